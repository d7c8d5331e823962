"""Diagnostic (GPU): can RCCL run a 2-rank communicator whose ranks share one GPU?
Launched as: python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1
--master-port 29531 tools/rccl_same_device.py"""
import os

import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda:0"))
x = torch.full((27,), float(rank), dtype=torch.float64, device="cuda:0")
out = torch.zeros((2, 27), dtype=torch.float64, device="cuda:0")
dist.all_gather_into_tensor(out, x)
torch.cuda.synchronize()
print(f"rank {rank}: all_gather ok {out[:, 0].tolist()} rccl {torch.cuda.nccl.version()}", flush=True)
dist.destroy_process_group()
