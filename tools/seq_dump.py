"""Track a synthetic sequence through the pipelined loop (bench.py's path) and dump the
per-frame GPU results + raw input frames for offline comparison with the oracle
(tools/seq_compare.py).  usage: seq_dump.py OUT.npz [n_frames] [P] [maxiter] [seed]"""
import ctypes as C
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "hand-pose-estimation_amd"), str(ROOT / "tests"), str(ROOT / "oracle")]
import hand_data  # noqa: E402
import hpe  # noqa: E402

out = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 400
P = int(sys.argv[3]) if len(sys.argv) > 3 else 256
maxiter = int(sys.argv[4]) if len(sys.argv) > 4 else 31
seed = int(sys.argv[5]) if len(sys.argv) > 5 else 7
gh = hpe.reference_hand(0)
ctx, lib = gh.ctx, gh.ctx.lib
poses = hand_data.trajectory(n, seed=seed, revert=0.02)
raw = np.array([gh.ctx.render_depth(th) for th in poses], dtype=np.float32)
ub, lb, sd = hpe.reference_bounds()
pso = hpe.PSO()
pso.set_pso_params(ub, lb, sd, 0.7298, 1.49618, 1.49618, maxiter, 1e-8, 1e-8)
pso._push(ctx)
state = torch.zeros(27, dtype=torch.float64, device="cuda:0")
state[:26] = torch.from_numpy(poses[0].copy())
torch.cuda.synchronize()
ctx.pipeline_begin(raw[0], True, True)
gx, gc, ev = [], [], []
tot = C.c_uint64(0)
ctx.check(lib.hpe_refine_eval_count(ctx.h, C.byref(tot), 1))
for f in range(n):
    ctx.track_pipelined(P, 1, state.data_ptr(), raw[f + 1] if f + 1 < n else None)
    ctx.check(lib.hpe_sync(ctx.h))
    torch.cuda.synchronize()
    s = state.cpu().numpy()
    gx.append(s[:26].copy())
    gc.append(s[26])
    ctx.check(lib.hpe_refine_eval_count(ctx.h, C.byref(tot), 1))
    ev.append(tot.value)
np.savez_compressed(out, raw=raw, poses=poses, gx=np.array(gx), gc=np.array(gc),
                    evals=np.array(ev), P=P, maxiter=maxiter)
print(f"dumped {n} frames to {out}")
