"""Diagnostic: the pipelined tracking loop with nothing else on the stream (no per-frame
timing events), wall time per frame.  Usage: python tools/loop_time.py [frames] [P]"""
import ctypes as C
import sys
import time
from pathlib import Path

import numpy as np
import torch

torch.cuda.set_device(0)
ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "hand-pose-estimation_amd"))
import hpe  # noqa: E402
from hpe import _lib, synth  # noqa: E402

nfr = int(sys.argv[1]) if len(sys.argv) > 1 else 40
P = int(sys.argv[2]) if len(sys.argv) > 2 else 256
hand = hpe.reference_hand()
ctx, lib = hand.ctx, hand.ctx.lib
poses = synth.trajectory(nfr + 4, 0)
raw = [np.ascontiguousarray(ctx.render_depth(th)) for th in poses]
ub, lb, sd = hpe.reference_bounds()
ctx.check(lib.hpe_set_pso_params(ctx.h, _lib.ptr(ub, C.c_double), _lib.ptr(lb, C.c_double),
                                 _lib.ptr(sd, C.c_double), 0.7298, 1.49618, 1.49618, 31, 1e-8, 1e-8))
st = torch.zeros(27, dtype=torch.float64, device="cuda:0")
for rep in range(2):
    st[:26] = torch.from_numpy(poses[0])
    torch.cuda.synchronize()
    ctx.pipeline_begin(raw[0])
    for f in range(3):  # warm-up (graph capture)
        ctx.track_pipelined(P, 1, st.data_ptr(), raw[f + 1])
    ctx.check(lib.hpe_sync(ctx.h))
    t0 = time.perf_counter()
    for f in range(3, nfr + 3):
        ctx.track_pipelined(P, 1, st.data_ptr(), raw[f + 1])
    ctx.check(lib.hpe_sync(ctx.h))
    el = time.perf_counter() - t0
    print({"rep": rep, "frames": nfr, "ms_per_frame": el / nfr * 1e3, "cost": float(st[26])})
