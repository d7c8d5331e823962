"""Diagnostic: host-side cost of each per-frame call of the end-to-end tracking loop."""
import ctypes as C
import sys
import time
from pathlib import Path

import numpy as np
import torch

torch.cuda.set_device(0)  # torch's HIP runtime first (as bench.py does)

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "hand-pose-estimation_amd"))
import hpe  # noqa: E402
from hpe import _lib, synth  # noqa: E402

hand = hpe.reference_hand()
ctx, lib = hand.ctx, hand.ctx.lib
poses = synth.trajectory(24, 0)
raw = [np.ascontiguousarray(ctx.render_depth(th)) for th in poses]
ub, lb, sd = hpe.reference_bounds()
ctx.check(lib.hpe_set_pso_params(ctx.h, _lib.ptr(ub, C.c_double), _lib.ptr(lb, C.c_double),
                                 _lib.ptr(sd, C.c_double), 0.7298, 1.49618, 1.49618, 31, 1e-8, 1e-8))
state = torch.zeros(27, dtype=torch.float64, device="cuda:0")
state[:26] = torch.from_numpy(poses[0])
torch.cuda.synchronize()
tp = ts = tt = 0.0
ctx.prepare_frame(0, raw[0])
for f in range(23):
    a = time.perf_counter()
    ctx.prepare_frame((f + 1) % 4, raw[f + 1])
    b = time.perf_counter()
    ctx.select_frame(f % 4)
    c = time.perf_counter()
    ctx.check(lib.hpe_track_frame_dev(ctx.h, 256, 1, C.c_void_p(state.data_ptr())))
    d = time.perf_counter()
    if f >= 3:
        tp += b - a; ts += c - b; tt += d - c
ctx.check(lib.hpe_sync(ctx.h))
n = 20
print(f"prepare {tp / n * 1e6:.1f} us  select {ts / n * 1e6:.1f} us  track(graph launch) {tt / n * 1e6:.1f} us")
# raw pinned memcpy alone
x = np.zeros_like(raw[0])
a = time.perf_counter()
for _ in range(100):
    np.copyto(x, raw[1])
print(f"numpy 307KB copy {(time.perf_counter() - a) / 100 * 1e6:.1f} us")
