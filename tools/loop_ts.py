"""Diagnostic: per-block wall-clock phases of k_pso_loop (grid-resident PSO) from the
timelines build (libhpe_rts.so, s_memrealtime at 100 MHz).  Per generation: the wait
(poll start -> every tag matched), how long after the LAST block of the previous
generation published its granules each block saw them, and the phases after it.
Usage: python tools/loop_ts.py [frames] [P]"""
import ctypes as C
import sys
from pathlib import Path

import numpy as np
import torch

torch.cuda.set_device(0)
ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "hand-pose-estimation_amd"))
import hpe  # noqa: E402
from hpe import _lib, synth  # noqa: E402

lib = _lib.load(ROOT / "hand-pose-estimation_amd" / "libhpe_rts.so")  # make timelines
_lib._lib = lib
lib.hpe_debug_blk_ts.restype = C.c_int
lib.hpe_debug_blk_ts.argtypes = [C.POINTER(C.c_uint64)]
nfr = int(sys.argv[1]) if len(sys.argv) > 1 else 4
P = int(sys.argv[2]) if len(sys.argv) > 2 else 256
GENS, BLK, PTS = 48, 256, 24
hand = hpe.reference_hand()
ctx = hand.ctx
poses = synth.trajectory(nfr + 1, 0)
raw = [np.ascontiguousarray(ctx.render_depth(th)) for th in poses]
ub, lb, sd = hpe.reference_bounds()
ctx.check(lib.hpe_set_pso_params(ctx.h, _lib.ptr(ub, C.c_double), _lib.ptr(lb, C.c_double),
                                 _lib.ptr(sd, C.c_double), 0.7298, 1.49618, 1.49618, 31, 1e-8, 1e-8))
st = torch.zeros(27, dtype=torch.float64, device="cuda:0")
st[:26] = torch.from_numpy(poses[0])
ctx.pipeline_begin(raw[0])
buf = np.zeros(GENS * BLK * PTS, dtype=np.uint64)
for f in range(nfr):
    ctx.track_pipelined(P, 1, st.data_ptr(), raw[f + 1])
    ctx.check(lib.hpe_sync(ctx.h))
    lib.hpe_debug_blk_ts(buf.ctypes.data_as(C.POINTER(C.c_uint64)))
ts = buf.reshape(GENS, BLK, PTS).astype(np.int64)
nb = min(P, BLK)
print("gen  period  wait(med/max)  seen-after-last-publish(med/max)  dec+vel+FK  eval  publish   [us]")
rows = []
for g in range(2, 31):
    t, tp = ts[g, :nb], ts[g - 1, :nb]
    if not t[:, 1].any() or not tp[:, 4].any():
        continue
    last_pub = tp[:, 4].max()
    wait = (t[:, 1] - t[:, 0]) / 100
    seen = (t[:, 1] - last_pub) / 100
    period = np.median(t[:, 1] - tp[:, 1]) / 100
    ph = [np.median(t[:, b] - t[:, a]) / 100 for a, b in ((1, 2), (2, 3), (3, 4))]
    rows.append([period, np.median(wait), wait.max(), np.median(seen), seen.max()] + ph)
    print(f"{g:3d}  {period:6.2f}  {np.median(wait):5.2f}/{wait.max():5.2f}    "
          f"{np.median(seen):5.2f}/{seen.max():5.2f}                     "
          f"{ph[0]:5.2f}  {ph[1]:5.2f}  {ph[2]:5.2f}")
r = np.array(rows)
print("mean ", " ".join(f"{v:6.2f}" for v in r.mean(0)))
