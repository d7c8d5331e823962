"""Diagnostic: per-block wall-clock phases of k_pso_gen from the timelines build
(libhpe_rts.so, s_memrealtime at 100 MHz).  Tracks a few pipelined frames and
analyses the generations of the last one.  Usage: python tools/blk_ts.py [frames] [P]"""
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
poses = synth.trajectory(nfr + 1, 0, revert=0.02)  # the bench sequence
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
rows = []
names = ["round1", "barrier1", "vel+FK", "eval", "tail"]
print("gen  span_us  ramp_us  gap_to_next_us | median phase us: " + " ".join(names) +
      " | max-block phase us")
for g in range(1, 31):
    t = ts[g, :nb]
    if not t[:, 0].any():
        continue
    t0, t1 = t[:, 0].min(), t[:, 5].max()
    ramp = (t[:, 0].max() - t0) / 100
    nxt = ts[g + 1, :nb, 0].min() if g + 1 < GENS and ts[g + 1, :nb, 0].any() else None
    gap = (nxt - t1) / 100 if nxt is not None else float("nan")
    ph = np.diff(t[:, :6], axis=1) / 100
    med = np.median(ph, axis=0)
    mx = ph.max(axis=0)
    rows.append((g, (t1 - t0) / 100, ramp, gap, *med, *mx))
    print(f"{g:3d} {(t1 - t0) / 100:8.2f} {ramp:8.2f} {gap:8.2f} | " +
          " ".join(f"{v:6.2f}" for v in med) + " | " + " ".join(f"{v:6.2f}" for v in mx))
    if g == 1 or g == 15:
        # finer points (median over blocks, us from entry): 6 round-1 loads landed,
        # 7 informant done, 1 pre-barrier, 2 post-barrier, 10 velocity done, 3 FK done,
        # 15 search start, 11 distances, 12 sqrt class, 13 index, 14 residual, 8 search done, 9 depth done, 4 eval done, 5 end
        rel = (t - t[:, :1]) / 100
        print("     points from entry:", " ".join(f"{k}:{np.median(rel[:, k]):.2f}"
                                            for k in (6, 7, 1, 2, 10, 3, 15, 11, 12, 13, 14, 8, 9, 4, 5)))
        print("     waves at the reduction:", " ".join(f"w{k - 16}:{np.median(rel[:, k]):.2f}"
                                                 for k in range(16, 24)))
r = np.array(rows)
print("mean span %.2f  ramp %.2f  gap %.2f | median phases %s" %
      (r[:, 1].mean(), r[:, 2].mean(), np.nanmean(r[:, 3]),
       " ".join(f"{v:.2f}" for v in r[:, 4:9].mean(axis=0))))
# where the last block to finish spent its time, per generation (critical block)
