"""Diagnostic (GPU): per-wave wall-clock phases of the wave-form generation k_pso_gen_w from
the timelines build (libhpe_rts.so, s_memrealtime at 100 MHz, lane 0 of each wave of the
first 256 workgroups).  One pso_evolve of P particles x 31 generations on a bench frame.
Usage: python tools/wave_ts.py P [wpp]"""
import ctypes as C
import os
import sys
from pathlib import Path

import numpy as np
import torch

torch.cuda.set_device(0)
ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "hand-pose-estimation_amd"))
P = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
os.environ["HPE_PSO_FORM"] = "wave"
if len(sys.argv) > 2:
    os.environ["HPE_PSO_WPP"] = sys.argv[2]
import hpe  # noqa: E402
from hpe import _lib, synth  # noqa: E402

lib = _lib.load(ROOT / "hand-pose-estimation_amd" / "libhpe_rts.so")
_lib._lib = lib
lib.hpe_debug_blk_ts.restype = C.c_int
lib.hpe_debug_blk_ts.argtypes = [C.POINTER(C.c_uint64)]
GENS, BLK, PTS = 48, 256, 24
hand = hpe.reference_hand()
pose = synth.trajectory(4, 0, revert=0.02)
om = hpe.observedmodel()
om.downsample = True
om.set_depth_mm(hand.ctx.render_depth(pose[3]))
cf = hpe.costfunc(hand, om)
ub, lb, sd = hpe.reference_bounds()
pso = hpe.PSO()
pso.set_pso_params(ub, lb, sd, 0.7298, 1.49618, 1.49618, 31, 1e-8, 1e-8)
bestp = np.zeros(26)
buf = np.zeros(GENS * BLK * PTS, dtype=np.uint64)
for rep in range(2):
    pso.pso_evolve(cf, pose[2].copy(), P, bestp)
    lib.hpe_debug_blk_ts(buf.ctypes.data_as(C.POINTER(C.c_uint64)))
ts = buf.reshape(GENS, BLK, PTS).astype(np.int64)
NPT = 11
names = ["entry->informant", "->hand staged", "barrier", "FK", "depth issue+filter tables",
         "search", "sums", "particle sum barrier", "pbest+pch", "pushes"]
print(f"P={P} wpp={os.environ.get('HPE_PSO_WPP', 'auto')}; the even waves of a sample of "
      f"workgroups (slot 2k + wave/2), medians over waves, us")
print("gen  span | " + " | ".join(names))
for g in range(1, 31):
    t = ts[g]
    w = np.concatenate([t[:, [2 * k + j for k in range(NPT)]] for j in range(2)], axis=0)  # (waves, NPT)
    w = w[w[:, 0] > 0]
    if not len(w):
        continue
    t0 = w[:, 0].min()
    end = w[:, 10][w[:, 10] > 0]
    span = ((end.max() if len(end) else w.max()) - t0) / 100
    med = []
    for k in range(NPT - 1):
        ok = (w[:, k] > 0) & (w[:, k + 1] > 0)
        med.append(np.median(w[ok, k + 1] - w[ok, k]) / 100 if ok.any() else float("nan"))
    st = (w[:, 0] - t0) / 100
    en = (end - t0) / 100 if len(end) else st
    print(f"{g:3d} {span:6.2f} | " + " | ".join(f"{v:5.2f}" for v in med) +
          f" | start p10/50/90 {np.percentile(st, 10):.2f}/{np.percentile(st, 50):.2f}/"
          f"{np.percentile(st, 90):.2f} end {np.percentile(en, 10):.2f}/{np.percentile(en, 50):.2f}/"
          f"{np.percentile(en, 90):.2f}")
