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
raw = buf.reshape(GENS, BLK, PTS)
ent = raw[:, :, 0:4].copy()  # entry stamps: clock | HW_ID << 40 | XCC_ID << 56
ts = (raw & np.uint64((1 << 40) - 1)).astype(np.int64)
names = ["entry->staged", "staged->searched(FK,filt)", "search", "sum->done(eval)", "pbest,pushes"]
pts = [0, 4, 8, 12, 16, 20]
print(f"P={P} wpp={os.environ.get('HPE_PSO_WPP', 'auto')}; medians over waves, us")
print("gen span ramp | " + " | ".join(names) + " | p90 start")
for g in range(1, 31):
    t = ts[g]
    w = np.stack([t[:, k:k + 4].reshape(-1) for k in pts], axis=1)  # (blocks*4, 6)
    w = w[w[:, 0] > 0]
    if not len(w):
        continue
    t0 = w[:, 0].min()
    ramp = (np.median(w[:, 0]) - t0) / 100
    ph = np.diff(w, axis=1) / 100
    ok = (w[:, 1:] > 0)  # the second wave of a particle (wpp 2) leaves before the last point
    med = [np.median(ph[ok[:, k], k]) if ok[:, k].any() else float("nan") for k in range(5)]
    end = w[:, 5][w[:, 5] > 0]
    print(f"{g:3d} {(max(end.max(), w[:, 4].max()) - t0) / 100:6.2f} {ramp:5.2f} | " +
          " | ".join(f"{v:5.2f}" for v in med) +
          f" | start spread {(np.percentile(w[:, 0], 90) - t0) / 100:5.2f}")

# placement of generation 10's sampled waves: start time vs (XCC, SE, CU) and the number of
# workgroups each CU ran
g = 10
e = ent[g].reshape(-1)
t = ts[g, :, 0:4].reshape(-1)
ok = e != 0
hw = (e[ok] >> np.uint64(40)) & np.uint64(0xFFFF)
xcc = (e[ok] >> np.uint64(56)) & np.uint64(0xF)
cu = ((hw >> np.uint64(8)) & np.uint64(0xF)).astype(int)
sh = ((hw >> np.uint64(12)) & np.uint64(1)).astype(int)
se = ((hw >> np.uint64(13)) & np.uint64(0x7)).astype(int)
simd = ((hw >> np.uint64(4)) & np.uint64(3)).astype(int)
slot = (hw & np.uint64(0xF)).astype(int)
st = (t[ok] - t[ok].min()) / 100
key = xcc.astype(int) * 1000 + se * 100 + sh * 16 + cu
print(f"gen {g}: {ok.sum()} sampled waves on {len(np.unique(key))} CUs, XCCs {sorted(set(xcc.tolist()))}")
late = st > 2.0
print(f"  started > 2 us after the first: {late.sum()} waves; early-wave slots {np.bincount(slot[~late])}; late-wave slots {np.bincount(slot[late]) if late.any() else []}")
per_cu = {}
for k, s_ in zip(key, st):
    per_cu.setdefault(k, []).append(s_)
cnt = np.array([len(v) for v in per_cu.values()])
print("  waves per sampled CU (histogram):", np.bincount(cnt))
ex = list(per_cu.items())[:4]
for k, v in ex:
    print(f"  CU {k}: starts {sorted(np.round(v, 2).tolist())}")
