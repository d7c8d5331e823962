"""Diagnostic: per-phase cycle breakdown of k_pso_gen and k_refine from the stamps
build (libhpe_stamps.so).  Usage: python tools/stamps.py [frames]"""
import ctypes as C
import sys
from pathlib import Path

import numpy as np
import torch

torch.cuda.set_device(0)  # torch's HIP runtime first

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "hand-pose-estimation_amd"))
import hpe  # noqa: E402
from hpe import _lib, synth  # noqa: E402

lib = _lib.load(ROOT / "hand-pose-estimation_amd" / "libhpe_stamps.so")
_lib._lib = lib  # make the package use the diagnostic build
nfr = int(sys.argv[1]) if len(sys.argv) > 1 else 4
P = int(sys.argv[2]) if len(sys.argv) > 2 else 256
hand = hpe.reference_hand()
ctx = hand.ctx
poses, sizes = synth.load_sequence(ctx, nfr + 1)
ub, lb, sd = hpe.reference_bounds()
ctx.check(lib.hpe_set_pso_params(ctx.h, _lib.ptr(ub, C.c_double), _lib.ptr(lb, C.c_double),
                                 _lib.ptr(sd, C.c_double), 0.7298, 1.49618, 1.49618, 31, 1e-8,
                                 1e-8))
st = np.zeros(64, dtype=np.uint64)
x = np.ascontiguousarray(poses[0])
ctx.select_frame(0)
lib.hpe_track_frame(ctx.h, P, 1, _lib.ptr(x, C.c_double), None)
lib.hpe_debug_stamps(st.ctypes.data_as(C.POINTER(C.c_uint64)))  # reset
names = {4: "gen: prologue (og + hand)", 5: "gen: block-0 span (cycles)",
         6: "gen: block-0 span (100MHz ticks)", 0: "gen: argmin+sig", 1: "gen: informant", 2: "gen: velocity", 3: "gen: pbest tail",
         10: "eval: fk", 11: "eval: search/align+depth+coll", 12: "eval: block_sum",
         13: "fk: trig phase", 14: "fk: chain+spheres phase", 15: "wave: depth issue",
         16: "wave: align frozen", 17: "wave: collision", 18: "wave: 3 reductions",
         20: "refine: corr eval", 21: "refine: grad evals", 22: "refine: goldstein",
         23: "refine: iter glue", 24: "prep (fused): band workgroups (incl. merge)",
         25: "prep (fused): DT workgroup", 19: "goldstein: speculated round",
         26: "opt: m=0 corr eval", 27: "opt: grad (2 waves)", 28: "opt: step tail (+m=0 re-match)"}
tot = np.zeros(64)
for f in range(1, nfr + 1):
    ctx.select_frame(f)
    ctx.check(lib.hpe_track_frame(ctx.h, P, 1, _lib.ptr(x, C.c_double), None))
    ctx.check(lib.hpe_sync(ctx.h))
    rc = lib.hpe_debug_stamps(st.ctypes.data_as(C.POINTER(C.c_uint64)))
    tot += st
# pipelined frames: next-frame preparation fused into the refine launch
import torch  # noqa: E402
raw = [np.ascontiguousarray(ctx.render_depth(th)) for th in poses]
stt = torch.zeros(27, dtype=torch.float64, device="cuda:0")
stt[:26] = torch.from_numpy(poses[0])
ctx.pipeline_begin(raw[0])
for f in range(nfr):
    ctx.track_pipelined(P, 1, stt.data_ptr(), raw[f + 1])
ctx.check(lib.hpe_sync(ctx.h))
lib.hpe_debug_stamps(st.ctypes.data_as(C.POINTER(C.c_uint64)))
tot[24] += st[24]; tot[25] += st[25]; tot[56] += st[56]; tot[57] += st[57]
print("stamps build:", rc)
for k, nm in names.items():
    n = tot[32 + k]
    if n:
        print(f"{nm:34s} laps {int(n):7d}  avg {tot[k] / n:10.1f} cyc  total/frame {tot[k] / nfr:12.0f} cyc")

# pso_optimise (test_full settings, P = 32): descent-phase breakdown of block 0
ctx.select_frame(1)
lib.hpe_debug_stamps(st.ctypes.data_as(C.POINTER(C.c_uint64)))  # reset
x = np.ascontiguousarray(poses[0]); bp = np.zeros(26); bc = C.c_double(0)
ctx.check(lib.hpe_set_pso_params(ctx.h, _lib.ptr(ub, C.c_double), _lib.ptr(lb, C.c_double),
                                 _lib.ptr(sd, C.c_double), 0.7298, 1.49618, 1.49618, 21, 1e-8,
                                 1e-8))
ctx.check(lib.hpe_pso_optimise(ctx.h, _lib.ptr(x, C.c_double), 32, _lib.ptr(bp, C.c_double),
                               C.byref(bc), None, 0))
lib.hpe_debug_stamps(st.ctypes.data_as(C.POINTER(C.c_uint64)))
print("pso_optimise P=32 maxiter=21 (20 descent launches, block 0):")
print("  goldstein searches %d: accepted %d, trials %d, down %d, up %d" %
      (st[32 + 9], st[9], st[30], st[7], st[8]))
for k in (26, 27, 19, 28, 15, 16, 17, 18):
    n = st[32 + k]
    if n:
        print(f"{names[k]:34s} laps {int(n):7d}  avg {st[k] / n:10.1f} cyc  per launch {st[k] / 20:12.0f} cyc")
