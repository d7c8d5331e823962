"""Diagnostic: wall-clock timeline of refine_init_pose (k_refine workgroup 0) from the
timelines build (libhpe_rts.so, s_memrealtime at 100 MHz), over pipelined frames.
Phases: corr = cal_cost2 with new correspondences, grad = the six central differences,
gold = one speculated Goldstein round, glue = the rest of an iteration.
Usage: python tools/ref_ts.py [frames] [P]"""
import ctypes as C
import sys
from collections import defaultdict
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
lib.hpe_debug_ref_ts.restype = C.c_int
lib.hpe_debug_ref_ts.argtypes = [C.POINTER(C.c_uint64)]
nfr = int(sys.argv[1]) if len(sys.argv) > 1 else 20
P = int(sys.argv[2]) if len(sys.argv) > 2 else 256
RT = 16384
hand = hpe.reference_hand()
ctx = hand.ctx
poses = synth.trajectory(nfr + 4, 0, revert=0.02)  # the bench sequence
raw = [np.ascontiguousarray(ctx.render_depth(th)) for th in poses]
ub, lb, sd = hpe.reference_bounds()
ctx.check(lib.hpe_set_pso_params(ctx.h, _lib.ptr(ub, C.c_double), _lib.ptr(lb, C.c_double),
                                 _lib.ptr(sd, C.c_double), 0.7298, 1.49618, 1.49618, 31, 1e-8, 1e-8))
st = torch.zeros(27, dtype=torch.float64, device="cuda:0")
st[:26] = torch.from_numpy(poses[0])
ctx.pipeline_begin(raw[0])
buf = np.zeros(RT, dtype=np.uint64)
dur = defaultdict(list)
per_frame = []
for f in range(nfr + 3):
    ctx.track_pipelined(P, 1, st.data_ptr(), raw[f + 1])
    ctx.check(lib.hpe_sync(ctx.h))
    lib.hpe_debug_ref_ts(buf.ctypes.data_as(C.POINTER(C.c_uint64)))
    if f < 3:
        continue
    ent = [(int(v) >> 8, int(v) & 0xff) for v in buf if v]
    if not ent:
        continue
    last = {}
    iters = rounds = 0
    rstart = None  # start of the current batch of node evaluations
    for t, ph in ent:
        if ph == 1:
            if 0 in last and iters == 0:
                dur["start"].append((t - last[0]) / 100.0)
        elif ph == 2:
            dur["corr"].append((t - last[1]) / 100.0); iters += 1
            rstart = t
        elif ph == 9:
            dur["  node0 eval"].append((t - rstart) / 100.0)
        elif ph == 8:
            dur["  barrier wait"].append((t - last[9]) / 100.0)
        elif ph == 3:
            dur["grad"].append((t - last[2]) / 100.0)
            rstart = t
        elif ph == 4:
            dur["gold round"].append((t - rstart) / 100.0); rounds += 1
            dur["  walk+copy"].append((t - last[8]) / 100.0)
            rstart = t
        elif ph == 5:
            dur["glue"].append((t - last[4]) / 100.0 if 4 in last else 0.0)
        last[ph] = t
    per_frame.append(((ent[-1][0] - ent[0][0]) / 100.0, iters, rounds))
for k, v in dur.items():
    v = np.array(v)
    print(f"{k:11s} n {len(v):5d}  median {np.median(v):7.2f} us  mean {v.mean():7.2f} us  "
          f"total/frame {v.sum() / len(per_frame):8.1f} us")
pf = np.array(per_frame)
print(f"refine per frame: {pf[:, 0].mean():.1f} us, {pf[:, 1].mean():.1f} iterations, "
      f"{pf[:, 2].mean():.1f} Goldstein rounds")
