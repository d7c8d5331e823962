"""Diagnostic: standalone k_prepare (observedmodel::next_frame on the GPU: depth, cloud,
scale, chamfer DT) timed with the library's per-dispatch events.
Usage: python tools/prep_time.py [frames]   (HPE_LIB_VARIANT selects a second build)"""
import ctypes as C
import sys
from pathlib import Path

import numpy as np
import torch

torch.cuda.set_device(0)
ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "hand-pose-estimation_amd"))
import hpe  # noqa: E402
from hpe import synth  # noqa: E402

nfr = int(sys.argv[1]) if len(sys.argv) > 1 else 16
hand = hpe.reference_hand()
ctx, lib = hand.ctx, hand.ctx.lib
poses = synth.trajectory(nfr, 0)
raw = [np.ascontiguousarray(ctx.render_depth(th)) for th in poses]
for f in range(nfr):  # warm-up
    ctx.prepare_frame(f % 4, raw[f])
ctx.check(lib.hpe_sync(ctx.h))
ctx.check(lib.hpe_profile_enable(ctx.h, 1))
for f in range(nfr):
    ctx.prepare_frame(f % 4, raw[f])
    ctx.check(lib.hpe_sync(ctx.h))
nl = C.c_int32(0); tot = C.c_double(0); mn = C.c_double(0); mx = C.c_double(0)
ctx.check(lib.hpe_profile_read_kernel(ctx.h, 4, C.byref(nl), C.byref(tot), C.byref(mn), C.byref(mx)))
print({"k_prepare_launches": nl.value, "avg_us": tot.value / max(nl.value, 1) * 1e3,
       "min_us": mn.value * 1e3, "max_us": mx.value * 1e3})
