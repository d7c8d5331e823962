"""Diagnostic: time of one refine_init_pose phase (correspondence eval, gradient batch or
speculated Goldstein round) on the product build, from kernel time / phase count.  Phase
counts come from the stamps build (libhpe_stamps.so), kernel times from the product
build's hipExtLaunchKernel events, on the same frames and x0."""
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

nfr = int(sys.argv[1]) if len(sys.argv) > 1 else 16
ds = (sys.argv[2] != "0") if len(sys.argv) > 2 else True


def run(libpath):
    lib = _lib.load(libpath)
    _lib._lib = lib
    hand = hpe.reference_hand()
    ctx = hand.ctx
    poses = synth.trajectory(nfr + 1, 0)
    for f in range(nfr + 1):
        ctx.prepare_frame(f, np.ascontiguousarray(ctx.render_depth(poses[f])), True, ds)
    ctx.check(lib.hpe_sync(ctx.h))
    st = np.zeros(64, dtype=np.uint64)
    lib.hpe_debug_stamps(st.ctypes.data_as(C.POINTER(C.c_uint64)))
    ctx.check(lib.hpe_profile_enable(ctx.h, 1))
    ev = C.c_int32(0)
    evals = 0
    for f in range(1, nfr + 1):
        ctx.select_frame(f)
        x = np.ascontiguousarray(poses[f - 1])
        ctx.check(lib.hpe_refine_init_pose(ctx.h, _lib.ptr(x, C.c_double), C.byref(ev)))
        evals += ev.value
    nl = C.c_int32(0); tot = C.c_double(0); mn = C.c_double(0); mx = C.c_double(0)
    ctx.check(lib.hpe_profile_read_kernel(ctx.h, 1, C.byref(nl), C.byref(tot), C.byref(mn), C.byref(mx)))
    lib.hpe_debug_stamps(st.ctypes.data_as(C.POINTER(C.c_uint64)))
    return tot.value * 1e3 / nl.value, evals / nfr, st


us, ev, _ = run(ROOT / "hand-pose-estimation_amd" / "libhpe.so")
_lib._lib = None
_, _, st = run(ROOT / "hand-pose-estimation_amd" / "libhpe_stamps.so")
iters = st[32 + 20] / nfr
rounds = st[32 + 19] / nfr
phases = 2 * iters + rounds
print(f"N={'250' if ds else 'full'}: refine {us:.1f} us/frame, {ev:.1f} evals, {iters:.2f} iterations, "
      f"{rounds:.2f} Goldstein rounds -> {phases:.1f} phases, {us / phases:.2f} us/phase")
