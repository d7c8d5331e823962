"""Diagnostic: Goldstein decision paths of refine_init_pose and pso_optimise from the
stamps build (libhpe_stamps.so, hpe_debug_gold_log).  Prints how searches end, how many
speculated rounds they take, and the most common decision prefixes -- the input for
choosing which nodes the eight waves speculate."""
import collections
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
lib.hpe_debug_gold_log.argtypes = [C.POINTER(C.c_uint64), C.c_int]
_lib._lib = lib
N = 65537
buf = np.zeros(N, dtype=np.uint64)


def read_log():
    lib.hpe_debug_gold_log(buf.ctypes.data_as(C.POINTER(C.c_uint64)), N)
    n = int(min(buf[0], N - 1))
    return buf[1:1 + n].copy()


def report(name, log, depth=3):
    it = (log >> np.uint64(32)) & np.uint64(0xff)
    acc = (log >> np.uint64(40)) & np.uint64(1)
    path = log & np.uint64(0xffffffff)
    print(f"== {name}: {len(log)} searches, accepted {int(acc.sum())}, exhausted "
          f"{int((it >= 30).sum())}, trials avg {it.mean():.2f}")
    print("   balanced depth-%d rounds avg %.2f" % (depth, np.ceil(it / depth).mean()))
    seqs = collections.Counter()
    for p, n, a in zip(path.tolist(), it.tolist(), acc.tolist()):
        dec = "".join("U" if (p >> k) & 1 else "D" for k in range(n - (1 if a else 0)))
        seqs[dec + ("A" if a else "X")] += 1
    for s, c in seqs.most_common(25):
        print(f"   {c:6d}  {s}")


hand = hpe.reference_hand()
ctx = hand.ctx
nfr = int(sys.argv[1]) if len(sys.argv) > 1 else 8
poses, sizes = synth.load_sequence(ctx, nfr + 1)
ub, lb, sd = hpe.reference_bounds()
ctx.check(lib.hpe_set_pso_params(ctx.h, _lib.ptr(ub, C.c_double), _lib.ptr(lb, C.c_double),
                                 _lib.ptr(sd, C.c_double), 0.7298, 1.49618, 1.49618, 31, 1e-8,
                                 1e-8))
x = np.ascontiguousarray(poses[0])
read_log()
for f in range(1, nfr + 1):
    ctx.select_frame(f)
    ctx.check(lib.hpe_track_frame(ctx.h, 256, 1, _lib.ptr(x, C.c_double), None))
ctx.check(lib.hpe_sync(ctx.h))
log_refine = read_log()
report("refine_init_pose (tracking loop)", log_refine)
ctx.check(lib.hpe_set_pso_params(ctx.h, _lib.ptr(ub, C.c_double), _lib.ptr(lb, C.c_double),
                                 _lib.ptr(sd, C.c_double), 0.7298, 1.49618, 1.49618, 21, 1e-8,
                                 1e-8))
x = np.ascontiguousarray(poses[0]); bp = np.zeros(26); bc = C.c_double(0)
ctx.select_frame(1)
ctx.check(lib.hpe_pso_optimise(ctx.h, _lib.ptr(x, C.c_double), 32, _lib.ptr(bp, C.c_double),
                               C.byref(bc), None, 0))
log_opt = read_log()
report("pso_optimise descent (P=32, 20 generations)", log_opt)
out = ROOT / "gpurun_out"
out.mkdir(exist_ok=True)
np.savez(out / "gold_log.npz", refine=log_refine, optimise=log_opt)
