"""Time pso_optimise (PSO.cpp:539-712) on the GPU for test_full's settings (P = 32,
maxiter = 200) and report per-kernel device times."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "hand-pose-estimation_amd"), str(ROOT / "oracle"), str(ROOT / "tests")]
import torch  # noqa: E402  (HIP runtime first)

torch.cuda.init()
import numpy as np  # noqa: E402

import hand_data  # noqa: E402
import hpe  # noqa: E402
import oracle_np  # noqa: E402
from hpe import _lib  # noqa: E402


def main():
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    maxiter = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    downsample = (sys.argv[3] != "0") if len(sys.argv) > 3 else True  # testmodel.cpp:64
    gh = hpe.reference_hand(device=0)
    geo, rad = hand_data.geometry_cm()
    nh = oracle_np.Hand(geo, rad)
    truth = hand_data.trajectory(2, seed=21)[1]
    om = hpe.observedmodel()
    om.downsample = downsample
    om.set_depth_mm(oracle_np.render_depth_mm(nh, truth))
    cf = hpe.costfunc(gh, om)
    ub, lb, sd = oracle_np.reference_bounds()
    pso = hpe.PSO()
    pso.set_pso_params(ub, lb, sd, 0.7298, 1.49618, 1.49618, maxiter, 1e-8, 1e-8)
    bp = np.zeros(26)
    pso.pso_optimise(cf, oracle_np.X0.copy(), P, bp)  # warm-up (allocations)
    ctx = cf.ctx
    ctx.lib.hpe_profile_enable(ctx.h, 1)
    t0 = time.perf_counter()
    pso.pso_optimise(cf, oracle_np.X0.copy(), P, bp)
    wall = time.perf_counter() - t0
    out = {"P": P, "maxiter": maxiter, "n": int(cf._obs_n()) if hasattr(cf, "_obs_n") else None,
           "downsample": downsample, "wall_ms": wall * 1e3, "cost": pso.last_gbest_cost}
    import ctypes as C
    for name, k in (("k_opt_descent", _lib.PROF_OPT_DESCENT), ("k_opt_move", _lib.PROF_OPT_MOVE)):
        n = C.c_int32(0); tot = C.c_double(0); mn = C.c_double(0); mx = C.c_double(0)
        ctx.lib.hpe_profile_read_kernel(ctx.h, k, C.byref(n), C.byref(tot), C.byref(mn), C.byref(mx))
        out[name] = {"launches": n.value, "avg_us": 1e3 * tot.value / max(n.value, 1),
                     "min_us": 1e3 * mn.value, "max_us": 1e3 * mx.value}
    ctx.lib.hpe_profile_enable(ctx.h, 0)
    print(out)


if __name__ == "__main__":
    main()
