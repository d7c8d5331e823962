"""pso_optimise GPU vs C oracle, generation by generation: how fast do the gbest traces
separate?  (Each descent step differentiates with eps 1e-5; last-ulp cost differences grow
over the generations, so long runs are compared through their traces' early agreement.)"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "hand-pose-estimation_amd"), str(ROOT / "oracle"), str(ROOT / "tests")]
import torch  # noqa: E402

torch.cuda.init()
import numpy as np  # noqa: E402

import hand_data  # noqa: E402
import hpe  # noqa: E402
import oracle_c  # noqa: E402
import oracle_np  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 8
M = int(sys.argv[2]) if len(sys.argv) > 2 else 30
geo, rad = hand_data.geometry_cm()
nh = oracle_np.Hand(geo, rad)
truth = hand_data.trajectory(2, seed=21)[1]
d = oracle_np.render_depth_mm(nh, truth)
o = oracle_c.load(build=False)
h = o.hand(geo, rad)
ob = o.preprocess(d, downsample=True)
ub, lb, sd = oracle_np.reference_bounds()
w, c1, c2 = 0.7298, 1.49618, 1.49618
rb, rc, rtr = o.pso_optimise(h, ob, oracle_np.X0.copy(), P, M, lb, ub, sd, w, c1, c2)
gh = hpe.reference_hand(device=0)
om = hpe.observedmodel()
om.downsample = True
om.set_depth_mm(d)
cf = hpe.costfunc(gh, om)
pso = hpe.PSO()
pso.set_pso_params(ub, lb, sd, w, c1, c2, M, 1e-8, 1e-8)
bp = np.zeros(26)
pso.pso_optimise(cf, oracle_np.X0.copy(), P, bp)
gtr = pso.last_optimise_trace
for g in range(M - 1):
    print("gen %3d  gpu %.15g  oracle %.15g  rel %.3g" % (g + 1, gtr[g], rtr[g],
                                                         abs(gtr[g] - rtr[g]) / abs(rtr[g])))
print("final |dbestp| %.3g" % np.abs(bp - rb).max())
