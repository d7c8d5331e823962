"""Diagnostic (GPU): dump the results of one build (HPE_LIB_VARIANT) on the config-2 frame
for a bitwise A/B of two builds: FK spheres, costs, refine, pso_evolve, tracked frame.
Usage: python tools/ab_dump.py out.npz"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "hand-pose-estimation_amd"), str(ROOT / "oracle"), str(ROOT / "tests")]
import torch  # noqa: E402

torch.cuda.is_available()
import hand_data  # noqa: E402
import hpe  # noqa: E402
import oracle_np  # noqa: E402

gh = hpe.reference_hand(device=0)
poses = hand_data.trajectory(4, seed=2)
depth = gh.ctx.render_depth(poses[3])
om = hpe.observedmodel()
om.downsample = True
om.set_depth_mm(depth)
cf = hpe.costfunc(gh, om)
ub, lb, sd = oracle_np.reference_bounds()
out = {"depth": depth}
th = np.stack([poses[k] for k in range(4)])
out["cost"] = np.array([cf.cal_cost(t.copy()) for t in th])
pso = hpe.PSO()
pso.set_pso_params(ub, lb, sd, 0.7298, 1.49618, 1.49618, 31, 1e-8, 1e-8)
x = poses[2].copy()
pso.refine_init_pose(x, cf)
out["refine"] = x.copy()
out["refine_evals"] = pso.last_refine_evals
b = np.zeros(26)
pso.pso_evolve(cf, x.copy(), 256, b)
out["pso_from_refined"] = b.copy()
out["pso_cost"] = pso.last_gbest_cost
g, c, t = pso.trace(cf)
out["trace_g"], out["trace_c"], out["trace_t"] = g, c, t
x = poses[2].copy()
out["track_cost"] = pso.track_frame(cf, x, 256, refine=True)
out["track_x"] = x.copy()
out["cal_cost_track_x"] = cf.cal_cost(x.copy())
g2, c2, t2 = pso.trace(cf)
out["track_trace_last"] = g2[-1]
x = poses[2].copy()
out["track_cost2"] = pso.track_frame(cf, x, 256, refine=True)
x = out["refine"].copy()
out["track_norefine_cost"] = pso.track_frame(cf, x, 256, refine=False)
out["track_norefine_x"] = x.copy()
np.savez(sys.argv[1], **out)
print({k: (v if np.ndim(v) == 0 else np.asarray(v).ravel()[:3]) for k, v in out.items() if k != "depth"})
