"""Generate the golden fixtures of tests/golden/ from the numpy restatement
(oracle/oracle_np.py), which is written independently of the C oracle
(oracle/hpe_oracle.c).  The reference itself cannot be built or run here (Armadillo and
OpenCV are absent) and ships no tests or expected values (§4), so
these fixtures pin the C oracle and the GPU path to a second restatement of the same
reference lines.

Run from the repo root:  python tests/golden/make_golden.py
"""
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
sys.path[:0] = [str(ROOT / "oracle"), str(ROOT / "tests")]

import hand_data  # noqa: E402
import oracle_np  # noqa: E402


def main():
    geo, rad = hand_data.geometry_cm()
    hand = oracle_np.Hand(geo, rad)
    rng = np.random.default_rng(2024)

    # FK: x0, random poses, bound extremes (handmodel.cpp:259-298)
    ub, lb, sd = oracle_np.reference_bounds()
    th = np.vstack([oracle_np.X0, ub, lb, hand_data.random_thetas(rng, 13, spread=2.0)])
    S = np.zeros((len(th), 48, 3)); J = np.zeros((len(th), 21, 3))
    for i, t in enumerate(th):
        S[i], J[i] = hand.build_hand_model(t, return_joints=True)
    np.savez_compressed(HERE / "fk.npz", theta=th, spheres=S, joints=J)

    # one frame: render -> preprocess (observedmodel.cpp:110-219, 272-369)
    truth = hand_data.trajectory(4, seed=17)[3]
    depth_mm = oracle_np.render_depth_mm(hand, truth)
    obs_ds, nfull = oracle_np.preprocess(depth_mm, downsample=True)
    obs_full, _ = oracle_np.preprocess(depth_mm, downsample=False)
    np.savez_compressed(HERE / "frame.npz", truth=truth, depth_mm=depth_mm,
                        depth_cm=obs_ds.depth, dt=obs_ds.dt, cloud=obs_ds.cloud,
                        cloud_full_every37=obs_full.cloud[::37], scale=obs_ds.scale, dtmax=obs_ds.dtmax,
                        nfull=nfull)

    # costs on the down-sampled frame (costfunc.cpp:31-127)
    th = np.vstack([truth, hand_data.random_thetas(rng, 23, x0=truth, spread=0.5)])
    cost = np.array([oracle_np.cal_cost(hand, obs_ds, t) for t in th])
    terms = np.zeros((len(th), 3)); match = np.zeros((len(th), obs_ds.cloud.shape[0]), np.int32)
    cost2 = np.zeros(len(th))
    for i, t in enumerate(th):
        cost2[i], match[i], terms[i] = oracle_np.cal_cost2(hand, obs_ds, t)
    np.savez_compressed(HERE / "costs.npz", theta=th, cost=cost, cost2=cost2, terms=terms,
                        match=match)

    # PSO (PSO.cpp:717-886, Philox draws) and refine (PSO.cpp:183-266)
    x0 = oracle_np.X0.copy()
    bestp, bestcost, trace = oracle_np.pso_evolve(hand, obs_ds, x0, 8, 4, lb, ub, sd)
    refined = oracle_np.refine_init_pose(hand, obs_ds, x0)
    u = np.array([oracle_np.u01(1000, s, g, i, k) for s in (1, 2, 3, 4) for g in (0, 1, 7)
                  for i in (0, 5) for k in (0, 1, 25)])
    np.savez_compressed(HERE / "pso.npz", x0=x0, P=8, maxiter=4, bestp=bestp,
                        bestcost=bestcost, trace=np.array(trace), refined=refined,
                        normals=oracle_np.normals(1000, 4), u01=u)
    make_optimise(hand, obs_ds)
    for f in sorted(HERE.glob("*.npz")):
        print(f.name, f.stat().st_size)


def make_optimise(hand=None, obs=None):
    """pso_optimise (PSO.cpp:539-712) on the golden frame: 8 particles, maxiter 4,
    set_pso_params' w, c1, c2 of test_full (testmodel.cpp:101-111)."""
    if hand is None:
        geo, rad = hand_data.geometry_cm()
        hand = oracle_np.Hand(geo, rad)
        f = np.load(HERE / "frame.npz")
        obs = oracle_np.Obs(f["depth_cm"], f["dt"], f["cloud"], float(f["scale"]))
    ub, lb, sd = oracle_np.reference_bounds()
    x0 = oracle_np.X0.copy()
    w, c1, c2 = 0.7298, 1.49618, 1.49618
    bestp, bestcost, trace = oracle_np.pso_optimise(hand, obs, x0, 8, 4, lb, ub, sd, w, c1, c2)
    np.savez_compressed(HERE / "optimise.npz", x0=x0, P=8, maxiter=4, w=w, c1=c1, c2=c2,
                        bestp=bestp, bestcost=bestcost, trace=np.array(trace))


if __name__ == "__main__":
    if sys.argv[1:] == ["optimise"]:
        make_optimise()
    else:
        main()
