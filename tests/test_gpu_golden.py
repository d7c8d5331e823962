"""The HIP path (through the C ABI) against the committed golden fixtures of the numpy
restatement (tests/golden/make_golden.py).  Tolerances as test_gpu_parity.py: FK 1e-9 cm,
costs relative 1e-9, correspondences tie-aware, PSO / refine pose 1e-6."""
from pathlib import Path

import numpy as np
import pytest

import oracle_np

pytestmark = pytest.mark.gpu
G = Path(__file__).resolve().parent / "golden"


def _load(name):
    return dict(np.load(G / name, allow_pickle=False))


@pytest.fixture(scope="module")
def setup():
    import hpe
    gh = hpe.reference_hand(0)
    f = _load("frame.npz")
    om = hpe.observedmodel(); om.downsample = True; om.set_depth_mm(f["depth_mm"])
    return gh, om, hpe.costfunc(gh, om), f


def test_fk_golden_gpu(setup):
    gh = setup[0]
    g = _load("fk.npz")
    S, J = gh.build_batch(g["theta"])
    np.testing.assert_allclose(S, g["spheres"], rtol=0, atol=1e-9)
    np.testing.assert_allclose(J, g["joints"], rtol=0, atol=1e-9)


def test_costs_golden_gpu(setup):
    gh, om, cf, f = setup
    np.testing.assert_array_equal(om.get_ptncloud(), f["cloud"])
    g = _load("costs.npz")
    c, m = cf.cal_cost_batch(g["theta"], return_match=True)
    np.testing.assert_allclose(c, g["cost"], rtol=1e-9)
    c2 = cf.cal_cost_batch(g["theta"], with_collision=True)
    np.testing.assert_allclose(c2, g["cost2"], rtol=1e-9)
    cloud = f["cloud"].astype(np.float32)
    for i, t in enumerate(g["theta"]):
        diff = np.nonzero(m[i] != g["match"][i])[0]
        if len(diff):  # tie-aware: equidistant in float
            S = oracle_np.Hand(*__import__("hand_data").geometry_cm()).build_hand_model(t)
            s = S.astype(np.float32)
            d1 = np.linalg.norm(cloud[diff] - s[m[i][diff]], axis=1)
            d2 = np.linalg.norm(cloud[diff] - s[g["match"][i][diff]], axis=1)
            assert np.all(np.abs(d1 - d2) <= 4 * np.spacing(np.maximum(d1, d2)))


def test_pso_refine_golden_gpu(setup):
    import hpe
    gh, om, cf, f = setup
    g = _load("pso.npz")
    ub, lb, sd = oracle_np.reference_bounds()
    pso = hpe.PSO()
    pso.set_pso_params(ub, lb, sd, 0.7298, 1.49618, 1.49618, int(g["maxiter"]), 1e-8, 1e-8)
    bp = np.zeros(26)
    pso.pso_evolve(cf, g["x0"], int(g["P"]), bp)
    np.testing.assert_allclose(bp, g["bestp"], rtol=0, atol=1e-6)
    assert abs(pso.last_gbest_cost - g["bestcost"]) <= 1e-8 * abs(g["bestcost"])
    gt, _, _ = pso.trace(cf)
    np.testing.assert_allclose(gt, g["trace"], rtol=1e-8)
    x = g["x0"].copy()
    pso.refine_init_pose(x, cf)
    np.testing.assert_allclose(x, g["refined"], rtol=0, atol=1e-6)


def test_pso_optimise_golden_gpu(setup):
    """pso_optimise against the numpy restatement's fixture (tolerances as in
    test_gpu_parity.test_pso_optimise)."""
    import hpe
    gh, om, cf, f = setup
    g = _load("optimise.npz")
    ub, lb, sd = oracle_np.reference_bounds()
    pso = hpe.PSO()
    pso.set_pso_params(ub, lb, sd, float(g["w"]), float(g["c1"]), float(g["c2"]),
                       int(g["maxiter"]), 1e-8, 1e-8)
    bp = np.zeros(26)
    assert pso.pso_optimise(cf, g["x0"], int(g["P"]), bp) == 1
    np.testing.assert_allclose(bp, g["bestp"], rtol=0, atol=1e-5)
    assert abs(pso.last_gbest_cost - g["bestcost"]) <= 1e-7 * abs(g["bestcost"])
    np.testing.assert_allclose(pso.last_optimise_trace, g["trace"], rtol=1e-7)
