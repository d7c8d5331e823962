"""The C oracle against the golden fixtures of the numpy restatement
(tests/golden/make_golden.py).  Two independent restatements of the reference lines
must agree before either is trusted as the parity oracle.

Tolerances: FK 1e-12 cm (numpy vs glibc sin/cos may differ by an ulp); costs relative
1e-12; correspondences, distance transform, cloud exact; PSO pose 1e-9, refine pose 1e-7.
"""
from pathlib import Path

import numpy as np
import pytest

import hand_data
import oracle_np

G = Path(__file__).resolve().parent / "golden"


def _load(name):
    return dict(np.load(G / name, allow_pickle=False))


@pytest.fixture(scope="module")
def frame(oracle):
    f = _load("frame.npz")
    return f, oracle.preprocess(f["depth_mm"], downsample=True)


def test_fk_golden(oracle, ora_hand):
    g = _load("fk.npz")
    for i, t in enumerate(g["theta"]):
        S, J = oracle.build(ora_hand, t, joints=True)
        np.testing.assert_allclose(S, g["spheres"][i], rtol=0, atol=1e-12)
        np.testing.assert_allclose(J, g["joints"][i], rtol=0, atol=1e-12)


def test_preprocess_golden(oracle, frame):
    f, obs = frame
    np.testing.assert_array_equal(obs.cloud, f["cloud"])
    np.testing.assert_array_equal(obs.dt, f["dt"])
    np.testing.assert_array_equal(obs.depth, f["depth_cm"])
    assert obs.dtmax == f["dtmax"]
    assert abs(obs.scale - f["scale"]) <= 1e-13 * abs(f["scale"])  # mean: summation order
    full = oracle.preprocess(f["depth_mm"], downsample=False)
    assert full.n == int(f["nfull"])
    np.testing.assert_array_equal(full.cloud[::37], f["cloud_full_every37"])


def test_costs_golden(oracle, ora_hand, frame):
    f, obs = frame
    g = _load("costs.npz")
    c = oracle.eval_costs(ora_hand, obs, g["theta"])
    np.testing.assert_allclose(c, g["cost"], rtol=1e-12)
    c2 = oracle.eval_costs(ora_hand, obs, g["theta"], with_collision=True)
    np.testing.assert_allclose(c2, g["cost2"], rtol=1e-12)
    for i, t in enumerate(g["theta"]):
        cr, tr, mr = oracle.terms(ora_hand, obs, t)
        np.testing.assert_array_equal(mr, g["match"][i])
        np.testing.assert_allclose(tr, g["terms"][i], rtol=1e-12, atol=1e-300)


def test_pso_refine_golden(oracle, ora_hand, frame):
    f, obs = frame
    g = _load("pso.npz")
    ub, lb, sd = oracle_np.reference_bounds()
    bp, bc, tr = oracle.pso_evolve(ora_hand, obs, g["x0"], int(g["P"]), int(g["maxiter"]),
                                   lb, ub, sd, seed=1000)
    np.testing.assert_allclose(bp, g["bestp"], rtol=0, atol=1e-9)
    assert abs(bc - g["bestcost"]) <= 1e-12 * abs(g["bestcost"])
    np.testing.assert_allclose(tr["gbest"], g["trace"], rtol=1e-12)
    x, _ = oracle.refine(ora_hand, obs, g["x0"])
    # central differences (eps 1e-5) turn last-ulp cost differences (numpy's pairwise sum
    # vs Armadillo's 2-accumulator order) into ~1e-8 gradient differences
    np.testing.assert_allclose(x, g["refined"], rtol=0, atol=1e-7)
    # the decision-margin instrumentation the sequence tests rely on: refine took at least
    # one Goldstein test, so its smallest margin is finite and non-negative
    m = oracle.refine_last_margin()
    assert 0.0 <= m < float("inf")


def test_pso_optimise_golden(oracle, ora_hand, frame):
    """pso_optimise (PSO.cpp:539-712).  Each descent step's central difference (eps 1e-5)
    amplifies last-ulp cost differences between the two restatements; over 30 descent
    steps per particle they reach ~2e-7 in the pose, 2e-9 in the cost."""
    f, obs = frame
    g = _load("optimise.npz")
    ub, lb, sd = oracle_np.reference_bounds()
    bp, bc, tr = oracle.pso_optimise(ora_hand, obs, g["x0"], int(g["P"]), int(g["maxiter"]),
                                     lb, ub, sd, float(g["w"]), float(g["c1"]),
                                     float(g["c2"]), seed=1000)
    np.testing.assert_allclose(bp, g["bestp"], rtol=0, atol=1e-6)
    assert abs(bc - g["bestcost"]) <= 1e-8 * abs(g["bestcost"])
    np.testing.assert_allclose(tr, g["trace"], rtol=1e-8)


def test_draws_golden(oracle):
    g = _load("pso.npz")
    u = [oracle.u01(1000, s, gg, i, k) for s in (1, 2, 3, 4) for gg in (0, 1, 7)
         for i in (0, 5) for k in (0, 1, 25)]
    np.testing.assert_array_equal(np.array(u), g["u01"])
    np.testing.assert_allclose(oracle.normals(1000, 4), g["normals"], rtol=0, atol=1e-15)
