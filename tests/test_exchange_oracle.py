"""The oracle's mirror of the opt-in per-generation exchange (hpe_set_exchange; an
ICP-PSO style extension, NOT the reference's algorithm, whose gbest never enters the
velocity, PSO.cpp:824-832).  CPU checks of the mirror itself: without an exchange the
lockstep subswarms are exactly the independent pso_evolve runs; with one, every swarm
still returns a particle it evaluated (its cost is cal_cost of its pose) and the
exchange changes the trajectories."""
import numpy as np

import hand_data
import oracle_np


def _frame(oracle):
    hand = oracle_np.Hand(*hand_data.geometry_cm())
    poses = hand_data.trajectory(3, seed=21)
    return poses, oracle.preprocess(oracle_np.render_depth_mm(hand, poses[2]))


def test_no_exchange_is_independent_swarms(oracle, ora_hand):
    poses, obs = _frame(oracle)
    ub, lb, sd = oracle_np.reference_bounds()
    seeds = [1000, 1001, 1002]
    bp, bc = oracle.pso_evolve_xch(ora_hand, obs, poses[1], 32, 8, lb, ub, sd, seeds, 0)
    for r, sd_ in enumerate(seeds):
        rb, rc, _ = oracle.pso_evolve(ora_hand, obs, poses[1], 32, 8, lb, ub, sd, seed=sd_)
        np.testing.assert_array_equal(bp[r], rb)
        assert bc[r] == rc


def test_exchange_changes_swarms_consistently(oracle, ora_hand):
    poses, obs = _frame(oracle)
    ub, lb, sd = oracle_np.reference_bounds()
    seeds = [1000, 1001]
    b0, c0 = oracle.pso_evolve_xch(ora_hand, obs, poses[1], 32, 11, lb, ub, sd, seeds, 0)
    b2, c2 = oracle.pso_evolve_xch(ora_hand, obs, poses[1], 32, 11, lb, ub, sd, seeds, 2)
    assert not np.array_equal(b0, b2)
    for r in range(2):  # each swarm's gbest is a pose it evaluated, at its cal_cost
        assert abs(oracle.cal_cost(ora_hand, obs, b2[r]) - c2[r]) <= 1e-12 * abs(c2[r])
    # every = maxiter - 1 or more: the only candidate exchange point is the last
    # generation, which has no successor, so nothing changes
    b9, c9 = oracle.pso_evolve_xch(ora_hand, obs, poses[1], 32, 11, lb, ub, sd, seeds, 10)
    np.testing.assert_array_equal(b9, b0)
