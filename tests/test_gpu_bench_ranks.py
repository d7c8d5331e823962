"""Config 5's multi-rank path end to end on ONE GPU: `bench.py --gpus 2 --backend gloo
--same-device --config subswarm8` runs two ranks (one process each, both on cuda:0), each
tracking the same frames with its own 1024-particle subswarm (seed 1000 + rank, wave form)
through the pipelined HIP loop, and exchanging {bestp, cost} once per frame through
hpe.dist.exchange_best (gloo through host memory here, RCCL on the 8-GPU
node).  The state after frame 0 must equal the oracle's best of the two subswarms tracking
that frame: refine_init_pose + pso_evolve(seed 1000 + r) + cal_cost(bestp)
(testmodel.cpp:124-138, PSO.cpp:717-722).  Tolerances as test_gpu_configs.py."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import hand_data
from hand_data import REFINE_RIGID
import oracle_np

pytestmark = pytest.mark.gpu


def _bench_ranks(dump, *extra):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, str(hand_data.ROOT / "bench.py"), "--gpus", "2", "--backend", "gloo",
           "--same-device", "--config", "subswarm8", "--steps", "3", "--warmup", "1",
           "--no-cpu-baseline", "--dump", str(dump), *extra]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    return json.loads(lines[0])


def test_bench_two_ranks_same_device_gloo(tmp_path, oracle, ora_hand):
    dump = tmp_path / "dump"
    r = _bench_ranks(dump)
    assert r["n_gpus"] == 2 and r["config"]["particles"] == 1024 and r["value"] > 0
    # the multi-rank self-verification the 8-GPU run will carry (bench.py rank_report)
    rk = r["ranks"]
    assert rk["world_size_pg"] == 2 and rk["backend"] == "gloo" and rk["same_device_mode"]
    assert len(rk["devices"]) == 2 and not rk["devices_distinct"]  # both on cuda:0
    assert all(d["pci"] == rk["devices"][0]["pci"] for d in rk["devices"])
    assert rk["final_state_identical"]
    assert 0 < rk["ms_per_step_min"] <= rk["ms_per_step_max"]
    assert rk["exchange_us"]["frames"] == 3 and rk["exchange_us"]["mean"] > 0
    # the N > 1 line carries the N = 1 figure of its own loop form and
    # names the refine form it ran (item 5)
    assert r["scaling_baseline_ms_per_step"] > 0 and r["per_frame_graph_ms_per_step"] is None
    assert r["config"]["refine_form"] and r["config"]["refine_kernel"]
    st = [np.load(dump / f"states_rank{k}.npy") for k in range(2)]
    assert st[0].shape == (4, 27)
    np.testing.assert_array_equal(st[0], st[1])  # every rank adopts the same winner
    raw0, x0 = np.load(dump / "raw0.npy"), np.load(dump / "x0.npy")
    obs = oracle.preprocess(raw0)
    ub, lb, sd = oracle_np.reference_bounds()
    res = []
    for rank in range(2):
        xr, _ = oracle.refine(ora_hand, obs, x0, rigid=REFINE_RIGID)
        xr, _, _ = oracle.pso_evolve(ora_hand, obs, xr, 1024, 31, lb, ub, sd, seed=1000 + rank)
        res.append((oracle.cal_cost(ora_hand, obs, xr), rank, xr))
    assert res[0][0] != res[1][0]
    cbest, _, xbest = min(res, key=lambda e: (e[0], e[1]))
    np.testing.assert_allclose(st[0][0, :26], xbest, rtol=0, atol=1e-6)
    assert abs(st[0][0, 26] - cbest) <= 1e-8 * abs(cbest)


def test_bench_two_ranks_generation_exchange(tmp_path, oracle, ora_hand):
    """The opt-in ICP-PSO style exchange (--exchange gen:10, hpe_set_exchange; NOT the
    reference algorithm): every 10 generations the two ranks' best pbest is all-gathered
    and the best injected as an extra informant.  Frame 0 against the oracle's lockstep
    mirror of the two subswarms (ora_pso_evolve_xch), then the per-frame best-of-2."""
    dump = tmp_path / "dump"
    r = _bench_ranks(dump, "--exchange", "gen:10")
    assert "every 10 generations" in r["config"]["exchange"]
    st = [np.load(dump / f"states_rank{k}.npy") for k in range(2)]
    np.testing.assert_array_equal(st[0], st[1])
    raw0, x0 = np.load(dump / "raw0.npy"), np.load(dump / "x0.npy")
    obs = oracle.preprocess(raw0)
    ub, lb, sd = oracle_np.reference_bounds()
    xr, _ = oracle.refine(ora_hand, obs, x0, rigid=REFINE_RIGID)
    bp, bc = oracle.pso_evolve_xch(ora_hand, obs, xr, 1024, 31, lb, ub, sd, [1000, 1001], 10)
    ind, _ = oracle.pso_evolve_xch(ora_hand, obs, xr, 1024, 31, lb, ub, sd, [1000, 1001], 0)
    assert not np.array_equal(bp, ind)  # the exchange changed the swarms
    k = int(np.argmin(bc))
    np.testing.assert_allclose(st[0][0, :26], bp[k], rtol=0, atol=1e-6)
    assert abs(st[0][0, 26] - bc[k]) <= 1e-8 * abs(bc[k])
