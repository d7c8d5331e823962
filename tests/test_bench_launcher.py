"""bench.py's multi-GPU entry on the CPU: `python bench.py --gpus 2` from a plain
invocation re-launches itself under torch.distributed.run (one process per rank) and
relays rank 0's JSON line; with --stub the ranks exchange stub tracker states over gloo
through hpe.dist.exchange_best (the per-frame best-of-subswarms step, SURVEY.md §8e,
replacing the OpenMP loop of PSO.cpp:848-861 across devices)."""
import json
import os
import subprocess
import sys

import hand_data


def _bench(*args, timeout=240):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, str(hand_data.ROOT / "bench.py"), *args],
                         capture_output=True, text=True, timeout=timeout, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    return json.loads(lines[0])


def test_self_launch_two_ranks_stub():
    r = _bench("--gpus", "2", "--stub", "--steps", "3", "--warmup", "1")
    assert r["n_gpus"] == 2 and r["steps"] == 3 and r["stub"]
    # frame 3: rank 0 has cost 10 + 3 % 2 = 11, rank 1 10 + 10 % 2 = 10 -> rank 1 wins
    assert r["winner_rank"] == 1 and r["winner_cost"] == 10.0
    assert r["value"] > 0
    # the multi-rank self-verification (bench.py rank_report)
    rk = r["ranks"]
    assert rk["world_size_pg"] == 2 and rk["backend"] == "gloo"
    assert rk["devices_distinct"] and len(rk["devices"]) == 2
    assert rk["final_state_identical"]
    assert 0 < rk["ms_per_step_min"] <= rk["ms_per_step_max"]


def test_single_rank_stub():
    r = _bench("--stub", "--steps", "2", "--warmup", "0")
    assert r["n_gpus"] == 1 and r["winner_rank"] == 0


def test_frames_per_graph_defaults(monkeypatch):
    """The frame loop bench.py times: on one GPU, and with N > 1 over the library exchange
    (hpe_subswarm_init, the default with nccl: the all-gather inside the frames' graphs), the
    raw frames resident in HBM, 8 frames per graph (hpe_track_raw_sequence_dev); with the torch
    or gloo exchange, --dump or a per-generation exchange, one graph per frame (the step sits
    between frames); an explicit value wins where allowed and is refused where a step sits
    between frames."""
    import importlib
    import pytest
    sys.path.insert(0, str(hand_data.ROOT))
    bench = importlib.import_module("bench")

    def parse(*argv):
        monkeypatch.setattr(sys, "argv", ["bench.py", *argv])
        return bench.parse()

    assert parse().frames_per_graph == 8
    assert parse("--resident").frames_per_graph == 8
    assert parse("--gpus", "2").frames_per_graph == 8
    assert parse("--gpus", "2").exchange_form == "library" and parse("--gpus", "2").lib_exchange
    assert parse("--gpus", "2", "--exchange-form", "torch").frames_per_graph == 0
    assert parse("--gpus", "2", "--backend", "gloo").frames_per_graph == 0
    assert parse("--gpus", "2", "--backend", "gloo").exchange_form == "torch"
    assert parse("--subswarm-world1").frames_per_graph == 8
    assert parse("--subswarm-world1").lib_exchange and not parse().lib_exchange
    assert parse("--dump", "/tmp/x").frames_per_graph == 0
    assert parse("--exchange", "gen:5").frames_per_graph == 0
    assert parse("--frames-per-graph", "0").frames_per_graph == 0
    assert parse("--frames-per-graph", "4").frames_per_graph == 4
    for bad in (("--gpus", "2", "--exchange-form", "torch", "--frames-per-graph", "8"),
                ("--gpus", "2", "--backend", "gloo", "--exchange-form", "library"),
                ("--gpus", "2", "--subswarm-world1"),
                ("--exchange", "gen:5", "--frames-per-graph", "8")):
        with pytest.raises(SystemExit):
            parse(*bad)
