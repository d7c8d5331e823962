"""RCCL on the box: the multi-GPU exchange's collective (hpe.dist.exchange_best's
all_gather_into_tensor) through torch.distributed's "nccl" backend (= RCCL on ROCm).  Only
one GPU is available to the tests, and RCCL refuses two ranks on one device, so this runs
a one-rank process group: it initialises an RCCL communicator on the device, tracks one
frame with the HIP library, and all-gathers the tracker state on the tracker's own stream
(as bench.py does per frame) -- the library, the communicator and the stream ordering are
exercised on hardware; the N-rank logic itself is covered by the gloo tests."""
import os
import subprocess
import sys

import pytest

import hand_data

pytestmark = pytest.mark.gpu

SCRIPT = r'''
import os, socket, sys
import numpy as np
import torch
import torch.distributed as dist
sys.path.insert(0, os.path.join(os.environ["HPE_ROOT"], "hand-pose-estimation_amd"))
import hpe
from hpe import synth
torch.cuda.set_device(0)
with socket.socket() as s:
    s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]
dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                        device_id=torch.device("cuda", 0))
hand = hpe.reference_hand(device=0)
ctx = hand.ctx
ub, lb, sd = hpe.reference_bounds()
pso = hpe.PSO()
pso.set_pso_params(ub, lb, sd, 0.7298, 1.49618, 1.49618, 6, 1e-8, 1e-8)
pso._push(ctx)
poses = synth.trajectory(2, 0, revert=0.02)
raw = [np.ascontiguousarray(ctx.render_depth(th)) for th in poses]
state = torch.zeros(27, dtype=torch.float64, device="cuda:0")
state[:26] = torch.from_numpy(poses[0])
torch.cuda.synchronize()
ctx.pipeline_begin(raw[0])
ctx.track_pipelined(64, 1, state.data_ptr(), raw[1])
ext = torch.cuda.ExternalStream(ctx.lib.hpe_stream(ctx.h), device="cuda:0")
gathered = torch.zeros(27, dtype=torch.float64, device="cuda:0")
with torch.cuda.stream(ext):
    dist.all_gather_into_tensor(gathered, state)
ctx.check(ctx.lib.hpe_sync(ctx.h))
torch.cuda.synchronize()
s, g = state.cpu().numpy(), gathered.cpu().numpy()
assert np.isfinite(s).all() and np.array_equal(s, g), (s, g)
v = torch.cuda.nccl.version()
print("RCCL", ".".join(map(str, v)) if isinstance(v, tuple) else v, "backend", dist.get_backend(),
      "cost", s[26])
hand.ctx.close()
dist.destroy_process_group()
'''


def test_rccl_one_rank_allgather_on_tracker_stream(tmp_path):
    env = dict(os.environ, HPE_ROOT=str(hand_data.ROOT))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    f = tmp_path / "rccl1.py"
    f.write_text(SCRIPT)
    out = subprocess.run([sys.executable, str(f)], capture_output=True, text=True, timeout=240,
                         env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    assert "RCCL" in out.stdout and "backend nccl" in out.stdout, out.stdout
    print(out.stdout.strip())


SCRIPT_LIB = r'''
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.environ["HPE_ROOT"], "hand-pose-estimation_amd"))
import hpe
from hpe import synth
from hpe.dist import library_exchange
torch.cuda.set_device(0)
hand = hpe.reference_hand(device=0)
ctx = hand.ctx
ub, lb, sd = hpe.reference_bounds()
pso = hpe.PSO()
P, n = 256, 16
pso.set_pso_params(ub, lb, sd, 0.7298, 1.49618, 1.49618, 31, 1e-8, 1e-8)
pso._push(ctx)
poses = synth.trajectory(n + 1, 0, revert=0.02)
raw = np.stack([np.ascontiguousarray(ctx.render_depth(th)) for th in poses]).astype(np.float32)
d_raw = torch.from_numpy(raw).to("cuda:0")

def run(fpg):
    state = torch.zeros(27, dtype=torch.float64, device="cuda:0")
    state[:26] = torch.from_numpy(poses[0])
    hist = torch.zeros(n * 27, dtype=torch.float64, device="cuda:0")
    torch.cuda.synchronize()
    ctx.track_raw_sequence(P, 1, state.data_ptr(), d_raw.data_ptr(), n, True, True,
                           frames_per_graph=fpg, d_hist_ptr=hist.data_ptr())
    ctx.check(ctx.lib.hpe_sync(ctx.h))
    return state.cpu().numpy(), hist.cpu().numpy().reshape(n, 27)

def pipelined():
    state = torch.zeros(27, dtype=torch.float64, device="cuda:0")
    state[:26] = torch.from_numpy(poses[0])
    torch.cuda.synchronize()
    ctx.pipeline_begin(raw[0])
    out = []
    for f in range(4):
        ctx.track_pipelined(P, 1, state.data_ptr(), raw[f + 1])
        ctx.check(ctx.lib.hpe_sync(ctx.h))
        out.append(state.cpu().numpy())
    return np.array(out)

def seq(fpg):  # the offline sequence API over device-prepared slots
    state = torch.zeros(27, dtype=torch.float64, device="cuda:0")
    state[:26] = torch.from_numpy(poses[0])
    hist = torch.zeros(n * 27, dtype=torch.float64, device="cuda:0")
    torch.cuda.synchronize()
    ctx.track_sequence(P, 1, state.data_ptr(), 0, n, fpg, hist.data_ptr())
    ctx.check(ctx.lib.hpe_sync(ctx.h))
    return state.cpu().numpy(), hist.cpu().numpy().reshape(n, 27)

for f in range(n):
    ctx.prepare_frame(f, raw[f])
ctx.check(ctx.lib.hpe_sync(ctx.h))
plain, plain_h = run(8)
plain_p = pipelined()
plain_s, plain_sh = seq(8)
info = library_exchange(ctx)  # world 1: no process group, the library's own communicator
assert info["nranks"] == 1 and info["rank"] == 0 and info["rccl_version"] > 0, info
g0 = ctx.subswarm_info(gathered=True)["gathered"]
assert np.isnan(g0).all()  # nothing exchanged yet
c0 = ctx.graph_captures()
a, a_h = run(8)           # captures the chunk graphs WITH the exchange (epoch bumped)
c1 = ctx.graph_captures()
b, b_h = run(8)           # replays them
c2 = ctx.graph_captures()
assert c1 > c0 and c2 == c1, (c0, c1, c2)
assert np.array_equal(a, plain) and np.array_equal(b, plain), (a - plain)
assert np.array_equal(a_h, plain_h) and np.array_equal(b_h, plain_h)
g = ctx.subswarm_info(gathered=True)["gathered"]
assert np.array_equal(g[0], plain), (g[0], plain)  # this rank's row: the last frame's result
# one graph per frame (frames_per_graph 1) and the per-frame pipelined form, with the exchange
c, c_h = run(1)
assert np.array_equal(c, plain) and np.array_equal(c_h, plain_h)
for fpg in (8, 3):
    e, e_h = seq(fpg)
    assert np.array_equal(e, plain_s) and np.array_equal(e_h, plain_sh), fpg
assert np.array_equal(pipelined(), plain_p)
# direct launches (profiling): one exchange event pair per frame
ctx.check(ctx.lib.hpe_profile_enable(ctx.h, 1))
assert np.array_equal(pipelined(), plain_p)
import ctypes as Cc
nl = Cc.c_int32(0); tot = Cc.c_double(0); mn = Cc.c_double(0); mx = Cc.c_double(0)
ctx.check(ctx.lib.hpe_profile_read_kernel(ctx.h, hpe._lib.PROF_EXCHANGE, Cc.byref(nl), Cc.byref(tot),
                                          Cc.byref(mn), Cc.byref(mx)))
ctx.check(ctx.lib.hpe_profile_enable(ctx.h, 0))
assert nl.value == 4, nl.value
# the fallback form (exchange on, direct launches): the same bits, nothing captured
assert ctx.subswarm_info()["in_graphs"]
ctx.subswarm_enable(True, direct=True)
assert not ctx.subswarm_info()["in_graphs"]
c3 = ctx.graph_captures()
f, f_h = run(8)
assert np.array_equal(f, plain) and np.array_equal(f_h, plain_h)
assert ctx.graph_captures() == c3
ctx.subswarm_enable(True)
assert ctx.subswarm_info()["in_graphs"]
# suspended: the plain loop again, bit for bit
ctx.subswarm_enable(False)
d, d_h = run(8)
assert np.array_equal(d, plain) and np.array_equal(d_h, plain_h)
ctx.subswarm_enable(True)
ctx.subswarm_fini()
assert ctx.subswarm_info()["nranks"] == 0
print("LIBRCCL", info["rccl_version"], "captures", c0, c1, c2, "exchange_us",
      tot.value / max(nl.value, 1) * 1e3, "cost", plain[26])
hand.ctx.close()
'''


def test_library_exchange_captured_world1(tmp_path):
    """the library's own subswarm exchange (hpe_subswarm_init: an RCCL
    communicator in libhpe.so; after every tracked frame an all-gather of {bestp, cost} and the
    pick) captured INTO the raw-sequence chunk graphs, on a one-rank communicator (RCCL refuses
    two ranks on one GPU).  The captured form must give per-frame {bestp, cost} (the history
    rows) and the final state bit-identical to the plain N = 1 run; the replay captures
    nothing; the frame results went through the gather buffer (this rank's row is the last
    frame's state, NaN before; the all-gather is in place, so at one rank RCCL moves nothing);
    one graph per frame (every pick a k_pick_best launch) and the per-frame pipelined form
    agree too; direct launches time one exchange per frame; the fallback form (exchange on,
    no graphs: hpe_subswarm_enable 2) gives the same bits; suspending the exchange gives the
    plain loop again."""
    env = dict(os.environ, HPE_ROOT=str(hand_data.ROOT))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    f = tmp_path / "librccl1.py"
    f.write_text(SCRIPT_LIB)
    out = subprocess.run([sys.executable, str(f)], capture_output=True, text=True, timeout=240,
                         env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    assert "LIBRCCL" in out.stdout, out.stdout
    print(out.stdout.strip())


SCRIPT_LIB_WAVE = r'''
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.environ["HPE_ROOT"], "hand-pose-estimation_amd"))
import hpe
from hpe import synth
from hpe.dist import library_exchange
torch.cuda.set_device(0)
hand = hpe.reference_hand(device=0)
ctx = hand.ctx
ub, lb, sd = hpe.reference_bounds()
pso = hpe.PSO()
P, n = 1024, 5                       # config 5's per-rank swarm: the wave form, 2 waves/particle
pso.set_pso_params(ub, lb, sd, 0.7298, 1.49618, 1.49618, 11, 1e-8, 1e-8)
pso.seed = 1003                      # rank 3's stream
pso._push(ctx)
poses = synth.trajectory(n + 1, 4, revert=0.02)
raw = np.stack([np.ascontiguousarray(ctx.render_depth(th)) for th in poses]).astype(np.float32)
d_raw = torch.from_numpy(raw).to("cuda:0")

def run(fpg):
    state = torch.zeros(27, dtype=torch.float64, device="cuda:0")
    state[:26] = torch.from_numpy(poses[0])
    hist = torch.zeros(n * 27, dtype=torch.float64, device="cuda:0")
    torch.cuda.synchronize()
    ctx.track_raw_sequence(P, 1, state.data_ptr(), d_raw.data_ptr(), n, True, True,
                           frames_per_graph=fpg, d_hist_ptr=hist.data_ptr())
    ctx.check(ctx.lib.hpe_sync(ctx.h))
    return state.cpu().numpy(), hist.cpu().numpy().reshape(n, 27)

plain, plain_h = run(8)
library_exchange(ctx)
for fpg in (8, 2):
    a, a_h = run(fpg)
    assert np.array_equal(a, plain) and np.array_equal(a_h, plain_h), fpg
print("LIBRCCL_WAVE ok", plain[26])
hand.ctx.close()
'''


def test_library_exchange_captured_world1_wave_form(tmp_path):
    """The same one-rank check on config 5's per-rank loop (1024 particles: the wave form at
    two waves per particle, seed 1003), chunks of 8 and 2 frames."""
    env = dict(os.environ, HPE_ROOT=str(hand_data.ROOT))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    f = tmp_path / "librccl_wave.py"
    f.write_text(SCRIPT_LIB_WAVE)
    out = subprocess.run([sys.executable, str(f)], capture_output=True, text=True, timeout=240,
                         env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    assert "LIBRCCL_WAVE ok" in out.stdout, out.stdout


def test_pick_best_kernel_equals_torch_pick_best():
    """hpe_pick_best (the per-frame best of N in one launch, used after the RCCL all-gather)
    against hpe.dist.pick_best on the same gathered rows: random costs, equal costs (lowest
    rank wins), NaN costs (never win), +inf / -inf costs, world 1 .. 64."""
    import ctypes as C

    import numpy as np
    import torch

    import hpe
    from hpe.dist import pick_best
    hand = hpe.reference_hand(device=0)
    ctx = hand.ctx
    rng = np.random.default_rng(5)
    for world in (1, 2, 3, 8, 64):
        for case in range(6):
            g = rng.normal(size=(world, 27))
            c = rng.uniform(1, 10, size=world)
            if case == 1:
                c[:] = 4.0
            elif case == 2:
                c[rng.integers(world)] = np.nan
            elif case == 3:
                c[:] = np.nan
            elif case == 4:
                c[rng.integers(world)] = np.inf
                c[rng.integers(world)] = np.nan
            elif case == 5:
                c[rng.integers(world)] = -np.inf
            g[:, 26] = c
            gt = torch.from_numpy(g.ravel().copy()).to("cuda:0")
            st = torch.zeros(27, dtype=torch.float64, device="cuda:0")
            torch.cuda.synchronize()
            ctx.check(ctx.lib.hpe_pick_best(ctx.h, C.c_void_p(gt.data_ptr()), world,
                                            C.c_void_p(st.data_ptr())))
            ctx.check(ctx.lib.hpe_sync(ctx.h))
            want = pick_best(torch.from_numpy(g.copy())).numpy()
            got = st.cpu().numpy()
            assert np.array_equal(got, want, equal_nan=True), (world, case)
    assert ctx.lib.hpe_pick_best(ctx.h, None, 2, None) == hpe._lib.HPE_E_ARG
    gt = torch.zeros(27 * 65, dtype=torch.float64, device="cuda:0")
    assert ctx.lib.hpe_pick_best(ctx.h, C.c_void_p(gt.data_ptr()), 65,
                                 C.c_void_p(gt.data_ptr())) == hpe._lib.HPE_E_ARG
    ctx.close()
