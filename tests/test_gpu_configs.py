"""GPU parity at the BASELINE.json workloads (the configs bench.py times), against the C
oracle on the same frames, seeds and x0.

  config 1  hpe_track (the C++ test_full driver) at 32 particles x maxiter 11, 10 frames
  config 2  one frame, 256 particles x maxiter 31 (30 generations), N = 250 and N = full,
            through pso_evolve (traces compared) and through the tracked frame
  config 3  the 400-frame sequence, 256 x 31, refine on, temporal prior, through the
            pipelined loop bench.py runs (hpe_track_pipelined, raw depth in)
  config 4  one frame, 4096 particles x maxiter 41 in the auto (wave) form; and 4096 x
            maxiter 6 at N = full (the multi-item search with the point prefetch)
  config 3  also 20 frames at N = full (the multi-workgroup refine + fused preparation)
  config 5  every rank's subswarm (1024 x maxiter 31, seed 1000 + r, r = 0..7) on this GPU,
            and the best-of-8 pick over them

Tolerances (as test_gpu_parity.py): pose |diff| <= 1e-6, cost relative 1e-8, gbest /
stagnation-count / topology traces exact (gbest relative 1e-8).  Reference:
testmodel.cpp:104-139, PSO.cpp:717-886 (informant topology :790-812).
"""
import numpy as np
import pytest

import hand_data
from hand_data import REFINE_RIGID
import oracle_np

pytestmark = pytest.mark.gpu

POSE_TOL, COST_RTOL = 1e-6, 1e-8
# long sequences (test_config3), tightened to the measured values (VERDICT r5 item 2;
# DESIGN.md §2 has the bounds and the measurements side by side).  Round 5, 400 frames:
# pose 2.19e-7, cost 3.1e-8, drift 2.8e-7, 6-7 mismatched frames of at most 2 flips each;
# 20 full-cloud frames: pose 5.3e-9
SEQ_POSE_TOL, SEQ_COST_RTOL = 5e-7, 5e-8
SEQ_DRIFT_TOL = 1e-6       # the free-running oracle's largest distance from the GPU trajectory
SEQ_MAX_MISMATCH = 12      # refine eval-count mismatches over the 400 frames
SEQ_MAX_FLIPS = 2          # near-tie decisions one mismatched frame may need inverted
FULL_SEQ_POSE_TOL = 1e-7   # the 20 full-cloud frames
# A refine whose evaluation count differs from the oracle's must have flipped a near-tie:
# the oracle's own run from the same x0 took some decision (Goldstein test, PSO.cpp:459-474,
# or the loop's tol > eps, :234) with a relative margin below this (a typical frame's
# smallest margin is ~1e-5; the fp64 sums' order alone moves a cost by ~1e-16 relative;
# measured: the 9 mismatched frames of the 400-frame sequence at 1.6e-16 .. 2.4e-15)
TIE_MARGIN = 1e-13


def _gpu_refine(gh, raw, x0, downsample=True):
    """The GPU's refine_init_pose of one raw frame from x0 (the same kernel and operations as
    inside the tracking loop): (refined pose, evaluation count)."""
    import hpe
    om = hpe.observedmodel()
    om.downsample = downsample
    om.set_depth_mm(raw)
    cf = hpe.costfunc(gh, om)
    x = np.array(x0, dtype=np.float64)
    pso = hpe.PSO()
    pso.refine_init_pose(x, cf)
    return x, pso.last_refine_evals


def _tie_replay(oracle, ora_hand, obs, x0, gpu_evals, gh=None, raw=None, rigid=REFINE_RIGID,
                downsample=True):
    """A refine whose evaluation count differs from the oracle's must be the oracle's own
    run with near-tie decisions (margin < TIE_MARGIN) inverted: hand_data.tie_replay
    replays one, then two, flipped ties and returns the flips whose replay takes exactly
    the GPU's evaluation count AND reaches the GPU's refined pose within 1e-6 (the GPU's
    refine of the same frame from the same x0, when gh / raw are given); None: no near-tie
    explains it.  rigid=False replays the reference's operation order (the chain)."""
    pose = None
    if gh is not None:
        pose, ev = _gpu_refine(gh, raw, x0, downsample)
        assert ev == gpu_evals, (ev, gpu_evals)  # the loop's refine, reproduced
    return hand_data.tie_replay(oracle, ora_hand, obs, x0, gpu_evals, rigid, TIE_MARGIN, pose=pose)


@pytest.fixture(scope="module")
def gh():
    import hpe
    return hpe.reference_hand(device=0)


def _cost_eq(a, b, rtol=COST_RTOL):
    """Relative rtol; an empty frame's NaN (lambda = 48/0, costfunc.cpp:372) must be NaN
    on both sides."""
    if np.isnan(b):
        return bool(np.isnan(a))
    return abs(a - b) <= rtol * abs(b)


def _pso(maxiter):
    import hpe
    ub, lb, sd = oracle_np.reference_bounds()
    p = hpe.PSO()
    p.set_pso_params(ub, lb, sd, 0.7298, 1.49618, 1.49618, maxiter, 1e-8, 1e-8)
    return p


def _costfunc(gh, depth, downsample):
    import hpe
    om = hpe.observedmodel()
    om.downsample = downsample
    om.set_depth_mm(depth)
    return hpe.costfunc(gh, om)


def _check_pso(pso, cf, bestp, rb, rc, tr):
    np.testing.assert_allclose(bestp, rb, rtol=0, atol=POSE_TOL)
    assert abs(pso.last_gbest_cost - rc) <= COST_RTOL * abs(rc)
    g, cnt, topo = pso.trace(cf)
    np.testing.assert_allclose(g, tr["gbest"], rtol=COST_RTOL)
    assert np.array_equal(cnt, tr["count"])
    assert np.array_equal(topo, tr["topo"])


@pytest.mark.parametrize("downsample", [True, False])
def test_config2_single_frame_256x30(oracle, ora_hand, gh, downsample):
    """BASELINE config 2: 256 particles x 30 generations on one frame."""
    P, maxiter = 256, 31
    poses = hand_data.trajectory(4, seed=2)
    depth = gh.ctx.render_depth(poses[3])
    obs = oracle.preprocess(depth, downsample=downsample)
    assert (obs.n == 250) == downsample and (downsample or obs.n > 2048)
    cf = _costfunc(gh, depth, downsample)
    ub, lb, sd = oracle_np.reference_bounds()
    x0 = poses[2].copy()
    pso = _pso(maxiter)
    bestp = np.zeros(26)
    assert pso.pso_evolve(cf, x0, P, bestp) == 1
    rb, rc, tr = oracle.pso_evolve(ora_hand, obs, x0, P, maxiter, lb, ub, sd, seed=1000)
    _check_pso(pso, cf, bestp, rb, rc, tr)
    # the same frame as a tracked frame: refine, pso_evolve, cal_cost(bestp)
    x = x0.copy()
    c = pso.track_frame(cf, x, P, refine=True)
    xr, _ = oracle.refine(ora_hand, obs, x0, rigid=REFINE_RIGID)
    xr, _, _ = oracle.pso_evolve(ora_hand, obs, xr, P, maxiter, lb, ub, sd, seed=1000)
    cr = oracle.cal_cost(ora_hand, obs, xr)
    np.testing.assert_allclose(x, xr, rtol=0, atol=POSE_TOL)
    assert abs(c - cr) <= COST_RTOL * abs(cr)


def test_config4_large_swarm_4096x40(oracle, ora_hand, gh):
    """BASELINE config 4: 4096 particles x 40 generations (auto form = one wave per
    particle; informant in-degree and inbox sizes at their largest)."""
    P, maxiter = 4096, 41
    poses = hand_data.trajectory(3, seed=44)
    depth = gh.ctx.render_depth(poses[2])
    obs = oracle.preprocess(depth)
    cf = _costfunc(gh, depth, True)
    ub, lb, sd = oracle_np.reference_bounds()
    pso = _pso(maxiter)
    bestp = np.zeros(26)
    assert pso.pso_evolve(cf, poses[1], P, bestp) == 1
    rb, rc, tr = oracle.pso_evolve(ora_hand, obs, poses[1], P, maxiter, lb, ub, sd, seed=1000)
    _check_pso(pso, cf, bestp, rb, rc, tr)
    assert tr["count"].max() >= 0 and len(tr["topo"]) == 40


def test_config4_large_swarm_full_cloud(oracle, ora_hand, gh):
    """Config 4's swarm at N = full: 4096 particles (wave form) x maxiter 6 on a full cloud
    (> 2048 points: every lane searches several points, the next point loaded one item
    ahead, hpe_device.hpp search_align).  BASELINE.md §2: each config at N = 250 and full."""
    P, maxiter = 4096, 6
    poses = hand_data.trajectory(3, seed=45)
    depth = gh.ctx.render_depth(poses[2])
    obs = oracle.preprocess(depth, downsample=False)
    assert obs.n > 2048
    cf = _costfunc(gh, depth, False)
    ub, lb, sd = oracle_np.reference_bounds()
    pso = _pso(maxiter)
    bestp = np.zeros(26)
    assert pso.pso_evolve(cf, poses[1], P, bestp) == 1
    rb, rc, tr = oracle.pso_evolve(ora_hand, obs, poses[1], P, maxiter, lb, ub, sd, seed=1000)
    _check_pso(pso, cf, bestp, rb, rc, tr)


def test_config5_subswarm_ranks_1024x30(oracle, ora_hand, gh):
    """BASELINE config 5, one rank at a time on this GPU: rank r's subswarm is 1024
    particles x maxiter 31 in the auto (wave, P >= 1024) form with Philox seed 1000 + r
    (hpe.dist.subswarm_seed; the reference reseeds every call, PSO.cpp:717-722), each
    against oracle.pso_evolve(seed=1000 + r) with traces; then hpe.dist.pick_best (the
    per-frame exchange's choice) over the 8 GPU states picks the same rank
    and state as over the 8 oracle states."""
    import torch
    from hpe.dist import pick_best, subswarm_seed
    P, maxiter, world = 1024, 31, 8
    poses = hand_data.trajectory(3, seed=51)
    depth = gh.ctx.render_depth(poses[2])
    obs = oracle.preprocess(depth)
    cf = _costfunc(gh, depth, True)
    ub, lb, sd = oracle_np.reference_bounds()
    pso = _pso(maxiter)
    hip_states, ora_states = [], []
    for r in range(world):
        pso.seed = subswarm_seed(r)
        bestp = np.zeros(26)
        assert pso.pso_evolve(cf, poses[1], P, bestp) == 1
        rb, rc, tr = oracle.pso_evolve(ora_hand, obs, poses[1], P, maxiter, lb, ub, sd,
                                       seed=subswarm_seed(r))
        _check_pso(pso, cf, bestp, rb, rc, tr)
        hip_states.append(np.concatenate([bestp, [pso.last_gbest_cost]]))
        ora_states.append(np.concatenate([rb, [rc]]))
    hip_states, ora_states = np.array(hip_states), np.array(ora_states)
    assert len(set(ora_states[:, 26])) == world  # 8 distinct streams
    hb = pick_best(torch.from_numpy(hip_states)).numpy()
    ob = pick_best(torch.from_numpy(ora_states)).numpy()
    assert int(np.argmin(hip_states[:, 26])) == int(np.argmin(ora_states[:, 26]))
    np.testing.assert_allclose(hb[:26], ob[:26], rtol=0, atol=POSE_TOL)
    assert _cost_eq(hb[26], ob[26])


def _track_pipelined(gh, raw, P, maxiter, x0, downsample):
    """hpe_track_pipelined over the raw frames (bench.py's loop): per-frame pose, cost and
    the running refine evaluation count."""
    import ctypes as C
    import torch
    n = len(raw)
    ctx, lib = gh.ctx, gh.ctx.lib
    _pso(maxiter)._push(ctx)
    state = torch.zeros(27, dtype=torch.float64, device="cuda:0")
    state[:26] = torch.from_numpy(np.array(x0, dtype=np.float64))
    torch.cuda.synchronize()
    ctx.pipeline_begin(raw[0], True, downsample)
    gx, gc, gev = [], [], []
    tot = C.c_uint64(0)
    ctx.check(lib.hpe_refine_eval_count(ctx.h, C.byref(tot), 1))
    for f in range(n):
        ctx.track_pipelined(P, 1, state.data_ptr(), raw[f + 1] if f + 1 < n else None)
        ctx.check(lib.hpe_sync(ctx.h))
        torch.cuda.synchronize()
        s = state.cpu().numpy()
        gx.append(s[:26].copy())
        gc.append(s[26])
        ctx.check(lib.hpe_refine_eval_count(ctx.h, C.byref(tot), 1))
        gev.append(tot.value)
    gh.ctx.frame_token = None  # the pipeline owned the selected frame
    return np.array(gx), np.array(gc), gev


def test_config3_full_cloud_20_frames_pipelined(oracle, ora_hand, gh):
    """Config 3's loop at N = full: 20 tracked frames, 256 x 30, refine on, through the
    pipelined loop.  Full clouds (> 2048 points) take the multi-workgroup refine (64 helper
    workgroups own cloud slices) with the next frame's preparation workgroups in the same
    launch (testmodel.cpp:64 downsample = false; observedmodel.cpp:204-217 skipped).  Every
    frame against the oracle started from the GPU's previous pose, SEQ_* tolerances."""
    n, P, maxiter = 20, 256, 31
    poses = hand_data.trajectory(n, seed=8, revert=0.02)
    raw = [np.ascontiguousarray(gh.ctx.render_depth(th)) for th in poses]
    gx, gc, gev = _track_pipelined(gh, raw, P, maxiter, poses[0], False)
    ub, lb, sd = oracle_np.reference_bounds()
    dpose, ev_mismatch, margin = [], [], []
    for f in range(n):
        obs = oracle.preprocess(raw[f], downsample=False)
        assert obs.n > 2048
        x0 = poses[0] if f == 0 else gx[f - 1]
        xr, er = oracle.refine(ora_hand, obs, x0, rigid=REFINE_RIGID)
        margin.append(oracle.refine_last_margin())
        xr, _, _ = oracle.pso_evolve(ora_hand, obs, xr, P, maxiter, lb, ub, sd, seed=1000)
        cr = oracle.cal_cost(ora_hand, obs, xr)
        dpose.append(np.abs(gx[f] - xr).max())
        assert _cost_eq(gc[f], cr, SEQ_COST_RTOL), (f, gc[f], cr)
        if gev[f] != er:
            ev_mismatch.append((f, _tie_replay(oracle, ora_hand, obs, x0, gev[f], gh, raw[f],
                                               downsample=False)))
    dpose, margin = np.array(dpose), np.array(margin)
    print(f"{n} full-cloud frames: max |dpose| {dpose.max():.3g} (frame {int(dpose.argmax())}), "
          f"refine eval-count mismatches (frame, flipped tie's margin) {ev_mismatch}; frames "
          f"with a margin < {TIE_MARGIN:g}: {int((margin < TIE_MARGIN).sum())}")
    assert dpose.max() <= FULL_SEQ_POSE_TOL, f"frame {int(dpose.argmax())}: pose {dpose.max()}"
    assert len(ev_mismatch) <= 1
    assert all(m is not None for _, m in ev_mismatch), "an eval-count mismatch no near-tie explains"
    assert all(len(m) <= SEQ_MAX_FLIPS for _, m in ev_mismatch)


@pytest.fixture(scope="module")
def seq400(gh):
    """BASELINE config 3 on the GPU: 400 tracked frames, 256 x 30, refine on, x0 <- previous
    bestp (testmodel.cpp:117-139), through the pipelined loop of bench.py (raw float32 mm
    depth in, preprocessing on the GPU inside the previous frame's refine launch)."""
    n, P, maxiter = 400, 256, 31
    poses = hand_data.trajectory(n, seed=7, revert=0.02)  # stays in view
    raw = [np.ascontiguousarray(gh.ctx.render_depth(th)) for th in poses]
    gx, gc, gev = _track_pipelined(gh, raw, P, maxiter, poses[0], True)
    return dict(n=n, P=P, maxiter=maxiter, poses=poses, raw=raw, gx=gx, gc=gc, gev=gev)


def _seq400_check(oracle, ora_hand, gh, s, rigid):
    """Every frame against the oracle (rigid: the mirror of the GPU's hand-frame refine;
    not rigid: the reference's own operation order, the DH chain on every evaluation)
    started from the GPU's previous pose, and the oracle running free over the sequence."""
    n, P, maxiter, poses, raw, gx, gc, gev = (s[k] for k in ("n", "P", "maxiter", "poses", "raw",
                                                            "gx", "gc", "gev"))
    ub, lb, sd = oracle_np.reference_bounds()
    free = poses[0].copy()
    dpose, dcost, drift, ev_mismatch, margin = [], [], [], [], []
    for f in range(n):
        obs = oracle.preprocess(raw[f])
        x0 = poses[0] if f == 0 else gx[f - 1]
        xr, er = oracle.refine(ora_hand, obs, x0, rigid=rigid)
        margin.append(oracle.refine_last_margin())
        xr, _, _ = oracle.pso_evolve(ora_hand, obs, xr, P, maxiter, lb, ub, sd, seed=1000)
        cr = oracle.cal_cost(ora_hand, obs, xr)
        dpose.append(np.abs(gx[f] - xr).max())
        dcost.append(0.0 if _cost_eq(gc[f], cr, SEQ_COST_RTOL) and np.isnan(cr)
                     else abs(gc[f] - cr) / abs(cr))
        if gev[f] != er:
            ev_mismatch.append((f, _tie_replay(oracle, ora_hand, obs, x0, gev[f], gh, raw[f], rigid)))
        free, _ = oracle.refine(ora_hand, obs, free, rigid=rigid)
        free, _, _ = oracle.pso_evolve(ora_hand, obs, free, P, maxiter, lb, ub, sd, seed=1000)
        drift.append(np.abs(free - gx[f]).max())
    dpose, dcost, drift, margin = np.array(dpose), np.array(dcost), np.array(drift), np.array(margin)
    first = lambda a, t: (int(np.nonzero(a > t)[0][0]) if (a > t).any() else None)  # noqa: E731
    flips = max((len(m) for _, m in ev_mismatch if m is not None), default=0)
    print(f"400 frames vs the oracle's {'hand-frame mirror' if rigid else 'reference order (chain)'}: "
          f"per-frame max |dpose| {dpose.max():.3g} (frame {int(dpose.argmax())}), max dcost "
          f"{np.nanmax(dcost):.3g}, refine eval-count mismatches {len(ev_mismatch)}, most flips a "
          f"frame needed {flips}; free-running oracle: max drift {drift.max():.3g}, first frame "
          f"beyond {SEQ_DRIFT_TOL:g}: {first(drift, SEQ_DRIFT_TOL)}; mismatched frames (frame, flipped "
          f"ties (decision, margin)) {ev_mismatch}; frames with a margin < {TIE_MARGIN:g}: "
          f"{int((margin < TIE_MARGIN).sum())}, median margin {np.median(margin):.3g}")
    assert dpose.max() <= SEQ_POSE_TOL, f"frame {int(dpose.argmax())}: pose {dpose.max()}"
    assert np.all(dcost <= SEQ_COST_RTOL), f"frame {int(np.nanargmax(dcost))}: cost {dcost.max()}"
    assert len(ev_mismatch) <= SEQ_MAX_MISMATCH, f"{len(ev_mismatch)} mismatched frames"
    assert all(m is not None for _, m in ev_mismatch), "an eval-count mismatch no near-tie explains"
    assert flips <= SEQ_MAX_FLIPS, f"a mismatched frame needed {flips} flipped ties"
    assert drift.max() <= SEQ_DRIFT_TOL, f"free-running divergence from frame {first(drift, SEQ_DRIFT_TOL)}"


def test_config3_sequence_400_frames_pipelined(oracle, ora_hand, gh, seq400):
    """BASELINE config 3 (seq400) against the oracle's mirror of the GPU's refine form.

    Checked two ways: (1) every frame against the oracle started from the GPU's previous
    pose (per-frame parity, no accumulated history); (2) the oracle running free over the
    whole sequence, whose largest distance from the GPU trajectory is reported.

    Sequence tolerances (SEQ_*, at about 2x the round-5 measurements): per-frame pose 5e-7,
    cost relative 5e-8, free-running drift 1e-6, at most 12 eval-count mismatches of at
    most 2 flipped ties each.  The fp64 sums differ in order (DPP tree vs Armadillo's two
    accumulators, ~1e-16 relative), and refine's Goldstein comparisons (PSO.cpp:459-474)
    sit at that rounding floor once alpha * g'p is ~1e-13: on ~2 % of frames a decision
    flips, the refine takes a few evaluations more or fewer and the pose moves by up to
    ~2e-7 (round 5: 7 of 400 frames, max 1.73e-7; free-running drift 2.6e-7, DESIGN.md
    §2).  Each such frame must
    be the oracle's refine from the same x0 with one or two near-tie decisions (relative
    margin below TIE_MARGIN) inverted: replaying the oracle with them flipped takes exactly
    the GPU's evaluation count and reaches the GPU's refined pose (_tie_replay).  Single
    calls keep the exact eval count (test_gpu_parity.py)."""
    _seq400_check(oracle, ora_hand, gh, seq400, REFINE_RIGID)


def test_config3_sequence_400_frames_vs_reference_order(oracle, ora_hand, gh, seq400):
    """the same 400 GPU frames against the reference's own operation
    order -- the oracle's restatement of refine_init_pose with the DH chain on every
    evaluation (fingermodel.cpp:287-311 via handmodel.cpp:259-298, PSO.cpp:216-266) -- per
    frame and free-running, with the same tolerances.  An eval-count mismatch must be a
    replay of the chain refine with near-ties flipped that reaches the GPU's refined pose."""
    _seq400_check(oracle, ora_hand, gh, seq400, False)


def test_config1_hpe_track_32x10(tmp_path, oracle, ora_hand, np_hand):
    """BASELINE config 1's shape (32 particles x maxiter 11) through the C++ test_full
    driver over 10 .bin frames, against the oracle loop."""
    from test_gpu_facade import _run_track, _write_inputs
    n, P, maxiter = 10, 32, 11
    poses = hand_data.trajectory(n, seed=13)
    hand, frames, depth = _write_inputs(tmp_path, np_hand, poses)
    ub, lb, sd = oracle_np.reference_bounds()
    x = oracle_np.X0.copy()
    ref_c, ref_x = [], []
    for f in range(n):
        obs = oracle.preprocess(depth[f])
        x, _ = oracle.refine(ora_hand, obs, x, rigid=REFINE_RIGID)
        x, _, _ = oracle.pso_evolve(ora_hand, obs, x, P, maxiter, lb, ub, sd)
        ref_c.append(oracle.cal_cost(ora_hand, obs, x))
        ref_x.append(x.copy())
    c, xs = _run_track(hand, frames, n, P, maxiter, 1, tmp_path / "poses.txt")
    np.testing.assert_allclose(xs, np.array(ref_x), rtol=0, atol=POSE_TOL)
    np.testing.assert_allclose(c, np.array(ref_c), rtol=COST_RTOL, atol=0)
