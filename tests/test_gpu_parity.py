"""GPU parity: the HIP path (through the C ABI) against the C oracle on identical inputs.

Tolerances (north_star: "within a stated float tolerance"):
  * sphere centres / joints: |diff| <= 1e-9 cm (fp64 FK; only libm vs ocml sin/cos
    rounding can differ)
  * correspondences: identical, except a point whose two nearest float distances lie
    within 1 ulp of each other (FK rounding may move a float centre by 1 ulp); such
    points must still be matched to an equidistant sphere (tie-aware comparator)
  * costs: relative 1e-9 (fp64 accumulation order differs: tree vs Armadillo's
    2-accumulator sum)
  * PSO / refine / tracking: bestp |diff| <= 1e-6, cost relative 1e-8
"""
import numpy as np
import pytest

import hand_data
from hand_data import REFINE_RIGID
import oracle_np

pytestmark = pytest.mark.gpu

RTOL = 1e-9


@pytest.fixture(scope="module")
def hpe_mod():
    import hpe
    return hpe


@pytest.fixture(scope="module")
def gpu_hand(hpe_mod):
    return hpe_mod.reference_hand(device=0)


def _frame(np_hand, theta, downsample=True):
    return oracle_np.render_depth_mm(np_hand, theta)


def _obs_pair(oracle, gpu_hand, depth_mm, downsample=True):
    import hpe
    obs = oracle.preprocess(depth_mm, downsample=downsample)
    om = hpe.observedmodel()
    om.to_cm, om.downsample, om.focal_len = True, downsample, 241.42
    om.set_depth_mm(depth_mm)
    return obs, om


class _refine_form:
    """Run a test body with the context's refine in one form (hpe_set_refine_exact), the
    oracle mode to compare with as the value: rigid (the hand-frame mirror) unless exact."""

    def __init__(self, ctx, exact):
        self.ctx, self.exact = ctx, exact

    def __enter__(self):
        self.prev = self.ctx.refine_exact
        self.ctx.refine_exact = self.exact
        return not self.exact

    def __exit__(self, *exc):
        self.ctx.refine_exact = self.prev


def _match_equiv(obs, S, m_gpu, m_ref):
    """Tie-aware: a differing match must be (float-)equidistant to the reference one."""
    diff = np.nonzero(m_gpu != m_ref)[0]
    if len(diff) == 0:
        return True
    q = obs.cloud[diff].astype(np.float32)
    s = S.astype(np.float32)
    d_g = np.linalg.norm(q - s[m_gpu[diff]], axis=1)
    d_r = np.linalg.norm(q - s[m_ref[diff]], axis=1)
    return bool(np.all(np.abs(d_g - d_r) <= 4 * np.spacing(np.maximum(d_g, d_r))))


def test_render_matches_numpy(gpu_hand, np_hand):
    th = oracle_np.X0
    d_gpu = gpu_hand.ctx.render_depth(th)
    d_np = oracle_np.render_depth_mm(np_hand, th)
    assert ((d_gpu > 0) == (d_np > 0)).mean() > 0.9995
    both = (d_gpu > 0) & (d_np > 0)
    assert np.abs(d_gpu[both] - d_np[both]).max() < 1e-3


def test_preprocess_host_matches_oracle(oracle, np_hand):
    import hpe
    d = oracle_np.render_depth_mm(np_hand, oracle_np.X0)
    for ds in (True, False):
        a = hpe.preprocess_depth(d, downsample=ds)
        b = oracle.preprocess(d, downsample=ds)
        np.testing.assert_array_equal(a["cloud"], b.cloud)
        np.testing.assert_array_equal(a["dt"], b.dt)
        np.testing.assert_array_equal(a["depth_cm"], b.depth)
        assert a["scale"] == b.scale and a["dtmax"] == b.dtmax


def test_fk_spheres_and_joints(oracle, ora_hand, gpu_hand):
    rng = np.random.default_rng(1)
    th = np.vstack([oracle_np.X0, hand_data.random_thetas(rng, 63, spread=3.0)])
    th[5] = 0.0
    th[6, 0:3] = (180.0, -180.0, 90.0)
    S, J = gpu_hand.build_batch(th)
    for i in range(len(th)):
        Sr, Jr = oracle.build(ora_hand, th[i], joints=True)
        np.testing.assert_allclose(S[i], Sr, rtol=0, atol=1e-9)
        np.testing.assert_allclose(J[i], Jr, rtol=0, atol=1e-9)


@pytest.mark.parametrize("downsample", [True, False])
def test_eval_costs_and_matches(oracle, ora_hand, gpu_hand, np_hand, downsample):
    import hpe
    rng = np.random.default_rng(2)
    truth = hand_data.trajectory(3, seed=5)[2]
    d = oracle_np.render_depth_mm(np_hand, truth)
    obs, om = _obs_pair(oracle, gpu_hand, d, downsample)
    cf = hpe.costfunc(gpu_hand, om)
    P = 48 if downsample else 12
    th = hand_data.random_thetas(rng, P, x0=truth, spread=0.4)
    th[0] = truth
    cost, match = cf.cal_cost_batch(th, return_match=True)
    ref = oracle.eval_costs(ora_hand, obs, th)
    np.testing.assert_allclose(cost, ref, rtol=RTOL, atol=0)
    for i in range(P):
        S = oracle.build(ora_hand, th[i])
        mr = oracle.correspondences(obs, S)
        assert _match_equiv(obs, S, match[i], mr)
    cost2 = cf.cal_cost_batch(th, with_collision=True)
    ref2 = oracle.eval_costs(ora_hand, obs, th, with_collision=True)
    np.testing.assert_allclose(cost2, ref2, rtol=RTOL, atol=0)


def test_cal_cost2_terms_and_frozen(oracle, ora_hand, gpu_hand, np_hand):
    import hpe
    d = oracle_np.render_depth_mm(np_hand, oracle_np.X0)
    obs, om = _obs_pair(oracle, gpu_hand, d)
    cf = hpe.costfunc(gpu_hand, om)
    th = oracle_np.X0 + 2.0
    m = np.zeros(obs.n, dtype=np.int32)
    c = cf.cal_cost2(th, m, True)
    cr, tr, mr = oracle.terms(ora_hand, obs, th)
    assert abs(c - cr) <= RTOL * abs(cr)
    np.testing.assert_allclose(cf.last_terms, tr, rtol=RTOL, atol=1e-300)
    assert np.array_equal(m, mr)
    th2 = th.copy(); th2[0] += 1e-5
    c2 = cf.cal_cost2(th2, m, False)
    cr2, tr2, _ = oracle.terms(ora_hand, obs, th2, match=mr)
    assert abs(c2 - cr2) <= RTOL * abs(cr2)


def test_match_ties_lowest_index(oracle, ora_hand, gpu_hand):
    """Cloud points placed exactly on float midpoints of sphere pairs: BFMatcher keeps
    the first of equal distances (and equal sqrtf values)."""
    import hpe
    th = oracle_np.X0
    S = oracle.build(ora_hand, th).astype(np.float32).astype(np.float64)
    rng = np.random.default_rng(3)
    pts = []
    for _ in range(400):
        a, b = rng.choice(48, 2, replace=False)
        pts.append(0.5 * (S[a] + S[b]))
    pts += list(S)  # exact centres: distance 0
    cloud = np.array(pts)
    depth = np.zeros((240, 320)); dt = np.zeros((240, 320), np.float32)
    K = np.array([[241.42, 0, 160], [0, 241.42, 120], [0, 0, 1.0]])
    import oracle_c
    obs = oracle_c.Obs(depth, dt, cloud, 0.1, 0.0, K)
    gpu_hand.ctx.store_frame(3, depth, dt, cloud, 0.1, 0.0, K)
    gpu_hand.ctx.select_frame(3)
    gpu_hand.ctx.frame_token = None
    om = hpe.observedmodel(); om._obs = dict(cloud=cloud); om.token = -1
    cf = hpe.costfunc(gpu_hand, om)
    cf._sync_frame = lambda: None
    cost, match = cf.cal_cost_batch(th[None, :], return_match=True)
    mr = oracle.correspondences(obs, oracle.build(ora_hand, th))
    assert np.array_equal(match[0], mr)
    assert abs(cost[0] - oracle.cal_cost(ora_hand, obs, th)) <= RTOL * abs(cost[0])


@pytest.mark.parametrize("P,maxiter", [(32, 11), (7, 4), (1, 3), (64, 1)])
def test_pso_evolve(oracle, ora_hand, gpu_hand, np_hand, P, maxiter):
    import hpe
    truth = hand_data.trajectory(2, seed=9)[1]
    d = oracle_np.render_depth_mm(np_hand, truth)
    obs, om = _obs_pair(oracle, gpu_hand, d)
    cf = hpe.costfunc(gpu_hand, om)
    ub, lb, sd = oracle_np.reference_bounds()
    pso = hpe.PSO()
    pso.set_pso_params(ub, lb, sd, 0.7298, 1.49618, 1.49618, maxiter, 1e-8, 1e-8)
    bestp = np.zeros(26)
    x0 = oracle_np.X0.copy()
    assert pso.pso_evolve(cf, x0, P, bestp) == 1
    rb, rc, tr = oracle.pso_evolve(ora_hand, obs, x0, P, maxiter, lb, ub, sd, seed=1000)
    np.testing.assert_allclose(bestp, rb, rtol=0, atol=1e-6)
    assert abs(pso.last_gbest_cost - rc) <= 1e-8 * abs(rc)
    if maxiter > 1:
        g, cnt, topo = pso.trace(cf)
        np.testing.assert_allclose(g, tr["gbest"], rtol=1e-8)
        assert np.array_equal(cnt, tr["count"])
        assert np.array_equal(topo, tr["topo"])


@pytest.mark.parametrize("P,maxiter,downsample", [(16, 4, True), (5, 3, True), (1, 2, True),
                                                  (4, 2, False)])
def test_pso_optimise(oracle, ora_hand, gpu_hand, np_hand, P, maxiter, downsample):
    """pso_optimise (PSO.cpp:539-712).  Every descent step differentiates the cost with
    eps 1e-5, so last-ulp cost differences (tree vs 2-accumulator sums) grow to ~1e-7 in
    the pose over a generation's 10 steps: bestp |diff| <= 1e-5, costs relative 1e-7.
    downsample=False: a full-resolution cloud (> 2048 points), matchId in HBM."""
    import hpe
    truth = hand_data.trajectory(2, seed=21)[1]
    d = oracle_np.render_depth_mm(np_hand, truth)
    obs, om = _obs_pair(oracle, gpu_hand, d, downsample=downsample)
    assert (obs.n > 2048) == (not downsample)
    cf = hpe.costfunc(gpu_hand, om)
    ub, lb, sd = oracle_np.reference_bounds()
    w, c1, c2 = 0.7298, 1.49618, 1.49618
    pso = hpe.PSO()
    pso.set_pso_params(ub, lb, sd, w, c1, c2, maxiter, 1e-8, 1e-8)
    bestp = np.zeros(26)
    x0 = oracle_np.X0.copy()
    assert pso.pso_optimise(cf, x0, P, bestp) == 1
    rb, rc, tr = oracle.pso_optimise(ora_hand, obs, x0, P, maxiter, lb, ub, sd, w, c1, c2,
                                     seed=1000)
    print("pso_optimise P=%d maxiter=%d: |dbestp| %.3g, dcost %.3g" %
          (P, maxiter, np.abs(bestp - rb).max(), abs(pso.last_gbest_cost - rc) / abs(rc)))
    np.testing.assert_allclose(bestp, rb, rtol=0, atol=1e-5)
    assert abs(pso.last_gbest_cost - rc) <= 1e-7 * abs(rc)
    np.testing.assert_allclose(pso.last_optimise_trace, tr, rtol=1e-7)
    # the descent lowers the cost below pso_evolve-free initialisation
    assert tr[-1] <= tr[0]


@pytest.mark.parametrize("exact", [False, True])
def test_refine_init_pose(oracle, ora_hand, gpu_hand, np_hand, exact):
    """Both refine forms: the hand-frame one (default) against the oracle's mirror of it,
    the reference's chain (HPE_REFINE_EXACT) against the restatement; the exact evaluation
    count either way."""
    import hpe
    truth = hand_data.trajectory(2, seed=4)[1]
    d = oracle_np.render_depth_mm(np_hand, truth)
    obs, om = _obs_pair(oracle, gpu_hand, d)
    cf = hpe.costfunc(gpu_hand, om)
    x0 = oracle_np.X0.copy()
    with _refine_form(gpu_hand.ctx, exact) as rigid:
        x_ref, ev_ref = oracle.refine(ora_hand, obs, x0, rigid=rigid)
        pso = hpe.PSO()
        x = x0.copy()
        pso.refine_init_pose(x, cf)
    assert pso.last_refine_evals == ev_ref
    np.testing.assert_allclose(x, x_ref, rtol=0, atol=1e-6)
    # and the hand-frame form is within the tracking tolerance of the reference's order
    x_chain, _ = oracle.refine(ora_hand, obs, x0, rigid=False)
    np.testing.assert_allclose(x, x_chain, rtol=0, atol=1e-6)


@pytest.mark.parametrize("exact", [False, True])
@pytest.mark.parametrize("npts", [256, 257, 1500])
def test_refine_staged_cloud_sizes(oracle, ora_hand, gpu_hand, np_hand, npts, exact):
    """refine_init_pose on clouds staged in LDS at the sizes around its two paths: N <= 256
    keeps each lane's matchIds in registers and spreads the correspondence items by SIMD
    load; 256 < N <= 2048 runs the plain strided search and LDS alignment.  The frame keeps
    the first npts foreground pixels of a rendered hand (no down-sampling)."""
    import hpe
    truth = hand_data.trajectory(2, seed=4)[1]
    d = oracle_np.render_depth_mm(np_hand, truth)
    fg = np.flatnonzero(d)
    assert len(fg) > npts
    d2 = np.zeros_like(d)
    d2.flat[fg[:npts]] = d.flat[fg[:npts]]
    obs, om = _obs_pair(oracle, gpu_hand, d2, downsample=False)
    assert obs.n == npts
    cf = hpe.costfunc(gpu_hand, om)
    x0 = oracle_np.X0.copy()
    with _refine_form(gpu_hand.ctx, exact) as rigid:
        x_ref, ev_ref = oracle.refine(ora_hand, obs, x0, rigid=rigid)
        pso = hpe.PSO()
        x = x0.copy()
        pso.refine_init_pose(x, cf)
    assert pso.last_refine_evals == ev_ref
    np.testing.assert_allclose(x, x_ref, rtol=0, atol=1e-6)


@pytest.mark.parametrize("exact", [False, True])
@pytest.mark.parametrize("mw", ["1", "0"])
def test_refine_full_cloud(oracle, ora_hand, np_hand, mw, exact, monkeypatch):
    """refine_init_pose on a full-resolution cloud (> 2048 points): the multi-workgroup
    form (mw=1: 64 helper workgroups own cloud slices, partial sums folded in a fixed
    order) and the single-workgroup form (HPE_REFINE_MW=0) both match the oracle, with
    the reference's evaluation count."""
    import hpe
    monkeypatch.setenv("HPE_REFINE_MW", mw)
    gh = hpe.reference_hand(device=0)  # the context reads HPE_REFINE_MW at creation
    truth = hand_data.trajectory(2, seed=4)[1]
    d = oracle_np.render_depth_mm(np_hand, truth)
    obs, om = _obs_pair(oracle, gh, d, downsample=False)
    assert obs.n > 2048
    cf = hpe.costfunc(gh, om)
    x0 = oracle_np.X0.copy()
    gh.ctx.refine_exact = exact
    x_ref, ev_ref = oracle.refine(ora_hand, obs, x0, rigid=not exact)
    pso = hpe.PSO()
    x = x0.copy()
    pso.refine_init_pose(x, cf)
    assert pso.last_refine_evals == ev_ref
    np.testing.assert_allclose(x, x_ref, rtol=0, atol=1e-6)
    x2 = x0.copy()  # deterministic: a second call gives the same bits
    pso.refine_init_pose(x2, cf)
    assert np.array_equal(x, x2)


def test_track_sequence(oracle, ora_hand, gpu_hand, np_hand):
    """test_full's loop (testmodel.cpp:117-139) on 3 synthetic frames, 32 particles."""
    import hpe
    poses = hand_data.trajectory(3, seed=11)
    ub, lb, sd = oracle_np.reference_bounds()
    pso = hpe.PSO()
    pso.set_pso_params(ub, lb, sd, 0.7298, 1.49618, 1.49618, 6, 1e-8, 1e-8)
    x_gpu = oracle_np.X0.copy(); x_ref = oracle_np.X0.copy()
    om = hpe.observedmodel(); om.downsample = True
    cf = hpe.costfunc(gpu_hand, om)
    for f in range(3):
        d = oracle_np.render_depth_mm(np_hand, poses[f])
        om.set_depth_mm(d)
        obs = oracle.preprocess(d)
        c = pso.track_frame(cf, x_gpu, 32, refine=True)
        x_ref, _ = oracle.refine(ora_hand, obs, x_ref, rigid=REFINE_RIGID)
        x_ref, _, _ = oracle.pso_evolve(ora_hand, obs, x_ref, 32, 6, lb, ub, sd)
        cr = oracle.cal_cost(ora_hand, obs, x_ref)
        np.testing.assert_allclose(x_gpu, x_ref, rtol=0, atol=1e-6)
        assert abs(c - cr) <= 1e-8 * abs(cr)


def test_edge_small_clouds(oracle, ora_hand, gpu_hand):
    """N = 1 and the degenerate down-sample (N_full < 250 -> 250 copies of point 0)."""
    import hpe
    d = np.zeros((240, 320), np.float32)
    d[120:125, 150:160] = 320.0  # 50 pixels at 32 cm
    for ds in (True, False):
        obs = oracle.preprocess(d, downsample=ds)
        om = hpe.observedmodel(); om.downsample = ds; om.set_depth_mm(d)
        cf = hpe.costfunc(gpu_hand, om)
        th = np.vstack([oracle_np.X0, oracle_np.X0 + 3])
        np.testing.assert_allclose(cf.cal_cost_batch(th), oracle.eval_costs(ora_hand, obs, th),
                                   rtol=RTOL)
    d1 = np.zeros((240, 320), np.float32); d1[100, 200] = 300.0
    obs = oracle.preprocess(d1, downsample=False)
    om = hpe.observedmodel(); om.set_depth_mm(d1)
    cf = hpe.costfunc(gpu_hand, om)
    np.testing.assert_allclose(cf.cal_cost_batch(oracle_np.X0[None]),
                               oracle.eval_costs(ora_hand, obs, oracle_np.X0[None]), rtol=RTOL)


def test_edge_large_cloud(oracle, ora_hand, gpu_hand, np_hand):
    """A frame whose foreground covers most of the image (a rendered hand in front of a
    240 x 200 block at 60 cm: ~50k points, full resolution): costs and correspondences of
    a particle batch against the oracle, and refine_init_pose (multi-workgroup form)."""
    import hpe
    truth = hand_data.trajectory(2, seed=4)[1]
    d = oracle_np.render_depth_mm(np_hand, truth)
    d = np.where(d > 0, d, 0).astype(np.float32)
    blk = np.zeros_like(d)
    blk[:, 60:260] = 600.0
    d = np.where(d > 0, d, blk)
    obs, om = _obs_pair(oracle, gpu_hand, d, downsample=False)
    assert obs.n > 40000
    cf = hpe.costfunc(gpu_hand, om)
    th = np.vstack([truth, truth + 2, oracle_np.X0])
    np.testing.assert_allclose(cf.cal_cost_batch(th), oracle.eval_costs(ora_hand, obs, th),
                               rtol=RTOL)
    x_ref, ev_ref = oracle.refine(ora_hand, obs, truth.copy(), rigid=REFINE_RIGID)
    pso = hpe.PSO()
    x = truth.copy()
    pso.refine_init_pose(x, cf)
    assert pso.last_refine_evals == ev_ref
    np.testing.assert_allclose(x, x_ref, rtol=0, atol=1e-6)


def test_edge_empty_frame_optimisers(oracle, ora_hand, gpu_hand):
    """An all-background frame (N = 0): lambda = 48/0, so every cost is NaN as in the
    reference (costfunc.cpp:372); no pbest ever improves, gbest stays zeros (PSO.cpp:546),
    refine's searches fail and leave x0 unchanged with the reference's eval count."""
    import hpe
    d = np.zeros((240, 320), np.float32)
    obs = oracle.preprocess(d, downsample=False)
    assert obs.n == 0
    om = hpe.observedmodel(); om.set_depth_mm(d)
    cf = hpe.costfunc(gpu_hand, om)
    ub, lb, sd = oracle_np.reference_bounds()
    pso = hpe.PSO()
    pso.set_pso_params(ub, lb, sd, 0.7298, 1.49618, 1.49618, 3, 1e-8, 1e-8)
    x0 = oracle_np.X0.copy()
    bp = np.zeros(26)
    pso.pso_evolve(cf, x0, 8, bp)
    rb, rc, _ = oracle.pso_evolve(ora_hand, obs, x0, 8, 3, lb, ub, sd, seed=1000)
    np.testing.assert_array_equal(bp, rb)
    assert pso.last_gbest_cost == rc
    x = x0.copy()
    pso.refine_init_pose(x, cf)
    xr, evr = oracle.refine(ora_hand, obs, x0, rigid=REFINE_RIGID)
    np.testing.assert_array_equal(x, xr)
    assert pso.last_refine_evals == evr
    pso.pso_optimise(cf, x0, 4, bp)
    ob, oc, _ = oracle.pso_optimise(ora_hand, obs, x0, 4, 3, lb, ub, sd, 0.7298, 1.49618,
                                    1.49618, seed=1000)
    np.testing.assert_array_equal(bp, ob)
    assert pso.last_gbest_cost == oc


@pytest.mark.parametrize("form,P,wpp", [("wave", 1024, 2), ("wave", 1030, 1), ("wave", 7, 2),
                                         ("block", 8, 0)])
def test_edge_empty_frame_every_form(oracle, ora_hand, form, P, wpp, monkeypatch):
    """An all-background frame (N = 0) in every generation form: the wave form at
    one and two waves per particle (the filter search's prologue must read no point), on a
    fresh context whose empty slot has no cloud arrays at all, and the workgroup form's
    filter cal_cost, chosen by the cloud BOUND of a device-prepared full-cloud frame (76,800)
    that turns out empty.  Results as the oracle's: NaN costs, gbest zeros and its cost 1e100
    (PSO.cpp:739-746), the tracked frame's cal_cost(bestp) NaN."""
    import ctypes as C

    import hpe
    monkeypatch.setenv("HPE_PSO_FORM", form)
    if wpp:
        monkeypatch.setenv("HPE_PSO_WPP", str(wpp))
    gh = hpe.reference_hand(device=0)  # fresh context (forms read at hpe_create)
    d = np.zeros((240, 320), np.float32)
    obs = oracle.preprocess(d, downsample=False)
    assert obs.n == 0
    ub, lb, sd = oracle_np.reference_bounds()
    pso = hpe.PSO()
    pso.set_pso_params(ub, lb, sd, 0.7298, 1.49618, 1.49618, 3, 1e-8, 1e-8)
    x0 = oracle_np.X0.copy()
    rb, rc, _ = oracle.pso_evolve(ora_hand, obs, x0, P, 3, lb, ub, sd, seed=1000)
    if form == "wave":
        om = hpe.observedmodel(); om.set_depth_mm(d)
        cf = hpe.costfunc(gh, om)
        bp = np.zeros(26)
        pso.pso_evolve(cf, x0, P, bp)
        np.testing.assert_array_equal(bp, rb)
        assert pso.last_gbest_cost == rc  # 1e100: no pbest ever beat the initial gbest
    else:  # a tracked frame on the device-prepared slot: refine + pso_evolve + cal_cost
        ctx = gh.ctx
        ctx.prepare_frame(1, d, True, False)
        ctx.select_frame(1)
        pso._push(ctx)
        x = x0.copy(); c = C.c_double(0)
        ctx.check(ctx.lib.hpe_track_frame(ctx.h, P, 1, hpe._lib.ptr(x, C.c_double), C.byref(c)))
        xr, _ = oracle.refine(ora_hand, obs, x0, rigid=REFINE_RIGID)
        rb, rc, _ = oracle.pso_evolve(ora_hand, obs, xr, P, 3, lb, ub, sd, seed=1000)
        np.testing.assert_array_equal(x, rb)
        assert np.isnan(c.value) and np.isnan(oracle.cal_cost(ora_hand, obs, rb))
    gh.ctx.close()


@pytest.mark.parametrize("P,maxiter,wpp", [(32, 11, 0), (7, 4, 0), (1, 3, 0), (1030, 3, 0),
                                           (32, 11, 1), (1030, 3, 2), (7, 4, 2)])
def test_pso_evolve_wave_form(oracle, ora_hand, np_hand, P, maxiter, wpp, monkeypatch):
    """The wave-form generation kernels (used for large swarms) against the oracle,
    including a ragged last workgroup (P not a multiple of the particles per workgroup), with
    one or two waves per particle (wpp 0: the context's choice)."""
    import hpe
    monkeypatch.setenv("HPE_PSO_FORM", "wave")
    if wpp:
        monkeypatch.setenv("HPE_PSO_WPP", str(wpp))
    gh = hpe.reference_hand(device=0)  # context created with the wave form forced
    truth = hand_data.trajectory(2, seed=9)[1]
    d = oracle_np.render_depth_mm(np_hand, truth)
    obs, om = _obs_pair(oracle, gh, d)
    cf = hpe.costfunc(gh, om)
    ub, lb, sd = oracle_np.reference_bounds()
    pso = hpe.PSO()
    pso.set_pso_params(ub, lb, sd, 0.7298, 1.49618, 1.49618, maxiter, 1e-8, 1e-8)
    bestp = np.zeros(26)
    x0 = oracle_np.X0.copy()
    assert pso.pso_evolve(cf, x0, P, bestp) == 1
    rb, rc, tr = oracle.pso_evolve(ora_hand, obs, x0, P, maxiter, lb, ub, sd, seed=1000)
    np.testing.assert_allclose(bestp, rb, rtol=0, atol=1e-6)
    assert abs(pso.last_gbest_cost - rc) <= 1e-8 * abs(rc)
    g, cnt, topo = pso.trace(cf)
    np.testing.assert_allclose(g, tr["gbest"], rtol=1e-8)
    assert np.array_equal(cnt, tr["count"]) and np.array_equal(topo, tr["topo"])


@pytest.mark.parametrize("wpp", [1, 2])
def test_wave_form_cooperative_fk_bit_identical(oracle, ora_hand, np_hand, wpp, monkeypatch):
    """The wave form's workgroup-cooperative FK (fk_coop, the default) against each wave's
    own FK (HPE_FK_COOP=0), at one and two waves per particle: the same operations per item,
    so the same pose, cost and traces bit for bit (and both against the oracle)."""
    import hpe
    monkeypatch.setenv("HPE_PSO_FORM", "wave")
    monkeypatch.setenv("HPE_PSO_WPP", str(wpp))
    truth = hand_data.trajectory(2, seed=11)[1]
    d = oracle_np.render_depth_mm(np_hand, truth)
    ub, lb, sd = oracle_np.reference_bounds()
    out = {}
    for coop in ("1", "0"):
        monkeypatch.setenv("HPE_FK_COOP", coop)
        gh = hpe.reference_hand(device=0)
        obs, om = _obs_pair(oracle, gh, d)
        cf = hpe.costfunc(gh, om)
        pso = hpe.PSO()
        pso.set_pso_params(ub, lb, sd, 0.7298, 1.49618, 1.49618, 4, 1e-8, 1e-8)
        bestp = np.zeros(26)
        assert pso.pso_evolve(cf, oracle_np.X0.copy(), 1030, bestp) == 1
        out[coop] = (bestp.copy(), pso.last_gbest_cost, pso.trace(cf))
    assert np.array_equal(out["1"][0], out["0"][0])
    assert out["1"][1] == out["0"][1]
    for a, b in zip(out["1"][2], out["0"][2]):
        assert np.array_equal(a, b)
    rb, rc, _ = oracle.pso_evolve(ora_hand, obs, oracle_np.X0.copy(), 1030, 4, lb, ub, sd, seed=1000)
    np.testing.assert_allclose(out["1"][0], rb, rtol=0, atol=1e-6)
    assert abs(out["1"][1] - rc) <= 1e-8 * abs(rc)


@pytest.mark.parametrize("form", ["wave", "wave2", "block"])
@pytest.mark.parametrize("n_ties", [400, 4000])
def test_wave_form_filter_search_ties(oracle, ora_hand, n_ties, form, monkeypatch):
    """The filter search (hpe_device.hpp bf_filter_lane: the wave form at one and two waves
    per particle, and the workgroup form's cal_cost above 256 points) on points that defeat
    its estimate: float midpoints of centre pairs (exact and near ties, decided by the exact
    search), the centres themselves (d2 = 0) and far outliers (the error bound E >= 0.5 sends
    them the exact way), with a swarm whose particles all sit at the pose the cloud was built
    from (std 0): every evaluation of the init and generation kernels must equal the oracle's
    cal_cost, whose match takes the first of equal distances.  A wrong pick changes the
    alignment term (the radii differ)."""
    import hpe
    import oracle_c
    monkeypatch.setenv("HPE_PSO_FORM", "block" if form == "block" else "wave")
    if form != "block":
        monkeypatch.setenv("HPE_PSO_WPP", "2" if form == "wave2" else "1")
    gh = hpe.reference_hand(device=0)
    th = oracle_np.X0
    S = oracle.build(ora_hand, th).astype(np.float32).astype(np.float64)
    rng = np.random.default_rng(4)
    pts = []
    for _ in range(n_ties):
        a, b = rng.choice(48, 2, replace=False)
        pts.append(0.5 * (S[a] + S[b]))
    pts += list(S)
    for k in range(6):  # outliers 400 and 1200 cm from the hand (E >= 0.5 from ~360 cm on)
        v = np.zeros(3)
        v[k % 3] = (-1) ** k * (400.0 if k < 3 else 1200.0)
        pts.append(S[21] + v)
    cloud = np.array(pts)
    depth = np.zeros((240, 320)); dt = np.zeros((240, 320), np.float32)
    K = np.array([[241.42, 0, 160], [0, 241.42, 120], [0, 0, 1.0]])
    obs = oracle_c.Obs(depth, dt, cloud, 0.1, 0.0, K)
    gh.ctx.store_frame(3, depth, dt, cloud, 0.1, 0.0, K)
    gh.ctx.select_frame(3)
    gh.ctx.frame_token = None
    om = hpe.observedmodel(); om._obs = dict(cloud=cloud); om.token = -1
    cf = hpe.costfunc(gh, om)
    cf._sync_frame = lambda: None
    ub, lb, _ = oracle_np.reference_bounds()
    pso = hpe.PSO()
    pso.set_pso_params(ub, lb, np.zeros(26), 0.7298, 1.49618, 1.49618, 2, 1e-8, 1e-8)
    bestp = np.zeros(26)
    assert pso.pso_evolve(cf, th.copy(), 1024, bestp) == 1
    ref = oracle.cal_cost(ora_hand, obs, th)
    assert abs(pso.last_gbest_cost - ref) <= RTOL * abs(ref)
    g, _, _ = pso.trace(cf)
    np.testing.assert_allclose(g, ref, rtol=RTOL)
    np.testing.assert_array_equal(bestp, th)


@pytest.mark.parametrize("P,maxiter", [(1024, 4), (1030, 3)])
def test_pso_evolve_block_form_inbox_counts(oracle, ora_hand, np_hand, P, maxiter, monkeypatch):
    """The workgroup-per-particle generation kernel at the edge of its per-receiver inbox
    counts (InboxCounts in the kernel arguments, P <= KIN_MAX = 1024) and just above it
    (every receiver reads the K slots of both variants), against the oracle."""
    import hpe
    monkeypatch.setenv("HPE_PSO_FORM", "block")
    gh = hpe.reference_hand(device=0)  # context created with the block form forced
    truth = hand_data.trajectory(2, seed=5)[1]
    d = oracle_np.render_depth_mm(np_hand, truth)
    obs, om = _obs_pair(oracle, gh, d)
    cf = hpe.costfunc(gh, om)
    ub, lb, sd = oracle_np.reference_bounds()
    pso = hpe.PSO()
    pso.set_pso_params(ub, lb, sd, 0.7298, 1.49618, 1.49618, maxiter, 1e-8, 1e-8)
    bestp = np.zeros(26)
    x0 = oracle_np.X0.copy()
    assert pso.pso_evolve(cf, x0, P, bestp) == 1
    rb, rc, tr = oracle.pso_evolve(ora_hand, obs, x0, P, maxiter, lb, ub, sd, seed=1000)
    np.testing.assert_allclose(bestp, rb, rtol=0, atol=1e-6)
    assert abs(pso.last_gbest_cost - rc) <= 1e-8 * abs(rc)
    g, cnt, topo = pso.trace(cf)
    np.testing.assert_allclose(g, tr["gbest"], rtol=1e-8)
    assert np.array_equal(cnt, tr["count"]) and np.array_equal(topo, tr["topo"])
