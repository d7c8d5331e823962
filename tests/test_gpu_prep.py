"""GPU preprocessing (hpe_prepare_frame) against the host preprocessing
(hpe_preprocess_depth, itself bit-exact against the C oracle: tests/test_host.py).

Depth, cloud, distance transform, its max, the cloud size and the cm-per-pixel scale
(Armadillo's two-accumulator mean replayed in order) must be identical.
Edge cases as observedmodel has them: empty frame (250 zero points when down-sampling,
NaN scale), a single pixel, a full frame, frames touching the image border."""
import numpy as np
import pytest

import hand_data
from hand_data import REFINE_RIGID
import oracle_np

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gh():
    import hpe
    return hpe.reference_hand(device=0)


def _frames(np_hand):
    out = []
    for seed in (0, 3):
        for th in hand_data.trajectory(3, seed=seed):
            out.append(oracle_np.render_depth_mm(np_hand, th))
    e = np.zeros((240, 320), np.float32)
    one = e.copy(); one[100, 200] = 300.0
    full = np.full((240, 320), 455.5, np.float32)
    edge = e.copy(); edge[0:6, 0:9] = 250.0; edge[-4:, -7:] = 251.0; edge[120, :] = 260.0
    rng = np.random.default_rng(1)
    speck = np.where(rng.random((240, 320)) < 0.02, rng.uniform(200, 600, (240, 320)), 0).astype(np.float32)
    # the DT's forward scan starts at the first row holding a hand pixel (an even row at
    # or above it): first hand rows odd / even / last, a lone pixel in a corner column
    late = []
    for r, c in ((1, 5), (133, 160), (238, 0), (239, 319), (239, 0), (200, 319)):
        x = e.copy(); x[r, c] = 321.0
        late.append(x)
    band = e.copy(); band[133:140, 40:90] = 410.0; band[201, 300:320] = 415.0
    return out + [e, one, full, edge, speck, band] + late


def _check(a, b):
    np.testing.assert_array_equal(a["depth_cm"], b["depth_cm"])
    np.testing.assert_array_equal(a["dt"], b["dt"])
    np.testing.assert_array_equal(a["cloud"], b["cloud"])
    assert a["dtmax"] == b["dtmax"]
    if np.isnan(b["scale"]):
        assert np.isnan(a["scale"])
    else:
        assert a["scale"] == b["scale"]


@pytest.mark.parametrize("downsample", [True, False])
def test_prepare_matches_host(gh, np_hand, downsample):
    import hpe
    for k, d in enumerate(_frames(np_hand)):
        gh.ctx.prepare_frame(100 + k, d, downsample=downsample)
    for k, d in enumerate(_frames(np_hand)):
        _check(gh.ctx.frame_readback(100 + k), hpe.preprocess_depth(d, downsample=downsample))


def test_prepared_frames_track_like_oracle(gh, oracle, ora_hand, np_hand):
    """test_full's loop on device-prepared frames (prepared one frame ahead)."""
    import hpe
    poses = hand_data.trajectory(3, seed=12)
    depth = [oracle_np.render_depth_mm(np_hand, th) for th in poses]
    ub, lb, sd = oracle_np.reference_bounds()
    pso = hpe.PSO()
    pso.set_pso_params(ub, lb, sd, 0.7298, 1.49618, 1.49618, 6, 1e-8, 1e-8)
    pso._push(gh.ctx)
    x_gpu = oracle_np.X0.copy(); x_ref = oracle_np.X0.copy()
    gh.ctx.prepare_frame(200, depth[0])
    import ctypes as C
    from hpe._lib import ptr
    for f in range(3):
        if f + 1 < 3:
            gh.ctx.prepare_frame(200 + f + 1, depth[f + 1])
        gh.ctx.select_frame(200 + f)
        gh.ctx.frame_token = None
        cost = C.c_double(0)
        gh.ctx.check(gh.ctx.lib.hpe_track_frame(gh.ctx.h, 32, 1, ptr(x_gpu, C.c_double),
                                                C.byref(cost)))
        obs = oracle.preprocess(depth[f])
        x_ref, _ = oracle.refine(ora_hand, obs, x_ref, rigid=REFINE_RIGID)
        x_ref, _, _ = oracle.pso_evolve(ora_hand, obs, x_ref, 32, 6, lb, ub, sd)
        cr = oracle.cal_cost(ora_hand, obs, x_ref)
        np.testing.assert_allclose(x_gpu, x_ref, rtol=0, atol=1e-6)
        assert abs(cost.value - cr) <= 1e-8 * abs(cr)


@pytest.mark.parametrize("downsample", [True, False])
def test_pipelined_tracking_like_oracle(gh, oracle, ora_hand, np_hand, downsample):
    """hpe_track_pipelined: each frame is prepared inside the previous frame's refine launch
    (fused workgroups); the tracked poses / costs must equal the oracle's test_full loop on
    the same raw frames."""
    import ctypes as C
    import hpe
    poses = hand_data.trajectory(4, seed=19)
    depth = [oracle_np.render_depth_mm(np_hand, th) for th in poses]
    ub, lb, sd = oracle_np.reference_bounds()
    maxiter = 6 if downsample else 3
    P = 32 if downsample else 8
    pso = hpe.PSO()
    pso.set_pso_params(ub, lb, sd, 0.7298, 1.49618, 1.49618, maxiter, 1e-8, 1e-8)
    pso._push(gh.ctx)
    state = np.zeros(27)
    dbuf = C.c_void_p()
    rt = gh.ctx.lib
    import torch
    st = torch.zeros(27, dtype=torch.float64, device="cuda:0")
    st[:26] = torch.from_numpy(oracle_np.X0)
    torch.cuda.synchronize()
    gh.ctx.pipeline_begin(depth[0], downsample=downsample)
    x_ref = oracle_np.X0.copy()
    for f in range(4):
        gh.ctx.track_pipelined(P, 1, st.data_ptr(), depth[f + 1] if f + 1 < 4 else None)
        gh.ctx.check(rt.hpe_sync(gh.ctx.h))
        out = st.cpu().numpy()
        obs = oracle.preprocess(depth[f], downsample=downsample)
        x_ref, _ = oracle.refine(ora_hand, obs, x_ref, rigid=REFINE_RIGID)
        x_ref, _, _ = oracle.pso_evolve(ora_hand, obs, x_ref, P, maxiter, lb, ub, sd)
        cr = oracle.cal_cost(ora_hand, obs, x_ref)
        np.testing.assert_allclose(out[:26], x_ref, rtol=0, atol=1e-6)
        assert abs(out[26] - cr) <= 1e-8 * abs(cr)


def test_sequence_tracking_like_oracle_and_per_frame(gh, oracle, ora_hand, np_hand):
    """hpe_track_sequence_dev (offline test_full loop over resident frames, several frames
    per graph launch): every frame's {bestp, cost} equals the oracle's loop, and equals
    hpe_track_frame_dev frame by frame bit for bit, for chunks of 1, 3 (ragged: 3 + 3 + 1)
    and 8 frames; a second call replays the cached graphs to the same bits."""
    import ctypes as C
    import hpe
    import torch
    n, P, maxiter, s0 = 7, 32, 6, 400
    poses = hand_data.trajectory(n, seed=23)
    depth = [oracle_np.render_depth_mm(np_hand, th) for th in poses]
    ub, lb, sd = oracle_np.reference_bounds()
    pso = hpe.PSO()
    pso.set_pso_params(ub, lb, sd, 0.7298, 1.49618, 1.49618, maxiter, 1e-8, 1e-8)
    pso._push(gh.ctx)
    for f in range(n):
        gh.ctx.prepare_frame(s0 + f, depth[f])
    rt = gh.ctx.lib
    # per-frame reference on the GPU: select + hpe_track_frame_dev
    st = torch.zeros(27, dtype=torch.float64, device="cuda:0")
    st[:26] = torch.from_numpy(oracle_np.X0)
    per_frame = []
    for f in range(n):
        gh.ctx.select_frame(s0 + f)
        gh.ctx.check(rt.hpe_track_frame_dev(gh.ctx.h, P, 1, C.c_void_p(st.data_ptr())))
        gh.ctx.check(rt.hpe_sync(gh.ctx.h))
        per_frame.append(st.cpu().numpy().copy())
    per_frame = np.array(per_frame)
    # the oracle's test_full loop
    x_ref = oracle_np.X0.copy()
    for f in range(n):
        obs = oracle.preprocess(depth[f])
        x_ref, _ = oracle.refine(ora_hand, obs, x_ref, rigid=REFINE_RIGID)
        x_ref, _, _ = oracle.pso_evolve(ora_hand, obs, x_ref, P, maxiter, lb, ub, sd)
        cr = oracle.cal_cost(ora_hand, obs, x_ref)
        np.testing.assert_allclose(per_frame[f, :26], x_ref, rtol=0, atol=1e-6)
        assert abs(per_frame[f, 26] - cr) <= 1e-8 * abs(cr)
    hist = torch.empty((n, 27), dtype=torch.float64, device="cuda:0")  # one buffer: a graph key
    caps = C.c_uint64(0)
    seen = set()  # chunk lengths captured so far: a chunk graph is keyed by its shape only
    for it, K in enumerate((1, 3, 8, 3)):  # the last: cached graphs
        st[:26] = torch.from_numpy(oracle_np.X0)
        st[26] = 0.0
        hist.fill_(float("nan"))
        torch.cuda.synchronize()
        gh.ctx.check(rt.hpe_graph_captures(gh.ctx.h, C.byref(caps)))
        before = caps.value
        gh.ctx.track_sequence(P, 1, st.data_ptr(), s0, n, K, hist.data_ptr())
        gh.ctx.check(rt.hpe_sync(gh.ctx.h))
        gh.ctx.check(rt.hpe_graph_captures(gh.ctx.h, C.byref(caps)))
        h = hist.cpu().numpy()
        assert np.array_equal(h, per_frame), K
        assert np.array_equal(st.cpu().numpy(), per_frame[-1]), K
        # chunk graphs are keyed by shape, not slots: 7 frames in chunks of K capture one
        # graph per chunk length not seen before (none on the replay)
        lens = {min(K, n - f0) for f0 in range(0, n, K)}
        assert caps.value - before == len(lens - seen), (K, caps.value - before)
        seen |= lens
    # argument errors
    bad = rt.hpe_track_sequence_dev
    assert bad(gh.ctx.h, P, 1, C.c_void_p(st.data_ptr()), s0, 0, 0, None) == hpe._lib.HPE_E_ARG
    assert bad(gh.ctx.h, P, 1, C.c_void_p(st.data_ptr()), 4095, 2, 0, None) == hpe._lib.HPE_E_ARG
    assert bad(gh.ctx.h, P, 1, C.c_void_p(st.data_ptr()), s0, n, 33, None) == hpe._lib.HPE_E_ARG
    assert bad(gh.ctx.h, P, 1, None, s0, n, 0, None) == hpe._lib.HPE_E_ARG


def test_sequence_wave_form_tail_and_empty_frame(gh, np_hand):
    """in a sequence chunk the final kernel stages the next frame's
    descriptor into the one its own cal_cost(bestp) tail reads.  The tail runs when the
    generations used the wave form (P >= 1024: no same-eval shortcut) or when no cost beat
    1e100 (an empty frame: every cost NaN).  Every frame of the sequence must equal
    hpe_track_frame_dev frame by frame, bit for bit, NaNs included."""
    import ctypes as C
    import hpe
    import torch
    n, P, maxiter, s0 = 5, 1024, 3, 600
    poses = hand_data.trajectory(n, seed=29)
    depth = [oracle_np.render_depth_mm(np_hand, th) for th in poses]
    depth[2] = np.zeros_like(depth[2])  # empty frame: NaN scale, NaN costs, bestp = zeros
    ub, lb, sd = oracle_np.reference_bounds()
    pso = hpe.PSO()
    pso.set_pso_params(ub, lb, sd, 0.7298, 1.49618, 1.49618, maxiter, 1e-8, 1e-8)
    pso._push(gh.ctx)
    for f in range(n):
        gh.ctx.prepare_frame(s0 + f, depth[f])
    rt = gh.ctx.lib
    st = torch.zeros(27, dtype=torch.float64, device="cuda:0")
    per_frame = []
    for f in range(n):  # the frames tracked independently from X0 (refine off)
        st[:26] = torch.from_numpy(oracle_np.X0)
        gh.ctx.select_frame(s0 + f)
        gh.ctx.check(rt.hpe_track_frame_dev(gh.ctx.h, P, 0, C.c_void_p(st.data_ptr())))
        gh.ctx.check(rt.hpe_sync(gh.ctx.h))
        per_frame.append(st.cpu().numpy().copy())
    assert np.isnan(per_frame[2][26]) and not np.isnan(per_frame[1][26])
    hist = torch.empty((1, 27), dtype=torch.float64, device="cuda:0")
    for f in range(n):  # each frame as a one-frame sequence chunk that stages the next slot
        st[:26] = torch.from_numpy(oracle_np.X0)
        st[26] = 0.0
        hist.fill_(-1.0)
        torch.cuda.synchronize()
        gh.ctx.track_sequence(P, 0, st.data_ptr(), s0 + f, 1, 1, hist.data_ptr())
        gh.ctx.check(rt.hpe_sync(gh.ctx.h))
        assert np.array_equal(hist.cpu().numpy()[0], per_frame[f], equal_nan=True), f
    # and the whole sequence in one chunk (x0 chained): the same bits as the chained per-frame loop
    st[:26] = torch.from_numpy(oracle_np.X0)
    chained = []
    for f in range(n):
        gh.ctx.select_frame(s0 + f)
        gh.ctx.check(rt.hpe_track_frame_dev(gh.ctx.h, P, 0, C.c_void_p(st.data_ptr())))
        gh.ctx.check(rt.hpe_sync(gh.ctx.h))
        chained.append(st.cpu().numpy().copy())
    hist = torch.empty((n, 27), dtype=torch.float64, device="cuda:0")
    st[:26] = torch.from_numpy(oracle_np.X0)
    st[26] = 0.0
    torch.cuda.synchronize()
    gh.ctx.track_sequence(P, 0, st.data_ptr(), s0, n, 8, hist.data_ptr())
    gh.ctx.check(rt.hpe_sync(gh.ctx.h))
    assert np.array_equal(hist.cpu().numpy(), np.array(chained), equal_nan=True)


@pytest.mark.parametrize("downsample", [True, False])
def test_raw_sequence_like_pipelined_and_oracle(gh, oracle, ora_hand, np_hand, downsample):
    """hpe_track_raw_sequence_dev (raw frames resident in HBM, each next frame prepared inside
    the previous frame's refine launch through the device row cursor, several frames per
    graph): every frame's {bestp, cost} equals hpe_track_pipelined's frame by frame bit for
    bit and the oracle's test_full loop, for chunks of 1, 3 (odd: both buffer parities,
    ragged 3 + 3 + 1) and 8; graphs are keyed by chunk shape, so a replay captures none."""
    import ctypes as C
    import hpe
    import torch
    n = 7 if downsample else 3
    P, maxiter = (32, 6) if downsample else (8, 3)
    poses = hand_data.trajectory(n, seed=29)
    depth = [oracle_np.render_depth_mm(np_hand, th) for th in poses]
    ub, lb, sd = oracle_np.reference_bounds()
    pso = hpe.PSO()
    pso.set_pso_params(ub, lb, sd, 0.7298, 1.49618, 1.49618, maxiter, 1e-8, 1e-8)
    pso._push(gh.ctx)
    rt = gh.ctx.lib
    st = torch.zeros(27, dtype=torch.float64, device="cuda:0")
    st[:26] = torch.from_numpy(oracle_np.X0)
    torch.cuda.synchronize()
    gh.ctx.pipeline_begin(depth[0], downsample=downsample)
    per_frame = []
    for f in range(n):
        gh.ctx.track_pipelined(P, 1, st.data_ptr(), depth[f + 1] if f + 1 < n else None)
        gh.ctx.check(rt.hpe_sync(gh.ctx.h))
        per_frame.append(st.cpu().numpy().copy())
    per_frame = np.array(per_frame)
    x_ref = oracle_np.X0.copy()
    for f in range(n):
        obs = oracle.preprocess(depth[f], downsample=downsample)
        x_ref, _ = oracle.refine(ora_hand, obs, x_ref, rigid=REFINE_RIGID)
        x_ref, _, _ = oracle.pso_evolve(ora_hand, obs, x_ref, P, maxiter, lb, ub, sd)
        cr = oracle.cal_cost(ora_hand, obs, x_ref)
        np.testing.assert_allclose(per_frame[f, :26], x_ref, rtol=0, atol=1e-6)
        assert abs(per_frame[f, 26] - cr) <= 1e-8 * abs(cr)
    d_raw = torch.from_numpy(np.stack(depth).astype(np.float32)).to("cuda:0")
    hist = torch.empty((n, 27), dtype=torch.float64, device="cuda:0")
    caps = C.c_uint64(0)
    seen = set()
    for K in (1, 3, 8, 3):  # the last: cached graphs
        st[:26] = torch.from_numpy(oracle_np.X0)
        st[26] = 0.0
        hist.fill_(float("nan"))
        torch.cuda.synchronize()
        gh.ctx.check(rt.hpe_graph_captures(gh.ctx.h, C.byref(caps)))
        before = caps.value
        gh.ctx.track_raw_sequence(P, 1, st.data_ptr(), d_raw.data_ptr(), n,
                                  downsample=downsample, frames_per_graph=K,
                                  d_hist_ptr=hist.data_ptr())
        gh.ctx.check(rt.hpe_sync(gh.ctx.h))
        gh.ctx.check(rt.hpe_graph_captures(gh.ctx.h, C.byref(caps)))
        assert np.array_equal(hist.cpu().numpy(), per_frame), K
        assert np.array_equal(st.cpu().numpy(), per_frame[-1]), K
        # one graph per chunk shape (length, first buffer's parity, last frame prepares more)
        shapes = {(min(K, n - f0), f0 & 1, f0 + K < n) for f0 in range(0, n, K)}
        assert caps.value - before == len(shapes - seen), (K, caps.value - before)
        seen |= shapes
    bad = rt.hpe_track_raw_sequence_dev
    sp = C.c_void_p(st.data_ptr())
    assert bad(gh.ctx.h, P, 1, sp, C.c_void_p(d_raw.data_ptr()), 0, 1, 1, 241.42, 0, None) == hpe._lib.HPE_E_ARG
    assert bad(gh.ctx.h, P, 1, sp, None, n, 1, 1, 241.42, 0, None) == hpe._lib.HPE_E_ARG
    assert bad(gh.ctx.h, P, 1, sp, C.c_void_p(d_raw.data_ptr()), n, 1, 1, 241.42, 33, None) == hpe._lib.HPE_E_ARG
    assert bad(gh.ctx.h, P, 1, sp, C.c_void_p(d_raw.data_ptr()), n, 1, 1, 0.0, 0, None) == hpe._lib.HPE_E_ARG


def test_raw_sequence_edges(gh, np_hand):
    """hpe_track_raw_sequence_dev at the edges: one frame (nothing prepared after it),
    frames_per_graph larger than the sequence, the largest chunk (HPE_SEQ_MAX_CHUNK), and a
    call after a pipelined sequence (which it ends) -- each equal to the per-frame
    pipelined loop bit for bit."""
    import hpe
    import torch
    n, P, maxiter = 5, 16, 4
    poses = hand_data.trajectory(n, seed=31)
    depth = [oracle_np.render_depth_mm(np_hand, th) for th in poses]
    ub, lb, sd = oracle_np.reference_bounds()
    pso = hpe.PSO()
    pso.set_pso_params(ub, lb, sd, 0.7298, 1.49618, 1.49618, maxiter, 1e-8, 1e-8)
    pso._push(gh.ctx)
    rt = gh.ctx.lib
    st = torch.zeros(27, dtype=torch.float64, device="cuda:0")

    def pipelined(m):
        st[:26] = torch.from_numpy(oracle_np.X0)
        st[26] = 0.0
        torch.cuda.synchronize()
        gh.ctx.pipeline_begin(depth[0])
        out = []
        for f in range(m):
            gh.ctx.track_pipelined(P, 1, st.data_ptr(), depth[f + 1] if f + 1 < m else None)
            gh.ctx.check(rt.hpe_sync(gh.ctx.h))
            out.append(st.cpu().numpy().copy())
        return np.array(out)

    ref = pipelined(n)
    d_raw = torch.from_numpy(np.stack(depth).astype(np.float32)).to("cuda:0")
    hist = torch.empty((n, 27), dtype=torch.float64, device="cuda:0")
    for m, K in ((1, 0), (1, 8), (n, 32), (n, n + 3)):
        st[:26] = torch.from_numpy(oracle_np.X0)
        st[26] = 0.0
        hist.fill_(float("nan"))
        torch.cuda.synchronize()
        gh.ctx.track_raw_sequence(P, 1, st.data_ptr(), d_raw.data_ptr(), m,
                                  frames_per_graph=K, d_hist_ptr=hist.data_ptr())
        gh.ctx.check(rt.hpe_sync(gh.ctx.h))
        h = hist.cpu().numpy()
        assert np.array_equal(h[:m], ref[:m]), (m, K)
        assert np.isnan(h[m:]).all(), (m, K)  # rows past the sequence untouched
    # a pipelined sequence in progress, then a raw sequence: it starts over cleanly
    st[:26] = torch.from_numpy(oracle_np.X0)
    torch.cuda.synchronize()
    gh.ctx.pipeline_begin(depth[0])
    gh.ctx.track_pipelined(P, 1, st.data_ptr(), depth[1])
    gh.ctx.check(rt.hpe_sync(gh.ctx.h))
    st[:26] = torch.from_numpy(oracle_np.X0)
    st[26] = 0.0
    torch.cuda.synchronize()
    gh.ctx.track_raw_sequence(P, 1, st.data_ptr(), d_raw.data_ptr(), n, frames_per_graph=2,
                              d_hist_ptr=hist.data_ptr())
    gh.ctx.check(rt.hpe_sync(gh.ctx.h))
    assert np.array_equal(hist.cpu().numpy(), ref)
