"""Known-answer tests pinning the C oracle (no GPU).

The reference ships no tests or golden outputs, so the oracle is
pinned by analytic facts of the reference's own model on its own data files
(misc/hgeo.dat, misc/rad.dat) and by published test vectors of the draw generator.
"""
import math

import numpy as np
import pytest

import hand_data
import oracle_np


def test_philox_random123_kat(oracle):
    """Philox4x32-10 known-answer vectors of Random123 (kat_vectors)."""
    assert oracle.philox([0, 0, 0, 0], [0, 0]) == [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]
    assert oracle.philox([0xffffffff] * 4, [0xffffffff] * 2) == \
        [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]
    assert oracle.philox([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344],
                         [0xa4093822, 0x299f31d0]) == [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]


def test_u01_range_and_normals(oracle):
    u = np.array([oracle.u01(1000, 2, g, i, d) for g in range(3) for i in range(20)
                  for d in range(26)])
    assert u.min() >= 0.0 and u.max() < 1.0
    assert abs(u.mean() - 0.5) < 0.02
    n = oracle.normals(1000, 400)
    assert abs(n.mean()) < 0.02 and abs(n.std() - 1.0) < 0.02


def _digit_joints(oracle, h, theta):
    """hand_joints rows (handmodel.cpp:291-296) + the per-digit base joint."""
    _, J = oracle.build(h, theta, joints=True)
    return J


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_fk_bone_lengths(oracle, ora_hand, seed):
    """Consecutive joints of every digit are exactly the DH segment lengths apart
    (fingermodel.cpp:142-155 L5..L7; thumbmodel.cpp:150-163 L1..L3), and the MCP joint
    is L0/L4 from the hand position (T01/Trf translation)."""
    geo, _ = hand_data.geometry_cm()
    rng = np.random.default_rng(seed)
    th = hand_data.random_thetas(rng, 1, spread=2.0)[0]
    J = _digit_joints(oracle, ora_hand, th)
    wrist = J[0]
    # rows 1-4 index, 5-8 middle, 9-12 ring, 13-16 little, 17-20 thumb (joints 1..4)
    for k, d in enumerate((1, 2, 3, 4, 0)):
        rows = J[1 + 4 * k:5 + 4 * k]
        L = geo[4 * d:4 * d + 4]
        assert abs(np.linalg.norm(rows[0] - wrist) - L[0]) < 1e-12
        for s in range(3):
            assert abs(np.linalg.norm(rows[s + 1] - rows[s]) - L[s + 1]) < 1e-12


def test_fk_sphere_placement(oracle, ora_hand):
    """Spheres lie on the segments at t = 1/3 steps (finger palm segment) and
    t = 1/2, 1 elsewhere (fingermodel.cpp:223-265, thumbmodel.cpp:242-272); y, z
    negated (handmodel.cpp:288)."""
    th = oracle_np.X0.copy()
    S = oracle.build(ora_hand, th)
    _, J = oracle.build(ora_hand, th, joints=True)
    Su = S * np.array([1, -1, -1])
    # index finger: spheres 8..17; joints 1..4 are J rows 1..4
    j1, j2, j3, j4 = J[1], J[2], J[3], J[4]
    np.testing.assert_allclose(Su[11], j1, atol=1e-12)   # palm segment end (t = 1)
    np.testing.assert_allclose(Su[12], 0.5 * (j1 + j2), atol=1e-12)
    np.testing.assert_allclose(Su[13], j2, atol=1e-12)
    np.testing.assert_allclose(Su[15], j3, atol=1e-12)
    np.testing.assert_allclose(Su[17], j4, atol=1e-12)
    # palm segment: 4 equally spaced spheres
    d = np.diff(Su[8:12], axis=0)
    np.testing.assert_allclose(d[0], d[1], atol=1e-12)
    np.testing.assert_allclose(d[1], d[2], atol=1e-12)
    # thumb: spheres 0..7 at midpoints / ends of its 4 segments; sphere 1 is joint 1
    np.testing.assert_allclose(Su[1], J[17], atol=1e-12)
    np.testing.assert_allclose(Su[7], J[20], atol=1e-12)


def test_fk_rigid_translation(oracle, ora_hand):
    """Translating the pose translates every sphere (T00, fingermodel.cpp:157-160)."""
    th = oracle_np.X0.copy()
    S0 = oracle.build(ora_hand, th)
    th2 = th.copy()
    th2[3:6] += (1.5, -2.0, 0.25)
    S1 = oracle.build(ora_hand, th2)
    np.testing.assert_allclose(S1 - S0, np.tile([1.5, 2.0, -0.25], (48, 1)), atol=1e-12)


def _blank_obs(cloud=None, scale=0.1, dtmax=0.0):
    import oracle_c
    depth = np.zeros((240, 320))
    dt = np.zeros((240, 320), np.float32)
    K = np.array([[241.42, 0, 160], [0, 241.42, 120], [0, 0, 1.0]])
    if cloud is None:
        cloud = np.zeros((1, 3))
    return oracle_c.Obs(depth, dt, cloud, scale, dtmax, K)


def test_depth_penalty_branches(oracle, ora_hand):
    """Per-branch values of costfunc.cpp:274-300 on hand-built centres."""
    import ctypes as C
    obs = _blank_obs(scale=0.1, dtmax=7.0)
    r = np.array(hand_data.geometry_cm()[1])
    S = np.zeros((48, 3))
    # every sphere off-image (behind the camera: z_unnegated < 0 -> projection flips,
    # far off): (dtmax*scale + r)^2
    S[:, 2] = 1.0  # negated frame z = +1 -> camera z = -1
    S[:, 0] = 1000.0
    Sc = S.copy()
    pen = oracle.lib.ora_depth_penalty(C.byref(ora_hand), C.byref(obs.s),
                                       Sc.ctypes.data_as(C.POINTER(C.c_double)))
    assert abs(pen - np.sum((7.0 * 0.1 + r) ** 2)) < 1e-9
    # on-image, depth 0 -> (DT*scale + r)^2 ; depth D != 0 -> max(0, D - z)^2
    obs.depth[120, 160] = 35.0
    obs.dt[121, 161] = 4.0
    S = np.zeros((48, 3))
    S[:, 0] = 1000.0
    S[:, 2] = 1.0
    S[0] = (0.0, 0.0, -30.0)            # projects to (160, 120): D = 35 -> (35-30)^2
    S[1] = (1.0 / 241.42 * 30.0 * 1.001, -1.0 / 241.42 * 30.0 * 1.001, -30.0)  # (161, 121)
    S[2] = (0.0, 0.0, -40.0)            # D = 35 < z -> 0
    Sc = S.copy()
    pen = oracle.lib.ora_depth_penalty(C.byref(ora_hand), C.byref(obs.s),
                                       Sc.ctypes.data_as(C.POINTER(C.c_double)))
    expect = 25.0 + (4.0 * 0.1 + r[1]) ** 2 + 0.0 + np.sum((7.0 * 0.1 + r[3:]) ** 2)
    assert abs(pen - expect) < 1e-9
    # the reference un-negates the caller's matrix in place (costfunc.cpp:249)
    np.testing.assert_array_equal(Sc[:, 1:], -S[:, 1:])


def test_collision_known_pair(oracle, ora_hand):
    """self_collision_penalty (costfunc.cpp:130-197): only rows 2..7 of adjacent digits
    interact; two coincident spheres contribute (r_a + r_b)^2."""
    import ctypes as C
    r = np.array(hand_data.geometry_cm()[1])
    S = np.arange(48 * 3, dtype=float).reshape(48, 3) * 100.0  # all far apart
    S[12] = S[2]  # thumb row 2 coincides with index row 12
    pen = oracle.lib.ora_collision(C.byref(ora_hand), S.ctypes.data_as(C.POINTER(C.c_double)))
    assert abs(pen - (r[2] + r[12]) ** 2) < 1e-12
    S[8] = S[3]  # index row 8 is not in the collision set
    pen2 = oracle.lib.ora_collision(C.byref(ora_hand), S.ctypes.data_as(C.POINTER(C.c_double)))
    assert pen2 == pen


def test_align_exact_fit(oracle, ora_hand):
    """A point on a sphere surface has zero alignment residual (costfunc.cpp:346-377)."""
    th = oracle_np.X0
    S = oracle.build(ora_hand, th)
    r = np.array(hand_data.geometry_cm()[1])
    # points on the surface of sphere j facing away from every other sphere's centre
    pts = S[[20, 30]] + np.array([[0, 0, 1.0]]) * r[[20, 30]][:, None]
    obs = _blank_obs(cloud=pts)
    m = oracle.correspondences(obs, S)
    import ctypes as C
    a = oracle.lib.ora_align(C.byref(ora_hand), C.byref(obs.s),
                             S.ctypes.data_as(C.POINTER(C.c_double)),
                             m.ctypes.data_as(C.POINTER(C.c_int32)))
    assert a < 1e-20 or np.any(m != [20, 30])


def test_correspondence_first_index_ties(oracle, ora_hand):
    """BFMatcher keeps the first of equal distances (OpenCV batchDistance, K = 1)."""
    S = np.zeros((48, 3))
    S[:, 0] = np.arange(48) * 10.0
    S[5] = (0.0, 2.0, 0.0)
    S[9] = (0.0, -2.0, 0.0)   # equidistant from the origin with sphere 5 ... and 0 at 0
    pts = np.array([[0.0, 0.0, 1.0], [0.0, 0.0, 0.0]])
    obs = _blank_obs(cloud=pts)
    m = oracle.correspondences(obs, S)
    assert list(m) == [0, 0]
    S[0] = (100.0, 0, 0)
    m = oracle.correspondences(obs, S)
    assert list(m) == [5, 5]   # 5 and 9 tie; the lower index wins


def test_dist_transform_known_values(oracle):
    """5x5 chamfer (OpenCV CV_DIST_L2 mask 5): a single hand pixel gives the mask
    weights 1, 1.4 (91750/65536), 2.1969 (143976/65536) around it."""
    d = np.zeros((240, 320))
    d[100, 100] = 30.0
    dt = oracle.dist_transform(d)
    assert dt[100, 100] == 0
    assert dt[100, 101] == np.float32(1.0)
    assert dt[101, 101] == np.float32(91750 / 65536)
    assert dt[102, 101] == np.float32(143976 / 65536)
    assert dt[100, 103] == np.float32(3.0)
    # monotone away from the pixel, bounded by a euclidean-ish envelope
    assert dt[0, 0] > 100 and dt[0, 0] < 1.1 * math.hypot(100, 100)


def test_preprocess_geometry(oracle):
    """Back-projection of observedmodel.cpp:130-161 and the 250-point down-sample."""
    d = np.zeros((240, 320), np.float32)
    d[120, 160] = 300.0   # principal point, 30 cm
    d[130, 170] = 400.0
    obs = oracle.preprocess(d, downsample=False)
    assert obs.n == 2
    np.testing.assert_allclose(obs.cloud[0], [0.0, -0.0, -30.0])
    np.testing.assert_allclose(obs.cloud[1], [10 * 40.0 / 241.42, -10 * 40.0 / 241.42, -40.0])
    ds = oracle.preprocess(d, downsample=True)
    assert ds.n == 250 and np.all(ds.cloud == ds.cloud[0])  # N < 250: k * 0 == row 0


def test_check_constraints_quirk_via_pso(oracle, ora_hand):
    """Above-max clamps to the MIN bound (PSO.cpp:372): with ub tiny and the particles
    pushed above it, every finite bestp dim must lie in [lb, ub]."""
    d = np.zeros((240, 320), np.float32)
    d[100:140, 140:180] = 320.0
    obs = oracle.preprocess(d)
    ub, lb, sd = oracle_np.reference_bounds()
    lb2 = lb.copy(); ub2 = ub.copy()
    lb2[6:] = 0.0
    ub2[6:] = 1e-3
    bp, bc, tr = oracle.pso_evolve(ora_hand, obs, oracle_np.X0, 8, 4, lb2, ub2, sd)
    assert np.all(bp[6:] >= lb2[6:])


def _gt_matrix(oracle, ora_hand, poses, rng, noise_mm=4.0):
    """A frames x 63 ground-truth matrix in the MSRA layout costfunc.cpp:476-507 reads:
    row f = the 21 joints of poses[f] in mm, joint j at columns 3j..3j+2, with y and z
    negated (the reference flips its model joints to compare, :492), plus noise."""
    rows = []
    for th in poses:
        _, J = oracle.build(ora_hand, th, joints=True)
        g = J * 10.0
        g[:, 1:3] *= -1
        rows.append((g + rng.normal(scale=noise_mm, size=g.shape)).ravel())
    return np.array(rows)


def test_gnd_truth_err_oracles(oracle, ora_hand, np_hand):
    """costfunc.cpp:476-507: the C oracle (Armadillo's column-major
    matrix, reshape(3,21) fill, two-accumulator sum), the numpy restatement and the
    product's host mirror agree; zero at the true pose; a known six-joint offset."""
    import hpe
    rng = np.random.default_rng(12)
    poses = hand_data.trajectory(5, seed=12)
    gt = _gt_matrix(oracle, ora_hand, poses, rng)
    for f, th in enumerate(poses[::-1]):  # estimate = a different pose of the sequence
        _, J = oracle.build(ora_hand, th, joints=True)
        Jn = np_hand.build_hand_model(th, return_joints=True)[1]
        np.testing.assert_allclose(Jn, J, rtol=0, atol=1e-12)
        ref = oracle.gnd_truth_err(J, gt, f)
        assert ref > 0
        assert abs(oracle_np.gnd_truth_err(J, gt, f) - ref) <= 4 * np.spacing(ref)
        assert hpe.gnd_truth_err(J, gt[f]) == ref  # same operation order: bit-identical
    _, J = oracle.build(ora_hand, poses[2], joints=True)
    exact = _gt_matrix(oracle, ora_hand, poses, rng, noise_mm=0.0)
    assert oracle.gnd_truth_err(J, exact, 2) == 0.0
    shifted = exact.copy()
    shifted[2, [3 * j + 1 for j in (0, 4, 8, 12, 16, 20)]] += 2.5  # 2.5 mm along y
    assert abs(oracle.gnd_truth_err(J, shifted, 2) - 15.0) < 1e-12
    # only the wrist and the five tips count: moving joint 1 changes nothing
    other = exact.copy()
    other[2, 3:6] += 100.0
    assert oracle.gnd_truth_err(J, other, 2) == 0.0
