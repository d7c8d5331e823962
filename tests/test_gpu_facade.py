"""GPU parity of the host C++ façade (hpe_facade.hpp: the reference's handmodel /
observedmodel / costfunc / PSO names over the C ABI) and of the term-level costfunc API.

hpe_track is test_full (testmodel.cpp:27-146) written against the façade: the same
.bin frames, hand files and call sequence.  Its per-frame costs and poses must match the
C oracle running the same sequence (tolerances as test_gpu_parity.py: pose 1e-6,
cost relative 1e-8).
"""
import json
import re
import subprocess

import numpy as np
import pytest

import hand_data
from hand_data import REFINE_RIGID
import oracle_np

pytestmark = pytest.mark.gpu

PKG = hand_data.ROOT / "hand-pose-estimation_amd"


def _write_inputs(tmp_path, np_hand, poses):
    d = json.loads(hand_data.HAND_JSON.read_text())
    hand = tmp_path / "misc"
    hand.mkdir()
    (hand / "hgeo.dat").write_text("\n".join(repr(float(v)) for v in d["hgeo_mm"]) + "\n")
    (hand / "rad.dat").write_text("\n".join(repr(float(v)) for v in d["rad_mm"]) + "\n")
    frames = tmp_path / "Subject1"
    frames.mkdir()
    depth = []
    for f, th in enumerate(poses):
        dm = oracle_np.render_depth_mm(np_hand, th).astype(np.float32)
        dm.tofile(frames / f"{f:06d}_depth.bin")
        depth.append(dm)
    return hand, frames, depth


def _run_track(hand, frames, n, P, maxiter, fused, pose_out):
    exe = PKG / "hpe_track"
    assert exe.exists(), "build hand-pose-estimation_amd (make) first"
    out = subprocess.run([str(exe), "--hand", str(hand), "--frames", str(frames), "--n", str(n),
                          "--particles", str(P), "--maxiter", str(maxiter), "--refine", "1",
                          "--fused", str(fused), "--pose-out", str(pose_out)],
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    costs = [float(m) for m in re.findall(r"frame\d{6}-cost: (\S+)", out.stdout)]
    assert len(costs) == n, out.stdout
    return np.array(costs), np.loadtxt(pose_out).reshape(n, 26)


def test_cpp_driver_matches_oracle(tmp_path, oracle, ora_hand, np_hand):
    n, P, maxiter = 3, 32, 6
    poses = hand_data.trajectory(n, seed=21)
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
    ref_c, ref_x = np.array(ref_c), np.array(ref_x)
    for fused in (0, 1):
        c, xs = _run_track(hand, frames, n, P, maxiter, fused, tmp_path / f"poses{fused}.txt")
        np.testing.assert_allclose(xs, ref_x, rtol=0, atol=1e-6)
        np.testing.assert_allclose(c, ref_c, rtol=1e-8, atol=0)


def test_cpp_facade_api(tmp_path, np_hand):
    """tests/cpp/facade_gpu.cpp drives every façade method once on the GPU and prints
    the values; they must equal the Python mirror's (same library, same inputs)."""
    src = hand_data.ROOT / "tests" / "cpp" / "facade_gpu.cpp"
    exe = tmp_path / "facade_gpu"
    subprocess.run(["g++", "-O1", "-std=c++17", "-o", str(exe), str(src),
                    f"-I{PKG / 'facade'}", f"-L{PKG}", "-lhpe_facade", "-lhpe",
                    f"-Wl,-rpath,{PKG}"], check=True, timeout=120)
    hand, frames, depth = _write_inputs(tmp_path, np_hand, hand_data.trajectory(1, seed=3))
    out = subprocess.run([str(exe), str(hand), str(frames) + "/"], capture_output=True,
                         text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    vals = dict(l.split("=", 1) for l in out.stdout.split() if "=" in l)
    import hpe
    gh = hpe.reference_hand(0)
    om = hpe.observedmodel(); om.downsample = True; om.set_depth_mm(depth[0])
    cf = hpe.costfunc(gh, om)
    th = oracle_np.X0 + 1.5
    assert float(vals["cal_cost"]) == cf.cal_cost(th)
    m = np.zeros(len(om.get_ptncloud()), np.int32)
    assert float(vals["cal_cost2"]) == cf.cal_cost2(th, m, True)
    S = gh.build_hand_model(th)
    assert float(vals["S0x"]) == S[0, 0] and float(vals["S47z"]) == S[47, 2]
    assert float(vals["align"]) == cf.align_models(gh.get_radii(), S, om.get_ptncloud(), m)
    assert float(vals["collision"]) == cf.self_collision_penalty(S, gh.get_radii())
    assert float(vals["depth"]) == cf.depth_penalty(None, None, S.copy(), None, 0.0)
    assert int(vals["m_sum"]) == int(m.sum())


def test_term_api_matches_oracle(oracle, ora_hand, np_hand):
    """align_models / depth_penalty / self_collision_penalty / compute_correspondences on a
    sphere matrix (costfunc.cpp:130-377) against the oracle's terms."""
    import hpe
    gh = hpe.reference_hand(0)
    truth = hand_data.trajectory(2, seed=8)[1]
    d = oracle_np.render_depth_mm(np_hand, truth)
    obs = oracle.preprocess(d)
    om = hpe.observedmodel(); om.downsample = True; om.set_depth_mm(d)
    cf = hpe.costfunc(gh, om)
    rng = np.random.default_rng(4)
    for th in hand_data.random_thetas(rng, 6, x0=truth, spread=0.5):
        cr, tr, mr = oracle.terms(ora_hand, obs, th)
        S = oracle.build(ora_hand, th)
        m = np.zeros(obs.n, np.int32)
        cf.compute_correspondences(om.get_ptncloud(), S, m)
        assert np.array_equal(m, mr)
        np.testing.assert_allclose(cf.align_models(gh.get_radii(), S, om.get_ptncloud(), m),
                                   tr[0], rtol=1e-9)
        Sd = S.copy()
        np.testing.assert_allclose(cf.depth_penalty(None, None, Sd, None, 0.0), tr[1],
                                   rtol=1e-9, atol=1e-300)
        np.testing.assert_array_equal(Sd[:, 1:], -S[:, 1:])  # un-negated like :249
        np.testing.assert_allclose(cf.self_collision_penalty(S, gh.get_radii()), tr[2],
                                   rtol=1e-9, atol=1e-300)


def test_gnd_truth_err_gpu_joints(tmp_path, oracle, ora_hand, np_hand):
    """costfunc::gnd_truth_err (costfunc.cpp:476-507) on joints built by
    the GPU FK (hpe_build_spheres joints_out), through the Python mirror and through the
    C++ façade (arma mat, column-major, reshape(3,21) fill, y/z flip), against the C
    oracle on its own FK joints.  Tolerance: the joints agree to 1e-9 cm (fp64 FK, only
    sin/cos rounding differs), so the mm error sums agree to 1e-7 mm absolute."""
    import hpe
    from test_oracle_kat import _gt_matrix
    rng = np.random.default_rng(41)
    poses = hand_data.trajectory(6, seed=41)
    gt = _gt_matrix(oracle, ora_hand, poses, rng)
    est = poses[::-1].copy()  # score pose 5-f against ground-truth row f
    gh = hpe.reference_hand(0)
    om = hpe.observedmodel(); om.downsample = True
    om.set_depth_mm(oracle_np.render_depth_mm(np_hand, poses[0]))
    cf = hpe.costfunc(gh, om)
    ref, mirror = [], []
    for f, th in enumerate(est):
        _, J = oracle.build(ora_hand, th, joints=True)
        ref.append(oracle.gnd_truth_err(J, gt, f))
        gh.build_hand_model(th)  # GPU FK -> hand_joints
        np.testing.assert_allclose(gh.hand_joints, J, rtol=0, atol=1e-9)
        mirror.append(cf.gnd_truth_err(gt, f))
    np.testing.assert_allclose(mirror, ref, rtol=0, atol=1e-7)
    # the C++ façade on the same inputs
    src = hand_data.ROOT / "tests" / "cpp" / "facade_gpu.cpp"
    exe = tmp_path / "facade_gpu"
    subprocess.run(["g++", "-O1", "-std=c++17", "-o", str(exe), str(src),
                    f"-I{PKG / 'facade'}", f"-L{PKG}", "-lhpe_facade", "-lhpe",
                    f"-Wl,-rpath,{PKG}"], check=True, timeout=120)
    hand, frames, _ = _write_inputs(tmp_path, np_hand, poses[:1])
    gtf, pf = tmp_path / "gt.txt", tmp_path / "poses.txt"
    with open(gtf, "w") as fh:
        fh.write(f"{len(gt)}\n")
        np.savetxt(fh, gt, fmt="%.17g")
    np.savetxt(pf, est, fmt="%.17g")
    out = subprocess.run([str(exe), str(hand), str(frames) + "/", str(gtf), str(pf)],
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    vals = dict(l.split("=", 1) for l in out.stdout.split() if "=" in l)
    fac = [float(vals[f"gte{f}"]) for f in range(len(est))]
    np.testing.assert_allclose(fac, ref, rtol=0, atol=1e-7)
    assert fac == mirror  # same joints, same operation order


def test_c_subswarm_exchange_world1(tmp_path, np_hand):
    """tests/cpp/subswarm_c.c: the library's subswarm exchange driven from plain C through
    include/hpe.h alone (INTEGRATION.md "Several GPUs"; no torch, no HIP headers): the
    test_full loop over host frames tracked plain, on a one-rank communicator, and in the
    exchange's direct-launch form -- every frame's {pose, cost} bit-identical."""
    src = hand_data.ROOT / "tests" / "cpp" / "subswarm_c.c"
    exe = tmp_path / "subswarm_c"
    subprocess.run(["gcc", "-O1", "-std=c11", "-o", str(exe), str(src),
                    f"-I{hand_data.ROOT / 'include'}", f"-L{PKG}", "-lhpe",
                    f"-Wl,-rpath,{PKG}"], check=True, timeout=120)
    poses = hand_data.trajectory(6, seed=17)
    hand, _, _ = _write_inputs(tmp_path, np_hand, poses[:0])
    pf = tmp_path / "poses.txt"
    pf.write_text("\n".join(" ".join(repr(float(v)) for v in p) for p in poses) + "\n")
    out = subprocess.run([str(exe), str(hand), str(pf), str(len(poses))], capture_output=True,
                         text=True, timeout=240)
    assert out.returncode == 0, (out.returncode, out.stderr[-2000:])
    assert "subswarm_c ok" in out.stdout and "nranks=1" in out.stdout, out.stdout
    print(out.stdout.strip())
