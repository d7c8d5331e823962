"""CPU-side checks of the product library and façade (no GPU compute calls):

* libhpe.so loads and exports exactly the entry points include/hpe.h declares;
* the host preprocessing in libhpe.so (observedmodel.cpp:110-219, 272-369) equals the C
  oracle bit for bit (it runs on the host in the product too);
* error paths fail loudly: no device -> HPE_E_NODEVICE, bad sphere counts -> HPE_E_ARG;
* the C++ façade compiles against arma_lite, keeps the reference's size-error behaviour
  and aborts on an unreadable .bin like observedmodel.cpp:290-293.
"""
import ctypes as C
import re
import signal
import subprocess

import numpy as np
import pytest

import hand_data
import oracle_np

ROOT = hand_data.ROOT
PKG = ROOT / "hand-pose-estimation_amd"


def _decls():
    txt = (ROOT / "include" / "hpe.h").read_text()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return set(re.findall(r"\b(hpe_[a-z0-9_]+)\s*\(", txt))


@pytest.fixture(scope="module")
def lib():
    from hpe import _lib
    return _lib.load()


def test_abi_exports_match_header(lib):
    from hpe import _lib
    declared = _decls()
    assert len(declared) >= 20
    assert declared == set(_lib.SIGNATURES), declared ^ set(_lib.SIGNATURES)
    nm = subprocess.run(["nm", "-D", "--defined-only", str(PKG / "libhpe.so")],
                        capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (hpe_[a-z0-9_]+)$", nm, flags=re.M))
    assert declared <= exported, declared - exported
    assert lib.hpe_abi_version() == 1


def test_abi_no_cxx_types_in_header():
    txt = (ROOT / "include" / "hpe.h").read_text()
    assert 'extern "C"' in txt
    for bad in ("std::", "torch", "template", "class ", "hipStream_t"):
        assert bad not in re.sub(r"/\*.*?\*/", "", txt, flags=re.S)


def test_errors_fail_loudly(lib):
    from hpe import _lib
    p = _lib.HandParams()
    h = C.c_void_p()
    assert lib.hpe_create(C.byref(h), 0, C.byref(p)) == _lib.HPE_E_ARG  # sphere counts
    p.tb_spheres[:] = (2, 2, 2, 2)
    p.fg_spheres[:] = (4, 2, 2, 2)
    import torch
    if not torch.cuda.is_available():
        assert lib.hpe_create(C.byref(h), 0, C.byref(p)) == _lib.HPE_E_NODEVICE
    assert lib.hpe_create(C.byref(h), 10 ** 6, C.byref(p)) == _lib.HPE_E_NODEVICE
    assert lib.hpe_eval_costs(None, None, 1, 0, None, None) == _lib.HPE_E_ARG
    # the subswarm exchange's entry points (no context / no buffer: refused, nothing loaded)
    assert lib.hpe_subswarm_unique_id(None) == _lib.HPE_E_ARG
    idb = (C.c_ubyte * _lib.SUBSWARM_ID_BYTES)()
    assert lib.hpe_subswarm_init(None, idb, 2, 0) == _lib.HPE_E_ARG
    assert lib.hpe_subswarm_enable(None, 1) == _lib.HPE_E_ARG
    assert lib.hpe_subswarm_fini(None) == _lib.HPE_E_ARG
    assert lib.hpe_subswarm_info(None, None, None, None, None, None) == _lib.HPE_E_ARG
    assert lib.hpe_pick_best(None, None, 2, None) == _lib.HPE_E_ARG
    import hpe
    with pytest.raises(hpe.HpeError):
        hpe.Context(p, device=10 ** 6)


@pytest.mark.parametrize("downsample", [True, False])
def test_host_preprocess_matches_oracle(oracle, np_hand, downsample):
    import hpe
    for seed in (0, 7):
        th = hand_data.trajectory(3, seed=seed)[-1]
        d = oracle_np.render_depth_mm(np_hand, th)
        a = hpe.preprocess_depth(d, downsample=downsample)
        b = oracle.preprocess(d, downsample=downsample)
        np.testing.assert_array_equal(a["cloud"], b.cloud)
        np.testing.assert_array_equal(a["dt"], b.dt)
        np.testing.assert_array_equal(a["depth_cm"], b.depth)
        assert a["scale"] == b.scale and a["dtmax"] == b.dtmax
        np.testing.assert_array_equal(a["K"].ravel(), np.asarray(b.K).ravel())


def test_host_preprocess_empty_frame(oracle):
    import hpe
    d = np.zeros((240, 320), np.float32)
    a = hpe.preprocess_depth(d, downsample=False)
    b = oracle.preprocess(d, downsample=False)
    assert len(a["cloud"]) == 0 == b.n
    assert np.isnan(a["scale"]) and np.isnan(b.scale)
    np.testing.assert_array_equal(a["dt"], b.dt)


@pytest.fixture(scope="module")
def facade_host(tmp_path_factory):
    if not (PKG / "libhpe_facade.so").exists():
        subprocess.run(["make", "-C", str(PKG), "libhpe_facade.so"], check=True, timeout=600)
    exe = tmp_path_factory.mktemp("fh") / "facade_host"
    subprocess.run(["g++", "-O1", "-std=c++17", "-Wall", "-o", str(exe),
                    str(ROOT / "tests" / "cpp" / "facade_host.cpp"), f"-I{PKG / 'facade'}",
                    f"-L{PKG}", "-lhpe_facade", "-lhpe", f"-Wl,-rpath,{PKG}"],
                   check=True, timeout=120)
    return exe


def test_facade_size_errors_zero_fill(facade_host):
    out = subprocess.run([str(facade_host)], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "facade_host ok" in out.stdout
    assert "20 params are needed" in out.stdout  # handmodel.cpp:178-181 message


def test_facade_missing_bin_aborts(facade_host):
    out = subprocess.run([str(facade_host), "abort"], capture_output=True, text=True, timeout=60)
    assert out.returncode == -signal.SIGABRT
    assert "open file for input failed" in out.stderr


def test_dim_restore_python_mirror():
    """PSO::dim_restore (PSO.cpp:160-180) in the Python mirror: rows copied, DIP = 2/3 PIP."""
    import hpe
    ti = 1.5 * np.arange(22) - 7.25
    out = np.zeros(26)
    hpe.PSO().dim_restore(ti, out)
    src = list(range(13)) + [-12, 13, 14, 15, -15, 16, 17, 18, -18, 19, 20, 21, -21]
    want = np.array([ti[k] if k >= 0 else 2. / 3 * ti[-k] for k in src])
    assert np.array_equal(out, want)
    with pytest.raises(IndexError):
        hpe.PSO().dim_restore(np.zeros(20), out)


def test_gnd_truth_err_host():
    """costfunc.cpp:476-507 restated on the host joints: zero at the true pose, and the
    six-joint sum for a known offset."""
    import hpe
    rng = np.random.default_rng(0)
    hj = rng.normal(size=(21, 3))
    gt = hj * 10.0
    gt[:, 1:3] *= -1
    assert hpe.gnd_truth_err(hj, gt.ravel()) == 0.0
    gt2 = gt.copy()
    gt2[[0, 4, 8, 12, 16, 20], 0] += 3.0  # 3 mm along x on the wrist and the five tips
    assert abs(hpe.gnd_truth_err(hj, gt2.ravel()) - 18.0) < 1e-12
