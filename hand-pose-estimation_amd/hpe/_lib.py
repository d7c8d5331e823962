"""ctypes binding of include/hpe.h (libhpe.so, built in-tree by the package Makefile).

The product path has no CPU fallback: if libhpe.so is missing or no gfx950 device is
visible, the calls raise.  The binding only marshals plain pointers and sizes.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

PKG_DIR = Path(__file__).resolve().parent.parent  # hand-pose-estimation_amd/
LIB_PATH = PKG_DIR / "libhpe.so"

PROF_PSO_GEN, PROF_REFINE, PROF_PSO_INIT, PROF_PSO_FINAL, PROF_PREP = 0, 1, 2, 3, 4
PROF_OPT_DESCENT, PROF_OPT_MOVE, PROF_SWARM_BEST, PROF_EXCHANGE = 5, 6, 7, 8
SUBSWARM_ID_BYTES = 128
HPE_OK, HPE_E_ARG, HPE_E_HIP, HPE_E_STATE, HPE_E_NOMEM, HPE_E_NODEVICE = 0, -1, -2, -3, -4, -5

dp = C.POINTER(C.c_double)
fp = C.POINTER(C.c_float)
ip = C.POINTER(C.c_int32)


class HandParams(C.Structure):
    _fields_ = [("geo_cm", C.c_double * 20), ("radii_cm", C.c_double * 48),
                ("cmc_deg", C.c_double * 5), ("spacing_cm", C.c_double * 5),
                ("tb_spheres", C.c_int32 * 4), ("fg_spheres", C.c_int32 * 4)]


class Frame(C.Structure):
    _fields_ = [("depth_cm", dp), ("dt", fp), ("cloud", dp), ("n", C.c_int32),
                ("scale", C.c_double), ("dtmax", C.c_double), ("K", C.c_double * 9)]


# name -> (restype, argtypes); the list IS the exported C ABI (tests check it against
# include/hpe.h)
SIGNATURES = {
    "hpe_abi_version": (C.c_int, []),
    "hpe_last_error": (C.c_char_p, [C.c_void_p]),
    "hpe_create": (C.c_int, [C.POINTER(C.c_void_p), C.c_int, C.POINTER(HandParams)]),
    "hpe_destroy": (C.c_int, [C.c_void_p]),
    "hpe_stream": (C.c_void_p, [C.c_void_p]),
    "hpe_sync": (C.c_int, [C.c_void_p]),
    "hpe_preprocess_depth": (C.c_int, [fp, C.c_int, C.c_int, C.c_double, dp, fp, dp, ip, dp,
                                       dp, dp]),
    "hpe_store_frame": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(Frame)]),
    "hpe_select_frame": (C.c_int, [C.c_void_p, C.c_int]),
    "hpe_set_frame": (C.c_int, [C.c_void_p, C.POINTER(Frame)]),
    "hpe_prepare_frame": (C.c_int, [C.c_void_p, C.c_int, fp, C.c_int, C.c_int, C.c_double]),
    "hpe_frame_readback": (C.c_int, [C.c_void_p, C.c_int, dp, fp, dp, ip, dp, dp]),
    "hpe_pipeline_begin": (C.c_int, [C.c_void_p, fp, C.c_int, C.c_int, C.c_double]),
    "hpe_track_pipelined": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_void_p, fp]),
    "hpe_track_raw_sequence_dev": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_void_p,
                                             C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_double,
                                             C.c_int, C.c_void_p]),
    "hpe_build_spheres": (C.c_int, [C.c_void_p, dp, C.c_int, dp, dp]),
    "hpe_eval_costs": (C.c_int, [C.c_void_p, dp, C.c_int, C.c_int, dp, ip]),
    "hpe_cal_cost2": (C.c_int, [C.c_void_p, dp, ip, C.c_int, dp, dp]),
    "hpe_eval_spheres": (C.c_int, [C.c_void_p, dp, C.c_int, C.c_int, ip, dp]),
    "hpe_set_pso_params": (C.c_int, [C.c_void_p, dp, dp, dp, C.c_double, C.c_double,
                                     C.c_double, C.c_int, C.c_double, C.c_double]),
    "hpe_set_seed": (C.c_int, [C.c_void_p, C.c_uint64]),
    "hpe_pso_evolve": (C.c_int, [C.c_void_p, dp, C.c_int, dp, dp]),
    "hpe_pso_optimise": (C.c_int, [C.c_void_p, dp, C.c_int, dp, dp, dp, C.c_int]),
    "hpe_pso_trace": (C.c_int, [C.c_void_p, dp, ip, ip, C.c_int]),
    "hpe_refine_init_pose": (C.c_int, [C.c_void_p, dp, ip]),
    "hpe_set_refine_exact": (C.c_int, [C.c_void_p, C.c_int]),
    "hpe_graph_captures": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint64)]),
    "hpe_set_exchange": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]),
    "hpe_pick_best": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]),
    "hpe_subswarm_unique_id": (C.c_int, [C.c_void_p]),
    "hpe_subswarm_init": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_int]),
    "hpe_subswarm_enable": (C.c_int, [C.c_void_p, C.c_int]),
    "hpe_subswarm_fini": (C.c_int, [C.c_void_p]),
    "hpe_subswarm_info": (C.c_int, [C.c_void_p, ip, ip, ip, ip, dp]),
    "hpe_get_refine_exact": (C.c_int, [C.c_void_p]),
    "hpe_track_frame": (C.c_int, [C.c_void_p, C.c_int, C.c_int, dp, dp]),
    "hpe_track_frame_dev": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_void_p]),
    "hpe_track_sequence_dev": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int,
                                         C.c_int, C.c_int, C.c_void_p]),
    "hpe_profile_enable": (C.c_int, [C.c_void_p, C.c_int]),
    "hpe_profile_read": (C.c_int, [C.c_void_p, ip, dp, dp, dp]),
    "hpe_profile_read_kernel": (C.c_int, [C.c_void_p, C.c_int, ip, dp, dp, dp]),
    "hpe_refine_eval_count": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint64), C.c_int]),
    "hpe_render_depth": (C.c_int, [C.c_void_p, dp, C.c_double, fp]),
    "hpe_debug_stamps": (C.c_int, [C.POINTER(C.c_uint64)]),
}

# hpe_exchange_fn: int (*)(void *user, double *d_ext, int generation)
EXCHANGE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_int)

_lib = None


def load(path: os.PathLike | str | None = None):
    """Load libhpe.so (raises if it is absent: there is no fallback path)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    # HPE_LIB_VARIANT=<file in the package dir>: A/B a second in-tree build (tools only)
    variant = os.environ.get("HPE_LIB_VARIANT")
    p = Path(path) if path else (PKG_DIR / variant if variant else LIB_PATH)
    if not p.exists():
        raise RuntimeError(f"{p} not built: run `make -C {PKG_DIR}` (no CPU fallback exists)")
    lib = C.CDLL(str(p))
    for name, (res, args) in SIGNATURES.items():
        if variant and not path and not hasattr(lib, name):
            continue  # an older build under A/B: entry points added since are absent
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    if path is None:
        _lib = lib
    return lib


class HpeError(RuntimeError):
    pass


def ptr(a: np.ndarray, ctype):
    return a.ctypes.data_as(C.POINTER(ctype))


def as_f64(a, shape=None):
    a = np.ascontiguousarray(a, dtype=np.float64)
    if shape is not None:
        a = a.reshape(shape)
    return a
