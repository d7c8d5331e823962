"""ctypes wrapper of oracle/liboracle_hpe.so -- TEST INFRASTRUCTURE (the checker).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
"""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

ORACLE_DIR = Path(__file__).resolve().parent
LIB = ORACLE_DIR / "liboracle_hpe.so"

dp = C.POINTER(C.c_double)
fp = C.POINTER(C.c_float)
ip = C.POINTER(C.c_int32)


class OraHand(C.Structure):
    _fields_ = [("geo", C.c_double * 20), ("radii", C.c_double * 48), ("cmc", C.c_double * 5),
                ("spacing", C.c_float * 5), ("F", C.c_double * 80), ("T10", C.c_double * 80)]


class OraObs(C.Structure):
    _fields_ = [("n", C.c_int), ("cloud", dp), ("depth", dp), ("dt", fp), ("dtmax", C.c_double),
                ("scale", C.c_double), ("K", C.c_double * 9)]


class OraTrace(C.Structure):
    _fields_ = [("gbest_trace", dp), ("fmin_trace", dp), ("count_trace", ip),
                ("topo_trace", ip), ("pcost0", dp)]


def _p(a, t):
    return a.ctypes.data_as(C.POINTER(t)) if a is not None else None


class Obs:
    """Keeps the numpy buffers alive behind an OraObs."""

    def __init__(self, depth_cm, dt, cloud, scale, dtmax, K):
        self.depth = np.ascontiguousarray(depth_cm, dtype=np.float64)
        self.dt = np.ascontiguousarray(dt, dtype=np.float32)
        self.cloud = np.ascontiguousarray(cloud, dtype=np.float64).reshape(-1, 3)
        self.scale, self.dtmax = float(scale), float(dtmax)
        self.K = np.asarray(K, dtype=np.float64).reshape(9)
        self.s = OraObs(len(self.cloud), _p(self.cloud, C.c_double), _p(self.depth, C.c_double),
                        _p(self.dt, C.c_float), self.dtmax, self.scale,
                        (C.c_double * 9)(*self.K))

    @property
    def n(self):
        return len(self.cloud)


class Oracle:
    def __init__(self, lib):
        self.lib = lib
        L = lib
        L.ora_hand_init.argtypes = [C.POINTER(OraHand), dp, dp, dp, dp]
        L.ora_build_hand_model.argtypes = [C.POINTER(OraHand), dp, dp, dp]
        L.ora_correspondences.argtypes = [C.POINTER(OraObs), dp, ip]
        L.ora_align.argtypes = [C.POINTER(OraHand), C.POINTER(OraObs), dp, ip]
        L.ora_align.restype = C.c_double
        L.ora_depth_penalty.argtypes = [C.POINTER(OraHand), C.POINTER(OraObs), dp]
        L.ora_depth_penalty.restype = C.c_double
        L.ora_collision.argtypes = [C.POINTER(OraHand), dp]
        L.ora_collision.restype = C.c_double
        L.ora_cal_cost.argtypes = [C.POINTER(OraHand), C.POINTER(OraObs), dp]
        L.ora_cal_cost.restype = C.c_double
        L.ora_cal_cost2.argtypes = [C.POINTER(OraHand), C.POINTER(OraObs), dp, ip, C.c_int, dp]
        L.ora_cal_cost2.restype = C.c_double
        L.ora_eval_costs.argtypes = [C.POINTER(OraHand), C.POINTER(OraObs), dp, C.c_int, C.c_int,
                                     dp, C.c_int]
        L.ora_philox4x32_10.argtypes = [C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                        C.POINTER(C.c_uint32)]
        L.ora_u01.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32]
        L.ora_u01.restype = C.c_double
        L.ora_normals.argtypes = [C.c_uint64, C.c_int, dp]
        L.ora_pso_evolve.argtypes = [C.POINTER(OraHand), C.POINTER(OraObs), dp, C.c_int, C.c_int,
                                     dp, dp, dp, C.c_uint64, dp, dp, C.POINTER(OraTrace), C.c_int]
        L.ora_pso_optimise.argtypes = [C.POINTER(OraHand), C.POINTER(OraObs), dp, C.c_int,
                                       C.c_int, dp, dp, dp, C.c_double, C.c_double, C.c_double,
                                       C.c_uint64, dp, dp, dp, C.c_int]
        L.ora_pso_optimise.restype = C.c_int
        L.ora_refine_init_pose.argtypes = [C.POINTER(OraHand), C.POINTER(OraObs), dp]
        L.ora_refine_init_pose.restype = C.c_int
        L.ora_refine_last_margin.restype = C.c_double
        L.ora_pso_evolve_xch.argtypes = [C.POINTER(OraHand), C.POINTER(OraObs), dp, C.c_int,
                                         C.c_int, dp, dp, dp, C.POINTER(C.c_uint64), C.c_int,
                                         C.c_int, dp, dp, C.c_int]
        L.ora_pso_evolve_xch.restype = C.c_int
        L.ora_refine_ex.argtypes = [C.POINTER(OraHand), C.POINTER(OraObs), dp, C.c_int,
                                    C.POINTER(C.c_int), C.c_int, dp, C.c_int,
                                    C.POINTER(C.c_int)]
        L.ora_refine_ex.restype = C.c_int
        L.ora_rigid_spheres.argtypes = [C.POINTER(OraHand), dp, dp, dp]
        L.ora_rigid_spheres.restype = None
        L.ora_gnd_truth_err.argtypes = [dp, dp, C.c_int, C.c_int]
        L.ora_gnd_truth_err.restype = C.c_double
        L.ora_dist_transform.argtypes = [dp, fp]
        L.ora_preprocess.argtypes = [fp, C.c_int, C.c_int, C.c_double, dp, fp, dp, ip, dp, dp, dp]

    # ---- hand / model
    def hand(self, geo_cm, radii_cm, cmc=(150.0, 107.5, 89.8, 76.5, 59.6),
             spacing=(-1.86, -1.86, 0.0, 1.91, 3.84)):
        h = OraHand()
        g = np.ascontiguousarray(geo_cm, dtype=np.float64)
        r = np.ascontiguousarray(radii_cm, dtype=np.float64)
        c = np.ascontiguousarray(cmc, dtype=np.float64)
        s = np.ascontiguousarray(spacing, dtype=np.float64)
        self.lib.ora_hand_init(C.byref(h), _p(g, C.c_double), _p(r, C.c_double),
                               _p(c, C.c_double), _p(s, C.c_double))
        return h

    def build(self, h, theta, joints=False):
        th = np.ascontiguousarray(theta, dtype=np.float64)
        S = np.zeros((48, 3)); J = np.zeros((21, 3))
        self.lib.ora_build_hand_model(C.byref(h), _p(th, C.c_double), _p(S, C.c_double),
                                      _p(J, C.c_double))
        return (S, J) if joints else S

    def correspondences(self, obs, S):
        S = np.ascontiguousarray(S, dtype=np.float64)
        m = np.zeros(max(obs.n, 1), dtype=np.int32)
        self.lib.ora_correspondences(C.byref(obs.s), _p(S, C.c_double), _p(m, C.c_int32))
        return m[:obs.n]

    def terms(self, h, obs, theta, match=None):
        """(align, depth, collision) as cal_cost2 computes them."""
        th = np.ascontiguousarray(theta, dtype=np.float64)
        m = np.zeros(max(obs.n, 1), dtype=np.int32) if match is None else \
            np.ascontiguousarray(match, dtype=np.int32)
        t = np.zeros(3)
        c = self.lib.ora_cal_cost2(C.byref(h), C.byref(obs.s), _p(th, C.c_double),
                                   _p(m, C.c_int32), int(match is None), _p(t, C.c_double))
        return c, t, m[:obs.n]

    def cal_cost(self, h, obs, theta):
        th = np.ascontiguousarray(theta, dtype=np.float64)
        return self.lib.ora_cal_cost(C.byref(h), C.byref(obs.s), _p(th, C.c_double))

    def cal_cost2(self, h, obs, theta, match, compute_corr):
        th = np.ascontiguousarray(theta, dtype=np.float64)
        return self.lib.ora_cal_cost2(C.byref(h), C.byref(obs.s), _p(th, C.c_double),
                                      _p(match, C.c_int32), int(compute_corr), None)

    def eval_costs(self, h, obs, thetas, with_collision=False, nthreads=0):
        th = np.ascontiguousarray(thetas, dtype=np.float64).reshape(-1, 26)
        out = np.zeros(len(th))
        self.lib.ora_eval_costs(C.byref(h), C.byref(obs.s), _p(th, C.c_double), len(th),
                                int(with_collision), _p(out, C.c_double), int(nthreads))
        return out

    # ---- draws
    def philox(self, ctr, key):
        c = (C.c_uint32 * 4)(*ctr); k = (C.c_uint32 * 2)(*key); o = (C.c_uint32 * 4)()
        self.lib.ora_philox4x32_10(c, k, o)
        return list(o)

    def u01(self, seed, stream, gen, idx, k):
        return self.lib.ora_u01(seed, stream, gen, idx, k)

    def normals(self, seed, P):
        out = np.zeros((P, 26))
        self.lib.ora_normals(seed, P, _p(out, C.c_double))
        return out

    # ---- optimiser
    def pso_evolve(self, h, obs, x0, P, maxiter, lb, ub, sd, seed=1000, nthreads=0):
        x = np.ascontiguousarray(x0, dtype=np.float64)
        lb, ub, sd = (np.ascontiguousarray(a, dtype=np.float64) for a in (lb, ub, sd))
        bp = np.zeros(26); bc = C.c_double(0)
        G = max(maxiter - 1, 1)
        tg = np.zeros(G); tf = np.zeros(G); tc = np.zeros(G, dtype=np.int32)
        tt = np.zeros(G, dtype=np.int32); p0 = np.zeros(P)
        tr = OraTrace(_p(tg, C.c_double), _p(tf, C.c_double), _p(tc, C.c_int32),
                      _p(tt, C.c_int32), _p(p0, C.c_double))
        self.lib.ora_pso_evolve(C.byref(h), C.byref(obs.s), _p(x, C.c_double), P, maxiter,
                                _p(lb, C.c_double), _p(ub, C.c_double), _p(sd, C.c_double),
                                seed, _p(bp, C.c_double), C.byref(bc), C.byref(tr), nthreads)
        n = maxiter - 1
        return bp, bc.value, dict(gbest=tg[:n], fmin=tf[:n], count=tc[:n], topo=tt[:n],
                                  pcost0=p0)

    def pso_evolve_xch(self, h, obs, x0, P, maxiter, lb, ub, sd, seeds, every, nthreads=0):
        """R subswarms (seeds) with the opt-in per-generation exchange every `every`
        generations (hpe_set_exchange's mirror; every = 0: independent swarms).  Returns
        (bestp R x 26, bestcost R)."""
        x = np.ascontiguousarray(x0, dtype=np.float64)
        lb, ub, sd = (np.ascontiguousarray(a, dtype=np.float64) for a in (lb, ub, sd))
        sa = np.ascontiguousarray(seeds, dtype=np.uint64)
        R = len(sa)
        bp = np.zeros((R, 26)); bc = np.zeros(R)
        self.lib.ora_pso_evolve_xch(C.byref(h), C.byref(obs.s), _p(x, C.c_double), P, maxiter,
                                    _p(lb, C.c_double), _p(ub, C.c_double), _p(sd, C.c_double),
                                    _p(sa, C.c_uint64), R, every, _p(bp, C.c_double),
                                    _p(bc, C.c_double), nthreads)
        return bp, bc

    def pso_optimise(self, h, obs, x0, P, maxiter, lb, ub, sd, w, c1, c2, seed=1000,
                     nthreads=0):
        """PSO.cpp:539-712 (descent + global-best PSO); returns bestp, gbest cost and the
        gbest cost after each of the maxiter-1 generations."""
        x = np.ascontiguousarray(x0, dtype=np.float64)
        lb, ub, sd = (np.ascontiguousarray(a, dtype=np.float64) for a in (lb, ub, sd))
        bp = np.zeros(26); bc = C.c_double(0)
        tg = np.zeros(max(maxiter - 1, 1))
        self.lib.ora_pso_optimise(C.byref(h), C.byref(obs.s), _p(x, C.c_double), P, maxiter,
                                  _p(lb, C.c_double), _p(ub, C.c_double), _p(sd, C.c_double),
                                  w, c1, c2, seed, _p(bp, C.c_double), C.byref(bc),
                                  _p(tg, C.c_double), nthreads)
        return bp, bc.value, tg[:max(maxiter - 1, 0)]

    def refine(self, h, obs, x0, rigid=False):
        """refine_init_pose (PSO.cpp:183-266); rigid=True: the mirror of the GPU's default
        hand-frame refine (test infrastructure, not the reference's operation order)."""
        x = np.array(x0, dtype=np.float64)
        if rigid:
            ev = self.lib.ora_refine_ex(C.byref(h), C.byref(obs.s), _p(x, C.c_double), 1, None,
                                        0, None, 0, None)
        else:
            ev = self.lib.ora_refine_init_pose(C.byref(h), C.byref(obs.s), _p(x, C.c_double))
        return x, ev

    def refine_log(self, h, obs, x0, rigid=False, flips=(), cap=4096):
        """refine with the decision log: (x, evals, margins) where margins[k] is decision
        k's relative margin; the decisions numbered in flips are inverted (near-tie
        replay)."""
        x = np.array(x0, dtype=np.float64)
        m = np.zeros(cap)
        nd = C.c_int(0)
        fl = np.ascontiguousarray(list(flips), dtype=np.int32)
        ev = self.lib.ora_refine_ex(C.byref(h), C.byref(obs.s), _p(x, C.c_double),
                                    1 if rigid else 0, _p(fl, C.c_int) if len(fl) else None,
                                    len(fl), _p(m, C.c_double), cap, C.byref(nd))
        return x, ev, m[:min(nd.value, cap)].copy()

    def rigid_spheres(self, h, x0, theta):
        """Spheres of theta by the hand-frame mirror (centres from x0's digits), 48 x 3."""
        a = np.ascontiguousarray(x0, dtype=np.float64)
        t = np.ascontiguousarray(theta, dtype=np.float64)
        S = np.zeros(144)
        self.lib.ora_rigid_spheres(C.byref(h), _p(a, C.c_double), _p(t, C.c_double),
                                   _p(S, C.c_double))
        return S.reshape(48, 3)

    def refine_last_margin(self):
        """The smallest relative decision margin of the last refine() (test
        instrumentation, hpe_oracle.c margin_note)."""
        return float(self.lib.ora_refine_last_margin())

    # ---- evaluation
    def gnd_truth_err(self, hand_joints, gnd_truth, frame):
        """costfunc.cpp:476-507; gnd_truth (frames, 63) in mm, handed over in Armadillo's
        column-major layout as the reference's `mat &gnd_truth`."""
        hj = np.ascontiguousarray(hand_joints, dtype=np.float64).reshape(63)
        g = np.asfortranarray(np.asarray(gnd_truth, dtype=np.float64).reshape(-1, 63))
        return self.lib.ora_gnd_truth_err(_p(hj, C.c_double), _p(g, C.c_double), g.shape[0],
                                          int(frame))

    # ---- preprocessing
    def dist_transform(self, depth_cm):
        d = np.ascontiguousarray(depth_cm, dtype=np.float64)
        out = np.zeros(d.shape, dtype=np.float32)
        self.lib.ora_dist_transform(_p(d, C.c_double), _p(out, C.c_float))
        return out

    def preprocess(self, depth_mm, to_cm=True, downsample=True, focal=241.42):
        d = np.ascontiguousarray(depth_mm, dtype=np.float32).reshape(240, 320)
        dc = np.zeros((240, 320)); dt = np.zeros((240, 320), dtype=np.float32)
        cloud = np.zeros((76800, 3)); n = C.c_int32(0)
        sc = C.c_double(0); dm = C.c_double(0); K = np.zeros(9)
        self.lib.ora_preprocess(_p(d, C.c_float), int(to_cm), int(downsample), focal,
                                _p(dc, C.c_double), _p(dt, C.c_float), _p(cloud, C.c_double),
                                C.byref(n), C.byref(sc), C.byref(dm), _p(K, C.c_double))
        return Obs(dc, dt, cloud[:n.value], sc.value, dm.value, K)


_oracle = None


def load(build=True):
    global _oracle
    if _oracle is None:
        if build and not LIB.exists():
            subprocess.run(["make", "-C", str(ORACLE_DIR)], check=True,
                           stdout=subprocess.DEVNULL)
        _oracle = Oracle(C.CDLL(str(LIB)))
    return _oracle
