"""hpe -- Python host mirror of the reference's PSO / costfunc / handmodel API.

Same class and method names, argument meaning and in-place (non-const reference)
semantics as /root/reference/src/{handmodel,observedmodel,costfunc,PSO}.h, over the
C ABI of include/hpe.h (libhpe.so: gfx950 HIP kernels).  numpy arrays stand in for
Armadillo vec/mat/uvec: a 26-vector theta, a (48, 3) sphere matrix, an int32 matchId.
Every compute call runs on the GPU; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import json
from pathlib import Path

import numpy as np

from . import _lib
from ._lib import HpeError, ptr

__all__ = ["handmodel", "observedmodel", "costfunc", "PSO", "reference_hand", "HpeError",
           "gnd_truth_err",
           "Context", "preprocess_depth", "reference_bounds", "X0"]

IMG_H, IMG_W = 240, 320
# testmodel.cpp:34-40
TB_SPHERES = (2, 2, 2, 2)
FG_SPHERES = (4, 2, 2, 2)
SPACING = (-1.86, -1.86, 0.0, 1.91, 3.84)
CMC = (150.0, 107.5, 89.8, 76.5, 59.6)
X0 = np.array([0, -10, -40, 0, 3, 32, 6, 9, 8, 9, 3, 9, 9, 6, 1, 9, 8, 7, 4, 8, 7, 6, 2,
               7, 7, 7], dtype=np.float64)


def reference_bounds():
    """ub, lb, std of testmodel.cpp:74-98."""
    ub = np.zeros(26); lb = np.zeros(26); sd = np.zeros(26)
    ub[0:3], ub[3:6], lb[0:3], lb[3:6] = 180, 100, -180, -100
    for k in range(5):
        ub[6 + 4 * k:10 + 4 * k] = (15, 90, 110, 90)
        lb[6 + 4 * k:10 + 4 * k] = (-15, 0, 0, 0)
    sd[0:3], sd[3:6], sd[6:26] = 9.0, 7.0, 9.0
    return ub, lb, sd


def _check(lib, ctx, rc):
    if rc != 0:
        msg = lib.hpe_last_error(ctx).decode() if ctx else ""
        raise HpeError(f"hpe error {rc}: {msg}")


class Context:
    """One hpe_ctx: device buffers, the hand constants and one HIP stream."""

    def __init__(self, params: _lib.HandParams, device: int = 0):
        self.lib = _lib.load()
        self._h = C.c_void_p()
        rc = self.lib.hpe_create(C.byref(self._h), device, C.byref(params))
        if rc != 0:
            raise HpeError(f"hpe_create failed ({rc}): no gfx950 device {device}?")
        self.device = device
        self.frame_token = None

    @property
    def h(self):
        return self._h

    def check(self, rc):
        _check(self.lib, self._h, rc)

    def close(self):
        if self._h:
            self.lib.hpe_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- frames
    @property
    def refine_exact(self) -> bool:
        """True: refine_init_pose places spheres by the reference's DH chain on every
        evaluation; False (default): the hand-frame form (hpe_set_refine_exact).

        The two forms differ in fp64 operation order only (centres within 1e-12 cm).  Over
        the 400-frame sequence test the default form's refine took a different number of
        evaluations than the reference-order oracle on 6 frames, each a replayed near-tie
        (relative margin < 1e-13), and the tracked poses stayed within 2.2e-7 per frame and
        2.8e-7 of the free-running reference-order oracle."""
        return bool(self.lib.hpe_get_refine_exact(self.h))

    @refine_exact.setter
    def refine_exact(self, exact: bool):
        self.check(self.lib.hpe_set_refine_exact(self.h, 1 if exact else 0))

    def store_frame(self, slot, depth_cm, dt, cloud, scale, dtmax, K):
        depth_cm = np.ascontiguousarray(depth_cm, dtype=np.float64)
        dt = np.ascontiguousarray(dt, dtype=np.float32)
        cloud = np.ascontiguousarray(cloud, dtype=np.float64).reshape(-1, 3)
        f = _lib.Frame(ptr(depth_cm, C.c_double), ptr(dt, C.c_float), ptr(cloud, C.c_double),
                       len(cloud), float(scale), float(dtmax),
                       (C.c_double * 9)(*np.asarray(K, dtype=np.float64).ravel()))
        self.check(self.lib.hpe_store_frame(self._h, slot, C.byref(f)))

    def select_frame(self, slot):
        self.check(self.lib.hpe_select_frame(self._h, slot))

    def prepare_frame(self, slot, depth_mm, to_cm=True, downsample=True, focal=241.42):
        """observedmodel::next_frame on the GPU into `slot` (asynchronous)."""
        d = np.ascontiguousarray(depth_mm, dtype=np.float32).reshape(IMG_H, IMG_W)
        self.check(self.lib.hpe_prepare_frame(self._h, slot, ptr(d, C.c_float), int(to_cm),
                                              int(downsample), float(focal)))

    def pipeline_begin(self, depth_mm, to_cm=True, downsample=True, focal=241.42):
        d = np.ascontiguousarray(depth_mm, dtype=np.float32).reshape(IMG_H, IMG_W)
        self.check(self.lib.hpe_pipeline_begin(self._h, ptr(d, C.c_float), int(to_cm),
                                               int(downsample), float(focal)))

    def track_pipelined(self, num_p, refine, d_state_ptr, next_depth_mm=None):
        """Track the pipeline's current frame into the 27 device doubles at d_state_ptr and
        prepare next_depth_mm (host) as the following frame."""
        nd = None
        if next_depth_mm is not None:
            nd = np.ascontiguousarray(next_depth_mm, dtype=np.float32).reshape(IMG_H, IMG_W)
        self.check(self.lib.hpe_track_pipelined(self._h, int(num_p), int(refine),
                                                C.c_void_p(d_state_ptr),
                                                ptr(nd, C.c_float) if nd is not None else None))

    def track_sequence(self, num_p, refine, d_state_ptr, first_slot, n, frames_per_graph=0,
                       d_hist_ptr=None):
        """Track resident frames first_slot .. first_slot+n-1 in order (test_full's loop),
        frames_per_graph of them per graph launch; frame f's {bestp, cost} to d_hist_ptr +
        27 f (device, optional).  Asynchronous on the context stream."""
        self.check(self.lib.hpe_track_sequence_dev(
            self._h, int(num_p), int(refine), C.c_void_p(d_state_ptr), int(first_slot), int(n),
            int(frames_per_graph), C.c_void_p(d_hist_ptr) if d_hist_ptr else None))

    def track_raw_sequence(self, num_p, refine, d_state_ptr, d_raw_ptr, n, to_cm=True,
                           downsample=True, focal=241.42, frames_per_graph=0, d_hist_ptr=None):
        """Track n raw depth frames resident in HBM (d_raw_ptr: n x 240x320 float mm) in
        order (test_full's loop), each next frame prepared inside the previous frame's
        refine launch, frames_per_graph per graph launch; frame f's {bestp, cost} to
        d_hist_ptr + 27 f (device, optional).  Asynchronous on the context stream."""
        self.check(self.lib.hpe_track_raw_sequence_dev(
            self._h, int(num_p), int(refine), C.c_void_p(d_state_ptr), C.c_void_p(d_raw_ptr),
            int(n), int(to_cm), int(downsample), float(focal), int(frames_per_graph),
            C.c_void_p(d_hist_ptr) if d_hist_ptr else None))

    # ---- multi-GPU subswarms: the library's own per-frame exchange (hpe_subswarm_init)
    def subswarm_init(self, uid: bytes, nranks: int, rank: int):
        """Join the RCCL communicator named by uid (hpe.subswarm_unique_id() on rank 0, shared
        with every rank); collective.  Every tracked frame then ends with the all-gather of
        {bestp, cost} over the ranks and the best-of-N pick, inside the frame's graph."""
        b = (C.c_ubyte * _lib.SUBSWARM_ID_BYTES).from_buffer_copy(bytes(uid))
        self.check(self.lib.hpe_subswarm_init(self._h, b, int(nranks), int(rank)))

    def subswarm_enable(self, on, direct=False):
        """Suspend (False) / resume (True) the exchange; direct=True resumes it with direct
        launches instead of captured graphs (the library's own fallback form)."""
        self.check(self.lib.hpe_subswarm_enable(self._h, (2 if direct else 1) if on else 0))

    def subswarm_fini(self):
        self.check(self.lib.hpe_subswarm_fini(self._h))

    def subswarm_info(self, gathered=False):
        """{"nranks", "rank", "rccl_version", "in_graphs"[, "gathered": (nranks, 27) rows]}."""
        n = C.c_int32(0); r = C.c_int32(0); v = C.c_int32(0); ig = C.c_int32(0)
        self.check(self.lib.hpe_subswarm_info(self._h, C.byref(n), C.byref(r), C.byref(v),
                                              C.byref(ig), None))
        out = {"nranks": n.value, "rank": r.value, "rccl_version": v.value,
               "in_graphs": bool(ig.value)}
        if gathered and n.value:
            g = np.zeros((n.value, 27))
            self.check(self.lib.hpe_subswarm_info(self._h, None, None, None, None,
                                                  ptr(g, C.c_double)))
            out["gathered"] = g
        return out

    def graph_captures(self) -> int:
        n = C.c_uint64(0)
        self.check(self.lib.hpe_graph_captures(self._h, C.byref(n)))
        return n.value

    def frame_readback(self, slot):
        depth = np.zeros((IMG_H, IMG_W)); dt = np.zeros((IMG_H, IMG_W), dtype=np.float32)
        cloud = np.zeros((IMG_H * IMG_W, 3)); n = C.c_int32(0)
        scale = C.c_double(0); dtmax = C.c_double(0)
        self.check(self.lib.hpe_frame_readback(self._h, slot, ptr(depth, C.c_double),
                                               ptr(dt, C.c_float), ptr(cloud, C.c_double),
                                               C.byref(n), C.byref(scale), C.byref(dtmax)))
        return dict(depth_cm=depth, dt=dt, cloud=cloud[:n.value].copy(), scale=scale.value,
                    dtmax=dtmax.value)

    def render_depth(self, theta, focal=241.42):
        th = _lib.as_f64(theta, (26,))
        out = np.zeros((IMG_H, IMG_W), dtype=np.float32)
        self.check(self.lib.hpe_render_depth(self._h, ptr(th, C.c_double), focal,
                                             ptr(out, C.c_float)))
        return out


def subswarm_unique_id() -> bytes:
    """RCCL's ncclGetUniqueId (128 bytes) for hpe_subswarm_init; call on one rank."""
    lib = _lib.load()
    b = (C.c_ubyte * _lib.SUBSWARM_ID_BYTES)()
    rc = lib.hpe_subswarm_unique_id(b)
    if rc != 0:
        raise HpeError(f"hpe_subswarm_unique_id failed ({rc}): RCCL not loadable?")
    return bytes(b)


def preprocess_depth(depth_mm, to_cm=True, downsample=True, focal=241.42):
    """observedmodel preprocessing (host C++ in libhpe.so; no GPU needed)."""
    lib = _lib.load()
    d = np.ascontiguousarray(depth_mm, dtype=np.float32).reshape(IMG_H, IMG_W)
    depth_cm = np.zeros((IMG_H, IMG_W)); dt = np.zeros((IMG_H, IMG_W), dtype=np.float32)
    cloud = np.zeros((IMG_H * IMG_W, 3)); n = C.c_int32(0)
    scale = C.c_double(0); dtmax = C.c_double(0); K = np.zeros(9)
    rc = lib.hpe_preprocess_depth(ptr(d, C.c_float), int(to_cm), int(downsample), focal,
                                  ptr(depth_cm, C.c_double), ptr(dt, C.c_float),
                                  ptr(cloud, C.c_double), C.byref(n), C.byref(scale),
                                  C.byref(dtmax), ptr(K, C.c_double))
    if rc != 0:
        raise HpeError(f"hpe_preprocess_depth failed ({rc})")
    return dict(depth_cm=depth_cm, dt=dt, cloud=cloud[:n.value].copy(), scale=scale.value,
                dtmax=dtmax.value, K=K.reshape(3, 3))


class handmodel:
    """handmodel(h_geo, h_spacing, tb_spheres, fg_spheres, h_CMC, sphR)
    (handmodel.h:9-10): lengths/radii in cm."""

    def __init__(self, h_geo, h_spacing, tb_spheres, fg_spheres, h_CMC, sphR, device=0):
        p = _lib.HandParams()
        p.geo_cm[:] = [float(x) for x in np.asarray(h_geo).ravel()]
        p.radii_cm[:] = [float(x) for x in np.asarray(sphR).ravel()]
        p.cmc_deg[:] = [float(x) for x in np.asarray(h_CMC).ravel()]
        p.spacing_cm[:] = [float(x) for x in np.asarray(h_spacing).ravel()]
        p.tb_spheres[:] = [int(x) for x in np.asarray(tb_spheres).ravel()]
        p.fg_spheres[:] = [int(x) for x in np.asarray(fg_spheres).ravel()]
        self.params = p
        self.ctx = Context(p, device)
        self.spheres_radii = np.asarray(sphR, dtype=np.float64).copy()
        self.hand_joints = np.zeros((21, 3))

    def get_radii(self):
        return self.spheres_radii

    def build_hand_model(self, h_theta, sphere_centres=None):
        """handmodel.cpp:259-298; fills sphere_centres (48,3) in place if given."""
        th = _lib.as_f64(h_theta, (1, 26))
        S = np.zeros((1, 48, 3)); J = np.zeros((1, 21, 3))
        self.ctx.check(self.ctx.lib.hpe_build_spheres(self.ctx.h, ptr(th, C.c_double), 1,
                                                      ptr(S, C.c_double), ptr(J, C.c_double)))
        self.hand_joints = J[0]
        if sphere_centres is not None:
            sphere_centres[...] = S[0]
        return S[0]

    def build_batch(self, thetas):
        th = _lib.as_f64(thetas).reshape(-1, 26)
        S = np.zeros((len(th), 48, 3)); J = np.zeros((len(th), 21, 3))
        self.ctx.check(self.ctx.lib.hpe_build_spheres(self.ctx.h, ptr(th, C.c_double), len(th),
                                                      ptr(S, C.c_double), ptr(J, C.c_double)))
        return S, J


def reference_hand(device=0):
    """The hand of test_full (testmodel.cpp:33-52) from the committed misc/*.dat values."""
    d = json.loads((Path(__file__).parent / "hand_subject1.json").read_text())
    geo = np.array(d["hgeo_mm"]) / 10.0
    rad = np.array(d["rad_mm"]) / 10.0
    return handmodel(geo, SPACING, TB_SPHERES, FG_SPHERES, CMC, rad, device=device)


class observedmodel:
    """observedmodel (observedmodel.h): .bin depth frames -> cloud, depth, DT, scale."""

    _token = 0

    def __init__(self):
        self.path = "../handModelling/Release_2014_5_28/Subject1/"
        self.filename = "000001_depth.bin"
        self.imgW, self.imgH = 240, 320
        self.to_cm, self.downsample, self.focal_len = True, False, 241.42
        self._obs = None

    def init_observation(self, dpath, dfname, mm_to_cm, imW, imH, foclen, downsampling):
        self.path, self.filename = dpath, dfname
        self.imgW, self.imgH = imW, imH
        self.to_cm, self.focal_len, self.downsample = mm_to_cm, foclen, downsampling
        self.load_data()

    def load_data(self):
        """observedmodel.cpp:272-310: headerless float32 mm, 240 x 320 row-major."""
        p = Path(self.path) / self.filename
        if not p.exists():
            raise FileNotFoundError(f"error: open file for input failed! ({p})")
        self.set_depth_mm(np.fromfile(p, dtype=np.float32))

    def set_depth_mm(self, depth_mm):
        """Use an in-memory frame (e.g. a synthetic one) instead of a .bin file."""
        self._obs = preprocess_depth(depth_mm, self.to_cm, self.downsample, self.focal_len)
        observedmodel._token += 1
        self.token = observedmodel._token

    def next_frame(self, name):
        self.filename = name
        self.load_data()
        return self

    def get_ptncloud(self): return self._obs["cloud"]
    def get_depthmap(self): return self._obs["depth_cm"]
    def get_disttran(self): return self._obs["dt"]
    def get_camera_mat(self): return self._obs["K"]
    def get_img_scale(self): return self._obs["scale"]
    def get_dtmax(self): return self._obs["dtmax"]


class costfunc:
    """costfunc(handmodel*, observedmodel*) (costfunc.h:25-41)."""

    def __init__(self, handM: handmodel, observed: observedmodel):
        self.hand, self.observation = handM, observed
        self.ctx = handM.ctx

    def _sync_frame(self):
        o = self.observation
        if self.ctx.frame_token != o.token:
            d = o._obs
            self.ctx.store_frame(0, d["depth_cm"], d["dt"], d["cloud"], d["scale"],
                                 d["dtmax"], d["K"])
            self.ctx.select_frame(0)
            self.ctx.frame_token = o.token

    def cal_cost(self, theta):
        return float(self.cal_cost_batch(np.asarray(theta).reshape(1, 26))[0])

    def cal_cost_batch(self, thetas, with_collision=False, return_match=False):
        """The OpenMP particle loops of PSO.cpp:748,848 as one launch."""
        self._sync_frame()
        th = _lib.as_f64(thetas).reshape(-1, 26)
        cost = np.zeros(len(th))
        n = len(self.observation.get_ptncloud())
        m = np.zeros((len(th), n), dtype=np.int32) if return_match else None
        self.ctx.check(self.ctx.lib.hpe_eval_costs(
            self.ctx.h, ptr(th, C.c_double), len(th), int(with_collision),
            ptr(cost, C.c_double), ptr(m, C.c_int32) if m is not None else None))
        return (cost, m) if return_match else cost

    def cal_cost2(self, theta, matchId, compute_corr, debug=False):
        """costfunc.cpp:31-86; matchId (int32, len N) is filled in place when
        compute_corr, read otherwise."""
        self._sync_frame()
        th = _lib.as_f64(theta, (26,))
        if matchId.dtype != np.int32 or not matchId.flags.c_contiguous:
            raise TypeError("matchId must be a contiguous int32 array")
        cost = C.c_double(0); terms = np.zeros(3)
        self.ctx.check(self.ctx.lib.hpe_cal_cost2(self.ctx.h, ptr(th, C.c_double),
                                                  ptr(matchId, C.c_int32), int(compute_corr),
                                                  C.byref(cost), ptr(terms, C.c_double)))
        if debug:
            print(terms[0]); print(terms[1]); print(terms[2], "\n")
        self.last_terms = terms
        return cost.value

    def gnd_truth_err(self, gnd_truth, frame):
        """costfunc.cpp:476-507: wrist + finger-tip error (mm) of the hand_joints left by the
        last build_hand_model against row `frame` of gnd_truth (frames x 63)."""
        return gnd_truth_err(self.hand.hand_joints, np.asarray(gnd_truth)[frame])

    # ---- term-level API on a sphere matrix (costfunc.cpp:130-377), one launch each
    def _sphere_terms(self, spheres, matchId=None):
        self._sync_frame()
        S = _lib.as_f64(spheres, (48, 3))
        n = len(self.observation.get_ptncloud())
        corr = matchId is None
        m = np.zeros(n, dtype=np.int32) if corr else np.ascontiguousarray(matchId, dtype=np.int32)
        terms = np.zeros(3)
        self.ctx.check(self.ctx.lib.hpe_eval_spheres(self.ctx.h, ptr(S, C.c_double), 1, int(corr),
                                                     ptr(m, C.c_int32), ptr(terms, C.c_double)))
        return terms, m

    def _same_cloud(self, ptncloud):
        own = self.observation.get_ptncloud()
        if ptncloud is not own and not np.array_equal(np.asarray(ptncloud), own):
            raise ValueError("the device path evaluates the observation's own point cloud")

    def compute_correspondences(self, ptns, sphM, matchId):
        """costfunc.cpp:306-343: nearest sphere centre per cloud point (BFMatcher, fp32,
        first index on ties).  matchId (int32, len N) is filled in place."""
        self._same_cloud(ptns)
        _, m = self._sphere_terms(sphM)
        matchId[...] = m
        return matchId

    def align_models(self, spheresR, spheresM, ptncloud, matchId):
        """costfunc.cpp:346-377: (48/N) sum (|p - S[m]| - r[m])^2 with the given matchId."""
        self._same_cloud(ptncloud)
        if not np.array_equal(np.asarray(spheresR, dtype=np.float64), self.hand.spheres_radii):
            raise ValueError("the device path uses the hand's own radii")
        return float(self._sphere_terms(spheresM, matchId)[0][0])

    def depth_penalty(self, cam_mat, depthmp, spheres, disttrans, scale):
        """costfunc.cpp:227-304 on the observation's depth / DT / scale.  Like the
        reference it un-negates y and z of `spheres` in place (:249)."""
        val = float(self._sphere_terms(spheres)[0][1])
        spheres[:, 1:3] *= -1
        return val

    def self_collision_penalty(self, spheresM, spheresR):
        """costfunc.cpp:130-197: adjacent-digit sphere overlap penalty."""
        return float(self._sphere_terms(spheresM)[0][2])


def gnd_truth_err(hand_joints, gt_row):
    """costfunc.cpp:476-507 for one frame: gt_row holds 63 values (joint j at 3j..3j+2, mm);
    hand_joints is the (21, 3) cm matrix of build_hand_model (handmodel.cpp:291-296)."""
    gt = np.asarray(gt_row, dtype=np.float64).reshape(21, 3)
    hj = np.asarray(hand_joints, dtype=np.float64) * 10.0
    hj[:, 1:3] *= -1
    e = gt - hj
    d = [float(np.sqrt((e[j, 0] * e[j, 0] + e[j, 1] * e[j, 1]) + e[j, 2] * e[j, 2]))
         for j in (0, 4, 8, 12, 16, 20)]
    return ((d[0] + d[2]) + d[4]) + ((d[1] + d[3]) + d[5])


class PSO:
    """PSO (PSO.h:15-72)."""

    def __init__(self):
        self.w, self.c1, self.c2 = 0.7298, 1.49618, 1.49618  # PSO.cpp:29-34
        self.maxiter, self.minstep, self.minfunc = 100, 1e-6, 1e-6
        self.theta_max = self.theta_min = self.theta_std = None
        self.seed = 1000  # arma_rng::set_seed(1000), PSO.cpp:722

    def set_pso_params(self, upperbound, lowerbound, std, omega, phip, phig, maxIter,
                       minStep, minFunc):
        self.theta_max = _lib.as_f64(upperbound, (26,)).copy()
        self.theta_min = _lib.as_f64(lowerbound, (26,)).copy()
        self.theta_std = _lib.as_f64(std, (26,)).copy()
        self.w, self.c1, self.c2 = omega, phip, phig
        self.maxiter, self.minstep, self.minfunc = maxIter, minStep, minFunc

    def dim_restore(self, theta_in, theta_out):
        """PSO.cpp:160-180: 22 -> 26 DOF in place, each finger's DIP = 2/3 of its PIP
        (rows 13, 17, 21, 25); theta_out must hold 26 values."""
        ti = np.asarray(theta_in, dtype=np.float64).ravel()
        if ti.size < 22 or np.asarray(theta_out).size < 26:
            raise IndexError("Mat::rows(): indices out of bounds or incorrectly used")
        theta_out[0:13] = ti[0:13]
        theta_out[13] = 2. / 3 * ti[12]
        for f in range(3):  # middle, ring, little
            o, i = 14 + 4 * f, 13 + 3 * f
            theta_out[o:o + 3] = ti[i:i + 3]
            theta_out[o + 3] = 2. / 3 * ti[i + 2]

    def _push(self, ctx):
        ctx.check(ctx.lib.hpe_set_pso_params(
            ctx.h, ptr(self.theta_max, C.c_double), ptr(self.theta_min, C.c_double),
            ptr(self.theta_std, C.c_double), self.w, self.c1, self.c2, int(self.maxiter),
            self.minstep, self.minfunc))
        ctx.check(ctx.lib.hpe_set_seed(ctx.h, C.c_uint64(self.seed)))

    def pso_evolve(self, optfunc: costfunc, x0, num_particles, bestp):
        """PSO.cpp:717-886: bestp (26,) filled in place; returns 1."""
        ctx = optfunc.ctx
        optfunc._sync_frame()
        self._push(ctx)
        x = _lib.as_f64(x0, (26,))
        out = np.zeros(26); bc = C.c_double(0)
        ctx.check(ctx.lib.hpe_pso_evolve(ctx.h, ptr(x, C.c_double), int(num_particles),
                                         ptr(out, C.c_double), C.byref(bc)))
        bestp[...] = out
        self.last_gbest_cost = bc.value
        return 1

    def pso_optimise(self, optfunc: costfunc, x0, num_p, bestp):
        """PSO.cpp:539-712 (descent + global-best PSO with omega / phip / phig of
        set_pso_params): bestp (26,) filled in place; returns 1.  The gbest cost after each
        generation is kept in last_optimise_trace."""
        ctx = optfunc.ctx
        optfunc._sync_frame()
        self._push(ctx)
        x = _lib.as_f64(x0, (26,))
        out = np.zeros(26); bc = C.c_double(0)
        G = max(self.maxiter - 1, 0)
        tr = np.zeros(max(G, 1))
        ctx.check(ctx.lib.hpe_pso_optimise(ctx.h, ptr(x, C.c_double), int(num_p),
                                           ptr(out, C.c_double), C.byref(bc),
                                           ptr(tr, C.c_double), G))
        bestp[...] = out
        self.last_gbest_cost = bc.value
        self.last_optimise_trace = tr[:G]
        return 1

    def trace(self, optfunc: costfunc):
        G = self.maxiter - 1
        g = np.zeros(max(G, 1)); cnt = np.zeros(max(G, 1), dtype=np.int32)
        topo = np.zeros(max(G, 1), dtype=np.int32)
        ctx = optfunc.ctx
        ctx.check(ctx.lib.hpe_pso_trace(ctx.h, ptr(g, C.c_double), ptr(cnt, C.c_int32),
                                        ptr(topo, C.c_int32), G))
        return g[:G], cnt[:G], topo[:G]

    def refine_init_pose(self, x0, optfunc: costfunc):
        """PSO.cpp:216-266: x0 (26,) refined in place."""
        ctx = optfunc.ctx
        optfunc._sync_frame()
        x = _lib.as_f64(x0, (26,)).copy()
        ev = C.c_int32(0)
        ctx.check(ctx.lib.hpe_refine_init_pose(ctx.h, ptr(x, C.c_double), C.byref(ev)))
        x0[...] = x
        self.last_refine_evals = ev.value

    def track_frame(self, optfunc: costfunc, x0, num_particles, refine=True):
        """testmodel.cpp:126-138 in one call: refine, pso_evolve, cal_cost(bestp);
        x0 <- bestp in place; returns the frame cost."""
        ctx = optfunc.ctx
        optfunc._sync_frame()
        self._push(ctx)
        x = _lib.as_f64(x0, (26,)).copy()
        c = C.c_double(0)
        ctx.check(ctx.lib.hpe_track_frame(ctx.h, int(num_particles), int(refine),
                                          ptr(x, C.c_double), C.byref(c)))
        x0[...] = x
        return c.value
