"""oracle/oracle_np.py -- independent numpy restatement of the reference hot path.

TEST INFRASTRUCTURE ONLY.  Used by tests/ (cross-check of the C oracle, golden
fixture generation via tests/golden/make_golden.py) and never by the product.

It is written independently of oracle/hpe_oracle.c (vectorised over spheres /
points / pixels, numpy reductions) so that agreement between the two is
evidence that both restate the reference correctly.  Citations are
/root/reference/src file:line.  Parity status: see oracle/hpe_oracle.h.
"""
from __future__ import annotations

import math
import numpy as np

PI = math.acos(-1.0)  # fingermodel.cpp:8
NS, DOF, H, W = 48, 26, 240, 320

# testmodel.cpp:34-40
TB_SPHERES = (2, 2, 2, 2)
FG_SPHERES = (4, 2, 2, 2)
SPACING = (-1.86, -1.86, 0.0, 1.91, 3.84)
CMC = (150.0, 107.5, 89.8, 76.5, 59.6)
X0 = np.array([0, -10, -40, 0, 3, 32, 6, 9, 8, 9, 3, 9, 9, 6, 1, 9, 8, 7, 4, 8, 7, 6, 2,
               7, 7, 7], dtype=np.float64)


def reference_bounds():
    """testmodel.cpp:74-98: ub, lb, std."""
    ub = np.zeros(26); lb = np.zeros(26); sd = np.zeros(26)
    ub[0:3] = 180; ub[3:6] = 100
    lb[0:3] = -180; lb[3:6] = -100
    for k in range(5):
        ub[6 + 4 * k:10 + 4 * k] = (15, 90, 110, 90)
        lb[6 + 4 * k:10 + 4 * k] = (-15, 0, 0, 0)
    sd[0:3] = 9.0; sd[3:6] = 7.0; sd[6:26] = 9.0
    return ub, lb, sd


def deg2rad(a):
    return a / 180.0 * PI


def _rz(a, L=0.0):
    c, s = math.cos(a), math.sin(a)
    return np.array([[c, -s, 0, L * c], [s, c, 0, L * s], [0, 0, 1, 0], [0, 0, 0, 1.0]])


def _mm(A, B):
    """4x4 product with k-ordered, non-fused sums (python floats)."""
    C = np.zeros((4, 4))
    for i in range(4):
        for j in range(4):
            acc = float(A[i, 0]) * float(B[0, j])
            for k in range(1, 4):
                acc = acc + float(A[i, k]) * float(B[k, j])
            C[i, j] = acc
    return C


class Hand:
    """handmodel + finger/thumb fixed transforms (handmodel.cpp:10-85,
    fingermodel.cpp:106-132, thumbmodel.cpp:112-138)."""

    def __init__(self, geo_cm, radii_cm, cmc=CMC, spacing=SPACING):
        self.geo = np.asarray(geo_cm, dtype=np.float64).reshape(5, 4)
        self.radii = np.asarray(radii_cm, dtype=np.float64)
        self.cmc = np.asarray(cmc, dtype=np.float64)
        self.spacing = np.asarray(spacing, dtype=np.float32)  # float member
        self.F, self.T10 = [], []
        for d in range(5):
            L0 = float(self.geo[d, 0])
            sp = self.spacing[d]
            n = deg2rad(float(self.cmc[d]))
            self.F.append(_rz(n, L0))
            sp2 = float(np.float32(sp * sp))           # float*float product
            a = math.sqrt(L0 * L0 + sp2 - 2 * L0 * float(sp) * math.cos(n))
            beta = math.asin(math.sin(n) * float(sp) / a)
            T = _rz(beta)
            if d == 0:
                T[0, 3] = -a * math.cos(beta); T[1, 3] = -a * math.sin(beta)
            else:
                T[0, 3] = -L0 * math.sin(n) * math.cos(beta)
                T[1, 3] = -L0 * math.sin(n) * math.sin(beta)
            self.T10.append(T)

    # fingermodel.cpp:270-317 / thumbmodel.cpp:276-318
    def _joints(self, d, th4, gb, gp):
        g = self.geo[d]
        a = [deg2rad(float(t)) for t in th4]
        A = np.array([[math.cos(a[0]), 0, -math.sin(a[0]), 0],
                      [math.sin(a[0]), 0, math.cos(a[0]), 0], [0, -1, 0, 0], [0, 0, 0, 1.0]])
        if d == 0:
            pc = deg2rad(float(self.cmc[0])) + PI
            c2, s2 = math.cos(a[1]), math.sin(a[1])
            B = np.array([[c2, -s2 * math.cos(pc), s2 * math.sin(pc), g[1] * c2],
                          [s2, c2 * math.cos(pc), -c2 * math.sin(pc), g[1] * s2],
                          [0, math.sin(pc), math.cos(pc), 0], [0, 0, 0, 1.0]])
        else:
            B = _rz(a[1], g[1])
        C3, C4 = _rz(a[2], g[2]), _rz(a[3], g[3])
        tz, ty, tx = deg2rad(float(gb[0]) + 180), deg2rad(float(gb[1])), deg2rad(float(gb[2]))
        Rz = _rz(tz)
        Ry = np.array([[math.cos(ty), 0, math.sin(ty), 0], [0, 1, 0, 0],
                       [-math.sin(ty), 0, math.cos(ty), 0], [0, 0, 0, 1.0]])
        Rx = np.array([[1, 0, 0, 0], [0, math.cos(tx), -math.sin(tx), 0],
                       [0, math.sin(tx), math.cos(tx), 0], [0, 0, 0, 1.0]])
        T00 = np.eye(4); T00[0:3, 3] = gp
        cur = _mm(T00, _mm(_mm(Rz, Ry), Rx))
        chain = [self.F[d], _mm(A, B), C3, C4]
        J = np.zeros((5, 3))
        for i in range(4):
            if i == 1:
                J[0] = _mm(cur, self.T10[d])[0:3, 3]
            cur = _mm(cur, chain[i])
            J[i + 1] = cur[0:3, 3]
        return J

    def build_hand_model(self, theta, return_joints=False):
        """handmodel.cpp:259-298 -> S (48,3), y and z negated."""
        th = np.asarray(theta, dtype=np.float64)
        rows, joints = [], []
        for d in range(5):
            J = self._joints(d, th[6 + 4 * d:10 + 4 * d], th[0:3], th[3:6])
            joints.append(J)
            ns = TB_SPHERES if d == 0 else FG_SPHERES
            for i in range(4):
                if i == 0 and d != 0:
                    t = 1.0 / (ns[0] - 1)
                    js = range(0, ns[0])
                else:
                    t = 1.0 / ns[i]
                    js = range(1, ns[i] + 1)
                for j in js:
                    rows.append((1.0 - t * j) * J[i] + (t * j) * J[i + 1])
        S = np.array(rows)
        S[:, 1:3] *= -1
        if return_joints:
            hj = np.zeros((21, 3))
            hj[0] = th[3:6]
            for k, d in enumerate((1, 2, 3, 4, 0)):
                hj[1 + 4 * k:5 + 4 * k] = joints[d][1:5]
            return S, hj
        return S


def correspondences(cloud, S):
    """costfunc.cpp:306-343 (BFMatcher NORM_L2 on float32, first minimum)."""
    q = np.asarray(cloud, dtype=np.float64).astype(np.float32)
    s = np.asarray(S, dtype=np.float64).astype(np.float32)
    t = q[:, None, :] - s[None, :, :]
    d2 = (t[..., 0] * t[..., 0] + t[..., 1] * t[..., 1]) + t[..., 2] * t[..., 2]
    dist = np.sqrt(d2.astype(np.float32))
    return np.argmin(dist, axis=1).astype(np.int32)  # first occurrence on ties


def align(radii, S, cloud, match):
    """costfunc.cpp:346-377."""
    d = cloud - S[match]
    nd = np.sqrt((d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2])
    return float(np.sum((nd - radii[match]) ** 2)) * (48.0 / len(cloud))


def depth_penalty(radii, S, K, depth, dt, dtmax, scale):
    """costfunc.cpp:227-304 (on un-negated centres)."""
    x, y, z = S[:, 0], -S[:, 1], -S[:, 2]
    pu = (K[0, 0] * x + K[0, 1] * y) + K[0, 2] * z
    pv = (K[1, 0] * x + K[1, 1] * y) + K[1, 2] * z
    pw = (K[2, 0] * x + K[2, 1] * y) + K[2, 2] * z
    with np.errstate(invalid="ignore", divide="ignore"):
        u, v = np.floor(pu / pw), np.floor(pv / pw)
    pen = 0.0
    for i in range(NS):
        if 0 <= u[i] < W and 0 <= v[i] < H:
            D = depth[int(v[i]), int(u[i])]
            if D != 0:
                pen += max(0.0, D - z[i]) ** 2
            else:
                pen += (float(dt[int(v[i]), int(u[i])]) * scale + radii[i]) ** 2
        else:
            pen += (dtmax * scale + radii[i]) ** 2
    return pen


def collision(radii, S):
    """costfunc.cpp:130-197."""
    base = (2, 12, 22, 32, 42)
    pen = 0.0
    for p in range(4):
        a = base[p] + np.arange(36) // 6
        b = base[p + 1] + np.arange(36) % 6
        d = S[b] - S[a]
        dist = np.sqrt((d[:, 0] ** 2 + d[:, 1] ** 2) + d[:, 2] ** 2)
        v = (radii[b] + radii[a]) - dist
        pen += float(np.sum(v[v > 0] ** 2))
    return pen


def gnd_truth_err(hand_joints, gnd_truth, frame):
    """costfunc.cpp:476-507.  gnd_truth: (frames, 63) mm; .row(frame).reshape(3, 21) is a
    column-major fill (:486-487), i.e. joint j = row[3j:3j+3]; hand_joints (21, 3) cm
    from build_hand_model, scaled to mm with y and z negated (:491-492); the six
    distances of wrist + finger tips {0, 4, 8, 12, 16, 20} summed by numpy here (pairwise
    order -- the C oracle keeps Armadillo's two accumulators; they agree to an ulp)."""
    row = np.asarray(gnd_truth, dtype=np.float64)[frame]
    gt = row.reshape(21, 3)  # == reshape(3, 21, order='F').T
    hj = np.asarray(hand_joints, dtype=np.float64) * 10.0
    hj = hj * np.array([1.0, -1.0, -1.0])
    diff = gt - hj
    dist = np.sqrt(np.square(diff[:, 0]) + np.square(diff[:, 1]) + np.square(diff[:, 2]))
    return float(np.sum(dist[[0, 4, 8, 12, 16, 20]]))


class Obs:
    def __init__(self, depth_cm, dt, cloud, scale, K=None, focal=241.42):
        self.depth = depth_cm
        self.dt = dt
        self.cloud = cloud
        self.scale = scale
        self.dtmax = float(dt.max())
        self.K = K if K is not None else np.array([[focal, 0, 160.0], [0, focal, 120.0],
                                                   [0, 0, 1.0]])


def cal_cost(hand, obs, theta):
    """costfunc.cpp:89-127."""
    S = hand.build_hand_model(theta)
    m = correspondences(obs.cloud, S)
    return align(hand.radii, S, obs.cloud, m) + depth_penalty(
        hand.radii, S, obs.K, obs.depth, obs.dt, obs.dtmax, obs.scale)


def cal_cost2(hand, obs, theta, match=None):
    """costfunc.cpp:31-86; returns (cost, match, terms)."""
    S = hand.build_hand_model(theta)
    if match is None:
        match = correspondences(obs.cloud, S)
    a = align(hand.radii, S, obs.cloud, match)
    d = depth_penalty(hand.radii, S, obs.K, obs.depth, obs.dt, obs.dtmax, obs.scale)
    c = collision(hand.radii, S)
    return a + d + c, match, (a, d, c)


# ---------------------------------------------------------------- draws
M0, M1, W0, W1 = 0xD2511F53, 0xCD9E8D57, 0x9E3779B9, 0xBB67AE85
MASK = 0xFFFFFFFF


def philox4x32_10(ctr, key):
    c = list(ctr); k0, k1 = key
    for r in range(10):
        if r:
            k0 = (k0 + W0) & MASK; k1 = (k1 + W1) & MASK
        p0 = M0 * c[0]; p1 = M1 * c[2]
        c = [((p1 >> 32) ^ c[1] ^ k0) & MASK, p1 & MASK, ((p0 >> 32) ^ c[3] ^ k1) & MASK,
             p0 & MASK]
    return c


ST_NORMAL, ST_RP, ST_RG, ST_LINK = 1, 2, 3, 4
ST_OPT_PERM, ST_OPT_RP, ST_OPT_RG, ST_OPT_NORMAL = 5, 6, 7, 8


def u01(seed, stream, gen, idx, k):
    out = philox4x32_10((k >> 1, idx, gen, stream), (seed & MASK, (seed >> 32) & MASK))
    p = (k & 1) * 2
    return ((out[p] << 21) | (out[p + 1] >> 11)) * 2.0 ** -53


def normals(seed, P):
    out = np.zeros((P, 26))
    for i in range(P):
        for q in range(13):
            u1 = u01(seed, ST_NORMAL, 0, i, 2 * q)
            u2 = u01(seed, ST_NORMAL, 0, i, 2 * q + 1)
            r = math.sqrt(-2.0 * math.log(1.0 - u1))
            t = (2.0 * PI) * u2
            out[i, 2 * q] = r * math.cos(t)
            out[i, 2 * q + 1] = r * math.sin(t)
    return out


def pso_evolve(hand, obs, x0, P, maxiter, lb, ub, sd, seed=1000, cost_fn=None):
    """PSO.cpp:717-886 with the Philox stream.  Returns (bestp, bestcost, gbest_trace)."""
    cost_fn = cost_fn or (lambda th: cal_cost(hand, obs, th))
    x = x0[None, :] + normals(seed, P) * sd[None, :]
    v = np.zeros_like(x)
    pb = x.copy()
    pc = np.array([cost_fn(x[i]) for i in range(P)])
    gcost, gpos = 1e100, np.zeros(26)
    for i in range(P):
        if pc[i] < gcost:
            gcost, gpos = pc[i], x[i].copy()
    W1 = 1.0 / (2 * math.log(2)); C1 = 0.5 + math.log(2)
    count, L, trace = 100, None, []
    for g in range(1, maxiter):
        if count > 0:
            L = np.eye(P, dtype=bool)
            for s in range(P):
                for k in range(3):
                    r = int(math.floor(u01(seed, ST_LINK, g, s, k) * (P - 1) + 0.5))
                    L[s, r] = True
        for i in range(P):
            conn = np.nonzero(L[:, i])[0]
            inf = int(conn[np.argmin(pc[conn])])
            for d in range(26):
                rp = u01(seed, ST_RP, g, i, d)
                rg = u01(seed, ST_RG, g, i, d)
                nv = W1 * v[i, d] + (C1 * rp) * (pb[i, d] - x[i, d])
                if inf != i:
                    nv = nv + (C1 * rg) * (pb[inf, d] - x[i, d])
                v[i, d] = nv
            x[i] = x[i] + v[i]
            lo = x[i] < lb; hi = x[i] > ub
            x[i][lo] = lb[lo]; x[i][hi] = lb[hi]
            v[i][lo | hi] = 0.0
        for i in range(P):
            f = cost_fn(x[i])
            if f < pc[i]:
                pc[i] = f; pb[i] = x[i].copy()
        fid = int(np.argmin(pc))
        if pc[fid] < gcost:
            gpos, gcost, count = x[fid].copy(), pc[fid], 0
        else:
            count += 1
        trace.append(gcost)
    return gpos, gcost, trace


def _goldstein(hand, obs, x, g, match, fk):
    """PSO.cpp:438-480 with the default 30 iterations; returns tk."""
    a, b, alpha = 0.0, 1e100, 0.5
    p = -g
    gp = float(np.dot(g, p))
    for _ in range(30):
        f1 = cal_cost2(hand, obs, x + alpha * p, match)[0]
        if f1 <= fk + 0.25 * alpha * gp:
            if f1 >= fk + 0.75 * alpha * gp:
                return alpha
            a = alpha
            alpha = min(2 * alpha, 0.5 * (alpha + b))
        else:
            b = alpha
            alpha = 0.5 * (a + alpha)
    return 0.0


def pso_optimise(hand, obs, x0, P, maxiter, lb, ub, sd, w, c1, c2, seed=1000):
    """PSO.cpp:539-712: per generation, 10 single-coordinate Goldstein descent steps per
    particle (cal_gradient :380-405), then the global-best velocity update.  Philox
    streams 5..8 replace Armadillo's randi / randu / randn.  Returns (bestp, cost, trace)."""
    nrm = np.zeros((P, 26))
    for i in range(P):
        for q in range(13):
            u1 = u01(seed, ST_OPT_NORMAL, 0, i, 2 * q)
            u2 = u01(seed, ST_OPT_NORMAL, 0, i, 2 * q + 1)
            r = math.sqrt(-2.0 * math.log(1.0 - u1))
            t = (2.0 * PI) * u2
            nrm[i, 2 * q], nrm[i, 2 * q + 1] = r * math.cos(t), r * math.sin(t)
    x = x0[None, :] + nrm * sd[None, :]
    v = np.zeros_like(x)
    pb = x.copy()
    pc = np.array([cal_cost(hand, obs, x[i]) for i in range(P)])
    gcost, gpos = 1e100, np.zeros(26)
    for i in range(P):
        if pc[i] < gcost:
            gcost, gpos = pc[i], x[i].copy()
    trace = []

    def clamp(xi, vi):
        lo = xi < lb; hi = xi > ub
        xi[lo] = lb[lo]; xi[hi] = lb[hi]
        vi[lo | hi] = 0.0

    for g in range(1, maxiter):
        for i in range(P):
            th = x[i].copy()
            match = None
            for m in range(10):
                fk, mk, _ = cal_cost2(hand, obs, th, None if m == 0 else match)
                match = mk
                sel = min(25, int(math.floor(u01(seed, ST_OPT_PERM, g, i, m) * 26)))
                xp = th.copy(); xm = th.copy()
                xp[sel] += 1e-5; xm[sel] -= 1e-5
                gr = np.zeros(26)
                gr[sel] = (cal_cost2(hand, obs, xp, match)[0] -
                           cal_cost2(hand, obs, xm, match)[0]) / (2 * 1e-5)
                tk = _goldstein(hand, obs, th, gr, match, fk)
                th = th - tk * gr
                f2, mk, _ = cal_cost2(hand, obs, th, None if m == 0 else match)
                match = mk
                if f2 < pc[i]:
                    pc[i] = f2; pb[i] = th.copy()
            clamp(th, v[i])
            x[i] = th
        fid = int(np.argmin(pc))
        if pc[fid] < gcost:
            gpos, gcost = x[fid].copy(), pc[fid]
        for i in range(P):
            for d in range(26):
                rp = u01(seed, ST_OPT_RP, g, i, d)
                rg = u01(seed, ST_OPT_RG, g, i, d)
                v[i, d] = (w * v[i, d] + (c1 * rp) * (pb[i, d] - x[i, d])) + \
                    (c2 * rg) * (gpos[d] - x[i, d])
            x[i] = x[i] + v[i]
            clamp(x[i], v[i])
        for i in range(P):
            f = cal_cost(hand, obs, x[i])
            if f < pc[i]:
                pc[i] = f; pb[i] = x[i].copy()
        fid = int(np.argmin(pc))
        if pc[fid] < gcost:
            gpos, gcost = x[fid].copy(), pc[fid]
        trace.append(gcost)
    return gpos, gcost, trace


def refine_init_pose(hand, obs, x0):
    """PSO.cpp:183-266 (cal_grad + goldstein, blocks [0..2] and [3..5])."""
    x0 = np.array(x0, dtype=np.float64)
    for (s0, s1) in ((0, 2), (3, 5)):
        tol, cnt, it = 1.0, 0, 0
        while tol > 1e-6 and it < 15 and cnt < 1:
            fk, match, _ = cal_cost2(hand, obs, x0)
            g = np.zeros(26)
            for i in range(s0, s1 + 1):
                xp = x0.copy(); xm = x0.copy()
                xp[i] += 1e-5; xm[i] -= 1e-5
                g[i] = (cal_cost2(hand, obs, xp, match)[0] -
                        cal_cost2(hand, obs, xm, match)[0]) / (2 * 1e-5)
            a, b, alpha, tk = 0.0, 1e100, 0.5, 0.0
            p = -g
            gp = float(np.dot(g, p))
            for _ in range(30):
                f1 = cal_cost2(hand, obs, x0 + alpha * p, match)[0]
                if f1 <= fk + 0.25 * alpha * gp:
                    if f1 >= fk + 0.75 * alpha * gp:
                        tk = alpha
                        break
                    a = alpha
                    alpha = min(2 * alpha, 0.5 * (alpha + b))
                else:
                    b = alpha
                    alpha = 0.5 * (a + alpha)
            if tk == 0:
                cnt += 1
            x0 = x0 - tk * g
            tol = math.sqrt(float(np.sum(g * g)))
            it += 1
    return x0


# ------------------------------------------------------- preprocessing
HV, DIAG, LONG = 65536, 91750, 143976
INIT = 0x7FFFFFFF >> 2


def dist_transform(depth_cm):
    """cv::distanceTransform(inverted, CV_DIST_L2, 5) restated as row min-plus scans."""
    Hh, Ww = depth_cm.shape
    T = np.full((Hh + 4, Ww + 4), INIT, dtype=np.int64)
    hand = depth_cm != 0
    col = np.arange(Ww, dtype=np.int64)
    for i in range(Hh):
        r = i + 2
        up2, up1 = T[r - 2], T[r - 1]
        a = np.minimum.reduce([up2[1:Ww + 1] + LONG, up2[3:Ww + 3] + LONG, up1[0:Ww] + LONG,
                               up1[1:Ww + 1] + DIAG, up1[2:Ww + 2] + HV,
                               up1[3:Ww + 3] + DIAG, up1[4:Ww + 4] + LONG])
        a = np.where(hand[i], 0, a)
        # T_j = min(a_j, T_{j-1} + HV), T_{-1} = INIT
        a = np.minimum(a, INIT + HV + HV * col)
        T[r, 2:Ww + 2] = np.minimum.accumulate(a - HV * col) + HV * col
    for i in range(Hh - 1, -1, -1):
        r = i + 2
        dn1, dn2 = T[r + 1], T[r + 2]
        cur = T[r, 2:Ww + 2]
        b = np.minimum.reduce([cur, dn2[3:Ww + 3] + LONG, dn2[1:Ww + 1] + LONG,
                               dn1[4:Ww + 4] + LONG, dn1[3:Ww + 3] + DIAG, dn1[2:Ww + 2] + HV,
                               dn1[1:Ww + 1] + DIAG, dn1[0:Ww] + LONG])
        rc = col[::-1]
        b = np.minimum(b, INIT + HV + HV * rc)
        T[r, 2:Ww + 2] = (np.minimum.accumulate((b - HV * rc)[::-1]) + HV * col)[::-1]
    return (T[2:Hh + 2, 2:Ww + 2].astype(np.float32) * np.float32(1.0 / 65536)).astype(np.float32)


def preprocess(depth_mm, to_cm=True, downsample=True, focal=241.42):
    """observedmodel.cpp:110-219 + 272-369.  Returns Obs plus the full cloud size."""
    D = np.asarray(depth_mm, dtype=np.float32).reshape(H, W).astype(np.float64)
    if to_cm:
        D = D / 10.0
    rr, cc = np.nonzero(D)  # row-major pixel order
    Z = D[rr, cc]
    X = ((cc - 160.0) * Z) / focal
    Y = ((rr - 120.0) * Z) / focal
    cloud = np.stack([X, -Y, -Z], axis=1)
    pu = (focal * X + 0.0 * Y) + 160.0 * Z
    eu = (focal * (X + 2.0) + 0.0 * Y) + 160.0 * Z
    pw = (0.0 * X + 0.0 * Y) + 1.0 * Z
    dn = np.abs(np.floor(eu / pw) - np.floor(pu / pw))
    cm = 2.0 / dn[dn != 0]
    scale = float(np.mean(cm)) if len(cm) else float("nan")
    nfull = len(cloud)
    if downsample:
        f = nfull // 250
        cloud = cloud[np.arange(250) * f] if nfull else np.zeros((250, 3))
    dt = dist_transform(D)
    return Obs(D, dt, cloud, scale, focal=focal), nfull


# ------------------------------------------------------- synthetic frames
def render_depth_mm(hand, theta, focal=241.42):
    """Synthetic 240x320 float32 depth (mm, zero background) of the 48-sphere
    model: front-most ray/sphere hit per pixel centre."""
    S = hand.build_hand_model(theta)
    C = np.stack([S[:, 0], -S[:, 1], -S[:, 2]], axis=1)  # camera frame
    rr, cc = np.mgrid[0:H, 0:W]
    dx = (cc - 160.0) / focal; dy = (rr - 120.0) / focal
    dd = dx * dx + dy * dy + 1.0
    best = np.full((H, W), np.inf)
    for j in range(NS):
        b = dx * C[j, 0] + dy * C[j, 1] + C[j, 2]
        c = C[j] @ C[j] - hand.radii[j] ** 2
        disc = b * b - dd * c
        ok = disc >= 0
        t = np.where(ok, (b - np.sqrt(np.where(ok, disc, 0))) / dd, np.inf)
        t = np.where(t > 0, t, np.inf)
        best = np.minimum(best, t)
    out = np.where(np.isfinite(best), best * 10.0, 0.0).astype(np.float32)
    return out


def load_reference_hand(misc_dir):
    geo = np.loadtxt(f"{misc_dir}/hgeo.dat") / 10.0
    rad = np.loadtxt(f"{misc_dir}/rad.dat") / 10.0
    return Hand(geo, rad)
