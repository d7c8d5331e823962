// hpe_device.hpp -- device data layout and block-cooperative building blocks of the
// MI355X PSO / costfunc / handmodel hot path (gfx950, wave64).
//
// One workgroup (HPE_NT = 512 threads = 8 waves) evaluates one particle:
//   fk_block      26-DOF forward kinematics -> 48 sphere centres (fp64) in LDS
//                 (handmodel.cpp:259-298, fingermodel.cpp:70-317, thumbmodel.cpp:76-318)
//   match_align   N x 48 nearest-centre search (fp32, BFMatcher semantics) fused
//                 with the fp64 alignment residual (costfunc.cpp:306-377)
//   depth/collide 48 projections + depth/DT gathers, 144 collision pairs
//                 (costfunc.cpp:227-304, 130-197)
// The file is compiled with -ffp-contract=off: every product is rounded before the
// add, as in the x86-64 reference build; the structured matrix products below skip
// only terms that are exact zeros (x + a*0 == x) or exact unit factors (a*1 == a),
// so they reproduce the reference's 4x4 k-ordered sums bit for bit.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hpe_layout.hpp"

struct __align__(16) Smem {
    float4 Sf[HPE_NS];        // fp32 centres for the search
    double S[HPE_NS][3];      // fp64 centres, y/z negated
    double AB[5][12];
    double J[5][5][3];        // joints per digit (hand_joints source)
    double th[32];
    double sn[24], cs[24];
    double red[HPE_NW][4];
    double dscal[8];
    int iscal[8];
};

__device__ __forceinline__ double deg2rad(double a) {
    return a / 180.0 * 3.141592653589793115997963468544185161590576171875;  // fingermodel.cpp:203
}

// ---------------------------------------------------------------- FK
// Step A: 23 lanes, one sincos each (3 global + 20 digit angles).
// Step B: 60 lanes, one entry each of AB = A(a1)*B(a2) per digit (T12*T23 / T01*T12).
// Step C: 15 lanes (digit, row): each carries ONE ROW of the left-multiplied chain
//         cur = T00*Tgb*F*AB*C3*C4 -- row r of a left product depends only on row r
//         of the left factor, so no exchange is needed -- and writes coordinate r of
//         that digit's spheres.
__device__ __forceinline__ void fk_block(Smem &sm, const DevHand *__restrict__ H) {
    const int t = threadIdx.x;
    if (t < 23) {
        double a;
        if (t == 0) a = deg2rad(sm.th[0] + 180);  // TWS, fingermodel.cpp:91
        else if (t < 3) a = deg2rad(sm.th[t]);    // ANG, ROT
        else a = deg2rad(sm.th[6 + (t - 3)]);     // digit angles, handmodel.cpp:141-146
        double s, c;
        sincos(a, &s, &c);
        sm.sn[t] = s;
        sm.cs[t] = c;
    }
    __syncthreads();
    if (t < 60) {
        const int d = t / 12, e = t % 12, i = e >> 2, j = e & 3;
        const double c1 = sm.cs[3 + 4 * d], s1 = sm.sn[3 + 4 * d];
        const double c2 = sm.cs[4 + 4 * d], s2 = sm.sn[4 + 4 * d];
        const double L1 = H->L[d][1], tc = H->twc[d], ts = H->tws[d];
        double a0, a1, a2;  // row i of A = [[c1,0,-s1,0],[s1,0,c1,0],[0,-1,0,0]]
        if (i == 0) { a0 = c1; a1 = 0; a2 = -s1; }
        else if (i == 1) { a0 = s1; a1 = 0; a2 = c1; }
        else { a0 = 0; a1 = -1; a2 = 0; }
        double b0, b1, b2;  // column j of B (thumbmodel.cpp:150-153; fingers: tc=1, ts=0)
        if (j == 0) { b0 = c2; b1 = s2; b2 = 0; }
        else if (j == 1) { b0 = -s2 * tc; b1 = c2 * tc; b2 = ts; }
        else if (j == 2) { b0 = s2 * ts; b1 = -c2 * ts; b2 = tc; }
        else { b0 = L1 * c2; b1 = L1 * s2; b2 = 0; }
        sm.AB[d][e] = (a0 * b0 + a1 * b1) + a2 * b2;  // + A(i,3)*B(3,j) = +0
    }
    __syncthreads();
    if (t < 15) {
        const int d = t / 3, r = t % 3;
        const double cz = sm.cs[0], sz = sm.sn[0], cy = sm.cs[1], sy = sm.sn[1];
        const double cxr = sm.cs[2], sxr = sm.sn[2];
        double z0, z1, z2;  // row r of Rz
        if (r == 0) { z0 = cz; z1 = -sz; z2 = 0; }
        else if (r == 1) { z0 = sz; z1 = cz; z2 = 0; }
        else { z0 = 0; z1 = 0; z2 = 1; }
        // (Rz*Ry) row r, Ry = [[cy,0,sy],[0,1,0],[-sy,0,cy]]
        const double q0 = z0 * cy + z2 * (-sy);
        const double q1 = z1;
        const double q2 = z0 * sy + z2 * cy;
        // Tgb row r = q * Rx, Rx = [[1,0,0],[0,cx,-sx],[0,sx,cx]]; cur0 = T00*Tgb
        const double g0 = q0;
        const double g1 = q1 * cxr + q2 * sxr;
        const double g2 = q1 * (-sxr) + q2 * cxr;
        const double u = sm.th[3 + r];
        // cur1 = cur0 * F  (rotation about z + translation L0)
        const double h0 = g0 * H->Fc[d] + g1 * H->Fs[d];
        const double h1 = g0 * (-H->Fs[d]) + g1 * H->Fc[d];
        const double h2 = g2;
        const double h3 = (g0 * H->FLc[d] + g1 * H->FLs[d]) + u;
        const double J1 = h3;
        const double J0 = (h0 * H->T10x[d] + h1 * H->T10y[d]) + h3;  // (cur*T10) at i == 1
        // cur2 = cur1 * AB
        const double *AB = sm.AB[d];
        const double k0 = (h0 * AB[0] + h1 * AB[4]) + h2 * AB[8];
        const double k1 = (h0 * AB[1] + h1 * AB[5]) + h2 * AB[9];
        const double k3 = ((h0 * AB[3] + h1 * AB[7]) + h2 * AB[11]) + h3;
        const double J2 = k3;
        // cur3 = cur2 * C3, C4 translation only
        const double c3 = sm.cs[5 + 4 * d], s3 = sm.sn[5 + 4 * d];
        const double c4 = sm.cs[6 + 4 * d], s4 = sm.sn[6 + 4 * d];
        const double L2 = H->L[d][2], L3 = H->L[d][3];
        const double m0 = k0 * c3 + k1 * s3;
        const double m1 = k0 * (-s3) + k1 * c3;
        const double m3 = (k0 * (L2 * c3) + k1 * (L2 * s3)) + k3;
        const double J3 = m3;
        const double J4 = (m0 * (L3 * c4) + m1 * (L3 * s4)) + m3;
        const double J[5] = {J0, J1, J2, J3, J4};
#pragma unroll
        for (int k = 0; k < 5; ++k) sm.J[d][k][r] = J[k];
        // spheres (fingermodel.cpp:208-267, thumbmodel.cpp:227-274)
        const double sg = (r == 0) ? 1.0 : -1.0;  // cols(1,2) *= -1 (handmodel.cpp:288)
        int idx = (d == 0) ? 0 : 8 + 10 * (d - 1);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if (i == 0 && d != 0) {
                const double tt = 1. / 3;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const double v = (1. - tt * j) * J[0] + (tt * j) * J[1];
                    sm.S[idx][r] = v * sg;
                    ((float *)&sm.Sf[idx])[r] = (float)(v * sg);
                    ++idx;
                }
            } else {
#pragma unroll
                for (int j = 1; j < 3; ++j) {
                    const double v = (1. - 0.5 * j) * J[i] + (0.5 * j) * J[i + 1];
                    sm.S[idx][r] = v * sg;
                    ((float *)&sm.Sf[idx])[r] = (float)(v * sg);
                    ++idx;
                }
            }
        }
    }
    __syncthreads();
}

// ---------------------------------------------------------------- reductions
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// Sum three per-thread doubles over the block in a fixed order; result in every thread.
__device__ __forceinline__ void block_sum3(Smem &sm, double &a, double &b, double &c) {
    a = wave_sum(a);
    b = wave_sum(b);
    c = wave_sum(c);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        sm.red[w][0] = a;
        sm.red[w][1] = b;
        sm.red[w][2] = c;
    }
    __syncthreads();
    double ra = 0, rb = 0, rc = 0;
#pragma unroll
    for (int k = 0; k < HPE_NW; ++k) {
        ra += sm.red[k][0];
        rb += sm.red[k][1];
        rc += sm.red[k][2];
    }
    a = ra;
    b = rb;
    c = rc;
    __syncthreads();
}

// ---------------------------------------------------------------- cost terms
// depth_penalty term of sphere i (costfunc.cpp:249-300); S is un-negated on the fly.
__device__ __forceinline__ double depth_term(const Smem &sm, int i, const DevObs &o,
                                             const DevHand *__restrict__ H) {
    const double x = sm.S[i][0], y = sm.S[i][1] * -1, z = sm.S[i][2] * -1;
    const double pu = (o.K[0] * x + o.K[1] * y) + o.K[2] * z;
    const double pv = (o.K[3] * x + o.K[4] * y) + o.K[5] * z;
    const double pw = (o.K[6] * x + o.K[7] * y) + o.K[8] * z;
    const double dx = floor(pu / pw), dy = floor(pv / pw);
    const double r = H->radii[i];
    if (dx >= 0 && dx < HPE_IMG_W && dy >= 0 && dy < HPE_IMG_H) {
        const int pix = (int)dy * HPE_IMG_W + (int)dx;
        const double djc = o.depth[pix];
        if (djc != 0.0) {
            const double tt = djc - z;
            const double diff = (0.0 < tt) ? tt : 0.0;
            return diff * diff;
        }
        const double dd = (double)o.dt[pix] * o.scale + r;
        return dd * dd;
    }
    const double md = o.dtmax * o.scale + r;
    return md * md;
}

// one of the 144 self-collision pairs (costfunc.cpp:150-193)
__device__ __forceinline__ double collide_term(const Smem &sm, int t,
                                               const DevHand *__restrict__ H) {
    const int p = t / 36, k = t % 36;
    const int a = 2 + 10 * p + k / 6, b = 2 + 10 * (p + 1) + k % 6;
    const double dx = sm.S[b][0] - sm.S[a][0], dy = sm.S[b][1] - sm.S[a][1],
                 dz = sm.S[b][2] - sm.S[a][2];
    const double v = (H->radii[b] + H->radii[a]) - sqrt((dx * dx + dy * dy) + dz * dz);
    return v > 0 ? v * v : 0.0;
}

// Largest float whose correctly rounded sqrt equals sqrtf(m): BFMatcher compares
// sqrtf(d2) (OpenCV batchDistL2_32f) with first-index ties, so the match is the
// first j with d2[j] <= hi_sqrt_class(min_j d2[j]).  sqrt double->float is
// innocuous double rounding (53 >= 2*24+2), mid^2 is exact in double.
__device__ __forceinline__ float hi_sqrt_class(float m) {
    const float s = (float)sqrt((double)m);
    const float sn = __uint_as_float(__float_as_uint(s) + 1u);
    const double mid = 0.5 * ((double)s + (double)sn);
    const double mid2 = mid * mid;
    float h = (float)mid2;
    if ((double)h >= mid2) h = __uint_as_float(__float_as_uint(h) - 1u);
    return h;
}

// Fused correspondence search + alignment residual.  Two lanes (t, t^1) share a point,
// 24 spheres each; returns this thread's partial sum of (|p - S[m]| - r[m])^2.
template <bool STORE_MATCH>
__device__ __forceinline__ double match_align(const Smem &sm, const DevObs &o,
                                              const DevHand *__restrict__ H,
                                              int32_t *__restrict__ match) {
    double acc = 0.0;
    const int h = threadIdx.x & 1;
    const float4 *Sf = sm.Sf + 24 * h;
    for (int it = threadIdx.x; it < 2 * o.n; it += HPE_NT) {
        const int p = it >> 1;
        const double X = o.cx[p], Y = o.cy[p], Z = o.cz[p];
        const float qx = (float)X, qy = (float)Y, qz = (float)Z;
        float d2[24];
        float m = __builtin_inff();
#pragma unroll
        for (int j = 0; j < 24; ++j) {
            const float4 s = Sf[j];
            const float t0 = qx - s.x, t1 = qy - s.y, t2 = qz - s.z;
            d2[j] = (t0 * t0 + t1 * t1) + t2 * t2;
            m = fminf(m, d2[j]);
        }
        m = fminf(m, __shfl_xor(m, 1));
        const float hi = hi_sqrt_class(m);
        int idx = 1 << 20;
#pragma unroll
        for (int j = 23; j >= 0; --j) idx = (d2[j] <= hi) ? j : idx;
        idx += 24 * h;
        idx = min(idx, __shfl_xor(idx, 1));
        if (h == 0) {
            if (idx >= HPE_NS) idx = 0;  // all-NaN point: reference is undefined (trainIdx -1)
            const double dx = X - sm.S[idx][0], dy = Y - sm.S[idx][1], dz = Z - sm.S[idx][2];
            const double e = sqrt((dx * dx + dy * dy) + dz * dz) - H->radii[idx];
            acc += e * e;
            if (STORE_MATCH) match[p] = idx;
        }
    }
    return acc;
}

// Alignment with frozen correspondences (cal_cost2(..., compute_corr=false)).
__device__ __forceinline__ double align_frozen(const Smem &sm, const DevObs &o,
                                               const DevHand *__restrict__ H,
                                               const int32_t *__restrict__ match) {
    double acc = 0.0;
    for (int p = threadIdx.x; p < o.n; p += HPE_NT) {
        const int idx = match[p];
        const double dx = o.cx[p] - sm.S[idx][0], dy = o.cy[p] - sm.S[idx][1],
                     dz = o.cz[p] - sm.S[idx][2];
        const double e = sqrt((dx * dx + dy * dy) + dz * dz) - H->radii[idx];
        acc += e * e;
    }
    return acc;
}

enum EvalMode { EV_COST = 0, EV_COST2_CORR = 1, EV_COST2_FROZEN = 2, EV_COST_STORE = 3 };

// Whole-block evaluation of the particle whose theta is in sm.th.  Every thread
// returns the total; terms (align, depth, collision) optionally via sm.dscal[0..2].
template <int MODE>
__device__ __forceinline__ double eval_block(Smem &sm, const DevObs &o,
                                             const DevHand *__restrict__ H,
                                             int32_t *__restrict__ match) {
    fk_block(sm, H);
    const int t = threadIdx.x;
    // issue the depth gathers first: their latency hides under the search
    double dep = (t < HPE_NS) ? depth_term(sm, t, o, H) : 0.0;
    double al;
    if (MODE == EV_COST2_FROZEN) al = align_frozen(sm, o, H, match);
    else if (MODE == EV_COST2_CORR || MODE == EV_COST_STORE) al = match_align<true>(sm, o, H, match);
    else al = match_align<false>(sm, o, H, nullptr);
    const bool coll = (MODE == EV_COST2_CORR || MODE == EV_COST2_FROZEN);
    double co = (coll && t < 144) ? collide_term(sm, t, H) : 0.0;
    block_sum3(sm, al, dep, co);
    const double align = al * o.lambda;
    if (t == 0) {
        sm.dscal[0] = align;
        sm.dscal[1] = dep;
        sm.dscal[2] = co;
    }
    if (!coll) return align + dep;
    return (align + dep) + co;
}

// ---------------------------------------------------------------- Philox4x32-10
__device__ __forceinline__ double philox_u01(uint64_t seed, uint32_t stream, uint32_t gen,
                                             uint32_t idx, uint32_t k) {
    uint32_t c0 = k >> 1, c1 = idx, c2 = gen, c3 = stream;
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r > 0) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        const uint32_t lo0 = 0xD2511F53u * c0, hi0 = __umulhi(0xD2511F53u, c0);
        const uint32_t lo1 = 0xCD9E8D57u * c2, hi1 = __umulhi(0xCD9E8D57u, c2);
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0;
        c1 = lo1;
        c2 = n2;
        c3 = lo0;
    }
    const uint32_t a = (k & 1u) ? c2 : c0, b = (k & 1u) ? c3 : c1;
    const uint64_t u53 = ((uint64_t)a << 21) | (b >> 11);
    return (double)u53 * 0x1.0p-53;
}

enum { ST_NORMAL = 1, ST_RP = 2, ST_RG = 3, ST_LINK = 4 };
