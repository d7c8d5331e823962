// hpe_device.hpp -- device building blocks of the MI355X PSO / costfunc / handmodel
// hot path (gfx950, wave64).
//
//   fk_wave       26-DOF forward kinematics of one particle by ONE wave -> 48 sphere
//                 centres (fp64 + fp32 copies) in that wave's LDS workspace
//                 (handmodel.cpp:259-298, fingermodel.cpp:70-317, thumbmodel.cpp:76-318)
//   search_align  N x 48 nearest-centre search (fp32, BFMatcher semantics) fused with
//                 the fp64 alignment residual, by NT threads      (costfunc.cpp:306-377)
//   depth_term / collide_term                                  (costfunc.cpp:227-304, 130-197)
//   eval_block    one particle per workgroup (PSO generations, batch evaluation)
//   eval_wave     one particle per wave with frozen correspondences (refine)
//
// Compiled with -ffp-contract=off: every product is rounded before the add, as in the
// x86-64 reference build.  The structured matrix products skip only terms that are
// exact zeros (x + a*0 == x for finite a) or exact unit factors (a*1 == a), so they
// reproduce the reference's k-ordered 4x4 sums bit for bit; only sin/cos (ocml vs
// glibc, both < 1 ulp) can differ.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "hpe_layout.hpp"

// Diagnostic phase stamps (libhpe_stamps.so only, -DHPE_STAMPS=1; the product build
// compiles them out).  Thread 0 of block 0 accumulates shader-clock cycles per phase.
#ifndef HPE_STAMPS
#define HPE_STAMPS 0
#endif
__device__ unsigned long long hpe_stamps[64];
#if HPE_STAMPS
#define HPE_GOLD_LOG 65536
__device__ unsigned long long hpe_gold_log[1 + HPE_GOLD_LOG];  // [0] = count
#endif
// Per-block wall-clock stamps of k_pso_gen (100 MHz s_memrealtime, comparable across CUs):
// [generation][block][point], written by thread 0 (diagnostic build only).
#define BT_GENS 48
#define BT_BLK 256
#define BT_PTS 24
#if HPE_STAMPS
__device__ unsigned long long hpe_blk_ts[BT_GENS * BT_BLK * BT_PTS];
#define BLK_TS(g, k)                                                                       \
    do {                                                                                   \
        if (threadIdx.x == 0 && (g) < BT_GENS && blockIdx.x < BT_BLK)                      \
            hpe_blk_ts[((g) * BT_BLK + blockIdx.x) * BT_PTS + (k)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
// the same from lane 0 of every wave (point k + wave) of every (gridDim.x / BT_BLK)-th
// workgroup (a sample spread over the grid)
#define WAVE_TS(g, k)                                                                      \
    do {                                                                                   \
        const unsigned st_ = (gridDim.x + BT_BLK - 1) / BT_BLK;                            \
        if ((threadIdx.x & 63) == 0 && (g) < BT_GENS && blockIdx.x % st_ == 0)             \
            hpe_blk_ts[((g) * BT_BLK + blockIdx.x / st_) * BT_PTS + (k) + (threadIdx.x >> 6)] = \
                __builtin_amdgcn_s_memrealtime();                                          \
    } while (0)
// the entry stamp with the wave's placement: low 40 bits of the 100 MHz clock, HW_ID bits
// 15:0 (wave slot, SIMD, CU, SH, SE) at 40, XCC_ID at 56
#define WAVE_TS_ID(g)                                                                      \
    do {                                                                                   \
        const unsigned st_ = (gridDim.x + BT_BLK - 1) / BT_BLK;                            \
        if ((threadIdx.x & 63) == 0 && (g) < BT_GENS && blockIdx.x % st_ == 0) {           \
            const unsigned long long hw_ = __builtin_amdgcn_s_getreg((31 << 11) | 4);      \
            const unsigned long long xc_ = __builtin_amdgcn_s_getreg((3 << 11) | 20);      \
            hpe_blk_ts[((g) * BT_BLK + blockIdx.x / st_) * BT_PTS + (threadIdx.x >> 6)] =   \
                (__builtin_amdgcn_s_memrealtime() & 0xFFFFFFFFFFull) | ((hw_ & 0xFFFF) << 40) | \
                ((xc_ & 0xF) << 56);                                                       \
        }                                                                                  \
    } while (0)
// finer points (k < 12) of the even waves of every sampled workgroup: slot 2 k + wave / 2
#define WAVE_TS2(g, k)                                                                     \
    do {                                                                                   \
        const unsigned st_ = (gridDim.x + BT_BLK - 1) / BT_BLK;                            \
        if ((threadIdx.x & 64) == 0 && (threadIdx.x & 63) == 0 && (g) < BT_GENS &&          \
            blockIdx.x % st_ == 0)                                                         \
            hpe_blk_ts[((g) * BT_BLK + blockIdx.x / st_) * BT_PTS + 2 * (k) + (threadIdx.x >> 7)] = \
                __builtin_amdgcn_s_memrealtime();                                          \
    } while (0)
#else
#define WAVE_TS2(g, k) \
    do {               \
    } while (0)
#define WAVE_TS_ID(g) \
    do {              \
    } while (0)
#define WAVE_TS(g, k) \
    do {              \
    } while (0)
#define BLK_TS(g, k) \
    do {             \
    } while (0)
#endif
// Refine timeline (diagnostic build only): thread 0 of workgroup 0 appends
// (s_memrealtime << 8 | phase) at phase boundaries, the count kept in LDS.
#define RT_LOG 16384
#if HPE_STAMPS
__device__ unsigned long long hpe_ref_ts[RT_LOG];
#define REF_TS(cnt, ph)                                                                    \
    do {                                                                                   \
        if (threadIdx.x == 0 && blockIdx.x == 0) {                                         \
            const unsigned k_ = (cnt)++;                                                   \
            if (k_ < RT_LOG) hpe_ref_ts[k_] = (__builtin_amdgcn_s_memrealtime() << 8) | (ph); \
        }                                                                                  \
    } while (0)
#else
#define REF_TS(cnt, ph) \
    do {                \
    } while (0)
#endif
// HPE_NO_LAPS: a diagnostic build with the wall-clock logs (BLK_TS, WAVE_TS, REF_TS) but
// without the per-phase cycle laps below, whose global read-modify-writes on thread 0 of
// block 0 would stretch the phases being timed.
#ifndef HPE_NO_LAPS
#define HPE_NO_LAPS 0
#endif
struct StampClock {
    unsigned long long t, t0 = 0, r0 = 0;
    // whole-kernel span of block 0: shader cycles into slot k, 100 MHz ticks into k + 1
    __device__ __forceinline__ void begin() {
        if (HPE_STAMPS && !HPE_NO_LAPS && blockIdx.x == 0 && threadIdx.x == 0) {
            t0 = __builtin_amdgcn_s_memtime();
            r0 = __builtin_amdgcn_s_memrealtime();
            t = t0;
        }
    }
    __device__ __forceinline__ void span(int k) {
        if (HPE_STAMPS && !HPE_NO_LAPS && blockIdx.x == 0 && threadIdx.x == 0) {
            hpe_stamps[k] += __builtin_amdgcn_s_memtime() - t0;
            hpe_stamps[k + 1] += __builtin_amdgcn_s_memrealtime() - r0;
            hpe_stamps[32 + k] += 1;
            hpe_stamps[32 + k + 1] += 1;
        }
    }
    __device__ __forceinline__ void start() {
        if (HPE_STAMPS && !HPE_NO_LAPS && blockIdx.x == 0 && threadIdx.x == 0) t = __builtin_amdgcn_s_memtime();
    }
    __device__ __forceinline__ void lap(int k) {
        if (HPE_STAMPS && !HPE_NO_LAPS && blockIdx.x == 0 && threadIdx.x == 0) {
            const unsigned long long n = __builtin_amdgcn_s_memtime();
            hpe_stamps[k] += n - t;
            hpe_stamps[32 + k] += 1;
            t = n;
        }
    }
};

// Per-evaluating-wave LDS workspace.
struct __align__(16) FkSm {
    float Sp[3][HPE_NS];     // fp32 centres for the search, one row per coordinate
    double S[HPE_NS][3];     // fp64 centres, y/z negated (handmodel.cpp:288)
    double J[5][5][3];       // joints per digit (hand_joints source)
    double th[32];           // the particle
    double sn[24], cs[24];   // 3 global + 20 digit angles
};

// The filter search's per-particle tables (bf_filter_lane).  FILT_PTS: points per pass in
// the workgroup form's filter search (one table read serves them all).
#ifndef FILT_PTS
#define FILT_PTS 2
#endif
struct __align__(16) FiltSm {
    float ax[HPE_NS], ay[HPE_NS], az[HPE_NS], aw[HPE_NS];  // -2 s'_j, |s'_j|^2 + 1
};
struct FiltC {
    float ox, oy, oz;  // origin
    float K;           // R + 1
};

// Block-level workspace (one particle per workgroup).
struct __align__(16) Smem {
    DevHand hand;  // hand constants staged from HBM (lane-indexed reads stay in LDS)
    FkSm fk;
    double red[16][4];
    double dscal[8];
    int iscal[16];
    double draws[2 * HPE_DOF];  // rp, rg of the generation (k_pso_gen)
    double pbr[32];             // own pbest row at entry (k_pso_gen's pushes)
    FiltSm flt;                 // the filter search's tables (cal_cost of large clouds)
    FiltC fltc;
};

// Global-memory pointers.  Pointers read from memory (the frame descriptor DevObs) are
// generic to the compiler, so their loads become flat_load, which count on BOTH vmcnt and
// lgkmcnt: every later LDS or scalar-load wait then also waits for the HBM round trip.
// Loading through an address_space(1) pointer gives global_load (vmcnt only).
#define HPE_GAS __attribute__((address_space(1)))
template <class T>
__device__ __forceinline__ const HPE_GAS T *gp(const T *p) {
    return (const HPE_GAS T *)p;
}

// Cloud + correspondences, either in LDS (staged; generic pointers into a __shared__
// array, whose address space the compiler infers) or in HBM (CloudGlobal).
template <class P>
struct CloudT {
    P cx, cy, cz;
    int n;
};
using CloudView = CloudT<const double *>;
using CloudGlobal = CloudT<const HPE_GAS double *>;

// Copy the hand constants into LDS in two halves: hand_word() issues this thread's load
// (unconditional, so no branch forces an early wait), hand_put() stores it once the
// caller has issued its other loads; the caller synchronises before use.
template <int NT>
__device__ __forceinline__ double hand_word(const DevHand *__restrict__ src) {
    constexpr int NWD = (int)(sizeof(DevHand) / 8);
    static_assert(sizeof(DevHand) % 8 == 0 && NWD <= NT, "one 8-byte hand word per thread");
    const int q = threadIdx.x < NWD ? threadIdx.x : NWD - 1;
    return gp((const double *)src)[q];
}
template <int NT>
__device__ __forceinline__ void hand_put(DevHand &dst, double v) {
    if (threadIdx.x < (int)(sizeof(DevHand) / 8)) ((double *)&dst)[threadIdx.x] = v;
}
template <int NT>
__device__ __forceinline__ void stage_hand(DevHand &dst, const DevHand *__restrict__ src) {
    hand_put<NT>(dst, hand_word<NT>(src));
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// fp64 sqrt, bit-identical to the compiler's correctly rounded expansion of sqrt(): for
// 2^-767 <= x < inf that expansion scales by 2^0 (its v_ldexp pair and the 0 / inf class
// select are identities), so hpe_sqrt_nr runs the same rsq + Newton fma sequence without
// them; every other input (0, tiny, negative, inf, NaN) is recomputed with sqrt() itself
// on a branch the cost terms' squared distances practically never enter (callers with
// several roots fix them up behind ONE branch, so the roots stay one basic block).
// tools/sqrt_check.hip compares hpe_sqrt with sqrt bitwise.
// (2^-767 <= x < inf as two integer operations on the high word: both bounds have a zero
// low word, and negative values, -0 and NaN fall outside the unsigned range)
__device__ __forceinline__ bool hpe_sqrt_direct(double x) {
    const unsigned hi = (unsigned)((unsigned long long)__double_as_longlong(x) >> 32);
    return hi - 0x10000000u < 0x7FF00000u - 0x10000000u;
}
__device__ __forceinline__ double hpe_sqrt_nr(double x) {
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y, h = y * 0.5;
    const double r = __builtin_fma(-h, g, 0.5);
    g = __builtin_fma(g, r, g);
    h = __builtin_fma(h, r, h);
    double d = __builtin_fma(-g, g, x);
    g = __builtin_fma(d, h, g);
    d = __builtin_fma(-g, g, x);
    return __builtin_fma(d, h, g);
}
__device__ __forceinline__ double hpe_sqrt(double x) {
    double g = hpe_sqrt_nr(x);
    if (!hpe_sqrt_direct(x)) g = sqrt(x);
    return g;
}

__device__ __forceinline__ double deg2rad(double a) {
    return a / 180.0 * 3.141592653589793115997963468544185161590576171875;  // fingermodel.cpp:203
}

// ---------------------------------------------------------------- FK (one wave)
// Phase 1: 23 lanes, one sincos each (TWS, ANG, ROT and the 20 digit angles).
// Phase 2: 15 lanes (digit d, row r).  Row r of a left-multiplied product depends only
//          on row r of the left factor, so each lane carries ONE ROW of
//          cur = T00*Tgb*F*(A*B)*C3*C4 with no exchange; the 9 entries of A*B it needs
//          (T12*T23 / T01*T12) are independent of the chain and overlap with it.  The
//          lane then writes coordinate r of its digit's spheres.
// The global position u = theta[3..5] enters every joint translation only as the
// innermost addend (T00 is a pure translation, fingermodel.cpp:157-160, 289):
//   J1 = X1 + u,  J0 = X0 + J1,  J2 = X2 + J1,  J3 = X3 + J2,  J4 = X4 + J3
// with X0..X4 depending on the rotations and digit angles only.  FK_STORE_X keeps them;
// FK_TRANSLATE rebuilds the joints of a theta that differs from the stored one only in
// u with those five adds -- the same operations in the same order, so bit-identical.
enum FkMode { FK_FULL = 0, FK_STORE_X = 1, FK_TRANSLATE = 2 };
struct FkX {
    double x[15][5];
};

// ocml's fp64 sincos as an out-of-line call: inside the refine's loops the inlined
// version's ~20 polynomial constants are hoisted out of the loop and spilled.
struct SinCos {
    double s, c;
};
__device__ __noinline__ SinCos sincos_outline(double a) {
    SinCos r;
    sincos(a, &r.s, &r.c);
    return r;
}

// A sphere centre as FK stores it (y and z negated): lane l < 48 gets sphere l's
// coordinates in registers, so its depth projection needs no LDS round trip.
struct SphXYZ {
    double x, y, z;
};

// thr (optional): theta[l] of this lane l < 26, already in a register where the caller
// computed it (it still stores f.th for the chain phase): the trig phase then runs on
// lanes 0..2 and 6..25 from that register, without the LDS round trip of the permuted read.
template <int MODE, bool OUTLINE_TRIG = false>
__device__ __forceinline__ void fk_wave_t(FkSm &f, const DevHand *__restrict__ H, FkX *X,
                                          SphXYZ *own = nullptr, const double *thr = nullptr) {
    const int l = threadIdx.x & 63;
    StampClock sc;
    sc.start();
    // hand constants of this lane's chain row and sphere items, loaded before the trig so
    // their latency is not behind the phase fences
    const int dl = (l < 15) ? l / 3 : 0;
    const double L2 = H->L[dl][2], L3 = H->L[dl][3];
    const double Fc = H->Fc[dl], Fs = H->Fs[dl], FLc = H->FLc[dl], FLs = H->FLs[dl];
    const double T10x = H->T10x[dl], T10y = H->T10y[dl];
    const double L1 = H->L[dl][1], tc = H->twc[dl], ts = H->tws[dl];
    const int sl = (l < HPE_NS) ? l : HPE_NS - 1;  // this lane's sphere
    const int sd = H->dg[sl], sa = H->ja[sl];
    const double swa = H->wa[sl], swb = H->wb[sl];
    if (MODE != FK_TRANSLATE) {
        // slot k of sn / cs: TWS (fingermodel.cpp:91), ANG, ROT, then the 20 digit angles
        // (handmodel.cpp:141-146) = theta[k < 3 ? k : k + 3]
        const int k = thr ? (l < 3 ? l : l - 3) : l;
        if (thr ? (l < 3 || (l >= 6 && l < 26)) : (l < 23)) {
            // one unconditional LDS read per lane (per-lane branches would serialise three
            // read round trips)
            const double th = thr ? *thr : f.th[l < 3 ? l : 6 + (l - 3)];
            const double a = deg2rad(k == 0 ? th + 180 : th);
            double s, c;
            if (OUTLINE_TRIG) {
                const SinCos r = sincos_outline(a);
                s = r.s;
                c = r.c;
            } else {
                sincos(a, &s, &c);
            }
            f.sn[k] = s;
            f.cs[k] = c;
        }
        wave_sync();
    }
    sc.lap(13);
    if (l < 15) {
        const int d = l / 3, r = l - 3 * (l / 3);
        const double u = f.th[3 + r];
        double X0, X1, X2, X3, X4;
        if (MODE == FK_TRANSLATE) {
            X0 = X->x[l][0];
            X1 = X->x[l][1];
            X2 = X->x[l][2];
            X3 = X->x[l][3];
            X4 = X->x[l][4];
        } else {
            const double c1 = f.cs[3 + 4 * d], s1 = f.sn[3 + 4 * d];
            const double c2 = f.cs[4 + 4 * d], s2 = f.sn[4 + 4 * d];
            const double c3 = f.cs[5 + 4 * d], s3 = f.sn[5 + 4 * d];
            const double c4 = f.cs[6 + 4 * d], s4 = f.sn[6 + 4 * d];
            // Columns 0, 1, 3 of A*B with A = [[c1,0,-s1,0],[s1,0,c1,0],[0,-1,0,0]] and
            // B = [[c2,-s2*tc,s2*ts,L1*c2],[s2,c2*tc,-c2*ts,L1*s2],[0,ts,tc,0]]
            // (thumbmodel.cpp:144-153; fingers tc = 1, ts = 0, fingermodel.cpp:137-145).
            // Each entry is the reference's k-ordered sum with its exact-zero terms dropped.
            const double b01 = -s2 * tc, b11 = c2 * tc, L1c2 = L1 * c2, L1s2 = L1 * s2;
            const double AB00 = c1 * c2, AB10 = s1 * c2, AB20 = -s2;
            const double AB01 = c1 * b01 + (-s1) * ts, AB11 = s1 * b01 + c1 * ts, AB21 = -b11;
            const double AB03 = c1 * L1c2, AB13 = s1 * L1c2, AB23 = -L1s2;
            const double cz = f.cs[0], sz = f.sn[0], cy = f.cs[1], sy = f.sn[1];
            const double cxr = f.cs[2], sxr = f.sn[2];
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
            // cur1 = cur0 * F  (rotation about z + translation L0); its translation is X1 + u
            const double h0 = g0 * Fc + g1 * Fs;
            const double h1 = g0 * (-Fs) + g1 * Fc;
            const double h2 = g2;
            X1 = g0 * FLc + g1 * FLs;
            X0 = h0 * T10x + h1 * T10y;  // (cur*T10) at i == 1
            // cur2 = cur1 * AB
            const double k0 = (h0 * AB00 + h1 * AB10) + h2 * AB20;
            const double k1 = (h0 * AB01 + h1 * AB11) + h2 * AB21;
            X2 = (h0 * AB03 + h1 * AB13) + h2 * AB23;
            // cur3 = cur2 * C3, then the translation of cur3 * C4
            const double m0 = k0 * c3 + k1 * s3;
            const double m1 = k0 * (-s3) + k1 * c3;
            X3 = k0 * (L2 * c3) + k1 * (L2 * s3);
            X4 = m0 * (L3 * c4) + m1 * (L3 * s4);
            if (MODE == FK_STORE_X) {
                X->x[l][0] = X0;
                X->x[l][1] = X1;
                X->x[l][2] = X2;
                X->x[l][3] = X3;
                X->x[l][4] = X4;
            }
        }
        const double J1 = X1 + u;
        const double J0 = X0 + J1;
        const double J2 = X2 + J1;
        const double J3 = X3 + J2;
        const double J4 = X4 + J3;
        f.J[d][0][r] = J0;
        f.J[d][1][r] = J1;
        f.J[d][2][r] = J2;
        f.J[d][3][r] = J3;
        f.J[d][4][r] = J4;
    }
    wave_sync();
    // spheres (fingermodel.cpp:208-267, thumbmodel.cpp:227-274): lane l < 48 places sphere
    // l, its three coordinates, weights from the hand tables; cols(1,2) *= -1
    // (handmodel.cpp:288).  Its six joint reads are issued first (unconditional: lanes >= 48
    // read sphere 47's), so they share one LDS round trip; the centre stays in the lane's
    // registers for the caller's depth projection (own).
    double ja[3], jb[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        ja[r] = f.J[sd][sa][r];
        jb[r] = f.J[sd][sa + 1][r];
    }
    double vs[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        const double v = swa * ja[r] + swb * jb[r];
        vs[r] = (r == 0) ? v : v * -1;
    }
    if (l < HPE_NS) {
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            f.S[l][r] = vs[r];
            f.Sp[r][l] = (float)vs[r];
        }
    }
    if (own) *own = (l < HPE_NS) ? SphXYZ{vs[0], vs[1], vs[2]} : SphXYZ{0.0, 0.0, 0.0};
    wave_sync();
    sc.lap(14);
}

// FK of NP particles by the whole workgroup (the wave form, round 5): the three phases of fk_wave_t with their items spread over the workgroup's
// threads instead of each wave running its own particle's phases on 23, 15 and 48 of its
// lanes -- trig on NP x 23 threads, chain rows on NP x 15, spheres on NP x 48 -- with a
// workgroup barrier after each.  The per-item operations are fk_wave_t's (FK_FULL, inline
// trig), so the centres are the same bits; fk[p * STRIDE] is particle p's workspace (STRIDE:
// waves per particle).  Every thread of the workgroup calls it.
template <int NP, int STRIDE>
__device__ __forceinline__ void fk_coop(FkSm *fk, const DevHand *__restrict__ H) {
    const int t = threadIdx.x;
    // this thread's chain row and sphere item, their hand constants loaded first
    const int pc = min(t / 15, NP - 1), l = t - 15 * (t / 15);
    const int dl = (t < NP * 15) ? l / 3 : 0;
    const double L2 = H->L[dl][2], L3 = H->L[dl][3];
    const double Fc = H->Fc[dl], Fs = H->Fs[dl], FLc = H->FLc[dl], FLs = H->FLs[dl];
    const double T10x = H->T10x[dl], T10y = H->T10y[dl];
    const double L1 = H->L[dl][1], tc = H->twc[dl], ts = H->tws[dl];
    const int ps = min(t / HPE_NS, NP - 1), sl = (t < NP * HPE_NS) ? t - HPE_NS * (t / HPE_NS) : HPE_NS - 1;
    const int sd = H->dg[sl], sa = H->ja[sl];
    const double swa = H->wa[sl], swb = H->wb[sl];
    if (t < NP * 23) {  // trig: slot k of particle t / 23 (fk_wave_t phase 1)
        const int pt = t / 23, k = t - 23 * pt;
        FkSm &f = fk[pt * STRIDE];
        const double th = f.th[k < 3 ? k : 6 + (k - 3)];
        const double a = deg2rad(k == 0 ? th + 180 : th);
        double sn, cs;
        sincos(a, &sn, &cs);
        f.sn[k] = sn;
        f.cs[k] = cs;
    }
    __syncthreads();
    if (t < NP * 15) {  // chain row r of digit d of particle pc (fk_wave_t phase 2, FK_FULL)
        FkSm &f = fk[pc * STRIDE];
        const int d = l / 3, r = l - 3 * (l / 3);
        const double u = f.th[3 + r];
        const double c1 = f.cs[3 + 4 * d], s1 = f.sn[3 + 4 * d];
        const double c2 = f.cs[4 + 4 * d], s2 = f.sn[4 + 4 * d];
        const double c3 = f.cs[5 + 4 * d], s3 = f.sn[5 + 4 * d];
        const double c4 = f.cs[6 + 4 * d], s4 = f.sn[6 + 4 * d];
        const double b01 = -s2 * tc, b11 = c2 * tc, L1c2 = L1 * c2, L1s2 = L1 * s2;
        const double AB00 = c1 * c2, AB10 = s1 * c2, AB20 = -s2;
        const double AB01 = c1 * b01 + (-s1) * ts, AB11 = s1 * b01 + c1 * ts, AB21 = -b11;
        const double AB03 = c1 * L1c2, AB13 = s1 * L1c2, AB23 = -L1s2;
        const double cz = f.cs[0], sz = f.sn[0], cy = f.cs[1], sy = f.sn[1];
        const double cxr = f.cs[2], sxr = f.sn[2];
        double z0, z1, z2;
        if (r == 0) { z0 = cz; z1 = -sz; z2 = 0; }
        else if (r == 1) { z0 = sz; z1 = cz; z2 = 0; }
        else { z0 = 0; z1 = 0; z2 = 1; }
        const double q0 = z0 * cy + z2 * (-sy);
        const double q1 = z1;
        const double q2 = z0 * sy + z2 * cy;
        const double g0 = q0;
        const double g1 = q1 * cxr + q2 * sxr;
        const double g2 = q1 * (-sxr) + q2 * cxr;
        const double h0 = g0 * Fc + g1 * Fs;
        const double h1 = g0 * (-Fs) + g1 * Fc;
        const double h2 = g2;
        const double X1 = g0 * FLc + g1 * FLs;
        const double X0 = h0 * T10x + h1 * T10y;
        const double k0 = (h0 * AB00 + h1 * AB10) + h2 * AB20;
        const double k1 = (h0 * AB01 + h1 * AB11) + h2 * AB21;
        const double X2 = (h0 * AB03 + h1 * AB13) + h2 * AB23;
        const double m0 = k0 * c3 + k1 * s3;
        const double m1 = k0 * (-s3) + k1 * c3;
        const double X3 = k0 * (L2 * c3) + k1 * (L2 * s3);
        const double X4 = m0 * (L3 * c4) + m1 * (L3 * s4);
        const double J1 = X1 + u;
        const double J0 = X0 + J1;
        const double J2 = X2 + J1;
        const double J3 = X3 + J2;
        const double J4 = X4 + J3;
        f.J[d][0][r] = J0;
        f.J[d][1][r] = J1;
        f.J[d][2][r] = J2;
        f.J[d][3][r] = J3;
        f.J[d][4][r] = J4;
    }
    __syncthreads();
    if (t < NP * HPE_NS) {  // sphere sl of particle ps (fk_wave_t phase 3)
        FkSm &f = fk[ps * STRIDE];
        double ja[3], jb[3];
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            ja[r] = f.J[sd][sa][r];
            jb[r] = f.J[sd][sa + 1][r];
        }
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            const double v = swa * ja[r] + swb * jb[r];
            const double vs = (r == 0) ? v : v * -1;
            f.S[sl][r] = vs;
            f.Sp[r][sl] = (float)vs;
        }
    }
    __syncthreads();
}

template <bool OUTLINE_TRIG = false>
__device__ __forceinline__ void fk_wave(FkSm &f, const DevHand *__restrict__ H,
                                        SphXYZ *own = nullptr, const double *thr = nullptr) {
    fk_wave_t<FK_FULL, OUTLINE_TRIG>(f, H, nullptr, own, thr);
}

// ---------------------------------------------------------------- reductions
// Wave-wide fp64 sum without LDS: DPP butterflies inside each 16-lane row, then the four
// row sums are combined in a fixed order through v_readlane.  Deterministic; all lanes
// receive the total.
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double readlane_f64(double v, int lane) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
    return __hiloint2double(hi, lo);
}
// A value every lane of the workgroup computed identically (from the same LDS words by the
// same operations), made provably wave-uniform for the compiler: control flow that decides
// barriers must not look divergent to it (a barrier under divergent control flow is
// undefined behaviour in the HIP model).  Bit-exact: every lane holds it.
__device__ __forceinline__ double uniform_f64(double v) {
    const int lo = __builtin_amdgcn_readfirstlane(__double2loint(v));
    const int hi = __builtin_amdgcn_readfirstlane(__double2hiint(v));
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double row_sum16(double v) {
    v += dpp_f64<0xB1>(v);   // quad_perm [1,0,3,2]
    v += dpp_f64<0x4E>(v);   // quad_perm [2,3,0,1]
    v += dpp_f64<0x141>(v);  // row_half_mirror
    v += dpp_f64<0x140>(v);  // row_mirror
    return v;
}
__device__ __forceinline__ double wave_sum(double v) {
    v = row_sum16(v);
    return ((readlane_f64(v, 0) + readlane_f64(v, 16)) + readlane_f64(v, 32)) +
           readlane_f64(v, 48);
}
template <int CTRL>
__device__ __forceinline__ int dpp_i32(int v) {
    return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xf, 0xf, false);
}
// Lexicographic (v, idx) minimum over the wave (Armadillo min(index): first minimum wins).
// v must not be NaN.  Returns the winner's idx and payload in every lane.
__device__ __forceinline__ void wave_argmin_lex(double v, int idx, int pay, int &out_idx,
                                                int &out_pay, double *out_min = nullptr) {
    double m = v;
    m = fmin(m, dpp_f64<0xB1>(m));
    m = fmin(m, dpp_f64<0x4E>(m));
    m = fmin(m, dpp_f64<0x141>(m));
    m = fmin(m, dpp_f64<0x140>(m));
    const double mn = fmin(fmin(readlane_f64(m, 0), readlane_f64(m, 16)),
                           fmin(readlane_f64(m, 32), readlane_f64(m, 48)));
    if (out_min) *out_min = mn;
    int c = (v == mn) ? idx : 0x7fffffff;
    c = min(c, dpp_i32<0xB1>(c));
    c = min(c, dpp_i32<0x4E>(c));
    c = min(c, dpp_i32<0x141>(c));
    c = min(c, dpp_i32<0x140>(c));
    const int mi = min(min(__builtin_amdgcn_readlane(c, 0), __builtin_amdgcn_readlane(c, 16)),
                       min(__builtin_amdgcn_readlane(c, 32), __builtin_amdgcn_readlane(c, 48)));
    const unsigned long long b = __ballot(v == mn && idx == mi);
    out_idx = mi;
    out_pay = __builtin_amdgcn_readlane(pay, (int)__ffsll((long long)b) - 1);
}

// The same over lanes 0..15 only (row 0; the other lanes are ignored): four DPP steps per
// key inside the row and one readlane each, instead of the cross-row readlane chains.
__device__ __forceinline__ void row0_argmin_lex(double v, int idx, int pay, int &out_idx,
                                                int &out_pay, double *out_min = nullptr) {
    double m = v;
    m = fmin(m, dpp_f64<0xB1>(m));
    m = fmin(m, dpp_f64<0x4E>(m));
    m = fmin(m, dpp_f64<0x141>(m));
    m = fmin(m, dpp_f64<0x140>(m));
    const double mn = readlane_f64(m, 0);
    if (out_min) *out_min = mn;
    int c = (v == mn) ? idx : 0x7fffffff;
    c = min(c, dpp_i32<0xB1>(c));
    c = min(c, dpp_i32<0x4E>(c));
    c = min(c, dpp_i32<0x141>(c));
    c = min(c, dpp_i32<0x140>(c));
    const int mi = __builtin_amdgcn_readlane(c, 0);
    const unsigned long long b = __ballot(v == mn && idx == mi) & 0xffffull;
    out_idx = mi;
    out_pay = __builtin_amdgcn_readlane(pay, (int)__ffsll((long long)b) - 1);
}

// three independent sums interleaved for ILP
__device__ __forceinline__ void wave_sum3(double &a, double &b, double &c) {
    a += dpp_f64<0xB1>(a); b += dpp_f64<0xB1>(b); c += dpp_f64<0xB1>(c);
    a += dpp_f64<0x4E>(a); b += dpp_f64<0x4E>(b); c += dpp_f64<0x4E>(c);
    a += dpp_f64<0x141>(a); b += dpp_f64<0x141>(b); c += dpp_f64<0x141>(c);
    a += dpp_f64<0x140>(a); b += dpp_f64<0x140>(b); c += dpp_f64<0x140>(c);
    a = ((readlane_f64(a, 0) + readlane_f64(a, 16)) + readlane_f64(a, 32)) + readlane_f64(a, 48);
    b = ((readlane_f64(b, 0) + readlane_f64(b, 16)) + readlane_f64(b, 32)) + readlane_f64(b, 48);
    c = ((readlane_f64(c, 0) + readlane_f64(c, 16)) + readlane_f64(c, 32)) + readlane_f64(c, 48);
}

__device__ __forceinline__ void wave_sum2(double &a, double &b) {
    a += dpp_f64<0xB1>(a); b += dpp_f64<0xB1>(b);
    a += dpp_f64<0x4E>(a); b += dpp_f64<0x4E>(b);
    a += dpp_f64<0x141>(a); b += dpp_f64<0x141>(b);
    a += dpp_f64<0x140>(a); b += dpp_f64<0x140>(b);
    a = ((readlane_f64(a, 0) + readlane_f64(a, 16)) + readlane_f64(a, 32)) + readlane_f64(a, 48);
    b = ((readlane_f64(b, 0) + readlane_f64(b, 16)) + readlane_f64(b, 32)) + readlane_f64(b, 48);
}

// Sum three per-thread doubles over NT threads in a fixed order; result in every thread.
// REUSE = false: the caller never touches `red` again in this kernel, so the trailing
// barrier that protects it is skipped.  c is not reduced when TWO (it stays 0).
template <int NT, bool REUSE = true, bool TWO = false>
__device__ __forceinline__ void block_sum3(double (*red)[4], double &a, double &b, double &c) {
    if (TWO) wave_sum2(a, b);
    else wave_sum3(a, b, c);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        red[w][0] = a;
        red[w][1] = b;
        red[w][2] = c;
    }
    __syncthreads();
    double ra = 0, rb = 0, rc = 0;
#pragma unroll
    for (int k = 0; k < NT / 64; ++k) {
        ra += red[k][0];
        rb += red[k][1];
        rc += red[k][2];
    }
    a = ra;
    b = rb;
    c = TWO ? 0.0 : rc;
    if (REUSE) __syncthreads();
}

// Sum one per-thread double over NT threads in a fixed order; result in every thread.
// The cost kernels sum each lane's total (align * lambda + depth + collision) once
// instead of the three terms separately: the same cost to the last bits (the reference's
// own sums run in yet another order) for one wave reduction instead of three.
template <int NT, bool REUSE = true>
__device__ __forceinline__ double block_sum1(double (*red)[4], double v) {
    v = wave_sum(v);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) red[w][0] = v;
    __syncthreads();
    double r = 0;
#pragma unroll
    for (int k = 0; k < NT / 64; ++k) r += red[k][0];
    if (REUSE) __syncthreads();
    return r;
}

// ---------------------------------------------------------------- rigid refine FK
// refine_init_pose moves only theta0..5 (PSO.cpp:225-227): the 20 digit angles are fixed
// for the whole call.  Every joint is u + Rg * x with Rg = Rz(theta0 + 180) Ry(theta1)
// Rx(theta2) (fingermodel.cpp:165-180) and x depending on the digit angles only
// (T00 * Tgb is the first factor of every chain, fingermodel.cpp:289), and a sphere is an
// affine combination of two joints, so
//     S_k = negate_yz(Rg * q_k + u),   q_k = the hand-frame centre,
// with q_k = the reference FK at theta0 = -180, theta1..5 = 0 (Tgb = I, u = 0 exactly:
// sincos(0) = (0, 1)) with y, z un-negated.  The self-collision penalty depends on the
// pairwise distances only, so it is a constant C of the call.  A refine node then costs
// three sincos and a 3x3 rotation (block 2, translation only: P_k + u with P_k = Rg * q_k
// of the block's fixed rotation) instead of the 5-digit DH chains.  Not the reference's
// operation order: spheres agree with the chain to ~1e-14 cm and costs to ~1e-15
// relative (DESIGN.md §2 states the tolerance; HPE_REFINE_EXACT=1 selects the chain).
struct __align__(16) RigidSm {
    double q[HPE_NS][3];  // hand-frame centres
    double P[HPE_NS][3];  // Rg(x0) q_k, block 2
    double C;             // self_collision_penalty (costfunc.cpp:130-197), rigid-invariant
};

// Row r of Rg from the three angles' sines / cosines: row r of Rz, then * Ry, then * Rx
// (fingermodel.cpp:165-180), the products with Rz's constant 0 / 1 entries left out (they
// only add a signed zero; oracle/hpe_oracle.c rigid_rows forms the same operations).
__device__ __forceinline__ void rigid_row(int r, double sz, double cz, double sy, double cy,
                                          double sx, double cx, double &g0, double &g1,
                                          double &g2) {
    if (r == 2) {  // (0, 0, 1) * Ry * Rx
        g0 = -sy;
        g1 = cy * sx;
        g2 = cy * cx;
        return;
    }
    const double z0 = (r == 0) ? cz : sz, z1 = (r == 0) ? -sz : cz;  // (z0, z1, 0)
    const double q0 = z0 * cy;
    const double q1 = z1;
    const double q2 = z0 * sy;
    g0 = q0;
    g1 = q1 * cx + q2 * sx;
    g2 = q1 * (-sx) + q2 * cx;
}

// Spheres of the refine node whose theta[l] is thl (lanes 0..25; lanes 0..2 and 3..5 are
// read, the digits are in R.q) into f.S / f.Sp; lane l < 48 keeps its centre in own.
// MODE 0: rotation block (trig on lanes 0..2, Rg rows, Rg q + u); MODE 1: translation
// block (P + u); MODE 2: store P = Rg q into Pout (u ignored, f untouched).
enum RigidMode { RG_ROT = 0, RG_TRANS = 1, RG_STORE_P = 2 };
#ifndef HPE_RIGID_OUTLINE_TRIG
#define HPE_RIGID_OUTLINE_TRIG 1
#endif
template <int MODE, bool OUTLINE_TRIG = HPE_RIGID_OUTLINE_TRIG>
__device__ __forceinline__ void rigid_wave(FkSm &f, const RigidSm &R, double thl,
                                           SphXYZ *own = nullptr, double (*Pout)[3] = nullptr) {
    const int l = threadIdx.x & 63;
    const int sl = l < HPE_NS ? l : HPE_NS - 1;
    const double a0 = MODE == RG_TRANS ? R.P[sl][0] : R.q[sl][0];
    const double a1 = MODE == RG_TRANS ? R.P[sl][1] : R.q[sl][1];
    const double a2 = MODE == RG_TRANS ? R.P[sl][2] : R.q[sl][2];
    double v[3];
    const double u[3] = {readlane_f64(thl, 3), readlane_f64(thl, 4), readlane_f64(thl, 5)};
    if (MODE == RG_TRANS) {
        v[0] = a0 + u[0];
        v[1] = a1 + u[1];
        v[2] = a2 + u[2];
    } else {
        double s = 0.0, c = 1.0;
        if (l < 3) {  // TWS, ANG, ROT (fingermodel.cpp:91-93)
            const double a = deg2rad(l == 0 ? thl + 180 : thl);
            if (OUTLINE_TRIG) {
                const SinCos r = sincos_outline(a);
                s = r.s;
                c = r.c;
            } else {
                sincos(a, &s, &c);
            }
        }
        const double sz = readlane_f64(s, 0), cz = readlane_f64(c, 0);
        const double sy = readlane_f64(s, 1), cy = readlane_f64(c, 1);
        const double sx = readlane_f64(s, 2), cx = readlane_f64(c, 2);
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            double g0, g1, g2;
            rigid_row(r, sz, cz, sy, cy, sx, cx, g0, g1, g2);
            const double p = (g0 * a0 + g1 * a1) + g2 * a2;
            if (MODE == RG_STORE_P) {
                if (l < HPE_NS) Pout[l][r] = p;
            }
            v[r] = p + u[r];
        }
        if (MODE == RG_STORE_P) return;
    }
    v[1] = v[1] * -1;  // handmodel.cpp:288
    v[2] = v[2] * -1;
    if (l < HPE_NS) {
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            f.S[l][r] = v[r];
            f.Sp[r][l] = (float)v[r];
        }
    }
    if (own) *own = (l < HPE_NS) ? SphXYZ{v[0], v[1], v[2]} : SphXYZ{0.0, 0.0, 0.0};
    wave_sync();
}

// ---------------------------------------------------------------- cost terms
// depth_penalty term of sphere i (costfunc.cpp:249-300); S is un-negated on the fly.
// Two halves, so that the gathers' L2 round trip overlaps the caller's other work:
//   depth_issue  projection + BOTH gathers (depth and DT at a clamped pixel), issued
//                unconditionally by every lane (sphere index clamped);
//   depth_finish waits for them (an empty asm consumes the loaded registers, so the
//                compiler can neither wait earlier nor sink a load into the reference's
//                branches) and evaluates the branches as selects; 0 where !use.
struct DepthG {
    double djc, z, r;
    float dtp;
    bool in;
};
__device__ __forceinline__ DepthG depth_issue_at(const SphXYZ &c, int i, const DevObs &o,
                                                 const DevHand *__restrict__ H) {
    i = i < HPE_NS ? i : HPE_NS - 1;
    const double x = c.x, y = c.y * -1, z = c.z * -1;
    double pu, pv, pw;
    if (o.K[1] == 0.0 && o.K[3] == 0.0 && o.K[6] == 0.0 && o.K[7] == 0.0 && o.K[8] == 1.0) {
        // the pinhole K of every frame (focal, principal point): the zero terms only add a
        // signed zero, which changes no value here; a non-finite coordinate leaves the
        // sphere off-image either way (general form: pw NaN, this form: dx or dy non-finite)
        pu = o.K[0] * x + o.K[2] * z;
        pv = o.K[4] * y + o.K[5] * z;
        pw = z;
    } else {
        pu = (o.K[0] * x + o.K[1] * y) + o.K[2] * z;
        pv = (o.K[3] * x + o.K[4] * y) + o.K[5] * z;
        pw = (o.K[6] * x + o.K[7] * y) + o.K[8] * z;
    }
    const double dx = floor(pu / pw), dy = floor(pv / pw);
    DepthG d;
    d.in = dx >= 0 && dx < HPE_IMG_W && dy >= 0 && dy < HPE_IMG_H;  // NaN: off-image
    const int pix = d.in ? (int)dy * HPE_IMG_W + (int)dx : 0;
    d.djc = gp(o.depth)[pix];
    d.dtp = gp(o.dt)[pix];
    d.z = z;
    d.r = H->radii[i];
    return d;
}
__device__ __forceinline__ DepthG depth_issue(const FkSm &f, int i, const DevObs &o,
                                              const DevHand *__restrict__ H) {
    const int ic = i < HPE_NS ? i : HPE_NS - 1;
    return depth_issue_at(SphXYZ{f.S[ic][0], f.S[ic][1], f.S[ic][2]}, i, o, H);
}
// md2p (optional): the off-image value md * md below, computed ahead by the caller with the
// same operations for the same sphere (the refine: once per call, not per evaluation).
__device__ __forceinline__ double depth_off_sq(const DevObs &o, double r) {
    const double md = o.dtmax * o.scale + r;  // off-image: max of the DT (:298)
    return md * md;
}
__device__ __forceinline__ double depth_finish(DepthG d, const DevObs &o, bool use,
                                               const double *md2p = nullptr) {
    asm volatile("" : "+v"(d.djc), "+v"(d.dtp));
    const double tt = d.djc - d.z;
    const double diff = (0.0 < tt) ? tt : 0.0;  // std::max(0.0, tt)
    const double dd = (double)d.dtp * o.scale + d.r;
    const double md2 = md2p ? *md2p : depth_off_sq(o, d.r);
    const double v = !d.in ? md2 : (d.djc != 0.0) ? diff * diff : dd * dd;
    return use ? v : 0.0;
}
// Block form: wave 0 (its lanes 0..47 are the spheres) issues; the other waves keep a
// zero DepthG, so they spend no VALU time on the projections while they search.
__device__ __forceinline__ DepthG depth_issue_w0(const FkSm &f, const DevObs &o,
                                                 const DevHand *__restrict__ H) {
    DepthG d{0.0, 0.0, 0.0, 0.f, false};
    if (threadIdx.x < 64) d = depth_issue(f, threadIdx.x, o, H);
    return d;
}
__device__ __forceinline__ double depth_term(const FkSm &f, int i, const DevObs &o,
                                             const DevHand *__restrict__ H) {
    return depth_finish(depth_issue(f, i, o, H), o, true);
}

// one of the 144 self-collision pairs (costfunc.cpp:150-193), as a load half and an
// arithmetic half (the same operations as collide_term)
struct CollPair {
    double ax, ay, az, bx, by, bz, ra, rb;
};
__device__ __forceinline__ CollPair collide_load(const FkSm &f, int t, const DevHand *__restrict__ H) {
    const int p = t / 36, k = t % 36;
    const int a = 2 + 10 * p + k / 6, b = 2 + 10 * (p + 1) + k % 6;
    return CollPair{f.S[a][0], f.S[a][1], f.S[a][2], f.S[b][0], f.S[b][1], f.S[b][2],
                    H->radii[a], H->radii[b]};
}
__device__ __forceinline__ double collide_d2(const CollPair &c) {
    const double dx = c.bx - c.ax, dy = c.by - c.ay, dz = c.bz - c.az;
    return (dx * dx + dy * dy) + dz * dz;
}
__device__ __forceinline__ double collide_value(const CollPair &c, double root) {
    const double v = (c.rb + c.ra) - root;
    return v > 0 ? v * v : 0.0;
}
__device__ __forceinline__ double collide_term(const FkSm &f, int t,
                                               const DevHand *__restrict__ H) {
    const int p = t / 36, k = t % 36;
    const int a = 2 + 10 * p + k / 6, b = 2 + 10 * (p + 1) + k % 6;
    const double dx = f.S[b][0] - f.S[a][0], dy = f.S[b][1] - f.S[a][1],
                 dz = f.S[b][2] - f.S[a][2];
    const double v = (H->radii[b] + H->radii[a]) - sqrt((dx * dx + dy * dy) + dz * dz);
    return v > 0 ? v * v : 0.0;
}

// Largest float whose correctly rounded sqrt equals sqrtf(m): BFMatcher compares
// sqrtf(d2) (OpenCV batchDistL2_32f) with first-index ties, so the match is the first
// j with d2[j] <= hi_sqrt_class(min_j d2[j]).  double->float rounding of a double sqrt
// is innocuous double rounding (53 >= 2*24+2); mid^2 is exact in double.
__device__ __forceinline__ float hi_sqrt_class(float m) {
    const float s = (float)sqrt((double)m);
    const float sn = __uint_as_float(__float_as_uint(s) + 1u);
    const double mid = 0.5 * ((double)s + (double)sn);
    const double mid2 = mid * mid;
    float h = (float)mid2;
    if ((double)h >= mid2) h = __uint_as_float(__float_as_uint(h) - 1u);
    return h;
}

// key = j if (bits(d2) <= hb) else j | 2^31 (unsigned order: the first j at or below hb
// is the minimum key), as two plain VALU ops: the sign bit of hb - bits(d2) masked in
// over j (the compiler would otherwise rebuild it as v_cmp + v_cndmask through VCC, one
// s_nop hazard each).  For non-negative floats the sign bit is exactly bits(d2) > hb.
template <int J>
__device__ __forceinline__ unsigned sqrt_class_key(int hb, float d2) {
    unsigned k;
    asm("v_sub_u32 %0, %1, %2\n\tv_and_or_b32 %0, %0, %3, %4"
        : "=&v"(k)
        : "v"(hb), "v"(__float_as_int(d2)), "s"(0x80000000u), "i"(J));
    return k;
}

// BFMatcher's match for the point (qx, qy, qz) over the 48 centres by a lane pair (this
// lane: the 24 of half h), with the matched sphere's fp64 centre and radius (lanes h == 0).
// Every lane of the wave calls it (DPP partner exchange, wave votes).
struct BfOut {
    int idx, ic;
    double cx, cy, cz, cr;
};
// fp32 squared distances of the query (qx, qy, qz) to the 24 centres SX/SY/SZ[0..23] (two
// per packed op: the same IEEE results as the scalar form), and their minimum.
__device__ __forceinline__ float bf_d2_24(const float *SX, const float *SY, const float *SZ,
                                          float qx, float qy, float qz, float (&d2)[24]) {
    typedef float f2 __attribute__((ext_vector_type(2)));  // packed fp32 (v_pk_*_f32)
    const f2 q2x = {qx, qx}, q2y = {qy, qy}, q2z = {qz, qz};
#pragma unroll
    for (int j = 0; j < 24; j += 2) {
        const f2 sx = *(const f2 *)(SX + j), sy = *(const f2 *)(SY + j),
                 sz = *(const f2 *)(SZ + j);
        const f2 t0 = q2x - sx, t1 = q2y - sy, t2 = q2z - sz;
        const f2 d = (t0 * t0 + t1 * t1) + t2 * t2;
        d2[j] = d.x;
        d2[j + 1] = d.y;
    }
    // minimum as a three-level tree of 3-way mins (v_min3_f32), not a 12-deep chain
    float m3[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) m3[k] = fminf(fminf(d2[3 * k], d2[3 * k + 1]), d2[3 * k + 2]);
    float m = fminf(fminf(fminf(m3[0], m3[1]), m3[2]), fminf(fminf(m3[3], m3[4]), m3[5]));
    return fminf(m, fminf(m3[6], m3[7]));
}
// first j in 0..23 with bits(d2[j]) <= hb, branch-free: key_j = j, or j | 2^31 when
// d2[j] > hb (non-negative floats order like their bit patterns), then an unsigned min
// tree.  Returns the smallest key (>= 64: no such j).
__device__ __forceinline__ unsigned bf_first_le_24(const float (&d2)[24], int hb) {
    unsigned key[24];
#define HPE_KEY(J) key[J] = sqrt_class_key<J>(hb, d2[J]);
    HPE_KEY(0) HPE_KEY(1) HPE_KEY(2) HPE_KEY(3) HPE_KEY(4) HPE_KEY(5) HPE_KEY(6) HPE_KEY(7)
    HPE_KEY(8) HPE_KEY(9) HPE_KEY(10) HPE_KEY(11) HPE_KEY(12) HPE_KEY(13) HPE_KEY(14)
    HPE_KEY(15) HPE_KEY(16) HPE_KEY(17) HPE_KEY(18) HPE_KEY(19) HPE_KEY(20) HPE_KEY(21)
    HPE_KEY(22) HPE_KEY(23)
#undef HPE_KEY
#pragma unroll
    for (int j = 0; j < 24; j += 3) key[j] = min(min(key[j], key[j + 1]), key[j + 2]);
    return min(min(min(key[0], key[3]), min(key[6], key[9])),
               min(min(key[12], key[15]), min(key[18], key[21])));
}
__device__ __forceinline__ BfOut bf_search(const FkSm &f, const DevHand *__restrict__ H,
                                           const float *SX, const float *SY, const float *SZ,
                                           float qx, float qy, float qz, int h,
                                           int g_ts = BT_GENS) {
    float d2[24];
    float m = bf_d2_24(SX, SY, SZ, qx, qy, qz, d2);
    BLK_TS(g_ts, 11);
    m = fminf(m, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(m), 0xB1, 0xf, 0xf,
                                                           false)));  // partner lane t^1
    // the first j of this half at or below hb, then the partner lane's half
    auto first_le = [&](int hb) {
        const unsigned kx = bf_first_le_24(d2, hb);
        const int ix = (kx >= 64u) ? (1 << 20) : (int)kx + 24 * h;
        return min(ix, __builtin_amdgcn_mov_dpp(ix, 0xB1, 0xf, 0xf, false));
    };
    // BFMatcher's match is the first j with d2[j] <= hi = hi_sqrt_class(m) (the sqrt
    // class of the minimum), and hi lies within 4 ulps above m (the class of s =
    // sqrtf(m) is narrower than 2 s ulp(s) <= 4 ulp(m)).  So the first j within 5 ulps
    // is the match whenever its own d2 IS the minimum; only otherwise (a sphere within
    // 5 ulps of the nearest, ahead of it: rare) is the exact class needed, by the whole
    // wave.  The check recomputes that sphere's fp32 d2 with the search's operations.
    int idx = first_le(__float_as_int(m) + 5);
    // the candidate's fp64 centre and radius, read ONCE: the exact check uses the float
    // of the centre (= Sp) and, unless the rare exact-class path moves idx, the
    // alignment uses them as they are (one LDS round trip on the chain, not two)
    int ic = idx < HPE_NS ? idx : 0;  // >= 48: all-NaN point (reference undefined)
    double cx = 0, cy = 0, cz = 0, cr = 0;
    bool exact = true;
    if (h == 0) {
        cx = f.S[ic][0];
        cy = f.S[ic][1];
        cz = f.S[ic][2];
        cr = H->radii[ic];
        const float tx = qx - (float)cx, ty = qy - (float)cy, tz = qz - (float)cz;
        const float dc = (tx * tx + ty * ty) + tz * tz;
        exact = (dc == m);  // false for NaN
    }
    if (__ballot(!exact)) {
        idx = first_le(__float_as_int(hi_sqrt_class(m)));
        ic = idx < HPE_NS ? idx : 0;
        if (h == 0) {
            cx = f.S[ic][0];
            cy = f.S[ic][1];
            cz = f.S[ic][2];
            cr = H->radii[ic];
        }
    }
    return BfOut{idx, ic, cx, cy, cz, cr};
}

// Fused correspondence search + alignment residual over NT threads.  Two lanes
// (t, t^1) share a point, 24 spheres each; returns this thread's partial sum of
// (|p - S[m]| - r[m])^2 and optionally stores m.
struct Pt {
    double x, y, z;
};

template <class CV>
__device__ __forceinline__ Pt load_pt(const CV &cv, int it) {
    const int p = it >> 1;
    if (it < 2 * cv.n) return Pt{cv.cx[p], cv.cy[p], cv.cz[p]};
    return Pt{0, 0, 0};
}
// pre: the point of item threadIdx.x, loaded early by the caller (load_pt) so its
// latency hides under FK.
// gt: this thread's index among the NT threads searching for the particle.
// stride / max_items (LDS cloud only): items gt, gt + stride, ... at most max_items of them
// (the refine's correspondence search spreads its items unevenly over the waves).
template <int NT, bool STORE_MATCH, class CV>
__device__ __forceinline__ double search_align(const FkSm &f, const CV &cv,
                                               const DevHand *__restrict__ H,
                                               int32_t *__restrict__ match, Pt pre,
                                               int gt = -1, int g_ts = BT_GENS,
                                               int stride = NT, int max_items = 1 << 30) {
    if (gt < 0) gt = threadIdx.x;
    double acc = 0.0;
    const int h = gt & 1;
    const float *SX = f.Sp[0] + 24 * h, *SY = f.Sp[1] + 24 * h, *SZ = f.Sp[2] + 24 * h;
    BLK_TS(g_ts, 15);
    auto item = [&](int it, const Pt &q) {
        const int p = it >> 1;
        const double X = q.x, Y = q.y, Z = q.z;
        const float qx = (float)X, qy = (float)Y, qz = (float)Z;
        const BfOut r = bf_search(f, H, SX, SY, SZ, qx, qy, qz, h, g_ts);
        const int idx = r.idx, ic = r.ic;
        const double cx = r.cx, cy = r.cy, cz = r.cz, cr = r.cr;
        if (HPE_STAMPS) asm volatile("" ::"v"(idx));
        BLK_TS(g_ts, 13);
        if (h == 0) {
            const double dx = X - cx, dy = Y - cy, dz = Z - cz;
            const double e = sqrt((dx * dx + dy * dy) + dz * dz) - cr;
            acc += e * e;
            if (STORE_MATCH) match[p] = ic;
        }
        if (HPE_STAMPS) asm volatile("" ::"v"(acc));
        BLK_TS(g_ts, 14);
    };
    if (std::is_same<CV, CloudGlobal>::value && 2 * cv.n > NT) {
        // Several items per lane from HBM (full cloud, wave form): the next item's point
        // is loaded one item ahead (unconditionally, at a clamped index), so its L2 round
        // trip overlaps this item's search instead of opening every iteration.  (An LDS
        // cloud, refine and pso_optimise, keeps the plain loop: no register cost.)
        Pt q = pre;
        for (int it = gt; it < 2 * cv.n; it += NT) {
            const int pn = min((it + NT) >> 1, cv.n - 1);
            const Pt qn = Pt{cv.cx[pn], cv.cy[pn], cv.cz[pn]};
            item(it, q);
            q = qn;
        }
    } else {
        int k = 0;
        for (int it = gt; it < 2 * cv.n && k < max_items; it += stride, ++k)
            item(it, it == gt ? pre : load_pt(cv, it));
    }
    return acc;
}

// BFMatcher's match for one point by ONE lane over all 48 centres (the wave form's search:
// no partner lane, so nothing a lane does per point is repeated by a second lane), as two
// halves of 24 with d2 in registers one half at a time.  Half X's candidate cX is its first
// j within 5 ulps of its own minimum mX.  If mA <= mB, m = mA and the whole search's first
// j within 5 ulps of m lies in A (A's minimum qualifies): cA.  If mA > mB + 5 ulps, no
// centre of A is within 5 ulps of m = mB: cB.  Either way the candidate equals bf_search's
// first pass and is the match when its d2 IS m (the same check); otherwise, or when the
// two minima are within 5 ulps of each other, the exact class is taken over both halves
// again (rare).
__device__ __forceinline__ BfOut bf_search_lane(const FkSm &f, const DevHand *__restrict__ H,
                                                float qx, float qy, float qz) {
    float d2[24];
    const float mA = bf_d2_24(f.Sp[0], f.Sp[1], f.Sp[2], qx, qy, qz, d2);
    const unsigned kA = bf_first_le_24(d2, __float_as_int(mA) + 5);
    const float mB = bf_d2_24(f.Sp[0] + 24, f.Sp[1] + 24, f.Sp[2] + 24, qx, qy, qz, d2);
    const unsigned kB = bf_first_le_24(d2, __float_as_int(mB) + 5);
    const float m = fminf(mA, mB);
    int idx = (mA <= mB) ? (int)kA : (__float_as_int(mA) > __float_as_int(mB) + 5) ? (int)kB + 24 : 64;
    int ic = idx < HPE_NS ? idx : 0;
    double cx = f.S[ic][0], cy = f.S[ic][1], cz = f.S[ic][2], cr = H->radii[ic];
    const float tx = qx - (float)cx, ty = qy - (float)cy, tz = qz - (float)cz;
    const float dc = (tx * tx + ty * ty) + tz * tz;
    if (!(idx < HPE_NS && dc == m)) {  // (false for NaN)
        const int hb = __float_as_int(hi_sqrt_class(m));
        bf_d2_24(f.Sp[0], f.Sp[1], f.Sp[2], qx, qy, qz, d2);
        const unsigned xa = bf_first_le_24(d2, hb);
        bf_d2_24(f.Sp[0] + 24, f.Sp[1] + 24, f.Sp[2] + 24, qx, qy, qz, d2);
        const unsigned xb = bf_first_le_24(d2, hb);
        idx = (xa < 64u) ? (int)xa : (xb < 64u) ? (int)xb + 24 : (1 << 20);
        ic = idx < HPE_NS ? idx : 0;  // >= 48: all-NaN point (reference undefined)
        cx = f.S[ic][0];
        cy = f.S[ic][1];
        cz = f.S[ic][2];
        cr = H->radii[ic];
    }
    return BfOut{idx, ic, cx, cy, cz, cr};
}

// The wave form's fused search + alignment (costfunc.cpp:306-377): lane l takes points
// l, l + 64, ... of an HBM cloud, the next point loaded one ahead; returns the lane's
// partial sum of (|p - S[m]| - r[m])^2.  pre = load_pt1(cv, lane).
template <class CV>
__device__ __forceinline__ Pt load_pt1(const CV &cv, int p) {
    if (p < cv.n) return Pt{cv.cx[p], cv.cy[p], cv.cz[p]};
    return Pt{0, 0, 0};
}
template <class CV>
__device__ __forceinline__ double search_align_lane(const FkSm &f, const CV &cv,
                                                    const DevHand *__restrict__ H, Pt pre) {
    double acc = 0.0;
    Pt q = pre;
    for (int p = threadIdx.x & 63; p < cv.n; p += 64) {
        // the centres are re-read from LDS per point (broadcast reads): hoisted out of the
        // loop, the 144 floats would take the registers of every other wave on the SIMD
        asm volatile("" ::: "memory");
        const int pn = min(p + 64, cv.n - 1);
        const Pt qn = Pt{cv.cx[pn], cv.cy[pn], cv.cz[pn]};
        const BfOut r = bf_search_lane(f, H, (float)q.x, (float)q.y, (float)q.z);
        const double dx = q.x - r.cx, dy = q.y - r.cy, dz = q.z - r.cz;
        const double e = sqrt((dx * dx + dy * dy) + dz * dz) - r.cr;
        acc += e * e;
        q = qn;
    }
    return acc;
}

// ---------------------------------------------------------------- filter search (wave form)
// BFMatcher's match decided from a cheap fp32 estimate of every d2, with the exact search
// only for the points whose estimate cannot decide it.  Per particle (filt_setup): an origin
// o (a central centre), s'_j = Sp_j - o, and per centre (-2 s'_j, |s'_j|^2 + 1) in LDS; per
// point q' = (float)p - o, Q = |q'|^2 and
//     a_j = ((|s'_j|^2 + 1) + Q) + q'.(-2 s'_j)          (one add + three fma per centre)
// which estimates D_j + 1, D_j = |(float)p - Sp_j|^2 (real), within
//     |a_j - (D_j + 1)| <= 11.1 u ((|q'| + |s'_j|)^2 + 1) <= 22.3 u (Q + R + 1),  u = 2^-24,
// R = max_j |s'_j|^2 (the fp32 rounding of the estimate, 9.0 u, and of the two translations,
// 2.01 u).  E = 64 u (Q + R + 1) bounds it with margin; E < 1/2 keeps every a_j positive, so
// their bit patterns order like their values.  Keys (bits(a_j) & ~63) | j give, through a
// min / second-min tree, the smallest key K1 (j* = K1 & 63) and the next K2: every other j has
// a_j >= v2 = float(K2 & ~63), and a_j* <= v1 = float(K1 | 63).  If v2 - v1 > 2E + M,
// M = 32 u (v1 + E), then D_j - D_j* > 23.2 u D_j* for every j != j*, so the reference's fp32
// d2 (within 5.01 u of D) of every other centre lies above the sqrt class of d2_j* (4 ulps,
// <= 8 u): j* is BFMatcher's match, whatever the ties in the estimate.  Otherwise (two centres
// within the bound: ~0.06 % of points on the bench sequence), bf_search_lane decides exactly.
// NaN or infinite inputs fail the test (comparisons with NaN are false) and go the exact way.
__device__ __forceinline__ float wave_max_f32(float v) {  // v >= 0 (or NaN: result unspecified)
    v = fmaxf(v, __int_as_float(dpp_i32<0xB1>(__float_as_int(v))));
    v = fmaxf(v, __int_as_float(dpp_i32<0x4E>(__float_as_int(v))));
    v = fmaxf(v, __int_as_float(dpp_i32<0x141>(__float_as_int(v))));
    v = fmaxf(v, __int_as_float(dpp_i32<0x140>(__float_as_int(v))));
    return fmaxf(fmaxf(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0)),
                       __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16))),
                 fmaxf(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32)),
                       __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48))));
}
// One wave, after FK (f's fp32 centres visible to the wave): (sx, sy, sz) = this lane's fp32
// centre, on = lane < 48.  The origin is centre FILT_ORIGIN, the most central of the model
// (over random poses its farthest centre is 9.3 cm away on average, the centres' mean 9.1):
// one broadcast LDS read instead of three wave sums.  The caller syncs before the search
// reads fs.
#define FILT_ORIGIN 21
__device__ __forceinline__ FiltC filt_setup_f(FiltSm &fs, const FkSm &f, float sx, float sy,
                                              float sz, bool on) {
    const int l = threadIdx.x & 63;
    FiltC c;
    c.ox = f.Sp[0][FILT_ORIGIN];
    c.oy = f.Sp[1][FILT_ORIGIN];
    c.oz = f.Sp[2][FILT_ORIGIN];
    const float tx = sx - c.ox, ty = sy - c.oy, tz = sz - c.oz;
    const float r2 = (tx * tx + ty * ty) + tz * tz;
    c.K = wave_max_f32(on ? r2 : 0.0f) + 1.0f;
    if (on) {
        fs.ax[l] = -2.0f * tx;
        fs.ay[l] = -2.0f * ty;
        fs.az[l] = -2.0f * tz;
        fs.aw[l] = r2 + 1.0f;
    }
    return c;
}
// the same from this lane's fp64 centre in registers (FK's own)
__device__ __forceinline__ FiltC filt_setup(FiltSm &fs, const FkSm &f, const SphXYZ &own) {
    const bool on = (threadIdx.x & 63) < HPE_NS;
    return filt_setup_f(fs, f, (float)own.x, (float)own.y, (float)own.z, on);
}
__device__ __forceinline__ unsigned med3_u32(unsigned a, unsigned b, unsigned c) {
    unsigned r;
    asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
struct Min2 {
    unsigned m, s;  // smallest, second smallest
};
__device__ __forceinline__ Min2 min2_leaf(unsigned a, unsigned b, unsigned c) {
    return Min2{min(min(a, b), c), med3_u32(a, b, c)};
}
// the second smallest of the union is the smaller of the second smallest minimum and the
// smallest second (the minimum's own group provides it, every other group's second exceeds
// that group's minimum)
__device__ __forceinline__ Min2 min2_merge3(Min2 a, Min2 b, Min2 c) {
    return Min2{min(min(a.m, b.m), c.m), min(med3_u32(a.m, b.m, c.m), min(min(a.s, b.s), c.s))};
}
__device__ __forceinline__ Min2 min2_merge2(Min2 a, Min2 b) {
    return Min2{min(a.m, b.m), med3_u32(a.m, b.m, min(a.s, b.s))};
}
template <int J0>
__device__ __forceinline__ Min2 filt_half(const FiltSm &fs, float qx, float qy, float qz, float Q) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    typedef float f2 __attribute__((ext_vector_type(2)));
    const f2 q2x = {qx, qx}, q2y = {qy, qy}, q2z = {qz, qz}, q2w = {Q, Q};
    unsigned key[24];
#pragma unroll
    for (int j = 0; j < 24; j += 4) {
        const f4 ax = *(const f4 *)(fs.ax + J0 + j), ay = *(const f4 *)(fs.ay + J0 + j),
                 az = *(const f4 *)(fs.az + J0 + j), aw = *(const f4 *)(fs.aw + J0 + j);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const f2 wx = h ? f2{ax.z, ax.w} : f2{ax.x, ax.y};
            const f2 wy = h ? f2{ay.z, ay.w} : f2{ay.x, ay.y};
            const f2 wz = h ? f2{az.z, az.w} : f2{az.x, az.y};
            const f2 ww = h ? f2{aw.z, aw.w} : f2{aw.x, aw.y};
            f2 a = ww + q2w;
            a = __builtin_elementwise_fma(q2x, wx, a);
            a = __builtin_elementwise_fma(q2y, wy, a);
            a = __builtin_elementwise_fma(q2z, wz, a);
            key[j + 2 * h] = __float_as_uint(a.x);
            key[j + 2 * h + 1] = __float_as_uint(a.y);
        }
    }
#define HPE_FKEY(J) asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(key[J]) : "v"(key[J]), "s"(0xFFFFFFC0u), "i"(J0 + J));
    HPE_FKEY(0) HPE_FKEY(1) HPE_FKEY(2) HPE_FKEY(3) HPE_FKEY(4) HPE_FKEY(5) HPE_FKEY(6)
    HPE_FKEY(7) HPE_FKEY(8) HPE_FKEY(9) HPE_FKEY(10) HPE_FKEY(11) HPE_FKEY(12) HPE_FKEY(13)
    HPE_FKEY(14) HPE_FKEY(15) HPE_FKEY(16) HPE_FKEY(17) HPE_FKEY(18) HPE_FKEY(19) HPE_FKEY(20)
    HPE_FKEY(21) HPE_FKEY(22) HPE_FKEY(23)
#undef HPE_FKEY
    Min2 L[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) L[k] = min2_leaf(key[3 * k], key[3 * k + 1], key[3 * k + 2]);
    return min2_merge3(min2_merge3(L[0], L[1], L[2]), min2_merge3(L[3], L[4], L[5]),
                       min2_merge2(L[6], L[7]));
}
__device__ __forceinline__ BfOut bf_filter_lane(const FkSm &f, const FiltSm &fs, const FiltC &c,
                                                const DevHand *__restrict__ H, float qx,
                                                float qy, float qz) {
    const float px = qx - c.ox, py = qy - c.oy, pz = qz - c.oz;
    const float Q = (px * px + py * py) + pz * pz;
    const Min2 r = min2_merge2(filt_half<0>(fs, px, py, pz, Q), filt_half<24>(fs, px, py, pz, Q));
    constexpr float U64 = 64.0f / 16777216.0f, U32 = 32.0f / 16777216.0f;
    const float E = (Q + c.K) * U64;
    const float v1 = __uint_as_float(r.m | 63u), v2 = __uint_as_float(r.s & ~63u);
    const float M = (v1 + E) * U32;
    if ((v2 - v1 > E * 2.0f + M) && (E < 0.5f)) {
        const int ic = (int)(r.m & 63u);
        return BfOut{ic, ic, f.S[ic][0], f.S[ic][1], f.S[ic][2], H->radii[ic]};
    }
    return bf_search_lane(f, H, qx, qy, qz);
}
// Two points per pass sharing every table read (the workgroup form at N = full, where a
// thread has many points and registers to spare): filt_half for points 0 and 1.
template <int J0, int U>
__device__ __forceinline__ void filt_half2(const FiltSm &fs, const float (&px)[U],
                                           const float (&py)[U], const float (&pz)[U],
                                           const float (&Q)[U], Min2 (&out)[U]) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    typedef float f2 __attribute__((ext_vector_type(2)));
    unsigned key[U][24];
#pragma unroll
    for (int j = 0; j < 24; j += 4) {
        const f4 ax = *(const f4 *)(fs.ax + J0 + j), ay = *(const f4 *)(fs.ay + J0 + j),
                 az = *(const f4 *)(fs.az + J0 + j), aw = *(const f4 *)(fs.aw + J0 + j);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const f2 wx = h ? f2{ax.z, ax.w} : f2{ax.x, ax.y};
            const f2 wy = h ? f2{ay.z, ay.w} : f2{ay.x, ay.y};
            const f2 wz = h ? f2{az.z, az.w} : f2{az.x, az.y};
            const f2 ww = h ? f2{aw.z, aw.w} : f2{aw.x, aw.y};
#pragma unroll
            for (int u = 0; u < U; ++u) {
                f2 a = ww + f2{Q[u], Q[u]};
                a = __builtin_elementwise_fma(f2{px[u], px[u]}, wx, a);
                a = __builtin_elementwise_fma(f2{py[u], py[u]}, wy, a);
                a = __builtin_elementwise_fma(f2{pz[u], pz[u]}, wz, a);
                key[u][j + 2 * h] = __float_as_uint(a.x);
                key[u][j + 2 * h + 1] = __float_as_uint(a.y);
            }
        }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
#define HPE_FKEY(J) asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(key[u][J]) : "v"(key[u][J]), "s"(0xFFFFFFC0u), "i"(J0 + J));
        HPE_FKEY(0) HPE_FKEY(1) HPE_FKEY(2) HPE_FKEY(3) HPE_FKEY(4) HPE_FKEY(5) HPE_FKEY(6)
        HPE_FKEY(7) HPE_FKEY(8) HPE_FKEY(9) HPE_FKEY(10) HPE_FKEY(11) HPE_FKEY(12) HPE_FKEY(13)
        HPE_FKEY(14) HPE_FKEY(15) HPE_FKEY(16) HPE_FKEY(17) HPE_FKEY(18) HPE_FKEY(19) HPE_FKEY(20)
        HPE_FKEY(21) HPE_FKEY(22) HPE_FKEY(23)
#undef HPE_FKEY
        Min2 L[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) L[k] = min2_leaf(key[u][3 * k], key[u][3 * k + 1], key[u][3 * k + 2]);
        out[u] = min2_merge3(min2_merge3(L[0], L[1], L[2]), min2_merge3(L[3], L[4], L[5]),
                             min2_merge2(L[6], L[7]));
    }
}
// bf_filter_lane for U points (the same test per point, the exact search where it fails)
template <int U>
__device__ __forceinline__ void bf_filter_lane2(const FkSm &f, const FiltSm &fs, const FiltC &c,
                                                const DevHand *__restrict__ H, const float (&qx)[U],
                                                const float (&qy)[U], const float (&qz)[U],
                                                BfOut (&r)[U]) {
    float px[U], py[U], pz[U], Q[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        px[u] = qx[u] - c.ox;
        py[u] = qy[u] - c.oy;
        pz[u] = qz[u] - c.oz;
        Q[u] = (px[u] * px[u] + py[u] * py[u]) + pz[u] * pz[u];
    }
    Min2 ma[U], mb[U];
    filt_half2<0, U>(fs, px, py, pz, Q, ma);
    filt_half2<24, U>(fs, px, py, pz, Q, mb);
    constexpr float U64 = 64.0f / 16777216.0f, U32 = 32.0f / 16777216.0f;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const Min2 m = min2_merge2(ma[u], mb[u]);
        const float E = (Q[u] + c.K) * U64;
        const float v1 = __uint_as_float(m.m | 63u), v2 = __uint_as_float(m.s & ~63u);
        const float M = (v1 + E) * U32;
        if ((v2 - v1 > E * 2.0f + M) && (E < 0.5f)) {
            const int ic = (int)(m.m & 63u);
            r[u] = BfOut{ic, ic, f.S[ic][0], f.S[ic][1], f.S[ic][2], H->radii[ic]};
        } else {
            r[u] = bf_search_lane(f, H, qx[u], qy[u], qz[u]);
        }
    }
}
// search_align_filt over points p0, p0 + step, ... U per pass (p, p + step, ...), the next
// pass's points loaded one pass ahead; pre = the point p0.  A pass's points past the cloud
// are evaluated at a clamped index and not added.  An empty cloud reads nothing (its
// arrays may be unallocated): n is uniform, so the early return is too.
template <int U, class CV>
__device__ __forceinline__ double search_align_filt2(const FkSm &f, const FiltSm &fs,
                                                     const FiltC &c, const CV &cv,
                                                     const DevHand *__restrict__ H, Pt pre,
                                                     int p0, int step) {
    double acc = 0.0;
    if (cv.n <= 0) return acc;
    const int n1 = cv.n - 1;
    Pt q[U];
    q[0] = pre;
#pragma unroll
    for (int u = 1; u < U; ++u) {
        const int pu = min(p0 + u * step, n1);
        q[u] = Pt{cv.cx[pu], cv.cy[pu], cv.cz[pu]};
    }
    for (int p = p0; p < cv.n; p += U * step) {
        asm volatile("" ::: "memory");  // the tables re-read from LDS per pass (registers)
        Pt qn[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int pu = min(p + (U + u) * step, n1);
            qn[u] = Pt{cv.cx[pu], cv.cy[pu], cv.cz[pu]};
        }
        float qx[U], qy[U], qz[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            qx[u] = (float)q[u].x;
            qy[u] = (float)q[u].y;
            qz[u] = (float)q[u].z;
        }
        BfOut r[U];
        bf_filter_lane2<U>(f, fs, c, H, qx, qy, qz, r);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const double dx = q[u].x - r[u].cx, dy = q[u].y - r[u].cy, dz = q[u].z - r[u].cz;
            const double e = sqrt((dx * dx + dy * dy) + dz * dz) - r[u].cr;
            if (u == 0 || p + u * step < cv.n) acc += e * e;
            q[u] = qn[u];
        }
    }
    return acc;
}
// points p0, p0 + step, ... of an HBM cloud, the next one loaded one ahead; pre = that of p0
template <class CV>
__device__ __forceinline__ double search_align_filt(const FkSm &f, const FiltSm &fs,
                                                    const FiltC &c, const CV &cv,
                                                    const DevHand *__restrict__ H, Pt pre,
                                                    int p0, int step) {
    double acc = 0.0;
    Pt q = pre;
    for (int p = p0; p < cv.n; p += step) {
        asm volatile("" ::: "memory");  // the tables re-read from LDS per point (registers)
        const int pn = min(p + step, cv.n - 1);
        const Pt qn = Pt{cv.cx[pn], cv.cy[pn], cv.cz[pn]};
        const BfOut r = bf_filter_lane(f, fs, c, H, (float)q.x, (float)q.y, (float)q.z);
        const double dx = q.x - r.cx, dy = q.y - r.cy, dz = q.z - r.cz;
        const double e = sqrt((dx * dx + dy * dy) + dz * dz) - r.cr;
        acc += e * e;
        q = qn;
    }
    return acc;
}

// Alignment with frozen correspondences (cal_cost2(..., compute_corr=false)) over
// `stride` lanes starting at `lane0`: per point e = |p - S[m]| - r[m], sum of e^2.
template <class CV>
__device__ __forceinline__ double align_frozen(const FkSm &f, const CV &cv,
                                               const DevHand *__restrict__ H,
                                               const int32_t *__restrict__ match, int lane0,
                                               int stride) {
    // fixed trip count of 4 points per lane per chunk, predicated (no divergent tail).
    // The four points' reads are issued in two batches (match + point, then the matched
    // sphere), each pinned by an empty asm that needs all of them: left to itself the
    // compiler of a kernel at the VGPR cap (k_refine) ran the points one after another,
    // five dependent LDS round trips each.
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    for (int base = 0; base < cv.n; base += 4 * stride) {
        const int n1 = cv.n - 1;
        int p[4], id[4];
        double px[4], py[4], pz[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            p[k] = base + lane0 + k * stride;
            const int q = min(p[k], n1);
            id[k] = match[q];
            px[k] = cv.cx[q];
            py[k] = cv.cy[q];
            pz[k] = cv.cz[q];
        }
        asm volatile("" : "+v"(id[0]), "+v"(id[1]), "+v"(id[2]), "+v"(id[3]), "+v"(px[0]),
                     "+v"(px[1]), "+v"(px[2]), "+v"(px[3]), "+v"(py[0]), "+v"(py[1]),
                     "+v"(py[2]), "+v"(py[3]), "+v"(pz[0]), "+v"(pz[1]), "+v"(pz[2]), "+v"(pz[3]));
        double sx[4], sy[4], sz[4], sr[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            sx[k] = f.S[id[k]][0];
            sy[k] = f.S[id[k]][1];
            sz[k] = f.S[id[k]][2];
            sr[k] = H->radii[id[k]];
        }
        asm volatile("" : "+v"(sx[0]), "+v"(sx[1]), "+v"(sx[2]), "+v"(sx[3]), "+v"(sy[0]),
                     "+v"(sy[1]), "+v"(sy[2]), "+v"(sy[3]), "+v"(sz[0]), "+v"(sz[1]),
                     "+v"(sz[2]), "+v"(sz[3]), "+v"(sr[0]), "+v"(sr[1]), "+v"(sr[2]), "+v"(sr[3]));
        double d2[4], rt[4], e[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const double dx = px[k] - sx[k], dy = py[k] - sy[k], dz = pz[k] - sz[k];
            d2[k] = (dx * dx + dy * dy) + dz * dz;
            rt[k] = hpe_sqrt_nr(d2[k]);
        }
        if (!(hpe_sqrt_direct(d2[0]) && hpe_sqrt_direct(d2[1]) && hpe_sqrt_direct(d2[2]) &&
              hpe_sqrt_direct(d2[3]))) {
#pragma unroll
            for (int k = 0; k < 4; ++k) rt[k] = hpe_sqrt_direct(d2[k]) ? rt[k] : sqrt(d2[k]);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const double r = rt[k] - sr[k];
            e[k] = r * r;
        }
        a0 += (p[0] < cv.n) ? e[0] : 0.0;
        a1 += (p[1] < cv.n) ? e[1] : 0.0;
        a2 += (p[2] < cv.n) ? e[2] : 0.0;
        a3 += (p[3] < cv.n) ? e[3] : 0.0;
    }
    return (a0 + a1) + (a2 + a3);
}

// The frozen matchIds of one lane for clouds of at most 256 points (the reference's
// down-sampled cloud, N = 250): those of points l + 64 k, loaded once per refine iteration
// after the correspondence search, so a node evaluation's alignment issues the point and
// matched-sphere reads together (one LDS round trip instead of two).
#define FP_MAX 256
struct FrozenPts {
    int id[4];
};
template <class CV>
__device__ __forceinline__ void load_frozen_pts(FrozenPts &fp, const CV &cv,
                                                const int32_t *__restrict__ match, int l) {
#pragma unroll
    for (int k = 0; k < 4; ++k) fp.id[k] = cv.n > 0 ? match[min(l + 64 * k, cv.n - 1)] : 0;
}
// align_frozen over the lane's points (n <= FP_MAX): the same per-point operations
template <class CV>
__device__ __forceinline__ double align_frozen_pts(const FkSm &f, const FrozenPts &fp,
                                                   const CV &cv, const DevHand *__restrict__ H,
                                                   int l) {
    double px[4], py[4], pz[4], sx[4], sy[4], sz[4], sr[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int q = min(l + 64 * k, max(cv.n - 1, 0));  // (n = 0: every term masked below)
        px[k] = cv.cx[q];
        py[k] = cv.cy[q];
        pz[k] = cv.cz[q];
        sx[k] = f.S[fp.id[k]][0];
        sy[k] = f.S[fp.id[k]][1];
        sz[k] = f.S[fp.id[k]][2];
        sr[k] = H->radii[fp.id[k]];
    }
    asm volatile("" : "+v"(sx[0]), "+v"(sx[1]), "+v"(sx[2]), "+v"(sx[3]), "+v"(sy[0]),
                 "+v"(sy[1]), "+v"(sy[2]), "+v"(sy[3]), "+v"(sz[0]), "+v"(sz[1]),
                 "+v"(sz[2]), "+v"(sz[3]), "+v"(sr[0]), "+v"(sr[1]), "+v"(sr[2]), "+v"(sr[3]),
                 "+v"(px[0]), "+v"(px[1]), "+v"(px[2]), "+v"(px[3]), "+v"(py[0]), "+v"(py[1]),
                 "+v"(py[2]), "+v"(py[3]), "+v"(pz[0]), "+v"(pz[1]), "+v"(pz[2]), "+v"(pz[3]));
    const int n = cv.n;
    double d2[4], rt[4], e[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const double dx = px[k] - sx[k], dy = py[k] - sy[k], dz = pz[k] - sz[k];
        d2[k] = (dx * dx + dy * dy) + dz * dz;
        rt[k] = hpe_sqrt_nr(d2[k]);
    }
    if (!(hpe_sqrt_direct(d2[0]) && hpe_sqrt_direct(d2[1]) && hpe_sqrt_direct(d2[2]) &&
          hpe_sqrt_direct(d2[3]))) {
#pragma unroll
        for (int k = 0; k < 4; ++k) rt[k] = hpe_sqrt_direct(d2[k]) ? rt[k] : sqrt(d2[k]);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const double r = rt[k] - sr[k];
        e[k] = (l + 64 * k < n) ? r * r : 0.0;
    }
    return (e[0] + e[1]) + (e[2] + e[3]);
}

#ifndef HPE_SETPRIO_FROM
#define HPE_SETPRIO_FROM 4  // first wave of a 512-thread block raised during the search
#endif
enum EvalMode { EV_COST = 0, EV_COST2_CORR = 1, EV_COST2_FROZEN = 2, EV_COST_STORE = 3 };

// cal_cost of the particle in f.th by WPP waves of one workgroup (the throughput form used
// when there are many more particles than CUs): each wave runs FK on its own workspace (the
// same operations on the same inputs: the same bits) and searches points l + 64 sub,
// l + 64 (sub + WPP), ...; sub 0 adds the depth terms.  WPP = 2 or 4 (swarms of at most one
// particle per SIMD) cuts the search's latency; the wave totals are added in sub order
// through xpart (indexed by wave) behind a workgroup barrier that every wave reaches.
// All lanes of the particle's waves return the total; pre = load_pt1(cv, l + 64 sub).
// COOP: FK by the whole workgroup (fk_coop over its NPW / WPP particles, particle p's
// centres in fks[p * WPP], read by all its waves); otherwise each wave runs its own (fk_wave
// on fks[w]).
template <int WPP, bool COOP, int NPW, class CV>
__device__ __forceinline__ double eval_wave_cost(FkSm *fks, FiltSm &fs, const DevObs &o,
                                                 const CV &cv, const DevHand *__restrict__ H,
                                                 Pt pre, int sub, double *xpart,
                                                 int g_ts = BT_GENS) {
    const int l = threadIdx.x & 63;
    FkSm &f = fks[COOP ? (threadIdx.x >> 6) - sub : (threadIdx.x >> 6)];
    SphXYZ own;
    if (COOP) {
        fk_coop<NPW / WPP, WPP>(fks, H);
        const int sl = l < HPE_NS ? l : HPE_NS - 1;
        own = SphXYZ{f.S[sl][0], f.S[sl][1], f.S[sl][2]};
        if (l >= HPE_NS) own = SphXYZ{0.0, 0.0, 0.0};
    } else {
        fk_wave(f, H, &own);
    }
    WAVE_TS2(g_ts, 4);
    const DepthG dg = depth_issue_at(own, l, o, H);
    const FiltC fc = filt_setup(fs, f, own);
    wave_sync();
    WAVE_TS2(g_ts, 5);
    // two or four waves per particle (small swarms, registers to spare): two points per
    // pass share each table read; one wave per particle stays at 128 VGPRs with one
    double al = WPP > 1 ? search_align_filt2<2>(f, fs, fc, cv, H, pre, l + 64 * sub, 64 * WPP)
                        : search_align_filt(f, fs, fc, cv, H, pre, l + 64 * sub, 64 * WPP);
    if (HPE_STAMPS) asm volatile("" ::"v"(al));
    WAVE_TS2(g_ts, 6);
    double dep = depth_finish(dg, o, l < HPE_NS && sub == 0);
    const double part = wave_sum(al * o.lambda + dep);
    if (HPE_STAMPS) asm volatile("" ::"v"(part));
    WAVE_TS2(g_ts, 7);
    if (WPP == 1) return part;
    const int w = threadIdx.x >> 6;
    if (l == 0) xpart[w] = part;
    __syncthreads();
    double tot = xpart[w - sub];
#pragma unroll
    for (int k = 1; k < WPP; ++k) tot += xpart[w - sub + k];
    return tot;
}

__device__ __forceinline__ CloudGlobal obs_cloud(const DevObs &o) {
    return CloudGlobal{gp(o.cx), gp(o.cy), gp(o.cz), o.n};
}

// Whole-block evaluation of the particle in sm.fk.th (wave 0 does FK, NT threads the
// search).  Every thread returns the total; terms (align, depth, collision) go to
// sm.dscal[0..2].
// FK = false: the caller has already placed the centres in sm.fk.S / Sp (hpe_eval_spheres).
// own_w0 (FK = false): the centres wave 0's FK (run by the caller) left in its registers,
// projected here without re-reading them from LDS; otherwise read from sm.fk.
template <int MODE, int NT, bool FK = true, bool FILT = false, class CV>
__device__ __forceinline__ double eval_block(Smem &sm, const DevObs &o, const CV &cv,
                                             const DevHand *__restrict__ H,
                                             int32_t *__restrict__ match, Pt pre,
                                             int g_ts = BT_GENS, const SphXYZ *own_w0 = nullptr,
                                             bool with_depth = true) {
    StampClock sc;
    sc.start();
    const int t = threadIdx.x;
    SphXYZ own{0.0, 0.0, 0.0};
    if (FK) {
        if (t < 64) fk_wave(sm.fk, H, &own);
        __syncthreads();
    } else if (own_w0) {
        own = *own_w0;
    }
    sc.lap(10);
    // FILT (the host's choice for frames of more than NT / 2 points, N = full): cal_cost over
    // the HBM cloud by the filter search, one thread per point (bf_filter_lane: the same
    // matches, about half the instructions of the lane-pair search); wave 0 builds the
    // tables, one barrier publishes them.  Every kernel of a frame makes the same choice.
    constexpr bool filt = FILT && MODE == EV_COST && std::is_same<CV, CloudGlobal>::value;
    Pt pre1{0.0, 0.0, 0.0};
    FiltC fc{0.f, 0.f, 0.f, 0.f};
    if constexpr (filt) {
        pre1 = load_pt1(cv, t);
        if (t < 64) {
            const int sl = t < HPE_NS ? t : 0;
            const FiltC c = filt_setup_f(sm.flt, sm.fk, sm.fk.Sp[0][sl], sm.fk.Sp[1][sl],
                                         sm.fk.Sp[2][sl], t < HPE_NS);
            if (t == 0) sm.fltc = c;
        }
        __syncthreads();
        fc = sm.fltc;
    }
    // wave 0 issues the depth gathers first (after the barrier: the other waves start
    // searching at once): their latency hides under the search
    DepthG dg{0.0, 0.0, 0.0, 0.f, false};
    if (t < 64 && with_depth) dg = (FK || own_w0) ? depth_issue_at(own, t, o, H) : depth_issue(sm.fk, t, o, H);
    // Waves 4..7 share the SIMDs with waves 0..3 and lose the age arbitration: they reached
    // the reduction ~0.5 us after waves 1..3.  Static priority for that half during the
    // search (MI355X_MICROARCH.md, two waves per SIMD, item 4).
    const bool young = NT == 512 && (t >> 6) >= HPE_SETPRIO_FROM;
    if (young) __builtin_amdgcn_s_setprio(1);
    double al;
    if (MODE == EV_COST2_FROZEN) al = align_frozen(sm.fk, cv, H, match, t, NT);
    else if (MODE == EV_COST2_CORR || MODE == EV_COST_STORE)
        al = search_align<NT, true>(sm.fk, cv, H, match, pre);
    else if (filt) al = search_align_filt2<FILT_PTS>(sm.fk, sm.flt, fc, cv, H, pre1, t, NT);
    else al = search_align<NT, false>(sm.fk, cv, H, nullptr, pre, -1, g_ts);
    if (young) __builtin_amdgcn_s_setprio(0);
    const bool coll = (MODE == EV_COST2_CORR || MODE == EV_COST2_FROZEN);
    double co = (coll && t < 144) ? collide_term(sm.fk, t, H) : 0.0;
    BLK_TS(g_ts, 8);
    double dep = depth_finish(dg, o, with_depth && t < HPE_NS);
    BLK_TS(g_ts, 9);
    if (HPE_STAMPS) asm volatile("" ::"v"(al), "v"(dep));
    WAVE_TS(g_ts, 16);
    sc.lap(11);
    if constexpr (!(MODE == EV_COST2_CORR || MODE == EV_COST2_FROZEN)) {
        // cal_cost (the PSO's evaluations): the lane totals summed once (block_sum1); the
        // separate terms are not formed
        const double tot = block_sum1<NT, false>(sm.red, al * o.lambda + dep);
        sc.lap(12);
        if (t == 0) {
            sm.dscal[0] = __builtin_nan("");
            sm.dscal[1] = __builtin_nan("");
            sm.dscal[2] = 0.0;
        }
        return tot;
    }
    block_sum3<NT, false>(sm.red, al, dep, co);
    sc.lap(12);
    const double align = al * o.lambda;
    if (t == 0) {
        sm.dscal[0] = align;
        sm.dscal[1] = dep;
        sm.dscal[2] = co;
    }
    if (!coll) return align + dep;
    return (align + dep) + co;
}

// One wave evaluates cal_cost2(f.th, match, false): FK, frozen alignment over the
// whole cloud, depth, collision; wave-local synchronisation only.  All lanes return
// the total.
// Xt != nullptr: f.th differs from the theta of Xt only in the global position
// (FK_TRANSLATE).
// In two halves: frozen_head (FK, the depth gathers issued, the collision sum) needs no
// correspondences, so the refine runs it for the gradient points while the previous
// correspondence search is still being reduced; frozen_tail (frozen alignment, depth,
// the three wave sums) reads matchId.
struct FrozenHead {
    DepthG dg;
    double co;
};
template <bool OUTLINE_TRIG = false>
__device__ __forceinline__ FrozenHead frozen_head(FkSm &f, const DevObs &o,
                                                  const DevHand *__restrict__ H,
                                                  FkX *Xt = nullptr, const double *thr = nullptr) {
    SphXYZ own;
    if (Xt) fk_wave_t<FK_TRANSLATE>(f, H, Xt, &own);
    else fk_wave<OUTLINE_TRIG>(f, H, &own, thr);
    const int l = threadIdx.x & 63;
    FrozenHead r;
    r.dg = depth_issue_at(own, l, o, H);
    // three pairs per lane (the third for lanes 0..15, computed by every lane at a clamped
    // index and selected): every LDS read of the three is issued before any is used, so
    // they share one round trip
    CollPair cp[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) cp[k] = collide_load(f, k < 2 ? l + 64 * k : ((l < 16) ? l + 128 : l), H);
    asm volatile("" ::"v"(cp[0].ax), "v"(cp[1].ax), "v"(cp[2].ax));
    double d2[3], rt[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        d2[k] = collide_d2(cp[k]);
        rt[k] = hpe_sqrt_nr(d2[k]);
    }
    if (!(hpe_sqrt_direct(d2[0]) && hpe_sqrt_direct(d2[1]) && hpe_sqrt_direct(d2[2]))) {
#pragma unroll
        for (int k = 0; k < 3; ++k) rt[k] = hpe_sqrt_direct(d2[k]) ? rt[k] : sqrt(d2[k]);
    }
    r.co = collide_value(cp[0], rt[0]) + collide_value(cp[1], rt[1]) +
           ((l < 16) ? collide_value(cp[2], rt[2]) : 0.0);
    return r;
}
// frozen_head of the rigid refine (rigid_wave above): the collision is the constant R.C,
// added by the caller after the sum.
template <int MODE>
__device__ __forceinline__ FrozenHead rigid_head(FkSm &f, const DevObs &o,
                                                 const DevHand *__restrict__ H,
                                                 const RigidSm &R, double thl) {
    SphXYZ own;
    rigid_wave<MODE>(f, R, thl, &own);
    FrozenHead r;
    r.dg = depth_issue_at(own, threadIdx.x & 63, o, H);
    r.co = 0.0;
    return r;
}
// RIGID (hand-frame refine): no collision term (it is the call's constant, added by the
// caller), and md2p carries the lane's off-image depth value computed once per call.  The
// lane total al * lambda + dep is >= +0, so leaving out "+ 0.0" changes no bit.
template <bool RIGID = false, class CV>
__device__ __forceinline__ double frozen_tail(const FkSm &f, const DevObs &o, const CV &cv,
                                              const DevHand *__restrict__ H,
                                              const int32_t *__restrict__ match,
                                              FrozenHead hd, const FrozenPts *fp = nullptr,
                                              const double *md2p = nullptr) {
    const int l = threadIdx.x & 63;
    double al = fp ? align_frozen_pts(f, *fp, cv, H, l) : align_frozen(f, cv, H, match, l, 64);
    double co = hd.co;
    if (!RIGID) asm volatile("" ::"v"(co));  // complete before depth_finish's wait for the gathers
    const double dep = depth_finish(hd.dg, o, l < HPE_NS, md2p);
    // one wave sum of the lane totals (the three terms' sums in another order: the same
    // value to the last bits, as any order of the reference's own sums)
    if (RIGID) return wave_sum(al * o.lambda + dep);
    return wave_sum((al * o.lambda + dep) + co);
}
template <bool OUTLINE_TRIG = false, class CV>
__device__ __forceinline__ double eval_wave_frozen(FkSm &f, const DevObs &o,
                                                   const CV &cv,
                                                   const DevHand *__restrict__ H,
                                                   const int32_t *__restrict__ match,
                                                   FkX *Xt = nullptr, const double *thr = nullptr,
                                                   const FrozenPts *fp = nullptr) {
    return frozen_tail(f, o, cv, H, match, frozen_head<OUTLINE_TRIG>(f, o, H, Xt, thr), fp);
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
        // each 32 x 32 -> 64 product as ONE v_mad_u64_u32 (the compiler emits a mul_lo /
        // mul_hi pair: two quarter-rate instructions for one)
        uint64_t p0, p1;
        asm("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(p0) : "s"(0xD2511F53u), "v"(c0) : "vcc");
        asm("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(p1) : "s"(0xCD9E8D57u), "v"(c2) : "vcc");
        const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
        const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
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

