// hpe_prep.hpp -- observedmodel preprocessing on the GPU:
//   depth mm -> cm                                   (observedmodel.cpp:296-308)
//   point cloud of the non-zero pixels, row-major    (observedmodel.cpp:110-169)
//   cm-per-pixel scale = mean of 2 / |d(u,v)|        (observedmodel.cpp:171-202)
//   down-sample to rows k * floor(N / 250)           (observedmodel.cpp:204-217)
//   5x5 chamfer distance transform of the background (observedmodel.cpp:313-358,
//     OpenCV distanceTransform(CV_DIST_L2, 5): 16.16 fixed point, weights 1 / 1.4 / 2.1969)
//
// Workgroups (PREP_WG of them, PREP_NT threads each, in one launch):
//   PREP_BANDS "band" workgroups: 30 image rows each -- depth, per-pixel cloud point and
//     scale term, compacted in pixel order within the band.  The last band to finish
//     merges: band offsets, the scale mean replayed in Armadillo's order (two alternating
//     sequential accumulators), the (down-sampled) cloud.
//   one DT workgroup: the chamfer raster scans by ONE wave, lane l holding columns
//     5l..5l+4, rows in registers; the in-row dependency T_c = min(a_c, T_{c-1} + 1) is a
//     prefix minimum (lane-serial over 5 columns, DPP across lanes).  Integer min-plus
//     arithmetic: exactly the raster-scan values.
// Results equal hpe_preprocess_depth bit for bit.  Hand-offs between workgroups follow
// MI355X_MICROARCH.md (inter-workgroup visibility): every storing wave waits for its
// stores, workgroup barrier, agent release, arrival counter; the last arriver acquires.
#pragma once
#include "hpe_device.hpp"

#define PREP_NT 512
#define PREP_BANDS 8
#define PREP_WG (PREP_BANDS + 1)
#define PREP_ROWS (HPE_IMG_H / PREP_BANDS)      // 30
#define PREP_BAND_PIX (PREP_ROWS * HPE_IMG_W)  // 9600
#define PREP_CH 4096                           // scale terms staged in LDS per pass
#define DT_HV 65536
#define DT_DIAG 91750
#define DT_LONG 143976
#define DT_INIT (0x7FFFFFFF >> 2)

struct PrepInfo {
    int n_full, n;
    double scale, dtmax;
    int band_n[PREP_BANDS], band_h[PREP_BANDS];  // points / scale terms per band
};

// Arguments of one frame preparation (device pointers of the destination slot).
struct PrepArgs {
    const float *raw;
    int to_cm, downsample;
    double focal;
    double *depth_cm, *cx, *cy, *cz, *tmp, *ctb;
    float *dt;
    int *dtf;
    PrepInfo *info;
    DevObs *obs_out;
    unsigned *ctr;  // [0] bands arrived, [1] (merged cloud, DT) arrived, [2] DT has its mask
    // resident raw sequences (hpe_track_raw_sequence_dev): raw is the sequence's first frame
    // and the frame prepared is the one after the device row cursor's (*raw_row + 1), so a
    // captured chunk graph serves every chunk; null: raw is the frame itself
    const int *raw_row;
    unsigned long long raw_stride;  // floats per raw frame
};

// LDS layout: chunk[PREP_CH] doubles | acc1, flag (64 B) | wcnt, hcnt | mask bits | wmax
constexpr int prep_lds_bytes() {
    return PREP_CH * 8 + 64 + 2 * (PREP_NT / 64) * 4 + HPE_IMG_W * HPE_IMG_H / 32 * 4 + 64;
}

// inclusive prefix minimum over lanes 0..63 of a wave (DPP row shifts + row broadcasts)
__device__ __forceinline__ int wave_prefix_min(int v) {
    const int id = 0x7FFFFFFF;
    v = min(v, __builtin_amdgcn_update_dpp(id, v, 0x111, 0xf, 0xf, false));  // row_shr:1
    v = min(v, __builtin_amdgcn_update_dpp(id, v, 0x112, 0xf, 0xf, false));  // row_shr:2
    v = min(v, __builtin_amdgcn_update_dpp(id, v, 0x114, 0xf, 0xf, false));  // row_shr:4
    v = min(v, __builtin_amdgcn_update_dpp(id, v, 0x118, 0xf, 0xf, false));  // row_shr:8
    v = min(v, __builtin_amdgcn_update_dpp(id, v, 0x142, 0xa, 0xf, false));  // row_bcast:15
    v = min(v, __builtin_amdgcn_update_dpp(id, v, 0x143, 0xc, 0xf, false));  // row_bcast:31
    return v;
}
// inclusive prefix minimum of five values in two levels of v_min3
__device__ __forceinline__ void scan5_min(const int q[5], int p[5]) {
    p[0] = q[0];
    p[1] = min(q[0], q[1]);
    p[2] = min(min(q[0], q[1]), q[2]);
    p[3] = min(min(p[1], q[2]), q[3]);
    p[4] = min(min(p[2], q[3]), q[4]);
}
// value of lane l-1 (lane 0: fill) / lane l+1 (lane 63: fill)
__device__ __forceinline__ int from_left(int v, int fill) {
    return __builtin_amdgcn_update_dpp(fill, v, 0x138, 0xf, 0xf, false);  // wave_shr:1
}
__device__ __forceinline__ int from_right(int v, int fill) {
    return __builtin_amdgcn_update_dpp(fill, v, 0x130, 0xf, 0xf, false);  // wave_shl:1
}

// Producer side of a hand-off, then the arrival; returns (to every thread) whether this
// workgroup arrived last of `parties` (it then holds an agent acquire).
__device__ __forceinline__ bool prep_arrive_last(unsigned *ctr, unsigned parties, int *flag) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's stores are out
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned old = atomicAdd(ctr, 1u);
        const bool last = (old == parties - 1);
        if (last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            *ctr = 0u;  // ready for the next frame (the kernel boundary orders it)
        }
        *flag = last ? 1 : 0;
    }
    __syncthreads();
    return __builtin_amdgcn_readfirstlane(*flag) != 0;  // decides exits and barriers (§7)
}

// The same for many arriving workgroups: one counter per shard (blockIdx % ARRIVE_SHARDS,
// each on its own 128-B line) and a top counter the last of every shard increments, so
// no address takes more than parties / ARRIVE_SHARDS + ARRIVE_SHARDS atomics (hundreds of
// same-address atomics serialise at ~11-13 ns each).  ctr: ARRIVE_SHARDS * 32 + 1 words,
// reset by the last arriver.
#define ARRIVE_SHARDS 16
__device__ __forceinline__ bool arrive_last_sharded(unsigned *ctr, unsigned parties, int *flag) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned s = blockIdx.x % ARRIVE_SHARDS;
        const unsigned used = parties < ARRIVE_SHARDS ? parties : ARRIVE_SHARDS;
        const unsigned size = parties / ARRIVE_SHARDS + (s < parties % ARRIVE_SHARDS ? 1u : 0u);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        bool last = false;
        if (atomicAdd(&ctr[s * 32], 1u) == size - 1) {  // last of its shard
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "agent");
            last = atomicAdd(&ctr[ARRIVE_SHARDS * 32], 1u) == used - 1;
        }
        if (last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            for (int k = 0; k < ARRIVE_SHARDS; ++k) ctr[k * 32] = 0u;  // for the next launch
            ctr[ARRIVE_SHARDS * 32] = 0u;
        }
        *flag = last ? 1 : 0;
    }
    __syncthreads();
    return __builtin_amdgcn_readfirstlane(*flag) != 0;  // decides exits and barriers (§7)
}

// ---- band workgroup b: rows [30b, 30b + 30)
__device__ __forceinline__ void prep_band(const PrepArgs &a, int b, unsigned char *lds) {
    constexpr int W = HPE_IMG_W, NWV = PREP_NT / 64;
    int *wcnt = (int *)(lds + PREP_CH * 8 + 64), *hcnt = wcnt + NWV;
    const int t = threadIdx.x, w = t >> 6, l = t & 63;
    const double focal = a.focal;
    const double c0 = 320 / 2., c1 = 240 / 2.;
    const double Kv[9] = {focal, 0.0, c0, 0.0, focal, c1, 0.0, 0.0, 1.0};
    const int pbase = b * PREP_BAND_PIX;
    double *tmpb = a.tmp + 3 * (size_t)pbase, *ctbb = a.ctb + pbase;
    int base = 0, ncm = 0;
    if (t == 0) {  // after the DT workgroup's raw reads (bounded: ~1 ms, then go anyway)
        for (int i = 0; i < 4096 && __hip_atomic_load(&a.ctr[2], __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT) == 0u; ++i)
            __builtin_amdgcn_s_sleep(8);
    }
    __syncthreads();
    // the band's raw pixels, all loads in flight at once (unconditional, clamped): one
    // round trip, also when the raw frame is read from pinned host memory over PCIe
    constexpr int NPASS = (PREP_BAND_PIX + PREP_NT - 1) / PREP_NT;
    float rvs[NPASS];
#pragma unroll
    for (int k = 0; k < NPASS; ++k) rvs[k] = a.raw[pbase + min(k * PREP_NT + t, PREP_BAND_PIX - 1)];
#pragma unroll
    for (int k = 0; k < NPASS; ++k) {
        const int p0 = k * PREP_NT;
        const int q = p0 + t, pix = pbase + q;
        const bool in = q < PREP_BAND_PIX;
        const float rv = rvs[k];
        const double Z = a.to_cm ? (double)rv / 10. : (double)rv;
        if (in) a.depth_cm[pix] = Z;
        const bool nz = in && Z != 0;
        const unsigned long long bm = __ballot(nz);
        const int wpre = __popcll(bm & ((1ull << l) - 1));
        double contrib = 0, X = 0, Y = 0;
        bool has = false;
        if (nz) {
            const int r = pix / W, c = pix - W * r;
            X = ((c - c0) * Z) / focal;
            Y = ((r - c1) * Z) / focal;
            const double ww = (Kv[6] * X + Kv[7] * Y) + Kv[8] * Z;
            const double u = (Kv[0] * X + Kv[1] * Y) + Kv[2] * Z;
            const double v = (Kv[3] * X + Kv[4] * Y) + Kv[5] * Z;
            const double Xe = X + 2.0;
            const double we = (Kv[6] * Xe + Kv[7] * Y) + Kv[8] * Z;
            const double ue = (Kv[0] * Xe + Kv[1] * Y) + Kv[2] * Z;
            const double ve = (Kv[3] * Xe + Kv[4] * Y) + Kv[5] * Z;
            const double du = floor(ue / we) - floor(u / ww);
            const double dv = floor(ve / we) - floor(v / ww);
            const double dn = sqrt(du * du + dv * dv);
            if (dn != 0) {
                contrib = 2.0 / dn;
                has = true;
            }
        }
        const unsigned long long bh = __ballot(has);
        const int hpre = __popcll(bh & ((1ull << l) - 1));
        if (l == 0) {
            wcnt[w] = __popcll(bm);
            hcnt[w] = __popcll(bh);
        }
        __syncthreads();
        int off = base, hoff = ncm, tot = 0, htot = 0;
#pragma unroll
        for (int k = 0; k < NWV; ++k) {
            off += (k < w) ? wcnt[k] : 0;
            hoff += (k < w) ? hcnt[k] : 0;
            tot += wcnt[k];
            htot += hcnt[k];
        }
        if (nz) {
            const int idx = off + wpre;
            tmpb[3 * idx + 0] = X;
            tmpb[3 * idx + 1] = Y * -1;
            tmpb[3 * idx + 2] = Z * -1;
        }
        if (has) ctbb[hoff + hpre] = contrib;  // the mean's terms, in pixel order
        base += tot;
        ncm += htot;
        __syncthreads();
    }
    if (t == 0) {
        a.info->band_n[b] = base;
        a.info->band_h[b] = ncm;
    }
}

// ---- merge (the last band to arrive): offsets, the scale mean, the (down-sampled) cloud
__device__ __forceinline__ void prep_merge(const PrepArgs &a, unsigned char *lds) {
    double *chunk = (double *)lds;
    double *acc1p = chunk + PREP_CH;
    const int t = threadIdx.x;
    int noff[PREP_BANDS + 1], hoff[PREP_BANDS + 1];
    noff[0] = hoff[0] = 0;
#pragma unroll
    for (int b = 0; b < PREP_BANDS; ++b) {
        noff[b + 1] = noff[b] + a.info->band_n[b];
        hoff[b + 1] = hoff[b] + a.info->band_h[b];
    }
    const int n_full = noff[PREP_BANDS], ncm = hoff[PREP_BANDS];
    // arma::mean = accumulate / n: two accumulators take the terms alternately, each a
    // sequential sum (arrayops::accumulate); threads 0 and 1 replay them from LDS chunks
    double acc = 0;
    for (int b0 = 0; b0 < ncm; b0 += PREP_CH) {
        const int m = min(PREP_CH, ncm - b0);
        for (int k = t; k < m; k += PREP_NT) {
            const int g = b0 + k;
            int b = 0;
#pragma unroll
            for (int q = 1; q < PREP_BANDS; ++q) b = (g >= hoff[q]) ? q : b;
            chunk[k] = a.ctb[(size_t)b * PREP_BAND_PIX + (g - hoff[b])];
        }
        __syncthreads();
        if (t < 2) {  // eight LDS reads in flight ahead of the dependent adds
            int k = ((b0 + t) & 1) ? 1 : 0;
            for (; k + 14 < m; k += 16) {
                double v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) v[u] = chunk[k + 2 * u];
#pragma unroll
                for (int u = 0; u < 8; ++u) acc += v[u];
            }
            for (; k < m; k += 2) acc += chunk[k];
        }
        __syncthreads();
    }
    if (t == 1) *acc1p = acc;
    const int n = a.downsample ? 250 : n_full;
    const int f = n_full / 250;
    for (int k = t; k < n; k += PREP_NT) {
        double x = 0, y = 0, z = 0;
        const int src = a.downsample ? k * f : k;
        if (!a.downsample || n_full > 0) {
            int b = 0;
#pragma unroll
            for (int q = 1; q < PREP_BANDS; ++q) b = (src >= noff[q]) ? q : b;
            const double *p = a.tmp + 3 * ((size_t)b * PREP_BAND_PIX + (src - noff[b]));
            x = p[0];
            y = p[1];
            z = p[2];
        }
        a.cx[k] = x;
        a.cy[k] = y;
        a.cz[k] = z;
    }
    __syncthreads();
    if (t == 0) {
        a.info->n_full = n_full;
        a.info->n = n;
        a.info->scale = ncm ? (acc + *acc1p) / ncm : __builtin_nan("");
    }
}

// ---- DT workgroup: mask bits by all waves, the raster scans by wave 0
__device__ __forceinline__ void prep_dt(const PrepArgs &a, unsigned char *lds) {
    constexpr int W = HPE_IMG_W, H = HPE_IMG_H;
    unsigned *msk = (unsigned *)(lds + PREP_CH * 8 + 64 + 2 * (PREP_NT / 64) * 4);
    float *wmaxp = (float *)(msk + W * H / 32);
    const int t = threadIdx.x, l = t & 63;
    // hand = non-zero raw depth: 150 pixels per thread in three batches of 50 loads, the
    // next batch in flight while one is folded (unconditional: no branch splits them into
    // one round trip each; the raw frame may sit in pinned host memory, behind PCIe)
    constexpr int NPT = W * H / PREP_NT, B = NPT / 3;  // 150 pixels per thread, 3 batches
    static_assert(W * H % PREP_NT == 0 && NPT % 3 == 0, "whole batches");
    float va[B], vb[B];
    auto issue = [&](float (&v)[B], int k0) {
#pragma unroll
        for (int q = 0; q < B; ++q) v[q] = a.raw[(k0 + q) * PREP_NT + t];
    };
    auto fold = [&](const float (&v)[B], int k0) {
#pragma unroll
        for (int q = 0; q < B; ++q) {
            const unsigned long long bm = __ballot(v[q] != 0.f);
            const int pix = (k0 + q) * PREP_NT + t;
            if ((l & 31) == 0) msk[pix >> 5] = (unsigned)(bm >> (l & 32));
        }
    };
    issue(va, 0);
    issue(vb, B);
    fold(va, 0);
    issue(va, 2 * B);  // the third batch lands while the second is folded
    fold(vb, B);
    fold(va, 2 * B);
    // the band workgroups hold their own raw reads until here (a scheduling hint only):
    // when the frame sits in host memory the DT, the longer chain, gets PCIe to itself
    if (t == 0) __hip_atomic_store(&a.ctr[2], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int *rfirst = (int *)(msk + W * H / 32 + 1);
    if (t == 0) {
        msk[W * H / 32] = 0u;  // the two-word window of the last pixels
        *rfirst = 0x7FFFFFFF;
    }
    __syncthreads();
    for (int k = t; k < W * H / 32; k += PREP_NT) {  // first mask word holding a hand pixel
        if (msk[k] != 0u) {
            atomicMin(rfirst, k);
            break;
        }
    }
    __syncthreads();
    // The forward pass starts at the first row r0 holding a hand pixel.  Above it every
    // forward value is >= DT_INIT; with a hand pixel anywhere, every pixel's final value is
    // finite (< DT_INIT: a forward path right/down from some hand pixel, then a backward
    // path up/left, stays inside the image), so forward values >= DT_INIT never win a min
    // and any such value gives the same result: the rows above r0 start from DT_INIT, as
    // row 0 does, and the backward pass reads DT_INIT for them.  No hand pixel: r0 = 0.
    const int r0 = (*rfirst == 0x7FFFFFFF) ? 0 : *rfirst / (W / 32);
    if (t < 64) {
        // forward pass: lane l owns columns c0..c0+4; u1 / u2 = rows r-1 / r-2 at columns
        // c0-2 .. c0+6 (halo from the neighbour lanes)
        const int c0 = 5 * l;
        int u1[9], u2[9];
#pragma unroll
        for (int i = 0; i < 9; ++i) u1[i] = u2[i] = DT_INIT;
        // rows in pairs from the even row at or above r0 (a row above r0 scanned from
        // DT_INIT is as good as unscanned, see above), two rows per trip
        static_assert(H % 2 == 0, "forward rows in pairs");
        auto row = [&](int r) {
            const int pix0 = r * W + c0;
            const unsigned long long mw =
                ((unsigned long long)msk[(pix0 >> 5) + 1] << 32) | msk[pix0 >> 5];
            const unsigned hb = (unsigned)(mw >> (pix0 & 31));
            int q[5], p[5];
#pragma unroll
            for (int k = 0; k < 5; ++k) {
                const int i = k + 2;
                // grouped by weight: min over the LONG, DIAG and HV neighbours, then the add
                const int mL = min(min(u2[i - 1], u2[i + 1]), min(u1[i - 2], u1[i + 2]));
                const int mD = min(u1[i - 1], u1[i + 1]);
                const int av = min(min(mL + DT_LONG, mD + DT_DIAG), u1[i] + DT_HV);
                // hand pixel -> 0: bit k sign-extended, then av & ~mask in one v_bfi
                const int m = __builtin_amdgcn_sbfe((int)hb, k, 1);
                q[k] = (av & ~m) - DT_HV * (c0 + k);
            }
            scan5_min(q, p);  // p[k] = min(q[0..k]), depth 2
            const int ex = from_left(wave_prefix_min(p[4]), 0x7FFFFFFF);  // lanes < l
            int T[5];
#pragma unroll
            for (int k = 0; k < 5; ++k) {
                // min(min(p, ex) + HV c, INIT + HV (c+1)) == min(p, ex, INIT + HV) + HV c
                T[k] = min(min(p[k], ex), DT_INIT + DT_HV) + DT_HV * (c0 + k);
                a.dtf[pix0 + k] = T[k];
            }
#pragma unroll
            for (int i = 0; i < 9; ++i) u2[i] = u1[i];
            u1[0] = from_left(T[3], DT_INIT);
            u1[1] = from_left(T[4], DT_INIT);
#pragma unroll
            for (int k = 0; k < 5; ++k) u1[k + 2] = T[k];
            u1[7] = from_right(T[0], DT_INIT);
            u1[8] = from_right(T[1], DT_INIT);
        };
        for (int r = r0 & ~1; r < H; r += 2) {
            row(r);
            row(r + 1);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        // backward pass: lane l owns columns cb-k (cb = 319 - 5l, k = 0..4), i.e. scan
        // index j = 5l + k; d1 / d2 = rows r+1 / r+2 at scan positions j-2 .. j+6
        const int cb = W - 1 - 5 * l;
        int d1[9], d2[9];
#pragma unroll
        for (int i = 0; i < 9; ++i) d1[i] = d2[i] = DT_INIT;
        float mx = 0.f;
        const float sc = 1.f / 65536;
        // forward values three rows ahead: row r's values are loaded while row r+3 is
        // scanned, into the register slot row r+3 just consumed (three slots, the loop
        // unrolled by three, so no register copy makes a row wait for newer loads);
        // unconditional loads of a clamped row
        int f0[5], f1[5], f2[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            f0[k] = a.dtf[(H - 1) * W + cb - k];
            f1[k] = a.dtf[(H - 2) * W + cb - k];
            f2[k] = a.dtf[(H - 3) * W + cb - k];
        }
        auto step = [&](int r, int (&fs)[5]) {
            int fw[5];
#pragma unroll
            for (int k = 0; k < 5; ++k) fw[k] = (r >= r0) ? fs[k] : DT_INIT;  // rows above r0: not scanned
            const int rn = r >= 3 ? r - 3 : 0;
#pragma unroll
            for (int k = 0; k < 5; ++k) fs[k] = a.dtf[rn * W + cb - k];
            int q[5], p[5];
#pragma unroll
            for (int k = 0; k < 5; ++k) {
                const int i = k + 2;
                const int mL = min(min(d2[i - 1], d2[i + 1]), min(d1[i - 2], d1[i + 2]));
                const int mD = min(d1[i - 1], d1[i + 1]);
                const int bv = min(min(fw[k], mL + DT_LONG), min(mD + DT_DIAG, d1[i] + DT_HV));
                q[k] = bv - DT_HV * (5 * l + k);
            }
            scan5_min(q, p);
            const int ex = from_left(wave_prefix_min(p[4]), 0x7FFFFFFF);
            int T[5];
#pragma unroll
            for (int k = 0; k < 5; ++k) {
                const int j = 5 * l + k;
                T[k] = min(min(p[k], ex), DT_INIT + DT_HV) + DT_HV * j;
                const float v = (float)T[k] * sc;
                a.dt[r * W + cb - k] = v;
                mx = v > mx ? v : mx;
            }
#pragma unroll
            for (int i = 0; i < 9; ++i) d2[i] = d1[i];
            d1[0] = from_left(T[3], DT_INIT);
            d1[1] = from_left(T[4], DT_INIT);
#pragma unroll
            for (int k = 0; k < 5; ++k) d1[k + 2] = T[k];
            d1[7] = from_right(T[0], DT_INIT);
            d1[8] = from_right(T[1], DT_INIT);
        };
        static_assert(H % 3 == 0, "backward rows in threes");
        for (int r = H - 1; r >= 2; r -= 3) {
            step(r, f0);
            step(r - 1, f1);
            step(r - 2, f2);
        }
        for (int off = 32; off > 0; off >>= 1) {
            const float o = __shfl_xor(mx, off);
            mx = o > mx ? o : mx;
        }
        if (l == 0) *wmaxp = mx;
    }
    __syncthreads();
    if (t == 0) a.info->dtmax = *wmaxp;
}

// The frame descriptor every tracking kernel reads.
__device__ __forceinline__ void prep_write_descriptor(const PrepArgs &a) {
    const PrepInfo *pi = a.info;
    DevObs od;
    od.cx = a.cx;
    od.cy = a.cy;
    od.cz = a.cz;
    od.depth = a.depth_cm;
    od.dt = a.dt;
    od.n = pi->n;
    od.lambda = (double)HPE_NS / (double)pi->n;  // costfunc.cpp:372
    od.scale = pi->scale;
    od.dtmax = pi->dtmax;
    const double Kv[9] = {a.focal, 0.0, 320 / 2., 0.0, a.focal, 240 / 2., 0.0, 0.0, 1.0};
    for (int k = 0; k < 9; ++k) od.K[k] = Kv[k];
    *a.obs_out = od;
}

// One preparing workgroup (index g in [0, PREP_WG)); the last to finish writes the
// descriptor.
__device__ __forceinline__ void prep_workgroup(const PrepArgs &a0, int g, unsigned char *lds) {
    int *flag = (int *)(lds + PREP_CH * 8 + 8);
    PrepArgs a = a0;
    if (a0.raw_row) a.raw = a0.raw + (size_t)(*a0.raw_row + 1) * a0.raw_stride;
    if (g < PREP_BANDS) {
        prep_band(a, g, lds);
        if (!prep_arrive_last(a.ctr, PREP_BANDS, flag)) return;
        prep_merge(a, lds);
    } else {
        prep_dt(a, lds);
    }
    if (prep_arrive_last(a.ctr + 1, 2, flag) && threadIdx.x == 0) {
        prep_write_descriptor(a);
        a.ctr[2] = 0u;  // every band is past its wait: ready for the next frame
    }
}

__global__ __launch_bounds__(PREP_NT) void k_prepare(PrepArgs a) {
    __shared__ __align__(16) unsigned char lds[prep_lds_bytes()];
    prep_workgroup(a, blockIdx.x, lds);
}
