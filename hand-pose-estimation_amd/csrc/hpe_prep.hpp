// hpe_prep.hpp -- observedmodel preprocessing on the GPU, one
// workgroup per frame, so a frame is prepared on a side stream while the previous one is
// tracked:
//   depth mm -> cm                                   (observedmodel.cpp:296-308)
//   point cloud of the non-zero pixels, row-major    (observedmodel.cpp:110-169)
//   cm-per-pixel scale = mean of 2 / |d(u,v)|        (observedmodel.cpp:171-202)
//   down-sample to rows k * floor(N / 250)           (observedmodel.cpp:204-217)
//   5x5 chamfer distance transform of the background (observedmodel.cpp:313-358,
//     OpenCV distanceTransform(CV_DIST_L2, 5): 16.16 fixed point, weights 1 / 1.4 / 2.1969)
// The DT is integer min-plus arithmetic, so the row scans (T_c = min(a_c, T_{c-1} + 1))
// computed as block prefix minima give exactly the raster-scan values.  The cloud and
// depth are the host's arithmetic (-ffp-contract=off) and the scale mean is summed in
// Armadillo's order (two alternating sequential accumulators): bit-identical results.
#pragma once
#include "hpe_device.hpp"

#define PREP_NT 1024
#define PREP_CH 4096  // scale terms staged in LDS per pass
#define DT_HV 65536
#define DT_DIAG 91750
#define DT_LONG 143976
#define DT_INIT (0x7FFFFFFF >> 2)

struct PrepInfo {
    int n_full, n;
    double scale, dtmax;
};

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

// One chamfer row step over 320 columns held by threads 0..319 (5 waves): returns
// T_j = min(a_j, T_{j-1} + HV) with T_{-1} = INIT, via a prefix minimum of a_j - HV*j.
__device__ __forceinline__ int dt_row_scan(int a, int j, int *wmin) {
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    int v = wave_prefix_min(a - DT_HV * j);
    if (l == 63 && w < 5) wmin[w] = v;
    __syncthreads();
    int pre = 0x7FFFFFFF;
    for (int k = 0; k < w && k < 5; ++k) pre = min(pre, wmin[k]);
    v = min(v, pre);
    __syncthreads();
    return min(v + DT_HV * j, DT_INIT + DT_HV * (j + 1));
}

__global__ __launch_bounds__(PREP_NT) void k_preprocess(
    const float *__restrict__ raw, int to_cm, int downsample, double focal,
    double *__restrict__ depth_cm, float *__restrict__ dt, double *__restrict__ cx,
    double *__restrict__ cy, double *__restrict__ cz, double *__restrict__ tmp,
    double *__restrict__ ctb,
    int *__restrict__ dtf, DevObs *__restrict__ obs_out, PrepInfo *__restrict__ info) {
    constexpr int W = HPE_IMG_W, H = HPE_IMG_H, NPIX = W * H, NWV = PREP_NT / 64;
    __shared__ int wcnt[NWV], hcnt[NWV];
    __shared__ double wsum[NWV][2];
    __shared__ double chunk[PREP_CH];
    __shared__ int ring[3][W + 4];
    __shared__ int wmin[8];
    __shared__ float wmax[NWV];
    const int t = threadIdx.x, w = t >> 6, l = t & 63;
    const double c0 = 320 / 2., c1 = 240 / 2.;
    const double Kv[9] = {focal, 0.0, c0, 0.0, focal, c1, 0.0, 0.0, 1.0};
    // ---- A: depth, cloud compaction (row-major), scale contributions; 1024 pixels a pass
    int base = 0, ncm = 0;
    double acc0 = 0, acc1 = 0;  // threads 0 / 1: even / odd terms of the scale mean
    for (int p0 = 0; p0 < NPIX; p0 += PREP_NT) {
        const int pix = p0 + t;
        const double Z = to_cm ? (double)raw[pix] / 10. : (double)raw[pix];
        depth_cm[pix] = Z;
        const bool nz = Z != 0;
        const unsigned long long b = __ballot(nz);
        const int wpre = __popcll(b & ((1ull << l) - 1));
        double contrib = 0;
        bool has = false;
        double X = 0, Y = 0;
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
            wcnt[w] = __popcll(b);
            hcnt[w] = __popcll(bh);
        }
        __syncthreads();
        int off = base, hoff = ncm, tot = 0, htot = 0;
        for (int k = 0; k < NWV; ++k) {
            off += (k < w) ? wcnt[k] : 0;
            hoff += (k < w) ? hcnt[k] : 0;
            tot += wcnt[k];
            htot += hcnt[k];
        }
        if (nz) {
            const int idx = off + wpre;
            tmp[3 * idx + 0] = X;
            tmp[3 * idx + 1] = Y * -1;
            tmp[3 * idx + 2] = Z * -1;
        }
        if (has) ctb[hoff + hpre] = contrib;  // the mean's terms, in pixel order
        base += tot;
        ncm += htot;
        __syncthreads();
    }
    const int n_full = base;
    // arma::mean = accumulate / n: two accumulators take the terms alternately, each a
    // sequential sum (arrayops::accumulate); threads 0 and 1 replay them from LDS chunks
    for (int b0 = 0; b0 < ncm; b0 += PREP_CH) {
        const int m = min(PREP_CH, ncm - b0);
        for (int k = t; k < m; k += PREP_NT) chunk[k] = ctb[b0 + k];
        __syncthreads();
        if (t < 2) {
            double a = (t == 0) ? acc0 : acc1;
            for (int k = (b0 + t) & 1 ? 1 : 0; k < m; k += 2) a += chunk[k];
            if (t == 0) acc0 = a;
            else acc1 = a;
        }
        __syncthreads();
    }
    if (t == 1) wsum[0][1] = acc1;
    __syncthreads();
    if (t == 0) acc1 = wsum[0][1];
    // ---- B: down-sample (observedmodel.cpp:204-217) into the slot's SoA cloud
    const int n = downsample ? 250 : n_full;
    const int f = n_full / 250;
    for (int k = t; k < n; k += PREP_NT) {
        double x = 0, y = 0, z = 0;
        const int src = downsample ? k * f : k;
        if (!downsample || n_full > 0) {
            x = tmp[3 * src + 0];
            y = tmp[3 * src + 1];
            z = tmp[3 * src + 2];
        }
        cx[k] = x;
        cy[k] = y;
        cz[k] = z;
    }
    // ---- C: distance transform, rows in sequence, columns in parallel (threads < 320)
    const bool col = t < W;
    for (int k = t; k < 3 * (W + 4); k += PREP_NT) (&ring[0][0])[k] = DT_INIT;
    __syncthreads();
    // forward pass (mask rows r-2, r-1 and the left neighbour)
    double dnext = col ? depth_cm[t] : 0.0;
    for (int r = 0; r < H; ++r) {
        const double dcur = dnext;
        if (col && r + 1 < H) dnext = depth_cm[(r + 1) * W + t];
        int a = 0;
        if (col && dcur == 0) {
            const int *u2 = ring[(r + 1) % 3], *u1 = ring[(r + 2) % 3];  // rows r-2, r-1
            const int j = t + 2;
            a = min(min(min(u2[j - 1] + DT_LONG, u2[j + 1] + DT_LONG),
                        min(u1[j - 2] + DT_LONG, u1[j - 1] + DT_DIAG)),
                    min(min(u1[j] + DT_HV, u1[j + 1] + DT_DIAG), u1[j + 2] + DT_LONG));
        }
        const int T = dt_row_scan(col ? a : 0x3FFFFFFF, t, wmin);
        if (col) {
            ring[r % 3][t + 2] = T;
            dtf[r * W + t] = T;
        }
        __syncthreads();
    }
    // backward pass (rows r+1, r+2 and the right neighbour): column c = W-1-t
    for (int k = t; k < 3 * (W + 4); k += PREP_NT) (&ring[0][0])[k] = DT_INIT;
    __syncthreads();
    const int c = W - 1 - t;
    float mx = 0.f;
    int fnext = col ? dtf[(H - 1) * W + c] : 0;
    const float sc = 1.f / 65536;
    for (int r = H - 1; r >= 0; --r) {
        const int fcur = fnext;
        if (col && r > 0) fnext = dtf[(r - 1) * W + c];
        int b = 0;
        if (col) {
            const int *d1 = ring[(r + 1) % 3], *d2 = ring[(r + 2) % 3];  // rows r+1, r+2
            const int j = c + 2;
            b = min(min(min(fcur, d2[j + 1] + DT_LONG), min(d2[j - 1] + DT_LONG, d1[j + 2] + DT_LONG)),
                    min(min(d1[j + 1] + DT_DIAG, d1[j] + DT_HV),
                        min(d1[j - 1] + DT_DIAG, d1[j - 2] + DT_LONG)));
        }
        const int T = dt_row_scan(col ? b : 0x3FFFFFFF, t, wmin);
        if (col) {
            ring[r % 3][c + 2] = T;
            const float v = (float)T * sc;
            dt[r * W + c] = v;
            mx = v > mx ? v : mx;
        }
        __syncthreads();
    }
    // ---- D: max(DT), the frame descriptor
    for (int off = 32; off > 0; off >>= 1) {
        const float o = __shfl_xor(mx, off);
        mx = o > mx ? o : mx;
    }
    if (l == 0) wmax[w] = mx;
    __syncthreads();
    if (t == 0) {
        float m = wmax[0];
        for (int k = 1; k < NWV; ++k) m = wmax[k] > m ? wmax[k] : m;
        const double scale = ncm ? (acc0 + acc1) / ncm : __builtin_nan("");
        DevObs od;
        od.cx = cx;
        od.cy = cy;
        od.cz = cz;
        od.depth = depth_cm;
        od.dt = dt;
        od.n = n;
        od.lambda = (double)HPE_NS / (double)n;  // costfunc.cpp:372
        od.scale = scale;
        od.dtmax = m;
        for (int k = 0; k < 9; ++k) od.K[k] = Kv[k];
        *obs_out = od;
        info->n_full = n_full;
        info->n = n;
        info->scale = scale;
        info->dtmax = m;
    }
}
