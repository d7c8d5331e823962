// tools/mfma_check.hip -- diagnostic: the MFMA-filtered correspondence search
// (hpe_device.hpp mfma_match, HPE_MFMA_SEARCH) against bf_search on random hand-sized sphere
// sets and points: on-surface points, points on the bisector of two spheres (fp32 ties),
// points far from the hand, NaN points.  Every match must equal bf_search's; prints the
// mismatch count and how often the filter sent a wave to bf_search.  Not part of the product.
// Build: hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -DHPE_MFMA_SEARCH=1 \
//        tools/mfma_check.hip -o tools/mfma_check
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../hand-pose-estimation_amd/csrc/hpe_device.hpp"

#define SETS 512     // sphere sets (one workgroup each)
#define PTS 1024     // points per set

__global__ __launch_bounds__(64) void k_check(const float *__restrict__ sph, const float *__restrict__ pts,
                                              const DevHand *__restrict__ H, unsigned *__restrict__ out) {
    __shared__ FkSm f;
    const int b = blockIdx.x, l = threadIdx.x, r = l & 31;
    if (l < HPE_NS) {
        for (int k = 0; k < 3; ++k) {
            const float v = sph[(b * HPE_NS + l) * 3 + k];
            f.Sp[k][l] = v;
            f.S[l][k] = (double)v;
        }
    }
    __syncthreads();
    const MfmaSph ms = mfma_sph(f);
    unsigned bad = 0, fall = 0;
    for (int tile = 0; tile < PTS / 32; ++tile) {
        const float *p = pts + ((size_t)b * PTS + 32 * tile + r) * 3;
        const int idx = mfma_match(f, ms, p[0], p[1], p[2]);
        const int h2 = l & 1;
        const float *q = pts + ((size_t)b * PTS + 32 * tile + (l >> 1)) * 3;
        const BfOut rb = bf_search(f, H, f.Sp[0] + 24 * h2, f.Sp[1] + 24 * h2, f.Sp[2] + 24 * h2,
                                   q[0], q[1], q[2], h2);
        const int ref = __shfl(rb.idx, 2 * r);
        if (__ballot(idx < 0)) ++fall;
        if (idx >= 0 && idx != ref) ++bad;
    }
    atomicAdd(&out[0], bad);
    if (l == 0) atomicAdd(&out[1], fall);
}


// fp16 subnormal A inputs: does the MFMA flush them?  out = sum of 2^-20 * 1 over k
__global__ void k_denorm(float *out) {
    const int l = threadIdx.x;
    const _Float16 d = (_Float16)0x1p-20f, z = (_Float16)0.f, o = (_Float16)1.f;
    const hpe_h8 a = (l >> 5) == 0 ? hpe_h8{d, z, z, z, z, z, z, z} : hpe_h8{z, z, z, z, z, z, z, z};
    const hpe_h8 b = (l >> 5) == 0 ? hpe_h8{o, z, z, z, z, z, z, z} : hpe_h8{z, z, z, z, z, z, z, z};
    const hpe_f16x zero = {};
    const hpe_f16x e = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, zero, 0, 0, 0);
    out[l] = e[0];
}

// cycles per 32-point tile: mode 0 = mfma_match alone (no fallback taken), 1 = bf_search alone;
// 8 waves per workgroup (two per SIMD), one workgroup per CU, 32 tiles per wave
__global__ __launch_bounds__(512) void k_time(const float *__restrict__ sph, const float *__restrict__ pts,
                                              const DevHand *__restrict__ H, int mode,
                                              unsigned long long *__restrict__ cyc, int *__restrict__ sink) {
    __shared__ FkSm f;
    const int b = blockIdx.x % SETS, t = threadIdx.x, l = t & 63, w = t >> 6, r = l & 31;
    if (t < HPE_NS) {
        for (int k = 0; k < 3; ++k) {
            const float v = sph[(b * HPE_NS + t) * 3 + k];
            f.Sp[k][t] = v;
            f.S[t][k] = (double)v;
        }
    }
    __syncthreads();
    int acc = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (mode == 0) {
        const MfmaSph ms = mfma_sph(f);
        for (int tile = w; tile < PTS / 32; tile += 8) {
            const float *p = pts + ((size_t)b * PTS + 32 * tile + r) * 3;
            acc += mfma_match(f, ms, p[0], p[1], p[2]);
        }
    } else {
        for (int tile = w; tile < PTS / 32; tile += 8) {
            const int h2 = l & 1;
            const float *q = pts + ((size_t)b * PTS + 32 * tile + (l >> 1)) * 3;
            acc += bf_search(f, H, f.Sp[0] + 24 * h2, f.Sp[1] + 24 * h2, f.Sp[2] + 24 * h2, q[0], q[1], q[2], h2).idx;
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    sink[blockIdx.x * 512 + t] = acc;
    if (l == 0) atomicAdd(cyc, t1 - t0);
}

int main() {
    std::mt19937 g(7);
    std::uniform_real_distribution<float> U(-1.f, 1.f);
    std::vector<float> sph((size_t)SETS * HPE_NS * 3), pts((size_t)SETS * PTS * 3);
    for (int b = 0; b < SETS; ++b) {
        const float cx = 10 * U(g), cy = 10 * U(g), cz = -45 + 10 * U(g);
        const float span = (b % 4 == 3) ? 60.f : 12.f;  // every fourth set: a stretched hand
        for (int s = 0; s < HPE_NS; ++s) {
            sph[(b * HPE_NS + s) * 3 + 0] = cx + span * U(g);
            sph[(b * HPE_NS + s) * 3 + 1] = cy + span * U(g);
            sph[(b * HPE_NS + s) * 3 + 2] = cz + 0.5f * span * U(g);
        }
        for (int i = 0; i < PTS; ++i) {
            float *p = &pts[((size_t)b * PTS + i) * 3];
            const int a = g() % HPE_NS, c = g() % HPE_NS;
            const float *A = &sph[(b * HPE_NS + a) * 3], *B = &sph[(b * HPE_NS + c) * 3];
            const int kind = i % 8;
            if (kind < 4) {  // near a sphere surface
                for (int k = 0; k < 3; ++k) p[k] = A[k] + 1.2f * U(g);
            } else if (kind < 7) {  // on the bisector of two spheres (ties in fp32)
                float d[3], v[3], w[3];
                for (int k = 0; k < 3; ++k) {
                    d[k] = B[k] - A[k];
                    v[k] = U(g);
                }
                w[0] = d[1] * v[2] - d[2] * v[1];
                w[1] = d[2] * v[0] - d[0] * v[2];
                w[2] = d[0] * v[1] - d[1] * v[0];
                const float t = (kind == 6) ? 1e-6f * U(g) : 0.f;
                for (int k = 0; k < 3; ++k) p[k] = 0.5f * (A[k] + B[k]) + 0.3f * w[k] + t * d[k];
            } else if (i % 64 == 7) {  // far away / non-finite
                p[0] = (i % 128 == 7) ? NAN : 400.f;
                p[1] = 0.f;
                p[2] = -40.f;
            } else {
                for (int k = 0; k < 3; ++k) p[k] = A[k] + 5.f * U(g);
            }
        }
    }
    float *ds, *dp;
    unsigned *dout;
    DevHand *dh;
    if (hipMalloc(&ds, sph.size() * 4) != hipSuccess || hipMalloc(&dp, pts.size() * 4) != hipSuccess ||
        hipMalloc(&dout, 8) != hipSuccess || hipMalloc(&dh, sizeof(DevHand)) != hipSuccess)
        return 1;
    (void)hipMemset(dh, 0, sizeof(DevHand));
    (void)hipMemcpy(ds, sph.data(), sph.size() * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(dp, pts.data(), pts.size() * 4, hipMemcpyHostToDevice);
    (void)hipMemset(dout, 0, 8);
    hipLaunchKernelGGL(k_check, dim3(SETS), dim3(64), 0, 0, ds, dp, (const DevHand *)dh, dout);
    unsigned out[2];
    (void)hipMemcpy(out, dout, 8, hipMemcpyDeviceToHost);
    printf("points %d, mismatches %u, tiles sent to bf_search %u of %d\n", SETS * PTS, out[0], out[1],
           SETS * PTS / 32);
    float *dd;
    (void)hipMalloc(&dd, 64 * 4);
    hipLaunchKernelGGL(k_denorm, dim3(1), dim3(64), 0, 0, dd);
    float dn[64];
    (void)hipMemcpy(dn, dd, 64 * 4, hipMemcpyDeviceToHost);
    printf("fp16 subnormal 2^-20 through the MFMA: %g (flushed: 0)\n", dn[0]);
    // timing on points without ties (surface points only)
    for (int b = 0; b < SETS; ++b)
        for (int i = 0; i < PTS; ++i) {
            float *p = &pts[((size_t)b * PTS + i) * 3];
            const float *A = &sph[(b * HPE_NS + (i * 7) % HPE_NS) * 3];
            for (int k = 0; k < 3; ++k) p[k] = A[k] + 1.2f * U(g);
        }
    (void)hipMemcpy(dp, pts.data(), pts.size() * 4, hipMemcpyHostToDevice);
    unsigned long long *dc;
    int *sink;
    (void)hipMalloc(&dc, 8);
    (void)hipMalloc(&sink, 256 * 512 * 4);
    for (int mode = 0; mode < 2; ++mode)
        for (int rep = 0; rep < 2; ++rep) {
            (void)hipMemset(dc, 0, 8);
            hipLaunchKernelGGL(k_time, dim3(256), dim3(512), 0, 0, ds, dp, (const DevHand *)dh, mode, dc, sink);
            unsigned long long c;
            (void)hipMemcpy(&c, dc, 8, hipMemcpyDeviceToHost);
            printf("%s: %.0f cycles per tile per wave (8 waves / CU)\n", mode ? "bf_search" : "mfma_match",
                   (double)c / (256.0 * 8 * (PTS / 32 / 8)));
        }
    return out[0] != 0;
}
