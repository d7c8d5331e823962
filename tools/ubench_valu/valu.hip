// Diagnostic: VALU throughput per wave-instruction on gfx950 for the instruction mixes of
// the wave form (fp32 scalar / packed, fp64, integer multiply, bit ops), at W waves per SIMD.
// Each lane runs 8 independent chains of REP instructions; cycles per wave-instruction per
// SIMD = elapsed shader cycles * 4 SIMDs / (waves * instructions).
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP 256
#define OP8(S) S(0) S(1) S(2) S(3) S(4) S(5) S(6) S(7)

template <int K>
__global__ __launch_bounds__(256) void k_valu(float *out, int n, unsigned long long *cyc) {
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    float a[8], b[8];
    double d[8];
    unsigned u[8];
    for (int i = 0; i < 8; ++i) {
        a[i] = threadIdx.x * 0.001f + i;
        b[i] = a[i] * 0.5f;
        d[i] = a[i];
        u[i] = threadIdx.x * 7 + i;
    }
    for (int r = 0; r < n; ++r) {
#pragma unroll
        for (int k = 0; k < REP / 8; ++k) {
            if (K == 0) {  // v_fma_f32
#define S(i) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a[i]) : "v"(b[i]), "v"(b[i]));
                OP8(S)
#undef S
            } else if (K == 1) {  // v_pk_fma_f32
#define S(i) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(d[i]) : "v"(d[i]), "v"(d[i]));
                OP8(S)
#undef S
            } else if (K == 2) {  // v_pk_add_f32
#define S(i) asm volatile("v_pk_add_f32 %0, %1, %0" : "+v"(d[i]) : "v"(d[i]));
                OP8(S)
#undef S
            } else if (K == 3) {  // v_fma_f64
#define S(i) asm volatile("v_fma_f64 %0, %1, %1, %0" : "+v"(d[i]) : "v"(d[i]));
                OP8(S)
#undef S
            } else if (K == 4) {  // v_add_f64
#define S(i) asm volatile("v_add_f64 %0, %1, %0" : "+v"(d[i]) : "v"(d[i]));
                OP8(S)
#undef S
            } else if (K == 5) {  // v_mul_lo_u32
#define S(i) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(u[i]) : "v"(u[i]));
                OP8(S)
#undef S
            } else if (K == 6) {  // v_mul_hi_u32
#define S(i) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(u[i]) : "v"(u[i]));
                OP8(S)
#undef S
            } else if (K == 7) {  // v_mad_u64_u32
#define S(i) asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %1, %0" : "+v"(d[i]) : "v"(u[i]) : "s0", "s1");
                OP8(S)
#undef S
            } else if (K == 8) {  // v_and_or_b32
#define S(i) asm volatile("v_and_or_b32 %0, %0, %1, %1" : "+v"(u[i]) : "v"(u[i]));
                OP8(S)
#undef S
            } else if (K == 9) {  // v_min3_u32
#define S(i) asm volatile("v_min3_u32 %0, %0, %1, %1" : "+v"(u[i]) : "v"(u[i]));
                OP8(S)
#undef S
            } else if (K == 10) {  // v_xor_b32
#define S(i) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(u[i]) : "v"(u[i]));
                OP8(S)
#undef S
            } else if (K == 11) {  // v_mul_f64
#define S(i) asm volatile("v_mul_f64 %0, %1, %0" : "+v"(d[i]) : "v"(d[i]));
                OP8(S)
#undef S
            } else if (K == 12) {  // v_cvt_f32_f64
#define S(i) asm volatile("v_cvt_f32_f64 %0, %1" : "=v"(a[i]) : "v"(d[i]));
                OP8(S)
#undef S
            } else if (K == 13) {  // v_rsq_f64
#define S(i) asm volatile("v_rsq_f64 %0, %0" : "+v"(d[i]));
                OP8(S)
#undef S
            } else if (K == 14) {  // v_med3_u32
#define S(i) asm volatile("v_med3_u32 %0, %0, %1, %1" : "+v"(u[i]) : "v"(u[i]));
                OP8(S)
#undef S
            } else if (K == 15) {  // v_pk_mul_f32
#define S(i) asm volatile("v_pk_mul_f32 %0, %1, %0" : "+v"(d[i]) : "v"(d[i]));
                OP8(S)
#undef S
            } else if (K == 16) {  // v_min3_f32
#define S(i) asm volatile("v_min3_f32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(b[i]));
                OP8(S)
#undef S
            } else if (K == 17) {  // v_med3_f32
#define S(i) asm volatile("v_med3_f32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(b[i]));
                OP8(S)
#undef S
            } else if (K == 18) {  // v_min_f32 (VOP2)
#define S(i) asm volatile("v_min_f32 %0, %0, %1" : "+v"(a[i]) : "v"(b[i]));
                OP8(S)
#undef S
            } else if (K == 19) {  // v_min_u32 (VOP2)
#define S(i) asm volatile("v_min_u32 %0, %0, %1" : "+v"(u[i]) : "v"(u[i]));
                OP8(S)
#undef S
            } else if (K == 20) {  // v_mov_b32_sdwa byte 0
#define S(i) asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_0 dst_unused:UNUSED_PRESERVE src0_sel:DWORD" : "+v"(u[i]) : "v"(u[(i + 1) & 7]));
                OP8(S)
#undef S
            } else if (K == 21) {  // v_sub_u32 (VOP2)
#define S(i) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(u[i]) : "v"(u[i]));
                OP8(S)
#undef S
            } else if (K == 22) {  // v_cndmask_b32 (VOP2, vcc)
#define S(i) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(u[i]) : "v"(u[i]));
                OP8(S)
#undef S
            } else if (K == 23) {  // v_add_f32 (VOP2)
#define S(i) asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[i]) : "v"(b[i]));
                OP8(S)
#undef S
            } else if (K == 24) {  // v_mul_f32 (VOP2)
#define S(i) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a[i]) : "v"(b[i]));
                OP8(S)
#undef S
            } else if (K == 25) {  // v_and_b32 (VOP2)
#define S(i) asm volatile("v_and_b32 %0, %0, %1" : "+v"(u[i]) : "v"(u[i]));
                OP8(S)
#undef S
            } else if (K == 26) {  // v_max_f64
#define S(i) asm volatile("v_max_f64 %0, %1, %0" : "+v"(d[i]) : "v"(d[i]));
                OP8(S)
#undef S
            }
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0;
    for (int i = 0; i < 8; ++i) s += a[i] + (float)d[i] + (float)u[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int K>
static void run(const char *name, float *out, unsigned long long *cyc, int wps) {
    const int nblk = 256 * wps, n = 64;
    hipLaunchKernelGGL(k_valu<K>, dim3(nblk), dim3(256), 0, 0, out, n, cyc);
    hipDeviceSynchronize();
    unsigned long long h[2048];
    hipMemcpy(h, cyc, nblk * 8, hipMemcpyDeviceToHost);
    double mx = 0, mean = 0;
    for (int b = 0; b < nblk; ++b) { mx = h[b] > mx ? h[b] : mx; mean += h[b]; }
    mean /= nblk;
    // per SIMD: wps waves, each n*REP instructions
    printf("%-16s waves/SIMD %d: %.2f cyc per wave-instruction per SIMD (mean span), %.2f (max)\n",
           name, wps, mean / (wps * (double)n * REP), mx / (wps * (double)n * REP));
}

int main() {
    float *out;
    unsigned long long *cyc;
    (void)hipMalloc(&out, 2048 * 256 * 4);
    (void)hipMalloc(&cyc, 2048 * 8);
    for (int wps : {4, 1}) {
        run<0>("v_fma_f32", out, cyc, wps);
        run<23>("v_add_f32", out, cyc, wps);
        run<24>("v_mul_f32", out, cyc, wps);
        run<1>("v_pk_fma_f32", out, cyc, wps);
        run<16>("v_min3_f32", out, cyc, wps);
        run<17>("v_med3_f32", out, cyc, wps);
        run<18>("v_min_f32", out, cyc, wps);
        run<19>("v_min_u32", out, cyc, wps);
        run<9>("v_min3_u32", out, cyc, wps);
        run<20>("v_mov_b32_sdwa", out, cyc, wps);
        run<21>("v_sub_u32", out, cyc, wps);
        run<22>("v_cndmask_b32", out, cyc, wps);
        run<25>("v_and_b32", out, cyc, wps);
        run<8>("v_and_or_b32", out, cyc, wps);
        run<3>("v_fma_f64", out, cyc, wps);
        run<26>("v_max_f64", out, cyc, wps);
        if (wps == 1) break;
    }
    return 0;
}
