// tools/ubench.hip -- diagnostic microbenchmarks of the device building blocks (not part
// of the product).  One workgroup, one wave measuring, s_memtime deltas averaged over
// repetitions: latency of each piece in isolation, without other waves contending.
// Build: hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 tools/ubench.hip
#include <cstdio>
#include <cstring>
#include <vector>

#include "../hand-pose-estimation_amd/csrc/hpe_device.hpp"
#include "../hand-pose-estimation_amd/csrc/hpe_host.hpp"

#define REPS 64

__device__ __forceinline__ unsigned long long now() {
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

// out[k] = average cycles of test k
__global__ __launch_bounds__(256) void k_ubench(const DevHand *Hg, DevObs o, int32_t *match_g, double *sink,
                         unsigned long long *out) {
    __shared__ FkSm f;
    __shared__ DevHand hs;
    __shared__ double cloud[3 * 256];
    __shared__ int32_t mt[256];
    const int t = threadIdx.x;
    for (int q = t; q < (int)(sizeof(DevHand) / 8); q += blockDim.x)
        ((double *)&hs)[q] = ((const double *)Hg)[q];
    for (int p = t; p < o.n && p < 256; p += blockDim.x) {
        cloud[p] = o.cx[p];
        cloud[256 + p] = o.cy[p];
        cloud[512 + p] = o.cz[p];
        mt[p] = p % 48;
    }
    if (t < 26) f.th[t] = 5.0 + t;
    __syncthreads();
    if (t >= 64) return;
    const CloudView cv{cloud, cloud + 256, cloud + 512, o.n < 256 ? o.n : 256};
    double acc = 0;
    unsigned long long t0, t1;
    // 0: fk_wave with H in LDS
    t0 = now();
    for (int r = 0; r < REPS; ++r) {
        if (t < 26) f.th[t] += 1e-3;
        wave_sync();
        fk_wave(f, &hs);
    }
    t1 = now();
    if (t == 0) out[0] = (t1 - t0) / REPS;
    // 1: fk_wave with H in global memory
    t0 = now();
    for (int r = 0; r < REPS; ++r) {
        if (t < 26) f.th[t] += 1e-3;
        wave_sync();
        fk_wave(f, Hg);
    }
    t1 = now();
    if (t == 0) out[1] = (t1 - t0) / REPS;
    // 2: eval_wave_frozen, LDS cloud/match, H in LDS
    t0 = now();
    for (int r = 0; r < REPS; ++r) {
        if (t < 26) f.th[t] += 1e-3;
        wave_sync();
        acc += eval_wave_frozen(f, o, cv, &hs, mt);
    }
    t1 = now();
    if (t == 0) out[2] = (t1 - t0) / REPS;
    // 3: wave_sum3
    double a = t, b = 2 * t, c = 3 * t;
    t0 = now();
    for (int r = 0; r < REPS; ++r) {
        wave_sum3(a, b, c);
        a += 1;
    }
    t1 = now();
    acc += a + b + c;
    if (t == 0) out[3] = (t1 - t0) / REPS;
    // 4: depth_term (global gathers)
    t0 = now();
    for (int r = 0; r < REPS; ++r) {
        double d = (t < 48) ? depth_term(f, t, o, &hs) : 0.0;
        acc += d;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (t < 26) f.th[t] += d * 1e-30;
    }
    t1 = now();
    if (t == 0) out[4] = (t1 - t0) / REPS;
    // 5: align_frozen only (LDS)
    t0 = now();
    for (int r = 0; r < REPS; ++r) acc += align_frozen(f, cv, &hs, mt, t, 64);
    t1 = now();
    if (t == 0) out[5] = (t1 - t0) / REPS;
    // 6: collision (3 pairs per lane)
    t0 = now();
    for (int r = 0; r < REPS; ++r)
        acc += collide_term(f, t, &hs) + collide_term(f, t + 64, &hs) +
               ((t < 16) ? collide_term(f, t + 128, &hs) : 0.0);
    t1 = now();
    if (t == 0) out[6] = (t1 - t0) / REPS;
    // 7: one dependent global load chain (L2-resident)
    const double *pp = o.cx;
    t0 = now();
    int idx = 0;
    for (int r = 0; r < REPS; ++r) {
        double v = pp[idx];
        idx = (int)(v * 0.0) + (r & 7);
        acc += v;
    }
    t1 = now();
    if (t == 0) out[7] = (t1 - t0) / REPS;
    // 8: sincos fp64 alone (23 lanes)
    double ang = 0.1 * t;
    t0 = now();
    for (int r = 0; r < REPS; ++r) {
        double s, cc;
        sincos(ang, &s, &cc);
        ang = s + cc * 1e-3;
    }
    t1 = now();
    acc += ang;
    if (t == 0) out[8] = (t1 - t0) / REPS;
    // 9: fp64 sqrt chain
    double q = 2.0 + t;
    t0 = now();
    for (int r = 0; r < REPS; ++r) q = sqrt(q) + 1.0;
    t1 = now();
    acc += q;
    if (t == 0) out[9] = (t1 - t0) / REPS;
    // 10: fp64 dependent add chain (16 per rep)
    double z = t;
    t0 = now();
    for (int r = 0; r < REPS; ++r) {
#pragma unroll
        for (int u = 0; u < 16; ++u) z = z * 1.0000001 + 1e-9;
    }
    t1 = now();
    acc += z;
    if (t == 0) out[10] = (t1 - t0) / REPS;
    // 15: fk_wave + depth_issue + depth_finish (the FK -> gather chain, nothing overlapped)
    t0 = now();
    for (int r = 0; r < REPS; ++r) {
        if (t < 26) f.th[t] += 1e-3;
        wave_sync();
        fk_wave(f, &hs);
        const DepthG dg = depth_issue(f, t, o, &hs);
        acc += depth_finish(dg, o, t < HPE_NS);
    }
    t1 = now();
    if (t == 0) out[15] = (t1 - t0) / REPS;
    // 16: fk_wave + align_frozen
    t0 = now();
    for (int r = 0; r < REPS; ++r) {
        if (t < 26) f.th[t] += 1e-3;
        wave_sync();
        fk_wave(f, &hs);
        acc += align_frozen(f, cv, &hs, mt, t, 64);
    }
    t1 = now();
    if (t == 0) out[16] = (t1 - t0) / REPS;
    // 17: fk_wave + depth_issue + align_frozen + depth_finish (no collision, no sum)
    t0 = now();
    for (int r = 0; r < REPS; ++r) {
        if (t < 26) f.th[t] += 1e-3;
        wave_sync();
        fk_wave(f, &hs);
        const DepthG dg = depth_issue(f, t, o, &hs);
        double al = align_frozen(f, cv, &hs, mt, t, 64);
        acc += al + depth_finish(dg, o, t < HPE_NS);
    }
    t1 = now();
    if (t == 0) out[17] = (t1 - t0) / REPS;
    // 18: fk_wave_t<FK_TRANSLATE> (no trig, no chain: joints from X + spheres)
    __shared__ FkX X;
    fk_wave_t<FK_STORE_X>(f, &hs, &X);
    t0 = now();
    for (int r = 0; r < REPS; ++r) {
        if (t < 26) f.th[t] += 1e-3;
        wave_sync();
        fk_wave_t<FK_TRANSLATE>(f, &hs, &X);
    }
    t1 = now();
    if (t == 0) out[18] = (t1 - t0) / REPS;
    // 19: fp64 a / 180.0 dependent chain
    double dv = 1.0 + t;
    t0 = now();
    for (int r = 0; r < REPS; ++r) dv = dv / 180.0 + 3.0;
    t1 = now();
    acc += dv;
    if (t == 0) out[19] = (t1 - t0) / REPS;
    // 20: the trig phase of fk_wave alone (th LDS read, deg2rad, sincos, LDS write, sync)
    t0 = now();
    for (int r = 0; r < REPS; ++r) {
        if (t < 23) {
            const double th = f.th[t < 3 ? t : 6 + (t - 3)];
            const double a = deg2rad(t == 0 ? th + 180 : th);
            double s, c;
            sincos(a, &s, &c);
            f.sn[t] = s;
            f.cs[t] = c;
        }
        wave_sync();
        if (t < 26) f.th[t] += f.sn[t % 23] * 1e-30;
        wave_sync();
    }
    t1 = now();
    if (t == 0) out[20] = (t1 - t0) / REPS;
    // 21: fk + depth + align + collision (batched loads), no wave sum
    t0 = now();
    for (int r = 0; r < REPS; ++r) {
        if (t < 26) f.th[t] += 1e-3;
        wave_sync();
        fk_wave(f, &hs);
        const DepthG dg = depth_issue(f, t, o, &hs);
        double al = align_frozen(f, cv, &hs, mt, t, 64);
        CollPair cp[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) cp[k] = collide_load(f, k < 2 ? t + 64 * k : ((t < 16) ? t + 128 : t), &hs);
        asm volatile("" ::"v"(cp[0].ax), "v"(cp[1].ax), "v"(cp[2].ax));
        double co = collide_value(cp[0]) + collide_value(cp[1]) + ((t < 16) ? collide_value(cp[2]) : 0.0);
        asm volatile("" ::"v"(co));
        acc += (al + depth_finish(dg, o, t < HPE_NS)) + co;
    }
    t1 = now();
    if (t == 0) out[21] = (t1 - t0) / REPS;
    // 22: eval_wave_frozen's sequence written out (21 + wave_sum3)
    t0 = now();
    for (int r = 0; r < REPS; ++r) {
        if (t < 26) f.th[t] += 1e-3;
        wave_sync();
        fk_wave(f, &hs);
        const DepthG dg = depth_issue(f, t, o, &hs);
        double al = align_frozen(f, cv, &hs, mt, t, 64);
        CollPair cp[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) cp[k] = collide_load(f, k < 2 ? t + 64 * k : ((t < 16) ? t + 128 : t), &hs);
        asm volatile("" ::"v"(cp[0].ax), "v"(cp[1].ax), "v"(cp[2].ax));
        double co = collide_value(cp[0]) + collide_value(cp[1]) + ((t < 16) ? collide_value(cp[2]) : 0.0);
        asm volatile("" ::"v"(co));
        double dep = depth_finish(dg, o, t < HPE_NS);
        wave_sum3(al, dep, co);
        acc += (al * o.lambda + dep) + co;
    }
    t1 = now();
    if (t == 0) out[22] = (t1 - t0) / REPS;
    // 23: eval_wave_frozen again (order effects)
    t0 = now();
    for (int r = 0; r < REPS; ++r) {
        if (t < 26) f.th[t] += 1e-3;
        wave_sync();
        acc += eval_wave_frozen(f, o, cv, &hs, mt);
    }
    t1 = now();
    if (t == 0) out[23] = (t1 - t0) / REPS;
    sink[t] = acc;
}

// block-level pieces (512 threads)
__global__ __launch_bounds__(HPE_NT) void k_ubench_block(const DevHand *Hg, DevObs o, double *sink,
                                                        unsigned long long *out) {
    __shared__ Smem sm;
    const int t = threadIdx.x;
    stage_hand<HPE_NT>(sm.hand, Hg);
    if (t < 26) sm.fk.th[t] = 5.0 + t;
    __syncthreads();
    const DevHand *H = &sm.hand;
    const CloudGlobal cv = obs_cloud(o);
    double acc = 0;
    unsigned long long t0, t1;
    // 11: eval_block<EV_COST, 512>
    t0 = now();
    for (int r = 0; r < REPS; ++r) {
        if (t < 26) sm.fk.th[t] += 1e-3;
        __syncthreads();
        acc += eval_block<EV_COST, HPE_NT>(sm, o, cv, H, nullptr, load_pt(cv, t));
    }
    t1 = now();
    if (t == 0) out[11] = (t1 - t0) / REPS;
    // 12: search_align<512> alone (FK done above)
    t0 = now();
    for (int r = 0; r < REPS; ++r) {
        acc += search_align<HPE_NT, false>(sm.fk, cv, H, nullptr, load_pt(cv, t));
        __syncthreads();
    }
    t1 = now();
    if (t == 0) out[12] = (t1 - t0) / REPS;
    // 13: block_sum3<512>
    double a = t, b = t, c = t;
    t0 = now();
    for (int r = 0; r < REPS; ++r) {
        block_sum3<HPE_NT>(sm.red, a, b, c);
        a += 1;
    }
    t1 = now();
    acc += a + b + c;
    if (t == 0) out[13] = (t1 - t0) / REPS;
    // 14: fk by wave 0 + __syncthreads
    t0 = now();
    for (int r = 0; r < REPS; ++r) {
        if (t < 26) sm.fk.th[t] += 1e-3;
        __syncthreads();
        if (t < 64) fk_wave(sm.fk, H);
        __syncthreads();
    }
    t1 = now();
    if (t == 0) out[14] = (t1 - t0) / REPS;
    sink[t] = acc;
}

int main() {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        printf("no device\n");
        return 1;
    }
    hpe_hand_params p;
    std::memset(&p, 0, sizeof(p));
    for (int k = 0; k < 20; ++k) p.geo_cm[k] = 2.0 + 0.1 * k;
    for (int k = 0; k < 48; ++k) p.radii_cm[k] = 1.0;
    const double cmc[5] = {150, 107.5, 89.8, 76.5, 59.6}, spc[5] = {-1.86, -1.86, 0, 1.91, 3.84};
    for (int k = 0; k < 5; ++k) {
        p.cmc_deg[k] = cmc[k];
        p.spacing_cm[k] = spc[k];
    }
    DevHand h;
    hpe::build_dev_hand(p, h);
    DevHand *dh;
    hipMalloc(&dh, sizeof(DevHand));
    hipMemcpy(dh, &h, sizeof(h), hipMemcpyHostToDevice);
    const int N = 250;
    std::vector<double> cl(3 * N);
    for (int i = 0; i < 3 * N; ++i) cl[i] = (i % 97) * 0.01 - (i < 2 * N ? 0 : 32);
    double *dc, *dd;
    float *dt;
    hipMalloc(&dc, sizeof(double) * 3 * N);
    hipMemcpy(dc, cl.data(), sizeof(double) * 3 * N, hipMemcpyHostToDevice);
    hipMalloc(&dd, sizeof(double) * 76800);
    hipMemset(dd, 0, sizeof(double) * 76800);
    hipMalloc(&dt, sizeof(float) * 76800);
    hipMemset(dt, 0, sizeof(float) * 76800);
    DevObs o;
    o.cx = dc; o.cy = dc + N; o.cz = dc + 2 * N;
    o.depth = dd; o.dt = dt; o.n = N; o.lambda = 48.0 / N; o.scale = 0.1; o.dtmax = 100;
    const double K[9] = {241.42, 0, 160, 0, 241.42, 120, 0, 0, 1};
    std::memcpy(o.K, K, sizeof(K));
    int32_t *dm;
    hipMalloc(&dm, sizeof(int32_t) * N);
    double *sink;
    hipMalloc(&sink, sizeof(double) * 1024);
    unsigned long long *dout;
    hipMalloc(&dout, sizeof(unsigned long long) * 32);
    hipMemset(dout, 0, sizeof(unsigned long long) * 32);
    const char *names[] = {"fk_wave (H in LDS)", "fk_wave (H in HBM)", "eval_wave_frozen N=250",
                           "wave_sum3", "depth_term (48 lanes, gathers)", "align_frozen N=250",
                           "collision 144 pairs", "dependent global load (L2)",
                           "sincos f64 (dependent)", "sqrt f64 (dependent)",
                           "16 dependent f64 mul+add", "eval_block<COST,512> N=250",
                           "search_align<512> N=250", "block_sum3<512>", "fk (wave 0) + syncs",
                           "fk + depth (no overlap)", "fk + align_frozen", "fk + depth + align",
                           "fk TRANSLATE (joints+spheres)", "f64 a/180 (dependent)",
                           "trig phase alone", "fk+depth+align+coll", "written-out frozen eval",
                           "eval_wave_frozen again"};
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(k_ubench, dim3(1), dim3(256), 0, 0, dh, o, dm, sink, dout);
        hipLaunchKernelGGL(k_ubench_block, dim3(1), dim3(HPE_NT), 0, 0, dh, o, sink, dout);
        hipDeviceSynchronize();
    }
    unsigned long long out[32];
    hipMemcpy(out, dout, sizeof(out), hipMemcpyDeviceToHost);
    for (int k = 0; k < 24; ++k) printf("%-34s %8llu cycles\n", names[k], out[k]);
    return 0;
}
