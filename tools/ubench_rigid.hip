// tools/ubench_rigid.hip -- diagnostic microbenchmark of the hand-frame refine node
// (hpe_device.hpp rigid_wave / rigid_head / frozen_tail), not part of the product.
// One workgroup; NW waves (argv[1], default 1) each evaluate nodes concurrently, wave 0
// times them with s_memtime: the latency of each piece alone and with 2 waves per SIMD.
// Build: hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -o tools/ubench_rigid \
//        tools/ubench_rigid.hip hand-pose-estimation_amd/csrc/hpe_host.cpp
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../hand-pose-estimation_amd/csrc/hpe_device.hpp"
#include "../hand-pose-estimation_amd/csrc/hpe_host.hpp"

#define REPS 64
#define NT 512

__device__ __forceinline__ unsigned long long now() {
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

__global__ __launch_bounds__(NT) void k_ub(const DevHand *Hg, DevObs o, double *sink,
                                           unsigned long long *out, int nw) {
    __shared__ FkSm fs[8];
    __shared__ DevHand hs;
    __shared__ RigidSm R;
    __shared__ double cloud[3 * 256];
    __shared__ int32_t mt[256];
    const int t = threadIdx.x, w = t >> 6, l = t & 63;
    for (int q = t; q < (int)(sizeof(DevHand) / 8); q += blockDim.x)
        ((double *)&hs)[q] = ((const double *)Hg)[q];
    for (int p = t; p < o.n && p < 256; p += blockDim.x) {
        cloud[p] = o.cx[p];
        cloud[256 + p] = o.cy[p];
        cloud[512 + p] = o.cz[p];
        mt[p] = p % 48;
    }
    if (t < 144) (&R.q[0][0])[t] = 0.5 * (t % 7) - 1.0;
    if (t < 144) (&R.P[0][0])[t] = 0.25 * (t % 5);
    if (t == 0) R.C = 1.0;
    __syncthreads();
    if (w >= nw) return;
    FkSm &f = fs[w];
    const CloudView cv{cloud, cloud + 256, cloud + 512, o.n < 256 ? o.n : 256};
    FrozenPts fp;
    load_frozen_pts(fp, cv, mt, l);
    double acc = 0, thl = (l < 26) ? 5.0 + l : 0.0;
    unsigned long long t0, t1;
    int k = 0;
#define TIMED(...)                                       \
    t0 = now();                                          \
    for (int r = 0; r < REPS; ++r) {                     \
        __VA_ARGS__;                                     \
    }                                                    \
    t1 = now();                                          \
    if (t == 0) out[k] = (t1 - t0) / REPS;               \
    ++k;
    // 0: rigid_wave rotation block (out-of-line sincos)
    TIMED(thl += 1e-3; rigid_wave<RG_ROT>(f, R, thl));
    // 1: rigid_wave rotation block, inlined sincos
    TIMED(thl += 1e-3; (rigid_wave<RG_ROT, false>(f, R, thl)));
    // 2: rigid_wave translation block
    TIMED(thl += 1e-3; rigid_wave<RG_TRANS>(f, R, thl));
    // 3: depth issue + finish on the stored centres (48 lanes)
    TIMED(const DepthG dg = depth_issue(f, l, o, &hs); const double d = depth_finish(dg, o, l < 48);
          acc += d; thl += d * 1e-30);
    // 4: align_frozen_pts (4 points per lane, matchIds in registers)
    TIMED(const double a = align_frozen_pts(f, fp, cv, &hs, l); acc += a; thl += a * 1e-30);
    // 5: wave_sum
    TIMED(thl = wave_sum(thl) * 1e-3 + 1.0);
    // 6: full node, rotation block: rigid_head + frozen_tail (+ C)
    TIMED(thl += 1e-3; const FrozenHead hd = rigid_head<RG_ROT>(f, o, &hs, R, thl);
          const double v = frozen_tail(f, o, cv, &hs, mt, hd, &fp) + R.C; acc += v;
          thl += v * 1e-30);
    // 7: full node, translation block
    TIMED(thl += 1e-3; const FrozenHead hd = rigid_head<RG_TRANS>(f, o, &hs, R, thl);
          const double v = frozen_tail(f, o, cv, &hs, mt, hd, &fp) + R.C; acc += v;
          thl += v * 1e-30);
    // 8: the exact chain node (fk_wave + depth + alignment + collision + sum), for scale
    TIMED(thl += 1e-3; if (l < 26) f.th[l] = thl; wave_sync();
          const double v = eval_wave_frozen<true>(f, o, cv, &hs, mt, nullptr, &thl, &fp);
          acc += v; thl += v * 1e-30);
    // 9: sincos_outline alone (dependent)
    TIMED(const SinCos sc = sincos_outline(thl); thl = sc.s + sc.c * 1e-3);
    // 10: deg2rad + sincos inline (dependent)
    TIMED(double s, c; sincos(deg2rad(thl), &s, &c); thl = s + c * 1e-3);
    // 11: projection of a centre (two fp64 divisions) without the gathers
    TIMED(const double x = thl, y = thl * 0.5, z = 30.0 + thl;
          const double pu = (o.K[0] * x + o.K[1] * y) + o.K[2] * z;
          const double pv = (o.K[3] * x + o.K[4] * y) + o.K[5] * z;
          const double pw = (o.K[6] * x + o.K[7] * y) + o.K[8] * z;
          thl = floor(pu / pw) * 1e-3 + floor(pv / pw) * 1e-4 + 1.0);
    sink[t] = acc + thl;
}

int main(int argc, char **argv) {
    const int nw = argc > 1 ? atoi(argv[1]) : 1;
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
    std::memset(&o, 0, sizeof(o));
    o.cx = dc; o.cy = dc + N; o.cz = dc + 2 * N;
    o.depth = dd; o.dt = dt; o.n = N; o.lambda = 48.0 / N; o.scale = 0.1; o.dtmax = 100;
    const double K[9] = {241.42, 0, 160, 0, 241.42, 120, 0, 0, 1};
    std::memcpy(o.K, K, sizeof(K));
    double *sink;
    hipMalloc(&sink, sizeof(double) * NT);
    unsigned long long *dout;
    hipMalloc(&dout, sizeof(unsigned long long) * 32);
    hipMemset(dout, 0, sizeof(unsigned long long) * 32);
    const char *names[] = {"rigid_wave ROT (outline sincos)", "rigid_wave ROT (inline sincos)",
                           "rigid_wave TRANS", "depth issue+finish", "align_frozen_pts",
                           "wave_sum", "node ROT (head+tail)", "node TRANS (head+tail)",
                           "exact chain node", "sincos_outline (dep)", "deg2rad+sincos (dep)",
                           "projection (2 fp64 div)"};
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(k_ub, dim3(1), dim3(NT), 0, 0, dh, o, sink, dout, nw);
        hipDeviceSynchronize();
    }
    unsigned long long out[32];
    hipMemcpy(out, dout, sizeof(out), hipMemcpyDeviceToHost);
    printf("waves evaluating concurrently: %d\n", nw);
    for (int k = 0; k < 12; ++k) printf("%-34s %8llu cycles\n", names[k], out[k]);
    return 0;
}
