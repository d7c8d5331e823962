// Residency census (diagnostic): how many 256-thread workgroups a CU admits at once for a
// given VGPR / LDS footprint.  Every workgroup records its start time (100 MHz clock) and
// placement, then holds its CU for HOLD_US; a workgroup that starts later than HOLD_US / 2
// after the first was queued behind a resident one.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define HOLD_US 40

template <int NV, int LDSB, int NS = 0>
__global__ __launch_bounds__(256) void k_census(unsigned long long *out, int pad) {
    __shared__ float lds[LDSB / 4];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0) {
        const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
        const unsigned xc = __builtin_amdgcn_s_getreg((3 << 11) | 20);
        out[(blockIdx.x * 4 + (threadIdx.x >> 6)) * 2] = t0;
        out[(blockIdx.x * 4 + (threadIdx.x >> 6)) * 2 + 1] = ((unsigned long long)xc << 32) | hw;
    }
    lds[threadIdx.x % (LDSB / 4)] = (float)pad;
    // occupy NV VGPRs: the asm clobbers registers up to v(NV-1)
    if (NV >= 128) asm volatile("v_mov_b32 v127, 0" ::: "v127");
    else if (NV >= 120) asm volatile("v_mov_b32 v119, 0" ::: "v119");
    else if (NV >= 104) asm volatile("v_mov_b32 v103, 0" ::: "v103");
    else asm volatile("v_mov_b32 v63, 0" ::: "v63");
    if (NS >= 100) asm volatile("s_mov_b32 s99, 0" ::: "s99");
    else if (NS >= 96) asm volatile("s_mov_b32 s95, 0" ::: "s95");
    else if (NS >= 80) asm volatile("s_mov_b32 s79, 0" ::: "s79");
    while (__builtin_amdgcn_s_memrealtime() - t0 < HOLD_US * 100) __builtin_amdgcn_s_sleep(10);
    __syncthreads();
    if (lds[(threadIdx.x + 1) % (LDSB / 4)] == 12345.f) out[0] = 0;
}

template <int NV, int LDSB, int NS = 0>
static void run(const char *name, int nblk) {
    unsigned long long *d;
    std::vector<unsigned long long> h(nblk * 8);
    hipMalloc(&d, h.size() * 8);
    hipMemset(d, 0, h.size() * 8);
    for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL((k_census<NV, LDSB, NS>), dim3(nblk), dim3(256), 0, 0, d, rep);
    hipDeviceSynchronize();
    hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
    unsigned long long tmin = ~0ull;
    for (int w = 0; w < nblk * 4; ++w) tmin = h[2 * w] < tmin ? h[2 * w] : tmin;
    int late = 0, slotmax = 0;
    for (int w = 0; w < nblk * 4; ++w) {
        if (h[2 * w] - tmin > 300) ++late;  // 3 us
        const int slot = (int)(h[2 * w + 1] & 0xF);
        slotmax = slot > slotmax ? slot : slotmax;
    }
    hipFuncAttributes fa;
    hipFuncGetAttributes(&fa, (const void *)k_census<NV, LDSB, NS>);
    int occ = 0;
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_census<NV, LDSB, NS>, 256, 0);
    printf("%-22s blocks %5d: late waves %5d of %5d (%.0f%% of blocks), max wave slot %d; numRegs %d, API blocks/CU %d\n",
           name, nblk, late, nblk * 4, 100.0 * late / (nblk * 4), slotmax, fa.numRegs, occ);
    hipFree(d);
}

int main() {
    run<128, 16992>("vgpr128 lds17k", 1024);
    run<128, 16992, 80>("vgpr128 lds17k s80", 1024);
    run<128, 16992, 96>("vgpr128 lds17k s96", 1024);
    run<128, 16992, 100>("vgpr128 lds17k s100", 1024);
    run<64, 1024, 96>("vgpr64 lds1k s96", 2048);
    run<64, 1024, 100>("vgpr64 lds1k s100", 2048);
    return 0;
}
