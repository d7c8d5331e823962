// tools/ubench_grid.hip -- is a grid-resident PSO generation loop worth building?
// (diagnostic, not part of the product)
//
// Models the cross-block data flow of one k_pso_gen generation at P = 256 blocks x 512
// threads (one block per CU): every block reads the 256 {tag, pbest cost} granules of the
// previous generation (the gmin reduction's inputs) plus NIB inbox granules, does W ticks
// of work (100 MHz s_memrealtime; the in-kernel chain of a generation is ~4.5 us), then
// publishes its own granule.  Two forms:
//   launch      one launch per generation, G launches captured in a hipGraph (today's
//               k_pso_gen structure: the kernel boundary orders the generations);
//   persistent  ONE launch, generations separated by polling the granules' tags: 16-B
//               sc1 stores of {tag, value} (one instruction, untorn), 16-B sc1 load polls
//               by wave 0 (MI355X_MICROARCH.md hand-off table, row 1: data-tagged
//               granules need no separate flag), bounded (an abort flag ends every block).
// Prints us per generation for both forms at W = 0 and W = 450 ticks.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tools/ubench_grid tools/ubench_grid.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define NB 256    // blocks = particles
#define NT 512    // threads per block
#define NIB 24    // inbox granules read per block (both topology variants)
#define POLL_MAX 400000

struct __align__(16) Gran {
    unsigned long long tag;
    double val;
};

// 16-B loads / stores with the sc1 cache policy (aux bit 4 = SC1 on gfx950) through a
// buffer resource, so the compiler tracks their vmcnt itself (several loads in flight).
typedef unsigned int u4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), 0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ Gran ld_sc1(__amdgpu_buffer_rsrc_t r, int off) {
    const u4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16);
    Gran g;
    g.tag = ((unsigned long long)v.y << 32) | v.x;
    g.val = __hiloint2double((int)v.w, (int)v.z);
    return g;
}
__device__ __forceinline__ void st_sc1(__amdgpu_buffer_rsrc_t r, int off, Gran g) {
    u4 v;
    v.x = (unsigned)g.tag;
    v.y = (unsigned)(g.tag >> 32);
    v.z = (unsigned)__double2loint(g.val);
    v.w = (unsigned)__double2hiint(g.val);
    __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 16);
}

__device__ __forceinline__ void spin(unsigned w) {
    if (!w) return;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < w) __builtin_amdgcn_s_sleep(1);
}

// launch form: one generation; the boundary makes generation g-1's plain stores visible
__global__ __launch_bounds__(NT) void k_launch(Gran *gr, const Gran *ib, int g, unsigned w,
                                               double *sink) {
    __shared__ double red[NT / 64];
    const int b = blockIdx.x, t = threadIdx.x;
    double m = 1e300;
    if (t < 64) {
        const Gran *src = gr + ((g - 1) & 1) * NB;
        for (int k = t; k < NB; k += 64) m = fmin(m, src[k].val);
        if (t < NIB) m = fmin(m, ib[b * NIB + t].val);
        for (int o = 32; o > 0; o >>= 1) m = fmin(m, __shfl_xor(m, o));
        if (t == 0) red[0] = m;
    }
    __syncthreads();
    m = red[0];
    spin(w + (b % 7) * 3);
    __syncthreads();
    if (t == 0) gr[(g & 1) * NB + b] = Gran{(unsigned long long)g, m + b};
    if (t == 1) sink[b] = m;
}

// persistent form: G generations in one launch
__global__ __launch_bounds__(NT) void k_persist(Gran *gr, Gran *ib, int G, unsigned w,
                                                int *abort_flag, double *sink,
                                                unsigned long long *polls) {
    __shared__ double red[NT / 64];
    __shared__ int bail;
    const int b = blockIdx.x, t = threadIdx.x;
    double m = 0;
    unsigned long long np = 0;
    for (int g = 1; g < G; ++g) {
        if (t < 64) {
            const __amdgpu_buffer_rsrc_t rg = rsrc(gr + ((g - 1) & 1) * NB);
            const __amdgpu_buffer_rsrc_t ri = rsrc(ib + (size_t)((g - 1) & 1) * NB * NIB + b * NIB);
            bool ok = false;
            int tries = 0;
            double mm = 1e300;
            while (!ok) {
                // five 16-B loads in flight per lane, unconditional (the inbox slot clamped)
                Gran q[5];
#pragma unroll
                for (int k = 0; k < 4; ++k) q[k] = ld_sc1(rg, 16 * (t + 64 * k));
                q[4] = ld_sc1(ri, 16 * (t < NIB ? t : 0));
                bool mine = true;
                mm = 1e300;
#pragma unroll
                for (int k = 0; k < 5; ++k) {
                    mine = mine && q[k].tag == (unsigned long long)(g - 1);
                    mm = fmin(mm, q[k].val);
                }
                ok = __all(mine);
                ++np;
                if (!ok) {
                    ++tries;
                    if (tries > POLL_MAX ||
                        ((tries & 63) == 0 && __hip_atomic_load(abort_flag, __ATOMIC_RELAXED,
                                                                __HIP_MEMORY_SCOPE_AGENT))) {
                        if (t == 0) __hip_atomic_store(abort_flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        ok = true;
                        tries = -1;
                    } else {
                        __builtin_amdgcn_s_sleep(1);
                    }
                }
            }
            for (int o = 32; o > 0; o >>= 1) mm = fmin(mm, __shfl_xor(mm, o));
            if (t == 0) {
                red[0] = mm;
                bail = tries < 0;
            }
        }
        __syncthreads();
        if (bail) break;
        m = red[0];
        spin(w + (b % 7) * 3);
        __syncthreads();
        // publish: one 16-B sc1 store per granule (this block's cost, and its inbox pushes
        // to NIB receivers modelled as granules to block (b + k) % NB)
        if (t == 0) st_sc1(rsrc(gr + (g & 1) * NB), 16 * b, Gran{(unsigned long long)g, m + b});
        if (t >= 64 && t < 64 + NIB) {
            const int r = (b + 1 + (t - 64) * 7) % NB, s = (t - 64);
            st_sc1(rsrc(ib + (size_t)(g & 1) * NB * NIB), 16 * (r * NIB + s), Gran{(unsigned long long)g, m});
        }
    }
    if (t == 0) {
        sink[b] = m;
        polls[b] = np;
    }
}

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            return 1;                                                              \
        }                                                                          \
    } while (0)

int main() {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        printf("no device\n");
        return 1;
    }
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    int occ = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_persist, NT, 0));
    printf("CUs %d, k_persist blocks/CU %d\n", prop.multiProcessorCount, occ);
    if (occ * prop.multiProcessorCount < NB) {
        printf("grid not co-resident: skipping the persistent form\n");
        return 1;
    }
    Gran *gr, *ib;
    int *abort_flag;
    double *sink;
    unsigned long long *polls;
    CK(hipMalloc(&gr, sizeof(Gran) * 2 * NB));
    CK(hipMalloc(&ib, sizeof(Gran) * 2 * NB * NIB));
    CK(hipMalloc(&abort_flag, sizeof(int)));
    CK(hipMalloc(&sink, sizeof(double) * NB));
    CK(hipMalloc(&polls, sizeof(unsigned long long) * NB));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int G = 31;
    for (unsigned w : {0u, 450u}) {
        // initial granules: tag 0 everywhere (generation 0 published)
        std::vector<Gran> init(2 * NB * NIB, Gran{0ull, 1.0});
        CK(hipMemcpy(gr, init.data(), sizeof(Gran) * 2 * NB, hipMemcpyHostToDevice));
        CK(hipMemcpy(ib, init.data(), sizeof(Gran) * 2 * NB * NIB, hipMemcpyHostToDevice));
        // launch form in a graph
        hipGraph_t graph;
        hipGraphExec_t exec;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
        for (int g = 1; g < G; ++g)
            hipLaunchKernelGGL(k_launch, dim3(NB), dim3(NT), 0, s, gr, ib, g, w, sink);
        CK(hipStreamEndCapture(s, &graph));
        CK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
        float best_l = 1e30f, best_p = 1e30f;
        for (int rep = 0; rep < 20; ++rep) {
            CK(hipEventRecord(e0, s));
            CK(hipGraphLaunch(exec, s));
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (rep >= 2 && ms < best_l) best_l = ms;
        }
        // persistent form
        int bad = 0;
        unsigned long long pmax = 0, psum = 0;
        for (int rep = 0; rep < 20; ++rep) {
            CK(hipMemcpy(gr, init.data(), sizeof(Gran) * 2 * NB, hipMemcpyHostToDevice));
            CK(hipMemcpy(ib, init.data(), sizeof(Gran) * 2 * NB * NIB, hipMemcpyHostToDevice));
            CK(hipMemset(abort_flag, 0, sizeof(int)));
            CK(hipEventRecord(e0, s));
            hipLaunchKernelGGL(k_persist, dim3(NB), dim3(NT), 0, s, gr, ib, G, w, abort_flag, sink, polls);
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            int ab = 0;
            CK(hipMemcpy(&ab, abort_flag, sizeof(int), hipMemcpyDeviceToHost));
            bad |= ab;
            std::vector<unsigned long long> np(NB);
            CK(hipMemcpy(np.data(), polls, sizeof(unsigned long long) * NB, hipMemcpyDeviceToHost));
            for (auto v : np) {
                pmax = v > pmax ? v : pmax;
                psum += v;
            }
            if (rep >= 2 && ms < best_p) best_p = ms;
        }
        printf("W=%3u ticks: launch form %.3f us/gen (%d launches, graph)   persistent %.3f us/gen "
               "(one launch, %d generations)%s   polls/gen/block avg %.2f max %.0f\n",
               w, 1e3f * best_l / (G - 1), G - 1, 1e3f * best_p / (G - 1), G - 1,
               bad ? "  ABORTED (not co-resident?)" : "", (double)psum / (20.0 * NB * (G - 1)),
               (double)pmax / (G - 1));
        CK(hipGraphExecDestroy(exec));
        CK(hipGraphDestroy(graph));
    }
    return 0;
}
