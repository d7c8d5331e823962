// tools/ubench_launch.hip -- diagnostic: the kernel-to-kernel boundary of a chain of dependent
// launches replayed as one hipGraph (the shape of a tracked frame's 30 generations): G
// launches of B workgroups x 512 threads, each workgroup reading one word the previous launch
// wrote and writing one, and optionally a 1 MB scatter of stores (dirty L2 lines at the
// boundary).  Prints the replay time per launch.  Not part of the product.
// Build: hipcc -O3 --offload-arch=gfx950 tools/ubench_launch.hip -o tools/ubench_launch
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ __launch_bounds__(512) void k_step(const unsigned *__restrict__ in, unsigned *__restrict__ out,
                                              double *__restrict__ scratch, int g, int dirty) {
    const int b = blockIdx.x, t = threadIdx.x;
    __shared__ unsigned s;
    if (t == 0) s = in[(b * 7 + g) % gridDim.x];
    __syncthreads();
    if (dirty == 1) scratch[((size_t)b * 512 + t) % (1 << 17)] = (double)(s + g);  // 1 MB of lines
    if (dirty == 2)  // the same stores, nontemporal
        __builtin_nontemporal_store((double)(s + g), &scratch[((size_t)b * 512 + t) % (1 << 17)]);
    if (t == 0) out[b] = s + 1;
}

// dirty == 3: the same chain with no kernel argument at all: the words live in __device__
// arrays whose addresses are link-time constants (no kernarg load before the first load)
__device__ unsigned g_a[4096], g_b[4096];
template <int PAR>
__global__ __launch_bounds__(512) void k_static() {
    const int b = blockIdx.x, t = threadIdx.x;
    const unsigned *in = PAR ? g_b : g_a;
    unsigned *out = PAR ? g_a : g_b;
    __shared__ unsigned s;
    if (t == 0) s = in[(b * 7 + PAR) % gridDim.x];
    __syncthreads();
    if (t == 0) out[b] = s + 1;
}

static void launch(int B, int g, int dirty, hipStream_t st, unsigned *a, unsigned *b, double *scr) {
    if (dirty == 3) {
        if (g & 1) hipLaunchKernelGGL(k_static<1>, dim3(B), dim3(512), 0, st);
        else hipLaunchKernelGGL(k_static<0>, dim3(B), dim3(512), 0, st);
        return;
    }
    hipLaunchKernelGGL(k_step, dim3(B), dim3(512), 0, st, (g & 1) ? b : a, (g & 1) ? a : b, scr, g, dirty);
}

int main(int argc, char **argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 256, G = argc > 2 ? atoi(argv[2]) : 30;
    const int dirty = argc > 3 ? atoi(argv[3]) : 0;
    unsigned *a, *b;
    double *scr;
    hipMalloc(&a, 4 * B);
    hipMalloc(&b, 4 * B);
    hipMalloc(&scr, 8 << 17);
    hipMemset(a, 0, 4 * B);
    hipStream_t st;
    hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    hipGraph_t gr;
    hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal);
    for (int g = 0; g < G; ++g) launch(B, g, dirty, st, a, b, scr);
    hipStreamEndCapture(st, &gr);
    hipGraphExec_t ex;
    hipGraphInstantiate(&ex, gr, nullptr, nullptr, 0);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int w = 0; w < 5; ++w) hipGraphLaunch(ex, st);
    hipStreamSynchronize(st);
    const int R = 50;
    hipEventRecord(e0, st);
    for (int r = 0; r < R; ++r) hipGraphLaunch(ex, st);
    hipEventRecord(e1, st);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    printf("B=%d G=%d dirty=%d: %.3f us per launch (graph replay, %d graphs)\n", B, G, dirty,
           ms * 1e3 / (R * G), R);
    // the same chain launched directly
    hipEventRecord(e0, st);
    for (int r = 0; r < 10; ++r)
        for (int g = 0; g < G; ++g) launch(B, g, dirty, st, a, b, scr);
    hipEventRecord(e1, st);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    printf("B=%d G=%d dirty=%d: %.3f us per launch (direct launches)\n", B, G, dirty, ms * 1e3 / (10 * G));
    return 0;
}
