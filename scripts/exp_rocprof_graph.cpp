// Minimal reproducer (diagnostic, not product) for the SIGSEGV that `rocprofv3 --kernel-trace`
// raises inside librocprofiler-sdk when a process replays hipGraphs of kernels with large
// parameter blocks (profiles/r05_rocprof_segv.txt).  No engine code: one
// kernel whose by-value argument is KB bytes, a graph of N such nodes (each with distinct
// argument bytes), replayed R times.  Without the tracer this runs clean; the engine's decode
// graphs have the same shape (~190 nodes with 0.2-0.5 KB kernel arguments each).
// Build: hipcc --offload-arch=gfx950 -O2 -std=c++17 -o exp_rocprof_graph exp_rocprof_graph.cpp
// Run:   rocprofv3 --kernel-trace --stats -d <dir> -- ./exp_rocprof_graph [nodes] [replays]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <int KB>
struct Big {
    unsigned w[KB / 4];
};

template <int KB>
__global__ void k_big(Big<KB> a, unsigned* out) {
    unsigned s = 0;
    for (int i = threadIdx.x; i < KB / 4; i += blockDim.x) s ^= a.w[i];
    if (s == 0x9e3779b9u) out[blockIdx.x] = s;
}

template <int KB>
static void run(int nodes, int replays, unsigned* out, hipStream_t st) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
    for (int n = 0; n < nodes; ++n) {
        Big<KB> a;
        for (int i = 0; i < KB / 4; ++i) a.w[i] = (unsigned)(n * 131 + i);
        hipLaunchKernelGGL(k_big<KB>, dim3(4), dim3(64), 0, st, a, out);
    }
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int r = 0; r < replays; ++r) CK(hipGraphLaunch(ge, st));
    CK(hipStreamSynchronize(st));
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    printf("kernarg %d B: %d nodes x %d replays ok\n", KB, nodes, replays);
    fflush(stdout);
}

int main(int argc, char** argv) {
    const int nodes = argc > 1 ? atoi(argv[1]) : 200;
    const int replays = argc > 2 ? atoi(argv[2]) : 200;
    hipStream_t st;
    CK(hipStreamCreate(&st));
    unsigned* out;
    CK(hipMalloc(&out, 4096));
    run<256>(nodes, replays, out, st);
    run<512>(nodes, replays, out, st);
    run<1024>(nodes, replays, out, st);
    run<2048>(nodes, replays, out, st);
    return 0;
}
