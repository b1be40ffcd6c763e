// Grid-barrier experiment (diagnostic, not product).  Question: what does one grid-wide barrier
// cost on MI355X for a persistent grid of one 1024-thread workgroup per CU, and is data written
// before it by one XCD visible after it on the others?
//   MODE 0: every thread __threadfence(), workgroup barrier, thread 0 atomicAdd + acquire spin
//   MODE 1: workgroup barrier, thread 0 release fetch_add + acquire spin (agent scope)
//   MODE 2: as 1, but the spin is a relaxed load and one acquire fence after it
// Every spin has a time limit (s_memrealtime, 100 MHz): a grid that is not co-resident ends
// with an error count instead of hanging.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o scripts/exp_gridbar scripts/exp_gridbar.cpp
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr unsigned long long kLimit = 100000000ull / 5;   // 200 ms of s_memrealtime ticks

template <int MODE>
__device__ __forceinline__ bool grid_bar(unsigned* ctr, unsigned target, unsigned long long t0) {
    bool ok = true;
    if (MODE == 0) __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) {
        if (MODE == 0) atomicAdd(ctr, 1u);
        else __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        for (;;) {
            unsigned v = MODE == 2 ? __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                   : __hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
            if (v >= target) break;
            if (__builtin_amdgcn_s_memrealtime() - t0 > kLimit) { ok = false; break; }
            __builtin_amdgcn_s_sleep(1);
        }
        if (MODE == 2) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
    return ok;
}

template <int MODE>
__global__ __launch_bounds__(1024) void bar_kernel(unsigned* ctr, int* buf, int nstage, int* err,
                                                  unsigned long long* tm) {
    const int wg = blockIdx.x, nwg = gridDim.x, tid = threadIdx.x;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    int bad = 0;
    for (int s = 0; s < nstage; ++s) {
        int* b = buf + (s & 1) * nwg * 64;
        if (tid < 64) b[wg * 64 + tid] = s * 4096 + wg;
        if (!grid_bar<MODE>(ctr, (unsigned)(s + 1) * nwg, t0)) { bad += 1000000; break; }
        if (tid < 64) {
            const int o = (wg + 37 + s) % nwg;
            if (b[o * 64 + tid] != s * 4096 + o) ++bad;
        }
    }
    if (bad) atomicAdd(err, bad);
    if (tid == 0) tm[wg] = __builtin_amdgcn_s_memrealtime() - t0;
}

template <int MODE>
void run(int nwg, int nstage) {
    unsigned* ctr;
    int *buf, *err;
    unsigned long long* tm;
    CK(hipMalloc(&ctr, 4));
    CK(hipMalloc(&buf, 2 * nwg * 64 * 4));
    CK(hipMalloc(&err, 4));
    CK(hipMalloc(&tm, nwg * 8));
    for (int rep = 0; rep < 3; ++rep) {
        CK(hipMemset(ctr, 0, 4));
        CK(hipMemset(err, 0, 4));
        CK(hipMemset(buf, 0xff, 2 * nwg * 64 * 4));
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        CK(hipEventRecord(a));
        hipLaunchKernelGGL(bar_kernel<MODE>, dim3(nwg), dim3(1024), 0, 0, ctr, buf, nstage, err, tm);
        CK(hipEventRecord(b));
        CK(hipDeviceSynchronize());
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        int e;
        CK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
        std::vector<unsigned long long> t(nwg);
        CK(hipMemcpy(t.data(), tm, nwg * 8, hipMemcpyDeviceToHost));
        unsigned long long mx = 0;
        for (auto v : t) mx = v > mx ? v : mx;
        printf("mode %d nwg %d stages %d: %.3f ms total, %.3f us/barrier (in-kernel %.3f us), errors %d\n", MODE, nwg,
               nstage, ms, 1000.0 * ms / nstage, mx / 100.0 / nstage, e);
    }
}

int main(int argc, char** argv) {
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    int occ = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, bar_kernel<0>, 1024, 0));
    printf("CUs %d, 1024-thread workgroups per CU %d\n", cus, occ);
    const int nstage = 2000;
    for (int nwg : {cus / 2, cus}) {
        run<0>(nwg, nstage);
        run<1>(nwg, nstage);
        run<2>(nwg, nstage);
    }
    return 0;
}
