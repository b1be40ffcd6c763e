// Grid-barrier experiment (diagnostic, not product).  Question: what does one grid-wide barrier
// cost on MI355X for a persistent grid of one 1024-thread workgroup per CU, and which store /
// load forms make data written before it on one XCD visible after it on the others?
//
// Barrier: every workgroup publishes its epoch in its own 128-byte flag slot (no shared counter:
// same-address atomics serialise), then wave 0 polls all the slots (4 per lane).
// Data: word i of a shared array is written by workgroup i % nwg, so every 128-byte line holds
// words of 32 workgroups spread over all 8 XCDs; after the barrier every workgroup reads and
// checks every word.
//   DATA 0: data stores and loads plain (expected stale: the writer's L2 is write-back)
//   DATA 1: stores agent-scope (sc1), loads plain
//   DATA 2: stores agent-scope (sc1), loads agent-scope (sc1)
//   DATA 3: stores sc1, loads plain after an agent acquire fence (L2 invalidate)
//   FRESH:  1: a fresh buffer region per stage (no line was read before it was written);
//           0: one region rewritten every stage (stale lines from the previous read are likely)
// Every poll has a time limit (s_memrealtime, 100 MHz): a grid that is not co-resident ends with
// a timeout count instead of hanging.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o scripts/exp_gridbar scripts/exp_gridbar.cpp
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr unsigned long long kLimit = 100000000ull / 5;   // 200 ms of s_memrealtime ticks
constexpr int kWords = 4096;                              // shared words per stage

__device__ __forceinline__ void st_agent(int* p, int v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ int ld_agent(const int* p) { return __hip_atomic_load(const_cast<int*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// returns false (in every thread) on timeout
__device__ __forceinline__ bool grid_bar(int* flags, int epoch, unsigned long long t0, int* lds_ok) {
    // every wave's stores done before the workgroup publishes
    __builtin_amdgcn_s_waitcnt(0);   // vmcnt(0) expcnt(0) lgkmcnt(0)
    __syncthreads();
    const int nwg = gridDim.x;
    if (threadIdx.x < 64) {
        if (threadIdx.x == 0) st_agent(flags + blockIdx.x * 32, epoch);
        bool ok = true;
        for (;;) {
            bool all = true;
            for (int w = threadIdx.x; w < nwg; w += 64) all = all && ld_agent(flags + w * 32) >= epoch;
            if (__all(all)) break;
            if (__builtin_amdgcn_s_memrealtime() - t0 > kLimit) { ok = false; break; }
            __builtin_amdgcn_s_sleep(1);
        }
        if (threadIdx.x == 0) *lds_ok = ok;
    }
    __syncthreads();
    return *lds_ok;
}

template <int DATA, int FRESH>
__global__ __launch_bounds__(1024) void bar_kernel(int* flags, int* buf, int nstage, int* err,
                                                  unsigned long long* tm) {
    __shared__ int lds_ok;
    const int wg = blockIdx.x, nwg = gridDim.x, tid = threadIdx.x;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    int bad = 0, tmo = 0;
    for (int s = 0; s < nstage; ++s) {
        int* b = buf + (FRESH ? (long long)s * kWords : 0);
        for (int i = wg + nwg * tid; i < kWords && tid < kWords / nwg + 1; i += nwg * 1024) {
            const int v = s * 65536 + i;
            if (DATA == 0) b[i] = v; else st_agent(b + i, v);
        }
        if (!grid_bar(flags, s + 1, t0, &lds_ok)) { tmo = 1; break; }
        if (DATA == 3) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        for (int i = tid; i < kWords; i += 1024) {
            const int v = DATA == 2 ? ld_agent(b + i) : b[i];
            if (v != s * 65536 + i) ++bad;
        }
    }
    if (bad) atomicAdd(err, bad);
    if (tmo && tid == 0) atomicAdd(err + 1, 1);
    if (tid == 0) tm[wg] = __builtin_amdgcn_s_memrealtime() - t0;
}

// Tagged data instead of a barrier: word i of stage s is the pair {value, s + 1} written by
// one 8-byte agent-scope store; readers poll the words they need until every tag is s + 1.
// Double-buffered by stage parity: a workgroup that sees all of stage s's words knows every
// workgroup finished reading stage s - 1 (each writes its stage-s words after its stage-s-1 reads).
//   POLL 0: agent-scope (sc1) loads;  POLL 1: plain loads (a stale L2 line would never update)
__device__ __forceinline__ void st_agent2(long long* p, long long v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ long long ld_agent2(const long long* p) { return __hip_atomic_load(const_cast<long long*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

template <int POLL>
__global__ __launch_bounds__(1024) void tag_kernel(long long* buf, int nstage, int* err, unsigned long long* tm) {
    const int wg = blockIdx.x, nwg = gridDim.x, tid = threadIdx.x;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    int bad = 0, tmo = 0;
    for (int s = 0; s < nstage && !tmo; ++s) {
        long long* b = buf + (s & 1) * kWords;
        for (int i = wg + nwg * tid; i < kWords && tid < kWords / nwg + 1; i += nwg * 1024)
            st_agent2(b + i, ((long long)(s + 1) << 32) | (unsigned)(s * 65536 + i));
        for (int i = tid; i < kWords; i += 1024) {
            long long v;
            for (;;) {
                if (POLL == 1) asm volatile("" ::: "memory");
                v = POLL == 0 ? ld_agent2(b + i) : b[i];
                if ((int)(v >> 32) == s + 1) break;
                if (__builtin_amdgcn_s_memrealtime() - t0 > kLimit) { tmo = 1; break; }
                __builtin_amdgcn_s_sleep(1);
            }
            if (tmo) break;
            if ((int)v != s * 65536 + i) ++bad;
        }
    }
    if (bad) atomicAdd(err, bad);
    if (tmo) atomicAdd(err + 1, 1);
    if (tid == 0) tm[wg] = __builtin_amdgcn_s_memrealtime() - t0;
}

template <int POLL>
void run_tag(int nwg, int nstage) {
    long long* buf;
    int* err;
    unsigned long long* tm;
    CK(hipMalloc(&buf, 2 * kWords * 8));
    CK(hipMalloc(&err, 8));
    CK(hipMalloc(&tm, nwg * 8));
    for (int rep = 0; rep < 2; ++rep) {
        CK(hipMemset(err, 0, 8));
        CK(hipMemset(buf, 0, 2 * kWords * 8));
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        CK(hipEventRecord(a));
        hipLaunchKernelGGL((tag_kernel<POLL>), dim3(nwg), dim3(1024), 0, 0, buf, nstage, err, tm);
        CK(hipEventRecord(b));
        CK(hipDeviceSynchronize());
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        int ev[2];
        CK(hipMemcpy(ev, err, 8, hipMemcpyDeviceToHost));
        printf("tagged poll %d nwg %d stages %d: %.3f us/stage, bad words %d, timed-out threads %d\n", POLL, nwg, nstage,
               1000.0 * ms / nstage, ev[0], ev[1]);
    }
    CK(hipFree(buf));
    CK(hipFree(err));
    CK(hipFree(tm));
}

template <int DATA, int FRESH>
void run(int nwg, int nstage) {
    int *flags, *buf, *err;
    unsigned long long* tm;
    CK(hipMalloc(&flags, nwg * 128));
    const size_t nbuf = (size_t)(FRESH ? nstage : 1) * kWords * 4;
    CK(hipMalloc(&buf, nbuf));
    CK(hipMalloc(&err, 8));
    CK(hipMalloc(&tm, nwg * 8));
    for (int rep = 0; rep < 2; ++rep) {
        CK(hipMemset(flags, 0, nwg * 128));
        CK(hipMemset(err, 0, 8));
        CK(hipMemset(buf, 0xff, nbuf));
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        CK(hipEventRecord(a));
        hipLaunchKernelGGL((bar_kernel<DATA, FRESH>), dim3(nwg), dim3(1024), 0, 0, flags, buf, nstage, err, tm);
        CK(hipEventRecord(b));
        CK(hipDeviceSynchronize());
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        int ev[2];
        CK(hipMemcpy(ev, err, 8, hipMemcpyDeviceToHost));
        printf("data %d fresh %d nwg %d stages %d: %.3f us/stage, bad words %d (of %lld), timeouts %d\n", DATA, FRESH,
               nwg, nstage, 1000.0 * ms / nstage, ev[0], (long long)nwg * nstage * kWords, ev[1]);
    }
    CK(hipFree(flags));
    CK(hipFree(buf));
    CK(hipFree(err));
    CK(hipFree(tm));
}

int main() {
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    printf("CUs %d\n", cus);
    const int nstage = 1000;
    for (int nwg : {cus}) {
        run<1, 1>(nwg, nstage);
        run<2, 1>(nwg, nstage);
        run_tag<0>(nwg, nstage);
        run_tag<0>(nwg / 2, nstage);
        run_tag<1>(nwg, 50);
    }
    return 0;
}
