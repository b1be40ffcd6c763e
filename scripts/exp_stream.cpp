// Streaming micro-benchmark (diagnostic, not product): what one decode-GEMV-sized launch can
// read from HBM, by workgroup shape and register-ring depth, with and without a per-item
// VALU load similar to the Q4_K dot.  Each workgroup streams a contiguous slice of a buffer
// larger than the 256 MiB Infinity Cache; the timed launches rotate over 8 such buffers.
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/exp_stream scripts/exp_stream.cpp
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__device__ __forceinline__ u32x4 ldg(const unsigned char* p) {
    return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
}

// WORK: 0 = xor the loads, 1 = ~45 VALU ops per 16 B (the Q4_K dot's shape)
template <int D, int WORK>
__global__ void stream_k(const unsigned char* buf, size_t bytes_per_wg, unsigned* out) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const unsigned char* base = buf + (size_t)blockIdx.x * bytes_per_wg;
    // wave w streams 1 KB chunks w, w+nw, ...
    const size_t nchunks = bytes_per_wg / 1024;
    u32x4 ring[D];
    size_t c = wave;
#pragma unroll
    for (int k = 0; k < D - 1; ++k) {
        ring[k] = ldg(base + (c < nchunks ? c : 0) * 1024 + lane * 16);
        c += nw;
    }
    unsigned acc = 0;
    int a0 = lane * 0x01010101, a1 = lane * 0x02020202;
    for (size_t it = wave; it < nchunks; it += (size_t)nw * D) {
#pragma unroll
        for (int k = 0; k < D; ++k) {
            ring[(k + D - 1) % D] = ldg(base + (c < nchunks ? c : 0) * 1024 + lane * 16);
            c += nw;
            const u32x4 v = ring[k];
            if (it + (size_t)k * nw < nchunks) {
                if (WORK == 0) {
                    acc ^= v.x ^ v.y ^ v.z ^ v.w;
                } else {
                    int dlo = 0, dhi = 0;
                    dlo = __builtin_amdgcn_sdot4(v.x & 0x0F0F0F0F, a0, dlo, false);
                    dlo = __builtin_amdgcn_sdot4(v.y & 0x0F0F0F0F, a1, dlo, false);
                    dlo = __builtin_amdgcn_sdot4(v.z & 0x0F0F0F0F, a0, dlo, false);
                    dlo = __builtin_amdgcn_sdot4(v.w & 0x0F0F0F0F, a1, dlo, false);
                    dhi = __builtin_amdgcn_sdot4((v.x >> 4) & 0x0F0F0F0F, a1, dhi, false);
                    dhi = __builtin_amdgcn_sdot4((v.y >> 4) & 0x0F0F0F0F, a0, dhi, false);
                    dhi = __builtin_amdgcn_sdot4((v.z >> 4) & 0x0F0F0F0F, a1, dhi, false);
                    dhi = __builtin_amdgcn_sdot4((v.w >> 4) & 0x0F0F0F0F, a0, dhi, false);
                    const unsigned sc = (v.x >> (lane & 7)) & 0x3F3F, mm = (v.y >> (lane & 3)) & 0x3F3F;
                    const int S = (int)(sc & 0xFF) * dlo + (int)(sc >> 8) * dhi;
                    const int M = (int)(mm & 0xFF) * a0 + (int)(mm >> 8) * a1;
                    const float f = (float)(v.z & 0xFFFF) * 1e-3f * (float)S - (float)(v.w & 0xFFFF) * 1e-3f * (float)M;
                    acc += __float_as_uint(f);
                }
            }
        }
    }
    if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

typedef void (*Fn)(const unsigned char*, size_t, unsigned*);

template <int D, int W>
Fn pick() { return stream_k<D, W>; }

int main(int argc, char** argv) {
    const size_t mb = argc > 1 ? atoi(argv[1]) : 50;          // MB per launch (the FFN gate/up is 50.8)
    const size_t bytes = mb << 20;
    const int nbuf = 8;
    std::vector<unsigned char*> bufs(nbuf);
    for (auto& b : bufs) {
        CK(hipMalloc(&b, bytes + (1 << 20)));
        CK(hipMemset(b, 1, bytes + (1 << 20)));
    }
    unsigned* out;
    CK(hipMalloc(&out, 4096 * 4));
    struct Cfg { int nw, d, w; Fn fn; };
    std::vector<Cfg> cfgs = {
        {8, 2, 0, pick<2, 0>()}, {8, 4, 0, pick<4, 0>()}, {8, 8, 0, pick<8, 0>()},
        {16, 2, 0, pick<2, 0>()}, {16, 4, 0, pick<4, 0>()}, {4, 8, 0, pick<8, 0>()},
        {8, 4, 1, pick<4, 1>()}, {8, 8, 1, pick<8, 1>()}, {16, 2, 1, pick<2, 1>()}, {16, 4, 1, pick<4, 1>()},
    };
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int grid : {256, 512}) {
        const size_t per = bytes / grid / 1024 * 1024;
        for (auto& c : cfgs) {
            for (int i = 0; i < 16; ++i)
                hipLaunchKernelGGL(c.fn, dim3(grid), dim3(c.nw * 64), 0, nullptr, bufs[i % nbuf], per, out);
            CK(hipDeviceSynchronize());
            const int reps = 64;
            std::vector<float> ts;
            for (int i = 0; i < reps; ++i) {
                CK(hipEventRecord(a, nullptr));
                hipLaunchKernelGGL(c.fn, dim3(grid), dim3(c.nw * 64), 0, nullptr, bufs[i % nbuf], per, out);
                CK(hipEventRecord(b, nullptr));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                ts.push_back(ms * 1000.f);
            }
            // back-to-back (graph-like) rate: 64 launches, one pair of events
            CK(hipEventRecord(a, nullptr));
            for (int i = 0; i < reps; ++i)
                hipLaunchKernelGGL(c.fn, dim3(grid), dim3(c.nw * 64), 0, nullptr, bufs[i % nbuf], per, out);
            CK(hipEventRecord(b, nullptr));
            CK(hipEventSynchronize(b));
            float msb;
            CK(hipEventElapsedTime(&msb, a, b));
            std::sort(ts.begin(), ts.end());
            const double med = ts[ts.size() / 2];
            const double btb = msb * 1000.0 / reps;
            printf("grid %3d nw %2d D %d work %d: single %7.2f us (%5.2f TB/s)  back-to-back %7.2f us (%5.2f TB/s)\n",
                   grid, c.nw, c.d, c.w, med, (double)per * grid / med / 1e6, btb, (double)per * grid / btb / 1e6);
        }
    }
    return 0;
}
