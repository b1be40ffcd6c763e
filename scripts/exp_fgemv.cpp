// Decode-GEMV design experiment (diagnostic, not product).  Question: a batch-1 GEMV whose
// waves issue ALL their weight loads at entry (one unit per wave, many workgroups: the streaming
// floor of exp_gemv2) needs its activation already quantised.  What does a 7B Q4_K_M step cost
// when that quantised activation is produced
//   sep    by a separate one-workgroup quant kernel between producer and consumer,
//   ticket by the producer's last-arriving workgroup (arrival counters, write-through stores),
//   pro    by every consumer workgroup itself (RMSNorm + Q8_K per workgroup),
// against the bare streaming floor (no activation at all)?
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I../include -o exp_fgemv exp_fgemv.cpp
#include "../blama_amd/csrc/qdot.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

using namespace mi;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

// ---- activation layout in global memory and LDS: q8 [nb][256] | bsum [nb][16] int | d [nb] (16-B padded)
__host__ __device__ inline int act_bytes(int nb) { return nb * 256 + nb * 64 + ((nb * 4 + 15) & ~15); }

struct FA {
    const uint8_t* A[4];
    const uint8_t* B[4];
    int rows, nb, units;
    float* out;
    const char* act;          // MODE 0: quantised activation
    const float* x;           // MODE 1: x and the norm weight
    const float* nw;
    // ticket epilogues
    unsigned* cnt;            // TK 1: [nblk_out] per-block counters; TK 2: [8] group + [1] top
    char* act_out;            // the next launch's activation
    const float* nw_next;     // TK 2: the norm weight of the next activation
    double* part;             // TK 2: per-workgroup sum of squares
    const float* resid;       // TK 2: residual (x_in); out = y + resid
};

__device__ __forceinline__ void wait_vm_asm0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ __forceinline__ unsigned fold(const Kq<T_Q4_K>::Ld& l) { return l.qs.x ^ l.qs.y ^ l.qs.z ^ l.qs.w ^ l.hdr.x ^ l.hdr.y ^ l.hdr.z ^ l.hdr.w; }
__device__ __forceinline__ unsigned fold(const Kq<T_Q6_K>::Ld& l) {
    return l.ql.x ^ l.ql.y ^ l.ql.z ^ l.ql.w ^ l.qh.x ^ l.qh.y ^ l.qh.z ^ l.qh.w ^ l.sc0 ^ l.sc1 ^ l.d;
}
template <int T> constexpr int nloads() { return T == T_Q4_K ? 2 : T == T_Q5_K ? 3 : T == T_Q6_K ? 4 : 3; }

// Q8_K of the activation held as 4 floats per lane, one 256-block per wave, into `dst` (global
// or LDS layout act_bytes)
__device__ __forceinline__ void q8k_to(char* dst, int nb, int blk, const float v[4], int lane) {
    quant_q8k_block(v, lane, reinterpret_cast<int8_t*>(dst + blk * 256), reinterpret_cast<int*>(dst + nb * 256) + blk * 16,
                    reinterpret_cast<float*>(dst + nb * 256 + nb * 64) + blk);
}

// MODE 0: quantised activation from global; MODE 1: RMSNorm + Q8_K per workgroup; MODE 9: floor (no activation)
// TK 0: plain store; TK 1: SwiGLU pair + per-256-block ticket quantising h into act_out;
// TK 2: residual add + global two-level ticket: RMSNorm(out) * nw_next -> act_out
template <int T, int NW, int RW, int C, int MODE, int TK>
__global__ __launch_bounds__(NW * 64) void fgemv(FA a) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    using K = Kq<T>;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int sbl = lane >> 3, j = lane & 7;
    const int nb = a.nb;
    const int u = blockIdx.x * NW + wave;
    const bool uv = u < a.units;
    const int uc = uv ? u : a.units - 1;
    constexpr bool PAIR = TK == 1 || TK == 3;
    // ---- activation requests first (they retire before the weights: vmcnt is in order)
    const int abytes = act_bytes(nb);
    f32x4 xv[2], wv[2];
    if (MODE == 0) {
        for (int o = threadIdx.x * 16; o < abytes; o += NW * 64 * 16)
            __builtin_amdgcn_global_load_lds(gptr(reinterpret_cast<const int*>(a.act + o)),
                                             (__attribute__((address_space(3))) void*)(lds + o), 16, 0, 0);
    } else if (MODE == 1) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int blk = wave + i * NW;
            if (blk < nb) {
                xv[i] = gptr(reinterpret_cast<const f32x4*>(a.x))[blk * 64 + lane];
                wv[i] = gptr(reinterpret_cast<const f32x4*>(a.nw))[blk * 64 + lane];
            }
        }
    }
    asm volatile("" ::: "memory");
    // ---- every weight load of the wave
    typename K::Ld w[RW][C];
    const uint8_t* rp[RW][4];
#pragma unroll
    for (int r = 0; r < RW; ++r) {
        const long long row = PAIR ? uc : (long long)uc * RW + r;
        const long long rr = row < a.rows ? row : a.rows - 1;
#pragma unroll
        for (int p = 0; p < 4; ++p)
            rp[r][p] = rfl_ptr(((PAIR && r == 1) ? a.B[p] : a.A[p]) + rr * nb * PlaneBytes<T>::b[p]);
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const int sb = 8 * c + sbl;
            w[r][c] = K::bload(rp[r], sb < nb ? sb : nb - 1, j, !uv || sb >= nb);
        }
    }
    if (MODE == 9) {
        unsigned f = 0;
#pragma unroll
        for (int r = 0; r < RW; ++r)
#pragma unroll
            for (int c = 0; c < C; ++c) f ^= fold(w[r][c]);
        if (f == 0x9e3779b9u) a.out[u] = (float)f;
        return;
    }
    if (MODE == 0) {
        // the activation landed (it was issued before the RW*C*nl weight loads)
        __builtin_amdgcn_s_waitcnt((((RW * C * nloads<T>()) & 15)) | (((RW * C * nloads<T>()) >> 4) << 14) | (0x7 << 4) | (0xF << 8));
        __builtin_amdgcn_s_barrier();
    } else {
        double* red = reinterpret_cast<double*>(lds + abytes);
        double s = 0.0;
#pragma unroll
        for (int i = 0; i < 2; ++i)
            if (wave + i * NW < nb) {
                s += (double)(xv[i].x * xv[i].x); s += (double)(xv[i].y * xv[i].y);
                s += (double)(xv[i].z * xv[i].z); s += (double)(xv[i].w * xv[i].w);
            }
        s = wave_sum63_d(s);
        if (lane == 63) red[wave] = s;
        __syncthreads();
        double tot = 0.0;
        for (int k = 0; k < NW; ++k) tot += red[k];
        const float scale = 1.0f / sqrtf((float)(tot / (double)(nb * 256)) + 1e-5f);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int blk = wave + i * NW;
            if (blk < nb) {
                float v[4] = {(xv[i].x * scale) * wv[i].x, (xv[i].y * scale) * wv[i].y, (xv[i].z * scale) * wv[i].z,
                              (xv[i].w * scale) * wv[i].w};
                q8k_to(lds, nb, blk, v, lane);
            }
        }
        __syncthreads();
    }
    // ---- dots
    Act av;
    av.q8k = reinterpret_cast<const int8_t*>(lds);
    av.bsum = reinterpret_cast<const int*>(lds + nb * 256);
    av.dk = reinterpret_cast<const float*>(lds + nb * 256 + nb * 64);
    float y[RW];
#pragma unroll
    for (int r = 0; r < RW; ++r) {
        float acc = 0.0f;
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const int sb0 = 8 * c + sbl;
            const int sb = sb0 < nb ? sb0 : nb - 1;
            const float p = K::dot(w[r][c], K::act(av, sb, j), j);
            acc += sb0 < nb ? p : 0.0f;
        }
        y[r] = wave_sum63(acc);
    }
    if (TK == 3) {
        if (lane == 63 && uv) a.out[u] = silu_f(y[0]) * y[1];
        return;
    }
    if (TK == 0) {
        if (lane == 63 && uv)
#pragma unroll
            for (int r = 0; r < RW; ++r) a.out[(long long)u * RW + r] = y[r];
        return;
    }
    if (TK == 1) {
        // h[u] = silu(gate) * up, write-through; the 256-block of u completes when its 256/NW workgroups arrived
        if (lane == 63 && uv) st_sc1(a.out + u, silu_f(y[0]) * y[1]);
        wait_vm_asm0();
        __syncthreads();
        int* flag = reinterpret_cast<int*>(lds + abytes);
        const int blk = (blockIdx.x * NW) >> 8;
        if (threadIdx.x == 0) {
            const unsigned need = 256 / NW;
            const unsigned old = __hip_atomic_fetch_add(a.cnt + blk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            flag[0] = old == need - 1 ? 1 : 0;
        }
        __syncthreads();
        if (flag[0] && wave == 0) {
            float v[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) v[k] = ld_sc1(a.out + blk * 256 + lane * 4 + k);
            q8k_to(a.act_out, a.units >> 8, blk, v, lane);
            if (lane == 0) __hip_atomic_store(a.cnt + blk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        return;
    }
    // TK 2: out[row] = y + resid[row] (write-through), the workgroup's sum of squares, two-level ticket
    double* red = reinterpret_cast<double*>(lds + abytes);
    int* flag = reinterpret_cast<int*>(lds + abytes + 8 * NW);
    {
        const long long row = (long long)u;
        float o = 0.0f;
        if (uv) o = y[0] + a.resid[row];
        if (lane == 63) {
            if (uv) st_sc1(a.out + row, o);
            red[wave] = uv ? (double)(o * o) : 0.0;
        }
    }
    wait_vm_asm0();
    __syncthreads();
    if (threadIdx.x == 0) {
        double s = 0.0;
        for (int k = 0; k < NW; ++k) s += red[k];
        __hip_atomic_store(a.part + blockIdx.x, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        wait_vm_asm0();
        const int g = blockIdx.x & 7;
        const unsigned ng = (gridDim.x - g + 7) / 8;
        const unsigned old = __hip_atomic_fetch_add(a.cnt + g * 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int last = 0;
        if (old == ng - 1) {
            const unsigned o2 = __hip_atomic_fetch_add(a.cnt + 8 * 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            last = o2 == 7 ? 1 : 0;
            __hip_atomic_store(a.cnt + g * 32, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        flag[0] = last;
    }
    __syncthreads();
    if (!flag[0]) return;
    // the last workgroup: sum the partials in workgroup order, RMSNorm, Q8_K of every block
    if (wave == 0) {
        double s = 0.0;
        for (int i = lane; i < (int)gridDim.x; i += 64) s += __hip_atomic_load(a.part + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s = wave_sum63_d(s);
        if (lane == 63) red[0] = s;
        if (lane == 0) __hip_atomic_store(a.cnt + 8 * 32, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    const float scale = 1.0f / sqrtf((float)(red[0] / (double)a.rows) + 1e-5f);
    const int nbo = a.rows >> 8;
    for (int blk = wave; blk < nbo; blk += NW) {
        float v[4];
        const f32x4 wn = gptr(reinterpret_cast<const f32x4*>(a.nw_next))[blk * 64 + lane];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = ld_sc1(a.out + blk * 256 + lane * 4 + k) * scale;
        v[0] *= wn.x; v[1] *= wn.y; v[2] *= wn.z; v[3] *= wn.w;
        q8k_to(a.act_out, nbo, blk, v, lane);
    }
}

// RMSNorm (NORM 1) or plain Q8_K of x[K] -> act, one workgroup of 16 waves
template <int NORM>
__global__ __launch_bounds__(1024) void quant_kernel(const float* x, const float* nw, int K, char* act) {
    __shared__ double red[16];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int nb = K >> 8;
    f32x4 xv[4], wv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int blk = wave + 16 * i;
        if (blk < nb) {
            xv[i] = gptr(reinterpret_cast<const f32x4*>(x))[blk * 64 + lane];
            if (NORM) wv[i] = gptr(reinterpret_cast<const f32x4*>(nw))[blk * 64 + lane];
        }
    }
    float scale = 1.0f;
    if (NORM) {
        double s = 0.0;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (wave + 16 * i < nb) {
                s += (double)(xv[i].x * xv[i].x); s += (double)(xv[i].y * xv[i].y);
                s += (double)(xv[i].z * xv[i].z); s += (double)(xv[i].w * xv[i].w);
            }
        s = wave_sum63_d(s);
        if (lane == 63) red[wave] = s;
        __syncthreads();
        double t = 0.0;
        for (int k = 0; k < 16; ++k) t += red[k];
        scale = 1.0f / sqrtf((float)(t / (double)K) + 1e-5f);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int blk = wave + 16 * i;
        if (blk < nb) {
            float v[4] = {xv[i].x, xv[i].y, xv[i].z, xv[i].w};
            if (NORM) { v[0] = (v[0] * scale) * wv[i].x; v[1] = (v[1] * scale) * wv[i].y; v[2] = (v[2] * scale) * wv[i].z; v[3] = (v[3] * scale) * wv[i].w; }
            q8k_to(act, nb, blk, v, lane);
        }
    }
}

// Infinity-Cache prefetch of byte ranges (a side stream): default-policy 16-B loads, folded
struct PfRanges {
    const uint8_t* p[8];
    long long n[8];   // bytes (multiple of 16)
    int cnt;
};
__global__ __launch_bounds__(256) void mall_prefetch(PfRanges r) {
    unsigned f = 0;
    for (int k = 0; k < r.cnt; ++k) {
        const u32x4* p = reinterpret_cast<const u32x4*>(r.p[k]);
        const long long n16 = r.n[k] / 16;
        for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n16; i += (long long)gridDim.x * 256 * 4) {
            u32x4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const long long ii = i + (long long)u * gridDim.x * 256;
                v[u] = ii < n16 ? *gptr(p + ii) : u32x4{0u, 0u, 0u, 0u};
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) f ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
        }
    }
    if (f == 0x9e3779b9u) reinterpret_cast<unsigned*>(const_cast<uint8_t*>(r.p[0]))[0] = f;
}

// ---------------------------------------------------------------------------------------------
struct Mat {
    int type, rows, nb;
    uint8_t* p[4];
    size_t bytes;
};
static Mat make_mat(int type, int rows, int K) {
    Mat m{type, rows, K / 256, {nullptr, nullptr, nullptr, nullptr}, 0};
    const int pb4[4] = {128, 16, 0, 0}, pb6[4] = {128, 64, 16, 2};
    const int* pb = type == T_Q4_K ? pb4 : pb6;
    size_t off[4], tot = 0;
    for (int p = 0; p < 4; ++p) {
        off[p] = tot;
        tot += ((size_t)rows * m.nb * pb[p] + 4096 + 255) & ~(size_t)255;
    }
    uint8_t* base;
    CK(hipMalloc(&base, tot));
    std::vector<uint8_t> h(tot);
    uint32_t s = 12345u + rows * 7 + K;
    for (size_t i = 0; i < tot; ++i) { s = s * 1664525u + 1013904223u; h[i] = (uint8_t)(s >> 24); }
    auto f16 = [](float f) { __half x = __float2half(f); return *reinterpret_cast<uint16_t*>(&x); };
    if (type == T_Q4_K) {
        for (size_t r = 0; r < (size_t)rows * m.nb; ++r) {
            uint16_t* hd = reinterpret_cast<uint16_t*>(&h[off[1] + r * 16]);
            hd[0] = f16(1e-3f); hd[1] = f16(5e-4f);
        }
    } else {
        for (size_t r = 0; r < (size_t)rows * m.nb; ++r) *reinterpret_cast<uint16_t*>(&h[off[3] + r * 2]) = f16(1e-3f);
    }
    CK(hipMemcpy(base, h.data(), tot, hipMemcpyHostToDevice));
    for (int p = 0; p < 4; ++p) m.p[p] = base + off[p];
    m.bytes = (size_t)rows * m.nb * (type == T_Q4_K ? 144 : 210);
    return m;
}

typedef void (*KFn)(FA);
struct Launch {
    int kind;          // 0 gemv, 1 quant norm, 2 quant plain, 3 prefetch fork (side stream), 4 join
    PfRanges pf;
    int pf_grid;
    KFn fn;
    int nw, grid, smem;
    FA a;
    const float* qx; const float* qnw; int qK; char* qact;
    size_t bytes;
};
static hipStream_t g_side = nullptr;
static std::vector<hipEvent_t> g_evs;
static size_t g_ev_i = 0;
static hipEvent_t next_ev() {
    if (g_ev_i == g_evs.size()) {
        hipEvent_t ev;
        CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        g_evs.push_back(ev);
    }
    return g_evs[g_ev_i++];
}
static void run(const Launch& L, hipStream_t s) {
    if (L.kind == 3) {   // fork: the side stream waits for the main stream's progress, then prefetches
        hipEvent_t ev = next_ev();
        CK(hipEventRecord(ev, s));
        CK(hipStreamWaitEvent(g_side, ev, 0));
        hipLaunchKernelGGL(mall_prefetch, dim3(L.pf_grid), dim3(256), 0, g_side, L.pf);
        return;
    }
    if (L.kind == 4) {   // join
        hipEvent_t ev = next_ev();
        CK(hipEventRecord(ev, g_side));
        CK(hipStreamWaitEvent(s, ev, 0));
        return;
    }
    if (L.kind == 0) hipLaunchKernelGGL(L.fn, dim3(L.grid), dim3(L.nw * 64), L.smem, s, L.a);
    else if (L.kind == 1) hipLaunchKernelGGL(quant_kernel<1>, dim3(1), dim3(1024), 0, s, L.qx, L.qnw, L.qK, L.qact);
    else hipLaunchKernelGGL(quant_kernel<0>, dim3(1), dim3(1024), 0, s, L.qx, L.qnw, L.qK, L.qact);
}
static Launch mk_quant(int norm, const float* x, const float* nw, int K, char* act) {
    Launch L{};
    L.kind = norm ? 1 : 2;
    L.qx = x; L.qnw = nw; L.qK = K; L.qact = act;
    return L;
}

template <int T, int NW, int RW, int C, int MODE, int TK>
static Launch mk(const Mat& A, const Mat* B, FA base) {
    Launch L{};
    L.kind = 0;
    L.fn = fgemv<T, NW, RW, C, MODE, TK>;
    L.nw = NW;
    FA& a = L.a;
    a = base;
    for (int p = 0; p < 4; ++p) { a.A[p] = A.p[p]; a.B[p] = B ? B->p[p] : A.p[p]; }
    a.rows = A.rows; a.nb = A.nb;
    a.units = (TK == 1 || TK == 3) ? A.rows : (A.rows + RW - 1) / RW;
    L.grid = (a.units + NW - 1) / NW;
    L.smem = act_bytes(A.nb) + 8 * NW + 64;
    L.bytes = A.bytes + (B ? B->bytes : 0);
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(L.fn), hipFuncAttributeMaxDynamicSharedMemorySize, 65536));
    return L;
}

static void time_kind(const char* name, std::vector<Launch> Ls, hipStream_t s) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int i = 0; i < 8; ++i) run(Ls[i % Ls.size()], s);
    CK(hipStreamSynchronize(s));
    hipGraph_t g; hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int i = 0; i < 64; ++i) run(Ls[i % Ls.size()], s);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(e0, s));
    for (int r = 0; r < 4; ++r) CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    const double btb = ms * 1e3 / 256.0;
    printf("%-40s grid %5d  graph %7.2f us (%4.2f TB/s)\n", name, Ls[0].grid, btb, Ls[0].bytes / btb / 1e6);
    fflush(stdout);
    CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g));
}

int main(int argc, char** argv) {
    const int what = argc > 1 ? atoi(argv[1]) : 3;
    hipStream_t s;
    CK(hipStreamCreate(&s));
    float *x, *x2, *nw, *h, *out;
    char *actA, *actB, *actC, *actD;
    unsigned* cnt;
    double* part;
    CK(hipMalloc(&x, 65536 * 4)); CK(hipMalloc(&x2, 65536 * 4)); CK(hipMalloc(&nw, 65536 * 4));
    CK(hipMalloc(&h, 65536 * 4)); CK(hipMalloc(&out, 65536 * 4));
    for (char** p : {&actA, &actB, &actC, &actD}) CK(hipMalloc(p, 65536));
    CK(hipMalloc(&cnt, 4096 * 4)); CK(hipMemset(cnt, 0, 4096 * 4));
    CK(hipMalloc(&part, 8192 * 8));
    {
        std::vector<float> hx(65536), hw(65536, 1.0f);
        for (int i = 0; i < 65536; ++i) hx[i] = 0.01f * (float)((i * 37) % 101 - 50);
        CK(hipMemcpy(x, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(x2, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(nw, hw.data(), hw.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(h, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
    }
    hipLaunchKernelGGL(quant_kernel<1>, dim3(1), dim3(1024), 0, s, x, nw, 4096, actA);
    hipLaunchKernelGGL(quant_kernel<1>, dim3(1), dim3(1024), 0, s, x, nw, 4096, actB);
    hipLaunchKernelGGL(quant_kernel<1>, dim3(1), dim3(1024), 0, s, x, nw, 4096, actC);
    hipLaunchKernelGGL(quant_kernel<0>, dim3(1), dim3(1024), 0, s, h, nw, 11008, actD);
    CK(hipStreamSynchronize(s));
    FA b{};
    b.out = out; b.x = x; b.nw = nw; b.cnt = cnt; b.part = part; b.nw_next = nw; b.resid = x2;
    const int nrot = 6;
    if (what & 1) {
        std::vector<Mat> wo, gate, up, down4, down6, qkv;
        for (int i = 0; i < nrot; ++i) {
            wo.push_back(make_mat(T_Q4_K, 4096, 4096));
            gate.push_back(make_mat(T_Q4_K, 11008, 4096));
            up.push_back(make_mat(T_Q4_K, 11008, 4096));
            down4.push_back(make_mat(T_Q4_K, 4096, 11008));
            down6.push_back(make_mat(T_Q6_K, 4096, 11008));
            qkv.push_back(make_mat(T_Q4_K, 12288, 4096));
        }
        auto many = [&](auto f) { std::vector<Launch> v; for (int i = 0; i < nrot; ++i) v.push_back(f(i)); return v; };
#define KIND(name, expr) time_kind(name, many([&](int i) { return expr; }), s)
        FA bA = b; bA.act = actA;
        FA bD = b; bD.act = actD;
        FA bT1 = b; bT1.act = actA; bT1.out = h; bT1.act_out = actD;
        FA bT2 = b; bT2.act = actD; bT2.out = x2; bT2.act_out = actA; bT2.resid = x;
        KIND("floor  WO q4k nw8", (mk<T_Q4_K, 8, 1, 2, 9, 0>(wo[i], nullptr, bA)));
        KIND("act    WO q4k nw8", (mk<T_Q4_K, 8, 1, 2, 0, 0>(wo[i], nullptr, bA)));
        KIND("act    WO q4k nw4", (mk<T_Q4_K, 4, 1, 2, 0, 0>(wo[i], nullptr, bA)));
        KIND("act    WO q4k nw16", (mk<T_Q4_K, 16, 1, 2, 0, 0>(wo[i], nullptr, bA)));
        KIND("rms    WO q4k nw8", (mk<T_Q4_K, 8, 1, 2, 1, 0>(wo[i], nullptr, bA)));
        KIND("floor  QKV q4k nw8 rw2", (mk<T_Q4_K, 8, 2, 2, 9, 0>(qkv[i], nullptr, bA)));
        KIND("act    QKV q4k nw8 rw2", (mk<T_Q4_K, 8, 2, 2, 0, 0>(qkv[i], nullptr, bA)));
        KIND("rms    QKV q4k nw8 rw2", (mk<T_Q4_K, 8, 2, 2, 1, 0>(qkv[i], nullptr, bA)));
        KIND("floor  UP q4k nw8 pair", (mk<T_Q4_K, 8, 2, 2, 9, 1>(gate[i], &up[i], bT1)));
        KIND("act    UP q4k nw8 pair ticket", (mk<T_Q4_K, 8, 2, 2, 0, 1>(gate[i], &up[i], bT1)));
        KIND("act    UP q4k nw4 pair ticket", (mk<T_Q4_K, 4, 2, 2, 0, 1>(gate[i], &up[i], bT1)));
        KIND("rms    UP q4k nw8 pair ticket", (mk<T_Q4_K, 8, 2, 2, 1, 1>(gate[i], &up[i], bT1)));
        KIND("floor  DOWN q4k nw8", (mk<T_Q4_K, 8, 1, 6, 9, 0>(down4[i], nullptr, bD)));
        KIND("act    DOWN q4k nw8", (mk<T_Q4_K, 8, 1, 6, 0, 0>(down4[i], nullptr, bD)));
        KIND("act    DOWN q4k nw8 ticket", (mk<T_Q4_K, 8, 1, 6, 0, 2>(down4[i], nullptr, bT2)));
        KIND("floor  DOWN q6k nw8", (mk<T_Q6_K, 8, 1, 6, 9, 0>(down6[i], nullptr, bD)));
        KIND("act    DOWN q6k nw8", (mk<T_Q6_K, 8, 1, 6, 0, 0>(down6[i], nullptr, bD)));
        KIND("act    DOWN q6k nw8 ticket", (mk<T_Q6_K, 8, 1, 6, 0, 2>(down6[i], nullptr, bT2)));
        KIND("quant  norm 4096", (mk_quant(1, x, nw, 4096, actB)));
        KIND("quant  plain 11008", (mk_quant(0, h, nw, 11008, actD)));
#undef KIND
    }
    if (what & 2) {
        // a 7B Q4_K_M-like step: 32 layers x {QKV, [attention out quant], WO, gate/up, down} + the head
        const int L = 32;
        std::vector<Launch> floor_, sep, tick, pro, sep3;
        std::vector<PfRanges> lay;
        size_t bytes = 0;
        FA bq = b; bq.act = actA;                           // QKV reads act A
        FA bw = b; bw.act = actB;                           // WO reads act B (attention output)
        FA bg = b; bg.act = actC; bg.out = h;               // gate/up reads act C -> h
        FA bd = b; bd.act = actD;                           // down reads act D (h)
        for (int l = 0; l < L; ++l) {
            const bool more = l < L / 8 || l >= 7 * L / 8 || (l - L / 8) % 3 == 2;
            Mat qkv = make_mat(T_Q4_K, 12288, 4096), wo = make_mat(T_Q4_K, 4096, 4096);
            Mat g = make_mat(T_Q4_K, 11008, 4096), u = make_mat(T_Q4_K, 11008, 4096);
            Mat d = make_mat(more ? T_Q6_K : T_Q4_K, 4096, 11008);
            bytes += qkv.bytes + wo.bytes + g.bytes + u.bytes + d.bytes;
            {
                PfRanges r{};
                const Mat* ms[5] = {&qkv, &wo, &g, &u, &d};
                const int pb4[4] = {128, 16, 0, 0}, pb6[4] = {128, 64, 16, 2};
                for (const Mat* m : ms) {   // the planes of each matrix are one allocation from p[0]
                    const int* pb = m->type == T_Q4_K ? pb4 : pb6;
                    long long tot = 0;
                    for (int q = 0; q < 4; ++q) tot += ((long long)m->rows * m->nb * pb[q] + 4096 + 255) & ~255LL;
                    r.p[r.cnt] = m->p[0];
                    r.n[r.cnt++] = tot & ~15LL;
                }
                lay.push_back(r);
            }
            floor_.push_back(mk<T_Q4_K, 8, 2, 2, 9, 0>(qkv, nullptr, bq));
            floor_.push_back(mk<T_Q4_K, 8, 1, 2, 9, 0>(wo, nullptr, bw));
            floor_.push_back(mk<T_Q4_K, 8, 2, 2, 9, 1>(g, &u, bg));
            if (more) floor_.push_back(mk<T_Q6_K, 8, 1, 6, 9, 0>(d, nullptr, bd));
            else floor_.push_back(mk<T_Q4_K, 8, 1, 6, 9, 0>(d, nullptr, bd));
            // sep: every activation by a one-workgroup quant kernel
            FA bw2 = bw; bw2.out = x2;
            FA bd2 = bd; bd2.out = x;
            FA bgs = bg; bgs.act_out = actD;
            sep.push_back(mk<T_Q4_K, 8, 2, 2, 0, 0>(qkv, nullptr, bq));
            sep.push_back(mk_quant(0, out, nw, 4096, actB));   // attention output
            sep.push_back(mk<T_Q4_K, 8, 1, 2, 0, 0>(wo, nullptr, bw2));
            sep.push_back(mk_quant(1, x2, nw, 4096, actC));
            sep.push_back(mk<T_Q4_K, 8, 2, 2, 0, 3>(g, &u, bgs));
            sep.push_back(mk_quant(0, h, nw, 11008, actD));
            if (more) sep.push_back(mk<T_Q6_K, 8, 1, 6, 0, 0>(d, nullptr, bd2));
            else sep.push_back(mk<T_Q4_K, 8, 1, 6, 0, 0>(d, nullptr, bd2));
            sep.push_back(mk_quant(1, x, nw, 4096, actA));
            // sep3: sep with the attention output quantised by the attention kernel itself
            sep3.push_back(mk<T_Q4_K, 8, 2, 2, 0, 0>(qkv, nullptr, bq));
            sep3.push_back(mk<T_Q4_K, 8, 1, 2, 0, 0>(wo, nullptr, bw2));
            sep3.push_back(mk_quant(1, x2, nw, 4096, actC));
            sep3.push_back(mk<T_Q4_K, 8, 2, 2, 0, 3>(g, &u, bgs));
            sep3.push_back(mk_quant(0, h, nw, 11008, actD));
            if (more) sep3.push_back(mk<T_Q6_K, 8, 1, 6, 0, 0>(d, nullptr, bd2));
            else sep3.push_back(mk<T_Q4_K, 8, 1, 6, 0, 0>(d, nullptr, bd2));
            sep3.push_back(mk_quant(1, x, nw, 4096, actA));
            // ticket: WO and down publish the next activation themselves (gate/up too, per block)
            FA bwt = bw; bwt.out = x2; bwt.resid = x; bwt.act_out = actC; bwt.cnt = cnt + 1024;
            FA bdt = bd; bdt.out = x; bdt.resid = x2; bdt.act_out = actA; bdt.cnt = cnt + 2048;
            tick.push_back(mk<T_Q4_K, 8, 2, 2, 0, 0>(qkv, nullptr, bq));
            tick.push_back(mk_quant(0, out, nw, 4096, actB));
            tick.push_back(mk<T_Q4_K, 8, 1, 2, 0, 2>(wo, nullptr, bwt));
            tick.push_back(mk<T_Q4_K, 8, 2, 2, 0, 1>(g, &u, bgs));
            if (more) tick.push_back(mk<T_Q6_K, 8, 1, 6, 0, 2>(d, nullptr, bdt));
            else tick.push_back(mk<T_Q4_K, 8, 1, 6, 0, 2>(d, nullptr, bdt));
            // pro: the RMSNorm activations built in every consumer workgroup
            FA bqp = bq; bqp.x = x;
            FA bgp = bgs; bgp.x = x2;
            pro.push_back(mk<T_Q4_K, 8, 2, 2, 1, 0>(qkv, nullptr, bqp));
            pro.push_back(mk_quant(0, out, nw, 4096, actB));
            pro.push_back(mk<T_Q4_K, 8, 1, 2, 0, 0>(wo, nullptr, bw2));
            pro.push_back(mk<T_Q4_K, 8, 2, 2, 1, 1>(g, &u, bgp));
            if (more) pro.push_back(mk<T_Q6_K, 8, 1, 6, 0, 0>(d, nullptr, bd2));
            else pro.push_back(mk<T_Q4_K, 8, 1, 6, 0, 0>(d, nullptr, bd2));
        }
        Mat o = make_mat(T_Q6_K, 32000, 4096);
        bytes += o.bytes;
        FA bo = b; bo.act = actA;
        floor_.push_back(mk<T_Q6_K, 8, 1, 2, 9, 0>(o, nullptr, bo));
        sep.push_back(mk<T_Q6_K, 8, 1, 2, 0, 0>(o, nullptr, bo));
        tick.push_back(mk<T_Q6_K, 8, 1, 2, 0, 0>(o, nullptr, bo));
        pro.push_back(mk<T_Q6_K, 8, 1, 2, 0, 0>(o, nullptr, bo));
        // the same chains with the next layer's weights prefetched into the Infinity Cache on a side
        // stream when a layer starts (every launch of layer l marks its start: kind 3 before it)
        auto with_pf = [&](const std::vector<Launch>& st, int per_layer, int grid) {
            std::vector<Launch> o;
            for (size_t i = 0; i < st.size(); ++i) {
                const int l = (int)(i / per_layer);
                if (i % per_layer == 0 && (size_t)i < (size_t)per_layer * L && l + 1 < L) {
                    Launch f{};
                    f.kind = 3;
                    f.pf = lay[l + 1];
                    f.pf_grid = grid;
                    o.push_back(f);
                }
                o.push_back(st[i]);
            }
            Launch j{};
            j.kind = 4;
            o.push_back(j);
            return o;
        };
        CK(hipStreamCreateWithFlags(&g_side, hipStreamNonBlocking));
        const auto floor_pf = with_pf(floor_, 4, 128);
        const auto sep3_pf64 = with_pf(sep3, 7, 64);
        const auto sep3_pf128 = with_pf(sep3, 7, 128);
        const auto sep3_pf256 = with_pf(sep3, 7, 256);
        const char* names[9] = {"floor", "sep", "ticket", "pro", "sep3", "floor+pf", "sep3+pf64", "sep3+pf128", "sep3+pf256"};
        for (int pass = 0; pass < 9; ++pass) {
            g_ev_i = 0;
            const auto& st = pass == 0 ? floor_ : pass == 1 ? sep : pass == 2 ? tick : pass == 3 ? pro : pass == 4 ? sep3
                           : pass == 5 ? floor_pf : pass == 6 ? sep3_pf64 : pass == 7 ? sep3_pf128 : sep3_pf256;
            hipGraph_t g; hipGraphExec_t ge;
            CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
            for (const auto& Lc : st) run(Lc, s);
            CK(hipStreamEndCapture(s, &g));
            CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
            for (int i = 0; i < 3; ++i) CK(hipGraphLaunch(ge, s));
            CK(hipStreamSynchronize(s));
            hipEvent_t e0, e1;
            CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
            const int reps = 20;
            CK(hipEventRecord(e0, s));
            for (int i = 0; i < reps; ++i) CK(hipGraphLaunch(ge, s));
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1));
            const double per = ms / reps;
            printf("chain %-8s: %zu launches, %.3f GB, %.3f ms/step = %.1f tok/s, %.2f TB/s\n", names[pass], st.size(),
                   bytes / 1e9, per, 1e3 / per, bytes / per / 1e9);
            fflush(stdout);
            CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g));
            if (pass == 2) {
                // the ticket protocol's result against the separate quant kernel's (the last down -> act A)
                std::vector<char> t1(65536), t2(65536);
                CK(hipMemcpy(t1.data(), actA, act_bytes(16), hipMemcpyDeviceToHost));
                hipLaunchKernelGGL(quant_kernel<1>, dim3(1), dim3(1024), 0, s, x, nw, 4096, actA);
                CK(hipStreamSynchronize(s));
                CK(hipMemcpy(t2.data(), actA, act_bytes(16), hipMemcpyDeviceToHost));
                int diff = 0;
                for (int i = 0; i < act_bytes(16); ++i) diff += t1[i] != t2[i];
                printf("ticket act vs quant kernel: %d differing bytes of %d\n", diff, act_bytes(16));
            }
        }
    }
    return 0;
}
