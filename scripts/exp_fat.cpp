// Decode-GEMV design experiment (diagnostic, not product), round 6.  Question: can the batch-1
// step drop its separate activation-quantisation launches (RMSNorm + Q8_K of x before QKV and
// gate/up, Q8_K of h before down) by having every consumer workgroup build the quantised
// activation itself, if the workgroups are FAT (about one per CU, several units per wave: the
// per-workgroup prologue is paid 256 times, not 768-1376 times)?
//   act   : the activation arrives quantised (as the r05 engine), thin or fat workgroups
//   rms   : x + the norm weight; RMSNorm (double sum) + Q8_K per workgroup
//   plain : h; Q8_K per workgroup
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I../include -o exp_fat exp_fat.cpp
#include "../blama_amd/csrc/qdot.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

using namespace mi;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

// activation layout: q8 [nb][256] | bsum [nb][16] int | d [nb] (16-B padded)
__host__ __device__ inline int act_bytes(int nb) { return nb * 256 + nb * 64 + ((nb * 4 + 15) & ~15); }

struct FA {
    const uint8_t* A[4];
    const uint8_t* B[4];
    int rows, nb, units;
    float* out;
    const char* act;          // MODE 0
    const float* x;           // MODE 1 / 2
    const float* nw;          // MODE 1
    const float* resid;       // EPI 2: out = y + resid
};

__device__ __forceinline__ void q8k_to(char* dst, int nb, int blk, const float v[4], int lane) {
    quant_q8k_block(v, lane, reinterpret_cast<int8_t*>(dst + blk * 256), reinterpret_cast<int*>(dst + nb * 256) + blk * 16,
                    reinterpret_cast<float*>(dst + nb * 256 + nb * 64) + blk);
}
template <int T> constexpr int nloads() { return T == T_Q4_K ? 2 : T == T_Q5_K ? 3 : T == T_Q6_K ? 4 : 3; }

// NW waves, UPW units per wave (a workgroup owns units [u0, u1) of unit_range over the grid, wave w
// takes u0 + w + k*NW), C 8-superblock chunks per row, RW rows per unit (PAIR: gate/up pair).
// MODE 0 act / 1 rms / 2 plain.  EPI 0 store, 1 SwiGLU, 2 residual add.
template <int T, int NW, int UPW, int RW, int C, int MODE, int EPI>
__global__ __launch_bounds__(NW * 64) void fat(FA a) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    using K = Kq<T>;
    constexpr bool PAIR = EPI == 1;
    constexpr int ABW = (8 * C + NW - 1) / NW;   // activation blocks per wave (MODE 1/2)
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int sbl = lane >> 3, j = lane & 7;
    const int nb = a.nb;
    int u0, u1;
    unit_range(a.units, gridDim.x, blockIdx.x, u0, u1);
    const int abytes = act_bytes(nb);
    f32x4 xv[ABW], wv[ABW];
    if (MODE == 0) {
        for (int o = threadIdx.x * 16; o < abytes; o += NW * 64 * 16)
            __builtin_amdgcn_global_load_lds(gptr(reinterpret_cast<const int*>(a.act + o)),
                                             (__attribute__((address_space(3))) void*)(lds + o), 16, 0, 0);
    } else {
#pragma unroll
        for (int i = 0; i < ABW; ++i) {
            const int blk = wave + i * NW;
            if (blk < nb) {
                xv[i] = gptr(reinterpret_cast<const f32x4*>(a.x))[blk * 64 + lane];
                if (MODE == 1) wv[i] = gptr(reinterpret_cast<const f32x4*>(a.nw))[blk * 64 + lane];
            }
        }
    }
    float res[UPW];
    if (EPI == 2) {
#pragma unroll
        for (int k = 0; k < UPW; ++k) {
            const int u = u0 + wave + k * NW;
            const uint8_t* rb = reinterpret_cast<const uint8_t*>(rfl_ptr(a.resid));
            res[k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(buf_rsrc(rb), oob((unsigned)u * 4, u >= u1), 0, 0));
        }
    }
    asm volatile("" ::: "memory");
    typename K::Ld w[UPW][RW][C];
#pragma unroll
    for (int k = 0; k < UPW; ++k) {
        const int u = u0 + wave + k * NW;
        const bool uv = u < u1;
        const int uc = uv ? u : u1 - 1;
#pragma unroll
        for (int r = 0; r < RW; ++r) {
            const long long row = PAIR ? uc : (long long)uc * RW + r;
            const long long rr = row < a.rows ? row : a.rows - 1;
            const uint8_t* rp[4];
#pragma unroll
            for (int p = 0; p < 4; ++p) rp[p] = rfl_ptr(((PAIR && r == 1) ? a.B[p] : a.A[p]) + rr * nb * PlaneBytes<T>::b[p]);
#pragma unroll
            for (int c = 0; c < C; ++c) {
                const int sb = 8 * c + sbl;
                w[k][r][c] = K::bload(rp, sb < nb ? sb : nb - 1, j, !uv || sb >= nb);
            }
        }
    }
    if (MODE == 0) {
        constexpr int NL = UPW * RW * C * nloads<T>() + (EPI == 2 ? UPW : 0);
        __builtin_amdgcn_s_waitcnt(((NL & 15)) | (((NL >> 4) & 3) << 14) | (0x7 << 4) | (0xF << 8));
        __builtin_amdgcn_s_barrier();
    } else {
        double* red = reinterpret_cast<double*>(lds + abytes);
        float scale = 1.0f;
        if (MODE == 1) {
            double s = 0.0;
#pragma unroll
            for (int i = 0; i < ABW; ++i)
                if (wave + i * NW < nb) {
                    s += (double)(xv[i].x * xv[i].x); s += (double)(xv[i].y * xv[i].y);
                    s += (double)(xv[i].z * xv[i].z); s += (double)(xv[i].w * xv[i].w);
                }
            s = wave_sum63_d(s);
            if (lane == 63) red[wave] = s;
            __syncthreads();
            double tot = 0.0;
#pragma unroll
            for (int k = 0; k < NW; ++k) tot += red[k];
            scale = 1.0f / sqrtf((float)(tot / (double)(nb * 256)) + 1e-5f);
        }
#pragma unroll
        for (int i = 0; i < ABW; ++i) {
            const int blk = wave + i * NW;
            if (blk < nb) {
                float v[4] = {xv[i].x, xv[i].y, xv[i].z, xv[i].w};
                if (MODE == 1) {
                    v[0] = (v[0] * scale) * wv[i].x; v[1] = (v[1] * scale) * wv[i].y;
                    v[2] = (v[2] * scale) * wv[i].z; v[3] = (v[3] * scale) * wv[i].w;
                }
                q8k_to(lds, nb, blk, v, lane);
            }
        }
        __syncthreads();
    }
    Act av;
    av.q8k = reinterpret_cast<const int8_t*>(lds);
    av.bsum = reinterpret_cast<const int*>(lds + nb * 256);
    av.dk = reinterpret_cast<const float*>(lds + nb * 256 + nb * 64);
#pragma unroll
    for (int k = 0; k < UPW; ++k) {
        const int u = u0 + wave + k * NW;
        float y[RW];
#pragma unroll
        for (int r = 0; r < RW; ++r) {
            float acc = 0.0f;
#pragma unroll
            for (int c = 0; c < C; ++c) {
                const int sb0 = 8 * c + sbl;
                const int sb = sb0 < nb ? sb0 : nb - 1;
                const float p = K::dot(w[k][r][c], K::act(av, sb, j), j);
                acc += sb0 < nb ? p : 0.0f;
            }
            y[r] = wave_sum63(acc);
        }
        if (lane == 63 && u < u1) {
            if (EPI == 1) a.out[u] = silu_f(y[0]) * y[1];
            else if (EPI == 2) a.out[u] = y[0] + res[k];
            else
#pragma unroll
                for (int r = 0; r < RW; ++r) a.out[(long long)u * RW + r] = y[r];
        }
    }
}

// RMSNorm (NORM 1) or plain Q8_K of x[K] -> act: one workgroup per 256-block (the engine's dv_quant)
template <int NORM>
__global__ __launch_bounds__(256) void quant_kernel(const float* x, const float* nw, int K, char* act) {
    __shared__ double red[4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int b = blockIdx.x, nb = K >> 8;
    const f32x4 v = gptr(reinterpret_cast<const f32x4*>(x))[b * 64 + lane];
    float scale = 1.0f;
    f32x4 wn = {1.0f, 1.0f, 1.0f, 1.0f};
    if (NORM) {
        wn = gptr(reinterpret_cast<const f32x4*>(nw))[b * 64 + lane];
        double sq = 0.0;
        const int n4 = K >> 2;
        for (int i0 = tid; i0 < n4; i0 += 8 * 256) {
            f32x4 y[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) if (i0 + k * 256 < n4) y[k] = gptr(reinterpret_cast<const f32x4*>(x))[i0 + k * 256];
#pragma unroll
            for (int k = 0; k < 8; ++k)
                if (i0 + k * 256 < n4) {
                    sq += (double)(y[k].x * y[k].x); sq += (double)(y[k].y * y[k].y);
                    sq += (double)(y[k].z * y[k].z); sq += (double)(y[k].w * y[k].w);
                }
        }
        sq = wave_sum63_d(sq);
        if (lane == 63) red[wave] = sq;
        __syncthreads();
        double tot = 0.0;
        for (int k = 0; k < 4; ++k) tot += red[k];
        scale = 1.0f / sqrtf((float)(tot / (double)K) + 1e-5f);
    }
    if (wave != 0) return;
    float q[4] = {v.x, v.y, v.z, v.w};
    if (NORM) { q[0] = (q[0] * scale) * wn.x; q[1] = (q[1] * scale) * wn.y; q[2] = (q[2] * scale) * wn.z; q[3] = (q[3] * scale) * wn.w; }
    q8k_to(act, nb, b, q, lane);
}

// The quant kernel with extra workgroups that prefetch a consumer GEMV's weights into the L2 of
// the XCD each consumer workgroup will run on (workgroup b -> XCD b % 8, round-robin placement).
// Workgroups [0, nqp) quantise (nqp = the block count rounded up to 8), the rest prefetch.
struct PF {
    const uint8_t* p[8];
    int pb[8];            // bytes per row of each plane
    int np;
    int rows, rows_per_wg, cons_wgs;   // consumer: rows, rows per workgroup, grid
    int max_wgs;          // prefetch consumer workgroups b < max_wgs only
};
template <int NORM>
__global__ __launch_bounds__(256) void qpf_kernel(const float* x, const float* nw, int K, char* act, int nqp, PF pf) {
    __shared__ double red[4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nb = K >> 8;
    if ((int)blockIdx.x < nqp) {
        const int b = blockIdx.x;
        if (b >= nb) return;
        const f32x4 v = gptr(reinterpret_cast<const f32x4*>(x))[b * 64 + lane];
        float scale = 1.0f;
        f32x4 wn = {1.0f, 1.0f, 1.0f, 1.0f};
        if (NORM) {
            wn = gptr(reinterpret_cast<const f32x4*>(nw))[b * 64 + lane];
            double sq = 0.0;
            const int n4 = K >> 2;
            for (int i0 = tid; i0 < n4; i0 += 8 * 256) {
                f32x4 y[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) if (i0 + k * 256 < n4) y[k] = gptr(reinterpret_cast<const f32x4*>(x))[i0 + k * 256];
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    if (i0 + k * 256 < n4) {
                        sq += (double)(y[k].x * y[k].x); sq += (double)(y[k].y * y[k].y);
                        sq += (double)(y[k].z * y[k].z); sq += (double)(y[k].w * y[k].w);
                    }
            }
            sq = wave_sum63_d(sq);
            if (lane == 63) red[wave] = sq;
            __syncthreads();
            double tot = 0.0;
            for (int k = 0; k < 4; ++k) tot += red[k];
            scale = 1.0f / sqrtf((float)(tot / (double)K) + 1e-5f);
        }
        if (wave != 0) return;
        float q[4] = {v.x, v.y, v.z, v.w};
        if (NORM) { q[0] = (q[0] * scale) * wn.x; q[1] = (q[1] * scale) * wn.y; q[2] = (q[2] * scale) * wn.z; q[3] = (q[3] * scale) * wn.w; }
        q8k_to(act, nb, b, q, lane);
        return;
    }
    const int p = (int)blockIdx.x - nqp;
    const int xcd = p & 7, rank = p >> 3, R = ((int)gridDim.x - nqp) >> 3;
    const int lim = min(pf.cons_wgs, pf.max_wgs);
    unsigned f = 0;
    for (int b = xcd + 8 * rank; b < lim; b += 8 * R) {
        const long long r0 = (long long)b * pf.rows_per_wg;
        const long long r1 = min((long long)pf.rows, r0 + pf.rows_per_wg);
        for (int q = 0; q < pf.np; ++q) {
            const u32x4* base = reinterpret_cast<const u32x4*>(pf.p[q] + r0 * pf.pb[q]);
            const int n16 = (int)((r1 - r0) * pf.pb[q] / 16);
            for (int i = tid; i < n16; i += 4 * 256) {
                u32x4 v[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) v[u] = i + u * 256 < n16 ? *gptr(base + i + u * 256) : u32x4{0u, 0u, 0u, 0u};
#pragma unroll
                for (int u = 0; u < 4; ++u) f ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
            }
        }
    }
    if (f == 0x9e3779b9u) act[65535] = 1;
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
    int kind;          // 0 gemv, 1 quant norm, 2 quant plain, 3 qpf norm, 4 qpf plain
    PF pf; int pf_wgs;
    KFn fn;
    int nw, grid, smem;
    FA a;
    const float* qx; const float* qnw; int qK; char* qact;
    size_t bytes;
};
static void run(const Launch& L, hipStream_t s) {
    if (L.kind == 0) hipLaunchKernelGGL(L.fn, dim3(L.grid), dim3(L.nw * 64), L.smem, s, L.a);
    else if (L.kind == 1) hipLaunchKernelGGL(quant_kernel<1>, dim3(L.qK / 256), dim3(256), 0, s, L.qx, L.qnw, L.qK, L.qact);
    else if (L.kind == 2) hipLaunchKernelGGL(quant_kernel<0>, dim3(L.qK / 256), dim3(256), 0, s, L.qx, L.qnw, L.qK, L.qact);
    else {
        const int nqp = (L.qK / 256 + 7) / 8 * 8;
        if (L.kind == 3) hipLaunchKernelGGL(qpf_kernel<1>, dim3(nqp + L.pf_wgs), dim3(256), 0, s, L.qx, L.qnw, L.qK, L.qact, nqp, L.pf);
        else hipLaunchKernelGGL(qpf_kernel<0>, dim3(nqp + L.pf_wgs), dim3(256), 0, s, L.qx, L.qnw, L.qK, L.qact, nqp, L.pf);
    }
}
// the quant launch Q with the prefetch of GEMV G's weights (its first `frac` of workgroups)
static Launch with_pf(Launch Q, const Launch& G, const struct Mat& A, const struct Mat* B, int rw, double frac, int pf_wgs);
static Launch mk_quant(int norm, const float* x, const float* nw, int K, char* act) {
    Launch L{};
    L.kind = norm ? 1 : 2;
    L.qx = x; L.qnw = nw; L.qK = K; L.qact = act;
    return L;
}
// grid 0: one unit per wave slot (thin: units / (NW*UPW))
template <int T, int NW, int UPW, int RW, int C, int MODE, int EPI>
static Launch mk(const Mat& A, const Mat* B, FA base, int grid) {
    Launch L{};
    L.kind = 0;
    L.fn = fat<T, NW, UPW, RW, C, MODE, EPI>;
    L.nw = NW;
    FA& a = L.a;
    a = base;
    for (int p = 0; p < 4; ++p) { a.A[p] = A.p[p]; a.B[p] = B ? B->p[p] : A.p[p]; }
    a.rows = A.rows; a.nb = A.nb;
    a.units = EPI == 1 ? A.rows : (A.rows + RW - 1) / RW;
    L.grid = grid > 0 ? grid : (a.units + NW * UPW - 1) / (NW * UPW);
    if ((a.units + L.grid - 1) / L.grid > NW * UPW) { printf("grid %d too small for %d units\n", L.grid, a.units); exit(1); }
    L.smem = act_bytes(A.nb) + 8 * NW + 64;
    L.bytes = A.bytes + (B ? B->bytes : 0);
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(L.fn), hipFuncAttributeMaxDynamicSharedMemorySize, 65536));
    return L;
}

static Launch with_pf(Launch Q, const Launch& G, const Mat& A, const Mat* B, int rw, double frac, int pf_wgs) {
    Q.kind = Q.kind == 1 ? 3 : 4;
    PF& p = Q.pf;
    p = PF{};
    const int pb4[4] = {128, 16, 0, 0}, pb6[4] = {128, 64, 16, 2};
    const int* pb = A.type == T_Q4_K ? pb4 : pb6;
    for (const Mat* m : {&A, B}) {
        if (!m) continue;
        for (int q = 0; q < 4; ++q)
            if (pb[q]) { p.p[p.np] = m->p[q]; p.pb[p.np] = pb[q] * m->nb; ++p.np; }
    }
    p.rows = A.rows;
    // rows per consumer workgroup: units per workgroup (NW * UPW over the grid) * rows per unit
    const int units = G.a.units;
    p.rows_per_wg = (units + G.grid - 1) / G.grid * rw;
    p.cons_wgs = G.grid;
    p.max_wgs = (int)(frac * G.grid);
    Q.pf_wgs = pf_wgs;
    return Q;
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
    printf("%-44s grid %5d  graph %7.2f us (%4.2f TB/s)\n", name, Ls[0].grid, btb, Ls[0].bytes / btb / 1e6);
    fflush(stdout);
    CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g));
}

static double time_chain(const char* name, const std::vector<Launch>& st, size_t bytes, hipStream_t s) {
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
    printf("chain %-10s: %zu launches, %.3f GB, %.3f ms/step = %.1f tok/s, %.2f TB/s\n", name, st.size(), bytes / 1e9, per,
           1e3 / per, bytes / per / 1e9);
    fflush(stdout);
    CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g));
    return per;
}

int main(int argc, char** argv) {
    const int what = argc > 1 ? atoi(argv[1]) : 3;
    hipStream_t s;
    CK(hipStreamCreate(&s));
    float *x, *x2, *nw, *h, *out;
    char *actA, *actB, *actC, *actD;
    CK(hipMalloc(&x, 65536 * 4)); CK(hipMalloc(&x2, 65536 * 4)); CK(hipMalloc(&nw, 65536 * 4));
    CK(hipMalloc(&h, 65536 * 4)); CK(hipMalloc(&out, 65536 * 4));
    for (char** p : {&actA, &actB, &actC, &actD}) CK(hipMalloc(p, 65536));
    {
        std::vector<float> hx(65536), hw(65536, 1.0f);
        for (int i = 0; i < 65536; ++i) hx[i] = 0.01f * (float)((i * 37) % 101 - 50);
        CK(hipMemcpy(x, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(x2, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(nw, hw.data(), hw.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(h, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
    }
    hipLaunchKernelGGL(quant_kernel<1>, dim3(16), dim3(256), 0, s, x, nw, 4096, actA);
    hipLaunchKernelGGL(quant_kernel<1>, dim3(16), dim3(256), 0, s, x, nw, 4096, actB);
    hipLaunchKernelGGL(quant_kernel<1>, dim3(16), dim3(256), 0, s, x, nw, 4096, actC);
    hipLaunchKernelGGL(quant_kernel<0>, dim3(43), dim3(256), 0, s, h, nw, 11008, actD);
    CK(hipStreamSynchronize(s));
    FA b{};
    b.out = out; b.x = x; b.nw = nw; b.resid = x2;
    const int nrot = 6;
    if (what & 1) {
        std::vector<Mat> wo, gu_g, gu_u, down4, down6, qkv;
        for (int i = 0; i < nrot; ++i) {
            wo.push_back(make_mat(T_Q4_K, 4096, 4096));
            gu_g.push_back(make_mat(T_Q4_K, 11008, 4096));
            gu_u.push_back(make_mat(T_Q4_K, 11008, 4096));
            down4.push_back(make_mat(T_Q4_K, 4096, 11008));
            down6.push_back(make_mat(T_Q6_K, 4096, 11008));
            qkv.push_back(make_mat(T_Q4_K, 12288, 4096));
        }
        auto many = [&](auto f) { std::vector<Launch> v; for (int i = 0; i < nrot; ++i) v.push_back(f(i)); return v; };
#define KIND(name, expr) time_kind(name, many([&](int i) { return expr; }), s)
        FA bA = b; bA.act = actA;
        FA bD = b; bD.act = actD; bD.x = h;
        KIND("thin act   QKV  nw8 u1", (mk<T_Q4_K, 8, 1, 2, 2, 0, 0>(qkv[i], nullptr, bA, 0)));
        KIND("fat  act   QKV  nw8 u3", (mk<T_Q4_K, 8, 3, 2, 2, 0, 0>(qkv[i], nullptr, bA, 256)));
        KIND("thin rms   QKV  nw8 u1", (mk<T_Q4_K, 8, 1, 2, 2, 1, 0>(qkv[i], nullptr, bA, 0)));
        KIND("fat  rms   QKV  nw8 u3", (mk<T_Q4_K, 8, 3, 2, 2, 1, 0>(qkv[i], nullptr, bA, 256)));
        KIND("fat  rms   QKV  nw16 u2 g192", (mk<T_Q4_K, 16, 2, 2, 2, 1, 0>(qkv[i], nullptr, bA, 192)));
        KIND("fat  rms   QKV  nw8 u2 g384", (mk<T_Q4_K, 8, 2, 2, 2, 1, 0>(qkv[i], nullptr, bA, 384)));
        KIND("thin act   UP   nw8 u1", (mk<T_Q4_K, 8, 1, 2, 2, 0, 1>(gu_g[i], &gu_u[i], bA, 0)));
        KIND("fat  act   UP   nw16 u3", (mk<T_Q4_K, 16, 3, 2, 2, 0, 1>(gu_g[i], &gu_u[i], bA, 256)));
        KIND("fat  rms   UP   nw16 u3", (mk<T_Q4_K, 16, 3, 2, 2, 1, 1>(gu_g[i], &gu_u[i], bA, 256)));
        KIND("fat  rms   UP   nw8 u3 g512", (mk<T_Q4_K, 8, 3, 2, 2, 1, 1>(gu_g[i], &gu_u[i], bA, 512)));
        KIND("fat  rms   UP   nw16 u2 g512", (mk<T_Q4_K, 16, 2, 2, 2, 1, 1>(gu_g[i], &gu_u[i], bA, 512)));
        KIND("thin act   WO   nw8 u1", (mk<T_Q4_K, 8, 1, 1, 2, 0, 2>(wo[i], nullptr, bA, 0)));
        KIND("fat  act   WO   nw16 u1", (mk<T_Q4_K, 16, 1, 1, 2, 0, 2>(wo[i], nullptr, bA, 256)));
        KIND("thin act   DN4  nw8 u1", (mk<T_Q4_K, 8, 1, 1, 6, 0, 2>(down4[i], nullptr, bD, 0)));
        KIND("thin plain DN4  nw8 u1", (mk<T_Q4_K, 8, 1, 1, 6, 2, 2>(down4[i], nullptr, bD, 0)));
        KIND("fat  act   DN4  nw16 u1", (mk<T_Q4_K, 16, 1, 1, 6, 0, 2>(down4[i], nullptr, bD, 256)));
        KIND("fat  plain DN4  nw16 u1", (mk<T_Q4_K, 16, 1, 1, 6, 2, 2>(down4[i], nullptr, bD, 256)));
        KIND("thin act   DN6  nw8 u1", (mk<T_Q6_K, 8, 1, 1, 6, 0, 2>(down6[i], nullptr, bD, 0)));
        KIND("fat  act   DN6  nw16 u1", (mk<T_Q6_K, 16, 1, 1, 6, 0, 2>(down6[i], nullptr, bD, 256)));
        KIND("fat  plain DN6  nw16 u1", (mk<T_Q6_K, 16, 1, 1, 6, 2, 2>(down6[i], nullptr, bD, 256)));
        KIND("fat  plain DN6  nw8 u1 g512", (mk<T_Q6_K, 8, 1, 1, 6, 2, 2>(down6[i], nullptr, bD, 512)));
        KIND("quant  norm 4096", (mk_quant(1, x, nw, 4096, actB)));
        KIND("quant  plain 11008", (mk_quant(0, h, nw, 11008, actD)));
#undef KIND
    }
    if (what & 2) {
        // a 7B Q4_K_M-like step: 32 layers x {QKV, [attention out quant], WO, gate/up, down} + the head
        const int L = 32;
        std::vector<Launch> sep3, fat3, pro;
        size_t bytes = 0;
        FA bq = b; bq.act = actA; bq.x = x; bq.out = out;          // QKV: act A / x
        FA bw = b; bw.act = actB; bw.out = x2; bw.resid = x;       // WO: act B (attention output) -> x2
        FA bg = b; bg.act = actC; bg.x = x2; bg.out = h;           // gate/up: act C / x2 -> h
        FA bd = b; bd.act = actD; bd.x = h; bd.out = x; bd.resid = x2;   // down: act D / h -> x
        for (int l = 0; l < L; ++l) {
            const bool more = l < L / 8 || l >= 7 * L / 8 || (l - L / 8) % 3 == 2;
            Mat qkv = make_mat(T_Q4_K, 12288, 4096), wo = make_mat(T_Q4_K, 4096, 4096);
            Mat g = make_mat(T_Q4_K, 11008, 4096), u = make_mat(T_Q4_K, 11008, 4096);
            Mat d = make_mat(more ? T_Q6_K : T_Q4_K, 4096, 11008);
            bytes += qkv.bytes + wo.bytes + g.bytes + u.bytes + d.bytes;
            // sep3: the r05 engine's form (thin workgroups, quant launches before gate/up, down, QKV)
            sep3.push_back(mk<T_Q4_K, 8, 1, 2, 2, 0, 0>(qkv, nullptr, bq, 0));
            sep3.push_back(mk_quant(0, out, nw, 4096, actB));   // stand-in for the attention launch
            sep3.push_back(mk<T_Q4_K, 8, 1, 1, 2, 0, 2>(wo, nullptr, bw, 0));
            sep3.push_back(mk_quant(1, x2, nw, 4096, actC));
            sep3.push_back(mk<T_Q4_K, 8, 1, 2, 2, 0, 1>(g, &u, bg, 0));
            sep3.push_back(mk_quant(0, h, nw, 11008, actD));
            if (more) sep3.push_back(mk<T_Q6_K, 8, 1, 1, 6, 0, 2>(d, nullptr, bd, 0));
            else sep3.push_back(mk<T_Q4_K, 8, 1, 1, 6, 0, 2>(d, nullptr, bd, 0));
            sep3.push_back(mk_quant(1, x, nw, 4096, actA));
            // fat3: fat workgroups, the same quant launches
            fat3.push_back(mk<T_Q4_K, 8, 3, 2, 2, 0, 0>(qkv, nullptr, bq, 256));
            fat3.push_back(mk_quant(0, out, nw, 4096, actB));
            fat3.push_back(mk<T_Q4_K, 16, 1, 1, 2, 0, 2>(wo, nullptr, bw, 256));
            fat3.push_back(mk_quant(1, x2, nw, 4096, actC));
            fat3.push_back(mk<T_Q4_K, 16, 3, 2, 2, 0, 1>(g, &u, bg, 256));
            fat3.push_back(mk_quant(0, h, nw, 11008, actD));
            if (more) fat3.push_back(mk<T_Q6_K, 16, 1, 1, 6, 0, 2>(d, nullptr, bd, 256));
            else fat3.push_back(mk<T_Q4_K, 16, 1, 1, 6, 0, 2>(d, nullptr, bd, 256));
            fat3.push_back(mk_quant(1, x, nw, 4096, actA));
            // pro: fat workgroups building their own activation (no quant launches but the attention stand-in)
            pro.push_back(mk<T_Q4_K, 8, 3, 2, 2, 1, 0>(qkv, nullptr, bq, 256));
            pro.push_back(mk_quant(0, out, nw, 4096, actB));
            pro.push_back(mk<T_Q4_K, 16, 1, 1, 2, 0, 2>(wo, nullptr, bw, 256));
            pro.push_back(mk<T_Q4_K, 16, 3, 2, 2, 1, 1>(g, &u, bg, 256));
            if (more) pro.push_back(mk<T_Q6_K, 16, 1, 1, 6, 2, 2>(d, nullptr, bd, 256));
            else pro.push_back(mk<T_Q4_K, 16, 1, 1, 6, 2, 2>(d, nullptr, bd, 256));
        }
        Mat o = make_mat(T_Q6_K, 32000, 4096);
        bytes += o.bytes;
        FA bo = b; bo.act = actA;
        sep3.push_back(mk<T_Q6_K, 8, 1, 1, 2, 0, 0>(o, nullptr, bo, 0));
        fat3.push_back(mk<T_Q6_K, 8, 1, 1, 2, 0, 0>(o, nullptr, bo, 0));
        pro.push_back(mk<T_Q6_K, 8, 1, 1, 2, 0, 0>(o, nullptr, bo, 0));
        for (int rep = 0; rep < 2; ++rep) {
            time_chain("sep3", sep3, bytes, s);
            time_chain("fat3", fat3, bytes, s);
            time_chain("pro", pro, bytes, s);
        }
    }
    if (what & 4) {
        // pairs: [quant; GEMV] vs [quant + prefetch of the GEMV's weights into L2; GEMV], cold weights
        // (enough rotations to exceed the 256 MB Infinity Cache)
        struct K { const char* name; int type, rows, K, pair, rw, nrot; };
        const K ks[] = {{"QKV", T_Q4_K, 12288, 4096, 0, 2, 14}, {"WO", T_Q4_K, 4096, 4096, 0, 1, 40},
                        {"UP", T_Q4_K, 11008, 4096, 1, 2, 6}, {"DN4", T_Q4_K, 4096, 11008, 0, 1, 14},
                        {"DN6", T_Q6_K, 4096, 11008, 0, 1, 10}};
        for (const K& k : ks) {
            std::vector<Mat> A, B;
            for (int i = 0; i < k.nrot; ++i) {
                A.push_back(make_mat(k.type, k.rows, k.K));
                if (k.pair) B.push_back(make_mat(k.type, k.rows, k.K));
            }
            auto gemv = [&](int i) {
                FA bb = b;
                bb.act = k.K == 4096 ? actA : actD;
                bb.out = k.pair ? h : out;
                if (k.type == T_Q6_K) return mk<T_Q6_K, 8, 1, 1, 6, 0, 2>(A[i], nullptr, bb, 0);
                if (k.pair) return mk<T_Q4_K, 8, 1, 2, 2, 0, 1>(A[i], &B[i], bb, 0);
                if (k.K == 11008) return mk<T_Q4_K, 8, 1, 1, 6, 0, 2>(A[i], nullptr, bb, 0);
                if (k.rw == 2) return mk<T_Q4_K, 8, 1, 2, 2, 0, 0>(A[i], nullptr, bb, 0);
                return mk<T_Q4_K, 8, 1, 1, 2, 0, 2>(A[i], nullptr, bb, 0);
            };
            const Launch q = k.K == 4096 ? mk_quant(1, x, nw, 4096, actA) : mk_quant(0, h, nw, 11008, actD);
            for (int variant = 0; variant < 7; ++variant) {
                const double fr[7] = {0, 1.0, 1.0, 1.0, 0.5, 0.5, 0.25};
                const int wg[7] = {0, 256, 512, 1024, 256, 512, 256};
                std::vector<Launch> st;
                for (int i = 0; i < k.nrot; ++i) {
                    const Launch g = gemv(i);
                    st.push_back(variant == 0 ? q : with_pf(q, g, A[i], k.pair ? &B[i] : nullptr, k.rw, fr[variant], wg[variant]));
                    st.push_back(g);
                }
                std::vector<Launch> rep;
                for (int r = 0; r < 64 / k.nrot + 1; ++r) rep.insert(rep.end(), st.begin(), st.end());
                char name[96];
                snprintf(name, sizeof name, "%s pair pf frac %.2f wgs %d", k.name, fr[variant], wg[variant]);
                const double ms = time_chain(name, rep, 0, s);
                printf("   -> %.2f us per pair\n", ms * 1e3 / (rep.size() / 2));
            }
            // the quant launch alone and the GEMV alone, same rotation
            std::vector<Launch> qa, ga;
            for (int i = 0; i < 64; ++i) { qa.push_back(q); ga.push_back(gemv(i % k.nrot)); }
            printf("   quant alone %.2f us, gemv alone %.2f us\n", time_chain("q", qa, 0, s) * 1e3 / 64, time_chain("g", ga, 0, s) * 1e3 / 64);
        }
    }
    return 0;
}
