// Causal attention of a physical batch of query tokens over the f16 KV cache on gfx950 f16
// MFMA (v_mfma_f32_32x32x16_f16): prompt ingestion and batched verification at any context
// length (row N1 of SURVEY.md §8 / DESIGN.md §4).
//
// Numerics are the ggml b5187 CPU graph's (llm_build_kqv, flash_attn off), as in the VALU
// kernels of kernels.hip: q rounded to f16 (the f16 vec_dot_type), KQ = sum f16(q) k in f32,
// w = KQ * scale, masked to -inf where the cell is after the token (cell_pos > pos, or a later
// cell); soft_max with the exact global max, the sum of expf(w - max) in double and
// p = expf(w - max) * (float)(1/sum); KQV = sum f16(p) v in f32.  The softmax is therefore
// three passes over the cells (max, sum, weighted V) -- an online softmax would round p
// before the sum is known.  Only fp32 summation orders differ from the CPU.
//
// Geometry.  A workgroup is one query head x 64 tokens (2 waves, a 32-token tile each); the
// 32-cell chunks of K and V are staged once per workgroup in LDS (V transposed) and shared,
// the next chunk's loads in flight while the current one is computed.
// S^T = K Q^T per chunk (D: lane = token, registers = cells), so a token's softmax statistics
// are lane-local, and S^T's registers are directly the B operand of O^T = V^T P^T (the
// accumulator-as-operand idiom: element j of k-step s = register 8s + j = cell
// 16s + 8(j>>2) + 4h + (j&3), which the V^T operand reads at the same cells).
#include "kernels.h"
#include <hip/hip_runtime.h>

namespace mi {
namespace amf {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f16x16 __attribute__((ext_vector_type(16)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

constexpr int WT = 2;          // token tiles (waves) per workgroup
constexpr int CH = 32;         // cells per chunk

__device__ __forceinline__ unsigned pack2(float a, float b) {
    const unsigned lo = __half_as_ushort(__float2half_rn(a)), hi = __half_as_ushort(__float2half_rn(b));
    return lo | (hi << 16);
}
__device__ __forceinline__ half8 as_h8(u32x4 v) { return __builtin_bit_cast(half8, v); }

template <int HD>
__global__ __launch_bounds__(64 * WT) void attn_mfma_kernel(const AttnParams P, int ntok, float* out) {
    constexpr int KS = HD / 16;          // k-steps of KQ
    constexpr int HB = HD / 32;          // 32-wide output blocks
    constexpr int KST = HD + 8;          // K row stride (halfs): 16-B aligned, staggered banks
    constexpr int VST = CH + 4;          // V^T row stride (halfs): 72 B
    __shared__ __attribute__((aligned(16))) _Float16 ks[CH * KST];
    __shared__ __attribute__((aligned(16))) _Float16 vt[HD * VST];
    __shared__ int cps[CH];
    __shared__ int last_cell;
    const int hq = blockIdx.x;                      // query head
    const int R = P.n_head / P.n_head_kv;
    const int g = hq / R;                           // its kv head
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int col = lane & 31, h = lane >> 5;
    const int t0 = blockIdx.y * (32 * WT) + 32 * w;   // this wave's token tile
    const int tok = t0 + col;                       // this lane's query token (D column)
    const bool tv = tok < ntok;
    const int qcell = tv ? P.tokpos[tok * 4 + 2] : -1;
    const int qpos = tv ? P.tokpos[tok * 4 + 1] : 0;
    // the workgroup's last cell (its last valid token's) and this wave's
    if (tid == 0) {
        const int lt = min(ntok, (int)(blockIdx.y + 1) * 32 * WT) - 1;
        last_cell = P.tokpos[lt * 4 + 2];
    }
    int wlast = -1;
    {
        const int lt = min(ntok, t0 + 32) - 1;
        if (lt >= t0) wlast = P.tokpos[lt * 4 + 2];
    }
    // Q^T fragments (B operand): lane (token col, half h), k-step s: q[tok][16s + 8h .. +7] as f16
    u32x4 qf[KS];
    {
        const float* qrow = P.q + (long long)(tv ? tok : 0) * P.n_head * HD + (long long)hq * HD;
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const float4 a = *reinterpret_cast<const float4*>(qrow + 16 * s + 8 * h);
            const float4 b = *reinterpret_cast<const float4*>(qrow + 16 * s + 8 * h + 4);
            qf[s] = tv ? u32x4{pack2(a.x, a.y), pack2(a.z, a.w), pack2(b.x, b.y), pack2(b.z, b.w)}
                       : u32x4{0u, 0u, 0u, 0u};
        }
    }
    __syncthreads();
    const int ncell = last_cell + 1;
    float mx = -INFINITY, inv = 0.0f;
    double sum = 0.0;
    f16x16 o[HB];
#pragma unroll
    for (int b = 0; b < HB; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[b][r] = 0.0f;

    constexpr int SEG = HD / 8;                     // 16-B pieces per cell row
    constexpr int NPC = CH * SEG / (64 * WT);       // pieces per thread per chunk
    static_assert(CH * SEG % (64 * WT) == 0, "chunk pieces split evenly over the threads");
    for (int pass = 0; pass < 3; ++pass) {
        // the next chunk's K (and V) in registers, issued before the current chunk is computed
        u32x4 kr[NPC], vr_[NPC];
        int cpr = 0;
        auto fetch = [&](int c0) {
#pragma unroll
            for (int i = 0; i < NPC; ++i) {
                const int pc = tid + 64 * WT * i;
                const int cl = pc / SEG, sg = pc % SEG;
                const int c = min(c0 + cl, P.n_ctx - 1);
                const long long ga = (long long)c * P.kv_dim + (long long)g * HD + sg * 8;
                kr[i] = *reinterpret_cast<const u32x4*>(P.kcache + ga);
                if (pass == 2) {   // cells past the batch's last are zero (p = 0 there; 0 * stale bits)
                    const u32x4 z = {0u, 0u, 0u, 0u};
                    vr_[i] = c0 + cl <= last_cell ? *reinterpret_cast<const u32x4*>(P.vcache + ga) : z;
                }
            }
            if (tid < CH) cpr = P.cell_pos[min(c0 + tid, P.n_ctx - 1)];
        };
        fetch(0);
        for (int c0 = 0; c0 < ncell; c0 += CH) {
            // ---- stage K (and V^T in the last pass) of cells c0 .. c0+31, and their positions
            __syncthreads();
#pragma unroll
            for (int i = 0; i < NPC; ++i) {
                const int pc = tid + 64 * WT * i;
                const int cl = pc / SEG, sg = pc % SEG;
                *reinterpret_cast<u32x4*>(&ks[cl * KST + sg * 8]) = kr[i];
                if (pass == 2) {
                    const unsigned vw[4] = {vr_[i].x, vr_[i].y, vr_[i].z, vr_[i].w};
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        vt[(sg * 8 + 2 * e) * VST + cl] = __ushort_as_half((unsigned short)(vw[e] & 0xFFFFu));
                        vt[(sg * 8 + 2 * e + 1) * VST + cl] = __ushort_as_half((unsigned short)(vw[e] >> 16));
                    }
                }
            }
            if (tid < CH) cps[tid] = cpr;
            __syncthreads();
            if (c0 + CH < ncell) fetch(c0 + CH);
            if (c0 > wlast) continue;                   // wave-uniform: nothing of this tile here
            // ---- S^T = K Q^T: lane = token, register r = cell c0 + (r&3) + 8(r>>2) + 4h
            f16x16 st;
#pragma unroll
            for (int r = 0; r < 16; ++r) st[r] = 0.0f;
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                const u32x4 kf = *reinterpret_cast<const u32x4*>(&ks[col * KST + 16 * s + 8 * h]);
                st = __builtin_amdgcn_mfma_f32_32x32x16_f16(as_h8(kf), as_h8(qf[s]), st, 0, 0, 0);
            }
            float wv[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int cl = (r & 3) + 8 * (r >> 2) + 4 * h;
                const int c = c0 + cl;
                const bool ok = tv && c <= qcell && cps[cl] <= qpos;
                wv[r] = ok ? st[r] * P.scale : -INFINITY;
            }
            if (pass == 0) {
#pragma unroll
                for (int r = 0; r < 16; ++r) mx = fmaxf(mx, wv[r]);
            } else if (pass == 1) {
#pragma unroll
                for (int r = 0; r < 16; ++r) sum += (double)expf(wv[r] - mx);
            } else {
                // p = f16(expf(w - max) * inv): the B operand of k-steps 0 (registers 0-7), 1 (8-15)
                u32x4 pf[2];
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    float p[8];
#pragma unroll
                    for (int j = 0; j < 8; ++j) p[j] = tv ? expf(wv[8 * s + j] - mx) * inv : 0.0f;
                    pf[s] = u32x4{pack2(p[0], p[1]), pack2(p[2], p[3]), pack2(p[4], p[5]), pack2(p[6], p[7])};
                }
#pragma unroll
                for (int b = 0; b < HB; ++b) {
#pragma unroll
                    for (int s = 0; s < 2; ++s) {
                        // V^T operand: row hd = 32b + col, cells 16s + 4h + 0..3 and 16s + 8 + 4h + 0..3
                        const _Float16* vr = &vt[(32 * b + col) * VST + 16 * s + 4 * h];
                        const u32x2 lo = *reinterpret_cast<const u32x2*>(vr);
                        const u32x2 hi = *reinterpret_cast<const u32x2*>(vr + 8);
                        const u32x4 vf = {lo.x, lo.y, hi.x, hi.y};
                        o[b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(as_h8(vf), as_h8(pf[s]), o[b], 0, 0, 0);
                    }
                }
            }
        }
        if (pass == 0) {
            mx = fmaxf(mx, __shfl_xor(mx, 32, 64));   // the token's other half of the cells
        } else if (pass == 1) {
            const long long b = __double_as_longlong(sum);
            const int lo = __shfl_xor((int)b, 32, 64), hi = __shfl_xor((int)(b >> 32), 32, 64);
            const double other = __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
            const double tot = h == 0 ? sum + other : other + sum;   // same order in both halves
            inv = (float)(1.0 / tot);
        }
    }
    // ---- O^T: lane = token, register r of block b = hd 32b + (r&3) + 8(r>>2) + 4h
    if (!tv) return;
    float* orow = out + (long long)tok * P.n_head * HD + (long long)hq * HD;
#pragma unroll
    for (int b = 0; b < HB; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) orow[32 * b + (r & 3) + 8 * (r >> 2) + 4 * h] = o[b][r];
}

}  // namespace amf

bool attn_mfma_supported(int head_dim) { return head_dim == 64 || head_dim == 128; }

void launch_attn_mfma(const AttnParams& p, int ntok, float* out, hipStream_t s) {
    if (ntok < 1) return;
    if (p.n_head % p.n_head_kv) throw Error("attn_mfma: n_head must be a multiple of n_head_kv");
    const dim3 grid(p.n_head, (ntok + 32 * amf::WT - 1) / (32 * amf::WT));
    if (p.head_dim == 128) hipLaunchKernelGGL(amf::attn_mfma_kernel<128>, grid, dim3(64 * amf::WT), 0, s, p, ntok, out);
    else if (p.head_dim == 64) hipLaunchKernelGGL(amf::attn_mfma_kernel<64>, grid, dim3(64 * amf::WT), 0, s, p, ntok, out);
    else throw Error("attn_mfma: head_dim 64 or 128");
    MI_HIP(hipGetLastError());
}

}  // namespace mi
