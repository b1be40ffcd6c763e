// Causal attention of a physical batch of query tokens over the f16 KV cache on gfx950 f16
// MFMA (v_mfma_f32_32x32x16_f16): prompt ingestion and batched verification at any context
// length (row N1 of SURVEY.md §8 / DESIGN.md §4).
//
// Numerics are the ggml b5187 CPU graph's (llm_build_kqv, flash_attn off), as in the VALU
// kernels of kernels.hip: q rounded to f16 (the f16 vec_dot_type), KQ = sum f16(q) k in f32,
// w = KQ * scale, masked to -inf where the cell is after the token (cell_pos > pos, or a later
// cell); soft_max with the exact global max, the sum of expf(w - max) in double and
// p = expf(w - max) * (float)(1/sum); KQV = sum f16(p) v in f32.  The softmax needs the max
// before any exponential and the whole sum before any p (an online softmax would round p
// before the sum is known); only fp32 / double summation orders differ from the CPU.
//
// Geometry.  A workgroup is one query head x one 32-token tile, 8 waves; the tile's 32-cell
// chunks are dealt to the waves round-robin (chunk c -> wave c % 8), so every wave holds its
// chunks' scores in registers:
//   S^T = K Q^T per chunk (D: lane = token, register r = cell (r&3) + 8(r>>2) + 4h), K straight
//   from the cache into the A operand (16 B per lane and k-step), so a token's softmax
//   statistics are lane-local; the waves' maxima and double sums are combined through LDS in
//   wave order.  O^T = V^T P^T: P^T is the S^T accumulator itself (registers 8s..8s+7 are the
//   B operand of k-step s, k-permuted), V^T comes from the wave's V chunk staged row-major in
//   LDS (XOR-swizzled 256-B rows) and read with ds_read_b64_tr_b16.  The 8 waves' O^T
//   partials are added in a fixed tree order through LDS.
// Up to 8 * CPR chunks (CPR per wave) the scores are computed once and kept in registers over
// the three softmax passes.  Past that a wave computes them twice, CPR chunks at a time: pass 1
// takes the max and, against its running max, the double sum (rescaled to the global max at the
// end: the terms' float rounding is the only difference from the direct sum); pass 3 recomputes
// them for p = f16(expf(w - max) * (1/sum)), exactly as the CPU rounds p.
#include "kernels.h"
#include <hip/hip_runtime.h>

namespace mi {
namespace amf {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef __fp16 trv4 __attribute__((__vector_size__(4 * sizeof(__fp16))));   // ds_read_tr16_b64 result
typedef float f16x16 __attribute__((ext_vector_type(16)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

constexpr int NW = 8;          // waves per workgroup (cell groups of one token tile)
constexpr int CH = 32;         // cells per chunk
constexpr int CPR = 2;         // chunks per wave whose scores stay in registers

__device__ __forceinline__ unsigned pack2(float a, float b) {
    const unsigned lo = __half_as_ushort(__float2half_rn(a)), hi = __half_as_ushort(__float2half_rn(b));
    return lo | (hi << 16);
}
__device__ __forceinline__ half8 as_h8(u32x4 v) { return __builtin_bit_cast(half8, v); }

// byte offset of 16-B chunk `ch` (0..HD/8-1) of row `row` in a [CH][HD] f16 image of 2*HD-byte
// rows, XOR-swizzled so that the transposed reads of the PV operand are conflict-free
// (cdna_hip_programming.md T10 layout (b), generalised to HD/8 chunks per row)
template <int HD>
__device__ __forceinline__ int vimg_off(int row, int ch) {
    constexpr int NCH = HD / 8;
    const int x = (((row & 3) << 2) | ((row >> 2) & 3)) & (NCH - 1);
    return row * (2 * HD) + 16 * (ch ^ x);
}

template <int HD>
__global__ __launch_bounds__(64 * NW) void attn_mfma_kernel(const AttnParams P, int ntok, float* out) {
    constexpr int KS = HD / 16;          // k-steps of KQ
    constexpr int HB = HD / 32;          // 32-wide output blocks
    constexpr int VPL = CH * HD / 8 / 64;   // 16-B pieces of a V chunk per lane
    constexpr int VIMG = CH * HD * 2;    // bytes of one V chunk image
    // LDS (dynamic, NW * VIMG bytes): one V chunk image per wave, reused for the partial-output
    // tree; then the exchanges
    extern __shared__ __attribute__((aligned(16))) char vimg[];
    __shared__ float xmax[NW][32];
    __shared__ double xsum[NW][32];
    const int hq = blockIdx.x;                      // query head
    const int R = P.n_head / P.n_head_kv;
    const int g = hq / R;                           // its kv head
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int col = lane & 31, h = lane >> 5;
    // the token tile: the last (longest causal extent) first, so that the short tiles fill in
    // behind the long ones (one workgroup per CU at 8 waves x ~250 VGPRs)
    const int t0 = (gridDim.y - 1 - blockIdx.y) * 32;
    const int tok = t0 + col;                       // this lane's query token (D column)
    const bool tv = tok < ntok;
    const int qcell = tv ? P.tokpos[tok * 4 + 2] : -1;
    const int qpos = tv ? P.tokpos[tok * 4 + 1] : 0;
    const __half* kbase = P.kcache + (long long)g * HD;
    const __half* vbase = P.vcache + (long long)g * HD;
    auto kload = [&](int c, u32x4 (&kf)[KS], i32x4 (&cp)[4]) {
        const int c0 = c * CH;
        const int cr = min(c0 + col, P.n_ctx - 1);  // the A operand row this lane supplies
#pragma unroll
        for (int s = 0; s < KS; ++s) kf[s] = *reinterpret_cast<const u32x4*>(kbase + (long long)cr * P.kv_dim + 16 * s + 8 * h);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int cb = c0 + 8 * q + 4 * h;
            if (cb + 3 < P.n_ctx) {
                cp[q] = *reinterpret_cast<const i32x4*>(P.cell_pos + cb);
            } else {   // the cache's last cells (cells past n_ctx are masked by cell <= qcell)
#pragma unroll
                for (int e = 0; e < 4; ++e) cp[q][e] = P.cell_pos[min(cb + e, P.n_ctx - 1)];
            }
        }
    };
    // the wave's first chunk (w) is loaded at entry, before the tile's extent is known: a chunk
    // past it is unused
    u32x4 kf0[KS];
    i32x4 cp0[4];
    kload(w, kf0, cp0);
    // the tile's last cell (its last valid token's): the causal end of every token in it
    const int wlast = __builtin_amdgcn_readfirstlane(P.tokpos[(min(ntok, t0 + 32) - 1) * 4 + 2]);
    const int nch = wlast / CH + 1;                 // chunks of the tile
    const int myn = nch > w ? (nch - w + NW - 1) / NW : 0;   // this wave's chunks: w, w+8, ...
    const int nround = (myn + CPR - 1) / CPR;
    const bool keep = nround <= 1;                  // scores computed once, kept in registers

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
    // scores of chunk c into st: masked, scaled w (lane = token, register r = cell (r&3)+8(r>>2)+4h);
    // kload (above) issues the chunk's K rows and cell positions, kcompute runs the MFMAs and the mask
    auto kcompute = [&](int c, const u32x4 (&kf)[KS], const i32x4 (&cp)[4], f16x16& st) {
        const int c0 = c * CH;
#pragma unroll
        for (int r = 0; r < 16; ++r) st[r] = 0.0f;
#pragma unroll
        for (int s = 0; s < KS; ++s) st = __builtin_amdgcn_mfma_f32_32x32x16_f16(as_h8(kf[s]), as_h8(qf[s]), st, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int cell = c0 + (r & 3) + 8 * (r >> 2) + 4 * h;
            const int pos = cp[r >> 2][r & 3];
            const bool ok = tv && cell <= qcell && pos <= qpos;
            st[r] = ok ? st[r] * P.scale : -INFINITY;
        }
    };
    auto scores = [&](int c, f16x16& st) {
        u32x4 kf[KS];
        i32x4 cp[4];
        kload(c, kf, cp);
        kcompute(c, kf, cp, st);
    };

    // ---- pass 1: the token's max over every cell ------------------------------------------------
    // (a wave that cannot keep its scores also sums expf(w - m) against its running max m, in
    // double, rescaling by exp(m_old - m_new) when m grows; at the end the sum is rescaled to the
    // global max: the scores are computed twice instead of three times, and the sum differs from
    // the direct one by float rounding of its terms only)
    f16x16 st[CPR];
    float mx = -INFINITY;
    double srun = 0.0;
    if (keep) {
#pragma unroll
        for (int i = 0; i < CPR; ++i) {
            if (i < myn) {
                if (i == 0) kcompute(w, kf0, cp0, st[i]);   // (loaded at entry)
                else scores(w + NW * i, st[i]);
#pragma unroll
                for (int r = 0; r < 16; ++r) mx = fmaxf(mx, st[i][r]);
            }
        }
    } else {
        // chunk by chunk, the next chunk's K rows in flight during this one's MFMAs
        auto step = [&](int k, const u32x4 (&kf)[KS], const i32x4 (&cp)[4]) {
            f16x16 sc;
            kcompute(w + NW * k, kf, cp, sc);
            float cm = -INFINITY;
#pragma unroll
            for (int r = 0; r < 16; ++r) cm = fmaxf(cm, sc[r]);
            if (cm > mx) {
                if (mx != -INFINITY) srun *= exp((double)mx - (double)cm);
                mx = cm;
            }
            if (mx != -INFINITY) {
#pragma unroll
                for (int r = 0; r < 16; ++r) srun += (double)expf(sc[r] - mx);
            }
        };
        u32x4 kf1[KS];
        i32x4 cp1[4];
        for (int k = 0; k < myn; k += 2) {
            if (k + 1 < myn) kload(w + NW * (k + 1), kf1, cp1);
            step(k, kf0, cp0);
            if (k + 1 >= myn) break;
            if (k + 2 < myn) kload(w + NW * (k + 2), kf0, cp0);
            step(k + 1, kf1, cp1);
        }
    }
    const float mlane = mx;   // this lane's own max (the running max of srun)
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));         // the token's other half of the cells
    if (h == 0) xmax[w][col] = mx;
    __syncthreads();
    float M = xmax[0][col];
#pragma unroll
    for (int k = 1; k < NW; ++k) M = fmaxf(M, xmax[k][col]);

    // V chunk c: piece i of this lane = row (lane + 64 i) / (HD/8), chunk (lane + 64 i) % (HD/8);
    // rows past the tile's last cell are zero (p = 0 there, and 0 * stale bits could be NaN)
    u32x4 vr[VPL];
    auto vload = [&](int c) {
#pragma unroll
        for (int i = 0; i < VPL; ++i) {
            const int pc = lane + 64 * i;
            const int row = pc / (HD / 8), ch = pc % (HD / 8);
            const int cell = c * CH + row;
            const u32x4 z = {0u, 0u, 0u, 0u};
            vr[i] = cell <= wlast ? *reinterpret_cast<const u32x4*>(vbase + (long long)min(cell, P.n_ctx - 1) * P.kv_dim + 8 * ch) : z;
        }
    };
    if (myn > 0) vload(w);   // the first chunk's V in flight during pass 2

    // ---- pass 2: the sum of expf(w - M) in double, waves added in order ------------------------
    double sum = 0.0;
    if (keep) {
#pragma unroll
        for (int i = 0; i < CPR; ++i) {
            if (i < myn) {
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const float e = expf(st[i][r] - M);
                    sum += (double)e;
                    st[i][r] = e;   // kept for pass 3: one expf per score
                }
            }
        }
    } else if (mlane != -INFINITY) {
        sum = srun * exp((double)mlane - (double)M);
    }
    {
        const long long b = __double_as_longlong(sum);
        const int lo = __shfl_xor((int)b, 32, 64), hi = __shfl_xor((int)(b >> 32), 32, 64);
        const double other = __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
        sum = h == 0 ? sum + other : other + sum;   // same order in both halves
    }
    if (h == 0) xsum[w][col] = sum;
    __syncthreads();
    double tot = 0.0;
#pragma unroll
    for (int k = 0; k < NW; ++k) tot += xsum[k][col];
    const float inv = (float)(1.0 / tot);

    // ---- pass 3: O^T += V^T P^T over the wave's chunks --------------------------------------------
    f16x16 o[HB];
#pragma unroll
    for (int b = 0; b < HB; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[b][r] = 0.0f;
    char* const vw = vimg + w * VIMG;
    // (recomputed scores: the next chunk's K rows in flight during this chunk's PV)
    u32x4 kfp[KS];
    i32x4 cpp[4];
    if (!keep && myn > 0) kload(w, kfp, cpp);
    for (int rd = 0; rd < nround; ++rd) {
#pragma unroll
        for (int i = 0; i < CPR; ++i) {
            const int k = rd * CPR + i;
            if (k < myn) {
                const int c = w + NW * k;
                if (!keep) {
                    kcompute(c, kfp, cpp, st[i]);
                    if (k + 1 < myn) kload(c + NW, kfp, cpp);
                }
                // stage this chunk's V (wave-private image; the previous chunk's reads are done:
                // ds ops of one wave complete in order)
#pragma unroll
                for (int j = 0; j < VPL; ++j) {
                    const int pc = lane + 64 * j;
                    *reinterpret_cast<u32x4*>(vw + vimg_off<HD>(pc / (HD / 8), pc % (HD / 8))) = vr[j];
                }
                if (k + 1 < myn) vload(c + NW);     // the next chunk's V in flight during this one
                // p = f16(expf(w - M) * inv): the B operand of k-steps 0 (registers 0-7), 1 (8-15)
                u32x4 pf[2];
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    float p[8];
#pragma unroll
                    for (int j = 0; j < 8; ++j)
                        p[j] = tv ? (keep ? st[i][8 * s + j] : expf(st[i][8 * s + j] - M)) * inv : 0.0f;
                    pf[s] = u32x4{pack2(p[0], p[1]), pack2(p[2], p[3]), pack2(p[4], p[5]), pack2(p[6], p[7])};
                }
                __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): the V image is written
#pragma unroll
                for (int b = 0; b < HB; ++b) {
#pragma unroll
                    for (int s = 0; s < 2; ++s) {
                        // V^T operand of lane (hd row 32b + col, half h), k-step s: cells
                        // 16s + 4h + 0..3 (elements 0-3) and 16s + 8 + 4h + 0..3 (elements 4-7),
                        // two transposed reads of 4 rows x 16 columns per 16-lane group
                        const int gq = (lane >> 2) & 3, gp = lane & 3;       // lane 4q+p of its group
                        const int colb = 32 * b + 16 * ((lane >> 4) & 1) + 4 * gp;   // first hd of the lane's address
                        const int r0 = 16 * s + 4 * h + gq, r1 = r0 + 8;
                        const int o0 = vimg_off<HD>(r0, colb >> 3) + 2 * (colb & 7);
                        const int o1 = vimg_off<HD>(r1, colb >> 3) + 2 * (colb & 7);
                        const u32x2 lo = __builtin_bit_cast(u32x2, __builtin_amdgcn_ds_read_tr16_b64_v4f16(
                            (__attribute__((address_space(3))) trv4*)(vw + o0)));
                        const u32x2 hi = __builtin_bit_cast(u32x2, __builtin_amdgcn_ds_read_tr16_b64_v4f16(
                            (__attribute__((address_space(3))) trv4*)(vw + o1)));
                        const u32x4 vf = {lo.x, lo.y, hi.x, hi.y};
                        o[b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(as_h8(vf), as_h8(pf[s]), o[b], 0, 0, 0);
                    }
                }
            }
        }
    }

    // ---- the waves' partials, added in a fixed tree: ((0+4)+(2+6)) + ((1+5)+(3+7)) ----------------
    // each partial is [HB][16 registers][64 lanes] f32 = HD * 128 B, inside the writer's V images
    __syncthreads();   // every wave is done with its V image
    float* const red = reinterpret_cast<float*>(vimg);
    for (int hw = NW / 2; hw >= 1; hw >>= 1) {
        if (w >= hw && w < 2 * hw) {
            float* dst = red + (w - hw) * (HD * 32);
#pragma unroll
            for (int b = 0; b < HB; ++b)
#pragma unroll
                for (int r = 0; r < 16; ++r) dst[(b * 16 + r) * 64 + lane] = o[b][r];
        }
        __syncthreads();
        if (w < hw) {
            const float* src = red + w * (HD * 32);
#pragma unroll
            for (int b = 0; b < HB; ++b)
#pragma unroll
                for (int r = 0; r < 16; ++r) o[b][r] += src[(b * 16 + r) * 64 + lane];
        }
        __syncthreads();
    }
    // ---- O^T: lane = token, register r of block b = hd 32b + (r&3) + 8(r>>2) + 4h
    if (w != 0 || !tv) return;
    float* orow = out + (long long)tok * P.n_head * HD + (long long)hq * HD;
#pragma unroll
    for (int b = 0; b < HB; ++b)
#pragma unroll
        for (int q = 0; q < 4; ++q)
            *reinterpret_cast<float4*>(orow + 32 * b + 8 * q + 4 * h) =
                float4{o[b][4 * q], o[b][4 * q + 1], o[b][4 * q + 2], o[b][4 * q + 3]};
}

}  // namespace amf

bool attn_mfma_supported(int head_dim) { return head_dim == 64 || head_dim == 128; }

void launch_attn_mfma(const AttnParams& p, int ntok, float* out, hipStream_t s) {
    if (ntok < 1) return;
    if (p.n_head % p.n_head_kv) throw Error("attn_mfma: n_head must be a multiple of n_head_kv");
    if (p.n_ctx < 4) throw Error("attn_mfma: n_ctx must be at least 4");
    const dim3 grid(p.n_head, (ntok + 31) / 32);
    const size_t lds = (size_t)amf::NW * amf::CH * p.head_dim * 2;
    static bool attr = false;
    if (!attr) {
        MI_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(amf::attn_mfma_kernel<128>), hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024));
        MI_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(amf::attn_mfma_kernel<64>), hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024));
        attr = true;
    }
    if (p.head_dim == 128) hipLaunchKernelGGL(amf::attn_mfma_kernel<128>, grid, dim3(64 * amf::NW), lds, s, p, ntok, out);
    else if (p.head_dim == 64) hipLaunchKernelGGL(amf::attn_mfma_kernel<64>, grid, dim3(64 * amf::NW), lds, s, p, ntok, out);
    else throw Error("attn_mfma: head_dim 64 or 128");
    MI_HIP(hipGetLastError());
}

}  // namespace mi
