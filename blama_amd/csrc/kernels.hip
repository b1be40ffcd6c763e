// HIP kernels for gfx950 (CDNA4, wave64).  Batch-1 decode of a LLaMA-family
// GGUF model: fused quantised GEMVs (Q4_K/Q5_K/Q6_K/Q8_0), RMSNorm, RoPE, KV
// append, attention over the f16 cache, SwiGLU, MoE routing and top-k.
//
// Numerics mirror the ggml CPU path of llama.cpp b5187 (the reference's
// verifier, Model::Params{.gpu=false}, inference/code/llama/Model.cpp:13-16):
// activations are quantised to Q8_K / Q8_0 exactly as quantize_row_q8_K_ref /
// quantize_row_q8_0 do, so every per-block integer dot product equals the
// CPU's bit for bit; only the fp32 accumulation order differs.  The whole
// file is compiled with -ffp-contract=off so that no a*b+c is silently fused
// where ggml rounds twice.
#include "kernels.h"
#include "qdot.h"
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdlib>
#include <cstring>
#include <algorithm>

namespace mi {

// ---------------------------------------------------------------------------
// Batched GEMM (prompt ingestion): gemv_t's weight ring and integer dots, with every
// loaded weight chunk dotted against up to GEMM_NT tokens' activations in LDS.
// Correctness first: the prologue reads its parameters straight from kernarg and
// quantises the NT activation rows without the decode kernel's latency tricks
// (one launch streams the weights once for NT tokens).
// ---------------------------------------------------------------------------
template <int T, int D>
__global__ __launch_bounds__(512) void gemm_t(const GemmParams P) {
    constexpr int NW = 8, NT = GEMM_NT;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    using Kk = Kq<T>;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int sbl = lane >> 3, j = lane & 7;
    const int nb = P.K >> 8;
    const int cpr = (nb + 7) >> 3;
    const int ntok = P.ntok;
    const ActLayout L = act_layout(P.K, P.need_q8k, P.need_q80);
    float* rope = reinterpret_cast<float*>(smem + NT * L.slot_bytes);            // [NT][n_rot/2][2]
    double* red = reinterpret_cast<double*>(rope + NT * ((P.n_rot / 2) * 2 + 2)); // [NT][NW]
    __shared__ int tp_pos[NT], tp_cell[NT];
    if (threadIdx.x < NT) {
        const int t = threadIdx.x < ntok ? threadIdx.x : ntok - 1;
        tp_pos[threadIdx.x] = P.tokpos ? P.tokpos[t * 4 + 1] : 0;
        tp_cell[threadIdx.x] = P.tokpos ? P.tokpos[t * 4 + 2] : 0;
    }
    // ---- prologue: RMSNorm (double sum, ggml order of rounding) + quantisation of NT rows
    const auto w4 = gptr(reinterpret_cast<const f32x4*>(P.norm_w));
    if (P.pro == PRO_RMSNORM) {
        for (int t = 0; t < NT; ++t) {
            double sacc = 0.0;
            if (t < ntok) {
                const auto x4 = gptr(reinterpret_cast<const f32x4*>(P.x + (long long)t * P.x_stride));
                for (int blk = wave; blk < nb; blk += NW) {
                    const f32x4 v = x4[blk * 64 + lane];
                    sacc += (double)(v.x * v.x);
                    sacc += (double)(v.y * v.y);
                    sacc += (double)(v.z * v.z);
                    sacc += (double)(v.w * v.w);
                }
            }
            sacc = wave_sum63_d(sacc);
            if (lane == 63) red[t * NW + wave] = sacc;
        }
    }
    __syncthreads();
    for (int t = 0; t < ntok; ++t) {
        float scale = 1.0f;
        if (P.pro == PRO_RMSNORM) {
            double tot = 0.0;
            for (int w = 0; w < NW; ++w) tot += red[t * NW + w];
            scale = 1.0f / sqrtf((float)(tot / (double)P.K) + P.eps);
        }
        char* base = smem + t * L.slot_bytes;
        const auto x4 = gptr(reinterpret_cast<const f32x4*>(P.x + (long long)t * P.x_stride));
        for (int blk = wave; blk < nb; blk += NW) {
            const f32x4 xv = x4[blk * 64 + lane];
            float v[4] = {xv.x, xv.y, xv.z, xv.w};
            if (P.pro == PRO_RMSNORM) {
                const f32x4 w = w4[blk * 64 + lane];
                v[0] = (v[0] * scale) * w.x;
                v[1] = (v[1] * scale) * w.y;
                v[2] = (v[2] * scale) * w.z;
                v[3] = (v[3] * scale) * w.w;
            }
            if (P.need_q8k)
                quant_q8k_block(v, lane, reinterpret_cast<int8_t*>(base + L.q8k) + blk * 256,
                                reinterpret_cast<int*>(base + L.bsum) + blk * 16,
                                reinterpret_cast<float*>(base + L.dk) + blk);
            if (P.need_q80)
                quant_q80_block(v, lane, reinterpret_cast<int8_t*>(base + L.q80) + blk * 256,
                                reinterpret_cast<float*>(base + L.d0) + blk * 8);
        }
    }
    __syncthreads();
    if (P.n_rot > 0) {   // RoPE table of each token's position (ggml_rope_cache_init)
        for (int t = wave; t < ntok; t += NW) {
            float* rt = rope + t * ((P.n_rot / 2) * 2 + 2);
            for (int i = lane; i < P.n_rot / 2; i += 64) {
                float theta = (float)tp_pos[t];
                for (int kk = 0; kk < i; ++kk) theta = theta * P.theta_scale;
                const float ff = P.freq_factors ? P.freq_factors[i] : 1.0f;
                const float th = P.freq_scale * (theta / ff);
                rt[2 * i] = cosf(th);
                rt[2 * i + 1] = sinf(th);
            }
        }
    }
    __syncthreads();

    // ---- weight stream: the gemv_t ring over this wave's units
    const int W = P.grid * NW;
    int u0, u1;
    unit_range(P.units, W, blockIdx.x * NW + wave, u0, u1);
    const int n_items = (u1 - u0) * cpr;
    const bool adj = P.pair == PAIR_ADJ;
    struct Slot { typename Kk::Ld a, b; };
    Slot ring[D];
    int iu = u0, ic = 0, park = 0;
    const uint8_t* pa[4];
    const uint8_t* pb[4];
    auto bases = [&](int u) {
        const long long ra = adj ? 2LL * u : u;
        long long rb = adj ? ra + 1 : u;
        if (adj && rb >= P.A.rows) rb = ra;   // odd tail: re-read row A, result unused
        const QMat& MB = adj ? P.A : P.B;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            pa[i] = P.A.p[i] + ra * nb * PlaneBytes<T>::b[i];
            pb[i] = MB.p[i] + rb * nb * PlaneBytes<T>::b[i];
        }
    };
    bases(u0 < P.units ? u0 : P.units - 1);
    auto issue = [&](Slot& S) {
        const int sb = park ? 0 : ic * 8 + sbl;
        const int jj = park ? 0 : j;
        S.a = Kk::load(pa, sb, jj);
        S.b = Kk::load(pb, sb, jj);
        if (iu < u1 && ++ic == cpr) {
            ic = 0;
            if (++iu < u1) bases(iu);
            else park = 1;
        }
    };
#pragma unroll
    for (int k = 0; k < D - 1; ++k) issue(ring[k]);

    int cu = u0, cc = 0;
    float accA[NT], accB[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) accA[t] = accB[t] = 0.0f;
    auto consume = [&](const Slot& S) {
        const int sb = cc * 8 + sbl;
        const bool lv = sb < nb;
        const int sbc = lv ? sb : nb - 1;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            if (t < ntok) {
                const typename Kk::AR ar = Kk::act(act_view(smem, L, t), sbc, j);
                const float da = Kk::dot(S.a, ar, j), db = Kk::dot(S.b, ar, j);
                accA[t] += lv ? da : 0.0f;
                accB[t] += lv ? db : 0.0f;
            }
        }
        if (++cc == cpr) {
            const long long ra = adj ? 2LL * cu : cu, rb = adj ? ra + 1 : cu;
            const bool hasB = !adj || rb < P.A.rows;
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                if (t >= ntok) continue;
                const float yA = wave_sum63(accA[t]);
                const float yB = wave_sum63(accB[t]);
                accA[t] = accB[t] = 0.0f;
                if (lane != 63) continue;
                float* out = P.out + (long long)t * P.out_stride;
                const float* res = P.resid ? P.resid + (long long)t * P.out_stride : nullptr;
                switch (P.epi) {
                case EPI_STORE:
                    out[ra] = yA;
                    if (hasB) out[rb] = yB;
                    break;
                case EPI_ADD: {
                    const float r0 = res[ra], r1 = hasB ? res[rb] : 0.0f;
                    out[ra] = yA + r0;
                    if (hasB) out[rb] = yB + r1;
                    break;
                }
                case EPI_ROPE_Q:
                case EPI_ROPE_K: {
                    const float* rt = rope + t * ((P.n_rot / 2) * 2 + 2);
                    const int i0 = (int)(ra % P.head_dim);
                    float o0 = yA, o1 = yB;
                    if (i0 < P.n_rot) {
                        const float cs = rt[i0], sn = rt[i0 + 1];
                        o0 = yA * cs - yB * sn;
                        o1 = yA * sn + yB * cs;
                    }
                    if (P.epi == EPI_ROPE_Q) {
                        out[ra] = o0;
                        out[rb] = o1;
                    } else {
                        __half* kr = P.kcache + (long long)tp_cell[t] * P.kv_dim;
                        kr[ra] = __float2half_rn(o0);
                        kr[rb] = __float2half_rn(o1);
                        if (cu == 0) P.cell_pos[tp_cell[t]] = tp_pos[t];
                    }
                    break;
                }
                case EPI_V: {
                    __half* vr = P.vcache + (long long)tp_cell[t] * P.kv_dim;
                    vr[ra] = __float2half_rn(yA);
                    if (hasB) vr[rb] = __float2half_rn(yB);
                    break;
                }
                case EPI_SWIGLU:
                    out[cu] = silu_f(yA) * yB;
                    break;
                default: break;
                }
            }
            cc = 0;
            ++cu;
        }
    };
    for (int base = 0; base < n_items; base += D) {
#pragma unroll
        for (int k = 0; k < D; ++k) {
            issue(ring[(k + D - 1) % D]);
            if (base + k < n_items) consume(ring[k]);
        }
    }
}

typedef void (*GemmFn)(const GemmParams);
static GemmFn gemm_fn(int type);
void init_gemm_attributes() {
    for (int t : {T_Q4_K, T_Q5_K, T_Q6_K, T_Q8_0})
        MI_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_fn(t)),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024));
}
static GemmFn gemm_fn(int type) {
    switch (type) {
    case T_Q4_K: return gemm_t<T_Q4_K, 4>;
    case T_Q5_K: return gemm_t<T_Q5_K, 4>;
    case T_Q6_K: return gemm_t<T_Q6_K, 4>;
    case T_Q8_0: return gemm_t<T_Q8_0, 4>;
    default: return nullptr;
    }
}

static size_t gemm_smem_bytes(const GemmParams& p) {
    const ActLayout L = act_layout(p.K, p.need_q8k, p.need_q80);
    return (size_t)GEMM_NT * L.slot_bytes + (size_t)GEMM_NT * ((p.n_rot / 2) * 2 + 2) * 4 + GEMM_NT * 8 * 8 + 64;
}

void launch_gemm(const GemmParams& p_in, hipStream_t s) {
    GemmParams p = p_in;
    if (p.K % 256 != 0) throw Error("gemm: K must be a multiple of 256");
    if (p.ntok < 1 || p.ntok > GEMM_NT) throw Error("gemm: 1..GEMM_NT tokens per launch");
    if (p.pair == PAIR_AB && p.B.type != p.A.type) throw Error("gemm: a pair must share its quant type");
    if (p.epi == EPI_MOE_DOWN) throw Error("gemm: MoE launches are served token by token");
    p.need_q8k = p.A.type != T_Q8_0;
    p.need_q80 = p.A.type == T_Q8_0;
    const int g = (p.units + 7) / 8;
    p.grid = g < 1 ? 1 : (g > 256 ? 256 : g);
    if ((long long)p.units * p.grid * 8 >= (1LL << 32)) throw Error("gemm: too many units");
    const size_t smem = gemm_smem_bytes(p);
    if (smem > 150 * 1024) throw Error("gemm: activations of GEMM_NT tokens do not fit LDS");
    GemmFn fn = gemm_fn(p.A.type);
    if (!fn) throw Error("gemm: unsupported quant type");
    hipLaunchKernelGGL(fn, dim3(p.grid), dim3(512), smem, s, p);
    MI_HIP(hipGetLastError());
}


// ---------------------------------------------------------------------------
// Exact ggml dequantisation of one element (dequantize_row_*, ggml-quants.c)
// ---------------------------------------------------------------------------
__device__ __forceinline__ void scale_min_k4(int t, const uint8_t* s, int& sc, int& m) {
    if (t < 4) { sc = s[t] & 63; m = s[t + 4] & 63; }
    else { sc = (s[t + 4] & 0xF) | ((s[t - 4] >> 6) << 4); m = (s[t + 4] >> 4) | ((s[t] >> 6) << 4); }
}

__device__ float dequant_elem(const QMat& M, long long row, int col) {
    const int sb = col >> 8, i = col & 255;
    const long long sbi = row * M.nb + sb;
    switch (M.type) {
    case T_Q4_K:
    case T_Q5_K: {
        const bool q5 = M.type == T_Q5_K;
        const uint8_t* qs = M.p[0] + sbi * 128;
        const uint8_t* hdr = M.p[q5 ? 2 : 1] + sbi * 16;
        const float d = h2f(hdr[0] | (hdr[1] << 8)), dmin = h2f(hdr[2] | (hdr[3] << 8));
        const int c = i >> 6, l = i & 63;
        const int t = 2 * c + (l >= 32);
        const int ll = l & 31;
        int q = (l < 32) ? (qs[32 * c + ll] & 0xF) : (qs[32 * c + ll] >> 4);
        if (q5) {
            const uint8_t* qh = M.p[1] + sbi * 32;
            q += ((qh[ll] >> t) & 1) ? 16 : 0;
        }
        int sc, m;
        scale_min_k4(t, hdr + 4, sc, m);
        const float d1 = d * (float)sc, m1 = dmin * (float)m;
        return d1 * (float)q - m1;
    }
    case T_Q6_K: {
        const uint8_t* ql = M.p[0] + sbi * 128;
        const uint8_t* qh = M.p[1] + sbi * 64;
        const int8_t* sc = reinterpret_cast<const int8_t*>(M.p[2] + sbi * 16);
        const uint8_t* dp = M.p[3] + sbi * 2;
        const float d = h2f(dp[0] | (dp[1] << 8));
        const int h = i >> 7, r = i & 127, quarter = r >> 5, l = r & 31;
        const int is = l / 16;
        const uint8_t L = ql[64 * h + l + ((quarter & 1) ? 32 : 0)];
        const int lo4 = (quarter < 2) ? (L & 0xF) : (L >> 4);
        const int hb = (qh[32 * h + l] >> (2 * quarter)) & 3;
        const int q = (lo4 | (hb << 4)) - 32;
        const int s = sc[8 * h + is + 2 * quarter];
        return (d * (float)s) * (float)q;
    }
    case T_Q8_0: {
        const int8_t q = reinterpret_cast<const int8_t*>(M.p[0] + sbi * 256)[i];
        const uint8_t* dp = M.p[1] + sbi * 16 + (i >> 5) * 2;
        return (float)q * h2f(dp[0] | (dp[1] << 8));
    }
    case T_F32:
        return reinterpret_cast<const float*>(M.p[0])[row * M.K + col];
    case T_F16:
        return __half2float(reinterpret_cast<const __half*>(M.p[0])[row * M.K + col]);
    default:
        return 0.0f;
    }
}

// get_rows(tok_embd, token) (+ get_rows(position_embd, pos) for GPT-2, llm_build_gpt2's
// inpL = ggml_add(tok rows, pos rows))
__global__ void embed_kernel(const EmbedParams P) {
    const long long tok = P.tokpos[0];
    const long long pos = P.tokpos[1];
    if (P.step && blockIdx.x == 0 && threadIdx.x == 0) *P.step += 1u;
    for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < P.n_embd; c += gridDim.x * blockDim.x) {
        const float e = dequant_elem(P.E, tok, c);
        P.out[c] = P.has_pos ? e + dequant_elem(P.P, pos, c) : e;
    }
}

__global__ void embed_multi_kernel(const EmbedParams P) {
    const long long tok = P.tokpos[blockIdx.y * 4];
    const long long pos = P.tokpos[blockIdx.y * 4 + 1];
    float* out = P.out + (long long)blockIdx.y * P.n_embd;
    for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < P.n_embd; c += gridDim.x * blockDim.x) {
        const float e = dequant_elem(P.E, tok, c);
        out[c] = P.has_pos ? e + dequant_elem(P.P, pos, c) : e;
    }
}

void launch_embed_multi(const EmbedParams& p, int ntok, hipStream_t s) {
    hipLaunchKernelGGL(embed_multi_kernel, dim3((p.n_embd + 255) / 256, ntok), dim3(256), 0, s, p);
    MI_HIP(hipGetLastError());
}

void launch_embed(const EmbedParams& p, hipStream_t s) {
    hipLaunchKernelGGL(embed_kernel, dim3((p.n_embd + 255) / 256), dim3(256), 0, s, p);
    MI_HIP(hipGetLastError());
}

__global__ void dequant_rows_kernel(const QMat M, int row0, int nrows, float* out) {
    const long long n = (long long)nrows * M.K;
    for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x)
        out[e] = dequant_elem(M, row0 + e / M.K, (int)(e % M.K));
}

void launch_dequant_rows(const QMat& m, int row0, int nrows, float* out, hipStream_t s) {
    long long n = (long long)nrows * m.K;
    int grid = (int)std::min<long long>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(dequant_rows_kernel, dim3(grid), dim3(256), 0, s, m, row0, nrows, out);
    MI_HIP(hipGetLastError());
}

__global__ void quantize_q8k_kernel(const float* x, int K, int8_t* q, float* d, int* bsums) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int blk = blockIdx.x * (blockDim.x >> 6) + wave;
    if (blk >= K / 256) return;
    const float4 xv = reinterpret_cast<const float4*>(x)[blk * 64 + lane];
    const float v[4] = {xv.x, xv.y, xv.z, xv.w};
    quant_q8k_block(v, lane, q + blk * 256, bsums + blk * 16, d + blk);
}

void launch_quantize_q8k(const float* x, int K, int8_t* q, float* d, int* bsums, hipStream_t s) {
    const int nb = K / 256;
    hipLaunchKernelGGL(quantize_q8k_kernel, dim3((nb + 3) / 4), dim3(256), 0, s, x, K, q, d, bsums);
    MI_HIP(hipGetLastError());
}

// ---------------------------------------------------------------------------
// Attention of one query token over the f16 cache, split over cells, in two
// launches so that the softmax weights can be rounded exactly as the CPU graph
// rounds them (non-flash path, Instance.hpp:25 flash_attn=false):
//   KQ  = ggml_mul_mat(k, q):  q is converted to the f16 vec_dot_type, s = k.q
//   ggml_soft_max_ext(KQ, mask, 1/sqrt(hd)): w = s*scale, e = expf(w - max),
//        sum in double, p = e * (float)(1/sum)
//   KQV = ggml_mul_mat(v, kq): p is converted to f16, o = sum_c f16(p_c) v_c
// Rounding p to f16 needs the head's global max and sum before any weight is
// formed, so:
//   attn_scores_kernel  grid (n_head_kv, ATTN_SMAX): split s writes w_c of its
//                       cells for the R = n_head/n_head_kv query heads of kv
//                       head g, and the split's max per head.
//   attn_pv_kernel      same grid: global max from the split maxes, the sum of
//                       expf(w - max) over ALL cells (every split recomputes it
//                       in the same fixed order -> identical in every split),
//                       then sum_c f16(p_c) v_c over its own cells -> part_o.
// The WO GEMV's PRO_ATTN prologue adds the splits' partials in split order.
// Only the order of the fp32 sums differs from the CPU's.
// Lane layout: LPC = head_dim/8 lanes hold one cache row (8 halves = one
// 16-byte load each); a wave covers CPW = 64/LPC cells per step.
// ---------------------------------------------------------------------------
// U: cell steps whose cache loads are in flight together.  The first step's loads are issued at
// entry, ahead of the loads the arithmetic waits on first (q; the split maxima and scores), so
// the cache round trip overlaps them.
template <int R, int LPC, int U>
__global__ __launch_bounds__(256) void attn_scores_kernel(const AttnParams P) {
    constexpr int CPW = 64 / LPC;
    constexpr int HD = LPC * 8;
    __shared__ float red[4][R];
    // kv head, and the first of the R q heads this workgroup serves (qsplit: one q head each)
    const int g = P.qsplit ? (int)blockIdx.x / P.qsplit : (int)blockIdx.x, s = blockIdx.y;
    const int gq = P.qsplit ? (int)blockIdx.x : (int)blockIdx.x * R;
#ifdef MI_STAMPS
    unsigned long long* const stp = P.stamps ? P.stamps + (blockIdx.y * gridDim.x + blockIdx.x) * 8 : nullptr;
    if (stp && threadIdx.x == 0) stp[0] = __builtin_amdgcn_s_memrealtime();
#endif
    const int ncell = P.tokpos[2] + 1, qpos = P.tokpos[1];
    int chunk, nsplit;
    attn_split(ncell, chunk, nsplit);
    if (s >= nsplit) return;
    const int c0 = s * chunk, c1 = min(ncell, c0 + chunk);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int L = lane % LPC, G = lane / LPC;
    const long long row_off = (long long)g * HD + L * 8;
    u32x4 kk[U];
    int cpos[U];
    auto fetch = [&](int cb) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int c = cb + u * 4 * CPW + G;
            c = c < c1 ? c : c1 - 1;
            kk[u] = *reinterpret_cast<const u32x4*>(P.kcache + (long long)c * P.kv_dim + row_off);
            cpos[u] = P.cell_pos[c];
        }
    };
    fetch(c0 + wave * CPW);
    float q[R][8];
#pragma unroll
    for (int t = 0; t < R; ++t) {
        const float4* qp = reinterpret_cast<const float4*>(P.q + (long long)(gq + t) * HD + L * 8);
        const float4 a = qp[0], b = qp[1];
        const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) q[t][e] = __half2float(__float2half_rn(v[e]));
    }
    float mx[R];
#pragma unroll
    for (int t = 0; t < R; ++t) mx[t] = -INFINITY;
    for (int cb = c0 + wave * CPW; cb < c1; cb += 4 * CPW * U) {
        if (cb != c0 + wave * CPW) fetch(cb);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int c = cb + u * 4 * CPW + G;
            const bool valid = c < c1 && cpos[u] <= qpos;
            const unsigned kw[4] = {kk[u].x, kk[u].y, kk[u].z, kk[u].w};
            float kf[8];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                kf[2 * e] = h2f(kw[e]);
                kf[2 * e + 1] = h2f(kw[e] >> 16);
            }
#pragma unroll
            for (int t = 0; t < R; ++t) {
                float d = 0.0f;
#pragma unroll
                for (int e = 0; e < 8; ++e) d = fmaf(q[t][e], kf[e], d);
#pragma unroll
                for (int off = LPC / 2; off > 0; off >>= 1) d += __shfl_xor(d, off, 64);
                const float w = valid ? d * P.scale : -INFINITY;
                mx[t] = fmaxf(mx[t], w);
                if (L == 0 && c < c1) P.scores[(long long)(gq + t) * P.n_ctx + c] = w;
            }
        }
    }
#pragma unroll
    for (int t = 0; t < R; ++t) {
        const float m = wave_max(mx[t]);
        if (lane == 0) red[wave][t] = m;
    }
    __syncthreads();
    if (threadIdx.x < R) {
        const int t = threadIdx.x;
        const float m = fmaxf(fmaxf(red[0][t], red[1][t]), fmaxf(red[2][t], red[3][t]));
        P.smax[s * P.n_head + gq + t] = m;
    }
#ifdef MI_STAMPS
    if (stp && threadIdx.x == 0) stp[4] = __builtin_amdgcn_s_memrealtime();
#endif
}

template <int R, int LPC, int U>
__global__ __launch_bounds__(256) void attn_pv_kernel(const AttnParams P) {
    constexpr int CPW = 64 / LPC;
    constexpr int HD = LPC * 8;
    __shared__ double dred[4][R];
    __shared__ float gm[R], ginv[R];
    __shared__ float red_o[4][R][HD];
    // kv head, and the first of the R q heads this workgroup serves (qsplit: one q head each)
    const int g = P.qsplit ? (int)blockIdx.x / P.qsplit : (int)blockIdx.x, s = blockIdx.y;
    const int gq = P.qsplit ? (int)blockIdx.x : (int)blockIdx.x * R;
#ifdef MI_STAMPS
    unsigned long long* const stp = P.stamps2 ? P.stamps2 + (blockIdx.y * gridDim.x + blockIdx.x) * 8 : nullptr;
    if (stp && threadIdx.x == 0) stp[0] = __builtin_amdgcn_s_memrealtime();
#endif
    const int ncell = P.tokpos[2] + 1;
    int chunk, nsplit;
    attn_split(ncell, chunk, nsplit);
    if (s >= nsplit) return;
    const int c0 = s * chunk, c1 = min(ncell, c0 + chunk);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int L = lane % LPC, G = lane / LPC;
    const long long row_off = (long long)g * HD + L * 8;
    u32x4 vv[U];
    auto fetch = [&](int cb) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int c = cb + u * 4 * CPW + G;
            c = c < c1 ? c : c1 - 1;
            vv[u] = *reinterpret_cast<const u32x4*>(P.vcache + (long long)c * P.kv_dim + row_off);
        }
    };
    fetch(c0 + wave * CPW);   // in flight while the softmax statistics are formed
    // global max of every head of the group
    float M[R];
#pragma unroll
    for (int t = 0; t < R; ++t) {
        float m = -INFINITY;
        for (int k = 0; k < nsplit; ++k) m = fmaxf(m, P.smax[k * P.n_head + gq + t]);
        M[t] = m;
    }
    // sum over all cells of expf(w - max), in double, fixed order
#pragma unroll
    for (int t = 0; t < R; ++t) {
        const float* w = P.scores + (long long)(gq + t) * P.n_ctx;
        double acc = 0.0;
        for (int c = tid; c < ncell; c += 256) acc += (double)expf(w[c] - M[t]);
        acc = wave_sum_d(acc);
        if (lane == 0) dred[wave][t] = acc;
    }
    __syncthreads();
    if (tid < R) {
        const double tot = ((dred[0][tid] + dred[1][tid]) + dred[2][tid]) + dred[3][tid];
        ginv[tid] = (float)(1.0 / tot);
        gm[tid] = M[tid];
    }
    __syncthreads();
    float o[R][8];
#pragma unroll
    for (int t = 0; t < R; ++t)
#pragma unroll
        for (int e = 0; e < 8; ++e) o[t][e] = 0.0f;
    for (int cb = c0 + wave * CPW; cb < c1; cb += 4 * CPW * U) {
        if (cb != c0 + wave * CPW) fetch(cb);
        float pw[U][R];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int c = cb + u * 4 * CPW + G;
            const bool in = c < c1;
            c = in ? c : c1 - 1;
#pragma unroll
            for (int t = 0; t < R; ++t) {
                const float w = P.scores[(long long)(gq + t) * P.n_ctx + c];
                // ggml_vec_soft_max_f32 then the f16 vec_dot_type conversion of KQV's src1
                const float p = expf(w - gm[t]) * ginv[t];
                pw[u][t] = in ? __half2float(__float2half_rn(p)) : 0.0f;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const unsigned vw[4] = {vv[u].x, vv[u].y, vv[u].z, vv[u].w};
            float vf[8];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                vf[2 * e] = h2f(vw[e]);
                vf[2 * e + 1] = h2f(vw[e] >> 16);
            }
#pragma unroll
            for (int t = 0; t < R; ++t)
#pragma unroll
                for (int e = 0; e < 8; ++e) o[t][e] = fmaf(pw[u][t], vf[e], o[t][e]);
        }
    }
    // sum the CPW cell groups of the wave, then the 4 waves in fixed order
#pragma unroll
    for (int t = 0; t < R; ++t)
#pragma unroll
        for (int off = LPC; off < 64; off <<= 1)
#pragma unroll
            for (int e = 0; e < 8; ++e) o[t][e] += __shfl_xor(o[t][e], off, 64);
    if (G == 0) {
#pragma unroll
        for (int t = 0; t < R; ++t)
#pragma unroll
            for (int e = 0; e < 8; ++e) red_o[wave][t][L * 8 + e] = o[t][e];
    }
    __syncthreads();
    for (int i = tid; i < R * HD; i += 256) {
        const int t = i / HD, d = i % HD;
        const float acc = ((red_o[0][t][d] + red_o[1][t][d]) + red_o[2][t][d]) + red_o[3][t][d];
        P.part_o[((long long)s * P.n_head + gq + t) * HD + d] = acc;
    }
#ifdef MI_STAMPS
    if (stp && threadIdx.x == 0) stp[4] = __builtin_amdgcn_s_memrealtime();
#endif
}

// Contexts past ATTN_SHORT cells in ONE launch: grid (n_head, ATTN_SMAX), one q head per
// workgroup row, split s of the head's cells per column (attn_split's chunks).  The split keeps its
// scaled scores in LDS; the splits of a head exchange their maxima, then their partial sums of
// expf(w - M) in double, through flag lines (agent-scope stores, bounded polls), so every split
// rounds p = f16(expf(w - M) * (1/S)) with the head's global M and S -- the CPU graph's softmax --
// without the scores' round trip through global memory and the second launch of
// attn_scores_kernel / attn_pv_kernel.  The V chunk's loads are issued before the exchange.
// The splits of one head are co-resident (n_head * 16 workgroups of 4 waves fit the chip many
// times over); a poll gives up after 2 s and flags the step invalid (xerr) instead of hanging.
__device__ __forceinline__ unsigned ld_ag(const unsigned* p) {
    return __hip_atomic_load(const_cast<unsigned*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <int LPC>
__global__ __launch_bounds__(256) void attn_long_kernel(const AttnParams P) {
    constexpr int CPW = 64 / LPC;
    constexpr int HD = LPC * 8;
    constexpr int U = 4;
    extern __shared__ __attribute__((aligned(16))) float sw[];   // [chunk] scaled scores
    __shared__ float redm[4];
    __shared__ double dred[4];
    __shared__ float stat[2];                                     // M, inv
    __shared__ float red_o[4][HD];
    const int h = blockIdx.x, s = blockIdx.y;
    const int g = h / (P.n_head / P.n_head_kv);
    const int ncell = P.tokpos[2] + 1, qpos = P.tokpos[1];
    int chunk, nsplit;
    attn_split(ncell, chunk, nsplit);
    if (s >= nsplit) return;
    const int c0 = s * chunk, c1 = min(ncell, c0 + chunk);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int L = lane % LPC, G = lane / LPC;
    const long long row_off = (long long)g * HD + L * 8;
    // strictly increasing over (step, layer, phase) for any depth
    const unsigned epoch = *P.step * (2u * (unsigned)max(P.n_layer, 1) + 2u) + 2u * (unsigned)P.layer;
    unsigned* const fl = P.xflags + (long long)h * ATTN_SMAX * 32;
    u32x4 kk[U];
    int cpos[U];
    auto fetch_k = [&](int cb) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int c = cb + u * 4 * CPW + G;
            c = c < c1 ? c : c1 - 1;
            kk[u] = *reinterpret_cast<const u32x4*>(P.kcache + (long long)c * P.kv_dim + row_off);
            cpos[u] = P.cell_pos[c];
        }
    };
    fetch_k(c0 + wave * CPW);
    float q[8];
    {
        const float4* qp = reinterpret_cast<const float4*>(P.q + (long long)h * HD + L * 8);
        const float4 a = qp[0], b = qp[1];
        const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) q[e] = __half2float(__float2half_rn(v[e]));
    }
    // 1. scaled KQ of the split's cells into LDS, the split's max
    float mx = -INFINITY;
    for (int cb = c0 + wave * CPW; cb < c1; cb += 4 * CPW * U) {
        if (cb != c0 + wave * CPW) fetch_k(cb);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int c = cb + u * 4 * CPW + G;
            const bool valid = c < c1 && cpos[u] <= qpos;
            const unsigned kw[4] = {kk[u].x, kk[u].y, kk[u].z, kk[u].w};
            float d = 0.0f;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                d = fmaf(q[2 * e], h2f(kw[e]), d);
                d = fmaf(q[2 * e + 1], h2f(kw[e] >> 16), d);
            }
#pragma unroll
            for (int off = LPC / 2; off > 0; off >>= 1) d += __shfl_xor(d, off, 64);
            const float w = valid ? d * P.scale : -INFINITY;
            mx = fmaxf(mx, w);
            if (L == 0 && c < c1) sw[c - c0] = w;
        }
    }
    // the V chunk a wave reads first: waves 1-3 issue it before the exchange; wave 0, which polls,
    // after it (vmcnt retires in issue order: a flag load would wait behind it)
    u32x4 vv[U];
    auto fetch_v = [&](int cb) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int c = cb + u * 4 * CPW + G;
            c = c < c1 ? c : c1 - 1;
            vv[u] = *reinterpret_cast<const u32x4*>(P.vcache + (long long)c * P.kv_dim + row_off);
        }
    };
    mx = wave_max(mx);
    if (lane == 0) redm[wave] = mx;
    __syncthreads();
    // publish this split's value of phase ph (stored by thread 0 before), then wait for every
    // split's (wave 0); false after a timeout
    auto exchange = [&](int ph) -> bool {
        bool ok = true;
        if (wave == 0) {
            const unsigned tgt = epoch + 1u + (unsigned)ph;
            if (lane == 0) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the value's store completed
                __hip_atomic_store(fl + s * 32, tgt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            for (;;) {
                const unsigned f = lane < nsplit ? ld_ag(fl + lane * 32) : tgt;
                if (__all((int)(f - tgt) >= 0)) break;
                if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {
                    ok = false;
                    if (lane == 0 && P.xerr) __hip_atomic_store(P.xerr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    break;
                }
            }
            asm volatile("" ::: "memory");
        }
        return ok;
    };
    if (tid == 0) {
        const float m = fmaxf(fmaxf(redm[0], redm[1]), fmaxf(redm[2], redm[3]));
        __hip_atomic_store(P.xmax + h * ATTN_SMAX + s, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (wave != 0) fetch_v(c0 + wave * CPW);
    exchange(0);
    if (wave == 0) {
        float m = lane < nsplit ? __hip_atomic_load(P.xmax + h * ATTN_SMAX + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                : -INFINITY;
        m = wave_max(m);
        if (lane == 0) stat[0] = m;
    }
    __syncthreads();
    const float M = stat[0];
    // 2. the split's sum of expf(w - M) in double; the head's sum in split order
    double acc = 0.0;
    for (int c = c0 + tid; c < c1; c += 256) acc += (double)expf(sw[c - c0] - M);
    acc = wave_sum_d(acc);
    if (lane == 0) dred[wave] = acc;
    __syncthreads();
    if (tid == 0) {
        const double ss = ((dred[0] + dred[1]) + dred[2]) + dred[3];
        __hip_atomic_store(P.xsum + h * ATTN_SMAX + s, ss, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    exchange(1);
    if (tid == 0) {
        double v[ATTN_SMAX];
#pragma unroll
        for (int k = 0; k < ATTN_SMAX; ++k)
            v[k] = k < nsplit ? __hip_atomic_load(P.xsum + h * ATTN_SMAX + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0;
        double tot = 0.0;
        for (int k = 0; k < nsplit; ++k) tot += v[k];
        stat[1] = (float)(1.0 / tot);
    }
    if (wave == 0) fetch_v(c0 + wave * CPW);
    __syncthreads();
    const float inv = stat[1];
    // 3. sum over the split's cells of f16(p_c) v_c
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = 0.0f;
    for (int cb = c0 + wave * CPW; cb < c1; cb += 4 * CPW * U) {
        if (cb != c0 + wave * CPW) fetch_v(cb);
        float pw[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int c = cb + u * 4 * CPW + G;
            const bool in = c < c1;
            const float p = expf(sw[(in ? c : c1 - 1) - c0] - M) * inv;   // ggml_vec_soft_max_f32, f16 vec_dot_type
            pw[u] = in ? __half2float(__float2half_rn(p)) : 0.0f;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const unsigned vw[4] = {vv[u].x, vv[u].y, vv[u].z, vv[u].w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                o[2 * e] = fmaf(pw[u], h2f(vw[e]), o[2 * e]);
                o[2 * e + 1] = fmaf(pw[u], h2f(vw[e] >> 16), o[2 * e + 1]);
            }
        }
    }
#pragma unroll
    for (int off = LPC; off < 64; off <<= 1)
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] += __shfl_xor(o[e], off, 64);
    if (G == 0) {
#pragma unroll
        for (int e = 0; e < 8; ++e) red_o[wave][L * 8 + e] = o[e];
    }
    __syncthreads();
    for (int d = tid; d < HD; d += 256)
        P.part_o[((long long)s * P.n_head + h) * HD + d] = ((red_o[0][d] + red_o[1][d]) + red_o[2][d]) + red_o[3][d];
}

// Short contexts (<= ATTN_SHORT cells): the same arithmetic as the two kernels above with a
// single split, in one launch.  One workgroup per kv head keeps its scores in LDS, so no
// other workgroup's result is needed between the softmax statistics and the PV sum.
// HG > 1 (the streaming decode step): HG such groups of 4 waves in one workgroup, one kv head (or,
// qsplit, one q head) each, so that a workgroup's R * HG q heads cover whole 256-blocks of the
// output, which it then also quantises into P.act_out (the WO launch's activation).
template <int R, int LPC, int HG>
__global__ __launch_bounds__(256 * HG) void attn_fused_kernel(const AttnParams P) {
    constexpr int CPW = 64 / LPC;
    constexpr int HD = LPC * 8;
    __shared__ float sw[HG][R][ATTN_SHORT];
    __shared__ float redm[HG][4][R];
    __shared__ double dred[HG][4][R];
    __shared__ float gm[HG][R], ginv[HG][R];
    __shared__ float red_o[HG][4][R][HD];
    const int grp = (int)threadIdx.x >> 8;
    const int unit = (int)blockIdx.x * HG + grp;   // this group's kv head (qsplit: q head)
    // kv head, and the first of the R q heads this group serves (qsplit: one q head each)
    const int g = P.qsplit ? unit / P.qsplit : unit;
    const int gq = P.qsplit ? unit : unit * R;
    const int tok = blockIdx.y;   // query token (launch_attn_multi); 0 for a decode step
#ifdef MI_STAMPS
    unsigned long long* const stp = P.stamps && tok == 0 ? P.stamps + blockIdx.x * 8 : nullptr;
    if (stp && threadIdx.x == 0) stp[0] = __builtin_amdgcn_s_memrealtime();
#endif
    const int* tp = P.tokpos + 4 * tok;
    const int tp2 = tp[2], qpos = tp[1];
    const float* qrow = P.q + (long long)tok * P.n_head * HD;
    float* orow = P.part_o + (long long)tok * P.n_head * HD;
    const int tid = threadIdx.x & 255, lane = tid & 63, wave = tid >> 6;
    const int L = lane % LPC, G = lane / LPC;
    const long long row_off = (long long)g * HD + L * 8;
    constexpr int U = 4;
    // The first chunk of K, V and cell positions is fetched at entry, before the cell count
    // arrives, so the token-position, K and V round trips overlap instead of chaining.  Cells
    // past the count are clamped to the cache and masked by select below, never by arithmetic.
    // (the first TWO chunks of a wave: a decode step within 128 cells makes no dependent cache
    // round trip after entry)
    constexpr int STRIDE = 4 * CPW * U;   // cells between a wave's chunks
    u32x4 k0[U], v0[U], k1[U], v1[U];
    int cp0[U], cp1[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int c = min(wave * CPW + u * 4 * CPW + G, P.n_ctx - 1);
        const int c1 = min(wave * CPW + STRIDE + u * 4 * CPW + G, P.n_ctx - 1);
        k0[u] = *reinterpret_cast<const u32x4*>(P.kcache + (long long)c * P.kv_dim + row_off);
        v0[u] = *reinterpret_cast<const u32x4*>(P.vcache + (long long)c * P.kv_dim + row_off);
        cp0[u] = P.cell_pos[c];
        k1[u] = *reinterpret_cast<const u32x4*>(P.kcache + (long long)c1 * P.kv_dim + row_off);
        v1[u] = *reinterpret_cast<const u32x4*>(P.vcache + (long long)c1 * P.kv_dim + row_off);
        cp1[u] = P.cell_pos[c1];
    }
    const int ncell = min(tp2 + 1, ATTN_SHORT);
    float q[R][8];
#pragma unroll
    for (int t = 0; t < R; ++t) {
        const float4* qp = reinterpret_cast<const float4*>(qrow + (long long)(gq + t) * HD + L * 8);
        const float4 a = qp[0], b = qp[1];
        const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) q[t][e] = __half2float(__float2half_rn(v[e]));
    }
    // 1. scaled KQ of every cell into LDS, and the per-head max
    float mx[R];
#pragma unroll
    for (int t = 0; t < R; ++t) mx[t] = -INFINITY;
    for (int cb = wave * CPW; cb < ncell; cb += 4 * CPW * U) {
        u32x4 kk[U];
        int cpos[U];
        if (cb == wave * CPW) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                kk[u] = k0[u];
                cpos[u] = cp0[u];
            }
        } else if (cb == wave * CPW + STRIDE) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                kk[u] = k1[u];
                cpos[u] = cp1[u];
            }
        } else {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                int c = cb + u * 4 * CPW + G;
                c = c < ncell ? c : ncell - 1;
                kk[u] = *reinterpret_cast<const u32x4*>(P.kcache + (long long)c * P.kv_dim + row_off);
                cpos[u] = P.cell_pos[c];
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int c = cb + u * 4 * CPW + G;
            const bool valid = c < ncell && cpos[u] <= qpos;
            const unsigned kw[4] = {kk[u].x, kk[u].y, kk[u].z, kk[u].w};
            float kf[8];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                kf[2 * e] = h2f(kw[e]);
                kf[2 * e + 1] = h2f(kw[e] >> 16);
            }
#pragma unroll
            for (int t = 0; t < R; ++t) {
                float d = 0.0f;
#pragma unroll
                for (int e = 0; e < 8; ++e) d = fmaf(q[t][e], kf[e], d);
#pragma unroll
                for (int off = LPC / 2; off > 0; off >>= 1) d += __shfl_xor(d, off, 64);
                const float w = valid ? d * P.scale : -INFINITY;
                mx[t] = fmaxf(mx[t], w);
                if (L == 0 && c < ncell) sw[grp][t][c] = w;
            }
        }
    }
#pragma unroll
    for (int t = 0; t < R; ++t) {
        const float m = wave_max(mx[t]);
        if (lane == 0) redm[grp][wave][t] = m;
    }
    __syncthreads();
    // 2. sum over all cells of expf(w - max), in double, fixed order (as attn_pv_kernel)
#pragma unroll
    for (int t = 0; t < R; ++t) {
        const float M = fmaxf(fmaxf(redm[grp][0][t], redm[grp][1][t]), fmaxf(redm[grp][2][t], redm[grp][3][t]));
        double acc = 0.0;
        for (int c = tid; c < ncell; c += 256) acc += (double)expf(sw[grp][t][c] - M);
        acc = wave_sum_d(acc);
        if (lane == 0) dred[grp][wave][t] = acc;
        if (tid == 0) gm[grp][t] = M;
    }
    __syncthreads();
    if (tid < R) ginv[grp][tid] = (float)(1.0 / (((dred[grp][0][tid] + dred[grp][1][tid]) + dred[grp][2][tid]) + dred[grp][3][tid]));
    __syncthreads();
    // 3. sum_c f16(p_c) v_c
    float o[R][8];
#pragma unroll
    for (int t = 0; t < R; ++t)
#pragma unroll
        for (int e = 0; e < 8; ++e) o[t][e] = 0.0f;
    for (int cb = wave * CPW; cb < ncell; cb += 4 * CPW * U) {
        u32x4 vv[U];
        float pw[U][R];
        const bool first = cb == wave * CPW, second = cb == wave * CPW + STRIDE;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int c = cb + u * 4 * CPW + G;
            const bool in = c < ncell;
            c = in ? c : ncell - 1;
            if (first || second) {   // prefetched at entry; a cell past the count may hold non-finite bits
                const u32x4 z = {0u, 0u, 0u, 0u};
                vv[u] = in ? (first ? v0[u] : v1[u]) : z;
            } else {
                vv[u] = *reinterpret_cast<const u32x4*>(P.vcache + (long long)c * P.kv_dim + row_off);
            }
#pragma unroll
            for (int t = 0; t < R; ++t) {
                const float p = expf(sw[grp][t][c] - gm[grp][t]) * ginv[grp][t];
                pw[u][t] = in ? __half2float(__float2half_rn(p)) : 0.0f;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const unsigned vw[4] = {vv[u].x, vv[u].y, vv[u].z, vv[u].w};
            float vf[8];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                vf[2 * e] = h2f(vw[e]);
                vf[2 * e + 1] = h2f(vw[e] >> 16);
            }
#pragma unroll
            for (int t = 0; t < R; ++t)
#pragma unroll
                for (int e = 0; e < 8; ++e) o[t][e] = fmaf(pw[u][t], vf[e], o[t][e]);
        }
    }
#pragma unroll
    for (int t = 0; t < R; ++t)
#pragma unroll
        for (int off = LPC; off < 64; off <<= 1)
#pragma unroll
            for (int e = 0; e < 8; ++e) o[t][e] += __shfl_xor(o[t][e], off, 64);
    if (G == 0) {
#pragma unroll
        for (int t = 0; t < R; ++t)
#pragma unroll
            for (int e = 0; e < 8; ++e) red_o[grp][wave][t][L * 8 + e] = o[t][e];
    }
    __syncthreads();
    for (int i = tid; i < R * HD; i += 256) {
        const int t = i / HD, d = i % HD;
        orow[(long long)(gq + t) * HD + d] = ((red_o[grp][0][t][d] + red_o[grp][1][t][d]) + red_o[grp][2][t][d]) + red_o[grp][3][t][d];
    }
    if ((P.act_out.act && gridDim.y == 1) || P.act_q8.q) {
        // the WO launch's quantised activation: this workgroup's R * HG heads are whole 256-blocks
        // (launch_attn / launch_attn_multi check), one wave per block; element e of the workgroup's
        // span lies in group e / (R * HD), head (e / HD) % R.  A decode step writes act_layout
        // (act_out); a short batch, token blockIdx.y's row of the batch GEMMs' format (act_q8)
        constexpr int NE = HG * R * HD;
        const int e0 = (int)blockIdx.x * HG * (P.qsplit ? 1 : R) * HD;
        const int gw = (int)threadIdx.x >> 6;
        for (int b = gw; b < NE / 256; b += 4 * HG) {
            float v[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int e = b * 256 + lane * 4 + k, gg = e / (R * HD), t = (e / HD) % R, d = e % HD;
                v[k] = ((red_o[gg][0][t][d] + red_o[gg][1][t][d]) + red_o[gg][2][t][d]) + red_o[gg][3][t][d];
            }
            if (P.act_q8.q) quant_actq8_block(P.act_q8, tok, e0 / 256 + b, v, lane);
            else dv_quant_block(P.act_out, e0 / 256 + b, v, lane);
        }
    }
#ifdef MI_STAMPS
    if (stp && threadIdx.x == 0) stp[4] = __builtin_amdgcn_s_memrealtime();
#endif
}

// The streaming decode step's attention (one token, contexts within ATTN_SHORT cells, the output
// quantised into P.act_out): attn_fused_kernel's arithmetic for one q head per group (R = 1: a kv
// head per group, or a q head of a GQA kv head with qsplit), with NWV waves per group -- twice the
// fused kernel's 4, so each wave walks half the cells -- and the score reductions on DPP (the
// fused kernel's ds_bpermute shuffles were one LDS round trip each).  f16(q) . k over the f16
// cache, scale, causal mask by cell position, the exact softmax (global max; the double sum of
// expf(w - max); p = f16(e * (1/sum))), sum_c f16(p_c) v_c; then whole 256-blocks of the output
// (HG groups) quantised as the WO launch's activation.
template <int CTRL, int RMASK>
__device__ __forceinline__ float dppf(float v, float old) {
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(v), CTRL, RMASK, 0xf, false));
}
// max over the wave of any floats (-inf identity), every lane
__device__ __forceinline__ float wave_max_any(float v) {
    const float ni = -INFINITY;
    v = fmaxf(v, dppf<0x111, 0xf>(v, ni));
    v = fmaxf(v, dppf<0x112, 0xf>(v, ni));
    v = fmaxf(v, dppf<0x114, 0xf>(v, ni));
    v = fmaxf(v, dppf<0x118, 0xf>(v, ni));
    v = fmaxf(v, dppf<0x142, 0xa>(v, ni));
    v = fmaxf(v, dppf<0x143, 0xc>(v, ni));
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
template <int LPC, int HG, int NWV>
__global__ __launch_bounds__(64 * NWV * HG) void attn_dec_kernel(const AttnParams P) {
    static_assert(LPC == 8 || LPC == 16, "head_dim 64 or 128");
    constexpr int HD = LPC * 8, CPW = 64 / LPC, NT = 64 * NWV, STEP = NWV * CPW;
    // the steps of the first 128 cells: q, then the cache rows and positions, requested at entry
    // (buffer loads parked past the descriptor for steps at or past ncell: zeros, no memory
    // access; K before V, which is needed last); past that, a loop.  The depth barely matters:
    // 1, 2, 3 and 4 steps (32-128 cells at 8 waves) measured within 0.8 % of each other, the
    // first 256 cells at entry 1-2 % slower (profiles/r06_fuse_ab.txt)
    constexpr int UM = (128 + STEP - 1) / STEP;
    __shared__ float sw[HG][ATTN_SHORT];
    __shared__ float redm[HG][NWV];
    __shared__ double dred[HG][NWV];
    __shared__ float red_o[HG][NWV][HD];
    const int grp = (int)threadIdx.x / NT;
    const int tid = (int)threadIdx.x % NT, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int unit = (int)blockIdx.x * HG + grp;   // this group's q head
    const int g = P.qsplit ? unit / P.qsplit : unit;   // its kv head
    const int L = lane % LPC, G = lane / LPC;
    const int tok = blockIdx.y;   // query token of a short batch (launch_attn_multi); 0 for a decode step
    const int tp2 = P.tokpos[4 * tok + 2], qpos = P.tokpos[4 * tok + 1];
    const int ncell = min(tp2 + 1, ATTN_SHORT);
    float q[8];
    const float* qrow = P.q + (long long)tok * P.n_head * HD;
    const f32x4 qa = gptr(reinterpret_cast<const f32x4*>(qrow + (long long)unit * HD + L * 8))[0];
    const f32x4 qb = gptr(reinterpret_cast<const f32x4*>(qrow + (long long)unit * HD + L * 8))[1];
    const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc(const_cast<__half*>(rfl_ptr(P.kcache + (long long)g * HD)), 0, 0x7FFFFFFF, 0x00020000);
    const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(const_cast<__half*>(rfl_ptr(P.vcache + (long long)g * HD)), 0, 0x7FFFFFFF, 0x00020000);
    const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(const_cast<int*>(P.cell_pos), 0, 0x7FFFFFFF, 0x00020000);
    u32x4 k0[UM], v0[UM];
    int cp0[UM];
    unsigned ko[UM];
#pragma unroll
    for (int u = 0; u < UM; ++u) {
        const bool park = wave * CPW + u * STEP >= ncell;
        const unsigned c = (unsigned)min(wave * CPW + u * STEP + G, ncell - 1);
        ko[u] = oob((c * (unsigned)P.kv_dim + (unsigned)L * 8u) * 2u, park);
        k0[u] = __builtin_amdgcn_raw_buffer_load_b128(rk, ko[u], 0, 0);
        cp0[u] = (int)__builtin_amdgcn_raw_buffer_load_b32(rc, oob(c * 4u, park), 0, 0);
    }
#pragma unroll
    for (int u = 0; u < UM; ++u) v0[u] = __builtin_amdgcn_raw_buffer_load_b128(rv, ko[u], 0, 0);
    {
        const float t[8] = {qa.x, qa.y, qa.z, qa.w, qb.x, qb.y, qb.z, qb.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) q[e] = __half2float(__float2half_rn(t[e]));
    }
    auto cvt8 = [](const u32x4& w, float (&f)[8]) {
        const unsigned ww[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            f[2 * e] = h2f(ww[e]);
            f[2 * e + 1] = h2f(ww[e] >> 16);
        }
    };
    // 1. scaled KQ of every cell into LDS (lane L == 0 of each cell's group), the wave's maximum
    float mx = -INFINITY;
    auto score = [&](int c, const u32x4& kk, int cp) {
        float kf[8];
        cvt8(kk, kf);
        float d = 0.0f;
#pragma unroll
        for (int e = 0; e < 8; ++e) d = fmaf(q[e], kf[e], d);
        d += dppf<0xB1, 0xf>(d, 0.0f);    // quad_perm [1,0,3,2]
        d += dppf<0x4E, 0xf>(d, 0.0f);    // quad_perm [2,3,0,1]: every lane its quad's sum
        d += dppf<0x141, 0xf>(d, 0.0f);   // row_half_mirror: the 8-lane group's sum
        if (LPC == 16) d += dppf<0x140, 0xf>(d, 0.0f);   // row_mirror: the 16-lane row's
        const bool valid = c < ncell && cp <= qpos;
        const float w = valid ? d * P.scale : -INFINITY;
        mx = fmaxf(mx, w);
        if (L == 0 && c < ncell) sw[grp][c] = w;
    };
#pragma unroll
    for (int u = 0; u < UM; ++u) {
        const int c = wave * CPW + u * STEP + G;
        if (wave * CPW + u * STEP < ncell) score(c, k0[u], cp0[u]);
    }
    for (int cb = wave * CPW + UM * STEP; cb < ncell; cb += STEP) {
        const int c = min(cb + G, ncell - 1);
        const u32x4 kk = *gptr(reinterpret_cast<const u32x4*>(P.kcache + (long long)c * P.kv_dim + (long long)g * HD + L * 8));
        const int cp = gptr(P.cell_pos)[c];
        score(cb + G, kk, cp);
    }
    const float wm = wave_max_any(mx);
    if (lane == 0) redm[grp][wave] = wm;
    __syncthreads();
    float M = redm[grp][0];
#pragma unroll
    for (int w = 1; w < NWV; ++w) M = fmaxf(M, redm[grp][w]);
    // 2. sum over every cell of expf(w - M) in double, fixed order (a cell per thread, waves in order)
    {
        double acc = 0.0;
        for (int c = tid; c < ncell; c += NT) acc += (double)expf(sw[grp][c] - M);
        acc = wave_sum63_d(acc);
        if (lane == 63) dred[grp][wave] = acc;
    }
    __syncthreads();
    double tot = 0.0;
#pragma unroll
    for (int w = 0; w < NWV; ++w) tot += dred[grp][w];
    const float inv = (float)(1.0 / tot);
    // 3. sum_c f16(p_c) v_c over the wave's cells, then the wave's cell groups, then the waves in order
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = 0.0f;
    auto pv = [&](int c, const u32x4& vv) {
        float vf[8];
        cvt8(vv, vf);
        const bool in = c < ncell;
        const float p = expf(sw[grp][in ? c : 0] - M) * inv;   // ggml_vec_soft_max_f32, f16 vec_dot_type
        const float pw = in ? __half2float(__float2half_rn(p)) : 0.0f;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = fmaf(pw, vf[e], o[e]);
    };
#pragma unroll
    for (int u = 0; u < UM; ++u) {
        const int c = wave * CPW + u * STEP + G;
        if (wave * CPW + u * STEP < ncell) pv(c, v0[u]);
    }
    for (int cb = wave * CPW + UM * STEP; cb < ncell; cb += STEP) {
        const int c = min(cb + G, ncell - 1);
        const u32x4 vv = *gptr(reinterpret_cast<const u32x4*>(P.vcache + (long long)c * P.kv_dim + (long long)g * HD + L * 8));
        pv(cb + G, vv);
    }
#pragma unroll
    for (int off = LPC; off < 64; off <<= 1)
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] += __shfl_xor(o[e], off, 64);
    if (G == 0) {
#pragma unroll
        for (int e = 0; e < 8; ++e) red_o[grp][wave][L * 8 + e] = o[e];
    }
    __syncthreads();
    // (no fp32 copy of the output: the streaming WO launch reads only the quantised one)
    // the WO launch's quantised activation: the workgroup's HG heads are whole 256-blocks, one
    // wave per block; element e of the workgroup's span is head e / HD, dim e % HD
    constexpr int NE = HG * HD;
    const int gw = (int)threadIdx.x >> 6;
    const int e0 = (int)blockIdx.x * NE;
    for (int b = gw; b < NE / 256; b += HG * NWV) {
        float v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int e = b * 256 + lane * 4 + k, gg = e / HD, d = e % HD;
            float s = red_o[gg][0][d];
#pragma unroll
            for (int w = 1; w < NWV; ++w) s += red_o[gg][w][d];
            v[k] = s;
        }
        if (P.act_q8.q) quant_actq8_block(P.act_q8, tok, e0 / 256 + b, v, lane);   // a short batch's WO input
        else dv_quant_block(P.act_out, e0 / 256 + b, v, lane);
    }
}

typedef void (*AttnFn)(const AttnParams);
// Can `need` workgroups of attn_long_kernel (256 threads, `lds` dynamic LDS) be resident on the
// current device at once?  The splits of a head spin on each other, so they all must be.
static bool attn_long_resident(const void* fn, size_t lds, long long need) {
    int dev = 0, cus = 0, per_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess) return false;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return false;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 256, lds) != hipSuccess) return false;
    return (long long)per_cu * cus >= need;
}
// the split kernels issue the cache loads of 4 cell steps per wave together (8: no faster, r03)
template <int R, int LPC>
static void attn_fns_l(AttnFn& a, AttnFn& b, AttnFn& f) {
    a = attn_scores_kernel<R, LPC, 4>;
    b = attn_pv_kernel<R, LPC, 4>;
    f = attn_fused_kernel<R, LPC, 1>;
}
template <int R>
static void attn_fns_r(int hd, AttnFn& a, AttnFn& b, AttnFn& f) {
    switch (hd) {
    case 32: attn_fns_l<R, 4>(a, b, f); break;
    case 64: attn_fns_l<R, 8>(a, b, f); break;
    case 128: attn_fns_l<R, 16>(a, b, f); break;
    case 256: attn_fns_l<R, 32>(a, b, f); break;
    default: a = b = f = nullptr; break;
    }
}

// one q head per group (R = 1) of head_dim 64 / 128 for a quantising pick: the decode kernel with
// 8-16 waves per group (attn_dec_kernel), nwv its waves per group; null: the fused kernel serves it
struct AttnQuantPick;
static AttnFn attn_dec_pick(const AttnQuantPick& k, int r, int head_dim, int& nwv);

// the R = 1 fused kernel with hg groups of 4 waves (the streaming decode step's quantising form)
static AttnFn attn_fused_hg1(int hd, int hg) {
    switch (hd * 8 + hg) {
    case 128 * 8 + 1: return attn_fused_kernel<1, 16, 1>;
    case 128 * 8 + 2: return attn_fused_kernel<1, 16, 2>;
    case 64 * 8 + 1: return attn_fused_kernel<1, 8, 1>;
    case 64 * 8 + 2: return attn_fused_kernel<1, 8, 2>;
    case 64 * 8 + 4: return attn_fused_kernel<1, 8, 4>;
    default: return nullptr;
    }
}

// The quantising fused kernel for a head geometry -- the decode step's (launch_attn with
// act_out) and a short batch's (launch_attn_multi with act_q8): a workgroup serves whole 256-blocks
// of the output, hg groups of 4 waves, each group one kv head (R q heads) or, with few kv heads
// (qsplit), one q head.  One picker for the support query and both launchers.
struct AttnQuantPick {
    AttnFn f;
    int qsplit, hg, units;
};
static AttnQuantPick attn_quant_pick(int n_head, int n_head_kv, int head_dim) {
    AttnQuantPick k{nullptr, 0, 1, 0};
    if (n_head_kv <= 0 || n_head % n_head_kv) return k;
    const int r = n_head / n_head_kv;
    if (r != 1 && r != 2 && r != 4 && r != 8) return k;
    const bool qs = r > 1 && n_head_kv < 16;   // few kv heads: a group per q head
    const int per = (qs ? 1 : r) * head_dim;   // output elements of one group
    const int hg = per >= 256 ? 1 : 256 / per;
    const int units = qs ? n_head : n_head_kv;
    if (units % hg || per * hg % 256) return k;
    AttnFn f = nullptr;
    if (hg == 1 && !qs) {
        AttnFn fa = nullptr, fb = nullptr;
        switch (r) {
        case 1: attn_fns_r<1>(head_dim, fa, fb, f); break;
        case 2: attn_fns_r<2>(head_dim, fa, fb, f); break;
        case 4: attn_fns_r<4>(head_dim, fa, fb, f); break;
        case 8: attn_fns_r<8>(head_dim, fa, fb, f); break;
        default: break;
        }
    } else if (qs || r == 1) {
        f = attn_fused_hg1(head_dim, hg);
    }
    k.f = f;
    k.qsplit = qs ? r : 0;
    k.hg = hg;
    k.units = units;
    return k;
}

static AttnFn attn_dec_pick(const AttnQuantPick& k, int r, int head_dim, int& nwv) {
    nwv = 4;
    if (!(k.hg > 1 || k.qsplit || r == 1)) return nullptr;
    switch (head_dim * 8 + k.hg) {
    case 128 * 8 + 1: nwv = 16; return attn_dec_kernel<16, 1, 16>;
    case 128 * 8 + 2: nwv = 8; return attn_dec_kernel<16, 2, 8>;
    case 64 * 8 + 1: nwv = 16; return attn_dec_kernel<8, 1, 16>;
    case 64 * 8 + 2: nwv = 8; return attn_dec_kernel<8, 2, 8>;
    case 64 * 8 + 4: nwv = 4; return attn_dec_kernel<8, 4, 4>;
    default: return nullptr;
    }
}

bool attn_quant_supported(int n_head, int n_head_kv, int head_dim) {
    return attn_quant_pick(n_head, n_head_kv, head_dim).f != nullptr;
}

void launch_attn(const AttnParams& p, hipStream_t s) {
    if (p.n_head % p.n_head_kv) throw Error("attn: n_head must be a multiple of n_head_kv");
    const int r = p.n_head / p.n_head_kv;
    AttnFn fa = nullptr, fb = nullptr, ff = nullptr;
    switch (r) {
    case 1: attn_fns_r<1>(p.head_dim, fa, fb, ff); break;
    case 2: attn_fns_r<2>(p.head_dim, fa, fb, ff); break;
    case 4: attn_fns_r<4>(p.head_dim, fa, fb, ff); break;
    case 8: attn_fns_r<8>(p.head_dim, fa, fb, ff); break;
    default: break;
    }
    if (!fa) throw Error("attn: unsupported head_dim / GQA ratio (head_dim 32..256, ratio 1/2/4/8)");
    if (p.fused && p.act_out.act) {
        // the streaming decode step: the output also quantised, whole 256-blocks per workgroup
        const AttnQuantPick k = attn_quant_pick(p.n_head, p.n_head_kv, p.head_dim);
        if (!k.f || p.act_out.K != p.n_head * p.head_dim)
            throw Error("attn: no quantising decode kernel for this head geometry");
        AttnParams q = p;
        q.qsplit = k.qsplit;
        int nwv = 4;
        const AttnFn fd = attn_dec_pick(k, r, p.head_dim, nwv);
        if (fd) {
            hipLaunchKernelGGL(fd, dim3(k.units / k.hg), dim3(64 * nwv * k.hg), 0, s, q);
        } else {
            hipLaunchKernelGGL(k.f, dim3(k.units / k.hg), dim3(256 * k.hg), 0, s, q);
        }
        MI_HIP(hipGetLastError());
        return;
    }
    if (p.fused) {   // the caller guarantees <= ATTN_SHORT cells (the kernel clamps anyway)
        if (r > 1 && p.n_head_kv < 16) {   // few kv heads: one workgroup per q head (R=1 kernel)
            AttnFn f1 = nullptr, a1 = nullptr, b1 = nullptr;
            attn_fns_r<1>(p.head_dim, a1, b1, f1);
            AttnParams q = p;
            q.qsplit = r;
            hipLaunchKernelGGL(f1, dim3(p.n_head), dim3(256), 0, s, q);
            MI_HIP(hipGetLastError());
            return;
        }
        hipLaunchKernelGGL(ff, dim3(p.n_head_kv), dim3(256), 0, s, p);
        MI_HIP(hipGetLastError());
        return;
    }
    if (p.xflags && p.step && !p.long_off && (p.head_dim == 64 || p.head_dim == 128)) {
        // one launch, the splits of a q head exchanging their softmax statistics
        const size_t lds = (size_t)std::max(64, ((p.n_ctx + ATTN_SMAX - 1) / ATTN_SMAX + 63) / 64 * 64) * sizeof(float);
        auto fn = p.head_dim == 128 ? attn_long_kernel<16> : attn_long_kernel<8>;
        if (lds <= 64 * 1024 && attn_long_resident(reinterpret_cast<const void*>(fn), lds, (long long)p.n_head * ATTN_SMAX * std::max(1, p.long_share))) {
            hipLaunchKernelGGL(fn, dim3(p.n_head, ATTN_SMAX), dim3(256), lds, s, p);
            MI_HIP(hipGetLastError());
            return;
        }
    }
    if (r > 1 && p.n_head_kv < 16) {   // few kv heads: one workgroup per q head and split
        AttnFn f1 = nullptr, a1 = nullptr, b1 = nullptr;
        attn_fns_r<1>(p.head_dim, a1, b1, f1);
        AttnParams q = p;
        q.qsplit = r;
        hipLaunchKernelGGL(a1, dim3(p.n_head, ATTN_SMAX), dim3(256), 0, s, q);
        MI_HIP(hipGetLastError());
        hipLaunchKernelGGL(b1, dim3(p.n_head, ATTN_SMAX), dim3(256), 0, s, q);
        MI_HIP(hipGetLastError());
        return;
    }
    hipLaunchKernelGGL(fa, dim3(p.n_head_kv, ATTN_SMAX), dim3(256), 0, s, p);
    MI_HIP(hipGetLastError());
    hipLaunchKernelGGL(fb, dim3(p.n_head_kv, ATTN_SMAX), dim3(256), 0, s, p);
    MI_HIP(hipGetLastError());
}

void launch_attn_multi(const AttnParams& p_in, int ntok, float* out, hipStream_t s) {
    AttnParams p = p_in;
    p.part_o = out;
    p.fused = 1;
    if (ntok < 1) return;
    const int r = p.n_head / p.n_head_kv;
    if (p.act_q8.q) {
        // each token's output also quantised (a short batch's WO input): the decode step's
        // quantising geometry, whole 256-blocks per workgroup, one grid row per token
        const AttnQuantPick k = attn_quant_pick(p.n_head, p.n_head_kv, p.head_dim);
        if (!k.f || p.act_q8.K != p.n_head * p.head_dim || p.act_q8.ntok != ntok)
            throw Error("attn: no quantising batch kernel for this head geometry");
        p.qsplit = k.qsplit;
        // the decode kernel, one grid row per token, where it serves the geometry (20 / 64 claimed
        // tokens 3.38 / 5.15 -> 3.36 / 5.09 ms against the fused kernel, profiles/r06_short_attn_ab.txt)
        int nwv = 4;
        const AttnFn fd = attn_dec_pick(k, r, p.head_dim, nwv);
        if (fd) hipLaunchKernelGGL(fd, dim3(k.units / k.hg, ntok), dim3(64 * nwv * k.hg), 0, s, p);
        else hipLaunchKernelGGL(k.f, dim3(k.units / k.hg, ntok), dim3(256 * k.hg), 0, s, p);
        MI_HIP(hipGetLastError());
        return;
    }
    AttnFn fa = nullptr, fb = nullptr, ff = nullptr;
    switch (r) {
    case 1: attn_fns_r<1>(p.head_dim, fa, fb, ff); break;
    case 2: attn_fns_r<2>(p.head_dim, fa, fb, ff); break;
    case 4: attn_fns_r<4>(p.head_dim, fa, fb, ff); break;
    case 8: attn_fns_r<8>(p.head_dim, fa, fb, ff); break;
    default: break;
    }
    if (!ff || p.n_head % p.n_head_kv) throw Error("attn: unsupported head_dim / GQA ratio");
    hipLaunchKernelGGL(ff, dim3(p.n_head_kv, ntok), dim3(256), 0, s, p);
    MI_HIP(hipGetLastError());
}

// Stand-alone combine (same arithmetic as the PRO_ATTN prologue).
__global__ void attn_combine_kernel(const AttnPartials A, const int* tokpos, float* out) {
    int chunk, nsplit;
    attn_split(tokpos[2] + 1, chunk, nsplit);
    const int h = blockIdx.x;
    for (int d = threadIdx.x; d < A.head_dim; d += blockDim.x) {
        float acc = 0.0f;
        for (int s = 0; s < nsplit; ++s) acc += A.o[((long long)s * A.n_head + h) * A.head_dim + d];
        out[h * A.head_dim + d] = acc;
    }
}

// one wave per 256-block of the output: its 4 elements per lane summed over the splits in split
// order (split 0 first, then += 1, 2, ..), then dv_quant_block
__global__ __launch_bounds__(64) void attn_combine_quant_kernel(const AttnPartials A, const int* tokpos, const ActOut t) {
    int chunk, nsplit;
    attn_split(tokpos[2] + 1, chunk, nsplit);
    const int b = blockIdx.x, lane = threadIdx.x;
    const long long stride = (long long)A.n_head * A.head_dim;
    const f32x4* o = reinterpret_cast<const f32x4*>(A.o);
    f32x4 v = o[b * 64 + lane];
    for (int s0 = 1; s0 < nsplit; s0 += 4) {   // four splits' loads in flight, added in order
        f32x4 t4[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (s0 + j < nsplit) t4[j] = o[(s0 + j) * stride / 4 + b * 64 + lane];
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (s0 + j < nsplit) {
                v.x += t4[j].x;
                v.y += t4[j].y;
                v.z += t4[j].z;
                v.w += t4[j].w;
            }
    }
    const float q[4] = {v.x, v.y, v.z, v.w};
    dv_quant_block(t, b, q, lane);
}

void launch_attn_combine_quant(const AttnPartials& a, const int* tokpos, const ActOut& t, hipStream_t s) {
    if (t.K != a.n_head * a.head_dim || t.K % 256 || !t.act || t.norm_w) throw Error("attn combine: bad activation");
    hipLaunchKernelGGL(attn_combine_quant_kernel, dim3(t.K / 256), dim3(64), 0, s, a, tokpos, t);
    MI_HIP(hipGetLastError());
}

void launch_attn_combine(const AttnPartials& a, const int* tokpos, float* out, hipStream_t s) {
    hipLaunchKernelGGL(attn_combine_kernel, dim3(a.n_head), dim3(128), 0, s, a, tokpos, out);
    MI_HIP(hipGetLastError());
}

// ---------------------------------------------------------------------------
// Top-k: keys (orderable logit << 32 | ~id), larger key = better, so the order
// is logit descending then id ascending.  A wave holds 64 keys, one per lane,
// sorted descending by lane; two sorted lists merge into the top 64 of their
// union by c[i] = max(a[i], b[63-i]) (a bitonic sequence) and a 6-step
// half-cleaner.  Stage 1: each 1024-logit block -> 16 wave sorts -> LDS tree
// merge -> its top 64.  Stage 2: one workgroup merges the block lists.
// ---------------------------------------------------------------------------
typedef unsigned long long u64;
__device__ __forceinline__ u64 topk_key(float v, int id) {
    unsigned u = __float_as_uint(v);
    u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
    return ((u64)u << 32) | (u64)(0xFFFFFFFFu - (unsigned)id);
}
__device__ __forceinline__ u64 shfl_xor64(u64 v, int m) {
    const unsigned lo = __shfl_xor((unsigned)v, m, 64), hi = __shfl_xor((unsigned)(v >> 32), m, 64);
    return ((u64)hi << 32) | lo;
}
__device__ __forceinline__ u64 shfl64(u64 v, int src) {
    const unsigned lo = __shfl((unsigned)v, src, 64), hi = __shfl((unsigned)(v >> 32), src, 64);
    return ((u64)hi << 32) | lo;
}
__device__ __forceinline__ u64 wave_sort_desc(u64 x, int lane) {
#pragma unroll
    for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            const u64 y = shfl_xor64(x, j);
            const bool desc = (lane & k) == 0 || k == 64;
            const bool lower = (lane & j) == 0;
            const bool keep_max = lower == desc;
            x = keep_max ? (x > y ? x : y) : (x < y ? x : y);
        }
    }
    return x;
}
// a, b sorted descending across the wave -> top 64 of a U b, sorted descending
__device__ __forceinline__ u64 wave_merge_desc(u64 a, u64 b, int lane) {
    const u64 br = shfl64(b, 63 - lane);
    u64 x = a > br ? a : br;
#pragma unroll
    for (int j = 32; j > 0; j >>= 1) {
        const u64 y = shfl_xor64(x, j);
        x = (lane & j) == 0 ? (x > y ? x : y) : (x < y ? x : y);
    }
    return x;
}

// 16 waves each hold a sorted list; tree-merge them through LDS into wave 0.
__device__ __forceinline__ u64 block_merge16(u64 x, u64* lds, int wave, int lane) {
    for (int n = 16; n > 1; n >>= 1) {
        if (wave >= n / 2 && wave < n) lds[(wave - n / 2) * 64 + lane] = x;
        __syncthreads();
        if (wave < n / 2) x = wave_merge_desc(x, lds[wave * 64 + lane], lane);
        __syncthreads();
    }
    return x;
}

__global__ __launch_bounds__(1024) void topk_stage1(const float* logits, int n, u64* cand) {
    __shared__ u64 lds[8 * 64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int id = blockIdx.x * TOPK_BLOCK + wave * 64 + lane;
    u64 x = id < n ? topk_key(logits[id], id) : 0ULL;
    x = wave_sort_desc(x, lane);
    x = block_merge16(x, lds, wave, lane);
    if (wave == 0) cand[blockIdx.x * 64 + lane] = x;
}

__global__ __launch_bounds__(1024) void topk_stage2(const u64* cand, int nblk, const float* logits, int* ids,
                                                   float* vals, int* h_ids, float* h_vals) {
    __shared__ u64 lds[8 * 64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    u64 x = wave < nblk ? cand[wave * 64 + lane] : 0ULL;
    for (int b = wave + 16; b < nblk; b += 16) x = wave_merge_desc(x, cand[b * 64 + lane], lane);
    x = block_merge16(x, lds, wave, lane);
    if (wave == 0) {
        const int i = x ? (int)(0xFFFFFFFFu - (unsigned)(x & 0xFFFFFFFFu)) : -1;
        const float v = i >= 0 ? logits[i] : -INFINITY;
        ids[lane] = i;
        vals[lane] = v;
        if (h_ids) {
            h_ids[lane] = i;
            h_vals[lane] = v;
        }
    }
}

void launch_topk(const TopkParams& p, hipStream_t s) {
    const int nblk = topk_blocks(p.n);
    hipLaunchKernelGGL(topk_stage1, dim3(nblk), dim3(1024), 0, s, p.logits, p.n, p.cand);
    MI_HIP(hipGetLastError());
    hipLaunchKernelGGL(topk_stage2, dim3(1), dim3(1024), 0, s, p.cand, nblk, p.logits, p.ids, p.vals, p.h_ids,
                       p.h_vals);
    MI_HIP(hipGetLastError());
}

__global__ void gather_kernel(const float* logits, const int* ids, int n, float* out) {
    const int i = threadIdx.x + blockIdx.x * blockDim.x;
    if (i < n) out[i] = logits[ids[i]];
}

// rows of logits: out[i] = base[(i / k) * row_stride + ids[i]]
__global__ void gather_rows_kernel(const float* base, long long row_stride, const int* ids, int n, int k, float* out) {
    const int i = threadIdx.x + blockIdx.x * blockDim.x;
    if (i < n) out[i] = base[(long long)(i / k) * row_stride + ids[i]];
}

void launch_gather_rows(const float* base, long long row_stride, const int* ids, int n, int k, float* out,
                        hipStream_t s) {
    if (n <= 0 || k <= 0) return;
    hipLaunchKernelGGL(gather_rows_kernel, dim3((n + 255) / 256), dim3(256), 0, s, base, row_stride, ids, n, k, out);
    MI_HIP(hipGetLastError());
}

void launch_gather(const float* logits, const int* ids, int n, float* out, hipStream_t s) {
    if (n <= 0) return;
    hipLaunchKernelGGL(gather_kernel, dim3((n + 255) / 256), dim3(256), 0, s, logits, ids, n, out);
    MI_HIP(hipGetLastError());
}

// ---------------------------------------------------------------------------
// MoE router (build_moe_ffn, softmax gating, norm_w): one workgroup.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void router_kernel(const RouterParams P0) {
    __shared__ double redd[4];
    __shared__ float logit[64];
    __shared__ float prs[64], topp[64];
    __shared__ int topi[64];
    // token blockIdx.x of a batch (launch_router_multi); one token for the decode step
    RouterParams P = P0;
    P.x += (long long)blockIdx.x * P.x_stride;
    P.sel += blockIdx.x * P.n_used;
    P.selw += blockIdx.x * P.n_used;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (P.part) {   // the split WO's halves: x = (p0 + p1) + x, written back for the experts
        const float* p0 = P.part + (long long)blockIdx.x * P.n_embd;
        const float* p1 = P.part + ((long long)P.part_ntok + blockIdx.x) * P.n_embd;
        float* xw = const_cast<float*>(P.x);
        for (int i = tid; i < P.n_embd; i += 256) xw[i] = (p0[i] + p1[i]) + xw[i];
        __syncthreads();
    }
    // every load of a phase issued before its arithmetic (a serial loop of dependent loads took
    // ~40 us per token, measured): the row as float4 per lane, kept in registers (n_embd <= 4096)
    constexpr int RK = 16;
    const f32x4* x4 = reinterpret_cast<const f32x4*>(P.x);
    const f32x4* n4 = reinterpret_cast<const f32x4*>(P.norm_w);
    const int nk = P.n_embd / 256;   // float4 per lane
    f32x4 xv[RK];
#pragma unroll
    for (int k = 0; k < RK; ++k)
        if (k < nk) xv[k] = x4[k * 64 + lane];
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < RK; ++k)
        if (k < nk) {
            s += (double)(xv[k].x * xv[k].x);
            s += (double)(xv[k].y * xv[k].y);
            s += (double)(xv[k].z * xv[k].z);
            s += (double)(xv[k].w * xv[k].w);
        }
    s = wave_sum_d(s);   // (every wave holds the whole row: each computes the same sum)
    const float mean = (float)(__shfl(s, 0, 64) / (double)P.n_embd);
    const float scale = 1.0f / sqrtf(mean + P.eps);
    (void)redd;
    {   // x * scale * norm_w, in place
        f32x4 nv[RK];
#pragma unroll
        for (int k = 0; k < RK; ++k)
            if (k < nk) nv[k] = n4[k * 64 + lane];
#pragma unroll
        for (int k = 0; k < RK; ++k)
            if (k < nk)
                xv[k] = f32x4{(xv[k].x * scale) * nv[k].x, (xv[k].y * scale) * nv[k].y, (xv[k].z * scale) * nv[k].z,
                              (xv[k].w * scale) * nv[k].w};
    }
    // expert e handled by wave e%4: logits = W_e . (x*scale*w)
    for (int e = wave; e < P.n_expert; e += 4) {
        const f32x4* we = reinterpret_cast<const f32x4*>(P.w + (long long)e * P.n_embd);
        f32x4 wv[RK];
#pragma unroll
        for (int k = 0; k < RK; ++k)
            if (k < nk) wv[k] = we[k * 64 + lane];
        float acc = 0.0f;
#pragma unroll
        for (int k = 0; k < RK; ++k)
            if (k < nk) {
                acc = fmaf(wv[k].x, xv[k].x, acc);
                acc = fmaf(wv[k].y, xv[k].y, acc);
                acc = fmaf(wv[k].z, xv[k].z, acc);
                acc = fmaf(wv[k].w, xv[k].w, acc);
            }
        acc = wave_sum(acc);
        if (lane == 0) logit[e] = acc;
    }
    __syncthreads();
    // softmax over the experts and the top n_used, in wave 0 with one lane per expert (per-thread
    // arrays here would live in scratch memory: ~45 us per call, measured)
    if (wave == 0) {
        const int E = P.n_expert;
        const float lg = lane < E ? logit[lane] : -INFINITY;
        float mx = lg;   // the max is order-free
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off, 64));
        const float pe = lane < E ? expf(lg - mx) : 0.0f;
        prs[lane] = pe;
        __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
        __builtin_amdgcn_wave_barrier();
        // soft_max's double sum in expert order, then p = e * (1/sum)
        double sum = 0.0;
        for (int e = 0; e < E; ++e) sum += (double)prs[e];
        const float inv = (float)(1.0 / sum);
        const float pr = pe * inv;
        // ggml_argsort (desc; the selection sort above kept ties in index order) as a rank
        int rank = 0;
        for (int e = 0; e < E; ++e) {
            const float pq = __shfl(pr, e, 64);
            rank += (pq > pr || (pq == pr && e < lane)) ? 1 : 0;
        }
        if (lane < E && rank < P.n_used) {
            topi[rank] = lane;
            topp[rank] = pr;
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_wave_barrier();
        if (lane == 0) {
            float wsum = 0.0f;
            for (int k = 0; k < P.n_used; ++k) wsum += topp[k];
            for (int k = 0; k < P.n_used; ++k) { P.sel[k] = topi[k]; P.selw[k] = topp[k] / wsum; }
        }
    }
}

void launch_router(const RouterParams& p, hipStream_t s) { launch_router_multi(p, 1, s); }

void launch_router_multi(const RouterParams& p, int ntok, hipStream_t s) {
    if (p.n_expert > 64) throw Error("router: too many experts");
    if (p.n_embd % 256 || p.n_embd > 4096) throw Error("router: n_embd must be a multiple of 256, at most 4096");
    if (ntok < 1) return;
    hipLaunchKernelGGL(router_kernel, dim3(ntok), dim3(256), 0, s, p);
    MI_HIP(hipGetLastError());
}

// One workgroup: 256 threads, each over a contiguous range of the picks (so that the rows of an
// expert come in pick order = token ascending), per-thread counts per expert in LDS, then an
// exclusive scan over the threads per expert, padded expert offsets, and the row assignment.
__global__ __launch_bounds__(256) void moe_group_kernel(const int* sel, int n, int U, int E, int* grp, int* rows,
                                                        int* rowsel, int* pos, int rows_cap) {
    __shared__ int cnt[256][MOE_GROUP_MAXE];
    __shared__ int off[MOE_GROUP_MAXE + 1];
    const int t = threadIdx.x;
    const int per = (n + 255) / 256;
    const int i0 = min(n, t * per), i1 = min(n, i0 + per);
    for (int e = 0; e < E; ++e) cnt[t][e] = 0;
    for (int i = i0; i < i1; ++i) {
        const int e = sel[i];
        if (e >= 0 && e < E) cnt[t][e] += 1;
    }
    __syncthreads();
    if (t < E) {   // exclusive scan over the threads: this expert's rows before thread th's
        int run = 0;
        for (int th = 0; th < 256; ++th) {
            const int c = cnt[th][t];
            cnt[th][t] = run;
            run += c;
        }
        grp[E + 1 + t] = run;
    }
    __syncthreads();
    if (t == 0) {
        off[0] = 0;
        for (int e = 0; e < E; ++e) off[e + 1] = off[e] + (grp[E + 1 + e] + 31) / 32 * 32;
        for (int e = 0; e <= E; ++e) grp[e] = off[e];
    }
    __syncthreads();
    // padding rows (and every row past the last expert's) first, then the picks' rows
    for (int r = t; r < rows_cap; r += 256) {
        rows[r] = -1;
        rowsel[r] = -1;
    }
    __syncthreads();
    int used[MOE_GROUP_MAXE];
    for (int e = 0; e < E; ++e) used[e] = 0;
    for (int i = i0; i < i1; ++i) {
        const int e = sel[i];
        if (e < 0 || e >= E) continue;   // the router never picks one (checked on the decode path)
        const int r = off[e] + cnt[t][e] + used[e]++;
        rows[r] = i / U;
        rowsel[r] = r;
        pos[i] = r;
    }
}

void launch_moe_group(const int* sel, int n, int U, int E, int* grp, int* rows, int* rowsel, int* pos, int rows_cap,
                      hipStream_t s) {
    if (E < 1 || E > MOE_GROUP_MAXE) throw Error("moe_group: 1..16 experts");
    if (rows_cap < moe_rows_cap(n, E)) throw Error("moe_group: row capacity too small");
    hipLaunchKernelGGL(moe_group_kernel, dim3(1), dim3(256), 0, s, sel, n, U, E, grp, rows, rowsel, pos, rows_cap);
    MI_HIP(hipGetLastError());
}

__global__ void moe_combine_kernel(const float* y, const int* pos, const float* w, float* x, int n_embd) {
    const int t = blockIdx.y;
    const float* y0 = y + (long long)pos[2 * t] * n_embd;
    const float* y1 = y + (long long)pos[2 * t + 1] * n_embd;
    const float w0 = w[2 * t], w1 = w[2 * t + 1];
    float* xr = x + (long long)t * n_embd;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n_embd; i += gridDim.x * blockDim.x)
        xr[i] = (y0[i] * w0 + y1[i] * w1) + xr[i];   // as the decode GEMV's EPI_MOE_DOWN
}

void launch_moe_combine(const float* y, const int* pos, const float* w, float* x, int ntok, int n_embd,
                        hipStream_t s) {
    if (ntok < 1) return;
    hipLaunchKernelGGL(moe_combine_kernel, dim3((n_embd + 255) / 256, ntok), dim3(256), 0, s, y, pos, w, x, n_embd);
    MI_HIP(hipGetLastError());
}

// ---------------------------------------------------------------------------
// Load-time repack: GGUF blocks -> planes (one thread per superblock)
// ---------------------------------------------------------------------------
__global__ void repack_kernel(const uint8_t* raw, int type, long long nsb, uint8_t* p0, uint8_t* p1,
                              uint8_t* p2, uint8_t* p3) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < nsb;
         i += (long long)gridDim.x * blockDim.x) {
        if (type == T_Q4_K) {
            const uint8_t* b = raw + i * 144;
            for (int k = 0; k < 128; ++k) p0[i * 128 + k] = b[16 + k];
            for (int k = 0; k < 16; ++k) p1[i * 16 + k] = b[k];
        } else if (type == T_Q5_K) {
            const uint8_t* b = raw + i * 176;
            for (int k = 0; k < 128; ++k) p0[i * 128 + k] = b[48 + k];
            for (int k = 0; k < 32; ++k) p1[i * 32 + k] = b[16 + k];
            for (int k = 0; k < 16; ++k) p2[i * 16 + k] = b[k];
        } else if (type == T_Q6_K) {
            const uint8_t* b = raw + i * 210;
            for (int k = 0; k < 128; ++k) p0[i * 128 + k] = b[k];
            for (int k = 0; k < 64; ++k) p1[i * 64 + k] = b[128 + k];
            for (int k = 0; k < 16; ++k) p2[i * 16 + k] = b[192 + k];
            p3[i * 2] = b[208];
            p3[i * 2 + 1] = b[209];
        } else if (type == T_Q8_0) {
            const uint8_t* b = raw + i * 272;   // 8 blocks of 34
            for (int blk = 0; blk < 8; ++blk) {
                p1[i * 16 + blk * 2] = b[blk * 34];
                p1[i * 16 + blk * 2 + 1] = b[blk * 34 + 1];
                for (int k = 0; k < 32; ++k) p0[i * 256 + blk * 32 + k] = b[blk * 34 + 2 + k];
            }
        }
    }
}

void launch_repack(const uint8_t* raw, int type, long long rows, int K, uint8_t* const planes[4],
                   hipStream_t s) {
    const long long nsb = rows * (K / 256);
    const int grid = (int)std::min<long long>((nsb + 255) / 256, 8192);
    hipLaunchKernelGGL(repack_kernel, dim3(grid), dim3(256), 0, s, raw, type, nsb, planes[0], planes[1],
                       planes[2], planes[3]);
    MI_HIP(hipGetLastError());
}

// ---------------------------------------------------------------------------
// KV maintenance: K-shift (re-rotate cached K by a per-cell position delta,
// as llama.cpp's build_k_shift does with ggml_rope_ext on the f16 cache) and
// cell compaction (seq_rm).
// ---------------------------------------------------------------------------
__global__ void kv_shift_kernel(const KvShiftParams P) {
    const int cell = blockIdx.x, layer = blockIdx.y;
    const int delta = P.cell_delta[cell];
    if (delta == 0) return;
    __half* kr = P.kcache + ((long long)layer * P.n_ctx + cell) * P.kv_dim;
    const int pairs_per_head = P.head_dim / 2;
    for (int pi = threadIdx.x; pi < P.kv_dim / 2; pi += blockDim.x) {
        const int i = pi % pairs_per_head;          // pair index within head
        if (2 * i >= P.n_rot) continue;
        float theta = (float)delta;
        for (int k = 0; k < i; ++k) theta = theta * P.theta_scale;
        const float ff = P.freq_factors ? P.freq_factors[i] : 1.0f;
        const float th = P.freq_scale * (theta / ff);
        const float c = cosf(th), sn = sinf(th);
        const int head = pi / pairs_per_head;
        __half* e = kr + head * P.head_dim + 2 * i;
        const float x0 = __half2float(e[0]), x1 = __half2float(e[1]);
        e[0] = __float2half_rn(x0 * c - x1 * sn);
        e[1] = __float2half_rn(x0 * sn + x1 * c);
    }
}

void launch_kv_shift(const KvShiftParams& p, hipStream_t s) {
    if (p.n_cells <= 0) return;
    hipLaunchKernelGGL(kv_shift_kernel, dim3(p.n_cells, p.n_layer), dim3(256), 0, s, p);
    MI_HIP(hipGetLastError());
}

__global__ void kv_gather_kernel(const __half* cache, int n_ctx, int kv_dim, const int* src_cell, __half* dst) {
    const int cell = blockIdx.x, layer = blockIdx.y;
    const __half* sr = cache + ((long long)layer * n_ctx + src_cell[cell]) * kv_dim;
    __half* dr = dst + ((long long)layer * n_ctx + cell) * kv_dim;
    for (int i = threadIdx.x; i < kv_dim; i += blockDim.x) dr[i] = sr[i];
}

__global__ void kv_copy_kernel(const __half* src, int n_ctx, int kv_dim, int n, __half* dst) {
    const int cell = blockIdx.x, layer = blockIdx.y;
    const long long off = ((long long)layer * n_ctx + cell) * kv_dim;
    for (int i = threadIdx.x; i < kv_dim; i += blockDim.x) dst[off + i] = src[off + i];
}

void launch_kv_move(__half* cache, int n_layer, int n_ctx, int kv_dim, const int* src_cell, int n_dst,
                    __half* scratch, hipStream_t s) {
    if (n_dst <= 0) return;
    hipLaunchKernelGGL(kv_gather_kernel, dim3(n_dst, n_layer), dim3(256), 0, s, cache, n_ctx, kv_dim, src_cell,
                       scratch);
    MI_HIP(hipGetLastError());
    hipLaunchKernelGGL(kv_copy_kernel, dim3(n_dst, n_layer), dim3(256), 0, s, scratch, n_ctx, kv_dim, n_dst,
                       cache);
    MI_HIP(hipGetLastError());
}

}  // namespace mi
