// Prompt ingestion / batched verification on gfx950 int8 MFMA: the quantised GEMM of a
// physical batch of up to UB_MAX tokens (n_ubatch, reference Instance.hpp:24).
//
// The arithmetic is ggml b5187's CPU mul_mat for these types: the activation rows are
// quantised to Q8_K exactly as quantize_row_q8_K_ref (one row per token, as the CPU graph
// does for src1), and every weight row x activation row product is
//   Q4_K  sum_sb [ d_x d_y * sum_j sc_j * dot_j  -  dmin_x d_y * sum_j m_j * bsum_j ]
//   Q6_K  sum_sb [ d_x d_y * sum_g sc_g * dot_g ]                  (vec_dot_q*_K_q8_K)
// with the sub-block dots dot_j (32 elements; Q6_K: 16-element groups g) and the min terms
// computed EXACTLY in int32 by v_mfma_i32_32x32x32_i8, one MFMA per sub-block.  Only the
// fp32 sum across superblocks runs in another order than the CPU's.
//
// Geometry.  A wave computes a 32x32 D tile per MFMA, D[token][weight row]:
//   A operand = activations: lane l holds token l&31, k-half l>>5 (16 int8)
//   B operand = weights:     lane l holds weight row l&31, the same k-half
//   D: lane l, register r  = token (r&3) + 8(r>>2) + 4(l>>5), weight row l&31
// (the k order inside an MFMA does not matter: A and B share it; scripts/exp_mfma_layout.cpp
// checks the D map).  So every lane owns ONE weight row: its sub-block scales and mins are
// per-lane scalars, and the scale multiply is one full-rate v_mad_i32_i24 per result (|dot| < 2^17,
// |scale| < 2^7: the 24-bit product is exact; a plain int multiply would be quarter-rate
// v_mul_lo_u32).  The per-superblock float update is fused (fmaf): only fp32 rounding differs.
// A workgroup is 4 waves over one tile of 32 weight rows (16 gate/up pairs for SwiGLU) x 128
// tokens; the waves split the superblocks, and their partial sums meet in LDS in wave order
// (deterministic), after which wave w runs the epilogue of token tile w.  The 4 token groups
// of a row tile are placed on one XCD (blockIdx % 8), so their weight reads share its L2.
#include "kernels.h"
#include <hip/hip_runtime.h>
#include <cstdlib>

namespace mi {
namespace mmq {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <typename T>
__device__ __forceinline__ const __attribute__((address_space(1))) T* gp(const T* p) {
    return (const __attribute__((address_space(1))) T*)(p);
}
__device__ __forceinline__ float h2f(uint32_t bits) {
    return __half2float(__ushort_as_half(static_cast<unsigned short>(bits & 0xFFFFu)));
}
template <int CTRL, int RMASK>
__device__ __forceinline__ int dpp_i(int v) {
    return __builtin_amdgcn_update_dpp(0, v, CTRL, RMASK, 0xf, false);
}
template <int CTRL, int RMASK>
__device__ __forceinline__ double dpp_d(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = dpp_i<CTRL, RMASK>((int)b), hi = dpp_i<CTRL, RMASK>((int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
// full-wave double sum (fixed order), total in lane 63
__device__ __forceinline__ double wave_sum63_d(double v) {
    v += dpp_d<0x111, 0xf>(v);
    v += dpp_d<0x112, 0xf>(v);
    v += dpp_d<0x114, 0xf>(v);
    v += dpp_d<0x118, 0xf>(v);
    v += dpp_d<0x142, 0xa>(v);
    v += dpp_d<0x143, 0xc>(v);
    return v;
}
__device__ __forceinline__ float wave_max_pos(float v) {
#define MX(ctrl, rm) v = fmaxf(v, __int_as_float(dpp_i<ctrl, rm>(__float_as_int(v))))
    MX(0x111, 0xf); MX(0x112, 0xf); MX(0x114, 0xf); MX(0x118, 0xf); MX(0x142, 0xa); MX(0x143, 0xc);
#undef MX
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

__device__ __forceinline__ float silu(float x) { return x / (1.0f + expf(-x)); }

// ((p[0] + p[s]) + p[2s]) + ... over n parts, in part order, the loads of up to 8 parts issued
// together (a runtime-length loop of load-then-add pays one memory round trip per part)
template <typename V>
__device__ __forceinline__ V sum_parts(const V* p, long long stride, int n) {
    V v[7];
#pragma unroll
    for (int k = 1; k < 8; ++k)
        if (k < n) v[k - 1] = p[k * stride];
    V acc = p[0];
#pragma unroll
    for (int k = 1; k < 8; ++k)
        if (k < n) acc = acc + v[k - 1];
    for (int k = 8; k < n; k += 4) {   // (past 8 parts: 4 at a time)
        V w[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (k + q < n) w[q] = p[(k + q) * stride];
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (k + q < n) acc = acc + w[q];
    }
    return acc;
}


// ---------------------------------------------------------------------------
// Activation rows -> Q8_K (quantize_row_q8_K_ref), one workgroup per token row.
// Writes q in MFMA-fragment order (below), d transposed [nb][npad] (4 consecutive tokens = one
// 16-B load in the GEMM), and per superblock the 8 sub-block bsums split as 64*hi + lo (hi = floor(b/64),
// lo in 0..63): bytes 0-7 hi_j, 8-15 lo_j -- the int8 A operand of the MFMA that forms
// sum_j m_j*bsum_j = 64*sum m_j hi_j + sum m_j lo_j exactly.  Rows ntok..npad-1 are zero.
// ---------------------------------------------------------------------------
// QA_W waves per token row (16: one 256-element block each at K = 4096); XR blocks per wave at
// most (the host picks the smallest that covers K: fewer predicated copies, fewer registers)
template <int QA_W, int XR>
__global__ __launch_bounds__(64 * QA_W) void quant_act_kernel(const float* x, int x_stride, const float* norm_w,
                                                        float eps, ActQ8 a, const int* rows, const float* part, int nks,
                                                        int swiglu) {
    const int t = blockIdx.x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int nb = a.K >> 8;
    // this wave's blocks: w0, w0 + bst, ... (gridDim.y > 1, rows without a norm: the row's blocks
    // spread over gridDim.y workgroups)
    const int w0 = (int)blockIdx.y * QA_W + wave, bst = QA_W * (int)gridDim.y;
    __shared__ double red[QA_W];
    // MFMA-fragment order (one wave load = 1 KiB contiguous): q [tile][sb][j][h*32 + t%32][16 B],
    // element 32j + 16h + e of superblock sb of token t at byte e; bsb [tile][sb][t%32][16 B]
    const int tile = t >> 5, tr = t & 31;
    const int fj = lane >> 3, fh = (lane >> 2) & 1, fw = lane & 3;   // this lane's 4 elements
    int8_t* q = a.q + (long long)tile * nb * 8192 + fj * 1024 + (fh * 32 + tr) * 16 + 4 * fw;
    int8_t* bsb = a.q80 ? nullptr : a.bsb + ((long long)tile * nb * 32 + tr) * 16;
    if (t >= a.ntok || (rows && rows[t] < 0)) {   // padding rows (and MoE group padding) are zero
        for (int blk = w0; blk < nb; blk += bst) {
            *reinterpret_cast<int*>(q + blk * 8192) = 0;
            if (!a.q80 && lane < 4) reinterpret_cast<int*>(bsb + blk * 512)[lane] = 0;
            if (a.q80 && lane < 8) a.dT[(long long)(blk * 8 + lane) * a.npad + t] = 0.0f;
            if (!a.q80 && lane == 0) a.dT[(long long)blk * a.npad + t] = 0.0f;
        }
        return;
    }
    const f32x4* x4 = x ? reinterpret_cast<const f32x4*>(x + (long long)(rows ? rows[t] : t) * x_stride) : nullptr;
    // this wave's blocks read once, kept for the quantisation
    f32x4 xr[XR];
    if (swiglu) {   // silu(g) * u of the pair launch's parts: g = ((g0 + g1) + ...), u likewise
        const f32x4* p4 = reinterpret_cast<const f32x4*>(part + (long long)t * 2 * a.K);
        const long long kst = (long long)a.ntok * 2 * a.K / 4;   // one part, in f32x4
#pragma unroll
        for (int i = 0; i < XR; ++i) {
            const int blk = w0 + bst * i;
            if (blk < nb) {
                const f32x4 g = sum_parts(p4 + blk * 64 + lane, kst, nks);
                const f32x4 u = sum_parts(p4 + a.K / 4 + blk * 64 + lane, kst, nks);
                xr[i] = f32x4{silu(g.x) * u.x, silu(g.y) * u.y, silu(g.z) * u.z, silu(g.w) * u.w};
            }
            asm volatile("" ::: "memory");   // one block's part loads in flight at a time (registers)
        }
    } else {
#pragma unroll
        for (int i = 0; i < XR; ++i)
            if (w0 + bst * i < nb) xr[i] = x4[(w0 + bst * i) * 64 + lane];
    }
    if (part && !swiglu) {   // the split-K GEMM's nks partials: x = (((p0 + p1) + p2) + ...) + x (EPI_ADD's o + resid), written back
        f32x4* xw = reinterpret_cast<f32x4*>(const_cast<float*>(x) + (long long)t * x_stride);
#pragma unroll
        for (int i = 0; i < XR; ++i) {
            const int blk = w0 + bst * i;
            if (blk < nb) {
                const f32x4 acc = sum_parts(reinterpret_cast<const f32x4*>(part + (long long)t * a.K) + blk * 64 + lane,
                                            (long long)a.ntok * a.K / 4, nks);
                xr[i] = f32x4{acc.x + xr[i].x, acc.y + xr[i].y, acc.z + xr[i].z, acc.w + xr[i].w};
                xw[blk * 64 + lane] = xr[i];
            }
            asm volatile("" ::: "memory");   // one block's part loads in flight at a time (registers)
        }
    }
    float scale = 1.0f;
    if (norm_w) {   // ggml_compute_forward_rms_norm_f32: sum of squares in double
        double sacc = 0.0;
#pragma unroll
        for (int i = 0; i < XR; ++i) {
            if (w0 + bst * i < nb) {
                const f32x4 v = xr[i];
                sacc += (double)(v.x * v.x);
                sacc += (double)(v.y * v.y);
                sacc += (double)(v.z * v.z);
                sacc += (double)(v.w * v.w);
            }
        }
        sacc = wave_sum63_d(sacc);
        if (lane == 63) red[wave] = sacc;
        __syncthreads();
        double tot = 0.0;
#pragma unroll
        for (int k = 0; k < QA_W; ++k) tot += red[k];
        scale = 1.0f / sqrtf((float)(tot / (double)a.K) + eps);
    }
    const f32x4* w4 = reinterpret_cast<const f32x4*>(norm_w);
#pragma unroll
    for (int i = 0; i < XR; ++i) {
        const int blk = w0 + bst * i;
        if (blk >= nb) break;
        const f32x4 xv = xr[i];
        float v[4] = {xv.x, xv.y, xv.z, xv.w};
        if (norm_w) {
            const f32x4 w = w4[blk * 64 + lane];
            v[0] = (v[0] * scale) * w.x;   // ggml_vec_scale_f32, then ggml_mul
            v[1] = (v[1] * scale) * w.y;
            v[2] = (v[2] * scale) * w.z;
            v[3] = (v[3] * scale) * w.w;
        }
        if (a.q80) {   // quantize_row_q8_0 (x86 SIMD form): per 32 elements = 8 lanes
            float am = fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3])));
            am = fmaxf(am, __int_as_float(dpp_i<0xB1, 0xf>(__float_as_int(am))));
            am = fmaxf(am, __int_as_float(dpp_i<0x4E, 0xf>(__float_as_int(am))));
            am = fmaxf(am, __int_as_float(dpp_i<0x141, 0xf>(__float_as_int(am))));   // row_half_mirror
            const float d0 = am / 127.0f;
            const float id = am != 0.0f ? 127.0f / am : 0.0f;
            int qz[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) qz[k] = (int)rintf(v[k] * id);
            *reinterpret_cast<int*>(q + blk * 8192) =
                (qz[0] & 0xFF) | ((qz[1] & 0xFF) << 8) | ((qz[2] & 0xFF) << 16) | ((qz[3] & 0xFF) << 24);
            if ((lane & 7) == 0) a.dT[(long long)(blk * 8 + (lane >> 3)) * a.npad + t] = __half2float(__float2half_rn(d0));
            continue;
        }
        const float a0 = fabsf(v[0]), a1 = fabsf(v[1]), a2 = fabsf(v[2]), a3 = fabsf(v[3]);
        const float amax = wave_max_pos(fmaxf(fmaxf(a0, a1), fmaxf(a2, a3)));
        int qv[4];
        float d;
        if (amax == 0.0f) {
            qv[0] = qv[1] = qv[2] = qv[3] = 0;
            d = 0.0f;
        } else {   // max = the signed value at the FIRST index whose |x| is the maximum
            const int e = a0 == amax ? 0 : a1 == amax ? 1 : a2 == amax ? 2 : a3 == amax ? 3 : 4;
            const float mine = e == 0 ? v[0] : e == 1 ? v[1] : e == 2 ? v[2] : v[3];
            const unsigned long long m = __ballot(e < 4);
            const int src = __builtin_ctzll(m);
            const float mx = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(mine), src));
            const float iscale = -127.0f / mx;
#pragma unroll
            for (int k = 0; k < 4; ++k) qv[k] = min(127, (int)rintf(iscale * v[k]));
            d = 1.0f / iscale;
        }
        *reinterpret_cast<int*>(q + blk * 8192) =
            (qv[0] & 0xFF) | ((qv[1] & 0xFF) << 8) | ((qv[2] & 0xFF) << 16) | ((qv[3] & 0xFF) << 24);
        // the 32-element sub-block sums: lanes 8j..8j+7
        int sm = (qv[0] + qv[1]) + (qv[2] + qv[3]);
        sm += dpp_i<0xB1, 0xf>(sm);    // quad_perm [1,0,3,2]
        sm += dpp_i<0x4E, 0xf>(sm);    // quad_perm [2,3,0,1]
        sm += __shfl_xor(sm, 4, 64);   // the two quads of a sub-block
        if ((lane & 7) == 0) {
            const int j = lane >> 3;
            bsb[blk * 512 + j] = (int8_t)(sm >> 6);          // floor(b/64), -64..63
            bsb[blk * 512 + 8 + j] = (int8_t)(sm & 63);      // b - 64*floor(b/64), 0..63
        }
        if (lane == 0) a.dT[(long long)blk * a.npad + t] = d;
    }
}

// ggml_rope_cache_init (rope NORM) for every token of the batch: theta iterated from the
// position as the CPU does, table [ntok][n_rot/2] of (cos, sin).
__global__ void rope_table_kernel(const int* tokpos, int ntok, int n_rot, float theta_scale, float freq_scale,
                                  const float* freq_factors, float2* out) {
    const int t = blockIdx.x;
    if (t >= ntok) return;
    const int pos = tokpos[t * 4 + 1];
    for (int i = threadIdx.x; i < n_rot / 2; i += blockDim.x) {
        float theta = (float)pos;
        for (int k = 0; k < i; ++k) theta = theta * theta_scale;
        const float ff = freq_factors ? freq_factors[i] : 1.0f;
        const float th = freq_scale * (theta / ff);
        out[(long long)t * (n_rot / 2) + i] = make_float2(cosf(th), sinf(th));
    }
}


__device__ __forceinline__ v16i mfma(v4i a, v4i b) {
    const v16i z = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    return __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, z, 0, 0, 0);
}


// get_scale_min_k4 for the 8 sub-blocks of a Q4_K header {d, dmin, scales[12]}
__device__ __forceinline__ void q4k_scales(const u32x4 hd, int sc[8], int mn[8]) {
    const unsigned Y = hd.y, Z = hd.z, W = hd.w;   // bytes 0-3, 4-7, 8-11 of scales[12]
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        sc[j] = (Y >> (8 * j)) & 63;
        mn[j] = (Z >> (8 * j)) & 63;
        sc[4 + j] = ((W >> (8 * j)) & 0xF) | (((Y >> (8 * j + 6)) & 3) << 4);
        mn[4 + j] = ((W >> (8 * j + 4)) & 0xF) | (((Z >> (8 * j + 6)) & 3) << 4);
    }
}

// MFMA-order weight copy: one 32-row x superblock tile (lane = h*32 + c holds row c's bytes of
// k-half h; rows of a gate/up pair tile: c < 16 gate row 16*rt + c, c >= 16 up row 16*rt + c - 16)
//   Q4_K  [p 4][lane 64][16] qs bytes 32p + 16h.. | [c 32][16] header                       4608 B
//   Q6_K  the scaled weights w = (q - 32) * scale (|w| <= 4096, exact in int16) as two int8 MFMA
//         operands w = 64*hi + lo (hi -64..64, lo 0..63): [s 8][lane 64][16] hi of span s (superblock
//         elements 32s + 16h..) | the same for lo | [c 32][2] d                              16448 B
//         (a 32-element span holds two 16-element scale groups, one per k-half: with the scale
//         folded into the operand, one MFMA per span and operand carries the exact integer sum)
//   Q8_0  [j 8][lane 64][16] qs bytes 32j + 16h.. | [c 32][8 f16] d                            8704 B
//   Q5_K  as Q4_K, plus [lane 64][16] qh bytes 16h..: [p 4][lane][16] qs | qh | [c 32][16] header 5632 B
__host__ __device__ constexpr int mmq32_tile_bytes_d(int type) {
    return type == T_Q4_K ? 4608 : type == T_Q5_K ? 5632 : type == T_Q6_K ? 16448 : type == T_Q8_0 ? 8704 : 0;
}

__global__ void swizzle_kernel(const QMat A, const QMat B, int pair, uint8_t* dst) {
    const int nb = A.nb;
    const long long tile = blockIdx.x;   // rt * nb + sb
    const int rt = (int)(tile / nb), sb = (int)(tile % nb);
    const int TB = mmq32_tile_bytes_d(A.type);
    uint8_t* o = dst + tile * TB;
    for (int off = threadIdx.x; off < TB; off += blockDim.x) {
        int plane, c, byte;
        if (A.type == T_Q8_0) {
            if (off < 8192) {
                const int jj = off >> 10, ln = (off >> 4) & 63, e = off & 15;
                plane = 0; c = ln & 31; byte = 32 * jj + 16 * (ln >> 5) + e;
            } else {
                plane = 1; c = (off - 8192) >> 4; byte = (off - 8192) & 15;
            }
        } else if (A.type == T_Q4_K) {
            if (off < 4096) {
                const int p = off >> 10, ln = (off >> 4) & 63, e = off & 15;
                plane = 0; c = ln & 31; byte = 32 * p + 16 * (ln >> 5) + e;
            } else {
                plane = 1; c = (off - 4096) >> 4; byte = (off - 4096) & 15;
            }
        } else if (A.type == T_Q5_K) {
            if (off < 4096) {
                const int p = off >> 10, ln = (off >> 4) & 63, e = off & 15;
                plane = 0; c = ln & 31; byte = 32 * p + 16 * (ln >> 5) + e;
            } else if (off < 5120) {
                const int ln = (off - 4096) >> 4, e = off & 15;
                plane = 1; c = ln & 31; byte = 16 * (ln >> 5) + e;
            } else {
                plane = 2; c = (off - 5120) >> 4; byte = (off - 5120) & 15;
            }
        } else {   // Q6_K
            if (off < 16384) {   // w = (q - 32) * scale of element 32s + 16h + e (dequantize_row_q6_K)
                const int lo = off >= 8192, o2 = off & 8191;
                const int sp = o2 >> 10, ln = (o2 >> 4) & 63, e = o2 & 15;
                const int cc = ln & 31, h = ln >> 5, l = 16 * h + e, hf = sp >> 2, qq = sp & 3;
                const QMat& M = (pair && cc >= 16) ? B : A;
                long long row = pair ? 16LL * rt + (cc & 15) : 32LL * rt + cc;
                if (row >= M.rows) row = M.rows - 1;
                const long long b = row * nb + sb;
                const int ql = M.p[0][b * 128 + 64 * hf + l + 32 * (qq & 1)];
                const int qh = M.p[1][b * 64 + 32 * hf + l];
                const int sc = (int)(signed char)M.p[2][b * 16 + 8 * hf + 2 * qq + h];
                const int q = ((qq >= 2 ? ql >> 4 : ql & 0xF) | (((qh >> (2 * qq)) & 3) << 4)) - 32;
                const int w = q * sc;
                o[off] = (uint8_t)(lo ? (w & 63) : (w >> 6));
                continue;
            }
            plane = 3; c = (off - 16384) >> 1; byte = (off - 16384) & 1;
        }
        const QMat& M = (pair && c >= 16) ? B : A;
        long long row = pair ? 16LL * rt + (c & 15) : 32LL * rt + c;
        if (row >= M.rows) row = M.rows - 1;
        const int pb = A.type == T_Q8_0 ? (plane == 0 ? 256 : 16)
                     : A.type == T_Q4_K ? (plane == 0 ? 128 : 16)
                     : A.type == T_Q5_K ? (plane == 0 ? 128 : plane == 1 ? 32 : 16)
                                        : (plane == 0 ? 128 : plane == 1 ? 64 : plane == 2 ? 16 : 2);
        o[off] = M.p[plane][(row * nb + sb) * pb + byte];
    }
}

template <bool AB>
__device__ __forceinline__ void mmq_epilogue(const GemmParams& P, int tend, const float2* rope, int ttok0,
                                             int lane, int row, const float v[16], int epi, int nrows,
                                             float* out);

// The epilogue of one 32-token x 32-row D tile (v: this lane's 16 results).
template <bool AB>
__device__ __forceinline__ void mmq_epilogue(const GemmParams& P, int tend, const float2* rope, int ttok0,
                                             int lane, int row, const float v[16], int epi, int nrows,
                                             float* out) {
    const int col = lane & 31, h = lane >> 5;
    const bool roped = epi == EPI_ROPE_Q || epi == EPI_ROPE_K;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int tok = ttok0 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const float pv = __shfl_xor(v[r], AB ? 16 : 1, 64);   // SwiGLU partner / RoPE partner
        if (tok >= tend) continue;
        if (AB) {
            if (col >= 16 || row >= nrows) continue;
            out[(long long)tok * P.out_stride + row] = silu(v[r]) * pv;   // silu(gate) * up
            continue;
        }
        if (row >= nrows) continue;
        float o = v[r];
        if (roped) {
            const int i0 = row % P.head_dim;
            if (i0 < P.n_rot) {
                const float2 cs = rope[(long long)tok * (P.n_rot / 2) + i0 / 2];
                o = (col & 1) ? pv * cs.y + v[r] * cs.x : v[r] * cs.x - pv * cs.y;
            }
        }
        const int* tp = P.tokpos + tok * 4;
        switch (epi) {
        case EPI_STORE:
        case EPI_ROPE_Q: out[(long long)tok * P.out_stride + row] = o; break;
        case EPI_ADD: {
            const long long i = (long long)tok * P.out_stride + row;
            out[i] = o + P.resid[i];
            break;
        }
        case EPI_ROPE_K: {
            const int cell = tp[2];
            P.kcache[(long long)cell * P.kv_dim + row] = __float2half_rn(o);
            if (row == 0) P.cell_pos[cell] = tp[1];
            break;
        }
        case EPI_V: P.vcache[(long long)tp[2] * P.kv_dim + row] = __float2half_rn(o); break;
        default: break;
        }
    }
}

// =============================================================================================
// mmq2: the same arithmetic on a 128-token x 32*RT-column block per workgroup (8 waves: wave wv
// computes token tile wv & 3 x row tile wv >> 2, one 32x32 tile), its operands staged in LDS by
// LDS-DMA (global_load_lds_dwordx4):
//   * the weight tiles of the block's RT row tiles and the activation tiles of its 4 token tiles
//     for superblock sb + 1 land in one stage while superblock sb is computed from the other;
//     every piece address is a scalar base + a lane offset, computed once per token block;
//   * Q4_K / Q5_K: the 4 waves of a row tile first decode its superblock into int8 operand
//     planes of the SCALED weights sc_j * q (P0 + 8 P1 [+ 16 P2], every plane byte <= 105), so
//     the MFMAs accumulate sum_j sc_j * dot_j over the 8 sub-blocks themselves: the nibble
//     split and scale work is done once per row tile instead of once per wave, and the 16
//     integer multiply-adds per sub-block and result are gone (VALU was the bound: ~310 VALU
//     against 10 MFMAs per wave and superblock);
//   * Q6_K: the scaled hi/lo operands of the MFMA-order copy, accumulated by the MFMA; Q8_0:
//     one MFMA per 32-block and a float update per block (vec_dot_q8_0_q8_0's order);
//   * per 32x32 tile the integer sums are exact (the same int32 values as mmq32's) and the
//     per-superblock fp32 update is mmq32's.
// LDS: 2 stages of [RT weight slots of SLOT bytes][4 x 8 KiB activations][2 KiB bsb][dT: 1 KiB,
// Q8_0 4 KiB], then (Q4_K / Q5_K) the operand planes [RT][NPL][8 sub-blocks][64 lanes x 16 B].
// =============================================================================================
constexpr int MMQ_SEGS = 3;
struct MmqSegs {
    const uint8_t* sw[MMQ_SEGS];
    int rows[MMQ_SEGS];
    int epi[MMQ_SEGS];
    int n;
};

template <int T> struct M2 {
    static constexpr int RT = 2;                                        // row tiles per block
    static constexpr int NW = 4 * RT;                                    // waves: one 32x32 tile each
    static constexpr int TB = mmq32_tile_bytes_d(T);                    // bytes of a tile-superblock
    static constexpr int SLOT = (TB + 1023) / 1024 * 1024;
    static constexpr int A_OFF = RT * SLOT;
    static constexpr int BSB_OFF = A_OFF + 4 * 8192;
    static constexpr int DT_OFF = BSB_OFF + 2048;
    static constexpr int DT_KB = T == T_Q8_0 ? 4 : 1;
    static constexpr int STAGE = DT_OFF + DT_KB * 1024;
    static constexpr int NI = STAGE / 1024;                             // 1 KiB LDS-DMA pieces
    static constexpr int NIW = (NI + NW - 1) / NW;                      // per wave (some repeat)
    static constexpr int NPL = 2;                                       // K-quant operand planes
    static constexpr int PLANES = (T == T_Q4_K || T == T_Q5_K) ? RT * NPL * 8 * 1024 : 0;
    static constexpr int lds(int nst) { return nst * STAGE + PLANES; }
};

typedef __attribute__((address_space(3))) char lchar;
// register pins: the value is materialised at this point of the (volatile) instruction stream,
// so LDS reads issued before it stay in flight together instead of being sunk to their uses
__device__ __forceinline__ void pin(v4i& x) { asm volatile("" : "+v"(x)); }
__device__ __forceinline__ void pin_all() { asm volatile("" ::: "memory"); }
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
// the two 16-bit halves of x times s (v_pk_mul_lo_u16), each product < 65536
__device__ __forceinline__ unsigned wmul16(unsigned x, unsigned s) {
    u16x2 a;
    __builtin_memcpy(&a, &x, 4);
    const u16x2 r = a * u16x2{(unsigned short)s, (unsigned short)s};
    unsigned o;
    __builtin_memcpy(&o, &r, 4);
    return o;
}
// the bytes of x times s, every byte product < 256 (no carry between bytes): v_pk_mul_lo_u16
__device__ __forceinline__ unsigned bmul(unsigned x, unsigned s) {
    u16x2 a;
    __builtin_memcpy(&a, &x, 4);
    const u16x2 r = a * u16x2{(unsigned short)s, (unsigned short)s};
    unsigned o;
    __builtin_memcpy(&o, &r, 4);
    return o;
}
template <typename V>
__device__ __forceinline__ V lds_ld(const lchar* p) { return *reinterpret_cast<const __attribute__((address_space(3))) V*>(p); }

// The two int8 operand planes of the scaled weights sc_j * q of sub-blocks 2w, 2w + 1 of one row
// (lane) of a Q4_K / Q5_K tile, every byte <= 127:
//   Q4_K (sc = 8 sh + sl, q <= 15):  P0 = q * sl, P1 = q * sh,  sc q = P0 + 8 P1
//   Q5_K (q = lo4 + 16 hb <= 31):    p = sc * q <= 1953 (16-bit products),
//                                    P0 = p & 127, P1 = p >> 7,  sc q = P0 + 128 P1
// hd: the row's header, wq: its qs piece w, qh (Q5_K): its high bits.  o0 / o1: P0 / P1 of
// sub-block 2w, o2 / o3: of sub-block 2w + 1.  (r06: a copy holding these planes pre-decoded,
// 3.7x the tile bytes, measured slower -- the L2->LDS copies bound this GEMM)
template <int T>
__device__ __forceinline__ void q45_planes(const u32x4 hd, const u32x4 wq, const u32x4 qh, int w, u32x4& o0, u32x4& o1,
                                           u32x4& o2, u32x4& o3) {
    const unsigned Y = hd.y, W = hd.w;
    // get_scale_min_k4 for j = 2w, 2w + 1
    int s0, s1;
    if (w < 2) {
        s0 = (Y >> (16 * w)) & 63;
        s1 = (Y >> (16 * w + 8)) & 63;
    } else {
        const int k = 2 * w - 4;
        s0 = ((W >> (8 * k)) & 0xF) | (((Y >> (8 * k + 6)) & 3) << 4);
        s1 = ((W >> (8 * k + 8)) & 0xF) | (((Y >> (8 * k + 14)) & 3) << 4);
    }
    const unsigned q[4] = {wq.x, wq.y, wq.z, wq.w};
    unsigned* p0 = reinterpret_cast<unsigned*>(&o0);
    unsigned* p1 = reinterpret_cast<unsigned*>(&o1);
    unsigned* p2 = reinterpret_cast<unsigned*>(&o2);
    unsigned* p3 = reinterpret_cast<unsigned*>(&o3);
    if (T == T_Q4_K) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const unsigned lo = q[i] & 0x0F0F0F0Fu, hi = (q[i] >> 4) & 0x0F0F0F0Fu;
            p0[i] = bmul(lo, s0 & 7);
            p1[i] = bmul(lo, s0 >> 3);
            p2[i] = bmul(hi, s1 & 7);
            p3[i] = bmul(hi, s1 >> 3);
        }
    } else {
        const unsigned b[4] = {qh.x, qh.y, qh.z, qh.w};
        // 4 elements q (bytes) times s as 16-bit products, split into lo7 / hi bytes
        auto split = [](unsigned q5, unsigned sc, unsigned& lo, unsigned& hi) {
            const unsigned m02 = wmul16(q5 & 0x00FF00FFu, sc), m13 = wmul16((q5 >> 8) & 0x00FF00FFu, sc);
            lo = (m02 & 0x007F007Fu) | ((m13 & 0x007F007Fu) << 8);
            hi = ((m02 >> 7) & 0x001F001Fu) | (((m13 >> 7) & 0x001F001Fu) << 8);
        };
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const unsigned q5a = (q[i] & 0x0F0F0F0Fu) | (((b[i] >> (2 * w)) & 0x01010101u) << 4);
            const unsigned q5b = ((q[i] >> 4) & 0x0F0F0F0Fu) | (((b[i] >> (2 * w + 1)) & 0x01010101u) << 4);
            split(q5a, s0, p0[i], p1[i]);
            split(q5b, s1, p2[i], p3[i]);
        }
    }
}

// NST 2: two stages (copy of sb + 1 during sb), one workgroup per CU.  NST 1: one stage, copy and
// compute in turn, sized (LDS, <= 128 VGPRs) for two workgroups per CU that overlap each other.
template <int T, bool AB, int NST>
__global__ __launch_bounds__(64 * M2<T>::NW) __attribute__((amdgpu_waves_per_eu(NST == 1 ? 4 : 2)))
void mmq2_t(const GemmParams P, const ActQ8 act, const float2* rope, const MmqSegs S) {
    using C = M2<T>;
    constexpr int RT = C::RT;
    constexpr int NPL = C::NPL;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int w = wv & 3;                             // this wave's token tile
    const int wr = wv >> 2;                           // this wave's row tile (of the block's RT)
    const int col = lane & 31, h = lane >> 5;
    const int nb = P.K >> 8;
    // segments: S.n matrices of this type over the same activation in one grid (Q / K / V),
    // their row blocks concatenated; segment s: S.rows[s] rows, MFMA-order copy S.sw[s],
    // epilogue S.epi[s].  A plain or grouped launch is one segment.
    int nrb = 0;
#pragma unroll
    for (int i = 0; i < MMQ_SEGS; ++i)
        if (i < S.n) nrb += ((AB ? (S.rows[i] + 15) / 16 : (S.rows[i] + 31) / 32) + RT - 1) / RT;
    const int ntb = (act.npad + 127) / 128;           // token blocks
    const int TB = C::TB;
    // split-K: part kh of the grid's ksplit parts takes superblocks [nb kh / ks, nb (kh + 1) / ks)
    const int ks = P.ksplit > 1 ? P.ksplit : 1;
    const int nbid = (int)gridDim.x / ks;
    const int kh = (int)blockIdx.x / nbid, bid = (int)blockIdx.x % nbid;
    const int sb0 = nb * kh / ks, sb1 = nb * (kh + 1) / ks;
    int rb, tb_b, tb_e, base, tend, grp_e = 0;
    if (P.grp) {
        // grouped (MoE): blockIdx -> (token block, expert, row block), token block slowest: the
        // first blocks of every expert go first, an expert's later blocks (its tokens past 128)
        // after them, and a block past its expert's tokens exits
        const int nrb8 = (nrb + 7) / 8 * 8;
        const int per = nrb8 * P.grp_n;
        const int tbi = bid / per, rem = bid % per;
        const int e = rem / nrb8;
        grp_e = e;
        rb = rem % nrb8;
        if (rb >= nrb) return;
        base = P.grp[e];
        const int cnt = P.grp[P.grp_n + 1 + e];
        if (tbi * 128 >= cnt) return;
        tend = base + cnt;
        tb_b = tbi;
        tb_e = tbi + 1;
    } else {
        // blockIdx -> (row block, token block): the token blocks of a row block on one XCD
        const int b = bid, xcd = b & 7, slot = b >> 3;
        rb = (slot / ntb) * 8 + xcd;
        tb_b = slot % ntb;
        tb_e = tb_b + 1;
        base = 0;
        tend = act.ntok;
        if (rb >= nrb) return;
    }
    // this row block's segment
    int seg = 0;
#pragma unroll
    for (int i = 0; i < MMQ_SEGS - 1; ++i) {
        const int nrb_i = ((AB ? (S.rows[i] + 15) / 16 : (S.rows[i] + 31) / 32) + RT - 1) / RT;
        if (i + 1 < S.n && seg == i && rb >= nrb_i) {
            rb -= nrb_i;
            seg = i + 1;
        }
    }
    const int rows_s = seg == 0 ? S.rows[0] : seg == 1 ? S.rows[1] : S.rows[2];
    const int epi_s = seg == 0 ? S.epi[0] : seg == 1 ? S.epi[1] : S.epi[2];
    const int nrt = AB ? (rows_s + 15) / 16 : (rows_s + 31) / 32;
    const uint8_t* swA = seg == 0 ? S.sw[0] : seg == 1 ? S.sw[1] : S.sw[2];
    if (P.grp) swA += (long long)grp_e * P.grp_stride;
    const int tile_end = (tend + 31) / 32;            // tiles past the batch's (group's) last: clamped
  for (int tb = tb_b; tb < tb_e; ++tb) {
    // (grouped: the previous token block's last stage may still be read by other waves)
    if (tb != tb_b) __builtin_amdgcn_s_barrier();
    const int tok0 = base + tb * 128;
    const int tile0 = tok0 / 32;
    const int ntt = min(4, tile_end - tile0);         // token tiles of this block

    // ---- the LDS-DMA copy of superblock sb into stage st: piece i (1 KiB) of the stage image.
    // Every piece is a wave-uniform base (scalar registers) + a per-lane 32-bit offset; the bases
    // of superblock 0 and their per-superblock steps are computed once per token block.
    auto ubase = [](const void* p) {
        const unsigned long long v = reinterpret_cast<unsigned long long>(p);
        const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v), hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
        return reinterpret_cast<const uint8_t*>(((unsigned long long)hi << 32) | lo);
    };
    const uint8_t* pbase[C::NIW];
    unsigned pstep[C::NIW], pvo[C::NIW];
#pragma unroll
    for (int k = 0; k < C::NIW; ++k) {
        int i = wv + C::NW * k;
        if (i >= C::NI) i = C::NI - 1;                // a repeated piece: same bytes, same place
        const int off = i * 1024;                     // byte offset of the piece in the stage
        if (off < C::A_OFF) {                         // weight slot r, bytes o.. within it
            const int r = off / C::SLOT, o = off % C::SLOT;
            const int rt = min(rb * RT + r, nrt - 1);
            pbase[k] = ubase(swA + (long long)rt * nb * TB + o);
            pstep[k] = TB;
            pvo[k] = o + lane * 16 < TB ? lane * 16 : 0;   // past the tile: any valid bytes (padding)
        } else if (off < C::BSB_OFF) {                // activation tile t, 1 KiB piece j
            const int o = off - C::A_OFF, t = o >> 13, j = (o >> 10) & 7;
            const int tt = min(tile0 + t, tile_end - 1);
            pbase[k] = ubase(act.q + (long long)tt * nb * 8192 + j * 1024);
            pstep[k] = 8192;
            pvo[k] = lane * 16;
        } else if (off < C::DT_OFF) {                 // bsb of tiles 2q, 2q+1 (512 B each)
            // (tiles past the batch's last are clamped to it: their slots are never read, and
            // a batch of one or three tiles has no tile pair to read)
            const int q = (off - C::BSB_OFF) >> 10;
            const int tt = min(tile0 + 2 * q, tile_end - 1), t2 = min(tile0 + 2 * q + (lane >> 5), tile_end - 1);
            pbase[k] = ubase(act.q80 ? reinterpret_cast<const int8_t*>(act.q) : act.bsb + (long long)tt * nb * 512);
            pstep[k] = act.q80 ? 0u : 512u;
            pvo[k] = act.q80 ? 0u : (unsigned)((t2 - tt) * nb * 512 + (lane & 31) * 16);
        } else {                                      // dT: 128 tokens x 4 B per row of dT
            const int q = (off - C::DT_OFF) >> 10;    // Q8_0: rows 8sb + 2q, 8sb + 2q + 1
            pbase[k] = ubase(act.dT + (long long)(act.q80 ? 2 * q : 0) * act.npad + tok0);
            pstep[k] = (unsigned)(act.q80 ? 8 : 1) * act.npad * 4u;
            const int tk = min(4 * (lane & 31), act.npad - 4 - tok0);
            pvo[k] = (unsigned)(tk * 4 + (act.q80 ? (lane >> 5) * act.npad * 4 : 0));
        }
    }
    auto copy_stage = [&](int sb, int st) {
        char* base = smem + st * C::STAGE;
#pragma unroll
        for (int k = 0; k < C::NIW; ++k) {
            int i = wv + C::NW * k;
            if (i >= C::NI) i = C::NI - 1;
            // (written as one offset: `ub + pvo[k]` here drops the kernel's host stub, hipcc 7.2)
            const uint8_t* ub = pbase[k] + (size_t)((unsigned long long)sb * pstep[k] + pvo[k]);
            __builtin_amdgcn_global_load_lds(gp(ub), (__attribute__((address_space(3))) void*)(base + i * 1024), 16, 0, 0);
        }
    };

    float y[1][16];
#pragma unroll
    for (int e = 0; e < 16; ++e) y[0][e] = 0.0f;

    copy_stage(sb0, NST == 2 ? (sb0 & 1) : 0);
#pragma unroll 1
    for (int sb = sb0; sb < sb1; ++sb) {
        // this wave's copy of superblock sb landed, then the workgroup's (barrier; LDS-DMA is a
        // pending LDS write on the VM counter).  Past the barrier every wave is done with
        // superblock sb - 1, whose stage takes the copy of sb + 1 (in flight during this step)
        // and whose operand planes take this step's decode.
        __builtin_amdgcn_s_waitcnt((0x7 << 4) | (0xF << 8));   // vmcnt(0)
        __builtin_amdgcn_s_barrier();
        if (NST == 2 && sb + 1 < sb1) copy_stage(sb + 1, (sb + 1) & 1);
        const lchar* stg = (const lchar*)(smem + (NST == 2 ? (sb & 1) : 0) * C::STAGE);
        const lchar* A0 = stg + C::A_OFF + w * 8192 + lane * 16;       // this wave's token tile
        const lchar* dTw = stg + C::DT_OFF + (w * 32 + 4 * h) * 4;
        // a wave whose token tile is past the block's tokens (or row tile past the matrix) skips
        // its MFMAs (it still copies and decodes for the others): partial blocks, MoE groups
        const bool busy = w < ntt && rb * RT + wr < nrt;
        if (T == T_Q8_0) {
          if (busy) {
#pragma unroll 2
            for (int j = 0; j < 8; ++j) {
                const v4i a = lds_ld<v4i>(A0 + j * 1024);
                {
                    constexpr int r = 0;
                    const lchar* wt = stg + wr * C::SLOT;
                    const v4i wq = lds_ld<v4i>(wt + j * 1024 + lane * 16);
                    const unsigned dwp = lds_ld<unsigned>(wt + 8192 + col * 16 + (j >> 1) * 4);
                    const float dwj = h2f(dwp >> (16 * (j & 1)));
                    const v16i dj = mfma(a, wq);
                    const lchar* dT8 = dTw + (j >> 1) * 1024 + (j & 1) * 512;
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        const f32x4 dx4 = lds_ld<f32x4>(dT8 + 32 * g);
                        const float dx[4] = {dx4.x, dx4.y, dx4.z, dx4.w};
#pragma unroll
                        for (int i = 0; i < 4; ++i) y[r][4 * g + i] = fmaf((float)dj[4 * g + i], dwj * dx[i], y[r][4 * g + i]);
                    }
                    asm volatile("" ::: "memory");   // no LDS load hoisted across sub-blocks
                }
            }
          }
        } else if (T == T_Q4_K || T == T_Q5_K) {
            // (1) decode: the 4 waves of row tile wr turn its superblock into two int8 operand
            //     planes of the scaled weights sc_j * q, every byte <= 127:
            //       Q4_K (sc = 8 sh + sl, q <= 15):  P0 = q * sl, P1 = q * sh,  sc q = P0 + 8 P1
            //       Q5_K (q = lo4 + 16 hb <= 31):    p = sc * q <= 1953 (16-bit products),
            //                                        P0 = p & 127, P1 = p >> 7,  sc q = P0 + 128 P1
            //     and the MFMAs accumulate the scaled sub-block sums over all 8 sub-blocks exactly
            //     (no integer multiply per result); wave w decodes piece w (sub-blocks 2w, 2w + 1)
            //     for every lane's row.
            const lchar* wt = stg + wr * C::SLOT;
            lchar* pl = (lchar*)(smem + NST * C::STAGE) + wr * (NPL * 8 * 1024) + lane * 16;
            constexpr int HDO = T == T_Q5_K ? 5120 : 4096;
            {
                const u32x4 hd = lds_ld<u32x4>(wt + HDO + col * 16);
                const u32x4 wq = lds_ld<u32x4>(wt + w * 1024 + lane * 16);
                const u32x4 qh = T == T_Q5_K ? lds_ld<u32x4>(wt + 4096 + lane * 16) : u32x4{0, 0, 0, 0};
                u32x4 o0, o1, o2, o3;   // P0/P1 of sub-block 2w, P0/P1 of sub-block 2w + 1
                q45_planes<T>(hd, wq, qh, w, o0, o1, o2, o3);
                *reinterpret_cast<__attribute__((address_space(3))) u32x4*>(pl + (0 * 8 + 2 * w) * 1024) = o0;
                *reinterpret_cast<__attribute__((address_space(3))) u32x4*>(pl + (1 * 8 + 2 * w) * 1024) = o1;
                *reinterpret_cast<__attribute__((address_space(3))) u32x4*>(pl + (0 * 8 + 2 * w + 1) * 1024) = o2;
                *reinterpret_cast<__attribute__((address_space(3))) u32x4*>(pl + (1 * 8 + 2 * w + 1) * 1024) = o3;
                __builtin_amdgcn_s_waitcnt((0xF) | (0x3 << 14) | (0x7 << 4));   // lgkmcnt(0): planes written
                __builtin_amdgcn_s_barrier();
            }
            // (2) the MFMAs: token tile w x row tile wr, the planes accumulated over the sub-blocks
            if (busy) {
                constexpr int r = 0;
                const u32x4 hd = lds_ld<u32x4>(wt + HDO + col * 16);
                v16i acc0 = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, acc1 = acc0;
                const lchar* plr = (const lchar*)pl;
                // every operand of the superblock read first (at 2 waves per SIMD the LDS latency
                // is hidden only by reads in flight: counted waits, not lgkmcnt(0) per MFMA pair)
                v4i av[8], b0[8], b1[8];
                auto ld = [&](int j) {
                    av[j] = lds_ld<v4i>(A0 + j * 1024);
                    b0[j] = lds_ld<v4i>(plr + (0 * 8 + j) * 1024);
                    b1[j] = lds_ld<v4i>(plr + (1 * 8 + j) * 1024);
                };
                auto mm = [&](int j) {
                    if (NST == 2) {
                        pin(av[j]);
                        pin(b0[j]);
                        pin(b1[j]);
                    }
                    acc0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(av[j], b0[j], acc0, 0, 0, 0);
                    acc1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(av[j], b1[j], acc1, 0, 0, 0);
                };
                // sub-blocks 0-3 read, then 4-7 read while 0-3 run
#pragma unroll
                for (int j = 0; j < 4; ++j) ld(j);
                if (NST == 2) pin_all();
#pragma unroll
                for (int j = 4; j < 8; ++j) ld(j);
#pragma unroll
                for (int j = 0; j < 8; ++j) mm(j);
                // sum_j m_j*bsum_j: mins as int8 B operands, k 0-7 (against hi) / k 8-15 (against lo)
                const unsigned Y = hd.y, Z = hd.z, W = hd.w;
                const int m03 = (int)(Z & 0x3F3F3F3Fu);
                const int m47 = (int)(((W >> 4) & 0x0F0F0F0Fu) | ((Z >> 2) & 0x30303030u));
                (void)Y;
                const v4i bm1 = h == 0 ? v4i{m03, m47, 0, 0} : v4i{0, 0, 0, 0};
                const v4i bm2 = h == 0 ? v4i{0, 0, m03, m47} : v4i{0, 0, 0, 0};
                const v4i ab = h == 0 ? lds_ld<v4i>(stg + C::BSB_OFF + w * 512 + col * 16) : v4i{0, 0, 0, 0};
                const v16i x1 = mfma(ab, bm1);
                const v16i x2 = mfma(ab, bm2);
                const float dr = h2f(hd.x), dmr = h2f(hd.x >> 16);
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const f32x4 dx4 = lds_ld<f32x4>(dTw + 32 * g);
                    const float dx[4] = {dx4.x, dx4.y, dx4.z, dx4.w};
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int e = 4 * g + i;
                        const int S = acc0[e] + (T == T_Q5_K ? 128 : 8) * acc1[e];
                        const float d = dr * dx[i], dm = dmr * dx[i];
                        y[r][e] = fmaf(-dm, (float)(64 * x1[e] + x2[e]), fmaf(d, (float)S, y[r][e]));
                    }
                }
            }
        } else {   // Q6_K: the 8 spans of w = 64*hi + lo, each operand accumulated by the MFMA
            if (busy) {
                constexpr int r = 0;
                const lchar* wt = stg + wr * C::SLOT;
                v16i ah = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, al = ah;
                v4i av[8], bh[8], bl[8];   // operands read first (counted LDS waits)
#pragma unroll
                for (int sp = 0; sp < 8; ++sp) {
                    av[sp] = lds_ld<v4i>(A0 + sp * 1024);
                    bh[sp] = lds_ld<v4i>(wt + sp * 1024 + lane * 16);
                    bl[sp] = lds_ld<v4i>(wt + 8192 + sp * 1024 + lane * 16);
                }
#pragma unroll
                for (int sp = 0; sp < 8; ++sp) {
                    if (NST == 2) {
                        pin(av[sp]);
                        pin(bh[sp]);
                        pin(bl[sp]);
                    }
                    ah = __builtin_amdgcn_mfma_i32_32x32x32_i8(av[sp], bh[sp], ah, 0, 0, 0);
                    al = __builtin_amdgcn_mfma_i32_32x32x32_i8(av[sp], bl[sp], al, 0, 0, 0);
                }
                const float dr = h2f(lds_ld<unsigned short>(wt + 16384 + col * 2));
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const f32x4 dx4 = lds_ld<f32x4>(dTw + 32 * g);
                    const float dx[4] = {dx4.x, dx4.y, dx4.z, dx4.w};
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int e = 4 * g + i;
                        y[r][e] = fmaf(dr * dx[i], (float)(ah[e] * 64 + al[e]), y[r][e]);
                    }
                }
            }
        }
        __builtin_amdgcn_s_waitcnt((0xF) | (0x3 << 14) | (0x7 << 4));   // lgkmcnt(0): this wave's LDS reads done
        if (NST == 1 && sb + 1 < sb1) {   // the one stage is free once every wave is past it
            __builtin_amdgcn_s_barrier();
            copy_stage(sb + 1, 0);
        }
    }
    // ---- epilogue: token tile w, row tile rb*RT + wr (no LDS: the next block's copy may start)
    const int rt = rb * RT + wr;
    if (w < ntt && rt < nrt) {
        const int row = AB ? rt * 16 + (col & 15) : rt * 32 + col;
        // split-K: this part's partial sums, stored plainly; else the segment's epilogue
        if (P.ksplit > 1)
            mmq_epilogue<AB>(P, tend, rope, tok0 + 32 * w, lane, row, y[0], EPI_STORE, rows_s,
                             P.part + (long long)kh * P.ntok * P.out_stride);
        else
            mmq_epilogue<AB>(P, tend, rope, tok0 + 32 * w, lane, row, y[0], epi_s, rows_s, P.out);
    }
  }
}

// =============================================================================================
// mmqs: short batches (<= MMQS_MAX tokens: the verification sizes, Session.cpp:231-244) on the
// same int8 MFMAs, streamed like the decode GEMV instead of tiled like a GEMM.  At 20-64 tokens
// a weight byte feeds at most 2 MFMA token tiles, so the launch is an HBM stream: every weight
// byte is read once, straight into registers (no LDS staging, no per-superblock barrier), and
// the grid is spread over K as well as over rows so that enough waves are in flight:
//   * workgroup = MS_NW waves = MS_NW row tiles (32 rows; a gate/up pair tile: 16 + 16) x one
//     K-part of sbw superblocks; the part's activation tiles (all NT token tiles, bsums, d) are
//     LDS-DMA'd once at entry, shared by the waves;
//   * each wave issues the weight loads of its first D superblocks at entry and refills the ring
//     as it computes; the arithmetic per superblock is mmq2's (scaled int8 operand planes, the
//     mins by MFMA, the same fmaf update), so every per-part sum is mmq2's exactly;
//   * the K-parts write plain partial sums part[kp][ntok][pstride]; the consumer adds them in part
//     order: launch_quant_act (residual x, or silu(gate) * up for the FFN down input),
//     launch_qkv_finish (RoPE, KV append), launch_part_sum (output head, the last residual).
// =============================================================================================
constexpr int MS_NW = 4;     // waves (row tiles) per workgroup
constexpr int MS_SBW = 4;    // superblocks per K-part
struct MsArgs {
    const uint8_t* sw[MMQ_SEGS];   // MFMA-order copies
    int nrt[MMQ_SEGS];             // row tiles per segment
    int rows[MMQ_SEGS];
    int prow[MMQ_SEGS];            // the segment's first row in the partial row space
    int n;                         // segments
    int nrt_tot;
    int kp;                        // K-parts (grid = row blocks x kp)
    int sbw;                       // superblocks per K-part (<= MS_SBW)
    int nff;                       // pair launches: the up rows' offset in the partial row space
    float* part;                   // [kp][prows][pstride]
    int pstride;
    int prows;                     // rows of one part: the batch's tokens (grouped: the MoE rows)
    // grouped (MoE, mmqs1 only): blockIdx.y = expert e, whose rows [grp[e], + grp[grp_n + 1 + e])
    // of the activation (whole 32-row tiles, moe_group_kernel) read expert e's copy at
    // sw[0] + e * grp_stride; blockIdx.z = the 32-row tile within the expert
    const int* grp;
    int grp_n;
    long long grp_stride;
};
// 16-B weight loads per superblock of a row tile (NV) and the wave's ring depth (D)
template <int T> struct MsT;
template <> struct MsT<T_Q4_K> { static constexpr int NV = 5, D = 4; };    // qs [4] | header
template <> struct MsT<T_Q5_K> { static constexpr int NV = 6, D = 4; };    // qs [4] | qh | header
template <> struct MsT<T_Q6_K> { static constexpr int NV = 16, D = 2; };   // hi [8] | lo [8] (+ d)
template <> struct MsT<T_Q8_0> { static constexpr int NV = 9, D = 2; };    // qs [8] | d [8 x f16]
template <int T> struct MsW {
    u32x4 v[MsT<T>::NV];
    unsigned d6;   // Q6_K: the row's d
};
template <int T>
__device__ __forceinline__ MsW<T> ms_load(const uint8_t* tile, int lane) {
    const int col = lane & 31;
    MsW<T> w;
    auto ld = [&](int off) { return __builtin_nontemporal_load(gp(reinterpret_cast<const u32x4*>(tile + off))); };
    if (T == T_Q4_K || T == T_Q5_K) {
#pragma unroll
        for (int p = 0; p < 4; ++p) w.v[p] = ld(p * 1024 + lane * 16);
        if (T == T_Q5_K) w.v[4] = ld(4096 + lane * 16);
        w.v[MsT<T>::NV - 1] = ld((T == T_Q5_K ? 5120 : 4096) + col * 16);
        w.d6 = 0;
    } else if (T == T_Q6_K) {
#pragma unroll
        for (int sp = 0; sp < 8; ++sp) {
            w.v[sp] = ld(sp * 1024 + lane * 16);
            w.v[8 + sp] = ld(8192 + sp * 1024 + lane * 16);
        }
        w.d6 = __builtin_nontemporal_load(gp(reinterpret_cast<const unsigned short*>(tile + 16384 + col * 2)));
    } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) w.v[j] = ld(j * 1024 + lane * 16);
        w.v[8] = ld(8192 + col * 16);
        w.d6 = 0;
    }
    return w;
}
__device__ __forceinline__ v16i mfma_acc(v4i a, v4i b, v16i c) { return __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c, 0, 0, 0); }
__device__ __forceinline__ v4i as_v4i(const unsigned p[4]) { return v4i{(int)p[0], (int)p[1], (int)p[2], (int)p[3]}; }

// one superblock (local index s of the part) of this wave's row tile into y[NT][16]
template <int T, int NT>
__device__ __forceinline__ void ms_sb(const MsW<T>& w, int s, const char* lds, int QB, int DB, int lane,
                                      float y[NT][16]) {
    typedef __attribute__((address_space(3))) const char lc;
    const lc* L = (const lc*)lds;
    const int col = lane & 31, h = lane >> 5;
    (void)col;
    auto act = [&](int t, int j) {
        return *reinterpret_cast<const __attribute__((address_space(3))) v4i*>(L + (s * NT + t) * 8192 + j * 1024 + lane * 16);
    };
    auto dx4 = [&](int off) { return *reinterpret_cast<const __attribute__((address_space(3))) f32x4*>(L + off); };
    if (T == T_Q4_K || T == T_Q5_K) {
        const u32x4 hd = w.v[MsT<T>::NV - 1];
        int sc[8], mn[8];
        q4k_scales(hd, sc, mn);
        const v16i z = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        // [hf]: even / odd sub-blocks in separate accumulators -- four independent MFMA chains per
        // token tile instead of two (a dependent MFMA waits out its predecessor's latency)
        v16i acc0[2][NT], acc1[2][NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) acc0[0][t] = acc1[0][t] = acc0[1][t] = acc1[1][t] = z;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const unsigned q[4] = {w.v[p].x, w.v[p].y, w.v[p].z, w.v[p].w};
#pragma unroll
            for (int hf = 0; hf < 2; ++hf) {
                const int j = 2 * p + hf;
                unsigned P0[4], P1[4];
                if (T == T_Q4_K) {   // sc q = P0 + 8 P1 (P0 = q (sc & 7), P1 = q (sc >> 3), bytes <= 105)
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const unsigned nib = hf ? (q[i] >> 4) & 0x0F0F0F0Fu : q[i] & 0x0F0F0F0Fu;
                        P0[i] = bmul(nib, sc[j] & 7);
                        P1[i] = bmul(nib, sc[j] >> 3);
                    }
                } else {             // sc q = P0 + 128 P1 (q = lo4 + 16 hb <= 31)
                    const unsigned b[4] = {w.v[4].x, w.v[4].y, w.v[4].z, w.v[4].w};
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const unsigned q5 = ((hf ? q[i] >> 4 : q[i]) & 0x0F0F0F0Fu) | (((b[i] >> j) & 0x01010101u) << 4);
                        const unsigned m02 = wmul16(q5 & 0x00FF00FFu, sc[j]), m13 = wmul16((q5 >> 8) & 0x00FF00FFu, sc[j]);
                        P0[i] = (m02 & 0x007F007Fu) | ((m13 & 0x007F007Fu) << 8);
                        P1[i] = ((m02 >> 7) & 0x001F001Fu) | (((m13 >> 7) & 0x001F001Fu) << 8);
                    }
                }
                const v4i b0 = as_v4i(P0), b1 = as_v4i(P1);
#pragma unroll
                for (int t = 0; t < NT; ++t) {
                    const v4i a = act(t, j);
                    acc0[hf][t] = mfma_acc(a, b0, acc0[hf][t]);
                    acc1[hf][t] = mfma_acc(a, b1, acc1[hf][t]);
                }
            }
        }
        // sum_j m_j*bsum_j by MFMA (mmq2's form): bsums 64 hi + lo as A, the row's mins as B
        const unsigned Z = hd.z, W = hd.w;
        const int m03 = (int)(Z & 0x3F3F3F3Fu);
        const int m47 = (int)(((W >> 4) & 0x0F0F0F0Fu) | ((Z >> 2) & 0x30303030u));
        const v4i bm1 = h == 0 ? v4i{m03, m47, 0, 0} : v4i{0, 0, 0, 0};
        const v4i bm2 = h == 0 ? v4i{0, 0, m03, m47} : v4i{0, 0, 0, 0};
        const float dr = h2f(hd.x), dmr = h2f(hd.x >> 16);
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const v4i ab = h == 0 ? *reinterpret_cast<const __attribute__((address_space(3))) v4i*>(L + QB + (s * NT + t) * 1024 + col * 16)
                                  : v4i{0, 0, 0, 0};
            const v16i x1 = mfma(ab, bm1);
            const v16i x2 = mfma(ab, bm2);
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const f32x4 d4 = dx4(DB + s * 256 + (t * 32 + 8 * g + 4 * h) * 4);
                const float dx[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int e = 4 * g + i;
                    const int S = (acc0[0][t][e] + acc0[1][t][e]) + (T == T_Q5_K ? 128 : 8) * (acc1[0][t][e] + acc1[1][t][e]);
                    const float d = dr * dx[i], dm = dmr * dx[i];
                    y[t][e] = fmaf(-dm, (float)(64 * x1[e] + x2[e]), fmaf(d, (float)S, y[t][e]));
                }
            }
        }
    } else if (T == T_Q6_K) {
        const v16i z = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        v16i ah[2][NT], al[2][NT];   // [sp & 1]: four independent MFMA chains per token tile
#pragma unroll
        for (int t = 0; t < NT; ++t) ah[0][t] = al[0][t] = ah[1][t] = al[1][t] = z;
#pragma unroll
        for (int sp = 0; sp < 8; ++sp) {
            const unsigned ph[4] = {w.v[sp].x, w.v[sp].y, w.v[sp].z, w.v[sp].w};
            const unsigned pl[4] = {w.v[8 + sp].x, w.v[8 + sp].y, w.v[8 + sp].z, w.v[8 + sp].w};
            const v4i bh = as_v4i(ph), bl = as_v4i(pl);
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const v4i a = act(t, sp);
                ah[sp & 1][t] = mfma_acc(a, bh, ah[sp & 1][t]);
                al[sp & 1][t] = mfma_acc(a, bl, al[sp & 1][t]);
            }
        }
        const float dr = h2f(w.d6);
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const f32x4 d4 = dx4(DB + s * 256 + (t * 32 + 8 * g + 4 * h) * 4);
                const float dx[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int e = 4 * g + i;
                    y[t][e] = fmaf(dr * dx[i], (float)((ah[0][t][e] + ah[1][t][e]) * 64 + (al[0][t][e] + al[1][t][e])), y[t][e]);
                }
            }
    } else {   // Q8_0: one MFMA per 32-block, vec_dot_q8_0_q8_0's per-block float update
        const u32x4 hdr = w.v[8];
        const unsigned hw[4] = {hdr.x, hdr.y, hdr.z, hdr.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const unsigned pq[4] = {w.v[j].x, w.v[j].y, w.v[j].z, w.v[j].w};
            const v4i wq = as_v4i(pq);
            const float dwj = h2f(hw[j >> 1] >> (16 * (j & 1)));
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const v16i dj = mfma(act(t, j), wq);
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const f32x4 d4 = dx4(DB + (s * 8 + j) * 256 + (t * 32 + 8 * g + 4 * h) * 4);
                    const float dx[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
                    for (int i = 0; i < 4; ++i) y[t][4 * g + i] = fmaf((float)dj[4 * g + i], dwj * dx[i], y[t][4 * g + i]);
                }
            }
            // block j's updates before block j + 1's operand reads (volatile asm keeps its order, the
            // memory clobber keeps the LDS reads behind it): one block's MFMA results live at a time
#pragma unroll
            for (int t = 0; t < NT; ++t)
#pragma unroll
                for (int e = 0; e < 16; ++e) asm volatile("" : "+v"(y[t][e]));
            asm volatile("" ::: "memory");
        }
    }
}

template <int T, bool AB, int NT>
__global__ __launch_bounds__(64 * MS_NW) void mmqs_t(const MsArgs M, const ActQ8 act) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr bool KQ = T != T_Q8_0;
    constexpr int D = MsT<T>::D;
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int col = lane & 31, h = lane >> 5;
    const int nb = act.K >> 8;
    const int kp = (int)blockIdx.x % M.kp, rb = (int)blockIdx.x / M.kp;
    const int sb0 = kp * M.sbw, nsb = min(M.sbw, nb - sb0);   // (the host sizes kp: nsb >= 1)
    // LDS: q [s][t] 8 KiB | k-quants: bsb [s][t] 1 KiB, dT [s] 256 B | Q8_0: dT [s][j] 256 B
    const int QB = M.sbw * NT * 8192;
    const int DB = QB + (KQ ? M.sbw * NT * 1024 : 0);
    typedef __attribute__((address_space(3))) void lv;
    // (1) this part's activation pieces (every token tile), LDS-DMA spread over the waves
    for (int i = wv; i < nsb * NT * 8; i += MS_NW) {
        const int s = i / (NT * 8), t = (i >> 3) % NT, j = i & 7;
        const int8_t* src = act.q + ((long long)t * nb + sb0 + s) * 8192 + j * 1024 + lane * 16;
        __builtin_amdgcn_global_load_lds(gp(src), (lv*)(smem + (s * NT + t) * 8192 + j * 1024), 16, 0, 0);
    }
    const int tl = min(lane, act.npad - 1);   // dT: token lane (a 32-token batch: lanes 32.. repeat)
    if (KQ) {
        for (int i = wv; i < nsb * NT; i += MS_NW) {   // bsb of (s, t) = i: 32 tokens x 16 B, twice
            const int s = i / NT, t = i % NT;
            const int8_t* src = act.bsb + ((long long)t * nb + sb0 + s) * 512 + col * 16;
            __builtin_amdgcn_global_load_lds(gp(src), (lv*)(smem + QB + i * 1024), 16, 0, 0);
        }
        for (int s = wv; s < nsb; s += MS_NW)
            __builtin_amdgcn_global_load_lds(gp(act.dT + (long long)(sb0 + s) * act.npad + tl), (lv*)(smem + DB + s * 256), 4, 0, 0);
    } else {
        for (int i = wv; i < nsb * 8; i += MS_NW)     // rows 8 (sb0 + s) + j of the per-32 d
            __builtin_amdgcn_global_load_lds(gp(act.dT + (long long)(8 * sb0 + i) * act.npad + tl), (lv*)(smem + DB + i * 256), 4, 0, 0);
    }
    // (2) this wave's row tile and the first D superblocks of its weights
    int g = rb * MS_NW + wv;
    const bool busy = g < M.nrt_tot;
    if (!busy) g = M.nrt_tot - 1;
    int seg = 0, rt = g;
#pragma unroll
    for (int i = 0; i < MMQ_SEGS - 1; ++i)
        if (i + 1 < M.n && seg == i && rt >= M.nrt[i]) {
            rt -= M.nrt[i];
            seg = i + 1;
        }
    const uint8_t* swA = seg == 0 ? M.sw[0] : seg == 1 ? M.sw[1] : M.sw[2];
    const int rows_s = seg == 0 ? M.rows[0] : seg == 1 ? M.rows[1] : M.rows[2];
    const int prow_s = seg == 0 ? M.prow[0] : seg == 1 ? M.prow[1] : M.prow[2];
    constexpr int TB = mmq32_tile_bytes_d(T);
    const uint8_t* tile0 = swA + ((long long)rt * nb + sb0) * TB;
    MsW<T> w[D];
    // a busy wave waits for its DMA only (issued before its NLD weight loads: loads retire in
    // order), so superblock 0's dots start while the later ones are still arriving
    constexpr int NLD = D * (MsT<T>::NV + (T == T_Q6_K ? 1 : 0));
    static_assert(NLD <= 63, "vmcnt range");
    if (busy) {
#pragma unroll
        for (int d = 0; d < D; ++d) w[d] = ms_load<T>(tile0 + (long long)min(d, nsb - 1) * TB, lane);
        asm volatile("" ::: "memory");   // every ring load issued before the wait
        __builtin_amdgcn_s_waitcnt((NLD & 0xF) | ((NLD >> 4) << 14) | (0x7 << 4) | (0xF << 8));   // vmcnt(NLD)
    } else {
        __builtin_amdgcn_s_waitcnt((0x7 << 4) | (0xF << 8));   // vmcnt(0)
    }
    __builtin_amdgcn_s_barrier();
    if (!busy) return;
    float y[NT][16];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int e = 0; e < 16; ++e) y[t][e] = 0.0f;
    for (int i = 0; i < nsb; i += D) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const int s = i + d;
            if (s < nsb) {
                const MsW<T> cur = w[d];
                if (s + D < nsb) w[d] = ms_load<T>(tile0 + (long long)(s + D) * TB, lane);
                ms_sb<T, NT>(cur, s, smem, QB, DB, lane, y);
            }
        }
    }
    // (3) the partial sums of this part: lane = weight row, 16 tokens per token tile
    const int rr = AB ? rt * 16 + (col & 15) : rt * 32 + col;
    if (rr >= rows_s) return;
    const int prow = prow_s + (AB && col >= 16 ? M.nff : 0) + rr;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int tok = t * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            if (tok < act.ntok) M.part[((long long)kp * act.ntok + tok) * M.pstride + prow] = y[t][r];
        }
}

// mmqs1: the one-token-tile (<= 32 tokens) k-quant form with no LDS: a workgroup is ONE wave =
// one row tile x one K-part (4x the workgroups of mmqs_t, so a launch of few row blocks -- the 7B
// WO at 128 row tiles -- still covers every CU), and the wave streams its activation pieces
// (8 A operands, the bsums, the 16 token scales per superblock) through registers next to its
// weights, both DA / DW superblocks ahead.  No barrier, no LDS-DMA: every wait is the compiler's
// count of this wave's own loads.  Same arithmetic as ms_sb (sum for sum).
struct MsAct {
    v4i a[8];     // A operands of sub-blocks 0..7
    v4i ab;       // bsums (64 hi + lo) of token col (lanes h = 1: zero)
    f32x4 dx[4];  // d of tokens 8g + 4h .. + 3
};
__device__ __forceinline__ MsAct ms_act_load(const ActQ8& act, int sb, int lane) {
    const int col = lane & 31, h = lane >> 5;
    MsAct r;
    const int8_t* q = act.q + (long long)sb * 8192 + lane * 16;
#pragma unroll
    for (int j = 0; j < 8; ++j) r.a[j] = __builtin_nontemporal_load(gp(reinterpret_cast<const v4i*>(q + j * 1024)));
    const v4i b = *gp(reinterpret_cast<const v4i*>(act.bsb + (long long)sb * 512 + col * 16));
    r.ab = h == 0 ? b : v4i{0, 0, 0, 0};
#pragma unroll
    for (int g = 0; g < 4; ++g) r.dx[g] = *gp(reinterpret_cast<const f32x4*>(act.dT + (long long)sb * act.npad + 8 * g + 4 * h));
    return r;
}
template <int T>
__device__ __forceinline__ void ms1_sb(const MsW<T>& w, const MsAct& A, int lane, float y[16]) {
    const int h = lane >> 5;
    const v16i z = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    if (T == T_Q4_K || T == T_Q5_K) {
        const u32x4 hd = w.v[MsT<T>::NV - 1];
        int sc[8], mn[8];
        q4k_scales(hd, sc, mn);
        v16i acc0 = z, acc1 = z;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const unsigned q[4] = {w.v[p].x, w.v[p].y, w.v[p].z, w.v[p].w};
#pragma unroll
            for (int hf = 0; hf < 2; ++hf) {
                const int j = 2 * p + hf;
                unsigned P0[4], P1[4];
                if (T == T_Q4_K) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const unsigned nib = hf ? (q[i] >> 4) & 0x0F0F0F0Fu : q[i] & 0x0F0F0F0Fu;
                        P0[i] = bmul(nib, sc[j] & 7);
                        P1[i] = bmul(nib, sc[j] >> 3);
                    }
                } else {
                    const unsigned b[4] = {w.v[4].x, w.v[4].y, w.v[4].z, w.v[4].w};
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const unsigned q5 = ((hf ? q[i] >> 4 : q[i]) & 0x0F0F0F0Fu) | (((b[i] >> j) & 0x01010101u) << 4);
                        const unsigned m02 = wmul16(q5 & 0x00FF00FFu, sc[j]), m13 = wmul16((q5 >> 8) & 0x00FF00FFu, sc[j]);
                        P0[i] = (m02 & 0x007F007Fu) | ((m13 & 0x007F007Fu) << 8);
                        P1[i] = ((m02 >> 7) & 0x001F001Fu) | (((m13 >> 7) & 0x001F001Fu) << 8);
                    }
                }
                acc0 = mfma_acc(A.a[j], as_v4i(P0), acc0);
                acc1 = mfma_acc(A.a[j], as_v4i(P1), acc1);
            }
        }
        const unsigned Z = hd.z, W = hd.w;
        const int m03 = (int)(Z & 0x3F3F3F3Fu);
        const int m47 = (int)(((W >> 4) & 0x0F0F0F0Fu) | ((Z >> 2) & 0x30303030u));
        const v4i bm1 = h == 0 ? v4i{m03, m47, 0, 0} : v4i{0, 0, 0, 0};
        const v4i bm2 = h == 0 ? v4i{0, 0, m03, m47} : v4i{0, 0, 0, 0};
        const v16i x1 = mfma(A.ab, bm1);
        const v16i x2 = mfma(A.ab, bm2);
        const float dr = h2f(hd.x), dmr = h2f(hd.x >> 16);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const float dx[4] = {A.dx[g].x, A.dx[g].y, A.dx[g].z, A.dx[g].w};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int e = 4 * g + i;
                const int S = acc0[e] + (T == T_Q5_K ? 128 : 8) * acc1[e];
                const float d = dr * dx[i], dm = dmr * dx[i];
                y[e] = fmaf(-dm, (float)(64 * x1[e] + x2[e]), fmaf(d, (float)S, y[e]));
            }
        }
    } else {   // Q6_K
        v16i ah = z, al = z;
#pragma unroll
        for (int sp = 0; sp < 8; ++sp) {
            const unsigned ph[4] = {w.v[sp].x, w.v[sp].y, w.v[sp].z, w.v[sp].w};
            const unsigned pl[4] = {w.v[8 + sp].x, w.v[8 + sp].y, w.v[8 + sp].z, w.v[8 + sp].w};
            ah = mfma_acc(A.a[sp], as_v4i(ph), ah);
            al = mfma_acc(A.a[sp], as_v4i(pl), al);
        }
        const float dr = h2f(w.d6);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const float dx[4] = {A.dx[g].x, A.dx[g].y, A.dx[g].z, A.dx[g].w};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int e = 4 * g + i;
                y[e] = fmaf(dr * dx[i], (float)(ah[e] * 64 + al[e]), y[e]);
            }
        }
    }
}
template <int T> struct Ms1D { static constexpr int DW = 2, DA = 2; };
template <> struct Ms1D<T_Q6_K> { static constexpr int DW = 1, DA = 2; };

// LEAN: one-deep rings, sized for two waves per SIMD (mmqs1_lean_t)
template <int T, bool AB, bool G, bool LEAN>
__device__ __forceinline__ void mmqs1_body(const MsArgs& M, const ActQ8& act_in) {
    constexpr int DW = LEAN ? 1 : Ms1D<T>::DW, DA = LEAN ? 1 : Ms1D<T>::DA;
    const int lane = threadIdx.x & 63;
    const int col = lane & 31, h = lane >> 5;
    const int nb = act_in.K >> 8;
    const int kp = (int)blockIdx.x % M.kp, g = (int)blockIdx.x / M.kp;
    const int sb0 = kp * M.sbw, nsb = min(M.sbw, nb - sb0);
    // this workgroup's token rows: [r0, r0 + ntk) of the partial row space, read from the
    // activation's 32-row tile r0 / 32 (grouped: expert e's tile z; exits past its rows)
    ActQ8 act = act_in;
    int r0 = 0, ntk = act_in.ntok;
    long long eoff = 0;
    if (G) {
        const int e = blockIdx.y, z = blockIdx.z;
        const int cnt = M.grp[M.grp_n + 1 + e];
        if (z * 32 >= cnt) return;
        r0 = M.grp[e] + z * 32;
        ntk = min(32, cnt - z * 32);
        const int tt = r0 >> 5;
        act.q += (long long)tt * nb * 8192;
        act.bsb += (long long)tt * nb * 512;
        act.dT += tt * 32;
        eoff = (long long)e * M.grp_stride;
    }
    int seg = 0, rt = g;
#pragma unroll
    for (int i = 0; i < MMQ_SEGS - 1; ++i)
        if (i + 1 < M.n && seg == i && rt >= M.nrt[i]) {
            rt -= M.nrt[i];
            seg = i + 1;
        }
    const uint8_t* swA = seg == 0 ? M.sw[0] : seg == 1 ? M.sw[1] : M.sw[2];
    const int rows_s = seg == 0 ? M.rows[0] : seg == 1 ? M.rows[1] : M.rows[2];
    const int prow_s = seg == 0 ? M.prow[0] : seg == 1 ? M.prow[1] : M.prow[2];
    constexpr int TB = mmq32_tile_bytes_d(T);
    const uint8_t* tile0 = swA + eoff + ((long long)rt * nb + sb0) * TB;
    // activation first, then weights (loads retire in order: superblock 0's act is never queued
    // behind later weights)
    MsAct a[DA];
#pragma unroll
    for (int d = 0; d < DA; ++d) a[d] = ms_act_load(act, sb0 + min(d, nsb - 1), lane);
    MsW<T> w[DW];
#pragma unroll
    for (int d = 0; d < DW; ++d) w[d] = ms_load<T>(tile0 + (long long)min(d, nsb - 1) * TB, lane);
    float y[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) y[e] = 0.0f;
    // fully unrolled over the part's (at most MS_SBW) superblocks: every ring slot is a value of its
    // own, so a refill issued before the slot's dots needs no register copy
#pragma unroll
    for (int s = 0; s < MS_SBW; ++s) {
        if (s < nsb) {
            const MsAct ca = a[s % DA];
            const MsW<T> cw = w[s % DW];
            if (s + DA < nsb) a[s % DA] = ms_act_load(act, sb0 + s + DA, lane);
            if (s + DW < nsb) w[s % DW] = ms_load<T>(tile0 + (long long)(s + DW) * TB, lane);
            ms1_sb<T>(cw, ca, lane, y);
        }
    }
    const int rr = AB ? rt * 16 + (col & 15) : rt * 32 + col;
    if (rr >= rows_s) return;
    const int prow = prow_s + (AB && col >= 16 ? M.nff : 0) + rr;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int tok = (r & 3) + 8 * (r >> 2) + 4 * h;
        if (tok < ntk) M.part[((long long)kp * M.prows + r0 + tok) * M.pstride + prow] = y[r];
    }
}
template <int T, bool AB, bool G>
__global__ __launch_bounds__(64) void mmqs1_t(const MsArgs M, const ActQ8 act) { mmqs1_body<T, AB, G, false>(M, act); }
template <int T, bool AB, bool G>
__global__ __launch_bounds__(64, 2) void mmqs1_lean_t(const MsArgs M, const ActQ8 act) { mmqs1_body<T, AB, G, true>(M, act); }

// the sum of the K-parts in part order, with the consumer's epilogue: Q / K RoPE (ggml NORM, the
// rope table of the batch), Q to q, K / V to the f16 caches (and the cell positions)
__global__ __launch_bounds__(256) void qkv_finish_kernel(const QkvFinish F) {
    const int t = blockIdx.y;
    const int pr = blockIdx.x * 256 + threadIdx.x;   // row pair
    const int r = 2 * pr;
    if (r >= F.nq + F.nk + F.nv) return;
    const float2* p = reinterpret_cast<const float2*>(F.part + (long long)t * F.pstride + r);
    const float2 v = sum_parts(p, (long long)F.ntok * F.pstride / 2, F.kp);   // (pstride even: nq, nk, nv are)
    const float v0 = v.x, v1 = v.y;
    const int seg = r < F.nq ? 0 : r < F.nq + F.nk ? 1 : 2;
    const int row = seg == 0 ? r : seg == 1 ? r - F.nq : r - F.nq - F.nk;
    float o0 = v0, o1 = v1;
    if (seg < 2) {
        const int i0 = row % F.head_dim;
        if (i0 < F.n_rot) {   // mmq_epilogue's expressions: even v cos - pv sin, odd pv sin + v cos
            const float2 cs = F.rope[(long long)t * (F.n_rot / 2) + i0 / 2];
            o0 = v0 * cs.x - v1 * cs.y;
            o1 = v0 * cs.y + v1 * cs.x;
        }
    }
    const int* tp = F.tokpos + t * 4;
    if (seg == 0) {
        F.q[(long long)t * F.q_stride + row] = o0;
        F.q[(long long)t * F.q_stride + row + 1] = o1;
    } else {
        __half* c = (seg == 1 ? F.kcache : F.vcache) + (long long)tp[2] * F.kv_dim + row;
        c[0] = __float2half_rn(o0);
        c[1] = __float2half_rn(o1);
        if (seg == 1 && row == 0) F.cell_pos[tp[2]] = tp[1];
    }
}

// out[t][r] = ((p0 + p1) + ...) [+ resid[t][r]]; swiglu > 0: silu(sum of row r) * (sum of row
// swiglu + r) (a pair launch's gate and up rows)
__global__ __launch_bounds__(256) void part_sum_kernel(const float* part, int kp, int ntok, int rows, int pstride,
                                                       const float* resid, int rstride, float* out, int ostride,
                                                       int swiglu) {
    const int t = blockIdx.y;
    const int r = blockIdx.x * 256 + threadIdx.x;
    if (r >= rows) return;
    float acc = sum_parts(part + (long long)t * pstride + r, (long long)ntok * pstride, kp);
    if (swiglu) acc = silu(acc) * sum_parts(part + (long long)t * pstride + swiglu + r, (long long)ntok * pstride, kp);
    if (resid) acc = acc + resid[(long long)t * rstride + r];
    out[(long long)t * ostride + r] = acc;
}

template <int T, int NST> constexpr int m2_lds() { return M2<T>::lds(NST); }

}  // namespace mmq

void launch_quant_act(const float* x, int x_stride, const float* norm_w, float eps, const ActQ8& a, hipStream_t s,
                      const int* rows, const float* part, int nks, int swiglu) {
    if (part && (nks < 1 || nks > 64)) throw Error("quant_act: 1..64 split-K partials");
    // (swiglu with rows: the MoE rows of a grouped pair launch, rows[t] < 0 marking padding rows)
    if (swiglu && (!part || norm_w)) throw Error("quant_act: swiglu takes a pair launch's parts, no norm");
    if (!swiglu && !x) throw Error("quant_act: no input rows");
    if (a.K % 256) throw Error("quant_act: K must be a multiple of 256");
    if (part && !swiglu && (rows || x_stride != a.K)) throw Error("quant_act: split-K partials take a dense [ntok][K] x");
    // (more than UB_MAX rows only for the MoE rows of a batch: one per (token, slot), padded)
    if (a.npad % 32 || a.ntok > a.npad || a.npad > 4 * UB_MAX) throw Error("quant_act: bad token count");
    if (a.K > 65536) throw Error("quant_act: K past 65536");
    // a row without a norm needs no row-wide sum: its blocks go to ceil(nb / 16) workgroups, one
    // block per wave (the FFN down input: 3 at n_ff = 11008)
    const int nb = a.K / 256;
    const int ny = norm_w ? 1 : (nb + 15) / 16;
    const int xr = (nb + 16 * ny - 1) / (16 * ny);
    auto f = xr <= 1 ? mmq::quant_act_kernel<16, 1> : xr <= 2 ? mmq::quant_act_kernel<16, 2>
           : xr <= 4 ? mmq::quant_act_kernel<16, 4> : mmq::quant_act_kernel<16, 16>;
    hipLaunchKernelGGL(f, dim3(a.npad, ny), dim3(1024), 0, s, x, x_stride, norm_w, eps, a, rows, part, nks, swiglu);
    MI_HIP(hipGetLastError());
}

void launch_rope_table(const int* tokpos, int ntok, int n_rot, float theta_scale, float freq_scale,
                       const float* freq_factors, float2* out, hipStream_t s) {
    if (ntok <= 0 || n_rot <= 0) return;
    hipLaunchKernelGGL(mmq::rope_table_kernel, dim3(ntok), dim3(64), 0, s, tokpos, ntok, n_rot, theta_scale,
                       freq_scale, freq_factors, out);
    MI_HIP(hipGetLastError());
}

bool mmq32_supported(int type) { return type == T_Q4_K || type == T_Q5_K || type == T_Q6_K || type == T_Q8_0; }

int mmq32_tile_bytes(int type) { return mmq::mmq32_tile_bytes_d(type); }

size_t mmq32_copy_bytes(const QMat& A, bool pair) {
    const long long nrt = pair ? (A.rows + 15) / 16 : (A.rows + 31) / 32;
    return (size_t)nrt * A.nb * mmq32_tile_bytes(A.type);
}


void launch_mmq32_swizzle(const QMat& A, const QMat* B, uint8_t* dst, hipStream_t s) {
    if (!mmq32_supported(A.type)) throw Error("mmq32 swizzle: Q4_K / Q5_K / Q6_K / Q8_0 only");
    if (B && (B->type != A.type || B->rows != A.rows || B->K != A.K)) throw Error("mmq32 swizzle: bad pair");
    const long long nrt = B ? (A.rows + 15) / 16 : (A.rows + 31) / 32;
    hipLaunchKernelGGL(mmq::swizzle_kernel, dim3((unsigned)(nrt * A.nb)), dim3(256), 0, s, A, B ? *B : A, B ? 1 : 0, dst);
    MI_HIP(hipGetLastError());
}

namespace {
bool mmq2_enabled() { return true; }
// one mmq2 launch over the segments S (all of p.A's type; one segment unless launch_mmq32_multi)
void launch_mmq2(const GemmParams& p, const mmq::MmqSegs& S, const ActQ8& act, const float2* rope, hipStream_t s) {
    const bool ab = p.pair == PAIR_AB;
    const int T = p.A.type;
    const int RT = mmq::M2<T_Q4_K>::RT;
    const int NWv = 4 * RT;
    int nrb = 0;
    for (int i = 0; i < S.n; ++i) nrb += ((ab ? (S.rows[i] + 15) / 16 : (S.rows[i] + 31) / 32) + RT - 1) / RT;
    const int ntb = (act.npad + 127) / 128;
    // grouped (MoE): a workgroup per (token block, expert, row block)
    const int g1 = (nrb + 7) / 8 * 8 * (p.grp ? p.grp_n * ((max(p.grp_max, 1) + 127) / 128) : ntb);
    if (p.ksplit > 1 && (p.grp || p.pair == PAIR_AB || p.epi != EPI_ADD || !p.part || S.n != 1 || p.A.nb < p.ksplit ||
                         (p.ksplit != 2 && p.ksplit != 4)))
        throw Error("mmq2: split-K (2 or 4 parts) is for a single EPI_ADD matrix with a partials buffer");
    const int g2 = g1 * (p.ksplit > 1 ? p.ksplit : 1);
    // one stage (two workgroups per CU) when the grid fills two workgroups per CU, else two stages
    // (one per CU).  7B 512-token prefill, one vs two stages: 15.5 vs 16.8 ms (same box, r04)
    static int n_cu = 0;
    if (!n_cu) {
        int dev = 0;
        MI_HIP(hipGetDevice(&dev));
        MI_HIP(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
    }
    const int nst = g2 >= 2 * n_cu ? 1 : 2;
    decltype(&mmq::mmq2_t<T_Q4_K, false, 2>) f2;
    int lds;
#define M2_PICK(NST_)                                                                                           \
    switch (T) {                                                                                                \
    case T_Q4_K: f2 = ab ? mmq::mmq2_t<T_Q4_K, true, NST_> : mmq::mmq2_t<T_Q4_K, false, NST_>; lds = mmq::m2_lds<T_Q4_K, NST_>(); break; \
    case T_Q5_K: f2 = ab ? mmq::mmq2_t<T_Q5_K, true, NST_> : mmq::mmq2_t<T_Q5_K, false, NST_>; lds = mmq::m2_lds<T_Q5_K, NST_>(); break; \
    case T_Q6_K: f2 = ab ? mmq::mmq2_t<T_Q6_K, true, NST_> : mmq::mmq2_t<T_Q6_K, false, NST_>; lds = mmq::m2_lds<T_Q6_K, NST_>(); break; \
    default: f2 = ab ? mmq::mmq2_t<T_Q8_0, true, NST_> : mmq::mmq2_t<T_Q8_0, false, NST_>; lds = mmq::m2_lds<T_Q8_0, NST_>(); break; \
    }
    if (nst == 1) { M2_PICK(1) } else { M2_PICK(2) }
#undef M2_PICK
    static bool attr_done[2][4][2] = {};
    const int ti = T == T_Q4_K ? 0 : T == T_Q5_K ? 1 : T == T_Q6_K ? 2 : 3;
    const int ni = nst == 1 ? 0 : 1;
    if (!attr_done[ni][ti][ab]) {
        MI_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(f2), hipFuncAttributeMaxDynamicSharedMemorySize, lds));
        attr_done[ni][ti][ab] = true;
    }
    hipLaunchKernelGGL(f2, dim3(g2), dim3(64 * NWv), (size_t)lds, s, p, act, rope, S);
    MI_HIP(hipGetLastError());
}
}  // namespace

void launch_mmq32_multi(const GemmParams* ps, int n, const ActQ8& act, const float2* rope, hipStream_t s) {
    bool one = n >= 2 && n <= mmq::MMQ_SEGS && mmq2_enabled();
    for (int i = 0; i < n && one; ++i)
        one = ps[i].A.type == ps[0].A.type && ps[i].pair != PAIR_AB && !ps[i].grp && ps[i].K == ps[0].K &&
              ps[i].A.sw && ps[i].A.K == ps[0].K && ps[i].epi != EPI_SWIGLU;
    if (!one) {
        for (int i = 0; i < n; ++i) launch_mmq32(ps[i], act, rope, s);
        return;
    }
    for (int i = 0; i < n; ++i) {   // the same checks as one launch each (the shared fields are ps[0]'s)
        const GemmParams& p = ps[i];
        if ((p.epi == EPI_ROPE_Q || p.epi == EPI_ROPE_K) && (!rope || p.head_dim % 2 || p.n_rot > p.head_dim))
            throw Error("mmq32: RoPE epilogue needs the rope table");
        if (p.out != ps[0].out || p.out_stride != ps[0].out_stride || p.resid != ps[0].resid)
            throw Error("mmq32 multi: the segments share one output buffer");
    }
    if (!mmq32_supported(ps[0].A.type)) throw Error("mmq32: Q4_K / Q5_K / Q6_K / Q8_0 only");
    if ((ps[0].A.type == T_Q8_0) != (act.q80 != 0)) throw Error("mmq32: Q8_0 weights take Q8_0 activations, k-quants Q8_K");
    if (act.K != ps[0].K) throw Error("mmq32: activation length differs from K");
    if (act.ntok < 1 || act.npad % 32 || act.npad > UB_MAX) throw Error("mmq32: bad token count");
    mmq::MmqSegs S{};
    S.n = n;
    for (int i = 0; i < n; ++i) {
        S.sw[i] = ps[i].A.sw;
        S.rows[i] = ps[i].A.rows;
        S.epi[i] = ps[i].epi;
    }
    launch_mmq2(ps[0], S, act, rope, s);
}

bool mmq2_active() { return mmq2_enabled(); }

void launch_mmq32(const GemmParams& p, const ActQ8& act, const float2* rope, hipStream_t s) {
    if (!mmq32_supported(p.A.type)) throw Error("mmq32: Q4_K / Q5_K / Q6_K / Q8_0 only");
    if ((p.A.type == T_Q8_0) != (act.q80 != 0)) throw Error("mmq32: Q8_0 weights take Q8_0 activations, k-quants Q8_K");
    if (act.K != p.K || p.A.K != p.K) throw Error("mmq32: activation length differs from K");
    const bool ab = p.pair == PAIR_AB;
    if (ab && (p.B.type != p.A.type || p.B.rows != p.A.rows || p.epi != EPI_SWIGLU))
        throw Error("mmq32: a pair launch is gate/up SwiGLU of one type");
    if (!ab && p.epi == EPI_SWIGLU) throw Error("mmq32: SwiGLU needs a pair");
    if ((p.epi == EPI_ROPE_Q || p.epi == EPI_ROPE_K) && (!rope || p.head_dim % 2 || p.n_rot > p.head_dim))
        throw Error("mmq32: RoPE epilogue needs the rope table");
    if (act.ntok < 1 || act.npad % 32 || act.npad > (p.grp ? 4 * UB_MAX : UB_MAX)) throw Error("mmq32: bad token count");
    if (!p.A.sw) throw Error("mmq32: the matrix has no MFMA-order copy");
    mmq::MmqSegs S{};
    S.n = 1;
    S.sw[0] = p.A.sw;
    S.rows[0] = p.A.rows;
    S.epi[0] = p.epi;
    launch_mmq2(p, S, act, rope, s);
}

// The Q4_K / Q5_K mmqs1 launches on the one-deep-ring, two-waves-per-SIMD form (214-220 VGPRs
// instead of 246-256 at one wave: 20-token verify 7B 3.61 -> 3.40 ms, Mixtral 18.2 -> 15.7 ms,
// same box, r05).  Q6_K keeps its two-deep ring at one wave (the lean form at two waves spills).

int mmqs_parts(int K) { return (K / 256 + mmq::MS_SBW - 1) / mmq::MS_SBW; }

int launch_mmqs(const QMat* const* mats, const int* prow, int n, bool pair, int nff, const ActQ8& act, float* part,
                int pstride, hipStream_t s) {
    if (n < 1 || n > mmq::MMQ_SEGS || (pair && n != 1)) throw Error("mmqs: 1..3 matrices (a pair: one)");
    const int T = mats[0]->type;
    if (!mmq32_supported(T)) throw Error("mmqs: Q4_K / Q5_K / Q6_K / Q8_0 only");
    if ((T == T_Q8_0) != (act.q80 != 0)) throw Error("mmqs: Q8_0 weights take Q8_0 activations, k-quants Q8_K");
    if (act.ntok < 1 || act.ntok > MMQS_MAX || (act.npad != 32 && act.npad != 64) || act.npad < act.ntok)
        throw Error("mmqs: 1..64 tokens");
    if (act.K % 256 || act.K <= 0) throw Error("mmqs: K must be a multiple of 256");
    mmq::MsArgs M{};
    M.n = n;
    for (int i = 0; i < n; ++i) {
        const QMat& A = *mats[i];
        if (A.type != T || A.K != act.K || !A.sw) throw Error("mmqs: the matrices share type and K, with MFMA-order copies");
        M.sw[i] = A.sw;
        M.rows[i] = A.rows;
        M.nrt[i] = pair ? (A.rows + 15) / 16 : (A.rows + 31) / 32;
        M.prow[i] = prow[i];
        M.nrt_tot += M.nrt[i];
        const int top = prow[i] + A.rows + (pair ? nff : 0);
        if (prow[i] < 0 || top > pstride || (pair && nff < A.rows)) throw Error("mmqs: partial rows past the stride");
    }
    // (half-width parts for the launches of few row blocks, 7B WO / V at 128 workgroups, measured no
    // faster: 20-token verify 3.46 vs 3.24 ms)
    M.sbw = mmq::MS_SBW;
    M.kp = mmqs_parts(act.K);
    M.nff = nff;
    M.part = part;
    M.pstride = pstride;
    M.prows = act.ntok;
    const int NT = act.npad / 32;
    const int KQ = T != T_Q8_0;
    const int lds = mmq::MS_SBW * NT * 8192 + (KQ ? mmq::MS_SBW * NT * 1024 + mmq::MS_SBW * 256 : mmq::MS_SBW * 8 * 256);
    // one token tile, k-quants: the one-wave register form (3.42 vs 3.50 ms for the LDS form, r05)
    if (NT == 1 && T != T_Q8_0) {
        decltype(&mmq::mmqs1_t<T_Q4_K, false, false>) f1 = nullptr;
        switch (T) {
        case T_Q4_K: f1 = pair ? mmq::mmqs1_lean_t<T_Q4_K, true, false> : mmq::mmqs1_lean_t<T_Q4_K, false, false>; break;
        case T_Q5_K: f1 = pair ? mmq::mmqs1_lean_t<T_Q5_K, true, false> : mmq::mmqs1_lean_t<T_Q5_K, false, false>; break;
        default: f1 = pair ? mmq::mmqs1_t<T_Q6_K, true, false> : mmq::mmqs1_t<T_Q6_K, false, false>; break;
        }
        hipLaunchKernelGGL(f1, dim3(M.nrt_tot * M.kp), dim3(64), 0, s, M, act);
        MI_HIP(hipGetLastError());
        return M.kp;
    }
    decltype(&mmq::mmqs_t<T_Q4_K, false, 1>) f = nullptr;
#define MS_PICK(TT)                                                                                 \
    f = pair ? (NT == 1 ? mmq::mmqs_t<TT, true, 1> : mmq::mmqs_t<TT, true, 2>)                     \
             : (NT == 1 ? mmq::mmqs_t<TT, false, 1> : mmq::mmqs_t<TT, false, 2>);
    switch (T) {
    case T_Q4_K: MS_PICK(T_Q4_K) break;
    case T_Q5_K: MS_PICK(T_Q5_K) break;
    case T_Q6_K: MS_PICK(T_Q6_K) break;
    default: MS_PICK(T_Q8_0) break;
    }
#undef MS_PICK
    static bool attr_done[4][2][2] = {};
    const int ti = T == T_Q4_K ? 0 : T == T_Q5_K ? 1 : T == T_Q6_K ? 2 : 3;
    if (!attr_done[ti][pair][NT - 1]) {
        MI_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(f), hipFuncAttributeMaxDynamicSharedMemorySize, lds));
        attr_done[ti][pair][NT - 1] = true;
    }
    const int grid = (M.nrt_tot + mmq::MS_NW - 1) / mmq::MS_NW * M.kp;
    hipLaunchKernelGGL(f, dim3(grid), dim3(64 * mmq::MS_NW), (size_t)lds, s, M, act);
    MI_HIP(hipGetLastError());
    return M.kp;
}

bool mmqs_grouped_supported(int type) { return type == T_Q4_K || type == T_Q5_K || type == T_Q6_K; }

int launch_mmqs_grouped(const QMat& A, bool pair, int nff, const ActQ8& act, float* part, int pstride, const int* grp,
                        int n_expert, int max_rows, hipStream_t s) {
    const int T = A.type;
    if (!mmqs_grouped_supported(T)) throw Error("mmqs grouped: Q4_K / Q5_K / Q6_K experts only");
    if (act.q80) throw Error("mmqs grouped: k-quant experts take Q8_K activations");
    if (!A.sw || A.K != act.K || act.K % 256 || act.K <= 0) throw Error("mmqs grouped: the experts' MFMA-order copies, K a multiple of 256");
    if (act.ntok != act.npad || act.npad % 32 || act.npad < 32) throw Error("mmqs grouped: the MoE rows are whole 32-row tiles");
    if (n_expert < 1 || n_expert > A.n_exp || max_rows < 1 || max_rows > MMQS_MAX) throw Error("mmqs grouped: bad expert / row count");
    if (A.rows + (pair ? nff : 0) > pstride || (pair && nff < A.rows)) throw Error("mmqs grouped: partial rows past the stride");
    mmq::MsArgs M{};
    M.n = 1;
    M.sw[0] = A.sw;
    M.rows[0] = A.rows;
    M.nrt[0] = M.nrt_tot = pair ? (A.rows + 15) / 16 : (A.rows + 31) / 32;
    M.prow[0] = 0;
    M.sbw = mmq::MS_SBW;
    M.kp = mmqs_parts(act.K);
    M.nff = nff;
    M.part = part;
    M.pstride = pstride;
    M.prows = act.ntok;
    M.grp = grp;
    M.grp_n = n_expert;
    M.grp_stride = A.sw_expert_stride;
    decltype(&mmq::mmqs1_t<T_Q4_K, false, true>) f1 = nullptr;
    switch (T) {
    case T_Q4_K: f1 = pair ? mmq::mmqs1_lean_t<T_Q4_K, true, true> : mmq::mmqs1_lean_t<T_Q4_K, false, true>; break;
    case T_Q5_K: f1 = pair ? mmq::mmqs1_lean_t<T_Q5_K, true, true> : mmq::mmqs1_lean_t<T_Q5_K, false, true>; break;
    default: f1 = pair ? mmq::mmqs1_t<T_Q6_K, true, true> : mmq::mmqs1_t<T_Q6_K, false, true>; break;
    }
    // an expert holds at most max_rows rows (one per token routed to it): ceil(max_rows / 32) tiles
    hipLaunchKernelGGL(f1, dim3(M.nrt_tot * M.kp, n_expert, (max_rows + 31) / 32), dim3(64), 0, s, M, act);
    MI_HIP(hipGetLastError());
    return M.kp;
}

void launch_qkv_finish(const QkvFinish& F, hipStream_t s) {
    if (F.ntok < 1 || F.kp < 1 || F.nq % 2 || F.nk % 2 || F.nv % 2 || F.head_dim % 2 || F.n_rot > F.head_dim || !F.rope)
        throw Error("qkv_finish: bad shape");
    const int npair = (F.nq + F.nk + F.nv) / 2;
    hipLaunchKernelGGL(mmq::qkv_finish_kernel, dim3((npair + 255) / 256, F.ntok), dim3(256), 0, s, F);
    MI_HIP(hipGetLastError());
}

void launch_part_sum(const float* part, int kp, int ntok, int rows, int pstride, const float* resid, int rstride,
                     float* out, int ostride, hipStream_t s, int swiglu) {
    if (ntok < 1 || kp < 1 || rows < 1 || rows + swiglu > pstride || (swiglu && swiglu < rows)) throw Error("part_sum: bad shape");
    hipLaunchKernelGGL(mmq::part_sum_kernel, dim3((rows + 255) / 256, ntok), dim3(256), 0, s, part, kp, ntok, rows, pstride,
                       resid, rstride, out, ostride, swiglu);
    MI_HIP(hipGetLastError());
}

}  // namespace mi
