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
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdlib>

namespace mi {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x4 ldg16(const uint8_t* p) {
    return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
}
__device__ __forceinline__ float h2f(uint32_t bits) {
    return __half2float(__ushort_as_half(static_cast<unsigned short>(bits & 0xFFFFu)));
}
__device__ __forceinline__ int dot4(int a, int b, int c) { return __builtin_amdgcn_sdot4(a, b, c, false); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
// Full-wave sum through DPP (row_shr 1/2/4/8, row_bcast 15/31): the total
// lands in lane 63.  Fixed combination order -> deterministic.
#define MI_DPP(v, ctrl, rmask) \
    __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), ctrl, rmask, 0xf, false))
__device__ __forceinline__ float wave_sum63(float v) {
    v += MI_DPP(v, 0x111, 0xf);   // row_shr:1
    v += MI_DPP(v, 0x112, 0xf);   // row_shr:2
    v += MI_DPP(v, 0x114, 0xf);   // row_shr:4
    v += MI_DPP(v, 0x118, 0xf);   // row_shr:8  -> lane 15 of each row holds the row sum
    v += MI_DPP(v, 0x142, 0xa);   // row_bcast:15 -> rows 1,3 add lane 15 of rows 0,2
    v += MI_DPP(v, 0x143, 0xc);   // row_bcast:31 -> rows 2,3 add lane 31
    return v;                     // lane 63 = total
}
#undef MI_DPP
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// ---------------------------------------------------------------------------
// Activation quantisation (per 256-block, one wave, 4 values per lane)
// ---------------------------------------------------------------------------

// quantize_row_q8_K_ref: max = signed value of the largest |x| (first index on
// ties), iscale = -127/max, q = min(127, nearest_int(iscale*x)), d = 1/iscale.
__device__ __forceinline__ void quant_q8k_block(const float v[4], int lane, int8_t* q8, int* bsum,
                                                float* dk) {
    float ab = fabsf(v[0]);
    int ib = 0;
#pragma unroll
    for (int e = 1; e < 4; ++e) if (fabsf(v[e]) > ab) { ab = fabsf(v[e]); ib = e; }
    unsigned hi = __float_as_uint(ab);
    unsigned lo = 0xFFFFFFFFu - (unsigned)(lane * 4 + ib);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        unsigned ohi = __shfl_xor(hi, o, 64), olo = __shfl_xor(lo, o, 64);
        if (ohi > hi || (ohi == hi && olo > lo)) { hi = ohi; lo = olo; }
    }
    const int idx = (int)(0xFFFFFFFFu - lo);
    const float mine = (idx & 3) == 0 ? v[0] : (idx & 3) == 1 ? v[1] : (idx & 3) == 2 ? v[2] : v[3];
    const float mx = __shfl(mine, idx >> 2, 64);
    int q[4];
    float d;
    if (__uint_as_float(hi) == 0.0f) {
        q[0] = q[1] = q[2] = q[3] = 0;
        d = 0.0f;
    } else {
        const float iscale = -127.0f / mx;
#pragma unroll
        for (int e = 0; e < 4; ++e) q[e] = min(127, (int)rintf(iscale * v[e]));
        d = 1.0f / iscale;
    }
    const int packed = (q[0] & 0xFF) | ((q[1] & 0xFF) << 8) | ((q[2] & 0xFF) << 16) | ((q[3] & 0xFF) << 24);
    reinterpret_cast<int*>(q8)[lane] = packed;
    int s = q[0] + q[1] + q[2] + q[3];
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    if ((lane & 3) == 0) bsum[lane >> 2] = s;
    if (lane == 0) *dk = d;
}

// x86 SIMD form of quantize_row_q8_0: d = fp16(amax/127), id = 127/amax,
// q = round-to-nearest-even(x*id).  8 lanes per 32-block.
__device__ __forceinline__ void quant_q80_block(const float v[4], int lane, int8_t* q8, float* d0) {
    float am = fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3])));
    am = fmaxf(am, __shfl_xor(am, 1, 64));
    am = fmaxf(am, __shfl_xor(am, 2, 64));
    am = fmaxf(am, __shfl_xor(am, 4, 64));
    const float d = am / 127.0f;
    const float id = am != 0.0f ? 127.0f / am : 0.0f;
    int q[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) q[e] = (int)rintf(v[e] * id);
    const int packed = (q[0] & 0xFF) | ((q[1] & 0xFF) << 8) | ((q[2] & 0xFF) << 16) | ((q[3] & 0xFF) << 24);
    reinterpret_cast<int*>(q8)[lane] = packed;
    if ((lane & 7) == 0) d0[lane >> 3] = __half2float(__float2half_rn(d));
}

// ---------------------------------------------------------------------------
// LDS layout of the GEMV prologue
// ---------------------------------------------------------------------------
struct ActLayout {
    int nb, q8k, q80, bsum, dk, d0, slot_bytes;
};
__host__ __device__ inline ActLayout act_layout(int K, int need_q8k, int need_q80) {
    ActLayout L;
    L.nb = K / 256;
    int off = 0;
    L.q8k = off; off += need_q8k ? L.nb * 256 : 0;
    L.q80 = off; off += need_q80 ? L.nb * 256 : 0;
    L.bsum = off; off += need_q8k ? L.nb * 64 : 0;
    L.dk = off; off += need_q8k ? ((L.nb * 4 + 15) & ~15) : 0;
    L.d0 = off; off += need_q80 ? L.nb * 32 : 0;
    L.slot_bytes = (off + 15) & ~15;
    return L;
}

struct Act {
    const int8_t* q8k;
    const int* bsum;
    const float* dk;
    const int8_t* q80;
    const float* d0;
};

__device__ __forceinline__ Act act_view(const char* smem, const ActLayout& L, int slot) {
    const char* b = smem + slot * L.slot_bytes;
    Act a;
    a.q8k = reinterpret_cast<const int8_t*>(b + L.q8k);
    a.bsum = reinterpret_cast<const int*>(b + L.bsum);
    a.dk = reinterpret_cast<const float*>(b + L.dk);
    a.q80 = reinterpret_cast<const int8_t*>(b + L.q80);
    a.d0 = reinterpret_cast<const float*>(b + L.d0);
    return a;
}

// ---------------------------------------------------------------------------
// Per-type superblock dot products.  A wave step covers SPS superblocks with
// LPS lanes each; each lane issues one aligned 16-byte load of the main
// quant plane (plus its side planes) and returns its fp32 partial.
// ---------------------------------------------------------------------------
template <int T> struct Kq;
template <int T> struct PlaneBytes;   // bytes per superblock of each plane (common.h plane_sb_bytes)
template <> struct PlaneBytes<T_Q4_K> { static constexpr int b[4] = {128, 16, 0, 0}; };
template <> struct PlaneBytes<T_Q5_K> { static constexpr int b[4] = {128, 32, 16, 0}; };
template <> struct PlaneBytes<T_Q6_K> { static constexpr int b[4] = {128, 64, 16, 2}; };
template <> struct PlaneBytes<T_Q8_0> { static constexpr int b[4] = {256, 16, 0, 0}; };

template <> struct Kq<T_Q4_K> {
    static constexpr int LPS = 8;
    struct Ld { u32x4 qs, hdr; };
    // rp: plane pointers at the start of the row (wave-uniform); sb = s*8 + sbl
    __device__ static Ld load(const uint8_t* const* rp, int sb, int j) {
        Ld l;
        l.qs = ldg16(rp[0] + sb * 128 + j * 16);
        l.hdr = ldg16(rp[1] + sb * 16);
        return l;
    }
    // the activation slice lane (sb, j) needs -- identical for every row
    struct AR { i32x4 alo, ahi; int bs_lo, bs_hi; float dx; };
    __device__ static AR act(const Act& a, int sb, int j) {
        const int g = j >> 1, half = j & 1;
        const int8_t* ab = a.q8k + sb * 256 + 64 * g + 16 * half;
        AR r;
        r.alo = *reinterpret_cast<const i32x4*>(ab);
        r.ahi = *reinterpret_cast<const i32x4*>(ab + 32);
        r.bs_lo = a.bsum[sb * 16 + 4 * g + half];
        r.bs_hi = a.bsum[sb * 16 + 4 * g + 2 + half];
        r.dx = a.dk[sb];
        return r;
    }
    __device__ static float dot(const Ld& l, const AR& r, int j) {
        const int g = j >> 1;
        const i32x4 alo = r.alo, ahi = r.ahi;
        int dlo = 0, dhi = 0;
        dlo = dot4(l.qs.x & 0x0F0F0F0F, alo.x, dlo);
        dlo = dot4(l.qs.y & 0x0F0F0F0F, alo.y, dlo);
        dlo = dot4(l.qs.z & 0x0F0F0F0F, alo.z, dlo);
        dlo = dot4(l.qs.w & 0x0F0F0F0F, alo.w, dlo);
        dhi = dot4((l.qs.x >> 4) & 0x0F0F0F0F, ahi.x, dhi);
        dhi = dot4((l.qs.y >> 4) & 0x0F0F0F0F, ahi.y, dhi);
        dhi = dot4((l.qs.z >> 4) & 0x0F0F0F0F, ahi.z, dhi);
        dhi = dot4((l.qs.w >> 4) & 0x0F0F0F0F, ahi.w, dhi);
        // get_scale_min_k4 for sub-blocks 2g, 2g+1 (bytes 2(g&1), 2(g&1)+1 of each header dword)
        const unsigned sh = (g & 1) * 16;
        const unsigned Y = l.hdr.y >> sh, Z = l.hdr.z >> sh, W = l.hdr.w >> sh;
        const unsigned SC = g < 2 ? (Y & 0x3F3Fu) : ((W & 0x0F0Fu) | ((Y >> 2) & 0x3030u));
        const unsigned MM = g < 2 ? (Z & 0x3F3Fu) : (((W >> 4) & 0x0F0Fu) | ((Z >> 2) & 0x3030u));
        const int S = (int)(SC & 0xFF) * dlo + (int)((SC >> 8) & 0xFF) * dhi;
        const int M = (int)(MM & 0xFF) * r.bs_lo + (int)((MM >> 8) & 0xFF) * r.bs_hi;
        const float d = h2f(l.hdr.x) * r.dx;
        const float dm = h2f(l.hdr.x >> 16) * r.dx;
        return d * (float)S - dm * (float)M;
    }
};

template <> struct Kq<T_Q5_K> {
    static constexpr int LPS = 8;
    struct Ld { u32x4 qs, qh, hdr; };
    __device__ static Ld load(const uint8_t* const* rp, int sb, int j) {
        Ld l;
        l.qs = ldg16(rp[0] + sb * 128 + j * 16);
        l.qh = ldg16(rp[1] + sb * 32 + (j & 1) * 16);
        l.hdr = ldg16(rp[2] + sb * 16);
        return l;
    }
    using AR = Kq<T_Q4_K>::AR;
    __device__ static AR act(const Act& a, int sb, int j) { return Kq<T_Q4_K>::act(a, sb, j); }
    __device__ static float dot(const Ld& l, const AR& r, int j) {
        const int g = j >> 1;
        const i32x4 alo = r.alo, ahi = r.ahi;
        const unsigned s0 = 2 * g, s1 = 2 * g + 1;
        int dlo = 0, dhi = 0;
#define Q5L(c) ((l.qs.c & 0x0F0F0F0Fu) | (((l.qh.c >> s0) & 0x01010101u) << 4))
#define Q5H(c) (((l.qs.c >> 4) & 0x0F0F0F0Fu) | (((l.qh.c >> s1) & 0x01010101u) << 4))
        dlo = dot4((int)Q5L(x), alo.x, dlo);
        dlo = dot4((int)Q5L(y), alo.y, dlo);
        dlo = dot4((int)Q5L(z), alo.z, dlo);
        dlo = dot4((int)Q5L(w), alo.w, dlo);
        dhi = dot4((int)Q5H(x), ahi.x, dhi);
        dhi = dot4((int)Q5H(y), ahi.y, dhi);
        dhi = dot4((int)Q5H(z), ahi.z, dhi);
        dhi = dot4((int)Q5H(w), ahi.w, dhi);
#undef Q5L
#undef Q5H
        const unsigned sh = (g & 1) * 16;
        const unsigned Y = l.hdr.y >> sh, Z = l.hdr.z >> sh, W = l.hdr.w >> sh;
        const unsigned SC = g < 2 ? (Y & 0x3F3Fu) : ((W & 0x0F0Fu) | ((Y >> 2) & 0x3030u));
        const unsigned MM = g < 2 ? (Z & 0x3F3Fu) : (((W >> 4) & 0x0F0Fu) | ((Z >> 2) & 0x3030u));
        const int S = (int)(SC & 0xFF) * dlo + (int)((SC >> 8) & 0xFF) * dhi;
        const int M = (int)(MM & 0xFF) * r.bs_lo + (int)((MM >> 8) & 0xFF) * r.bs_hi;
        const float d = h2f(l.hdr.x) * r.dx;
        const float dm = h2f(l.hdr.x >> 16) * r.dx;
        return d * (float)S - dm * (float)M;
    }
};

template <> struct Kq<T_Q6_K> {
    static constexpr int LPS = 8;
    struct Ld { u32x4 ql, qh; unsigned sc0, sc1, d; };
    __device__ static Ld load(const uint8_t* const* rp, int sb, int j) {
        Ld l;
        const int h = j >> 2, half = j & 1;
        l.ql = ldg16(rp[0] + sb * 128 + j * 16);
        l.qh = ldg16(rp[1] + sb * 64 + 32 * h + 16 * half);
        // scales 8h..8h+7: is_lo = 8h+2hq+half lives in word 0, is_hi = is_lo+4 in word 1
        typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
        const u32x2 sc = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(rp[2] + sb * 16) + h);
        l.sc0 = sc.x;
        l.sc1 = sc.y;
        l.d = __builtin_nontemporal_load(reinterpret_cast<const unsigned short*>(rp[3] + sb * 2));
        return l;
    }
    struct AR { i32x4 alo, ahi; int bs_lo, bs_hi; float dx; };
    __device__ static AR act(const Act& a, int sb, int j) {
        const int h = j >> 2, hq = (j >> 1) & 1, half = j & 1;
        const int e_lo = 128 * h + 32 * hq + 16 * half;
        const int8_t* ab = a.q8k + sb * 256 + e_lo;
        const int is_lo = 8 * h + 2 * hq + half;
        AR r;
        r.alo = *reinterpret_cast<const i32x4*>(ab);
        r.ahi = *reinterpret_cast<const i32x4*>(ab + 64);
        r.bs_lo = a.bsum[sb * 16 + is_lo];
        r.bs_hi = a.bsum[sb * 16 + is_lo + 4];
        r.dx = a.dk[sb];
        return r;
    }
    __device__ static float dot(const Ld& l, const AR& r, int j) {
        const int hq = (j >> 1) & 1, half = j & 1;
        const unsigned sh = hq * 2;
        const i32x4 alo = r.alo, ahi = r.ahi;
        int dlo = 0, dhi = 0;
#define Q6L(c) ((l.ql.c & 0x0F0F0F0Fu) | (((l.qh.c >> sh) & 0x03030303u) << 4))
#define Q6H(c) (((l.ql.c >> 4) & 0x0F0F0F0Fu) | (((l.qh.c >> (sh + 4)) & 0x03030303u) << 4))
        dlo = dot4((int)Q6L(x), alo.x, dlo);
        dlo = dot4((int)Q6L(y), alo.y, dlo);
        dlo = dot4((int)Q6L(z), alo.z, dlo);
        dlo = dot4((int)Q6L(w), alo.w, dlo);
        dhi = dot4((int)Q6H(x), ahi.x, dhi);
        dhi = dot4((int)Q6H(y), ahi.y, dhi);
        dhi = dot4((int)Q6H(z), ahi.z, dhi);
        dhi = dot4((int)Q6H(w), ahi.w, dhi);
#undef Q6L
#undef Q6H
        // unsigned 6-bit q times q8, minus 32*sum(q8) == sum((q-32)*q8) exactly
        const int bsh = 8 * (2 * hq + half);
        const int sc_lo = (int)(signed char)((l.sc0 >> bsh) & 0xFF);
        const int sc_hi = (int)(signed char)((l.sc1 >> bsh) & 0xFF);
        const int S = sc_lo * (dlo - 32 * r.bs_lo) + sc_hi * (dhi - 32 * r.bs_hi);
        const float d = h2f(l.d) * r.dx;
        return d * (float)S;
    }
};

template <> struct Kq<T_Q8_0> {
    static constexpr int LPS = 8;          // lane j owns block j (32 weights) of the superblock
    struct Ld { u32x4 q0, q1; unsigned d; };
    __device__ static Ld load(const uint8_t* const* rp, int sb, int j) {
        Ld l;
        l.q0 = ldg16(rp[0] + sb * 256 + j * 32);
        l.q1 = ldg16(rp[0] + sb * 256 + j * 32 + 16);
        l.d = __builtin_nontemporal_load(reinterpret_cast<const unsigned short*>(rp[1] + sb * 16 + j * 2));
        return l;
    }
    struct AR { i32x4 a0, a1; float d0; };
    __device__ static AR act(const Act& a, int sb, int j) {
        const int8_t* ab = a.q80 + sb * 256 + j * 32;
        AR r;
        r.a0 = *reinterpret_cast<const i32x4*>(ab);
        r.a1 = *reinterpret_cast<const i32x4*>(ab + 16);
        r.d0 = a.d0[sb * 8 + j];
        return r;
    }
    __device__ static float dot(const Ld& l, const AR& r, int j) {
        const i32x4 a0 = r.a0, a1 = r.a1;
        int s = 0;
        s = dot4((int)l.q0.x, a0.x, s);
        s = dot4((int)l.q0.y, a0.y, s);
        s = dot4((int)l.q0.z, a0.z, s);
        s = dot4((int)l.q0.w, a0.w, s);
        s = dot4((int)l.q1.x, a1.x, s);
        s = dot4((int)l.q1.y, a1.y, s);
        s = dot4((int)l.q1.z, a1.z, s);
        s = dot4((int)l.q1.w, a1.w, s);
        const float d = h2f(l.d) * r.d0;   // fp16(x.d) * fp16(y.d), then * sumi
        return d * (float)s;
    }
};

// ---------------------------------------------------------------------------
// The fused GEMV kernel, specialised per quant type T.
//
// Work decomposition: a unit is a pair of output rows (see kernels.h); a wave
// owns units gw, gw + W, gw + 2W, ... (W = waves in the grid).  A unit is
// streamed in "chunks" (one step of SPS superblocks for both rows), and the
// wave keeps D chunks in flight in a register ring: while chunk q is being
// reduced against the LDS activations, chunks q+1 .. q+D-1 are loading.  The
// first D-1 chunks are issued before the prologue so that the weight stream
// starts while the activations are normalised and quantised.
// ---------------------------------------------------------------------------
struct SmemPlan {
    ActLayout L;
    int act_bytes, rope_off, red_off, resid_off, total;
};
// resid_rows: residual values staged per workgroup (its contiguous unit range)
__host__ __device__ inline SmemPlan smem_plan(int K, int nslots, int need_q8k, int need_q80, int n_rot,
                                              int resid_rows) {
    SmemPlan P;
    P.L = act_layout(K, need_q8k, need_q80);
    P.act_bytes = P.L.slot_bytes * nslots;
    P.rope_off = P.act_bytes;
    P.red_off = P.rope_off + ((n_rot / 2) * 8 + 15) / 16 * 16;
    P.resid_off = P.red_off + 32 * 8;
    P.total = P.resid_off + ((resid_rows * 4 + 15) / 16) * 16;
    return P;
}
__host__ __device__ inline int resid_rows_per_wg(const GemvParams&) { return 0; }

__device__ __forceinline__ float silu_f(float x) { return x / (1.0f + expf(-x)); }

// Prologue (every workgroup, redundantly): RMSNorm of slot 0 if requested,
// quantisation of the activation slots into LDS, residual rows of this
// workgroup's unit range, and the RoPE cos/sin table of this token.
__device__ __forceinline__ void gemv_prologue(const GemvParams& P, char* smem, const SmemPlan& SP, int pos) {
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nwaves = blockDim.x >> 6;
    const ActLayout& L = SP.L;
    double* red = reinterpret_cast<double*>(smem + SP.red_off);
    if (P.pro < 0) return;   // debug: skip the prologue (timing ablation only)
    float scale = 1.0f;
    if (P.pro == PRO_RMSNORM) {
        // ggml_compute_forward_rms_norm_f32: sum of float squares in double
        double s = 0.0;
        const float4* x4 = reinterpret_cast<const float4*>(P.x[0]);
        for (int i = tid; i < P.K / 4; i += blockDim.x) {
            const float4 v = x4[i];
            s += (double)(v.x * v.x);
            s += (double)(v.y * v.y);
            s += (double)(v.z * v.z);
            s += (double)(v.w * v.w);
        }
        s = wave_sum_d(s);
        if (lane == 0) red[wave] = s;
        __syncthreads();
        double tot = 0.0;
        for (int w = 0; w < nwaves; ++w) tot += red[w];
        const float mean = (float)(tot / (double)P.K);
        scale = 1.0f / sqrtf(mean + P.eps);
    }
    for (int slot = 0; slot < P.nslots; ++slot) {
        char* base = smem + slot * L.slot_bytes;
        const float4* x4 = reinterpret_cast<const float4*>(P.x[slot]);
        const bool norm = slot == 0 && P.pro == PRO_RMSNORM;
        for (int blk = wave; blk < L.nb; blk += nwaves) {
            const float4 xv = x4[blk * 64 + lane];
            float v[4] = {xv.x, xv.y, xv.z, xv.w};
            if (norm) {
                const float4 w = reinterpret_cast<const float4*>(P.norm_w)[blk * 64 + lane];
                v[0] = (v[0] * scale) * w.x;   // ggml_vec_scale_f32 then ggml_mul
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
    // residual rows of this workgroup (in-place residual add: x[r] = W.a + x[r])
    const int rrows = resid_rows_per_wg(P);
    if (rrows > 0) {
        float* rs = reinterpret_cast<float*>(smem + SP.resid_off);
        const long long r0 = (long long)blockIdx.x * rrows;
        const long long nrow = P.seg[0].pair == PAIR_ADJ ? P.seg[0].A.rows : P.seg[0].units;
        for (int i = tid; i < rrows; i += blockDim.x) rs[i] = (r0 + i < nrow) ? P.seg[0].resid[r0 + i] : 0.0f;
    }
    // RoPE cache for this token's position (ggml_rope_cache_init, ext_factor 0, mscale 1)
    if (P.n_rot > 0 && wave == 0) {
        float* rope = reinterpret_cast<float*>(smem + SP.rope_off);
        for (int i = lane; i < P.n_rot / 2; i += 64) {
            float theta = (float)pos;
            for (int k = 0; k < i; ++k) theta = theta * P.theta_scale;
            const float ff = P.freq_factors ? P.freq_factors[i] : 1.0f;
            const float th = P.freq_scale * (theta / ff);
            rope[2 * i] = cosf(th);
            rope[2 * i + 1] = sinf(th);
        }
    }
}

struct UnitRef {
    int si;           // segment
    int lu;           // unit within segment
    long long ra, rb; // rows
    bool hasB;
};

__device__ __forceinline__ UnitRef unit_ref(const GemvParams& P, int u) {
    UnitRef c;
    int si = 0;
    while (si + 1 < P.nseg && u >= P.seg[si + 1].unit0) ++si;
    c.si = si;
    c.lu = u - P.seg[si].unit0;
    if (P.seg[si].pair == PAIR_ADJ) {
        c.ra = 2LL * c.lu;
        c.rb = c.ra + 1;
        c.hasB = c.rb < P.seg[si].A.rows;
    } else {
        c.ra = c.rb = c.lu;
        c.hasB = true;
    }
    return c;
}

// rva / rvb: residual values of rows A / B (loaded with the unit's weights)
__device__ __forceinline__ void gemv_epilogue(const GemvParams& P, const UnitRef& c, const float* rope,
                                              float rva, float rvb, float wa, float wb,
                                              int pos, int cell, float yA, float yB) {
    const GemvSeg& S = P.seg[c.si];
    const long long ra = c.ra, rb = c.rb;
    switch (S.epi) {
    case EPI_STORE:
        S.out[ra] = yA;
        if (c.hasB) S.out[rb] = yB;
        break;
    case EPI_ADD:
        S.out[ra] = yA + rva;
        if (c.hasB) S.out[rb] = yB + rvb;
        break;
    case EPI_ROPE_Q:
    case EPI_ROPE_K: {
        const int i0 = (int)(ra % P.head_dim);   // even
        float o0 = yA, o1 = yB;
        if (i0 < P.n_rot) {
            const float cs = rope[i0], sn = rope[i0 + 1];
            o0 = yA * cs - yB * sn;
            o1 = yA * sn + yB * cs;
        }
        if (S.epi == EPI_ROPE_Q) {
            S.out[ra] = o0;
            S.out[rb] = o1;
        } else {
            __half* kr = P.kcache + (long long)cell * P.kv_dim;
            kr[ra] = __float2half_rn(o0);
            kr[rb] = __float2half_rn(o1);
            if (c.lu == 0) P.cell_pos[cell] = pos;
        }
        break;
    }
    case EPI_V: {
        __half* vr = P.vcache + (long long)cell * P.kv_dim;
        vr[ra] = __float2half_rn(yA);
        if (c.hasB) vr[rb] = __float2half_rn(yB);
        break;
    }
    case EPI_SWIGLU:
        S.out[c.lu] = silu_f(yA) * yB;
        break;
    case EPI_MOE_DOWN:
        S.out[c.lu] = (yA * wa + yB * wb) + rva;
        break;
    default: break;
    }
}

// ---------------------------------------------------------------------------
// The fused GEMV kernel, specialised per quant type T, per NSW (superblock
// steps streamed by one wave per row, <= 2), per KS (waves of the workgroup
// that split one row pair's K range; KS*NSW*8 >= K/256) and per PF (units a
// wave keeps in flight: 1 = load, consume; 2 = the next unit's loads are issued
// before the current unit is consumed, so the wave's weight stream never stops).
//
// * Each wave keeps, for its NSW steps, the activation slice its lanes need in
//   registers (it is the same for every row), loaded from LDS once after the
//   prologue; the inner loop touches no LDS.
// * A unit (row pair) is loaded with all NSW x 2 row loads issued together
//   (8 lanes per superblock, aligned 16-B loads), the first unit before the
//   prologue so the weight stream starts while activations are quantised.
// * Groups of KS waves sweep the units grid-strided, so neighbouring groups (in
//   and across workgroups) stream neighbouring rows at the same time.
// * KS > 1: the KS waves' partial sums are combined through LDS in fixed
//   order (deterministic) by the group's first wave, which runs the epilogue.
//   The barrier is a bare s_barrier for the in-flight prefetch (no LDS-DMA is
//   pending, so __syncthreads emits no vmcnt drain).
// ---------------------------------------------------------------------------
template <int T, int NSW, int KS, int DUAL, int ROLE, int PF>
__global__ __launch_bounds__(GEMV_THREADS) void gemv_t(const GemvParams P) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    using K = Kq<T>;
    static_assert(K::LPS == 8, "8 lanes per superblock");
    constexpr int NW = GEMV_THREADS / 64;
    constexpr int NGRP = NW / KS;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform -> SGPRs
    const int grp = wave / KS, wk = wave % KS;
    const int sbl = lane >> 3, j = lane & 7;
    const SmemPlan SP = smem_plan(P.K, P.nslots, P.need_q8k, P.need_q80, P.n_rot, resid_rows_per_wg(P));
    const int nb = P.K >> 8;
    const int ns = (nb + 7) >> 3;
    // token position / cache cell and MoE routing results, read once
    int pos = 0, cell = 0;
    if (P.tokpos) {
        pos = __builtin_amdgcn_readfirstlane(P.tokpos[1]);
        cell = __builtin_amdgcn_readfirstlane(P.tokpos[2]);
    }
    int e0 = 0, e1 = 0;
    float w0 = 0.0f, w1 = 0.0f;
    if (P.sel) {
        e0 = __builtin_amdgcn_readfirstlane(P.sel[0]);
        e1 = __builtin_amdgcn_readfirstlane(P.sel[1]);
        w0 = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(P.selw[0])));
        w1 = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(P.selw[1])));
    }
    const int G_total = gridDim.x * NGRP;
    const int g0 = blockIdx.x * NGRP + grp;
    const int n_iter = (P.total_units + G_total - 1) / G_total;   // same for every wave of the workgroup

    struct Buf {
        typename K::Ld a[NSW], b[NSW];
        float ra, rb;   // residual values of the unit's rows (loaded with its weights: no late drain)
    };
    // Issue every load of unit u (u < total_units, wave-uniform).  Lanes past
    // the row's last superblock read into the next row / the plane's
    // 8-superblock tail padding; their products are masked.
    auto issue = [&](Buf& B, int u) {
        const UnitRef c = unit_ref(P, u);
        const GemvSeg& S = P.seg[c.si];
        const QMat& MB = S.pair == PAIR_ADJ ? S.A : S.B;
        const long long ea = S.expA == 0 ? e0 : S.expA == 1 ? e1 : 0;
        const long long eb = S.expB == 0 ? e0 : S.expB == 1 ? e1 : 0;
        const long long rb = c.hasB ? c.rb : c.ra;   // odd tail: re-read row A, result unused
        const uint8_t* ra_p[4];
        const uint8_t* rb_p[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            ra_p[i] = S.A.p[i] + ea * S.A.expert_stride[i] + c.ra * nb * PlaneBytes<T>::b[i];
            rb_p[i] = MB.p[i] + eb * MB.expert_stride[i] + rb * nb * PlaneBytes<T>::b[i];
        }
#pragma unroll
        for (int t = 0; t < NSW; ++t) {
            const int s = wk + t * KS;
            if (s < ns) {
                B.a[t] = K::load(ra_p, s * 8 + sbl, j);
                B.b[t] = K::load(rb_p, s * 8 + sbl, j);
            }
        }
        B.ra = B.rb = 0.0f;
        if (S.resid) {
            const long long ia = S.pair == PAIR_ADJ ? c.ra : c.lu;
            B.ra = S.resid[ia];
            B.rb = S.resid[S.pair == PAIR_ADJ ? rb : ia];
        }
    };

    Buf b0, b1;
    if (g0 < P.total_units) issue(b0, g0);
    gemv_prologue(P, smem, SP, pos);
    __syncthreads();
    const float* rope = reinterpret_cast<const float*>(smem + SP.rope_off);
    float* red = reinterpret_cast<float*>(smem + SP.red_off);   // prologue scratch, reused

    // this wave's activation slices (slot 0, and slot 1 for the dual-slot MoE down launch)
    typename K::AR arA[NSW], arB[NSW];
    {
        const Act a0 = act_view(smem, SP.L, 0);
        const Act a1 = act_view(smem, SP.L, DUAL ? 1 : 0);
#pragma unroll
        for (int t = 0; t < NSW; ++t) {
            const int s = wk + t * KS;
            const int sb = s * 8 + sbl;
            const int sbc = sb < nb ? sb : nb - 1;
            arA[t] = K::act(a0, sbc, j);
            if (DUAL) arB[t] = K::act(a1, sbc, j);
        }
    }

    // Consume unit u from B (u may be past the end: then only the barrier runs).
    auto consume = [&](const Buf& B, int u) {
        const bool valid = u < P.total_units;
        float accA = 0.0f, accB = 0.0f;
        if (valid) {
#pragma unroll
            for (int t = 0; t < NSW; ++t) {
                const int s = wk + t * KS;
                if (s < ns) {
                    const bool lv = s * 8 + sbl < nb;
                    const float pa = K::dot(B.a[t], arA[t], j);
                    const float pb = K::dot(B.b[t], DUAL ? arB[t] : arA[t], j);
                    accA += lv ? pa : 0.0f;
                    accB += lv ? pb : 0.0f;
                }
            }
        }
        float yA = wave_sum63(accA);
        float yB = wave_sum63(accB);
        if (KS == 1) {
            if (valid && lane == 63) gemv_epilogue(P, unit_ref(P, u), rope, B.ra, B.rb, w0, w1, pos, cell, yA, yB);
        } else {
            if (lane == 63) {
                red[(grp * KS + wk) * 2] = yA;
                red[(grp * KS + wk) * 2 + 1] = yB;
            }
            __syncthreads();
            if (valid && wk == 0 && lane == 63) {
                yA = red[grp * KS * 2];
                yB = red[grp * KS * 2 + 1];
#pragma unroll
                for (int k = 1; k < KS; ++k) {
                    yA += red[(grp * KS + k) * 2];
                    yB += red[(grp * KS + k) * 2 + 1];
                }
                gemv_epilogue(P, unit_ref(P, u), rope, B.ra, B.rb, w0, w1, pos, cell, yA, yB);
            }
            __syncthreads();
        }
    };

    int u = g0;
    if constexpr (PF == 1) {
        for (int it = 0; it < n_iter; ++it, u += G_total) {
            if (it > 0 && u < P.total_units) issue(b0, u);
            consume(b0, u);
        }
    } else {
        for (int it = 0; it < n_iter; it += 2, u += 2 * G_total) {
            if (u + G_total < P.total_units) issue(b1, u + G_total);
            consume(b0, u);
            if (it + 1 < n_iter) {
                if (u + 2 * G_total < P.total_units) issue(b0, u + 2 * G_total);
                consume(b1, u + G_total);
            }
        }
    }
}

constexpr int GEMV_MAX_NS = 8;

typedef void (*GemvFn)(const GemvParams);

// ns = superblock steps per row (ceil(K/256/8)) -> KS waves share a row pair,
// each wave streams NSW <= 2 steps.  ROLE: 0 generic, 1 FFN gate/up, 2 dual
// activation slot (MoE down).
template <int T, int ROLE, int PF>
static GemvFn gemv_fn_ns_pf(int ns) {
    constexpr int DUAL = ROLE == 2 ? 1 : 0;
    switch (ns) {
    case 1: return gemv_t<T, 1, 1, DUAL, ROLE, PF>;
    case 2: return gemv_t<T, 2, 1, DUAL, ROLE, PF>;
    case 3: case 4: return gemv_t<T, 2, 2, DUAL, ROLE, PF>;
    case 5: case 6: case 7: case 8: return gemv_t<T, 2, 4, DUAL, ROLE, PF>;
    default: return nullptr;
    }
}
// PF = 2 (double-buffered units) measured slower on Q4_K/Q8_0 and spills on
// Q5_K/Q6_K at 4 waves/SIMD: PF = 1 is the shipped variant.
template <int T, int ROLE>
static GemvFn gemv_fn_ns(int ns) { return gemv_fn_ns_pf<T, ROLE, 1>(ns); }

int gemv_ks(int ns) { return ns <= 2 ? 1 : ns <= 4 ? 2 : 4; }

template <int ROLE>
static GemvFn gemv_fn_t(int type, int ns) {
    switch (type) {
    case T_Q4_K: return gemv_fn_ns<T_Q4_K, ROLE>(ns);
    case T_Q5_K: return gemv_fn_ns<T_Q5_K, ROLE>(ns);
    case T_Q6_K: return gemv_fn_ns<T_Q6_K, ROLE>(ns);
    case T_Q8_0: return gemv_fn_ns<T_Q8_0, ROLE>(ns);
    default: return nullptr;
    }
}

// The FFN gate/up launch gets its own symbol (the bench's roofline kernel).
static GemvFn gemv_fn(int role, int type, int ns, int nslots) {
    if (nslots > 1) return gemv_fn_t<2>(type, ns);
    return role == ROLE_FFN_UP ? gemv_fn_t<1>(type, ns) : gemv_fn_t<0>(type, ns);
}

__global__ void attn_kernel(const AttnParams P);

void init_kernel_attributes() {
    const int types[4] = {T_Q4_K, T_Q5_K, T_Q6_K, T_Q8_0};
    for (int r : {ROLE_GENERIC, ROLE_FFN_UP})
        for (int t : types)
            for (int ns = 1; ns <= GEMV_MAX_NS; ++ns)
                for (int nsl = 1; nsl <= 2; ++nsl)
                    MI_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(gemv_fn(r, t, ns, nsl)),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    MI_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(attn_kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
}

size_t gemv_smem_bytes(const GemvParams& p) {
    return (size_t)smem_plan(p.K, p.nslots, p.need_q8k, p.need_q80, p.n_rot, resid_rows_per_wg(p)).total;
}

int gemv_ks(int ns);
int gemv_default_grid(const GemvParams& p) {
    // One 16-wave workgroup per CU (256 CUs): the per-workgroup prologue
    // (activation quantisation) is paid once per CU.  Small launches use
    // fewer workgroups so every group of KS waves still gets a unit.
    const int ks = gemv_ks((p.K / 256 + 7) / 8);
    const int groups_per_wg = (GEMV_THREADS / 64) / ks;
    const int g = (p.total_units + groups_per_wg - 1) / groups_per_wg;
    return g < 1 ? 1 : (g > 256 ? 256 : g);
}

void launch_gemv(const GemvParams& p_in, int role, int grid, hipStream_t s, hipEvent_t ev_start,
                 hipEvent_t ev_stop) {
    GemvParams p = p_in;
    if (p.K % 256 != 0) throw Error("gemv: K must be a multiple of 256");
    static const int dbg = getenv("MI_GEMV_DEBUG") ? atoi(getenv("MI_GEMV_DEBUG")) : 0;
    if (dbg & 1) p.pro = -1;
    if (dbg & 2) grid = 1024;
    if (grid <= 0) grid = gemv_default_grid(p);
    p.upw = 0;
    const size_t smem = gemv_smem_bytes(p);
    if (smem > 160 * 1024) throw Error("gemv: activation too large for LDS");
    const int type = p.seg[0].A.type;
    for (int i = 0; i < p.nseg; ++i)
        if (p.seg[i].A.type != type || (p.seg[i].pair == PAIR_AB && p.seg[i].B.type != type))
            throw Error("gemv: all matrices of one launch must share a quant type");
    const int ns = (p.K / 256 + 7) / 8;
    GemvFn fn = gemv_fn(role, type, ns, p.nslots);
    if (!fn) throw Error("gemv: unsupported quant type or K (K <= 16384)");
    if (ev_start || ev_stop)
        hipExtLaunchKernelGGL(fn, dim3(grid), dim3(GEMV_THREADS), smem, s, ev_start, ev_stop, 0, p);
    else
        hipLaunchKernelGGL(fn, dim3(grid), dim3(GEMV_THREADS), smem, s, p);
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

__global__ void embed_kernel(const EmbedParams P) {
    const long long tok = P.tokpos[0];
    for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < P.n_embd; c += gridDim.x * blockDim.x)
        P.out[c] = dequant_elem(P.E, tok, c);
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
// Attention for one query token over the f16 cache, one workgroup per q head.
// Mirrors the non-flash CPU graph (Instance.hpp:25 flash_attn=false):
//   KQ = mul_mat(K, q): q rounded to f16 (vec_dot_type F16), f32 sums
//   soft_max_ext(KQ*scale + mask): f32 exp, double sum, p = e * (float)(1/sum)
//   KQV = mul_mat(V^T, p): p rounded to f16, f32 sums
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void attn_kernel(const AttnParams P) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float* qf = reinterpret_cast<float*>(smem);                 // [head_dim]
    float* part = qf + 256;                                      // [4][head_dim] partial outputs
    double* redd = reinterpret_cast<double*>(part + 4 * 256);    // [8]
    float* redf = reinterpret_cast<float*>(redd + 8);            // [8]
    float* sc = redf + 8;                                        // [n_ctx] scores / probs
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int h = blockIdx.x;
    const int g = h / (P.n_head / P.n_head_kv);
    const int hd = P.head_dim;
    const int qpos = P.tokpos[1];
    const int ncell = P.tokpos[2] + 1;
    for (int d = tid; d < hd; d += 256) qf[d] = __half2float(__float2half_rn(P.q[h * hd + d]));
    __syncthreads();

    float lmax = -INFINITY;
    for (int c = tid; c < ncell; c += 256) {
        const uint8_t* kr = reinterpret_cast<const uint8_t*>(P.kcache + (long long)c * P.kv_dim + g * hd);
        float acc = 0.0f;
        for (int d = 0; d < hd; d += 8) {
            const u32x4 kv = *reinterpret_cast<const u32x4*>(kr + d * 2);
            const unsigned w[4] = {kv.x, kv.y, kv.z, kv.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                acc = fmaf(qf[d + 2 * e], h2f(w[e]), acc);
                acc = fmaf(qf[d + 2 * e + 1], h2f(w[e] >> 16), acc);
            }
        }
        float s = acc * P.scale;
        if (P.cell_pos[c] > qpos) s = -INFINITY;
        sc[c] = s;
        lmax = fmaxf(lmax, s);
    }
    lmax = wave_max(lmax);
    if (lane == 0) redf[wave] = lmax;
    __syncthreads();
    const float mx = fmaxf(fmaxf(redf[0], redf[1]), fmaxf(redf[2], redf[3]));
    double ls = 0.0;
    for (int c = tid; c < ncell; c += 256) {
        const float e = expf(sc[c] - mx);
        sc[c] = e;
        ls += (double)e;
    }
    ls = wave_sum_d(ls);
    if (lane == 0) redd[wave] = ls;
    __syncthreads();
    const double tot = redd[0] + redd[1] + redd[2] + redd[3];
    const float inv = (float)(1.0 / tot);

    // PV: lane owns dims [lane*dpl, +dpl); wave w owns cells w, w+4, ...
    const int dpl = hd >= 64 ? hd / 64 : 1;   // 1, 2 or 4
    const bool active = lane * dpl < hd;
    float o[4] = {0.f, 0.f, 0.f, 0.f};
    const __half* vb = P.vcache + g * hd + (active ? lane * dpl : 0);
#pragma unroll 4
    for (int c = wave; c < ncell; c += 4) {
        const float p = __half2float(__float2half_rn(sc[c] * inv));
        const __half* vr = vb + (long long)c * P.kv_dim;
        if (dpl == 2) {
            const unsigned w = *reinterpret_cast<const unsigned*>(vr);
            o[0] = fmaf(p, h2f(w), o[0]);
            o[1] = fmaf(p, h2f(w >> 16), o[1]);
        } else if (dpl == 4) {
            const uint2 w = *reinterpret_cast<const uint2*>(vr);
            o[0] = fmaf(p, h2f(w.x), o[0]);
            o[1] = fmaf(p, h2f(w.x >> 16), o[1]);
            o[2] = fmaf(p, h2f(w.y), o[2]);
            o[3] = fmaf(p, h2f(w.y >> 16), o[3]);
        } else {
            o[0] = fmaf(p, __half2float(vr[0]), o[0]);
        }
    }
    if (active)
        for (int e = 0; e < dpl; ++e) part[wave * 256 + lane * dpl + e] = o[e];
    __syncthreads();
    for (int d = tid; d < hd; d += 256)
        P.out[h * hd + d] = ((part[d] + part[256 + d]) + part[512 + d]) + part[768 + d];
}

void launch_attn(const AttnParams& p, hipStream_t s) {
    if (!(p.head_dim == 32 || p.head_dim == 64 || p.head_dim == 128 || p.head_dim == 256))
        throw Error("attn: unsupported head_dim");
    const size_t smem = (256 + 4 * 256) * 4 + 8 * 8 + 8 * 4 + (size_t)p.n_ctx * 4;
    if (smem > 160 * 1024) throw Error("attn: n_ctx too large for the LDS score buffer");
    hipLaunchKernelGGL(attn_kernel, dim3(p.n_head), dim3(256), smem, s, p);
    MI_HIP(hipGetLastError());
}

// ---------------------------------------------------------------------------
// Top-k: sort keys (orderable logit << 32 | ~id) descending.  Stage 1: each of
// 64 workgroups sorts its chunk and keeps 64; stage 2 merges 4096 candidates.
// ---------------------------------------------------------------------------
__device__ __forceinline__ unsigned long long topk_key(float v, int id) {
    unsigned u = __float_as_uint(v);
    u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
    return ((unsigned long long)u << 32) | (unsigned long long)(0xFFFFFFFFu - (unsigned)id);
}

__device__ void bitonic_desc(unsigned long long* k, int n) {
    for (int size = 2; size <= n; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int i = threadIdx.x; i < n; i += blockDim.x) {
                const int j = i ^ stride;
                if (j > i) {
                    const unsigned long long a = k[i], b = k[j];
                    const bool desc = (i & size) == 0;
                    if (desc ? (a < b) : (a > b)) { k[i] = b; k[j] = a; }
                }
            }
            __syncthreads();
        }
    }
}

__global__ __launch_bounds__(256) void topk_stage1(const float* logits, int n, int chunk, int p2,
                                                   unsigned long long* cand) {
    extern __shared__ unsigned long long keys[];
    const int begin = blockIdx.x * chunk;
    for (int i = threadIdx.x; i < p2; i += blockDim.x) {
        const int id = begin + i;
        keys[i] = (i < chunk && id < n) ? topk_key(logits[id], id) : 0ULL;
    }
    __syncthreads();
    bitonic_desc(keys, p2);
    for (int i = threadIdx.x; i < TOPK_MAX; i += blockDim.x)
        cand[blockIdx.x * TOPK_MAX + i] = i < p2 ? keys[i] : 0ULL;
}

__global__ __launch_bounds__(1024) void topk_stage2(const unsigned long long* cand, const float* logits, int* ids,
                                                   float* vals) {
    __shared__ unsigned long long keys[TOPK_GROUPS * TOPK_MAX];
    for (int i = threadIdx.x; i < TOPK_GROUPS * TOPK_MAX; i += blockDim.x) keys[i] = cand[i];
    __syncthreads();
    bitonic_desc(keys, TOPK_GROUPS * TOPK_MAX);
    for (int i = threadIdx.x; i < TOPK_MAX; i += blockDim.x) {
        const unsigned long long k = keys[i];
        const int id = k ? (int)(0xFFFFFFFFu - (unsigned)(k & 0xFFFFFFFFu)) : -1;
        ids[i] = id;
        vals[i] = id >= 0 ? logits[id] : -INFINITY;
    }
}

void launch_topk(const TopkParams& p, hipStream_t s) {
    const int chunk = (p.n + TOPK_GROUPS - 1) / TOPK_GROUPS;
    int p2 = 64;
    while (p2 < chunk) p2 <<= 1;
    if (p2 * 8 > 64 * 1024) throw Error("topk: vocabulary too large");
    hipLaunchKernelGGL(topk_stage1, dim3(TOPK_GROUPS), dim3(256), p2 * 8, s, p.logits, p.n, chunk, p2, p.cand);
    MI_HIP(hipGetLastError());
    hipLaunchKernelGGL(topk_stage2, dim3(1), dim3(1024), 0, s, p.cand, p.logits, p.ids, p.vals);
    MI_HIP(hipGetLastError());
}

__global__ void gather_kernel(const float* logits, const int* ids, int n, float* out) {
    const int i = threadIdx.x + blockIdx.x * blockDim.x;
    if (i < n) out[i] = logits[ids[i]];
}

void launch_gather(const float* logits, const int* ids, int n, float* out, hipStream_t s) {
    if (n <= 0) return;
    hipLaunchKernelGGL(gather_kernel, dim3((n + 255) / 256), dim3(256), 0, s, logits, ids, n, out);
    MI_HIP(hipGetLastError());
}

// ---------------------------------------------------------------------------
// MoE router (build_moe_ffn, softmax gating, norm_w): one workgroup.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void router_kernel(const RouterParams P) {
    __shared__ double redd[4];
    __shared__ float logit[64];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    double s = 0.0;
    for (int i = tid; i < P.n_embd; i += 256) s += (double)(P.x[i] * P.x[i]);
    s = wave_sum_d(s);
    if (lane == 0) redd[wave] = s;
    __syncthreads();
    const double tot = ((redd[0] + redd[1]) + redd[2]) + redd[3];
    const float mean = (float)(tot / (double)P.n_embd);
    const float scale = 1.0f / sqrtf(mean + P.eps);
    // expert e handled by wave e%4: logits = W_e . (x*scale*w)
    for (int e = wave; e < P.n_expert; e += 4) {
        const float* we = P.w + (long long)e * P.n_embd;
        float acc = 0.0f;
        for (int i = lane; i < P.n_embd; i += 64) acc = fmaf(we[i], (P.x[i] * scale) * P.norm_w[i], acc);
        acc = wave_sum(acc);
        if (lane == 0) logit[e] = acc;
    }
    __syncthreads();
    if (tid == 0) {
        float mx = -INFINITY;
        for (int e = 0; e < P.n_expert; ++e) mx = fmaxf(mx, logit[e]);
        float pr[64];
        double sum = 0.0;
        for (int e = 0; e < P.n_expert; ++e) { pr[e] = expf(logit[e] - mx); sum += (double)pr[e]; }
        const float inv = (float)(1.0 / sum);
        for (int e = 0; e < P.n_expert; ++e) pr[e] = pr[e] * inv;
        // ggml_argsort (desc) selection order, then ggml_top_k's first n_used
        int idx[64];
        for (int e = 0; e < P.n_expert; ++e) idx[e] = e;
        for (int a = 0; a < P.n_expert; ++a)
            for (int b = a + 1; b < P.n_expert; ++b)
                if (pr[idx[a]] < pr[idx[b]]) { int t = idx[a]; idx[a] = idx[b]; idx[b] = t; }
        float wsum = 0.0f;
        for (int k = 0; k < P.n_used; ++k) wsum += pr[idx[k]];
        for (int k = 0; k < P.n_used; ++k) { P.sel[k] = idx[k]; P.selw[k] = pr[idx[k]] / wsum; }
    }
}

void launch_router(const RouterParams& p, hipStream_t s) {
    if (p.n_expert > 64) throw Error("router: too many experts");
    hipLaunchKernelGGL(router_kernel, dim3(1), dim3(256), 0, s, p);
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
