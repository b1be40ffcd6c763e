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
#include <cstring>
#include <algorithm>

namespace mi {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// Pointers the GEMV reads from its LDS copy of the parameter block are generic
// to the compiler, which would emit flat_* accesses: those retire out of order
// (every wait becomes vmcnt(0) & lgkmcnt(0)) and would serialise the weight
// ring.  Every global access of the GEMV goes through gptr() -> global_*.
template <typename T>
__device__ __forceinline__ const __attribute__((address_space(1))) T* gptr(const T* p) {
    return (const __attribute__((address_space(1))) T*)(p);
}
template <typename T>
__device__ __forceinline__ __attribute__((address_space(1))) T* gptr_w(T* p) {
    return (__attribute__((address_space(1))) T*)(p);
}
// A wave-uniform pointer (e.g. read from LDS) moved to SGPRs.
template <typename T>
__device__ __forceinline__ T* rfl_ptr(T* p) {
    const unsigned long long v = reinterpret_cast<unsigned long long>(p);
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
    return reinterpret_cast<T*>(((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ u32x4 ldg16(const uint8_t* p) {
    return __builtin_nontemporal_load(gptr(reinterpret_cast<const u32x4*>(p)));
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
// DPP forms of the prologue reductions (__shfl_xor lowers to ds_bpermute: an
// LDS round trip per step, ~16 dependent ones per Q8_K block).
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
// Full-wave double sum, total in lane 63 (same scan as wave_sum63).
__device__ __forceinline__ double wave_sum63_d(double v) {
    v += dpp_d<0x111, 0xf>(v);
    v += dpp_d<0x112, 0xf>(v);
    v += dpp_d<0x114, 0xf>(v);
    v += dpp_d<0x118, 0xf>(v);
    v += dpp_d<0x142, 0xa>(v);
    v += dpp_d<0x143, 0xc>(v);
    return v;
}
// Full-wave max of non-negative floats (0 is the identity), broadcast to all lanes.
__device__ __forceinline__ float wave_max_pos(float v) {
#define MX(ctrl, rm) v = fmaxf(v, __int_as_float(dpp_i<ctrl, rm>(__float_as_int(v))))
    MX(0x111, 0xf); MX(0x112, 0xf); MX(0x114, 0xf); MX(0x118, 0xf); MX(0x142, 0xa); MX(0x143, 0xc);
#undef MX
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
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
    const float a0 = fabsf(v[0]), a1 = fabsf(v[1]), a2 = fabsf(v[2]), a3 = fabsf(v[3]);
    const float amax = wave_max_pos(fmaxf(fmaxf(a0, a1), fmaxf(a2, a3)));
    int q[4];
    float d;
    if (amax == 0.0f) {
        q[0] = q[1] = q[2] = q[3] = 0;
        d = 0.0f;
    } else {
        // the signed value at the FIRST index whose |x| is the maximum
        const int e = a0 == amax ? 0 : a1 == amax ? 1 : a2 == amax ? 2 : a3 == amax ? 3 : 4;
        const float mine = e == 0 ? v[0] : e == 1 ? v[1] : e == 2 ? v[2] : v[3];
        const unsigned long long m = __ballot(e < 4);
        const int src = __builtin_ctzll(m);
        const float mx = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(mine), src));
        const float iscale = -127.0f / mx;
#pragma unroll
        for (int k = 0; k < 4; ++k) q[k] = min(127, (int)rintf(iscale * v[k]));
        d = 1.0f / iscale;
    }
    const int packed = (q[0] & 0xFF) | ((q[1] & 0xFF) << 8) | ((q[2] & 0xFF) << 16) | ((q[3] & 0xFF) << 24);
    reinterpret_cast<int*>(q8)[lane] = packed;
    int sm = q[0] + q[1] + q[2] + q[3];
    sm += dpp_i<0xB1, 0xf>(sm);   // quad_perm [1,0,3,2]
    sm += dpp_i<0x4E, 0xf>(sm);   // quad_perm [2,3,0,1] -> every lane of the quad has its 16-sum
    if ((lane & 3) == 0) bsum[lane >> 2] = sm;
    if (lane == 0) *dk = d;
}

// x86 SIMD form of quantize_row_q8_0: d = fp16(amax/127), id = 127/amax,
// q = round-to-nearest-even(x*id).  8 lanes per 32-block.
__device__ __forceinline__ void quant_q80_block(const float v[4], int lane, int8_t* q8, float* d0) {
    float am = fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3])));
    am = fmaxf(am, __int_as_float(dpp_i<0xB1, 0xf>(__float_as_int(am))));
    am = fmaxf(am, __int_as_float(dpp_i<0x4E, 0xf>(__float_as_int(am))));
    am = fmaxf(am, __int_as_float(dpp_i<0x141, 0xf>(__float_as_int(am))));   // row_half_mirror
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
#ifdef MI_EXP_NOHDR   // bandwidth experiment only (wrong numerics): no header loads
        l.hdr = u32x4{0x3c003c00u, 0x01010101u, 0x01010101u, 0x01010101u};
#else
        l.hdr = ldg16(rp[1] + sb * 16);
#endif
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
        const u32x2 sc = __builtin_nontemporal_load(gptr(reinterpret_cast<const u32x2*>(rp[2] + sb * 16) + h));
        l.sc0 = sc.x;
        l.sc1 = sc.y;
        l.d = __builtin_nontemporal_load(gptr(reinterpret_cast<const unsigned short*>(rp[3] + sb * 2)));
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
        l.d = __builtin_nontemporal_load(gptr(reinterpret_cast<const unsigned short*>(rp[1] + sb * 16 + j * 2)));
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
// Work decomposition: a unit is a PAIR of output rows (see kernels.h).  Every
// wave owns a contiguous range of units (so a workgroup owns a contiguous
// range, whose residual rows it stages in LDS).  A unit's two rows are
// streamed in "chunks": one aligned 16-byte load per lane of the main quant
// plane plus its side planes, 8 superblocks per row and chunk (8 lanes per
// superblock).  The wave walks its (unit, chunk) items through a D-deep
// register ring: while item i is reduced against the LDS activations, items
// i+1 .. i+D-1 are in flight -- across unit boundaries, so a wave's weight
// stream never stops until its range is done.  The first D-1 items are issued
// before the prologue, so the stream starts while the activations are
// normalised and quantised.  Loads past the end of the range repeat the last
// item's addresses (cache hits) so that every ring step issues the same loads
// and the compiler's vmcnt bookkeeping stays exact (no wait-for-all).
// ---------------------------------------------------------------------------
struct SmemPlan {
    ActLayout L;
    int act_bytes, rope_off, resid_off, attn_off, red_off, total;
};
__host__ __device__ inline SmemPlan smem_plan(const GemvParams& p) {
    SmemPlan S;
    S.L = act_layout(p.K, p.need_q8k, p.need_q80);
    S.act_bytes = S.L.slot_bytes * p.nslots;
    S.rope_off = S.act_bytes;
    S.resid_off = S.rope_off + ((p.n_rot / 2) * 8 + 15) / 16 * 16;
    S.attn_off = S.resid_off + ((p.wg_units * 2 * 4 + 15) / 16) * 16;
    S.red_off = S.attn_off;
    S.total = S.red_off + 32 * 8;
    return S;
}

__device__ __forceinline__ float silu_f(float x) { return x / (1.0f + expf(-x)); }

__device__ __forceinline__ void unit_range(int total, int W, int gw, int& u0, int& u1) {
    // total * (gw + 1) < 2^32 (total <= 65536 units, W <= 4096 waves)
    u0 = (int)(((unsigned)total * (unsigned)gw) / (unsigned)W);
    u1 = (int)(((unsigned)total * (unsigned)(gw + 1)) / (unsigned)W);
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

// Scalar (constant-cache) load of a wave-uniform int written by an earlier
// kernel or copy: it retires on lgkmcnt, so waiting for it never waits for the
// weight stream (vector loads retire in order on vmcnt).
__device__ __forceinline__ int sload_i32(const int* p) {
    return *(const __attribute__((address_space(4))) int*)(p);
}

// Prologue, split in two so that its global loads are issued BEFORE the first
// weight load: vmcnt retires in issue order, so the prologue's waits then never
// wait for the weight stream.
//  pro_load:   this wave's activation blocks (blocks wave, wave+NW, ...; and the
//              RMSNorm weights) into registers, the residual values of this
//              workgroup's units.
//  pro_finish: (after the weight prefill) RMSNorm / attention combine, Q8_K or
//              Q8_0 quantisation into LDS, residuals and the RoPE table to LDS.
constexpr int PRO_MAXB = 8;   // activation blocks one wave keeps in registers
struct ProRegs {
    f32x4 x[PRO_MAXB], w[PRO_MAXB];
    i32x4 tp;                  // {token, pos, cell, -} (a vector load: a scalar one would
                              // hold every LDS wait behind it, lgkmcnt counts both)
    float ra, rb;
    float ff[2];              // RoPE freq factors of pairs lane, lane+64 (wave 0)
    int nsplit;               // PRO_ATTN: attention splits to add
    bool regs;                // blocks held in registers (else re-read in pro_finish)
    bool attn_regs;           // PRO_ATTN: the splits' partials held in x[] (block i, split s: x[i*nsplit+s])
};

// Entry loads: the activation, RMSNorm weight and token position.  Their pointers
// arrive preloaded in SGPRs (kernarg preload, the kernel's leading arguments), so
// these loads are in flight at once, racing the load of the parameter block.
__device__ __forceinline__ void pro_load_entry(ProRegs& R, const float* x0, const float* nw_, const int* tp, int nb,
                                               bool regs, bool rms, int nw, int wave, int lane) {
    R.tp = tp ? *gptr(reinterpret_cast<const i32x4*>(tp)) : i32x4{0, 0, 0, 0};
    R.regs = regs;
    if (regs) {
        const auto x4 = gptr(reinterpret_cast<const f32x4*>(x0));
        const auto w4 = gptr(reinterpret_cast<const f32x4*>(nw_));
#pragma unroll
        for (int i = 0; i < PRO_MAXB; ++i) {
            const int blk = wave + i * nw;
            if (blk < nb) {
                R.x[i] = x4[blk * 64 + lane];
                if (rms) R.w[i] = w4[blk * 64 + lane];
            }
        }
    }
}

// Loads that need the parameter block: RoPE freq factors, the attention partials
// (their count depends on the cell count in R.tp) and the residuals of this
// workgroup's units.  Returns whether any were issued.
__device__ __forceinline__ bool pro_load_rest(const GemvParams& P, ProRegs& R, int nb, int nw, int wave, int lane,
                                              int wg_u0, int wg_u1) {
    const int tid = threadIdx.x;
    bool any = false;
    R.ff[0] = R.ff[1] = 1.0f;
    if (P.freq_factors) {
        any = true;
        if (wave == 0) {
            if (lane < P.n_rot / 2) R.ff[0] = gptr(P.freq_factors)[lane];
            if (lane + 64 < P.n_rot / 2) R.ff[1] = gptr(P.freq_factors)[lane + 64];
        }
    }
    R.nsplit = 0;
    R.attn_regs = false;
    if (P.pro == PRO_ATTN) {
        any = true;
        int chunk;
        attn_split(__builtin_amdgcn_readfirstlane(R.tp.z) + 1, chunk, R.nsplit);
        const int bpw = (nb + nw - 1) / nw;   // blocks per wave
        R.attn_regs = P.nslots == 1 && R.nsplit * bpw <= PRO_MAXB;
        if (R.attn_regs) {
            const AttnPartials& A = P.attn;
#pragma unroll
            for (int k = 0; k < PRO_MAXB; ++k) {   // register k = (block i, split s)
                const int i = k / R.nsplit, s = k % R.nsplit;
                const int blk = wave + i * nw;
                if (i < bpw && blk < nb)
                    R.x[k] = *gptr(reinterpret_cast<const f32x4*>(
                        A.o + (long long)s * A.n_head * A.head_dim + blk * 256 + lane * 4));
            }
        }
    }
    // residual values of this workgroup's units (the in-place residual add reads
    // them before any wave of the workgroup overwrites its rows).  Residual
    // launches have one segment (launch_gemv checks), so the lookup is scalar.
    R.ra = R.rb = 0.0f;
    const GemvSeg& S0 = P.seg[0];
    if (S0.resid) {
        any = true;
        if (tid < wg_u1 - wg_u0) {
            const long long lu = wg_u0 + tid;
            if (S0.pair == PAIR_ADJ) {
                const long long ra = 2 * lu;
                R.ra = gptr(S0.resid)[ra];
                R.rb = gptr(S0.resid)[ra + 1 < S0.A.rows ? ra + 1 : ra];
            } else {
                R.ra = gptr(S0.resid)[lu];
                R.rb = gptr(S0.resid)[lu];   // a second load, not a copy (a copy waits for the load)
            }
        }
    }
    return any;
}

// RAW_BARRIER: LDS-DMA is in flight (gemv_ring_body), so the reduction's barrier must not
// wait vmcnt(0) (see lds_barrier).
template <bool RAW_BARRIER>
__device__ __forceinline__ void pro_finish(const GemvParams& P, const ProRegs& R, char* smem, const SmemPlan& SP,
                                           int pos, int ncell, int wg_u0, int wg_u1, int bid) {
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nwaves = blockDim.x >> 6;
    const ActLayout& L = SP.L;
    double* red = reinterpret_cast<double*>(smem + SP.red_off);
    {
        float* rs = reinterpret_cast<float*>(smem + SP.resid_off);
        if (tid < wg_u1 - wg_u0) {
            rs[2 * tid] = R.ra;
            rs[2 * tid + 1] = R.rb;
        }
    }
    float scale = 1.0f;
    if (P.pro == PRO_RMSNORM) {
        // ggml_compute_forward_rms_norm_f32: sum of float squares in double
        double s = 0.0;
        if (R.regs) {
#pragma unroll
            for (int i = 0; i < PRO_MAXB; ++i) {
                if (wave + i * nwaves < L.nb) {
                    const f32x4 v = R.x[i];
                    s += (double)(v.x * v.x);
                    s += (double)(v.y * v.y);
                    s += (double)(v.z * v.z);
                    s += (double)(v.w * v.w);
                }
            }
        } else {
            const auto x4 = gptr(reinterpret_cast<const f32x4*>(P.x[0]));
            for (int i = tid; i < P.K / 4; i += blockDim.x) {
                const f32x4 v = x4[i];
                s += (double)(v.x * v.x);
                s += (double)(v.y * v.y);
                s += (double)(v.z * v.z);
                s += (double)(v.w * v.w);
            }
        }
        s = wave_sum63_d(s);
        if (lane == 63) red[wave] = s;
#ifdef MI_STAMPS
        if (P.stamps && threadIdx.x == 0) P.stamps[bid * 8 + 5] = __builtin_amdgcn_s_memrealtime();
#endif
        if (RAW_BARRIER) {
            __builtin_amdgcn_s_waitcnt((0xF) | (0x3 << 14) | (0x7 << 4));   // lgkmcnt(0) only
            __builtin_amdgcn_s_barrier();
        } else {
            __syncthreads();
        }
#ifdef MI_STAMPS
        if (P.stamps && threadIdx.x == 0) P.stamps[bid * 8 + 6] = __builtin_amdgcn_s_memrealtime();
#endif
        double tot = 0.0;
        for (int w = 0; w < nwaves; ++w) tot += red[w];
        const float mean = (float)(tot / (double)P.K);
        scale = 1.0f / sqrtf(mean + P.eps);
    }
    int nsplit = 0;
    if (P.pro == PRO_ATTN) {
        int chunk;
        attn_split(ncell, chunk, nsplit);
    }
    auto quant = [&](char* base, int blk, float v[4]) {
        if (P.need_q8k)
            quant_q8k_block(v, lane, reinterpret_cast<int8_t*>(base + L.q8k) + blk * 256,
                            reinterpret_cast<int*>(base + L.bsum) + blk * 16,
                            reinterpret_cast<float*>(base + L.dk) + blk);
        if (P.need_q80)
            quant_q80_block(v, lane, reinterpret_cast<int8_t*>(base + L.q80) + blk * 256,
                            reinterpret_cast<float*>(base + L.d0) + blk * 8);
    };
    if (R.attn_regs) {
        // the attention splits' partial sums (prefetched), added in split order
#pragma unroll
        for (int i = 0; i < PRO_MAXB; ++i) {
            const int blk = wave + i * nwaves;
            if (i * R.nsplit < PRO_MAXB && blk < L.nb) {
                f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
                for (int k = 0; k < PRO_MAXB; ++k)
                    if (k / R.nsplit == i) acc += R.x[k];
                float v[4] = {acc.x, acc.y, acc.z, acc.w};
                quant(smem, blk, v);
            }
        }
    } else if (R.regs) {
#pragma unroll
        for (int i = 0; i < PRO_MAXB; ++i) {
            const int blk = wave + i * nwaves;
            if (blk < L.nb) {
                float v[4] = {R.x[i].x, R.x[i].y, R.x[i].z, R.x[i].w};
                if (P.pro == PRO_RMSNORM) {
                    v[0] = (v[0] * scale) * R.w[i].x;   // ggml_vec_scale_f32 then ggml_mul
                    v[1] = (v[1] * scale) * R.w[i].y;
                    v[2] = (v[2] * scale) * R.w[i].z;
                    v[3] = (v[3] * scale) * R.w[i].w;
                }
                quant(smem, blk, v);
            }
        }
    } else {
        for (int slot = 0; slot < P.nslots; ++slot) {
            char* base = smem + slot * L.slot_bytes;
            const auto x4 = gptr(reinterpret_cast<const f32x4*>(P.x[slot]));
            for (int blk = wave; blk < L.nb; blk += nwaves) {
                float v[4];
                if (slot == 0 && P.pro == PRO_ATTN) {
                    // the attention splits' partial sums, added in split order
                    const AttnPartials& A = P.attn;
                    const int e0 = blk * 256 + lane * 4;
                    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
                    for (int s = 0; s < nsplit; ++s) {
                        const f32x4 o =
                            *gptr(reinterpret_cast<const f32x4*>(A.o + (long long)s * A.n_head * A.head_dim + e0));
                        acc.x += o.x;
                        acc.y += o.y;
                        acc.z += o.z;
                        acc.w += o.w;
                    }
                    v[0] = acc.x; v[1] = acc.y; v[2] = acc.z; v[3] = acc.w;
                } else {
                    const f32x4 xv = x4[blk * 64 + lane];
                    v[0] = xv.x; v[1] = xv.y; v[2] = xv.z; v[3] = xv.w;
                    if (slot == 0 && P.pro == PRO_RMSNORM) {
                        const f32x4 w = gptr(reinterpret_cast<const f32x4*>(P.norm_w))[blk * 64 + lane];
                        v[0] = (v[0] * scale) * w.x;
                        v[1] = (v[1] * scale) * w.y;
                        v[2] = (v[2] * scale) * w.z;
                        v[3] = (v[3] * scale) * w.w;
                    }
                }
                quant(base, blk, v);
            }
        }
    }
    // RoPE cache for this token's position (ggml_rope_cache_init, ext_factor 0, mscale 1)
    if (P.n_rot > 0 && wave == 0) {
        float* rope = reinterpret_cast<float*>(smem + SP.rope_off);
        for (int i = lane; i < P.n_rot / 2; i += 64) {
            float theta = (float)pos;
            for (int k = 0; k < i; ++k) theta = theta * P.theta_scale;
            const float ff = i < 64 ? R.ff[0] : R.ff[1];
            const float th = P.freq_scale * (theta / ff);
            rope[2 * i] = cosf(th);
            rope[2 * i + 1] = sinf(th);
        }
    }
}

// Epilogue inputs, uniform and kept in SGPRs: per launch (EpiConst) and per
// segment (EpiSeg, re-read from the LDS parameters only when the consumer enters a
// new segment).
struct EpiConst {
    __half* kcache;
    __half* vcache;
    int* cell_pos;
    int head_dim, n_rot, kv_dim;
};
struct EpiSeg {
    float* out;
    int epi, pair, unit0, end, rows;
};
__device__ __forceinline__ EpiConst epi_const(const GemvParams& P) {
    EpiConst E;
    E.kcache = rfl_ptr(P.kcache);
    E.vcache = rfl_ptr(P.vcache);
    E.cell_pos = rfl_ptr(P.cell_pos);
    E.head_dim = __builtin_amdgcn_readfirstlane(P.head_dim);
    E.n_rot = __builtin_amdgcn_readfirstlane(P.n_rot);
    E.kv_dim = __builtin_amdgcn_readfirstlane(P.kv_dim);
    return E;
}
__device__ __forceinline__ EpiSeg epi_seg(const GemvParams& P, int u) {
    int si = 0;
    while (si + 1 < P.nseg && u >= P.seg[si + 1].unit0) ++si;
    const GemvSeg& S = P.seg[si];
    EpiSeg e;
    e.out = rfl_ptr(S.out);
    e.epi = __builtin_amdgcn_readfirstlane(S.epi);
    e.pair = __builtin_amdgcn_readfirstlane(S.pair);
    e.unit0 = __builtin_amdgcn_readfirstlane(S.unit0);
    e.end = __builtin_amdgcn_readfirstlane(S.unit0 + S.units);
    e.rows = __builtin_amdgcn_readfirstlane(S.A.rows);
    return e;
}

// rva / rvb: residual values of rows A / B
__device__ __forceinline__ void gemv_epilogue(const EpiConst& E, const EpiSeg& S, int u, const float* rope,
                                              float rva, float rvb, float wa, float wb,
                                              int pos, int cell, float yA, float yB) {
    const auto out = gptr_w(S.out);
    const int lu = u - S.unit0;
    const bool adj = S.pair == PAIR_ADJ;
    const long long ra = adj ? 2LL * lu : lu, rb = adj ? ra + 1 : lu;
    const bool hasB = !adj || rb < S.rows;
    switch (S.epi) {
    case EPI_STORE:
        out[ra] = yA;
        if (hasB) out[rb] = yB;
        break;
    case EPI_ADD:
        out[ra] = yA + rva;
        if (hasB) out[rb] = yB + rvb;
        break;
    case EPI_ROPE_Q:
    case EPI_ROPE_K: {
        const int i0 = (int)(ra % E.head_dim);   // even
        float o0 = yA, o1 = yB;
        if (i0 < E.n_rot) {
            const float cs = rope[i0], sn = rope[i0 + 1];
            o0 = yA * cs - yB * sn;
            o1 = yA * sn + yB * cs;
        }
        if (S.epi == EPI_ROPE_Q) {
            out[ra] = o0;
            out[rb] = o1;
        } else {
            const auto kr = gptr_w(reinterpret_cast<unsigned short*>(E.kcache + (long long)cell * E.kv_dim));
            kr[ra] = __half_as_ushort(__float2half_rn(o0));
            kr[rb] = __half_as_ushort(__float2half_rn(o1));
            if (lu == 0) gptr_w(E.cell_pos)[cell] = pos;
        }
        break;
    }
    case EPI_V: {
        const auto vr = gptr_w(reinterpret_cast<unsigned short*>(E.vcache + (long long)cell * E.kv_dim));
        vr[ra] = __half_as_ushort(__float2half_rn(yA));
        if (hasB) vr[rb] = __half_as_ushort(__float2half_rn(yB));
        break;
    }
    case EPI_SWIGLU:
        out[lu] = silu_f(yA) * yB;
        break;
    case EPI_MOE_DOWN:
        out[lu] = (yA * wa + yB * wb) + rva;
        break;
    default: break;
    }
}

constexpr int kGemvParamVecs = (int)((sizeof(GemvParams) + 15) / 16);

// The GEMV of one workgroup: workgroup `bid` of P.grid.  NW waves per workgroup, D-deep ring.
// ROLE (template only, so the roofline kernel has its own symbol): 0 generic, 1 FFN gate/up.
// DUAL: two activation slots (MoE down).
template <int T, int D, int NW, int DUAL>
__device__ __forceinline__ void gemv_body(const float* __restrict__ kx0, const float* __restrict__ knw,
                                          const int* __restrict__ ktp, int kflags, const GemvParams& Pk,
                                          u32x4* sparams, const int bid) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    using K = Kq<T>;
    static_assert(K::LPS == 8, "8 lanes per superblock");
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // The launch's parameter block (~1 KB of kernarg) is copied to LDS by one
    // 16-byte vector load per lane: a single memory round trip.  Reading the
    // fields straight from kernarg compiles to a chain of ~15 dependent scalar
    // loads (segment lookup, plane bases, ...), each a full memory latency, which
    // cost 5-10 us per launch before the first weight load was issued.
    ProRegs pr;
    pro_load_entry(pr, kx0, knw, ktp, (kflags & 0xFFFFF) >> 8, (kflags >> 20) & 1, (kflags >> 21) & 1, NW, wave,
                   lane);
    {
        const u32x4* src = reinterpret_cast<const u32x4*>(&Pk);
        for (int i = threadIdx.x; i < kGemvParamVecs; i += NW * 64) sparams[i] = src[i];
        __syncthreads();
    }
    const GemvParams& P = *reinterpret_cast<const GemvParams*>(sparams);
    const int sbl = lane >> 3, j = lane & 7;
    const SmemPlan SP = smem_plan(P);
    const int nb = P.K >> 8;
    const int cpr = (nb + 7) >> 3;   // chunks per row
    int e0 = 0, e1 = 0;
    float w0 = 0.0f, w1 = 0.0f;
    if (P.sel) {
        e0 = __builtin_amdgcn_readfirstlane(gptr(P.sel)[0]);
        e1 = __builtin_amdgcn_readfirstlane(gptr(P.sel)[1]);
        w0 = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(gptr(P.selw)[0])));
        w1 = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(gptr(P.selw)[1])));
    }
#ifdef MI_STAMPS   // diagnostic build only (scripts/exp_gemv_stamps)
#define MI_STAMP(k) \
    if (P.stamps && threadIdx.x == 0) P.stamps[bid * 8 + (k)] = __builtin_amdgcn_s_memrealtime();
#else
#define MI_STAMP(k)
#endif
    MI_STAMP(0)
    // P.grid == gridDim.x (set by launch_gemv; reading gridDim costs a hidden-kernarg round trip)
    const int W = P.grid * NW;
    int u0, u1, wg_u0, wg_u1, dummy;
    unit_range(P.total_units, W, bid * NW + wave, u0, u1);
    unit_range(P.total_units, P.grid, bid, wg_u0, dummy);
    unit_range(P.total_units, W, bid * NW + NW - 1, dummy, wg_u1);
    const int n_items = (u1 - u0) * cpr;

    struct Slot { typename K::Ld a, b; };
    Slot ring[D];
    // Issue cursor: unit iu, chunk ic and the plane bases of the unit's two rows, kept in
    // SGPRs.  Moving to the next unit of the same segment is a pointer increment; only a
    // segment change (or a PAIR_ADJ odd-row tail) re-derives the bases from the LDS copy of
    // the parameters (a chain of dependent LDS reads, ~0.4 us: far too slow per unit).
    int iu = u0, ic = 0;
    const uint8_t* pa[4] = {nullptr, nullptr, nullptr, nullptr};
    const uint8_t* pb[4] = {nullptr, nullptr, nullptr, nullptr};
    int fast_end = 0;          // units < fast_end advance by a pointer increment
    int step_rows = 0;         // rows per unit: 2 (PAIR_ADJ) or 1 (PAIR_AB)
    auto bases = [&](int u) {
        const UnitRef c = unit_ref(P, u);
        const GemvSeg& S = P.seg[c.si];
        const QMat& MB = S.pair == PAIR_ADJ ? S.A : S.B;
        const long long ea = S.expA == 0 ? e0 : S.expA == 1 ? e1 : 0;
        const long long eb = S.expB == 0 ? e0 : S.expB == 1 ? e1 : 0;
        const long long rb = c.hasB ? c.rb : c.ra;   // odd tail: re-read row A, result unused
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            pa[i] = rfl_ptr(S.A.p[i] + ea * S.A.expert_stride[i] + c.ra * nb * PlaneBytes<T>::b[i]);
            pb[i] = rfl_ptr(MB.p[i] + eb * MB.expert_stride[i] + rb * nb * PlaneBytes<T>::b[i]);
        }
        const int pair = __builtin_amdgcn_readfirstlane(S.pair);
        const int end = __builtin_amdgcn_readfirstlane(S.unit0 + S.units);
        const int rows = __builtin_amdgcn_readfirstlane(S.A.rows);
        step_rows = pair == PAIR_ADJ ? 2 : 1;
        fast_end = (pair == PAIR_ADJ && (rows & 1)) ? end - 1 : end;   // the odd tail takes the slow path
    };
    auto next_unit = [&](int u) {
        if (u < fast_end) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const long long d = (long long)step_rows * nb * PlaneBytes<T>::b[i];
                pa[i] += d;
                pb[i] += d;
            }
        } else {
            bases(u);
        }
    };
    bases(u0 < P.total_units ? u0 : P.total_units - 1);   // idle waves re-read a valid row
    // Issue the next item (past the end: the last item again, a cache hit).
    // Past the end of its range a wave keeps issuing (so every ring step issues the same
    // loads and the compiler's vmcnt bookkeeping stays exact), but "parked": every lane
    // reads the same 16 bytes of the last row, one request per load instead of 16 lines.
    int park_sb = -1;          // -1: streaming; else 0 (every lane at offset 0)
    auto issue = [&](Slot& S) {
        const int sb = park_sb < 0 ? ic * 8 + sbl : 0;
        const int jj = park_sb < 0 ? j : 0;
        S.a = K::load(pa, sb, jj);
        S.b = K::load(pb, sb, jj);
        if (iu < u1) {
            if (++ic == cpr) {
                ic = 0;
                if (++iu < u1) next_unit(iu);
                else { iu = u1; park_sb = 0; }   // park
            }
        }
    };

    // Wait for the prologue loads that needed the parameter block BEFORE issuing the
    // weight prefill.  Issued together, those requests of late CUs queue behind
    // every CU's prefill at the memory channels (measured: ~3 us to land); alone
    // they land in ~1 us and the prologue then computes while the prefill streams.
    if (pro_load_rest(P, pr, nb, NW, wave, lane, wg_u0, wg_u1)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int k = 0; k < D - 1; ++k) issue(ring[k]);
    MI_STAMP(1)
    const int pos = __builtin_amdgcn_readfirstlane(pr.tp.y);
    const int cell = __builtin_amdgcn_readfirstlane(pr.tp.z);
    pro_finish<false>(P, pr, smem, SP, pos, cell + 1, wg_u0, wg_u1, bid);
    MI_STAMP(7)
    __syncthreads();
    MI_STAMP(2)
    const float* rope = reinterpret_cast<const float*>(smem + SP.rope_off);
    const float* rs = reinterpret_cast<const float*>(smem + SP.resid_off);
    const Act a0 = act_view(smem, SP.L, 0);
    const Act a1 = act_view(smem, SP.L, DUAL ? 1 : 0);

    int cu = u0, cc = 0;
    float accA = 0.0f, accB = 0.0f;
    const EpiConst EC = epi_const(P);
    EpiSeg cseg = epi_seg(P, u0 < P.total_units ? u0 : P.total_units - 1);
    auto consume = [&](const Slot& S) {
        const int sb = cc * 8 + sbl;
        const bool lv = sb < nb;
        const int sbc = lv ? sb : nb - 1;
        const typename K::AR arA = K::act(a0, sbc, j);
        const float pa_ = K::dot(S.a, arA, j);
        float pb_;
        if (DUAL) {
            const typename K::AR arB = K::act(a1, sbc, j);
            pb_ = K::dot(S.b, arB, j);
        } else {
            pb_ = K::dot(S.b, arA, j);
        }
        accA += lv ? pa_ : 0.0f;
        accB += lv ? pb_ : 0.0f;
        if (++cc == cpr) {
            const float yA = wave_sum63(accA);
            const float yB = wave_sum63(accB);
            if (cu >= cseg.end) cseg = epi_seg(P, cu);   // segment change (rare)
            if (lane == 63) {
                const int i = cu - wg_u0;
                gemv_epilogue(EC, cseg, cu, rope, rs[2 * i], rs[2 * i + 1], w0, w1, pos, cell, yA, yB);
            }
            accA = accB = 0.0f;
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
        if (base == 0) { MI_STAMP(3) }
    }
    MI_STAMP(4)
#undef MI_STAMP
}

template <int T, int D, int NW, int DUAL, int ROLE>
__global__ __launch_bounds__(NW * 64) void gemv_t(const float* __restrict__ kx0, const float* __restrict__ knw,
                                                   const int* __restrict__ ktp, int kflags, const GemvParams Pk) {
    __shared__ __attribute__((aligned(16))) u32x4 sparams[kGemvParamVecs];
    gemv_body<T, D, NW, DUAL>(kx0, knw, ktp, kflags, Pk, sparams, blockIdx.x);
}

// Two quant types in one launch (the Q/K/V projections of a Q4_K_M / Q5_K_M layer whose
// attn_v is Q6_K): workgroups [0, P1.grid) run the T1 matrices, the rest the T2 ones, each
// half with its own unit split.  Saves one launch (its fixed entry/prologue cost) per such
// layer.  Both halves consume the same activation (Q8_K of the RMS-normed residual).
template <int T1, int T2, int D, int NW>
__global__ __launch_bounds__(NW * 64) void gemv_mix_t(const float* __restrict__ kx0, const float* __restrict__ knw,
                                                       const int* __restrict__ ktp, int kflags, const GemvParams P1,
                                                       const GemvParams P2) {
    __shared__ __attribute__((aligned(16))) u32x4 sparams[kGemvParamVecs];
    const int g1 = P1.grid;
    if ((int)blockIdx.x < g1) gemv_body<T1, D, NW, 0>(kx0, knw, ktp, kflags, P1, sparams, blockIdx.x);
    else gemv_body<T2, D, NW, 0>(kx0, knw, ktp, kflags, P2, sparams, blockIdx.x - g1);
}

// ---------------------------------------------------------------------------
// The GEMV with its weight stream staged through LDS by LDS-DMA (global_load_lds).
//
// gemv_body keeps its in-flight weights in registers: D-1 items per wave, which at the
// register budget of its prologue is ~50 KB per CU, ~2 us of the CU's share of HBM
// bandwidth -- less than the prologue (activation arrival, RMSNorm, Q8_K quantisation) takes,
// so HBM idles until the prologue is done.  Here every wave owns a private ring of D item
// slots in LDS, filled by global_load_lds: ~110 KB in flight per CU from the moment the
// prologue starts, no VGPRs held, and no cross-wave synchronisation in the stream (a wave
// only ever reads the slots it filled itself, so its own vmcnt orders it).
// An item is one 8-superblock chunk of the unit's two rows, every plane (Rq<T>::ROW bytes a
// row); the LDS image is lane-linear per plane, so the consumer's reads are the register
// ring's loads with an LDS base.
// ---------------------------------------------------------------------------
// One LDS-DMA of 16 bytes a lane (global_load_lds_dwordx4, non-temporal: decode weights are
// read once).  Inline asm, not __builtin_amdgcn_global_load_lds: with the builtin, hipcc
// (ROCm 7.2) tail-merges an exec-masked DMA (the 8-lane header planes) with the full-wave one
// after it into ONE instruction whose M0 comes from v_readfirstlane of a per-lane select --
// the wrong LDS base for every lane outside the first (found by the GEMV op tests).  M0 is
// written and restored inside the statement (it is compiler-reserved); hipcc does not count
// these loads, the ring's wait_vm() does.
__device__ __forceinline__ void gl16(const uint8_t* g, char* l) {
    const unsigned la = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)l;
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(g), "s"(la) : "memory");
}
// s_waitcnt vmcnt(N) and nothing else (expcnt 7, lgkmcnt 15 = no wait)
template <int N>
__device__ __forceinline__ void wait_vm() {
    static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
    __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}
// workgroup barrier that leaves LDS-DMA in flight: this wave's LDS accesses complete (the
// data other waves read after the barrier), then s_barrier; __syncthreads() would also wait
// vmcnt(0), draining every wave's ring.
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_s_waitcnt((0xF) | (0x3 << 14) | (0x7 << 4) | (0x0 << 8));   // lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
}

template <int T> struct Rq;
template <> struct Rq<T_Q4_K> {   // qs 8x128 | hdr 8x16
    static constexpr int ROW = 1152, G = 2;
    __device__ static int glds(const uint8_t* const* rp, int sb0, char* d, int lane) {
        gl16(rp[0] + sb0 * 128 + lane * 16, d);
        if (lane < 8) gl16(rp[1] + (sb0 + lane) * 16, d + 1024);
        return 0;
    }
    __device__ static Kq<T_Q4_K>::Ld lds(const char* s, int sbl, int j, int) {
        Kq<T_Q4_K>::Ld l;
        l.qs = *reinterpret_cast<const u32x4*>(s + sbl * 128 + j * 16);
        l.hdr = *reinterpret_cast<const u32x4*>(s + 1024 + sbl * 16);
        return l;
    }
};
template <> struct Rq<T_Q5_K> {   // qs 8x128 | qh 8x32 | hdr 8x16
    static constexpr int ROW = 1408, G = 3;
    __device__ static int glds(const uint8_t* const* rp, int sb0, char* d, int lane) {
        gl16(rp[0] + sb0 * 128 + lane * 16, d);
        if (lane < 16) gl16(rp[1] + sb0 * 32 + lane * 16, d + 1024);
        if (lane < 8) gl16(rp[2] + (sb0 + lane) * 16, d + 1280);
        return 0;
    }
    __device__ static Kq<T_Q5_K>::Ld lds(const char* s, int sbl, int j, int) {
        Kq<T_Q5_K>::Ld l;
        l.qs = *reinterpret_cast<const u32x4*>(s + sbl * 128 + j * 16);
        l.qh = *reinterpret_cast<const u32x4*>(s + 1024 + sbl * 32 + (j & 1) * 16);
        l.hdr = *reinterpret_cast<const u32x4*>(s + 1280 + sbl * 16);
        return l;
    }
};
template <> struct Rq<T_Q6_K> {   // ql 8x128 | qh 8x64 | scales 8x16 | d: 32 B holding 8x2
    static constexpr int ROW = 1696, G = 4;
    // The d plane has 2 bytes a superblock, so a chunk's 16 bytes need not be 16-B aligned: two
    // lanes fetch the 32 aligned bytes around them; returns the chunk's offset within those.
    __device__ static int glds(const uint8_t* const* rp, int sb0, char* d, int lane) {
        gl16(rp[0] + sb0 * 128 + lane * 16, d);
        if (lane < 32) gl16(rp[1] + sb0 * 64 + lane * 16, d + 1024);
        if (lane < 8) gl16(rp[2] + (sb0 + lane) * 16, d + 1536);
        const uint8_t* dp = rp[3] + sb0 * 2;
        const uint8_t* da = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(dp) & ~(uintptr_t)15);
        if (lane < 2) gl16(da + lane * 16, d + 1664);
        return (int)(dp - da);
    }
    __device__ static Kq<T_Q6_K>::Ld lds(const char* s, int sbl, int j, int doff) {
        typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
        Kq<T_Q6_K>::Ld l;
        const int h = j >> 2, half = j & 1;
        l.ql = *reinterpret_cast<const u32x4*>(s + sbl * 128 + j * 16);
        l.qh = *reinterpret_cast<const u32x4*>(s + 1024 + sbl * 64 + 32 * h + 16 * half);
        const u32x2 sc = *reinterpret_cast<const u32x2*>(s + 1536 + sbl * 16 + h * 8);
        l.sc0 = sc.x;
        l.sc1 = sc.y;
        l.d = *reinterpret_cast<const unsigned short*>(s + 1664 + doff + sbl * 2);
        return l;
    }
};
template <> struct Rq<T_Q8_0> {   // qs 8x256 | d 8x16
    static constexpr int ROW = 2176, G = 3;
    __device__ static int glds(const uint8_t* const* rp, int sb0, char* d, int lane) {
        gl16(rp[0] + sb0 * 256 + lane * 16, d);
        gl16(rp[0] + sb0 * 256 + 1024 + lane * 16, d + 1024);
        if (lane < 8) gl16(rp[1] + (sb0 + lane) * 16, d + 2048);
        return 0;
    }
    __device__ static Kq<T_Q8_0>::Ld lds(const char* s, int sbl, int j, int) {
        Kq<T_Q8_0>::Ld l;
        l.q0 = *reinterpret_cast<const u32x4*>(s + sbl * 256 + j * 32);
        l.q1 = *reinterpret_cast<const u32x4*>(s + sbl * 256 + j * 32 + 16);
        l.d = *reinterpret_cast<const unsigned short*>(s + 2048 + sbl * 16 + j * 2);
        return l;
    }
};

// LDS ring depth per type at 8 waves (ring = 8 x D x 2 x ROW bytes, ~105-113 KB)
template <int T> struct RingD;
template <> struct RingD<T_Q4_K> { static constexpr int D = 6; };
template <> struct RingD<T_Q5_K> { static constexpr int D = 5; };
template <> struct RingD<T_Q6_K> { static constexpr int D = 4; };
template <> struct RingD<T_Q8_0> { static constexpr int D = 3; };
constexpr int RING_NW = 8;
__host__ __device__ inline int ring_bytes(int t) {
    switch (t) {
    case T_Q4_K: return RING_NW * 6 * 2 * 1152;
    case T_Q5_K: return RING_NW * 5 * 2 * 1408;
    case T_Q6_K: return RING_NW * 4 * 2 * 1696;
    case T_Q8_0: return RING_NW * 3 * 2 * 2176;
    default: return 0;
    }
}

template <int T, int DUAL>
__device__ __forceinline__ void gemv_ring_body(const float* __restrict__ kx0, const float* __restrict__ knw,
                                               const int* __restrict__ ktp, int kflags, const GemvParams& Pk,
                                               u32x4* sparams, const int bid) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    using K = Kq<T>;
    using RQ = Rq<T>;
    constexpr int NW = RING_NW, D = RingD<T>::D, ITEM = 2 * RQ::ROW, GI = 2 * RQ::G;
    static_assert((D - 1) * GI < 64, "in-flight LDS-DMA count must fit vmcnt");
    static_assert(D <= 8, "8 bits of slot offsets per slot in 64");
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    ProRegs pr;
    pro_load_entry(pr, kx0, knw, ktp, (kflags & 0xFFFFF) >> 8, (kflags >> 20) & 1, (kflags >> 21) & 1, NW, wave,
                   lane);
    {
        const u32x4* src = reinterpret_cast<const u32x4*>(&Pk);
        for (int i = threadIdx.x; i < kGemvParamVecs; i += NW * 64) sparams[i] = src[i];
        __syncthreads();   // no LDS-DMA in flight yet: waits for the parameters (and x) only
    }
    const GemvParams& P = *reinterpret_cast<const GemvParams*>(sparams);
#ifdef MI_STAMPS   // diagnostic build only (scripts/timeline.py)
#define MI_STAMP(k) \
    if (P.stamps && threadIdx.x == 0) P.stamps[bid * 8 + (k)] = __builtin_amdgcn_s_memrealtime();
#else
#define MI_STAMP(k)
#endif
    MI_STAMP(0)
    const int sbl = lane >> 3, j = lane & 7;
    const SmemPlan SP = smem_plan(P);
    char* const ring = smem + ((SP.total + 15) & ~15) + wave * (D * ITEM);
    const int nb = P.K >> 8;
    const int cpr = (nb + 7) >> 3;   // chunks per row
    int e0 = 0, e1 = 0;
    float w0 = 0.0f, w1 = 0.0f;
    if (P.sel) {
        e0 = __builtin_amdgcn_readfirstlane(gptr(P.sel)[0]);
        e1 = __builtin_amdgcn_readfirstlane(gptr(P.sel)[1]);
        w0 = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(gptr(P.selw)[0])));
        w1 = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(gptr(P.selw)[1])));
    }
    const int W = P.grid * NW;
    int u0, u1, wg_u0, wg_u1, dummy;
    unit_range(P.total_units, W, bid * NW + wave, u0, u1);
    unit_range(P.total_units, P.grid, bid, wg_u0, dummy);
    unit_range(P.total_units, W, bid * NW + NW - 1, dummy, wg_u1);
    const int n_items = (u1 - u0) * cpr;

    int iu = u0, ic = 0, islot = 0;
    unsigned long long doffs = 0;   // per ring slot: the A and B rows' Rq::glds offsets (4 bits each)
    const uint8_t* pa[4] = {nullptr, nullptr, nullptr, nullptr};
    const uint8_t* pb[4] = {nullptr, nullptr, nullptr, nullptr};
    int fast_end = 0, step_rows = 0;
    auto bases = [&](int u) {
        const UnitRef c = unit_ref(P, u);
        const GemvSeg& S = P.seg[c.si];
        const QMat& MB = S.pair == PAIR_ADJ ? S.A : S.B;
        const long long ea = S.expA == 0 ? e0 : S.expA == 1 ? e1 : 0;
        const long long eb = S.expB == 0 ? e0 : S.expB == 1 ? e1 : 0;
        const long long rb = c.hasB ? c.rb : c.ra;   // odd tail: re-read row A, result unused
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            pa[i] = rfl_ptr(S.A.p[i] + ea * S.A.expert_stride[i] + c.ra * nb * PlaneBytes<T>::b[i]);
            pb[i] = rfl_ptr(MB.p[i] + eb * MB.expert_stride[i] + rb * nb * PlaneBytes<T>::b[i]);
        }
        const int pair = __builtin_amdgcn_readfirstlane(S.pair);
        const int end = __builtin_amdgcn_readfirstlane(S.unit0 + S.units);
        const int rows = __builtin_amdgcn_readfirstlane(S.A.rows);
        step_rows = pair == PAIR_ADJ ? 2 : 1;
        fast_end = (pair == PAIR_ADJ && (rows & 1)) ? end - 1 : end;
    };
    auto next_unit = [&](int u) {
        if (u < fast_end) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const long long d = (long long)step_rows * nb * PlaneBytes<T>::b[i];
                pa[i] += d;
                pb[i] += d;
            }
        } else {
            bases(u);
        }
    };
    bases(u0 < P.total_units ? u0 : P.total_units - 1);
    // Issue the next item into the next ring slot.  Past the end of its range a wave keeps
    // issuing the last item again (cache hits into a free slot), so every step issues exactly
    // GI LDS-DMA instructions and the counted vmcnt waits stay exact.
    auto issue = [&]() {
        char* slot = ring + islot * ITEM;
        const unsigned oa = (unsigned)RQ::glds(pa, ic * 8, slot, lane);
        const unsigned ob = (unsigned)RQ::glds(pb, ic * 8, slot + RQ::ROW, lane);
        doffs = (doffs & ~(0xFFull << (8 * islot))) | ((unsigned long long)(oa | (ob << 4)) << (8 * islot));
        islot = islot + 1 == D ? 0 : islot + 1;
        if (iu < u1) {
            if (++ic == cpr) {
                if (iu + 1 < u1) {
                    ic = 0;
                    ++iu;
                    next_unit(iu);
                } else {
                    ic = cpr - 1;   // park on the last item
                    iu = u1;
                }
            }
        }
    };
    pro_load_rest(P, pr, nb, NW, wave, lane, wg_u0, wg_u1);
    // Every ordinary load the prologue consumes has landed before the first LDS-DMA: hipcc does
    // not count the asm DMAs, so a wait it placed later for one of those loads would count
    // them as younger loads and drain the ring's prefill.  The builtin (not asm) tells hipcc.
    wait_vm<0>();
#pragma unroll
    for (int k = 0; k < D - 1; ++k) issue();
    MI_STAMP(1)
    const int pos = __builtin_amdgcn_readfirstlane(pr.tp.y);
    const int cell = __builtin_amdgcn_readfirstlane(pr.tp.z);
    pro_finish<true>(P, pr, smem, SP, pos, cell + 1, wg_u0, wg_u1, bid);
    MI_STAMP(7)
    lds_barrier();
    MI_STAMP(2)
    const float* rope = reinterpret_cast<const float*>(smem + SP.rope_off);
    const float* rs = reinterpret_cast<const float*>(smem + SP.resid_off);
    const Act a0 = act_view(smem, SP.L, 0);
    const Act a1 = act_view(smem, SP.L, DUAL ? 1 : 0);

    int cu = u0, cc = 0, cslot = 0;
    float accA = 0.0f, accB = 0.0f;
    const EpiConst EC = epi_const(P);
    EpiSeg cseg = epi_seg(P, u0 < P.total_units ? u0 : P.total_units - 1);
    for (int it = 0; it < n_items; ++it) {
        issue();
        wait_vm<(D - 1) * GI>();   // this item's GI transfers have landed (D-1 items stay in flight)
        const char* slot = ring + cslot * ITEM;
        const unsigned off = (unsigned)(doffs >> (8 * cslot)) & 0xFFu;
        cslot = cslot + 1 == D ? 0 : cslot + 1;
        const typename K::Ld la = RQ::lds(slot, sbl, j, (int)(off & 0xF));
        const typename K::Ld lb = RQ::lds(slot + RQ::ROW, sbl, j, (int)(off >> 4));
        const int sb = cc * 8 + sbl;
        const bool lv = sb < nb;
        const int sbc = lv ? sb : nb - 1;
        const typename K::AR arA = K::act(a0, sbc, j);
        const float pa_ = K::dot(la, arA, j);
        float pb_;
        if (DUAL) {
            const typename K::AR arB = K::act(a1, sbc, j);
            pb_ = K::dot(lb, arB, j);
        } else {
            pb_ = K::dot(lb, arA, j);
        }
        accA += lv ? pa_ : 0.0f;
        accB += lv ? pb_ : 0.0f;
        if (++cc == cpr) {
            const float yA = wave_sum63(accA);
            const float yB = wave_sum63(accB);
            if (cu >= cseg.end) cseg = epi_seg(P, cu);   // segment change (rare)
            if (lane == 63) {
                const int i = cu - wg_u0;
                gemv_epilogue(EC, cseg, cu, rope, rs[2 * i], rs[2 * i + 1], w0, w1, pos, cell, yA, yB);
            }
            accA = accB = 0.0f;
            cc = 0;
            ++cu;
        }
        if (it == 0) { MI_STAMP(3) }
    }
    MI_STAMP(4)
    wait_vm<0>();   // the parked transfers land before the wave (and its LDS) retires
#undef MI_STAMP
}

template <int T, int DUAL, int ROLE>
__global__ __launch_bounds__(RING_NW * 64) void gemv_r(const float* __restrict__ kx0, const float* __restrict__ knw,
                                                        const int* __restrict__ ktp, int kflags, const GemvParams Pk) {
    __shared__ __attribute__((aligned(16))) u32x4 sparams[kGemvParamVecs];
    gemv_ring_body<T, DUAL>(kx0, knw, ktp, kflags, Pk, sparams, blockIdx.x);
}

template <int T1, int T2>
__global__ __launch_bounds__(RING_NW * 64) void gemv_r_mix(const float* __restrict__ kx0, const float* __restrict__ knw,
                                                            const int* __restrict__ ktp, int kflags, const GemvParams P1,
                                                            const GemvParams P2) {
    __shared__ __attribute__((aligned(16))) u32x4 sparams[kGemvParamVecs];
    if ((int)blockIdx.x < P1.grid) gemv_ring_body<T1, 0>(kx0, knw, ktp, kflags, P1, sparams, blockIdx.x);
    else gemv_ring_body<T2, 0>(kx0, knw, ktp, kflags, P2, sparams, blockIdx.x - P1.grid);
}

// ---------------------------------------------------------------------------
// The K-split GEMV (gemv_k): the decode GEMV without a workgroup-wide prologue.
//
// gemv_body / gemv_ring_body quantise the whole activation into LDS before any wave can
// consume a weight: x arrives, RMSNorm (a workgroup reduction), Q8_K of every block, a
// barrier -- 4-6 us per launch during which the weight stream is throttled (the stamp
// timelines of profiles/r02_timeline_*.txt).  Here the waves of a workgroup split K instead:
// G = ceil(K/2048) groups of m waves; group g streams superblocks [8g, 8g+8) of every unit the
// workgroup owns, so each lane needs the activation of ONE 32-element slice only, for the
// whole launch.  Every wave builds that slice itself, in registers:
//   RMSNorm   each wave sums the squares of the full x (the same double sum in every wave, so
//             every wave gets the bit-identical scale) -- no barrier;
//   Q8_K      the 8 lanes of a superblock reduce its amax (and the sign of its first
//             maximal element, ggml's tie rule) by DPP; each lane quantises its own 32 values
//             and forms its own two 16-element bsums, exactly as quantize_row_q8_K_ref;
//   Q8_0      a lane owns a whole 32-block (quantize_row_q8_0's x86 form), no reduction.
// The weight ring is issued right after the parameter block arrives and the slice math runs
// while it is in flight.  A unit's G chunk partials meet in LDS and are added in chunk order
// (deterministic) by the epilogue threads after one barrier at the end.
// ---------------------------------------------------------------------------
template <int T> struct KAct;
// Q8_K element positions of lane j within its superblock (Kq<T>::act's slices): two runs of 16
__device__ __forceinline__ int kpos_lo_q45(int j) { return 64 * (j >> 1) + 16 * (j & 1); }
__device__ __forceinline__ int kpos_lo_q6(int j) { return 128 * (j >> 2) + 32 * ((j >> 1) & 1) + 16 * (j & 1); }

// max over the 8 lanes of a lane group (lanes 8k..8k+7), every lane gets it
__device__ __forceinline__ float max8(float v) {
    v = fmaxf(v, __int_as_float(dpp_i<0xB1, 0xf>(__float_as_int(v))));   // quad_perm [1,0,3,2]
    v = fmaxf(v, __int_as_float(dpp_i<0x4E, 0xf>(__float_as_int(v))));   // quad_perm [2,3,0,1]
    v = fmaxf(v, __int_as_float(dpp_i<0x141, 0xf>(__float_as_int(v))));  // row_half_mirror
    return v;
}
__device__ __forceinline__ int min8(int v) {
    v = min(v, dpp_i<0xB1, 0xf>(v));
    v = min(v, dpp_i<0x4E, 0xf>(v));
    v = min(v, dpp_i<0x141, 0xf>(v));
    return v;
}

// quantize_row_q8_K_ref on one 256-block held as 32 values per lane by 8 lanes: lo[16] are
// elements plo..plo+15 and hi[16] elements phi..phi+15 (plo < phi).  Returns this lane's
// packed int8 values and bsums, and the block's d.
__device__ __forceinline__ void q8k_slice(const float lo[16], const float hi[16], int plo, int phi, i32x4& alo,
                                          i32x4& ahi, int& bs_lo, int& bs_hi, float& dx) {
    float am = 0.0f;
#pragma unroll
    for (int e = 0; e < 16; ++e) am = fmaxf(am, fmaxf(fabsf(lo[e]), fabsf(hi[e])));
    const float amax = max8(am);
    int q[32];
    if (amax == 0.0f) {
#pragma unroll
        for (int e = 0; e < 32; ++e) q[e] = 0;
        dx = 0.0f;
    } else {
        // the signed value at the FIRST index whose |x| is the maximum: key = 2*index + sign
        int key = 1 << 20;
#pragma unroll
        for (int e = 15; e >= 0; --e)
            if (fabsf(hi[e]) == amax) key = 2 * (phi + e) + (hi[e] < 0.0f ? 1 : 0);
#pragma unroll
        for (int e = 15; e >= 0; --e)
            if (fabsf(lo[e]) == amax) key = 2 * (plo + e) + (lo[e] < 0.0f ? 1 : 0);
        key = min8(key);
        const float mx = (key & 1) ? -amax : amax;
        const float iscale = -127.0f / mx;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            q[e] = min(127, (int)rintf(iscale * lo[e]));
            q[16 + e] = min(127, (int)rintf(iscale * hi[e]));
        }
        dx = 1.0f / iscale;
    }
    int sl = 0, sh = 0;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        sl += q[e];
        sh += q[16 + e];
    }
    bs_lo = sl;
    bs_hi = sh;
    int pk[8];
#pragma unroll
    for (int w = 0; w < 8; ++w)
        pk[w] = (q[4 * w] & 0xFF) | ((q[4 * w + 1] & 0xFF) << 8) | ((q[4 * w + 2] & 0xFF) << 16) | ((q[4 * w + 3] & 0xFF) << 24);
    alo = i32x4{pk[0], pk[1], pk[2], pk[3]};
    ahi = i32x4{pk[4], pk[5], pk[6], pk[7]};
}

template <> struct KAct<T_Q4_K> {
    __device__ static void pos(int j, int& lo, int& hi) { lo = kpos_lo_q45(j); hi = lo + 32; }
    __device__ static Kq<T_Q4_K>::AR quant(const float lo[16], const float hi[16], int j) {
        int plo, phi;
        pos(j, plo, phi);
        Kq<T_Q4_K>::AR r;
        q8k_slice(lo, hi, plo, phi, r.alo, r.ahi, r.bs_lo, r.bs_hi, r.dx);
        return r;
    }
};
template <> struct KAct<T_Q5_K> {
    __device__ static void pos(int j, int& lo, int& hi) { KAct<T_Q4_K>::pos(j, lo, hi); }
    __device__ static Kq<T_Q5_K>::AR quant(const float lo[16], const float hi[16], int j) {
        return KAct<T_Q4_K>::quant(lo, hi, j);
    }
};
template <> struct KAct<T_Q6_K> {
    __device__ static void pos(int j, int& lo, int& hi) { lo = kpos_lo_q6(j); hi = lo + 64; }
    __device__ static Kq<T_Q6_K>::AR quant(const float lo[16], const float hi[16], int j) {
        int plo, phi;
        pos(j, plo, phi);
        Kq<T_Q6_K>::AR r;
        q8k_slice(lo, hi, plo, phi, r.alo, r.ahi, r.bs_lo, r.bs_hi, r.dx);
        return r;
    }
};
template <> struct KAct<T_Q8_0> {   // lane j: elements 32j..32j+31 = one Q8_0 block
    __device__ static void pos(int j, int& lo, int& hi) { lo = 32 * j; hi = lo + 16; }
    __device__ static Kq<T_Q8_0>::AR quant(const float lo[16], const float hi[16], int) {
        float am = 0.0f;
#pragma unroll
        for (int e = 0; e < 16; ++e) am = fmaxf(am, fmaxf(fabsf(lo[e]), fabsf(hi[e])));
        const float d = am / 127.0f;
        const float id = am != 0.0f ? 127.0f / am : 0.0f;
        int pk[8];
#pragma unroll
        for (int w = 0; w < 8; ++w) {
            const float* src = w < 4 ? lo + 4 * w : hi + 4 * (w - 4);
            int q0 = (int)rintf(src[0] * id), q1 = (int)rintf(src[1] * id), q2 = (int)rintf(src[2] * id),
                q3 = (int)rintf(src[3] * id);
            pk[w] = (q0 & 0xFF) | ((q1 & 0xFF) << 8) | ((q2 & 0xFF) << 16) | ((q3 & 0xFF) << 24);
        }
        Kq<T_Q8_0>::AR r;
        r.a0 = i32x4{pk[0], pk[1], pk[2], pk[3]};
        r.a1 = i32x4{pk[4], pk[5], pk[6], pk[7]};
        r.d0 = __half2float(__float2half_rn(d));
        return r;
    }
};

// K-split geometry: G chunk groups of m waves, NW = G*m <= 8 (two waves a SIMD: the
// prologue's x slices and the ring need the 256-VGPR budget)
__host__ __device__ inline int gemv_k_groups(int K) { return (K / 256 + 7) / 8; }
__host__ __device__ inline int gemv_k_waves(int K) {
    const int G = gemv_k_groups(K);
    return G * (8 / G);
}
template <int T> struct KRingD { static constexpr int D = 4; };   // register ring depth

// LDS: [params copy (static)] [rope table | resid | partials[wg_units][G] float2]
struct KPlan { int rope_off, resid_off, part_off, total; };
__host__ __device__ inline KPlan kplan(const GemvParams& p) {
    KPlan k;
    k.rope_off = 0;
    k.resid_off = ((p.n_rot / 2) * 8 + 15) / 16 * 16;
    k.part_off = k.resid_off + ((p.wg_units * 2 * 4 + 15) / 16) * 16;
    k.total = k.part_off + p.wg_units * gemv_k_groups(p.K) * 8;
    k.total = (k.total + 15) & ~15;   // then [16] doubles of RMSNorm shares (the kernel's red[])
    return k;
}

__device__ __forceinline__ void k_load_slice(const float* __restrict__ p, int e0, int e1, float lo[16], float hi[16]) {
#pragma unroll
    for (int v = 0; v < 4; ++v) {
        const f32x4 a = *gptr(reinterpret_cast<const f32x4*>(p + e0) + v);
        const f32x4 b = *gptr(reinterpret_cast<const f32x4*>(p + e1) + v);
        lo[4 * v] = a.x; lo[4 * v + 1] = a.y; lo[4 * v + 2] = a.z; lo[4 * v + 3] = a.w;
        hi[4 * v] = b.x; hi[4 * v + 1] = b.y; hi[4 * v + 2] = b.z; hi[4 * v + 3] = b.w;
    }
}

// This wave's share of ggml_compute_forward_rms_norm_f32's sum of squares: float4 i of x for
// i = lane + 64*(wave + NW*r); KX_PART float4 a lane are loaded at kernel entry (K <= 8192 at 8
// waves), the rest (larger K) after.  The shares meet in LDS in wave order.
constexpr int KX_PART = 4;

// kflags: K (bits 0-19) | RMSNorm prologue (21) | attention-combine prologue (22); for the
// attention prologue kx0 is split 0 of the attention partials.
template <int T, int D, int DUAL>
__device__ __forceinline__ void gemv_k_body(const float* __restrict__ kx0, const float* __restrict__ knw,
                                            const int* __restrict__ ktp, int kflags, const GemvParams& Pk,
                                            u32x4* sparams, const int bid) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    using K = Kq<T>;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int NW = blockDim.x >> 6;
    const int Kdim = kflags & 0xFFFFF;
    const int nb = Kdim >> 8;
    const int G = (nb + 7) >> 3;
    const int m = NW / G;
    const int g = wave / m, wk = wave - g * m;
    const int sbl = lane >> 3, j = lane & 7;
    const int sb = 8 * g + sbl;
    const bool lv = sb < nb;
    const bool rms = (kflags >> 21) & 1;
    const bool attn_pro = (kflags >> 22) & 1;
    int plo, phi;
    KAct<T>::pos(j, plo, phi);
    const int xe0 = (lv ? sb : 0) * 256 + plo, xe1 = (lv ? sb : 0) * 256 + phi;
    // ---- entry: loads that need only the direct arguments (this lane's activation slice of
    // slot 0, its norm weights, this wave's share of the RMSNorm sum, the token position) and
    // the parameter block: one round trip for all of them
    float xlo[16], xhi[16], wlo[16], whi[16];
    k_load_slice(kx0, xe0, xe1, xlo, xhi);
    if (rms) k_load_slice(knw, xe0, xe1, wlo, whi);
    f32x4 xr[KX_PART];
    const int n4 = Kdim / 4;
    if (rms) {
        const auto x4 = gptr(reinterpret_cast<const f32x4*>(kx0));
#pragma unroll
        for (int r = 0; r < KX_PART; ++r) {
            const int i = lane + 64 * (wave + NW * r);
            xr[r] = i < n4 ? x4[i] : f32x4{0.f, 0.f, 0.f, 0.f};
        }
    }
    const i32x4 tp = ktp ? *gptr(reinterpret_cast<const i32x4*>(ktp)) : i32x4{0, 0, 0, 0};
    {
        const u32x4* src = reinterpret_cast<const u32x4*>(&Pk);
        for (int i = threadIdx.x; i < kGemvParamVecs; i += blockDim.x) sparams[i] = src[i];
        __syncthreads();
    }
    const GemvParams& P = *reinterpret_cast<const GemvParams*>(sparams);
#ifdef MI_STAMPS   // diagnostic build only (scripts/timeline.py)
#define MI_STAMP(k) \
    if (P.stamps && threadIdx.x == 0) P.stamps[bid * 8 + (k)] = __builtin_amdgcn_s_memrealtime();
#else
#define MI_STAMP(k)
#endif
    MI_STAMP(0)
    const KPlan KP = kplan(P);
    double* red = reinterpret_cast<double*>(smem + KP.total);   // [NW] RMSNorm shares
    int e0 = 0, e1 = 0;
    float w0 = 0.0f, w1 = 0.0f;
    if (P.sel) {   // MoE: the experts decide the weight addresses
        e0 = __builtin_amdgcn_readfirstlane(gptr(P.sel)[0]);
        e1 = __builtin_amdgcn_readfirstlane(gptr(P.sel)[1]);
        w0 = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(gptr(P.selw)[0])));
        w1 = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(gptr(P.selw)[1])));
    }
    int wg_u0, wg_u1;
    unit_range(P.total_units, P.grid, bid, wg_u0, wg_u1);
    const int nwu = wg_u1 - wg_u0;
    const int u0 = wg_u0 + (int)(((unsigned)nwu * (unsigned)wk) / (unsigned)m);
    const int u1 = wg_u0 + (int)(((unsigned)nwu * (unsigned)(wk + 1)) / (unsigned)m);
    const int n_items = u1 - u0;
    // attention splits past the first (contexts over ATTN_SHORT cells): added in split order
    // before the prefetch -- a load issued behind it would wait for all of it
    if (attn_pro) {
        int chunk_, nsplit;
        attn_split(__builtin_amdgcn_readfirstlane(tp.z) + 1, chunk_, nsplit);
        const AttnPartials& A = P.attn;
        for (int s = 1; s < nsplit; ++s) {
            float lo[16], hi[16];
            k_load_slice(A.o + (long long)s * A.n_head * A.head_dim, xe0, xe1, lo, hi);
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                xlo[e] += lo[e];
                xhi[e] += hi[e];
            }
        }
    }
    // the other inputs of the prologue, issued before the prefetch, consumed after it
    float ylo[16], yhi[16];
    if (DUAL) k_load_slice(P.x[1], xe0, xe1, ylo, yhi);
    const bool rope_wave = P.n_rot > 0 && wave == NW - 1;
    float ff0 = 1.0f, ff1 = 1.0f;
    if (rope_wave && P.freq_factors) {
        if (lane < P.n_rot / 2) ff0 = gptr(P.freq_factors)[lane];
        if (lane + 64 < P.n_rot / 2) ff1 = gptr(P.freq_factors)[lane + 64];
    }

    // ---- the weight prefetch
    struct Slot { typename K::Ld a, b; };
    Slot ring[D];
    int iu = u0;
    const uint8_t* pa[4] = {nullptr, nullptr, nullptr, nullptr};
    const uint8_t* pb[4] = {nullptr, nullptr, nullptr, nullptr};
    int fast_end = 0, step_rows = 0;
    auto bases = [&](int u) {
        const UnitRef c = unit_ref(P, u);
        const GemvSeg& S = P.seg[c.si];
        const QMat& MB = S.pair == PAIR_ADJ ? S.A : S.B;
        const long long ea = S.expA == 0 ? e0 : S.expA == 1 ? e1 : 0;
        const long long eb = S.expB == 0 ? e0 : S.expB == 1 ? e1 : 0;
        const long long rb = c.hasB ? c.rb : c.ra;   // odd tail: re-read row A, result unused
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            pa[i] = rfl_ptr(S.A.p[i] + ea * S.A.expert_stride[i] + c.ra * nb * PlaneBytes<T>::b[i]);
            pb[i] = rfl_ptr(MB.p[i] + eb * MB.expert_stride[i] + rb * nb * PlaneBytes<T>::b[i]);
        }
        const int pair = __builtin_amdgcn_readfirstlane(S.pair);
        const int end = __builtin_amdgcn_readfirstlane(S.unit0 + S.units);
        const int rows = __builtin_amdgcn_readfirstlane(S.A.rows);
        step_rows = pair == PAIR_ADJ ? 2 : 1;
        fast_end = (pair == PAIR_ADJ && (rows & 1)) ? end - 1 : end;
    };
    auto next_unit = [&](int u) {
        if (u < fast_end) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const long long d = (long long)step_rows * nb * PlaneBytes<T>::b[i];
                pa[i] += d;
                pb[i] += d;
            }
        } else {
            bases(u);
        }
    };
    bases(u0 < P.total_units ? u0 : P.total_units - 1);
    // past the end of its range a wave re-issues its last item (cache hits) so every ring step
    // issues the same loads and hipcc's vmcnt bookkeeping stays exact
    const int sbi = lv ? sb : nb - 1;
    auto issue = [&](Slot& S) {
        S.a = K::load(pa, sbi, j);
        S.b = K::load(pb, sbi, j);
        if (iu + 1 < u1) next_unit(++iu);
    };
#pragma unroll
    for (int k = 0; k < D - 1; ++k) issue(ring[k]);
    MI_STAMP(1)
    // this wave's RMSNorm share: its x loads were issued at entry, before the ring, so waiting
    // for them here does not wait for the weights (loads retire in order); doing this before the
    // ring issue held the first weight loads back by one x round trip (r02 stamps: 1.2-2.8 us)
    if (rms) {
        double sacc = 0.0;
#pragma unroll
        for (int r = 0; r < KX_PART; ++r) {
            const f32x4 v = xr[r];
            sacc += (double)(v.x * v.x);
            sacc += (double)(v.y * v.y);
            sacc += (double)(v.z * v.z);
            sacc += (double)(v.w * v.w);
        }
        sacc = wave_sum63_d(sacc);
        if (lane == 63) red[wave] = sacc;
    }
    // residual values of this workgroup's units: needed only by the epilogue threads
    float ra = 0.0f, rbv = 0.0f;
    const bool has_resid = P.seg[0].resid && (int)threadIdx.x < nwu;
    if (has_resid) {
        const GemvSeg& S0 = P.seg[0];
        const long long lu = wg_u0 + threadIdx.x;
        if (S0.pair == PAIR_ADJ) {
            ra = gptr(S0.resid)[2 * lu];
            rbv = gptr(S0.resid)[2 * lu + 1 < S0.A.rows ? 2 * lu + 1 : 2 * lu];
        } else {
            ra = gptr(S0.resid)[lu];
            rbv = gptr(S0.resid)[lu];
        }
    }
    // ---- the activation slice, while the prefetch is in flight
    typename K::AR arA, arB;
    {
        if (rms) {
            __syncthreads();   // every wave's RMSNorm share is in LDS (loads stay in flight)
            double tot = 0.0;
            for (int w = 0; w < NW; ++w) tot += red[w];
            if (n4 > 64 * NW * KX_PART) {   // K > 8192 at 8 waves: the rest of the sum (rare)
                const auto x4 = gptr(reinterpret_cast<const f32x4*>(kx0));
                double sacc = 0.0;
                for (int i = lane + 64 * NW * KX_PART; i < n4; i += 64) {
                    const f32x4 v = x4[i];
                    sacc += (double)(v.x * v.x);
                    sacc += (double)(v.y * v.y);
                    sacc += (double)(v.z * v.z);
                    sacc += (double)(v.w * v.w);
                }
                sacc = wave_sum63_d(sacc);
                const long long b = __double_as_longlong(sacc);
                const int lo = __builtin_amdgcn_readlane((int)b, 63), hi = __builtin_amdgcn_readlane((int)(b >> 32), 63);
                tot += __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
            }
            const float mean = (float)(tot / (double)Kdim);
            const float scale = 1.0f / sqrtf(mean + P.eps);
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                xlo[e] = (xlo[e] * scale) * wlo[e];   // ggml_vec_scale_f32 then ggml_mul
                xhi[e] = (xhi[e] * scale) * whi[e];
            }
        }
        if (!lv) {
#pragma unroll
            for (int e = 0; e < 16; ++e) xlo[e] = xhi[e] = 0.0f;
        }
        arA = KAct<T>::quant(xlo, xhi, j);
        if (DUAL) {
            if (!lv) {
#pragma unroll
                for (int e = 0; e < 16; ++e) ylo[e] = yhi[e] = 0.0f;
            }
            arB = KAct<T>::quant(ylo, yhi, j);
        } else {
            arB = arA;
        }
    }
    const int pos = __builtin_amdgcn_readfirstlane(tp.y);
    const int cell = __builtin_amdgcn_readfirstlane(tp.z);
    float* rope = reinterpret_cast<float*>(smem + KP.rope_off);
    float* rs = reinterpret_cast<float*>(smem + KP.resid_off);
    float2* part = reinterpret_cast<float2*>(smem + KP.part_off);
    if (rope_wave) {   // ggml_rope_cache_init for this token's position (the epilogue reads it)
        for (int i = lane; i < P.n_rot / 2; i += 64) {
            float theta = (float)pos;
            for (int k = 0; k < i; ++k) theta = theta * P.theta_scale;
            const float ff = i < 64 ? ff0 : ff1;
            const float th = P.freq_scale * (theta / ff);
            rope[2 * i] = cosf(th);
            rope[2 * i + 1] = sinf(th);
        }
    }
    MI_STAMP(7)
    // ---- the stream: one item (this chunk of one unit's two rows) per unit
    int cu = u0;
    auto consume = [&](const Slot& S) {
        const float pa_ = K::dot(S.a, arA, j);
        const float pb_ = K::dot(S.b, arB, j);
        const float yA = wave_sum63(lv ? pa_ : 0.0f);
        const float yB = wave_sum63(lv ? pb_ : 0.0f);
        if (lane == 63) part[(cu - wg_u0) * G + g] = make_float2(yA, yB);
        ++cu;
    };
    for (int base = 0; base < n_items; base += D) {
#pragma unroll
        for (int k = 0; k < D; ++k) {
            issue(ring[(k + D - 1) % D]);
            if (base + k < n_items) consume(ring[k]);
        }
        if (base == 0) { MI_STAMP(3) }
    }
    if (has_resid) {
        rs[2 * threadIdx.x] = ra;
        rs[2 * threadIdx.x + 1] = rbv;
    }
    __syncthreads();
    MI_STAMP(2)
    // ---- epilogue: one thread per unit adds its G chunk partials in chunk order
    const EpiConst EC = epi_const(P);
    for (int i = threadIdx.x; i < nwu; i += blockDim.x) {
        const int u = wg_u0 + i;
        float yA = 0.0f, yB = 0.0f;
        for (int q = 0; q < G; ++q) {
            const float2 v = part[i * G + q];
            yA += v.x;
            yB += v.y;
        }
        int si = 0;
        while (si + 1 < P.nseg && u >= P.seg[si + 1].unit0) ++si;
        const GemvSeg& S = P.seg[si];
        EpiSeg es;
        es.out = S.out;
        es.epi = S.epi;
        es.pair = S.pair;
        es.unit0 = S.unit0;
        es.end = S.unit0 + S.units;
        es.rows = S.A.rows;
        gemv_epilogue(EC, es, u, rope, rs[2 * i], rs[2 * i + 1], w0, w1, pos, cell, yA, yB);
    }
    MI_STAMP(4)
#undef MI_STAMP
}

template <int T, int DUAL, int ROLE>
__global__ __launch_bounds__(512) void gemv_k(const float* __restrict__ kx0, const float* __restrict__ knw,
                                               const int* __restrict__ ktp, int kflags, const GemvParams Pk) {
    __shared__ __attribute__((aligned(16))) u32x4 sparams[kGemvParamVecs];
    gemv_k_body<T, KRingD<T>::D, DUAL>(kx0, knw, ktp, kflags, Pk, sparams, blockIdx.x);
}

template <int T1, int T2>
__global__ __launch_bounds__(512) void gemv_k_mix(const float* __restrict__ kx0, const float* __restrict__ knw,
                                                   const int* __restrict__ ktp, int kflags, const GemvParams P1,
                                                   const GemvParams P2) {
    __shared__ __attribute__((aligned(16))) u32x4 sparams[kGemvParamVecs];
    if ((int)blockIdx.x < P1.grid) gemv_k_body<T1, KRingD<T1>::D, 0>(kx0, knw, ktp, kflags, P1, sparams, blockIdx.x);
    else gemv_k_body<T2, KRingD<T2>::D, 0>(kx0, knw, ktp, kflags, P2, sparams, blockIdx.x - P1.grid);
}

typedef void (*GemvFn)(const float*, const float*, const int*, int, const GemvParams);
typedef void (*GemvMixFn)(const float*, const float*, const int*, int, const GemvParams, const GemvParams);

// Kernel configurations: waves per workgroup NW and ring depth D (one
// workgroup per CU).  MI_GEMV_CFG=n selects config n for every type
// (micro-benchmarks); otherwise gemv_cfg_for(type).
struct GemvCfg { int nw, d; };
constexpr GemvCfg kGemvCfgs[] = {{16, 2}, {8, 4}, {8, 3}, {16, 3}, {8, 6}, {8, 8}, {4, 8}};
constexpr int kNumGemvCfgs = sizeof(kGemvCfgs) / sizeof(kGemvCfgs[0]);
// Per launch role (measured on the 7B Q4_K_M decode, profiles/r01_*): the FFN gate/up
// launch (the largest, 50 MB) runs best with 16 waves x 2-deep rings, the others with 8 x 4.
// MI_GEMV_CFG / MI_GEMV_CFG_<ROLE> override (sweeps).
static int gemv_cfg_for(int type, int role) {
    static const int forced = getenv("MI_GEMV_CFG") ? atoi(getenv("MI_GEMV_CFG")) : -1;
    if (forced >= 0 && forced < kNumGemvCfgs) return forced;
    static const char* names[6] = {"MI_GEMV_CFG_QKV", "MI_GEMV_CFG_WO", "MI_GEMV_CFG_UP", "MI_GEMV_CFG_DOWN",
                                   "MI_GEMV_CFG_OUT", "MI_GEMV_CFG_GEN"};
    static int per_role[6] = {-2, -2, -2, -2, -2, -2};
    if (role >= 0 && role < 6) {
        if (per_role[role] == -2) per_role[role] = getenv(names[role]) ? atoi(getenv(names[role])) : -1;
        if (per_role[role] >= 0 && per_role[role] < kNumGemvCfgs) return per_role[role];
    }
    (void)type;
    return role == ROLE_FFN_UP ? 0 : 1;
}

template <int T, int DUAL, int ROLE>
static GemvFn gemv_fn_cfg(int cfg) {
    switch (cfg) {
    case 0: return gemv_t<T, 2, 16, DUAL, ROLE>;
    case 1: return gemv_t<T, 4, 8, DUAL, ROLE>;
    case 2: return gemv_t<T, 3, 8, DUAL, ROLE>;
    case 3: return gemv_t<T, 3, 16, DUAL, ROLE>;
    case 4: return gemv_t<T, 6, 8, DUAL, ROLE>;
    case 5: return gemv_t<T, 8, 8, DUAL, ROLE>;
    case 6: return gemv_t<T, 8, 4, DUAL, ROLE>;
    default: return nullptr;
    }
}

template <int DUAL, int ROLE>
static GemvFn gemv_fn_t(int type, int cfg) {
    switch (type) {
    case T_Q4_K: return gemv_fn_cfg<T_Q4_K, DUAL, ROLE>(cfg);
    case T_Q5_K: return gemv_fn_cfg<T_Q5_K, DUAL, ROLE>(cfg);
    case T_Q6_K: return gemv_fn_cfg<T_Q6_K, DUAL, ROLE>(cfg);
    case T_Q8_0: return gemv_fn_cfg<T_Q8_0, DUAL, ROLE>(cfg);
    default: return nullptr;
    }
}

static GemvFn gemv_fn(int role, int type, int nslots, int cfg) {
    if (nslots > 1) return gemv_fn_t<1, 2>(type, cfg);
    return role == ROLE_FFN_UP ? gemv_fn_t<0, 1>(type, cfg) : gemv_fn_t<0, 0>(type, cfg);
}


// Dynamic LDS a GEMV may use: 160 KB minus its static copy of the parameters.
constexpr int kGemvDynLds = 160 * 1024 - (int)((sizeof(GemvParams) + 15) / 16 * 16);

template <int T, int D> __global__ void gemm_t(const GemmParams P);
static void gemm_attrs();
static GemvMixFn gemv_mix_fn(int t1, int t2);

// Decode GEMV implementation: MI_GEMV=k (default: the K-split gemv_k), ring (the LDS-DMA ring
// gemv_r), reg (the register ring gemv_t with a workgroup prologue) -- A/B switches.
enum GemvImpl { GEMV_REG = 0, GEMV_RING = 1, GEMV_KSPLIT = 2 };
static int gemv_impl() {
    static const int impl = [] {
        const char* e = getenv("MI_GEMV");
        if (getenv("MI_GEMV_REG")) return (int)GEMV_REG;
        if (!e || !*e || !strcmp(e, "k")) return (int)GEMV_KSPLIT;
        if (!strcmp(e, "ring")) return (int)GEMV_RING;
        return (int)GEMV_REG;
    }();
    return impl;
}
static bool gemv_ring_on() { return gemv_impl() == GEMV_RING; }
static bool gemv_k_on(int K) { return gemv_impl() == GEMV_KSPLIT && gemv_k_groups(K) <= 8; }

template <int DUAL, int ROLE>
static GemvFn gemv_k_fn_t(int type) {
    switch (type) {
    case T_Q4_K: return gemv_k<T_Q4_K, DUAL, ROLE>;
    case T_Q5_K: return gemv_k<T_Q5_K, DUAL, ROLE>;
    case T_Q6_K: return gemv_k<T_Q6_K, DUAL, ROLE>;
    case T_Q8_0: return gemv_k<T_Q8_0, DUAL, ROLE>;
    default: return nullptr;
    }
}
static GemvFn gemv_k_fn(int role, int type, int nslots) {
    if (nslots > 1) return gemv_k_fn_t<1, 2>(type);
    return role == ROLE_FFN_UP ? gemv_k_fn_t<0, 1>(type) : gemv_k_fn_t<0, 0>(type);
}
static GemvMixFn gemv_k_mix_fn(int t1, int t2) {
    if (t1 == T_Q4_K && t2 == T_Q6_K) return gemv_k_mix<T_Q4_K, T_Q6_K>;
    if (t1 == T_Q5_K && t2 == T_Q6_K) return gemv_k_mix<T_Q5_K, T_Q6_K>;
    return nullptr;
}

template <int DUAL, int ROLE>
static GemvFn gemv_r_fn_t(int type) {
    switch (type) {
    case T_Q4_K: return gemv_r<T_Q4_K, DUAL, ROLE>;
    case T_Q5_K: return gemv_r<T_Q5_K, DUAL, ROLE>;
    case T_Q6_K: return gemv_r<T_Q6_K, DUAL, ROLE>;
    case T_Q8_0: return gemv_r<T_Q8_0, DUAL, ROLE>;
    default: return nullptr;
    }
}
static GemvFn gemv_r_fn(int role, int type, int nslots) {
    if (nslots > 1) return gemv_r_fn_t<1, 2>(type);
    return role == ROLE_FFN_UP ? gemv_r_fn_t<0, 1>(type) : gemv_r_fn_t<0, 0>(type);
}
static GemvMixFn gemv_r_mix_fn(int t1, int t2) {
    if (t1 == T_Q4_K && t2 == T_Q6_K) return gemv_r_mix<T_Q4_K, T_Q6_K>;
    if (t1 == T_Q5_K && t2 == T_Q6_K) return gemv_r_mix<T_Q5_K, T_Q6_K>;
    return nullptr;
}

void init_kernel_attributes() {
    gemm_attrs();
    const int types[4] = {T_Q4_K, T_Q5_K, T_Q6_K, T_Q8_0};
    for (int r : {ROLE_GENERIC, ROLE_FFN_UP})
        for (int t : types)
            for (int nsl = 1; nsl <= 2; ++nsl) {
                for (int c = 0; c < kNumGemvCfgs; ++c)
                    MI_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(gemv_fn(r, t, nsl, c)),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, kGemvDynLds));
                MI_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(gemv_r_fn(r, t, nsl)),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, kGemvDynLds));
            }
    for (int t1 : {T_Q4_K, T_Q5_K}) {
        MI_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(gemv_mix_fn(t1, T_Q6_K)),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, kGemvDynLds));
        MI_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(gemv_r_mix_fn(t1, T_Q6_K)),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, kGemvDynLds));
    }
}

// Units one workgroup owns at most (its residual staging in LDS).
static int wg_units_max(int total_units, int grid) { return (total_units + grid - 1) / grid + 1; }

size_t gemv_smem_bytes(const GemvParams& p) { return (size_t)smem_plan(p).total; }
// the LDS-DMA ring kernel: prologue plan, then the rings
static size_t gemv_r_smem_bytes(const GemvParams& p) {
    return (((size_t)smem_plan(p).total + 15) & ~(size_t)15) + (size_t)ring_bytes(p.seg[0].A.type);
}

static int gemv_waves(int type, int role, int K) {
    if (gemv_k_on(K)) return gemv_k_waves(K);
    return gemv_ring_on() ? RING_NW : kGemvCfgs[gemv_cfg_for(type, role)].nw;
}

int gemv_default_grid(const GemvParams& p, int role) {
    // One workgroup per CU (256 CUs).  Small launches use fewer workgroups so that every
    // wave (of a K group, for gemv_k) still gets a unit.
    int per = gemv_waves(p.seg[0].A.type, role, p.K);
    if (gemv_k_on(p.K)) per /= gemv_k_groups(p.K);
    const int g = (p.total_units + per - 1) / per;
    // at most one workgroup per CU by default; MI_GEMV_GRID raises the cap (A/B)
    static const int cap = getenv("MI_GEMV_GRID") ? std::max(1, atoi(getenv("MI_GEMV_GRID"))) : 256;
    return g < 1 ? 1 : (g > cap ? cap : g);
}

// Validates a launch and fixes its grid-dependent fields; returns the kernel configuration
// (register ring), -1 (LDS-DMA ring) or -2 (K-split).
static int gemv_prepare(GemvParams& p, int role, int grid) {
    if (p.K % 256 != 0) throw Error("gemv: K must be a multiple of 256");
    const int type = p.seg[0].A.type;
    for (int i = 0; i < p.nseg; ++i)
        if (p.seg[i].A.type != type || (p.seg[i].pair == PAIR_AB && p.seg[i].B.type != type))
            throw Error("gemv: all matrices of one launch must share a quant type");
    if (p.pro == PRO_ATTN && (p.attn.n_head * p.attn.head_dim != p.K || p.attn.head_dim % 4 != 0))
        throw Error("gemv: attention combine needs K == n_head*head_dim");
    const bool kk = gemv_k_on(p.K);
    const int cfg = kk ? -2 : gemv_ring_on() ? -1 : gemv_cfg_for(type, role);
    const int nw = gemv_waves(type, role, p.K);
    if (grid <= 0) grid = gemv_default_grid(p, role);
    if ((long long)p.total_units * grid * nw >= (1LL << 32))
        throw Error("gemv: too many units for the 32-bit unit split");
    p.wg_units = wg_units_max(p.total_units, grid);
    p.grid = grid;
    for (int i = 0; i < p.nseg; ++i)
        if (p.seg[i].resid && (p.nseg != 1 || p.wg_units > nw * 64))
            throw Error("gemv: residual launches must have one segment and <= 64*NW units per workgroup");
    const size_t lds = kk ? (size_t)kplan(p).total : cfg < 0 ? gemv_r_smem_bytes(p) : gemv_smem_bytes(p);
    if (lds > (size_t)kGemvDynLds) throw Error("gemv: activation too large for LDS");
    return cfg;
}

// leading arguments: K | flags (activation kept in registers, RMSNorm prologue)
static int gemv_kflags(const GemvParams& p, int nw) {
    const int nb = p.K / 256;
    const bool regs = p.pro != PRO_ATTN && p.nslots == 1 && nb <= PRO_MAXB * nw;
    const bool rms = p.pro == PRO_RMSNORM;
    return p.K | (regs ? 1 << 20 : 0) | (rms ? 1 << 21 : 0);
}

// gemv_k's leading arguments: K | RMSNorm (bit 21) | attention combine (bit 22); kx0 is the
// activation, or split 0 of the attention partials
static int gemv_k_kflags(const GemvParams& p) {
    return p.K | (p.pro == PRO_RMSNORM ? 1 << 21 : 0) | (p.pro == PRO_ATTN ? 1 << 22 : 0);
}
static const float* gemv_k_x0(const GemvParams& p) { return p.pro == PRO_ATTN ? p.attn.o : p.x[0]; }

void launch_gemv(const GemvParams& p_in, int role, int grid, hipStream_t s, hipEvent_t ev_start,
                 hipEvent_t ev_stop) {
    GemvParams p = p_in;
    const int cfg = gemv_prepare(p, role, grid);
    const int type = p.seg[0].A.type;
    GemvFn fn;
    size_t smem;
    int nw, kflags;
    const float* kx0 = p.x[0];
    if (cfg == -2) {
        fn = gemv_k_fn(role, type, p.nslots);
        smem = (size_t)kplan(p).total + 16 * sizeof(double);
        nw = gemv_k_waves(p.K);
        kflags = gemv_k_kflags(p);
        kx0 = gemv_k_x0(p);
    } else {
        const bool ring = cfg < 0;
        smem = ring ? gemv_r_smem_bytes(p) : gemv_smem_bytes(p);
        fn = ring ? gemv_r_fn(role, type, p.nslots) : gemv_fn(role, type, p.nslots, cfg);
        nw = ring ? RING_NW : kGemvCfgs[cfg].nw;
        kflags = gemv_kflags(p, nw);
    }
    if (!fn) throw Error("gemv: unsupported quant type");
    const dim3 block(nw * 64);
    const float* knw = p.pro == PRO_RMSNORM ? p.norm_w : nullptr;
    const int* ktp = p.tokpos;
    if (ev_start || ev_stop)
        hipExtLaunchKernelGGL(fn, dim3(p.grid), block, smem, s, ev_start, ev_stop, 0, kx0, knw, ktp, kflags, p);
    else
        hipLaunchKernelGGL(fn, dim3(p.grid), block, smem, s, kx0, knw, ktp, kflags, p);
    MI_HIP(hipGetLastError());
}

// Config 1 (8 waves, 4-deep ring) is the QKV role's; the pairs are the Q*_K_M layer mixes.
static GemvMixFn gemv_mix_fn(int t1, int t2) {
    if (t1 == T_Q4_K && t2 == T_Q6_K) return gemv_mix_t<T_Q4_K, T_Q6_K, 4, 8>;
    if (t1 == T_Q5_K && t2 == T_Q6_K) return gemv_mix_t<T_Q5_K, T_Q6_K, 4, 8>;
    return nullptr;
}

bool gemv_mix_supported(int t1, int t2, int role) {
    if (gemv_impl() == GEMV_KSPLIT) return gemv_k_mix_fn(t1, t2) != nullptr;
    if (gemv_ring_on()) return gemv_r_mix_fn(t1, t2) != nullptr;
    return gemv_mix_fn(t1, t2) != nullptr && gemv_cfg_for(t1, role) == 1 && gemv_cfg_for(t2, role) == 1;
}

void launch_gemv_mix(const GemvParams& p1_in, const GemvParams& p2_in, int role, hipStream_t s) {
    GemvParams p1 = p1_in, p2 = p2_in;
    const int t1 = p1.seg[0].A.type, t2 = p2.seg[0].A.type;
    const bool ring = gemv_ring_on();
    const bool kk = gemv_k_on(p1.K);
    GemvMixFn fn = kk ? gemv_k_mix_fn(t1, t2) : ring ? gemv_r_mix_fn(t1, t2) : gemv_mix_fn(t1, t2);
    if (!fn || !gemv_mix_supported(t1, t2, role)) throw Error("gemv: unsupported type pair for a mixed launch");
    if (p1.K != p2.K || p1.pro != p2.pro || p1.x[0] != p2.x[0] || p1.norm_w != p2.norm_w || p1.tokpos != p2.tokpos ||
        p1.nslots != 1 || p2.nslots != 1)
        throw Error("gemv: the halves of a mixed launch must share their activation");
    // split the 256 workgroups in proportion to the bytes each half streams
    auto bytes = [](const GemvParams& p) {
        double b = 0;
        for (int i = 0; i < p.nseg; ++i) b += (double)p.seg[i].A.rows * (p.K / block_elems(p.seg[i].A.type)) * block_bytes(p.seg[i].A.type);
        return b;
    };
    const int total = gemv_default_grid(p1, role) + gemv_default_grid(p2, role) >= 256 ? 256 : 128;
    const double b1 = bytes(p1), b2 = bytes(p2);
    int g1 = (int)(total * b1 / (b1 + b2) + 0.5);
    g1 = std::max(1, std::min(total - 1, std::min(g1, gemv_default_grid(p1, role))));
    const int g2 = std::min(total - g1, gemv_default_grid(p2, role));
    const int cfg = gemv_prepare(p1, role, g1);
    gemv_prepare(p2, role, g2);
    size_t smem;
    int nw, kflags;
    const float* kx0 = p1.x[0];
    if (kk) {
        smem = (size_t)std::max(kplan(p1).total, kplan(p2).total) + 16 * sizeof(double);
        nw = gemv_k_waves(p1.K);
        kflags = gemv_k_kflags(p1);
        kx0 = gemv_k_x0(p1);
    } else {
        smem = ring ? std::max(gemv_r_smem_bytes(p1), gemv_r_smem_bytes(p2))
                    : std::max(gemv_smem_bytes(p1), gemv_smem_bytes(p2));
        nw = ring ? RING_NW : kGemvCfgs[cfg].nw;
        kflags = gemv_kflags(p1, nw);
    }
    const dim3 block(nw * 64);
    const float* knw = p1.pro == PRO_RMSNORM ? p1.norm_w : nullptr;
    hipLaunchKernelGGL(fn, dim3(p1.grid + p2.grid), block, smem, s, kx0, knw, p1.tokpos, kflags, p1, p2);
    MI_HIP(hipGetLastError());
}

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
static void gemm_attrs() {
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

__global__ void embed_kernel(const EmbedParams P) {
    const long long tok = P.tokpos[0];
    for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < P.n_embd; c += gridDim.x * blockDim.x)
        P.out[c] = dequant_elem(P.E, tok, c);
}

__global__ void embed_multi_kernel(const EmbedParams P) {
    const long long tok = P.tokpos[blockIdx.y * 4];
    float* out = P.out + (long long)blockIdx.y * P.n_embd;
    for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < P.n_embd; c += gridDim.x * blockDim.x)
        out[c] = dequant_elem(P.E, tok, c);
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
template <int R, int LPC>
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
    const long long row_off = (long long)g * HD + L * 8;
    constexpr int U = 4;   // steps whose K loads are issued together
    for (int cb = c0 + wave * CPW; cb < c1; cb += 4 * CPW * U) {
        u32x4 kk[U];
        int cpos[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int c = cb + u * 4 * CPW + G;
            c = c < c1 ? c : c1 - 1;
            kk[u] = *reinterpret_cast<const u32x4*>(P.kcache + (long long)c * P.kv_dim + row_off);
            cpos[u] = P.cell_pos[c];
        }
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

template <int R, int LPC>
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
    constexpr int U = 4;
    for (int cb = c0 + wave * CPW; cb < c1; cb += 4 * CPW * U) {
        u32x4 vv[U];
        float pw[U][R];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int c = cb + u * 4 * CPW + G;
            const bool in = c < c1;
            c = in ? c : c1 - 1;
            vv[u] = *reinterpret_cast<const u32x4*>(P.vcache + (long long)c * P.kv_dim + row_off);
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

// Short contexts (<= ATTN_SHORT cells): the same arithmetic as the two kernels above with a
// single split, in one launch.  One workgroup per kv head keeps its scores in LDS, so no
// other workgroup's result is needed between the softmax statistics and the PV sum.
template <int R, int LPC>
__global__ __launch_bounds__(256) void attn_fused_kernel(const AttnParams P) {
    constexpr int CPW = 64 / LPC;
    constexpr int HD = LPC * 8;
    __shared__ float sw[R][ATTN_SHORT];
    __shared__ float redm[4][R];
    __shared__ double dred[4][R];
    __shared__ float gm[R], ginv[R];
    __shared__ float red_o[4][R][HD];
    // kv head, and the first of the R q heads this workgroup serves (qsplit: one q head each)
    const int g = P.qsplit ? (int)blockIdx.x / P.qsplit : (int)blockIdx.x;
    const int gq = P.qsplit ? (int)blockIdx.x : (int)blockIdx.x * R;
    const int tok = blockIdx.y;   // query token (launch_attn_multi); 0 for a decode step
#ifdef MI_STAMPS
    unsigned long long* const stp = P.stamps && tok == 0 ? P.stamps + blockIdx.x * 8 : nullptr;
    if (stp && threadIdx.x == 0) stp[0] = __builtin_amdgcn_s_memrealtime();
#endif
    const int* tp = P.tokpos + 4 * tok;
    const int tp2 = tp[2], qpos = tp[1];
    const float* qrow = P.q + (long long)tok * P.n_head * HD;
    float* orow = P.part_o + (long long)tok * P.n_head * HD;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int L = lane % LPC, G = lane / LPC;
    const long long row_off = (long long)g * HD + L * 8;
    constexpr int U = 4;
    // The first chunk of K, V and cell positions is fetched at entry, before the cell count
    // arrives, so the token-position, K and V round trips overlap instead of chaining.  Cells
    // past the count are clamped to the cache and masked by select below, never by arithmetic.
    u32x4 k0[U], v0[U];
    int cp0[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int c = min(wave * CPW + u * 4 * CPW + G, P.n_ctx - 1);
        k0[u] = *reinterpret_cast<const u32x4*>(P.kcache + (long long)c * P.kv_dim + row_off);
        v0[u] = *reinterpret_cast<const u32x4*>(P.vcache + (long long)c * P.kv_dim + row_off);
        cp0[u] = P.cell_pos[c];
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
                if (L == 0 && c < ncell) sw[t][c] = w;
            }
        }
    }
#pragma unroll
    for (int t = 0; t < R; ++t) {
        const float m = wave_max(mx[t]);
        if (lane == 0) redm[wave][t] = m;
    }
    __syncthreads();
    // 2. sum over all cells of expf(w - max), in double, fixed order (as attn_pv_kernel)
#pragma unroll
    for (int t = 0; t < R; ++t) {
        const float M = fmaxf(fmaxf(redm[0][t], redm[1][t]), fmaxf(redm[2][t], redm[3][t]));
        double acc = 0.0;
        for (int c = tid; c < ncell; c += 256) acc += (double)expf(sw[t][c] - M);
        acc = wave_sum_d(acc);
        if (lane == 0) dred[wave][t] = acc;
        if (tid == 0) gm[t] = M;
    }
    __syncthreads();
    if (tid < R) ginv[tid] = (float)(1.0 / (((dred[0][tid] + dred[1][tid]) + dred[2][tid]) + dred[3][tid]));
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
        const bool first = cb == wave * CPW;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int c = cb + u * 4 * CPW + G;
            const bool in = c < ncell;
            c = in ? c : ncell - 1;
            if (first) {   // prefetched at entry; a cell past the count may hold non-finite bits
                const u32x4 z = {0u, 0u, 0u, 0u};
                vv[u] = in ? v0[u] : z;
            } else {
                vv[u] = *reinterpret_cast<const u32x4*>(P.vcache + (long long)c * P.kv_dim + row_off);
            }
#pragma unroll
            for (int t = 0; t < R; ++t) {
                const float p = expf(sw[t][c] - gm[t]) * ginv[t];
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
            for (int e = 0; e < 8; ++e) red_o[wave][t][L * 8 + e] = o[t][e];
    }
    __syncthreads();
    for (int i = tid; i < R * HD; i += 256) {
        const int t = i / HD, d = i % HD;
        orow[(long long)(gq + t) * HD + d] = ((red_o[0][t][d] + red_o[1][t][d]) + red_o[2][t][d]) + red_o[3][t][d];
    }
#ifdef MI_STAMPS
    if (stp && threadIdx.x == 0) stp[4] = __builtin_amdgcn_s_memrealtime();
#endif
}

typedef void (*AttnFn)(const AttnParams);
template <int R>
static void attn_fns_r(int hd, AttnFn& a, AttnFn& b, AttnFn& f) {
    switch (hd) {
    case 32: a = attn_scores_kernel<R, 4>; b = attn_pv_kernel<R, 4>; f = attn_fused_kernel<R, 4>; break;
    case 64: a = attn_scores_kernel<R, 8>; b = attn_pv_kernel<R, 8>; f = attn_fused_kernel<R, 8>; break;
    case 128: a = attn_scores_kernel<R, 16>; b = attn_pv_kernel<R, 16>; f = attn_fused_kernel<R, 16>; break;
    case 256: a = attn_scores_kernel<R, 32>; b = attn_pv_kernel<R, 32>; f = attn_fused_kernel<R, 32>; break;
    default: a = b = f = nullptr; break;
    }
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
