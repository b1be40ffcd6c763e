// Device helpers shared by the decode GEMV (gemv.hip), the batch GEMMs and the other kernels:
// typed global pointers, DPP wave reductions, the ggml activation quantisers and the per-type
// superblock dot products (Kq<T>), which reproduce ggml b5187's vec_dot_q*_K_q8_K /
// vec_dot_q8_0_q8_0 integer arithmetic bit for bit.
#pragma once
#include "kernels.h"
#include <hip/hip_runtime.h>

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
// Buffer loads of a wave-uniform base (SGPR descriptor) with the cache policy nt.  An offset at or
// past GV_OOB is out of the descriptor's range: the load returns zeros without a memory access
// (the decode GEMV's ring issues such loads once a wave's items run out, so it never waits for a
// real round trip it does not need).
constexpr unsigned BUF_OOB = 0xFFFFFF00u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const uint8_t* base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base), 0, 0x7FFFFFFF, 0x00020000);
}
__device__ __forceinline__ u32x4 bld16(const uint8_t* base, unsigned off) {
    return __builtin_amdgcn_raw_buffer_load_b128(buf_rsrc(base), off, 0, 2);
}
__device__ __forceinline__ unsigned bld8x(const uint8_t* base, unsigned off, unsigned& hi) {
    typedef unsigned int u32x2_ __attribute__((ext_vector_type(2)));
    const u32x2_ v = __builtin_amdgcn_raw_buffer_load_b64(buf_rsrc(base), off, 0, 2);
    hi = v.y;
    return v.x;
}
__device__ __forceinline__ unsigned bld2(const uint8_t* base, unsigned off) {
    return __builtin_amdgcn_raw_buffer_load_b16(buf_rsrc(base), off, 0, 2);
}
__device__ __forceinline__ unsigned oob(unsigned off, bool park) { return park ? BUF_OOB : off; }
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
    // branch-free (selects only), so that the blocks a wave quantises back to back form one
    // basic block whose dependent chains (DPP max, division) the scheduler can interleave
    const float a0 = fabsf(v[0]), a1 = fabsf(v[1]), a2 = fabsf(v[2]), a3 = fabsf(v[3]);
    const float amax = wave_max_pos(fmaxf(fmaxf(a0, a1), fmaxf(a2, a3)));
    // the signed value at the FIRST index whose |x| is the maximum (amax == 0: every lane's
    // first element, unused)
    const int e = a0 == amax ? 0 : a1 == amax ? 1 : a2 == amax ? 2 : a3 == amax ? 3 : 4;
    const float mine = e == 0 ? v[0] : e == 1 ? v[1] : e == 2 ? v[2] : v[3];
    const unsigned long long m = __ballot(e < 4);
    const int src = __builtin_ctzll(m | (1ull << 63));
    const float mx = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(mine), src));
    const bool zero = amax == 0.0f;
    const float iscale = -127.0f / mx;
    int q[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) q[k] = zero ? 0 : min(127, (int)rintf(iscale * v[k]));
    const float d = zero ? 0.0f : 1.0f / iscale;
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
    // buffer-load form (decode GEMV ring): park = the wave has no item left (zeros, no access)
    __device__ static Ld bload(const uint8_t* const* rp, int sb, int j, bool park) {
        Ld l;
        l.qs = bld16(rp[0], oob(sb * 128 + j * 16, park));
        l.hdr = bld16(rp[1], oob(sb * 16, park));
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
        return finish(l.hdr, ScaleSel(j), dlo, dhi, r);
    }
    // get_scale_min_k4 for the lane's sub-blocks 2g, 2g+1 (g = j >> 1) without a lane-dependent
    // branch: bytes 2(g&1), 2(g&1)+1 of each header dword, then per-lane masks pick the g < 2
    // form (6 low bits of scales[is] / scales[is+4]) or the g >= 2 form (4 bits of scales[is+4]
    // | the top 2 bits of scales[is-4] / scales[is] << 4).  The masks depend on the lane only.
    struct ScaleSel {
        unsigned sh, lo6, lo4, hi2;
        __device__ explicit ScaleSel(int j) {
            const int g = j >> 1;
            sh = (unsigned)(g & 1) * 16;
            lo6 = g < 2 ? 0x3F3Fu : 0u;
            lo4 = g < 2 ? 0u : 0x0F0Fu;
            hi2 = g < 2 ? 0u : 0x3030u;
        }
    };
    // d * sum(sc * q.a) - dmin * sum(m * bsum), the scale products in 24-bit multiplies
    // (|dlo|, |dhi| <= 32*31*127, scales and mins 6-bit, |bsum| <= 16*127: exact)
    __device__ static float finish(const u32x4& hdr, const ScaleSel& q, int dlo, int dhi, const AR& r) {
        const unsigned Y = hdr.y >> q.sh, Z = hdr.z >> q.sh, W = hdr.w >> q.sh;
        const unsigned SC = (Y & q.lo6) | (W & q.lo4) | ((Y >> 2) & q.hi2);
        const unsigned MM = (Z & q.lo6) | ((W >> 4) & q.lo4) | ((Z >> 2) & q.hi2);
        const int S = __mul24((int)(SC & 0xFF), dlo) + __mul24((int)((SC >> 8) & 0xFF), dhi);
        const int M = __mul24((int)(MM & 0xFF), r.bs_lo) + __mul24((int)((MM >> 8) & 0xFF), r.bs_hi);
        const float d = h2f(hdr.x) * r.dx;
        const float dm = h2f(hdr.x >> 16) * r.dx;
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
    __device__ static Ld bload(const uint8_t* const* rp, int sb, int j, bool park) {
        Ld l;
        l.qs = bld16(rp[0], oob(sb * 128 + j * 16, park));
        l.qh = bld16(rp[1], oob(sb * 32 + (j & 1) * 16, park));
        l.hdr = bld16(rp[2], oob(sb * 16, park));
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
        return Kq<T_Q4_K>::finish(l.hdr, Kq<T_Q4_K>::ScaleSel(j), dlo, dhi, r);
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
    __device__ static Ld bload(const uint8_t* const* rp, int sb, int j, bool park) {
        Ld l;
        const int h = j >> 2, half = j & 1;
        l.ql = bld16(rp[0], oob(sb * 128 + j * 16, park));
        l.qh = bld16(rp[1], oob(sb * 64 + 32 * h + 16 * half, park));
        l.sc0 = bld8x(rp[2], oob(sb * 16 + 8 * h, park), l.sc1);
        l.d = bld2(rp[3], oob(sb * 2, park));
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
    __device__ static Ld bload(const uint8_t* const* rp, int sb, int j, bool park) {
        Ld l;
        l.q0 = bld16(rp[0], oob(sb * 256 + j * 32, park));
        l.q1 = bld16(rp[0], oob(sb * 256 + j * 32 + 16, park));
        l.d = bld2(rp[1], oob(sb * 16 + j * 2, park));
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

__device__ __forceinline__ float silu_f(float x) { return x / (1.0f + expf(-x)); }

// every storing wave, before its workgroup signals a hand-off (invisible to the compiler's waits)
__device__ __forceinline__ void drain_vm() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// ---------------------------------------------------------------------------
// Block b of a published activation (ActOut, kernels.h) from one wave's 4 values per lane
// ---------------------------------------------------------------------------
__device__ __forceinline__ void dv_quant_block(const ActOut& t, int b, const float v[4], int lane) {
    const ActLayout L = act_layout(t.K, t.q8k, t.q80);
    if (t.q8k)
        quant_q8k_block(v, lane, reinterpret_cast<int8_t*>(t.act + L.q8k + b * 256),
                        reinterpret_cast<int*>(t.act + L.bsum) + b * 16, reinterpret_cast<float*>(t.act + L.dk) + b);
    if (t.q80)
        quant_q80_block(v, lane, reinterpret_cast<int8_t*>(t.act + L.q80 + b * 256),
                        reinterpret_cast<float*>(t.act + L.d0) + b * 8);
}

// Block blk (256 elements, 4 per lane: elements 4 lane..) of token row t of a physical batch's
// activation, quantised as quantize_row_q8_K_ref (a.q80 = 0) or the x86 quantize_row_q8_0 (a.q80
// = 1) and stored in the batch GEMMs' format (ActQ8: MFMA A fragments, token-minor d, byte-split
// 32-element bsums) -- the arithmetic and layout of quant_act_kernel, shared with the attention
// kernel that quantises a short batch's output itself.
__device__ __forceinline__ void quant_actq8_block(const ActQ8& a, int t, int blk, const float v[4], int lane) {
    const int nb = a.K >> 8;
    const int tile = t >> 5, tr = t & 31;
    const int fj = lane >> 3, fh = (lane >> 2) & 1, fw = lane & 3;
    int8_t* q = a.q + (long long)tile * nb * 8192 + fj * 1024 + (fh * 32 + tr) * 16 + 4 * fw + (long long)blk * 8192;
    if (a.q80) {
        float am = fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3])));
        am = fmaxf(am, __int_as_float(dpp_i<0xB1, 0xf>(__float_as_int(am))));
        am = fmaxf(am, __int_as_float(dpp_i<0x4E, 0xf>(__float_as_int(am))));
        am = fmaxf(am, __int_as_float(dpp_i<0x141, 0xf>(__float_as_int(am))));   // row_half_mirror
        const float d0 = am / 127.0f;
        const float id = am != 0.0f ? 127.0f / am : 0.0f;
        int qz[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) qz[k] = (int)rintf(v[k] * id);
        *reinterpret_cast<int*>(q) = (qz[0] & 0xFF) | ((qz[1] & 0xFF) << 8) | ((qz[2] & 0xFF) << 16) | ((qz[3] & 0xFF) << 24);
        if ((lane & 7) == 0) a.dT[(long long)(blk * 8 + (lane >> 3)) * a.npad + t] = __half2float(__float2half_rn(d0));
        return;
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
    *reinterpret_cast<int*>(q) = (qv[0] & 0xFF) | ((qv[1] & 0xFF) << 8) | ((qv[2] & 0xFF) << 16) | ((qv[3] & 0xFF) << 24);
    // the 32-element sub-block sums: lanes 8j..8j+7
    int sm = (qv[0] + qv[1]) + (qv[2] + qv[3]);
    sm += dpp_i<0xB1, 0xf>(sm);    // quad_perm [1,0,3,2]
    sm += dpp_i<0x4E, 0xf>(sm);    // quad_perm [2,3,0,1]
    sm += __shfl_xor(sm, 4, 64);   // the two quads of a sub-block
    if ((lane & 7) == 0) {
        int8_t* bsb = a.bsb + ((long long)tile * nb * 32 + tr) * 16 + (long long)blk * 512;
        const int j = lane >> 3;
        bsb[j] = (int8_t)(sm >> 6);          // floor(b/64), -64..63
        bsb[8 + j] = (int8_t)(sm & 63);      // b - 64*floor(b/64), 0..63
    }
    if (lane == 0) a.dT[(long long)blk * a.npad + t] = d;
}

__device__ __forceinline__ void unit_range(int total, int W, int gw, int& u0, int& u1) {
    // total * (gw + 1) < 2^32 (total <= 65536 units, W <= 4096 waves)
    u0 = (int)(((unsigned)total * (unsigned)gw) / (unsigned)W);
    u1 = (int)(((unsigned)total * (unsigned)(gw + 1)) / (unsigned)W);
}

}  // namespace mi
