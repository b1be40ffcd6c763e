// Batch-1 decode GEMV for gfx950 (CDNA4, wave64): ggml_mul_mat of one token against a
// Q4_K / Q5_K / Q6_K / Q8_0 matrix, fused with its neighbours in
// llm_build_llama: the RMSNorm or attention-combine prologue, the Q8_K / Q8_0 activation
// quantisation of the CPU path, and the RoPE / KV-append / residual / SwiGLU / MoE epilogues.
//
// Numerics: every per-block integer dot is ggml b5187's vec_dot_q*_K_q8_K / vec_dot_q8_0_q8_0
// bit for bit (qdot.h); only the fp32 sum order across superblocks differs from the CPU's.
//
// Structure (measured, scripts/exp_gemv2.cpp, in-kernel stamps):
//  * A workgroup of GV_NW waves serves one segment.  A wave walks "items" -- one 8-superblock
//    chunk of the RW rows of one unit -- through a D-deep register ring: one aligned 16-byte load
//    per lane of the main quant plane (+ side planes), the next items in flight while one is
//    reduced against the activation in LDS.
//  * Request order (GvArgs::order).  Order 0: each wave issues its activation slices, then its
//    weight ring at once (no workgroup barrier: the barrier waited for the workgroup's last wave
//    to start), then builds its share of the activation.  Order 4: waves [0, npro) stage the
//    activation by LDS-DMA and build it while the other waves issue their rings; a wave that has
//    issued its ring runs its later instructions only as fast as the CU's memory pipeline drains
//    (back-pressure), so the prologue is kept off those waves.  Orders 1 and 2 (barrier / wait for
//    the own slice first) are A/B knobs.
//  * The ~0.5 KB parameter block is read with one vector load per lane and spread to scalars by
//    v_readlane; a workgroup's segment is a compile-time index (no dependent kernarg reads).
#include "qdot.h"
#include <hip/hip_ext.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace mi {

namespace {

constexpr int GV_NW = 16;       // waves per workgroup (one workgroup per CU)
constexpr int GV_ASTR = 272;    // LDS bytes per activation block: 256 int8 + 16 (b128 reads spread over banks)
constexpr int GV_KMAX = 14336;  // largest activation (Llama-3 / Mixtral n_ff)

struct GvSeg {
    const uint8_t* a[4];        // planes of A (expert 0, row 0)
    const uint8_t* b[4];        // PAIR_AB: planes of B
    float* out;
    const float* resid;
    const float* bias;          // optional per-row bias (GPT-2 projections)
    int units, blk0, nblk, rows;
    int epi, nq, nk, expA, expB, actB;
};

struct GvArgs {
    GvSeg seg[2];
    const float* x[2];
    const float* norm_w;
    const float* norm_b;        // PRO_LAYERNORM
    const unsigned short* gelu_tab;   // EPI_GELU: ggml_table_gelu_f16
    const float* attn_o;        // PRO_ATTN: split partials [split][attn_stride]
    const int* tokpos;
    int* cell_pos;
    __half* kcache;
    __half* vcache;
    const float* freq_factors;
    const int* sel;
    const float* selw;
    float eps, theta_scale, freq_scale;
    int K, pro, nslots, attn_nsplit, attn_stride, n_rot, head_dim, kv_dim;
    int order;                    // 0: weights right after the activation requests; 1: after a
                                  // workgroup barrier; 2: after this wave's activation landed;
                                  // 4: waves [0, npro) build the activation (staged by LDS-DMA)
                                  // while the others stream, then stream themselves
    int npro;                     // order 4: prologue waves
    int stage_off;                // order 4: LDS byte offset of the staged activation arrays
    int flag_off;                 // order 4: LDS byte offset of the [2][GV_NW] flag words
    int pre;                      // ring items issued before the prologue (the rest after it)
    unsigned long long* stamps;   // MI_STAMPS builds: [grid][8] s_memrealtime per workgroup
};

// LDS layout of one activation slot: Q8_K blocks [nb][GV_ASTR] | bsums [nb][16] int | d [nb]
// (padded to 16 B) | Q8_0 blocks [nb][GV_ASTR] | Q8_0 d [nb][8].  Then the RoPE table and the
// RMSNorm shares.
struct GvLds {
    int q8k, bsum, dk, q80, d0, slot;
};
__host__ __device__ inline GvLds gv_lds(int nb) {
    GvLds L;
    int o = 0;
    L.q8k = o; o += nb * GV_ASTR;
    L.bsum = o; o += nb * 64;
    L.dk = o; o += (nb * 4 + 15) & ~15;
    L.q80 = o; o += nb * GV_ASTR;
    L.d0 = o; o += nb * 32;
    L.slot = o;
    return L;
}
__host__ __device__ inline int gv_rope_off(int nb, int nslots) { return gv_lds(nb).slot * nslots; }
__host__ __device__ inline int gv_red_off(int nb, int nslots, int n_rot) {
    return gv_rope_off(nb, nslots) + (((n_rot / 2) * 8 + 15) & ~15);
}
__host__ inline size_t gv_lds_bytes(int nb, int nslots, int n_rot) {
    return (size_t)gv_red_off(nb, nslots, n_rot) + 2 * GV_NW * 8;   // two rounds of per-wave doubles
}
// order 4: the fp32 arrays the prologue waves stage (x, then the norm weight or the second
// slot), 1 KiB per 256-block each, after the rest; then the flag words
constexpr size_t GV_LDS_MAX = 160 * 1024;
__host__ inline int gv_stage_arrays(int pro, int nslots) {
    return 1 + ((pro == PRO_RMSNORM || nslots > 1) ? 1 : 0);
}

__device__ __forceinline__ int readfirstlane_i(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_s_waitcnt((0xF) | (0x3 << 14) | (0x7 << 4));   // lgkmcnt(0): LDS writes done; vmcnt untouched
    __builtin_amdgcn_s_barrier();
}

// The activation registers Kq<T>::dot needs for lane j of superblock sb, from the LDS slot.
template <int T> struct GvAct;
template <> struct GvAct<T_Q4_K> {
    __device__ static Kq<T_Q4_K>::AR get(const char* s, const GvLds& L, int sb, int j) {
        const int g = j >> 1, half = j & 1;
        const char* ab = s + L.q8k + sb * GV_ASTR + 64 * g + 16 * half;
        Kq<T_Q4_K>::AR r;
        r.alo = *reinterpret_cast<const i32x4*>(ab);
        r.ahi = *reinterpret_cast<const i32x4*>(ab + 32);
        const int* bs = reinterpret_cast<const int*>(s + L.bsum) + sb * 16 + 4 * g + half;
        r.bs_lo = bs[0];
        r.bs_hi = bs[2];
        r.dx = reinterpret_cast<const float*>(s + L.dk)[sb];
        return r;
    }
};
template <> struct GvAct<T_Q5_K> {
    __device__ static Kq<T_Q5_K>::AR get(const char* s, const GvLds& L, int sb, int j) {
        return GvAct<T_Q4_K>::get(s, L, sb, j);
    }
};
template <> struct GvAct<T_Q6_K> {
    __device__ static Kq<T_Q6_K>::AR get(const char* s, const GvLds& L, int sb, int j) {
        const int h = j >> 2, hq = (j >> 1) & 1, half = j & 1;
        const char* ab = s + L.q8k + sb * GV_ASTR + 128 * h + 32 * hq + 16 * half;
        Kq<T_Q6_K>::AR r;
        r.alo = *reinterpret_cast<const i32x4*>(ab);
        r.ahi = *reinterpret_cast<const i32x4*>(ab + 64);
        const int* bs = reinterpret_cast<const int*>(s + L.bsum) + sb * 16 + 8 * h + 2 * hq + half;
        r.bs_lo = bs[0];
        r.bs_hi = bs[4];
        r.dx = reinterpret_cast<const float*>(s + L.dk)[sb];
        return r;
    }
};
template <> struct GvAct<T_Q8_0> {
    __device__ static Kq<T_Q8_0>::AR get(const char* s, const GvLds& L, int sb, int j) {
        const char* ab = s + L.q80 + sb * GV_ASTR + 32 * j;
        Kq<T_Q8_0>::AR r;
        r.a0 = *reinterpret_cast<const i32x4*>(ab);
        r.a1 = *reinterpret_cast<const i32x4*>(ab + 16);
        r.d0 = reinterpret_cast<const float*>(s + L.d0)[sb * 8 + j];
        return r;
    }
};

// Which activation formats a workgroup of segment types (T0, T1) must build.
template <int T> __host__ __device__ constexpr bool gv_q80() { return T == T_Q8_0; }

// Loads of one ring item row (Kq<T>::bload): the persistent prefill waits for everything but
// these (vmcnt counts loads and stores in issue order).
template <int T> __host__ __device__ constexpr int gv_nl() {
    return T == T_Q4_K ? 2 : T == T_Q5_K ? 3 : T == T_Q6_K ? 4 : 3;
}
template <int N> __device__ __forceinline__ void wait_vm() {   // s_waitcnt vmcnt(N) only
    static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}
// Persistent kernel: item-rows of the next stage each wave pulls into L2 ahead of its ring while
// the grid barrier completes, and the dword loads that takes (one per 128-byte line and lane).
constexpr int GV_TOUCH = 6;
template <int T, int RW> __host__ __device__ constexpr int gv_touch_n() {
    int n = 0;
    for (int p = 0; p < 4; ++p) {
        const int b = p == 0 ? PlaneBytes<T>::b[0] : p == 1 ? PlaneBytes<T>::b[1] : p == 2 ? PlaneBytes<T>::b[2] : PlaneBytes<T>::b[3];
        if (b == 0) continue;
        const int lines = (8 * b + 127) / 128;
        n += RW * ((GV_TOUCH / RW * lines + 63) / 64);
    }
    return n;
}
struct GvNoWait {
    __device__ bool operator()() const { return true; }
    __device__ void mark() const {}   // the prologue is done (persistent diagnostics)
};
// Output stores: plain, or (persistent kernel) agent-scope write-through so that the workgroups of
// the other XCDs read them after the grid barrier
template <bool P> __device__ __forceinline__ void gst(float* p, float v) {
    if (P) __hip_atomic_store(gptr_w(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *gptr_w(p) = v;
}
template <bool P> __device__ __forceinline__ void gst(unsigned short* p, unsigned short v) {
    if (P) __hip_atomic_store(gptr_w(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *gptr_w(p) = v;
}
template <bool P> __device__ __forceinline__ void gst(int* p, int v) {
    if (P) __hip_atomic_store(gptr_w(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *gptr_w(p) = v;
}

// ---------------------------------------------------------------------------------------------
// One workgroup's work for segment SI of type T.
//   RW  rows per unit: 2 (PAIR_AB pairs, RoPE pairs of EPI_QKV) or 1
//   KB  activation blocks of 256 per wave held in registers by the prologue: ceil(nb / GV_NW)
//   D   register ring depth (items in flight per wave)
// ---------------------------------------------------------------------------------------------
//   GX  the GPT-2 extensions (LayerNorm prologue, bias and GELU epilogues) are compiled in
//   P   persistent step kernel (decode_step_kernel): the ring prefill is issued before `wait`
//       (the grid barrier that publishes the previous stage's outputs), the activation and the
//       residuals are loaded after it, and every output is stored write-through (agent scope)
//   ND  the launch has one activation slot (the FFN gate/up launch): no second-slot paths
template <int T, int SI, int RW, int KB, int D, bool GX, bool P = false, typename Wait = GvNoWait, bool ND = false>
__device__ __forceinline__ void gv_body(const GvArgs& a, char* lds, Wait&& wait = Wait()) {
    using K = Kq<T>;
    constexpr bool Q80 = gv_q80<T>();
    const GvSeg& S = a.seg[SI];
    // persistent kernel: the lane index is opaque per stage, so that the compiler does not hoist
    // every variant's lane-derived addresses out of the stage loop (and spill them)
    int tid_ = threadIdx.x;
    if (P) asm volatile("" : "+v"(tid_));
    const int lane = tid_ & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid_ >> 6);
    const int sbl = lane >> 3, j = lane & 7;
    const int nb = a.K >> 8;
    const int C = (nb + 7) >> 3;                       // 8-superblock chunks per row
    const int pro = a.pro;
    const int epi = S.epi;
    const bool dual = !ND && a.nslots > 1;
    const GvLds L = gv_lds(nb);
    const int slot_bytes = L.slot;
#ifdef MI_STAMPS   // diagnostic build only (scripts/timeline.py): 0 entry, 1 prefill issued,
                   // 2 activation in LDS, 3 first item consumed, 4 end
#define GV_STAMP(k) \
    if (a.stamps && threadIdx.x == 0) a.stamps[blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memrealtime();
    // order 4: the stamps of the last wave (a streaming wave) instead of wave 0's
#define GV_STAMPL(k) \
    if (a.stamps && threadIdx.x == 64 * (GV_NW - 1)) a.stamps[blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memrealtime();
#else
#define GV_STAMP(k)
#define GV_STAMPL(k)
#endif
    GV_STAMP(0)
#ifdef MI_STAMPS   // 6: the workgroup's last wave to start
    if (a.stamps && lane == 0) atomicMax(a.stamps + blockIdx.x * 8 + 6, (unsigned long long)__builtin_amdgcn_s_memrealtime());
#endif

    // ---- 1. MoE routing: the router's choice decides the weight addresses ----------------------
    int e0 = 0, e1 = 0;
    float w0 = 0.0f, w1 = 0.0f;
    const bool moe = S.expA >= 0 || S.expB >= 0;
    if (moe) {
        e0 = __builtin_amdgcn_readfirstlane(gptr(a.sel)[0]);
        e1 = __builtin_amdgcn_readfirstlane(gptr(a.sel)[1]);
        w0 = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(gptr(a.selw)[0])));
        w1 = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(gptr(a.selw)[1])));
    }

    // ---- 2. the weight ring: item = (unit, chunk) of this wave's units -------------------------
    // units are dealt wave-major over the segment's workgroups (unit u -> workgroup u % nblk), so
    // every workgroup -- every CU's share of the stream -- gets the same number of units +-1
    const int wg = (int)blockIdx.x - S.blk0;
    const int stride = S.nblk * GV_NW;                 // units between a wave's consecutive units
    const int u_first = wave * S.nblk + wg;
    const int n_units = u_first < S.units ? (S.units - u_first + stride - 1) / stride : 0;
    const int n_items = n_units * C;
    const bool ab = RW == 2 && (epi == EPI_SWIGLU || epi == EPI_MOE_DOWN);
    // row r of unit u: PAIR_AB: row u of A (r = 0) / of B (r = 1); else row RW*u + r of A
    const long long eA = S.expA == 0 ? e0 : S.expA == 1 ? e1 : 0;
    const long long eB = S.expB == 0 ? e0 : S.expB == 1 ? e1 : 0;
    const uint8_t* rp[RW][4];
    long long step[4];                                  // bytes between a row and the next unit's row
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const long long rowb = (long long)nb * PlaneBytes<T>::b[p];
        const long long ex = (long long)S.rows * rowb;   // one expert's plane bytes
        const long long r0 = ab ? u_first : (long long)u_first * RW;
        const long long rc = r0 < S.rows ? r0 : 0;       // a wave without units re-reads row 0 (parked)
#pragma unroll
        for (int r = 0; r < RW; ++r) {
            const bool isB = ab && r == 1;
            const uint8_t* base = isB ? S.b[p] + eB * ex : S.a[p] + eA * ex;
            long long row = ab ? rc : rc + r;
            if (row >= S.rows) row = S.rows - 1;         // an odd last pair re-reads its row (result unused)
            rp[r][p] = rfl_ptr(base + row * rowb);
        }
        step[p] = (ab ? (long long)stride : (long long)stride * RW) * rowb;
    }
    struct Slot {
        typename K::Ld w[RW];
        float2 res;
        float2 bia;
    };
    Slot ring[D];
    int iu = 0, ic = 0;                                 // issue cursor: unit index (0..n_units), chunk
    const bool has_res = S.resid != nullptr;
    const bool has_bias = GX && S.bias != nullptr && !ab;
    // the unit's residual values, with the unit's last chunk (item (iu_, ic_))
    auto res_load = [&](Slot& s, int iu_, int ic_, bool park) {
        const long long u = u_first + (long long)iu_ * stride;
        const long long r0 = ab ? u : u * RW;
        const bool rv = !park && ic_ == C - 1;
        const unsigned o0 = oob((unsigned)(r0 * 4), !rv);
        const unsigned o1 = oob((unsigned)((r0 + 1) * 4), !(rv && RW == 2 && !ab && r0 + 1 < S.rows));
        const uint8_t* rb = reinterpret_cast<const uint8_t*>(rfl_ptr(S.resid));
        s.res.x = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(buf_rsrc(rb), o0, 0, 0));
        s.res.y = RW == 2 && !ab ? __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(buf_rsrc(rb), o1, 0, 0)) : 0.0f;
    };
    // defer_res: the residual is the previous stage's output (persistent prefill before the barrier)
    auto issue = [&](Slot& s, bool defer_res) {
        const int sb0 = ic * 8 + sbl;
        const int sb = sb0 < nb ? sb0 : nb - 1;
        const bool park = iu >= n_units;               // no item left: out-of-range loads (zeros)
#pragma unroll
        for (int r = 0; r < RW; ++r) s.w[r] = K::bload(rp[r], sb, j, park);
        if (has_res && !defer_res) res_load(s, iu, ic, park);
        if (has_bias) {   // the unit's bias values, with the unit's last chunk
            const long long u = u_first + (long long)iu * stride;
            const long long r0 = u * RW;
            const bool rv = !park && ic == C - 1;
            const unsigned o0 = oob((unsigned)(r0 * 4), !rv);
            const unsigned o1 = oob((unsigned)((r0 + 1) * 4), !(rv && RW == 2 && r0 + 1 < S.rows));
            const uint8_t* bb = reinterpret_cast<const uint8_t*>(rfl_ptr(S.bias));
            s.bia.x = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(buf_rsrc(bb), o0, 0, 0));
            s.bia.y = RW == 2 ? __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(buf_rsrc(bb), o1, 0, 0)) : 0.0f;
        }
        if (!park && ++ic == C) {
            ic = 0;
            if (++iu < n_units) {
#pragma unroll
                for (int r = 0; r < RW; ++r)
#pragma unroll
                    for (int p = 0; p < 4; ++p) rp[r][p] += step[p];
            }
        }
    };
    if (P) {
        static_assert(!P || !GX, "the persistent kernel serves the LLaMA graph");
        // The next stage's weights stream while the grid barrier completes: waves 1-15 issue
        // their ring's first D-1 items into registers and touch the GV_TOUCH item-rows after
        // them into L2 (one dword load per 128-byte line, results discarded after the barrier);
        // wave 1 also touches wave 0's first items.  Wave 0 polls the barrier with no load in
        // flight (vmcnt retires in issue order: a flag load would wait behind a prefetch) and
        // issues its ring after it, from L2.  The stores of the previous stage (issued before
        // the prefetch) are complete before the workgroup publishes.
        constexpr int NTI = GV_TOUCH / RW;             // items touched per wave
        constexpr int NT = gv_touch_n<T, RW>();
        unsigned tv[2 * NT];
        // touch items [i0, i0 + NTI) of the wave whose first unit is uf (row pointers rb)
        auto touch = [&](const uint8_t* const (&rb)[RW][4], int nu, unsigned* out) {
            int nt = 0;
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                constexpr int bp[4] = {PlaneBytes<T>::b[0], PlaneBytes<T>::b[1], PlaneBytes<T>::b[2], PlaneBytes<T>::b[3]};
                if (bp[p] == 0) continue;
                const int lines = (8 * bp[p] + 127) / 128;   // 128-byte lines of one item-row of plane p
#pragma unroll
                for (int r = 0; r < RW; ++r) {
#pragma unroll
                    for (int i0 = 0; i0 < (NTI * ((8 * 256 + 127) / 128)); i0 += 64) {   // <= 2 loads per (plane, row)
                        if (i0 >= NTI * lines) break;
                        const int slot = i0 + lane;
                        const int item = (wave == 0 ? 0 : D - 1) + slot / lines, q = slot % lines;
                        const int ui = item / C, ci = item % C;
                        const bool valid = slot < NTI * lines && ui < nu;
                        const unsigned off = (unsigned)(ui * step[p] + (long long)ci * 8 * bp[p] + q * 128);
                        out[nt++] = __builtin_amdgcn_raw_buffer_load_b32(buf_rsrc(rb[r][p]), oob(off, !valid), 0, 0);
                    }
                }
            }
        };
        if (wave != 0) {
            const uint8_t* rb0[RW][4];
#pragma unroll
            for (int r = 0; r < RW; ++r)
#pragma unroll
                for (int p = 0; p < 4; ++p) rb0[r][p] = rp[r][p];
#pragma unroll
            for (int k = 0; k < D - 1; ++k) issue(ring[k], true);
            touch(rb0, n_units, tv);
            if (wave == 1) {   // wave 0's first items: its rows are wave 1's minus nblk units
                const int nu0 = wg < S.units ? (S.units - wg + stride - 1) / stride : 0;
                const uint8_t* rw0[RW][4];
#pragma unroll
                for (int p = 0; p < 4; ++p) {
                    const long long back = (long long)S.nblk * (ab ? 1 : RW) * nb * PlaneBytes<T>::b[p];
#pragma unroll
                    for (int r = 0; r < RW; ++r) rw0[r][p] = u_first < S.units ? rb0[r][p] - back : rb0[r][p];
                }
                touch(rw0, nu0, tv + NT);
                wait_vm<(D - 1) * RW * gv_nl<T>() + 2 * NT>();
            } else {
                wait_vm<(D - 1) * RW * gv_nl<T>() + NT>();
            }
        } else {
            wait_vm<0>();
        }
        if (!wait()) return;
        if (wave != 0) {
#pragma unroll
            for (int k = 0; k < NT; ++k) asm volatile("" ::"v"(tv[k]));   // retire the touches
            if (wave == 1) {
#pragma unroll
                for (int k = NT; k < 2 * NT; ++k) asm volatile("" ::"v"(tv[k]));
            }
        } else {
#pragma unroll
            for (int k = 0; k < D - 1; ++k) issue(ring[k], true);
        }
    }

    // ---- 3. entry loads: token position, the activation slices ---------------------------------
    const bool qkv = epi == EPI_QKV;
    const bool need_tp = qkv || (pro == PRO_ATTN && a.attn_nsplit == 0);
    i32x4 tp = {0, 0, 0, 0};
    const bool order4 = !P && a.order == 4;
    if (need_tp && !order4) tp = *gptr(reinterpret_cast<const i32x4*>(a.tokpos));
    double* red = reinterpret_cast<double*>(lds + gv_red_off(nb, a.nslots, a.n_rot));
    float* rope = reinterpret_cast<float*>(lds + gv_rope_off(nb, a.nslots));
    // ggml_rope_cache_init for this token's position (ext_factor 0, mscale 1) into LDS
    auto rope_table = [&](int pos_, float ff0_, float ff1_) {
        for (int i = lane; i < a.n_rot / 2; i += 64) {
            float theta = (float)pos_;
            for (int k = 0; k < i; ++k) theta = theta * a.theta_scale;
            const float ff = i < 64 ? ff0_ : ff1_;
            const float th = a.freq_scale * (theta / ff);
            rope[2 * i] = cosf(th);
            rope[2 * i + 1] = sinf(th);
        }
    };
    if (order4) {
        // ---- prologue waves (order 4) ----------------------------------------------------------
        // A wave that has issued its weight ring cannot run the prologue: its later instructions
        // wait behind the ring's requests in the CU's memory pipeline (back-pressure, ~4 us at a
        // decode launch's ~100 KB in flight per CU; in-kernel stamps).  So waves
        // [0, npro) build the activation -- their x / norm-weight blocks by LDS-DMA into a stage,
        // the RMSNorm partials exchanged through LDS flag words, then the Q8_K / Q8_0 blocks --
        // and issue their rings after it; the other waves issue their rings at once and wait for
        // the prologue waves' flags (and the RoPE wave's) before the first dot product.
        const int npro = a.npro;
        const bool pw = wave < npro;
        const bool need_w = pro == PRO_RMSNORM;
        char* const stage = lds + a.stage_off;
        // [2][GV_NW] flag words, through an LDS-typed pointer (a generic one would make them flat_*)
        volatile __attribute__((address_space(3))) int* const flg = (volatile __attribute__((address_space(3))) int*)(lds + a.flag_off);
        if (wave == 0 && lane < 2 * GV_NW) flg[lane] = 0;
        if (pw) {
            const float* xo = a.attn_o;
            const float* xs = a.x[0];
            asm volatile("" : "+s"(xo), "+s"(xs));
            const float* x0 = pro == PRO_ATTN ? xo : xs;
            for (int blk = wave; blk < nb; blk += npro) {
                __builtin_amdgcn_global_load_lds(gptr(x0 + blk * 256 + lane * 4),
                                                 (__attribute__((address_space(3))) void*)(stage + blk * 1024), 16, 0, 0);
                if (need_w)
                    __builtin_amdgcn_global_load_lds(gptr(a.norm_w + blk * 256 + lane * 4),
                                                     (__attribute__((address_space(3))) void*)(stage + (size_t)(nb + blk) * 1024), 16, 0, 0);
                if (dual)
                    __builtin_amdgcn_global_load_lds(gptr(a.x[1] + blk * 256 + lane * 4),
                                                     (__attribute__((address_space(3))) void*)(stage + (size_t)(nb + blk) * 1024), 16, 0, 0);
            }
        }
        float ff0 = 1.0f, ff1 = 1.0f;
        const bool rope_wave = qkv && a.n_rot > 0 && wave == GV_NW - 1;
        // the token position: prologue waves and the RoPE wave now, the other waves behind their ring
        if (need_tp && (pw || rope_wave)) tp = *gptr(reinterpret_cast<const i32x4*>(a.tokpos));
        if (rope_wave && a.freq_factors) {
            if (lane < a.n_rot / 2) ff0 = gptr(a.freq_factors)[lane];
            if (lane + 64 < a.n_rot / 2) ff1 = gptr(a.freq_factors)[lane + 64];
        }
        lds_barrier();   // the flag words are zero (the LDS-DMA stays in flight across it)
        // wait until flags[round][w] are set for every wave w in `mask` (one lane per wave)
        auto wait_flags = [&](int round, unsigned mask) {
            for (;;) {
                const bool ok = !((mask >> lane) & 1u) || flg[round * GV_NW + (lane & (GV_NW - 1))] != 0;
                if (__all(ok)) break;
                __builtin_amdgcn_s_sleep(1);
            }
        };
        const unsigned pmask = (1u << npro) - 1u;
        if (!pw) {
            if (rope_wave) {   // before its ring: the table is on the critical path of the epilogue
                rope_table(readfirstlane_i(tp.y), ff0, ff1);
                __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): the table is written
                if (lane == 0) flg[GV_NW + wave] = 1;
            }
#pragma unroll
            for (int k = 0; k < D - 1; ++k) issue(ring[k], false);
            if (need_tp && !rope_wave) tp = *gptr(reinterpret_cast<const i32x4*>(a.tokpos));
            GV_STAMPL(1)
        } else {
            wait_vm<0>();   // this wave's staged blocks landed
            float scale = 1.0f;
            if (pro == PRO_RMSNORM) {
                // ggml_compute_forward_rms_norm_f32: sum of float squares in double
                double sq = 0.0;
                for (int blk = wave; blk < nb; blk += npro) {
                    const f32x4 v = *reinterpret_cast<const f32x4*>(stage + blk * 1024 + lane * 16);
                    sq += (double)(v.x * v.x);
                    sq += (double)(v.y * v.y);
                    sq += (double)(v.z * v.z);
                    sq += (double)(v.w * v.w);
                }
                sq = wave_sum63_d(sq);
                if (lane == 63) red[wave] = sq;
                __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): the partial is written
                if (lane == 63) flg[wave] = 1;
                wait_flags(0, pmask);
                double tot = 0.0;
                for (int w = 0; w < npro; ++w) tot += red[w];
                scale = 1.0f / sqrtf((float)(tot / (double)a.K) + a.eps);
            }
            for (int blk = wave; blk < nb; blk += npro) {
                const f32x4 xv = *reinterpret_cast<const f32x4*>(stage + blk * 1024 + lane * 16);
                float v[4] = {xv.x, xv.y, xv.z, xv.w};
                if (pro == PRO_RMSNORM) {
                    const f32x4 wv = *reinterpret_cast<const f32x4*>(stage + (size_t)(nb + blk) * 1024 + lane * 16);
                    v[0] = (v[0] * scale) * wv.x;   // ggml_vec_scale_f32 then ggml_mul
                    v[1] = (v[1] * scale) * wv.y;
                    v[2] = (v[2] * scale) * wv.z;
                    v[3] = (v[3] * scale) * wv.w;
                }
                if (Q80)
                    quant_q80_block(v, lane, reinterpret_cast<int8_t*>(lds + L.q80 + blk * GV_ASTR),
                                    reinterpret_cast<float*>(lds + L.d0) + blk * 8);
                else
                    quant_q8k_block(v, lane, reinterpret_cast<int8_t*>(lds + L.q8k + blk * GV_ASTR),
                                    reinterpret_cast<int*>(lds + L.bsum) + blk * 16, reinterpret_cast<float*>(lds + L.dk) + blk);
                if (dual) {
                    const f32x4 yv = *reinterpret_cast<const f32x4*>(stage + (size_t)(nb + blk) * 1024 + lane * 16);
                    float y[4] = {yv.x, yv.y, yv.z, yv.w};
                    char* s1 = lds + slot_bytes;
                    if (Q80)
                        quant_q80_block(y, lane, reinterpret_cast<int8_t*>(s1 + L.q80 + blk * GV_ASTR),
                                        reinterpret_cast<float*>(s1 + L.d0) + blk * 8);
                    else
                        quant_q8k_block(y, lane, reinterpret_cast<int8_t*>(s1 + L.q8k + blk * GV_ASTR),
                                        reinterpret_cast<int*>(s1 + L.bsum) + blk * 16, reinterpret_cast<float*>(s1 + L.dk) + blk);
                }
            }
            __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): this wave's blocks are written
            if (lane == 0) flg[GV_NW + wave] = 1;
#ifdef MI_STAMPS   // 7 (order 4): the workgroup's last prologue wave done
            if (a.stamps && lane == 0) atomicMax(a.stamps + blockIdx.x * 8 + 7, (unsigned long long)__builtin_amdgcn_s_memrealtime());
#endif
#pragma unroll
            for (int k = 0; k < D - 1; ++k) issue(ring[k], false);
        }
        wait_flags(1, pmask | (rope_wave || (qkv && a.n_rot > 0) ? (1u << (GV_NW - 1)) : 0u));
        GV_STAMPL(2)
    } else {
        // ---- 3. entry loads: token position, the activation slices ---------------------------------
        const bool qkv = epi == EPI_QKV;
        const bool need_tp = qkv || (pro == PRO_ATTN && a.attn_nsplit == 0);
        i32x4 tp = {0, 0, 0, 0};
        if (need_tp) tp = *gptr(reinterpret_cast<const i32x4*>(a.tokpos));
        f32x4 xv[KB], wv[KB], yv[KB];
    #pragma unroll
        for (int i = 0; i < KB; ++i) {
            const int blk = wave + GV_NW * i;
            if (blk < nb) {
                // (values made opaque: a select of two addresses into the parameter copy would put it in scratch)
                const float* xo = a.attn_o;
                const float* xs = a.x[0];
                asm volatile("" : "+s"(xo), "+s"(xs));
                const float* x0 = pro == PRO_ATTN ? xo : xs;
                xv[i] = gptr(reinterpret_cast<const f32x4*>(x0))[blk * 64 + lane];
                if (pro == PRO_RMSNORM || (GX && pro == PRO_LAYERNORM))
                    wv[i] = gptr(reinterpret_cast<const f32x4*>(a.norm_w))[blk * 64 + lane];
                if (dual) yv[i] = gptr(reinterpret_cast<const f32x4*>(a.x[1]))[blk * 64 + lane];
                else if (GX && pro == PRO_LAYERNORM) yv[i] = gptr(reinterpret_cast<const f32x4*>(a.norm_b))[blk * 64 + lane];
            }
        }
        float ff0 = 1.0f, ff1 = 1.0f;
        const bool rope_wave = qkv && a.n_rot > 0 && wave == GV_NW - 1;
        if (rope_wave && a.freq_factors) {
            if (lane < a.n_rot / 2) ff0 = gptr(a.freq_factors)[lane];
            if (lane + 64 < a.n_rot / 2) ff1 = gptr(a.freq_factors)[lane + 64];
        }
        if (P) {   // the residuals of the prefilled items (item k = unit k / C, chunk k % C)
            if (has_res) {
    #pragma unroll
                for (int k = 0; k < D - 1; ++k) res_load(ring[k], k / C, k % C, k / C >= n_units);
            }
        } else {
            // the activation requests ahead of the weight requests (a.order, measured: DESIGN.md §4)
            if (a.order == 1) __builtin_amdgcn_s_barrier();
            if (a.order == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    #ifdef MI_STAMPS   // 7 (order 2): the workgroup's last wave whose activation landed
            if (a.stamps && lane == 0 && a.order == 2)
                atomicMax(a.stamps + blockIdx.x * 8 + 7, (unsigned long long)__builtin_amdgcn_s_memrealtime());
    #endif
        }
        const int pre = P ? D - 1 : a.pre;
        if (!P) {
    #pragma unroll
            for (int k = 0; k < D - 1; ++k)
                if (k < pre) issue(ring[k], false);
        }
        GV_STAMP(1)

        // ---- 3. prologue: the activation into LDS while the weights stream ---------------------------
        float scale = 1.0f;
        if (pro == PRO_RMSNORM) {
            // ggml_compute_forward_rms_norm_f32: sum of float squares in double
            double s = 0.0;
    #pragma unroll
            for (int i = 0; i < KB; ++i)
                if (wave + GV_NW * i < nb) {
                    s += (double)(xv[i].x * xv[i].x);
                    s += (double)(xv[i].y * xv[i].y);
                    s += (double)(xv[i].z * xv[i].z);
                    s += (double)(xv[i].w * xv[i].w);
                }
            s = wave_sum63_d(s);
            if (lane == 63) red[wave] = s;
            lds_barrier();
            double tot = 0.0;
    #pragma unroll
            for (int w = 0; w < GV_NW; ++w) tot += red[w];
            scale = 1.0f / sqrtf((float)(tot / (double)a.K) + a.eps);
        }
        float mean = 0.0f;
        if (GX && pro == PRO_LAYERNORM) {
            // ggml_compute_forward_norm_f32: mean from a double sum, then the double sum of the
            // f32 squares of (x - mean), variance = (float)(sum2 / n)
            double s = 0.0;
    #pragma unroll
            for (int i = 0; i < KB; ++i)
                if (wave + GV_NW * i < nb) {
                    s += (double)xv[i].x;
                    s += (double)xv[i].y;
                    s += (double)xv[i].z;
                    s += (double)xv[i].w;
                }
            s = wave_sum63_d(s);
            if (lane == 63) red[wave] = s;
            lds_barrier();
            double tot = 0.0;
    #pragma unroll
            for (int w = 0; w < GV_NW; ++w) tot += red[w];
            mean = (float)(tot / (double)a.K);
            double s2 = 0.0;
    #pragma unroll
            for (int i = 0; i < KB; ++i)
                if (wave + GV_NW * i < nb) {
                    const float v0 = xv[i].x - mean, v1 = xv[i].y - mean, v2 = xv[i].z - mean, v3 = xv[i].w - mean;
                    s2 += (double)(v0 * v0);
                    s2 += (double)(v1 * v1);
                    s2 += (double)(v2 * v2);
                    s2 += (double)(v3 * v3);
                }
            s2 = wave_sum63_d(s2);
            if (lane == 63) red[GV_NW + wave] = s2;
            lds_barrier();
            double tot2 = 0.0;
    #pragma unroll
            for (int w = 0; w < GV_NW; ++w) tot2 += red[GV_NW + w];
            scale = 1.0f / sqrtf((float)(tot2 / (double)a.K) + a.eps);
        }
        if (pro == PRO_ATTN) {
            // the other splits of the attention partials (contexts past ATTN_SHORT cells), in split order
            int nsplit = a.attn_nsplit;
            if (nsplit == 0) {
                int chunk;
                attn_split(__builtin_amdgcn_readfirstlane(tp.z) + 1, chunk, nsplit);
            }
            if constexpr (KB == 1) {
                // four splits' loads in flight together, then added in split order
                for (int sp0 = 1; sp0 < nsplit; sp0 += 4) {
                    f32x4 t4[4];
    #pragma unroll
                    for (int j = 0; j < 4; ++j)
                        if (wave < nb && sp0 + j < nsplit)
                            t4[j] = gptr(reinterpret_cast<const f32x4*>(a.attn_o + (long long)(sp0 + j) * a.attn_stride))[wave * 64 + lane];
    #pragma unroll
                    for (int j = 0; j < 4; ++j)
                        if (wave < nb && sp0 + j < nsplit) xv[0] += t4[j];
                }
            } else {   // wider activations: no extra registers (they would cost the GEMV ring its occupancy)
                for (int sp = 1; sp < nsplit; ++sp) {
    #pragma unroll
                    for (int i = 0; i < KB; ++i) {
                        const int blk = wave + GV_NW * i;
                        if (blk < nb)
                            xv[i] += gptr(reinterpret_cast<const f32x4*>(a.attn_o + (long long)sp * a.attn_stride))[blk * 64 + lane];
                    }
                }
            }
        }
    #pragma unroll
        for (int i = 0; i < KB; ++i) {
            const int blk = wave + GV_NW * i;
            if (blk >= nb) continue;
            float v[4] = {xv[i].x, xv[i].y, xv[i].z, xv[i].w};
            if (pro == PRO_RMSNORM) {
                v[0] = (v[0] * scale) * wv[i].x;   // ggml_vec_scale_f32 then ggml_mul
                v[1] = (v[1] * scale) * wv[i].y;
                v[2] = (v[2] * scale) * wv[i].z;
                v[3] = (v[3] * scale) * wv[i].w;
            }
            if (GX && pro == PRO_LAYERNORM) {        // (x - mean) * scale, then ggml_mul, ggml_add
                v[0] = ((v[0] - mean) * scale) * wv[i].x + yv[i].x;
                v[1] = ((v[1] - mean) * scale) * wv[i].y + yv[i].y;
                v[2] = ((v[2] - mean) * scale) * wv[i].z + yv[i].z;
                v[3] = ((v[3] - mean) * scale) * wv[i].w + yv[i].w;
            }
            if (Q80)
                quant_q80_block(v, lane, reinterpret_cast<int8_t*>(lds + L.q80 + blk * GV_ASTR),
                                reinterpret_cast<float*>(lds + L.d0) + blk * 8);
            else
                quant_q8k_block(v, lane, reinterpret_cast<int8_t*>(lds + L.q8k + blk * GV_ASTR),
                                reinterpret_cast<int*>(lds + L.bsum) + blk * 16, reinterpret_cast<float*>(lds + L.dk) + blk);
            if (dual) {
                float y[4] = {yv[i].x, yv[i].y, yv[i].z, yv[i].w};
                char* s1 = lds + slot_bytes;
                if (Q80)
                    quant_q80_block(y, lane, reinterpret_cast<int8_t*>(s1 + L.q80 + blk * GV_ASTR),
                                    reinterpret_cast<float*>(s1 + L.d0) + blk * 8);
                else
                    quant_q8k_block(y, lane, reinterpret_cast<int8_t*>(s1 + L.q8k + blk * GV_ASTR),
                                    reinterpret_cast<int*>(s1 + L.bsum) + blk * 16, reinterpret_cast<float*>(s1 + L.dk) + blk);
            }
        }
        if (rope_wave) rope_table(readfirstlane_i(tp.y), ff0, ff1);
        lds_barrier();
    #pragma unroll
        for (int k = 0; k < D - 1; ++k)
            if (k >= pre) issue(ring[k], false);
        GV_STAMP(2)
        if (P) wait.mark();

    }
    const int pos = readfirstlane_i(tp.y);
    const int cell = readfirstlane_i(tp.z);
    // ---- 4. the stream: consume item i while items i+1 .. i+D-1 are in flight -----------------
    const char* act0 = lds;
    const char* actB = (dual && S.actB == 1) ? lds + slot_bytes : lds;
    float acc[RW];
#pragma unroll
    for (int r = 0; r < RW; ++r) acc[r] = 0.0f;
    int cu = 0, cc = 0;                                 // consume cursor
    auto consume = [&](const Slot& s) {
        const int sb0 = cc * 8 + sbl;
        const bool lv = sb0 < nb;
        const int sb = lv ? sb0 : nb - 1;
        const typename K::AR ar = GvAct<T>::get(act0, L, sb, j);
#pragma unroll
        for (int r = 0; r < RW; ++r) {
            float p;
            if (RW == 2 && r == 1 && dual) {
                const typename K::AR arB = GvAct<T>::get(actB, L, sb, j);
                p = K::dot(s.w[r], arB, j);
            } else {
                p = K::dot(s.w[r], ar, j);
            }
            acc[r] += lv ? p : 0.0f;
        }
        if (++cc == C) {
            float y[RW];
#pragma unroll
            for (int r = 0; r < RW; ++r) {
                y[r] = wave_sum63(acc[r]);
                acc[r] = 0.0f;
            }
            if (has_bias) {   // ggml_add of the projection bias
                y[0] += s.bia.x;
                if (RW == 2) y[RW - 1] += s.bia.y;
            }
            if (lane == 63) {
                const long long u = u_first + (long long)cu * stride;
                float* const out = S.out;
                if (ab) {
                    if (epi == EPI_SWIGLU) gst<P>(out + u, silu_f(y[0]) * y[RW - 1]);
                    else gst<P>(out + u, (y[0] * w0 + y[RW - 1] * w1) + s.res.x);   // EPI_MOE_DOWN
                } else {
                    const long long r0 = u * RW;
                    if (epi == EPI_QKV) {
                        // RoPE pairs (RW == 2): rows r0, r0+1 of Q or K; or two V rows
                        float o0 = y[0], o1 = y[RW - 1];
                        const bool isq = r0 < S.nq, isk = !isq && r0 < S.nq + S.nk;
                        if (isq || isk) {
                            const int i0 = (int)((isq ? r0 : r0 - S.nq) % a.head_dim);
                            if (i0 < a.n_rot) {
                                const float cs = rope[i0], sn = rope[i0 + 1];
                                o0 = y[0] * cs - y[RW - 1] * sn;
                                o1 = y[0] * sn + y[RW - 1] * cs;
                            }
                        }
                        if (isq) {
                            gst<P>(out + r0, o0);
                            gst<P>(out + r0 + 1, o1);
                        } else if (isk) {
                            const long long rk = r0 - S.nq;
                            unsigned short* const kr = reinterpret_cast<unsigned short*>(a.kcache + (long long)cell * a.kv_dim);
                            gst<P>(kr + rk, __half_as_ushort(__float2half_rn(o0)));
                            gst<P>(kr + rk + 1, __half_as_ushort(__float2half_rn(o1)));
                            if (rk == 0) gst<P>(a.cell_pos + cell, pos);
                        } else {
                            const long long rv = r0 - S.nq - S.nk;
                            unsigned short* const vr = reinterpret_cast<unsigned short*>(a.vcache + (long long)cell * a.kv_dim);
                            gst<P>(vr + rv, __half_as_ushort(__float2half_rn(o0)));
                            if (RW == 2 && r0 + 1 < S.rows) gst<P>(vr + rv + 1, __half_as_ushort(__float2half_rn(o1)));
                        }
                    } else {
#pragma unroll
                        for (int r = 0; r < RW; ++r) {
                            if (r0 + r >= S.rows) break;
                            const float v = r == 0 ? y[0] : y[RW - 1];
                            const float rv = r == 0 ? s.res.x : s.res.y;
                            float o = v;
                            if (epi == EPI_ADD) o = v + rv;
                            if (GX && epi == EPI_GELU) {   // ggml_vec_gelu_f32 (GGML_GELU_FP16 table)
                                const unsigned short hb = __half_as_ushort(__float2half_rn(v));
                                const float t = __half2float(__ushort_as_half(gptr(a.gelu_tab)[hb]));
                                o = v <= -10.0f ? 0.0f : (v >= 10.0f ? v : t);
                            }
                            gst<P>(out + r0 + r, o);
                        }
                    }
                }
            }
            cc = 0;
            ++cu;
        }
    };
    for (int base = 0; base < n_items; base += D) {
#pragma unroll
        for (int k = 0; k < D; ++k) {
            issue(ring[(k + D - 1) % D], false);
            if (base + k < n_items) consume(ring[k]);
            if (base + k == 0) {
                if (order4) { GV_STAMPL(3) } else { GV_STAMP(3) }
            }
        }
    }
    GV_STAMP(4)
#ifdef MI_STAMPS   // 5: the workgroup's last wave to finish
    if (a.stamps && lane == 0) atomicMax(a.stamps + blockIdx.x * 8 + 5, (unsigned long long)__builtin_amdgcn_s_memrealtime());
#endif
#undef GV_STAMP
#undef GV_STAMPL
}

// T1: -1 one segment; -2 two segments of type T0; else the type of segment 1.
// TAG: 1 for the FFN gate/up launches, so that the roofline kernel has a symbol of its own in
// kernel traces (the same code as the QKV launches of an all-Q4_K layer); 2 for the GPT-2
// launches (LayerNorm / bias / GELU compiled in, kept out of the LLaMA kernels' registers).
// The parameter block is read with ONE vector load per lane and spread to scalars with
// v_readlane: the compiler's kernarg scalar loads came in ~7 dependent rounds (each a scalar
// cache miss), ~2.4 us from entry to the first weight request (scripts/timeline.py).
__device__ __forceinline__ GvArgs gv_args_fetch(const GvArgs& ka) {
    constexpr int NW = (int)(sizeof(GvArgs) / 4);
    static_assert(sizeof(GvArgs) % 4 == 0 && NW <= 4 * 64, "parameter block layout");
    int lane = threadIdx.x & 63;
    asm volatile("" : "+v"(lane));
    const u32x4* src = reinterpret_cast<const u32x4*>(&ka);
    u32x4 v = {0u, 0u, 0u, 0u};
    if (lane < (NW + 3) / 4) v = src[lane];
    GvArgs l;
    unsigned* dst = reinterpret_cast<unsigned*>(&l);
#pragma unroll
    for (int i = 0; i < NW; ++i) dst[i] = __builtin_amdgcn_readlane(v[i & 3], i >> 2);
    return l;
}

template <int T0, int T1, int RW, int KB, int D, int TAG>
__global__ __launch_bounds__(GV_NW * 64) void gemv_kernel(const GvArgs ka) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const GvArgs a = gv_args_fetch(ka);
    if (T1 == -1 || (int)blockIdx.x < a.seg[1].blk0) gv_body<T0, 0, RW, KB, D, TAG == 2, false, GvNoWait, TAG == 1>(a, lds);
    else gv_body<(T1 < 0 ? T0 : T1), 1, RW, KB, D, TAG == 2, false, GvNoWait, TAG == 1>(a, lds);
}

typedef void (*GvFn)(const GvArgs);

// ring depth: items of one wave in flight (an item is RW rows x one 8-superblock chunk);
// KB activation blocks per wave (K <= 4096: 1, <= 8192: 2, <= 16384: 4 at 16 waves)
// (the 128-VGPR budget of a 16-wave workgroup: 4 one-row items, 3 two-row items; 2 for the
// wider Q5_K / Q6_K / Q8_0 two-row items)
template <int T, int RW> struct GvD {
    static constexpr int D = RW == 1 ? 4 : (T == T_Q4_K ? 3 : 2);
};

template <int T0, int T1, int RW, int TAG>
GvFn gv_fn_kb(int kb) {
    constexpr int D = GvD<T0, RW>::D < GvD<(T1 < 0 ? T0 : T1), RW>::D ? GvD<T0, RW>::D : GvD<(T1 < 0 ? T0 : T1), RW>::D;
    switch (kb) {
    case 1: return gemv_kernel<T0, T1, RW, 1, D, TAG>;
    case 2: return gemv_kernel<T0, T1, RW, 2, D, TAG>;
    case 4: return gemv_kernel<T0, T1, RW, 4, D, TAG>;
    default: return nullptr;
    }
}
// t1: -1 one segment, -2 two of type T0, else the second segment's type (Q6_K / Q8_0)
template <int T0, int RW>
GvFn gv_fn_pair(int t1, int kb, int tag) {
    switch (t1) {
    case -1: return tag == 2 ? gv_fn_kb<T0, -1, RW, 2>(kb)
                  : tag && RW == 2 ? gv_fn_kb<T0, -1, RW, 1>(kb) : gv_fn_kb<T0, -1, RW, 0>(kb);
    case -2: return gv_fn_kb<T0, -2, RW, 0>(kb);
    case T_Q6_K: return gv_fn_kb<T0, T_Q6_K, RW, 0>(kb);
    case T_Q8_0: return gv_fn_kb<T0, T_Q8_0, RW, 0>(kb);
    default: return nullptr;
    }
}
template <int RW>
GvFn gv_fn_rw(int t0, int t1, int kb, int tag) {
    switch (t0) {
    case T_Q4_K: return gv_fn_pair<T_Q4_K, RW>(t1, kb, tag);
    case T_Q5_K: return gv_fn_pair<T_Q5_K, RW>(t1, kb, tag);
    case T_Q6_K: return t1 == T_Q6_K ? nullptr : gv_fn_pair<T_Q6_K, RW>(t1, kb, tag);
    case T_Q8_0: return t1 >= 0 ? nullptr : gv_fn_pair<T_Q8_0, RW>(t1, kb, tag);
    default: return nullptr;
    }
}
// nseg segments of types t0 (, t1); tag: the FFN gate/up launch
GvFn gv_fn(int nseg, int t0, int t1, int rw, int kb, int tag) {
    const int k = nseg == 1 ? -1 : (t1 == t0 ? -2 : t1);
    return rw == 2 ? gv_fn_rw<2>(t0, k, kb, tag) : gv_fn_rw<1>(t0, k, kb, tag);
}

int gv_kb(int K) {
    const int nb = K / 256;
    const int kb = (nb + GV_NW - 1) / GV_NW;
    return kb <= 1 ? 1 : kb <= 2 ? 2 : kb <= 4 ? 4 : -1;
}

bool gv_rw2(const GemvSeg& s) { return s.pair == PAIR_AB || s.epi == EPI_QKV; }

long long seg_bytes(const GemvSeg& s) {
    auto mb = [](const QMat& q) {
        return (long long)q.rows * q.nb * ((long long)block_bytes(q.type) * 256 / block_elems(q.type));
    };
    return s.pair == PAIR_AB ? mb(s.A) + mb(s.B) : mb(s.A);
}

// dynamic LDS of a launch: the activation slots, RoPE table and reductions (+ the staged arrays)
size_t gv_lds_total(const GvArgs& a, int nb, int pro) {
    size_t b = gv_lds_bytes(nb, a.nslots, a.n_rot);
    if (a.order == 4) b = (size_t)a.flag_off + 2 * GV_NW * sizeof(int);
    return b;
}

// cap on workgroups: the weight ring keeps D items x RW rows in flight per wave
int gv_grid_cap() { return 256; }

}  // namespace

bool gemv_pair_supported(int t1, int t2) {
    if (t1 == t2) return is_quant(t1);
    return (t2 == T_Q6_K && (t1 == T_Q4_K || t1 == T_Q5_K)) ||
           (t2 == T_Q8_0 && (t1 == T_Q4_K || t1 == T_Q5_K || t1 == T_Q6_K));
}

int gemv_grid(const GemvParams& p) {
    int units = 0;
    for (int i = 0; i < p.nseg; ++i) {
        const GemvSeg& s = p.seg[i];
        const int rw = gv_rw2(s) ? 2 : 1;
        units += s.pair == PAIR_AB ? s.A.rows : (s.A.rows + rw - 1) / rw;
    }
    return std::max(p.nseg, std::min(gv_grid_cap(), (units + GV_NW - 1) / GV_NW));
}

void init_kernel_attributes() {
    init_gemm_attributes();
    const int types[4] = {T_Q4_K, T_Q5_K, T_Q6_K, T_Q8_0};
    for (int rw = 1; rw <= 2; ++rw)
        for (int kb : {1, 2, 4})
            for (int t0 : types)
                for (int t1 : {-1, t0, (int)T_Q6_K, (int)T_Q8_0}) {
                    for (int tag = 0; tag <= 2; ++tag) {
                        GvFn f = t1 < 0 ? gv_fn(1, t0, t0, rw, kb, tag) : gv_fn(2, t0, t1, rw, kb, tag);
                        if (f)
                            MI_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(f),
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)GV_LDS_MAX));
                    }
                }
}

// Validates a launch and fills its kernel arguments: grid (<= cap workgroups), the variant key.
struct GvKey {
    int nseg, t0, t1, rw, kb, tag;
};
static void gv_prepare(const GemvParams& p, int cap, GvArgs& a, int& grid_out, GvKey& key) {
    if (p.nseg < 1 || p.nseg > GEMV_MAX_SEG) throw Error("gemv: 1 or 2 segments per launch");
    if (p.K % 256 != 0 || p.K > GV_KMAX) throw Error("gemv: K must be a multiple of 256 and <= 14336");
    const bool rw2 = gv_rw2(p.seg[0]);
    for (int i = 0; i < p.nseg; ++i) {
        const GemvSeg& g = p.seg[i];
        if (gv_rw2(g) != rw2) throw Error("gemv: segments of one launch must share their unit shape");
        if (g.A.K != p.K || (g.pair == PAIR_AB && (g.B.K != p.K || g.B.type != g.A.type || g.B.rows != g.A.rows)))
            throw Error("gemv: matrix shapes do not match the activation");
        if (!is_quant(g.A.type)) throw Error("gemv: unsupported quant type");
        if (g.epi == EPI_QKV && (g.A.rows & 1)) throw Error("gemv: fused QKV rows must be even");
        if ((g.epi == EPI_SWIGLU || g.epi == EPI_MOE_DOWN) != (g.pair == PAIR_AB))
            throw Error("gemv: SwiGLU / MoE-down epilogues take a PAIR_AB segment");
        if ((g.epi == EPI_ADD || g.epi == EPI_MOE_DOWN) && !g.resid) throw Error("gemv: residual epilogue without resid");
        if (g.epi == EPI_GELU && (!p.gelu_tab || g.pair == PAIR_AB)) throw Error("gemv: GELU epilogue needs the table, one matrix");
        if (g.bias && g.pair == PAIR_AB) throw Error("gemv: no bias on a PAIR_AB segment");
    }
    if (p.nseg == 2 && !gemv_pair_supported(p.seg[0].A.type, p.seg[1].A.type))
        throw Error("gemv: unsupported pair of segment types");
    if (p.pro == PRO_ATTN && (p.attn.n_head * p.attn.head_dim != p.K)) throw Error("gemv: attention combine needs K == n_head*head_dim");
    if (p.nslots == 2 && (p.pro == PRO_RMSNORM || p.pro == PRO_LAYERNORM)) throw Error("gemv: a second activation slot is plain");
    if (p.pro == PRO_LAYERNORM && (!p.norm_w || !p.norm_b)) throw Error("gemv: layer norm needs its weight and bias");
    const int kb = gv_kb(p.K);
    bool gx = p.pro == PRO_LAYERNORM;
    for (int i = 0; i < p.nseg; ++i) gx = gx || p.seg[i].bias || p.seg[i].epi == EPI_GELU;
    if (gx && p.nseg != 1) throw Error("gemv: LayerNorm / bias / GELU launches take one segment");
    key.nseg = p.nseg;
    key.t0 = p.seg[0].A.type;
    key.t1 = p.seg[p.nseg - 1].A.type;
    key.rw = rw2 ? 2 : 1;
    key.kb = kb;
    key.tag = gx ? 2 : (p.nseg == 1 && p.seg[0].epi == EPI_SWIGLU && p.nslots <= 1 ? 1 : 0);

    std::memset(&a, 0, sizeof(a));
    // workgroups per segment in proportion to its bytes (at least one each)
    int units = 0;
    for (int i = 0; i < p.nseg; ++i) {
        const GemvSeg& sg = p.seg[i];
        units += sg.pair == PAIR_AB ? sg.A.rows : (sg.A.rows + key.rw - 1) / key.rw;
    }
    const int grid = std::max(p.nseg, std::min(cap, (units + GV_NW - 1) / GV_NW));
    long long tot = 0;
    for (int i = 0; i < p.nseg; ++i) tot += seg_bytes(p.seg[i]);
    int blk = 0;
    for (int i = 0; i < p.nseg; ++i) {
        const GemvSeg& g = p.seg[i];
        GvSeg& o = a.seg[i];
        for (int k = 0; k < 4; ++k) {
            o.a[k] = g.A.p[k];
            o.b[k] = g.pair == PAIR_AB ? g.B.p[k] : g.A.p[k];
        }
        o.out = g.out;
        o.resid = g.resid;
        o.bias = g.bias;
        o.rows = g.A.rows;
        o.units = g.pair == PAIR_AB ? g.A.rows : (g.A.rows + key.rw - 1) / key.rw;
        o.epi = g.epi;
        o.nq = g.nq;
        o.nk = g.nk;
        o.expA = g.expA;
        o.expB = g.expB;
        o.actB = g.actB;
        int nblk = i + 1 == p.nseg ? grid - blk
                                   : (int)std::max(1LL, std::min<long long>(grid - blk - 1, grid * seg_bytes(g) / std::max(1LL, tot)));
        nblk = std::max(1, std::min(nblk, (o.units + GV_NW - 1) / GV_NW));
        o.blk0 = blk;
        o.nblk = nblk;
        blk += nblk;
    }
    if (p.nseg == 1) a.seg[1].blk0 = blk;   // every workgroup is segment 0's
    a.x[0] = p.x[0];
    a.x[1] = p.nslots > 1 ? p.x[1] : p.x[0];
    a.norm_w = p.norm_w;
    a.norm_b = p.norm_b;
    a.gelu_tab = p.gelu_tab;
    a.attn_o = p.attn.o;
    a.tokpos = p.tokpos;
    a.cell_pos = p.cell_pos;
    a.kcache = p.kcache;
    a.vcache = p.vcache;
    a.freq_factors = p.freq_factors;
    a.sel = p.sel;
    a.selw = p.selw;
    a.eps = p.eps;
    a.theta_scale = p.theta_scale;
    a.freq_scale = p.freq_scale;
    a.K = p.K;
    a.pro = p.pro;
    a.nslots = p.nslots < 1 ? 1 : p.nslots;
    a.attn_nsplit = p.attn_nsplit;
    a.attn_stride = p.attn.n_head * p.attn.head_dim;
    a.n_rot = p.n_rot;
    a.head_dim = p.head_dim > 0 ? p.head_dim : 1;
    a.kv_dim = p.kv_dim;
    a.stamps = p.stamps;
    // default: prologue waves (order 4; +2 % decode over order 0 on two boxes)
    a.order = 4;
    a.pre = 8;
    // order 4 (prologue waves): not for the GPT-2 launches (LayerNorm) nor a WO launch that adds
    // the splits of a long-context attention; too wide to stage -> order 0
    if (a.order == 4 && (key.tag == 2 || p.pro == PRO_LAYERNORM || (p.pro == PRO_ATTN && p.attn_nsplit != 1))) a.order = 0;
    {
        const int nb = p.K / 256;
        // 8 from K = 4096 up: 556 vs 548 tok/s against ceil(nb/4) = 4 on the 7B, same box; 2 prologue
        // waves: 455.  Narrower K keeps ceil(nb/4), the r04 rule it was measured with
        a.npro = nb >= 16 ? 8 : (nb + 3) / 4;
        a.npro = std::max(1, std::min(a.npro, std::min(GV_NW - 2, nb)));
    }
    a.stage_off = (int)((gv_lds_bytes(p.K / 256, a.nslots, p.n_rot) + 15) & ~(size_t)15);
    a.flag_off = a.stage_off + gv_stage_arrays(p.pro, a.nslots) * (p.K / 256) * 1024;
    if (a.order == 4 && gv_lds_total(a, p.K / 256, p.pro) > GV_LDS_MAX) a.order = 0;
    for (int i = 0; i < p.nseg; ++i)
        if (p.seg[i].epi == EPI_QKV && (!p.tokpos || (p.n_rot > 0 && p.head_dim <= 0)))
            throw Error("gemv: QKV epilogue needs tokpos and the head geometry");
    if (gv_lds_total(a, p.K / 256, p.pro) > GV_LDS_MAX) throw Error("gemv: activation too large for LDS");
    grid_out = blk;
}

void launch_gemv(const GemvParams& p, hipStream_t s, hipEvent_t ev_start, hipEvent_t ev_stop) {
    GvArgs a;
    GvKey key;
    int grid = 0;
    gv_prepare(p, gv_grid_cap(), a, grid, key);
    GvFn fn = gv_fn(key.nseg, key.t0, key.t1, key.rw, key.kb, key.tag);
    if (!fn) throw Error("gemv: no kernel for this type / shape");
    const size_t smem = gv_lds_total(a, p.K / 256, p.pro);
    if (ev_start || ev_stop)
        hipExtLaunchKernelGGL(fn, dim3(grid), dim3(GV_NW * 64), smem, s, ev_start, ev_stop, 0, a);
    else
        hipLaunchKernelGGL(fn, dim3(grid), dim3(GV_NW * 64), smem, s, a);
    MI_HIP(hipGetLastError());
}

}  // namespace mi
