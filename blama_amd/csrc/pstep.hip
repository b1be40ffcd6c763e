// Persistent batch-1 decode step (gfx950, wave64): every layer of one dense LLaMA token in ONE
// launch -- the hot path of SURVEY.md §8a rows a5-a13 (RMSNorm, quantised mul_mat, RoPE, KV
// append, KQ / softmax / KQV, residual adds, SwiGLU) behind Session::doDecode's llama_decode
// (/root/reference/inference/code/llama/Session.cpp:381-392).
//
// Why one launch.  The launch form of the step (dgemv.hip) pays, per layer, eight dependent kernel
// boundaries (Q/K/V, attention, WO, FFN gate/up, FFN down and three activation quantisations),
// and HBM idles at every one of them while the next kernel's weight loads ramp up.  Here one
// workgroup per CU (grid = the CU count, all co-resident) runs the whole step:
//   * wave 0 is the LOADER: it streams this CU's share of every matrix of every layer, in the
//     order the step consumes them, into a ring of PS_NSLOT LDS slots by LDS-DMA
//     (global_load_lds_dwordx4, nt), running ahead of every data dependency by up to the ring --
//     the weight stream never stops for a hand-off;
//   * waves 1..7 are CONSUMERS: they gather each op's input from the other CUs, build the Q8_K
//     activation in LDS (RMSNorm in double + quantize_row_q8_K, bit for bit the CPU's rules),
//     run the per-superblock integer dots of their rows out of the ring (Kq<T>::dot, the same
//     arithmetic and lane order as dgemv_kernel) and publish their outputs.
// Hand-offs between CUs are 8-byte {tag, value} granules written by one sc1 store and swept by the
// consumers with sc1 loads until every tag equals the edge's epoch (MI355X guide, Guideline 16
// R2): no flags, fences or grid barriers.  Epoch = f(step counter, layer, edge): unique per step
// (the embedding launch counts steps), so nothing is re-zeroed between launches.  Every spin is
// bounded: on a timeout the wave writes a code to the host-mapped error word and exits; the host
// rolls the step back and the context returns to the launch form.
//
// Per layer (CU c, NCU CUs; units of an op split evenly, contiguous):
//   E_X   gather x (layer 0: the embedding row) -> rms_norm * attn_norm -> Q8_K (LDS)
//   QKV   RoPE pairs of the Q|K|V rows: q / k / v granules, f16 K / V rows into the cache
//   ATT   CUs c < n_embd/256: the q heads of output block c (exact softmax, f16 p, as attn_fused),
//         the block quantised to Q8_K and published as 81 granules (64 words, 16 bsums, d)
//   E_ATT gather the quantised attention output (WO's activation)
//   WO    x_a = y + x (residual) -> granules
//   E_XA  gather x_a -> rms_norm * ffn_norm -> Q8_K
//   GU    h = silu(gate) * up -> granules
//   E_H   gather h -> Q8_K
//   DN    x = y + x_a -> granules (the next layer's E_X); the last layer also stores x for the head
#include "qdot.h"

#include <algorithm>
#include <cstring>
#include <vector>

namespace mi {

namespace {

typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(3))) int lint;
typedef __attribute__((address_space(3))) char lchar;

constexpr int PS_NW = 8;           // waves per workgroup: 0 loader, 1..7 consumers
constexpr int PS_NC = PS_NW - 1;
constexpr int PS_NSLOT = 8;        // LDS ring slots at most (PsArgs::nslot; FULL / FREE words)
constexpr int PS_DEPTH = 3;        // slot fills the loader keeps in flight
constexpr int PS_MU = 2;           // units per consumer wave per slot (ups <= PS_NC * PS_MU)
constexpr int PS_MAXRES = 64;      // residual rows per CU (WO / down units)
constexpr int PS_MB = 8;           // activation blocks per consumer wave (K <= 7 * 8 * 256 = 14336)
constexpr int PS_ATT_W = 81;       // granules per quantised attention block: 64 q words, 16 bsums, d
constexpr int PS_CTL = 1024;       // LDS control block
constexpr unsigned long long PS_TIMEOUT = 25000000ull;   // 0.25 s of the 100 MHz real-time clock

enum { E_X = 0, E_QKV = 1, E_ATT = 2, E_XA = 3, E_H = 4, E_N = 8 };

}  // namespace

enum { PS_R_QKV = 0, PS_R_WO = 1, PS_R_GU = 2, PS_R_DN = 3 };

// ---- the step's plan (device memory, read-only during the launch) ----
struct PsOp {
    const uint8_t* a[4];      // planes of A
    const uint8_t* b[4];      // planes of B (gate/up: up)
    int type, role;           // role: PS_R_*
    int rows, units, ups;     // rows of A; units (QKV: RoPE pairs; GU: pairs; WO/DN: rows); units per slot
    int row0;                 // QKV: first row of this group within the layer's Q|K|V rows
    int K, nb, C;             // input length, superblocks, 8-superblock chunks per row
};
struct PsLayer {
    PsOp op[5];
    int n_op;
    const float* attn_norm;
    const float* ffn_norm;
    __half* kc;               // this layer's caches [n_ctx][kv_dim]
    __half* vc;
};

namespace {

// ------------------------------------------------------------------ helpers ----
// the plan is read-only for the launch: read it through the constant address space, so that it
// lands in SGPRs by scalar loads (a vector load would make the loader wait for its LDS-DMA)
template <typename T>
__device__ __forceinline__ T ld_const(const T* p) {
#if defined(__HIP_DEVICE_COMPILE__)
    return *(const __attribute__((address_space(4))) T*)(p);
#else
    return *p;
#endif
}
__device__ __forceinline__ unsigned long long rt_now() { return __builtin_amdgcn_s_memrealtime(); }

struct Guard {                 // bounded spin: false (and the error word set) after PS_TIMEOUT
    unsigned long long t0;
    unsigned n;
    __device__ Guard() : t0(0), n(0) {}
    __device__ bool ok(unsigned* err, unsigned code) {
        __builtin_amdgcn_s_sleep(1);
        if ((++n & 15) != 0) return true;
        const unsigned long long t = rt_now();
        if (t0 == 0) t0 = t;
        if (t - t0 < PS_TIMEOUT) return true;
        __hip_atomic_store(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return false;
    }
};

// the lane id, re-derived where it is used: a volatile asm cannot be hoisted, so the many inlined
// GEMV variants do not keep their lane-dependent constants alive across the whole step (spills)
__device__ __forceinline__ int fresh_lane() {
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

// two f16 (round to nearest even), the first in the low half: a K / V cache pair
__device__ __forceinline__ unsigned pack_h2(float a, float b) {
    return (unsigned)__half_as_ushort(__float2half_rn(a)) | ((unsigned)__half_as_ushort(__float2half_rn(b)) << 16);
}

__device__ __forceinline__ void lds_wait() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// wait until at most n vector-memory operations of this wave are outstanding (0..63)
__device__ __forceinline__ void vm_wait(int n) {
#define VMW(k) case k: __builtin_amdgcn_s_waitcnt(((k) & 15) | (((k) >> 4) << 14) | (0x7 << 4) | (0xF << 8)); break;
#define VMW8(b) VMW(b) VMW(b + 1) VMW(b + 2) VMW(b + 3) VMW(b + 4) VMW(b + 5) VMW(b + 6) VMW(b + 7)
    switch (n < 0 ? 0 : n > 63 ? 63 : n) {
        VMW8(0) VMW8(8) VMW8(16) VMW8(24) VMW8(32) VMW8(40) VMW8(48) VMW8(56)
    }
#undef VMW8
#undef VMW
}

// LDS words the loader touches, in inline asm: the compiler would otherwise wait for every
// outstanding LDS-DMA (vmcnt(0)) before each, as they might alias
__device__ __forceinline__ int lds_ld_asm(const lint* p) {
    int v;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    return v;
}
__device__ __forceinline__ void lds_st_asm(lint* p, int v) {
    asm volatile("ds_write_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : : "v"(p), "v"(v) : "memory");
}

__device__ __forceinline__ void put_granule(unsigned long long* g, unsigned tag, unsigned v) {
    __hip_atomic_store((gu64*)(g), ((unsigned long long)tag << 32) | v, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t g_rsrc(const unsigned long long* g) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned long long*>(g), 0, 0x7FFFFFFF, 0x00020000);
}
// two granules (16 B, sc1: past this CU's L1 to the coherent copy)
__device__ __forceinline__ u32x4 ld_gran2(__amdgpu_buffer_rsrc_t r, unsigned idx) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, idx * 8u, 0, 16);
}
__device__ __forceinline__ unsigned long long ld_gran(const unsigned long long* g, unsigned idx) {
    return __hip_atomic_load((const gu64*)(g) + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Q8_K of one 256-block held as 4 consecutive values per lane (quantize_row_q8_K_ref: the
// signed value at the FIRST index of the largest |x|, iscale = -127/max, q = min(127,
// nearest(iscale x)), d = 1/iscale); returns the packed q word, the 16-element sum in lanes
// 4k (bsum k) and d
struct Q8kLane {
    int packed, bsum;
    float d;
};
__device__ __forceinline__ Q8kLane q8k_lane(const float v[4], int lane) {
    const float a0 = fabsf(v[0]), a1 = fabsf(v[1]), a2 = fabsf(v[2]), a3 = fabsf(v[3]);
    const float amax = wave_max_pos(fmaxf(fmaxf(a0, a1), fmaxf(a2, a3)));
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
    Q8kLane r;
    r.d = zero ? 0.0f : 1.0f / iscale;
    r.packed = (q[0] & 0xFF) | ((q[1] & 0xFF) << 8) | ((q[2] & 0xFF) << 16) | ((q[3] & 0xFF) << 24);
    int sm = q[0] + q[1] + q[2] + q[3];
    sm += dpp_i<0xB1, 0xf>(sm);
    sm += dpp_i<0x4E, 0xf>(sm);
    r.bsum = sm;
    (void)lane;
    return r;
}

// ------------------------------------------------------------ LDS weights ----
// a row's planes inside a ring slot (LDS pointers)
struct LRow {
    const lchar* p[4];
};
template <int T> struct Lq;
template <> struct Lq<T_Q4_K> {
    __device__ static Kq<T_Q4_K>::Ld ld(const LRow& r, int sb, int j) {
        Kq<T_Q4_K>::Ld l;
        l.qs = *reinterpret_cast<const __attribute__((address_space(3))) u32x4*>(r.p[0] + sb * 128 + j * 16);
        l.hdr = *reinterpret_cast<const __attribute__((address_space(3))) u32x4*>(r.p[1] + sb * 16);
        return l;
    }
};
template <> struct Lq<T_Q5_K> {
    __device__ static Kq<T_Q5_K>::Ld ld(const LRow& r, int sb, int j) {
        Kq<T_Q5_K>::Ld l;
        l.qs = *reinterpret_cast<const __attribute__((address_space(3))) u32x4*>(r.p[0] + sb * 128 + j * 16);
        l.qh = *reinterpret_cast<const __attribute__((address_space(3))) u32x4*>(r.p[1] + sb * 32 + (j & 1) * 16);
        l.hdr = *reinterpret_cast<const __attribute__((address_space(3))) u32x4*>(r.p[2] + sb * 16);
        return l;
    }
};
template <> struct Lq<T_Q6_K> {
    __device__ static Kq<T_Q6_K>::Ld ld(const LRow& r, int sb, int j) {
        Kq<T_Q6_K>::Ld l;
        const int h = j >> 2, half = j & 1;
        l.ql = *reinterpret_cast<const __attribute__((address_space(3))) u32x4*>(r.p[0] + sb * 128 + j * 16);
        l.qh = *reinterpret_cast<const __attribute__((address_space(3))) u32x4*>(r.p[1] + sb * 64 + 32 * h + 16 * half);
        const __attribute__((address_space(3))) unsigned* sc =
            reinterpret_cast<const __attribute__((address_space(3))) unsigned*>(r.p[2] + sb * 16 + 8 * h);
        l.sc0 = sc[0];
        l.sc1 = sc[1];
        l.d = *reinterpret_cast<const __attribute__((address_space(3))) unsigned short*>(r.p[3] + sb * 2);
        return l;
    }
};

// ---- slot geometry: rows [ra, rb) of each matrix of the op, planes in order, each plane's
// bytes [align_down(ra RB), align_up(rb RB)) (16-B aligned regions; the arena pads every plane)
__device__ __forceinline__ int rows_per_unit(int role) { return role == PS_R_QKV ? 2 : 1; }
__device__ __forceinline__ int n_mats(int role) { return role == PS_R_GU ? 2 : 1; }

// plane p's region of rows [ra, rb) of matrix m: LDS offset (from the slot) and source bytes
struct Region {
    int off, lo, bytes;
};

}  // namespace

// ------------------------------------------------------------------ kernel ----
struct PsArgs {
    const PsLayer* layers;
    int n_layer, n_embd, n_ff, n_head, n_head_kv, head_dim, kv_dim, n_rot;
    float eps, theta_scale, freq_scale, kq_scale;
    const float* freq_factors;
    const int* tokpos;         // {token, pos, cell, -}
    int* cell_pos;
    const unsigned* step;      // decode steps so far (the embedding launch increments it first)
    const float* xin;          // the embedding row
    float* xout;               // the residual after the last layer (the head's input)
    unsigned long long* g_x;   // granules: x after down [n_embd]
    unsigned long long* g_qkv; // q | k | v [n_embd + 2 kv_dim]
    unsigned long long* g_att; // quantised attention output [n_embd / 256][PS_ATT_W]
    unsigned long long* g_xa;  // x after WO [n_embd]
    unsigned long long* g_h;   // FFN [n_ff]
    unsigned* err;             // host-mapped: a spin gave up (the step is invalid)
    unsigned long long* stamps; // diagnostics: [ncu][16] s_memrealtime stamps of layer stamp_layer (null: off)
    int stamp_layer;
    int slot_bytes;            // ring slot size
    int nslot;                 // ring slots
    int act_off;               // LDS offset of the activation / attention scratch region
    int ctl_off;               // LDS offset of the control block
};

namespace {

struct Ctl {                   // LDS control block layout (offsets from ctl_off)
    static constexpr int FULL = 0;        // int[PS_NSLOT]: fill seq + 1 of the slot's data
    static_assert(PS_NSLOT * 4 <= 32, "FULL / FREE words");
    static constexpr int FREE = 32;       // int[PS_NSLOT]: consumer releases of the slot
    static constexpr int SYNC = 64;       // int: consumer barrier counter
    static constexpr int GATH = 68;       // int: consumer waves sweeping another CU's data (the loader thins)
    static constexpr int RED = 128;       // double[8]: per-wave norm partials
    static constexpr int RES = 256;       // float[PS_MAXRES]: residual rows of this CU
    static constexpr int MISC = 512;      // float[PS_NC][4]: attention maxima
    static constexpr int DRED = 640;      // double[PS_NC][4]: attention sums
};

__device__ __forceinline__ void unit_span(int units, int cu, int ncu, int& u0, int& u1) {
    u0 = (int)(((long long)units * cu) / ncu);
    u1 = (int)(((long long)units * (cu + 1)) / ncu);
}

// the regions of a slot holding units [ua, ub) of op (wave-uniform arithmetic)
__device__ __forceinline__ int slot_regions(const PsOp& op, int ua, int ub, Region (&rg)[2][4]) {
    const int rpu = rows_per_unit(op.role);
    const int ra = ua * rpu, rb = min(ub * rpu, op.rows);
    const int np = op.type == T_Q4_K ? 2 : op.type == T_Q5_K ? 3 : 4;
    int off = 0;
    for (int m = 0; m < 2; ++m) {
        for (int p = 0; p < 4; ++p) {
            rg[m][p] = Region{off, 0, 0};
            if (m >= n_mats(op.role) || p >= np) continue;
            const int pb = (op.type == T_Q4_K ? (p == 0 ? 128 : 16)
                          : op.type == T_Q5_K ? (p == 0 ? 128 : p == 1 ? 32 : 16)
                          : (p == 0 ? 128 : p == 1 ? 64 : p == 2 ? 16 : 2)) * op.nb;
            const long long lo = ((long long)ra * pb) & ~15LL;
            const long long hi = ((long long)rb * pb + 15) & ~15LL;
            rg[m][p].lo = (int)lo;   // (plane offsets of one matrix fit in 31 bits: < 2 GB per plane)
            rg[m][p].bytes = (int)(hi - lo);
            off += (int)(hi - lo);
        }
    }
    return off;
}

// ---- the loader (wave 0) ----
__device__ __forceinline__ void ps_loader(const PsArgs& a, lchar* smem, int cu, int ncu) {
    const int lane = threadIdx.x & 63;
    const int nslot = a.nslot;
    lint* full = reinterpret_cast<lint*>(smem + a.ctl_off + Ctl::FULL);
    lint* fre = reinterpret_cast<lint*>(smem + a.ctl_off + Ctl::FREE);
    // fills in flight (up to PS_DEPTH): fill seq - nin .. seq - 1, c0 the oldest's DMA count
    int seq = 0, nin = 0, c0 = 0, c1 = 0, c2 = 0;
    auto mark_oldest = [&](int younger) {   // wait for the oldest in-flight fill, publish it
        vm_wait(younger);
        const int f = seq - nin;
        lds_st_asm(full + f % nslot, f + 1);
        c0 = c1;
        c1 = c2;
        --nin;
    };
    Guard g;
    for (int l = 0; l < a.n_layer; ++l) {
        const PsLayer* Lp = a.layers + l;
        const int n_op = ld_const(&Lp->n_op);
        if (a.stamps && l == a.stamp_layer && lane == 0) a.stamps[blockIdx.x * 16 + 13] = rt_now();
        for (int o = 0; o < n_op; ++o) {
            const PsOp op = ld_const(Lp->op + o);
            int u0, u1;
            unit_span(op.units, cu, ncu, u0, u1);
            for (int ua = u0; ua < u1; ua += op.ups) {
                const int ub = min(u1, ua + op.ups);
                const int s = seq % nslot, use = seq / nslot;
                if (use > 0 && lds_ld_asm(fre + s) < use * PS_NC) {
                    // the slot's previous data is still being read: publish what is in flight
                    // first, then wait for the release
                    while (nin > 0) mark_oldest(nin == 3 ? c1 + c2 : nin == 2 ? c1 : 0);
                    while (lds_ld_asm(fre + s) < use * PS_NC)
                        if (!g.ok(a.err, 0x101)) return;
                }
                Region rg[2][4];
                slot_regions(op, ua, ub, rg);
                lchar* dst = smem + s * a.slot_bytes;
                int cnt = 0;
#pragma unroll
                for (int m = 0; m < 2; ++m) {
#pragma unroll
                    for (int p = 0; p < 4; ++p) {
                        const int nbytes = rg[m][p].bytes;
                        if (nbytes == 0) continue;
                        const uint8_t* src = (m ? op.b[p] : op.a[p]) + rg[m][p].lo;
                        src = rfl_ptr(src);
                        for (int i0 = 0; i0 < nbytes; i0 += 1024) {
                            if (i0 + lane * 16 < nbytes)
                                __builtin_amdgcn_global_load_lds(
                                    gptr(reinterpret_cast<const unsigned*>(src + i0 + lane * 16)),
                                    (__attribute__((address_space(3))) void*)(dst + rg[m][p].off + i0), 16, 0, 2);
                            ++cnt;
                        }
                    }
                }
                if (nin == 0) c0 = cnt;
                else if (nin == 1) c1 = cnt;
                else c2 = cnt;
                ++nin;
                ++seq;
                if (nin == PS_DEPTH) mark_oldest(c1 + c2);   // PS_DEPTH 3: the two younger stay in flight
            }
        }
    }
    while (nin > 0) mark_oldest(nin == 3 ? c1 + c2 : nin == 2 ? c1 : 0);
    if (a.stamps && lane == 0) a.stamps[blockIdx.x * 16 + 14] = rt_now();
}

// ---- consumer-wave barrier (the loader never joins: LDS counter) ----
struct CSync {
    lint* ctr;
    int gen;
    __device__ bool wait(unsigned* err, unsigned code) {
        gen += PS_NC;
        lds_wait();
        if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        Guard g;
        while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < gen)
            if (!g.ok(err, code)) return false;
        asm volatile("" ::: "memory");
        return true;
    }
};

// ---- gather a float vector of nb 256-blocks: consumer wave cw holds blocks cw + 7 i, 4 values per lane
// (elements 256 b + 4 lane ..); from granules (tag) or, g == null, plain from x
template <int MB>
__device__ __forceinline__ bool gather_vec(const unsigned long long* g, const float* x, int nb, unsigned tag, int cw, int lane,
                           float (&v)[MB][4], unsigned* err, unsigned code) {
    lane = fresh_lane();
    if (!g) {
#pragma unroll
        for (int i = 0; i < MB; ++i) {
            const int b = cw + PS_NC * i;
            if (b < nb) {
                const f32x4 t = gptr(reinterpret_cast<const f32x4*>(x))[b * 64 + lane];
                v[i][0] = t.x; v[i][1] = t.y; v[i][2] = t.z; v[i][3] = t.w;
            }
        }
        return true;
    }
    const __amdgpu_buffer_rsrc_t r = g_rsrc(g);
    unsigned pend = 0;
#pragma unroll
    for (int i = 0; i < MB; ++i)
        if (cw + PS_NC * i < nb) pend |= 1u << i;
    Guard gd;
    while (pend) {
        u32x4 q0[MB], q1[MB];
#pragma unroll
        for (int i = 0; i < MB; ++i)
            if (pend & (1u << i)) {
                const unsigned idx = (unsigned)((cw + PS_NC * i) * 256 + lane * 4);
                q0[i] = ld_gran2(r, idx);
                q1[i] = ld_gran2(r, idx + 2);
            }
#pragma unroll
        for (int i = 0; i < MB; ++i)
            if (pend & (1u << i)) {
                const bool ok = q0[i].y == tag && q0[i].w == tag && q1[i].y == tag && q1[i].w == tag;
                if (__all(ok)) {
                    v[i][0] = __uint_as_float(q0[i].x);
                    v[i][1] = __uint_as_float(q0[i].z);
                    v[i][2] = __uint_as_float(q1[i].x);
                    v[i][3] = __uint_as_float(q1[i].z);
                    pend &= ~(1u << i);
                }
            }
        if (pend && !gd.ok(err, code)) return false;
    }
    return true;
}

// The activation of the next op from the gathered vector: rms_norm(v) * nw (nw set) or v, Q8_K into
// the LDS act region (act_layout(K, 1, 0)); the residual rows [r0, r1) of this CU into RES.
// Two consumer barriers: every wave is done with the previous activation before it is overwritten,
// and the new one is complete before any wave reads it.
template <int MB>
__device__ __forceinline__ bool build_act(const PsArgs& a, lchar* smem, CSync& cs, float (&v)[MB][4], const f32x4 (&w)[MB], int nb,
                          const float* nw, int r0, int r1, int cw, int lane, unsigned code) {
    lane = fresh_lane();
    __attribute__((address_space(3))) double* lred =
        reinterpret_cast<__attribute__((address_space(3))) double*>(smem + a.ctl_off + Ctl::RED);
    if (nw) {
        double s = 0.0;
#pragma unroll
        for (int i = 0; i < MB; ++i)
            if (cw + PS_NC * i < nb)
#pragma unroll
                for (int k = 0; k < 4; ++k) s += (double)(v[i][k] * v[i][k]);
        s = wave_sum63_d(s);
        if (lane == 63) lred[cw] = s;
    }
    if (!cs.wait(a.err, code)) return false;   // (1) the previous activation is no longer read
    float scale = 1.0f;
    if (nw) {
        double tot = 0.0;
#pragma unroll
        for (int k = 0; k < PS_NC; ++k) tot += lred[k];
        scale = 1.0f / sqrtf((float)(tot / (double)(nb * 256)) + a.eps);
    }
    const int K = nb * 256;
    lchar* act = smem + a.act_off;
    __attribute__((address_space(3))) float* res =
        reinterpret_cast<__attribute__((address_space(3))) float*>(smem + a.ctl_off + Ctl::RES);
#pragma unroll
    for (int i = 0; i < MB; ++i) {
        const int b = cw + PS_NC * i;
        if (b >= nb) continue;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int e = b * 256 + lane * 4 + k;
            if (e >= r0 && e < r1) res[e - r0] = v[i][k];
        }
        float y[4] = {v[i][0], v[i][1], v[i][2], v[i][3]};
        if (nw) {   // ggml_vec_scale_f32 then ggml_mul
            y[0] = (y[0] * scale) * w[i].x;
            y[1] = (y[1] * scale) * w[i].y;
            y[2] = (y[2] * scale) * w[i].z;
            y[3] = (y[3] * scale) * w[i].w;
        }
        const Q8kLane q = q8k_lane(y, lane);
        reinterpret_cast<lint*>(act + b * 256)[lane] = q.packed;
        if ((lane & 3) == 0) reinterpret_cast<lint*>(act + K)[b * 16 + (lane >> 2)] = q.bsum;
        if (lane == 0) reinterpret_cast<__attribute__((address_space(3))) float*>(act + K + nb * 64)[b] = q.d;
        __builtin_amdgcn_sched_barrier(0);   // one block at a time (interleaving them all spills)
    }
    return cs.wait(a.err, code + 1);   // (2) the activation is complete
}

// ---- one op's slots for consumer wave cw: loads of its units from the ring, release, dots, epilogue
struct OpCtx {
    int seq;          // ring fills consumed so far
    unsigned tag_out; // the tag of this op's outputs
    int res0;         // first unit of this CU's WO / down rows (RES index base)
    int last;         // the last layer (down also stores x)
    int l;
};

template <int T, int ROLE, int C>
__device__ __forceinline__ bool ps_op(const PsArgs& a, const PsLayer& L, const PsOp& op, lchar* smem, OpCtx& oc, int cu, int ncu,
                      int cw, int lane) {
    using KQ = Kq<T>;
    constexpr int RW = (ROLE == PS_R_QKV || ROLE == PS_R_GU) ? 2 : 1;
    lane = fresh_lane();
    const int sbl = lane >> 3, j = lane & 7;
    const int nb = op.nb;
    lint* full = reinterpret_cast<lint*>(smem + a.ctl_off + Ctl::FULL);
    lint* fre = reinterpret_cast<lint*>(smem + a.ctl_off + Ctl::FREE);
    const __attribute__((address_space(3))) float* res =
        reinterpret_cast<const __attribute__((address_space(3))) float*>(smem + a.ctl_off + Ctl::RES);
    const lchar* actb = smem + a.act_off;
    Act av;
    av.q8k = (const int8_t*)(actb);
    av.bsum = (const int*)(actb + nb * 256);
    av.dk = (const float*)(actb + nb * 256 + nb * 64);
    int u0, u1;
    unit_span(op.units, cu, ncu, u0, u1);
    i32x4 tp = {0, 0, 0, 0};
    if (ROLE == PS_R_QKV) tp = *gptr(reinterpret_cast<const i32x4*>(a.tokpos));
    // the activation slices this lane's dots read (the same for every row): once per op
    typename KQ::AR ar[C];
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const int sb0 = 8 * c + sbl;
        ar[c] = KQ::act(av, sb0 < nb ? sb0 : nb - 1, j);
    }
    for (int ua = u0; ua < u1; ua += op.ups) {
        const int ub = min(u1, ua + op.ups);
        const int s = oc.seq % a.nslot;
        {
            Guard g;
            while (__hip_atomic_load(full + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != oc.seq + 1)
                if (!g.ok(a.err, 0x110)) return false;
            asm volatile("" ::: "memory");
        }
        Region rg[2][4];
        slot_regions(op, ua, ub, rg);
        const lchar* sbase = smem + s * a.slot_bytes;
        // this wave's units of the slot: u = ua + cw + 7 k.  Each unit's weights are read from the
        // slot into registers, the slot released after the wave's last unit is read, then its dots
        const int nmine = ub - ua > cw ? (ub - ua - cw + PS_NC - 1) / PS_NC : 0;
        if (nmine == 0) {
            if (lane == 0) __hip_atomic_fetch_add(fre + s, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        oc.seq++;
        for (int k = 0; k < nmine; ++k) {
            const int u = ua + cw + PS_NC * k;
            typename KQ::Ld w[RW][C];
#pragma unroll
            for (int r = 0; r < RW; ++r) {
                const int m = ROLE == PS_R_GU ? r : 0;
                const int row = ROLE == PS_R_GU ? u : (ROLE == PS_R_QKV ? 2 * u + r : u);
                const int rr = min(row, op.rows - 1);
                LRow lr;
#pragma unroll
                for (int p = 0; p < 4; ++p) {
                    const int pb = (T == T_Q4_K ? (p == 0 ? 128 : 16)
                                  : T == T_Q5_K ? (p == 0 ? 128 : p == 1 ? 32 : 16)
                                  : (p == 0 ? 128 : p == 1 ? 64 : p == 2 ? 16 : 2)) * nb;
                    lr.p[p] = sbase + rg[m][p].off + ((long long)rr * pb - rg[m][p].lo);
                }
#pragma unroll
                for (int c = 0; c < C; ++c) {
                    const int sb = 8 * c + sbl;
                    w[r][c] = Lq<T>::ld(lr, sb < nb ? sb : nb - 1, j);
                }
            }
            if (k == nmine - 1) {   // the slot's bytes this wave needs are in registers: release it
                lds_wait();
                if (lane == 0) __hip_atomic_fetch_add(fre + s, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            float y[RW];
#pragma unroll
            for (int r = 0; r < RW; ++r) {
                float acc = 0.0f;
#pragma unroll
                for (int c = 0; c < C; ++c) {
                    const int sb0 = 8 * c + sbl;
                    const float p = KQ::dot(w[r][c], ar[c], j);
                    acc += sb0 < nb ? p : 0.0f;
                }
                y[r] = wave_sum63(acc);
            }
            if (lane != 63) continue;
            if (ROLE == PS_R_QKV) {
                const int R = op.row0 + 2 * u;   // row within Q | K | V
                float o0 = y[0], o1 = y[RW - 1];
                const bool isq = R < a.n_embd, isk = !isq && R < a.n_embd + a.kv_dim;
                const int i0 = (isq ? R : R - a.n_embd) % a.head_dim;
                if ((isq || isk) && i0 < a.n_rot) {   // ggml_rope_cache_init (ext_factor 0, mscale 1), then rotate
                    const float ff = a.freq_factors ? gptr(a.freq_factors)[i0 / 2] : 1.0f;
                    float theta = (float)tp.y;
                    for (int k2 = 0; k2 < i0 / 2; ++k2) theta = theta * a.theta_scale;
                    const float th = a.freq_scale * (theta / ff);
                    const float cs = cosf(th), sn = sinf(th);
                    o0 = y[0] * cs - y[RW - 1] * sn;
                    o1 = y[0] * sn + y[RW - 1] * cs;
                }
                const int cell = tp.z;
                if (isk) {
                    const int rk = R - a.n_embd;
                    *gptr_w(reinterpret_cast<unsigned*>(L.kc + (long long)cell * a.kv_dim + rk)) = pack_h2(o0, o1);
                    if (rk == 0) *gptr_w(a.cell_pos + cell) = tp.y;
                } else if (!isq) {
                    const int rv = R - a.n_embd - a.kv_dim;
                    *gptr_w(reinterpret_cast<unsigned*>(L.vc + (long long)cell * a.kv_dim + rv)) = pack_h2(o0, o1);
                }
                put_granule(a.g_qkv + R, oc.tag_out, __float_as_uint(o0));
                put_granule(a.g_qkv + R + 1, oc.tag_out, __float_as_uint(o1));
            } else if (ROLE == PS_R_GU) {
                put_granule(a.g_h + u, oc.tag_out, __float_as_uint(silu_f(y[0]) * y[RW - 1]));
            } else {   // WO / down: the residual add
                const float xo = y[0] + res[u - oc.res0];
                if (ROLE == PS_R_WO) {
                    put_granule(a.g_xa + u, oc.tag_out, __float_as_uint(xo));
                } else {
                    put_granule(a.g_x + u, oc.tag_out, __float_as_uint(xo));
                    if (oc.last) *gptr_w(a.xout + u) = xo;
                }
            }
        }
    }
    return true;
}

template <int T, int ROLE>
__device__ __forceinline__ bool ps_op_c(const PsArgs& a, const PsLayer& L, const PsOp& op, lchar* smem, OpCtx& oc, int cu, int ncu,
                        int cw, int lane) {
    switch (op.C) {
    case 1: return ps_op<T, ROLE, 1>(a, L, op, smem, oc, cu, ncu, cw, lane);
    case 2: return ps_op<T, ROLE, 2>(a, L, op, smem, oc, cu, ncu, cw, lane);
    case 4: return ps_op<T, ROLE, 4>(a, L, op, smem, oc, cu, ncu, cw, lane);
    default: break;
    }
    if constexpr (ROLE == PS_R_DN) {
        switch (op.C) {
        case 3: return ps_op<T, ROLE, 3>(a, L, op, smem, oc, cu, ncu, cw, lane);
        case 6: return ps_op<T, ROLE, 6>(a, L, op, smem, oc, cu, ncu, cw, lane);
        case 7: return ps_op<T, ROLE, 7>(a, L, op, smem, oc, cu, ncu, cw, lane);
        default: break;
        }
    }
    __hip_atomic_store(a.err, 0x1F0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return false;
}
template <int ROLE>
__device__ __forceinline__ bool ps_op_t(const PsArgs& a, const PsLayer& L, const PsOp& op, lchar* smem, OpCtx& oc, int cu, int ncu,
                        int cw, int lane) {
    switch (op.type) {
    case T_Q4_K: return ps_op_c<T_Q4_K, ROLE>(a, L, op, smem, oc, cu, ncu, cw, lane);
    case T_Q5_K: return ps_op_c<T_Q5_K, ROLE>(a, L, op, smem, oc, cu, ncu, cw, lane);
    case T_Q6_K: return ps_op_c<T_Q6_K, ROLE>(a, L, op, smem, oc, cu, ncu, cw, lane);
    default: break;
    }
    __hip_atomic_store(a.err, 0x1F1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return false;
}

// ---- attention of output block blk (q heads [blk hpb, (blk + 1) hpb)) on this CU's consumer waves ----
// The arithmetic of attn_fused_kernel: q rounded to f16, KQ over the f16 cache (this step's cell
// from the Q/K/V granules, rounded to f16 as its cache row is), scale, causal mask by cell position,
// the exact softmax (global max, double sum, p = f16(e * (1 / sum))), sum_c f16(p_c) v_c; then the
// block quantised to Q8_K and published.
template <int HD>
__device__ __forceinline__ bool ps_attention(const PsArgs& a, const PsLayer& L, lchar* smem, CSync& cs, int blk, unsigned tag_qkv,
                             unsigned tag_att, int cw, int lane) {
    constexpr int LPC = HD / 8;            // lanes per cell (8 dims each)
    constexpr int CPW = 64 / LPC;          // cells per wave step
    constexpr int HPB = 256 / HD;          // q heads per output block
    constexpr int KP = HPB >= 4 ? 1 : 8 / HPB;   // wave steps whose cache rows are requested up front
    lane = fresh_lane();
    const int Lh = lane % LPC, G = lane / LPC;
    const int r = a.n_head / a.n_head_kv;
    const i32x4 tp = *gptr(reinterpret_cast<const i32x4*>(a.tokpos));
    const int qpos = tp.y, ncell = min(tp.z + 1, ATTN_SHORT), cnew = tp.z;
    // 0. the cached cells' K / V rows and positions of this wave's first KP steps, all requested
    // before anything waits (under the weight stream every round trip costs microseconds)
    u32x4 kc[KP][HPB], vc[KP][HPB];
    int pc[KP];
#pragma unroll
    for (int k = 0; k < KP; ++k) {
        const int c = cw * CPW + k * PS_NC * CPW + G;
        const int cc = min(c, max(cnew - 1, 0));
        pc[k] = gptr(a.cell_pos)[cc];
#pragma unroll
        for (int t = 0; t < HPB; ++t) {
            const int hk = (blk * HPB + t) / r;
            kc[k][t] = *gptr(reinterpret_cast<const u32x4*>(L.kc + (long long)cc * a.kv_dim + hk * HD + Lh * 8));
            vc[k][t] = *gptr(reinterpret_cast<const u32x4*>(L.vc + (long long)cc * a.kv_dim + hk * HD + Lh * 8));
        }
    }
    // this step's q / k / v of the block's heads (granules; 8 consecutive dims per lane)
    float q[HPB][8], kn[HPB][8], vn[HPB][8];
    {
        const __amdgpu_buffer_rsrc_t rs = g_rsrc(a.g_qkv);
        Guard g;
        for (;;) {
            bool ok = true;
#pragma unroll
            for (int t = 0; t < HPB; ++t) {
                const int hq = blk * HPB + t, hk = hq / r;
                const unsigned iq = (unsigned)(hq * HD + Lh * 8);
                const unsigned ik = (unsigned)(a.n_embd + hk * HD + Lh * 8);
                const unsigned iv = (unsigned)(a.n_embd + a.kv_dim + hk * HD + Lh * 8);
#pragma unroll
                for (int e2 = 0; e2 < 4; ++e2) {
                    const u32x4 gq = ld_gran2(rs, iq + 2 * e2), gk = ld_gran2(rs, ik + 2 * e2), gv = ld_gran2(rs, iv + 2 * e2);
                    ok = ok && gq.y == tag_qkv && gq.w == tag_qkv && gk.y == tag_qkv && gk.w == tag_qkv && gv.y == tag_qkv &&
                         gv.w == tag_qkv;
                    q[t][2 * e2] = __half2float(__float2half_rn(__uint_as_float(gq.x)));
                    q[t][2 * e2 + 1] = __half2float(__float2half_rn(__uint_as_float(gq.z)));
                    kn[t][2 * e2] = __half2float(__float2half_rn(__uint_as_float(gk.x)));
                    kn[t][2 * e2 + 1] = __half2float(__float2half_rn(__uint_as_float(gk.z)));
                    vn[t][2 * e2] = __half2float(__float2half_rn(__uint_as_float(gv.x)));
                    vn[t][2 * e2 + 1] = __half2float(__float2half_rn(__uint_as_float(gv.z)));
                }
            }
            if (__all(ok)) break;
            if (!g.ok(a.err, 0x120)) return false;
        }
    }
    lchar* scr = smem + a.act_off;
    __attribute__((address_space(3))) float* sw = reinterpret_cast<__attribute__((address_space(3))) float*>(scr);
    __attribute__((address_space(3))) float* opart =
        reinterpret_cast<__attribute__((address_space(3))) float*>(scr + HPB * ATTN_SHORT * 4);
    __attribute__((address_space(3))) float* misc =
        reinterpret_cast<__attribute__((address_space(3))) float*>(smem + a.ctl_off + Ctl::MISC);
    __attribute__((address_space(3))) double* dred =
        reinterpret_cast<__attribute__((address_space(3))) double*>(smem + a.ctl_off + Ctl::DRED);
    // 8 f16 of a cache row -> floats
    auto cvt8 = [](const u32x4& w, float (&f)[8]) {
        const unsigned ww[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            f[2 * e] = h2f(ww[e]);
            f[2 * e + 1] = h2f(ww[e] >> 16);
        }
    };
    auto load_row = [&](const __half* cache, int c, int t) {
        const int hk = (blk * HPB + t) / r;
        return *gptr(reinterpret_cast<const u32x4*>(cache + (long long)c * a.kv_dim + hk * HD + Lh * 8));
    };
    // 1. scaled KQ of every cell (LDS), per-head maxima
    float mx[HPB];
#pragma unroll
    for (int t = 0; t < HPB; ++t) mx[t] = -INFINITY;
    const int nsteps = (ncell - cw * CPW + PS_NC * CPW - 1) / (PS_NC * CPW);
    auto score_step = [&](int k, const u32x4 (&kw)[HPB], int pos_c) {
        const int c = cw * CPW + k * PS_NC * CPW + G;
        const bool in = c < ncell;
        const bool isnew = !in || c == cnew;
        const bool valid = in && (isnew ? qpos : pos_c) <= qpos;
#pragma unroll
        for (int t = 0; t < HPB; ++t) {
            float kf[8];
            if (isnew) {
#pragma unroll
                for (int e = 0; e < 8; ++e) kf[e] = kn[t][e];
            } else {
                cvt8(kw[t], kf);
            }
            float d = 0.0f;
#pragma unroll
            for (int e = 0; e < 8; ++e) d = fmaf(q[t][e], kf[e], d);
#pragma unroll
            for (int off = LPC / 2; off > 0; off >>= 1) d += __shfl_xor(d, off, 64);
            const float wv = valid ? d * a.kq_scale : -INFINITY;
            mx[t] = fmaxf(mx[t], wv);
            if (Lh == 0 && in) sw[t * ATTN_SHORT + c] = wv;
        }
    };
#pragma unroll
    for (int k = 0; k < KP; ++k)
        if (k < nsteps) score_step(k, kc[k], pc[k]);
    for (int k = KP; k < nsteps; ++k) {
        const int c = min(cw * CPW + k * PS_NC * CPW + G, max(cnew - 1, 0));
        u32x4 kw[HPB];
#pragma unroll
        for (int t = 0; t < HPB; ++t) kw[t] = load_row(L.kc, c, t);
        score_step(k, kw, gptr(a.cell_pos)[c]);
    }
#pragma unroll
    for (int t = 0; t < HPB; ++t) {
        const float m = wave_max(mx[t]);
        if (lane == 0) misc[cw * 4 + t] = m;
    }
    if (!cs.wait(a.err, 0x130)) return false;
    float M[HPB];
#pragma unroll
    for (int t = 0; t < HPB; ++t) {
        float m = misc[t];
#pragma unroll
        for (int k = 1; k < PS_NC; ++k) m = fmaxf(m, misc[k * 4 + t]);
        M[t] = m;
    }
    // 2. sum of expf(w - max) in double: wave cw takes cells cw*64 + lane + 448 i
#pragma unroll
    for (int t = 0; t < HPB; ++t) {
        double acc = 0.0;
        for (int c = cw * 64 + lane; c < ncell; c += PS_NC * 64) acc += (double)expf(sw[t * ATTN_SHORT + c] - M[t]);
        acc = wave_sum63_d(acc);
        if (lane == 63) dred[cw * 4 + t] = acc;
    }
    if (!cs.wait(a.err, 0x131)) return false;
    float inv[HPB];
#pragma unroll
    for (int t = 0; t < HPB; ++t) {
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < PS_NC; ++k) s += dred[k * 4 + t];
        inv[t] = (float)(1.0 / s);
    }
    // 3. sum_c f16(p_c) v_c, this wave's cells (lane groups), then the waves' partials in order
    float o[HPB][8];
#pragma unroll
    for (int t = 0; t < HPB; ++t)
#pragma unroll
        for (int e = 0; e < 8; ++e) o[t][e] = 0.0f;
    auto pv_step = [&](int k, const u32x4 (&vw)[HPB]) {
        const int c = cw * CPW + k * PS_NC * CPW + G;
        const bool in = c < ncell;
        const int cc = in ? c : cnew;
#pragma unroll
        for (int t = 0; t < HPB; ++t) {
            float vf[8];
            if (cc == cnew) {
#pragma unroll
                for (int e = 0; e < 8; ++e) vf[e] = vn[t][e];
            } else {
                cvt8(vw[t], vf);
            }
            const float p = expf(sw[t * ATTN_SHORT + cc] - M[t]) * inv[t];   // ggml_vec_soft_max_f32, f16 vec_dot_type
            const float pw = in ? __half2float(__float2half_rn(p)) : 0.0f;
#pragma unroll
            for (int e = 0; e < 8; ++e) o[t][e] = fmaf(pw, vf[e], o[t][e]);
        }
    };
#pragma unroll
    for (int k = 0; k < KP; ++k)
        if (k < nsteps) pv_step(k, vc[k]);
    for (int k = KP; k < nsteps; ++k) {
        const int c = min(cw * CPW + k * PS_NC * CPW + G, max(cnew - 1, 0));
        u32x4 vw[HPB];
#pragma unroll
        for (int t = 0; t < HPB; ++t) vw[t] = load_row(L.vc, c, t);
        pv_step(k, vw);
    }
#pragma unroll
    for (int t = 0; t < HPB; ++t)
#pragma unroll
        for (int off = LPC; off < 64; off <<= 1)
#pragma unroll
            for (int e = 0; e < 8; ++e) o[t][e] += __shfl_xor(o[t][e], off, 64);
    if (G == 0) {
#pragma unroll
        for (int t = 0; t < HPB; ++t)
#pragma unroll
            for (int e = 0; e < 8; ++e) opart[cw * 256 + t * HD + Lh * 8 + e] = o[t][e];
    }
    if (!cs.wait(a.err, 0x132)) return false;
    if (cw == 0) {   // the block's 256 outputs (4 per lane), waves added in order, quantised, published
        float v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float s = opart[lane * 4 + k];
#pragma unroll
            for (int w2 = 1; w2 < PS_NC; ++w2) s += opart[w2 * 256 + lane * 4 + k];
            v[k] = s;
        }
        const Q8kLane qb = q8k_lane(v, lane);
        unsigned long long* gb = a.g_att + (long long)blk * PS_ATT_W;
        put_granule(gb + lane, tag_att, (unsigned)qb.packed);
        if ((lane & 3) == 0) put_granule(gb + 64 + (lane >> 2), tag_att, (unsigned)qb.bsum);
        if (lane == 0) put_granule(gb + 80, tag_att, __float_as_uint(qb.d));
    }
    return true;
}

// WO's activation: the quantised attention blocks (nb of them), consumer wave cw taking blocks cw + 7 i
__device__ __forceinline__ bool gather_att(const PsArgs& a, lchar* smem, CSync& cs, int nb, unsigned tag, int cw, int lane) {
    lane = fresh_lane();
    lint* gath = reinterpret_cast<lint*>(smem + a.ctl_off + Ctl::GATH);
    if (lane == 0) __hip_atomic_fetch_add(gath, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    unsigned qv[PS_MB], bs[PS_MB], dv[PS_MB];
    unsigned pend = 0;
#pragma unroll
    for (int i = 0; i < PS_MB; ++i)
        if (cw + PS_NC * i < nb) pend |= 1u << i;
    Guard g;
    while (pend) {
#pragma unroll
        for (int i = 0; i < PS_MB; ++i) {
            if (!(pend & (1u << i))) continue;
            const unsigned base = (unsigned)((cw + PS_NC * i) * PS_ATT_W);
            const unsigned long long x0 = ld_gran(a.g_att, base + lane);
            const unsigned long long x1 = ld_gran(a.g_att, base + 64 + (lane & 15));
            const unsigned long long x2 = ld_gran(a.g_att, base + 80);
            const bool ok = (unsigned)(x0 >> 32) == tag && (unsigned)(x1 >> 32) == tag && (unsigned)(x2 >> 32) == tag;
            if (__all(ok)) {
                qv[i] = (unsigned)x0;
                bs[i] = (unsigned)x1;
                dv[i] = (unsigned)x2;
                pend &= ~(1u << i);
            }
        }
        if (pend && !g.ok(a.err, 0x140)) return false;
    }
    if (lane == 0) __hip_atomic_fetch_add(gath, -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (!cs.wait(a.err, 0x141)) return false;   // every wave is done with the previous activation
    const int K = nb * 256;
    lchar* act = smem + a.act_off;
#pragma unroll
    for (int i = 0; i < PS_MB; ++i) {
        const int b = cw + PS_NC * i;
        if (b >= nb) continue;
        reinterpret_cast<lint*>(act + b * 256)[lane] = (int)qv[i];
        if (lane < 16) reinterpret_cast<lint*>(act + K)[b * 16 + lane] = (int)bs[i];
        if (lane == 0) reinterpret_cast<lint*>(act + K + nb * 64)[b] = (int)dv[i];
    }
    return cs.wait(a.err, 0x142);
}

__device__ __forceinline__ bool ps_layer_attention(const PsArgs& a, const PsLayer& L, lchar* smem, CSync& cs, int blk, unsigned tq,
                                   unsigned ta, int cw, int lane) {
    // every wave is done with QKV's activation before the scores overwrite it
    if (!cs.wait(a.err, 0x12F)) return false;
    lint* gath = reinterpret_cast<lint*>(smem + a.ctl_off + Ctl::GATH);
    if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(gath, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    bool ok = false, known = true;
    switch (a.head_dim) {
    case 64: ok = ps_attention<64>(a, L, smem, cs, blk, tq, ta, cw, lane); break;
    case 128: ok = ps_attention<128>(a, L, smem, cs, blk, tq, ta, cw, lane); break;
    case 256: ok = ps_attention<256>(a, L, smem, cs, blk, tq, ta, cw, lane); break;
    default: known = false; break;
    }
    if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(gath, -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (known) return ok;
    __hip_atomic_store(a.err, 0x1F2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return false;
}

__device__ __forceinline__ void ps_stamp(const PsArgs& a, int l, int k, int cw, int lane) {
    if (a.stamps && l == a.stamp_layer && cw == 0 && lane == 0)
        a.stamps[blockIdx.x * 16 + k] = rt_now();
}

__device__ __forceinline__ unsigned ps_tag(unsigned step, int n_layer, int l, int e) {
    return step * (unsigned)(n_layer * E_N + E_N) + (unsigned)(l * E_N + e) + 1u;
}

// gather a vector edge and build the next activation from it, sized by the blocks per wave
template <int MB>
__device__ __forceinline__ bool edge_mb(const PsArgs& a, lchar* smem, CSync& cs, const unsigned long long* g, const float* x,
                                        int nb, unsigned tag, const float* nw, int r0, int r1, int cw, int lane, unsigned code,
                                        int l, int st) {
    float v[MB][4];
    f32x4 w[MB];   // the norm weight, requested before the gather waits
    if (nw) {
        const int ln = fresh_lane();
#pragma unroll
        for (int i = 0; i < MB; ++i)
            if (cw + PS_NC * i < nb) w[i] = gptr(reinterpret_cast<const f32x4*>(nw))[(cw + PS_NC * i) * 64 + ln];
    }
    lint* gath = reinterpret_cast<lint*>(smem + a.ctl_off + Ctl::GATH);
    if (lane == 0) __hip_atomic_fetch_add(gath, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    const bool ok = gather_vec<MB>(g, x, nb, tag, cw, lane, v, a.err, code);
    if (lane == 0) __hip_atomic_fetch_add(gath, -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (!ok) return false;
    ps_stamp(a, l, st, cw, lane);
    return build_act<MB>(a, smem, cs, v, w, nb, nw, r0, r1, cw, lane, code + 2);
}
__device__ __forceinline__ bool edge(const PsArgs& a, lchar* smem, CSync& cs, const unsigned long long* g, const float* x, int nb,
                                     unsigned tag, const float* nw, int r0, int r1, int cw, int lane, unsigned code, int l,
                                     int st) {
    if (nb <= 3 * PS_NC) return edge_mb<3>(a, smem, cs, g, x, nb, tag, nw, r0, r1, cw, lane, code, l, st);
    if (nb <= 5 * PS_NC) return edge_mb<5>(a, smem, cs, g, x, nb, tag, nw, r0, r1, cw, lane, code, l, st);
    return edge_mb<PS_MB>(a, smem, cs, g, x, nb, tag, nw, r0, r1, cw, lane, code, l, st);
}

__device__ __forceinline__ void ps_consumer(const PsArgs& a, lchar* smem, int cu, int ncu, int cw, int lane) {
    CSync cs{reinterpret_cast<lint*>(smem + a.ctl_off + Ctl::SYNC), 0};
    const unsigned step = *gptr(a.step);
    const int nbe = a.n_embd / 256, nbf = a.n_ff / 256;
    OpCtx oc{0, 0, 0, 0, 0};
    for (int l = 0; l < a.n_layer; ++l) {
        PsLayer L;
        {
            const PsLayer* Lp = a.layers + l;
            L.n_op = ld_const(&Lp->n_op);
            L.attn_norm = ld_const(&Lp->attn_norm);
            L.ffn_norm = ld_const(&Lp->ffn_norm);
            L.kc = ld_const(&Lp->kc);
            L.vc = ld_const(&Lp->vc);
        }
        const PsOp* const ops = a.layers[l].op;
        oc.l = l;
        oc.last = l == a.n_layer - 1;
        // residual rows of this CU (WO / down share one partition of n_embd rows)
        int r0, r1;
        unit_span(a.n_embd, cu, ncu, r0, r1);
        oc.res0 = r0;
        // E_X: the layer input, rms_norm * attn_norm -> Q8_K
        ps_stamp(a, l, 0, cw, lane);
        if (!edge(a, smem, cs, l == 0 ? nullptr : a.g_x, a.xin, nbe, ps_tag(step, a.n_layer, l - 1, E_X), L.attn_norm, r0, r1,
                  cw, lane, 0x150, l, 1))
            return;
        ps_stamp(a, l, 2, cw, lane);
        // Q / K / V groups
        oc.tag_out = ps_tag(step, a.n_layer, l, E_QKV);
        const int nq = L.n_op - 3;
        for (int o = 0; o < nq; ++o)
            if (!ps_op_t<PS_R_QKV>(a, L, ld_const(ops + o), smem, oc, cu, ncu, cw, lane)) return;
        ps_stamp(a, l, 3, cw, lane);
        // attention (CUs 0 .. nbe-1)
        if (cu < nbe) {
            if (!ps_layer_attention(a, L, smem, cs, cu, oc.tag_out, ps_tag(step, a.n_layer, l, E_ATT), cw, lane)) return;
        }
        ps_stamp(a, l, 4, cw, lane);
        if (!gather_att(a, smem, cs, nbe, ps_tag(step, a.n_layer, l, E_ATT), cw, lane)) return;
        ps_stamp(a, l, 5, cw, lane);
        // WO + residual
        oc.tag_out = ps_tag(step, a.n_layer, l, E_XA);
        if (!ps_op_t<PS_R_WO>(a, L, ld_const(ops + nq), smem, oc, cu, ncu, cw, lane)) return;
        ps_stamp(a, l, 6, cw, lane);
        // E_XA: rms_norm * ffn_norm -> Q8_K; the residual of down
        if (!edge(a, smem, cs, a.g_xa, nullptr, nbe, oc.tag_out, L.ffn_norm, r0, r1, cw, lane, 0x160, l, 7)) return;
        ps_stamp(a, l, 8, cw, lane);
        // gate / up + SwiGLU
        oc.tag_out = ps_tag(step, a.n_layer, l, E_H);
        if (!ps_op_t<PS_R_GU>(a, L, ld_const(ops + nq + 1), smem, oc, cu, ncu, cw, lane)) return;
        ps_stamp(a, l, 9, cw, lane);
        // E_H: h -> Q8_K
        if (!edge(a, smem, cs, a.g_h, nullptr, nbf, oc.tag_out, nullptr, 0, 0, cw, lane, 0x170, l, 10)) return;
        ps_stamp(a, l, 11, cw, lane);
        // down + residual
        oc.tag_out = ps_tag(step, a.n_layer, l, E_X);
        if (!ps_op_t<PS_R_DN>(a, L, ld_const(ops + nq + 2), smem, oc, cu, ncu, cw, lane)) return;
        ps_stamp(a, l, 12, cw, lane);
    }
}

__global__ __launch_bounds__(PS_NW * 64) void ps_step_kernel(const PsArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    lchar* smem = (lchar*)(smem_raw);
    const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int cu = blockIdx.x, ncu = gridDim.x;
    // the control block starts zeroed (LDS is not), then the roles split for good
    if (threadIdx.x < 64) reinterpret_cast<lint*>(smem + a.ctl_off)[threadIdx.x] = 0;
    if (a.stamps && threadIdx.x == 0) a.stamps[blockIdx.x * 16 + 15] = rt_now();
    __syncthreads();
    if (wave == 0) ps_loader(a, smem, cu, ncu);
    else ps_consumer(a, smem, cu, ncu, wave - 1, lane);
}

}  // namespace

// ------------------------------------------------------------------- host ----
struct PsStep {
    PsArgs args;
    PsLayer* d_layers = nullptr;
    unsigned long long* gran = nullptr;
    int ncu = 0;
    size_t lds = 0;
    long long bytes = 0;
};

namespace {
int ps_plane_bytes_row(int type, int nb) {
    int s = 0;
    for (int p = 0; p < plane_count(type); ++p) s += plane_sb_bytes(type, p) * nb;
    return s;
}
int ps_chunks(int nb) {
    const int c = (nb + 7) / 8;
    return c == 5 ? 6 : c;
}
}  // namespace

PsStep* ps_create(const PsConfig& c, const std::vector<PsLayerDesc>& layers, std::string* why) {
    auto fail = [&](const std::string& w) -> PsStep* {
        if (why) *why = w;
        return nullptr;
    };
    int dev = 0, ncu = 0;
    MI_HIP(hipGetDevice(&dev));
    MI_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    if (c.n_layer <= 0 || (int)layers.size() != c.n_layer) return fail("layer table");
    if (c.n_embd % 256 || c.n_ff % 256) return fail("n_embd / n_ff not multiples of 256");
    if (c.head_dim != 64 && c.head_dim != 128 && c.head_dim != 256) return fail("head_dim");
    if (c.n_head_kv <= 0 || c.n_head % c.n_head_kv || c.n_head * c.head_dim != c.n_embd) return fail("head geometry");
    const int nbe = c.n_embd / 256, nbf = c.n_ff / 256;
    if (nbe > ncu || nbe > PS_NC * PS_MB || nbf > PS_NC * PS_MB) return fail("activation wider than the gather");
    if ((c.n_embd + ncu - 1) / ncu > PS_MAXRES) return fail("residual rows per CU");
    const int hpb = 256 / c.head_dim;
    const int act_region = std::max(((int)act_layout(std::max(c.n_embd, c.n_ff), 1, 0).slot_bytes + 15) / 16 * 16,
                                    hpb * ATTN_SHORT * 4 + PS_NC * 256 * 4);
    const int lds_max = 160 * 1024;
    const int nslot = 6;
    const int slot = ((lds_max - act_region - PS_CTL) / nslot) & ~1023;
    if (slot < 8192) return fail("LDS");
    auto* s = new PsStep();
    std::vector<PsLayer> hl(c.n_layer);
    long long bytes = 0;
    for (int l = 0; l < c.n_layer; ++l) {
        const PsLayerDesc& d = layers[l];
        PsLayer& L = hl[l];
        std::memset(&L, 0, sizeof(L));
        if (d.n_op < 4 || d.n_op > 5) { delete s; return fail("op count"); }
        L.n_op = d.n_op;
        L.attn_norm = d.attn_norm;
        L.ffn_norm = d.ffn_norm;
        L.kc = d.kc;
        L.vc = d.vc;
        for (int o = 0; o < d.n_op; ++o) {
            const PsOpDesc& od = d.op[o];
            PsOp& op = L.op[o];
            const int t = od.A.type;
            if (t != T_Q4_K && t != T_Q5_K && t != T_Q6_K) { delete s; return fail("matrix type"); }
            const bool gu = od.role == PS_R_GU;
            if (gu && (od.B.type != t || od.B.rows != od.A.rows || od.B.K != od.A.K)) { delete s; return fail("gate/up pair"); }
            if (od.A.n_exp > 1) { delete s; return fail("MoE"); }
            for (int p = 0; p < 4; ++p) {
                op.a[p] = od.A.p[p];
                op.b[p] = gu ? od.B.p[p] : od.A.p[p];
            }
            op.type = t;
            op.role = od.role;
            op.rows = od.A.rows;
            op.K = od.A.K;
            op.nb = od.A.nb;
            op.row0 = od.row0;
            op.C = ps_chunks(op.nb);
            const int want_k = od.role == PS_R_DN ? c.n_ff : c.n_embd;
            if (op.K != want_k) { delete s; return fail("matrix width"); }
            const bool cok = op.C == 1 || op.C == 2 || op.C == 4 ||
                             (od.role == PS_R_DN && (op.C == 3 || op.C == 6 || op.C == 7));
            if (!cok) { delete s; return fail("chunks per row"); }
            if (od.role == PS_R_QKV && (op.rows & 1)) { delete s; return fail("odd Q/K/V group"); }
            const int rpu = od.role == PS_R_QKV ? 2 : 1;
            op.units = od.role == PS_R_QKV ? op.rows / 2 : op.rows;
            const int nm = gu ? 2 : 1;
            const int unit_bytes = rpu * nm * ps_plane_bytes_row(t, op.nb);
            const int fit = (slot - 32 * plane_count(t) * nm) / unit_bytes;
            if (fit < 1) { delete s; return fail("a unit does not fit a ring slot"); }
            op.ups = std::min(fit, PS_NC * PS_MU);
            bytes += (long long)nm * op.rows * op.nb * block_bytes(t);
        }
    }
    MI_HIP(hipMalloc(&s->d_layers, sizeof(PsLayer) * c.n_layer));
    MI_HIP(hipMemcpy(s->d_layers, hl.data(), sizeof(PsLayer) * c.n_layer, hipMemcpyHostToDevice));
    const size_t ng = (size_t)c.n_embd + (c.n_embd + 2 * c.kv_dim) + (size_t)nbe * PS_ATT_W + c.n_embd + c.n_ff;
    MI_HIP(hipMalloc(&s->gran, ng * 8));
    MI_HIP(hipMemset(s->gran, 0, ng * 8));
    PsArgs& a = s->args;
    std::memset(&a, 0, sizeof(a));
    a.layers = s->d_layers;
    a.n_layer = c.n_layer;
    a.n_embd = c.n_embd;
    a.n_ff = c.n_ff;
    a.n_head = c.n_head;
    a.n_head_kv = c.n_head_kv;
    a.head_dim = c.head_dim;
    a.kv_dim = c.kv_dim;
    a.n_rot = c.n_rot;
    a.eps = c.eps;
    a.theta_scale = c.theta_scale;
    a.freq_scale = c.freq_scale;
    a.kq_scale = c.kq_scale;
    a.freq_factors = c.freq_factors;
    a.tokpos = c.tokpos;
    a.cell_pos = c.cell_pos;
    a.step = c.step;
    a.xin = c.xin;
    a.xout = c.xout;
    a.g_x = s->gran;
    a.g_qkv = a.g_x + c.n_embd;
    a.g_att = a.g_qkv + c.n_embd + 2 * c.kv_dim;
    a.g_xa = a.g_att + (size_t)nbe * PS_ATT_W;
    a.g_h = a.g_xa + c.n_embd;
    a.err = c.err;
    a.slot_bytes = slot;
    a.nslot = nslot;
    a.act_off = nslot * slot;
    a.ctl_off = a.act_off + act_region;
    s->lds = (size_t)a.ctl_off + PS_CTL;
    s->ncu = ncu;
    s->bytes = bytes;
    MI_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(ps_step_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)s->lds));
    int per_cu = 0;
    MI_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, ps_step_kernel, PS_NW * 64, s->lds));
    if (per_cu < 1) {
        ps_destroy(s);
        return fail("the step's workgroup does not fit a CU");
    }
    return s;
}

void ps_destroy(PsStep* s) {
    if (!s) return;
    if (s->d_layers) hipFree(s->d_layers);
    if (s->gran) hipFree(s->gran);
    delete s;
}

void ps_launch(const PsStep* s, hipStream_t st) {
    hipLaunchKernelGGL(ps_step_kernel, dim3(s->ncu), dim3(PS_NW * 64), s->lds, st, s->args);
    MI_HIP(hipGetLastError());
}

long long ps_bytes(const PsStep* s) { return s ? s->bytes : 0; }

int ps_arm_stamps(PsStep* s, unsigned long long* dev, int layer) {
    if (!s) return 0;
    s->args.stamps = dev;
    s->args.stamp_layer = layer;
    return s->ncu;
}

}  // namespace mi
