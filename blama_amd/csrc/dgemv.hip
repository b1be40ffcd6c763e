// Batch-1 decode GEMV, streaming form (gfx950, wave64): ggml_mul_mat of one token against a
// Q4_K / Q5_K / Q6_K / Q8_0 matrix for the dense LLaMA decode step within
// ATTN_SHORT cells.  Same integer arithmetic as gemv.hip (Kq<T>, qdot.h: ggml b5187's
// vec_dot_q*_K_q8_K / vec_dot_q8_0_q8_0 bit for bit per superblock); what differs is the shape:
//
//  * One unit (a row, a RoPE row pair or a gate/up row pair) per wave, 8-wave workgroups, a grid
//    of units / 8 workgroups (~500-1400, more than are resident: the hardware deals the rest out
//    as workgroups retire).  Every weight load of a wave is issued at entry -- no ring, nothing
//    waits on the activation before the weights are in flight (the streaming floor measured by
//    scripts/exp_gemv2.cpp / exp_fgemv.cpp).
//  * The activation arrives quantised (Q8_K and/or Q8_0, act_layout) by its own small launch
//    (dv_quant_kernel: rms_norm(x) * norm_w for the QKV, gate/up and head inputs) or by the
//    producer (the attention kernel quantises its output for WO, whole 256-blocks per workgroup);
//    each workgroup loads those few KB ahead of its weights and copies them into LDS.  Measured
//    alternatives (scripts/exp_fgemv.cpp, profiles/r05_exp_fgemv*.txt): publishing
//    the activation inside the producing launch by arrival tickets cost 6-10 us per launch; an
//    rms-norm prologue in every QKV / gate/up workgroup (DV_QKVN / DV_SWIGLUN) 8-9 % slower for 7B
//    and Llama-3-8B but 17 % faster for TinyLlama; the FFN down launch quantising h itself in
//    every workgroup (DV_ADDQ) 1-1.5 % slower per 7B token but 4-5 % faster for TinyLlama -- so
//    the step quantises in-launch for small models only (n_ff * n_embd <= 2^24; bit-identical to
//    the dv_quant launches; profiles/r06_hq_ab.txt, r06_nq_ab.txt); an Infinity-Cache prefetch of the next layer's weights from a side stream slowed the
//    chain 1.7-2.6x.
//    Every sum is taken in a fixed order: results are bit-reproducible.
#include "qdot.h"
#include <hip/hip_ext.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>

namespace mi {

namespace {

constexpr int DV_NW = 8;       // waves per workgroup
constexpr int DV_ACT_LD = 5;   // 16-B activation loads per lane: act bytes <= 5 x 8 KiB

// DV_ADDQ: DV_ADD whose workgroups quantise the fp32 activation (hraw, no norm) into LDS themselves;
// DV_QKVN / DV_SWIGLUN: DV_QKV / DV_SWIGLU whose workgroups build rms_norm(hraw) * norm_w so
enum DvRole { DV_QKV = 0, DV_ADD = 1, DV_SWIGLU = 2, DV_STORE = 3, DV_ADDQ = 4, DV_QKVN = 5, DV_SWIGLUN = 6 };
constexpr int dv_base(int r) { return r == DV_ADDQ ? DV_ADD : r == DV_QKVN ? DV_QKV : r == DV_SWIGLUN ? DV_SWIGLU : r; }


struct DvSeg {
    const uint8_t* a[4];        // planes of A
    const uint8_t* b[4];        // DV_SWIGLU: planes of B (up)
    float* out;
    int rows, units, blk0, nblk;
    int nq, nk;                 // DV_QKV: rows of Q and K in A (the rest are V)
};

struct DvArgs {
    DvSeg seg[2];
    const char* act;            // this launch's activation, act_layout(K, q8k, q80)
    int act_bytes, K, q8k, q80;
    const float* resid;         // DV_ADD
    const float* hraw;          // DV_ADDQ / _QKVN / _SWIGLUN: the fp32 activation (K floats)
    const float* norm_w;        // DV_QKVN / DV_SWIGLUN
    float eps;
    int red_off;                // DV_QKVN / DV_SWIGLUN: LDS offset of the 4 waves' sums of squares
    const int* tokpos;          // DV_QKV: {token, pos, cell, -}
    int* cell_pos;
    __half* kcache;
    __half* vcache;
    const float* freq_factors;
    float theta_scale, freq_scale;
    int n_rot, head_dim, kv_dim;
};

__device__ __forceinline__ void dv_lds_barrier() {
    __builtin_amdgcn_s_waitcnt((0xF) | (0x3 << 14) | (0x7 << 4));   // lgkmcnt(0); vmcnt untouched
    __builtin_amdgcn_s_barrier();
}

// One workgroup's work for segment SI of type T.  RW: rows per unit (2: DV_QKV RoPE pairs /
// DV_SWIGLU gate-up pairs); C: 8-superblock chunks per row (ceil(K / 2048)).
template <int T, int SI, int RW, int C, int ROLE0>
__device__ __forceinline__ void dv_body(const DvArgs& a, char* lds) {
    constexpr int ROLE = dv_base(ROLE0);
    using K = Kq<T>;
    const DvSeg& S = a.seg[SI];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int sbl = lane >> 3, j = lane & 7;
    const int nb = a.K >> 8;
    const int wg = (int)blockIdx.x - S.blk0;
    const int u = wg * DV_NW + wave;
    const bool uv = u < S.units;
    const int uc = uv ? u : S.units - 1;
    constexpr bool ADD = ROLE == DV_ADD;
    constexpr bool RAWQ = ROLE0 == DV_ADDQ;
    constexpr bool NORMQ = ROLE0 == DV_QKVN || ROLE0 == DV_SWIGLUN;
    constexpr int NP = NORMQ ? 2 * C : 1;   // NORMQ: pieces tid + 256 k of waves 0-3 (dv_quant_kernel's)
    const int n4 = a.K >> 2;
    constexpr int NLD = DV_ACT_LD;
    const ActLayout L = act_layout(a.K, a.q8k, a.q80);
    // ---- 1. the activation and the epilogue's inputs, requested before any weight (loads retire
    // in order: the compiler's wait for them is then a count that leaves the weights in flight)
    u32x4 av[RAWQ || NORMQ ? 1 : NLD];
    f32x4 hv[RAWQ ? C : 1];   // DV_ADDQ: blocks wave, wave + 8, .. (nb <= 8 C), 4 floats per lane
    f32x4 xv[NP], nv[NP];
    if constexpr (NORMQ) {
        if (wave < 4) {
            const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.hraw), 0, a.K * 4, 0x00020000);
            const __amdgpu_buffer_rsrc_t nr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.norm_w), 0, a.K * 4, 0x00020000);
#pragma unroll
            for (int k = 0; k < NP; ++k) {
                const int i = tid + 256 * k;
                xv[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, oob(i * 16, i >= n4), 0, 0));
                nv[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(nr, oob(i * 16, i >= n4), 0, 0));
            }
        }
    } else if constexpr (RAWQ) {
        const __amdgpu_buffer_rsrc_t hr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.hraw), 0, a.K * 4, 0x00020000);
#pragma unroll
        for (int k = 0; k < C; ++k) {
            const int b = wave + DV_NW * k;
            hv[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(hr, oob((b * 64 + lane) * 16, b >= nb), 0, 0));
        }
    } else {
        const __amdgpu_buffer_rsrc_t ar = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(a.act), 0, a.act_bytes, 0x00020000);
#pragma unroll
        for (int k = 0; k < NLD; ++k) av[k] = __builtin_amdgcn_raw_buffer_load_b128(ar, (k * DV_NW * 64 + tid) * 16, 0, 0);
    }
    i32x4 tp = {0, 0, 0, 0};
    if (ROLE == DV_QKV) tp = *gptr(reinterpret_cast<const i32x4*>(a.tokpos));
    float res = 0.0f;
    if (ADD) {
        const uint8_t* rb = reinterpret_cast<const uint8_t*>(rfl_ptr(a.resid));
        res = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(buf_rsrc(rb), oob((unsigned)uc * 4, !uv), 0, 0));
    }
    // DV_QKV: the RoPE pair index of this unit and its frequency factor (Llama-3 rope_freqs)
    const int r0 = RW * uc;
    const bool isq = ROLE == DV_QKV && r0 < S.nq;
    const bool isk = ROLE == DV_QKV && !isq && r0 < S.nq + S.nk;
    const int i0 = (ROLE == DV_QKV && (isq || isk)) ? (isq ? r0 : r0 - S.nq) % a.head_dim : 0;
    const bool roped = (isq || isk) && i0 < a.n_rot;
    float ff = 1.0f;
    if (ROLE == DV_QKV && a.freq_factors) {
        const uint8_t* fb = reinterpret_cast<const uint8_t*>(rfl_ptr(a.freq_factors));
        ff = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(buf_rsrc(fb), oob((unsigned)(i0 / 2) * 4, !roped), 0, 0));
    }
    asm volatile("" ::: "memory");

    // ---- 2. every weight load of this wave
    typename K::Ld w[RW][C];
#pragma unroll
    for (int r = 0; r < RW; ++r) {
        long long row = ROLE == DV_SWIGLU ? uc : (long long)uc * RW + r;
        if (row >= S.rows) row = S.rows - 1;            // an odd last pair re-reads its row (unused)
        const uint8_t* rp[4];
#pragma unroll
        for (int p = 0; p < 4; ++p)
            rp[p] = rfl_ptr(((ROLE == DV_SWIGLU && r == 1) ? S.b[p] : S.a[p]) + row * nb * PlaneBytes<T>::b[p]);
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const int sb = 8 * c + sbl;
            w[r][c] = K::bload(rp, sb < nb ? sb : nb - 1, j, !uv || sb >= nb);
        }
    }

    // ---- 3. the activation into LDS (the waits the compiler puts here leave the weights in flight)
    if constexpr (NORMQ) {   // dv_quant_kernel with the norm: the same sums in the same order, waves 0-3
        double* red = reinterpret_cast<double*>(lds + a.red_off);
        if (wave < 4) {
            double sq = 0.0;
#pragma unroll
            for (int k = 0; k < NP; ++k)
                if (tid + 256 * k < n4) {
                    sq += (double)(xv[k].x * xv[k].x);
                    sq += (double)(xv[k].y * xv[k].y);
                    sq += (double)(xv[k].z * xv[k].z);
                    sq += (double)(xv[k].w * xv[k].w);
                }
            sq = wave_sum63_d(sq);
            if (lane == 63) red[wave] = sq;
        }
        dv_lds_barrier();
        if (wave < 4) {
            double tot = 0.0;
#pragma unroll
            for (int k = 0; k < 4; ++k) tot += red[k];
            const float scale = 1.0f / sqrtf((float)(tot / (double)a.K) + a.eps);
            const ActOut t{a.K, a.q8k, a.q80, lds, nullptr, 0.0f};
#pragma unroll
            for (int k = 0; k < NP; ++k) {
                const int b = wave + 4 * k;   // piece tid + 256 k = block b's lane piece
                if (b < nb) {
                    const float q[4] = {(xv[k].x * scale) * nv[k].x, (xv[k].y * scale) * nv[k].y,
                                        (xv[k].z * scale) * nv[k].z, (xv[k].w * scale) * nv[k].w};
                    dv_quant_block(t, b, q, lane);
                }
            }
        }
    } else if constexpr (RAWQ) {   // dv_quant_kernel's arithmetic without the norm, block by block into LDS
        const ActOut t{a.K, a.q8k, a.q80, lds, nullptr, 0.0f};
#pragma unroll
        for (int k = 0; k < C; ++k) {
            const int b = wave + DV_NW * k;
            if (b < nb) {
                const float q[4] = {hv[k].x, hv[k].y, hv[k].z, hv[k].w};
                dv_quant_block(t, b, q, lane);
            }
        }
    } else {
#pragma unroll
        for (int k = 0; k < NLD; ++k) {
            const int o = (k * DV_NW * 64 + tid) * 16;
            if (o < a.act_bytes) *reinterpret_cast<u32x4*>(lds + o) = av[k];
        }
    }
    dv_lds_barrier();

    // ---- 4. the dot products: lane 63 holds each row's sum
    const Act act = act_view(lds, L, 0);
    float y[RW];
#pragma unroll
    for (int r = 0; r < RW; ++r) {
        float acc = 0.0f;
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const int sb0 = 8 * c + sbl;
            const int sb = sb0 < nb ? sb0 : nb - 1;
            const float p = K::dot(w[r][c], K::act(act, sb, j), j);
            acc += sb0 < nb ? p : 0.0f;
        }
        y[r] = wave_sum63(acc);
    }

    // ---- 5. epilogue (lane 63)
    if (lane != 63 || !uv) return;
    if (ROLE == DV_QKV) {
        float o0 = y[0], o1 = y[RW - 1];
        if (roped) {   // ggml_rope_cache_init (ext_factor 0, mscale 1) for this pair, then rotate
            float theta = (float)tp.y;
            for (int k = 0; k < i0 / 2; ++k) theta = theta * a.theta_scale;
            const float th = a.freq_scale * (theta / ff);
            const float cs = cosf(th), sn = sinf(th);
            o0 = y[0] * cs - y[RW - 1] * sn;
            o1 = y[0] * sn + y[RW - 1] * cs;
        }
        const int cell = tp.z;
        if (isq) {
            S.out[r0] = o0;
            S.out[r0 + 1] = o1;
        } else if (isk) {
            const int rk = r0 - S.nq;
            __half* kr = a.kcache + (long long)cell * a.kv_dim;
            kr[rk] = __float2half_rn(o0);
            kr[rk + 1] = __float2half_rn(o1);
            if (rk == 0) a.cell_pos[cell] = tp.y;
        } else {
            const int rv = r0 - S.nq - S.nk;
            __half* vr = a.vcache + (long long)cell * a.kv_dim;
            vr[rv] = __float2half_rn(o0);
            if (r0 + 1 < S.rows) vr[rv + 1] = __float2half_rn(o1);
        }
    } else if (ROLE == DV_SWIGLU) {
        S.out[u] = silu_f(y[0]) * y[RW - 1];
    } else if (ADD) {
        S.out[u] = y[0] + res;
    } else {
        S.out[u] = y[0];
    }
}

// T1: -1 one segment, else the type of segment 1 (a mixed-type Q/K/V launch)
template <int T0, int T1, int RW, int C, int ROLE>
__global__ __launch_bounds__(DV_NW * 64) void dgemv_kernel(const DvArgs a) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    if (T1 < 0 || (int)blockIdx.x < a.seg[1].blk0) dv_body<T0, 0, RW, C, ROLE>(a, lds);
    else dv_body<(T1 < 0 ? T0 : T1), 1, RW, C, ROLE>(a, lds);
}

typedef void (*DvFn)(const DvArgs);

// chunks per row: K <= 2048 -> 1, 4096 -> 2, 8192 -> 4 (the n_embd-wide inputs); the FFN down
// input (n_ff) also 3 (5632), 6 (11008), 7 (14336)
template <int T0, int T1, int RW, int ROLE>
DvFn dv_fn_c(int c) {
    switch (c) {
    case 1: return dgemv_kernel<T0, T1, RW, 1, ROLE>;
    case 2: return dgemv_kernel<T0, T1, RW, 2, ROLE>;
    case 4: return dgemv_kernel<T0, T1, RW, 4, ROLE>;
    default: break;
    }
    if constexpr (dv_base(ROLE) == DV_ADD) {
        switch (c) {
        case 3: return dgemv_kernel<T0, T1, RW, 3, ROLE>;
        case 6: return dgemv_kernel<T0, T1, RW, 6, ROLE>;
        case 7: return dgemv_kernel<T0, T1, RW, 7, ROLE>;
        default: break;
        }
    }
    return nullptr;
}
template <int T0, int ROLE>
DvFn dv_fn_t1(int t1, int c) {
    constexpr int RW = (dv_base(ROLE) == DV_QKV || dv_base(ROLE) == DV_SWIGLU) ? 2 : 1;
    if (t1 < 0) return dv_fn_c<T0, -1, RW, ROLE>(c);
    if constexpr (dv_base(ROLE) == DV_QKV) {   // mixed-type Q/K/V launches only
        switch (t1) {
        case T_Q6_K: return dv_fn_c<T0, T_Q6_K, RW, ROLE>(c);
        case T_Q8_0: return dv_fn_c<T0, T_Q8_0, RW, ROLE>(c);
        default: return nullptr;
        }
    }
    return nullptr;
}
template <int ROLE>
DvFn dv_fn_role(int t0, int t1, int c) {
    switch (t0) {
    case T_Q4_K: return dv_fn_t1<T_Q4_K, ROLE>(t1, c);
    case T_Q5_K: return dv_fn_t1<T_Q5_K, ROLE>(t1, c);
    case T_Q6_K: return t1 == T_Q6_K ? nullptr : dv_fn_t1<T_Q6_K, ROLE>(t1, c);
    case T_Q8_0: return t1 >= 0 ? nullptr : dv_fn_t1<T_Q8_0, ROLE>(t1, c);
    default: return nullptr;
    }
}
DvFn dv_fn(int role, int t0, int t1, int c) {
    switch (role) {
    case DV_QKV: return dv_fn_role<DV_QKV>(t0, t1, c);
    case DV_ADD: return dv_fn_role<DV_ADD>(t0, t1, c);
    case DV_ADDQ: return dv_fn_role<DV_ADDQ>(t0, t1, c);
    case DV_QKVN: return c <= 4 ? dv_fn_role<DV_QKVN>(t0, t1, c) : nullptr;
    case DV_SWIGLUN: return c <= 4 ? dv_fn_role<DV_SWIGLUN>(t0, t1, c) : nullptr;
    case DV_SWIGLU: return dv_fn_role<DV_SWIGLU>(t0, t1, c);
    case DV_STORE: return dv_fn_role<DV_STORE>(t0, t1, c);
    default: return nullptr;
    }
}
int dv_chunks(int K) {
    const int c = (K / 256 + 7) / 8;
    return c == 5 ? 6 : c;
}


// rms_norm(x) * norm_w (norm_w set) or x itself, quantised: one workgroup per 256-block.  With the
// norm, each 4-wave workgroup reads the whole row and takes its sum of squares in double (every
// workgroup in the same order: thread-strided 16-B pieces, the wave's DPP tree, the 4 waves in
// order -- so all blocks see one scale, and the result is bit-reproducible); without it, one wave
// reads its block.  ggml_compute_forward_rms_norm_f32 + ggml_mul, then quantize_row_q8_K /
// quantize_row_q8_0 (x86 form).  (r06: one wave per block standing in for the four, no LDS or
// barrier, bit-identical, measured 635-637 vs 644-647 tok/s: not kept, profiles/r06_dvq_ab.txt.)
constexpr int DQ_NORM_W = 4;   // waves per workgroup with the norm
__global__ __launch_bounds__(DQ_NORM_W * 64) void dv_quant_kernel(const float* x, const ActOut t) {
    __shared__ double red[DQ_NORM_W];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int b = blockIdx.x;
    const f32x4 v = gptr(reinterpret_cast<const f32x4*>(x))[b * 64 + lane];   // (waves > 0: unused)
    float scale = 1.0f;
    f32x4 wn = {1.0f, 1.0f, 1.0f, 1.0f};
    if (t.norm_w) {
        wn = gptr(reinterpret_cast<const f32x4*>(t.norm_w))[b * 64 + lane];
        double sq = 0.0;
        const int n4 = t.K >> 2;
        // this thread's pieces tid, tid + 256, ... requested together (DQ_LD at a time: a
        // load-then-add loop waited out one memory round trip per piece), summed in that order
        constexpr int DQ_LD = 8;   // K <= 8192 in one round
        for (int i0 = tid; i0 < n4; i0 += DQ_LD * DQ_NORM_W * 64) {
            f32x4 y[DQ_LD];
#pragma unroll
            for (int k = 0; k < DQ_LD; ++k) {
                const int i = i0 + k * DQ_NORM_W * 64;
                if (i < n4) y[k] = gptr(reinterpret_cast<const f32x4*>(x))[i];
            }
#pragma unroll
            for (int k = 0; k < DQ_LD; ++k) {
                if (i0 + k * DQ_NORM_W * 64 < n4) {
                    sq += (double)(y[k].x * y[k].x);
                    sq += (double)(y[k].y * y[k].y);
                    sq += (double)(y[k].z * y[k].z);
                    sq += (double)(y[k].w * y[k].w);
                }
            }
        }
        sq = wave_sum63_d(sq);
        if (lane == 63) red[wave] = sq;
        __syncthreads();
        double tot = 0.0;
#pragma unroll
        for (int k = 0; k < DQ_NORM_W; ++k) tot += red[k];
        scale = 1.0f / sqrtf((float)(tot / (double)t.K) + t.eps);
    }
    if (wave != 0) return;
    float q[4] = {v.x, v.y, v.z, v.w};
    if (t.norm_w) {   // ggml_vec_scale_f32 then ggml_mul
        q[0] = (q[0] * scale) * wn.x;
        q[1] = (q[1] * scale) * wn.y;
        q[2] = (q[2] * scale) * wn.z;
        q[3] = (q[3] * scale) * wn.w;
    }
    dv_quant_block(t, b, q, lane);
}

}  // namespace

size_t dv_act_bytes(int K, int q8k, int q80) { return (size_t)act_layout(K, q8k, q80).slot_bytes; }

void launch_dv_quant(const float* x, const ActOut& t, hipStream_t s) {
    if (t.K % 256 || t.K <= 0 || !t.act || (!t.q8k && !t.q80)) throw Error("dv_quant: unsupported shape");
    hipLaunchKernelGGL(dv_quant_kernel, dim3(t.K / 256), dim3(t.norm_w ? DQ_NORM_W * 64 : 64), 0, s, x, t);
    MI_HIP(hipGetLastError());
}

namespace {
int dv_role(const GemvParams& p) {
    const GemvSeg& g = p.seg[0];
    // (a launch given the fp32 activation x[0] instead of a quantised one: ADD without a norm,
    // Q/K/V and SwiGLU with rms_norm * norm_w, quantised in every workgroup)
    const bool raw = !p.act_in && p.x[0];
    if (raw && (g.epi == EPI_ADD) == (p.norm_w != nullptr)) return -1;
    return g.epi == EPI_QKV ? (raw ? DV_QKVN : DV_QKV) : g.epi == EPI_ADD ? (raw ? DV_ADDQ : DV_ADD)
         : g.epi == EPI_SWIGLU ? (raw ? DV_SWIGLUN : DV_SWIGLU) : g.epi == EPI_STORE && !raw ? DV_STORE : -1;
}
}  // namespace

bool dgemv_supported(const GemvParams& p) {
    if (p.nseg < 1 || p.nseg > 2 || p.K % 256 || (!p.act_q8k && !p.act_q80) ||
        dv_act_bytes(p.K, p.act_q8k, p.act_q80) > (size_t)DV_ACT_LD * DV_NW * 64 * 16)
        return false;
    const GemvSeg& g = p.seg[0];
    const int role = dv_role(p);
    if (role < 0 || g.bias || g.expA >= 0 || g.expB >= 0) return false;
    if (p.nseg == 2 && (dv_base(role) != DV_QKV || p.seg[1].epi != EPI_QKV)) return false;
    if ((role == DV_QKVN || role == DV_SWIGLUN) && p.K > 4 * 256 * 2 * dv_chunks(p.K)) return false;
    return dv_fn(role, g.A.type, p.nseg == 2 ? p.seg[1].A.type : -1, dv_chunks(p.K)) != nullptr;
}

void launch_dgemv(const GemvParams& p, hipStream_t s, hipEvent_t ev_start, hipEvent_t ev_stop) {
    if (!p.act_in && !p.x[0]) throw Error("dgemv: no activation");
    if (!dgemv_supported(p)) throw Error("dgemv: unsupported launch shape");
    const GemvSeg& g0 = p.seg[0];
    const int role0 = dv_role(p);
    const int role = dv_base(role0);
    const int rw = (role == DV_QKV || role == DV_SWIGLU) ? 2 : 1;
    DvArgs a;
    std::memset(&a, 0, sizeof(a));
    int blk = 0;
    for (int i = 0; i < p.nseg; ++i) {
        const GemvSeg& g = p.seg[i];
        if (g.A.K != p.K) throw Error("dgemv: matrix shape does not match the activation");
        if (role == DV_SWIGLU && (g.pair != PAIR_AB || g.B.type != g.A.type || g.B.rows != g.A.rows))
            throw Error("dgemv: SwiGLU needs a gate/up pair of one type and shape");
        if (role == DV_QKV && (g.A.rows & 1)) throw Error("dgemv: fused QKV rows must be even");
        DvSeg& o = a.seg[i];
        for (int k = 0; k < 4; ++k) {
            o.a[k] = g.A.p[k];
            o.b[k] = role == DV_SWIGLU ? g.B.p[k] : g.A.p[k];
        }
        o.out = g.out;
        o.rows = g.A.rows;
        o.units = role == DV_SWIGLU ? g.A.rows : (g.A.rows + rw - 1) / rw;
        o.nq = g.nq;
        o.nk = g.nk;
        o.blk0 = blk;
        o.nblk = (o.units + DV_NW - 1) / DV_NW;
        blk += o.nblk;
    }
    if (p.nseg == 1) a.seg[1].blk0 = blk;
    a.act = p.act_in;
    a.K = p.K;
    a.q8k = p.act_q8k;
    a.q80 = p.act_q80;
    a.act_bytes = (int)dv_act_bytes(p.K, p.act_q8k, p.act_q80);
    a.resid = g0.resid;
    a.tokpos = p.tokpos;
    a.cell_pos = p.cell_pos;
    a.kcache = p.kcache;
    a.vcache = p.vcache;
    a.freq_factors = p.freq_factors;
    a.theta_scale = p.theta_scale;
    a.freq_scale = p.freq_scale;
    a.n_rot = p.n_rot;
    a.head_dim = p.head_dim > 0 ? p.head_dim : 1;
    a.kv_dim = p.kv_dim;
    a.hraw = p.x[0];
    a.norm_w = p.norm_w;
    a.eps = p.eps;
    const size_t actb = (dv_act_bytes(p.K, p.act_q8k, p.act_q80) + 15) / 16 * 16;
    a.red_off = (int)actb;
    if (role0 == DV_ADDQ && p.K > DV_NW * 256 * dv_chunks(p.K)) throw Error("dgemv: activation too long to quantise in-launch");
    if (role == DV_ADD && !g0.resid) throw Error("dgemv: residual epilogue without resid");
    if (role == DV_QKV && !p.tokpos) throw Error("dgemv: QKV epilogue needs tokpos");
    const DvFn fn = dv_fn(role0, g0.A.type, p.nseg == 2 ? p.seg[1].A.type : -1, dv_chunks(p.K));
    const size_t smem = actb + (role0 == DV_QKVN || role0 == DV_SWIGLUN ? 4 * sizeof(double) : 0);
    if (ev_start || ev_stop)
        hipExtLaunchKernelGGL(fn, dim3(blk), dim3(DV_NW * 64), smem, s, ev_start, ev_stop, 0, a);
    else
        hipLaunchKernelGGL(fn, dim3(blk), dim3(DV_NW * 64), smem, s, a);
    MI_HIP(hipGetLastError());
}

}  // namespace mi
