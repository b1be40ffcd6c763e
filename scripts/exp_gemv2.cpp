// Decode-GEMV design experiment (diagnostic, not product).  Question: what does a batch-1
// Q4_K / Q6_K GEMV cost per launch when every weight load of the wave is issued at kernel
// entry (before the activation prologue), with no ring and no parameter-block copy, and what
// does a 7B Q4_K_M step cost as a chain of such launches?
//   PRO 0: activation pre-quantised (Q8_K in global) -> LDS
//   PRO 1: RMSNorm (double sum) + Q8_K of x in every workgroup
//   PRO 2: Q8_K of x (no norm) in every workgroup
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o scripts/exp_gemv2 scripts/exp_gemv2.cpp
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int Q4K = 12, Q6K = 14;

template <typename T>
__device__ __forceinline__ const __attribute__((address_space(1))) T* gp(const T* p) {
    return (const __attribute__((address_space(1))) T*)(p);
}
__device__ __forceinline__ u32x4 ldg16(const uint8_t* p) { return __builtin_nontemporal_load(gp(reinterpret_cast<const u32x4*>(p))); }
__device__ __forceinline__ float h2f(uint32_t b) { return __half2float(__ushort_as_half((unsigned short)(b & 0xFFFF))); }
__device__ __forceinline__ int dot4(int a, int b, int c) { return __builtin_amdgcn_sdot4(a, b, c, false); }
template <int CTRL, int RMASK>
__device__ __forceinline__ int dpp_i(int v) { return __builtin_amdgcn_update_dpp(0, v, CTRL, RMASK, 0xf, false); }
template <int CTRL, int RMASK>
__device__ __forceinline__ double dpp_d(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = dpp_i<CTRL, RMASK>((int)b), hi = dpp_i<CTRL, RMASK>((int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ float wsum63(float v) {
#define D_(c, r) v += __int_as_float(dpp_i<c, r>(__float_as_int(v)))
    D_(0x111, 0xf); D_(0x112, 0xf); D_(0x114, 0xf); D_(0x118, 0xf); D_(0x142, 0xa); D_(0x143, 0xc);
#undef D_
    return v;
}
__device__ __forceinline__ double wsum63_d(double v) {
    v += dpp_d<0x111, 0xf>(v); v += dpp_d<0x112, 0xf>(v); v += dpp_d<0x114, 0xf>(v);
    v += dpp_d<0x118, 0xf>(v); v += dpp_d<0x142, 0xa>(v); v += dpp_d<0x143, 0xc>(v);
    return v;
}
__device__ __forceinline__ float wmax_pos(float v) {
#define M_(c, r) v = fmaxf(v, __int_as_float(dpp_i<c, r>(__float_as_int(v))))
    M_(0x111, 0xf); M_(0x112, 0xf); M_(0x114, 0xf); M_(0x118, 0xf); M_(0x142, 0xa); M_(0x143, 0xc);
#undef M_
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_s_waitcnt((0xF) | (0x3 << 14) | (0x7 << 4));   // lgkmcnt(0) only
    __builtin_amdgcn_s_barrier();
}

struct GV {
    const uint8_t* A[4];
    const uint8_t* B[4];
    const float* x;
    const float* nw;
    const int8_t* q8;
    const int* bsum;
    const float* dk;
    float* out;
    int rows, nb, units;
    unsigned long long* st;   // STAMPS builds: [grid][4] s_memrealtime (entry, act ready, first compute done, end)
};

// LDS activation: q8 at sb*ASTR (padded stride), bsum [nb*16], dk [nb], red [32] doubles
constexpr int ASTR = 272;
__host__ __device__ inline int lds_bytes(int nb) { return nb * ASTR + nb * 64 + ((nb * 4 + 15) & ~15) + 32 * 8; }

template <int T> struct Kq;
template <> struct Kq<Q4K> {
    static constexpr int pb[4] = {128, 16, 0, 0};
    struct Ld { u32x4 qs, hdr; __device__ unsigned fold() const { return qs.x ^ qs.y ^ qs.z ^ qs.w ^ hdr.x ^ hdr.y ^ hdr.z ^ hdr.w; } };
    __device__ static Ld load(const uint8_t* const* rp, int sb, int j) {
        Ld l; l.qs = ldg16(rp[0] + sb * 128 + j * 16); l.hdr = ldg16(rp[1] + sb * 16); return l;
    }
    __device__ static float dot(const Ld& l, const char* act, int nb, int sb, int j) {
        const int g = j >> 1, half = j & 1;
        const int8_t* ab = reinterpret_cast<const int8_t*>(act) + sb * ASTR + 64 * g + 16 * half;
        const i32x4 alo = *reinterpret_cast<const i32x4*>(ab);
        const i32x4 ahi = *reinterpret_cast<const i32x4*>(ab + 32);
        const int* bs = reinterpret_cast<const int*>(act + nb * ASTR);
        const int bs_lo = bs[sb * 16 + 4 * g + half], bs_hi = bs[sb * 16 + 4 * g + 2 + half];
        const float dx = reinterpret_cast<const float*>(act + nb * ASTR + nb * 64)[sb];
        int dlo = 0, dhi = 0;
        dlo = dot4(l.qs.x & 0x0F0F0F0F, alo.x, dlo); dlo = dot4(l.qs.y & 0x0F0F0F0F, alo.y, dlo);
        dlo = dot4(l.qs.z & 0x0F0F0F0F, alo.z, dlo); dlo = dot4(l.qs.w & 0x0F0F0F0F, alo.w, dlo);
        dhi = dot4((l.qs.x >> 4) & 0x0F0F0F0F, ahi.x, dhi); dhi = dot4((l.qs.y >> 4) & 0x0F0F0F0F, ahi.y, dhi);
        dhi = dot4((l.qs.z >> 4) & 0x0F0F0F0F, ahi.z, dhi); dhi = dot4((l.qs.w >> 4) & 0x0F0F0F0F, ahi.w, dhi);
        const unsigned sh = (g & 1) * 16;
        const unsigned Y = l.hdr.y >> sh, Z = l.hdr.z >> sh, W = l.hdr.w >> sh;
        const unsigned SC = g < 2 ? (Y & 0x3F3Fu) : ((W & 0x0F0Fu) | ((Y >> 2) & 0x3030u));
        const unsigned MM = g < 2 ? (Z & 0x3F3Fu) : (((W >> 4) & 0x0F0Fu) | ((Z >> 2) & 0x3030u));
        const int S = (int)(SC & 0xFF) * dlo + (int)((SC >> 8) & 0xFF) * dhi;
        const int M = (int)(MM & 0xFF) * bs_lo + (int)((MM >> 8) & 0xFF) * bs_hi;
        return h2f(l.hdr.x) * dx * (float)S - h2f(l.hdr.x >> 16) * dx * (float)M;
    }
};
template <> struct Kq<Q6K> {
    static constexpr int pb[4] = {128, 64, 16, 2};
    struct Ld { u32x4 ql, qh; unsigned sc0, sc1, d;
        __device__ unsigned fold() const { return ql.x ^ ql.y ^ ql.z ^ ql.w ^ qh.x ^ qh.y ^ qh.z ^ qh.w ^ sc0 ^ sc1 ^ d; } };
    __device__ static Ld load(const uint8_t* const* rp, int sb, int j) {
        Ld l;
        const int h = j >> 2, half = j & 1;
        l.ql = ldg16(rp[0] + sb * 128 + j * 16);
        l.qh = ldg16(rp[1] + sb * 64 + 32 * h + 16 * half);
        const u32x2 sc = __builtin_nontemporal_load(gp(reinterpret_cast<const u32x2*>(rp[2] + sb * 16) + h));
        l.sc0 = sc.x; l.sc1 = sc.y;
        l.d = __builtin_nontemporal_load(gp(reinterpret_cast<const unsigned short*>(rp[3] + sb * 2)));
        return l;
    }
    __device__ static float dot(const Ld& l, const char* act, int nb, int sb, int j) {
        const int h = j >> 2, hq = (j >> 1) & 1, half = j & 1;
        const int8_t* ab = reinterpret_cast<const int8_t*>(act) + sb * ASTR + 128 * h + 32 * hq + 16 * half;
        const i32x4 alo = *reinterpret_cast<const i32x4*>(ab);
        const i32x4 ahi = *reinterpret_cast<const i32x4*>(ab + 64);
        const int is_lo = 8 * h + 2 * hq + half;
        const int* bs = reinterpret_cast<const int*>(act + nb * ASTR);
        const int bs_lo = bs[sb * 16 + is_lo], bs_hi = bs[sb * 16 + is_lo + 4];
        const float dx = reinterpret_cast<const float*>(act + nb * ASTR + nb * 64)[sb];
        const unsigned shq = hq * 2;
        int dlo = 0, dhi = 0;
#define Q6L(c) ((l.ql.c & 0x0F0F0F0Fu) | (((l.qh.c >> shq) & 0x03030303u) << 4))
#define Q6H(c) (((l.ql.c >> 4) & 0x0F0F0F0Fu) | (((l.qh.c >> (shq + 4)) & 0x03030303u) << 4))
        dlo = dot4((int)Q6L(x), alo.x, dlo); dlo = dot4((int)Q6L(y), alo.y, dlo);
        dlo = dot4((int)Q6L(z), alo.z, dlo); dlo = dot4((int)Q6L(w), alo.w, dlo);
        dhi = dot4((int)Q6H(x), ahi.x, dhi); dhi = dot4((int)Q6H(y), ahi.y, dhi);
        dhi = dot4((int)Q6H(z), ahi.z, dhi); dhi = dot4((int)Q6H(w), ahi.w, dhi);
#undef Q6L
#undef Q6H
        const int bsh = 8 * (2 * hq + half);
        const int sc_lo = (int)(signed char)((l.sc0 >> bsh) & 0xFF);
        const int sc_hi = (int)(signed char)((l.sc1 >> bsh) & 0xFF);
        const int S = sc_lo * (dlo - 32 * bs_lo) + sc_hi * (dhi - 32 * bs_hi);
        return h2f(l.d) * dx * (float)S;
    }
};

// Q8_K of one 256-block by one wave (4 values per lane) into the LDS activation
__device__ __forceinline__ void q8k_block(const float v[4], int lane, char* act, int nb, int blk) {
    const float a0 = fabsf(v[0]), a1 = fabsf(v[1]), a2 = fabsf(v[2]), a3 = fabsf(v[3]);
    const float amax = wmax_pos(fmaxf(fmaxf(a0, a1), fmaxf(a2, a3)));
    int q[4] = {0, 0, 0, 0};
    float d = 0.0f;
    if (amax != 0.0f) {
        const int e = a0 == amax ? 0 : a1 == amax ? 1 : a2 == amax ? 2 : a3 == amax ? 3 : 4;
        const float mine = e == 0 ? v[0] : e == 1 ? v[1] : e == 2 ? v[2] : v[3];
        const unsigned long long m = __ballot(e < 4);
        const float mx = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(mine), __builtin_ctzll(m)));
        const float iscale = -127.0f / mx;
#pragma unroll
        for (int k = 0; k < 4; ++k) q[k] = min(127, (int)rintf(iscale * v[k]));
        d = 1.0f / iscale;
    }
    reinterpret_cast<int*>(act + blk * ASTR)[lane] =
        (q[0] & 0xFF) | ((q[1] & 0xFF) << 8) | ((q[2] & 0xFF) << 16) | ((q[3] & 0xFF) << 24);
    int sm = q[0] + q[1] + q[2] + q[3];
    sm += dpp_i<0xB1, 0xf>(sm);
    sm += dpp_i<0x4E, 0xf>(sm);
    if ((lane & 3) == 0) reinterpret_cast<int*>(act + nb * ASTR)[blk * 16 + (lane >> 2)] = sm;
    if (lane == 0) reinterpret_cast<float*>(act + nb * ASTR + nb * 64)[blk] = d;
}


template <int T, int NW, int RW, int C, int PRO, int PAIR, int LOOP, int ORDER = 1, int PIPE = 2,
          int MAXBPW = (C * 8 + NW - 1) / NW>
__global__ __launch_bounds__(NW * 64) void gv(GV a) {
    extern __shared__ __attribute__((aligned(16))) char act[];
    using K = Kq<T>;
#ifdef STAMPS
    if (a.st && threadIdx.x == 0) a.st[blockIdx.x * 4 + 0] = __builtin_amdgcn_s_memrealtime();
#define STAMP(k) if (a.st && threadIdx.x == 0) a.st[blockIdx.x * 4 + (k)] = __builtin_amdgcn_s_memrealtime();
#else
#define STAMP(k)
#endif
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int sbl = lane >> 3, j = lane & 7;
    const int nb = a.nb;
    const int stride = gridDim.x * NW;
    int u = blockIdx.x * NW + wave;
    typename K::Ld w0[RW][C], w1[RW][C];
    auto load = [&](typename K::Ld (&w)[RW][C], int uu) {
        uu = uu < a.units ? uu : a.units - 1;
#pragma unroll
        for (int r = 0; r < RW; ++r) {
            const long long row = PAIR ? uu : (long long)uu * RW + r;
            const long long rr = row < a.rows ? row : a.rows - 1;
            const uint8_t* rp[4];
#pragma unroll
            for (int p = 0; p < 4; ++p) rp[p] = ((PAIR && r == 1) ? a.B[p] : a.A[p]) + rr * nb * K::pb[p];
#pragma unroll
            for (int c = 0; c < C; ++c) {
                const int sb = 8 * c + sbl;
                w[r][c] = K::load(rp, sb < nb ? sb : nb - 1, j);
            }
        }
    };
    auto compute = [&](const typename K::Ld (&w)[RW][C], int uu) {
        float y[RW];
#pragma unroll
        for (int r = 0; r < RW; ++r) {
            float acc = 0.0f;
#pragma unroll
            for (int c = 0; c < C; ++c) {
                const int sb = 8 * c + sbl;
                const float p = K::dot(w[r][c], act, nb, sb < nb ? sb : nb - 1, j);
                acc += sb < nb ? p : 0.0f;
            }
            y[r] = wsum63(acc);
        }
        if (lane == 63 && uu < a.units) {
            if (PAIR) {
                a.out[uu] = y[0] / (1.0f + expf(-y[0])) * y[1];
            } else {
#pragma unroll
                for (int r = 0; r < RW; ++r)
                    if ((long long)uu * RW + r < a.rows) a.out[(long long)uu * RW + r] = y[r];
            }
        }
    };
    // ---- activation loads FIRST (they retire before the weights: vmcnt is in order)
    f32x4 xv[MAXBPW], wv[MAXBPW];
    i32x4 qv[4];
    int bsv = 0;
    float dkv = 0.0f;
    if (PRO == 0) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int i = threadIdx.x + k * NW * 64;
            if (i < nb * 16) qv[k] = *gp(reinterpret_cast<const i32x4*>(a.q8) + i);
        }
        if ((int)threadIdx.x < nb * 16) bsv = gp(a.bsum)[threadIdx.x];
        if ((int)threadIdx.x < nb) dkv = gp(a.dk)[threadIdx.x];
    } else {
#pragma unroll
        for (int i = 0; i < MAXBPW; ++i) {
            const int blk = wave + i * NW;
            if (blk < nb) {
                xv[i] = gp(reinterpret_cast<const f32x4*>(a.x))[blk * 64 + lane];
                if (PRO == 1) wv[i] = gp(reinterpret_cast<const f32x4*>(a.nw))[blk * 64 + lane];
            }
        }
    }
    // ORDER 1: every wave's activation requests ahead of any weight request of this CU (a
    // barrier that waits for no counter); ORDER 2: the activation lands before the weights go
    if (ORDER == 1) __builtin_amdgcn_s_barrier();
    if (ORDER == 2) { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
    load(w0, u);
    if (LOOP && PIPE == 2) load(w1, u + stride);
    // ---- prologue: the activation into LDS while the weights stream
    if (PRO == 0) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int i = threadIdx.x + k * NW * 64;
            if (i < nb * 16) *reinterpret_cast<i32x4*>(act + (i >> 4) * ASTR + (i & 15) * 16) = qv[k];
        }
        if ((int)threadIdx.x < nb * 16) reinterpret_cast<int*>(act + nb * ASTR)[threadIdx.x] = bsv;
        if ((int)threadIdx.x < nb) reinterpret_cast<float*>(act + nb * ASTR + nb * 64)[threadIdx.x] = dkv;
    } else {
        float scale = 1.0f;
        if (PRO == 1) {
            double s = 0.0;
#pragma unroll
            for (int i = 0; i < MAXBPW; ++i)
                if (wave + i * NW < nb) {
                    s += (double)(xv[i].x * xv[i].x); s += (double)(xv[i].y * xv[i].y);
                    s += (double)(xv[i].z * xv[i].z); s += (double)(xv[i].w * xv[i].w);
                }
            s = wsum63_d(s);
            double* red = reinterpret_cast<double*>(act + lds_bytes(nb) - 32 * 8);
            if (lane == 63) red[wave] = s;
            lds_barrier();
            double tot = 0.0;
            for (int w = 0; w < NW; ++w) tot += red[w];
            scale = 1.0f / sqrtf((float)(tot / (double)(nb * 256)) + 1e-5f);
        }
#pragma unroll
        for (int i = 0; i < MAXBPW; ++i) {
            const int blk = wave + i * NW;
            if (blk < nb) {
                float v[4] = {xv[i].x, xv[i].y, xv[i].z, xv[i].w};
                if (PRO == 1) {
                    v[0] = (v[0] * scale) * wv[i].x; v[1] = (v[1] * scale) * wv[i].y;
                    v[2] = (v[2] * scale) * wv[i].z; v[3] = (v[3] * scale) * wv[i].w;
                }
                q8k_block(v, lane, act, nb, blk);
            }
        }
    }
    lds_barrier();
    STAMP(1)
    if (!LOOP) {
        compute(w0, u);
        __syncthreads();
        STAMP(3)
        return;
    }
    if (PIPE == 1) {   // one unit in flight per wave: refill right after its compute
        for (int first = 1;; first = 0) {
            compute(w0, u);
            if (first) { STAMP(2) }
            u += stride;
            if (u >= a.units) break;
            load(w0, u);
        }
        __syncthreads();
        STAMP(3)
        return;
    }
    // w0 = unit u, w1 = unit u + stride in flight; refill each buffer after its compute
    for (int first = 1;; first = 0) {
        compute(w0, u);
        if (first) { STAMP(2) }
        u += stride;
        if (u >= a.units) break;
        load(w0, u + stride);
        compute(w1, u);
        u += stride;
        if (u >= a.units) break;
        load(w1, u + stride);
    }
    __syncthreads();
    STAMP(3)
}

// streaming floor: the same loads, xor-reduced, no prologue
template <int T, int NW, int RW, int C, int PAIR>
__global__ __launch_bounds__(NW * 64) void gv_floor(GV a) {
    using K = Kq<T>;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int sbl = lane >> 3, j = lane & 7;
    const int nb = a.nb;
    const int u = min(blockIdx.x * NW + wave, a.units - 1);
    unsigned acc = 0;
#pragma unroll
    for (int r = 0; r < RW; ++r) {
        const long long row = PAIR ? u : (long long)u * RW + r;
        const long long rr = row < a.rows ? row : a.rows - 1;
        const uint8_t* rp[4];
#pragma unroll
        for (int p = 0; p < 4; ++p) rp[p] = ((PAIR && r == 1) ? a.B[p] : a.A[p]) + rr * nb * K::pb[p];
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const int sb = 8 * c + sbl;
            acc ^= K::load(rp, sb < nb ? sb : nb - 1, j).fold();
        }
    }
    if (acc == 0x9e3779b9u) a.out[u] = (float)acc;
}

typedef void (*KFn)(GV);

struct Mat {   // one quantised matrix, planes in one allocation
    int type, rows, nb;
    uint8_t* p[4];
    size_t bytes;
};
static Mat make_mat(int type, int rows, int K) {
    Mat m{type, rows, K / 256, {nullptr, nullptr, nullptr, nullptr}, 0};
    const int pb4[4] = {128, 16, 0, 0}, pb6[4] = {128, 64, 16, 2};
    const int* pb = type == Q4K ? pb4 : pb6;
    size_t off[4], tot = 0;
    for (int p = 0; p < 4; ++p) {
        off[p] = tot;
        tot += ((size_t)rows * m.nb * pb[p] + 4096 + 255) & ~(size_t)255;
    }
    uint8_t* base;
    CK(hipMalloc(&base, tot));
    // bytes: pseudo-random; Q4_K headers / Q6_K d: small f16 scales
    std::vector<uint8_t> h(tot);
    uint32_t s = 12345u + rows * 7 + K;
    for (size_t i = 0; i < tot; ++i) { s = s * 1664525u + 1013904223u; h[i] = (uint8_t)(s >> 24); }
    auto f16 = [](float f) { __half x = __float2half(f); return *reinterpret_cast<uint16_t*>(&x); };
    if (type == Q4K) {
        for (size_t r = 0; r < (size_t)rows * m.nb; ++r) {
            uint16_t* hd = reinterpret_cast<uint16_t*>(&h[off[1] + r * 16]);
            hd[0] = f16(1e-3f); hd[1] = f16(5e-4f);
        }
    } else {
        for (size_t r = 0; r < (size_t)rows * m.nb; ++r) *reinterpret_cast<uint16_t*>(&h[off[3] + r * 2]) = f16(1e-3f);
    }
    CK(hipMemcpy(base, h.data(), tot, hipMemcpyHostToDevice));
    for (int p = 0; p < 4; ++p) m.p[p] = base + off[p];
    m.bytes = (size_t)rows * m.nb * (type == Q4K ? 144 : 210);
    return m;
}

struct Launch {
    KFn fn;
    int nw, grid, smem;
    GV a;
    size_t bytes;
};
static void run(const Launch& L, hipStream_t s) { hipLaunchKernelGGL(L.fn, dim3(L.grid), dim3(L.nw * 64), L.smem, s, L.a); }

template <int T, int NW, int RW, int C, int PRO, int PAIR, int LOOP, int ORDER = 1, int PIPE = 2>
static Launch mk(const Mat& A, const Mat* B, const float* x, const float* nw, const int8_t* q8, const int* bs,
                 const float* dk, float* out, int grid_cap = 0) {
    Launch L;
    L.fn = gv<T, NW, RW, C, PRO, PAIR, LOOP, ORDER, PIPE>;
    L.nw = NW;
    GV& a = L.a;
    for (int p = 0; p < 4; ++p) { a.A[p] = A.p[p]; a.B[p] = B ? B->p[p] : A.p[p]; }
    a.x = x; a.nw = nw; a.q8 = q8; a.bsum = bs; a.dk = dk; a.out = out;
    a.rows = A.rows; a.nb = A.nb; a.st = nullptr;
    a.units = PAIR ? A.rows : (A.rows + RW - 1) / RW;
    L.grid = (a.units + NW - 1) / NW;
    if (LOOP && grid_cap > 0) L.grid = std::min(L.grid, grid_cap);
    L.smem = lds_bytes(A.nb);
    L.bytes = A.bytes + (B ? B->bytes : 0);
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(L.fn), hipFuncAttributeMaxDynamicSharedMemorySize, 65536));
    return L;
}
template <int T, int NW, int RW, int C, int PAIR>
static Launch mk_floor(const Mat& A, const Mat* B, float* out) {
    Launch L;
    L.fn = gv_floor<T, NW, RW, C, PAIR>;
    L.nw = NW;
    GV& a = L.a;
    for (int p = 0; p < 4; ++p) { a.A[p] = A.p[p]; a.B[p] = B ? B->p[p] : A.p[p]; }
    a.out = out; a.rows = A.rows; a.nb = A.nb; a.st = nullptr;
    a.units = PAIR ? A.rows : (A.rows + RW - 1) / RW;
    L.grid = (a.units + NW - 1) / NW;
    L.smem = 0;
    L.bytes = A.bytes + (B ? B->bytes : 0);
    return L;
}

// time one launch kind over nrot weight copies (rotation defeats the 256 MiB Infinity Cache)
static unsigned long long* g_st = nullptr;
static void time_kind(const char* name, std::vector<Launch> Ls, hipStream_t s) {
#ifdef STAMPS
    {
        // one launch after 8 back-to-back ones; phases per workgroup (us, 100 MHz clock)
        for (auto& L : Ls) L.a.st = nullptr;
        for (int i = 0; i < 8; ++i) run(Ls[i % Ls.size()], s);
        Launch L = Ls[0];
        L.a.st = g_st;
        CK(hipMemsetAsync(g_st, 0, 8192 * 4 * 8, s));
        run(L, s);
        CK(hipStreamSynchronize(s));
        std::vector<unsigned long long> h(L.grid * 4);
        CK(hipMemcpy(h.data(), g_st, h.size() * 8, hipMemcpyDeviceToHost));
        unsigned long long t0 = ~0ull, tend = 0, e1 = 0;
        std::vector<double> act, first, end, entry;
        for (int g = 0; g < L.grid; ++g) t0 = std::min(t0, h[g * 4]);
        for (int g = 0; g < L.grid; ++g) {
            entry.push_back((h[g * 4] - t0) / 100.0);
            act.push_back((h[g * 4 + 1] - h[g * 4]) / 100.0);
            if (h[g * 4 + 2]) first.push_back((h[g * 4 + 2] - h[g * 4]) / 100.0);
            end.push_back((h[g * 4 + 3] - h[g * 4]) / 100.0);
            tend = std::max(tend, h[g * 4 + 3]);
        }
        auto med = [](std::vector<double> v) { if (v.empty()) return -1.0; std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
        auto mx = [](std::vector<double> v) { return v.empty() ? -1.0 : *std::max_element(v.begin(), v.end()); };
        printf("  stamps %-36s entry spread %5.2f  act %5.2f (max %5.2f)  first %5.2f  end %5.2f (max %5.2f)  span %5.2f us\n",
               name, mx(entry), med(act), mx(act), med(first), med(end), mx(end), (tend - t0) / 100.0);
        (void)e1;
        for (auto& L2 : Ls) L2.a.st = nullptr;
    }
#endif
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int i = 0; i < 8; ++i) run(Ls[i % Ls.size()], s);
    CK(hipStreamSynchronize(s));
    std::vector<float> single;
    for (int i = 0; i < 48; ++i) {
        CK(hipEventRecord(e0, s));
        run(Ls[i % Ls.size()], s);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        single.push_back(ms * 1e3f);
    }
    std::sort(single.begin(), single.end());
    // back to back, as a graph
    hipGraph_t g; hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int i = 0; i < 64; ++i) run(Ls[i % Ls.size()], s);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(e0, s));
    for (int r = 0; r < 4; ++r) CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    const double btb = ms * 1e3 / 256.0;
    const double by = (double)Ls[0].bytes;
    printf("%-44s grid %5d  single %7.2f us (%4.2f TB/s)  graph %7.2f us (%4.2f TB/s)\n", name, Ls[0].grid,
           single[single.size() / 2], by / single[single.size() / 2] / 1e6, btb, by / btb / 1e6);
    fflush(stdout);
    CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g));
}

int main(int argc, char** argv) {
    const int nrot = 6;
    hipStream_t s;
    CK(hipStreamCreate(&s));
    float *x, *nw, *dk, *out, *h;
    int8_t* q8;
    int* bs;
    CK(hipMalloc(&x, 16384 * 4)); CK(hipMalloc(&nw, 16384 * 4)); CK(hipMalloc(&dk, 64 * 4));
    CK(hipMalloc(&out, 65536 * 4)); CK(hipMalloc(&h, 65536 * 4));
    CK(hipMalloc(&q8, 16384)); CK(hipMalloc(&bs, 16384 * 4));
    CK(hipMalloc(&g_st, 8192 * 4 * 8));
    {
        std::vector<float> hx(16384), hw(16384, 1.0f);
        for (int i = 0; i < 16384; ++i) hx[i] = 0.01f * (float)((i * 37) % 101 - 50);
        CK(hipMemcpy(x, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(nw, hw.data(), hw.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(h, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemset(q8, 3, 16384)); CK(hipMemset(bs, 0, 16384 * 4));
        std::vector<float> hd(64, 1e-2f);
        CK(hipMemcpy(dk, hd.data(), 64 * 4, hipMemcpyHostToDevice));
    }
    const bool single = argc < 2 || atoi(argv[1]) != 2;
    const bool chain = argc < 2 || atoi(argv[1]) != 1;
    if (single) {
        std::vector<Mat> wo, gate, up, down4, down6, qkv;
        for (int i = 0; i < nrot; ++i) {
            wo.push_back(make_mat(Q4K, 4096, 4096));
            gate.push_back(make_mat(Q4K, 11008, 4096));
            up.push_back(make_mat(Q4K, 11008, 4096));
            down4.push_back(make_mat(Q4K, 4096, 11008));
            down6.push_back(make_mat(Q6K, 4096, 11008));
            qkv.push_back(make_mat(Q4K, 12288, 4096));
        }
        auto many = [&](auto f) { std::vector<Launch> v; for (int i = 0; i < nrot; ++i) v.push_back(f(i)); return v; };
#define KIND(name, expr) time_kind(name, many([&](int i) { return expr; }), s)
        KIND("floor  WO q4k nw8 rw1", (mk_floor<Q4K, 8, 1, 2, 0>(wo[i], nullptr, out)));
        KIND("plain  WO nw8  o1", (mk<Q4K, 8, 1, 2, 2, 0, 0, 1>(wo[i], nullptr, x, nw, q8, bs, dk, out)));
        KIND("plain  WO nw16 o1", (mk<Q4K, 16, 1, 2, 2, 0, 0, 1>(wo[i], nullptr, x, nw, q8, bs, dk, out)));
        KIND("plain  WO nw8  o2", (mk<Q4K, 8, 1, 2, 2, 0, 0, 2>(wo[i], nullptr, x, nw, q8, bs, dk, out)));
        KIND("plain  WO nw8  o0", (mk<Q4K, 8, 1, 2, 2, 0, 0, 0>(wo[i], nullptr, x, nw, q8, bs, dk, out)));
        KIND("rms    WO nw16 o1", (mk<Q4K, 16, 1, 2, 1, 0, 0, 1>(wo[i], nullptr, x, nw, q8, bs, dk, out)));
        KIND("floor  QKV q4k nw8 rw1", (mk_floor<Q4K, 8, 1, 2, 0>(qkv[i], nullptr, out)));
        KIND("rms    QKV nw16 o1 oneshot", (mk<Q4K, 16, 1, 2, 1, 0, 0, 1>(qkv[i], nullptr, x, nw, q8, bs, dk, out)));
        KIND("rms    QKV nw8  o1 l256 p1", (mk<Q4K, 8, 1, 2, 1, 0, 1, 1, 1>(qkv[i], nullptr, x, nw, q8, bs, dk, out, 256)));
        KIND("rms    QKV nw16 o1 l256 p1", (mk<Q4K, 16, 1, 2, 1, 0, 1, 1, 1>(qkv[i], nullptr, x, nw, q8, bs, dk, out, 256)));
        KIND("rms    QKV nw8  o1 l256 p2", (mk<Q4K, 8, 1, 2, 1, 0, 1, 1, 2>(qkv[i], nullptr, x, nw, q8, bs, dk, out, 256)));
        KIND("rms    QKV nw8  o2 l256 p1", (mk<Q4K, 8, 1, 2, 1, 0, 1, 2, 1>(qkv[i], nullptr, x, nw, q8, bs, dk, out, 256)));
        KIND("rms    QKV nw8  o1 l512 p1", (mk<Q4K, 8, 1, 2, 1, 0, 1, 1, 1>(qkv[i], nullptr, x, nw, q8, bs, dk, out, 512)));
        KIND("floor  UP  q4k nw8 pair", (mk_floor<Q4K, 8, 2, 2, 1>(gate[i], &up[i], out)));
        KIND("rms    UP  nw8  o1 l256 p1", (mk<Q4K, 8, 2, 2, 1, 1, 1, 1, 1>(gate[i], &up[i], x, nw, q8, bs, dk, out, 256)));
        KIND("rms    UP  nw16 o1 l256 p1", (mk<Q4K, 16, 2, 2, 1, 1, 1, 1, 1>(gate[i], &up[i], x, nw, q8, bs, dk, out, 256)));
        KIND("rms    UP  nw8  o1 l256 p2", (mk<Q4K, 8, 2, 2, 1, 1, 1, 1, 2>(gate[i], &up[i], x, nw, q8, bs, dk, out, 256)));
        KIND("rms    UP  nw8  o1 l512 p1", (mk<Q4K, 8, 2, 2, 1, 1, 1, 1, 1>(gate[i], &up[i], x, nw, q8, bs, dk, out, 512)));
        KIND("rms    UP  nw4  o1 l512 p2", (mk<Q4K, 4, 2, 2, 1, 1, 1, 1, 2>(gate[i], &up[i], x, nw, q8, bs, dk, out, 512)));
        KIND("rms    UP  nw8  o2 l256 p1", (mk<Q4K, 8, 2, 2, 1, 1, 1, 2, 1>(gate[i], &up[i], x, nw, q8, bs, dk, out, 256)));
        KIND("floor  DOWN q4k nw8 rw1", (mk_floor<Q4K, 8, 1, 6, 0>(down4[i], nullptr, out)));
        KIND("plain  DOWN4 nw16 o1", (mk<Q4K, 16, 1, 6, 2, 0, 0, 1>(down4[i], nullptr, h, nw, q8, bs, dk, out)));
        KIND("plain  DOWN4 nw8  o1", (mk<Q4K, 8, 1, 6, 2, 0, 0, 1>(down4[i], nullptr, h, nw, q8, bs, dk, out)));
        KIND("plain  DOWN4 nw8  o1 l256 p1", (mk<Q4K, 8, 1, 6, 2, 0, 1, 1, 1>(down4[i], nullptr, h, nw, q8, bs, dk, out, 256)));
        KIND("plain  DOWN4 nw4  o1 l256 p2", (mk<Q4K, 4, 1, 6, 2, 0, 1, 1, 2>(down4[i], nullptr, h, nw, q8, bs, dk, out, 256)));
        KIND("plain  DOWN4 nw16 o2", (mk<Q4K, 16, 1, 6, 2, 0, 0, 2>(down4[i], nullptr, h, nw, q8, bs, dk, out)));
        KIND("floor  DOWN q6k nw8 rw1", (mk_floor<Q6K, 8, 1, 6, 0>(down6[i], nullptr, out)));
        KIND("plain  DOWN6 nw16 o1", (mk<Q6K, 16, 1, 6, 2, 0, 0, 1>(down6[i], nullptr, h, nw, q8, bs, dk, out)));
        KIND("plain  DOWN6 nw8  o1 l256 p1", (mk<Q6K, 8, 1, 6, 2, 0, 1, 1, 1>(down6[i], nullptr, h, nw, q8, bs, dk, out, 256)));
#undef KIND
    }
    if (chain) {
        // a 7B Q4_K_M-like step: 32 layers x {QKV, WO, gate/up, down (Q6_K on the use_more_bits
        // layers)} + the Q6_K output head, as one captured graph
        const int L = 32;
        std::vector<Launch> step, step_b, step_c, step_floor;
        size_t bytes = 0;
        for (int l = 0; l < L; ++l) {
            const bool more = l < L / 8 || l >= 7 * L / 8 || (l - L / 8) % 3 == 2;
            Mat qkv = make_mat(Q4K, 12288, 4096), wo = make_mat(Q4K, 4096, 4096);
            Mat g = make_mat(Q4K, 11008, 4096), u = make_mat(Q4K, 11008, 4096);
            Mat d = make_mat(more ? Q6K : Q4K, 4096, 11008);
            // A: the previous best (no ordering barrier, 2 units in flight)
            step.push_back(mk<Q4K, 16, 1, 2, 1, 0, 1, 0, 2>(qkv, nullptr, x, nw, q8, bs, dk, out, 256));
            step.push_back(mk<Q4K, 16, 1, 2, 2, 0, 0, 0>(wo, nullptr, out, nw, q8, bs, dk, h));
            step.push_back(mk<Q4K, 8, 2, 2, 1, 1, 1, 0, 2>(g, &u, x, nw, q8, bs, dk, h, 256));
            if (more) step.push_back(mk<Q6K, 16, 1, 6, 2, 0, 0, 0>(d, nullptr, h, nw, q8, bs, dk, out));
            else step.push_back(mk<Q4K, 16, 1, 6, 2, 0, 0, 0>(d, nullptr, h, nw, q8, bs, dk, out));
            // B: activation first (barrier), one unit in flight per wave, 8 waves
            step_b.push_back(mk<Q4K, 8, 1, 2, 1, 0, 1, 1, 1>(qkv, nullptr, x, nw, q8, bs, dk, out, 256));
            step_b.push_back(mk<Q4K, 8, 1, 2, 2, 0, 0, 1>(wo, nullptr, out, nw, q8, bs, dk, h));
            step_b.push_back(mk<Q4K, 8, 2, 2, 1, 1, 1, 1, 1>(g, &u, x, nw, q8, bs, dk, h, 256));
            if (more) step_b.push_back(mk<Q6K, 8, 1, 6, 2, 0, 1, 1, 1>(d, nullptr, h, nw, q8, bs, dk, out, 256));
            else step_b.push_back(mk<Q4K, 8, 1, 6, 2, 0, 1, 1, 1>(d, nullptr, h, nw, q8, bs, dk, out, 256));
            // C: activation first, 16 waves one-shot / loops
            step_c.push_back(mk<Q4K, 16, 1, 2, 1, 0, 1, 1, 1>(qkv, nullptr, x, nw, q8, bs, dk, out, 256));
            step_c.push_back(mk<Q4K, 16, 1, 2, 2, 0, 0, 1>(wo, nullptr, out, nw, q8, bs, dk, h));
            step_c.push_back(mk<Q4K, 16, 2, 2, 1, 1, 1, 1, 1>(g, &u, x, nw, q8, bs, dk, h, 256));
            if (more) step_c.push_back(mk<Q6K, 16, 1, 6, 2, 0, 0, 1>(d, nullptr, h, nw, q8, bs, dk, out));
            else step_c.push_back(mk<Q4K, 16, 1, 6, 2, 0, 0, 1>(d, nullptr, h, nw, q8, bs, dk, out));
            step_floor.push_back(mk_floor<Q4K, 8, 1, 2, 0>(qkv, nullptr, out));
            step_floor.push_back(mk_floor<Q4K, 8, 1, 2, 0>(wo, nullptr, out));
            step_floor.push_back(mk_floor<Q4K, 8, 2, 2, 1>(g, &u, out));
            if (more) step_floor.push_back(mk_floor<Q6K, 8, 1, 6, 0>(d, nullptr, out));
            else step_floor.push_back(mk_floor<Q4K, 8, 1, 6, 0>(d, nullptr, out));
            bytes += qkv.bytes + wo.bytes + g.bytes + u.bytes + d.bytes;
        }
        Mat o = make_mat(Q6K, 32000, 4096);
        step.push_back(mk<Q6K, 16, 1, 2, 1, 0, 1, 0, 2>(o, nullptr, x, nw, q8, bs, dk, out, 256));
        step_b.push_back(mk<Q6K, 8, 1, 2, 1, 0, 1, 1, 1>(o, nullptr, x, nw, q8, bs, dk, out, 256));
        step_c.push_back(mk<Q6K, 16, 1, 2, 1, 0, 1, 1, 1>(o, nullptr, x, nw, q8, bs, dk, out, 256));
        step_floor.push_back(mk_floor<Q6K, 8, 1, 2, 0>(o, nullptr, out));
        bytes += o.bytes;
        const char* names[4] = {"prev", "o1-nw8-p1", "o1-nw16", "floor"};
        for (int pass = 0; pass < 4; ++pass) {
            const auto& st = pass == 0 ? step : pass == 1 ? step_b : pass == 2 ? step_c : step_floor;
            hipGraph_t g; hipGraphExec_t ge;
            CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
            for (const auto& Lc : st) run(Lc, s);
            CK(hipStreamEndCapture(s, &g));
            CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
            for (int i = 0; i < 3; ++i) CK(hipGraphLaunch(ge, s));
            CK(hipStreamSynchronize(s));
            hipEvent_t e0, e1;
            CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
            const int reps = 20;
            CK(hipEventRecord(e0, s));
            for (int i = 0; i < reps; ++i) CK(hipGraphLaunch(ge, s));
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1));
            const double per = ms / reps;
            printf("chain %-8s: %zu launches, %.3f GB, %.3f ms/step = %.1f tok/s, %.2f TB/s\n", names[pass],
                   st.size(), bytes / 1e9, per, 1e3 / per, bytes / per / 1e9);
            fflush(stdout);
        }
    }
    return 0;
}
