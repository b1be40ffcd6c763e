/* C restatement of the ggml CPU path of llama.cpp tag b5187 for the llama graph.
 *
 * TEST INFRASTRUCTURE ONLY -- the checker and the CPU baseline, never part of
 * the product (blama_amd/ never links or loads it).  ggml is a third-party
 * dependency of the reference (pinned at
 * /root/reference/inference/code/CMakeLists.txt:35) that is not present here;
 * this file restates the published scalar algorithms of
 *   ggml/src/ggml-quants.c          dequantize_row_*, quantize_row_q8_K_ref
 *   ggml/src/ggml-cpu/ggml-cpu-quants.c  ggml_vec_dot_{q4_K,q5_K,q6_K}_q8_K,
 *                                   ggml_vec_dot_q8_0_q8_0 (generic paths),
 *                                   quantize_row_q8_0 (x86 SIMD rounding)
 *   ggml/src/ggml-cpu/ggml-cpu.c    rms_norm, rope (NORM), soft_max, silu,
 *                                   ggml_vec_dot_f16 (double accumulation)
 *   src/llama-model.cpp             llm_build_llama (batch-1 decode order)
 * independently of oracle/ggml_ref.py (numpy), against which tests cross-check
 * it.  Reference call sites: Model.cpp:13-16 (gpu=false selects this path),
 * Session.cpp:388 (llama_decode), Session.cpp:24 (logits).
 *
 * Parity of the quant formats is "unpinned" (no reference test covers them;
 * SURVEY.md §8c5): see oracle/ggml_ref.py's header.
 */
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define QK_K 256
enum { T_F32 = 0, T_F16 = 1, T_Q8_0 = 8, T_Q4_K = 12, T_Q5_K = 13, T_Q6_K = 14 };

/* ---------------------------------------------------------------- fp16 ---- */
static float h2f(uint16_t h) {
    const uint32_t s = (uint32_t)(h >> 15) << 31, e = (h >> 10) & 0x1F, m = h & 0x3FF;
    uint32_t u;
    if (e == 0) {
        if (m == 0) u = s;
        else {   /* subnormal */
            float f = (float)m * (1.0f / 16777216.0f);
            memcpy(&u, &f, 4);
            u |= s;
        }
    } else if (e == 31) u = s | 0x7F800000 | (m << 13);
    else u = s | ((e + 112) << 23) | (m << 13);
    float f;
    memcpy(&f, &u, 4);
    return f;
}

static uint16_t f2h(float f) {   /* round to nearest even (F16C _cvtss_sh(x, 0)) */
    uint32_t x;
    memcpy(&x, &f, 4);
    const uint32_t sign = (x >> 16) & 0x8000;
    const uint32_t ax = x & 0x7FFFFFFF;
    if (ax >= 0x7F800000) return (uint16_t)(sign | 0x7C00 | (ax > 0x7F800000 ? 0x200 : 0));
    if (ax >= 0x477FF000) return (uint16_t)(sign | 0x7C00);   /* rounds to inf */
    if (ax < 0x38800000) {                                      /* subnormal half */
        float a;
        memcpy(&a, &ax, 4);
        const float r = a * 16777216.0f;                        /* units of 2^-24 */
        float ri = rintf(r);
        return (uint16_t)(sign | (uint32_t)ri);
    }
    const uint32_t mant = ax & 0x7FFFFF, exp = (ax >> 23) - 112;
    uint32_t h = (exp << 10) | (mant >> 13);
    const uint32_t rem = mant & 0x1FFF;
    if (rem > 0x1000 || (rem == 0x1000 && (h & 1))) h++;
    return (uint16_t)(sign | h);
}

/* --------------------------------------------------- activation quant ---- */
typedef struct { float d; int8_t qs[QK_K]; int16_t bsums[QK_K / 16]; } q8k_t;
typedef struct { float d; int8_t qs[32]; } q80_t;   /* d already rounded through fp16 */

static int nearest_int(float f) {
    float v = f + 12582912.f;
    int i;
    memcpy(&i, &v, 4);
    return (i & 0x007fffff) - 0x00400000;
}

void orc_quantize_q8_K(const float* x, int K, q8k_t* y) {   /* quantize_row_q8_K_ref */
    for (int b = 0; b < K / QK_K; ++b, x += QK_K) {
        float mx = 0, amax = 0;
        for (int j = 0; j < QK_K; ++j) {
            const float ax = fabsf(x[j]);
            if (ax > amax) { amax = ax; mx = x[j]; }
        }
        if (amax == 0) {
            y[b].d = 0;
            memset(y[b].qs, 0, QK_K);
            memset(y[b].bsums, 0, sizeof(y[b].bsums));
            continue;
        }
        const float iscale = -127.f / mx;
        for (int j = 0; j < QK_K; ++j) {
            const int v = nearest_int(iscale * x[j]);
            y[b].qs[j] = (int8_t)(v < 127 ? v : 127);
        }
        for (int j = 0; j < QK_K / 16; ++j) {
            int s = 0;
            for (int i = 0; i < 16; ++i) s += y[b].qs[j * 16 + i];
            y[b].bsums[j] = (int16_t)s;
        }
        y[b].d = 1 / iscale;
    }
}

static void quantize_q8_0(const float* x, int K, q80_t* y) {   /* x86 SIMD quantize_row_q8_0 */
    for (int b = 0; b < K / 32; ++b, x += 32) {
        float amax = 0;
        for (int j = 0; j < 32; ++j) amax = fmaxf(amax, fabsf(x[j]));
        const float d = amax / 127.f;
        const float id = amax != 0.0f ? 127.f / amax : 0.0f;
        y[b].d = h2f(f2h(d));
        for (int j = 0; j < 32; ++j) y[b].qs[j] = (int8_t)rintf(x[j] * id);
    }
}

/* ----------------------------------------------------------- vec_dot ---- */
static void scale_min_k4(int j, const uint8_t* q, uint8_t* d, uint8_t* m) {
    if (j < 4) { *d = q[j] & 63; *m = q[j + 4] & 63; }
    else { *d = (q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4); *m = (q[j + 4] >> 4) | ((q[j - 0] >> 6) << 4); }
}

/* ORC_ALT=1: sum the 8 float lanes in reverse order -- a second, equally valid
 * fp32 accumulation order, used to measure how far two correct implementations
 * drift apart on a given model (test infrastructure only) */
static int g_alt = -1;
static int alt_order(void) {
    if (g_alt < 0) g_alt = getenv("ORC_ALT") != NULL;
    return g_alt;
}
/* switch the accumulation order in-process (tests measure the algorithm's own noise floor) */
void orc_set_alt(int on) { g_alt = on ? 1 : 0; }
static float lane_sum(const float* sums, float init) {
    float s = init;
    if (alt_order()) for (int l = 7; l >= 0; --l) s += sums[l];
    else for (int l = 0; l < 8; ++l) s += sums[l];
    return s;
}

/* ggml_vec_dot_q4_K_q8_K / q5_K (generic): exact integer sums per sub-block,
 * per-lane float accumulators sums[8], mins subtracted per superblock. */
static float dot_q45_K(const uint8_t* row, int K, const q8k_t* y, int q5) {
    const int bb = q5 ? 176 : 144;
    float sums[8] = {0};
    float sumf = 0;
    for (int i = 0; i < K / QK_K; ++i) {
        const uint8_t* blk = row + (size_t)i * bb;
        const uint8_t* sc = blk + 4;
        const uint8_t* qh = q5 ? blk + 16 : NULL;
        const uint8_t* qs = blk + (q5 ? 48 : 16);
        int8_t a[QK_K];
        for (int c = 0; c < 4; ++c)
            for (int l = 0; l < 32; ++l) {
                a[64 * c + l] = (int8_t)((qs[32 * c + l] & 0xF) + (q5 && (qh[l] >> (2 * c) & 1) ? 16 : 0));
                a[64 * c + 32 + l] = (int8_t)((qs[32 * c + l] >> 4) + (q5 && (qh[l] >> (2 * c + 1) & 1) ? 16 : 0));
            }
        uint8_t scl[8], mn[8];
        for (int j = 0; j < 8; ++j) scale_min_k4(j, sc, &scl[j], &mn[j]);
        int sumi = 0;
        for (int j = 0; j < QK_K / 16; ++j) sumi += y[i].bsums[j] * mn[j / 2];
        int32_t aux32[8] = {0};
        const int8_t* q8 = y[i].qs;
        for (int j = 0; j < QK_K / 32; ++j)
            for (int k = 0; k < 4; ++k)
                for (int l = 0; l < 8; ++l) aux32[l] += scl[j] * (q8[32 * j + 8 * k + l] * a[32 * j + 8 * k + l]);
        uint16_t dh, dmh;
        memcpy(&dh, blk, 2);
        memcpy(&dmh, blk + 2, 2);
        const float d = h2f(dh) * y[i].d;
        for (int l = 0; l < 8; ++l) sums[l] += d * aux32[l];
        const float dmin = h2f(dmh) * y[i].d;
        sumf -= dmin * sumi;
    }
    return lane_sum(sums, sumf);
}

static float dot_q6_K(const uint8_t* row, int K, const q8k_t* y) {   /* ggml_vec_dot_q6_K_q8_K */
    float sums[8] = {0};
    for (int i = 0; i < K / QK_K; ++i) {
        const uint8_t* blk = row + (size_t)i * 210;
        const uint8_t* ql = blk;
        const uint8_t* qh = blk + 128;
        const int8_t* sc = (const int8_t*)(blk + 192);
        int8_t a[QK_K];
        for (int h = 0; h < 2; ++h)
            for (int l = 0; l < 32; ++l) {
                a[128 * h + l] = (int8_t)(((ql[64 * h + l] & 0xF) | (((qh[32 * h + l] >> 0) & 3) << 4)) - 32);
                a[128 * h + l + 32] = (int8_t)(((ql[64 * h + l + 32] & 0xF) | (((qh[32 * h + l] >> 2) & 3) << 4)) - 32);
                a[128 * h + l + 64] = (int8_t)(((ql[64 * h + l] >> 4) | (((qh[32 * h + l] >> 4) & 3) << 4)) - 32);
                a[128 * h + l + 96] = (int8_t)(((ql[64 * h + l + 32] >> 4) | (((qh[32 * h + l] >> 6) & 3) << 4)) - 32);
            }
        int32_t aux32[8] = {0};
        const int8_t* q8 = y[i].qs;
        for (int j = 0; j < QK_K / 16; ++j)
            for (int k = 0; k < 2; ++k)
                for (int l = 0; l < 8; ++l) aux32[l] += sc[j] * (q8[16 * j + 8 * k + l] * a[16 * j + 8 * k + l]);
        uint16_t dh;
        memcpy(&dh, blk + 208, 2);
        const float d = h2f(dh) * y[i].d;
        for (int l = 0; l < 8; ++l) sums[l] += d * aux32[l];
    }
    return lane_sum(sums, 0.0f);
}

static float dot_q8_0(const uint8_t* row, int K, const q80_t* y) {   /* ggml_vec_dot_q8_0_q8_0 */
    float sumf = 0;
    const int nb = K / 32;
    /* ORC_ALT: the blocks summed last to first -- an fp32 order as valid as the generic loop's
       (the AVX2 path keeps 8 running sums; ggml-cpu's block order differs between its paths) */
    for (int bi = 0; bi < nb; ++bi) {
        const int b = alt_order() ? nb - 1 - bi : bi;
        const uint8_t* blk = row + (size_t)b * 34;
        const int8_t* q = (const int8_t*)(blk + 2);
        int sumi = 0;
        for (int j = 0; j < 32; ++j) sumi += q[j] * y[b].qs[j];
        uint16_t dh;
        memcpy(&dh, blk, 2);
        sumf += sumi * (h2f(dh) * y[b].d);
    }
    return sumf;
}

/* ---------------------------------------------- x86 AVX2 dot kernels ---- *
 * The CPU-baseline leg of bench.py times the reference's CPU path; on x86 ggml b5187 runs the
 * AVX2 forms of these dots (ggml-cpu-quants.c ggml_vec_dot_{q4_K,q5_K,q6_K}_q8_K,
 * ggml_vec_dot_q8_0_q8_0 under __AVX2__), not the generic loops above.  These restate that
 * technique: maddubs of the unsigned quants against the signed Q8 bytes, madd by the sub-block
 * scales, an int32 vector per superblock converted once and fused into 8 float lanes by d.  Every
 * integer is the one the generic loop forms; only the fp32 lane grouping differs (so results
 * match the scalar loops to rounding, not bit for bit).  Off by default: the parity tests keep
 * the generic order (orc_set_simd / ORC_SIMD=1 switch it on for timing). */
#include <immintrin.h>
static int g_simd = -1;
static int use_simd(void) {
    if (g_simd < 0) g_simd = getenv("ORC_SIMD") != NULL && atoi(getenv("ORC_SIMD")) != 0;
    return g_simd;
}
void orc_set_simd(int on) { g_simd = on ? 1 : 0; }
static float hsum8(__m256 v) {
    __m128 a = _mm_add_ps(_mm256_castps256_ps128(v), _mm256_extractf128_ps(v, 1));
    a = _mm_add_ps(a, _mm_movehl_ps(a, a));
    a = _mm_add_ss(a, _mm_movehdup_ps(a));
    return _mm_cvtss_f32(a);
}
/* Q4_K (q5 = 0) / Q5_K (q5 = 1) */
static float dot_q45_K_avx2(const uint8_t* row, int K, const q8k_t* y, int q5) {
    const int bb = q5 ? 176 : 144;
    const __m256i m4 = _mm256_set1_epi8(0x0F), m1 = _mm256_set1_epi8(0x01);
    __m256 acc = _mm256_setzero_ps();
    float summ = 0.0f;
    for (int i = 0; i < K / QK_K; ++i) {
        const uint8_t* blk = row + (size_t)i * bb;
        const uint8_t* qs = blk + (q5 ? 48 : 16);
        uint8_t scl[8], mn[8];
        for (int j = 0; j < 8; ++j) scale_min_k4(j, blk + 4, &scl[j], &mn[j]);
        int sumi_m = 0;
        for (int j = 0; j < QK_K / 16; ++j) sumi_m += y[i].bsums[j] * mn[j / 2];
        const __m256i qhv = q5 ? _mm256_loadu_si256((const __m256i*)(blk + 16)) : _mm256_setzero_si256();
        __m256i sumi = _mm256_setzero_si256();
        for (int c = 0; c < 4; ++c) {
            const __m256i qb = _mm256_loadu_si256((const __m256i*)(qs + 32 * c));
            __m256i lo = _mm256_and_si256(qb, m4), hi = _mm256_and_si256(_mm256_srli_epi16(qb, 4), m4);
            if (q5) {
                lo = _mm256_add_epi8(lo, _mm256_slli_epi16(_mm256_and_si256(_mm256_srli_epi16(qhv, 2 * c), m1), 4));
                hi = _mm256_add_epi8(hi, _mm256_slli_epi16(_mm256_and_si256(_mm256_srli_epi16(qhv, 2 * c + 1), m1), 4));
            }
            const __m256i yl = _mm256_loadu_si256((const __m256i*)(y[i].qs + 64 * c));
            const __m256i yh = _mm256_loadu_si256((const __m256i*)(y[i].qs + 64 * c + 32));
            const __m256i pl = _mm256_madd_epi16(_mm256_set1_epi16(scl[2 * c]), _mm256_maddubs_epi16(lo, yl));
            const __m256i ph = _mm256_madd_epi16(_mm256_set1_epi16(scl[2 * c + 1]), _mm256_maddubs_epi16(hi, yh));
            sumi = _mm256_add_epi32(sumi, _mm256_add_epi32(pl, ph));
        }
        uint16_t dh, dmh;
        memcpy(&dh, blk, 2);
        memcpy(&dmh, blk + 2, 2);
        acc = _mm256_fmadd_ps(_mm256_set1_ps(h2f(dh) * y[i].d), _mm256_cvtepi32_ps(sumi), acc);
        summ -= h2f(dmh) * y[i].d * sumi_m;
    }
    return hsum8(acc) + summ;
}
static float dot_q6_K_avx2(const uint8_t* row, int K, const q8k_t* y) {
    const __m256i m4 = _mm256_set1_epi8(0x0F), m3 = _mm256_set1_epi8(0x03), m32 = _mm256_set1_epi8(32);
    __m256 acc = _mm256_setzero_ps();
    for (int i = 0; i < K / QK_K; ++i) {
        const uint8_t* blk = row + (size_t)i * 210;
        const int8_t* sc = (const int8_t*)(blk + 192);
        __m256i sumi = _mm256_setzero_si256();
        for (int h = 0; h < 2; ++h) {
            const __m256i l0 = _mm256_loadu_si256((const __m256i*)(blk + 64 * h));
            const __m256i l1 = _mm256_loadu_si256((const __m256i*)(blk + 64 * h + 32));
            const __m256i qh = _mm256_loadu_si256((const __m256i*)(blk + 128 + 32 * h));
            const __m256i q[4] = {
                _mm256_or_si256(_mm256_and_si256(l0, m4), _mm256_slli_epi16(_mm256_and_si256(qh, m3), 4)),
                _mm256_or_si256(_mm256_and_si256(l1, m4), _mm256_slli_epi16(_mm256_and_si256(_mm256_srli_epi16(qh, 2), m3), 4)),
                _mm256_or_si256(_mm256_and_si256(_mm256_srli_epi16(l0, 4), m4), _mm256_slli_epi16(_mm256_and_si256(_mm256_srli_epi16(qh, 4), m3), 4)),
                _mm256_or_si256(_mm256_and_si256(_mm256_srli_epi16(l1, 4), m4), _mm256_slli_epi16(_mm256_and_si256(_mm256_srli_epi16(qh, 6), m3), 4))};
            for (int g = 0; g < 4; ++g) {   /* elements 128 h + 32 g ..: scales 8 h + 2 g, + 1 */
                const __m256i yv = _mm256_loadu_si256((const __m256i*)(y[i].qs + 128 * h + 32 * g));
                const __m256i p = _mm256_sub_epi16(_mm256_maddubs_epi16(q[g], yv), _mm256_maddubs_epi16(m32, yv));
                const int j = 8 * h + 2 * g;
                const __m256i s = _mm256_setr_epi16(sc[j], sc[j], sc[j], sc[j], sc[j], sc[j], sc[j], sc[j], sc[j + 1],
                                                    sc[j + 1], sc[j + 1], sc[j + 1], sc[j + 1], sc[j + 1], sc[j + 1], sc[j + 1]);
                sumi = _mm256_add_epi32(sumi, _mm256_madd_epi16(s, p));
            }
        }
        uint16_t dh;
        memcpy(&dh, blk + 208, 2);
        acc = _mm256_fmadd_ps(_mm256_set1_ps(h2f(dh) * y[i].d), _mm256_cvtepi32_ps(sumi), acc);
    }
    return hsum8(acc);
}
static float dot_q8_0_avx2(const uint8_t* row, int K, const q80_t* y) {
    __m256 acc = _mm256_setzero_ps();
    for (int b = 0; b < K / 32; ++b) {
        const uint8_t* blk = row + (size_t)b * 34;
        const __m256i x = _mm256_loadu_si256((const __m256i*)(blk + 2));
        const __m256i v = _mm256_loadu_si256((const __m256i*)y[b].qs);
        /* signed x signed: |x| maddubs (v with x's sign), as ggml's mul_sum_i8_pairs_float */
        const __m256i p = _mm256_madd_epi16(_mm256_set1_epi16(1), _mm256_maddubs_epi16(_mm256_sign_epi8(x, x), _mm256_sign_epi8(v, x)));
        uint16_t dh;
        memcpy(&dh, blk, 2);
        acc = _mm256_fmadd_ps(_mm256_set1_ps(h2f(dh) * y[b].d), _mm256_cvtepi32_ps(p), acc);
    }
    return hsum8(acc);
}

static size_t row_bytes(int t, int K) {
    switch (t) {
    case T_Q4_K: return (size_t)K / 256 * 144;
    case T_Q5_K: return (size_t)K / 256 * 176;
    case T_Q6_K: return (size_t)K / 256 * 210;
    case T_Q8_0: return (size_t)K / 32 * 34;
    case T_F32: return (size_t)K * 4;
    case T_F16: return (size_t)K * 2;
    default: return 0;
    }
}

/* y[M] = W . x (ggml_mul_mat with one activation column) */
int orc_gemv(int type, const void* w, int rows, int K, const float* x, float* y) {
    const uint8_t* W = (const uint8_t*)w;
    const size_t rb = row_bytes(type, K);
    if (!rb) return -1;
    q8k_t* a8k = NULL;
    q80_t* a80 = NULL;
    if (type == T_Q4_K || type == T_Q5_K || type == T_Q6_K) {
        a8k = (q8k_t*)malloc(sizeof(q8k_t) * (K / QK_K));
        orc_quantize_q8_K(x, K, a8k);
    } else if (type == T_Q8_0) {
        a80 = (q80_t*)malloc(sizeof(q80_t) * (K / 32));
        quantize_q8_0(x, K, a80);
    }
#pragma omp parallel for schedule(static)
    for (int r = 0; r < rows; ++r) {
        const uint8_t* row = W + (size_t)r * rb;
        float v = 0;
        const int simd = use_simd();
        switch (type) {
        case T_Q4_K: v = simd ? dot_q45_K_avx2(row, K, a8k, 0) : dot_q45_K(row, K, a8k, 0); break;
        case T_Q5_K: v = simd ? dot_q45_K_avx2(row, K, a8k, 1) : dot_q45_K(row, K, a8k, 1); break;
        case T_Q6_K: v = simd ? dot_q6_K_avx2(row, K, a8k) : dot_q6_K(row, K, a8k); break;
        case T_Q8_0: v = simd ? dot_q8_0_avx2(row, K, a80) : dot_q8_0(row, K, a80); break;
        case T_F32: {
            const float* f = (const float*)row;
            double s = 0;   /* ggml_vec_dot_f32 scalar path accumulates in ggml_float */
            for (int k = 0; k < K; ++k) s += (double)(f[k] * x[k]);
            v = (float)s;
            break;
        }
        default: break;
        }
        y[r] = v;
    }
    free(a8k);
    free(a80);
    return 0;
}

/* dequantize_row_* for one row (get_rows of the token embedding) */
static void dequant_row(int type, const uint8_t* row, int K, float* y) {
    if (type == T_F32) { memcpy(y, row, (size_t)K * 4); return; }
    if (type == T_F16) { for (int k = 0; k < K; ++k) { uint16_t h; memcpy(&h, row + 2 * k, 2); y[k] = h2f(h); } return; }
    if (type == T_Q8_0) {
        for (int b = 0; b < K / 32; ++b) {
            uint16_t dh;
            memcpy(&dh, row + b * 34, 2);
            const float d = h2f(dh);
            for (int j = 0; j < 32; ++j) y[b * 32 + j] = ((const int8_t*)(row + b * 34 + 2))[j] * d;
        }
        return;
    }
    if (type == T_Q6_K) {
        for (int i = 0; i < K / QK_K; ++i) {
            const uint8_t* blk = row + (size_t)i * 210;
            uint16_t dh;
            memcpy(&dh, blk + 208, 2);
            const float d = h2f(dh);
            const uint8_t* ql = blk;
            const uint8_t* qh = blk + 128;
            const int8_t* sc = (const int8_t*)(blk + 192);
            float* o = y + i * QK_K;
            for (int n = 0; n < 2; ++n) {
                for (int l = 0; l < 32; ++l) {
                    const int is = l / 16;
                    const int q1 = ((ql[l] & 0xF) | (((qh[l] >> 0) & 3) << 4)) - 32;
                    const int q2 = ((ql[l + 32] & 0xF) | (((qh[l] >> 2) & 3) << 4)) - 32;
                    const int q3 = ((ql[l] >> 4) | (((qh[l] >> 4) & 3) << 4)) - 32;
                    const int q4 = ((ql[l + 32] >> 4) | (((qh[l] >> 6) & 3) << 4)) - 32;
                    o[l] = d * sc[is] * q1;
                    o[l + 32] = d * sc[is + 2] * q2;
                    o[l + 64] = d * sc[is + 4] * q3;
                    o[l + 96] = d * sc[is + 6] * q4;
                }
                o += 128; ql += 64; qh += 32; sc += 8;
            }
        }
        return;
    }
    const int q5 = type == T_Q5_K;
    const int bb = q5 ? 176 : 144;
    for (int i = 0; i < K / QK_K; ++i) {
        const uint8_t* blk = row + (size_t)i * bb;
        uint16_t dh, dmh;
        memcpy(&dh, blk, 2);
        memcpy(&dmh, blk + 2, 2);
        const float d = h2f(dh), mn = h2f(dmh);
        const uint8_t* qh = blk + 16;
        const uint8_t* q = blk + (q5 ? 48 : 16);
        float* o = y + i * QK_K;
        for (int c = 0; c < 4; ++c) {
            uint8_t s1, m1, s2, m2;
            scale_min_k4(2 * c, blk + 4, &s1, &m1);
            scale_min_k4(2 * c + 1, blk + 4, &s2, &m2);
            const float d1 = d * s1, mm1 = mn * m1, d2 = d * s2, mm2 = mn * m2;
            for (int l = 0; l < 32; ++l) {
                const int lo = (q[32 * c + l] & 0xF) + (q5 && (qh[l] >> (2 * c) & 1) ? 16 : 0);
                const int hi = (q[32 * c + l] >> 4) + (q5 && (qh[l] >> (2 * c + 1) & 1) ? 16 : 0);
                o[64 * c + l] = d1 * lo - mm1;
                o[64 * c + 32 + l] = d2 * hi - mm2;
            }
        }
    }
}

/* --------------------------------------------------------- the model ---- */
typedef struct {
    int n_vocab, n_embd, n_layer, n_head, n_head_kv, n_ff, n_rot, n_expert, n_expert_used;
    float eps, rope_base;
} orc_hparams;

typedef struct { int type; const uint8_t* data; int64_t ne0, ne1, ne2; } orc_tensor;

typedef struct {
    orc_hparams hp;
    int n_ctx, n_cells;
    orc_tensor tok_embd, output, output_norm;
    orc_tensor* layer;    /* [n_layer][12]: attn_norm q k v o ffn_norm gate up down gate_inp */
    uint16_t *kc, *vc;    /* [n_layer][n_ctx][kv_dim] fp16 */
    int* cell_pos;
} orc_model;

enum { L_ATTN_NORM, L_Q, L_K, L_V, L_O, L_FFN_NORM, L_GATE, L_UP, L_DOWN, L_GATE_INP, L_N };

orc_model* orc_create(const orc_hparams* hp, int n_ctx) {
    orc_model* m = (orc_model*)calloc(1, sizeof(orc_model));
    m->hp = *hp;
    m->n_ctx = n_ctx;
    m->layer = (orc_tensor*)calloc((size_t)hp->n_layer * L_N, sizeof(orc_tensor));
    const size_t kvd = (size_t)hp->n_head_kv * (hp->n_embd / hp->n_head);
    m->kc = (uint16_t*)calloc((size_t)hp->n_layer * n_ctx * kvd, 2);
    m->vc = (uint16_t*)calloc((size_t)hp->n_layer * n_ctx * kvd, 2);
    m->cell_pos = (int*)calloc(n_ctx, sizeof(int));
    return m;
}

void orc_free(orc_model* m) {
    if (!m) return;
    free(m->layer); free(m->kc); free(m->vc); free(m->cell_pos); free(m);
}

int orc_set_tensor(orc_model* m, const char* name, int type, const void* data, int64_t ne0, int64_t ne1, int64_t ne2) {
    orc_tensor t = {type, (const uint8_t*)data, ne0, ne1, ne2};
    if (!strcmp(name, "token_embd.weight")) { m->tok_embd = t; return 0; }
    if (!strcmp(name, "output.weight")) { m->output = t; return 0; }
    if (!strcmp(name, "output_norm.weight")) { m->output_norm = t; return 0; }
    int l;
    char rest[64];
    if (sscanf(name, "blk.%d.%63s", &l, rest) != 2 || l < 0 || l >= m->hp.n_layer) return 1;
    static const char* names[L_N] = {"attn_norm.weight", "attn_q.weight", "attn_k.weight", "attn_v.weight",
                                     "attn_output.weight", "ffn_norm.weight", "ffn_gate.weight", "ffn_up.weight",
                                     "ffn_down.weight", "ffn_gate_inp.weight"};
    static const char* exps[3] = {"ffn_gate_exps.weight", "ffn_up_exps.weight", "ffn_down_exps.weight"};
    for (int i = 0; i < L_N; ++i)
        if (!strcmp(rest, names[i])) { m->layer[l * L_N + i] = t; return 0; }
    for (int i = 0; i < 3; ++i)
        if (!strcmp(rest, exps[i])) { m->layer[l * L_N + L_GATE + i] = t; return 0; }
    return 1;
}

static void rms_norm_mul(const float* x, const float* w, int n, float eps, float* y) {
    double sum = 0.0;
    for (int i = 0; i < n; ++i) sum += (double)(x[i] * x[i]);
    const float mean = (float)(sum / n);
    const float scale = 1.0f / sqrtf(mean + eps);
    for (int i = 0; i < n; ++i) y[i] = (x[i] * scale) * w[i];
}

static void rope(float* x, int n_heads, int hd, int n_rot, int pos, float base) {
    const float ts = powf(base, -2.0f / n_rot);
    float cs[512], sn[512];
    float theta = (float)pos;
    static int use_f = -1;   /* ORC_ROPE_F=1: libm cosf/sinf (sensitivity experiments) */
    if (use_f < 0) use_f = getenv("ORC_ROPE_F") != NULL;
    for (int i = 0; i < n_rot / 2; ++i) {
        /* correctly rounded cos/sin of the float angle (ggml calls libm cosf/sinf,
           which are within 1 ulp of this; the numpy oracle and the HIP engine
           use the correctly rounded value) */
        cs[i] = use_f ? cosf(theta) : (float)cos((double)theta);
        sn[i] = use_f ? sinf(theta) : (float)sin((double)theta);
        theta *= ts;
    }
    for (int h = 0; h < n_heads; ++h)
        for (int i = 0; i < n_rot / 2; ++i) {
            float* e = x + h * hd + 2 * i;
            const float x0 = e[0], x1 = e[1];
            e[0] = x0 * cs[i] - x1 * sn[i];
            e[1] = x0 * sn[i] + x1 * cs[i];
        }
}

static void mm(const orc_tensor* t, int expert, const float* x, float* y) {
    const int K = (int)t->ne0, M = (int)t->ne1;
    const uint8_t* base = t->data + (size_t)expert * M * row_bytes(t->type, K);
    orc_gemv(t->type, base, M, K, x, y);
}

static float silu(float v) { return v / (1.0f + expf(-v)); }

/* ORC_TRACE=1: print a checksum of every intermediate vector (debugging aid) */
static void trace(const char* what, int l, const float* v, int n) {
    static int on = -1;
    if (on < 0) on = getenv("ORC_TRACE") != NULL;
    if (!on) return;
    double s = 0.0, a = 0.0;
    for (int i = 0; i < n; ++i) { s += v[i]; a += fabs(v[i]); }
    fprintf(stderr, "L%d %-5s sum=%.9g abs=%.9g\n", l, what, s, a);
}

/* one llama_decode of `token` at position max(cell_pos)+1; logits -> out[n_vocab] */
/* Test diagnostics: over the MoE layers of the last orc_decode, the smallest gap between the
 * router probability of the last expert picked and the best one left out (INFINITY: dense).  A
 * gap near zero is a routing near-tie, which any other fp32 order may resolve the other way. */
static float g_moe_margin = INFINITY;
float orc_last_moe_margin(void) { return g_moe_margin; }

int orc_decode(orc_model* m, int token, float* out) {
    g_moe_margin = INFINITY;
    const orc_hparams* hp = &m->hp;
    const int d = hp->n_embd, hd = d / hp->n_head, kvd = hp->n_head_kv * hd, ff = hp->n_ff;
    if (m->n_cells >= m->n_ctx) return 1;
    int pos = 0;
    for (int c = 0; c < m->n_cells; ++c) if (m->cell_pos[c] + 1 > pos) pos = m->cell_pos[c] + 1;
    const int cell = m->n_cells;
    float* x = (float*)malloc(sizeof(float) * d);
    float* cur = (float*)malloc(sizeof(float) * d);
    float* q = (float*)malloc(sizeof(float) * d);
    float* k = (float*)malloc(sizeof(float) * kvd);
    float* v = (float*)malloc(sizeof(float) * kvd);
    float* att = (float*)malloc(sizeof(float) * d);
    float* g = (float*)malloc(sizeof(float) * ff);
    float* u = (float*)malloc(sizeof(float) * ff);
    float* dn = (float*)malloc(sizeof(float) * d);
    float* acc = (float*)malloc(sizeof(float) * d);
    dequant_row(m->tok_embd.type, m->tok_embd.data + (size_t)token * row_bytes(m->tok_embd.type, d), d, x);
    const float kq_scale = 1.0f / sqrtf((float)hd);
    const int ratio = hp->n_head / hp->n_head_kv;
    for (int l = 0; l < hp->n_layer; ++l) {
        const orc_tensor* L = m->layer + l * L_N;
        rms_norm_mul(x, (const float*)L[L_ATTN_NORM].data, d, hp->eps, cur);
        mm(&L[L_Q], 0, cur, q);
        mm(&L[L_K], 0, cur, k);
        mm(&L[L_V], 0, cur, v);
        rope(q, hp->n_head, hd, hp->n_rot, pos, hp->rope_base);
        rope(k, hp->n_head_kv, hd, hp->n_rot, pos, hp->rope_base);
        trace("q", l, q, d); trace("k", l, k, kvd); trace("v", l, v, kvd);
        uint16_t* kc = m->kc + ((size_t)l * m->n_ctx) * kvd;
        uint16_t* vc = m->vc + ((size_t)l * m->n_ctx) * kvd;
        for (int i = 0; i < kvd; ++i) { kc[(size_t)cell * kvd + i] = f2h(k[i]); vc[(size_t)cell * kvd + i] = f2h(v[i]); }
        const int nc = cell + 1;
#pragma omp parallel for schedule(static)
        for (int h = 0; h < hp->n_head; ++h) {
            const int gk = h / ratio;
            float* s = (float*)malloc(sizeof(float) * nc);
            float qh[512];
            for (int e = 0; e < hd; ++e) qh[e] = h2f(f2h(q[h * hd + e]));   /* vec_dot_type F16 */
            float mx = -INFINITY;
            for (int c = 0; c < nc; ++c) {
                double sd = 0.0;   /* ggml_vec_dot_f16 scalar: ggml_float accumulation */
                const uint16_t* kr = kc + (size_t)c * kvd + gk * hd;
                for (int e = 0; e < hd; ++e) sd += (double)(qh[e] * h2f(kr[e]));
                float w = (float)sd * kq_scale;
                if (c != cell && m->cell_pos[c] > pos) w = -INFINITY;
                s[c] = w;
                if (w > mx) mx = w;
            }
            double sum = 0.0;
            for (int c = 0; c < nc; ++c) { const float e = expf(s[c] - mx); s[c] = e; sum += (double)e; }
            const float inv = (float)(1.0 / sum);
            for (int c = 0; c < nc; ++c) s[c] = h2f(f2h(s[c] * inv));
            for (int e = 0; e < hd; ++e) {
                double o = 0.0;
                for (int c = 0; c < nc; ++c) o += (double)(s[c] * h2f(vc[(size_t)c * kvd + gk * hd + e]));
                att[h * hd + e] = (float)o;
            }
            free(s);
        }
        trace("att", l, att, d);
        mm(&L[L_O], 0, att, dn);
        for (int i = 0; i < d; ++i) x[i] = dn[i] + x[i];
        trace("x1", l, x, d);
        rms_norm_mul(x, (const float*)L[L_FFN_NORM].data, d, hp->eps, cur);
        trace("cur", l, cur, d);
        if (hp->n_expert == 0) {
            mm(&L[L_GATE], 0, cur, g);
            mm(&L[L_UP], 0, cur, u);
            trace("g", l, g, ff); trace("u", l, u, ff);
            for (int i = 0; i < ff; ++i) g[i] = silu(g[i]) * u[i];
            trace("h", l, g, ff);
            mm(&L[L_DOWN], 0, g, dn);
            trace("dn", l, dn, d);
            for (int i = 0; i < d; ++i) x[i] = dn[i] + x[i];
        } else {
            float lg[64], pr[64];
            orc_gemv(T_F32, L[L_GATE_INP].data, hp->n_expert, d, cur, lg);
            float mxl = -INFINITY;
            for (int e = 0; e < hp->n_expert; ++e) if (lg[e] > mxl) mxl = lg[e];
            double sm = 0;
            for (int e = 0; e < hp->n_expert; ++e) { pr[e] = expf(lg[e] - mxl); sm += pr[e]; }
            const float inv = (float)(1.0 / sm);
            for (int e = 0; e < hp->n_expert; ++e) pr[e] *= inv;
            int idx[64];
            for (int e = 0; e < hp->n_expert; ++e) idx[e] = e;
            for (int a = 0; a < hp->n_expert; ++a)
                for (int b = a + 1; b < hp->n_expert; ++b)
                    if (pr[idx[a]] < pr[idx[b]]) { int t = idx[a]; idx[a] = idx[b]; idx[b] = t; }
            if (hp->n_expert_used < hp->n_expert)   /* the last pick's lead over the first expert left out */
                g_moe_margin = fminf(g_moe_margin, pr[idx[hp->n_expert_used - 1]] - pr[idx[hp->n_expert_used]]);
            float ws = 0;
            for (int kk = 0; kk < hp->n_expert_used; ++kk) ws += pr[idx[kk]];
            for (int i = 0; i < d; ++i) acc[i] = 0;
            for (int kk = 0; kk < hp->n_expert_used; ++kk) {
                const int e = idx[kk];
                const float w = pr[e] / ws;
                mm(&L[L_GATE], e, cur, g);
                mm(&L[L_UP], e, cur, u);
                for (int i = 0; i < ff; ++i) g[i] = silu(g[i]) * u[i];
                mm(&L[L_DOWN], e, g, dn);
                for (int i = 0; i < d; ++i) acc[i] = kk == 0 ? dn[i] * w : acc[i] + dn[i] * w;
            }
            for (int i = 0; i < d; ++i) x[i] = acc[i] + x[i];
        }
    }
    rms_norm_mul(x, (const float*)m->output_norm.data, d, hp->eps, cur);
    const orc_tensor* out_t = m->output.data ? &m->output : &m->tok_embd;
    mm(out_t, 0, cur, out);
    m->cell_pos[cell] = pos;
    m->n_cells++;
    free(x); free(cur); free(q); free(k); free(v); free(att); free(g); free(u); free(dn); free(acc);
    return 0;
}

void orc_kv_clear(orc_model* m) { m->n_cells = 0; }
int orc_n_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
