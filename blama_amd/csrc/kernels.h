// Kernel parameter blocks and host-side launchers (implemented in kernels.hip).
#pragma once
#include "common.h"
#include <vector>

namespace mi {

// ---- decode GEMV (gemv.hip) -------------------------------------------------
// One launch computes one or two "segments" (a matrix, or a gate/up pair) against one
// activation: ggml_mul_mat of batch 1 with the CPU path's integer arithmetic (activations
// quantised to Q8_K / Q8_0, per-block integer dots), fused with the producer's epilogue.
enum Pair { PAIR_ADJ = 0, PAIR_AB = 1 };
enum Epi {
    EPI_STORE = 0,    // out[r] = y
    EPI_ADD = 1,      // out[r] = y + resid[r]            (residual add, llm_build_llama)
    EPI_QKV = 2,      // fused Q|K|V rows: rows < nq -> RoPE -> out (f32 q); rows < nq+nk ->
                      // RoPE -> f16 K cache row of this token's cell; the rest -> f16 V cache
    EPI_ROPE_Q = 3,   // batch GEMM epilogues (gemm_t / mmq32): RoPE -> out
    EPI_ROPE_K = 4,   //   RoPE -> f16 K cache
    EPI_V = 7,        //   -> f16 V cache
    EPI_SWIGLU = 5,   // out[u] = silu(yA) * yB            (LLM_FFN_SILU + LLM_FFN_PAR)
    EPI_MOE_DOWN = 6, // out[u] = (yA*wA + yB*wB) + resid[u] (build_moe_ffn aggregation)
    EPI_GELU = 8,     // out[r] = gelu(y + bias[r])       (llm_build_gpt2 FFN: LLM_FFN_GELU, LLM_FFN_SEQ)
};
// Every epilogue but SwiGLU / MoE-down adds GemvSeg::bias[r] to y first when it is set (the
// ggml_add of a GPT-2 projection bias, before RoPE-less KV append, residual add or GELU).
enum Pro {
    PRO_PLAIN = 0,    // activation = x[0] (and x[1] for a second slot)
    PRO_RMSNORM = 1,  // activation = rms_norm(x[0]) * norm_w
    PRO_ATTN = 2,     // activation = the attention partials of the splits, added in split order
    PRO_LAYERNORM = 3,// activation = layer_norm(x[0]) * norm_w + norm_b  (build_norm LLM_NORM)
};

struct GemvSeg {
    QMat A, B;            // B: the PAIR_AB partner (gate/up: up; MoE down: the same tensor)
    int pair, epi;
    int nq, nk;           // EPI_QKV: rows of Q and K in A (the rest are V)
    int expA, expB;       // MoE: slot in sel[] choosing the expert of A / B (-1: dense)
    int actB;             // activation slot of the B rows (MoE down: 1)
    float* out;
    const float* resid;   // EPI_ADD / EPI_MOE_DOWN (may alias out)
    const float* bias;    // optional per-row bias (GPT-2), added before the epilogue
};

// Attention split over cells: split s of q head h holds the partial sum
// O_s = sum_{c in s} f16(p_c) v_c with the head's exact softmax weights p (the
// global max and sum are known before the weights are rounded; see
// attn_pv_kernel).  A split covers `chunk` cells, chunk = max(64,
// ceil(ncell / ATTN_SMAX) rounded up to 64), so there are at most ATTN_SMAX
// splits.
constexpr int ATTN_SMAX = 16;
// Contexts up to ATTN_SHORT cells are served by one fused launch, one workgroup per kv head
// (scores in LDS, exact softmax, PV): one split.  Longer ones split over cells.
constexpr int ATTN_SHORT = 512;
__host__ __device__ inline void attn_split(int ncell, int& chunk, int& nsplit) {
    if (ncell <= ATTN_SHORT) {
        chunk = ncell;
        nsplit = 1;
        return;
    }
    int c = (ncell + ATTN_SMAX - 1) / ATTN_SMAX;
    c = (c + 63) & ~63;
    chunk = c < 64 ? 64 : c;
    nsplit = (ncell + chunk - 1) / chunk;
}
struct AttnPartials {
    const float* o;            // [ATTN_SMAX][n_head][head_dim]
    int n_head, head_dim;
};

// Q8_K / Q8_0 activations of a physical batch (launch_quant_act; layout below)
struct ActQ8 {
    int8_t* q;                 // [npad/32][K/256][8][64][16]: MFMA A fragments (mmq.hip quant_act_kernel)
    float* dT;                 // [K/256][npad]  (Q8_K d, token-minor)
    int8_t* bsb;               // [npad/32][K/256][32][16]: sub-block bsums as 64*hi + lo (bytes 0-7 hi, 8-15 lo)
    int K;
    int ntok, npad;            // tokens; rows allocated (ntok rounded up to 32, <= UB_MAX)
    int q80;                   // 1: Q8_0 activations (for Q8_0 weights): dT is [K/32][npad] f16-rounded d, no bsb
};
// ---- a quantised activation a decode launch publishes for the next one (the attention kernel for
// the streaming WO launch) ----
// Layout in global memory: act_layout(K, q8k, q80) of qdot.h (the Q8_K blocks, the Q8_0 blocks,
// the Q8_K sub-block sums and scales, the Q8_0 scales), the same bytes the consumer copies into
// LDS.  norm_w set: the activation is rms_norm(x) * norm_w (ggml's rms_norm then mul).
struct ActOut {
    int K;                    // length (multiple of 256)
    int q8k, q80;             // formats to write (Q8_K for k-quant consumers, Q8_0 for Q8_0 ones)
    char* act;                // destination
    const float* norm_w;      // optional
    float eps;
};

constexpr int GEMV_MAX_SEG = 2;
struct GemvParams {
    GemvSeg seg[GEMV_MAX_SEG];
    int nseg;
    int pro;                  // Pro
    int nslots;               // 1, or 2 (MoE down: x[1] feeds the B rows)
    const float* x[2];
    const float* norm_w;
    const float* norm_b;      // PRO_LAYERNORM bias
    float eps;
    int K;                    // activation length (multiple of 256, <= 14336)
    const unsigned short* gelu_tab;   // EPI_GELU: ggml_table_gelu_f16 (65536 f16 bit patterns)
    // RoPE / KV cache (EPI_QKV)
    const int* tokpos;        // {token, pos, cell, -}
    int* cell_pos;            // cell -> position (written with the K rows)
    float theta_scale, freq_scale;
    int n_rot, head_dim;
    const float* freq_factors;
    __half* kcache;           // this layer's K cache [n_ctx][kv_dim]
    __half* vcache;
    int kv_dim;
    // MoE routing results
    const int* sel;
    const float* selw;
    AttnPartials attn;        // PRO_ATTN input
    int attn_nsplit;          // PRO_ATTN: splits to add (0: from the cell count in tokpos)
    unsigned long long* stamps;   // diagnostics (MI_STAMPS builds): per-workgroup stamps [grid][8]
    // streaming form (launch_dgemv, dense LLaMA decode within ATTN_SHORT cells): the activation
    // arrives quantised, act_layout(K, act_q8k, act_q80) at act_in (pro / x / norm_w unused)
    const char* act_in;
    int act_q8k, act_q80;
};

void init_kernel_attributes();   // once per device, before any graph capture
// the streaming form (dgemv.hip): p.act_in set; the events as launch_gemv's
void launch_dgemv(const GemvParams& p, hipStream_t s, hipEvent_t ev_start = nullptr, hipEvent_t ev_stop = nullptr);
bool dgemv_supported(const GemvParams& p);            // a compiled variant serves this launch
size_t dv_act_bytes(int K, int q8k, int q80);         // bytes of a quantised activation
// ev_start/ev_stop (optional): recorded at the kernel's own start and end (hipExtLaunchKernel)
// -- the bench's in-kernel timing of one launch.
void launch_gemv(const GemvParams& p, hipStream_t s, hipEvent_t ev_start = nullptr, hipEvent_t ev_stop = nullptr);
// whether one launch can carry segments of these two quant types
bool gemv_pair_supported(int t1, int t2);
// workgroups of a launch
int gemv_grid(const GemvParams& p);
void init_gemm_attributes();     // the batch GEMMs' LDS limits (kernels.hip)

struct AttnParams;

// ---- batched quantised GEMM over up to GEMM_NT tokens (prompt ingestion) ----
// The GEMV's integer arithmetic per token (Q8_K / Q8_0 activations, per-block integer
// dots), with every weight load used for GEMM_NT tokens: a prompt of n tokens streams
// the weights n/GEMM_NT times instead of n times.  Dense models; one matrix (or a
// gate/up pair) per launch; epilogues as the GEMV's, per token.
constexpr int GEMM_NT = 8;
struct GemmParams {
    QMat A, B;                 // B: PAIR_AB partner (gate/up)
    int pair, epi, units;
    int ntok;                  // tokens in this launch (1..GEMM_NT)
    int K;
    int pro;                   // PRO_PLAIN or PRO_RMSNORM
    const float* x;            // [ntok][x_stride]
    int x_stride;
    const float* norm_w;
    float eps;
    float* out;                // [ntok][out_stride]
    int out_stride;
    const float* resid;        // EPI_ADD: [ntok][out_stride] (may alias out)
    const int* tokpos;         // [ntok][4] {token, pos, cell, 0}
    int* cell_pos;
    float theta_scale, freq_scale;
    int n_rot, head_dim;
    const float* freq_factors;
    __half* kcache;            // this layer's caches
    __half* vcache;
    int kv_dim;
    int need_q8k, need_q80;
    int grid;                  // set by launch_gemm
    // mmq32 grouped launch (MoE prompt batches): expert e's MFMA-order copy is A.sw + e*grp_stride,
    // its activation rows [grp[e], grp[e] + grp[grp_n + 1 + e]) (launch_moe_group's layout)
    const int* grp;
    long long grp_stride;
    int grp_n;
    int grp_max;   // mmq2 grouped: the most rows one expert can have (the batch's tokens)
    // mmq2 split over K (EPI_ADD of a dense prompt batch): ksplit (2 or 4) parts of the superblocks
    // write their partial sums to part[ksplit][ntok][out_stride] (no residual); the next
    // launch_quant_act over the same buffer adds them, x = ((p0 + p1) + ...) + x, writes x back and
    // quantises it
    int ksplit;
    float* part;
};
void launch_gemm(const GemmParams& p, hipStream_t s);

// ---- token embedding: get_rows(tok_embd, token) with ggml dequantisation ----
struct EmbedParams {
    QMat E;                    // quant planes, or E.p[0] = raw f32/f16 rows
    const int* tokpos;
    float* out;
    int n_embd;
    QMat P;                    // GPT-2: learned position embedding (row = the token's position),
    int has_pos;               // added to the token row (ggml_add of the two get_rows)
    unsigned* step;            // optional: incremented once per launch (decode step counter)
};
void launch_embed(const EmbedParams& p, hipStream_t s);
// rms_norm(x) * a.norm_w (or x itself) of one row, quantised into a.act (dgemv.hip; one workgroup
// per 256-block)
void launch_dv_quant(const float* x, const ActOut& a, hipStream_t s);

// ---- attention over the f16 cache: KQ -> soft_max -> KQV, split over cells ----
// Two launches, grid (n_head_kv, ATTN_SMAX) each; the WO GEMV's PRO_ATTN
// prologue adds the splits' partials.
struct AttnParams {
    const float* q;            // [n_head*hd] (roped)
    const __half* kcache;      // [n_ctx][kv_dim]
    const __half* vcache;
    const int* tokpos;
    const int* cell_pos;
    float* scores;             // [n_head][n_ctx] scaled KQ (scratch)
    float* smax;               // [ATTN_SMAX][n_head] split maxima (scratch)
    float* part_o;             // [ATTN_SMAX][n_head][hd]
    int n_head, n_head_kv, head_dim, kv_dim, n_ctx;
    float scale;
    unsigned long long* stamps;    // diagnostics (MI_STAMPS builds): scores / pv launches
    unsigned long long* stamps2;
    int fused;                     // 1: the single-launch kernel (the context has <= ATTN_SHORT cells)
    int qsplit;                    // fused kernel: 0 = a workgroup per kv head; R = a workgroup per q head
    // contexts past ATTN_SHORT cells in ONE launch (attn_long_kernel): the splits of a q head
    // exchange their maxima and partial sums through these (null: the two-launch split kernels)
    unsigned* xflags;              // [n_head][ATTN_SMAX][32]: the exchange's flag lines
    float* xmax;                   // [n_head][ATTN_SMAX]
    double* xsum;                  // [n_head][ATTN_SMAX]
    const unsigned* step;          // decode steps so far (the embedding launch counts them)
    int layer;                     // this layer (the exchange's epoch: step * (2 * n_layer + 2) + 2 * layer + phase)
    int n_layer;                   // layers per step (the epoch's stride; 0 = one layer)
    unsigned* xerr;                // host-mapped: an exchange timed out (the step is invalid)
    // contexts that may run attention on this device at once: the single launch is used only when
    // that many grids of n_head * ATTN_SMAX workgroups are co-resident (occupancy x CUs)
    int long_share;
    int long_off;                  // 1: never the single launch (an exchange timed out before)
    ActOut act_out;                // fused kernel, decode (act_out.act set): the output also quantised
                                   // (a workgroup serves whole 256-blocks of it: 256 / (R * hd) kv heads)
    ActQ8 act_q8;                  // fused kernel, a short batch (act_q8.q set; launch_attn_multi): each
                                   // token's output quantised in the batch GEMMs' format, same blocks
};
void launch_attn(const AttnParams& p, hipStream_t s);
// a decode attention launch can also quantise its output (AttnParams::act_out) for this geometry
bool attn_quant_supported(int n_head, int n_head_kv, int head_dim);
// Combine the partials into out[n_head*hd] (tests / the eager debug path).
void launch_attn_combine(const AttnPartials& a, const int* tokpos, float* out, hipStream_t s);
// The same sum of the splits (split order, as gemv.hip's PRO_ATTN prologue), quantised into t
// (t.K == n_head * head_dim): the streaming WO launch's activation past ATTN_SHORT cells.
void launch_attn_combine_quant(const AttnPartials& a, const int* tokpos, const ActOut& t, hipStream_t s);

// ---- top-k over logits (sorted by logit desc, id asc), k <= 64 ----
// Stage 1: every 1024-logit block -> its sorted top 64 (wave bitonic sorts +
// merges); stage 2: one workgroup merges the block lists.
constexpr int TOPK_MAX = 64;
constexpr int TOPK_BLOCK = 1024;
inline int topk_blocks(int n) { return (n + TOPK_BLOCK - 1) / TOPK_BLOCK; }
struct TopkParams {
    const float* logits;
    int n;
    unsigned long long* cand;  // [topk_blocks(n) * TOPK_MAX]
    int* ids;                  // [TOPK_MAX] (device)
    float* vals;
    int* h_ids;                // optional: also written straight to mapped host memory
    float* h_vals;
};
void launch_topk(const TopkParams& p, hipStream_t s);

// ---- gather logits at ids ----
void launch_gather(const float* logits, const int* ids, int n, float* out, hipStream_t s);
// n = rows*k ids, k per row: out[i] = base[(i / k) * row_stride + ids[i]]
void launch_gather_rows(const float* base, long long row_stride, const int* ids, int n, int k, float* out,
                        hipStream_t s);

// ---- MoE router: softmax gating + top-k + weight normalisation ----
struct RouterParams {
    const float* x;            // residual stream (pre-norm)
    const float* norm_w;
    float eps;
    const float* w;            // F32 [n_expert][n_embd]
    int n_embd, n_expert, n_used;
    int* sel;                  // [token][n_used]
    float* selw;
    long long x_stride;        // elements between token rows (launch_router_multi)
    // (batch, optional) split-K partials of the WO GEMM that produced x, [2][ntok][n_embd]:
    // x = (p0 + p1) + x first, written back (GemmParams::ksplit)
    const float* part;
    int part_ntok;
};
void launch_router(const RouterParams& p, hipStream_t s);
// the router of ntok token rows x[t * x_stride] -> sel/selw [t][n_used] (one workgroup each)
void launch_router_multi(const RouterParams& p, int ntok, hipStream_t s);
// build_moe_ffn's aggregation over a physical batch: x[t] = (y[pos[t][0]]*w[t][0] + y[pos[t][1]]*w[t][1])
// + x[t] (ggml_mul by the weights, ggml_add of the slots in slot order, then the residual add);
// y holds the experts' down outputs in compact rows (grouped by expert)
// Groups the n (token, slot) picks of a physical batch (sel[t*U + k] = expert) by expert on the
// device: expert e's rows are [grp[e], grp[e] + cnt_e) with grp[e] a multiple of 32 (whole MFMA
// token tiles), tokens ascending within an expert; grp = {off[0..E], cnt[0..E-1]}.  rows[r] = the
// source token of row r (-1 for padding, up to rows_cap), rowsel[r] = r or -1, pos[t*U + k] = row.
constexpr int MOE_GROUP_MAXE = 16;
inline int moe_rows_cap(int n, int E) { return (n + E * 31 + 31) / 32 * 32; }
void launch_moe_group(const int* sel, int n, int U, int E, int* grp, int* rows, int* rowsel, int* pos, int rows_cap,
                      hipStream_t s);
void launch_moe_combine(const float* y, const int* pos, const float* w, float* x, int ntok, int n_embd,
                        hipStream_t s);

// ---- load-time repack of GGUF blocks into planes ----
void launch_repack(const uint8_t* raw, int type, long long rows, int K, uint8_t* const planes[4],
                   hipStream_t s);

// ---- KV cache maintenance (context shift / self-extend K re-rotation) ----
struct KvShiftParams {
    __half* kcache;            // all layers [n_layer][n_ctx][kv_dim]
    int n_layer, n_ctx, kv_dim, head_dim, n_rot;
    const int* cell_delta;     // per cell position delta (0 = untouched)
    int n_cells;
    float theta_scale, freq_scale;
    const float* freq_factors;
};
void launch_kv_shift(const KvShiftParams& p, hipStream_t s);
void launch_kv_move(__half* cache, int n_layer, int n_ctx, int kv_dim, const int* src_cell,
                    int n_dst, __half* scratch, hipStream_t s);

// ---- single-op entry points used by the op-level parity tests ----
void launch_dequant_rows(const QMat& m, int row0, int nrows, float* out, hipStream_t s);
void launch_quantize_q8k(const float* x, int K, int8_t* q, float* d, int* bsums, hipStream_t s);

// embedding rows of ntok tokens (tokpos[t*4]) -> out[t*n_embd]
void launch_embed_multi(const EmbedParams& p, int ntok, hipStream_t s);
// causal attention of ntok query tokens (q [ntok][n_head*hd]) over <= ATTN_SHORT cells;
// out [ntok][n_head*hd] (the fused single-split arithmetic per token)
void launch_attn_multi(const AttnParams& p, int ntok, float* out, hipStream_t s);


// ---- causal attention of ntok query tokens (q [ntok][n_head*hd]) on f16 MFMA (attn_mfma.hip):
// any number of cells (<= n_ctx); out [ntok][n_head*hd]; head_dim 64 or 128 ----
bool attn_mfma_supported(int head_dim);
void launch_attn_mfma(const AttnParams& p, int ntok, float* out, hipStream_t s);

// ---- int8-MFMA GEMM over a physical batch of up to UB_MAX tokens (mmq.hip) ----
// Prompt ingestion and batched verification: activations quantised to Q8_K once per matrix
// input (launch_quant_act), then v_mfma_i32_32x32x32_i8 per sub-block (launch_mmq32).
constexpr int UB_MAX = 512;    // n_ubatch (reference Instance.hpp:24)
// rows (optional): token t of the batch reads row rows[t] of x (the tokens routed to one expert)
// part (optional): the split-K partial sums of the GEMM that produced x (see GemmParams::ksplit):
// x = ((p0 + p1) + ...) + x first, written back
// swiglu: part holds the gate/up parts of a pair launch ([nks][ntok][2 K]: gate rows, then up
// rows); the row quantised is silu(sum gate) * (sum up) (x unused)
void launch_quant_act(const float* x, int x_stride, const float* norm_w, float eps, const ActQ8& a, hipStream_t s,
                      const int* rows = nullptr, const float* part = nullptr, int nks = 2, int swiglu = 0);
// whether prompt-batch GEMMs take the mmq2 path (the only one with ksplit)
bool mmq2_active();
// ggml_rope_cache_init per token of the batch: out [ntok][n_rot/2] (cos, sin)
void launch_rope_table(const int* tokpos, int ntok, int n_rot, float theta_scale, float freq_scale,
                       const float* freq_factors, float2* out, hipStream_t s);
bool mmq32_supported(int type);
// Bytes of one 32-row x superblock tile of the MFMA-order copy; total bytes of a copy of A
// (pair = gate/up: A and B in one copy, 16 rows of each per tile).
int mmq32_tile_bytes(int type);
size_t mmq32_copy_bytes(const QMat& A, bool pair);
// Builds the MFMA-order copy of A (and B for a pair) into dst from the planes.
void launch_mmq32_swizzle(const QMat& A, const QMat* B, uint8_t* dst, hipStream_t s);
// GemmParams: A (B = up for PAIR_AB / EPI_SWIGLU), epi, K, out/out_stride, resid, tokpos [ntok][4],
// RoPE fields (rope table from launch_rope_table), caches; the tokens are act's.
void launch_mmq32(const GemmParams& p, const ActQ8& act, const float2* rope, hipStream_t s);
// several matrices of one type over the same activation (Q / K / V) as ONE mmq2 launch when they
// qualify (no pairs, no grouping, a shared output buffer), else one launch each
void launch_mmq32_multi(const GemmParams* ps, int n, const ActQ8& act, const float2* rope, hipStream_t s);

// ---- short batches (<= MMQS_MAX tokens, mmq.hip mmqs): a split-K streaming int8-MFMA GEMM ----
// The matrices (one type; a gate/up pair: one QMat, its pair copy) over act (npad 32 or 64) write
// the plain partial sums of their K-parts to part[kp][ntok][pstride], matrix i's rows from prow[i]
// (a pair: gate rows from prow[0], up rows from prow[0] + nff).  Returns kp (mmqs_parts(K)).  The
// consumer adds the parts in order: launch_quant_act (part / swiglu), launch_qkv_finish,
// launch_part_sum.
constexpr int MMQS_MAX = 64;
int mmqs_parts(int K);
int launch_mmqs(const QMat* const* mats, const int* prow, int n, bool pair, int nff, const ActQ8& act, float* part,
                int pstride, hipStream_t s);
// The routed experts of a short MoE batch (build_moe_ffn's mul_mat_id): act holds the MoE rows
// (moe_group_kernel: expert e's at [grp[e], + grp[n_expert + 1 + e]), whole 32-row tiles, at most
// max_rows each), and expert e's rows multiply its own matrix; the parts go to
// part[kp][act.ntok][pstride] at the same rows (a pair: up rows from nff).  Returns kp.
bool mmqs_grouped_supported(int type);
int launch_mmqs_grouped(const QMat& A, bool pair, int nff, const ActQ8& act, float* part, int pstride, const int* grp,
                        int n_expert, int max_rows, hipStream_t s);
// Q / K / V from the parts of their GEMMs (rows [Q | K | V] of part): RoPE NORM of Q and K (the
// batch's rope table), Q -> q [ntok][q_stride], K / V -> the f16 caches at the tokens' cells
struct QkvFinish {
    const float* part;
    int pstride, kp, ntok;
    int nq, nk, nv;
    float* q;
    int q_stride;
    __half* kcache;
    __half* vcache;
    int kv_dim;
    int* cell_pos;
    const int* tokpos;
    const float2* rope;
    int n_rot, head_dim;
};
void launch_qkv_finish(const QkvFinish& F, hipStream_t s);
// out[t][r] = ((p0 + p1) + ...) [+ resid[t][r]] over rows [0, rows) of the parts; swiglu > 0 (a
// pair launch's parts, up rows from swiglu): silu(sum gate) * (sum up)
void launch_part_sum(const float* part, int kp, int ntok, int rows, int pstride, const float* resid, int rstride,
                     float* out, int ostride, hipStream_t s, int swiglu = 0);

}  // namespace mi
