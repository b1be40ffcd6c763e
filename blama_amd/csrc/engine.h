// Engine internals: GGUF parsing, the device-resident model and the decode
// context.  The public surface is the C ABI in include/mi_engine.h.
#pragma once
#include <mutex>
#include <cstdlib>
#include "common.h"
#include "kernels.h"
#include "mi_engine.h"

#include <functional>
#include <map>
#include <memory>
#include <string>
#include <vector>

namespace mi {

// ---------------------------------------------------------------- GGUF ----
struct GgufValue {
    int type = -1;                // gguf_type
    long long i = 0;
    double f = 0.0;
    std::string s;
    int arr_type = -1;
    long long arr_n = 0;
    std::vector<std::string> arr_s;
    std::vector<double> arr_num;
};

struct GgufTensor {
    std::string name;
    int type = 0;
    int n_dims = 0;
    long long ne[4] = {1, 1, 1, 1};
    unsigned long long offset = 0;   // within the data section
    size_t nbytes = 0;
};

struct Gguf {
    std::map<std::string, GgufValue> kv;
    std::vector<GgufTensor> tensors;
    size_t data_offset = 0;          // start of the data section in the file
    // parse the header (metadata + tensor infos) from a memory image
    void parse(const uint8_t* data, size_t size);
    const GgufValue* get(const std::string& k) const {
        auto it = kv.find(k);
        return it == kv.end() ? nullptr : &it->second;
    }
    long long get_int(const std::string& k, long long def) const;
    double get_float(const std::string& k, double def) const;
    std::string get_str(const std::string& k, const std::string& def) const;
    const GgufTensor* tensor(const std::string& name) const;
};

// --------------------------------------------------------------- model ----
struct HParams {
    int n_vocab = 0, n_embd = 0, n_layer = 0, n_head = 0, n_head_kv = 0, n_ff = 0, n_ctx_train = 0;
    int n_rot = 0, head_dim = 0, n_expert = 0, n_expert_used = 0;
    float eps = 1e-5f, rope_base = 10000.0f, freq_scale = 1.0f;
    int arch = 0;                       // ARCH_LLAMA (llm_build_llama) or ARCH_GPT2 (llm_build_gpt2)
};
enum { ARCH_LLAMA = 0, ARCH_GPT2 = 1 };

struct Layer {
    float* attn_norm = nullptr;
    float* ffn_norm = nullptr;
    QMat wq{}, wk{}, wv{}, wo{};
    QMat gate{}, up{}, down{};          // dense FFN, or the *_exps tensors for MoE
    float* router = nullptr;            // ffn_gate_inp (F32) for MoE
    // Q, K, V as 1-3 groups of adjacent same-type rows (the arena stores the planes of a group's
    // tensors back to back, so a group is one matrix to the decode GEMV): group g holds nq[g] Q
    // rows, then nk[g] K rows, then V rows
    int n_qkv = 0;
    QMat qkv[3]{};
    int qkv_nq[3] = {0, 0, 0}, qkv_nk[3] = {0, 0, 0};
    // GPT-2: LayerNorm biases and the projection biases (attn_qkv is the one fused QKV group)
    float *attn_norm_b = nullptr, *ffn_norm_b = nullptr;
    float *bqkv = nullptr, *bo = nullptr, *bup = nullptr, *bdown = nullptr;
};

struct Model {
    HParams hp;
    Gguf gguf;
    std::vector<std::string> tokens;
    std::vector<int> token_type;
    std::vector<float> token_score;     // SPM merge scores (tokenizer.ggml.scores)
    std::string tok_model;              // tokenizer.ggml.model ("llama" = SPM, "gpt2" = BPE)
    std::vector<std::string> merges;    // tokenizer.ggml.merges (BPE: "left right", rank = index)
    int bos = -1, eos = -1, eot = -1;
    bool add_bos = true;
    int device = 0;
    bool vocab_only = false;

    uint8_t* arena = nullptr;
    size_t arena_bytes = 0;
    // MFMA-order copies of the layer matrices and the output head for prompt batches (mmq32),
    // built from the arena on the device the first time a context needs them (replicas build
    // their own after the arena broadcast): one more weight-sized allocation, HBM for speed
    uint8_t* mmq_arena = nullptr;
    size_t mmq_bytes = 0;
    std::mutex mmq_mu;
    // false when the copy does not fit (the batch path then uses the v_dot4 GEMM).  The copies are
    // taken from the arena once: writes to the arena (mi_model_arena, mi_model_replicate) must
    // come before the first context (mi_model_replicate checks this).
    bool ensure_mmq_copies();
    long long weight_bytes = 0;         // GGUF bytes streamed per token (all but tok_embd)
    long long type_bytes[32] = {0};

    QMat tok_embd{};
    QMat pos_embd{};                    // GPT-2 learned positions (position_embd.weight)
    QMat output{};
    float* output_norm = nullptr;
    float* output_norm_b = nullptr;     // GPT-2
    unsigned short* gelu_tab = nullptr; // GPT-2: ggml_table_gelu_f16 on the device
    float* rope_freqs = nullptr;
    std::vector<Layer> layers;

    ~Model();
    // data: the GGUF image (header at least; tensor data unless no_upload/vocab_only)
    void load(const uint8_t* data, size_t size, const mi_model_params& p);
    const QMat* find_qmat(const std::string& name) const;
};

// ------------------------------------------------------------- context ----
int dev_chain_contexts(int device);   // live contexts on the device

struct Ctx {
    Model* m = nullptr;
    int device = 0;
    uint32_t n_ctx = 0, n_batch = 0, n_ubatch = 0;
    int kv_dim = 0;
    hipStream_t stream = nullptr;

    // device buffers
    __half* kcache = nullptr;           // [n_layer][n_ctx][kv_dim]
    __half* vcache = nullptr;
    __half* kv_scratch = nullptr;       // compaction scratch (allocated lazily)
    int* cell_pos = nullptr;            // [n_ctx]
    int* tokpos = nullptr;              // {token, pos, cell, 0}
    float *x = nullptr, *q = nullptr, *attn = nullptr, *h = nullptr, *h2 = nullptr, *logits = nullptr;
    unsigned long long* cand = nullptr;
    int* topk_ids = nullptr;
    float* topk_vals = nullptr;
    int* sel = nullptr;
    float* selw = nullptr;
    int* gather_ids = nullptr;
    float* gather_out = nullptr;
    int* cell_delta = nullptr;
    int* move_src = nullptr;
    float* part_o = nullptr;            // split-K attention partials [ATTN_SMAX][n_head][hd]
    float* attn_smax = nullptr;         // [ATTN_SMAX][n_head] split maxima
    float* attn_scores = nullptr;       // [n_head][n_ctx] scaled KQ
    // the single-launch long-context attention's exchange (attn_long_kernel) and the step counter
    unsigned* attn_xflags = nullptr;    // [n_head][ATTN_SMAX][32]
    float* attn_xmax = nullptr;
    double* attn_xsum = nullptr;
    unsigned* step_ctr = nullptr;       // decode steps so far (incremented by the embedding launch)
    unsigned* h_attn_xerr = nullptr;    // host-mapped: an exchange timed out
    unsigned* d_attn_xerr = nullptr;
    // batched prompt ingestion (dense models): GEMM_NT rows of residual / q / attention / FFN
    bool batch_ok = false;
    float *xb = nullptr, *qb = nullptr, *attnb = nullptr, *hb = nullptr;
    int* tokpos_b = nullptr;            // [GEMM_NT][4]
    int* h_tokpos_b = nullptr;          // pinned ring [kTokbRing][GEMM_NT][4]
    long long tokb_slot = 0;
    static constexpr int kTokbRing = 256;
    static constexpr int kBatchRows = UB_MAX;
    bool mmq_ok = false;                // int8-MFMA GEMM for prompt chunks (all layers Q4_K / Q6_K)
    // physical batches of up to UB_MAX tokens on mmq32 (mmq.hip): activations, rope table
    int8_t* ub_q = nullptr;             // Q8_K rows [UB_MAX][kmax]
    float* ub_dT = nullptr;             // [kmax/256][UB_MAX]
    int8_t* ub_bsb = nullptr;           // [UB_MAX][kmax/256][16]
    float2* ub_rope = nullptr;          // [UB_MAX][n_rot/2]
    float* ub_part = nullptr;           // [2][UB_MAX][n_embd] split-K partials (dense models; MI_MMQ_KSPLIT=0: off)
    // short batches (<= mmqs_max tokens, dense models): the split-K streaming GEMM's partial sums
    // [kp][ntok][rows] of every launch (mmq.hip mmqs; MI_MMQS_MAX=0: off)
    float* ub_spart = nullptr;
    int mmqs_max = 0;
    bool out_mmq = false;               // the output head is mmq32-capable (batched logits of every token)
    bool ub_q80 = false;                // the layer matrices are Q8_0: Q8_0 batch activations
    bool attn_mfma = false;             // batch attention on f16 MFMA (attn_mfma.hip); MI_ATTN_VALU=1: VALU kernel
    // MI_OUT_ALL: logits of every token of the last decode call, [out_rows][n_vocab]
    float* logits_all = nullptr;
    int logits_all_cap = 0;
    int out_rows = 0;                   // rows of logits_all valid (0: the last decode was MI_OUT_LAST)
    int topk_row = -1;                  // output row the mapped top-k buffers hold (-1: the last token)
    // diagnostics (MI_STAMPS builds only): s_memrealtime stamps of every
    // workgroup of every launch of the last enqueued step [launch][wg][8]
    static constexpr int kStampLaunches = 320, kStampWgs = 512;
    unsigned long long* stamps = nullptr;

    // pinned host buffers
    int* h_tokpos = nullptr;            // ring of kTokRing x 4 ints
    int* h_topk_ids = nullptr;
    float* h_topk_vals = nullptr;
    float* h_logits = nullptr;
    float* h_gather = nullptr;
    int* d_h_topk_ids = nullptr;        // device views of h_topk_ids / h_topk_vals
    float* d_h_topk_vals = nullptr;
    long long tok_slot = 0;

    // host mirror of the cache cells
    std::vector<int> h_cell_pos;
    int n_cells = 0;
    int pos_max = -1;
    bool logits_valid = false;

    // decode graphs (with / without the output head).  With profiling on, the
    // full step is split in three graphs around one layer's FFN gate/up GEMV so
    // that plain HIP events on the stream bracket exactly that launch.
    // MI_NO_GRAPH=1: launch every kernel eagerly (profilers that cannot trace
    // graph-launched kernels); the default replays one hipGraph per step
    bool use_graphs = getenv("MI_NO_GRAPH") == nullptr;
    // [attention mode]: 1 = the context fits the fused short-attention launch (ATTN_SHORT
    // cells), 0 = split attention; the host knows the cell count of every step.
    hipGraphExec_t g_full[2] = {nullptr, nullptr}, g_nolog[2] = {nullptr, nullptr};
    hipGraphExec_t g_seg[2][3] = {{nullptr, nullptr, nullptr}, {nullptr, nullptr, nullptr}};
    int attn_fused = 0;                 // mode of the step being enqueued
    bool attn_long_off = false;         // an exchange of attn_long_kernel timed out: split kernels only
    bool unsynced = false;              // decodes enqueued since the last sync()
    int undo_cells = 0, undo_pos = -1;  // n_cells / pos_max at the last sync (xerr rollback)
    int prof_layer = -1;
    hipEvent_t prof_ev[2] = {nullptr, nullptr};
    bool prof_pending = false;
    long long prof_bytes = 0;            // algorithmic bytes of the timed launch (mi_prof_bytes)
    int seg_filter = -1;                // -1: enqueue everything; else only ops of this segment

    static constexpr int kTokRing = 8192;

    // streaming decode step (dgemv.hip) for dense LLaMA contexts within ATTN_SHORT cells: every GEMV
    // reads its activation quantised -- WO's from the attention kernel, the others' from a
    // dv_quant launch (rms_norm'd x, or h) -- from sp_act[role]
    struct SpLayer {
        int fA, fB, fC, fD;             // activation formats of QKV, WO, gate/up, down: bit 0 Q8_K, bit 1 Q8_0
    };
    bool sp_ok = false;                 // false: the gemv_kernel graph (GPT-2)
    std::vector<SpLayer> sp;
    int sp_fH = 0;                      // the output head's activation formats
    char* sp_mem = nullptr;
    char* sp_act[5] = {};               // QKV, WO, gate/up, down, head inputs
    bool sp_setup();
    void enqueue_step_sp(bool with_logits);
    struct LayerBufs {
        const float* x_in;              // residual stream into the layer
        float *q, *po, *xa, *h, *h2, *xf;   // q, attention output, residual after WO, FFN (2nd expert), after down
    };
    void layer_ops(int l, const LayerBufs& B, const std::function<void(const GemvParams&, int)>& gemv,
                   const std::function<void(const AttnParams&)>& attn,
                   const std::function<void(const RouterParams&)>& router);

    Ctx(Model* model, uint32_t n_ctx, uint32_t n_batch, uint32_t n_ubatch);
    ~Ctx();
    void enqueue_step(bool with_logits);
    void enqueue_output(const float* xrow, unsigned long long* stamps_slab);
    void enqueue_layer_gpt2(int l, const GemvParams& base, __half* kl, __half* vl, float kq_scale,
                            const std::function<unsigned long long*()>& stamp);
    void decode_batch(const int32_t* tokens, int n);
    void decode_ubatch(const int32_t* tokens, int n, bool all);
    // the layers of one short physical batch on mmqs; returns the residual parts still to add
    // into xb (pend_k parts of ub_spart)
    int ubatch_layers_short(int nt);
    void enqueue_ubatch_short(int nt, bool all, int c0, bool last);
    ActQ8 ub_act(int K, int ntok, int type) const;   // the activation format `type`'s matrices read
    bool hp_dense() const { return m->hp.n_expert == 0; }
    // a second activation set (Q8_0) for a model mixing Q8_0 and k-quant matrices
    int8_t* ub_q0 = nullptr;
    float* ub_dT0 = nullptr;
    // MoE prompt batches: router picks and weights [token][n_used], the tokens grouped by expert on
    // the device (moe_rows: source token of each (expert, token) row, -1 for padding; moe_pos: the
    // row of each (token, slot)), the experts' down outputs [row][n_embd]
    float* yb = nullptr;
    int* sel_b = nullptr;
    float* selw_b = nullptr;
    int* moe_rows = nullptr;
    int* moe_pos = nullptr;
    int* moe_rowsel = nullptr;          // row r or -1 (padding): the down projection's input rows
    int* moe_grp = nullptr;             // launch_moe_group's {offsets, counts}
    int8_t* moe_q = nullptr;            // the rows' Q8_K / Q8_0 activations (moe_rows_cap rows)
    float* moe_dT = nullptr;
    int8_t* moe_bsb = nullptr;
    void moe_ffn_batch(int l, int nt, const float* pend = nullptr);
    // a short MoE batch's routed experts on the grouped mmqs (every expert matrix a k-quant)
    void moe_ffn_short(int l, int nt);
    bool moe_short = false;
    bool short_ok() const { return hp_dense() || moe_short; }
    const float* out_row(int row) const;   // device logits of output row `row` (-1: the last)
    hipGraphExec_t build_graph(bool with_logits, int seg);
    void invalidate_graphs();
    int decode(const int32_t* tokens, int n, bool all = false);
    void sync();
    int topk(int row, int k, int32_t* ids, float* vals);
    int gather(int row, const int32_t* ids, int n, float* out);
    int gather_rows(int row0, int nrows, const int32_t* ids, int k, float* out);
    int* grows_ids = nullptr;           // gather_rows buffers (grown on demand)
    float* grows_out = nullptr;
    float* h_grows = nullptr;
    size_t grows_cap = 0;
    const float* logits_host(int row);
    void kv_clear();
    int kv_seq_rm(int p0, int p1);
    int kv_seq_shift(int p0, int p1, int delta, int div);
    size_t state_size() const;
    size_t state_get(uint8_t* dst, size_t size);
    size_t state_set(const uint8_t* src, size_t size);
    int prof_read(float* us, int n);
    long long ffn_bytes() const;
};

}  // namespace mi
