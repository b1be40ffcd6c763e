/* mi_engine.h -- C ABI of the MI355X-native quantized-inference engine.
 *
 * This is the drop-in boundary for Blama's hot path.  Blama's inference layer
 * (bl::llama, /root/reference/inference/code/llama) binds the llama.cpp C API
 * (llama.h, llama.cpp tag b5187); the entry points below replace the hot-path
 * subset of it.  Each declaration cites the reference call
 * site whose llama.h function it replaces.
 *
 * Conventions: plain C types only; functions returning pointers return NULL on
 * error and functions returning int32_t return a negative value on error, with
 * the message available from mi_last_error() (thread-local).  mi_decode keeps
 * llama_decode's convention: 0 = ok, 1 = no KV space, < 0 = error
 * (checked "!= 0" at Session.cpp:388).  One context is used by one thread at a
 * time (Server.cpp:36); a model may back several contexts.
 */
#ifndef MI_ENGINE_H
#define MI_ENGINE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mi_model mi_model;
typedef struct mi_ctx mi_ctx;

typedef struct mi_model_params {
    int32_t device_ordinal; /* HIP device; Model.cpp:18-21 binds the first GPU */
    int32_t cpu_only;       /* Model::Params::gpu=false -- not served here: returns NULL */
    int32_t vocab_only;     /* Model::Params::vocabOnly: parse metadata/vocab, no weights */
    int32_t no_upload;      /* allocate the weight arena but leave it unfilled (replica
                               that receives the weights by RCCL broadcast) */
} mi_model_params;

/* Last error message of this thread ("" if none). */
const char* mi_last_error(void);

/* ---- model: replaces llama_model_load_from_file / llama_model_free
 *      (Model.cpp:52, Model.hpp:55) ---- */
mi_model* mi_model_load(const char* gguf_path, const mi_model_params* params);
/* Same, from a GGUF image in host memory (with no_upload/vocab_only only the
 * header -- metadata and tensor infos -- needs to be present). */
mi_model* mi_model_load_from_memory(const void* data, size_t size, const mi_model_params* params);
void mi_model_free(mi_model* model);

/* hparams / vocab queries: llama_vocab_n_tokens (Session.cpp:27),
 * llama_model_n_ctx_train (Model.cpp:41), llama_vocab_bos/eos (Instance.cpp:91-92),
 * llama_vocab_get_add_bos (Model.cpp:45), llama_model_meta_val_str (Model.cpp:57) */
int32_t mi_model_n_vocab(const mi_model* model);
int32_t mi_model_n_ctx_train(const mi_model* model);
int32_t mi_model_n_embd(const mi_model* model);
int32_t mi_model_n_layer(const mi_model* model);
int32_t mi_model_n_head(const mi_model* model);
int32_t mi_model_n_head_kv(const mi_model* model);
int32_t mi_model_n_ff(const mi_model* model);
int32_t mi_model_n_expert(const mi_model* model);
int32_t mi_model_token_bos(const mi_model* model);
int32_t mi_model_token_eos(const mi_model* model);
int32_t mi_model_add_bos(const mi_model* model);
int32_t mi_model_token_is_eog(const mi_model* model, int32_t token);
/* Text of a vocabulary entry (raw GGUF piece); returns its length or < 0. */
int32_t mi_model_token_text(const mi_model* model, int32_t token, char* buf, int32_t size);
/* Vocabulary for the host tokenizer (Vocab.cpp:37-72 -> llama_tokenize / llama_token_to_piece):
 * entries in tokenizer.ggml.tokens, SPM merge score, llama_token_type (1 normal, 2 unknown,
 * 3 control, 4 user-defined, 5 unused, 6 byte), and tokenizer.ggml.model ("llama" = SPM). */
int32_t mi_model_n_tokens(const mi_model* model);
float mi_model_token_score(const mi_model* model, int32_t token);
int32_t mi_model_token_type(const mi_model* model, int32_t token);
int32_t mi_model_tokenizer(const mi_model* model, char* buf, int32_t size);
int32_t mi_model_meta_str(const mi_model* model, const char* key, char* buf, int32_t size);
/* BPE vocabularies (tokenizer.ggml.model "gpt2", e.g. Llama-3): tokenizer.ggml.merges, rank = index;
 * mi_model_merge returns the length of merge i ("left right") or < 0. */
int32_t mi_model_n_merges(const mi_model* model);
int32_t mi_model_merge(const mi_model* model, int32_t i, char* buf, int32_t size);
/* Bytes of quantised weights a decode step streams (all tensors but tok_embd; of an MoE expert
 * tensor only the n_expert_used experts a token is routed to). */
int64_t mi_model_weight_bytes(const mi_model* model);
/* The device weight arena (one allocation) -- for the replica broadcast. */
int32_t mi_model_arena(const mi_model* model, void** dev_ptr, size_t* bytes);
/* Replicas for concurrent sessions (one worker per replica, Server.cpp:36): fills
 * the weight arenas of models[1..n-1] -- each loaded from the same GGUF with no_upload, i.e. the
 * header only -- from models[0].  Devices other than models[0]'s receive the arena by one RCCL
 * broadcast over xGMI (ncclCommInitAll over the distinct devices, root models[0]); further
 * replicas on a device take a device-to-device copy.  Call before any mi_ctx_create on the
 * replicas (their prompt-batch weight copies are built from the arena then).  0 ok, < 0 error. */
int32_t mi_model_replicate(mi_model* const* models, int32_t n);
/* Per ggml type id (0..31): bytes of weights of that type (the GGUF's byte histogram). */
int32_t mi_model_type_histogram(const mi_model* model, int64_t* bytes_by_type, int32_t n);

/* ---- context: replaces llama_init_from_model / llama_free (Instance.cpp:36);
 *      n_ctx 0 = training context (Instance.hpp:22) ---- */
mi_ctx* mi_ctx_create(mi_model* model, uint32_t n_ctx, uint32_t n_batch, uint32_t n_ubatch);
void mi_ctx_free(mi_ctx* ctx);
uint32_t mi_n_ctx(const mi_ctx* ctx);     /* llama_n_ctx   (Session.cpp:57,72,162,322) */
uint32_t mi_n_batch(const mi_ctx* ctx);   /* llama_n_batch (Session.cpp:381) */

/* llama_decode(llama_batch_get_one(tokens, n)) (Session.cpp:388, Instance.cpp:115):
 * tokens take positions pos_max+1...; asynchronous on the context's stream.
 * out_mode MI_OUT_LAST = logits of the last token only (llama_batch_get_one);
 * MI_OUT_ALL = logits of every token (a batch with logits[i] = true for all i), n <= n_batch:
 * output row i is the distribution after token i -- one batched pass in place of the
 * per-token decodes of Session::fillCtx (Session.cpp:231-244). */
#define MI_OUT_LAST 0
#define MI_OUT_ALL 1
int32_t mi_decode(mi_ctx* ctx, const int32_t* tokens, int32_t n, int32_t out_mode);

/* Output rows: -1 = the last token's; 0..n-1 after an MI_OUT_ALL decode of n tokens (row 0 only
 * after MI_OUT_LAST).  Top-k of an output row, sorted by logit descending then id ascending;
 * k <= 64.  Replaces fillLogits + std::sort + first 10 (Session.cpp:246-261) and
 * feeds the sampler chain's top_k(40) stage (Sampler.cpp:15-97).  Synchronises. */
int32_t mi_topk(mi_ctx* ctx, int32_t row, int32_t k, int32_t* ids, float* logits);
/* Logits of an output row at the given ids (Session.cpp:263-282).  Synchronises. */
int32_t mi_gather(mi_ctx* ctx, int32_t row, const int32_t* ids, int32_t n, float* out);
/* Batched form of mi_gather for a verification pass: rows row0 .. row0+n_rows-1, k ids per row
 * (ids and out are [n_rows][k]).  Returns n_rows*k or < 0.  Synchronises. */
int32_t mi_gather_rows(mi_ctx* ctx, int32_t row0, int32_t n_rows, const int32_t* ids, int32_t k, float* out);
/* Full-vocabulary escape hatch: llama_get_logits_ith(ctx, -1) (Session.cpp:24,
 * Sampler.cpp:111).  Context-owned; valid until the next decode.  Synchronises. */
const float* mi_logits(mi_ctx* ctx, int32_t row);
void mi_synchronize(mi_ctx* ctx);         /* llama_synchronize (Session.cpp:54) */

/* KV cache (single sequence): llama_kv_self_clear (Session.cpp:53),
 * llama_kv_self_seq_rm / seq_add / seq_div (Session.cpp:341-342, 359-361).
 * p1 < 0 means "to the end". */
void mi_kv_clear(mi_ctx* ctx);
int32_t mi_kv_seq_rm(mi_ctx* ctx, int32_t p0, int32_t p1);
int32_t mi_kv_seq_add(mi_ctx* ctx, int32_t p0, int32_t p1, int32_t delta);
int32_t mi_kv_seq_div(mi_ctx* ctx, int32_t p0, int32_t p1, int32_t d);
int32_t mi_kv_pos_max(const mi_ctx* ctx); /* -1 when empty */
int32_t mi_kv_n_cells(const mi_ctx* ctx);

/* State save/restore: llama_state_get_size / get_data / set_data (Session.cpp:291-304). */
size_t mi_state_size(mi_ctx* ctx);
size_t mi_state_get(mi_ctx* ctx, uint8_t* dst, size_t size);
size_t mi_state_set(mi_ctx* ctx, const uint8_t* src, size_t size);

/* ---- measurement: HIP events on the context's stream bracketing the FFN
 * gate/up GEMV launch of `layer` in every output-producing decode step (the
 * step's graph is split in three around it); layer < 0 disables.
 * mi_prof_read returns 1 and that launch's duration (microseconds) once per
 * timed step, 0 if no step was timed since the last read. ---- */
int32_t mi_prof_enable(mi_ctx* ctx, int32_t layer);
int32_t mi_prof_read(mi_ctx* ctx, float* us, int32_t n);
/* Algorithmic HBM bytes of one FFN gate/up launch (weights + activation in/out). */
int64_t mi_prof_ffn_bytes(const mi_ctx* ctx);
/* Algorithmic HBM bytes of the launch mi_prof_read last timed (the FFN gate/up launch). */
int64_t mi_prof_bytes(const mi_ctx* ctx);
/* Diagnostics: the form the context's decode steps take: 1 the streaming GEMV
 * launches (dgemv.hip; MoE: the attention half, the experts on gemv_kernel), 0 the gemv_kernel graph
 * (GPT-2); -1 for a null context. */
int32_t mi_decode_path(const mi_ctx* ctx);
/* Diagnostics: copies the per-workgroup s_memrealtime stamps (100 MHz) of the
 * first n_launch launches of the last decode step, [launch][512][8] uint64, to
 * out.  Returns the number of launches copied; 0 unless the library is the
 * diagnostic build (libmi_engine_stamps.so, compiled with -DMI_STAMPS). */
int32_t mi_debug_stamps(mi_ctx* ctx, uint64_t* out, int32_t n_launch);

/* ---- op-level entry points (host buffers in/out) used by the parity tests ----
 * raw_blocks: GGUF-layout blocks of a rows x K matrix of ggml type `type`. */
int32_t mi_op_gemv(int32_t device, int32_t type, const void* raw_blocks, int32_t rows, int32_t K,
                   const float* x, float* y);
int32_t mi_op_dequant(int32_t device, int32_t type, const void* raw_blocks, int32_t rows, int32_t K,
                      float* out);
int32_t mi_op_quantize_q8_K(int32_t device, const float* x, int32_t K, int8_t* qs, float* d,
                            int32_t* bsums);
int32_t mi_op_topk(int32_t device, const float* logits, int32_t n, int32_t k, int32_t* ids, float* vals);
/* One decode step's attention (KQ -> soft_max -> KQV, Session.cpp:388's llama_decode inner
 * graph, flash_attn=false) of n_head f32 query heads over n_cells cells of an f16 K/V cache
 * [n_cells][n_head_kv*head_dim]; cells whose cell_pos > pos are masked.  out: [n_head*head_dim]. */
int32_t mi_op_attention(int32_t device, int32_t n_head, int32_t n_head_kv, int32_t head_dim, int32_t n_cells,
                        const float* q, const uint16_t* k_f16, const uint16_t* v_f16, const int32_t* cell_pos,
                        int32_t pos, float* out);
/* The prompt-batch GEMM (Session.cpp:381-392's n_ubatch physical batches; ntok <= MI_MMQS_MAX,
 * default 64: the short-batch GEMM mmqs, otherwise the tiled int8-MFMA GEMM mmq32) of
 * ntok <= 512 token rows x[ntok][K] against a rows x K Q4_K / Q5_K / Q6_K / Q8_0 matrix: each row's
 * activation is quantised to Q8_K (Q8_0 for Q8_0 weights) as the CPU graph does, then
 * y[t][r] = vec_dot(W_r, q(x_t)).  With raw_up non-NULL the launch is the FFN gate/up pair
 * (raw_blocks = gate): y[t][r] = silu(gate_r . q(x_t)) * (up_r . q(x_t)).  y: [ntok][rows]. */
int32_t mi_op_gemm(int32_t device, int32_t type, const void* raw_blocks, const void* raw_up, int32_t rows,
                   int32_t K, int32_t ntok, const float* x, float* y);
/* The prompt-batch attention (attn_mfma: f16 MFMA) of ntok query tokens q[ntok][n_head*head_dim]
 * over an f16 cache of n_cells cells: token t sits in cell tok_cell[t] at position tok_pos[t] and
 * sees the cells c <= tok_cell[t] whose cell_pos[c] <= tok_pos[t] (llm_build_llama's kq_mask).
 * tok_cell must be ascending.  out: [ntok][n_head*head_dim]. */
int32_t mi_op_attention_batch(int32_t device, int32_t n_head, int32_t n_head_kv, int32_t head_dim,
                              int32_t n_cells, int32_t ntok, const float* q, const uint16_t* k_f16,
                              const uint16_t* v_f16, const int32_t* cell_pos, const int32_t* tok_cell,
                              const int32_t* tok_pos, float* out);
/* Median device time (us) of `iters` launches of the GEMV above (micro-benchmark). */
/* The decode step's streaming GEMV (dgemv.hip), one launch: x quantised on the device (Q8_K /
 * Q8_0 as the matrices need), then role 0 Q/K/V rows without RoPE (a second matrix of another type
 * = a second segment; y = [A x | B x]), 1 y = A x + resid, 2 y = silu(A x) * (B x) (gate/up pair),
 * 3 y = A x, 4 as 1 with x quantised inside the launch by every workgroup (the FFN down launch
 * of small models).  type2/raw2/rows2: the second matrix (raw2 NULL: none). */
int32_t mi_op_dgemv(int32_t device, int32_t role, int32_t type, const void* raw_blocks, int32_t rows, int32_t K,
                    int32_t type2, const void* raw_blocks2, int32_t rows2, const float* x, const float* resid, float* y);
int32_t mi_op_gemv_bench(int32_t device, int32_t type, const void* raw_blocks, int32_t rows, int32_t K,
                         int32_t iters, float* median_us);

#ifdef __cplusplus
}
#endif
#endif /* MI_ENGINE_H */
