// Engine host code: GGUF parsing, weight residency and the batch-1 decode
// schedule captured into HIP graphs.
//
// Reference anchors (the llama.h functions this replaces):
//   llama_model_load_from_file  /root/reference/inference/code/llama/Model.cpp:52
//   llama_init_from_model       /root/reference/inference/code/llama/Instance.cpp:36
//   llama_decode                /root/reference/inference/code/llama/Session.cpp:388
//   llama_get_logits_ith        /root/reference/inference/code/llama/Session.cpp:24
//   llama_kv_self_*             /root/reference/inference/code/llama/Session.cpp:53,341-361
//   llama_state_*               /root/reference/inference/code/llama/Session.cpp:291-304
#include "engine.h"

#include <atomic>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstring>

namespace mi {

static thread_local std::string g_last_error;
void set_last_error(const std::string& s) { g_last_error = s; }
const char* last_error() { return g_last_error.c_str(); }

// ================================================================== GGUF ===
namespace {
struct Reader {
    const uint8_t* p;
    size_t n, pos = 0;
    void need(size_t k) {
        if (pos + k > n) throw Error("GGUF: truncated header");
    }
    template <class T> T rd() {
        need(sizeof(T));
        T v;
        std::memcpy(&v, p + pos, sizeof(T));
        pos += sizeof(T);
        return v;
    }
    std::string str() {
        const uint64_t len = rd<uint64_t>();
        need(len);
        std::string s(reinterpret_cast<const char*>(p + pos), len);
        pos += len;
        return s;
    }
};

enum { G_U8 = 0, G_I8, G_U16, G_I16, G_U32, G_I32, G_F32, G_BOOL, G_STR, G_ARR, G_U64, G_I64, G_F64 };

double read_num(Reader& r, int t, bool* is_float) {
    *is_float = false;
    switch (t) {
    case G_U8: return r.rd<uint8_t>();
    case G_I8: return r.rd<int8_t>();
    case G_U16: return r.rd<uint16_t>();
    case G_I16: return r.rd<int16_t>();
    case G_U32: return r.rd<uint32_t>();
    case G_I32: return r.rd<int32_t>();
    case G_F32: *is_float = true; return r.rd<float>();
    case G_BOOL: return r.rd<uint8_t>();
    case G_U64: return (double)r.rd<uint64_t>();
    case G_I64: return (double)r.rd<int64_t>();
    case G_F64: *is_float = true; return r.rd<double>();
    default: throw Error("GGUF: bad value type");
    }
}
}  // namespace

void Gguf::parse(const uint8_t* data, size_t size) {
    Reader r{data, size};
    if (size < 24 || std::memcmp(data, "GGUF", 4) != 0) throw Error("not a GGUF file");
    r.pos = 4;
    const uint32_t ver = r.rd<uint32_t>();
    if (ver != 2 && ver != 3) throw Error("unsupported GGUF version " + std::to_string(ver));
    const uint64_t nt = r.rd<uint64_t>(), nkv = r.rd<uint64_t>();
    for (uint64_t i = 0; i < nkv; ++i) {
        std::string key = r.str();
        GgufValue v;
        v.type = (int)r.rd<uint32_t>();
        if (v.type == G_STR) {
            v.s = r.str();
        } else if (v.type == G_ARR) {
            v.arr_type = (int)r.rd<uint32_t>();
            v.arr_n = (long long)r.rd<uint64_t>();
            if (v.arr_type == G_STR) {
                v.arr_s.reserve(v.arr_n);
                for (long long k = 0; k < v.arr_n; ++k) v.arr_s.push_back(r.str());
            } else {
                v.arr_num.reserve(v.arr_n);
                bool fl;
                for (long long k = 0; k < v.arr_n; ++k) v.arr_num.push_back(read_num(r, v.arr_type, &fl));
            }
        } else {
            bool fl;
            const double d = read_num(r, v.type, &fl);
            v.f = d;
            v.i = (long long)d;
        }
        kv.emplace(std::move(key), std::move(v));
    }
    for (uint64_t i = 0; i < nt; ++i) {
        GgufTensor t;
        t.name = r.str();
        t.n_dims = (int)r.rd<uint32_t>();
        if (t.n_dims < 1 || t.n_dims > 4) throw Error("GGUF: bad n_dims for " + t.name);
        long long n = 1;
        for (int d = 0; d < t.n_dims; ++d) { t.ne[d] = (long long)r.rd<uint64_t>(); n *= t.ne[d]; }
        t.type = (int)r.rd<uint32_t>();
        t.offset = r.rd<uint64_t>();
        const int be = block_elems(t.type), bb = block_bytes(t.type);
        if (bb == 0) {
            t.nbytes = 0;   // unsupported type: only an error if the tensor is used
        } else {
            if (n % be) throw Error("GGUF: tensor " + t.name + " not a whole number of blocks");
            t.nbytes = (size_t)(n / be) * bb;
        }
        tensors.push_back(t);
    }
    const long long align = get_int("general.alignment", 32);
    data_offset = (r.pos + align - 1) / align * align;
}

long long Gguf::get_int(const std::string& k, long long def) const {
    const GgufValue* v = get(k);
    return (v && v->type != G_STR && v->type != G_ARR) ? v->i : def;
}
double Gguf::get_float(const std::string& k, double def) const {
    const GgufValue* v = get(k);
    return (v && v->type != G_STR && v->type != G_ARR) ? v->f : def;
}
std::string Gguf::get_str(const std::string& k, const std::string& def) const {
    const GgufValue* v = get(k);
    return (v && v->type == G_STR) ? v->s : def;
}
const GgufTensor* Gguf::tensor(const std::string& name) const {
    for (const auto& t : tensors)
        if (t.name == name) return &t;
    return nullptr;
}

// ================================================================= model ===
Model::~Model() {
    if (arena || mmq_arena || gelu_tab) hipSetDevice(device);
    if (arena) hipFree(arena);
    if (mmq_arena) hipFree(mmq_arena);
    if (gelu_tab) hipFree(gelu_tab);
}

namespace {
// ggml_table_gelu_f16 (ggml-cpu.c init with GGML_GELU_FP16): fp16(ggml_gelu_f32(fp32(h))) for
// every f16 bit pattern h, ggml_gelu_f32(x) = 0.5f*x*(1.0f + tanhf(SQRT_2_OVER_PI*x*(1.0f +
// GELU_COEF_A*x*x))), evaluated on the host with the C library's tanhf (no FMA contraction:
// -ffp-contract=off), as the reference's CPU build evaluates it.
std::vector<unsigned short> gelu_table_host() {
    std::vector<unsigned short> t(65536);
    const float A = 0.044715f, K = 0.79788456080286535587989211986876f;
    for (int i = 0; i < 65536; ++i) {
        const unsigned short h = (unsigned short)i;
        _Float16 hf;
        std::memcpy(&hf, &h, 2);
        const float x = (float)hf;
        const float g = 0.5f * x * (1.0f + tanhf(K * x * (1.0f + A * x * x)));
        const _Float16 r = (_Float16)g;
        std::memcpy(&t[i], &r, 2);
    }
    return t;
}
}  // namespace

// Expert e of a MoE tensor as a matrix of its own (planes and MFMA-order copy offset).
QMat expert_view(const QMat& q, int e) {
    QMat v = q;
    for (int k = 0; k < 4; ++k)
        if (v.p[k]) v.p[k] += e * q.expert_stride[k];
    if (v.sw) v.sw += e * q.sw_expert_stride;
    return v;
}

bool Model::ensure_mmq_copies() {
    std::lock_guard<std::mutex> lk(mmq_mu);
    if (mmq_arena) return true;
    MI_HIP(hipSetDevice(device));
    // every mmq32-capable projection (gate and up as one pair copy; MoE: one copy per expert,
    // expert e at sw + e * sw_expert_stride) and the output head
    std::vector<std::pair<QMat*, QMat*>> todo;
    for (Layer& L : layers) {
        for (QMat* q : {&L.wq, &L.wk, &L.wv, &L.wo, &L.down})
            if (mmq32_supported(q->type)) todo.push_back({q, nullptr});
        if (mmq32_supported(L.gate.type) && L.up.type == L.gate.type) todo.push_back({&L.gate, &L.up});
    }
    if (mmq32_supported(output.type)) todo.push_back({&output, nullptr});
    auto experts = [](const QMat& q) { return std::max(1, q.n_exp); };
    size_t total = 0;
    std::vector<size_t> offs;
    for (auto& t : todo) {
        offs.push_back(total);
        const size_t one = mmq32_copy_bytes(*t.first, t.second != nullptr);
        total = (total + one * experts(*t.first) + 255) & ~size_t(255);
    }
    if (!total) return true;
    if (hipMalloc(&mmq_arena, total) != hipSuccess) {
        (void)hipGetLastError();   // clear the sticky error; the caller falls back
        mmq_arena = nullptr;
        return false;
    }
    mmq_bytes = total;
    for (size_t i = 0; i < todo.size(); ++i) {
        QMat& A = *todo[i].first;
        const size_t one = mmq32_copy_bytes(A, todo[i].second != nullptr);
        for (int e = 0; e < experts(A); ++e) {   // expert e's planes -> its own copy
            QMat a = expert_view(A, e), b = todo[i].second ? expert_view(*todo[i].second, e) : QMat{};
            launch_mmq32_swizzle(a, todo[i].second ? &b : nullptr, mmq_arena + offs[i] + one * e, nullptr);
        }
        A.sw = mmq_arena + offs[i];
        A.sw_expert_stride = (long long)one;
    }
    MI_HIP(hipDeviceSynchronize());
    return true;
}

const QMat* Model::find_qmat(const std::string&) const { return nullptr; }

namespace {
size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

struct Planned {
    const GgufTensor* t;
    size_t off[4];     // arena offsets of the planes (quant) or of the raw copy (p0)
    long long rows;    // rows across all experts
    int K;
    int experts;
};
}  // namespace

void Model::load(const uint8_t* data, size_t size, const mi_model_params& p) {
    device = p.device_ordinal;
    vocab_only = p.vocab_only != 0;
    gguf.parse(data, size);
    const std::string arch = gguf.get_str("general.architecture", "");
    if (arch != "llama" && arch != "gpt2")
        throw Error("unsupported architecture '" + arch + "' (this backend serves the llama and gpt2 graphs)");
    hp.arch = arch == "gpt2" ? ARCH_GPT2 : ARCH_LLAMA;
    auto key = [&](const char* k) { return arch + "." + k; };
    hp.n_embd = (int)gguf.get_int(key("embedding_length"), 0);
    hp.n_layer = (int)gguf.get_int(key("block_count"), 0);
    hp.n_ff = (int)gguf.get_int(key("feed_forward_length"), 0);
    hp.n_head = (int)gguf.get_int(key("attention.head_count"), 0);
    hp.n_head_kv = (int)gguf.get_int(key("attention.head_count_kv"), hp.n_head);
    hp.n_ctx_train = (int)gguf.get_int(key("context_length"), 2048);
    hp.eps = (float)gguf.get_float(key(hp.arch == ARCH_GPT2 ? "attention.layer_norm_epsilon"
                                                             : "attention.layer_norm_rms_epsilon"), 1e-5);
    hp.rope_base = (float)gguf.get_float(key("rope.freq_base"), 10000.0);
    const double fs = gguf.get_float(key("rope.scale_linear"), 0.0);
    hp.freq_scale = fs > 0.0 ? (float)(1.0 / fs) : 1.0f;
    hp.n_expert = (int)gguf.get_int(key("expert_count"), 0);
    hp.n_expert_used = (int)gguf.get_int(key("expert_used_count"), 0);
    if (hp.n_embd <= 0 || hp.n_layer <= 0 || hp.n_head <= 0) throw Error("GGUF: missing llama hparams");
    hp.head_dim = hp.n_embd / hp.n_head;
    hp.n_rot = hp.arch == ARCH_GPT2 ? 0 : (int)gguf.get_int(key("rope.dimension_count"), hp.head_dim);
    if (hp.arch == ARCH_GPT2 && hp.n_expert) throw Error("gpt2: no MoE");

    if (const GgufValue* tv = gguf.get("tokenizer.ggml.tokens")) tokens = tv->arr_s;
    if (const GgufValue* tt = gguf.get("tokenizer.ggml.token_type"))
        for (double d : tt->arr_num) token_type.push_back((int)d);
    if (const GgufValue* ts = gguf.get("tokenizer.ggml.scores"))
        for (double d : ts->arr_num) token_score.push_back((float)d);
    tok_model = gguf.get_str("tokenizer.ggml.model", "llama");
    if (const GgufValue* mv = gguf.get("tokenizer.ggml.merges")) merges = mv->arr_s;
    hp.n_vocab = (int)tokens.size();
    if (const GgufTensor* te = gguf.tensor("token_embd.weight")) hp.n_vocab = (int)te->ne[1];
    bos = (int)gguf.get_int("tokenizer.ggml.bos_token_id", 1);
    eos = (int)gguf.get_int("tokenizer.ggml.eos_token_id", 2);
    eot = (int)gguf.get_int("tokenizer.ggml.eot_token_id", -1);
    add_bos = gguf.get_int("tokenizer.ggml.add_bos_token", 1) != 0;
    if (vocab_only) return;
    if (p.cpu_only) throw Error("cpu_only models are served by the CPU reference path, not this engine");

    // ---- plan the arena ----
    std::vector<Planned> plan;
    size_t off = 0;
    auto add = [&](const std::string& name, bool required, int experts) -> int {
        const GgufTensor* t = gguf.tensor(name);
        if (!t) {
            if (required) throw Error("GGUF: missing tensor " + name);
            return -1;
        }
        Planned pl{};
        pl.t = t;
        pl.K = (int)t->ne[0];
        pl.experts = experts;
        pl.rows = t->ne[1] * (t->n_dims > 2 ? t->ne[2] : 1);
        if (is_quant(t->type)) {
            if (pl.K % 256) throw Error("tensor " + name + ": K not a multiple of 256");
            const long long nsb = pl.rows * (pl.K / 256);
            for (int k = 0; k < plane_count(t->type); ++k) {
                pl.off[k] = off;   // + 8 superblocks of tail padding read by idle GEMV lanes
                off = align256(off + (size_t)(nsb + kPlanePadSb) * plane_sb_bytes(t->type, k));
            }
        } else if (t->type == T_F32 || t->type == T_F16) {
            pl.off[0] = off;
            off = align256(off + t->nbytes);
        } else {
            throw Error("tensor " + name + ": unsupported ggml type " + std::to_string(t->type));
        }
        plan.push_back(pl);
        return (int)plan.size() - 1;
    };
    // Q/K/V of one layer as groups of adjacent same-type tensors whose planes are stored back to
    // back (plane k of the group = plane k of each tensor in order): one decode-GEMV matrix each
    auto add_group = [&](const std::vector<std::string>& names, std::vector<int>& idx) {
        std::vector<const GgufTensor*> ts;
        for (const auto& n : names) {
            const GgufTensor* t = gguf.tensor(n);
            if (!t) throw Error("GGUF: missing tensor " + n);
            ts.push_back(t);
        }
        const int type = ts[0]->type;
        const int K = (int)ts[0]->ne[0];
        if (!is_quant(type) || K % 256) throw Error("tensor " + names[0] + ": not a quantised matrix with K % 256 == 0");
        const size_t first = plan.size();
        for (const GgufTensor* t : ts) {
            if (t->type != type || (int)t->ne[0] != K) throw Error("add_group: mixed tensors");
            Planned pl{};
            pl.t = t;
            pl.K = K;
            pl.experts = 1;
            pl.rows = t->ne[1];
            plan.push_back(pl);
            idx.push_back((int)plan.size() - 1);
        }
        for (int k = 0; k < plane_count(type); ++k) {
            for (size_t i = first; i < plan.size(); ++i) {
                plan[i].off[k] = off;
                off += (size_t)plan[i].rows * (K / 256) * plane_sb_bytes(type, k);
            }
            off = align256(off + (size_t)kPlanePadSb * plane_sb_bytes(type, k));
        }
    };
    struct LayerIdx {
        int an, fn, q, k, v, o, g, u, d, r;
        std::vector<std::vector<int>> qkv_groups;
        int anb = -1, fnb = -1, bqkv = -1, bo = -1, bu = -1, bd = -1;   // GPT-2 biases
    };
    const bool gpt2 = hp.arch == ARCH_GPT2;
    const int i_te = add("token_embd.weight", true, 1);
    const int i_pe = gpt2 ? add("position_embd.weight", true, 1) : -1;
    const int i_on = add("output_norm.weight", true, 1);
    const int i_onb = gpt2 ? add("output_norm.bias", true, 1) : -1;
    int i_out = add("output.weight", false, 1);
    const int i_rf = add("rope_freqs.weight", false, 1);
    std::vector<LayerIdx> li(hp.n_layer);
    const int E = hp.n_expert > 0 ? hp.n_expert : 1;
    for (int l = 0; l < hp.n_layer && gpt2; ++l) {   // llm_build_gpt2's tensors (LLM_ARCH_GPT2)
        const std::string b = "blk." + std::to_string(l) + ".";
        LayerIdx& x = li[l];
        x.an = add(b + "attn_norm.weight", true, 1);
        x.anb = add(b + "attn_norm.bias", true, 1);
        x.fn = add(b + "ffn_norm.weight", true, 1);
        x.fnb = add(b + "ffn_norm.bias", true, 1);
        std::vector<int> idx;
        add_group({b + "attn_qkv.weight"}, idx);   // one fused [3 n_embd] x n_embd matrix
        x.qkv_groups.push_back(idx);
        x.q = x.k = x.v = idx[0];
        x.bqkv = add(b + "attn_qkv.bias", true, 1);
        x.o = add(b + "attn_output.weight", true, 1);
        x.bo = add(b + "attn_output.bias", true, 1);
        x.r = -1;
        x.g = x.u = add(b + "ffn_up.weight", true, 1);
        x.bu = add(b + "ffn_up.bias", true, 1);
        x.d = add(b + "ffn_down.weight", true, 1);
        x.bd = add(b + "ffn_down.bias", true, 1);
    }
    for (int l = 0; l < hp.n_layer && !gpt2; ++l) {
        const std::string b = "blk." + std::to_string(l) + ".";
        LayerIdx& x = li[l];
        x.an = add(b + "attn_norm.weight", true, 1);
        x.fn = add(b + "ffn_norm.weight", true, 1);
        {
            const std::string nq = b + "attn_q.weight", nk = b + "attn_k.weight", nv = b + "attn_v.weight";
            const GgufTensor *tq = gguf.tensor(nq), *tk = gguf.tensor(nk), *tv = gguf.tensor(nv);
            if (!tq || !tk || !tv) throw Error("GGUF: missing attention tensors in " + b);
            std::vector<std::vector<std::string>> groups;
            if (tq->type == tk->type && tk->type == tv->type) groups = {{nq, nk, nv}};
            else if (tq->type == tk->type) groups = {{nq, nk}, {nv}};
            else if (tk->type == tv->type) groups = {{nq}, {nk, nv}};
            else groups = {{nq}, {nk}, {nv}};
            std::vector<int> all;
            for (const auto& g : groups) {
                std::vector<int> idx;
                add_group(g, idx);
                x.qkv_groups.push_back(idx);
                all.insert(all.end(), idx.begin(), idx.end());
            }
            x.q = all[0];
            x.k = all[1];
            x.v = all[2];
        }
        x.o = add(b + "attn_output.weight", true, 1);
        if (hp.n_expert > 0) {
            x.r = add(b + "ffn_gate_inp.weight", true, 1);
            x.g = add(b + "ffn_gate_exps.weight", true, E);
            x.u = add(b + "ffn_up_exps.weight", true, E);
            x.d = add(b + "ffn_down_exps.weight", true, E);
        } else {
            x.r = -1;
            x.g = add(b + "ffn_gate.weight", true, 1);
            x.u = add(b + "ffn_up.weight", true, 1);
            x.d = add(b + "ffn_down.weight", true, 1);
        }
    }
    if (hp.n_expert > 0 && hp.n_expert_used != 2)
        throw Error("MoE: this build serves top-2 routing (expert_used_count=2)");
    arena_bytes = off;
    for (const auto& pl : plan) {
        // bytes one decode step streams: an expert tensor contributes the n_expert_used experts
        // the router picks (build_moe_ffn reads only those), not all n_expert of them
        if (pl.t->name != "token_embd.weight" && pl.t->name != "position_embd.weight")
            weight_bytes += pl.experts > 1 ? (long long)pl.t->nbytes / pl.experts * hp.n_expert_used
                                           : (long long)pl.t->nbytes;
        if (pl.t->type >= 0 && pl.t->type < 32) type_bytes[pl.t->type] += (long long)pl.t->nbytes;
    }
    if (i_out < 0) weight_bytes += (long long)plan[i_te].t->nbytes;   // tied output head

    MI_HIP(hipSetDevice(device));
    MI_HIP(hipMalloc(&arena, arena_bytes));

    // ---- upload + repack ----
    if (!p.no_upload) {
        size_t max_raw = 0;
        for (const auto& pl : plan)
            if (is_quant(pl.t->type)) max_raw = std::max(max_raw, pl.t->nbytes);
        uint8_t* staging = nullptr;
        if (max_raw) MI_HIP(hipMalloc(&staging, max_raw));
        for (const auto& pl : plan) {
            const size_t src = gguf.data_offset + pl.t->offset;
            if (src + pl.t->nbytes > size) {
                if (staging) hipFree(staging);
                throw Error("GGUF: tensor data of " + pl.t->name + " beyond the end of the image");
            }
            if (is_quant(pl.t->type)) {
                MI_HIP(hipMemcpy(staging, data + src, pl.t->nbytes, hipMemcpyHostToDevice));
                uint8_t* planes[4] = {arena + pl.off[0], arena + pl.off[1], arena + pl.off[2], arena + pl.off[3]};
                launch_repack(staging, pl.t->type, pl.rows, pl.K, planes, nullptr);
            } else {
                MI_HIP(hipMemcpy(arena + pl.off[0], data + src, pl.t->nbytes, hipMemcpyHostToDevice));
            }
        }
        MI_HIP(hipDeviceSynchronize());
        if (staging) hipFree(staging);
    }

    // ---- device views ----
    auto qm = [&](int idx) -> QMat {
        QMat m{};
        const Planned& pl = plan[idx];
        m.type = pl.t->type;
        m.K = pl.K;
        m.nb = pl.K / 256;
        m.rows = (int)(pl.rows / pl.experts);
        m.n_exp = pl.experts;
        if (is_quant(m.type)) {
            for (int k = 0; k < plane_count(m.type); ++k) {
                m.p[k] = arena + pl.off[k];
                m.expert_stride[k] = (long long)m.rows * m.nb * plane_sb_bytes(m.type, k);
            }
        } else {
            m.p[0] = arena + pl.off[0];
        }
        return m;
    };
    auto f32p = [&](int idx) -> float* {
        if (idx < 0) return nullptr;
        if (plan[idx].t->type != T_F32) throw Error("tensor " + plan[idx].t->name + " must be F32");
        return reinterpret_cast<float*>(arena + plan[idx].off[0]);
    };
    tok_embd = qm(i_te);
    if (i_pe >= 0) pos_embd = qm(i_pe);
    output_norm_b = f32p(i_onb);
    output = i_out >= 0 ? qm(i_out) : qm(i_te);
    if (!is_quant(output.type)) throw Error("output head must be a quantised tensor in this build");
    output_norm = f32p(i_on);
    rope_freqs = f32p(i_rf);
    layers.resize(hp.n_layer);
    for (int l = 0; l < hp.n_layer; ++l) {
        Layer& L = layers[l];
        const LayerIdx& x = li[l];
        L.attn_norm = f32p(x.an);
        L.ffn_norm = f32p(x.fn);
        L.wq = qm(x.q); L.wk = qm(x.k); L.wv = qm(x.v); L.wo = qm(x.o);
        L.gate = qm(x.g); L.up = qm(x.u); L.down = qm(x.d);
        L.router = f32p(x.r);
        L.attn_norm_b = f32p(x.anb);
        L.ffn_norm_b = f32p(x.fnb);
        L.bqkv = f32p(x.bqkv);
        L.bo = f32p(x.bo);
        L.bup = f32p(x.bu);
        L.bdown = f32p(x.bd);
        for (const QMat* m : {&L.wq, &L.wk, &L.wv, &L.wo, &L.gate, &L.up, &L.down})
            if (!is_quant(m->type)) throw Error("layer weights must be quantised (Q4_K/Q5_K/Q6_K/Q8_0)");
        if (gpt2) {   // the fused QKV rows: n_embd Q rows, n_embd K rows, n_embd V rows
            L.n_qkv = 1;
            L.qkv[0] = qm(x.qkv_groups[0][0]);
            L.qkv_nq[0] = hp.n_embd;
            L.qkv_nk[0] = hp.n_head_kv * hp.head_dim;
            if (L.qkv[0].rows != L.qkv_nq[0] + 2 * L.qkv_nk[0]) throw Error("gpt2: attn_qkv must have 3 n_embd rows");
            continue;
        }
        L.n_qkv = (int)x.qkv_groups.size();
        int seen = 0;   // Q rows, then K rows, then V rows across the groups
        for (int g = 0; g < L.n_qkv; ++g) {
            QMat m = qm(x.qkv_groups[g][0]);
            int nq = 0, nk = 0, rows = 0;
            for (int i : x.qkv_groups[g]) {
                const int r = (int)plan[i].rows;
                if (seen == 0) nq += r;
                else if (seen == 1) nk += r;
                rows += r;
                ++seen;
            }
            m.rows = rows;
            L.qkv[g] = m;
            L.qkv_nq[g] = nq;
            L.qkv_nk[g] = nk;
        }
    }
    if (gpt2) {
        const std::vector<unsigned short> t = gelu_table_host();
        MI_HIP(hipMalloc(&gelu_tab, t.size() * sizeof(unsigned short)));
        MI_HIP(hipMemcpy(gelu_tab, t.data(), t.size() * sizeof(unsigned short), hipMemcpyHostToDevice));
    }
}

// =============================================================== context ===
namespace {
std::vector<int> g_attr_done(64, 0);

namespace {
struct DevChain {
    std::mutex mu;
    std::atomic<int> nctx{0};  // live contexts on the device (attention co-residency budget)
};
DevChain& dev_chain(int device) {
    static std::mutex mu;
    static std::map<int, std::unique_ptr<DevChain>> chains;
    std::lock_guard<std::mutex> lk(mu);
    auto& c = chains[device];
    if (!c) c.reset(new DevChain());
    return *c;
}
}  // namespace

GemvSeg seg_of(const QMat& A, int pair, int epi, float* out) {
    GemvSeg g;
    std::memset(&g, 0, sizeof(g));
    g.A = A;
    g.B = A;
    g.pair = pair;
    g.epi = epi;
    g.expA = g.expB = -1;
    g.out = out;
    return g;
}
}  // namespace
int dev_chain_contexts(int device) { return dev_chain(device).nctx.load(); }

Ctx::Ctx(Model* model, uint32_t nctx, uint32_t nbatch, uint32_t nubatch) : m(model) {
    if (m->vocab_only) throw Error("cannot create a context on a vocab-only model");
    device = m->device;
    MI_HIP(hipSetDevice(device));
    n_ctx = nctx ? nctx : (uint32_t)m->hp.n_ctx_train;
    n_batch = std::min(nbatch ? nbatch : 2048u, n_ctx);   // "may be silently truncated to ctxSize"
    n_ubatch = nubatch ? std::min(nubatch, n_batch) : n_batch;
    const HParams& hp = m->hp;
    kv_dim = hp.n_head_kv * hp.head_dim;
    if (device < (int)g_attr_done.size() && !g_attr_done[device]) {
        init_kernel_attributes();
        g_attr_done[device] = 1;
    }
    MI_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    const size_t kvb = (size_t)hp.n_layer * n_ctx * kv_dim * sizeof(__half);
    MI_HIP(hipMalloc(&kcache, kvb));
    MI_HIP(hipMalloc(&vcache, kvb));
    MI_HIP(hipMemset(kcache, 0, kvb));
    MI_HIP(hipMemset(vcache, 0, kvb));
    MI_HIP(hipMalloc(&cell_pos, n_ctx * sizeof(int)));
    MI_HIP(hipMemset(cell_pos, 0, n_ctx * sizeof(int)));
    MI_HIP(hipMalloc(&tokpos, 4 * sizeof(int)));
    MI_HIP(hipMemset(tokpos, 0, 4 * sizeof(int)));
    const int big = std::max(hp.n_embd, hp.n_ff);
    MI_HIP(hipMalloc(&x, hp.n_embd * sizeof(float)));
    MI_HIP(hipMalloc(&q, hp.n_embd * sizeof(float)));
    MI_HIP(hipMalloc(&attn, hp.n_embd * sizeof(float)));
    MI_HIP(hipMalloc(&h, big * sizeof(float)));
    MI_HIP(hipMalloc(&h2, big * sizeof(float)));
    MI_HIP(hipMalloc(&logits, (size_t)hp.n_vocab * sizeof(float)));
    MI_HIP(hipMalloc(&cand, (size_t)topk_blocks(hp.n_vocab) * TOPK_MAX * sizeof(unsigned long long)));
    MI_HIP(hipMalloc(&part_o, (size_t)ATTN_SMAX * hp.n_head * hp.head_dim * sizeof(float)));
#ifdef MI_STAMPS
    MI_HIP(hipMalloc(&stamps, (size_t)kStampLaunches * kStampWgs * 8 * sizeof(unsigned long long)));
    MI_HIP(hipMemset(stamps, 0, (size_t)kStampLaunches * kStampWgs * 8 * sizeof(unsigned long long)));
#endif
    // GPT-2 prompts run token by token (one decode graph each): its batch kernels (LayerNorm,
    // biases, GELU) are not built
    batch_ok = hp.arch == ARCH_LLAMA && getenv("MI_NO_BATCH") == nullptr;
    if (batch_ok) {
        // MFMA batch path (decode_ubatch / mmq32) when every layer matrix is mmq32-capable (each
        // matrix reads the activation format of its type: Q8_0 activations for Q8_0 weights, Q8_K
        // for the k-quants); otherwise prompt chunks on the v_dot4 GEMM (decode_batch, dense only)
        mmq_ok = getenv("MI_NO_MMQ") == nullptr;
        bool any_k = false, any_0 = false;
        for (const Layer& L : m->layers)
            for (const QMat* q : {&L.wq, &L.wk, &L.wv, &L.wo, &L.gate, &L.up, &L.down}) {
                mmq_ok = mmq_ok && mmq32_supported(q->type);
                (q->type == T_Q8_0 ? any_0 : any_k) = true;
            }
        // the gate/up pair shares one MFMA-order copy (16 gate + 16 up rows per tile)
        for (const Layer& L : m->layers)
            mmq_ok = mmq_ok && L.gate.type == L.up.type && L.gate.rows == L.up.rows;
        const int NB = kBatchRows;
        // MoE: a row per (token, slot), each expert's rows padded to whole 32-row tiles
        const int hrows = hp.n_expert > 0 ? moe_rows_cap(NB * hp.n_expert_used, hp.n_expert) : NB;
        MI_HIP(hipMalloc(&xb, (size_t)NB * hp.n_embd * sizeof(float)));
        MI_HIP(hipMalloc(&qb, (size_t)NB * hp.n_embd * sizeof(float)));
        MI_HIP(hipMalloc(&attnb, (size_t)NB * hp.n_embd * sizeof(float)));
        MI_HIP(hipMalloc(&hb, (size_t)hrows * hp.n_ff * sizeof(float)));
        MI_HIP(hipMalloc(&tokpos_b, (size_t)NB * 4 * sizeof(int)));
        MI_HIP(hipHostMalloc(&h_tokpos_b, (size_t)kTokbRing * NB * 4 * sizeof(int)));
        const int kmax = std::max(hp.n_embd, hp.n_ff);
        if (mmq_ok) {
            // ub_q / ub_dT / ub_bsb: the k-quant (Q8_K) activations, or the Q8_0 ones when every
            // matrix is Q8_0; a model mixing both (Mixtral's Q8_0 attn_k / attn_v) has a second
            // set ub_q0 / ub_dT0 for Q8_0
            ub_q80 = !any_k;
            // no room for the copy: prompt batches fall back to the v_dot4 GEMM
            mmq_ok = m->ensure_mmq_copies();
            out_mmq = mmq_ok && mmq32_supported(m->output.type);
            attn_mfma = attn_mfma_supported(hp.head_dim);
            MI_HIP(hipMalloc(&ub_q, (size_t)UB_MAX * kmax));
            MI_HIP(hipMalloc(&ub_dT, (size_t)UB_MAX * (kmax / 32) * sizeof(float)));   // Q8_0: per 32
            MI_HIP(hipMalloc(&ub_bsb, (size_t)UB_MAX * (kmax / 256) * 16));
            if (any_k && any_0) {
                MI_HIP(hipMalloc(&ub_q0, (size_t)UB_MAX * kmax));
                MI_HIP(hipMalloc(&ub_dT0, (size_t)UB_MAX * (kmax / 32) * sizeof(float)));
            }
            if (hp.n_expert > 0) {   // routing of a physical batch, grouped rows, expert down outputs
                if (hp.n_expert > MOE_GROUP_MAXE) throw Error("MoE prompt batches: at most 16 experts");
                const int ns = NB * hp.n_expert_used;
                const int cap = moe_rows_cap(ns, hp.n_expert);
                MI_HIP(hipMalloc(&yb, (size_t)cap * hp.n_embd * sizeof(float)));
                MI_HIP(hipMalloc(&sel_b, (size_t)ns * sizeof(int)));
                MI_HIP(hipMalloc(&selw_b, (size_t)ns * sizeof(float)));
                MI_HIP(hipMalloc(&moe_rows, (size_t)cap * sizeof(int)));
                MI_HIP(hipMalloc(&moe_rowsel, (size_t)cap * sizeof(int)));
                MI_HIP(hipMalloc(&moe_pos, (size_t)ns * sizeof(int)));
                MI_HIP(hipMalloc(&moe_grp, (size_t)(2 * MOE_GROUP_MAXE + 1) * sizeof(int)));
                MI_HIP(hipMalloc(&moe_q, (size_t)cap * kmax));
                MI_HIP(hipMalloc(&moe_dT, (size_t)cap * (kmax / 32) * sizeof(float)));
                MI_HIP(hipMalloc(&moe_bsb, (size_t)cap * (kmax / 256) * 16));
            }
            MI_HIP(hipMalloc(&ub_rope, (size_t)UB_MAX * std::max(1, hp.n_rot / 2) * sizeof(float2)));
            // split-K partials of the residual GEMMs (WO, FFN down) of dense models
            if (mmq2_active())
                MI_HIP(hipMalloc(&ub_part, (size_t)2 * UB_MAX * hp.n_embd * sizeof(float)));
            mmqs_max = getenv("MI_MMQS_MAX") ? std::min(MMQS_MAX, std::max(0, atoi(getenv("MI_MMQS_MAX")))) : MMQS_MAX;
            // MoE: short batches when every expert matrix has the grouped form (k-quants)
            moe_short = hp.n_expert > 0;
            for (const Layer& L : m->layers)
                moe_short = moe_short && mmqs_grouped_supported(L.gate.type) && L.up.type == L.gate.type &&
                            mmqs_grouped_supported(L.down.type);
            if (mmqs_max > 0 && (hp.n_expert == 0 || moe_short)) {
                const size_t qkv = (size_t)hp.n_embd + 2 * (size_t)kv_dim;
                size_t per = std::max({(size_t)mmqs_parts(hp.n_embd) * std::max({qkv, (size_t)hp.n_embd, 2 * (size_t)hp.n_ff}),
                                       (size_t)mmqs_parts(hp.n_ff) * hp.n_embd});
                if (out_mmq) per = std::max(per, (size_t)mmqs_parts(hp.n_embd) * hp.n_vocab);
                size_t tot = per * MMQS_MAX;
                if (moe_short)   // the experts' parts over the MoE rows of MMQS_MAX tokens
                    tot = std::max(tot, std::max((size_t)mmqs_parts(hp.n_embd) * 2 * hp.n_ff, (size_t)mmqs_parts(hp.n_ff) * hp.n_embd) *
                                            (size_t)moe_rows_cap(MMQS_MAX * hp.n_expert_used, hp.n_expert));
                MI_HIP(hipMalloc(&ub_spart, tot * sizeof(float)));
            } else {
                moe_short = false;
                mmqs_max = 0;
            }
        }
        // MoE prompts need the MFMA path (the v_dot4 GEMM has no routed-expert form)
        if (hp.n_expert > 0 && !mmq_ok) batch_ok = false;
    }
    MI_HIP(hipMalloc(&attn_smax, (size_t)ATTN_SMAX * hp.n_head * sizeof(float)));
    MI_HIP(hipMalloc(&attn_scores, (size_t)hp.n_head * n_ctx * sizeof(float)));
    MI_HIP(hipMalloc(&attn_xflags, (size_t)hp.n_head * ATTN_SMAX * 32 * sizeof(unsigned)));
    MI_HIP(hipMemset(attn_xflags, 0, (size_t)hp.n_head * ATTN_SMAX * 32 * sizeof(unsigned)));
    MI_HIP(hipMalloc(&attn_xmax, (size_t)hp.n_head * ATTN_SMAX * sizeof(float)));
    MI_HIP(hipMalloc(&attn_xsum, (size_t)hp.n_head * ATTN_SMAX * sizeof(double)));
    MI_HIP(hipMalloc(&step_ctr, 16));
    MI_HIP(hipMemset(step_ctr, 0, 16));
    MI_HIP(hipHostMalloc(&h_attn_xerr, 16, hipHostMallocMapped | hipHostMallocCoherent));
    *h_attn_xerr = 0;
    MI_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&d_attn_xerr), h_attn_xerr, 0));
    MI_HIP(hipMalloc(&topk_ids, TOPK_MAX * sizeof(int)));
    MI_HIP(hipMalloc(&topk_vals, TOPK_MAX * sizeof(float)));
    MI_HIP(hipMalloc(&sel, 64 * sizeof(int)));
    MI_HIP(hipMalloc(&selw, 64 * sizeof(float)));
    MI_HIP(hipMemset(sel, 0, 64 * sizeof(int)));
    MI_HIP(hipMemset(selw, 0, 64 * sizeof(float)));
    MI_HIP(hipMalloc(&gather_ids, 4096 * sizeof(int)));
    MI_HIP(hipMalloc(&gather_out, 4096 * sizeof(float)));
    MI_HIP(hipMalloc(&cell_delta, n_ctx * sizeof(int)));
    MI_HIP(hipMalloc(&move_src, n_ctx * sizeof(int)));
    MI_HIP(hipHostMalloc(&h_tokpos, kTokRing * 4 * sizeof(int)));
    // the top-k kernel writes its result straight into these (coherent, mapped)
    MI_HIP(hipHostMalloc(&h_topk_ids, TOPK_MAX * sizeof(int), hipHostMallocMapped | hipHostMallocCoherent));
    MI_HIP(hipHostMalloc(&h_topk_vals, TOPK_MAX * sizeof(float), hipHostMallocMapped | hipHostMallocCoherent));
    MI_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&d_h_topk_ids), h_topk_ids, 0));
    MI_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&d_h_topk_vals), h_topk_vals, 0));
    MI_HIP(hipHostMalloc(&h_logits, (size_t)hp.n_vocab * sizeof(float)));
    MI_HIP(hipHostMalloc(&h_gather, 4096 * sizeof(float)));
    h_cell_pos.assign(n_ctx, 0);
    sp_ok = sp_setup();
    dev_chain(device).nctx++;
}

Ctx::~Ctx() {
    dev_chain(device).nctx--;
    hipSetDevice(device);
    if (stream) hipStreamSynchronize(stream);
    invalidate_graphs();
    for (auto e : prof_ev) if (e) hipEventDestroy(e);
    for (void* p : {(void*)kcache, (void*)vcache, (void*)kv_scratch, (void*)cell_pos, (void*)tokpos, (void*)x,
                    (void*)q, (void*)attn, (void*)h, (void*)h2, (void*)logits, (void*)cand, (void*)topk_ids,
                    (void*)topk_vals, (void*)sel, (void*)selw, (void*)gather_ids, (void*)gather_out,
                    (void*)cell_delta, (void*)move_src, (void*)part_o, (void*)attn_smax, (void*)attn_scores, (void*)stamps,
                    (void*)attn_xflags, (void*)attn_xmax, (void*)attn_xsum, (void*)step_ctr,
                    (void*)xb, (void*)qb, (void*)attnb, (void*)hb, (void*)tokpos_b, (void*)ub_q, (void*)ub_dT, (void*)ub_bsb, (void*)ub_rope, (void*)ub_part, (void*)ub_spart,
                    (void*)ub_q0, (void*)ub_dT0, (void*)yb, (void*)sel_b, (void*)selw_b, (void*)moe_rows, (void*)moe_pos,
                    (void*)moe_rowsel, (void*)moe_grp, (void*)moe_q, (void*)moe_dT, (void*)moe_bsb,
                    (void*)logits_all, (void*)grows_ids, (void*)grows_out, (void*)sp_mem})
        if (p) hipFree(p);
    for (void* p : {(void*)h_tokpos, (void*)h_topk_ids, (void*)h_topk_vals, (void*)h_logits, (void*)h_gather, (void*)h_grows,
                    (void*)h_tokpos_b, (void*)h_attn_xerr})
        if (p) hipHostFree(p);
    if (stream) hipStreamDestroy(stream);
}

void Ctx::invalidate_graphs() {
    for (int m = 0; m < 2; ++m) {
        for (hipGraphExec_t* g : {&g_full[m], &g_nolog[m], &g_seg[m][0], &g_seg[m][1], &g_seg[m][2]}) {
            if (*g) hipGraphExecDestroy(*g);
            *g = nullptr;
        }
    }
}

long long Ctx::ffn_bytes() const {
    const Layer& L = m->layers[0];
    auto mb = [](const QMat& q) { return (long long)q.rows * q.nb * ((long long)block_bytes(q.type) * 256 / block_elems(q.type)); };
    const HParams& hp = m->hp;
    const long long w = hp.n_expert > 0 ? 2 * (mb(L.gate) + mb(L.up)) : mb(L.gate) + mb(L.up);
    if (sp_ok)   // streaming path: x and the norm weight read (by every workgroup, L2-served), h written
        return w + (long long)hp.n_embd * 4 * 2 + (long long)hp.n_ff * 4;
    const long long act = (long long)hp.n_embd * 4 * 2 + (long long)hp.n_ff * 4 * (hp.n_expert > 0 ? 2 : 1);
    return w + act;   // weights + x and norm weight read + h written
}

// The ops of one llm_build_llama layer for the token in tokpos, as launch parameters handed to
// `gemv` (role: 0 QKV, 1 WO, 2 FFN gate/up, 3 FFN down), `attn` and `router` (the residual
// updated in place).
void Ctx::layer_ops(int l, const LayerBufs& B, const std::function<void(const GemvParams&, int)>& gemv,
                    const std::function<void(const AttnParams&)>& attn,
                    const std::function<void(const RouterParams&)>& router) {
    const HParams& hp = m->hp;
    const Layer& L = m->layers[l];
    __half* kl = kcache + (size_t)l * n_ctx * kv_dim;
    __half* vl = vcache + (size_t)l * n_ctx * kv_dim;
    const float theta_scale = std::pow(hp.rope_base, -2.0f / (float)hp.n_rot);
    const float kq_scale = 1.0f / std::sqrt((float)hp.head_dim);
    GemvParams base;
    std::memset(&base, 0, sizeof(base));
    base.tokpos = tokpos;
    base.cell_pos = cell_pos;
    base.head_dim = hp.head_dim;
    base.kv_dim = kv_dim;
    base.eps = hp.eps;
    base.nslots = 1;
    // ---- Q/K/V projections + RoPE + KV append: one launch per pair of row groups ----
    {
        GemvParams p = base;
        p.pro = PRO_RMSNORM;
        p.x[0] = B.x_in;
        p.norm_w = L.attn_norm;
        p.K = hp.n_embd;
        p.theta_scale = theta_scale;
        p.freq_scale = hp.freq_scale;
        p.n_rot = hp.n_rot;
        p.freq_factors = m->rope_freqs;
        p.kcache = kl;
        p.vcache = vl;
        for (int g = 0; g < L.n_qkv;) {
            p.nseg = 0;
            for (; g < L.n_qkv && p.nseg < GEMV_MAX_SEG; ++g) {
                if (p.nseg == 1 && !gemv_pair_supported(p.seg[0].A.type, L.qkv[g].type)) break;
                GemvSeg& sg = p.seg[p.nseg++];
                sg = seg_of(L.qkv[g], PAIR_ADJ, EPI_QKV, B.q);
                sg.nq = L.qkv_nq[g];
                sg.nk = L.qkv_nk[g];
            }
            gemv(p, 0);
        }
    }
    // ---- attention ----
    {
        AttnParams a{B.q, kl, vl, tokpos, cell_pos, attn_scores, attn_smax, B.po, hp.n_head, hp.n_head_kv, hp.head_dim,
                     kv_dim, (int)n_ctx, kq_scale};
        a.fused = attn_fused;
        a.xflags = attn_xflags;   // contexts past ATTN_SHORT: one launch (attn_long_kernel)
        a.xmax = attn_xmax;
        a.xsum = attn_xsum;
        a.step = step_ctr;
        a.layer = l;
        a.n_layer = hp.n_layer;
        a.xerr = d_attn_xerr;
        a.long_share = dev_chain(device).nctx.load();
        a.long_off = attn_long_off ? 1 : 0;
        attn(a);
    }
    // ---- output projection + residual (prologue: the attention splits combined) ----
    {
        GemvParams p = base;
        p.pro = PRO_ATTN;
        p.attn = AttnPartials{B.po, hp.n_head, hp.head_dim};
        p.attn_nsplit = attn_fused ? 1 : 0;   // the split graph reads the count from the cell count
        p.K = hp.n_embd;
        p.nseg = 1;
        p.seg[0] = seg_of(L.wo, PAIR_ADJ, EPI_ADD, B.xa);
        p.seg[0].resid = B.x_in;
        gemv(p, 1);
    }
    if (hp.n_expert > 0) {
        RouterParams rp{B.xa, L.ffn_norm, hp.eps, L.router, hp.n_embd, hp.n_expert, hp.n_expert_used, sel, selw, 0};
        router(rp);
    }
    // ---- FFN gate/up + SwiGLU ----
    {
        GemvParams p = base;
        p.pro = PRO_RMSNORM;
        p.x[0] = B.xa;
        p.norm_w = L.ffn_norm;
        p.K = hp.n_embd;
        const int nsl = hp.n_expert > 0 ? 2 : 1;
        if (hp.n_expert > 0) {   // expert ids/weights: only MoE launches wait for them
            p.sel = sel;
            p.selw = selw;
        }
        p.nseg = nsl;
        for (int k = 0; k < nsl; ++k) {
            p.seg[k] = seg_of(L.gate, PAIR_AB, EPI_SWIGLU, k == 0 ? B.h : B.h2);
            p.seg[k].B = L.up;
            if (hp.n_expert > 0) p.seg[k].expA = p.seg[k].expB = k;
        }
        gemv(p, 2);
    }
    // ---- FFN down + residual ----
    {
        GemvParams p = base;
        p.pro = PRO_PLAIN;
        p.x[0] = B.h;
        p.K = hp.n_ff;
        p.nseg = 1;
        if (hp.n_expert > 0) {
            p.sel = sel;
            p.selw = selw;
            p.nslots = 2;
            p.x[1] = B.h2;
            p.seg[0] = seg_of(L.down, PAIR_AB, EPI_MOE_DOWN, B.xf);
            p.seg[0].expA = 0;
            p.seg[0].expB = 1;
            p.seg[0].actB = 1;
        } else {
            p.seg[0] = seg_of(L.down, PAIR_ADJ, EPI_ADD, B.xf);
        }
        p.seg[0].resid = B.xa;
        gemv(p, 3);
    }
}

namespace {
// activation formats a set of matrices reads: bit 0 Q8_K (k-quants), bit 1 Q8_0
int act_fmt(std::initializer_list<int> types) {
    int f = 0;
    for (int t : types) f |= t == T_Q8_0 ? 2 : 1;
    return f;
}
}  // namespace

// The streaming decode step's buffers (dense LLaMA; DESIGN.md §4 "dgemv"), and whether every
// launch of the step has a compiled variant (GPT-2 keeps the gemv_kernel graph; MoE experts run on it).
bool Ctx::sp_setup() {
    const HParams& hp = m->hp;
    if (hp.arch != ARCH_LLAMA) return false;
    const bool moe = hp.n_expert > 0;   // MoE: the attention half streams, the experts keep gemv_kernel
    if (hp.n_embd % 256 || hp.n_ff % 256 || hp.n_head * hp.head_dim != hp.n_embd) return false;
    if (!attn_quant_supported(hp.n_head, hp.n_head_kv, hp.head_dim)) return false;
    const int nl = hp.n_layer;
    sp.assign(nl, SpLayer{});
    sp_fH = act_fmt({m->output.type});
    size_t act_max = 0;
    for (int l = 0; l < nl; ++l) {
        const Layer& L = m->layers[l];
        SpLayer& b = sp[l];
        b.fA = 0;
        for (int g = 0; g < L.n_qkv; ++g) b.fA |= act_fmt({L.qkv[g].type});
        b.fB = act_fmt({L.wo.type});
        b.fC = act_fmt({L.gate.type, L.up.type});
        b.fD = act_fmt({L.down.type});
        act_max = std::max(act_max, dv_act_bytes(hp.n_embd, b.fB & 1, b.fB >> 1));
    }
    // every launch must have a variant: the step's parameter checks, dry
    bool ok = true;
    for (int l = 0; l < nl && ok; ++l) {
        const Layer& L = m->layers[l];
        GemvParams p;
        std::memset(&p, 0, sizeof(p));
        p.K = hp.n_embd;
        p.act_in = reinterpret_cast<const char*>(x);   // (any non-null pointer: the checks only)
        p.act_q8k = sp[l].fA & 1;
        p.act_q80 = sp[l].fA >> 1;
        for (int g = 0; g < L.n_qkv && ok;) {
            p.nseg = 0;
            for (; g < L.n_qkv && p.nseg < GEMV_MAX_SEG; ++g) {
                if (p.nseg == 1 && !gemv_pair_supported(p.seg[0].A.type, L.qkv[g].type)) break;
                p.seg[p.nseg++] = seg_of(L.qkv[g], PAIR_ADJ, EPI_QKV, q);
            }
            ok = dgemv_supported(p);
        }
        GemvParams w = p;
        w.nseg = 1;
        w.seg[0] = seg_of(L.wo, PAIR_ADJ, EPI_ADD, x);
        w.act_q8k = sp[l].fB & 1;
        w.act_q80 = sp[l].fB >> 1;
        ok = ok && dgemv_supported(w);
        if (moe) continue;
        GemvParams gu = p;
        gu.nseg = 1;
        gu.seg[0] = seg_of(L.gate, PAIR_AB, EPI_SWIGLU, h);
        gu.seg[0].B = L.up;
        gu.act_q8k = sp[l].fC & 1;
        gu.act_q80 = sp[l].fC >> 1;
        ok = ok && L.gate.type == L.up.type && dgemv_supported(gu);
        GemvParams d = p;
        d.K = hp.n_ff;
        d.nseg = 1;
        d.seg[0] = seg_of(L.down, PAIR_ADJ, EPI_ADD, x);
        d.act_q8k = sp[l].fD & 1;
        d.act_q80 = sp[l].fD >> 1;
        ok = ok && dgemv_supported(d);
    }
    GemvParams hd;
    std::memset(&hd, 0, sizeof(hd));
    hd.K = hp.n_embd;
    hd.act_in = reinterpret_cast<const char*>(x);
    hd.nseg = 1;
    hd.seg[0] = seg_of(m->output, PAIR_ADJ, EPI_STORE, logits);
    hd.act_q8k = sp_fH & 1;
    hd.act_q80 = sp_fH >> 1;
    ok = ok && dgemv_supported(hd);
    if (!ok) {
        sp.clear();
        return false;
    }
    size_t act_n = 0, act_f = 0;
    for (int l = 0; l < nl; ++l) {
        const SpLayer& b = sp[l];
        for (int f : {b.fA, b.fB, b.fC}) act_n = std::max(act_n, dv_act_bytes(hp.n_embd, f & 1, f >> 1));
        act_f = std::max(act_f, dv_act_bytes(hp.n_ff, b.fD & 1, b.fD >> 1));
    }
    act_n = std::max(act_n, dv_act_bytes(hp.n_embd, sp_fH & 1, sp_fH >> 1));
    act_n = (act_n + 255) / 256 * 256;
    act_f = (act_f + 255) / 256 * 256;
    MI_HIP(hipSetDevice(device));
    MI_HIP(hipMalloc(&sp_mem, 4 * act_n + act_f));
    MI_HIP(hipMemset(sp_mem, 0, 4 * act_n + act_f));
    sp_act[0] = sp_mem;
    sp_act[1] = sp_mem + act_n;
    sp_act[2] = sp_mem + 2 * act_n;
    sp_act[4] = sp_mem + 3 * act_n;
    sp_act[3] = sp_mem + 4 * act_n;
    return true;
}

// One batch-1 decode step on the streaming kernels (any context length): the embedding, per layer
// dv_quant(rms_norm(x) * attn_norm) -> QKV -> attention (its output also quantised; past ATTN_SHORT
// cells the split attention + attn_combine_quant) -> WO + residual -> dv_quant(rms_norm
// * ffn_norm) -> gate/up -> dv_quant(h) (small models: inside the down launch) -> down + residual,
// then the output head and the top-k.
// Profiling segments as enqueue_step's (the gate/up launch of prof_layer carries the event pair).
void Ctx::enqueue_step_sp(bool with_logits) {
    // The FFN down launch quantises h in every workgroup itself (no dv_quant launch before it) when
    // that redundant work -- n_ff elements in each of n_embd / 8 workgroups -- is small: one launch
    // fewer per layer wins for TinyLlama (1398-1409 vs 1341-1342 tok/s), loses 1 % for 7B
    // (profiles/r06_hq_ab.txt).
    const HParams& hp = m->hp;
    const bool hq_down = (long long)hp.n_ff * hp.n_embd <= (1LL << 24);
    // The same rule for the normed inputs of Q/K/V and gate/up (dense models): their workgroups
    // build rms_norm(x) * norm_w and quantise it themselves, bit-identical to dv_quant_kernel. That
    // removes two more launches per layer: TinyLlama 1407-1412 -> 1639-1653 tok/s, but 7B 637-643 ->
    // 579-589 and Llama-3-8B 511 -> 470-480 (profiles/r06_nq_ab.txt).
    const bool nq_in = hq_down && hp.n_expert == 0 && hp.n_embd <= 8192;
    const bool moe = hp.n_expert > 0;
    int seg = 0;
    auto on = [&]() { return seg_filter < 0 || seg_filter == seg; };
    const float theta_scale = std::pow(hp.rope_base, -2.0f / (float)hp.n_rot);
    const float kq_scale = 1.0f / std::sqrt((float)hp.head_dim);
    auto act = [&](int role, int fmt, int K, const float* norm_w) {
        return ActOut{K, fmt & 1, fmt >> 1, sp_act[role], norm_w, hp.eps};
    };
    if (on()) {
        EmbedParams ep{m->tok_embd, tokpos, x, hp.n_embd, m->pos_embd, 0, step_ctr};
        launch_embed(ep, stream);
        if (!nq_in) launch_dv_quant(x, act(0, sp[0].fA, hp.n_embd, m->layers[0].attn_norm), stream);
    }
    for (int l = 0; l < hp.n_layer; ++l) {
        const Layer& L = m->layers[l];
        const SpLayer& b = sp[l];
        __half* kl = kcache + (size_t)l * n_ctx * kv_dim;
        __half* vl = vcache + (size_t)l * n_ctx * kv_dim;
        GemvParams base;
        std::memset(&base, 0, sizeof(base));
        base.tokpos = tokpos;
        base.cell_pos = cell_pos;
        base.head_dim = hp.head_dim;
        base.kv_dim = kv_dim;
        base.nslots = 1;
        base.K = hp.n_embd;
        {   // Q/K/V + RoPE + KV append
            GemvParams p = base;
            p.act_in = nq_in ? nullptr : sp_act[0];
            p.x[0] = nq_in ? x : nullptr;
            p.norm_w = nq_in ? L.attn_norm : nullptr;
            p.eps = hp.eps;
            p.act_q8k = b.fA & 1;
            p.act_q80 = b.fA >> 1;
            p.theta_scale = theta_scale;
            p.freq_scale = hp.freq_scale;
            p.n_rot = hp.n_rot;
            p.freq_factors = m->rope_freqs;
            p.kcache = kl;
            p.vcache = vl;
            for (int g = 0; g < L.n_qkv;) {
                p.nseg = 0;
                for (; g < L.n_qkv && p.nseg < GEMV_MAX_SEG; ++g) {
                    if (p.nseg == 1 && !gemv_pair_supported(p.seg[0].A.type, L.qkv[g].type)) break;
                    GemvSeg& sg = p.seg[p.nseg++];
                    sg = seg_of(L.qkv[g], PAIR_ADJ, EPI_QKV, q);
                    sg.nq = L.qkv_nq[g];
                    sg.nk = L.qkv_nk[g];
                }
                if (on()) launch_dgemv(p, stream);
            }
        }
        {   // attention, its output quantised for WO: <= ATTN_SHORT cells one fused launch (which
            // quantises); past that the split launch(es) of the r04 step, then the splits summed in
            // split order and quantised (attn_combine_quant_kernel)
            AttnParams a{q, kl, vl, tokpos, cell_pos, attn_scores, attn_smax, part_o, hp.n_head, hp.n_head_kv,
                         hp.head_dim, kv_dim, (int)n_ctx, kq_scale};
            if (attn_fused) {
                a.fused = 1;
                a.act_out = act(1, b.fB, hp.n_embd, nullptr);
                if (on()) launch_attn(a, stream);
            } else {
                a.fused = 0;
                a.xflags = attn_xflags;
                a.xmax = attn_xmax;
                a.xsum = attn_xsum;
                a.step = step_ctr;
                a.layer = l;
                a.n_layer = hp.n_layer;
                a.xerr = d_attn_xerr;
                a.long_share = dev_chain(device).nctx.load();
                a.long_off = attn_long_off ? 1 : 0;
                if (on()) {
                    launch_attn(a, stream);
                    launch_attn_combine_quant(AttnPartials{part_o, hp.n_head, hp.head_dim}, tokpos,
                                              act(1, b.fB, hp.n_embd, nullptr), stream);
                }
            }
        }
        {   // output projection + residual (in place), then rms_norm(x) * ffn_norm quantised
            GemvParams p = base;
            p.act_in = sp_act[1];
            p.act_q8k = b.fB & 1;
            p.act_q80 = b.fB >> 1;
            p.nseg = 1;
            p.seg[0] = seg_of(L.wo, PAIR_ADJ, EPI_ADD, x);
            p.seg[0].resid = x;
            if (on()) {
                launch_dgemv(p, stream);
                if (!moe && !nq_in) launch_dv_quant(x, act(2, b.fC, hp.n_embd, L.ffn_norm), stream);
            }
        }
        if (moe) {   // the routed experts on the r04 step's kernels (layer_ops' MoE FFN), x in place
            GemvParams gb = base;
            gb.eps = hp.eps;
            RouterParams rp{x, L.ffn_norm, hp.eps, L.router, hp.n_embd, hp.n_expert, hp.n_expert_used, sel, selw, 0};
            if (on()) launch_router(rp, stream);
            GemvParams p = gb;
            p.pro = PRO_RMSNORM;
            p.x[0] = x;
            p.norm_w = L.ffn_norm;
            p.sel = sel;
            p.selw = selw;
            p.nseg = 2;
            for (int k = 0; k < 2; ++k) {
                p.seg[k] = seg_of(L.gate, PAIR_AB, EPI_SWIGLU, k == 0 ? h : h2);
                p.seg[k].B = L.up;
                p.seg[k].expA = p.seg[k].expB = k;
            }
            if (l == prof_layer) seg = 1;
            const bool timed = l == prof_layer && seg_filter == 1;
            if (on()) launch_gemv(p, stream, timed ? prof_ev[0] : nullptr, timed ? prof_ev[1] : nullptr);
            if (l == prof_layer) seg = 2;
            GemvParams d = gb;
            d.pro = PRO_PLAIN;
            d.x[0] = h;
            d.x[1] = h2;
            d.nslots = 2;
            d.K = hp.n_ff;
            d.sel = sel;
            d.selw = selw;
            d.nseg = 1;
            d.seg[0] = seg_of(L.down, PAIR_AB, EPI_MOE_DOWN, x);
            d.seg[0].expA = 0;
            d.seg[0].expB = 1;
            d.seg[0].actB = 1;
            d.seg[0].resid = x;
            if (on()) {
                launch_gemv(d, stream);
                if (l + 1 < hp.n_layer)
                    launch_dv_quant(x, act(0, sp[l + 1].fA, hp.n_embd, m->layers[l + 1].attn_norm), stream);
                else if (with_logits)
                    launch_dv_quant(x, act(4, sp_fH, hp.n_embd, m->output_norm), stream);
            }
            continue;
        }
        {   // FFN gate/up + SwiGLU, then h quantised
            GemvParams p = base;
            p.act_in = nq_in ? nullptr : sp_act[2];
            p.x[0] = nq_in ? x : nullptr;
            p.norm_w = nq_in ? L.ffn_norm : nullptr;
            p.eps = hp.eps;
            p.act_q8k = b.fC & 1;
            p.act_q80 = b.fC >> 1;
            p.nseg = 1;
            p.seg[0] = seg_of(L.gate, PAIR_AB, EPI_SWIGLU, h);
            p.seg[0].B = L.up;
            if (l == prof_layer) seg = 1;
            const bool timed = l == prof_layer && seg_filter == 1;
            if (on()) launch_dgemv(p, stream, timed ? prof_ev[0] : nullptr, timed ? prof_ev[1] : nullptr);
            if (l == prof_layer) seg = 2;
            if (on() && !hq_down) launch_dv_quant(h, act(3, b.fD, hp.n_ff, nullptr), stream);
        }
        {   // FFN down + residual (in place), then the next layer's (or the output head's) input quantised
            GemvParams p = base;
            p.act_in = hq_down ? nullptr : sp_act[3];
            p.x[0] = h;
            p.K = hp.n_ff;
            p.act_q8k = b.fD & 1;
            p.act_q80 = b.fD >> 1;
            p.nseg = 1;
            p.seg[0] = seg_of(L.down, PAIR_ADJ, EPI_ADD, x);
            p.seg[0].resid = x;
            const bool next = (l + 1 < hp.n_layer && !nq_in) || (l + 1 == hp.n_layer && with_logits);
            const ActOut nx = l + 1 < hp.n_layer ? act(0, sp[l + 1].fA, hp.n_embd, m->layers[l + 1].attn_norm)
                                                 : act(4, sp_fH, hp.n_embd, m->output_norm);
            if (on()) {
                launch_dgemv(p, stream);
                if (next) launch_dv_quant(x, nx, stream);
            }
        }
    }
    if (with_logits && on()) {   // the output head, the top-k
        GemvParams p;
        std::memset(&p, 0, sizeof(p));
        p.K = hp.n_embd;
        p.act_in = sp_act[4];
        p.act_q8k = sp_fH & 1;
        p.act_q80 = sp_fH >> 1;
        p.nseg = 1;
        p.seg[0] = seg_of(m->output, PAIR_ADJ, EPI_STORE, logits);
        launch_dgemv(p, stream);
        TopkParams tp{logits, hp.n_vocab, cand, topk_ids, topk_vals, d_h_topk_ids, d_h_topk_vals};
        launch_topk(tp, stream);
    }
}

// One decode step for the token in tokpos (batch 1): the llm_build_llama graph.
// With seg_filter >= 0 only the ops of that profiling segment are enqueued
// (0: up to layer prof_layer's FFN gate/up, 1: that launch, 2: the rest).
void Ctx::enqueue_step(bool with_logits) {
    const HParams& hp = m->hp;
    if (sp_ok) {   // dense LLaMA at any context (past 512 cells: 474-481 vs 429-435 tok/s at 3968, r06)
        enqueue_step_sp(with_logits);
        return;
    }
    int seg = 0;
    int n_launch = 0;   // diagnostic stamps (MI_STAMPS builds only): one slab per launch
    auto stamp = [&]() -> unsigned long long* {
        if (!stamps || n_launch >= kStampLaunches) return nullptr;
        return stamps + (size_t)(n_launch++) * kStampWgs * 8;
    };
    auto on = [&]() { return seg_filter < 0 || seg_filter == seg; };
    EmbedParams ep{m->tok_embd, tokpos, x, hp.n_embd, m->pos_embd, hp.arch == ARCH_GPT2 ? 1 : 0, step_ctr};
    if (on()) launch_embed(ep, stream);
    const float kq_scale = 1.0f / std::sqrt((float)hp.head_dim);
    for (int l = 0; l < hp.n_layer; ++l) {
        if (hp.arch == ARCH_GPT2) {   // llm_build_gpt2: LayerNorm, biases, no RoPE, GELU MLP
            GemvParams base;
            std::memset(&base, 0, sizeof(base));
            base.tokpos = tokpos;
            base.cell_pos = cell_pos;
            base.head_dim = hp.head_dim;
            base.kv_dim = kv_dim;
            base.eps = hp.eps;
            base.nslots = 1;
            enqueue_layer_gpt2(l, base, kcache + (size_t)l * n_ctx * kv_dim, vcache + (size_t)l * n_ctx * kv_dim,
                               kq_scale, stamp);
            continue;
        }
        const LayerBufs B{x, q, part_o, x, h, h2, x};
        layer_ops(
            l, B,
            [&](const GemvParams& p0, int role) {
                GemvParams p = p0;
                p.stamps = stamp();
                if (role != 2) {
                    if (on()) launch_gemv(p, stream);
                    return;
                }
                if (l == prof_layer) seg = 1;
                // the profiled launch (segment 1, always eager) carries the event pair
                const bool timed = l == prof_layer && seg_filter == 1;
                if (on()) launch_gemv(p, stream, timed ? prof_ev[0] : nullptr, timed ? prof_ev[1] : nullptr);
                if (l == prof_layer) seg = 2;
            },
            [&](const AttnParams& a0) {
                AttnParams a = a0;
                a.stamps = stamp();
                a.stamps2 = stamp();
                if (on()) launch_attn(a, stream);
            },
            [&](const RouterParams& rp) {
                if (on()) launch_router(rp, stream);
            });
    }
    if (with_logits && on()) enqueue_output(x, stamp());
}

// One GPT-2 block (llm_build_gpt2, src/llama-model.cpp b5187) of the decode step:
//   cur = LayerNorm(x)*attn_norm + attn_norm_b -> wqkv + bqkv -> Q / K / V (no RoPE) -> KV append
//   attention -> wo + bo + x (residual);  LayerNorm(x)*ffn_norm + ffn_norm_b -> up + bup -> GELU
//   -> down + bdown + x
void Ctx::enqueue_layer_gpt2(int l, const GemvParams& base, __half* kl, __half* vl, float kq_scale,
                             const std::function<unsigned long long*()>& stamp) {
    const HParams& hp = m->hp;
    const Layer& L = m->layers[l];
    auto on = [&]() { return seg_filter < 0; };
    {
        GemvParams p = base;
        p.pro = PRO_LAYERNORM;
        p.x[0] = x;
        p.norm_w = L.attn_norm;
        p.norm_b = L.attn_norm_b;
        p.K = hp.n_embd;
        p.n_rot = 0;
        p.kcache = kl;
        p.vcache = vl;
        p.nseg = 1;
        p.seg[0] = seg_of(L.qkv[0], PAIR_ADJ, EPI_QKV, q);
        p.seg[0].nq = L.qkv_nq[0];
        p.seg[0].nk = L.qkv_nk[0];
        p.seg[0].bias = L.bqkv;
        p.stamps = stamp();
        if (on()) launch_gemv(p, stream);
    }
    {
        AttnParams a{q, kl, vl, tokpos, cell_pos, attn_scores, attn_smax, part_o, hp.n_head, hp.n_head_kv, hp.head_dim,
                     kv_dim, (int)n_ctx, kq_scale};
        a.fused = attn_fused;
        a.stamps = stamp();
        a.stamps2 = stamp();
        if (on()) launch_attn(a, stream);
    }
    {
        GemvParams p = base;
        p.pro = PRO_ATTN;
        p.attn = AttnPartials{part_o, hp.n_head, hp.head_dim};
        p.attn_nsplit = attn_fused ? 1 : 0;
        p.K = hp.n_embd;
        p.nseg = 1;
        p.seg[0] = seg_of(L.wo, PAIR_ADJ, EPI_ADD, x);
        p.seg[0].resid = x;
        p.seg[0].bias = L.bo;
        p.stamps = stamp();
        if (on()) launch_gemv(p, stream);
    }
    {
        GemvParams p = base;
        p.pro = PRO_LAYERNORM;
        p.x[0] = x;
        p.norm_w = L.ffn_norm;
        p.norm_b = L.ffn_norm_b;
        p.K = hp.n_embd;
        p.gelu_tab = m->gelu_tab;
        p.nseg = 1;
        p.seg[0] = seg_of(L.up, PAIR_ADJ, EPI_GELU, h);
        p.seg[0].bias = L.bup;
        p.stamps = stamp();
        if (on()) launch_gemv(p, stream);
    }
    {
        GemvParams p = base;
        p.pro = PRO_PLAIN;
        p.x[0] = h;
        p.K = hp.n_ff;
        p.nseg = 1;
        p.seg[0] = seg_of(L.down, PAIR_ADJ, EPI_ADD, x);
        p.seg[0].resid = x;
        p.seg[0].bias = L.bdown;
        p.stamps = stamp();
        if (on()) launch_gemv(p, stream);
    }
}

// final RMSNorm (GPT-2: LayerNorm) + output head GEMV of one residual row, then the top-k
void Ctx::enqueue_output(const float* xrow, unsigned long long* stamps_slab) {
    const HParams& hp = m->hp;
    GemvParams p;
    std::memset(&p, 0, sizeof(p));
    p.pro = hp.arch == ARCH_GPT2 ? PRO_LAYERNORM : PRO_RMSNORM;
    p.norm_b = m->output_norm_b;
    p.nslots = 1;
    p.x[0] = xrow;
    p.norm_w = m->output_norm;
    p.eps = hp.eps;
    p.K = hp.n_embd;
    p.tokpos = tokpos;
    p.nseg = 1;
    p.seg[0] = seg_of(m->output, PAIR_ADJ, EPI_STORE, logits);
    p.stamps = stamps_slab;
    launch_gemv(p, stream);
    TopkParams tp{logits, hp.n_vocab, cand, topk_ids, topk_vals, d_h_topk_ids, d_h_topk_vals};
    launch_topk(tp, stream);
}

hipGraphExec_t Ctx::build_graph(bool with_logits, int seg) {
    hipGraph_t g = nullptr;
    seg_filter = seg;
    MI_HIP(hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal));
    try {
        enqueue_step(with_logits);
    } catch (...) {
        seg_filter = -1;
        hipStreamEndCapture(stream, &g);
        if (g) hipGraphDestroy(g);
        throw;
    }
    seg_filter = -1;
    MI_HIP(hipStreamEndCapture(stream, &g));
    hipGraphExec_t ex = nullptr;
    MI_HIP(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
    MI_HIP(hipGraphDestroy(g));
    return ex;
}

// Prompt ingestion: n tokens in chunks of GEMM_NT, every weight matrix streamed once per
// chunk (launch_gemm), causal attention of the chunk's tokens (launch_attn_multi), the
// output head for the last token only (llama_batch_get_one: logits of the last token).
void Ctx::decode_batch(const int32_t* tokens, int n) {
    const HParams& hp = m->hp;
    const float theta_scale = std::pow(hp.rope_base, -2.0f / (float)hp.n_rot);
    const float kq_scale = 1.0f / std::sqrt((float)hp.head_dim);
    const int chunk = GEMM_NT;
    // one projection on the v_dot4 GEMM, which quantises its own rows
    auto proj = [&](GemmParams p, const float* x, int x_stride, const float* norm, bool) {
        p.x = x;
        p.x_stride = x_stride;
        p.norm_w = norm;
        p.pro = norm ? PRO_RMSNORM : PRO_PLAIN;
        launch_gemm(p, stream);
    };
    for (int c0 = 0; c0 < n; c0 += chunk) {
        const int nt = std::min(chunk, n - c0);
        const long long slot = tokb_slot++ % kTokbRing;
        if (slot == 0 && tokb_slot > 1) MI_HIP(hipStreamSynchronize(stream));
        int* hpos = h_tokpos_b + slot * kBatchRows * 4;
        for (int t = 0; t < nt; ++t) {
            const int pos = pos_max + 1, cell = n_cells;
            hpos[t * 4 + 0] = tokens[c0 + t];
            hpos[t * 4 + 1] = pos;
            hpos[t * 4 + 2] = cell;
            hpos[t * 4 + 3] = 0;
            h_cell_pos[cell] = pos;
            n_cells++;
            pos_max = pos;
        }
        MI_HIP(hipMemcpyAsync(tokpos_b, hpos, nt * 4 * sizeof(int), hipMemcpyHostToDevice, stream));
        EmbedParams ep{m->tok_embd, tokpos_b, xb, hp.n_embd};
        launch_embed_multi(ep, nt, stream);
        for (int l = 0; l < hp.n_layer; ++l) {
            const Layer& L = m->layers[l];
            __half* kl = kcache + (size_t)l * n_ctx * kv_dim;
            __half* vl = vcache + (size_t)l * n_ctx * kv_dim;
            GemmParams b;
            std::memset(&b, 0, sizeof(b));
            b.ntok = nt;
            b.tokpos = tokpos_b;
            b.cell_pos = cell_pos;
            b.theta_scale = theta_scale;
            b.freq_scale = hp.freq_scale;
            b.head_dim = hp.head_dim;
            b.freq_factors = m->rope_freqs;
            b.kcache = kl;
            b.vcache = vl;
            b.kv_dim = kv_dim;
            b.eps = hp.eps;
            // Q / K / V projections (+ RoPE, KV append)
            const QMat* mats[3] = {&L.wq, &L.wk, &L.wv};
            const int epis[3] = {EPI_ROPE_Q, EPI_ROPE_K, EPI_V};
            for (int i = 0; i < 3; ++i) {
                GemmParams p = b;
                p.A = *mats[i];
                p.pair = PAIR_ADJ;
                p.epi = epis[i];
                p.units = (mats[i]->rows + 1) / 2;
                p.K = hp.n_embd;
                p.out = qb;
                p.out_stride = hp.n_embd;
                p.n_rot = i < 2 ? hp.n_rot : 0;
                proj(p, xb, hp.n_embd, L.attn_norm, i == 0);   // the three share one quantisation
            }
            AttnParams a{qb, kl, vl, tokpos_b, cell_pos, attn_scores, attn_smax, attnb, hp.n_head, hp.n_head_kv,
                         hp.head_dim, kv_dim, (int)n_ctx, kq_scale};
            launch_attn_multi(a, nt, attnb, stream);
            {   // output projection + residual
                GemmParams p = b;
                p.A = L.wo;
                p.pair = PAIR_ADJ;
                p.epi = EPI_ADD;
                p.units = (L.wo.rows + 1) / 2;
                p.K = hp.n_embd;
                p.out = xb;
                p.resid = xb;
                p.out_stride = hp.n_embd;
                proj(p, attnb, hp.n_embd, nullptr, true);
            }
            {   // FFN gate/up + SwiGLU
                GemmParams p = b;
                p.A = L.gate;
                p.B = L.up;
                p.pair = PAIR_AB;
                p.epi = EPI_SWIGLU;
                p.units = L.gate.rows;
                p.K = hp.n_embd;
                p.out = hb;
                p.out_stride = hp.n_ff;
                proj(p, xb, hp.n_embd, L.ffn_norm, true);
            }
            {   // FFN down + residual
                GemmParams p = b;
                p.A = L.down;
                p.pair = PAIR_ADJ;
                p.epi = EPI_ADD;
                p.units = (L.down.rows + 1) / 2;
                p.K = hp.n_ff;
                p.out = xb;
                p.resid = xb;
                p.out_stride = hp.n_embd;
                proj(p, hb, hp.n_ff, nullptr, true);
            }
        }
        if (c0 + nt == n) enqueue_output(xb + (size_t)(nt - 1) * hp.n_embd, nullptr);
    }
    logits_valid = true;
}

// build_moe_ffn (src/llama-graph.cpp, b5187: softmax gating, top-2, weights normalised) over a
// physical batch, all on the device: the router of every token (the decode step's router_kernel),
// the (token, slot) picks grouped by expert (launch_moe_group: tokens ascending within an expert,
// each expert's rows whole 32-row MFMA tiles), one quantisation of every row, ONE grouped mmq32
// launch for the experts' gate/up + SwiGLU and one for their down projections (a workgroup per
// (expert, row tile) over that expert's token tiles), then every token's x += w0*y0 + w1*y1 in
// slot order (launch_moe_combine, the decode GEMV's EPI_MOE_DOWN arithmetic).  No host round trip.
void Ctx::moe_ffn_batch(int l, int nt, const float* pend) {
    const HParams& hp = m->hp;
    const Layer& L = m->layers[l];
    const int U = hp.n_expert_used, E = hp.n_expert;
    RouterParams rp{xb, L.ffn_norm, hp.eps, L.router, hp.n_embd, E, U, sel_b, selw_b, hp.n_embd, pend, nt};
    launch_router_multi(rp, nt, stream);
    const int cap = moe_rows_cap(nt * U, E);
    launch_moe_group(sel_b, nt * U, U, E, moe_grp, moe_rows, moe_rowsel, moe_pos, cap, stream);
    auto act_of = [&](int K, int type) {
        ActQ8 a;
        a.q = moe_q;
        a.dT = moe_dT;
        a.bsb = moe_bsb;
        a.K = K;
        a.ntok = cap;
        a.npad = cap;
        a.q80 = type == T_Q8_0 ? 1 : 0;
        return a;
    };
    GemmParams p;
    std::memset(&p, 0, sizeof(p));
    p.ntok = cap;
    p.tokpos = tokpos_b;
    p.grp = moe_grp;
    p.grp_n = E;
    p.grp_max = nt;
    // gate/up + SwiGLU: rms_norm(x) * ffn_norm of each row's token
    const ActQ8 act = act_of(hp.n_embd, L.gate.type);
    launch_quant_act(xb, hp.n_embd, L.ffn_norm, hp.eps, act, stream, moe_rows);
    p.A = L.gate;
    p.B = L.up;
    p.pair = PAIR_AB;
    p.epi = EPI_SWIGLU;
    p.K = hp.n_embd;
    p.out = hb;
    p.out_stride = hp.n_ff;
    p.grp_stride = L.gate.sw_expert_stride;
    launch_mmq32(p, act, ub_rope, stream);
    // down: every row of the FFN output, stored (weighted and summed by the combine)
    const ActQ8 a2 = act_of(hp.n_ff, L.down.type);
    launch_quant_act(hb, hp.n_ff, nullptr, hp.eps, a2, stream, moe_rowsel);
    GemmParams d = p;
    d.A = L.down;
    std::memset(&d.B, 0, sizeof(d.B));
    d.pair = PAIR_ADJ;
    d.epi = EPI_STORE;
    d.K = hp.n_ff;
    d.out = yb;
    d.out_stride = hp.n_embd;
    d.grp_stride = L.down.sw_expert_stride;
    launch_mmq32(d, a2, ub_rope, stream);
    launch_moe_combine(yb, moe_pos, selw_b, xb, nt, hp.n_embd, stream);
}

// The same build_moe_ffn over a short batch (<= MMQS_MAX tokens; x already holds the residual) on
// the grouped streaming GEMM: router, grouping, one quantisation of every MoE row, the experts'
// gate/up pair parts (launch_mmqs_grouped: workgroups per (row tile, K-part, expert, 32-row tile),
// each expert's matrix streamed once for the rows routed to it), SwiGLU of the parts quantised for
// down, down's parts, their sum per row, then every token's x += w0*y0 + w1*y1 in slot order.
void Ctx::moe_ffn_short(int l, int nt) {
    const HParams& hp = m->hp;
    const Layer& L = m->layers[l];
    const int U = hp.n_expert_used, E = hp.n_expert;
    RouterParams rp{xb, L.ffn_norm, hp.eps, L.router, hp.n_embd, E, U, sel_b, selw_b, hp.n_embd, nullptr, nt};
    launch_router_multi(rp, nt, stream);
    const int cap = moe_rows_cap(nt * U, E);
    launch_moe_group(sel_b, nt * U, U, E, moe_grp, moe_rows, moe_rowsel, moe_pos, cap, stream);
    auto act_of = [&](int K) {
        ActQ8 a;
        a.q = moe_q;
        a.dT = moe_dT;
        a.bsb = moe_bsb;
        a.K = K;
        a.ntok = cap;
        a.npad = cap;
        a.q80 = 0;
        return a;
    };
    const ActQ8 act = act_of(hp.n_embd);
    launch_quant_act(xb, hp.n_embd, L.ffn_norm, hp.eps, act, stream, moe_rows);
    // an expert receives each token at most once: at most nt rows
    const int kg = launch_mmqs_grouped(L.gate, true, hp.n_ff, act, ub_spart, 2 * hp.n_ff, moe_grp, E, nt, stream);
    const ActQ8 a2 = act_of(hp.n_ff);
    launch_quant_act(nullptr, hp.n_ff, nullptr, hp.eps, a2, stream, moe_rowsel, ub_spart, kg, 1);
    const int kd = launch_mmqs_grouped(L.down, false, 0, a2, ub_spart, hp.n_embd, moe_grp, E, nt, stream);
    launch_part_sum(ub_spart, kd, cap, hp.n_embd, hp.n_embd, nullptr, 0, yb, hp.n_embd, stream);
    launch_moe_combine(yb, moe_pos, selw_b, xb, nt, hp.n_embd, stream);
}

ActQ8 Ctx::ub_act(int K, int ntok, int type) const {
    const bool q80 = type == T_Q8_0;
    const bool second = q80 && !ub_q80 && ub_q0;   // the Q8_0 set of a mixed model
    ActQ8 a;
    a.q = second ? ub_q0 : ub_q;
    a.dT = second ? ub_dT0 : ub_dT;
    a.bsb = ub_bsb;
    a.K = K;
    a.ntok = ntok;
    a.npad = (ntok + 31) / 32 * 32;
    a.q80 = q80 ? 1 : 0;
    return a;
}

// Prompt ingestion / batched verification in physical batches of up to UB_MAX tokens on the
// int8-MFMA GEMM (mmq.hip): per layer every weight matrix is streamed once per batch; each
// activation is quantised to Q8_K once (RMSNorm fused) and shared by the matrices that read it.
// `all`: the output head runs over every token (rows of logits_all), else over the last one.
void Ctx::decode_ubatch(const int32_t* tokens, int n, bool all) {
    const HParams& hp = m->hp;
    const float theta_scale = std::pow(hp.rope_base, -2.0f / (float)hp.n_rot);
    const float kq_scale = 1.0f / std::sqrt((float)hp.head_dim);
    for (int c0 = 0; c0 < n; c0 += UB_MAX) {
        const int nt = std::min(UB_MAX, n - c0);
        const long long slot = tokb_slot++ % kTokbRing;
        if (slot == 0 && tokb_slot > 1) MI_HIP(hipStreamSynchronize(stream));
        int* hpos = h_tokpos_b + slot * kBatchRows * 4;
        for (int t = 0; t < nt; ++t) {
            const int pos = pos_max + 1, cell = n_cells;
            hpos[t * 4 + 0] = tokens[c0 + t];
            hpos[t * 4 + 1] = pos;
            hpos[t * 4 + 2] = cell;
            hpos[t * 4 + 3] = 0;
            h_cell_pos[cell] = pos;
            n_cells++;
            pos_max = pos;
        }
        MI_HIP(hipMemcpyAsync(tokpos_b, hpos, nt * 4 * sizeof(int), hipMemcpyHostToDevice, stream));
        if (mmqs_max > 0 && nt <= mmqs_max && short_ok()) {   // a short batch (its launches captured as a
            // hipGraph measured no faster: the GPU, not the enqueue, sets the pace)
            enqueue_ubatch_short(nt, all, c0, c0 + nt == n);
            continue;
        }
        EmbedParams ep{m->tok_embd, tokpos_b, xb, hp.n_embd};
        launch_embed_multi(ep, nt, stream);
        launch_rope_table(tokpos_b, nt, hp.n_rot, theta_scale, hp.freq_scale, m->rope_freqs, ub_rope, stream);
        const float* pend = nullptr;   // split-K partials not yet added into xb (the next quant_act does)
        // split-K parts of the residual GEMMs: 4 for short batches of dense models (verification
        // of tens of tokens: more workgroups, a quarter of the superblock steps each; 4 x nt rows
        // fit the 2 x UB_MAX partials buffer), else 2 (the MoE router adds 2)
        const int ks = hp_dense() && nt <= 64 ? 4 : 2;   // 4 x 64 rows fit the 2 x UB_MAX partials buffer
        for (int l = 0; l < hp.n_layer; ++l) {
            const Layer& L = m->layers[l];
            __half* kl = kcache + (size_t)l * n_ctx * kv_dim;
            __half* vl = vcache + (size_t)l * n_ctx * kv_dim;
            GemmParams b;
            std::memset(&b, 0, sizeof(b));
            b.ntok = nt;
            b.tokpos = tokpos_b;
            b.cell_pos = cell_pos;
            b.head_dim = hp.head_dim;
            b.n_rot = hp.n_rot;
            b.kcache = kl;
            b.vcache = vl;
            b.kv_dim = kv_dim;
            b.K = hp.n_embd;
            b.out_stride = hp.n_embd;
            // Q / K / V (+ RoPE, KV append) over one quantisation of rms_norm(x) * attn_norm per
            // activation format the three matrices read
            const QMat* mats[3] = {&L.wq, &L.wk, &L.wv};
            const int epis[3] = {EPI_ROPE_Q, EPI_ROPE_K, EPI_V};
            for (int f = 0; f < 2; ++f) {
                bool need = false;
                for (const QMat* q : mats) need = need || (q->type == T_Q8_0) == (f == 1);
                if (need) {
                    launch_quant_act(xb, hp.n_embd, L.attn_norm, hp.eps, ub_act(hp.n_embd, nt, f ? T_Q8_0 : T_Q4_K), stream,
                                     nullptr, pend, ks);
                    pend = nullptr;
                }
            }
            // the matrices of one type in one launch (7B: Q/K/V, or Q/K plus a Q6_K V)
            for (int i = 0; i < 3; ++i) {
                bool first = true;
                for (int j = 0; j < i; ++j) first = first && mats[j]->type != mats[i]->type;
                if (!first) continue;
                GemmParams ps[3];
                int n = 0;
                for (int j = i; j < 3; ++j) {
                    if (mats[j]->type != mats[i]->type) continue;
                    ps[n] = b;
                    ps[n].A = *mats[j];
                    ps[n].pair = PAIR_ADJ;
                    ps[n].epi = epis[j];
                    ps[n].out = qb;
                    ++n;
                }
                launch_mmq32_multi(ps, n, ub_act(hp.n_embd, nt, mats[i]->type), ub_rope, stream);
            }
            AttnParams a{qb, kl, vl, tokpos_b, cell_pos, attn_scores, attn_smax, attnb, hp.n_head, hp.n_head_kv,
                         hp.head_dim, kv_dim, (int)n_ctx, kq_scale};
            if (attn_mfma) launch_attn_mfma(a, nt, attnb, stream);
            else launch_attn_multi(a, nt, attnb, stream);
            {   // output projection + residual
                const ActQ8 act = ub_act(hp.n_embd, nt, L.wo.type);
                launch_quant_act(attnb, hp.n_embd, nullptr, hp.eps, act, stream);
                GemmParams p = b;
                p.A = L.wo;
                p.pair = PAIR_ADJ;
                p.epi = EPI_ADD;
                p.out = xb;
                p.resid = xb;
                if (ub_part && L.wo.nb >= ks) {   // parts of K; the FFN's quant_act adds them
                    p.ksplit = ks;
                    p.part = ub_part;
                    pend = ub_part;
                }
                launch_mmq32(p, act, ub_rope, stream);
            }
            if (hp.n_expert > 0) {   // routed experts (build_moe_ffn) + residual
                moe_ffn_batch(l, nt, pend);
                pend = nullptr;
                continue;
            }
            {   // FFN gate/up + SwiGLU
                const ActQ8 act = ub_act(hp.n_embd, nt, L.gate.type);
                launch_quant_act(xb, hp.n_embd, L.ffn_norm, hp.eps, act, stream, nullptr, pend, ks);
                pend = nullptr;
                GemmParams p = b;
                p.A = L.gate;
                p.B = L.up;
                p.pair = PAIR_AB;
                p.epi = EPI_SWIGLU;
                p.out = hb;
                p.out_stride = hp.n_ff;
                launch_mmq32(p, act, ub_rope, stream);
            }
            {   // FFN down + residual
                const ActQ8 act = ub_act(hp.n_ff, nt, L.down.type);
                launch_quant_act(hb, hp.n_ff, nullptr, hp.eps, act, stream);
                GemmParams p = b;
                p.A = L.down;
                p.pair = PAIR_ADJ;
                p.epi = EPI_ADD;
                p.K = hp.n_ff;
                p.out = xb;
                p.resid = xb;
                if (ub_part && L.down.nb >= ks && l + 1 < hp.n_layer) {   // the next layer's quant_act adds them
                    p.ksplit = ks;
                    p.part = ub_part;
                    pend = ub_part;
                }
                launch_mmq32(p, act, ub_rope, stream);
            }
        }
        if (all) {   // final norm + output head over every token of the batch
            const ActQ8 a_out = ub_act(hp.n_embd, nt, m->output.type);   // the head's own activation format
            launch_quant_act(xb, hp.n_embd, m->output_norm, hp.eps, a_out, stream);
            GemmParams p;
            std::memset(&p, 0, sizeof(p));
            p.A = m->output;
            p.pair = PAIR_ADJ;
            p.epi = EPI_STORE;
            p.K = hp.n_embd;
            p.ntok = nt;
            p.tokpos = tokpos_b;
            p.out = logits_all + (size_t)c0 * hp.n_vocab;
            p.out_stride = hp.n_vocab;
            launch_mmq32(p, a_out, ub_rope, stream);
            if (c0 + nt == n) {   // the last row also feeds `logits` and the mapped top-k
                MI_HIP(hipMemcpyAsync(logits, logits_all + (size_t)(n - 1) * hp.n_vocab, (size_t)hp.n_vocab * sizeof(float),
                                      hipMemcpyDeviceToDevice, stream));
                TopkParams tp{logits, hp.n_vocab, cand, topk_ids, topk_vals, d_h_topk_ids, d_h_topk_vals};
                launch_topk(tp, stream);
            }
        } else if (c0 + nt == n) {
            enqueue_output(xb + (size_t)(nt - 1) * hp.n_embd, nullptr);
        }
    }
    logits_valid = true;
}

// One short physical batch (tokens uploaded to tokpos_b): embedding, the rope table, the layers on
// mmqs, then the output -- every token's logits rows (`all`, rows c0.. of logits_all; the last
// chunk's last row also feeds `logits` and the top-k) or the last token's through the decode head.
void Ctx::enqueue_ubatch_short(int nt, bool all, int c0, bool last) {
    const HParams& hp = m->hp;
    const float theta_scale = std::pow(hp.rope_base, -2.0f / (float)hp.n_rot);
    EmbedParams ep{m->tok_embd, tokpos_b, xb, hp.n_embd};
    launch_embed_multi(ep, nt, stream);
    launch_rope_table(tokpos_b, nt, hp.n_rot, theta_scale, hp.freq_scale, m->rope_freqs, ub_rope, stream);
    const int pend_k = ubatch_layers_short(nt);
    if (all) {   // final norm + output head on mmqs, its parts summed into the logits rows
        const ActQ8 a_out = ub_act(hp.n_embd, nt, m->output.type);
        launch_quant_act(xb, hp.n_embd, m->output_norm, hp.eps, a_out, stream, nullptr, pend_k ? ub_spart : nullptr,
                         pend_k ? pend_k : 2);
        const QMat* mo[1] = {&m->output};
        const int pr[1] = {0};
        const int kp = launch_mmqs(mo, pr, 1, false, 0, a_out, ub_spart, hp.n_vocab, stream);
        launch_part_sum(ub_spart, kp, nt, hp.n_vocab, hp.n_vocab, nullptr, 0, logits_all + (size_t)c0 * hp.n_vocab,
                        hp.n_vocab, stream);
        if (last) {
            MI_HIP(hipMemcpyAsync(logits, logits_all + (size_t)(c0 + nt - 1) * hp.n_vocab, (size_t)hp.n_vocab * sizeof(float),
                                  hipMemcpyDeviceToDevice, stream));
            TopkParams tp{logits, hp.n_vocab, cand, topk_ids, topk_vals, d_h_topk_ids, d_h_topk_vals};
            launch_topk(tp, stream);
        }
    } else {
        // the last residual parts into xb (the next chunk, or the output, reads it)
        if (pend_k) launch_part_sum(ub_spart, pend_k, nt, hp.n_embd, hp.n_embd, xb, hp.n_embd, xb, hp.n_embd, stream);
        if (last) enqueue_output(xb + (size_t)(nt - 1) * hp.n_embd, nullptr);
    }
}

// One short physical batch (<= mmqs_max tokens) through the layers on the split-K streaming GEMM
// (mmq.hip mmqs): every launch writes K-part sums to ub_spart, and the next kernel adds them --
// quant_act (the residual, or SwiGLU of the gate/up parts), qkv_finish (RoPE, KV append).
// Returns the count of the last FFN down's parts, still to be added into xb.
int Ctx::ubatch_layers_short(int nt) {
    const HParams& hp = m->hp;
    const float kq_scale = 1.0f / std::sqrt((float)hp.head_dim);
    const int qkv_rows = hp.n_embd + 2 * kv_dim;
    int pend_k = 0;   // residual parts of ub_spart not yet added into xb
    for (int l = 0; l < hp.n_layer; ++l) {
        const Layer& L = m->layers[l];
        __half* kl = kcache + (size_t)l * n_ctx * kv_dim;
        __half* vl = vcache + (size_t)l * n_ctx * kv_dim;
        // Q / K / V: one quantisation of rms_norm(x) * attn_norm per activation format (the first
        // also adds the residual parts), the matrices of one type in one launch, rows [Q | K | V]
        const QMat* mats[3] = {&L.wq, &L.wk, &L.wv};
        const int prow[3] = {0, L.wq.rows, L.wq.rows + L.wk.rows};
        for (int f = 0; f < 2; ++f) {
            bool need = false;
            for (const QMat* q : mats) need = need || (q->type == T_Q8_0) == (f == 1);
            if (need) {
                launch_quant_act(xb, hp.n_embd, L.attn_norm, hp.eps, ub_act(hp.n_embd, nt, f ? T_Q8_0 : T_Q4_K), stream,
                                 nullptr, pend_k ? ub_spart : nullptr, pend_k ? pend_k : 2);
                pend_k = 0;
            }
        }
        int kp = 0;
        for (int i = 0; i < 3; ++i) {
            bool first = true;
            for (int j = 0; j < i; ++j) first = first && mats[j]->type != mats[i]->type;
            if (!first) continue;
            const QMat* ms[3];
            int pr[3], n = 0;
            for (int j = i; j < 3; ++j)
                if (mats[j]->type == mats[i]->type) {
                    ms[n] = mats[j];
                    pr[n++] = prow[j];
                }
            kp = launch_mmqs(ms, pr, n, false, 0, ub_act(hp.n_embd, nt, mats[i]->type), ub_spart, qkv_rows, stream);
        }
        QkvFinish F{ub_spart, qkv_rows, kp, nt, L.wq.rows, L.wk.rows, L.wv.rows, qb, hp.n_embd, kl, vl, kv_dim, cell_pos,
                    tokpos_b, ub_rope, hp.n_rot, hp.head_dim};
        launch_qkv_finish(F, stream);
        AttnParams a{qb, kl, vl, tokpos_b, cell_pos, attn_scores, attn_smax, attnb, hp.n_head, hp.n_head_kv,
                     hp.head_dim, kv_dim, (int)n_ctx, kq_scale};
        // within ATTN_SHORT cells the decode step's fused kernel, one workgroup per (kv head, token)
        // (20-token verify 3.52 -> 3.30 ms against the MFMA kernel's 32-token tiles; 64 tokens
        // equal, same box)
        const ActQ8 act_wo = ub_act(hp.n_embd, nt, L.wo.type);
        const bool qattn = attn_quant_supported(hp.n_head, hp.n_head_kv, hp.head_dim);
        if (attn_mfma && n_cells > ATTN_SHORT) {
            launch_attn_mfma(a, nt, attnb, stream);
            launch_quant_act(attnb, hp.n_embd, nullptr, hp.eps, act_wo, stream);
        } else if (qattn) {   // the fused kernel also quantises each token's output for W_o
            a.act_q8 = act_wo;
            launch_attn_multi(a, nt, attnb, stream);
        } else {
            launch_attn_multi(a, nt, attnb, stream);
            launch_quant_act(attnb, hp.n_embd, nullptr, hp.eps, act_wo, stream);
        }
        {   // output projection: parts of W_o attn, added to x by the FFN's quant_act
            const ActQ8& act = act_wo;
            const QMat* mo[1] = {&L.wo};
            const int pr[1] = {0};
            pend_k = launch_mmqs(mo, pr, 1, false, 0, act, ub_spart, hp.n_embd, stream);
        }
        if (hp.n_expert > 0) {   // routed experts: x += W_o parts first (the router reads x)
            launch_part_sum(ub_spart, pend_k, nt, hp.n_embd, hp.n_embd, xb, hp.n_embd, xb, hp.n_embd, stream);
            pend_k = 0;
            moe_ffn_short(l, nt);
            continue;
        }
        {   // FFN gate/up: parts of both, SwiGLU'd by the down input's quant_act
            const ActQ8 act = ub_act(hp.n_embd, nt, L.gate.type);
            launch_quant_act(xb, hp.n_embd, L.ffn_norm, hp.eps, act, stream, nullptr, ub_spart, pend_k);
            pend_k = 0;
            const QMat* mg[1] = {&L.gate};
            const int pr[1] = {0};
            const int kg = launch_mmqs(mg, pr, 1, true, hp.n_ff, act, ub_spart, 2 * hp.n_ff, stream);
            const ActQ8 a2 = ub_act(hp.n_ff, nt, L.down.type);
            launch_quant_act(nullptr, hp.n_ff, nullptr, hp.eps, a2, stream, nullptr, ub_spart, kg, 1);
            const QMat* md[1] = {&L.down};
            pend_k = launch_mmqs(md, pr, 1, false, 0, a2, ub_spart, hp.n_embd, stream);
        }
    }
    return pend_k;
}

int Ctx::decode(const int32_t* tokens, int n, bool all) {
    MI_HIP(hipSetDevice(device));
    if (n <= 0) throw Error("decode: empty batch");
    if (!unsynced) {   // the state a failed long-context exchange rolls back to
        undo_cells = n_cells;
        undo_pos = pos_max;
    }
    unsynced = true;
    for (int i = 0; i < n; ++i)
        if (tokens[i] < 0 || tokens[i] >= m->hp.n_vocab) throw Error("decode: token id out of range");
    if (n_cells + n > (int)n_ctx) return 1;   // no KV slot (llama_decode returns 1)
    if (m->hp.arch == ARCH_GPT2 && pos_max + n >= m->hp.n_ctx_train)
        throw Error("decode: gpt2 position past the learned position embeddings (n_ctx_train)");
    if (all && n > (int)n_batch) throw Error("decode: MI_OUT_ALL takes at most n_batch tokens");
    out_rows = 0;
    topk_row = -1;
    if (all && logits_all_cap < n) {   // every token's logits: [n_batch][n_vocab], allocated once
        if (logits_all) MI_HIP(hipFree(logits_all));
        logits_all = nullptr;
        MI_HIP(hipMalloc(&logits_all, (size_t)n_batch * m->hp.n_vocab * sizeof(float)));
        logits_all_cap = (int)n_batch;
    }
    // prompt ingestion through the batched GEMM when the context stays within the fused
    // attention's reach (dense models; MI_NO_BATCH=1 forces token-by-token decode)
    const bool fits = n >= 2 && batch_ok && hp_dense() && n_cells + n <= ATTN_SHORT && prof_layer < 0;
    // the MFMA batch path attends over any number of cells with the MFMA attention kernel
    const bool ub = n >= 2 && batch_ok && mmq_ok && prof_layer < 0 && (attn_mfma || n_cells + n <= ATTN_SHORT);
    if (ub && (!all || out_mmq)) {
        decode_ubatch(tokens, n, all);
        if (all) out_rows = n;
        return 0;
    }
    if (fits && !all) {
        decode_batch(tokens, n);
        return 0;
    }
    for (int i = 0; i < n; ++i) {
        const bool last = i == n - 1 || all;
        const int pos = pos_max + 1, cell = n_cells;
        attn_fused = cell + 1 <= ATTN_SHORT ? 1 : 0;   // this step attends over cell + 1 cells
        const long long slot = tok_slot++ % kTokRing;
        if (slot == 0 && tok_slot > 1) MI_HIP(hipStreamSynchronize(stream));
        int* hp = h_tokpos + slot * 4;
        hp[0] = tokens[i];
        hp[1] = pos;
        hp[2] = cell;
        hp[3] = 0;
        MI_HIP(hipMemcpyAsync(tokpos, hp, 4 * sizeof(int), hipMemcpyHostToDevice, stream));
        if (last && prof_layer >= 0 && prof_layer < m->hp.n_layer) {
            for (int k = 0; k < 2; ++k)
                if (!prof_ev[k]) MI_HIP(hipEventCreate(&prof_ev[k]));
            // graph up to the profiled launch, the launch itself eagerly with
            // hipExtLaunchKernel start/stop events, graph for the rest
            for (int k = 0; k < 3; ++k) {
                if (use_graphs && k != 1) {
                    if (!g_seg[attn_fused][k]) g_seg[attn_fused][k] = build_graph(true, k);
                    MI_HIP(hipGraphLaunch(g_seg[attn_fused][k], stream));
                } else {
                    seg_filter = k;
                    enqueue_step(true);
                    seg_filter = -1;
                }
            }
            prof_pending = true;
            prof_bytes = ffn_bytes();
        } else if (!use_graphs) {
            enqueue_step(last);
        } else {
            hipGraphExec_t& g = last ? g_full[attn_fused] : g_nolog[attn_fused];
            if (!g) g = build_graph(last, -1);
            MI_HIP(hipGraphLaunch(g, stream));
        }
        if (all)   // this token's logits -> row i
            MI_HIP(hipMemcpyAsync(logits_all + (size_t)i * m->hp.n_vocab, logits, (size_t)m->hp.n_vocab * sizeof(float),
                                  hipMemcpyDeviceToDevice, stream));
        h_cell_pos[cell] = pos;
        n_cells++;
        pos_max = pos;
    }
    if (all) out_rows = n;
    logits_valid = true;
    return 0;
}

void Ctx::sync() {
    MI_HIP(hipSetDevice(device));
    MI_HIP(hipStreamSynchronize(stream));
    const bool was_unsynced = unsynced;
    unsynced = false;
    if (h_attn_xerr && *h_attn_xerr) {   // an attention exchange gave up: the step's logits are invalid
        *h_attn_xerr = 0;
        logits_valid = false;
        // the cells decoded since the last good sync hold KV rows built from a wrong attention
        // output: drop them, and use the two-launch split kernels from now on
        if (was_unsynced) {
            n_cells = undo_cells;
            pos_max = undo_pos;
        }
        invalidate_graphs();
        attn_long_off = true;
        throw Error("long-context attention: the splits of a head were not co-resident (exchange timed out); "
                    "the step was rolled back and this context now uses the two-launch kernels");
    }
}

const float* Ctx::out_row(int row) const {
    if (row == -1) return logits;
    if (row < 0 || row >= std::max(out_rows, 1)) throw Error("output row out of range");
    if (out_rows == 0) return logits;   // MI_OUT_LAST: row 0 is the last token's
    return logits_all + (size_t)row * m->hp.n_vocab;
}

int Ctx::topk(int row, int k, int32_t* ids, float* vals) {
    if (!logits_valid) throw Error("no logits: decode a token first");
    if (k < 0 || k > TOPK_MAX) throw Error("topk: k must be in [0, 64]");
    if (out_rows > 0 && row == out_rows - 1) row = -1;   // the last row's top-k is already computed
    const float* src = out_row(row);
    if (src != logits || topk_row != -1) {   // another row than the mapped buffers hold
        MI_HIP(hipSetDevice(device));
        TopkParams tp{src, m->hp.n_vocab, cand, topk_ids, topk_vals, d_h_topk_ids, d_h_topk_vals};
        launch_topk(tp, stream);
        topk_row = src == logits ? -1 : row;
    }
    sync();
    for (int i = 0; i < k; ++i) {
        ids[i] = h_topk_ids[i];
        vals[i] = h_topk_vals[i];
    }
    return k;
}

int Ctx::gather(int row, const int32_t* ids, int n, float* out) {
    if (!logits_valid) throw Error("no logits: decode a token first");
    const float* src = out_row(row);
    if (n < 0 || n > 4096) throw Error("gather: n must be in [0, 4096]");
    for (int i = 0; i < n; ++i)
        if (ids[i] < 0 || ids[i] >= m->hp.n_vocab) throw Error("gather: id out of range");
    if (n == 0) return 0;
    MI_HIP(hipSetDevice(device));
    MI_HIP(hipMemcpyAsync(gather_ids, ids, n * sizeof(int), hipMemcpyHostToDevice, stream));
    launch_gather(src, gather_ids, n, gather_out, stream);
    MI_HIP(hipMemcpyAsync(h_gather, gather_out, n * sizeof(float), hipMemcpyDeviceToHost, stream));
    sync();
    std::memcpy(out, h_gather, n * sizeof(float));
    return n;
}

// Logits of rows row0..row0+nrows-1 at k ids each (ids [nrows][k]): the batched form of gather
// for a verification pass -- one copy in, one kernel, one copy out.
int Ctx::gather_rows(int row0, int nrows, const int32_t* ids, int k, float* out) {
    if (!logits_valid) throw Error("no logits: decode a token first");
    if (nrows < 0 || k < 0) throw Error("gather_rows: negative count");
    const size_t n = (size_t)nrows * k;
    if (n == 0) return 0;
    const int avail = out_rows > 0 ? out_rows : 1;
    if (row0 < 0 || row0 + nrows > avail) throw Error("gather_rows: output rows out of range");
    for (size_t i = 0; i < n; ++i)
        if (ids[i] < 0 || ids[i] >= m->hp.n_vocab) throw Error("gather_rows: id out of range");
    MI_HIP(hipSetDevice(device));
    if (n > grows_cap) {
        if (grows_ids) hipFree(grows_ids);
        if (grows_out) hipFree(grows_out);
        if (h_grows) hipHostFree(h_grows);
        grows_ids = nullptr; grows_out = nullptr; h_grows = nullptr; grows_cap = 0;
        MI_HIP(hipMalloc(&grows_ids, n * sizeof(int)));
        MI_HIP(hipMalloc(&grows_out, n * sizeof(float)));
        MI_HIP(hipHostMalloc(&h_grows, n * sizeof(float)));
        grows_cap = n;
    }
    const float* base = out_rows > 0 ? logits_all + (size_t)row0 * m->hp.n_vocab : logits;
    MI_HIP(hipMemcpyAsync(grows_ids, ids, n * sizeof(int), hipMemcpyHostToDevice, stream));
    launch_gather_rows(base, m->hp.n_vocab, grows_ids, (int)n, k, grows_out, stream);
    MI_HIP(hipMemcpyAsync(h_grows, grows_out, n * sizeof(float), hipMemcpyDeviceToHost, stream));
    sync();
    std::memcpy(out, h_grows, n * sizeof(float));
    return (int)n;
}

const float* Ctx::logits_host(int row) {
    if (!logits_valid) throw Error("no logits: decode a token first");
    const float* src = out_row(row);
    MI_HIP(hipSetDevice(device));
    MI_HIP(hipMemcpyAsync(h_logits, src, (size_t)m->hp.n_vocab * sizeof(float), hipMemcpyDeviceToHost, stream));
    sync();
    return h_logits;
}

void Ctx::kv_clear() {
    n_cells = 0;
    pos_max = -1;
    out_rows = 0;      // rows of the last MI_OUT_ALL pass belong to the cleared cache
    topk_row = -1;
}

// Remove cells with pos in [p0, p1); the survivors keep their order and are
// compacted to the front of the cache.
int Ctx::kv_seq_rm(int p0, int p1) {
    if (p0 < 0) p0 = 0;
    if (p1 < 0) p1 = INT_MAX;
    std::vector<int> keep;
    keep.reserve(n_cells);
    for (int c = 0; c < n_cells; ++c)
        if (h_cell_pos[c] < p0 || h_cell_pos[c] >= p1) keep.push_back(c);
    bool prefix = true;
    for (int j = 0; j < (int)keep.size(); ++j)
        if (keep[j] != j) { prefix = false; break; }
    if (!prefix) {
        MI_HIP(hipSetDevice(device));
        const HParams& hp = m->hp;
        if (!kv_scratch) MI_HIP(hipMalloc(&kv_scratch, (size_t)hp.n_layer * n_ctx * kv_dim * sizeof(__half)));
        MI_HIP(hipMemcpyAsync(move_src, keep.data(), keep.size() * sizeof(int), hipMemcpyHostToDevice, stream));
        launch_kv_move(kcache, hp.n_layer, n_ctx, kv_dim, move_src, (int)keep.size(), kv_scratch, stream);
        launch_kv_move(vcache, hp.n_layer, n_ctx, kv_dim, move_src, (int)keep.size(), kv_scratch, stream);
        std::vector<int> np(keep.size());
        for (size_t j = 0; j < keep.size(); ++j) np[j] = h_cell_pos[keep[j]];
        for (size_t j = 0; j < keep.size(); ++j) h_cell_pos[j] = np[j];
        MI_HIP(hipMemcpyAsync(cell_pos, h_cell_pos.data(), keep.size() * sizeof(int), hipMemcpyHostToDevice, stream));
        sync();
    }
    n_cells = (int)keep.size();
    pos_max = -1;
    for (int c = 0; c < n_cells; ++c) pos_max = std::max(pos_max, h_cell_pos[c]);
    return 0;
}

// seq_add (div == 0: pos += delta) / seq_div (pos /= div) over [p0, p1):
// positions change and cached K is re-rotated by the delta (K-shift).
int Ctx::kv_seq_shift(int p0, int p1, int delta, int div) {
    if (p0 < 0) p0 = 0;
    if (p1 < 0) p1 = INT_MAX;
    if (p0 == p1) return 0;
    if (div == 0 && delta == 0) return 0;
    if (div == 1) return 0;
    std::vector<int> dlt(n_cells, 0);
    bool any = false, neg = false;
    for (int c = 0; c < n_cells; ++c) {
        const int ps = h_cell_pos[c];
        if (ps >= p0 && ps < p1) {
            const int np = div ? ps / div : ps + delta;
            dlt[c] = np - ps;
            h_cell_pos[c] = np;
            any = any || dlt[c] != 0;
            neg = neg || np < 0;
        }
    }
    if (any) {
        MI_HIP(hipSetDevice(device));
        const HParams& hp = m->hp;
        MI_HIP(hipMemcpyAsync(cell_delta, dlt.data(), n_cells * sizeof(int), hipMemcpyHostToDevice, stream));
        KvShiftParams kp{kcache, hp.n_layer, (int)n_ctx, kv_dim, hp.head_dim, hp.n_rot, cell_delta, n_cells,
                         std::pow(hp.rope_base, -2.0f / (float)hp.n_rot), hp.freq_scale, m->rope_freqs};
        launch_kv_shift(kp, stream);
        MI_HIP(hipMemcpyAsync(cell_pos, h_cell_pos.data(), n_cells * sizeof(int), hipMemcpyHostToDevice, stream));
        sync();
    }
    if (neg) return kv_seq_rm(INT_MIN, 0);   // cells shifted below 0 are removed (llama.cpp semantics)
    pos_max = -1;
    for (int c = 0; c < n_cells; ++c) pos_max = std::max(pos_max, h_cell_pos[c]);
    return 0;
}

// ---- state: header | cell positions | K rows | V rows | last logits ----
namespace {
struct StateHdr {
    char magic[8];
    int32_t version, n_layer, kv_dim, n_vocab, n_cells, pos_max, logits_valid, pad;
};
}  // namespace

size_t Ctx::state_size() const {
    const HParams& hp = m->hp;
    return sizeof(StateHdr) + (size_t)n_cells * sizeof(int) +
           2 * (size_t)hp.n_layer * n_cells * kv_dim * sizeof(__half) + (size_t)hp.n_vocab * sizeof(float);
}

size_t Ctx::state_get(uint8_t* dst, size_t size) {
    const size_t need = state_size();
    if (size < need) throw Error("state_get: buffer too small");
    const HParams& hp = m->hp;
    StateHdr hd{};
    std::memcpy(hd.magic, "MISTATE1", 8);
    hd.version = 1;
    hd.n_layer = hp.n_layer;
    hd.kv_dim = kv_dim;
    hd.n_vocab = hp.n_vocab;
    hd.n_cells = n_cells;
    hd.pos_max = pos_max;
    hd.logits_valid = logits_valid ? 1 : 0;
    uint8_t* o = dst;
    std::memcpy(o, &hd, sizeof(hd));
    o += sizeof(hd);
    std::memcpy(o, h_cell_pos.data(), n_cells * sizeof(int));
    o += n_cells * sizeof(int);
    MI_HIP(hipSetDevice(device));
    sync();
    const size_t row = (size_t)n_cells * kv_dim * sizeof(__half);
    for (__half* cache : {kcache, vcache})
        for (int l = 0; l < hp.n_layer; ++l) {
            if (row) MI_HIP(hipMemcpy(o, cache + (size_t)l * n_ctx * kv_dim, row, hipMemcpyDeviceToHost));
            o += row;
        }
    if (logits_valid) MI_HIP(hipMemcpy(o, logits, (size_t)hp.n_vocab * sizeof(float), hipMemcpyDeviceToHost));
    else std::memset(o, 0, (size_t)hp.n_vocab * sizeof(float));
    return need;
}

size_t Ctx::state_set(const uint8_t* src, size_t size) {
    const HParams& hp = m->hp;
    StateHdr hd;
    if (size < sizeof(hd)) throw Error("state_set: truncated state");
    std::memcpy(&hd, src, sizeof(hd));
    if (std::memcmp(hd.magic, "MISTATE1", 8) != 0 || hd.n_layer != hp.n_layer || hd.kv_dim != kv_dim ||
        hd.n_vocab != hp.n_vocab)
        throw Error("state_set: state does not match this model");
    if (hd.n_cells < 0 || hd.n_cells > (int)n_ctx) throw Error("state_set: too many cells for this context");
    const size_t need = sizeof(hd) + (size_t)hd.n_cells * sizeof(int) +
                        2 * (size_t)hp.n_layer * hd.n_cells * kv_dim * sizeof(__half) + (size_t)hp.n_vocab * sizeof(float);
    if (size < need) throw Error("state_set: truncated state");
    const uint8_t* s = src + sizeof(hd);
    n_cells = hd.n_cells;
    pos_max = hd.pos_max;
    out_rows = 0;      // only the restored last-token row (-1 / 0) is valid after a restore
    topk_row = -1;
    std::memcpy(h_cell_pos.data(), s, n_cells * sizeof(int));
    s += n_cells * sizeof(int);
    MI_HIP(hipSetDevice(device));
    sync();
    if (n_cells) MI_HIP(hipMemcpy(cell_pos, h_cell_pos.data(), n_cells * sizeof(int), hipMemcpyHostToDevice));
    const size_t row = (size_t)n_cells * kv_dim * sizeof(__half);
    for (__half* cache : {kcache, vcache})
        for (int l = 0; l < hp.n_layer; ++l) {
            if (row) MI_HIP(hipMemcpy(cache + (size_t)l * n_ctx * kv_dim, s, row, hipMemcpyHostToDevice));
            s += row;
        }
    logits_valid = hd.logits_valid != 0;
    if (logits_valid) {
        MI_HIP(hipMemcpy(logits, s, (size_t)hp.n_vocab * sizeof(float), hipMemcpyHostToDevice));
        TopkParams tp{logits, hp.n_vocab, cand, topk_ids, topk_vals, d_h_topk_ids, d_h_topk_vals};
        launch_topk(tp, stream);
        sync();
    }
    return need;
}

int Ctx::prof_read(float* us, int n) {
    if (!prof_pending || n < 1) return 0;
    sync();
    float ms = 0.0f;
    MI_HIP(hipEventElapsedTime(&ms, prof_ev[0], prof_ev[1]));
    us[0] = ms * 1000.0f;
    prof_pending = false;
    return 1;
}

}  // namespace mi
