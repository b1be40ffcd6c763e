// bl::llama host surface on the MI355X engine.
//
// This is the C++ layer Blama's L4/L5 call (reference inference/code/llama/*.hpp). The names,
// parameter structs, call order and error messages are kept, so Server code and tests written
// against the reference port with small edits (INTEGRATION.md lists them: e.g. Model takes
// Params by value, there is no ChatFormat or lvocab()); they do not compile unchanged. Below
// it, every decode, logit extraction and KV operation goes through the engine's C ABI
// (include/mi_engine.h). There is no llama.cpp here.
//
// What is mirrored (reference file:line):
//   Token / TokenData / TokenDataVector       Token.hpp:9-17
//   TokenPrediction                           Session.hpp:20-27
//   Model{Params{gpu, vocabOnly, prefixInputsWithBos}}   Model.hpp:26-58
//   Vocab{tokenize, isEog, nTokens, tokenToString}       Vocab.hpp:16-34
//   Instance{InitParams, warmup, startSession, stopSession}   Instance.hpp:19-51
//   Session{InitParams, setInitialPrompt, complete, completeStream, fillCtx,
//           getState, setState, resetSampler}             Session.hpp:29-130
//   Sampler{Params, sample, accept, reset}                Sampler.hpp:22-115
//   LogitComparer / MetricsAggregator                     LogitComparer.hpp:12-34
//
// Not served (engine scope): Model::Params::gpu=false (the reference's CPU
// verifier), LoRA, control vectors, grammar constraints, encoder models.
#pragma once
#include <cstdint>
#include <memory>
#include <optional>
#include <random>
#include <span>
#include <stdexcept>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

#include "grammar.hpp"

struct mi_model;
struct mi_ctx;

namespace bl::llama {

using Token = std::int32_t;
inline constexpr Token Token_Invalid = -1;

struct TokenData {
    Token token;
    float logit;
};
using TokenDataVector = std::vector<TokenData>;

struct TokenPrediction {
    Token token = Token_Invalid;
    TokenDataVector logits;
    explicit operator bool() const { return token != Token_Invalid; }
};

class Model;

class Vocab {
public:
    explicit Vocab(const Model& model);
    // Tokenisation of `text` (llama_tokenize): SentencePiece (llm_tokenizer_spm) for "llama"
    // vocabularies, byte-level BPE with the GPT-2 or Llama-3 pre-tokenizer (llm_tokenizer_bpe)
    // for "gpt2" ones; addSpecial prepends BOS when the model asks for it, parseSpecial matches
    // control-token texts (e.g. "<s>", "<|begin_of_text|>") as single tokens.
    std::vector<Token> tokenize(std::string_view text, bool addSpecial, bool parseSpecial) const;
    Token decoderStartToken() const noexcept;
    bool isEog(Token token) const noexcept;
    int32_t nTokens() const noexcept;
    std::string tokenToString(Token token, bool special = true) const;
    Token bos() const noexcept { return m_bos; }
    Token eos() const noexcept { return m_eos; }
    // end-of-turn token (llama_vocab::token_eot): the GGUF's eot id, else a known end-of-turn
    // text found in the vocabulary, else -1 (LLAMA_TOKEN_NULL)
    Token eot() const noexcept { return m_eot; }
    // fill-in-the-middle tokens (llama_vocab_fim_pre/suf/mid, used by Session::pushPrompt for a
    // postfix, Session.cpp:142-159): tokenizer.ggml.fim_{pre,suf,mid}_token_id (or the older
    // prefix/suffix/middle keys), else a known FIM text in the vocabulary, else -1
    Token fimPre() const noexcept { return m_fimPre; }
    Token fimSuf() const noexcept { return m_fimSuf; }
    Token fimMid() const noexcept { return m_fimMid; }

private:
    void load();
    const Model& m_model;
    std::vector<std::string> m_text;
    std::vector<float> m_score;
    std::vector<int> m_type;
    std::unordered_map<std::string, Token> m_index;
    Token m_bos = -1, m_eos = -1, m_eot = -1, m_unk = 0;
    Token m_fimPre = -1, m_fimSuf = -1, m_fimMid = -1;
    bool m_spm = true;
    // byte-level BPE (tokenizer.ggml.model "gpt2": Llama-3 and GPT-2 vocabularies)
    bool m_bpe = false;
    int m_pre = 0;                           // pre-tokenizer: 0 GPT-2, 1 Llama-3 ("llama-bpe")
    bool m_ignoreMerges = false;             // Llama-3: a pre-token found whole in the vocab is one token
    std::unordered_map<std::string, int> m_rank;   // "left right" -> merge rank
    void bpeWord(std::string_view word, std::vector<Token>& out) const;
    bool m_loaded = false;
    friend class Model;
};

class Model {
public:
    struct Params {
        bool gpu = true;                   // Model.hpp:29; false = the reference's CPU verifier (not served)
        bool vocabOnly = false;
        bool prefixInputsWithBos = false;
        int device = 0;                    // HIP device of this replica (extension: one Model per GPU)
        bool noUpload = false;             // header only, weights filled by loadReplicas (extension)
        bool operator==(const Params& other) const noexcept = default;
    };
    // One Model per entry of `devices` (extension for the replica server): the first
    // parses and uploads the GGUF, the others read only its header and receive the weights from
    // it (mi_model_replicate: an RCCL broadcast across devices, device copies on one device).
    static std::vector<std::shared_ptr<Model>> loadReplicas(const std::string& gguf, const std::vector<int>& devices,
                                                            Params params);
    static std::vector<std::shared_ptr<Model>> loadReplicas(const std::string& gguf, const std::vector<int>& devices) {
        return loadReplicas(gguf, devices, Params{});
    }
    Model(const std::string& gguf, Params params);
    // Load from a GGUF image in memory (tests, replicas).
    Model(const void* data, size_t size, Params params);
    ~Model();
    Model(const Model&) = delete;
    Model& operator=(const Model&) = delete;

    const Params& params() const noexcept { return m_params; }
    uint32_t trainCtxLength() const noexcept;
    bool shouldAddBosToken() const noexcept;
    bool hasEncoder() const noexcept { return false; }
    bool prefixInputsWithBos() const noexcept { return m_params.prefixInputsWithBos; }

    mi_model* mmodel() noexcept { return m_model; }
    const mi_model* mmodel() const noexcept { return m_model; }
    const Vocab& vocab() const noexcept { return m_vocab; }

private:
    const Params m_params;
    mi_model* m_model = nullptr;
    Vocab m_vocab{*this};
};

class Sampler {
public:
    enum class SamplingType { Top_K, Top_P, Min_P, Typical_P, Temperature, XTC, Infill };
    struct Params {
        uint32_t rngSeed = 0;
        int32_t minKeep = 0;
        int32_t topK = 40;
        float topP = 0.95f;
        float minP = 0.05f;
        float tfsZ = 1.00f;
        float typicalP = 1.00f;
        float temp = 0.80f;
        float tempRange = 0.00f;
        float tempExp = 1.00f;
        struct RepetitionPenalty {
            int32_t numTokens = 64;
            float repeat = 1.00f;
            float freq = 0.00f;
            float present = 0.00f;
        } repetitionPenalty;
        std::vector<SamplingType> samplerSequence = {SamplingType::Top_K, SamplingType::Typical_P,
                                                     SamplingType::Top_P, SamplingType::Min_P,
                                                     SamplingType::Temperature};
        struct Mirostat {                  // Sampler.hpp:55-59
            int32_t ver = 0;               // 0 = disabled, 1 = mirostat, 2 = mirostat 2.0
            float tau = 5.00f;
            float eta = 0.10f;
        } mirostat;
        struct Xtc {                       // Sampler.hpp:60-64
            float probability = 0.00f;     // 0 = disabled
            float threshold = 0.10f;       // > 0.5 disables
        } xtc;
        std::string grammar;
        std::vector<std::pair<Token, float>> logitBias;
    };
    Sampler(Model& model, const Params& params);

    // Samples from the context's last logits.  With no logit bias and no active penalty, the
    // chain's first stage is top_k(topK) (topK <= 64), so the engine's sorted top-k is the same
    // candidate set (ties broken by id, which std::sort leaves unspecified).  Otherwise bias and
    // penalties can move tokens across the top-k boundary, so the chain runs on the full
    // vocabulary, as the reference's does (Sampler.cpp:30-41).
    // With a grammar (Params::grammar, GBNF, root rule "root"): the chain's pick is checked
    // against the grammar and, when it does not fit, the full vocabulary is resampled with the
    // grammar applied first (Sampler.cpp:126-173); grammarFirst applies it first always.
    Token sample(mi_ctx* ctx, int idx = -1, bool grammarFirst = false);
    void accept(Token id, bool acceptGrammar);
    void reset();
    const Grammar* grammar() const noexcept { return m_grammar.get(); }

    // The chain applied to a candidate list sorted by logit descending (exposed for tests).
    struct Candidate { Token id; float logit; float p; };
    Token applyChain(std::vector<Candidate>& cur);
    Token applyMirostat(std::vector<Candidate>& cur);

private:
    Model& m_model;
    Params m_params;
    float m_mu = 0.0f;                     // mirostat state (2 tau at start and on reset)
    std::mt19937 m_xtcRng;                 // llama_sampler_init_xtc's own generator
    std::mt19937 m_rng;
    std::vector<Token> m_prev;          // penalty window
    std::unique_ptr<Grammar> m_grammar;    // null: no grammar (llama_sampler_init_grammar of "")
    Token sampleChain(mi_ctx* ctx, int idx);
    Token sampleGrammarFirst(mi_ctx* ctx, int idx);
};

class Instance;

class Session {
public:
    struct InitParams {
        uint32_t gaFactor = 1;
        uint32_t gaWidth = 512;
        bool infiniteContext = true;
        uint32_t seed = 0;
        std::string grammar;
        float temperature = 0.80f;
        float topP = 0.95f;
        // fillCtx as one batched pass (mi_decode MI_OUT_ALL) instead of the reference's one decode
        // per claimed token.  Off by default: the serial form is bit-identical to generation
        // (t-integration.cpp:219-248); the batched rows match it within the GEMM's fp32 order.
        bool batchedVerify = false;
    };
    Session(Instance& instance, mi_ctx* ctx, InitParams params);
    Session(const Session&) = delete;
    Session& operator=(const Session&) = delete;
    ~Session();

    void setInitialPrompt(std::span<const Token> prompt);
    bool setState(std::span<uint8_t> state);
    struct CompleteParams {
        std::span<const Token> prompt;
        std::span<const Token> suffix;
        int32_t maxTokens = 0;
    };
    std::vector<TokenPrediction> complete(CompleteParams params);

    class StreamGenerator {
    public:
        StreamGenerator(Session& session, CompleteParams params) : m_session(session), m_params(params) {}
        TokenPrediction complete();
        void abort() { m_status = Status::Aborted; }
        enum class Status { InProgress, Completed, Aborted };
        Status status() const { return m_status; }

    private:
        Session& m_session;
        CompleteParams m_params;
        int32_t m_genTokens = 0;
        Status m_status = Status::InProgress;
    };
    StreamGenerator completeStream(CompleteParams params);

    std::vector<TokenPrediction> fillCtx(std::span<TokenPrediction> tokens);
    std::vector<uint8_t> getState();
    void resetSampler(const Sampler::Params& params);

private:
    enum class Source { InitialPrompt, InteractivePrompt, Generated };
    void pushPrompt(std::span<const Token> prompt, std::span<const Token> postfix = {});
    TokenPrediction getToken();
    void doDecode(std::span<const Token> tokens, Source src);
    void flushPendingState();
    TokenDataVector getLogitsFromCtx(int32_t topK);
    // logits at `tokens`' ids of output row `row` (-1: the last token's; 0..n-1 after a batched
    // fillCtx pass)
    TokenDataVector getLogitsFromCtx(const TokenDataVector& tokens, int32_t row = -1);
    void requireGenerating() const;

    struct State {
        enum class Phase { Initial, Generating, Streaming };
        Phase m_phase = Phase::Initial;
        Token m_currToken = Token_Invalid;
        unsigned maxTokens = 0;
        unsigned numKeep = 0;
        uint32_t gaIndex = 0;
        uint32_t numPast = 0;
    };

    Instance& m_instance;
    mi_ctx* m_ctx;
    std::unique_ptr<Sampler> m_sampler;
    InitParams m_params;
    State m_state;
};

class Instance {
public:
    struct InitParams {
        uint32_t ctxSize = 0;
        uint32_t batchSize = 2048;
        uint32_t ubatchSize = 512;
        bool flashAttn = false;
    };
    Instance(Model& model, InitParams params);
    ~Instance();
    Instance(const Instance&) = delete;
    Instance& operator=(const Instance&) = delete;

    void warmup();
    Session& startSession(const Session::InitParams params);
    void stopSession() noexcept;
    Model& model() const noexcept { return m_model; }
    mi_ctx* mctx() noexcept { return m_ctx; }

private:
    Model& m_model;
    mi_ctx* m_ctx = nullptr;
    std::optional<Session> m_session;
};

struct ComparisonMetrics {
    float top1Match;
    float distance;
    float jsd;
};

class LogitComparer {
public:
    static ComparisonMetrics compare(const TokenDataVector& data1, const TokenDataVector& data2);
    static float logitSimilarity(const TokenDataVector& data1, const TokenDataVector& data2);
};

struct MetricsAggregator {
    float pushAndVerify(std::span<const ComparisonMetrics> m);

private:
    std::vector<ComparisonMetrics> metrics;
};

}  // namespace bl::llama
