// bl::llama host surface on the MI355X engine (see llama.hpp for the mirrored reference files).
#include "llama.hpp"
#include "unicode_cats.hpp"
#include <array>

#include "mi_engine.h"

#include <algorithm>
#include <cmath>
#include <limits>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <queue>
#include <sstream>

namespace bl::llama {

namespace {
// throw_ex{} << ... in the reference (bstl/throw_stdex.hpp): std::runtime_error with the text.
struct Fail {
    std::ostringstream os;
    template <typename T>
    Fail& operator<<(const T& v) {
        os << v;
        return *this;
    }
    [[noreturn]] void raise() { throw std::runtime_error(os.str()); }
};
#define BL_THROW(msg) \
    do { Fail f_; f_ << msg; f_.raise(); } while (0)

std::string last_error() {
    const char* e = mi_last_error();
    return e ? std::string(e) : std::string();
}

constexpr int kTypeNormal = 1, kTypeUnknown = 2, kTypeControl = 3, kTypeUserDefined = 4, kTypeByte = 6;
const std::string kSpace = "\xe2\x96\x81";   // U+2581, SentencePiece's whitespace

std::string escape_whitespace(std::string_view s) {
    std::string o;
    o.reserve(s.size() * 2);
    for (char c : s) {
        if (c == ' ') o += kSpace;
        else o += c;
    }
    return o;
}
std::string unescape_whitespace(const std::string& s) {
    std::string o;
    o.reserve(s.size());
    for (size_t i = 0; i < s.size();) {
        if (s.compare(i, kSpace.size(), kSpace) == 0) {
            o += ' ';
            i += kSpace.size();
        } else {
            o += s[i++];
        }
    }
    return o;
}
size_t utf8_len(unsigned char c) {
    static const size_t lut[16] = {1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 2, 2, 3, 4};
    return lut[c >> 4];
}

// ---- byte-level BPE (llm_tokenizer_bpe, unicode.cpp) ----
// GPT-2's bytes_to_unicode: printable bytes map to themselves, the rest to U+0100.. in byte order
const std::array<uint32_t, 256>& byte_to_cp() {
    static const std::array<uint32_t, 256> t = [] {
        std::array<uint32_t, 256> m{};
        uint32_t n = 0;
        for (int b = 0; b < 256; ++b) {
            const bool keep = (b >= 33 && b <= 126) || (b >= 161 && b <= 172) || (b >= 174);
            m[b] = keep ? (uint32_t)b : 256 + n++;
        }
        return m;
    }();
    return t;
}
void put_utf8(std::string& o, uint32_t cp) {
    if (cp < 0x80) o += (char)cp;
    else if (cp < 0x800) { o += (char)(0xC0 | (cp >> 6)); o += (char)(0x80 | (cp & 0x3F)); }
    else if (cp < 0x10000) { o += (char)(0xE0 | (cp >> 12)); o += (char)(0x80 | ((cp >> 6) & 0x3F)); o += (char)(0x80 | (cp & 0x3F)); }
    else { o += (char)(0xF0 | (cp >> 18)); o += (char)(0x80 | ((cp >> 12) & 0x3F)); o += (char)(0x80 | ((cp >> 6) & 0x3F)); o += (char)(0x80 | (cp & 0x3F)); }
}
// UTF-8 -> code points with the byte offset of each (an invalid sequence is one U+FFFD per byte)
void cps_of(std::string_view s, std::vector<uint32_t>& cp, std::vector<size_t>& off) {
    cp.clear();
    off.clear();
    for (size_t i = 0; i < s.size();) {
        const unsigned char c = (unsigned char)s[i];
        size_t n = c < 0x80 ? 1 : (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : (c >> 3) == 30 ? 4 : 0;
        uint32_t v = 0xFFFD;
        if (n && i + n <= s.size()) {
            v = n == 1 ? c : n == 2 ? (c & 0x1F) : n == 3 ? (c & 0x0F) : (c & 0x07);
            for (size_t k = 1; k < n; ++k) {
                const unsigned char d = (unsigned char)s[i + k];
                if ((d & 0xC0) != 0x80) { n = 0; break; }
                v = (v << 6) | (d & 0x3F);
            }
        }
        if (!n || i + n > s.size()) { n = 1; v = 0xFFFD; }
        cp.push_back(v);
        off.push_back(i);
        i += n;
    }
    off.push_back(s.size());
}
template <size_t N>
bool in_ranges(const unicode::CpRange (&r)[N], uint32_t c) {
    size_t lo = 0, hi = N;
    while (lo < hi) {
        const size_t mid = (lo + hi) / 2;
        if (c < r[mid].lo) hi = mid;
        else if (c > r[mid].hi) lo = mid + 1;
        else return true;
    }
    return false;
}
bool is_L(uint32_t c) { return c < 0x80 ? ((c | 32) >= 'a' && (c | 32) <= 'z') : in_ranges(unicode::kLetter, c); }
bool is_N(uint32_t c) { return c < 0x80 ? (c >= '0' && c <= '9') : in_ranges(unicode::kNumber, c); }
bool is_S(uint32_t c) {   // \s: Unicode White_Space
    return (c >= 9 && c <= 13) || c == 32 || c == 0x85 || c == 0xA0 || c == 0x1680 || (c >= 0x2000 && c <= 0x200A) ||
           c == 0x2028 || c == 0x2029 || c == 0x202F || c == 0x205F || c == 0x3000;
}
bool is_nl(uint32_t c) { return c == '\r' || c == '\n'; }
uint32_t lower_ascii(uint32_t c) { return (c >= 'A' && c <= 'Z') ? c + 32 : c; }

// Length (code points) of the pre-token starting at i: the first alternative of the regex that
// matches there, with the regex's greedy / backtracking semantics (unicode.cpp's hand-written
// splitters do the same).
//   Llama-3: (?:'[sS]|'[tT]|'[rR][eE]|'[vV][eE]|'[mM]|'[lL][lL]|'[dD])|[^\r\n\p{L}\p{N}]?\p{L}+|
//            \p{N}{1,3}| ?[^\s\p{L}\p{N}]+[\r\n]*|\s*[\r\n]+|\s+(?!\S)|\s+
//   GPT-2:   's|'t|'re|'ve|'m|'ll|'d| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+
size_t pretok_len(const std::vector<uint32_t>& c, size_t i, bool llama3) {
    const size_t n = c.size();
    auto other = [&](uint32_t x) { return !is_S(x) && !is_L(x) && !is_N(x); };
    if (c[i] == '\'' && i + 1 < n) {
        const uint32_t a = llama3 ? lower_ascii(c[i + 1]) : c[i + 1];
        if (a == 's' || a == 't' || a == 'm' || a == 'd') return 2;
        if (i + 2 < n) {
            const uint32_t b = llama3 ? lower_ascii(c[i + 2]) : c[i + 2];
            if ((a == 'r' && b == 'e') || (a == 'v' && b == 'e') || (a == 'l' && b == 'l')) return 3;
        }
    }
    size_t j = i;
    if (llama3) {
        if (!is_nl(c[j]) && !is_L(c[j]) && !is_N(c[j]) && j + 1 < n && is_L(c[j + 1])) ++j;
        if (is_L(c[j])) {
            while (j < n && is_L(c[j])) ++j;
            return j - i;
        }
        if (is_N(c[i])) {
            j = i;
            while (j < n && j - i < 3 && is_N(c[j])) ++j;
            return j - i;
        }
    } else {
        if (c[j] == ' ' && j + 1 < n && is_L(c[j + 1])) ++j;
        if (is_L(c[j])) {
            while (j < n && is_L(c[j])) ++j;
            return j - i;
        }
        j = i;
        if (c[j] == ' ' && j + 1 < n && is_N(c[j + 1])) ++j;
        if (is_N(c[j])) {
            while (j < n && is_N(c[j])) ++j;
            return j - i;
        }
    }
    j = i;
    if (c[j] == ' ' && j + 1 < n && other(c[j + 1])) ++j;
    if (other(c[j])) {
        while (j < n && other(c[j])) ++j;
        if (llama3)
            while (j < n && is_nl(c[j])) ++j;
        return j - i;
    }
    if (is_S(c[i])) {
        size_t e = i;
        while (e < n && is_S(c[e])) ++e;
        if (llama3) {   // \s*[\r\n]+ : up to the run's last CR/LF
            size_t last = n;
            for (size_t k = i; k < e; ++k)
                if (is_nl(c[k])) last = k;
            if (last != n) return last + 1 - i;
        }
        if (e == n) return e - i;       // \s+(?!\S) at the end of the text
        if (e - i >= 2) return e - i - 1;   // \s+(?!\S): leave the last space to the next word
        return e - i;                   // \s+
    }
    return 1;
}
}  // namespace

// ------------------------------------------------------------------ Model ---
Model::Model(const std::string& gguf, Params params) : m_params(params) {
    if (!params.gpu)
        BL_THROW("Model::Params::gpu=false (the CPU verifier) is not served by the MI355X engine");
    mi_model_params mp{params.device, 0, params.vocabOnly ? 1 : 0, params.noUpload ? 1 : 0};
    m_model = mi_model_load(gguf.c_str(), &mp);
    if (!m_model) BL_THROW("Failed to load model " << gguf << ": " << last_error());
    m_vocab.load();
}

Model::Model(const void* data, size_t size, Params params) : m_params(params) {
    if (!params.gpu)
        BL_THROW("Model::Params::gpu=false (the CPU verifier) is not served by the MI355X engine");
    mi_model_params mp{params.device, 0, params.vocabOnly ? 1 : 0, params.noUpload ? 1 : 0};
    m_model = mi_model_load_from_memory(data, size, &mp);
    if (!m_model) BL_THROW("Failed to load model: " << last_error());
    m_vocab.load();
}

Model::~Model() {
    if (m_model) mi_model_free(m_model);
}

std::vector<std::shared_ptr<Model>> Model::loadReplicas(const std::string& gguf, const std::vector<int>& devices,
                                                        Params params) {
    if (devices.empty()) BL_THROW("loadReplicas: no device");
    std::vector<std::shared_ptr<Model>> out;
    Params p = params;
    p.device = devices[0];
    p.noUpload = false;
    out.push_back(std::make_shared<Model>(gguf, p));   // parses and repacks the weights once
    for (size_t i = 1; i < devices.size(); ++i) {
        Params r = params;
        r.device = devices[i];
        r.noUpload = true;                             // header only: the arena is filled below
        out.push_back(std::make_shared<Model>(gguf, r));
    }
    if (out.size() > 1) {
        std::vector<mi_model*> ms;
        for (auto& m : out) ms.push_back(m->mmodel());
        if (mi_model_replicate(ms.data(), (int32_t)ms.size()) != 0) BL_THROW("loadReplicas: " << last_error());
    }
    return out;
}

uint32_t Model::trainCtxLength() const noexcept {
    // a vocab-only model has no weights and reports no training context (t-integration.cpp:35)
    return m_params.vocabOnly ? 0u : (uint32_t)std::max(0, mi_model_n_ctx_train(m_model));
}

bool Model::shouldAddBosToken() const noexcept { return mi_model_add_bos(m_model) == 1; }

// ------------------------------------------------------------------ Vocab ---
Vocab::Vocab(const Model& model) : m_model(model) {}

void Vocab::load() {
    const mi_model* m = m_model.mmodel();
    const int n = mi_model_n_tokens(m);
    m_text.resize(std::max(0, n));
    m_score.resize(m_text.size());
    m_type.resize(m_text.size());
    std::string buf;
    for (int i = 0; i < n; ++i) {
        const int len = mi_model_token_text(m, i, nullptr, 0);
        buf.assign((size_t)len + 1, '\0');
        mi_model_token_text(m, i, buf.data(), len + 1);
        m_text[i].assign(buf.data(), (size_t)len);
        m_score[i] = mi_model_token_score(m, i);
        m_type[i] = mi_model_token_type(m, i);
        m_index.emplace(m_text[i], i);
    }
    m_bos = mi_model_token_bos(m);
    m_eos = mi_model_token_eos(m);
    for (int i = 0; i < n; ++i)
        if (m_type[i] == kTypeUnknown) { m_unk = i; break; }
    // the engine's end-of-generation set is {eos, tokenizer.ggml.eot_token_id}
    for (int i = 0; i < n && m_eot < 0; ++i)
        if (i != m_eos && mi_model_token_is_eog(m, i) == 1) m_eot = i;
    for (const char* t : {"<|eot_id|>", "<|im_end|>", "<|end|>", "<end_of_turn>", "<|endoftext|>", "<EOT>"}) {
        if (m_eot >= 0) break;
        auto it = m_index.find(t);
        if (it != m_index.end()) m_eot = it->second;
    }
    // FIM ids (llama_vocab::impl::load: the GGUF keys, then the b5187 text auto-detection)
    auto meta_id = [&](std::initializer_list<const char*> keys) -> Token {
        for (const char* k : keys) {
            char v[32] = {0};
            if (mi_model_meta_str(m, k, v, sizeof v) > 0) {
                const long id = std::strtol(v, nullptr, 10);
                if (id >= 0 && id < n) return (Token)id;
            }
        }
        return -1;
    };
    auto text_id = [&](std::initializer_list<const char*> texts) -> Token {
        for (const char* t : texts) {
            auto it = m_index.find(t);
            if (it != m_index.end()) return it->second;
        }
        return -1;
    };
    m_fimPre = meta_id({"tokenizer.ggml.fim_pre_token_id", "tokenizer.ggml.prefix_token_id"});
    m_fimSuf = meta_id({"tokenizer.ggml.fim_suf_token_id", "tokenizer.ggml.suffix_token_id"});
    m_fimMid = meta_id({"tokenizer.ggml.fim_mid_token_id", "tokenizer.ggml.middle_token_id"});
    if (m_fimPre < 0)
        m_fimPre = text_id({"<|fim_prefix|>", "<fim-prefix>", "<fim_prefix>", "<｜fim▁begin｜>",
                            "<PRE>", "▁<PRE>"});
    if (m_fimSuf < 0)
        m_fimSuf = text_id({"<|fim_suffix|>", "<fim-suffix>", "<fim_suffix>", "<｜fim▁hole｜>",
                            "<SUF>", "▁<SUF>"});
    if (m_fimMid < 0)
        m_fimMid = text_id({"<|fim_middle|>", "<fim-middle>", "<fim_middle>", "<｜fim▁end｜>",
                            "<MID>", "▁<MID>"});
    char tk[32] = {0};
    mi_model_tokenizer(m, tk, sizeof tk);
    m_spm = std::string(tk) == "llama";
    m_bpe = std::string(tk) == "gpt2";
    if (m_bpe) {
        // llama_vocab::impl::load: tokenizer.ggml.pre picks the pre-tokenizer; the Llama-3 family
        // also takes a whole pre-token from the vocabulary before merging (ignore_merges)
        char pre[64] = {0};
        const std::string p = mi_model_meta_str(m, "tokenizer.ggml.pre", pre, sizeof pre) > 0 ? pre : "default";
        if (p == "llama3" || p == "llama-v3" || p == "llama-bpe" || p == "falcon3") {
            m_pre = 1;
            m_ignoreMerges = true;
        } else if (p == "gpt-2" || p == "default") {
            m_pre = 0;
        } else {
            BL_THROW("tokenizer: BPE pre-tokenizer '" << p << "' is not served (llama-bpe, gpt-2)");
        }
        const int nm = mi_model_n_merges(m);
        for (int i = 0; i < nm; ++i) {
            const int len = mi_model_merge(m, i, nullptr, 0);
            buf.assign((size_t)len + 1, '\0');
            mi_model_merge(m, i, buf.data(), len + 1);
            m_rank.emplace(std::string(buf.data(), (size_t)len), i);
        }
    }
    m_loaded = true;
}

int32_t Vocab::nTokens() const noexcept { return (int32_t)m_text.size(); }
bool Vocab::isEog(Token token) const noexcept { return mi_model_token_is_eog(m_model.mmodel(), token) == 1; }
Token Vocab::decoderStartToken() const noexcept { return m_bos; }

std::string Vocab::tokenToString(Token token, bool special) const {
    if (token < 0 || token >= nTokens()) return {};
    const std::string& t = m_text[token];
    if (m_bpe && (m_type[token] == kTypeNormal || m_type[token] == 0)) {   // byte-level: back to bytes
        static const std::unordered_map<uint32_t, unsigned char> back = [] {
            std::unordered_map<uint32_t, unsigned char> m;
            for (int b = 0; b < 256; ++b) m.emplace(byte_to_cp()[b], (unsigned char)b);
            return m;
        }();
        std::vector<uint32_t> cp;
        std::vector<size_t> off;
        cps_of(t, cp, off);
        std::string o;
        for (size_t i = 0; i < cp.size(); ++i) {
            auto it = back.find(cp[i]);
            if (it != back.end()) o += (char)it->second;
            else o.append(t, off[i], off[i + 1] - off[i]);
        }
        return o;
    }
    switch (m_type[token]) {
    case kTypeNormal: return unescape_whitespace(t);
    case kTypeUnknown: return "\xe2\x96\x85";   // U+2585, what llama_token_to_piece prints
    case kTypeControl: return special ? t : std::string();
    case kTypeUserDefined: return t;
    case kTypeByte:
        if (t.size() == 6 && t.rfind("<0x", 0) == 0) return std::string(1, (char)std::stoi(t.substr(3, 2), nullptr, 16));
        return t;
    default: return {};
    }
}

// One pre-token of a BPE vocabulary (llm_tokenizer_bpe_session::tokenize): byte-encode it, then
// merge adjacent symbols lowest merge rank first (leftmost on ties); symbols missing from the
// vocabulary fall back to their single byte-characters.
void Vocab::bpeWord(std::string_view word, std::vector<Token>& out) const {
    std::string enc;
    for (unsigned char b : word) put_utf8(enc, byte_to_cp()[b]);
    if (m_ignoreMerges) {
        auto it = m_index.find(enc);
        if (it != m_index.end()) { out.push_back(it->second); return; }
    }
    struct Sym { int prev, next; size_t off, n; };
    std::vector<Sym> sym;
    for (size_t off = 0; off < enc.size();) {
        const size_t n = std::min(utf8_len((unsigned char)enc[off]), enc.size() - off);
        sym.push_back({(int)sym.size() - 1, (int)sym.size() + 1, off, n});
        off += n;
    }
    if (sym.empty()) return;
    sym.back().next = -1;
    struct Bigram { int left, right, rank; size_t size; };
    auto worse = [](const Bigram& a, const Bigram& b) { return a.rank > b.rank || (a.rank == b.rank && a.left > b.left); };
    std::priority_queue<Bigram, std::vector<Bigram>, decltype(worse)> q(worse);
    auto try_pair = [&](int l, int r) {
        if (l < 0 || r < 0) return;
        std::string key = enc.substr(sym[l].off, sym[l].n);
        key += ' ';
        key.append(enc, sym[r].off, sym[r].n);
        auto it = m_rank.find(key);
        if (it != m_rank.end()) q.push({l, r, it->second, sym[l].n + sym[r].n});
    };
    for (size_t i = 1; i < sym.size(); ++i) try_pair((int)i - 1, (int)i);
    while (!q.empty()) {
        const Bigram b = q.top();
        q.pop();
        Sym& L = sym[b.left];
        Sym& R = sym[b.right];
        if (L.n == 0 || R.n == 0 || L.n + R.n != b.size || L.next != b.right) continue;   // stale
        L.n += R.n;
        R.n = 0;
        L.next = R.next;
        if (R.next >= 0) sym[R.next].prev = b.left;
        try_pair(L.prev, b.left);
        try_pair(b.left, L.next);
    }
    for (int i = 0; i != -1; i = sym[i].next) {
        const std::string t = enc.substr(sym[i].off, sym[i].n);
        auto it = m_index.find(t);
        if (it != m_index.end()) { out.push_back(it->second); continue; }
        for (size_t k = 0; k < t.size();) {   // each character alone, where the vocabulary has it
            const size_t n = std::min(utf8_len((unsigned char)t[k]), t.size() - k);
            auto bt = m_index.find(t.substr(k, n));
            if (bt != m_index.end()) out.push_back(bt->second);
            k += n;
        }
    }
}

std::vector<Token> Vocab::tokenize(std::string_view text, bool addSpecial, bool parseSpecial) const {
    if (!m_spm && !m_bpe) BL_THROW("tokenizer: only SentencePiece (llama) and byte-level BPE (gpt2) vocabularies are served");
    std::vector<Token> out;
    if (addSpecial && m_model.shouldAddBosToken() && m_bos >= 0) out.push_back(m_bos);

    // 1. split the text at special-token texts (control tokens only when parseSpecial), longest first
    struct Frag { bool tok; Token id; std::string_view s; };
    std::vector<Frag> frags{{false, -1, text}};
    std::vector<Token> specials;
    for (int i = 0; i < nTokens(); ++i)
        if ((m_type[i] == kTypeControl && parseSpecial) || m_type[i] == kTypeUserDefined)
            if (!m_text[i].empty()) specials.push_back(i);
    std::stable_sort(specials.begin(), specials.end(),
                     [&](Token a, Token b) { return m_text[a].size() > m_text[b].size(); });
    for (Token sp : specials) {
        const std::string& st = m_text[sp];
        std::vector<Frag> next;
        for (const Frag& f : frags) {
            if (f.tok) { next.push_back(f); continue; }
            size_t pos = 0;
            while (true) {
                const size_t hit = f.s.find(st, pos);
                if (hit == std::string_view::npos) break;
                if (hit > pos) next.push_back({false, -1, f.s.substr(pos, hit - pos)});
                next.push_back({true, sp, {}});
                pos = hit + st.size();
            }
            if (pos < f.s.size()) next.push_back({false, -1, f.s.substr(pos)});
        }
        frags.swap(next);
    }

    if (m_bpe) {   // 2'. byte-level BPE: pre-tokenize each raw fragment, then merge each pre-token
        std::vector<uint32_t> cp;
        std::vector<size_t> off;
        for (const Frag& f : frags) {
            if (f.tok) { out.push_back(f.id); continue; }
            cps_of(f.s, cp, off);
            for (size_t i = 0; i < cp.size();) {
                const size_t n = pretok_len(cp, i, m_pre == 1);
                bpeWord(f.s.substr(off[i], off[i + n] - off[i]), out);
                i += n;
            }
        }
        return out;
    }
    // 2. SentencePiece BPE over each raw fragment (llm_tokenizer_spm semantics)
    bool prev_special = true;   // a raw fragment at the start or after a special token gets a space prefix
    for (const Frag& f : frags) {
        if (f.tok) {
            out.push_back(f.id);
            prev_special = true;
            continue;
        }
        std::string s = prev_special ? std::string(" ") : std::string();
        s += f.s;
        s = escape_whitespace(s);
        prev_special = false;
        struct Sym { int prev, next; size_t off, n; };
        std::vector<Sym> sym;
        for (size_t off = 0; off < s.size();) {
            const size_t n = std::min(utf8_len((unsigned char)s[off]), s.size() - off);
            sym.push_back({(int)sym.size() - 1, (int)sym.size() + 1, off, n});
            off += n;
        }
        if (sym.empty()) continue;
        sym.back().next = -1;
        struct Bigram { int left, right; float score; size_t size; };
        auto worse = [](const Bigram& a, const Bigram& b) {
            return a.score < b.score || (a.score == b.score && a.left > b.left);
        };
        std::priority_queue<Bigram, std::vector<Bigram>, decltype(worse)> q(worse);
        std::unordered_map<std::string, std::pair<int, int>> merged_from;
        auto try_pair = [&](int l, int r) {
            if (l < 0 || r < 0) return;
            const std::string t = s.substr(sym[l].off, sym[l].n + sym[r].n);
            auto it = m_index.find(t);
            if (it == m_index.end()) return;
            q.push({l, r, m_score[it->second], t.size()});
            merged_from[t] = {l, r};
        };
        for (size_t i = 1; i < sym.size(); ++i) try_pair((int)i - 1, (int)i);
        while (!q.empty()) {
            const Bigram b = q.top();
            q.pop();
            Sym& L = sym[b.left];
            Sym& R = sym[b.right];
            if (L.n == 0 || R.n == 0 || L.n + R.n != b.size) continue;   // stale
            L.n += R.n;
            R.n = 0;
            L.next = R.next;
            if (R.next >= 0) sym[R.next].prev = b.left;
            try_pair(L.prev, b.left);
            try_pair(b.left, L.next);
        }
        std::function<void(const Sym&)> emit = [&](const Sym& y) {
            const std::string t = s.substr(y.off, y.n);
            auto it = m_index.find(t);
            if (it != m_index.end()) { out.push_back(it->second); return; }
            auto mf = merged_from.find(t);
            if (mf == merged_from.end()) {   // byte fallback
                for (unsigned char c : t) {
                    char hex[8];
                    std::snprintf(hex, sizeof hex, "<0x%02X>", c);
                    auto bt = m_index.find(hex);
                    out.push_back(bt != m_index.end() ? bt->second : m_unk);
                }
                return;
            }
            emit(sym[mf->second.first]);
            emit(sym[mf->second.second]);
        };
        for (int i = 0; i != -1; i = sym[i].next) emit(sym[i]);
    }
    return out;
}

// ---------------------------------------------------------------- Sampler ---
Sampler::Sampler(Model& model, const Params& params)
    : m_model(model), m_params(params), m_mu(2.0f * params.mirostat.tau), m_xtcRng(params.rngSeed), m_rng(params.rngSeed) {
    if (params.mirostat.ver > 2) BL_THROW("Unsupported mirostat version");   // Sampler.cpp:67-69
    if (!params.grammar.empty()) m_grammar = std::make_unique<Grammar>(params.grammar, "root");
}

void Sampler::accept(Token id, bool acceptGrammar) {
    if (acceptGrammar && m_grammar) m_grammar->accept(m_model.vocab(), id);   // Sampler.cpp:100-106
    m_prev.push_back(id);
    const size_t w = (size_t)std::max(0, m_params.repetitionPenalty.numTokens);
    if (m_prev.size() > w) m_prev.erase(m_prev.begin(), m_prev.end() - (std::ptrdiff_t)w);
}

void Sampler::reset() {
    if (m_grammar) m_grammar->reset();
    m_prev.clear();
    m_rng.seed(m_params.rngSeed);   // llama_sampler_dist reset re-seeds
    m_xtcRng.seed(m_params.rngSeed);
    m_mu = 2.0f * m_params.mirostat.tau;
}

namespace {
void softmax(std::vector<Sampler::Candidate>& c) {   // sorted desc on entry
    const float mx = c[0].logit;
    float sum = 0.0f;
    for (auto& x : c) {
        x.p = std::exp(x.logit - mx);
        sum += x.p;
    }
    for (auto& x : c) x.p /= sum;
}
}  // namespace

// llama.cpp b5187 sampler chain semantics (llama-sampling.cpp), on a list sorted by logit desc.
Token Sampler::applyChain(std::vector<Candidate>& cur) {
    const Params& P = m_params;
    const size_t min_keep = (size_t)std::max(0, P.minKeep);
    for (auto& [tok, bias] : P.logitBias)
        for (auto& c : cur)
            if (c.id == tok) c.logit += bias;
    if (!P.logitBias.empty())
        std::stable_sort(cur.begin(), cur.end(), [](auto& a, auto& b) { return a.logit > b.logit; });
    const auto& rp = P.repetitionPenalty;
    if (rp.numTokens != 0 && !(rp.repeat == 1.0f && rp.freq == 0.0f && rp.present == 0.0f)) {
        std::unordered_map<Token, int> cnt;
        for (Token t : m_prev) cnt[t]++;
        for (auto& c : cur) {
            auto it = cnt.find(c.id);
            if (it == cnt.end()) continue;
            c.logit = c.logit <= 0 ? c.logit * rp.repeat : c.logit / rp.repeat;
            c.logit -= (float)it->second * rp.freq + (it->second > 0 ? 1.0f : 0.0f) * rp.present;
        }
        std::stable_sort(cur.begin(), cur.end(), [](auto& a, auto& b) { return a.logit > b.logit; });
    }
    if (P.mirostat.ver == 1 || P.mirostat.ver == 2) return applyMirostat(cur);
    for (SamplingType st : P.samplerSequence) {
        switch (st) {
        case SamplingType::Top_K: {
            size_t k = P.topK <= 0 ? cur.size() : (size_t)P.topK;
            k = std::min(std::max(k, min_keep), cur.size());
            cur.resize(k);
            break;
        }
        case SamplingType::Typical_P: {   // llama_sampler_typical_apply (locally typical sampling)
            if (P.typicalP >= 1.0f) break;
            softmax(cur);
            float entropy = 0.0f;
            for (auto& c : cur) entropy += -c.p * std::log(c.p);
            std::vector<float> shifted(cur.size());
            for (size_t i = 0; i < cur.size(); ++i) shifted[i] = std::fabs(-std::log(cur[i].p) - entropy);
            std::vector<size_t> idx(cur.size());
            for (size_t i = 0; i < idx.size(); ++i) idx[i] = i;
            std::sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return shifted[a] < shifted[b]; });
            float cum = 0.0f;
            size_t last = idx.size();
            for (size_t i = 0; i < idx.size(); ++i) {
                cum += cur[idx[i]].p;
                // min_keep is size_t there: min_keep 0 makes (min_keep - 1) the maximum value, so
                // the set is never cut (reproduced as is)
                if (cum > P.typicalP && i >= min_keep - 1) { last = i + 1; break; }
            }
            std::vector<Candidate> nw;
            for (size_t i = 0; i < last; ++i) nw.push_back(cur[idx[i]]);
            std::stable_sort(nw.begin(), nw.end(), [](auto& a, auto& b) { return a.logit > b.logit; });
            cur.swap(nw);
            break;
        }
        case SamplingType::Top_P: {
            if (P.topP >= 1.0f) break;
            softmax(cur);
            float cum = 0.0f;
            size_t last = cur.size();
            for (size_t i = 0; i < cur.size(); ++i) {
                cum += cur[i].p;
                if (cum >= P.topP && i + 1 >= min_keep) { last = i + 1; break; }
            }
            cur.resize(last);
            break;
        }
        case SamplingType::Min_P: {
            if (P.minP <= 0.0f || cur.empty()) break;
            const float min_logit = cur[0].logit + std::log(P.minP);
            size_t i = 1;
            for (; i < cur.size(); ++i)
                if (cur[i].logit < min_logit && i >= min_keep) break;
            cur.resize(i);
            break;
        }
        case SamplingType::XTC: {   // llama_sampler_xtc_apply: drop the top choices above threshold
            if (P.xtc.probability <= 0.0f || P.xtc.threshold > 0.5f || cur.size() < 2) break;
            std::uniform_real_distribution<float> u(0.0f, 1.0f);
            if (u(m_xtcRng) > P.xtc.probability) break;
            softmax(cur);
            size_t pos_last = 0;
            for (size_t i = 0; i < cur.size(); ++i) {
                if (cur[i].p >= P.xtc.threshold) pos_last = i;
                else break;
            }
            if (cur.size() - pos_last >= min_keep && pos_last > 0) cur.erase(cur.begin(), cur.begin() + (std::ptrdiff_t)pos_last);
            break;
        }
        case SamplingType::Temperature:
            if (P.tempRange > 0.0f) {   // llama_sampler_temp_ext_apply: entropy-scaled temperature
                if (cur.size() <= 1) break;
                const float min_t = std::max(0.0f, P.temp - P.tempRange), max_t = P.temp + P.tempRange;
                softmax(cur);
                const float max_entropy = -std::log(1.0f / (float)cur.size());
                float entropy = 0.0f;
                for (auto& c : cur)
                    if (c.p > 0.0f) entropy -= c.p * std::log(c.p);
                const float dyn_t = min_t + (max_t - min_t) * std::pow(entropy / max_entropy, P.tempExp);
                for (auto& c : cur) c.logit /= dyn_t;
                break;
            }
            if (P.temp <= 0.0f) {
                cur.resize(1);   // greedy: keep the max (list is sorted)
            } else {
                for (auto& c : cur) c.logit /= P.temp;
            }
            break;
        case SamplingType::Infill: {   // llama_sampler_infill_apply (fill-in-the-middle)
            const Vocab& voc = m_model.vocab();
            softmax(cur);
            float p_txt = 0.0f, p_eog = 0.0f;
            for (auto& c : cur) (voc.isEog(c.id) ? p_eog : p_txt) += c.p;
            if (3 * p_eog * (float)cur.size() > p_txt) {   // end of generation is likely: EOG only
                std::vector<Candidate> nw;
                for (auto& c : cur)
                    if (voc.isEog(c.id)) nw.push_back(c);
                cur.swap(nw);
                break;
            }
            // merge each token into another whose piece it prefixes (the likelier one keeps both)
            std::vector<std::string> piece(cur.size());
            for (size_t i = 0; i < cur.size(); ++i) piece[i] = voc.tokenToString(cur[i].id, false);
            const float NEG = -std::numeric_limits<float>::infinity();
            for (size_t i0 = 0; i0 < cur.size(); ++i0) {
                for (size_t i1 = 0; i1 < cur.size(); ++i1) {
                    if (cur[i0].logit == NEG) break;
                    if (i0 == i1 || cur[i1].logit == NEG) continue;
                    const std::string &a = piece[i0], &b = piece[i1];
                    if (!a.empty() && a.size() <= b.size() && b.compare(0, a.size(), a) == 0) {
                        size_t dst = i0, src = i1;
                        if (cur[i1].p > cur[i0].p) std::swap(dst, src);
                        cur[dst].p += cur[src].p;
                        cur[src].logit = NEG;
                        cur[src].p = 0.0f;
                    }
                }
            }
            // keep EOG and text tokens with p >= 0.2, then text tokens >= 1 / (n_text + 1)
            size_t n_txt = 0;
            float psum = 0.0f;
            std::vector<Candidate> nw;
            for (auto& c : cur) {
                const bool eog = voc.isEog(c.id);
                if (c.p < 0.2f && !eog) continue;
                n_txt += !eog;
                psum += c.p;
                nw.push_back(c);
            }
            if (n_txt == 0) {   // nothing but EOG left: the end-of-turn token
                cur.assign(1, Candidate{voc.eot(), 1.0f, 1.0f});
                break;
            }
            for (auto& c : nw) c.p /= psum;
            const float th = 1.0f / (float)(n_txt + 1);
            cur.clear();
            for (auto& c : nw)
                if (c.p >= th || voc.isEog(c.id)) cur.push_back(c);
            break;
        }
        default: BL_THROW("Unsupported sampler type");
        }
    }
    softmax(cur);
    std::vector<float> p(cur.size());
    for (size_t i = 0; i < cur.size(); ++i) p[i] = cur[i].p;
    std::discrete_distribution<int> dist(p.begin(), p.end());
    return cur[(size_t)dist(m_rng)].id;
}

// Sampler.cpp:47-70: temp, then mirostat (v1: llama_sampler_mirostat_apply with m = 100; v2:
// llama_sampler_mirostat_v2_apply) sampling from its own target surprise mu.
Token Sampler::applyMirostat(std::vector<Candidate>& cur) {
    const Params& P = m_params;
    if (P.temp <= 0.0f) cur.resize(1);
    else for (auto& c : cur) c.logit /= P.temp;
    softmax(cur);
    if (P.mirostat.ver == 1) {
        const int m = 100;
        float sum_ti_bi = 0.0f, sum_ti_sq = 0.0f;
        for (size_t i = 0; i < (size_t)(m - 1) && i + 1 < cur.size(); ++i) {
            const float t_i = std::log((float)(i + 2) / (float)(i + 1));
            const float b_i = std::log(cur[i].p / cur[i + 1].p);
            sum_ti_bi += t_i * b_i;
            sum_ti_sq += t_i * t_i;
        }
        const float s_hat = sum_ti_bi / sum_ti_sq;
        const float eps_hat = s_hat - 1;
        const float n_vocab = (float)mi_model_n_vocab(m_model.mmodel());
        const float k = std::pow((eps_hat * std::pow(2.0f, m_mu)) / (1 - std::pow(n_vocab, -eps_hat)), 1 / s_hat);
        // int(k) as llama.cpp converts it on x86: out of range or NaN gives INT_MIN, so top-1
        const int ki = (k >= -2147483648.0f && k < 2147483648.0f) ? (int)k : INT32_MIN;
        cur.resize(std::min(cur.size(), (size_t)std::max(ki, 1)));
    } else {
        size_t keep = 0;
        while (keep < cur.size() && !(-std::log2(cur[keep].p) > m_mu)) ++keep;
        cur.resize(std::max<size_t>(keep, 1));
    }
    softmax(cur);
    std::vector<float> p(cur.size());
    for (size_t i = 0; i < cur.size(); ++i) p[i] = cur[i].p;
    std::discrete_distribution<int> dist(p.begin(), p.end());
    const size_t idx = (size_t)dist(m_rng);
    const float observed = -std::log2(cur[idx].p);
    m_mu = m_mu - P.mirostat.eta * (observed - P.mirostat.tau);
    return cur[idx].id;
}

Token Sampler::sample(mi_ctx* ctx, int idx, bool grammarFirst) {
    if (m_grammar && grammarFirst) return sampleGrammarFirst(ctx, idx);
    const Token id = sampleChain(ctx, idx);
    if (!m_grammar || m_grammar->allows(m_model.vocab(), id)) return id;
    // resampling: the grammar on the whole vocabulary first, then the chain (Sampler.cpp:158-172)
    return sampleGrammarFirst(ctx, idx);
}

Token Sampler::sampleGrammarFirst(mi_ctx* ctx, int idx) {
    const float* lg = mi_logits(ctx, idx);
    if (!lg) BL_THROW("sampling: " << last_error());
    const int32_t n = mi_model_n_vocab(m_model.mmodel());
    std::vector<int32_t> ids((size_t)n);
    std::vector<float> v(lg, lg + n);
    for (int32_t i = 0; i < n; ++i) ids[(size_t)i] = i;
    m_grammar->apply(m_model.vocab(), ids.data(), v.data(), (size_t)n);
    std::vector<Candidate> cur((size_t)n);
    bool any = false;
    for (int32_t i = 0; i < n; ++i) {
        cur[(size_t)i] = {i, v[(size_t)i], 0.0f};
        any = any || v[(size_t)i] != -INFINITY;
    }
    if (!any) BL_THROW("no selected token during re-sampling - check your sampling configuration");
    std::stable_sort(cur.begin(), cur.end(), [](auto& a, auto& b) { return a.logit > b.logit; });
    return applyChain(cur);
}

Token Sampler::sampleChain(mi_ctx* ctx, int idx) {
    std::vector<Candidate> cur;
    // The GPU top-k may stand in for the vocabulary only when nothing before top_k in the chain
    // (logit_bias, penalties: Sampler.cpp:30-41) can move a token across the top-k boundary.
    const auto& rp = m_params.repetitionPenalty;
    const bool penalties = rp.numTokens != 0 && !(rp.repeat == 1.0f && rp.freq == 0.0f && rp.present == 0.0f);
    if (m_params.mirostat.ver == 0 && m_params.topK > 0 && m_params.topK <= 64 && m_params.samplerSequence.size() &&
        m_params.samplerSequence[0] == SamplingType::Top_K && m_params.logitBias.empty() && !penalties) {
        const int k = m_params.topK;
        std::vector<int32_t> ids(k);
        std::vector<float> lg(k);
        if (mi_topk(ctx, idx, k, ids.data(), lg.data()) < 0) BL_THROW("sampling: " << last_error());
        for (int i = 0; i < k; ++i) cur.push_back({ids[i], lg[i], 0.0f});
    } else {   // full vocabulary: the chain does not start with a top-k the engine can serve
        const float* lg = mi_logits(ctx, idx);
        if (!lg) BL_THROW("sampling: " << last_error());
        const int32_t n = mi_model_n_vocab(m_model.mmodel());
        cur.resize((size_t)n);
        for (int32_t i = 0; i < n; ++i) cur[(size_t)i] = {i, lg[i], 0.0f};
        std::stable_sort(cur.begin(), cur.end(), [](auto& a, auto& b) { return a.logit > b.logit; });
    }
    if (cur.empty()) BL_THROW("no selected token during sampling - check your sampling configuration");
    return applyChain(cur);
}

// --------------------------------------------------------------- Instance ---
Instance::Instance(Model& model, InitParams params) : m_model(model) {
    m_ctx = mi_ctx_create(model.mmodel(), params.ctxSize, params.batchSize, params.ubatchSize);
    if (!m_ctx) BL_THROW("Failed to create llama context");
}

Instance::~Instance() {
    m_session.reset();
    if (m_ctx) mi_ctx_free(m_ctx);
}

void Instance::warmup() {
    std::vector<Token> t;
    if (m_model.vocab().bos() >= 0) t.push_back(m_model.vocab().bos());
    if (m_model.vocab().eos() >= 0) t.push_back(m_model.vocab().eos());
    if (t.empty()) t.push_back(0);
    mi_decode(m_ctx, t.data(), (int32_t)t.size(), MI_OUT_LAST);
    mi_kv_clear(m_ctx);
    mi_synchronize(m_ctx);
}

Session& Instance::startSession(const Session::InitParams params) {
    if (m_session.has_value()) BL_THROW("Session is already started. Stop it to start a new one.");
    m_session.emplace(*this, m_ctx, params);
    return *m_session;
}

void Instance::stopSession() noexcept { m_session.reset(); }

// ---------------------------------------------------------------- Session ---
Session::Session(Instance& instance, mi_ctx* ctx, InitParams params)
    : m_instance(instance), m_ctx(ctx), m_params(std::move(params)) {
    Sampler::Params sp;
    sp.rngSeed = m_params.seed;
    sp.topP = m_params.topP;
    sp.temp = m_params.temperature;
    sp.grammar = m_params.grammar;
    m_sampler = std::make_unique<Sampler>(instance.model(), sp);
    mi_kv_clear(m_ctx);
    mi_synchronize(m_ctx);
    m_state.maxTokens = mi_n_ctx(m_ctx) - 4;
}

Session::~Session() {
    try {
        flushPendingState();
    } catch (...) {
    }
}

void Session::setInitialPrompt(std::span<const Token> prompt) {
    if (m_state.m_phase != State::Phase::Initial) BL_THROW("Session already started");
    Token only = Token_Invalid;
    m_state.numKeep = std::min<uint32_t>((uint32_t)prompt.size(), m_state.maxTokens);
    if (prompt.empty()) {
        only = m_instance.model().vocab().bos();
        prompt = {&only, 1};
    }
    if (prompt.size() > m_state.maxTokens)
        BL_THROW("Initial prompt too long. Got " << prompt.size() << " tokens, max: " << mi_n_ctx(m_ctx) - 4);
    if (m_params.gaFactor != 1 && m_params.gaWidth % m_params.gaFactor != 0)
        BL_THROW("Group-attention width " << m_params.gaWidth << " must be a multiple of group-attention factor "
                                          << m_params.gaFactor);
    doDecode(prompt, Source::InitialPrompt);
    m_state.m_phase = State::Phase::Generating;
}

void Session::pushPrompt(std::span<const Token> prompt, std::span<const Token> postfix) {
    if (m_state.m_phase != State::Phase::Generating) BL_THROW("Session hasn't started yet");
    flushPendingState();
    if (prompt.empty() && postfix.empty()) BL_THROW("Prompt and postfix are empty");
    m_sampler->reset();
    std::vector<Token> toks;
    const Vocab& voc = m_instance.model().vocab();
    if (m_instance.model().prefixInputsWithBos()) toks.push_back(voc.bos());
    // a postfix is framed by the FIM tokens (Session.cpp:142-159); a model without one of them
    // skips it (the reference logs a warning there)
    auto add = [&](Token t) { if (t >= 0) toks.push_back(t); };
    if (!postfix.empty()) add(voc.fimPre());
    toks.insert(toks.end(), prompt.begin(), prompt.end());
    if (!postfix.empty()) {
        add(voc.fimSuf());
        toks.insert(toks.end(), postfix.begin(), postfix.end());
        add(voc.fimMid());
    }
    if (toks.size() > m_state.maxTokens)
        BL_THROW("Prompt too long. Got " << toks.size() << " tokens, max: " << mi_n_ctx(m_ctx) - 4);
    doDecode(toks, Source::InteractivePrompt);
}

TokenPrediction Session::getToken() {
    if (m_state.m_phase != State::Phase::Generating && m_state.m_phase != State::Phase::Streaming)
        BL_THROW("Session hasn't started yet");
    flushPendingState();
    m_state.m_currToken = m_sampler->sample(m_ctx);
    if (m_instance.model().vocab().isEog(m_state.m_currToken)) m_state.m_currToken = Token_Invalid;
    TokenPrediction p;
    p.token = m_state.m_currToken;
    p.logits = getLogitsFromCtx(10);
    return p;
}

std::vector<TokenPrediction> Session::complete(CompleteParams params) {
    if (m_state.m_phase != State::Phase::Generating) BL_THROW("Session hasn't started yet");
    flushPendingState();
    if (!params.prompt.empty() || !params.suffix.empty()) pushPrompt(params.prompt, params.suffix);
    std::vector<TokenPrediction> out;
    for (int32_t i = 0; i < params.maxTokens; ++i) {
        TokenPrediction p = getToken();
        if (p.token == Token_Invalid) break;
        out.push_back(std::move(p));
    }
    return out;
}

Session::StreamGenerator Session::completeStream(CompleteParams params) {
    if (m_state.m_phase != State::Phase::Generating) BL_THROW("Session hasn't started yet");
    flushPendingState();
    if (!params.prompt.empty() || !params.suffix.empty()) pushPrompt(params.prompt, params.suffix);
    m_state.m_phase = State::Phase::Streaming;
    return StreamGenerator(*this, params);
}

TokenPrediction Session::StreamGenerator::complete() {
    if (m_session.m_state.m_phase != State::Phase::Streaming || m_status != Status::InProgress) return {};
    TokenPrediction p = m_session.getToken();
    if (p.token == Token_Invalid || ++m_genTokens >= m_params.maxTokens) {
        m_session.m_state.m_phase = State::Phase::Generating;
        m_status = Status::Completed;
    }
    return p;
}

std::vector<TokenPrediction> Session::fillCtx(std::span<TokenPrediction> tokens) {
    std::vector<TokenPrediction> out;
    out.reserve(tokens.size());
    // Batched verification: the reference pushes the claimed tokens one decode at a time
    // (Session.cpp:231-244).  When no context shift or Self-Extend step can fall inside the
    // run, the same tokens go through mi_decode(MI_OUT_ALL) in n_batch chunks and row i holds
    // the distribution after token i -- what the i-th single-token decode leaves behind.
    // Only with InitParams::batchedVerify (the serial loop below is bit-identical to generation).
    requireGenerating();
    flushPendingState();
    const uint32_t n = (uint32_t)tokens.size();
    const uint32_t batch = mi_n_batch(m_ctx);
    // Not with prefixInputsWithBos: the serial loop's pushPrompt decodes a BOS before every
    // claimed token, which changes every position after the first.
    if (m_params.batchedVerify && n > 0 && m_params.gaFactor == 1 && m_state.numPast + n < mi_n_ctx(m_ctx) &&
        batch > 0 && !m_instance.model().prefixInputsWithBos()) {
        // the sampler ends as the serial loop leaves it: pushPrompt resets it (RNG re-seeded,
        // penalty window and mirostat state cleared) before each token, so only the last
        // claimed token is in its history (Session.cpp:123)
        m_sampler->reset();
        m_sampler->accept(tokens[n - 1].token, false);
        for (uint32_t c0 = 0; c0 < n; c0 += batch) {
            const uint32_t nc = std::min(batch, n - c0);
            std::vector<Token> ids(nc);
            for (uint32_t i = 0; i < nc; ++i) ids[i] = tokens[c0 + i].token;
            if (mi_decode(m_ctx, ids.data(), (int32_t)nc, MI_OUT_ALL) != 0) BL_THROW("Failed to decode tokens");
            m_state.numPast += nc;
            // every row's claimed ids (each once, in id order, as the reference's vocabulary scan
            // yields them) in one gather: rows padded to the longest list with their first id
            std::vector<std::vector<int32_t>> rid(nc);
            size_t k = 0;
            for (uint32_t i = 0; i < nc; ++i) {
                for (const TokenData& t : tokens[c0 + i].logits)
                    if (t.token >= 0 && t.token < m_instance.model().vocab().nTokens()) rid[i].push_back(t.token);
                std::sort(rid[i].begin(), rid[i].end());
                rid[i].erase(std::unique(rid[i].begin(), rid[i].end()), rid[i].end());
                k = std::max(k, rid[i].size());
            }
            std::vector<int32_t> flat(nc * k, 0);
            for (uint32_t i = 0; i < nc; ++i)
                for (size_t j = 0; j < k; ++j) flat[i * k + j] = rid[i].empty() ? 0 : rid[i][std::min(j, rid[i].size() - 1)];
            std::vector<float> lg(flat.size());
            if (k > 0 && mi_gather_rows(m_ctx, 0, (int32_t)nc, flat.data(), (int32_t)k, lg.data()) < 0)
                BL_THROW("gather: " << last_error());
            for (uint32_t i = 0; i < nc; ++i) {
                TokenPrediction r;
                r.token = tokens[c0 + i].token;
                r.logits.resize(rid[i].size());
                for (size_t j = 0; j < rid[i].size(); ++j) r.logits[j] = {rid[i][j], lg[i * k + j]};
                std::stable_sort(r.logits.begin(), r.logits.end(),
                                 [](const TokenData& a, const TokenData& b) { return a.logit > b.logit; });
                out.push_back(std::move(r));
            }
        }
        return out;
    }
    for (const TokenPrediction& t : tokens) {
        pushPrompt({&t.token, 1}, {});
        TokenPrediction r;
        r.token = t.token;
        r.logits = getLogitsFromCtx(t.logits);
        out.push_back(std::move(r));
    }
    return out;
}

void Session::requireGenerating() const {
    if (m_state.m_phase != State::Phase::Generating && m_state.m_phase != State::Phase::Streaming)
        BL_THROW("Session hasn't started yet");
}

TokenDataVector Session::getLogitsFromCtx(int32_t topK) {
    requireGenerating();
    flushPendingState();
    // GPU top-k in place of the full-vocabulary host copy + std::sort (Session.cpp:246-261)
    std::vector<int32_t> ids(topK);
    std::vector<float> lg(topK);
    if (mi_topk(m_ctx, -1, topK, ids.data(), lg.data()) < 0) BL_THROW("top-k: " << last_error());
    TokenDataVector r(topK);
    for (int32_t i = 0; i < topK; ++i) r[i] = {ids[i], lg[i]};
    return r;
}

TokenDataVector Session::getLogitsFromCtx(const TokenDataVector& tokens, int32_t row) {
    requireGenerating();
    flushPendingState();
    // the reference scans the vocabulary in id order keeping ids in `tokens`: each id once
    std::vector<int32_t> ids;
    for (const TokenData& t : tokens)
        if (t.token >= 0 && t.token < m_instance.model().vocab().nTokens()) ids.push_back(t.token);
    std::sort(ids.begin(), ids.end());
    ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
    std::vector<float> lg(ids.size());
    if (!ids.empty() && mi_gather(m_ctx, row, ids.data(), (int32_t)ids.size(), lg.data()) < 0)
        BL_THROW("gather: " << last_error());
    TokenDataVector r(ids.size());
    for (size_t i = 0; i < ids.size(); ++i) r[i] = {ids[i], lg[i]};
    std::stable_sort(r.begin(), r.end(), [](const TokenData& a, const TokenData& b) { return a.logit > b.logit; });
    return r;
}

std::vector<uint8_t> Session::getState() {
    if (m_state.m_phase != State::Phase::Generating) BL_THROW("Session hasn't started yet");
    flushPendingState();
    const size_t n = mi_state_size(m_ctx);
    std::vector<uint8_t> st(n);
    if (mi_state_get(m_ctx, st.data(), n) != n) BL_THROW("Failed to get state");
    return st;
}

bool Session::setState(std::span<uint8_t> state) {
    if (m_state.m_phase != State::Phase::Initial) BL_THROW("Session already started");
    if (mi_state_set(m_ctx, state.data(), state.size()) != state.size()) BL_THROW("Failed to set state");
    m_state.m_phase = State::Phase::Generating;
    return true;
}

void Session::doDecode(std::span<const Token> tokens, Source src) {
    if (tokens.size() > m_state.maxTokens) tokens = tokens.first(m_state.maxTokens);
    const uint32_t ctxLen = mi_n_ctx(m_ctx);
    if (m_params.gaFactor == 1) {
        // context shift: keep numKeep, drop half of the rest, slide the tail down (K re-rotated)
        if (m_state.numPast + tokens.size() >= ctxLen) {
            if (!m_params.infiniteContext) BL_THROW("context limit of " << ctxLen << " reached");
            const uint32_t numLeft = m_state.numPast - m_state.numKeep;
            const int numDiscard = (int)(numLeft / 2);
            mi_kv_seq_rm(m_ctx, (int32_t)m_state.numKeep, (int32_t)(m_state.numKeep + numDiscard));
            mi_kv_seq_add(m_ctx, (int32_t)(m_state.numKeep + numDiscard), (int32_t)m_state.numPast, -numDiscard);
            m_state.numPast -= (uint32_t)numDiscard;
        }
    } else {
        // Self-Extend group attention
        const uint32_t gaFactor = m_params.gaFactor, gaWidth = m_params.gaWidth;
        while (m_state.numPast >= m_state.gaIndex + gaWidth) {
            const int ib = (int)((gaFactor * m_state.gaIndex) / gaWidth);
            const int bd = (int)((gaWidth / gaFactor) * (gaFactor - 1));
            const int dd = (int)(gaWidth / gaFactor) - ib * bd - (int)gaWidth;
            const int gi = (int)m_state.gaIndex;
            mi_kv_seq_add(m_ctx, gi, (int32_t)m_state.numPast, ib * bd);
            mi_kv_seq_div(m_ctx, gi + ib * bd, gi + ib * bd + (int)gaWidth, (int)gaFactor);
            mi_kv_seq_add(m_ctx, gi + ib * bd + (int)gaWidth, (int32_t)m_state.numPast + ib * bd, dd);
            m_state.numPast -= (uint32_t)bd;
            m_state.gaIndex += gaWidth / gaFactor;
        }
    }
    for (Token t : tokens) m_sampler->accept(t, src == Source::Generated);
    const uint32_t batch = mi_n_batch(m_ctx);
    while (!tokens.empty()) {
        auto b = tokens.size() > batch ? tokens.first(batch) : tokens;
        tokens = tokens.subspan(b.size());
        if (mi_decode(m_ctx, b.data(), (int32_t)b.size(), MI_OUT_LAST) != 0) BL_THROW("Failed to decode tokens");
        m_state.numPast += (uint32_t)b.size();
    }
}

void Session::flushPendingState() {
    if (m_state.m_currToken != Token_Invalid) {
        const Token t = m_state.m_currToken;
        m_state.m_currToken = Token_Invalid;
        doDecode({&t, 1}, Source::Generated);
    }
}

void Session::resetSampler(const Sampler::Params& params) {
    m_sampler = std::make_unique<Sampler>(m_instance.model(), params);
}

// ---------------------------------------------------------- LogitComparer ---
namespace {
// softmax over a list sorted desc: its first logit is the max (LogitComparer.cpp:8-28)
std::unordered_map<Token, float> probs(const TokenDataVector& d) {
    std::unordered_map<Token, float> r(d.size());
    const float top = d[0].logit;
    float z = 0.0f;
    for (const TokenData& t : d) {
        const float e = std::exp(t.logit - top);
        r[t.token] = e;
        z += e;
    }
    for (auto& kv : r) kv.second /= z;
    return r;
}
float sum_sq(const TokenData* d, size_t n) {
    float s = 0.0f;
    for (size_t i = 0; i < n; ++i) s += d[i].logit * d[i].logit;
    return s;
}
float kl_to(const std::unordered_map<Token, float>& P, const std::unordered_map<Token, float>& M) {
    float kl = 0.0f;
    for (const auto& [tok, p] : P) {
        auto it = M.find(tok);
        if (p > 0.0f && it != M.end() && it->second > 0.0f) kl += p * std::log(p / it->second);
    }
    return kl;
}
}  // namespace

ComparisonMetrics LogitComparer::compare(const TokenDataVector& a, const TokenDataVector& b) {
    // the reference reads a[0]/b[0] unchecked (LogitComparer.cpp:39-55); this server faces the
    // network, so an empty list is an error, not undefined behaviour
    if (a.empty() || b.empty()) throw std::runtime_error("LogitComparer: empty logits");
    ComparisonMetrics m;
    m.top1Match = a[0].token == b[0].token ? 1.0f : 0.0f;
    const size_t n = std::min(a.size(), b.size());
    const float da = sum_sq(a.data(), n), db = sum_sq(b.data(), n);
    m.distance = std::fabs(da - db) / std::max(da, db);
    const auto pa = probs(a), pb = probs(b);
    std::unordered_map<Token, float> mid;   // Jensen-Shannon over the shared ids, natural log
    for (const auto& [tok, p] : pa) {
        auto it = pb.find(tok);
        if (it != pb.end()) mid[tok] = (p + it->second) / 2.0f;
    }
    m.jsd = (kl_to(pa, mid) + kl_to(pb, mid)) / 2.0f;
    return m;
}

float LogitComparer::logitSimilarity(const TokenDataVector& a, const TokenDataVector& b) {
    std::unordered_map<Token, float> lb;
    for (const TokenData& t : b) lb[t.token] = t.logit;
    float num = 0.0f, den = 0.0f;
    for (const TokenData& t : a) {
        const float w = std::fabs(t.logit);
        float sim = 0.0f;
        auto it = lb.find(t.token);
        if (it != lb.end()) sim = 1.0f - std::fabs(t.logit - it->second) / std::fabs(std::max(t.logit, it->second));
        num += w * sim;
        den += w;
    }
    return den > 0.0f ? num / den : 0.0f;
}

float MetricsAggregator::pushAndVerify(std::span<const ComparisonMetrics> m) {
    metrics.insert(metrics.end(), m.begin(), m.end());
    double total = 0.0;
    for (const ComparisonMetrics& x : metrics) total += 0.5 * (1.0f - x.distance) + 0.5 * (1.0f - x.jsd);
    return float(total / metrics.size());
}

}  // namespace bl::llama
