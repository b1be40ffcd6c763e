// GBNF grammar-constrained sampling for the bl::llama Sampler.
//
// The reference builds `llama_sampler_init_grammar(vocab, params.grammar, "root")` and, per
// sampled token, checks it against the grammar and resamples with the grammar applied first on
// a rejection (inference/code/llama/Sampler.cpp:16, 126-173); generated tokens advance the
// grammar (Sampler.cpp:100-106, Session.cpp:374-377).  The arithmetic lives in llama.cpp b5187
// (src/llama-grammar.cpp, not vendored): this file restates its published algorithm --
//   * the GBNF parser (llama_grammar_parser): rules `name ::= alternates`, literals with \x \u \U
//     \t \r \n escapes, character classes [..] / [^..] with ranges, `.`, groups, rule references,
//     comments, and the repetition rewrites of *, +, ?, {m}, {m,}, {m,n} into generated rules;
//   * undefined-rule, missing-root and left-recursion checks;
//   * the pushdown recogniser: a set of element stacks advanced over rule references
//     (llama_grammar_advance_stack), one code point at a time (llama_grammar_accept), with the
//     partial-UTF-8 state carried across tokens (decode_utf8, llama_grammar_match_partial_char);
//   * the candidate filter (llama_grammar_apply_impl): an end-of-generation token is allowed only
//     when some stack is empty, an empty piece never, any other token iff some stack can consume
//     all of its code points (and the trailing partial sequence can still match).
// Parity is unpinned (llama.cpp is not vendored; tests/cpp/t_bl_llama.cpp "grammar" checks the
// language each construct defines).
#pragma once
#include <cstdint>
#include <map>
#include <string>
#include <vector>

namespace bl::llama {

class Vocab;

class Grammar {
public:
    enum ElemType : uint8_t {   // llama_gretype
        END = 0, ALT = 1, RULE_REF = 2, CHAR = 3, CHAR_NOT = 4, CHAR_RNG_UPPER = 5, CHAR_ALT = 6, CHAR_ANY = 7,
    };
    struct Elem {
        ElemType type;
        uint32_t value;
    };
    struct Partial {            // llama_partial_utf8
        uint32_t value = 0;
        int n_remain = 0;
    };
    using Stack = std::vector<const Elem*>;

    // Parses `text`; throws std::runtime_error on a syntax error, an undefined rule, a missing
    // `root` symbol or left recursion (where llama_sampler_init_grammar gives no grammar).
    Grammar(const std::string& text, const std::string& root = "root");
    Grammar(const Grammar&) = delete;              // stacks point into this object's rules
    Grammar& operator=(const Grammar&) = delete;

    // llama_grammar_apply_impl on (id, logit) pairs: rejected tokens get -INFINITY.
    void apply(const Vocab& vocab, const int32_t* ids, float* logits, size_t n) const;
    // whether one token is allowed now (the Sampler's single-token check, Sampler.cpp:146-156)
    bool allows(const Vocab& vocab, int32_t id) const;
    // llama_grammar_accept_impl: advance over the token's piece; throws if that empties the
    // stacks (and on an end-of-generation token when no stack is complete)
    void accept(const Vocab& vocab, int32_t id);
    void reset();               // back to the initial stacks (llama_sampler_reset)

    // the recogniser on plain text (tests): does the grammar accept `s` as a prefix / whole?
    bool acceptsPrefix(const std::string& s) const;
    bool acceptsComplete(const std::string& s) const;
    size_t nRules() const { return m_rules.size(); }

private:
    std::vector<std::vector<Elem>> m_rules;
    std::map<std::string, uint32_t> m_symbols;
    uint32_t m_root = 0;
    std::vector<Stack> m_initial, m_stacks;
    Partial m_partial;

    void advance(const Stack& st, std::vector<Stack>& out) const;
    std::vector<Stack> acceptChar(const std::vector<Stack>& stacks, uint32_t chr) const;
    bool tokenAllowed(const std::string& piece) const;
};

}  // namespace bl::llama
