// GBNF grammar engine: a restatement of llama.cpp b5187's src/llama-grammar.cpp algorithm
// (see grammar.hpp for the mapping and the reference call sites).
#include "grammar.hpp"

#include "llama.hpp"

#include <algorithm>
#include <cmath>
#include <stdexcept>

namespace bl::llama {

namespace {

using Elem = Grammar::Elem;
using Rule = std::vector<Elem>;

bool end_of_seq(const Elem* p) { return p->type == Grammar::END || p->type == Grammar::ALT; }

// decode_utf8 (llama-grammar.cpp): code points of `src` continuing a partial sequence, the
// terminating 0, and the partial sequence the text ends in
std::pair<std::vector<uint32_t>, Grammar::Partial> decode_utf8(const std::string& src, Grammar::Partial start) {
    static const int lookup[] = {1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 2, 2, 3, 4};
    const char* pos = src.c_str();
    std::vector<uint32_t> cps;
    cps.reserve(src.size() + 1);
    uint32_t value = start.value;
    int n_remain = start.n_remain;
    while (*pos != 0 && n_remain > 0) {   // continue the previous token's sequence
        const uint8_t next = (uint8_t)*pos;
        if ((next >> 6) != 2) {
            cps.push_back(0);
            return {std::move(cps), Grammar::Partial{0, -1}};
        }
        value = (value << 6) + (next & 0x3F);
        ++pos;
        --n_remain;
    }
    if (start.n_remain > 0 && n_remain == 0) cps.push_back(value);
    while (*pos != 0) {
        const uint8_t first = (uint8_t)*pos;
        n_remain = lookup[first >> 4] - 1;
        if (n_remain < 0) {   // invalid sequence
            cps.clear();
            cps.push_back(0);
            return {std::move(cps), Grammar::Partial{0, n_remain}};
        }
        const uint8_t mask = (uint8_t)((1 << (7 - n_remain)) - 1);
        value = first & mask;
        ++pos;
        while (*pos != 0 && n_remain > 0) {
            value = (value << 6) + ((uint8_t)*pos & 0x3F);
            ++pos;
            --n_remain;
        }
        if (n_remain == 0) cps.push_back(value);
    }
    cps.push_back(0);
    return {std::move(cps), Grammar::Partial{value, n_remain}};
}

// llama_grammar_match_char: (matched, element after the char / class)
std::pair<bool, const Elem*> match_char(const Elem* pos, uint32_t chr) {
    bool found = false;
    const bool positive = pos->type == Grammar::CHAR || pos->type == Grammar::CHAR_ANY;
    do {
        if (pos[1].type == Grammar::CHAR_RNG_UPPER) {
            found = found || (pos->value <= chr && chr <= pos[1].value);
            pos += 2;
        } else if (pos->type == Grammar::CHAR_ANY) {
            found = true;
            pos += 1;
        } else {
            found = found || pos->value == chr;
            pos += 1;
        }
    } while (pos->type == Grammar::CHAR_ALT);
    return {found == positive, pos};
}

// llama_grammar_match_partial_char: can the partial sequence still complete to a match?
bool match_partial_char(const Elem* pos, Grammar::Partial partial) {
    const bool positive = pos->type == Grammar::CHAR || pos->type == Grammar::CHAR_ANY;
    const uint32_t pv = partial.value;
    const int n_remain = partial.n_remain;
    if (n_remain < 0 || (n_remain == 1 && pv < 2)) return false;   // invalid, or overlong 7-bit
    uint32_t low = pv << (n_remain * 6);
    const uint32_t high = low | ((1u << (n_remain * 6)) - 1);
    if (low == 0) {
        if (n_remain == 2) low = 1u << 11;
        else if (n_remain == 3) low = 1u << 16;
    }
    do {
        if (pos[1].type == Grammar::CHAR_RNG_UPPER) {
            if (pos->value <= high && low <= pos[1].value) return positive;
            pos += 2;
        } else if (pos->type == Grammar::CHAR_ANY) {
            return true;
        } else {
            if (low <= pos->value && pos->value <= high) return positive;
            pos += 1;
        }
    } while (pos->type == Grammar::CHAR_ALT);
    return !positive;
}

// ---- the parser (llama_grammar_parser) ----
struct Parser {
    std::map<std::string, uint32_t>& symbols;
    std::vector<Rule>& rules;

    static bool is_word(char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || c == '-' || (c >= '0' && c <= '9'); }
    static bool is_digit(char c) { return c >= '0' && c <= '9'; }

    uint32_t symbol_id(const char* s, size_t n) {
        const uint32_t next = (uint32_t)symbols.size();
        return symbols.emplace(std::string(s, n), next).first->second;
    }
    uint32_t generate_symbol(const std::string& base) {
        const uint32_t next = (uint32_t)symbols.size();
        symbols[base + '_' + std::to_string(next)] = next;
        return next;
    }
    void add_rule(uint32_t id, const Rule& r) {
        if (rules.size() <= id) rules.resize(id + 1);
        rules[id] = r;
    }
    static const char* parse_space(const char* p, bool newline_ok) {
        while (*p == ' ' || *p == '\t' || *p == '#' || (newline_ok && (*p == '\r' || *p == '\n'))) {
            if (*p == '#') {
                while (*p && *p != '\r' && *p != '\n') ++p;
            } else {
                ++p;
            }
        }
        return p;
    }
    static const char* parse_name(const char* s) {
        const char* p = s;
        while (is_word(*p)) ++p;
        if (p == s) throw std::runtime_error(std::string("expecting name at ") + s);
        return p;
    }
    static const char* parse_int(const char* s) {
        const char* p = s;
        while (is_digit(*p)) ++p;
        if (p == s) throw std::runtime_error(std::string("expecting integer at ") + s);
        return p;
    }
    static std::pair<uint32_t, const char*> parse_hex(const char* s, int size) {
        const char* p = s;
        const char* end = s + size;
        uint32_t v = 0;
        for (; p < end && *p; ++p) {
            v <<= 4;
            const char c = *p;
            if ('a' <= c && c <= 'f') v += (uint32_t)(c - 'a' + 10);
            else if ('A' <= c && c <= 'F') v += (uint32_t)(c - 'A' + 10);
            else if ('0' <= c && c <= '9') v += (uint32_t)(c - '0');
            else break;
        }
        if (p != end) throw std::runtime_error("expecting " + std::to_string(size) + " hex chars at " + s);
        return {v, p};
    }
    // one code point of plain UTF-8 (the parser's decode_utf8)
    static std::pair<uint32_t, const char*> utf8_one(const char* s) {
        static const int lookup[] = {1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 2, 2, 3, 4};
        const uint8_t first = (uint8_t)*s;
        const int len = lookup[first >> 4];
        const uint8_t mask = (uint8_t)((1 << (8 - len)) - 1);
        uint32_t v = first & mask;
        const char* p = s + 1;
        for (int i = 1; i < len && *p; ++i, ++p) v = (v << 6) + ((uint8_t)*p & 0x3F);
        return {v, p};
    }
    static std::pair<uint32_t, const char*> parse_char(const char* s) {
        if (*s == '\\') {
            switch (s[1]) {
            case 'x': return parse_hex(s + 2, 2);
            case 'u': return parse_hex(s + 2, 4);
            case 'U': return parse_hex(s + 2, 8);
            case 't': return {'\t', s + 2};
            case 'r': return {'\r', s + 2};
            case 'n': return {'\n', s + 2};
            case '\\': case '"': case '[': case ']': return {(uint32_t)(uint8_t)s[1], s + 2};
            default: throw std::runtime_error(std::string("unknown escape at ") + s);
            }
        } else if (*s) {
            return utf8_one(s);
        }
        throw std::runtime_error("unexpected end of input");
    }

    const char* parse_sequence(const char* src, const std::string& rule_name, Rule& out, bool nested) {
        size_t last_sym_start = out.size();
        const char* pos = src;
        // S{m,n} -> S (m times) S'(n-m), S'(k) ::= S S'(k-1) | ; S{m,} -> S (m times) S', S' ::= S S' |
        auto repetitions = [&](int min_times, int max_times) {
            if (last_sym_start == out.size())
                throw std::runtime_error(std::string("expecting preceding item to */+/?/{ at ") + pos);
            const Rule prev(out.begin() + (std::ptrdiff_t)last_sym_start, out.end());
            if (min_times == 0) out.resize(last_sym_start);
            else
                for (int i = 1; i < min_times; ++i) out.insert(out.end(), prev.begin(), prev.end());
            uint32_t last_rec = 0;
            const int n_opt = max_times < 0 ? 1 : max_times - min_times;
            Rule rec(prev);
            for (int i = 0; i < n_opt; ++i) {
                rec.resize(prev.size());
                const uint32_t rec_id = generate_symbol(rule_name);
                if (i > 0 || max_times < 0) rec.push_back({Grammar::RULE_REF, max_times < 0 ? rec_id : last_rec});
                rec.push_back({Grammar::ALT, 0});
                rec.push_back({Grammar::END, 0});
                add_rule(rec_id, rec);
                last_rec = rec_id;
            }
            if (n_opt > 0) out.push_back({Grammar::RULE_REF, last_rec});
        };
        while (*pos) {
            if (*pos == '"') {   // literal
                ++pos;
                last_sym_start = out.size();
                while (*pos != '"') {
                    if (!*pos) throw std::runtime_error("unexpected end of input");
                    auto c = parse_char(pos);
                    pos = c.second;
                    out.push_back({Grammar::CHAR, c.first});
                }
                pos = parse_space(pos + 1, nested);
            } else if (*pos == '[') {   // character class
                ++pos;
                Grammar::ElemType start = Grammar::CHAR;
                if (*pos == '^') {
                    ++pos;
                    start = Grammar::CHAR_NOT;
                }
                last_sym_start = out.size();
                while (*pos != ']') {
                    if (!*pos) throw std::runtime_error("unexpected end of input");
                    auto c = parse_char(pos);
                    pos = c.second;
                    out.push_back({last_sym_start < out.size() ? Grammar::CHAR_ALT : start, c.first});
                    if (pos[0] == '-' && pos[1] != ']') {
                        if (!pos[1]) throw std::runtime_error("unexpected end of input");
                        auto e = parse_char(pos + 1);
                        pos = e.second;
                        out.push_back({Grammar::CHAR_RNG_UPPER, e.first});
                    }
                }
                pos = parse_space(pos + 1, nested);
            } else if (is_word(*pos)) {   // rule reference
                const char* name_end = parse_name(pos);
                const uint32_t ref = symbol_id(pos, (size_t)(name_end - pos));
                pos = parse_space(name_end, nested);
                last_sym_start = out.size();
                out.push_back({Grammar::RULE_REF, ref});
            } else if (*pos == '(') {   // group -> synthesized rule
                pos = parse_space(pos + 1, true);
                const uint32_t sub = generate_symbol(rule_name);
                pos = parse_alternates(pos, rule_name, sub, true);
                last_sym_start = out.size();
                out.push_back({Grammar::RULE_REF, sub});
                if (*pos != ')') throw std::runtime_error(std::string("expecting ')' at ") + pos);
                pos = parse_space(pos + 1, nested);
            } else if (*pos == '.') {
                last_sym_start = out.size();
                out.push_back({Grammar::CHAR_ANY, 0});
                pos = parse_space(pos + 1, nested);
            } else if (*pos == '*') {
                pos = parse_space(pos + 1, nested);
                repetitions(0, -1);
            } else if (*pos == '+') {
                pos = parse_space(pos + 1, nested);
                repetitions(1, -1);
            } else if (*pos == '?') {
                pos = parse_space(pos + 1, nested);
                repetitions(0, 1);
            } else if (*pos == '{') {
                pos = parse_space(pos + 1, nested);
                if (!is_digit(*pos)) throw std::runtime_error(std::string("expecting an int at ") + pos);
                const char* ie = parse_int(pos);
                const int mn = (int)std::stoul(std::string(pos, (size_t)(ie - pos)));
                pos = parse_space(ie, nested);
                int mx = -1;
                if (*pos == '}') {
                    mx = mn;
                    pos = parse_space(pos + 1, nested);
                } else if (*pos == ',') {
                    pos = parse_space(pos + 1, nested);
                    if (is_digit(*pos)) {
                        const char* je = parse_int(pos);
                        mx = (int)std::stoul(std::string(pos, (size_t)(je - pos)));
                        pos = parse_space(je, nested);
                    }
                    if (*pos != '}') throw std::runtime_error(std::string("expecting '}' at ") + pos);
                    pos = parse_space(pos + 1, nested);
                } else {
                    throw std::runtime_error(std::string("expecting ',' at ") + pos);
                }
                repetitions(mn, mx);
            } else {
                break;
            }
        }
        return pos;
    }

    const char* parse_alternates(const char* src, const std::string& rule_name, uint32_t rule_id, bool nested) {
        Rule rule;
        const char* pos = parse_sequence(src, rule_name, rule, nested);
        while (*pos == '|') {
            rule.push_back({Grammar::ALT, 0});
            pos = parse_space(pos + 1, true);
            pos = parse_sequence(pos, rule_name, rule, nested);
        }
        rule.push_back({Grammar::END, 0});
        add_rule(rule_id, rule);
        return pos;
    }

    const char* parse_rule(const char* src) {
        const char* name_end = parse_name(src);
        const char* pos = parse_space(name_end, false);
        const size_t n = (size_t)(name_end - src);
        const uint32_t id = symbol_id(src, n);
        const std::string name(src, n);
        if (!(pos[0] == ':' && pos[1] == ':' && pos[2] == '=')) throw std::runtime_error(std::string("expecting ::= at ") + pos);
        pos = parse_space(pos + 3, true);
        pos = parse_alternates(pos, name, id, false);
        if (*pos == '\r') pos += pos[1] == '\n' ? 2 : 1;
        else if (*pos == '\n') ++pos;
        else if (*pos) throw std::runtime_error(std::string("expecting newline or end at ") + pos);
        return parse_space(pos, true);
    }

    void parse(const char* src) {
        const char* pos = parse_space(src, true);
        while (*pos) pos = parse_rule(pos);
        for (const Rule& r : rules) {
            if (r.empty()) throw std::runtime_error("Undefined rule");
            for (const Elem& e : r)
                if (e.type == Grammar::RULE_REF && (e.value >= rules.size() || rules[e.value].empty())) {
                    for (const auto& kv : symbols)
                        if (kv.second == e.value) throw std::runtime_error("Undefined rule identifier '" + kv.first + "'");
                    throw std::runtime_error("Undefined rule");
                }
        }
    }
};

// llama_grammar_detect_left_recursion
bool left_recursion(const std::vector<Rule>& rules, size_t i, std::vector<bool>& visited, std::vector<bool>& in_progress,
                    std::vector<bool>& may_be_empty) {
    if (in_progress[i]) return true;
    in_progress[i] = true;
    const Rule& rule = rules[i];
    bool at_start = true;
    for (size_t k = 0; k < rule.size(); ++k) {
        if (end_of_seq(&rule[k])) {
            if (at_start) {
                may_be_empty[i] = true;
                break;
            }
            at_start = true;
        } else {
            at_start = false;
        }
    }
    bool recurse = true;
    for (size_t k = 0; k < rule.size(); ++k) {
        if (rule[k].type == Grammar::RULE_REF && recurse) {
            if (left_recursion(rules, rule[k].value, visited, in_progress, may_be_empty)) return true;
            if (!may_be_empty[rule[k].value]) recurse = false;
        } else if (end_of_seq(&rule[k])) {
            recurse = true;
        } else {
            recurse = false;
        }
    }
    in_progress[i] = false;
    visited[i] = true;
    return false;
}

}  // namespace

Grammar::Grammar(const std::string& text, const std::string& root) {
    Parser ps{m_symbols, m_rules};
    try {
        ps.parse(text.c_str());
    } catch (const std::exception& e) {
        throw std::runtime_error(std::string("error parsing grammar: ") + e.what());
    }
    auto it = m_symbols.find(root);
    if (it == m_symbols.end()) throw std::runtime_error("grammar does not contain a '" + root + "' symbol");
    m_root = it->second;
    const size_t n = m_rules.size();
    std::vector<bool> visited(n), in_progress(n), may_be_empty(n);
    for (size_t i = 0; i < n; ++i)
        if (!visited[i] && left_recursion(m_rules, i, visited, in_progress, may_be_empty))
            throw std::runtime_error("unsupported grammar, left recursion detected for nonterminal at index " +
                                     std::to_string(i));
    // one initial stack per alternate of the root rule
    const Elem* pos = m_rules[m_root].data();
    for (;;) {
        Stack st;
        if (!end_of_seq(pos)) st.push_back(pos);
        advance(st, m_initial);
        while (!end_of_seq(pos)) ++pos;
        if (pos->type == ALT) ++pos;
        else break;
    }
    m_stacks = m_initial;
}

// llama_grammar_advance_stack: expand rule references on top of the stack until a character
// element (or nothing) is on top; collect the distinct results
void Grammar::advance(const Stack& st, std::vector<Stack>& out) const {
    if (st.empty()) {
        if (std::find(out.begin(), out.end(), st) == out.end()) out.push_back(st);
        return;
    }
    const Elem* pos = st.back();
    switch (pos->type) {
    case RULE_REF: {
        const Elem* sub = m_rules[pos->value].data();
        do {
            Stack ns(st.begin(), st.end() - 1);
            if (!end_of_seq(pos + 1)) ns.push_back(pos + 1);   // the rest of this sequence
            if (!end_of_seq(sub)) ns.push_back(sub);           // the alternate's first element
            advance(ns, out);
            while (!end_of_seq(sub)) ++sub;
            if (sub->type == ALT) ++sub;
            else break;
        } while (true);
        break;
    }
    case CHAR:
    case CHAR_NOT:
    case CHAR_ANY:
        if (std::find(out.begin(), out.end(), st) == out.end()) out.push_back(st);
        break;
    default:
        throw std::runtime_error("grammar: unexpected element on a stack");
    }
}

// llama_grammar_accept: the stacks after one code point
std::vector<Grammar::Stack> Grammar::acceptChar(const std::vector<Stack>& stacks, uint32_t chr) const {
    std::vector<Stack> out;
    for (const Stack& st : stacks) {
        if (st.empty()) continue;
        auto m = match_char(st.back(), chr);
        if (!m.first) continue;
        Stack ns(st.begin(), st.end() - 1);
        if (!end_of_seq(m.second)) ns.push_back(m.second);
        advance(ns, out);
    }
    return out;
}

// llama_grammar_reject_candidates for one piece: allowed iff some stack consumes every full code
// point and then either ends complete with no partial sequence left, or has a character element
// on top that the partial sequence can still complete to (or there is no partial sequence)
bool Grammar::tokenAllowed(const std::string& piece) const {
    auto dec = decode_utf8(piece, m_partial);
    const std::vector<uint32_t>& cps = dec.first;
    std::vector<Stack> cur = m_stacks;
    for (size_t i = 0; i + 1 < cps.size(); ++i) {
        // a completed stack rejects further code points (reject_candidates_for_stack, empty stack)
        cur = acceptChar(cur, cps[i]);
        if (cur.empty()) return false;
    }
    for (const Stack& st : cur) {
        if (st.empty()) {
            if (dec.second.n_remain == 0) return true;
        } else if (dec.second.n_remain == 0 || match_partial_char(st.back(), dec.second)) {
            return true;
        }
    }
    return false;
}

bool Grammar::allows(const Vocab& vocab, int32_t id) const {
    if (vocab.isEog(id)) {
        for (const Stack& st : m_stacks)
            if (st.empty()) return true;
        return false;
    }
    const std::string piece = vocab.tokenToString(id, true);
    if (piece.empty() || piece[0] == 0) return false;
    return tokenAllowed(piece);
}

void Grammar::apply(const Vocab& vocab, const int32_t* ids, float* logits, size_t n) const {
    for (size_t i = 0; i < n; ++i)
        if (!allows(vocab, ids[i])) logits[i] = -INFINITY;
}

void Grammar::accept(const Vocab& vocab, int32_t id) {
    if (vocab.isEog(id)) {
        for (const Stack& st : m_stacks)
            if (st.empty()) return;
        throw std::runtime_error("grammar: end of generation before the grammar is complete");
    }
    const std::string piece = vocab.tokenToString(id, true);
    auto dec = decode_utf8(piece, m_partial);
    for (size_t i = 0; i + 1 < dec.first.size(); ++i) m_stacks = acceptChar(m_stacks, dec.first[i]);
    m_partial = dec.second;
    if (m_stacks.empty()) throw std::runtime_error("Unexpected empty grammar stack after accepting piece: " + piece);
}

void Grammar::reset() {
    m_stacks = m_initial;
    m_partial = Partial{};
}

bool Grammar::acceptsPrefix(const std::string& s) const {
    auto dec = decode_utf8(s, Partial{});
    std::vector<Stack> cur = m_initial;
    for (size_t i = 0; i + 1 < dec.first.size(); ++i) {
        cur = acceptChar(cur, dec.first[i]);
        if (cur.empty()) return false;
    }
    return true;
}

bool Grammar::acceptsComplete(const std::string& s) const {
    auto dec = decode_utf8(s, Partial{});
    std::vector<Stack> cur = m_initial;
    for (size_t i = 0; i + 1 < dec.first.size(); ++i) {
        cur = acceptChar(cur, dec.first[i]);
        if (cur.empty()) return false;
    }
    for (const Stack& st : cur)
        if (st.empty()) return true;
    return false;
}

}  // namespace bl::llama
