// Tests of the bl::llama host surface (blama_amd/host) in the shape of the reference's own tests:
// inference/test/t-LogitComparer.cpp and t-integration.cpp.  Models are synthetic GGUFs written
// by the pytest wrapper (tests/test_host.py), so the reference's gpt2 text KATs (" Bush", ...)
// become token-level checks.
//
// usage: t_bl_llama [cpu] [gpu] --model=<gguf> --vocab=<gguf> --out=<file>
#include "llama.hpp"
#include "mi_engine.h"
#include "minitest.hpp"
#include "server.hpp"
#include "wire.hpp"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <future>
#include <unordered_set>

namespace {
std::string g_model, g_vocab, g_out, g_in;
void setup(int argc, char** argv, std::vector<std::string>& groups) {
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        if (a.rfind("--model=", 0) == 0) g_model = a.substr(8);
        else if (a.rfind("--vocab=", 0) == 0) g_vocab = a.substr(8);
        else if (a.rfind("--out=", 0) == 0) g_out = a.substr(6);
        else if (a.rfind("--in=", 0) == 0) g_in = a.substr(5);
        else groups.push_back(a);
    }
}
using namespace bl::llama;
const std::vector<Token> kPrompt = {1, 300, 301, 302, 303, 400, 77, 5};
}  // namespace

// ---------------------------------------------------------------- CPU ----
TEST_CASE_G("compare - no model", "cpu") {   // t-LogitComparer.cpp:13-39
    TokenDataVector tdv1, tdv2;
    float logitValue = 17.5f;
    for (int32_t i = 0; i < 10; i++) {
        tdv1.push_back({i, logitValue});
        tdv2.push_back({i, logitValue});
        logitValue -= 0.5f;
    }
    CHECK(LogitComparer::logitSimilarity(tdv1, tdv2) == 1.0f);
    auto metrics = LogitComparer::compare(tdv1, tdv2);
    CHECK(metrics.top1Match == 1.0f);
    CHECK(metrics.distance == 0.0f);
    CHECK(metrics.jsd == 0.0f);
    MetricsAggregator agg;
    CHECK(agg.pushAndVerify({&metrics, 1}) == 1.0f);
}

TEST_CASE_G("compare - perturbed", "cpu") {
    TokenDataVector a, b;
    for (int32_t i = 0; i < 10; i++) {
        a.push_back({i, 12.0f - i});
        b.push_back({i == 0 ? 1 : i == 1 ? 0 : i, 12.0f - i + (i == 3 ? 0.25f : 0.0f)});
    }
    auto m = LogitComparer::compare(a, b);
    CHECK(m.top1Match == 0.0f);   // ids 0 and 1 swapped at the top
    CHECK(m.distance > 0.0f && m.distance < 0.01f);
    CHECK(m.jsd > 0.0f && m.jsd < 0.2f);
    const float sim = LogitComparer::logitSimilarity(a, b);
    CHECK(sim < 1.0f && sim > 0.9f);
    MetricsAggregator agg;
    const float s1 = agg.pushAndVerify({&m, 1});
    auto same = LogitComparer::compare(a, a);
    const float s2 = agg.pushAndVerify({&same, 1});   // running mean over both steps
    CHECK(s2 > s1 && s2 < 1.0f);
}

TEST_CASE_G("sampler chain", "cpu") {
    REQUIRE(!g_vocab.empty());
    Model model(g_vocab, {.vocabOnly = true});
    auto make = [](std::vector<Sampler::Candidate>& c) {
        c.clear();
        for (int i = 0; i < 40; ++i) c.push_back({100 + i, 8.0f - 0.25f * i, 0.0f});
    };
    std::vector<Sampler::Candidate> c;
    Sampler::Params greedy;
    greedy.temp = 0.0f;
    Sampler g(model, greedy);
    make(c);
    CHECK(g.applyChain(c) == 100);                  // temp <= 0: the top candidate
    Sampler::Params p;
    p.rngSeed = 1234;
    Sampler s1(model, p), s2(model, p);
    std::vector<Token> a, b;
    for (int i = 0; i < 16; ++i) {
        make(c); a.push_back(s1.applyChain(c));
        make(c); b.push_back(s2.applyChain(c));
    }
    CHECK(a == b);                                  // same seed, same draws
    s1.reset();
    std::vector<Token> a2;
    for (int i = 0; i < 16; ++i) { make(c); a2.push_back(s1.applyChain(c)); }
    CHECK(a2 == a);                                 // reset re-seeds (pushPrompt semantics)
    for (Token t : a) CHECK(t >= 100 && t < 140);
    // min_p 0.05 at temp 1 keeps logits >= top + ln 0.05 = top - 3.0: at most 13 candidates
    Sampler::Params q;
    q.temp = 1.0f;
    q.topP = 1.0f;
    Sampler s3(model, q);
    int maxid = 0;
    for (int i = 0; i < 400; ++i) { make(c); maxid = std::max(maxid, s3.applyChain(c) - 100); }
    CHECK(maxid <= 12);
}

// The stages after the reference's default chain (Sampler.cpp:47-95): mirostat v1/v2, typical_p,
// dynamic temperature, XTC.  Parity unpinned (llama.cpp is not vendored in the reference); these
// check each stage's defining property on a geometric candidate list.
TEST_CASE_G("sampler stages", "cpu") {
    REQUIRE(!g_vocab.empty());
    Model model(g_vocab, {.vocabOnly = true});
    auto make = [](std::vector<Sampler::Candidate>& c, float step) {
        c.clear();
        for (int i = 0; i < 40; ++i) c.push_back({100 + i, 8.0f - step * i, 0.0f});
    };
    std::vector<Sampler::Candidate> c;
    auto draws = [&](const Sampler::Params& p, float step, int n) {
        Sampler s(model, p);
        std::vector<Token> out;
        for (int i = 0; i < n; ++i) { make(c, step); out.push_back(s.applyChain(c) - 100); }
        return out;
    };
    auto distinct = [](const std::vector<Token>& v) {
        return (int)std::unordered_set<Token>(v.begin(), v.end()).size();
    };
    Sampler::Params base;
    base.rngSeed = 7;
    base.temp = 1.0f;
    base.topK = 0;
    base.topP = 1.0f;
    base.minP = 0.0f;
    // XTC always on, threshold 0.1: at step 0.25 the top four have p >= 0.1 (0.221 .. 0.104),
    // so the first three are removed and nothing below id 3 is ever drawn
    {
        Sampler::Params p = base;
        p.samplerSequence = {Sampler::SamplingType::XTC, Sampler::SamplingType::Temperature};
        p.xtc = {1.0f, 0.1f};
        auto v = draws(p, 0.25f, 300);
        CHECK(*std::min_element(v.begin(), v.end()) == 3);
        p.xtc = {1.0f, 0.6f};   // threshold > 0.5 disables
        v = draws(p, 0.25f, 300);
        CHECK(*std::min_element(v.begin(), v.end()) == 0);
    }
    // mirostat: a low target surprise keeps the draws near the top, a high one spreads them;
    // the same seed repeats the same draws (mu restarts at 2 tau)
    for (int ver : {1, 2}) {
        Sampler::Params p = base;
        p.mirostat = {ver, 1.0f, 0.1f};
        auto lo = draws(p, 0.25f, 300);
        CHECK(lo == draws(p, 0.25f, 300));
        // v1's k = (eps 2^mu / (1 - n_vocab^-eps))^(1/s) leaves int range for a large mu, and
        // the x86 conversion then gives top-1 (as llama.cpp's int(k) does): tau 5 keeps k finite
        p.mirostat.tau = ver == 1 ? 5.0f : 10.0f;
        auto hi = draws(p, 0.1f, 300);   // flatter list: the full 40 are in reach
        CHECK(*std::max_element(lo.begin(), lo.end()) <= 8);
        CHECK(distinct(hi) >= 15);
    }
    {
        Sampler::Params p = base;
        p.mirostat.ver = 3;
        CHECK_THROWS(Sampler(model, p));
    }
    // typical_p with min_keep 0 never cuts (llama.cpp's size_t min_keep - 1); with min_keep 1 it
    // keeps the candidates whose surprise is nearest the entropy, which excludes the top one here
    {
        Sampler::Params p = base;
        auto ref = draws(p, 0.25f, 200);
        p.typicalP = 0.3f;
        CHECK(draws(p, 0.25f, 200) == ref);
        p.minKeep = 1;
        auto v = draws(p, 0.25f, 200);
        CHECK(v != ref);
        CHECK(std::count(v.begin(), v.end(), 0) == 0);
    }
    // dynamic temperature: temp 0.5 +- 0.5 on a peaked list (low entropy) is near greedy; on a
    // flat list (normalised entropy 1) it is temp 1 over all 40
    {
        Sampler::Params p = base;
        p.temp = 0.5f;
        p.tempRange = 0.5f;
        auto peaked = draws(p, 3.0f, 200);
        CHECK(std::count(peaked.begin(), peaked.end(), 0) == 200);
        CHECK(distinct(draws(p, 0.0f, 400)) >= 30);
    }
    // infill: a token absorbs the tokens its piece prefixes, text below 0.2 is dropped, and a
    // likely end of generation leaves only the EOG tokens
    {
        const Vocab& voc = model.vocab();
        Token a = -1, b = -1;
        std::vector<Token> text;
        for (Token i = 0; i < voc.nTokens(); ++i) {
            const std::string s = voc.tokenToString(i, false);
            if (s.empty() || voc.isEog(i)) continue;
            text.push_back(i);
        }
        for (Token i : text)
            for (Token j : text) {
                const std::string si = voc.tokenToString(i, false), sj = voc.tokenToString(j, false);
                if (a < 0 && i != j && si.size() >= 2 && si.size() < sj.size() && sj.compare(0, si.size(), si) == 0) {
                    a = i;
                    b = j;
                }
            }
        REQUIRE(a >= 0 && voc.eos() >= 0);
        std::vector<Token> filler;
        for (Token t : text)
            if (t != a && t != b && filler.size() < 10) filler.push_back(t);
        Sampler::Params p = base;
        p.samplerSequence = {Sampler::SamplingType::Infill, Sampler::SamplingType::Temperature};
        Sampler s(model, p), plain(model, base);
        auto build = [&](float la, float lb, float leos, float lf) {
            c.clear();
            c.push_back({a, la, 0});
            c.push_back({b, lb, 0});
            for (Token t : filler) c.push_back({t, lf, 0});
            c.push_back({voc.eos(), leos, 0});
            std::stable_sort(c.begin(), c.end(), [](auto& x, auto& y) { return x.logit > y.logit; });
        };
        int got_a = 0, plain_b = 0;
        for (int i = 0; i < 200; ++i) {
            build(5.0f, 4.9f, -10.0f, 0.0f);
            got_a += s.applyChain(c) == a;       // b merged into a; fillers < 0.2
            build(5.0f, 4.9f, -10.0f, 0.0f);
            plain_b += plain.applyChain(c) == b;
        }
        CHECK(got_a == 200);
        CHECK(plain_b > 40);
        build(0.0f, 0.0f, 3.0f, 0.0f);           // 3 p_eog n > p_text: EOG only
        CHECK(s.applyChain(c) == voc.eos());
        build(0.0f, -5.0f, -10.0f, 0.0f);        // flat text, none >= 0.2 after merging: EOT
        if (filler.size() == 10) CHECK(s.applyChain(c) == voc.eot());
    }
}

TEST_CASE_G("vocab only", "cpu") {   // t-integration.cpp:25-43
    REQUIRE(!g_vocab.empty());
    Model model(g_vocab, {.vocabOnly = true});
    CHECK(model.params().gpu);
    CHECK(model.params().vocabOnly);
    CHECK(model.trainCtxLength() == 0);
    CHECK(model.shouldAddBosToken());
    CHECK_FALSE(model.hasEncoder());
    auto& vocab = model.vocab();
    // the test vocabulary (tests/test_host.py) has merges up to "▁hello" and "▁world"
    auto t = vocab.tokenize("hello world", true, true);
    REQUIRE(t.size() == 3);
    CHECK(t[0] == vocab.bos());
    CHECK(vocab.tokenToString(t[1]) == " hello");
    CHECK(vocab.tokenToString(t[2]) == " world");
    CHECK(vocab.tokenize("hello world", false, true) == std::vector<Token>(t.begin() + 1, t.end()));
    // a control token's text is one token when parseSpecial, plain text otherwise
    auto sp = vocab.tokenize("hello</s>", false, true);
    REQUIRE(sp.size() == 2);
    CHECK(sp[1] == vocab.eos());
    CHECK(vocab.isEog(vocab.eos()));
    auto nsp = vocab.tokenize("hello</s>", false, false);
    CHECK(nsp.size() > 2);
    // bytes missing from the vocabulary fall back to <0xXX> tokens
    auto by = vocab.tokenize("\xc3\xa9", false, false);
    std::string back;
    for (Token x : by) back += vocab.tokenToString(x);
    CHECK(back == " \xc3\xa9");
}

// GBNF grammars (llama-grammar.cpp b5187 restated in blama_amd/host/grammar.cpp; parity unpinned):
// the language of each construct, the parser's errors, and the token-level filter the Sampler
// applies (Sampler.cpp:126-173) with partial UTF-8 across byte tokens.
TEST_CASE_G("grammar", "cpu") {
    {
        Grammar g("root ::= \"a\" [0-9]+ (\"x\" | \"yz\")?\n");
        CHECK(g.acceptsComplete("a12"));
        CHECK(g.acceptsComplete("a1x"));
        CHECK(g.acceptsComplete("a1yz"));
        CHECK_FALSE(g.acceptsComplete("a"));
        CHECK(g.acceptsPrefix("a"));
        CHECK(g.acceptsPrefix("a1y"));
        CHECK_FALSE(g.acceptsComplete("a1y"));
        CHECK_FALSE(g.acceptsPrefix("b"));
        CHECK_FALSE(g.acceptsPrefix("a1xy"));
    }
    {   // bounded repetitions: S{m}, S{m,}, S{m,n}
        Grammar g("root ::= \"ab\"{2,3} c\nc ::= [c]{1} d{2,}\nd ::= \"d\"");
        CHECK(g.acceptsComplete("ababcdd"));
        CHECK(g.acceptsComplete("abababcddddd"));
        CHECK_FALSE(g.acceptsComplete("abcdd"));
        CHECK_FALSE(g.acceptsPrefix("abababab"));
        CHECK_FALSE(g.acceptsComplete("ababcd"));
    }
    {   // classes, negation, any char, escapes, comments, unicode ranges, multi-line alternates
        Grammar g("# a comment\nroot ::= item (\",\" item)*   # trailing comment\n"
                  "item ::= [^,\\x5D\\n]+ | \"\\u00e9\" [\\u03b1-\\u03c9] |\n    \"<\" . \">\"\n");
        CHECK(g.acceptsComplete("abc,d e"));
        CHECK(g.acceptsComplete("\xc3\xa9\xce\xb2"));       // "é" then a greek small letter
        CHECK(g.acceptsComplete("\xc3\xa9" "A"));           // ... and by the first alternative
        CHECK_FALSE(g.acceptsComplete("\n"));
        CHECK(g.acceptsComplete("<,>,x"));                   // "." takes the comma inside <>
        CHECK_FALSE(g.acceptsPrefix("a]"));
        CHECK_FALSE(g.acceptsComplete("a,"));
    }
    // parser errors (llama_sampler_init_grammar yields no grammar for these)
    auto throws = [](const char* txt) {
        try { Grammar g(txt); } catch (const std::runtime_error&) { return true; }
        return false;
    };
    CHECK(throws("root ::= foo\n"));                     // undefined rule
    CHECK(throws("root ::= root \"a\" | \"b\"\n"));      // left recursion
    CHECK(throws("item ::= \"a\"\n"));                   // no root
    CHECK(throws("root ::= \"\\q\"\n"));                 // unknown escape
    CHECK(throws("root ::= \"a\" {,2}\n"));              // expecting an int
    CHECK(throws("root ::= ( \"a\"\n"));                 // unbalanced group
    CHECK(throws("root ::= * \"a\"\n"));                 // repetition without an item

    // token level over the test vocabulary
    REQUIRE(!g_vocab.empty());
    Model model(g_vocab, {.vocabOnly = true});
    auto& voc = model.vocab();
    const Token hello = voc.tokenize("hello", false, true).back(), world = voc.tokenize("world", false, true).back();
    REQUIRE(voc.tokenToString(hello) == " hello");
    {
        Grammar g("root ::= \" hello\" \" world\"\n");
        CHECK(g.allows(voc, hello));
        CHECK_FALSE(g.allows(voc, world));
        CHECK_FALSE(g.allows(voc, voc.eos()));               // EOG only once a stack is complete
        std::vector<int32_t> ids = {hello, world, voc.eos()};
        std::vector<float> lg = {1.0f, 2.0f, 3.0f};
        g.apply(voc, ids.data(), lg.data(), ids.size());
        CHECK(lg[0] == 1.0f && lg[1] == -INFINITY && lg[2] == -INFINITY);
        g.accept(voc, hello);
        CHECK(g.allows(voc, world));
        CHECK_FALSE(g.allows(voc, hello));
        g.accept(voc, world);
        CHECK(g.allows(voc, voc.eos()));
        CHECK_FALSE(g.allows(voc, hello));                   // a complete stack takes nothing more
        bool threw = false;
        try { g.accept(voc, hello); } catch (const std::runtime_error&) { threw = true; }
        CHECK(threw);                                        // "Unexpected empty grammar stack"
        g.reset();
        CHECK(g.allows(voc, hello) && !g.allows(voc, world));
    }
    {   // a two-byte character split over byte-fallback tokens (partial UTF-8 state)
        const auto by = voc.tokenize("\xc3\xa9", false, false);
        REQUIRE(by.size() >= 2);
        const Token b0 = by[by.size() - 2], b1 = by[by.size() - 1];
        REQUIRE(voc.tokenToString(b0) == "\xc3" && voc.tokenToString(b1) == "\xa9");
        Grammar g("root ::= \"\\u00e9\"\n");
        CHECK(g.allows(voc, b0));                            // 0xC3 can still complete to U+00E9
        CHECK_FALSE(g.allows(voc, b1));                      // a continuation byte cannot start
        g.accept(voc, b0);
        CHECK(g.allows(voc, b1));
        CHECK_FALSE(g.allows(voc, b0));                      // 0xC3 does not continue 0xC3
        CHECK_FALSE(g.allows(voc, voc.eos()));
        g.accept(voc, b1);
        CHECK(g.allows(voc, voc.eos()));
        Grammar h("root ::= [a-z]\n");
        CHECK_FALSE(h.allows(voc, b0));                      // U+00C0..U+00FF is past [a-z]
    }
    {   // the Sampler: generated tokens advance the grammar, prompt tokens do not; reset rewinds
        Sampler::Params p;
        p.grammar = "root ::= \" hello\" \" world\"";
        Sampler s(model, p);
        REQUIRE(s.grammar() != nullptr);
        s.accept(world, false);                              // prompt token: grammar untouched
        CHECK(s.grammar()->allows(voc, hello));
        s.accept(hello, true);
        CHECK(s.grammar()->allows(voc, world));
        s.reset();
        CHECK(s.grammar()->allows(voc, hello));
        Sampler::Params bad;
        bad.grammar = "root ::= nope";
        bool threw = false;
        try { Sampler t(model, bad); } catch (const std::runtime_error&) { threw = true; }
        CHECK(threw);
    }
}

// tests/test_tokenizer_bpe.py: tokenise every line of --in (hex-encoded UTF-8) with the vocab-only
// model --vocab (parseSpecial, no BOS) and write the ids, one line per text, to --out
TEST_CASE_G("tokenize file", "tok") {
    REQUIRE(!g_vocab.empty() && !g_in.empty() && !g_out.empty());
    Model model(g_vocab, {.vocabOnly = true});
    std::ifstream in(g_in);
    std::ofstream out(g_out);
    std::string line;
    while (std::getline(in, line)) {
        std::string text;
        for (size_t i = 0; i + 1 < line.size(); i += 2) text += (char)std::stoi(line.substr(i, 2), nullptr, 16);
        const auto ids = model.vocab().tokenize(text, false, true);
        for (size_t i = 0; i < ids.size(); ++i) out << (i ? " " : "") << ids[i];
        out << "\n";
        std::string back;   // tokenToString of the ids concatenates to the text again
        for (Token t : ids) back += model.vocab().tokenToString(t);
        CHECK(back == text);
    }
}

TEST_CASE_G("wire format", "cpu") {   // HttpServerMain.cpp:37-94, 259-288
    using server::Server;
    namespace wire = server::wire;
    Server::CompleteReponse gen;
    gen.push_back({" he said \"hi\"\n\t\x01", 301, {{301, 17.25f}, {7, -0.1f}, {1234567, 3.14159274f}}});
    gen.push_back({"\xc3\xa9\xe2\x82\xac", 77, {{77, 1e-30f}, {5, -1.17549435e-38f}, {9, 0.333333343f}}});
    const std::string body = wire::completeBody(gen);
    const auto j = bl::json::parse(body);
    CHECK(j.at("text").as_string() == gen[0].tokenStr + gen[1].tokenStr);
    auto back = wire::toCompleteResponse(j);
    REQUIRE(back.size() == gen.size());
    for (size_t i = 0; i < gen.size(); ++i) {
        CHECK(back[i].tokenStr == gen[i].tokenStr);
        CHECK(back[i].tokenId == gen[i].tokenId);
        REQUIRE(back[i].logits.size() == gen[i].logits.size());
        for (size_t k = 0; k < gen[i].logits.size(); ++k) {
            CHECK(back[i].logits[k].tokenId == gen[i].logits[k].tokenId);
            CHECK(std::memcmp(&back[i].logits[k].logit, &gen[i].logits[k].logit, 4) == 0);   // float-exact
        }
    }
    // request keys: "prompt" required, the rest optional with the Server.hpp:25-32 defaults
    auto p = wire::toCompleteParams(bl::json::parse(R"({"prompt": "a\u00e9\ud83d\ude00"})"));
    CHECK(p.prompt == "a\xc3\xa9\xf0\x9f\x98\x80");
    CHECK(p.maxTokens == 0u);
    CHECK(p.seed == 0u);
    CHECK(p.temperature == 0.8f);
    CHECK(p.topP == 0.95f);
    p = wire::toCompleteParams(bl::json::parse(
        R"({"prompt":"x","max_tokens":16,"seed":42,"suffix":"y","temp":0.5,"top_p":0.9})"));
    CHECK(p.maxTokens == 16u);
    CHECK(p.seed == 42u);
    CHECK(p.suffix == "y");
    CHECK(p.temperature == 0.5f);
    CHECK(p.topP == 0.9f);
    auto p2 = wire::toCompleteParams(bl::json::parse(bl::json::dump(wire::fromCompleteParams(p))));
    CHECK(p2.prompt == p.prompt && p2.maxTokens == p.maxTokens && p2.seed == p.seed);
    CHECK(p2.temperature == p.temperature && p2.topP == p.topP && p2.suffix == p.suffix);
    CHECK_THROWS(wire::toCompleteParams(bl::json::parse(R"({"max_tokens": 3})")));
    CHECK_THROWS(bl::json::parse("{\"prompt\": }"));
    CHECK_THROWS(bl::json::parse("[1, 2"));
    // invalid UTF-8 (byte-fallback tokens) becomes U+FFFD per maximal subpart; ids/logits intact
    const std::string fffd = "\xef\xbf\xbd";
    auto enc = [](std::string s) { bl::json::Value v = bl::json::Value::string(std::move(s)); return bl::json::parse(bl::json::dump(v)).as_string(); };
    CHECK(enc("\xe2") == fffd);
    CHECK(enc("a\xe2\x96") == "a" + fffd);                 // truncated 3-byte sequence: one U+FFFD
    CHECK(enc("\xe2\x96\x81") == "\xe2\x96\x81");          // complete: kept
    CHECK(enc("\xc0\xaf") == fffd + fffd);                 // overlong lead: each byte invalid
    CHECK(enc("\xed\xa0\x80") == fffd + fffd + fffd);      // surrogate: 0xA0 outside ED's range
    CHECK(enc("\xf0\x9f\x98\x80x\xff") == "\xf0\x9f\x98\x80x" + fffd);
    CHECK((float)bl::json::parse(wire::verifyBody(0.975f)).at("result").as_number() == 0.975f);
    // network-facing validation: empty or oversized claimed logit lists, non-JSON numbers,
    // out-of-range integers, deep nesting
    CHECK_THROWS(wire::toCompleteResponse(bl::json::parse(R"({"tokenData":[{"str":"","id":0,"logits":[]}]})")));
    CHECK_THROWS(wire::toCompleteParams(bl::json::parse(R"({"prompt":"x","seed":-1e300})")));
    CHECK_THROWS(wire::toCompleteParams(bl::json::parse(R"({"prompt":"x","max_tokens":1.5})")));
    CHECK_THROWS(wire::toCompleteParams(bl::json::parse(R"({"prompt":"x","temp":1e300})")));
    CHECK(wire::toCompleteParams(bl::json::parse(R"({"prompt":"x","seed":4294967295})")).seed == 4294967295u);
    CHECK_THROWS(bl::json::parse("nan"));
    CHECK_THROWS(bl::json::parse("[inf]"));
    CHECK_THROWS(bl::json::parse("0x10"));
    CHECK_THROWS(bl::json::parse("1e999"));
    CHECK_THROWS(bl::json::parse("+1"));
    CHECK(bl::json::parse("-0.5e-3").as_number() == -0.5e-3);
    CHECK_THROWS(bl::json::parse(std::string(100000, '[')));
    CHECK(bl::json::parse(std::string(200, '[') + std::string(200, ']')).is_array());
    CHECK_THROWS(LogitComparer::compare({}, {{1, 1.0f}}));
}

// ---------------------------------------------------------------- GPU ----
TEST_CASE_G("session", "gpu") {   // t-integration.cpp:124-250
    REQUIRE(!g_model.empty());
    Model model(g_model, {});
    CHECK(model.params().gpu);
    CHECK(model.trainCtxLength() == 256);
    Instance inst(model, {});
    inst.warmup();
    {   // no initialization
        auto& s = inst.startSession({});
        CHECK_THROWS_WITH(s.complete({}), "Session hasn't started yet");
        CHECK_THROWS_WITH(s.completeStream({.prompt = kPrompt}), "Session hasn't started yet");
        CHECK_THROWS_WITH(s.getState(), "Session hasn't started yet");
        inst.stopSession();
    }
    {   // double initialization
        auto& s = inst.startSession({});
        s.setInitialPrompt(kPrompt);
        CHECK_THROWS_WITH(s.setState({}), "Session already started");
        inst.stopSession();
    }
    Token first = Token_Invalid;
    {   // generating phase
        auto& s = inst.startSession({});
        s.setInitialPrompt(kPrompt);
        auto p = s.complete({.maxTokens = 1});
        REQUIRE(p.size() == 1);
        first = p[0].token;
        CHECK(p[0].logits.size() == 10);
        for (size_t i = 1; i < p[0].logits.size(); ++i) CHECK(p[0].logits[i - 1].logit >= p[0].logits[i].logit);
        const std::vector<Token> more = {410, 411, 412};
        auto p2 = s.complete({.prompt = more, .maxTokens = 1});
        REQUIRE(p2.size() == 1);
        CHECK(s.getState().size() > 0);
        inst.stopSession();
    }
    {   // generation streaming: same seed, same first token as complete()
        auto& s = inst.startSession({});
        s.setInitialPrompt(kPrompt);
        auto stream = s.completeStream({.maxTokens = 1});
        auto p = stream.complete();
        CHECK(p.token == first);
        CHECK(stream.status() == Session::StreamGenerator::Status::Completed);
        CHECK(stream.complete().token == Token_Invalid);
        inst.stopSession();
    }
    {   // single session
        auto& s = inst.startSession({});
        (void)s;
        CHECK_THROWS_WITH(inst.startSession({}), "Session is already started. Stop it to start a new one.");
        inst.stopSession();
    }
}

TEST_CASE_G("sampler bias beyond top-k", "gpu") {   // Sampler.cpp:30-41: bias before top_k
    Model model(g_model, {});
    Instance inst(model, {});
    REQUIRE(mi_decode(inst.mctx(), kPrompt.data(), (int32_t)kPrompt.size(), MI_OUT_LAST) == 0);
    const float* lg = mi_logits(inst.mctx(), -1);
    REQUIRE(lg != nullptr);
    const int32_t n = mi_model_n_vocab(model.mmodel());
    Token low = 0;
    for (int32_t i = 1; i < n; ++i)
        if (lg[i] < lg[low]) low = i;          // the lowest-ranked token: far outside the top 40
    Sampler::Params p;
    p.temp = 0.0f;                              // greedy
    p.logitBias = {{low, 1e4f}};
    Sampler s(model, p);
    CHECK(s.sample(inst.mctx()) == low);        // the bias lifts it over every other token
    Sampler::Params q;
    q.temp = 0.0f;
    Sampler plain(model, q);
    Token top = plain.sample(inst.mctx());
    q.repetitionPenalty.repeat = 1e6f;          // penalise the top token out of first place
    q.repetitionPenalty.numTokens = 64;
    Sampler pen(model, q);
    pen.accept(top, false);
    const Token second = pen.sample(inst.mctx());
    CHECK(second != top);
}

TEST_CASE_G("sampler stages on the logits", "gpu") {   // Sampler.cpp:47-96 over a real context
    Model model(g_model, {});
    Instance inst(model, {});
    REQUIRE(mi_decode(inst.mctx(), kPrompt.data(), (int32_t)kPrompt.size(), MI_OUT_LAST) == 0);
    const int32_t n = mi_model_n_vocab(model.mmodel());
    Sampler::Params g;
    g.temp = 0.0f;
    const Token top = Sampler(model, g).sample(inst.mctx());
    auto run = [&](const Sampler::Params& p) {
        Sampler s(model, p);
        std::vector<Token> out;
        for (int i = 0; i < 32; ++i) out.push_back(s.sample(inst.mctx()));
        return out;
    };
    std::vector<Sampler::Params> ps;
    for (int ver : {1, 2}) {            // mirostat: the full vocabulary, not the engine's top-k
        Sampler::Params p;
        p.rngSeed = 11;
        p.mirostat = {ver, 5.0f, 0.1f};
        ps.push_back(p);
    }
    {
        Sampler::Params p;               // XTC, typical and dynamic temperature after top-k
        p.rngSeed = 12;
        p.typicalP = 0.5f;
        p.minKeep = 1;
        p.tempRange = 0.3f;
        p.xtc = {0.5f, 0.1f};
        p.samplerSequence = {Sampler::SamplingType::Top_K, Sampler::SamplingType::Typical_P,
                             Sampler::SamplingType::XTC, Sampler::SamplingType::Temperature};
        ps.push_back(p);
    }
    {
        Sampler::Params p;               // infill after top-k
        p.rngSeed = 13;
        p.samplerSequence = {Sampler::SamplingType::Top_K, Sampler::SamplingType::Infill,
                             Sampler::SamplingType::Temperature};
        ps.push_back(p);
    }
    for (auto& p : ps) {
        auto a = run(p);
        CHECK(a == run(p));              // same seed, same draws
        for (Token t : a) CHECK((t >= 0 && t < n) || t == model.vocab().eot());
    }
    Sampler::Params p;                    // a near-zero target surprise: mirostat v2 is greedy
    p.mirostat = {2, 0.0f, 0.1f};
    CHECK(Sampler(model, p).sample(inst.mctx()) == top);
}

TEST_CASE_G("grammar sampling", "gpu") {   // Sampler.cpp:126-173 / Session.cpp:374-377 over a real context
    Model model(g_model, {});
    Instance inst(model, {});
    auto& voc = model.vocab();
    // the synthetic vocabulary's pieces are " t<i>" (and byte tokens): a finite language, so the
    // generation must spell one of its strings and then end on end-of-generation
    const std::string gram = "root ::= \" t1\" [0-9] [0-9] \" t2\" [0-9] [0-9]";
    Grammar check(gram);
    for (uint32_t seed : {5u, 6u}) {
        Session::InitParams ip;
        ip.seed = seed;
        ip.grammar = gram;
        auto& s = inst.startSession(ip);
        s.setInitialPrompt(kPrompt);
        auto p = s.complete({.maxTokens = 12});
        std::string text;
        for (auto& tp : p) text += voc.tokenToString(tp.token);
        CHECK(p.size() < 12);                 // stopped on EOG, the only token a complete grammar allows
        CHECK(check.acceptsComplete(text));
        inst.stopSession();
    }
    {   // without a grammar the same session samples outside that set
        Session::InitParams ip;
        ip.seed = 5;
        auto& s = inst.startSession(ip);
        s.setInitialPrompt(kPrompt);
        auto p = s.complete({.maxTokens = 6});
        bool outside = false;
        for (auto& tp : p) outside = outside || voc.tokenToString(tp.token).rfind(" t1", 0) != 0;
        CHECK(outside);
        inst.stopSession();
    }
}

TEST_CASE_G("filling ctx", "gpu") {   // t-integration.cpp:219-248: bit-identical verification
    Model model(g_model, {});
    Instance inst(model, {}), inst2(model, {});
    inst.warmup();
    inst2.warmup();
    auto& s = inst.startSession({});
    auto& s2 = inst2.startSession({});
    s.setInitialPrompt(kPrompt);
    s2.setInitialPrompt(kPrompt);
    auto p = s.complete({.maxTokens = 10});
    REQUIRE(p.size() > 0);
    auto p2 = s2.fillCtx(p);
    CHECK(p.size() == p2.size());
    for (size_t i = 0; i < p.size(); i++) {
        REQUIRE(p2[i].logits.size() == p[i].logits.size());
        for (size_t j = 0; j < p[i].logits.size(); j++) {
            CHECK(p[i].logits[j].token == p2[i].logits[j].token);
            CHECK(p[i].logits[j].logit == p2[i].logits[j].logit);
        }
    }
    // the Server::verify flow (Server.cpp:127-161) on a self-verification scores 1
    MetricsAggregator agg;
    float score = 0;
    for (size_t i = 0; i < p.size(); i++) {
        auto m = LogitComparer::compare(p[i].logits, p2[i].logits);
        score = agg.pushAndVerify({&m, 1});
    }
    CHECK(score == 1.0f);
}

TEST_CASE_G("filling ctx batched", "gpu") {   // fillCtx as one MI_OUT_ALL pass vs generation
    Model model(g_model, {});
    Instance inst(model, {}), inst2(model, {});
    auto& s = inst.startSession({});
    auto& s2 = inst2.startSession({.batchedVerify = true});
    s.setInitialPrompt(kPrompt);
    s2.setInitialPrompt(kPrompt);
    auto p = s.complete({.maxTokens = 24});
    REQUIRE(p.size() > 0);
    auto p2 = s2.fillCtx(p);
    REQUIRE(p.size() == p2.size());
    MetricsAggregator agg;
    float score = 0;
    for (size_t i = 0; i < p.size(); i++) {
        REQUIRE(p2[i].logits.size() == p[i].logits.size());
        CHECK(p2[i].token == p[i].token);
        float rms = 0;
        for (auto& l : p[i].logits) rms += l.logit * l.logit;
        rms = std::sqrt(rms / p[i].logits.size());
        for (auto& l : p[i].logits) {   // same ids (gathered), logits within the GEMM's fp32 order
            auto it = std::find_if(p2[i].logits.begin(), p2[i].logits.end(), [&](const TokenData& d) { return d.token == l.token; });
            REQUIRE(it != p2[i].logits.end());
            CHECK(std::fabs(it->logit - l.logit) <= 4e-3f * rms);
        }
        auto m = LogitComparer::compare(p[i].logits, p2[i].logits);
        CHECK(m.top1Match == 1.0f);
        score = agg.pushAndVerify({&m, 1});
    }
    CHECK(score >= 0.999f);
    // the batch decoded every claimed token: prompt + claimed cells in the cache
    CHECK(mi_kv_n_cells(inst2.mctx()) == (int32_t)(kPrompt.size() + p.size()));
}

TEST_CASE_G("states", "gpu") {   // t-integration.cpp:304-421
    Model model(g_model, {});
    Instance inst(model, {});
    std::vector<uint8_t> state;
    std::vector<Token> gen;
    {
        auto& s = inst.startSession({});
        s.setInitialPrompt(kPrompt);
        state = s.getState();
        for (auto& p : s.complete({.maxTokens = 6})) gen.push_back(p.token);
        inst.stopSession();
    }
    {
        auto& s = inst.startSession({});
        s.setState(state);
        std::vector<Token> again;
        for (auto& p : s.complete({.maxTokens = 6})) again.push_back(p.token);
        CHECK(again == gen);
        inst.stopSession();
    }
}

TEST_CASE_G("context shift", "gpu") {   // Session.cpp:324-347 through a long generation
    Model model(g_model, {});
    Instance inst(model, {.ctxSize = 32});
    auto& s = inst.startSession({});
    s.setInitialPrompt(kPrompt);
    auto p = s.complete({.maxTokens = 40});   // 8 + 40 > 32 - 4: shifts at least once
    CHECK(p.size() == 40);
    Instance inst2(model, {.ctxSize = 32});
    auto& s2 = inst2.startSession({.infiniteContext = false});
    s2.setInitialPrompt(kPrompt);
    CHECK_THROWS_WITH(s2.complete({.maxTokens = 40}), "context limit of 32 reached");
}

TEST_CASE_G("complete for the oracle", "gpu") {   // t-LogitComparer.cpp:41-79, GPU side
    REQUIRE(!g_out.empty());
    Model model(g_model, {});
    Instance inst(model, {});
    auto& s = inst.startSession({.seed = 7});
    s.setInitialPrompt(kPrompt);
    auto iRes = s.complete({.maxTokens = 12});
    std::ofstream f(g_out);
    for (auto& p : iRes) {
        f << p.token;
        for (auto& l : p.logits) {
            char buf[64];
            std::snprintf(buf, sizeof buf, " %d:%.9g", l.token, l.logit);
            f << buf;
        }
        f << "\n";
    }
    CHECK(iRes.size() == 12);
}

TEST_CASE_G("server", "gpu") {   // Server.cpp:45-77 and :127-161 through the worker thread
    using server::Server;
    auto model = std::make_shared<Model>(g_model, Model::Params{});
    Server srv(model);
    Server::CompleteRequestParams req;
    req.prompt = "hello world";
    req.maxTokens = 8;
    req.seed = 3;
    std::promise<Server::CompleteReponse> pc;
    srv.completeText(req, [&](Server::CompleteReponse r) { pc.set_value(std::move(r)); });
    auto resp = pc.get_future().get();
    REQUIRE(resp.size() == 8);
    for (auto& t : resp) {
        CHECK(t.logits.size() == 10);
        CHECK(t.tokenStr == model->vocab().tokenToString((Token)t.tokenId));
    }
    // the same request again: same seed, same completion (session per request)
    std::promise<Server::CompleteReponse> pc2;
    srv.completeText(req, [&](Server::CompleteReponse r) { pc2.set_value(std::move(r)); });
    auto resp2 = pc2.get_future().get();
    REQUIRE(resp2.size() == resp.size());
    for (size_t i = 0; i < resp.size(); ++i) CHECK(resp2[i].tokenId == resp[i].tokenId);
    // verify of its own completion after a JSON round trip scores 1 (to the fp32 order of the
    // batched verification pass: Session::InitParams::batchedVerify)
    auto wired = server::wire::toCompleteResponse(bl::json::parse(server::wire::completeBody(resp)));
    std::promise<float> pv;
    srv.verify(req, wired, [&](float s) { pv.set_value(s); });
    CHECK(pv.get_future().get() >= 0.999f);
    // a tampered completion scores below 1
    auto bad = resp;
    for (auto& t : bad)
        for (auto& l : t.logits) l.logit *= 1.5f;
    std::promise<float> pb;
    srv.verify(req, bad, [&](float s) { pb.set_value(s); });
    const float sb = pb.get_future().get();
    CHECK(sb < 0.95f);
    // an error on the worker reaches the error callback and the next request still runs
    auto huge = resp;             // a claimed token outside the vocabulary makes decode throw
    huge[0].tokenId = 1u << 30;
    std::promise<float> pe;
    srv.verify(req, huge, [&](float s) { pe.set_value(s); },
               [&](std::exception_ptr e) { pe.set_exception(e); });
    CHECK_THROWS(pe.get_future().get());
    std::promise<float> pv2;
    srv.verify(req, wired, [&](float s) { pv2.set_value(s); });
    CHECK(pv2.get_future().get() >= 0.999f);
}

TEST_CASE_G("server replicas", "gpu") {   // one Instance + worker per replica, least-loaded dispatch
    using server::Server;
    auto model = std::make_shared<Model>(g_model, Model::Params{});
    Server srv(std::vector<std::shared_ptr<Model>>{model, model});   // two contexts on one GPU
    REQUIRE(srv.replicas() == 2);
    Server::CompleteRequestParams req;
    req.prompt = "hello world";
    req.maxTokens = 8;
    req.seed = 3;
    constexpr int N = 8;
    std::vector<std::promise<Server::CompleteReponse>> pr(N);
    for (int i = 0; i < N; ++i)   // submitted together: the queue spreads them over both replicas
        srv.completeText(req, [&pr, i](Server::CompleteReponse r) { pr[i].set_value(std::move(r)); });
    std::vector<Server::CompleteReponse> out;
    for (auto& p : pr) out.push_back(p.get_future().get());
    for (int i = 1; i < N; ++i) {   // a session per request: same seed, same tokens on either replica
        REQUIRE(out[i].size() == out[0].size());
        for (size_t k = 0; k < out[0].size(); ++k) {
            CHECK(out[i][k].tokenId == out[0][k].tokenId);
            for (size_t j = 0; j < out[0][k].logits.size(); ++j)
                CHECK(out[i][k].logits[j].logit == out[0][k].logits[j].logit);
        }
    }
    auto served = srv.served();
    CHECK(served[0] + served[1] == (uint64_t)N);
    CHECK(served[0] >= 1);
    CHECK(served[1] >= 1);
    std::vector<std::promise<float>> pv(4);
    for (int i = 0; i < 4; ++i) srv.verify(req, out[i], [&pv, i](float s) { pv[i].set_value(s); });
    for (auto& p : pv) CHECK(p.get_future().get() >= 0.999f);
}

MINITEST_MAIN(setup)
