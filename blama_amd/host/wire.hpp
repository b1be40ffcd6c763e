// The JSON wire format of /complete and /verify_completion.  It follows the reference
// server/code/http/HttpServerMain.cpp:
//   toJson (:37-51)               CompleteReponse -> [{"str","id","logits":[{"id","logit"}]}]
//   toCompleteResponse (:53-70)   {"tokenData": [...]} -> CompleteReponse
//   toCompleteParams (:85-94)     "prompt" is required; "max_tokens", "seed", "suffix", "temp"
//                                 and "top_p" are optional
//   getCompleteResponse (:259-275) {"text": concatenated token strings, "tokenData": [...]}
//   getVerifyResponse (:277-288)  {"result": score}
// A logit is written with 9 significant digits, which reads back as the same float.  nlohmann
// gets the same round trip by storing the value as a double.
#pragma once
#include "json.hpp"
#include "server.hpp"

namespace bl::llama::server::wire {

using json::Value;

// Numbers come from the network: every conversion is range-checked (the parser already rejects
// nan/inf).  Integers must be integral and within [INT32_MIN, UINT32_MAX]; a negative value
// wraps as nlohmann's get<uint32_t> (a static_cast) would.
inline uint32_t to_u32(const Value& v, const char* what) {
    const double d = v.as_number();
    if (d != std::floor(d) || d < -2147483648.0 || d > 4294967295.0)
        throw std::runtime_error(std::string("json: ") + what + " is not a 32-bit integer");
    return (uint32_t)(int64_t)d;
}
inline float to_f32(const Value& v, const char* what) {
    const double d = v.as_number();
    if (!(std::fabs(d) <= 3.4028234663852886e38)) throw std::runtime_error(std::string("json: ") + what + " out of float range");
    return (float)d;
}
// Claimed top-k lists per token: the verifier gathers at most this many ids (mi_gather).
constexpr size_t kMaxClaimedLogits = 4096;

inline Value toJson(const Server::CompleteReponse& gen) {
    Value arr = Value::array();
    for (const auto& g : gen) {
        Value jt = Value::object();
        jt.set("str", Value::string(g.tokenStr));
        jt.set("id", Value::number(g.tokenId));
        Value jl = Value::array();
        for (const auto& l : g.logits) {
            Value e = Value::object();
            e.set("id", Value::number(l.tokenId));
            e.set("logit", Value::number(l.logit, true));
            jl.arr.push_back(std::move(e));
        }
        jt.set("logits", std::move(jl));
        arr.arr.push_back(std::move(jt));
    }
    return arr;
}

inline Server::CompleteReponse toCompleteResponse(const Value& j) {
    Server::CompleteReponse gen;
    const Value& toks = j.at("tokenData");
    if (!toks.is_array()) throw std::runtime_error("json: tokenData is not an array");
    gen.reserve(toks.arr.size());
    for (const Value& jt : toks.arr) {
        auto& g = gen.emplace_back();
        g.tokenStr = jt.at("str").as_string();
        g.tokenId = to_u32(jt.at("id"), "id");
        const Value& jl = jt.at("logits");
        if (!jl.is_array()) throw std::runtime_error("json: logits is not an array");
        if (jl.arr.empty() || jl.arr.size() > kMaxClaimedLogits)
            throw std::runtime_error("json: logits must hold 1.." + std::to_string(kMaxClaimedLogits) + " entries");
        g.logits.reserve(jl.arr.size());
        for (const Value& e : jl.arr) g.logits.push_back({to_u32(e.at("id"), "id"), to_f32(e.at("logit"), "logit")});
    }
    return gen;
}

inline Server::CompleteRequestParams toCompleteParams(const Value& j) {
    Server::CompleteRequestParams p;
    if (!j.is_object()) throw std::runtime_error("json: request is not an object");
    p.prompt = j.at("prompt").as_string();
    if (auto* v = j.find("max_tokens")) p.maxTokens = to_u32(*v, "max_tokens");
    if (auto* v = j.find("seed")) p.seed = to_u32(*v, "seed");
    if (auto* v = j.find("suffix")) p.suffix = v->as_string();
    if (auto* v = j.find("temp")) p.temperature = to_f32(*v, "temp");
    if (auto* v = j.find("top_p")) p.topP = to_f32(*v, "top_p");
    return p;
}

inline Value fromCompleteParams(const Server::CompleteRequestParams& p) {
    Value j = Value::object();
    j.set("prompt", Value::string(p.prompt));
    j.set("max_tokens", Value::number(p.maxTokens));
    j.set("seed", Value::number(p.seed));
    j.set("suffix", Value::string(p.suffix));
    j.set("temp", Value::number(p.temperature, true));
    j.set("top_p", Value::number(p.topP, true));
    return j;
}

inline std::string completeBody(const Server::CompleteReponse& gen) {
    std::string text;
    for (const auto& g : gen) text += g.tokenStr;
    Value out = Value::object();
    out.set("text", Value::string(text));
    out.set("tokenData", toJson(gen));
    return json::dump(out);
}

inline std::string verifyBody(float score) {
    Value out = Value::object();
    out.set("result", Value::number(score, true));
    return json::dump(out);
}

}  // namespace bl::llama::server::wire
