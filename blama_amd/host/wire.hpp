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
        g.tokenId = (uint32_t)(int64_t)jt.at("id").as_number();
        const Value& jl = jt.at("logits");
        if (!jl.is_array()) throw std::runtime_error("json: logits is not an array");
        g.logits.reserve(jl.arr.size());
        for (const Value& e : jl.arr)
            g.logits.push_back({(uint32_t)(int64_t)e.at("id").as_number(), (float)e.at("logit").as_number()});
    }
    return gen;
}

inline Server::CompleteRequestParams toCompleteParams(const Value& j) {
    Server::CompleteRequestParams p;
    if (!j.is_object()) throw std::runtime_error("json: request is not an object");
    p.prompt = j.at("prompt").as_string();
    if (auto* v = j.find("max_tokens")) p.maxTokens = (uint32_t)(int64_t)v->as_number();
    if (auto* v = j.find("seed")) p.seed = (uint32_t)(int64_t)v->as_number();
    if (auto* v = j.find("suffix")) p.suffix = v->as_string();
    if (auto* v = j.find("temp")) p.temperature = (float)v->as_number();
    if (auto* v = j.find("top_p")) p.topP = (float)v->as_number();
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
