// bl::llama::server::Server: see server.hpp for the reference mapping.
#include "server.hpp"
#include <cstdlib>

#include <cstdio>

namespace bl::llama::server {

Server::Server(std::shared_ptr<Model> model)
    : m_model(std::move(model)), m_instance(std::make_unique<Instance>(*m_model, Instance::InitParams{})) {
    m_instance->warmup();                                  // Server.cpp:37
    m_worker = std::thread([this] { run(); });
}

Server::~Server() {
    {
        std::lock_guard<std::mutex> lk(m_mu);
        m_stop = true;                                     // pending jobs still run (work guard reset)
    }
    m_cv.notify_all();
    if (m_worker.joinable()) m_worker.join();
}

void Server::post(std::function<void()> job, ErrorCb onError) {
    {
        std::lock_guard<std::mutex> lk(m_mu);
        m_jobs.emplace_back(std::move(job), std::move(onError));
    }
    m_cv.notify_one();
}

void Server::run() {
    for (;;) {
        std::pair<std::function<void()>, ErrorCb> job;
        {
            std::unique_lock<std::mutex> lk(m_mu);
            m_cv.wait(lk, [this] { return m_stop || !m_jobs.empty(); });
            if (m_jobs.empty()) return;
            job = std::move(m_jobs.front());
            m_jobs.pop_front();
        }
        try {
            job.first();
        } catch (...) {
            m_instance->stopSession();                     // the next request starts clean
            if (job.second) job.second(std::current_exception());
            else std::fprintf(stderr, "bl::llama::server: request failed with an exception\n");
        }
    }
}

void Server::completeText(CompleteRequestParams params, std::function<void(CompleteReponse)> cb, ErrorCb onError) {
    post([this, params = std::move(params), cb = std::move(cb)] {
        auto& session = m_instance->startSession({.seed = params.seed, .temperature = params.temperature,
                                                  .topP = params.topP});
        const Vocab& vocab = m_model->vocab();
        session.setInitialPrompt(vocab.tokenize(params.prompt, true, true));
        auto iRes = session.complete({.prompt = {}, .maxTokens = (int32_t)params.maxTokens});
        CompleteReponse response;
        response.reserve(iRes.size());
        for (const auto& tp : iRes) {
            auto& td = response.emplace_back();
            td.tokenStr = vocab.tokenToString(tp.token);
            td.tokenId = (uint32_t)tp.token;
            td.logits.reserve(tp.logits.size());
            for (const auto& l : tp.logits) td.logits.push_back({(uint32_t)l.token, l.logit});
        }
        cb(std::move(response));
        m_instance->stopSession();
    }, std::move(onError));
}

void Server::verify(CompleteRequestParams req, CompleteReponse resp, std::function<void(float)> cb, ErrorCb onError) {
    post([this, req = std::move(req), resp = std::move(resp), cb = std::move(cb)] {
        // the claimed tokens are pushed in one batched pass (BLAMA_SERIAL_VERIFY=1: one decode per
        // token, as Session.cpp:231-244, bit-identical to this server's own generation)
        static const bool batched = getenv("BLAMA_SERIAL_VERIFY") == nullptr;
        auto& session = m_instance->startSession({.seed = req.seed, .temperature = req.temperature,
                                                  .topP = req.topP, .batchedVerify = batched});
        session.setInitialPrompt(m_model->vocab().tokenize(req.prompt, true, true));
        std::vector<TokenPrediction> claimed;
        claimed.reserve(resp.size());
        for (const auto& td : resp) {
            auto& tp = claimed.emplace_back();
            tp.token = (Token)td.tokenId;
            tp.logits.reserve(td.logits.size());
            for (const auto& l : td.logits) tp.logits.push_back({(Token)l.tokenId, l.logit});
        }
        auto mine = session.fillCtx(claimed);
        MetricsAggregator agg;
        float score = 0;
        for (size_t i = 0; i < claimed.size(); i++) {
            auto m = LogitComparer::compare(claimed[i].logits, mine[i].logits);
            score = agg.pushAndVerify({&m, 1});
        }
        cb(score);
        m_instance->stopSession();
    }, std::move(onError));
}

}  // namespace bl::llama::server
