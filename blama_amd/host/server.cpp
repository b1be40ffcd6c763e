// bl::llama::server::Server: see server.hpp for the reference mapping.
#include "server.hpp"
#include <cstdlib>

#include <cstdio>
#include <stdexcept>

namespace bl::llama::server {

Server::Server(std::shared_ptr<Model> model) : Server(std::vector<std::shared_ptr<Model>>{std::move(model)}) {}

Server::Server(std::vector<std::shared_ptr<Model>> replicas) {
    if (replicas.empty()) throw std::runtime_error("Server: no model");
    for (auto& m : replicas) {
        auto r = std::make_unique<Replica>();
        r->model = std::move(m);
        r->instance = std::make_unique<Instance>(*r->model, Instance::InitParams{});
        r->instance->warmup();                             // Server.cpp:37
        m_reps.push_back(std::move(r));
    }
    for (auto& r : m_reps) {
        Replica* rp = r.get();
        rp->worker = std::thread([this, rp] { run(*rp); });
    }
}

Server::~Server() {
    {
        std::lock_guard<std::mutex> lk(m_mu);
        m_stop = true;                                     // pending jobs still run (work guard reset)
    }
    for (auto& r : m_reps) r->cv.notify_all();
    for (auto& r : m_reps)
        if (r->worker.joinable()) r->worker.join();
}

std::vector<uint64_t> Server::served() const {
    std::lock_guard<std::mutex> lk(m_mu);
    std::vector<uint64_t> v;
    for (const auto& r : m_reps) v.push_back(r->served);
    return v;
}

// least-loaded dispatch: the replica with the fewest queued + running requests
void Server::post(std::function<void(Replica&)> job, ErrorCb onError) {
    Replica* best = nullptr;
    {
        std::lock_guard<std::mutex> lk(m_mu);
        for (auto& r : m_reps)
            if (!best || r->load < best->load) best = r.get();
        best->jobs.emplace_back(std::move(job), std::move(onError));
        best->load++;
    }
    best->cv.notify_one();
}

void Server::run(Replica& r) {
    for (;;) {
        std::pair<std::function<void(Replica&)>, ErrorCb> job;
        {
            std::unique_lock<std::mutex> lk(m_mu);
            r.cv.wait(lk, [&] { return m_stop || !r.jobs.empty(); });
            if (r.jobs.empty()) return;
            job = std::move(r.jobs.front());
            r.jobs.pop_front();
        }
        try {
            job.first(r);
        } catch (...) {
            r.instance->stopSession();                     // the next request starts clean
            if (job.second) job.second(std::current_exception());
            else std::fprintf(stderr, "bl::llama::server: request failed with an exception\n");
        }
        std::lock_guard<std::mutex> lk(m_mu);
        r.load--;
        r.served++;
    }
}

void Server::completeText(CompleteRequestParams params, std::function<void(CompleteReponse)> cb, ErrorCb onError) {
    post([params = std::move(params), cb = std::move(cb)](Replica& rep) {
        auto& session = rep.instance->startSession({.seed = params.seed, .temperature = params.temperature,
                                                  .topP = params.topP});
        const Vocab& vocab = rep.model->vocab();
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
        rep.instance->stopSession();
    }, std::move(onError));
}

void Server::verify(CompleteRequestParams req, CompleteReponse resp, std::function<void(float)> cb, ErrorCb onError) {
    post([req = std::move(req), resp = std::move(resp), cb = std::move(cb)](Replica& rep) {
        // the claimed tokens are pushed in one batched pass (BLAMA_SERIAL_VERIFY=1: one decode per
        // token, as Session.cpp:231-244, bit-identical to this server's own generation)
        static const bool batched = getenv("BLAMA_SERIAL_VERIFY") == nullptr;
        auto& session = rep.instance->startSession({.seed = req.seed, .temperature = req.temperature,
                                                  .topP = req.topP, .batchedVerify = batched});
        session.setInitialPrompt(rep.model->vocab().tokenize(req.prompt, true, true));
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
        rep.instance->stopSession();
    }, std::move(onError));
}

}  // namespace bl::llama::server
