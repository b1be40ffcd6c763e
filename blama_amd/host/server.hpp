// bl::llama::server::Server on the MI355X engine: the request layer (L4) behind Blama's HTTP
// endpoints.  Mirrors reference server/code/server/Server.hpp:17-68.  The request and response
// structs, the completeText/verify flow and the single worker thread are the same:
//
//   completeText  Server.cpp:45-77    startSession{seed,temp,topP} -> tokenize(prompt, true, true)
//                                     -> setInitialPrompt -> complete{maxTokens} -> response
//                                     -> cb -> stopSession
//   verify        Server.cpp:127-161  startSession -> setInitialPrompt -> fillCtx(claimed)
//                                     -> LogitComparer::compare + MetricsAggregator per token -> cb(score)
//   worker        Server.cpp:36       every request runs on one thread, so one engine context
//                                     serves them in arrival order
//
// What differs:
// - The callbacks are std::function, where the reference uses itlib::ufunction.  itlib is not
//   in this image.
// - An optional error callback receives exceptions raised on the worker.  The reference lets
//   them escape the io_context thread.
// - chatComplete/chatVerify are not served: the chat templating is out of scope.
//
// - Replicas (extension): Server(models) runs one Instance and one worker thread per model
//   (one Model per GPU: Model::Params::device), and each request goes to the replica with the
//   fewest queued + running requests (lowest index on ties).  A replica is the reference's
//   single-worker server; requests are independent sessions, so nothing crosses replicas
//   (replicas only).  Server(model) is one replica, the reference's shape.
#pragma once
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "llama.hpp"

namespace bl::llama::server {

class Server {
public:
    explicit Server(std::shared_ptr<Model> model);
    // one replica per model (the same model may appear twice: two contexts on one GPU)
    explicit Server(std::vector<std::shared_ptr<Model>> replicas);
    ~Server();

    Server(const Server&) = delete;
    Server& operator=(const Server&) = delete;

    struct CompleteRequestParams {     // Server.hpp:25-32
        std::string prompt;
        uint32_t maxTokens = 0;
        uint32_t seed = 0;
        std::string suffix;
        float temperature = 0.8f;
        float topP = 0.95f;
    };

    struct TokenData {                 // Server.hpp:46-56
        std::string tokenStr;
        uint32_t tokenId = 0;
        struct LogitData {
            uint32_t tokenId = 0;
            float logit = 0;
        };
        std::vector<LogitData> logits;
    };

    using CompleteReponse = std::vector<TokenData>;   // (sic) Server.hpp:56
    using ErrorCb = std::function<void(std::exception_ptr)>;

    void completeText(CompleteRequestParams params, std::function<void(CompleteReponse)> cb,
                      ErrorCb onError = {});
    void verify(CompleteRequestParams req, CompleteReponse resp, std::function<void(float)> cb,
                ErrorCb onError = {});

    size_t replicas() const noexcept { return m_reps.size(); }
    // requests each replica has served so far (tests, load reports)
    std::vector<uint64_t> served() const;

private:
    struct Replica {
        std::shared_ptr<Model> model;
        std::unique_ptr<Instance> instance;
        std::deque<std::pair<std::function<void(Replica&)>, ErrorCb>> jobs;
        uint32_t load = 0;                 // queued + running requests
        uint64_t served = 0;
        std::condition_variable cv;
        std::thread worker;
    };
    void post(std::function<void(Replica&)> job, ErrorCb onError);
    void run(Replica& r);

    std::vector<std::unique_ptr<Replica>> m_reps;
    mutable std::mutex m_mu;               // guards every replica's queue, load and stop flag
    bool m_stop = false;
};

}  // namespace bl::llama::server
