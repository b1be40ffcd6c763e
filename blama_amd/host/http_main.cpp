// blama-http-server on the MI355X engine: the L5 executable.  Mirrors reference
// server/code/http/HttpServerMain.cpp:
//   POST /complete            (:311-318) -> {"text", "tokenData"}
//   POST /verify_completion   (:328-338) {"request", "response"} -> {"result"}
//   any other method          (:305-309) -> 400
//   any other path            (:350-354) -> 404
//   env BLAMA_HOST (default 0.0.0.0), BLAMA_PORT (default 7331), BLAMA_MODEL (:383-435),
//   validated with the reference's error messages
//
// What differs:
// - Plain POSIX sockets, one thread per connection and one request per connection.  The
//   reference uses Boost.Beast coroutines, and Boost is not in this image.  Every request
//   still runs on the Server's single worker, so the concurrency model is the reference's.
// - BLAMA_MODEL is required: the reference falls back to a gpt2 test file that is not here.
// - BLAMA_PORT=0 binds an ephemeral port.  The bound port is printed as
//   "Listening on port N".
// - A body that is not valid JSON, or a request that throws on the worker, gets a 500 with
//   the message in the body.  In the reference the exception ends the coroutine.
// - /chat/completions and /chat/verify_completion return 501: chat templating is out of scope.
// - A malformed request head or Content-Length gets a 400, a body over 64 MB a 413.
#include <arpa/inet.h>
#include <execinfo.h>
#include <net/if.h>
#include <netinet/in.h>
#include <signal.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <charconv>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <filesystem>
#include <future>
#include <iostream>
#include <limits>
#include <string>
#include <thread>

#include "server.hpp"
#include "wire.hpp"

namespace fs = std::filesystem;
using bl::llama::server::Server;
namespace wire = bl::llama::server::wire;

namespace {

struct Request {
    std::string method, target, body;
};

// Bodies above this are refused with 413 (the reference's Beast parser has its own limit).
constexpr size_t kMaxBody = 64u << 20;

enum class ReadStatus { Ok, Closed, BadRequest, TooLarge };

ReadStatus readRequest(int fd, Request& req) {
    std::string buf;
    char chunk[65536];
    size_t hdrEnd = std::string::npos;
    while ((hdrEnd = buf.find("\r\n\r\n")) == std::string::npos) {
        const ssize_t n = ::recv(fd, chunk, sizeof chunk, 0);
        if (n <= 0) return ReadStatus::Closed;
        buf.append(chunk, (size_t)n);
        if (buf.size() > (64u << 10) && buf.find("\r\n\r\n") == std::string::npos) return ReadStatus::TooLarge;
    }
    const std::string head = buf.substr(0, hdrEnd);
    const size_t sp1 = head.find(' '), sp2 = head.find(' ', sp1 + 1);
    if (sp1 == std::string::npos || sp2 == std::string::npos) return ReadStatus::BadRequest;
    req.method = head.substr(0, sp1);
    req.target = head.substr(sp1 + 1, sp2 - sp1 - 1);
    size_t clen = 0;
    size_t pos = head.find("\r\n");
    while (pos != std::string::npos && pos < head.size()) {
        const size_t next = head.find("\r\n", pos + 2);
        std::string line = head.substr(pos + 2, (next == std::string::npos ? head.size() : next) - pos - 2);
        const size_t colon = line.find(':');
        if (colon != std::string::npos) {
            std::string key = line.substr(0, colon);
            for (auto& c : key) c = (char)std::tolower((unsigned char)c);
            if (key == "content-length") {
                // digits only (optional surrounding blanks); no sign, no overflow
                size_t b = colon + 1, e = line.size();
                while (b < e && (line[b] == ' ' || line[b] == '\t')) ++b;
                while (e > b && (line[e - 1] == ' ' || line[e - 1] == '\t')) --e;
                unsigned long long v = 0;
                const auto r = std::from_chars(line.data() + b, line.data() + e, v, 10);
                if (b == e || r.ec != std::errc() || r.ptr != line.data() + e) return ReadStatus::BadRequest;
                if (v > kMaxBody) return ReadStatus::TooLarge;
                clen = (size_t)v;
            }
        }
        pos = next;
    }
    req.body = buf.substr(hdrEnd + 4);
    while (req.body.size() < clen) {
        const ssize_t n = ::recv(fd, chunk, std::min(sizeof chunk, clen - req.body.size()), 0);
        if (n <= 0) return ReadStatus::Closed;
        req.body.append(chunk, (size_t)n);
    }
    req.body.resize(clen);
    return ReadStatus::Ok;
}

void writeAll(int fd, const std::string& s) {
    size_t off = 0;
    while (off < s.size()) {
        const ssize_t n = ::send(fd, s.data() + off, s.size() - off, MSG_NOSIGNAL);
        if (n <= 0) return;
        off += (size_t)n;
    }
}

void respond(int fd, int status, const char* reason, const std::string& body, bool json) {
    std::string r = "HTTP/1.1 " + std::to_string(status) + " " + reason + "\r\n";
    r += "Server: blama-amd\r\n";
    if (json) r += "Content-Type: text/json\r\n";              // HttpServerMain.cpp:268
    r += "Access-Control-Allow-Origin: *\r\n";
    r += "Content-Length: " + std::to_string(body.size()) + "\r\n";
    r += "Connection: close\r\n\r\n";
    r += body;
    writeAll(fd, r);
}

void handleRequest(int fd, Server& server, const Request& req) {
    try {
        if (req.method != "POST") {
            respond(fd, 400, "Bad Request", "", false);
        } else if (req.target == "/complete") {
            auto params = wire::toCompleteParams(bl::json::parse(req.body));
            // shared: the worker may still be inside set_value when this thread wakes
            auto pr = std::make_shared<std::promise<Server::CompleteReponse>>();
            auto fut = pr->get_future();
            server.completeText(std::move(params), [pr](Server::CompleteReponse r) { pr->set_value(std::move(r)); },
                                [pr](std::exception_ptr e) { pr->set_exception(e); });
            respond(fd, 200, "OK", wire::completeBody(fut.get()), true);
        } else if (req.target == "/verify_completion") {
            const auto j = bl::json::parse(req.body);
            auto rreq = wire::toCompleteParams(j.at("request"));
            auto rrsp = wire::toCompleteResponse(j.at("response"));
            auto pr = std::make_shared<std::promise<float>>();
            auto fut = pr->get_future();
            server.verify(std::move(rreq), std::move(rrsp), [pr](float s) { pr->set_value(s); },
                          [pr](std::exception_ptr e) { pr->set_exception(e); });
            respond(fd, 200, "OK", wire::verifyBody(fut.get()), true);
        } else if (req.target == "/chat/completions" || req.target == "/chat/verify_completion") {
            respond(fd, 501, "Not Implemented", "chat templating is not served by this build", false);
        } else {
            respond(fd, 404, "Not Found", "", false);
        }
    } catch (const std::exception& e) {
        respond(fd, 500, "Internal Server Error", e.what(), false);
    }
}

// Runs on a detached thread: nothing may escape it (an escaping exception would terminate the
// whole server).
void handle(int fd, Server& server) noexcept {
    try {
        Request req;
        switch (readRequest(fd, req)) {
        case ReadStatus::Ok: handleRequest(fd, server, req); break;
        case ReadStatus::BadRequest: respond(fd, 400, "Bad Request", "malformed request head", false); break;
        case ReadStatus::TooLarge: respond(fd, 413, "Payload Too Large", "", false); break;
        case ReadStatus::Closed: break;
        }
    } catch (...) {
    }
    ::shutdown(fd, SHUT_WR);
    ::close(fd);
}

std::string modelFromEnv() {
    const char* model_env = std::getenv("BLAMA_MODEL");
    if (!model_env || std::string(model_env).empty())
        throw std::runtime_error("Environment variable not set or empty: BLAMA_MODEL");
    std::string path(model_env);
    if (!path.ends_with(".gguf")) throw std::runtime_error("BLAMA_MODEL does not end with .gguf: " + path);
    if (!fs::exists(path)) throw std::runtime_error("BLAMA_MODEL does not exist: " + path);
    if (!fs::is_regular_file(path)) throw std::runtime_error("BLAMA_MODEL is not a regular file: " + path);
    return path;
}

}  // namespace

int serve();

namespace {
std::atomic<bool> g_listening{false};

// A fatal signal before or while serving: name it and print a backtrace on stderr, then die of
// the same signal (the parent sees the signal number as the exit status).
void crash_handler(int sig) {
    char msg[64];
    int n = 0;
    for (const char* p = "blama-http-server: fatal signal "; *p; ++p) msg[n++] = *p;
    char d[8];
    int k = 0;
    for (int v = sig; v > 0 && k < 8; v /= 10) d[k++] = char('0' + v % 10);
    while (k > 0) msg[n++] = d[--k];
    msg[n++] = '\n';
    (void)!::write(2, msg, n);
    void* frames[64];
    const int nf = ::backtrace(frames, 64);
    ::backtrace_symbols_fd(frames, nf, 2);
    ::signal(sig, SIG_DFL);
    ::raise(sig);
}

void install_crash_handlers() {
    void* warm[1];
    ::backtrace(warm, 1);   // loads libgcc's unwinder now, not inside the handler
    for (int sig : {SIGSEGV, SIGBUS, SIGILL, SIGFPE, SIGABRT}) ::signal(sig, crash_handler);
    // a library calling exit() during start-up (before "Listening") says so
    std::atexit([] {
        if (!g_listening.load()) std::cerr << "blama-http-server: exit() called before the server was listening" << std::endl;
    });
}
}  // namespace

int main() {
    std::setvbuf(stdout, nullptr, _IOLBF, 0);   // stage lines reach a log file as they happen
    install_crash_handlers();
    try {
        return serve();
    } catch (const std::exception& e) {   // configuration errors: message and a non-zero exit
        std::cerr << "blama-http-server: " << e.what() << std::endl;
        g_listening = true;   // a reported configuration error, not a silent exit
        return 1;
    }
}

int serve() {
    ::signal(SIGPIPE, SIG_IGN);
    // BLAMA_HOST: an IPv4 or IPv6 address, as boost::asio::ip::make_address accepts it
    // (HttpServerMain.cpp:386); default 0.0.0.0
    sockaddr_storage ss{};
    socklen_t slen = sizeof(sockaddr_in);
    {
        auto* a4 = reinterpret_cast<sockaddr_in*>(&ss);
        a4->sin_family = AF_INET;
        a4->sin_addr.s_addr = htonl(INADDR_ANY);
    }
    if (const char* h = std::getenv("BLAMA_HOST")) {
        auto* a4 = reinterpret_cast<sockaddr_in*>(&ss);
        auto* a6 = reinterpret_cast<sockaddr_in6*>(&ss);
        if (::inet_pton(AF_INET, h, &a4->sin_addr) == 1) {
            a4->sin_family = AF_INET;
        } else {
            // an IPv6 literal, optionally with a %scope (link-local)
            std::string s6 = h, scope;
            if (const size_t pc = s6.find('%'); pc != std::string::npos) {
                scope = s6.substr(pc + 1);
                s6.resize(pc);
            }
            ss = sockaddr_storage{};
            if (::inet_pton(AF_INET6, s6.c_str(), &a6->sin6_addr) != 1) throw std::invalid_argument("Invalid BLAMA_HOST");
            a6->sin6_family = AF_INET6;
            if (!scope.empty()) {
                a6->sin6_scope_id = ::if_nametoindex(scope.c_str());
                if (a6->sin6_scope_id == 0) {
                    char* end = nullptr;
                    const unsigned long v = std::strtoul(scope.c_str(), &end, 10);
                    if (!end || *end) throw std::invalid_argument("Invalid BLAMA_HOST");
                    a6->sin6_scope_id = (uint32_t)v;
                }
            }
            slen = sizeof(sockaddr_in6);
        }
    }
    uint16_t port = 7331;
    if (const char* p = std::getenv("BLAMA_PORT")) {
        size_t idx = 0;
        const unsigned long v = std::stoul(p, &idx, 10);
        if (idx != std::strlen(p)) throw std::invalid_argument("Extra characters after BLAMA_PORT number");
        if (v > std::numeric_limits<uint16_t>::max()) throw std::out_of_range("Value exceeds uint16_t max");
        port = (uint16_t)v;
    }
    const std::string modelGguf = modelFromEnv();
    std::cout << "Loading model " << modelGguf << std::endl;
    // BLAMA_DEVICES=0,1,...: one replica (Model + Instance + worker) per listed GPU behind the
    // server's least-loaded dispatch (extension; default: device 0, the reference's one worker)
    // the first replica parses the GGUF; the others receive its weight arena (RCCL broadcast
    // across GPUs, a device copy on the same GPU) instead of re-reading the file
    std::vector<int> devices;
    {
        std::string devs = std::getenv("BLAMA_DEVICES") ? std::getenv("BLAMA_DEVICES") : "0";
        size_t at = 0;
        while (at <= devs.size()) {
            const size_t comma = devs.find(',', at);
            const std::string d = devs.substr(at, comma == std::string::npos ? std::string::npos : comma - at);
            size_t idx = 0;
            const int dev = std::stoi(d, &idx, 10);
            if (idx != d.size() || dev < 0) throw std::invalid_argument("BLAMA_DEVICES: bad device list");
            devices.push_back(dev);
            if (comma == std::string::npos) break;
            at = comma + 1;
        }
    }
    std::cerr << "blama-http-server: loading " << devices.size() << " replica(s)" << std::endl;
    auto replicas = bl::llama::Model::loadReplicas(modelGguf, devices);
    std::cerr << "blama-http-server: weights resident on every replica; creating instances" << std::endl;
    Server server(std::move(replicas));
    std::cerr << "blama-http-server: instances ready" << std::endl;

    const int lfd = ::socket(ss.ss_family, SOCK_STREAM, 0);
    const int one = 1;
    ::setsockopt(lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    if (ss.ss_family == AF_INET) reinterpret_cast<sockaddr_in*>(&ss)->sin_port = htons(port);
    else reinterpret_cast<sockaddr_in6*>(&ss)->sin6_port = htons(port);
    if (::bind(lfd, (sockaddr*)&ss, slen) != 0 || ::listen(lfd, 64) != 0) {
        std::perror("bind/listen");
        return 1;
    }
    socklen_t alen = sizeof ss;
    ::getsockname(lfd, (sockaddr*)&ss, &alen);
    const uint16_t bound = ss.ss_family == AF_INET ? reinterpret_cast<sockaddr_in*>(&ss)->sin_port
                                                   : reinterpret_cast<sockaddr_in6*>(&ss)->sin6_port;
    g_listening = true;
    std::cout << "Listening on port " << ntohs(bound) << std::endl;
    for (;;) {
        const int fd = ::accept(lfd, nullptr, nullptr);
        if (fd < 0) continue;
        std::thread([fd, &server] { handle(fd, server); }).detach();
    }
}
