// extern "C" implementation of include/mi_engine.h.  Every entry point
// catches exceptions and reports them through mi_last_error().
#include "engine.h"

#include <dlfcn.h>
#include <execinfo.h>
#include <fcntl.h>
#include <signal.h>
#include <rccl/rccl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

using namespace mi;

struct mi_model { Model impl; };
struct mi_ctx { std::unique_ptr<Ctx> impl; };

#define MI_TRY(fail) catch (const std::exception& e) { set_last_error(e.what()); return fail; } \
                     catch (...) { set_last_error("unknown error"); return fail; }

// ---- replicas: fill the arenas of header-only models (no_upload) from a loaded one ----
// Weights cross devices by one RCCL broadcast over xGMI (single process: ncclCommInitAll over the
// distinct devices, root = the loaded model's device); replicas on a device that already holds
// a filled arena take a device-to-device copy.  librccl is opened on first use (dlopen), so the
// engine carries no link-time RCCL dependency.
namespace {
struct Rccl {
    decltype(&ncclCommInitAll) init = nullptr;
    decltype(&ncclBroadcast) bcast = nullptr;
    decltype(&ncclGroupStart) gstart = nullptr;
    decltype(&ncclGroupEnd) gend = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclGetErrorString) err = nullptr;
    std::string load_error;     // why the library or a symbol is missing (dlerror() read once, here)
};
const Rccl& rccl() {
    static const Rccl r = [] {
        Rccl x;
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
        if (!h) {
            const char* e = dlerror();
            x.load_error = e ? e : "dlopen(librccl.so) failed";
            return x;
        }
        x.init = reinterpret_cast<decltype(x.init)>(dlsym(h, "ncclCommInitAll"));
        x.bcast = reinterpret_cast<decltype(x.bcast)>(dlsym(h, "ncclBroadcast"));
        x.gstart = reinterpret_cast<decltype(x.gstart)>(dlsym(h, "ncclGroupStart"));
        x.gend = reinterpret_cast<decltype(x.gend)>(dlsym(h, "ncclGroupEnd"));
        x.destroy = reinterpret_cast<decltype(x.destroy)>(dlsym(h, "ncclCommDestroy"));
        x.err = reinterpret_cast<decltype(x.err)>(dlsym(h, "ncclGetErrorString"));
        if (!x.init || !x.bcast || !x.gstart || !x.gend || !x.destroy) x.load_error = "missing symbols";
        return x;
    }();
    return r;
}
// Diagnostic (MI_SEGV_MAPS=1): on SIGSEGV / SIGBUS print the fault address, the faulting PC and
// every backtrace frame with the mapping that holds it (path + offset, from /proc/self/maps), so
// the frames of a crash inside the ROCm libraries can be symbolised offline (llvm-symbolizer
// --obj=<path> <offset>); then the default action.  Installed when a context is created, i.e.
// after any profiler's own handler.
char g_maps[1 << 20];
void segv_out(const char* s) { ssize_t r = write(2, s, strlen(s)); (void)r; }
void segv_where(const char* tag, unsigned long long a, int nmaps) {
    char line[512];
    const char* p = g_maps;
    const char* end = g_maps + nmaps;
    const char* prev = nullptr;
    while (p < end) {
        const char* nl = (const char*)memchr(p, '\n', end - p);
        if (!nl) nl = end;
        unsigned long long lo = 0, hi = 0, off = 0;
        if (sscanf(p, "%llx-%llx %*s %llx", &lo, &hi, &off) == 3 && a >= lo && a < hi) {
            const char* path = (const char*)memchr(p, '/', nl - p);
            const int pl = path ? (int)(nl - path) : 0;
            snprintf(line, sizeof line, "mi_segv %s 0x%llx = %.*s +0x%llx (mapping %.*s)\n", tag, a, pl, path ? path : "",
                     a - lo + off, (int)(nl - p), p);
            segv_out(line);
            return;
        }
        if (lo > a && prev) {   // unmapped: the mappings on either side
            const char* pn = (const char*)memchr(prev, '\n', end - prev);
            snprintf(line, sizeof line, "mi_segv %s 0x%llx unmapped, between\n  %.*s\n  %.*s\n", tag, a,
                     (int)((pn ? pn : end) - prev), prev, (int)(nl - p), p);
            segv_out(line);
            return;
        }
        prev = p;
        p = nl + 1;
    }
    snprintf(line, sizeof line, "mi_segv %s 0x%llx not found in maps\n", tag, a);
    segv_out(line);
}
void segv_handler(int sig, siginfo_t* si, void* ucv) {
    int fd = open("/proc/self/maps", O_RDONLY);
    int n = 0;
    if (fd >= 0) {
        for (ssize_t r; n < (int)sizeof(g_maps) - 1 && (r = read(fd, g_maps + n, sizeof(g_maps) - 1 - n)) > 0;) n += (int)r;
        close(fd);
    }
    char line[128];
    snprintf(line, sizeof line, "mi_segv signal %d fault address %p\n", sig, si ? si->si_addr : nullptr);
    segv_out(line);
    segv_where("fault", (unsigned long long)(si ? si->si_addr : nullptr), n);
    const ucontext_t* uc = reinterpret_cast<const ucontext_t*>(ucv);
    if (uc) segv_where("pc", (unsigned long long)uc->uc_mcontext.gregs[REG_RIP], n);
    void* fr[64];
    const int nf = backtrace(fr, 64);
    for (int i = 0; i < nf; ++i) {
        char tag[16];
        snprintf(tag, sizeof tag, "frame%02d", i);
        segv_where(tag, (unsigned long long)fr[i], n);
    }
    signal(sig, SIG_DFL);
    raise(sig);
}
void segv_maps_install() {
    static bool done = false;
    if (done || !getenv("MI_SEGV_MAPS")) return;
    done = true;
    void* warm[2];
    backtrace(warm, 2);   // loads the unwinder before any signal
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sa.sa_sigaction = segv_handler;
    sa.sa_flags = SA_SIGINFO;
    sigaction(SIGSEGV, &sa, nullptr);
    sigaction(SIGBUS, &sa, nullptr);
    segv_out("mi_segv: handler installed\n");
}
void nccl_ck(ncclResult_t r, const char* what) {
    if (r != ncclSuccess) throw Error(std::string("RCCL ") + what + ": " + (rccl().err ? rccl().err(r) : "error"));
}
}  // namespace

extern "C" {

const char* mi_last_error(void) { return last_error(); }

mi_model* mi_model_load_from_memory(const void* data, size_t size, const mi_model_params* params) {
    try {
        set_last_error("");
        mi_model_params p{0, 0, 0, 0};
        if (params) p = *params;
        if (p.cpu_only) throw Error("cpu_only: the CPU path is the reference's ggml backend, not this engine");
        auto* m = new mi_model();
        try {
            m->impl.load(static_cast<const uint8_t*>(data), size, p);
        } catch (...) {
            delete m;
            throw;
        }
        return m;
    }
    MI_TRY(nullptr)
}

mi_model* mi_model_load(const char* path, const mi_model_params* params) {
    try {
        if (!path) throw Error("null path");
        const int fd = ::open(path, O_RDONLY);
        if (fd < 0) throw Error(std::string("cannot open ") + path);
        struct stat st;
        if (fstat(fd, &st) != 0) { ::close(fd); throw Error("fstat failed"); }
        const size_t size = (size_t)st.st_size;
        void* map = mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
        ::close(fd);
        if (map == MAP_FAILED) throw Error(std::string("mmap failed for ") + path);
        mi_model* m = mi_model_load_from_memory(map, size, params);
        munmap(map, size);
        return m;
    }
    MI_TRY(nullptr)
}

void mi_model_free(mi_model* model) { delete model; }

int32_t mi_model_n_vocab(const mi_model* m) { return m ? m->impl.hp.n_vocab : -1; }
int32_t mi_model_n_ctx_train(const mi_model* m) { return m ? m->impl.hp.n_ctx_train : -1; }
int32_t mi_model_n_embd(const mi_model* m) { return m ? m->impl.hp.n_embd : -1; }
int32_t mi_model_n_layer(const mi_model* m) { return m ? m->impl.hp.n_layer : -1; }
int32_t mi_model_n_head(const mi_model* m) { return m ? m->impl.hp.n_head : -1; }
int32_t mi_model_n_head_kv(const mi_model* m) { return m ? m->impl.hp.n_head_kv : -1; }
int32_t mi_model_n_ff(const mi_model* m) { return m ? m->impl.hp.n_ff : -1; }
int32_t mi_model_n_expert(const mi_model* m) { return m ? m->impl.hp.n_expert : -1; }
int32_t mi_model_token_bos(const mi_model* m) { return m ? m->impl.bos : -1; }
int32_t mi_model_token_eos(const mi_model* m) { return m ? m->impl.eos : -1; }
int32_t mi_model_add_bos(const mi_model* m) { return m ? (m->impl.add_bos ? 1 : 0) : -1; }

int32_t mi_model_token_is_eog(const mi_model* m, int32_t token) {
    if (!m) return -1;
    return (token == m->impl.eos || (m->impl.eot >= 0 && token == m->impl.eot)) ? 1 : 0;
}

float mi_model_token_score(const mi_model* m, int32_t token) {
    if (!m || token < 0 || token >= (int)m->impl.token_score.size()) return 0.0f;
    return m->impl.token_score[token];
}

int32_t mi_model_token_type(const mi_model* m, int32_t token) {
    if (!m || token < 0 || token >= (int)m->impl.tokens.size()) return -1;
    if (token >= (int)m->impl.token_type.size()) return 1;   // LLAMA_TOKEN_TYPE_NORMAL
    return m->impl.token_type[token];
}

int32_t mi_model_n_tokens(const mi_model* m) { return m ? (int32_t)m->impl.tokens.size() : -1; }

int32_t mi_model_tokenizer(const mi_model* m, char* buf, int32_t size) {
    if (!m) return -1;
    const std::string& s = m->impl.tok_model;
    if (buf && size > 0) {
        const int n = std::min<int>((int)s.size(), size - 1);
        std::memcpy(buf, s.data(), n);
        buf[n] = 0;
    }
    return (int32_t)s.size();
}

int32_t mi_model_token_text(const mi_model* m, int32_t token, char* buf, int32_t size) {
    if (!m || token < 0 || token >= (int)m->impl.tokens.size()) { set_last_error("token out of range"); return -1; }
    const std::string& s = m->impl.tokens[token];
    if (buf && size > 0) {
        const int n = std::min<int>((int)s.size(), size - 1);
        std::memcpy(buf, s.data(), n);
        buf[n] = 0;
    }
    return (int32_t)s.size();
}

int32_t mi_model_n_merges(const mi_model* m) { return m ? (int32_t)m->impl.merges.size() : -1; }

int32_t mi_model_merge(const mi_model* m, int32_t i, char* buf, int32_t size) {
    if (!m || i < 0 || i >= (int)m->impl.merges.size()) { set_last_error("merge out of range"); return -1; }
    const std::string& s = m->impl.merges[i];
    if (buf && size > 0) {
        const int n = std::min<int>((int)s.size(), size - 1);
        std::memcpy(buf, s.data(), n);
        buf[n] = 0;
    }
    return (int32_t)s.size();
}

int32_t mi_model_meta_str(const mi_model* m, const char* key, char* buf, int32_t size) {
    if (!m || !key) return -1;
    const GgufValue* v = m->impl.gguf.get(key);
    if (!v) return -1;
    std::string s = v->type == 8 ? v->s : (v->type == 6 || v->type == 12) ? std::to_string(v->f) : std::to_string(v->i);
    if (buf && size > 0) {
        const int n = std::min<int>((int)s.size(), size - 1);
        std::memcpy(buf, s.data(), n);
        buf[n] = 0;
    }
    return (int32_t)s.size();
}

int64_t mi_model_weight_bytes(const mi_model* m) { return m ? m->impl.weight_bytes : -1; }

int32_t mi_model_arena(const mi_model* m, void** dev_ptr, size_t* bytes) {
    if (!m) return -1;
    if (dev_ptr) *dev_ptr = m->impl.arena;
    if (bytes) *bytes = m->impl.arena_bytes;
    return 0;
}


// One line per replication stage on stderr: a start-up that dies inside RCCL or HIP says where.
static void replicate_log(const std::string& what) {
    std::fprintf(stderr, "mi_engine: replicate: %s\n", what.c_str());
    std::fflush(stderr);
}

int32_t mi_model_replicate(mi_model* const* models, int32_t n) {
    int caller_dev = -1;
    (void)hipGetDevice(&caller_dev);
    // communicators and streams are released on every path (a throw after ncclCommInitAll included)
    struct Guard {
        std::vector<ncclComm_t> comms;
        std::vector<std::pair<int, hipStream_t>> streams;
        int dev;
        ~Guard() {
            for (auto& [d, s] : streams) {
                if (!s) continue;
                (void)hipSetDevice(d);
                (void)hipStreamSynchronize(s);
                (void)hipStreamDestroy(s);
            }
            for (ncclComm_t c : comms)
                if (c && rccl().destroy) rccl().destroy(c);
            if (dev >= 0) (void)hipSetDevice(dev);
        }
    } guard{{}, {}, caller_dev};
    try {
        if (!models || n < 1 || !models[0]) throw Error("replicate: no source model");
        const Model& src = models[0]->impl;
        if (!src.arena) throw Error("replicate: the source model has no weights");
        for (int i = 1; i < n; ++i) {
            const Model& d = models[i]->impl;
            if (!d.arena || d.arena_bytes != src.arena_bytes || d.gguf.tensors.size() != src.gguf.tensors.size())
                throw Error("replicate: replica " + std::to_string(i) + " was not loaded from the same GGUF header");
            // the MFMA-order copies are built from the arena when the first context needs them
            if (d.mmq_arena) throw Error("replicate: replica " + std::to_string(i) + " already has a context");
        }
        std::vector<int> filled(n, 0);
        filled[0] = 1;
        // one receiver per distinct device other than the source's (RCCL ranks 1..); MI_REPLICATE_RCCL=1
        // also sends the first same-device replica through a one-rank broadcast (exercises the path on
        // a single GPU)
        std::vector<int> devs = {src.device}, recv = {0};
        const bool force = getenv("MI_REPLICATE_RCCL") != nullptr;
        for (int i = 1; i < n; ++i) {
            const int dv = models[i]->impl.device;
            if (std::find(devs.begin(), devs.end(), dv) == devs.end()) {
                devs.push_back(dv);
                recv.push_back(i);
            }
        }
        int self_recv = -1;
        if (force && devs.size() == 1)
            for (int i = 1; i < n && self_recv < 0; ++i)
                if (models[i]->impl.device == src.device) self_recv = i;
        replicate_log(std::to_string(n) + " models, " + std::to_string(src.arena_bytes) + " B arena, " +
                      std::to_string(devs.size()) + " device(s)" + (self_recv > 0 ? ", one-rank RCCL broadcast forced" : ""));
        if (devs.size() > 1 || self_recv > 0) {
            const Rccl& R = rccl();
            if (!R.init || !R.bcast || !R.gstart || !R.gend || !R.destroy)
                throw Error("replicate: librccl not usable: " + R.load_error);
            const int nd = (int)devs.size();
            guard.comms.assign(nd, nullptr);
            replicate_log("ncclCommInitAll over " + std::to_string(nd) + " device(s)");
            nccl_ck(R.init(guard.comms.data(), nd, devs.data()), "ncclCommInitAll");
            replicate_log("communicators ready");
            for (int r = 0; r < nd; ++r) {
                MI_HIP(hipSetDevice(devs[r]));
                hipStream_t s = nullptr;
                MI_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
                guard.streams.emplace_back(devs[r], s);
            }
            replicate_log("ncclBroadcast of the arena");
            nccl_ck(R.gstart(), "ncclGroupStart");
            for (int r = 0; r < nd; ++r) {
                MI_HIP(hipSetDevice(devs[r]));
                uint8_t* dst = r == 0 ? (self_recv > 0 ? models[self_recv]->impl.arena : src.arena)
                                      : models[recv[r]]->impl.arena;
                nccl_ck(R.bcast(src.arena, dst, src.arena_bytes, ncclUint8, 0, guard.comms[r], guard.streams[r].second),
                        "ncclBroadcast");
            }
            nccl_ck(R.gend(), "ncclGroupEnd");
            for (auto& [d, s] : guard.streams) {
                MI_HIP(hipSetDevice(d));
                MI_HIP(hipStreamSynchronize(s));
            }
            replicate_log("broadcast complete");
            for (int r = 1; r < nd; ++r) filled[recv[r]] = 1;
            if (self_recv > 0) filled[self_recv] = 1;
        }
        // the rest: a copy from a filled arena on the same device (or a peer copy from the source)
        for (int i = 1; i < n; ++i) {
            if (filled[i]) continue;
            Model& d = models[i]->impl;
            const uint8_t* from = src.arena;
            int from_dev = src.device;
            for (int j = 0; j < n; ++j)
                if (filled[j] && models[j]->impl.device == d.device) { from = models[j]->impl.arena; from_dev = d.device; break; }
            replicate_log("replica " + std::to_string(i) + ": device copy " + std::to_string(from_dev) + " -> " +
                          std::to_string(d.device));
            MI_HIP(hipSetDevice(d.device));
            if (from_dev == d.device) MI_HIP(hipMemcpy(d.arena, from, src.arena_bytes, hipMemcpyDeviceToDevice));
            else MI_HIP(hipMemcpyPeer(d.arena, d.device, from, from_dev, src.arena_bytes));
            filled[i] = 1;
        }
        for (int i = 0; i < n; ++i) {
            MI_HIP(hipSetDevice(models[i]->impl.device));
            MI_HIP(hipDeviceSynchronize());
        }
        replicate_log("done");
        return 0;
    }
    MI_TRY(-1)
}

int32_t mi_model_type_histogram(const mi_model* m, int64_t* out, int32_t n) {
    if (!m || !out) return -1;
    const int k = std::min(n, 32);
    for (int i = 0; i < k; ++i) out[i] = m->impl.type_bytes[i];
    return k;
}

mi_ctx* mi_ctx_create(mi_model* model, uint32_t n_ctx, uint32_t n_batch, uint32_t n_ubatch) {
    try {
        if (!model) throw Error("null model");
        segv_maps_install();
        auto* c = new mi_ctx();
        try {
            c->impl.reset(new Ctx(&model->impl, n_ctx, n_batch, n_ubatch));
        } catch (...) {
            delete c;
            throw;
        }
        return c;
    }
    MI_TRY(nullptr)
}

void mi_ctx_free(mi_ctx* ctx) { delete ctx; }
uint32_t mi_n_ctx(const mi_ctx* c) { return c ? c->impl->n_ctx : 0; }
uint32_t mi_n_batch(const mi_ctx* c) { return c ? c->impl->n_batch : 0; }

int32_t mi_decode(mi_ctx* c, const int32_t* tokens, int32_t n, int32_t out_mode) {
    try {
        if (!c || !tokens) throw Error("null argument");
        if (out_mode != MI_OUT_LAST && out_mode != MI_OUT_ALL) throw Error("decode: out_mode must be MI_OUT_LAST or MI_OUT_ALL");
        return c->impl->decode(tokens, n, out_mode == MI_OUT_ALL);
    }
    MI_TRY(-1)
}

int32_t mi_topk(mi_ctx* c, int32_t row, int32_t k, int32_t* ids, float* logits) {
    try {
        if (!c || !ids || !logits) throw Error("null argument");
        return c->impl->topk(row, k, ids, logits);
    }
    MI_TRY(-1)
}

int32_t mi_gather(mi_ctx* c, int32_t row, const int32_t* ids, int32_t n, float* out) {
    try {
        if (!c || (n > 0 && (!ids || !out))) throw Error("null argument");
        return c->impl->gather(row, ids, n, out);
    }
    MI_TRY(-1)
}

int32_t mi_gather_rows(mi_ctx* c, int32_t row0, int32_t n_rows, const int32_t* ids, int32_t k, float* out) {
    try {
        if (!c || ((int64_t)n_rows * k > 0 && (!ids || !out))) throw Error("null argument");
        return c->impl->gather_rows(row0, n_rows, ids, k, out);
    }
    MI_TRY(-1)
}

const float* mi_logits(mi_ctx* c, int32_t row) {
    try {
        if (!c) throw Error("null ctx");
        return c->impl->logits_host(row);
    }
    MI_TRY(nullptr)
}

void mi_synchronize(mi_ctx* c) {
    try { if (c) c->impl->sync(); } catch (const std::exception& e) { set_last_error(e.what()); }
}

void mi_kv_clear(mi_ctx* c) { if (c) c->impl->kv_clear(); }

int32_t mi_kv_seq_rm(mi_ctx* c, int32_t p0, int32_t p1) {
    try { if (!c) throw Error("null ctx"); return c->impl->kv_seq_rm(p0, p1); }
    MI_TRY(-1)
}
int32_t mi_kv_seq_add(mi_ctx* c, int32_t p0, int32_t p1, int32_t delta) {
    try { if (!c) throw Error("null ctx"); return c->impl->kv_seq_shift(p0, p1, delta, 0); }
    MI_TRY(-1)
}
int32_t mi_kv_seq_div(mi_ctx* c, int32_t p0, int32_t p1, int32_t d) {
    try {
        if (!c) throw Error("null ctx");
        if (d <= 0) throw Error("seq_div: divisor must be positive");
        return c->impl->kv_seq_shift(p0, p1, 0, d);
    }
    MI_TRY(-1)
}
int32_t mi_kv_pos_max(const mi_ctx* c) { return c ? c->impl->pos_max : -1; }
int32_t mi_kv_n_cells(const mi_ctx* c) { return c ? c->impl->n_cells : -1; }

size_t mi_state_size(mi_ctx* c) { return c ? c->impl->state_size() : 0; }
size_t mi_state_get(mi_ctx* c, uint8_t* dst, size_t size) {
    try { if (!c || !dst) throw Error("null argument"); return c->impl->state_get(dst, size); }
    MI_TRY(0)
}
size_t mi_state_set(mi_ctx* c, const uint8_t* src, size_t size) {
    try { if (!c || !src) throw Error("null argument"); return c->impl->state_set(src, size); }
    MI_TRY(0)
}

int32_t mi_prof_enable(mi_ctx* c, int32_t layer) {
    if (!c) return -1;
    if (layer >= c->impl->m->hp.n_layer) layer = c->impl->m->hp.n_layer - 1;
    if (c->impl->prof_layer != layer) {
        c->impl->prof_layer = layer < 0 ? -1 : layer;
        c->impl->invalidate_graphs();
    }
    return 0;
}
int32_t mi_prof_read(mi_ctx* c, float* us, int32_t n) {
    try { if (!c || !us) throw Error("null argument"); return c->impl->prof_read(us, n); }
    MI_TRY(-1)
}
int64_t mi_prof_ffn_bytes(const mi_ctx* c) { return c ? c->impl->ffn_bytes() : -1; }
int64_t mi_prof_bytes(const mi_ctx* c) { return c ? c->impl->prof_bytes : -1; }

int32_t mi_decode_path(const mi_ctx* c) {
    if (!c) return -1;
    return c->impl->sp_ok ? 1 : 0;
}
int32_t mi_debug_stamps(mi_ctx* c, uint64_t* out, int32_t n_launch) {
    try {
        if (!c || !out) throw Error("null argument");
        mi::Ctx* x = c->impl.get();
        if (!x->stamps) return 0;
        n_launch = std::min(n_launch, (int32_t)mi::Ctx::kStampLaunches);
        x->sync();
        MI_HIP(hipMemcpy(out, x->stamps, (size_t)n_launch * mi::Ctx::kStampWgs * 8 * 8, hipMemcpyDeviceToHost));
        return n_launch;
    }
    MI_TRY(-1)
}

}  // extern "C"

// ------------------------------------------------------------- op level ---
namespace {
struct DevBuf {
    void* p = nullptr;
    explicit DevBuf(size_t n) { MI_HIP(hipMalloc(&p, n ? n : 16)); }
    ~DevBuf() { if (p) hipFree(p); }
    template <class T> T* as() { return static_cast<T*>(p); }
};

// Upload GGUF blocks and repack them into planes; returns the QMat view.
QMat upload_qmat(int type, const void* raw, int rows, int K, std::vector<std::unique_ptr<DevBuf>>& keep) {
    if (!is_quant(type)) throw Error("op: unsupported quant type");
    if (K % 256) throw Error("op: K must be a multiple of 256");
    const size_t nbytes = (size_t)rows * (K / block_elems(type)) * block_bytes(type);
    auto staging = std::make_unique<DevBuf>(nbytes);
    MI_HIP(hipMemcpy(staging->p, raw, nbytes, hipMemcpyHostToDevice));
    QMat m{};
    m.type = type;
    m.rows = rows;
    m.K = K;
    m.nb = K / 256;
    uint8_t* planes[4] = {nullptr, nullptr, nullptr, nullptr};
    for (int k = 0; k < plane_count(type); ++k) {
        keep.push_back(std::make_unique<DevBuf>((size_t)(rows * m.nb + kPlanePadSb) * plane_sb_bytes(type, k)));
        MI_HIP(hipMemset(keep.back()->p, 0, (size_t)(rows * m.nb + kPlanePadSb) * plane_sb_bytes(type, k)));
        planes[k] = keep.back()->as<uint8_t>();
        m.p[k] = planes[k];
    }
    launch_repack(staging->as<uint8_t>(), type, rows, K, planes, nullptr);
    MI_HIP(hipDeviceSynchronize());
    return m;
}

GemvParams single_gemv(const QMat& m, const float* x, float* y) {
    GemvParams p;
    std::memset(&p, 0, sizeof(p));
    p.pro = PRO_PLAIN;
    p.nslots = 1;
    p.x[0] = x;
    p.K = m.K;
    p.nseg = 1;
    p.seg[0].A = m;
    p.seg[0].B = m;
    p.seg[0].pair = PAIR_ADJ;
    p.seg[0].epi = EPI_STORE;
    p.seg[0].expA = p.seg[0].expB = -1;
    p.seg[0].out = y;
    return p;
}

void ensure_attrs(int device) {
    static std::vector<int> done(64, 0);
    if (device >= 0 && device < 64 && !done[device]) {
        init_kernel_attributes();
        done[device] = 1;
    }
}
}  // namespace

extern "C" {

int32_t mi_op_gemv(int32_t device, int32_t type, const void* raw, int32_t rows, int32_t K, const float* x, float* y) {
    try {
        MI_HIP(hipSetDevice(device));
        ensure_attrs(device);
        std::vector<std::unique_ptr<DevBuf>> keep;
        const QMat m = upload_qmat(type, raw, rows, K, keep);
        DevBuf dx(K * sizeof(float)), dy(rows * sizeof(float));
        MI_HIP(hipMemcpy(dx.p, x, K * sizeof(float), hipMemcpyHostToDevice));
        launch_gemv(single_gemv(m, dx.as<float>(), dy.as<float>()), nullptr);
        MI_HIP(hipDeviceSynchronize());
        MI_HIP(hipMemcpy(y, dy.p, rows * sizeof(float), hipMemcpyDeviceToHost));
        return 0;
    }
    MI_TRY(-1)
}

// The decode step's streaming GEMV (dgemv.hip) for one launch of a given role: x quantised on the
// device by dv_quant_kernel (no norm), then dgemv_kernel.  role 0 (Q/K/V, no RoPE: every row a Q
// row; a second matrix = a second segment of another type), 1 (residual add), 2 (SwiGLU of the pair
// A = gate, B = up), 3 (store), 4 (residual add with x quantised inside the launch, by every
// workgroup: the small models' FFN down).
int32_t mi_op_dgemv(int32_t device, int32_t role, int32_t type, const void* raw, int32_t rows, int32_t K, int32_t type2,
                    const void* raw2, int32_t rows2, const float* x, const float* resid, float* y) {
    try {
        MI_HIP(hipSetDevice(device));
        ensure_attrs(device);
        if (role < 0 || role > 4) throw Error("op_dgemv: role");
        const bool addq = role == 4;
        if (addq) role = 1;
        std::vector<std::unique_ptr<DevBuf>> keep;
        const QMat a = upload_qmat(type, raw, rows, K, keep);
        QMat b{};
        const bool two = raw2 && rows2 > 0;
        if (two) b = upload_qmat(type2, raw2, rows2, K, keep);
        if (role == 2 && (!two || type2 != type || rows2 != rows)) throw Error("op_dgemv: SwiGLU needs a pair");
        if ((role == 1 || role == 3) && two) throw Error("op_dgemv: one matrix for this role");
        const int out_rows = role == 0 ? rows + (two ? rows2 : 0) : rows;
        DevBuf dx(K * sizeof(float)), dy(out_rows * sizeof(float)), dr(out_rows * sizeof(float)), dtp(16);
        MI_HIP(hipMemcpy(dx.p, x, K * sizeof(float), hipMemcpyHostToDevice));
        if (role == 1) MI_HIP(hipMemcpy(dr.p, resid, rows * sizeof(float), hipMemcpyHostToDevice));
        MI_HIP(hipMemset(dtp.p, 0, 16));
        int fmt = 0;
        for (int t : {type, two ? type2 : type}) fmt |= t == T_Q8_0 ? 2 : 1;
        DevBuf act(dv_act_bytes(K, fmt & 1, fmt >> 1));
        launch_dv_quant(dx.as<float>(), ActOut{K, fmt & 1, fmt >> 1, act.as<char>(), nullptr, 1e-5f}, nullptr);
        GemvParams p;
        std::memset(&p, 0, sizeof(p));
        p.K = K;
        p.act_in = addq ? nullptr : act.as<char>();
        p.x[0] = addq ? dx.as<float>() : nullptr;
        p.act_q8k = fmt & 1;
        p.act_q80 = fmt >> 1;
        p.tokpos = dtp.as<int>();
        p.head_dim = 128;
        p.nseg = role == 0 && two ? 2 : 1;
        const int epi[4] = {EPI_QKV, EPI_ADD, EPI_SWIGLU, EPI_STORE};
        for (int s = 0; s < p.nseg; ++s) {
            GemvSeg& g = p.seg[s];
            g.A = s == 0 ? a : b;
            g.B = role == 2 ? b : g.A;
            g.pair = role == 2 ? PAIR_AB : PAIR_ADJ;
            g.epi = epi[role];
            g.expA = g.expB = -1;
            g.out = dy.as<float>() + (s == 0 ? 0 : rows);
            g.nq = g.A.rows;   // Q/K/V: every row a Q row, n_rot 0 (no rotation)
            g.resid = role == 1 ? dr.as<float>() : nullptr;
        }
        if (!dgemv_supported(p)) throw Error("op_dgemv: no compiled variant for this launch");
        launch_dgemv(p, nullptr);
        MI_HIP(hipDeviceSynchronize());
        MI_HIP(hipMemcpy(y, dy.p, out_rows * sizeof(float), hipMemcpyDeviceToHost));
        return 0;
    }
    MI_TRY(-1)
}

int32_t mi_op_gemv_bench(int32_t device, int32_t type, const void* raw, int32_t rows, int32_t K, int32_t iters,
                         float* median_us) {
    try {
        MI_HIP(hipSetDevice(device));
        ensure_attrs(device);
        std::vector<std::unique_ptr<DevBuf>> keep;
        const QMat m0 = upload_qmat(type, raw, rows, K, keep);
        // enough copies that consecutive launches stream from HBM, not the 256 MiB Infinity Cache
        size_t mbytes = 0;
        for (int k = 0; k < plane_count(type); ++k)
            mbytes += (size_t)(rows * m0.nb + kPlanePadSb) * plane_sb_bytes(type, k);
        const int copies = (int)std::min<size_t>(64, std::max<size_t>(1, (768ull << 20) / mbytes + 1));
        std::vector<QMat> mats(copies, m0);
        for (int c = 1; c < copies; ++c)
            for (int k = 0; k < plane_count(type); ++k) {
                const size_t n = (size_t)(rows * m0.nb + kPlanePadSb) * plane_sb_bytes(type, k);
                keep.push_back(std::make_unique<DevBuf>(n));
                MI_HIP(hipMemcpy(keep.back()->p, m0.p[k], n, hipMemcpyDeviceToDevice));
                mats[c].p[k] = keep.back()->as<uint8_t>();
            }
        DevBuf dx(K * sizeof(float)), dy(rows * sizeof(float));
        std::vector<float> hx(K);
        for (int i = 0; i < K; ++i) hx[i] = 0.5f + 0.001f * (float)(i % 97);
        MI_HIP(hipMemcpy(dx.p, hx.data(), K * sizeof(float), hipMemcpyHostToDevice));
        hipEvent_t a, b;
        MI_HIP(hipEventCreate(&a));
        MI_HIP(hipEventCreate(&b));
        std::vector<float> t;
        for (int i = 0; i < copies + 2; ++i)
            launch_gemv(single_gemv(mats[i % copies], dx.as<float>(), dy.as<float>()), nullptr);
        for (int i = 0; i < iters; ++i) {
            const GemvParams p = single_gemv(mats[i % copies], dx.as<float>(), dy.as<float>());
            MI_HIP(hipEventRecord(a, nullptr));
            launch_gemv(p, nullptr);
            MI_HIP(hipEventRecord(b, nullptr));
            MI_HIP(hipEventSynchronize(b));
            float ms = 0;
            MI_HIP(hipEventElapsedTime(&ms, a, b));
            t.push_back(ms * 1000.0f);
        }
        hipEventDestroy(a);
        hipEventDestroy(b);
        std::sort(t.begin(), t.end());
        *median_us = t.empty() ? 0.0f : t[t.size() / 2];
        return 0;
    }
    MI_TRY(-1)
}

int32_t mi_op_dequant(int32_t device, int32_t type, const void* raw, int32_t rows, int32_t K, float* out) {
    try {
        MI_HIP(hipSetDevice(device));
        std::vector<std::unique_ptr<DevBuf>> keep;
        const QMat m = upload_qmat(type, raw, rows, K, keep);
        DevBuf d((size_t)rows * K * sizeof(float));
        launch_dequant_rows(m, 0, rows, d.as<float>(), nullptr);
        MI_HIP(hipDeviceSynchronize());
        MI_HIP(hipMemcpy(out, d.p, (size_t)rows * K * sizeof(float), hipMemcpyDeviceToHost));
        return 0;
    }
    MI_TRY(-1)
}

int32_t mi_op_quantize_q8_K(int32_t device, const float* x, int32_t K, int8_t* qs, float* d, int32_t* bsums) {
    try {
        if (K % 256) throw Error("K must be a multiple of 256");
        MI_HIP(hipSetDevice(device));
        const int nb = K / 256;
        DevBuf dx(K * sizeof(float)), dq(K), dd(nb * sizeof(float)), db(nb * 16 * sizeof(int));
        MI_HIP(hipMemcpy(dx.p, x, K * sizeof(float), hipMemcpyHostToDevice));
        launch_quantize_q8k(dx.as<float>(), K, dq.as<int8_t>(), dd.as<float>(), db.as<int>(), nullptr);
        MI_HIP(hipDeviceSynchronize());
        MI_HIP(hipMemcpy(qs, dq.p, K, hipMemcpyDeviceToHost));
        MI_HIP(hipMemcpy(d, dd.p, nb * sizeof(float), hipMemcpyDeviceToHost));
        MI_HIP(hipMemcpy(bsums, db.p, nb * 16 * sizeof(int), hipMemcpyDeviceToHost));
        return 0;
    }
    MI_TRY(-1)
}

int32_t mi_op_topk(int32_t device, const float* logits, int32_t n, int32_t k, int32_t* ids, float* vals) {
    try {
        if (k < 0 || k > TOPK_MAX) throw Error("k must be in [0, 64]");
        MI_HIP(hipSetDevice(device));
        if (n < 1) throw Error("n must be positive");
        DevBuf dl(n * sizeof(float)), dc((size_t)topk_blocks(n) * TOPK_MAX * 8), di(TOPK_MAX * 4), dv(TOPK_MAX * 4);
        MI_HIP(hipMemcpy(dl.p, logits, n * sizeof(float), hipMemcpyHostToDevice));
        TopkParams tp{dl.as<float>(), n, dc.as<unsigned long long>(), di.as<int>(), dv.as<float>(), nullptr, nullptr};
        launch_topk(tp, nullptr);
        MI_HIP(hipDeviceSynchronize());
        std::vector<int> hi(TOPK_MAX);
        std::vector<float> hv(TOPK_MAX);
        MI_HIP(hipMemcpy(hi.data(), di.p, TOPK_MAX * 4, hipMemcpyDeviceToHost));
        MI_HIP(hipMemcpy(hv.data(), dv.p, TOPK_MAX * 4, hipMemcpyDeviceToHost));
        for (int i = 0; i < k; ++i) { ids[i] = hi[i]; vals[i] = hv[i]; }
        return k;
    }
    MI_TRY(-1)
}

int32_t mi_op_attention(int32_t device, int32_t n_head, int32_t n_head_kv, int32_t head_dim, int32_t n_cells,
                        const float* q, const uint16_t* k_f16, const uint16_t* v_f16, const int32_t* cell_pos,
                        int32_t pos, float* out) {
    try {
        if (n_head <= 0 || n_head_kv <= 0 || n_head % n_head_kv || n_cells <= 0 || head_dim <= 0)
            throw Error("attention: bad shape");
        MI_HIP(hipSetDevice(device));
        const int kv_dim = n_head_kv * head_dim, d = n_head * head_dim;
        const size_t kvb = (size_t)n_cells * kv_dim * sizeof(uint16_t);
        DevBuf dq(d * sizeof(float)), dk(kvb), dv(kvb), dcp(n_cells * sizeof(int)), dtp(4 * sizeof(int));
        DevBuf dsc((size_t)n_head * n_cells * sizeof(float)), dsm((size_t)ATTN_SMAX * n_head * sizeof(float));
        DevBuf dpo((size_t)ATTN_SMAX * d * sizeof(float)), dout(d * sizeof(float));
        MI_HIP(hipMemcpy(dq.p, q, d * sizeof(float), hipMemcpyHostToDevice));
        MI_HIP(hipMemcpy(dk.p, k_f16, kvb, hipMemcpyHostToDevice));
        MI_HIP(hipMemcpy(dv.p, v_f16, kvb, hipMemcpyHostToDevice));
        MI_HIP(hipMemcpy(dcp.p, cell_pos, n_cells * sizeof(int), hipMemcpyHostToDevice));
        const int tp[4] = {0, pos, n_cells - 1, 0};   // {token, query position, last cell}
        MI_HIP(hipMemcpy(dtp.p, tp, sizeof tp, hipMemcpyHostToDevice));
        AttnParams a{dq.as<float>(), dk.as<__half>(), dv.as<__half>(), dtp.as<int>(), dcp.as<int>(),
                     dsc.as<float>(), dsm.as<float>(), dpo.as<float>(), n_head, n_head_kv, head_dim, kv_dim,
                     n_cells, 1.0f / std::sqrt((float)head_dim)};
        a.fused = n_cells <= ATTN_SHORT ? 1 : 0;   // the decode graph's choice for this cell count
        // the decode graph's single-launch long-context kernel (exchange buffers zeroed, step 0)
        DevBuf dxf((size_t)n_head * ATTN_SMAX * 32 * sizeof(unsigned)), dxm((size_t)n_head * ATTN_SMAX * sizeof(float));
        DevBuf dxs((size_t)n_head * ATTN_SMAX * sizeof(double)), dst(16);
        MI_HIP(hipMemset(dxf.p, 0, (size_t)n_head * ATTN_SMAX * 32 * sizeof(unsigned)));
        MI_HIP(hipMemset(dst.p, 0, 16));
        a.xflags = dxf.as<unsigned>();
        a.xmax = dxm.as<float>();
        a.xsum = dxs.as<double>();
        a.step = dst.as<unsigned>();
        launch_attn(a, nullptr);
        launch_attn_combine(AttnPartials{dpo.as<float>(), n_head, head_dim}, dtp.as<int>(), dout.as<float>(), nullptr);
        MI_HIP(hipDeviceSynchronize());
        MI_HIP(hipMemcpy(out, dout.p, d * sizeof(float), hipMemcpyDeviceToHost));
        return 0;
    }
    MI_TRY(-1)
}

int32_t mi_op_gemm(int32_t device, int32_t type, const void* raw, const void* raw_up, int32_t rows, int32_t K,
                   int32_t ntok, const float* x, float* y) {
    try {
        if (!mmq32_supported(type)) throw Error("op_gemm: Q4_K / Q5_K / Q6_K / Q8_0 only");
        if (ntok < 1 || ntok > UB_MAX) throw Error("op_gemm: 1..512 token rows");
        if (rows < 1 || K < 256 || K % 256) throw Error("op_gemm: bad shape");
        MI_HIP(hipSetDevice(device));
        ensure_attrs(device);
        std::vector<std::unique_ptr<DevBuf>> keep;
        QMat A = upload_qmat(type, raw, rows, K, keep);
        QMat B = A;
        const bool pair = raw_up != nullptr;
        if (pair) B = upload_qmat(type, raw_up, rows, K, keep);
        DevBuf sw(mmq32_copy_bytes(A, pair));
        launch_mmq32_swizzle(A, pair ? &B : nullptr, sw.as<uint8_t>(), nullptr);
        A.sw = sw.as<uint8_t>();
        const int npad = (ntok + 31) / 32 * 32;
        DevBuf dx((size_t)ntok * K * sizeof(float)), dy((size_t)ntok * rows * sizeof(float));
        DevBuf dq((size_t)npad * K), ddT((size_t)npad * (K / 32) * sizeof(float)), dbs((size_t)npad * (K / 256) * 16);
        DevBuf dtp((size_t)ntok * 4 * sizeof(int));
        MI_HIP(hipMemset(dtp.p, 0, (size_t)ntok * 4 * sizeof(int)));
        MI_HIP(hipMemcpy(dx.p, x, (size_t)ntok * K * sizeof(float), hipMemcpyHostToDevice));
        ActQ8 act{dq.as<int8_t>(), ddT.as<float>(), dbs.as<int8_t>(), K, ntok, npad, type == T_Q8_0 ? 1 : 0};
        launch_quant_act(dx.as<float>(), K, nullptr, 0.0f, act, nullptr);
        // up to MMQS_MAX tokens: the short-batch GEMM (K-part sums, added by part_sum) as the
        // engine's verification batches take it; MI_MMQS_MAX=0: the tiled GEMM for every count
        const char* ms = getenv("MI_MMQS_MAX");
        const bool short_b = ntok <= (ms ? std::min(MMQS_MAX, std::max(0, atoi(ms))) : MMQS_MAX);   // as Ctx::Ctx clamps it
        if (short_b) {
            const int pst = pair ? 2 * rows : rows;
            DevBuf part((size_t)mmqs_parts(K) * ntok * pst * sizeof(float));
            const QMat* mats[1] = {&A};
            const int prow[1] = {0};
            const int kp = launch_mmqs(mats, prow, 1, pair, rows, act, part.as<float>(), pst, nullptr);
            launch_part_sum(part.as<float>(), kp, ntok, rows, pst, nullptr, 0, dy.as<float>(), rows, nullptr, pair ? rows : 0);
            MI_HIP(hipDeviceSynchronize());
        } else {
            GemmParams p;
            std::memset(&p, 0, sizeof(p));
            p.A = A;
            p.B = B;
            p.pair = pair ? PAIR_AB : PAIR_ADJ;
            p.epi = pair ? EPI_SWIGLU : EPI_STORE;
            p.K = K;
            p.ntok = ntok;
            p.tokpos = dtp.as<int>();
            p.out = dy.as<float>();
            p.out_stride = rows;
            launch_mmq32(p, act, nullptr, nullptr);
        }
        MI_HIP(hipDeviceSynchronize());
        MI_HIP(hipMemcpy(y, dy.p, (size_t)ntok * rows * sizeof(float), hipMemcpyDeviceToHost));
        return 0;
    }
    MI_TRY(-1)
}

int32_t mi_op_attention_batch(int32_t device, int32_t n_head, int32_t n_head_kv, int32_t head_dim, int32_t n_cells,
                              int32_t ntok, const float* q, const uint16_t* k_f16, const uint16_t* v_f16,
                              const int32_t* cell_pos, const int32_t* tok_cell, const int32_t* tok_pos, float* out) {
    try {
        if (n_head <= 0 || n_head_kv <= 0 || n_head % n_head_kv || n_cells <= 0 || ntok <= 0)
            throw Error("attention_batch: bad shape");
        if (!attn_mfma_supported(head_dim)) throw Error("attention_batch: head_dim 64 or 128");
        for (int t = 0; t < ntok; ++t) {
            if (tok_cell[t] < 0 || tok_cell[t] >= n_cells) throw Error("attention_batch: token cell out of range");
            if (t && tok_cell[t] <= tok_cell[t - 1]) throw Error("attention_batch: token cells must ascend");
        }
        MI_HIP(hipSetDevice(device));
        const int kv_dim = n_head_kv * head_dim, d = n_head * head_dim;
        const size_t kvb = (size_t)n_cells * kv_dim * sizeof(uint16_t);
        DevBuf dq((size_t)ntok * d * sizeof(float)), dk(kvb), dv(kvb), dcp(n_cells * sizeof(int));
        DevBuf dtp((size_t)ntok * 4 * sizeof(int)), dout((size_t)ntok * d * sizeof(float));
        std::vector<int> tp((size_t)ntok * 4, 0);
        for (int t = 0; t < ntok; ++t) {
            tp[t * 4 + 1] = tok_pos[t];
            tp[t * 4 + 2] = tok_cell[t];
        }
        MI_HIP(hipMemcpy(dq.p, q, (size_t)ntok * d * sizeof(float), hipMemcpyHostToDevice));
        MI_HIP(hipMemcpy(dk.p, k_f16, kvb, hipMemcpyHostToDevice));
        MI_HIP(hipMemcpy(dv.p, v_f16, kvb, hipMemcpyHostToDevice));
        MI_HIP(hipMemcpy(dcp.p, cell_pos, n_cells * sizeof(int), hipMemcpyHostToDevice));
        MI_HIP(hipMemcpy(dtp.p, tp.data(), tp.size() * sizeof(int), hipMemcpyHostToDevice));
        AttnParams a{dq.as<float>(), dk.as<__half>(), dv.as<__half>(), dtp.as<int>(), dcp.as<int>(),
                     nullptr, nullptr, nullptr, n_head, n_head_kv, head_dim, kv_dim,
                     n_cells, 1.0f / std::sqrt((float)head_dim)};
        launch_attn_mfma(a, ntok, dout.as<float>(), nullptr);
        MI_HIP(hipDeviceSynchronize());
        MI_HIP(hipMemcpy(out, dout.p, (size_t)ntok * d * sizeof(float), hipMemcpyDeviceToHost));
        return 0;
    }
    MI_TRY(-1)
}

}  // extern "C"
