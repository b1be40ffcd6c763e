// Shared definitions for the MI355X (gfx950) quantized-inference engine.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <cstdint>
#include <cstddef>
#include <string>
#include <stdexcept>

namespace mi {

// ggml_type ids (llama.cpp b5187 ggml.h) -- the GGUF tensor type field.
enum GgmlType : int {
    T_F32 = 0, T_F16 = 1, T_Q8_0 = 8, T_Q4_K = 12, T_Q5_K = 13, T_Q6_K = 14, T_Q8_K = 15,
};

constexpr int QK_K = 256;

// Bytes of one GGUF block and the elements it covers.
inline int block_elems(int t) { return (t == T_F32 || t == T_F16) ? 1 : (t == T_Q8_0 ? 32 : 256); }
inline int block_bytes(int t) {
    switch (t) {
    case T_F32: return 4; case T_F16: return 2; case T_Q8_0: return 34;
    case T_Q4_K: return 144; case T_Q5_K: return 176; case T_Q6_K: return 210;
    default: return 0;
    }
}
inline bool is_quant(int t) { return t == T_Q8_0 || t == T_Q4_K || t == T_Q5_K || t == T_Q6_K; }

// On-device layout of a quantised matrix.  GGUF rows are arrays of blocks
// whose sizes (144/176/210/34 B) are not all 16-B aligned; at load time each
// tensor is split into "planes" so that every per-lane 16-byte load of the
// GEMV kernels is aligned and every plane streams contiguously.  Planes are
// [row][superblock][bytes]; a superblock is 256 weights (8 Q8_0 blocks).
//   Q4_K: p0 qs[128]  p1 hdr[16] = {f16 d, f16 dmin, u8 scales[12]}
//   Q5_K: p0 qs[128]  p1 qh[32]  p2 hdr[16]
//   Q6_K: p0 ql[128]  p1 qh[64]  p2 i8 scales[16]  p3 f16 d
//   Q8_0: p0 qs[256]  p1 f16 d[8]
constexpr int kPlanePadSb = 16;  // tail padding (superblocks) after every plane (ring GEMV over-reads)
inline int plane_count(int t) {
    switch (t) { case T_Q4_K: return 2; case T_Q5_K: return 3; case T_Q6_K: return 4;
                 case T_Q8_0: return 2; default: return 0; }
}
inline int plane_sb_bytes(int t, int p) {
    static const int q4k[] = {128, 16}, q5k[] = {128, 32, 16}, q6k[] = {128, 64, 16, 2}, q80[] = {256, 16};
    switch (t) {
    case T_Q4_K: return q4k[p]; case T_Q5_K: return q5k[p]; case T_Q6_K: return q6k[p];
    case T_Q8_0: return q80[p]; default: return 0;
    }
}

struct QMat {                // device view of one (expert of a) quantised matrix
    const uint8_t* p[4];     // planes
    int type;
    int rows;
    int K;                   // input features (multiple of 256)
    int nb;                  // superblocks per row = K/256
    long long expert_stride[4];  // bytes between experts, per plane (0 if dense)
    // Prompt-batch copy in MFMA-fragment order (mmq.hip, built per context on first use; null if
    // none): [row tile of 32][superblock][tile bytes], for a gate/up pair on the gate matrix with
    // 16 gate + 16 up rows per tile.
    const uint8_t* sw;
    long long sw_expert_stride;  // bytes between the experts' MFMA-order copies (MoE)
    int n_exp;                   // experts stacked in the planes (MoE *_exps tensors), else 1
};

struct Error : std::runtime_error { using std::runtime_error::runtime_error; };

void set_last_error(const std::string& s);
const char* last_error();

#define MI_HIP(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) \
    throw ::mi::Error(std::string("HIP error ") + hipGetErrorString(e_) + " at " + __FILE__ + ":" + std::to_string(__LINE__)); } while (0)

}  // namespace mi
