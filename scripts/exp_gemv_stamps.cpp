// Diagnostic: where does a GEMV launch spend its time?  Launches one GEMV on
// cold caches (a 1 GiB write in between, as the decode's 4 GB weight stream
// leaves them) with per-workgroup s_memrealtime stamps (100 MHz) and prints,
// over workgroups, the stamp offsets from the earliest workgroup start.
// Build: make -C scripts exp_gemv_stamps   Run: ./scripts/exp_gemv_stamps [type rows K pro]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "../blama_amd/csrc/kernels.h"

using namespace mi;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

int main(int argc, char** argv) {
    const int type = argc > 1 ? atoi(argv[1]) : T_Q4_K;
    const int rows = argc > 2 ? atoi(argv[2]) : 4096;
    const int K = argc > 3 ? atoi(argv[3]) : 4096;
    const int pro = argc > 4 ? atoi(argv[4]) : PRO_PLAIN;
    init_kernel_attributes();
    const int nb = K / 256;
    const long long nsb = (long long)rows * nb;
    const size_t raw_bytes = (size_t)rows * (K / block_elems(type)) * block_bytes(type);
    std::vector<uint8_t> h(raw_bytes);
    srand(1);
    for (auto& b : h) b = rand() & 0xFF;
    // sane fp16 scales (exponent small) so nothing is inf/nan
    const int bb = block_bytes(type), be = block_elems(type);
    for (size_t blk = 0; blk < raw_bytes / bb; ++blk) {
        uint8_t* p = h.data() + blk * bb;
        uint16_t d = 0x1400;   // ~1e-3
        if (type == T_Q6_K) memcpy(p + 208, &d, 2);
        else { memcpy(p, &d, 2); if (type != T_Q8_0) memcpy(p + 2, &d, 2); }
    }
    (void)be;
    uint8_t* raw;
    CK(hipMalloc(&raw, raw_bytes));
    CK(hipMemcpy(raw, h.data(), raw_bytes, hipMemcpyHostToDevice));
    QMat m{};
    m.type = type; m.rows = rows; m.K = K; m.nb = nb;
    uint8_t* planes[4] = {nullptr, nullptr, nullptr, nullptr};
    for (int k = 0; k < plane_count(type); ++k) {
        CK(hipMalloc(&planes[k], (size_t)(nsb + kPlanePadSb) * plane_sb_bytes(type, k)));
        m.p[k] = planes[k];
    }
    launch_repack(raw, type, rows, K, planes, nullptr);
    // a second copy of the matrix: launch B runs the same code on cold weights
    uint8_t* planes2[4] = {nullptr, nullptr, nullptr, nullptr};
    QMat m2 = m;
    for (int k = 0; k < plane_count(type); ++k) {
        CK(hipMalloc(&planes2[k], (size_t)(nsb + kPlanePadSb) * plane_sb_bytes(type, k)));
        m2.p[k] = planes2[k];
    }
    launch_repack(raw, type, rows, K, planes2, nullptr);
    float *x, *y, *nw;
    CK(hipMalloc(&x, K * 4));
    CK(hipMalloc(&nw, K * 4));
    CK(hipMalloc(&y, rows * 4 + 64));
    std::vector<float> hx(K, 0.5f);
    CK(hipMemcpy(x, hx.data(), K * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(nw, hx.data(), K * 4, hipMemcpyHostToDevice));
    uint8_t* flush;
    const size_t fl = 1ull << 30;
    CK(hipMalloc(&flush, fl));
    unsigned long long* st;
    CK(hipMalloc(&st, 256 * 8 * 8));

    GemvParams p;
    memset(&p, 0, sizeof(p));
    p.pro = pro;
    p.nslots = 1;
    p.x[0] = x;
    p.norm_w = nw;
    p.eps = 1e-5f;
    p.K = K;
    p.nseg = 1;
    p.seg[0].A = m;
    p.seg[0].pair = PAIR_ADJ;
    p.seg[0].epi = EPI_STORE;
    p.seg[0].units = (rows + 1) / 2;
    p.seg[0].expA = p.seg[0].expB = -1;
    p.seg[0].out = y;
    p.total_units = p.seg[0].units;
    p.need_q8k = type != T_Q8_0;
    p.need_q80 = type == T_Q8_0;
    p.stamps = st;
    const int grid = gemv_default_grid(p);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const double mb = (double)raw_bytes / 1e6;
    printf("type %d rows %d K %d pro %d grid %d  (%.1f MB)\n", type, rows, K, pro, grid, mb);
    printf("   A = first launch after a 1 GiB write (cold code, x, weights); B = the same kernel right\n"
           "   after on a second copy of the matrix (warm code and x, cold weights)\n");
    printf("   event_us | stamp offsets (us) from first WG entry, median / max over WGs:\n");
    printf("            | issued       rms-arrive   rms-leave    pro-end      pro-barrier  1st-ring     end\n");
    unsigned long long* st2;
    CK(hipMalloc(&st2, 256 * 8 * 8));
    auto show = [&](const char* tag, float ms, unsigned long long* dst) {
        std::vector<unsigned long long> hs(grid * 8);
        CK(hipMemcpy(hs.data(), dst, grid * 64, hipMemcpyDeviceToHost));
        unsigned long long t0 = ~0ull;
        for (int g = 0; g < grid; ++g) t0 = std::min(t0, hs[g * 8]);
        printf("%s %8.2f |", tag, ms * 1000);
        for (int k : {1, 5, 6, 7, 2, 3, 4}) {
            std::vector<double> v;
            for (int g = 0; g < grid; ++g)
                if (hs[g * 8 + k]) v.push_back((hs[g * 8 + k] - t0) / 100.0);
            std::sort(v.begin(), v.end());
            if (v.empty()) printf("   -    /  -   ");
            else printf(" %5.2f/%6.2f ", v[v.size() / 2], v.back());
        }
        printf("\n");
    };
    hipEvent_t c, d;
    CK(hipEventCreate(&c));
    CK(hipEventCreate(&d));
    for (int it = 0; it < 4; ++it) {
        CK(hipMemsetAsync(flush, it, fl, nullptr));
        CK(hipMemsetAsync(st, 0, 256 * 64, nullptr));
        CK(hipMemsetAsync(st2, 0, 256 * 64, nullptr));
        CK(hipEventRecord(a, nullptr));
        p.stamps = st;
        p.seg[0].A = m;
        launch_gemv(p, ROLE_GENERIC, grid, nullptr);
        CK(hipEventRecord(b, nullptr));
        p.stamps = st2;
        p.seg[0].A = m2;
        launch_gemv(p, ROLE_GENERIC, grid, nullptr);
        CK(hipEventRecord(d, nullptr));
        CK(hipEventSynchronize(d));
        float ms, ms2, ms3;
        CK(hipEventElapsedTime(&ms, a, b));
        CK(hipEventElapsedTime(&ms2, b, d));
        show("A", ms, st);
        show("B", ms2, st2);
        // C: B's matrix again (warm TLB entries and Infinity Cache lines for its weights)
        CK(hipMemsetAsync(st2, 0, 256 * 64, nullptr));
        CK(hipEventRecord(a, nullptr));
        launch_gemv(p, ROLE_GENERIC, grid, nullptr);
        CK(hipEventRecord(b, nullptr));
        CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&ms3, a, b));
        show("C", ms3, st2);
    }
    return 0;
}
