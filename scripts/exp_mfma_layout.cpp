// Diagnostic: checks the operand / result lane layout assumed by the int8 MFMA GEMM
// (kernels.hip gemm_mfma_t) for v_mfma_i32_16x16x32_i8:
//   A (16x32): lane l holds A[l%16][8*(l/16) .. +7];  B (32x16): lane l holds B[8*(l/16) .. +7][l%16]
//   D (16x16): lane l, register i holds D[4*(l/16)+i][l%16]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef int v4i __attribute__((ext_vector_type(4)));
__global__ void k(const int8_t* A, const int8_t* B, int* D) {
    const int l = threadIdx.x;
    long a = 0, b = 0;
    int8_t* pa = reinterpret_cast<int8_t*>(&a);
    int8_t* pb = reinterpret_cast<int8_t*>(&b);
    for (int e = 0; e < 8; ++e) {
        pa[e] = A[(l % 16) * 32 + 8 * (l / 16) + e];
        pb[e] = B[(8 * (l / 16) + e) * 16 + (l % 16)];
    }
    v4i acc = {0, 0, 0, 0};
    acc = __builtin_amdgcn_mfma_i32_16x16x32_i8(a, b, acc, 0, 0, 0);
    for (int i = 0; i < 4; ++i) D[(4 * (l / 16) + i) * 16 + (l % 16)] = acc[i];
}
int main() {
    int8_t hA[16 * 32], hB[32 * 16];
    for (int i = 0; i < 16 * 32; ++i) hA[i] = (int8_t)((i * 37 + 11) % 255 - 127);
    for (int i = 0; i < 32 * 16; ++i) hB[i] = (int8_t)((i * 53 + 7) % 255 - 127);
    int8_t *dA, *dB;
    int* dD;
    hipMalloc(&dA, sizeof hA);
    hipMalloc(&dB, sizeof hB);
    hipMalloc(&dD, 256 * 4);
    hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
    hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dD);
    int hD[256];
    hipMemcpy(hD, dD, sizeof hD, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int r = 0; r < 16; ++r)
        for (int c = 0; c < 16; ++c) {
            int s = 0;
            for (int kk = 0; kk < 32; ++kk) s += hA[r * 32 + kk] * hB[kk * 16 + c];
            if (s != hD[r * 16 + c]) ++bad;
        }
    printf("mfma_i32_16x16x32_i8 layout: %s (%d mismatches)\n", bad ? "MISMATCH" : "ok", bad);
    return bad ? 1 : 0;
}
