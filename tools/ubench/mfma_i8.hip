// Lane maps and issue cost of the gfx950 i8 MFMAs that k_describe's row pass
// could use (v_mfma_i32_16x16x32_i8, v_mfma_i32_16x16x64_i8), checked with
// exact integer data against a host product (asymmetric A and B).
//   hipcc --offload-arch=gfx950 -O3 -o mfma_i8 mfma_i8.hip && ./mfma_i8
// Hypothesis (bf16 family, cdna_hip_programming.md §3): lane l holds
//   A[l & 15][K/4 * (l >> 4) + j], B[K/4 * (l >> 4) + j][l & 15], j < K/4,
//   C[4 * (l >> 4) + i][l & 15], i < 4.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x2v __attribute__((ext_vector_type(2)));

__global__ void k_mm32(const int8_t *A, const int8_t *B, int *C, uint64_t *cyc) {
    const int l = threadIdx.x;
    long a = 0, b = 0;
    for (int j = 0; j < 8; ++j) {
        a |= (long)(uint8_t)A[(l & 15) * 32 + 8 * (l >> 4) + j] << (8 * j);
        b |= (long)(uint8_t)B[(8 * (l >> 4) + j) * 16 + (l & 15)] << (8 * j);
    }
    i32x4 c = {0, 0, 0, 0};
    c = __builtin_amdgcn_mfma_i32_16x16x32_i8(a, b, c, 0, 0, 0);
    for (int i = 0; i < 4; ++i) C[(4 * (l >> 4) + i) * 16 + (l & 15)] = c[i];
    // issue cost: 64 dependent-free MFMAs on 4 accumulators
    i32x4 d0 = c, d1 = c, d2 = c, d3 = c;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < 16; ++r) {
        d0 = __builtin_amdgcn_mfma_i32_16x16x32_i8(a, b, d0, 0, 0, 0);
        d1 = __builtin_amdgcn_mfma_i32_16x16x32_i8(b, a, d1, 0, 0, 0);
        d2 = __builtin_amdgcn_mfma_i32_16x16x32_i8(a, a, d2, 0, 0, 0);
        d3 = __builtin_amdgcn_mfma_i32_16x16x32_i8(b, b, d3, 0, 0, 0);
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (l == 0) cyc[0] = t1 - t0;
    C[256 + l] = d0[0] + d1[1] + d2[2] + d3[3];
}

__global__ void k_mm64(const int8_t *A, const int8_t *B, int *C, uint64_t *cyc) {
    const int l = threadIdx.x;
    i32x4 a = {0, 0, 0, 0}, b = {0, 0, 0, 0};
    for (int j = 0; j < 16; ++j) {
        a[j >> 2] |= (int)(uint8_t)A[(l & 15) * 64 + 16 * (l >> 4) + j] << (8 * (j & 3));
        b[j >> 2] |= (int)(uint8_t)B[(16 * (l >> 4) + j) * 16 + (l & 15)] << (8 * (j & 3));
    }
    i32x4 c = {0, 0, 0, 0};
    c = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
    for (int i = 0; i < 4; ++i) C[(4 * (l >> 4) + i) * 16 + (l & 15)] = c[i];
    i32x4 d0 = c, d1 = c, d2 = c, d3 = c;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < 16; ++r) {
        d0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, d0, 0, 0, 0);
        d1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(b, a, d1, 0, 0, 0);
        d2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, a, d2, 0, 0, 0);
        d3 = __builtin_amdgcn_mfma_i32_16x16x64_i8(b, b, d3, 0, 0, 0);
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (l == 0) cyc[0] = t1 - t0;
    C[256 + l] = d0[0] + d1[1] + d2[2] + d3[3];
}

static int check(const char *name, int K, void (*kern)(const int8_t *, const int8_t *, int *, uint64_t *)) {
    std::vector<int8_t> A(16 * K), B(K * 16);
    for (int i = 0; i < 16 * K; ++i) A[i] = (int8_t)((i * 37 + 11) % 255 - 127);
    for (int i = 0; i < 16 * K; ++i) B[i] = (int8_t)((i * 53 + 5) % 251 - 125);
    int8_t *dA, *dB;
    int *dC;
    uint64_t *dcy;
    hipMalloc(&dA, A.size());
    hipMalloc(&dB, B.size());
    hipMalloc(&dC, (256 + 64) * 4);
    hipMalloc(&dcy, 8);
    hipMemcpy(dA, A.data(), A.size(), hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), B.size(), hipMemcpyHostToDevice);
    for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, dA, dB, dC, dcy);
    std::vector<int> C(256);
    uint64_t cy = 0;
    hipMemcpy(C.data(), dC, 256 * 4, hipMemcpyDeviceToHost);
    hipMemcpy(&cy, dcy, 8, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j) {
            int s = 0;
            for (int k = 0; k < K; ++k) s += A[i * K + k] * B[k * 16 + j];
            bad += s != C[i * 16 + j];
        }
    printf("%s: %d / 256 wrong under the assumed lane map; %.1f cycles (s_memtime) per MFMA, 4 accumulators\n", name,
           bad, cy / 64.0);
    hipFree(dA); hipFree(dB); hipFree(dC); hipFree(dcy);
    return bad;
}

int main() {
    int bad = check("v_mfma_i32_16x16x32_i8", 32, k_mm32);
    bad += check("v_mfma_i32_16x16x64_i8", 64, k_mm64);
    return bad ? 1 : 0;
}
