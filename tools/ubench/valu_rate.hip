// VALU issue rate per instruction kind: 8 waves per SIMD, each running
// independent chains of one instruction; prints ns per wave-instruction per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP8(X) X X X X X X X X
template <int K>
__global__ __launch_bounds__(256) void k_rate(uint32_t *out, int iters, uint32_t s) {
    uint32_t a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 + 1, a5 = a0 + 9, a6 = a0 ^ 5, a7 = a0 + 77;
    float f0 = a0, f1 = a1, f2 = a2, f3 = a3, f4 = a4, f5 = a5, f6 = a6, f7 = a7;
    for (int i = 0; i < iters; ++i) {
        if constexpr (K == 0) {   // v_pk_min_u16
            REP8(asm volatile("v_pk_min_u16 %0, %0, %8\n v_pk_min_u16 %1, %1, %8\n v_pk_min_u16 %2, %2, %8\n v_pk_min_u16 %3, %3, %8\n v_pk_min_u16 %4, %4, %8\n v_pk_min_u16 %5, %5, %8\n v_pk_min_u16 %6, %6, %8\n v_pk_min_u16 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s));)
        } else if constexpr (K == 1) {   // v_add_u32
            REP8(asm volatile("v_add_u32 %0, %0, %8\n v_add_u32 %1, %1, %8\n v_add_u32 %2, %2, %8\n v_add_u32 %3, %3, %8\n v_add_u32 %4, %4, %8\n v_add_u32 %5, %5, %8\n v_add_u32 %6, %6, %8\n v_add_u32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s));)
        } else if constexpr (K == 2) {   // v_perm_b32
            REP8(asm volatile("v_perm_b32 %0, %0, %1, %8\n v_perm_b32 %1, %1, %2, %8\n v_perm_b32 %2, %2, %3, %8\n v_perm_b32 %3, %3, %4, %8\n v_perm_b32 %4, %4, %5, %8\n v_perm_b32 %5, %5, %6, %8\n v_perm_b32 %6, %6, %7, %8\n v_perm_b32 %7, %7, %0, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s));)
        } else if constexpr (K == 3) {   // v_fma_f32
            REP8(asm volatile("v_fma_f32 %0, %0, %0, %8\n v_fma_f32 %1, %1, %1, %8\n v_fma_f32 %2, %2, %2, %8\n v_fma_f32 %3, %3, %3, %8\n v_fma_f32 %4, %4, %4, %8\n v_fma_f32 %5, %5, %5, %8\n v_fma_f32 %6, %6, %6, %8\n v_fma_f32 %7, %7, %7, %8" : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3), "+v"(f4), "+v"(f5), "+v"(f6), "+v"(f7) : "s"(s));)
        } else if constexpr (K == 4) {   // v_min_u32
            REP8(asm volatile("v_min_u32 %0, %0, %8\n v_min_u32 %1, %1, %8\n v_min_u32 %2, %2, %8\n v_min_u32 %3, %3, %8\n v_min_u32 %4, %4, %8\n v_min_u32 %5, %5, %8\n v_min_u32 %6, %6, %8\n v_min_u32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s));)
        } else if constexpr (K == 5) {   // v_max_f32
            REP8(asm volatile("v_max_f32 %0, %0, %8\n v_max_f32 %1, %1, %8\n v_max_f32 %2, %2, %8\n v_max_f32 %3, %3, %8\n v_max_f32 %4, %4, %8\n v_max_f32 %5, %5, %8\n v_max_f32 %6, %6, %8\n v_max_f32 %7, %7, %8" : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3), "+v"(f4), "+v"(f5), "+v"(f6), "+v"(f7) : "s"(s));)
        } else if constexpr (K == 6) {   // v_pk_max_f16
            REP8(asm volatile("v_pk_max_f16 %0, %0, %8\n v_pk_max_f16 %1, %1, %8\n v_pk_max_f16 %2, %2, %8\n v_pk_max_f16 %3, %3, %8\n v_pk_max_f16 %4, %4, %8\n v_pk_max_f16 %5, %5, %8\n v_pk_max_f16 %6, %6, %8\n v_pk_max_f16 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s));)
        } else if constexpr (K == 7) {   // v_max3_u32
            REP8(asm volatile("v_max3_u32 %0, %0, %8, %1\n v_max3_u32 %1, %1, %8, %2\n v_max3_u32 %2, %2, %8, %3\n v_max3_u32 %3, %3, %8, %4\n v_max3_u32 %4, %4, %8, %5\n v_max3_u32 %5, %5, %8, %6\n v_max3_u32 %6, %6, %8, %7\n v_max3_u32 %7, %7, %8, %0" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s));)
        } else if constexpr (K == 8) {   // v_pk_add_f32 (packed fp32)
            REP8(asm volatile("v_pk_add_f32 %0, %0, %4\n v_pk_add_f32 %1, %1, %4\n v_pk_add_f32 %2, %2, %4\n v_pk_add_f32 %3, %3, %4" : "+v"(*(double*)&f0), "+v"(*(double*)&f2), "+v"(*(double*)&f4), "+v"(*(double*)&f6) : "v"(0.0));)
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + (uint32_t)(f0 + f1 + f2 + f3 + f4 + f5 + f6 + f7);
}

template <int K>
void run(const char *name, uint32_t *d, int per_block_insts) {
    const int blocks = 256 * 8, iters = 2000;
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL(k_rate<K>, dim3(blocks), dim3(256), 0, 0, d, 10, 7u);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_rate<K>, dim3(blocks), dim3(256), 0, 0, d, iters, 7u);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    const double winst = (double)blocks * 4 * iters * per_block_insts;   // wave-instructions
    const double per_simd = winst / 1024.0;
    printf("%-14s %8.3f ms  %.3f ns per wave-instr per SIMD (%.2f cycles at 2.4 GHz)\n", name, ms, ms * 1e6 / per_simd, ms * 1e6 / per_simd * 2.4);
}

int main() {
    uint32_t *d; hipMalloc(&d, 4 * 256 * 256 * 8);
    run<0>("v_pk_min_u16", d, 64); run<1>("v_add_u32", d, 64); run<2>("v_perm_b32", d, 64);
    run<3>("v_fma_f32", d, 64); run<4>("v_min_u32", d, 64); run<5>("v_max_f32", d, 64);
    run<6>("v_pk_max_f16", d, 64); run<7>("v_max3_u32", d, 64); run<8>("v_pk_add_f32", d, 32);
    return 0;
}
