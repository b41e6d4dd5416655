// VALU issue rate per instruction kind and encoding: W waves per SIMD, each
// running 8 independent chains of one instruction; prints ns per
// wave-instruction per SIMD and, from s_memtime / s_memrealtime stamps taken
// around the loop by every workgroup (median), the shader clock the chip held
// during that launch, so the cycles per wave-instruction need no assumed clock.
//   VOP3 = 64-bit encoding (an SGPR operand, or a 3-source / packed op)
//   VOP2 = 32-bit encoding (_e32, VGPR src1)
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

#define REP8(X) X X X X X X X X
#define CH8(OP, A) OP " %0, " A "\n " OP " %1, " A "\n " OP " %2, " A "\n " OP " %3, " A "\n " \
                   OP " %4, " A "\n " OP " %5, " A "\n " OP " %6, " A "\n " OP " %7, " A "\n"

template <int K>
__global__ __launch_bounds__(256) void k_rate(uint32_t *out, uint64_t *stamps, int iters, uint32_t s) {
    uint32_t a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 + 1, a5 = a0 + 9, a6 = a0 ^ 5, a7 = a0 + 77;
    float f0 = a0, f1 = a1, f2 = a2, f3 = a3, f4 = a4, f5 = a5, f6 = a6, f7 = a7;
    uint32_t vs = s + threadIdx.x;   // a VGPR operand for the 32-bit encodings
    float vf = 1.0f + threadIdx.x * 1e-9f;
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; ++i) {
        if constexpr (K == 0) {   // v_pk_min_u16 (VOP3P)
            REP8(asm volatile(CH8("v_pk_min_u16", "%0, %8") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s));)
        } else if constexpr (K == 1) {   // v_add_u32 with an SGPR operand (VOP3)
            REP8(asm volatile(CH8("v_add_u32_e64", "%0, %8") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s));)
        } else if constexpr (K == 2) {   // v_perm_b32 (VOP3)
            REP8(asm volatile("v_perm_b32 %0, %0, %1, %8\n v_perm_b32 %1, %1, %2, %8\n v_perm_b32 %2, %2, %3, %8\n v_perm_b32 %3, %3, %4, %8\n v_perm_b32 %4, %4, %5, %8\n v_perm_b32 %5, %5, %6, %8\n v_perm_b32 %6, %6, %7, %8\n v_perm_b32 %7, %7, %0, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s));)
        } else if constexpr (K == 3) {   // v_fma_f32 (VOP3)
            REP8(asm volatile("v_fma_f32 %0, %0, %0, %8\n v_fma_f32 %1, %1, %1, %8\n v_fma_f32 %2, %2, %2, %8\n v_fma_f32 %3, %3, %3, %8\n v_fma_f32 %4, %4, %4, %8\n v_fma_f32 %5, %5, %5, %8\n v_fma_f32 %6, %6, %6, %8\n v_fma_f32 %7, %7, %7, %8" : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3), "+v"(f4), "+v"(f5), "+v"(f6), "+v"(f7) : "s"(s));)
        } else if constexpr (K == 4) {   // v_min_u32 with an SGPR operand (VOP3)
            REP8(asm volatile(CH8("v_min_u32_e64", "%0, %8") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s));)
        } else if constexpr (K == 5) {   // v_max_f32 with an SGPR operand (VOP3)
            REP8(asm volatile(CH8("v_max_f32_e64", "%0, %8") : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3), "+v"(f4), "+v"(f5), "+v"(f6), "+v"(f7) : "s"(s));)
        } else if constexpr (K == 6) {   // v_pk_max_f16 (VOP3P)
            REP8(asm volatile(CH8("v_pk_max_f16", "%0, %8") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s));)
        } else if constexpr (K == 7) {   // v_max3_u32 (VOP3)
            REP8(asm volatile("v_max3_u32 %0, %0, %8, %1\n v_max3_u32 %1, %1, %8, %2\n v_max3_u32 %2, %2, %8, %3\n v_max3_u32 %3, %3, %8, %4\n v_max3_u32 %4, %4, %8, %5\n v_max3_u32 %5, %5, %8, %6\n v_max3_u32 %6, %6, %8, %7\n v_max3_u32 %7, %7, %8, %0" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s));)
        } else if constexpr (K == 8) {   // v_pk_add_f32 (packed fp32, VOP3P)
            REP8(asm volatile("v_pk_add_f32 %0, %0, %4\n v_pk_add_f32 %1, %1, %4\n v_pk_add_f32 %2, %2, %4\n v_pk_add_f32 %3, %3, %4" : "+v"(*(double*)&f0), "+v"(*(double*)&f2), "+v"(*(double*)&f4), "+v"(*(double*)&f6) : "v"(0.0));)
        } else if constexpr (K == 9) {   // v_add_u32_e32 (VOP2, all VGPR)
            REP8(asm volatile(CH8("v_add_u32_e32", "%8, %0") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(vs));)
        } else if constexpr (K == 10) {  // v_min_u32_e32 (VOP2)
            REP8(asm volatile(CH8("v_min_u32_e32", "%8, %0") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(vs));)
        } else if constexpr (K == 11) {  // v_fmac_f32_e32 (VOP2)
            REP8(asm volatile(CH8("v_fmac_f32_e32", "%8, %8") : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3), "+v"(f4), "+v"(f5), "+v"(f6), "+v"(f7) : "v"(vf));)
        } else if constexpr (K == 12) {  // v_and_b32_e32 (VOP2)
            REP8(asm volatile(CH8("v_and_b32_e32", "%8, %0") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(vs));)
        } else if constexpr (K == 13) {  // v_add_u32_e64 with all-VGPR operands (VOP3 encoding, VOP2 opcode)
            REP8(asm volatile(CH8("v_add_u32_e64", "%8, %0") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(vs));)
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + (uint32_t)(f0 + f1 + f2 + f3 + f4 + f5 + f6 + f7);
    if (threadIdx.x == 0) {   // vector stores of the wave's stamps
        stamps[4 * blockIdx.x + 0] = t1 - t0;
        stamps[4 * blockIdx.x + 1] = r1 - r0;
    }
}

template <int K>
void run(const char *name, uint32_t *d, uint64_t *st, int per_iter_insts, int waves_per_simd) {
    const int blocks = 256 * waves_per_simd, iters = 2000;   // 256 threads = 4 waves = one per SIMD of a CU
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    for (int w = 0; w < 3; ++w)
        hipLaunchKernelGGL(k_rate<K>, dim3(blocks), dim3(256), 0, 0, d, st, iters, 7u);   // warm the clock
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_rate<K>, dim3(blocks), dim3(256), 0, 0, d, st, iters, 7u);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    std::vector<uint64_t> h(4 * blocks);
    hipMemcpy(h.data(), st, 8 * 4 * blocks, hipMemcpyDeviceToHost);
    std::vector<double> ghz(blocks);
    for (int b = 0; b < blocks; ++b) ghz[b] = h[4 * b + 1] ? 0.1 * (double)h[4 * b] / (double)h[4 * b + 1] : 0.0;
    std::nth_element(ghz.begin(), ghz.begin() + blocks / 2, ghz.end());
    const double clk = ghz[blocks / 2];
    const double winst = (double)blocks * 4 * iters * per_iter_insts;   // wave-instructions
    const double per_simd = winst / 1024.0;
    const double ns = ms * 1e6 / per_simd;
    printf("%-16s W=%-2d %8.3f ms  %.3f ns per wave-instr per SIMD  clock %.3f GHz (s_memtime)  %.2f cycles  "
           "(%.2f at 2.4 GHz)\n", name, waves_per_simd, ms, ns, clk, ns * clk, ns * 2.4);
}

int main() {
    uint32_t *d; hipMalloc(&d, 4 * 256 * 256 * 16);
    uint64_t *st; hipMalloc(&st, 8 * 4 * 256 * 16);
    for (int W : {8, 2}) {
        run<0>("v_pk_min_u16", d, st, 64, W); run<1>("v_add_u32_e64", d, st, 64, W); run<2>("v_perm_b32", d, st, 64, W);
        run<3>("v_fma_f32", d, st, 64, W); run<4>("v_min_u32_e64", d, st, 64, W); run<5>("v_max_f32_e64", d, st, 64, W);
        run<6>("v_pk_max_f16", d, st, 64, W); run<7>("v_max3_u32", d, st, 64, W); run<8>("v_pk_add_f32", d, st, 32, W);
        run<9>("v_add_u32_e32", d, st, 64, W); run<10>("v_min_u32_e32", d, st, 64, W);
        run<11>("v_fmac_f32_e32", d, st, 64, W); run<12>("v_and_b32_e32", d, st, 64, W);
        run<13>("v_add_u32_e64vv", d, st, 64, W);
    }
    run<9>("v_add_u32_e32", d, st, 64, 1); run<9>("v_add_u32_e32", d, st, 64, 4); run<9>("v_add_u32_e32", d, st, 64, 16);
    return 0;
}
