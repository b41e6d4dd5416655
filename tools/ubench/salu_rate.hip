// Issue rate of scalar ALU instructions per CU on gfx950: W waves per CU each
// run independent s_add_u32 chains (8 chains, 64 instructions per loop
// iteration); the chip-wide rate is SALU instructions / (kernel cycles x CUs).
// The CU has one scalar unit; this measures whether it issues one SALU
// instruction per clock (shared by all the CU's waves), the bound k_describe
// runs into (profiles/r03_salu_rate.txt).
//   hipcc --offload-arch=gfx950 -O3 -o salu_rate salu_rate.hip && ./salu_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define R8 "s_add_u32 %0, %0, %8\n s_add_u32 %1, %1, %8\n s_add_u32 %2, %2, %8\n s_add_u32 %3, %3, %8\n" \
           "s_add_u32 %4, %4, %8\n s_add_u32 %5, %5, %8\n s_add_u32 %6, %6, %8\n s_add_u32 %7, %7, %8\n"

__global__ void k_salu(uint32_t *out, int iters, uint32_t x, uint64_t *clk) {
    uint32_t a0 = x, a1 = x + 1, a2 = x + 2, a3 = x + 3, a4 = x + 4, a5 = x + 5, a6 = x + 6, a7 = x + 7;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
        asm volatile(R8 R8 R8 R8 R8 R8 R8 R8
                     : "+s"(a0), "+s"(a1), "+s"(a2), "+s"(a3), "+s"(a4), "+s"(a5), "+s"(a6), "+s"(a7)
                     : "s"(x)
                     : "scc");
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) {
        out[blockIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
        clk[2 * blockIdx.x] = t0;
        clk[2 * blockIdx.x + 1] = t1;
    }
}

// The same with v_add_u32 (full-rate VALU) in place of s_add_u32, for scale.
#define V8 "v_add_u32 %0, %0, %8\n v_add_u32 %1, %1, %8\n v_add_u32 %2, %2, %8\n v_add_u32 %3, %3, %8\n" \
           "v_add_u32 %4, %4, %8\n v_add_u32 %5, %5, %8\n v_add_u32 %6, %6, %8\n v_add_u32 %7, %7, %8\n"
__global__ void k_valu(uint32_t *out, int iters, uint32_t x, uint64_t *clk) {
    uint32_t a0 = x ^ threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
             a7 = a0 + 7;
    uint32_t y = x + (threadIdx.x & 1);
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
        asm volatile(V8 V8 V8 V8 V8 V8 V8 V8
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                     : "v"(y));
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t0;
        clk[2 * blockIdx.x + 1] = t1;
    }
}

int main() {
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount;
    const int iters = 2000;
    uint32_t *out;
    uint64_t *clk;
    hipMalloc(&out, 64 << 20);
    hipMalloc(&clk, 1 << 20);
    setvbuf(stdout, nullptr, _IONBF, 0);
    printf("CUs %d; per CU: waves, instructions per clock (s_memtime span of the slowest workgroup)\n", cus);
    for (int kind = 0; kind < 2; ++kind)
        for (int wpb : {1, 4}) {
            for (int bpc : {1, 2, 4, 8}) {
                const int blocks = cus * bpc;
                for (int rep = 0; rep < 2; ++rep) {
                    if (kind == 0) hipLaunchKernelGGL(k_salu, dim3(blocks), dim3(64 * wpb), 0, 0, out, iters, 3u, clk);
                    else hipLaunchKernelGGL(k_valu, dim3(blocks), dim3(64 * wpb), 0, 0, out, iters, 3u, clk);
                }
                hipDeviceSynchronize();
                std::vector<uint64_t> c(2 * blocks);
                hipMemcpy(c.data(), clk, c.size() * 8, hipMemcpyDeviceToHost);
                // (s_memtime is per-CU: take the longest workgroup span; all
                // workgroups of a launch are resident together)
                uint64_t span = 0;
                for (int b = 0; b < blocks; ++b) span = std::max(span, c[2 * b + 1] - c[2 * b]);
                const uint64_t t0 = 0, t1 = span;
                // s_memtime counts at the shader clock; instructions per CU:
                const double inst = (double)bpc * wpb * iters * 64.0;
                printf("%s  waves/CU %3d  per-CU %.3f instr/clk  (%.0f cycles)\n", kind == 0 ? "s_add_u32" : "v_add_u32",
                       bpc * wpb, inst / (double)(t1 - t0), (double)(t1 - t0));
            }
        }
    return 0;
}
