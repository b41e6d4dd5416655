// Issue cost per VALU opcode on gfx950, all operands in VGPRs unless the
// name says otherwise: 8 waves per SIMD, 8 independent chains per wave (every
// instruction's destination is read again 8 instructions later), 2000
// iterations of 64 instructions.  Cycles per wave-instruction per SIMD use the
// clock each launch held (s_memtime / s_memrealtime, median over workgroups).
// Finding this answers (profiles/r02_valu_ops.txt): which opcodes issue at the
// full wave64 rate (about 2 cycles) and which at half (about 4).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

#define REP8(X) X X X X X X X X
#define CH8(OP, A) OP " %0, " A "\n " OP " %1, " A "\n " OP " %2, " A "\n " OP " %3, " A "\n " \
                   OP " %4, " A "\n " OP " %5, " A "\n " OP " %6, " A "\n " OP " %7, " A "\n"
// %0..%7 = chain registers, %8 = x (VGPR), %9 = y (VGPR), %10 = s (SGPR)
#define OUTS "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
#define INS "v"(x), "v"(y), "s"(s)

#define OPK(NAME, TEXT, ...)                                                                       \
    __global__ __launch_bounds__(256) void k_##NAME(uint32_t *out, uint64_t *st, int iters, uint32_t s, \
                                                    uint32_t x0, uint32_t y0) {                      \
        uint32_t a0 = x0 ^ threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, \
                 a6 = a0 + 6, a7 = a0 + 7;                                                           \
        uint32_t x = x0 + (threadIdx.x & 1), y = y0;                                                 \
        const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();     \
        for (int i = 0; i < iters; ++i) { REP8(asm volatile(TEXT : OUTS : INS __VA_ARGS__);) }        \
        const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();     \
        out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;                 \
        if (threadIdx.x == 0) { st[2 * blockIdx.x] = t1 - t0; st[2 * blockIdx.x + 1] = r1 - r0; }    \
    }

#define ONE 0x3f800000u
// integer
OPK(add_u32, CH8("v_add_u32_e32", "%8, %0"))
OPK(sub_u32, CH8("v_sub_u32_e32", "%8, %0"))
OPK(and_b32, CH8("v_and_b32_e32", "%8, %0"))
OPK(or_b32, CH8("v_or_b32_e32", "%8, %0"))
OPK(xor_b32, CH8("v_xor_b32_e32", "%8, %0"))
OPK(lshrrev_b32, CH8("v_lshrrev_b32_e32", "%8, %0"))
OPK(lshlrev_b32, CH8("v_lshlrev_b32_e32", "%8, %0"))
OPK(min_u32, CH8("v_min_u32_e32", "%8, %0"))
OPK(max_u32, CH8("v_max_u32_e32", "%8, %0"))
OPK(min_i32, CH8("v_min_i32_e32", "%8, %0"))
OPK(mul_u32_u24, CH8("v_mul_u32_u24_e32", "%8, %0"))
OPK(mul_lo_u32, CH8("v_mul_lo_u32", "%8, %0"))
OPK(add_u32_sgpr, CH8("v_add_u32_e32", "%10, %0"))
OPK(add_u32_inline, CH8("v_add_u32_e32", "7, %0"))
OPK(add_u32_literal, CH8("v_add_u32_e32", "0x12345, %0"))
OPK(and_b32_literal, CH8("v_and_b32_e32", "0xff00ff, %0"))
// three-operand integer (VOP3)
OPK(add3_u32, CH8("v_add3_u32", "%0, %8, %9"))
OPK(lshl_add_u32, CH8("v_lshl_add_u32", "%0, 1, %8"))
OPK(lshl_or_b32, CH8("v_lshl_or_b32", "%8, 4, %0"))
OPK(and_or_b32, CH8("v_and_or_b32", "%0, %8, %9"))
OPK(or3_b32, CH8("v_or3_b32", "%0, %8, %9"))
OPK(xad_u32, CH8("v_xad_u32", "%0, %8, %9"))
OPK(min3_u32, CH8("v_min3_u32", "%0, %8, %9"))
OPK(max3_u32, CH8("v_max3_u32", "%0, %8, %9"))
OPK(med3_u32, CH8("v_med3_u32", "%0, %8, %9"))
OPK(mad_u32_u24, CH8("v_mad_u32_u24", "%0, %8, %9"))
OPK(bfe_u32, CH8("v_bfe_u32", "%0, %8, 8"))
OPK(bfi_b32, CH8("v_bfi_b32", "%8, %0, %9"))
OPK(alignbyte_b32, CH8("v_alignbyte_b32", "%0, %8, 1"))
OPK(alignbit_b32, CH8("v_alignbit_b32", "%0, %8, 3"))
OPK(perm_b32_vsel, CH8("v_perm_b32", "%0, %8, %9"))
OPK(perm_b32_ssel, CH8("v_perm_b32", "%0, %8, %10"))
OPK(sad_u8, CH8("v_sad_u8", "%0, %8, %9"))
OPK(sad_u32, CH8("v_sad_u32", "%0, %8, %9"))
OPK(msad_u8, CH8("v_msad_u8", "%0, %8, %9"))
OPK(cndmask_b32, CH8("v_cndmask_b32_e32", "%8, %0, vcc"), : "vcc")
OPK(bcnt_u32, CH8("v_bcnt_u32_b32", "%0, %8"))
OPK(dot4_u32_u8, CH8("v_dot4_u32_u8", "%8, %9, %0"))
OPK(dot2_u32_u16, CH8("v_dot2_u32_u16", "%8, %9, %0"))
// packed 16-bit (VOP3P)
OPK(pk_add_u16, CH8("v_pk_add_u16", "%0, %8"))
OPK(pk_sub_u16, CH8("v_pk_sub_u16", "%0, %8"))
OPK(pk_min_u16, CH8("v_pk_min_u16", "%0, %8"))
OPK(pk_max_u16, CH8("v_pk_max_u16", "%0, %8"))
OPK(pk_lshrrev_b16, CH8("v_pk_lshrrev_b16", "%8, %0"))
OPK(pk_mad_u16, CH8("v_pk_mad_u16", "%0, %8, %9"))
// 16-bit scalar-per-lane (VOP2 _e32 where it exists)
OPK(min_u16, CH8("v_min_u16_e32", "%8, %0"))
OPK(max_u16, CH8("v_max_u16_e32", "%8, %0"))
OPK(sub_u16, CH8("v_sub_u16_e32", "%8, %0"))
// float (x = 1.0f, y = 0: values stay finite and normal)
OPK(add_f32, CH8("v_add_f32_e32", "%9, %0"))
OPK(mul_f32, CH8("v_mul_f32_e32", "%8, %0"))
OPK(fmac_f32, CH8("v_fmac_f32_e32", "%8, %9"))
OPK(fma_f32, CH8("v_fma_f32", "%0, %8, %9"))
OPK(max_f32, CH8("v_max_f32_e32", "%8, %0"))
OPK(min_f32, CH8("v_min_f32_e32", "%8, %0"))
OPK(cvt_f32_u32, CH8("v_cvt_f32_u32_e32", "%0"))
OPK(cvt_u32_f32, CH8("v_cvt_u32_f32_e32", "%0"))
OPK(pk_add_f16, CH8("v_pk_add_f16", "%0, %9"))
OPK(pk_fma_f16, CH8("v_pk_fma_f16", "%0, %8, %9"))
OPK(rndne_f32, CH8("v_rndne_f32_e32", "%0"))
OPK(mov_b32, CH8("v_mov_b32_e32", "%8"))
// DPP / cross-lane
OPK(mov_dpp_shr1, CH8("v_mov_b32_dpp", "%8 row_shr:1 row_mask:0xf bank_mask:0xf"))
OPK(add_dpp_shr1, CH8("v_add_u32_dpp", "%8, %0 row_shr:1 row_mask:0xf bank_mask:0xf"))
OPK(min_dpp_shr1, CH8("v_min_u32_dpp", "%8, %0 row_shr:1 row_mask:0xf bank_mask:0xf"))

struct Op { const char *name; void (*k)(uint32_t *, uint64_t *, int, uint32_t, uint32_t, uint32_t); uint32_t x, y; };
#define E(N) {#N, k_##N, 3u, 5u}
#define EF(N) {#N, k_##N, ONE, 0u}
static const Op kOps[] = {
    E(add_u32), E(sub_u32), E(and_b32), E(or_b32), E(xor_b32), E(lshrrev_b32), E(lshlrev_b32), E(min_u32), E(max_u32),
    E(min_i32), E(mul_u32_u24), E(mul_lo_u32), E(add_u32_sgpr), E(add_u32_inline), E(add_u32_literal),
    E(and_b32_literal), E(add3_u32), E(lshl_add_u32), E(lshl_or_b32), E(and_or_b32), E(or3_b32), E(xad_u32),
    E(min3_u32), E(max3_u32), E(med3_u32), E(mad_u32_u24), E(bfe_u32), E(bfi_b32), E(alignbyte_b32),
    E(alignbit_b32), E(perm_b32_vsel), E(perm_b32_ssel), E(sad_u8), E(sad_u32), E(msad_u8), E(cndmask_b32),
    E(bcnt_u32), E(dot4_u32_u8), E(dot2_u32_u16), E(pk_add_u16), E(pk_sub_u16), E(pk_min_u16), E(pk_max_u16),
    E(pk_lshrrev_b16), E(pk_mad_u16), E(min_u16), E(max_u16), E(sub_u16), EF(add_f32), EF(mul_f32), EF(fmac_f32),
    EF(fma_f32), EF(max_f32), EF(min_f32), E(cvt_f32_u32), EF(cvt_u32_f32), E(pk_add_f16), E(pk_fma_f16),
    EF(rndne_f32), E(mov_b32), E(mov_dpp_shr1), E(add_dpp_shr1), E(min_dpp_shr1),
};

int main() {
    const int W = 8, blocks = 256 * W, iters = 2000;
    uint32_t *d; (void)hipMalloc(&d, 4 * 256 * blocks);
    uint64_t *st; (void)hipMalloc(&st, 16 * blocks);
    std::vector<uint64_t> h(2 * blocks);
    std::vector<double> ghz(blocks);
    printf("%-18s %9s %10s %8s\n", "opcode", "ms", "clock_GHz", "cycles");
    for (const Op &op : kOps) {
        for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(op.k, dim3(blocks), dim3(256), 0, 0, d, st, iters, 7u, op.x, op.y);
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(op.k, dim3(blocks), dim3(256), 0, 0, d, st, iters, 7u, op.x, op.y);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms; (void)hipEventElapsedTime(&ms, e0, e1);
        (void)hipMemcpy(h.data(), st, 16 * blocks, hipMemcpyDeviceToHost);
        for (int b = 0; b < blocks; ++b) ghz[b] = h[2 * b + 1] ? 0.1 * (double)h[2 * b] / (double)h[2 * b + 1] : 0.0;
        std::nth_element(ghz.begin(), ghz.begin() + blocks / 2, ghz.end());
        const double per_simd = (double)blocks * 4 * iters * 64 / 1024.0;
        printf("%-18s %9.3f %10.3f %8.2f\n", op.name, ms, ghz[blocks / 2], ms * 1e6 / per_simd * ghz[blocks / 2]);
        (void)hipEventDestroy(e0); (void)hipEventDestroy(e1);
    }
    return 0;
}
