// orbx_wave.h -- wave64 cross-lane primitives on DPP (row_shr / row_bcast),
// which stay in the VALU instead of round-tripping through LDS the way
// ds_bpermute-based shuffles do.  All require every lane of the wave active.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace orbx {

template <int Ctrl, int RowMask = 0xF>
__device__ inline uint32_t dpp_or(uint32_t old, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, Ctrl, RowMask, 0xF, false);
}

// Orders this wave's LDS accesses: everything before is visible to every lane
// after (no workgroup barrier).
__device__ inline void wave_lds_fence() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

constexpr int kRowShr1 = 0x111, kRowShr2 = 0x112, kRowShr4 = 0x114, kRowShr8 = 0x118;
constexpr int kRowBcast15 = 0x142, kRowBcast31 = 0x143;

// Inclusive prefix sum over the 64 lanes: six in-place v_add_u32_dpp.  (The
// compiler's form of the same DPP sums is a v_mov 0, a v_mov_dpp and a v_add
// per step when it does not fold them: 3x the VALU.)  A lane without a
// row_shr source adds 0 (bound_ctrl); rows outside a row_bcast's row_mask are
// not written, i.e. keep their sum.  The s_nop 1 before each step covers the
// two wait states a DPP read of a VGPR the previous VALU wrote needs (the
// compiler inserts none inside asm).
__device__ inline int wave_incl_scan_i32(int v) {
    asm volatile(
        "s_nop 1\n\t"
        "v_add_u32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "s_nop 1\n\t"
        "v_add_u32_dpp %0, %0, %0 row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "s_nop 1\n\t"
        "v_add_u32_dpp %0, %0, %0 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "s_nop 1\n\t"
        "v_add_u32_dpp %0, %0, %0 row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "s_nop 1\n\t"
        "v_add_u32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_add_u32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf\n\t"
        "s_nop 1"
        : "+v"(v));
    return v;
}

// The same scan into a new register, leaving v as it was (no copy when the
// caller still needs the lane's own count).
__device__ inline int wave_incl_scan_i32_to(int v) {
    int r;
    asm volatile(
        "s_nop 1\n\t"
        "v_add_u32_dpp %0, %1, %1 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "s_nop 1\n\t"
        "v_add_u32_dpp %0, %0, %0 row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "s_nop 1\n\t"
        "v_add_u32_dpp %0, %0, %0 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "s_nop 1\n\t"
        "v_add_u32_dpp %0, %0, %0 row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "s_nop 1\n\t"
        "v_add_u32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_add_u32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf\n\t"
        "s_nop 1"
        : "=&v"(r)
        : "v"(v));
    return r;
}

// Inclusive prefix sum of packed pairs of 32-bit counters (the halves are
// scanned independently: callers pack counts that never carry into bit 32).
__device__ inline uint64_t wave_incl_scan_u64(uint64_t v) {
    const uint32_t lo = (uint32_t)wave_incl_scan_i32((int)(uint32_t)v);
    const uint32_t hi = (uint32_t)wave_incl_scan_i32((int)(uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// Sum over the wave, returned in every lane.
__device__ inline int wave_sum_i32(int v) {
    return __builtin_amdgcn_readlane(wave_incl_scan_i32(v), 63);
}

// Minimum over the wave, returned in every lane.
__device__ inline uint32_t wave_min_u32(uint32_t v) {
    v = min(v, dpp_or<kRowShr1>(~0u, v));
    v = min(v, dpp_or<kRowShr2>(~0u, v));
    v = min(v, dpp_or<kRowShr4>(~0u, v));
    v = min(v, dpp_or<kRowShr8>(~0u, v));
    v = min(v, dpp_or<kRowBcast15, 0xA>(~0u, v));
    v = min(v, dpp_or<kRowBcast31, 0xC>(~0u, v));
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// Maximum over the wave, returned in every lane.
__device__ inline uint32_t wave_max_u32(uint32_t v) {
    v = max(v, dpp_or<kRowShr1>(0u, v));
    v = max(v, dpp_or<kRowShr2>(0u, v));
    v = max(v, dpp_or<kRowShr4>(0u, v));
    v = max(v, dpp_or<kRowShr8>(0u, v));
    v = max(v, dpp_or<kRowBcast15, 0xA>(0u, v));
    v = max(v, dpp_or<kRowBcast31, 0xC>(0u, v));
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

}  // namespace orbx
