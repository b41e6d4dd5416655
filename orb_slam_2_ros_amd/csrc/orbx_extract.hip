// orbx_extract.hip -- gfx950 kernels of the ORB extractor hot path.
//
// Stage                       reference (wjjcdy/orb_slam_2_ros)
//   k_resize   (x7 levels)    ComputePyramid, ORBextractor.cc:1152-1185 (+cv::resize)
//   k_blur     (all levels)   GaussianBlur 7x7 s=2, ORBextractor.cc:1128-1130
//   k_fast     (all cells)    cell loop + cv::FAST, ORBextractor.cc:820-863
//   k_quadtree (frame,level)  DistributeOctTree, ORBextractor.cc:561-787
//   k_describe (one wave/kp)  IC_Angle + computeOrbDescriptor + scaling,
//                             ORBextractor.cc:77-147, 1116-1148
// Every launch covers a whole batch of frames (grid.y / grid.z = frame).
// Integer / byte work bound by HBM, VALU issue or latency; k_describe runs its
// orientation moments and blur row pass as int8 MFMAs (15 per keypoint).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>

#include "orbx_device.h"
#include "orbx_math.h"
#include "orbx_wave.h"

namespace orbx {

// rBRIEF sampling points (ORBextractor.cc:150-408)
constexpr int kPatternPts[512][2] = {
#define ORBX_PATTERN_BEGIN
#define ORBX_PATTERN_END
#include "orb_pattern.inc"
#undef ORBX_PATTERN_BEGIN
#undef ORBX_PATTERN_END
};
// The descriptor's rotation multiplies them in float; k_describe fetches them
// as OCP fp8 e4m3fn (gfx950's format: every integer of magnitude <= 16 is
// exact) and widens a point (x, y) to an f32 pair with one
// v_cvt_pk_f32_fp8: lane l's 16 bytes are pairs 64 g + l, g = 0..3, as
// (x0, y0, x1, y1) -- one 16-byte load a lane instead of four.
constexpr uint32_t fp8_e4m3_int(int n) {   // n in [-15, 15]
    int a = n < 0 ? -n : n, e = 0;
    while (a >> (e + 1)) ++e;
    return n == 0 ? 0u : (uint32_t)((n < 0 ? 0x80 : 0) | ((e + 7) << 3) | (((a << 3) >> e) & 7));
}
struct PatternQ {
    uint32_t w[64][4];
    constexpr PatternQ() : w() {
        for (int l = 0; l < 64; ++l)
            for (int g = 0; g < 4; ++g) {
                const int j = 64 * g + l;
                w[l][g] = fp8_e4m3_int(kPatternPts[2 * j][0]) | fp8_e4m3_int(kPatternPts[2 * j][1]) << 8 |
                          fp8_e4m3_int(kPatternPts[2 * j + 1][0]) << 16 | fp8_e4m3_int(kPatternPts[2 * j + 1][1]) << 24;
            }
    }
};
constexpr bool pattern_in_fp8_range() {
    for (int i = 0; i < 512; ++i)
        for (int c = 0; c < 2; ++c)
            if (kPatternPts[i][c] < -15 || kPatternPts[i][c] > 15) return false;
    return true;
}
static_assert(pattern_in_fp8_range(), "the fp8 pattern table holds integers up to 15 exactly");
static_assert(fp8_e4m3_int(1) == 0x38 && fp8_e4m3_int(13) == 0x55 && fp8_e4m3_int(-3) == 0xC4, "e4m3fn, bias 7");

// c_disc_mask[ri][g]: byte k kept iff column 4g - 16 + k lies in row ri - 15
// of the orientation disc (kUmax, orbx_plan.h).
struct DiscMask {
    uint32_t m[32][8];
    constexpr DiscMask() : m() {
        for (int ri = 0; ri < 32; ++ri)
            for (int g = 0; g < 8; ++g) {
                uint32_t keep = 0;
                const int v = ri - 15, av = v < 0 ? -v : v;
                for (int k = 0; k < 4; ++k) {
                    const int u = 4 * g - 16 + k, au = u < 0 ? -u : u;
                    if (ri < 31 && au <= kUmax[av]) keep |= 0xFFu << (8 * k);
                }
                m[ri][g] = keep;
            }
    }
};
__constant__ DiscMask c_disc_mask = DiscMask();

// IC_Angle's moments on the matrix cores (k_describe): three int8 MFMAs over
// the staged patch (rows 0..47 as three 16-row tiles; the keypoint at patch
// column 23, so the disc, rows 6..36 and columns 8..38, lies in one 32-column
// window, columns 8..39).  Per (row tile rt, lane):
//   mask: the A-operand bytes kept, patch row 16 rt + (l & 15), window
//         columns 8 (l >> 4) + 0..7, inside the disc (kUmax);
//   b:    the B-operand bytes, k = 8 (l >> 4) + 0..7, output column j = l & 15:
//         j = 15: u = k - 15 (m10), j = 12 + rt: 1 (the rows' sums, weighted
//         by their v afterwards: m01), others 0.
constexpr int kDescKpCol = 23;   // the keypoint's patch column (k_describe staging)
struct MomTables {
    uint64_t mb[3][64][2];   // (mask, b): one 16-byte load a product
    constexpr MomTables() : mb() {
        for (int rt = 0; rt < 3; ++rt)
            for (int l = 0; l < 64; ++l) {
                uint64_t mk = 0, bb = 0;
                const int v = 16 * rt + (l & 15) - 21, av = v < 0 ? -v : v, j = l & 15;
                for (int jj = 0; jj < 8; ++jj) {
                    const int u = 8 + 8 * (l >> 4) + jj - kDescKpCol, au = u < 0 ? -u : u;
                    if (av <= 15 && au <= kUmax[av]) mk |= 0xFFull << (8 * jj);
                    const int w = j == 15 ? u : (j == 12 + rt ? 1 : 0);
                    bb |= (uint64_t)(uint8_t)(int8_t)w << (8 * jj);
                }
                mb[rt][l][0] = mk;
                mb[rt][l][1] = bb;
            }
    }
};

// Phase profiling (diagnostic build only, -DORBX_PHASE_PROF: tools/phase_prof.py):
// each wave adds the s_memtime cycles of its phases to g_phase[kernel][phase]
// (lane 0, vector atomics).  The product build compiles the marks away.
#ifdef ORBX_PHASE_PROF
// (256 slots per counter, by workgroup: one shared address per counter would
// serialise every wave's atomic at one L2 channel)
__device__ unsigned long long g_phase[3][8][256];
#define PHASE_START() uint64_t phase_t_ = __builtin_amdgcn_s_memtime()
#define PHASE_MARK(K, I)                                                                  \
    do {                                                                                  \
        const uint64_t phase_n_ = __builtin_amdgcn_s_memtime();                          \
        if ((threadIdx.x & 63) == 0)                                                      \
            atomicAdd(&g_phase[K][I][(blockIdx.x + 37 * blockIdx.y) & 255],              \
                      (unsigned long long)(phase_n_ - phase_t_));                         \
        phase_t_ = phase_n_;                                                              \
    } while (0)
#else
#define PHASE_START() uint64_t phase_t_ = 0; (void)phase_t_
#define PHASE_MARK(K, I) (void)0
#endif

// Per-phase instruction counts (tools/phase_valu.sh): a build with
// -DORBX_STOP_FAST=N / -DORBX_STOP_DESC=N compiles k_fast / k_describe only up
// to the end of phase N (k_fast: 1 staging, 2 iniThFAST compass + compaction,
// 3 its arc scores, 4 its NMS + output, no minThFAST pass; k_describe:
// 1 staging, 2 moments + row pass, 4 orientation + sample offsets + column
// pass), so SQ_INSTS_* differences between builds split the counts by phase.
// Results of such builds are wrong by design; 0 = the product.
#ifndef ORBX_STOP_FAST
#define ORBX_STOP_FAST 0
#endif
#ifndef ORBX_STOP_DESC
#define ORBX_STOP_DESC 0
#endif
constexpr int kStopFast = ORBX_STOP_FAST, kStopDesc = ORBX_STOP_DESC;

namespace {

constexpr int kThreads = 256;

__device__ inline const uint8_t *level_ptr(const DevPlan &p, const FrameBufs &fb, const LevelGeom &g,
                                           int l, int b, int &pitch) {
    if (l == 0) {
        pitch = fb.img0_pitch;
        return fb.img0 + (int64_t)b * fb.img0_stride;
    }
    pitch = g.pitch;
    return fb.pyr + (int64_t)b * p.pyr_bytes + g.pyr_off;
}

__device__ inline const uint8_t *level_ptr(const DevPlan &p, const FrameBufs &fb, int l, int b, int &pitch) {
    if (l == 0) {
        pitch = fb.img0_pitch;
        return fb.img0 + (int64_t)b * fb.img0_stride;
    }
    pitch = p.la[l].pitch;
    return fb.pyr + (int64_t)b * p.pyr_bytes + p.la[l].pyr_off;
}

// The dispatcher hands workgroup j (linear, x fastest) to XCD j % 8.  This
// maps j to a logical block index so that each XCD runs a contiguous range of
// logical blocks: consecutive blocks of one frame then share an XCD's L2
// (overlapping cell rings / keypoint patches hit instead of refetching).
constexpr int kXcds = 8;
__device__ inline int xcd_logical_block(int j, int n) {
    const int per = (int)((uint32_t)n / kXcds), rem = (int)((uint32_t)n % kXcds), xcd = (int)((uint32_t)j % kXcds),
              idx = (int)((uint32_t)j / kXcds);
    return xcd < rem ? xcd * (per + 1) + idx : rem * (per + 1) + (xcd - rem) * per + idx;
}

// (x, y) of the logical block of a 2-D grid.
__device__ inline void xcd_block_2d(int &bx, int &by) {
    const int n = gridDim.x * gridDim.y;
    const int L = xcd_logical_block(blockIdx.y * gridDim.x + blockIdx.x, n);
    // (the division runs on the VALU; readfirstlane hands the wave-uniform
    // results back to the scalar unit, so the code that depends on them stays SALU)
    by = __builtin_amdgcn_readfirstlane(L / gridDim.x);
    bx = __builtin_amdgcn_readfirstlane(L - by * gridDim.x);
}

// The same with the division by gridDim.x as a multiply-high by a host-made
// magic ceil(2^32 / gridDim.x), exact while (blocks) x gridDim.x < 2^32
// (checked by the launcher; magic 0 = divide): 3 scalar instructions instead of
// the ~20 of a 32-bit division.
__device__ inline void xcd_block_2d(int &bx, int &by, uint32_t magic) {
    const int n = gridDim.x * gridDim.y;
    const int L = xcd_logical_block(blockIdx.y * gridDim.x + blockIdx.x, n);
    by = magic ? (int)__umulhi((uint32_t)L, magic) : L / (int)gridDim.x;
    bx = L - by * (int)gridDim.x;
}

// The wave's index in its workgroup as a scalar: the compiler cannot prove
// threadIdx.x >> 6 wave-uniform, so everything derived from it would live in
// VGPRs and branch per lane.
__device__ inline int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }
// set bits of m below this lane (v_mbcnt_lo / hi: two VALU, where a masked popcount takes four)
// The lane mask of a comparison straight from its v_cmp (an SGPR pair).
// __ballot of a bool that also steers a branch is lowered as v_cndmask 0 / 1
// plus a second v_cmp; these keep the compare's own mask.
__device__ inline uint64_t lanes_lt(int a, int b) { return __builtin_amdgcn_sicmp(a, b, 40); }   // ICMP_SLT
__device__ inline uint64_t lanes_gt(int a, int b) { return __builtin_amdgcn_sicmp(a, b, 38); }   // ICMP_SGT

__device__ inline int mbcnt64(uint64_t m) {
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ inline int reflect101(int v, int n) {
    // BORDER_REFLECT_101 for the 3-px halo of a >= 4 px image.
    v = v < 0 ? -v : v;
    return v >= n ? 2 * n - v - 2 : v;
}

__device__ inline uint32_t pack_key(int x, int y, int score) {
    return (uint32_t)x | ((uint32_t)y << 12) | ((uint32_t)score << 24);
}

// ---- wave / block helpers (wave64) ----------------------------------------
// Exclusive scan of a[0..m) (uint64) in LDS by the whole NT-thread block.
// ws: NT / 64 uint64 of LDS scratch.  Returns the total.  Ends with a barrier.
template <int NT = kThreads>
__device__ uint64_t block_excl_scan_u64(uint64_t *a, int m, uint64_t *ws) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int per = (m + NT - 1) / NT;
    const int s = min(tid * per, m), e = min(s + per, m);
    uint64_t local = 0;
    for (int i = s; i < e; ++i) local += a[i];
    const uint64_t incl = wave_incl_scan_u64(local);
    if (lane == 63) ws[wave] = incl;
    __syncthreads();
    uint64_t base = 0, total = 0;
    for (int w = 0; w < NT / 64; ++w) {
        if (w < wave) base += ws[w];
        total += ws[w];
    }
    uint64_t run = base + incl - local;
    for (int i = s; i < e; ++i) {
        const uint64_t v = a[i];
        a[i] = run;
        run += v;
    }
    __syncthreads();
    return total;
}

// Exclusive scan of one int per thread across the block; returns total.
__device__ int block_excl_scan_i32(int v, int *total, int *ws) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int incl = wave_incl_scan_i32(v);
    if (lane == 63) ws[wave] = incl;
    __syncthreads();
    int base = 0, tot = 0;
    for (int w = 0; w < kThreads / 64; ++w) {
        if (w < wave) base += ws[w];
        tot += ws[w];
    }
    __syncthreads();
    *total = tot;
    return base + incl - v;
}

// Unsigned 24-bit multiply (v_mul_u32_u24, full rate); both operands must be
// in [0, 2^24), which every use below guarantees.
// (__umul24: the masked-product form let the compiler pick v_mul_lo_u32, a
// quarter-rate op, whenever one operand was a scalar it had proven small)
__device__ inline int mul24u(int a, int b) { return (int)__umul24((uint32_t)a, (uint32_t)b); }

// Small exact integer division for the index walks (a < 2^15, b <= 255).
__device__ inline int div_small(int a, int b) {
    return (int)(((float)a + 0.5f) * __builtin_amdgcn_rcpf((float)b));
}

// ===========================================================================
// Wave-cooperative staging of an image rectangle into LDS with aligned dword
// loads, NB in flight per lane before any LDS store (a rectangle of up to
// 64 * NB dwords costs one global round trip).  Pixel (r, c) of the
// rectangle lands at dst[r * ds + o + c]; returns o = x0 & 3.  The caller
// guarantees a 4-aligned image base and pitch and that the aligned span
// [x0 & ~3, x0 + nc rounded up to 4) lies inside the row's pitch.
// ===========================================================================
template <int NB = 8>
__device__ inline int wave_stage_rect(uint8_t *dst, int ds, const uint8_t *img, int pitch, int y0, int x0,
                                      int nr, int nc, int lane) {
    const int xa = x0 & ~3, o = x0 - xa;
    const int nd = (o + nc + 3) >> 2;
    const int total = nr * nd;
    const int dr = div_small(64, nd), dk = 64 - dr * nd;
    const int r_l = div_small(lane, nd), k_l = lane - r_l * nd;
    const uint8_t *base = img + (int64_t)y0 * pitch + xa;
    for (int i0 = 0, r0 = r_l, k0 = k_l; i0 < total; i0 += 64 * NB) {
        uint32_t v[NB];
        int r = r0, k = k0;
#pragma unroll
        for (int j = 0; j < NB; ++j) {
            if (i0 + 64 * j + lane < total) v[j] = *reinterpret_cast<const uint32_t *>(base + mul24u(r, pitch) + 4 * k);
            r += dr; k += dk; if (k >= nd) { k -= nd; ++r; }
        }
        r = r0; k = k0;
#pragma unroll
        for (int j = 0; j < NB; ++j) {
            if (i0 + 64 * j + lane < total) *reinterpret_cast<uint32_t *>(dst + mul24u(r, ds) + 4 * k) = v[j];
            r += dr; k += dk; if (k >= nd) { k -= nd; ++r; }
        }
        r0 = r; k0 = k;
    }
    return o;
}


// A raw buffer resource over a wave-uniform base: loads through it take a
// 32-bit per-lane offset plus a scalar offset, so no 64-bit address
// arithmetic runs on the VALU (2 VALU per global_load otherwise).  The range
// check is left open (the callers never read past their rectangles).
__device__ inline __amdgpu_buffer_rsrc_t wave_rsrc(const void *base) {
    const uint64_t a = reinterpret_cast<uint64_t>(base);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(((uint64_t)hi << 32) | lo), (short)0,
                                             0x7FFFFFF0, 0x00020000);
}

__device__ inline uint32_t buf_ld32(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
    return __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0);
}

// The same staging with a fixed lane -> (row in pass, dword) map, so each
// load's address is one uniform row offset plus a fixed per-lane offset (no
// per-load index walk): rows of at most 64 dwords go 64 / nd rows per pass;
// wider rows one row per pass in 64-dword chunks, NB rows per round.  BUF:
// buffer loads, the row offset a scalar operand and the lane offset a 32-bit
// VGPR (k_fast, k_describe: -2 % time); the resize windows (up to 24
// rows in flight) measured 2 % slower that way and keep global loads.
// X80: the bytes are stored XOR 0x80 (as signed I - 128, k_describe's int8 MFMAs).
// FO >= 0 (BUF only): the rectangle lands at dst column FO whatever x0's
// alignment (the loads are then unaligned dwords from x0 - FO; the buffer
// base stays 4-aligned and the remainder goes into the lane offset).
template <int NB = 8, bool BUF = true, bool X80 = false, int FO = -1>
__device__ inline int wave_stage_rows(uint8_t *dst, int ds, const uint8_t *img, int pitch, int y0, int x0, int nr,
                                      int nc, int lane) {
    constexpr uint32_t kX = X80 ? 0x80808080u : 0u;
    static_assert(FO < 0 || BUF, "a forced column offset needs the buffer loads");
    // (all wave-uniform: row offsets then come from the scalar unit)
    pitch = __builtin_amdgcn_readfirstlane(pitch);
    ds = __builtin_amdgcn_readfirstlane(ds);
    nr = __builtin_amdgcn_readfirstlane(nr);
    const int xs = FO >= 0 ? x0 - FO : x0;                  // first byte loaded
    const int xa = xs & ~3, o = FO >= 0 ? FO : x0 - xa;
    const int sh = FO >= 0 ? xs - xa : 0;                   // load misalignment
    const int nd = (o + nc + 3) >> 2;
    const uint8_t *gsrc = img + (int64_t)y0 * pitch + xa;
    const __amdgpu_buffer_rsrc_t src = wave_rsrc(gsrc);
    auto load = [&](int voff, int row) -> uint32_t {
        if constexpr (BUF) return buf_ld32(src, voff, __builtin_amdgcn_readfirstlane(row * pitch));
        else return *reinterpret_cast<const uint32_t *>(gsrc + mul24u(row, pitch) + voff);
    };
    if (nd > 64) {
        for (int c0 = 0; c0 < nd; c0 += 64) {
            const bool on = c0 + lane < nd;
            const int voff = 4 * (c0 + lane) + sh;
            for (int r0 = 0; r0 < nr; r0 += NB) {
                uint32_t v[NB];
#pragma unroll
                for (int j = 0; j < NB; ++j)
                    if (on && r0 + j < nr) v[j] = load(voff, r0 + j);
#pragma unroll
                for (int j = 0; j < NB; ++j)
                    if (on && r0 + j < nr) *reinterpret_cast<uint32_t *>(dst + mul24u(r0 + j, ds) + voff - sh) = v[j] ^ kX;
            }
        }
        return o;
    }
    const int R = __builtin_amdgcn_readfirstlane(div_small(64, nd));   // rows per pass (wave-uniform)
    const int rl = div_small(lane, nd), k = lane - mul24u(rl, nd);
    const int voff = mul24u(rl, pitch) + 4 * k + sh, loff = mul24u(rl, ds) + 4 * k;
    const int rmax = rl < R ? nr - rl : 0;   // this lane loads rows r0 + j R < rmax
    // the row offsets as scalar multiples of R * pitch (a v_mul_lo_u32 per
    // load otherwise: quarter rate, then a readfirstlane)
    const int Rp = __builtin_amdgcn_readfirstlane(R * pitch);
    for (int r0 = 0, s0 = 0; r0 < nr; r0 += NB * R, s0 += NB * Rp) {
        uint32_t v[NB];
#pragma unroll
        for (int j = 0; j < NB; ++j) {
            if constexpr (BUF) {
                if (r0 + mul24u(j, R) < rmax) v[j] = buf_ld32(src, voff, s0 + j * Rp);
            } else {
                if (r0 + j * R < rmax) v[j] = load(voff, r0 + j * R);
            }
        }
#pragma unroll
        for (int j = 0; j < NB; ++j)
            if constexpr (BUF) {
                if (r0 + mul24u(j, R) < rmax) *reinterpret_cast<uint32_t *>(dst + mul24u(r0 + mul24u(j, R), ds) + loff) = v[j] ^ kX;
            } else {
                if (r0 + j * R < rmax) *reinterpret_cast<uint32_t *>(dst + mul24u(r0 + j * R, ds) + loff) = v[j] ^ kX;
            }
    }
    return o;
}

// ===========================================================================
// K1: bilinear level l from level l-1 (cv::resize INTER_LINEAR 8U, OpenCV 3.2
// fixed point; SSE2 vertical rounding on the leading columns, scalar tail).
// Block = 256 x 8 output pixels; the source window it needs (<= kResRows x
// kResCols bytes, checked on the host) is staged in LDS by coalesced loads.
// Thread = 4 consecutive columns x 2 rows, one u32 store per row.
// ===========================================================================
constexpr int kResTW = 256, kResTH = 16, kResRows = 32, kResCols = 544;
typedef __attribute__((address_space(3))) uint8_t lds_u8;   // LDS byte (keeps ds_read_u8)
constexpr int kResRowsPerThread = kResTH / 4;

__global__ __launch_bounds__(kThreads) void k_resize(DevPlan p, FrameBufs fb, int l) {
    __shared__ uint8_t win[kResRows * kResCols];
    const LevelGeom g = p.lv[l];
    const LevelGeom gs = p.lv[l - 1];
    const int tid = threadIdx.x;
    const int L = xcd_logical_block((blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x,
                                    gridDim.x * gridDim.y * gridDim.z);
    const int bxy = L % (gridDim.x * gridDim.y), b = L / (gridDim.x * gridDim.y);
    const int x0 = (bxy % gridDim.x) * kResTW, y0 = (bxy / gridDim.x) * kResTH;
    const ResizeTap *xt = p.xtaps + g.xtab_off;
    const ResizeTap *yt = p.ytaps + g.ytab_off;
    // this thread's taps: 4 columns x kResRowsPerThread rows, fetched before the
    // window so their latency overlaps the staging loads
    const int xb = x0 + 4 * (tid & 63);
    const int yb = y0 + kResRowsPerThread * (tid >> 6);
    ResizeTap tx[4], ty[kResRowsPerThread];
#pragma unroll
    for (int k = 0; k < 4; ++k) tx[k] = xt[min(xb + k, g.w - 1)];
#pragma unroll
    for (int k = 0; k < kResRowsPerThread; ++k) ty[k] = yt[min(yb + k, g.h - 1)];
    const int xl = min(x0 + kResTW, g.w) - 1, yl = min(y0 + kResTH, g.h) - 1;
    const int c_lo = xt[x0].src, c_hi = min((int)xt[xl].src + 1, gs.w - 1);
    const int r_lo = min(max((int)yt[y0].src, 0), gs.h - 1);
    const int r_hi = min(max((int)yt[yl].src + 1, 0), gs.h - 1);
    const int nc = c_hi - c_lo + 1, nr = r_hi - r_lo + 1;
    int spitch;
    const uint8_t *src = level_ptr(p, fb, gs, l - 1, b, spitch);
    // each wave stages a quarter of the window's rows (aligned dword loads)
    const int wv = tid >> 6;
    const int ra = (nr * wv) >> 2, rb = (nr * (wv + 1)) >> 2;
    int o = c_lo & 3;
    if (rb > ra) o = wave_stage_rect(win + ra * kResCols, kResCols, src, spitch, r_lo + ra, c_lo, rb - ra, nc, tid & 63);
    __syncthreads();
    if (xb >= g.w) return;
    uint8_t *dst = fb.pyr + (int64_t)b * p.pyr_bytes + g.pyr_off;
    // An opaque 1: stops the load vectorizer from fusing the tap pair S[sx],
    // S[sx+1] into one unaligned ds_read_u16 (LDS unaligned-access stalls).
    int one = 1;
    asm volatile("" : "+s"(one));
#pragma unroll
    for (int rr = 0; rr < kResRowsPerThread; ++rr) {
        const int y = yb + rr;
        if (y >= g.h) break;
        const lds_u8 *S0 = (const lds_u8 *)(win + mul24u(min(max((int)ty[rr].src, 0), gs.h - 1) - r_lo, kResCols) + o - c_lo);
        const lds_u8 *S1 = (const lds_u8 *)(win + mul24u(min(max((int)ty[rr].src + 1, 0), gs.h - 1) - r_lo, kResCols) + o - c_lo);
        const int b0 = ty[rr].a0, b1 = ty[rr].a1;
        uint32_t packed = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            // Branch-free: tail columns carry coefficients (2048, 0) (orbx_plan.h);
            // every product fits 24-bit operands (S <= 255, a <= 2048, h < 2^20).
            const int sx = tx[k].src, sx1 = sx + one;
            const int h0 = mul24u(S0[sx], tx[k].a0) + mul24u(S0[sx1], tx[k].a1);
            const int h1 = mul24u(S1[sx], tx[k].a0) + mul24u(S1[sx1], tx[k].a1);
            // SSE2 columns: _mm_packs_epi32(h>>4); _mm_mulhi_epi16; _mm_adds_epi16; +2; >>2; packus
            const int v_simd = ((mul24u(h0 >> 4, b0) >> 16) + (mul24u(h1 >> 4, b1) >> 16) + 2) >> 2;
            // scalar tail: FixedPtCast<int, uchar, 22>
            const int v_tail = (mul24u(h0, b0) + mul24u(h1, b1) + (1 << 21)) >> 22;
            const int v = (tx[k].mode & 2) ? v_simd : v_tail;
            packed |= (uint32_t)min(max(v, 0), 255) << (8 * k);
        }
        *reinterpret_cast<uint32_t *>(dst + mul24u(y, g.pitch) + xb) = packed;
    }
}

// ===========================================================================
// K1 (wave tiles): the same resize with every wave independent.  A wave owns
// a 4*twg x (64/twg)*kResizeK output tile (ResizeWave, chosen per level so
// narrow levels waste few lanes), stages the source window it needs in its
// own LDS slice and writes 4 columns x kResizeK rows per lane.  The window
// bounds come from the same double/float arithmetic as the tap tables, so the
// staging loads and the tap loads go out together.  Per source row a lane
// reads 3 dwords, realigns them, gathers each column's pixel pair (S[sx],
// S[sx+1]) with one v_perm and applies the horizontal taps with one
// v_dot2_u32_u16; the vertical pass is OpenCV's fixed point as above.
// ===========================================================================
typedef unsigned short u16x2_t __attribute__((ext_vector_type(2)));
#ifndef ORBX_RS_REUSE
#define ORBX_RS_REUSE 1
#endif
#ifndef ORBX_RS_MULHI
#define ORBX_RS_MULHI 1
#endif

__host__ __device__ inline int resize_src_raw(int d, double scale) {
#ifdef __HIP_DEVICE_COMPILE__
    const float f = __double2float_rn(__dsub_rn(__dmul_rn(__dadd_rn((double)d, 0.5), scale), 0.5));
    return (int)floorf(f);
#else
    const float f = (float)((d + 0.5) * scale - 0.5);
    return floor_i(f);
#endif
}

// The SSE2 columns' vertical pass of 4 columns, packed into one dword:
// ((h0 >> 4) b0 >> 16) + ((h1 >> 4) b1 >> 16), + 2, >> 2 (each sum <= 1022),
// the >> 16 as the high half of (h & ~15) x (b << 12) (24-bit operands, bb =
// b << 12).  Two sums share a dword (s0 + s1 << 16 + 0x20002, no carry between
// the halves), one shift rounds both, one v_perm packs the four bytes.
__device__ inline uint32_t resize_vpass_simd(const uint32_t h0[4], const uint32_t h1[4], uint32_t bb0, uint32_t bb1) {
    uint32_t sm[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        sm[k] = (uint32_t)(((uint64_t)(h0[k] & 0xFFFF0u) * bb0) >> 32) + (uint32_t)(((uint64_t)(h1[k] & 0xFFFF0u) * bb1) >> 32);
    const uint32_t p01 = ((sm[1] << 16) + sm[0] + 0x00020002u) >> 2;
    const uint32_t p23 = ((sm[3] << 16) + sm[2] + 0x00020002u) >> 2;
    return __builtin_amdgcn_perm(p23, p01, 0x06040200u);
}

// One wave tile (ResizeWave) of level l of frame b; `win` is the wave's LDS
// slice (a.win_bytes).
template <int NB>
__device__ inline void resize_tile(const DevPlan &p, const FrameBufs &fb, int l, const ResizeWave &a, int b, int tile,
                                   int lane, uint8_t *win) {
    wave_lds_fence();   // the slice's previous window is consumed
    const int ty = tile / a.ntx, tx = tile - ty * a.ntx;
    const LevelArgs g = p.la[l], gs = p.la[l - 1];
    const int twg = a.twg, lr = lane >> a.twg_shift, lg = lane & (twg - 1);
    const int TH = (64 >> a.twg_shift) * kResizeK;
    const int x0 = tx * 4 * twg, y0 = ty * TH;
    const int xb = x0 + 4 * lg, yb = y0 + lr * kResizeK;
    // taps of this lane's 4 columns and kResizeK rows (independent of the window loads)
    // (buffer loads: 32-bit lane offsets from the wave's table bases)
    static_assert(sizeof(ResizeTap) == 8, "one dwordx2 a tap");
    const __amdgpu_buffer_rsrc_t xt = wave_rsrc(p.xtaps + a.xtab_off), yt = wave_rsrc(p.ytaps + a.ytab_off);
    ResizeTap txk[4], tyk[kResizeK];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        txk[k] = __builtin_bit_cast(ResizeTap, __builtin_amdgcn_raw_buffer_load_b64(xt, 8 * min(xb + k, g.w - 1), 0, 0));
#pragma unroll
    for (int k = 0; k < kResizeK; ++k)
        tyk[k] = __builtin_bit_cast(ResizeTap, __builtin_amdgcn_raw_buffer_load_b64(yt, 8 * min(yb + k, g.h - 1), 0, 0));
    // the source window: columns [c_lo, c_hi], rows [r_lo, r_hi] (as the tables)
    const int xl = min(x0 + 4 * twg, g.w) - 1, yl = min(y0 + TH, g.h) - 1;
    const int c_lo = min(max(resize_src_raw(x0, a.sx), 0), gs.w - 1);
    const int c_hi = min(max(resize_src_raw(xl, a.sx), 0) + 1, gs.w - 1);
    const int r_lo = min(max(resize_src_raw(y0, a.sy), 0), gs.h - 1);
    const int r_hi = min(max(resize_src_raw(yl, a.sy) + 1, 0), gs.h - 1);
    int spitch;
    const uint8_t *src = level_ptr(p, fb, l - 1, b, spitch);
    wave_stage_rows<NB, false>(win, a.win_stride, src, spitch, r_lo, c_lo, r_hi - r_lo + 1, c_hi - c_lo + 1, lane);
    // per-lane column constants: dword of the first source pixel, realignment,
    // and the v_perm selectors of the 4 pixel pairs (S[sx_k], S[sx_k + 1])
    const int rel0 = txk[0].src - (c_lo & ~3);
    const int q4 = (rel0 >> 2) * 4, o = rel0 & 3;
    uint32_t sel[4], coef[4];
    bool simd_all = true;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t r = (uint32_t)(txk[k].src - txk[0].src);
        sel[k] = r | 0x0C00u | ((r + 1) << 16) | 0x0C000000u;
        coef[k] = (uint32_t)(uint16_t)txk[k].a0 | ((uint32_t)(uint16_t)txk[k].a1 << 16);
        simd_all &= (txk[k].mode & 2) != 0;
    }
    wave_lds_fence();
    if (xb >= g.w) return;
    // (buffer stores: a 32-bit lane offset from the wave's level base, no
    // 64-bit address arithmetic per row)
    const __amdgpu_buffer_rsrc_t dst = wave_rsrc(fb.pyr + (int64_t)b * p.pyr_bytes + g.pyr_off);
    auto hrow = [&](int row, uint32_t h[4]) {
        const uint32_t *ap = reinterpret_cast<const uint32_t *>(win + mul24u(row - r_lo, a.win_stride) + q4);
        const uint32_t d0 = ap[0], d1 = ap[1], d2 = ap[2];
        const uint32_t w0 = __builtin_amdgcn_alignbyte(d1, d0, o), w1 = __builtin_amdgcn_alignbyte(d2, d1, o);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t pr = __builtin_amdgcn_perm(w1, w0, sel[k]);
            h[k] = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2_t, pr), __builtin_bit_cast(u16x2_t, coef[k]), 0u,
                                          false);
        }
    };
    // the horizontal pass of source row `prow` from the previous output row:
    // the next row's first source row is usually the previous one's second
#if ORBX_RS_REUSE
    uint32_t hp[4] = {0u, 0u, 0u, 0u};
    int prow = -1;
#endif
#pragma unroll
    for (int j = 0; j < kResizeK; ++j) {
        const int y = yb + j;
        if (y >= g.h) break;
        const int s0 = min(max((int)tyk[j].src, 0), gs.h - 1), s1 = min(max((int)tyk[j].src + 1, 0), gs.h - 1);
        const int b0 = tyk[j].a0, b1 = tyk[j].a1;
        uint32_t h0[4], h1[4];
#if ORBX_RS_REUSE
        if (s0 == prow) {
#pragma unroll
            for (int k = 0; k < 4; ++k) h0[k] = hp[k];
        } else {
            hrow(s0, h0);
        }
        hrow(s1, h1);
        prow = s1;
#pragma unroll
        for (int k = 0; k < 4; ++k) hp[k] = h1[k];
#else
        hrow(s0, h0);
        hrow(s1, h1);
#endif
        // SSE2 columns: _mm_packs_epi32(h>>4); _mm_mulhi_epi16; _mm_adds_epi16; +2; >>2
        // (h <= 255 * 2048: no saturation, result <= 255); the last < 16 columns
        // are the scalar tail FixedPtCast<int, uchar, 22>
        uint32_t packed = 0;
        if (simd_all) {
#if ORBX_RS_MULHI
            // ((h >> 4) * b) >> 16 as the high half of a 24 x 24-bit product:
            // (h & ~15) * (b << 12) = ((h >> 4) * b) << 16, both operands < 2^24
            const uint32_t bb0 = ((uint32_t)b0 & 0xFFFu) << 12, bb1 = ((uint32_t)b1 & 0xFFFu) << 12;   // (b <= 2048)
            packed = resize_vpass_simd(h0, h1, bb0, bb1);
#else
#pragma unroll
            for (int k = 0; k < 4; ++k)
                packed |= (((mul24u(h0[k] >> 4, b0) >> 16) + (mul24u(h1[k] >> 4, b1) >> 16) + 2) >> 2) << (8 * k);
#endif
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t v = (txk[k].mode & 2)
                                       ? ((mul24u(h0[k] >> 4, b0) >> 16) + (mul24u(h1[k] >> 4, b1) >> 16) + 2) >> 2
                                       : (mul24u(h0[k], b0) + mul24u(h1[k], b1) + (1 << 21)) >> 22;
                packed |= v << (8 * k);
            }
        }
        __builtin_amdgcn_raw_buffer_store_b32(packed, dst, mul24u(y, g.pitch) + xb, 0, 0);
    }
}

template <int NB>
__global__ __launch_bounds__(kThreads) void k_resize_w(DevPlan p, FrameBufs fb, int l, ResizeWave a, int B) {
    extern __shared__ __align__(16) uint8_t lds[];
    const int wave = wave_id(), lane = threadIdx.x & 63;
    const int L = xcd_logical_block(blockIdx.x, gridDim.x);
    const int t = L * 4 + wave;
    if (t >= a.ntiles * B) return;
    const int b = t / a.ntiles;
    resize_tile<NB>(p, fb, l, a, b, t - b * a.ntiles, lane, lds + wave * a.win_bytes);
}

// ===========================================================================
// K1 (direct wave tiles): the same tiles and arithmetic without the LDS
// window.  A lane's 4 columns read source bytes sx_0 .. sx_3 + 1, at most 7
// apart (plan_resize_waves), so each source row is ONE dword-aligned 12-byte
// buffer load (8 bytes from cs = min(sx_0, w_src - 8) after v_alignbyte; a
// pair byte past them, only the last column's S[sx + 1] whose coefficient is
// 0 there, is selected as zero).  The lane's column constants (load column,
// realignment, v_perm selectors, coefficients) and its rows' clamped source
// rows and vertical coefficients are host tables (ResizeCol, ResizeRow), so
// the kernel does no tap arithmetic.  The window staging (half of
// resize_tile's VALU: predicated loads and LDS stores a row) goes; L1/L2
// serve the rows the lanes share.  Unaligned 8-byte loads instead of the
// 12-byte aligned ones measured slower (resize 1.80 vs 1.52 ms a step,
// profiles/r05_ab_resize_direct.txt).
// ===========================================================================
#ifndef ORBX_RS_DIRECT
#define ORBX_RS_DIRECT 1
#endif

__device__ inline void resize_tile_direct(const DevPlan &p, const FrameBufs &fb, int l, const ResizeWave &a, int b,
                                          int tile, int lane) {
    const int ty = tile / a.ntx, tx = tile - ty * a.ntx;
    const LevelArgs g = p.la[l], gs = p.la[l - 1];
    const int twg = a.twg, lr = lane >> a.twg_shift, lg = lane & (twg - 1);
    const int TH = (64 >> a.twg_shift) * kResizeK;
    const int x0 = tx * 4 * twg, y0 = ty * TH;
    const int xb = x0 + 4 * lg, yb = y0 + lr * kResizeK;
    if (xb >= g.w) return;
    // this lane's column group and rows (host tables: no per-lane tap arithmetic)
    const __amdgpu_buffer_rsrc_t ct = wave_rsrc(p.rcols + a.col_off), rt = wave_rsrc(p.rrows + a.ytab_off);
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
    const u32x3 cg0 = __builtin_amdgcn_raw_buffer_load_b96(ct, 12 * xb, 0, 0);     // c, o, smask
    const u32x4 cg1 = __builtin_amdgcn_raw_buffer_load_b128(ct, 12 * xb + 16, 0, 0);   // sel
    const u32x4 cg2 = __builtin_amdgcn_raw_buffer_load_b128(ct, 12 * xb + 32, 0, 0);   // coef
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    u32x2 rw[kResizeK];
#pragma unroll
    for (int j = 0; j < kResizeK; ++j) rw[j] = __builtin_amdgcn_raw_buffer_load_b64(rt, 8 * min(yb + j, g.h - 1), 0, 0);
    int spitch;
    __amdgpu_buffer_rsrc_t src = wave_rsrc(level_ptr(p, fb, l - 1, b, spitch));
    spitch = __builtin_amdgcn_readfirstlane(spitch);
    if (l == 1) {
        // level 0 is the caller's image: the buffer's range ends at its last
        // row's last dword (a dword never crosses a page), so the dword loads
        // of the last row's right end cannot fault
        const uint64_t a0 = reinterpret_cast<uint64_t>(level_ptr(p, fb, 0, b, spitch));
        const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a0), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a0 >> 32));
        src = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(((uint64_t)hi << 32) | lo), (short)0,
                                                ((gs.h - 1) * spitch + gs.w + 3) & ~3, 0x00020000);
    }
    const int c = (int)cg0.x, o = (int)cg0.y;
    const uint32_t smask = cg0.z;
    const uint32_t sel[4] = {cg1.x, cg1.y, cg1.z, cg1.w}, coef[4] = {cg2.x, cg2.y, cg2.z, cg2.w};
    // every source row the lane needs, loaded before any is used; a row shared
    // with the previous output row is not loaded again (at the 1.2 factor 2 of
    // 3 output rows reuse one)
    u32x3 d0[kResizeK], d1[kResizeK];
    int s1p = -1;
#pragma unroll
    for (int j = 0; j < kResizeK; ++j) {
        const int s0 = (int)(rw[j].x & 0xFFFFu), s1 = (int)(rw[j].x >> 16);
        if (s0 != s1p) d0[j] = __builtin_amdgcn_raw_buffer_load_b96(src, mul24u(s0, spitch) + c, 0, 0);
        d1[j] = __builtin_amdgcn_raw_buffer_load_b96(src, mul24u(s1, spitch) + c, 0, 0);
        s1p = s1;
    }
    const __amdgpu_buffer_rsrc_t dst = wave_rsrc(fb.pyr + (int64_t)b * p.pyr_bytes + g.pyr_off);
    auto hrow = [&](u32x3 d, uint32_t h[4]) {
        const uint32_t w0 = __builtin_amdgcn_alignbyte(d.y, d.x, o), w1 = __builtin_amdgcn_alignbyte(d.z, d.y, o);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t pr = __builtin_amdgcn_perm(w1, w0, sel[k]);
            h[k] = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2_t, pr), __builtin_bit_cast(u16x2_t, coef[k]), 0u,
                                          false);
        }
    };
    uint32_t hp[4] = {0u, 0u, 0u, 0u};
    int prow = -1;
#pragma unroll
    for (int j = 0; j < kResizeK; ++j) {
        const int y = yb + j;
        if (y >= g.h) break;
        const int s0 = (int)(rw[j].x & 0xFFFFu), s1 = (int)(rw[j].x >> 16);
        const uint32_t bb0 = (rw[j].y & 0xFFFFu) << 12, bb1 = (rw[j].y >> 16) << 12;
        uint32_t h0[4], h1[4];
        if (s0 == prow) {
#pragma unroll
            for (int k = 0; k < 4; ++k) h0[k] = hp[k];
        } else {
            hrow(d0[j], h0);
        }
        hrow(d1[j], h1);
        prow = s1;
#pragma unroll
        for (int k = 0; k < 4; ++k) hp[k] = h1[k];
        uint32_t packed = 0;
        if (smask == 0xFu) {
            packed = resize_vpass_simd(h0, h1, bb0, bb1);
        } else {
            const uint32_t b0 = bb0 >> 12, b1 = bb1 >> 12;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t v = (smask >> k & 1u)
                                       ? ((mul24u(h0[k] >> 4, b0) >> 16) + (mul24u(h1[k] >> 4, b1) >> 16) + 2) >> 2
                                       : (mul24u(h0[k], b0) + mul24u(h1[k], b1) + (1 << 21)) >> 22;
                packed |= v << (8 * k);
            }
        }
        __builtin_amdgcn_raw_buffer_store_b32(packed, dst, mul24u(y, g.pitch) + xb, 0, 0);
    }
}

#ifndef ORBX_RSD_WPE
#define ORBX_RSD_WPE 0
#endif
__global__ __launch_bounds__(kThreads)
#if ORBX_RSD_WPE
__attribute__((amdgpu_waves_per_eu(ORBX_RSD_WPE)))
#endif
void k_resize_d(DevPlan p, FrameBufs fb, int l, ResizeWave a, int B) {
    const int wave = wave_id(), lane = threadIdx.x & 63;
    const int L = xcd_logical_block(blockIdx.x, gridDim.x);
    const int t = L * 4 + wave;
    if (t >= a.ntiles * B) return;
    const int b = t / a.ntiles;
    resize_tile_direct(p, fb, l, a, b, t - b * a.ntiles, lane);
}

// ===========================================================================
// K1 (regions): the whole pyramid of a frame in one launch for small batches.
// Block (region r, frame b) computes levels 1.. of its region with the level
// before each held in LDS: the level-l rectangle R_l it computes is its owned
// rectangle O_l plus what R_{l+1} reads (host plan, plan_pyr_regions), so the
// regions recompute their halos instead of waiting for each other, and only
// O_l is written to the pyramid.  Every pixel is the same fixed-point
// function of the same source pixels as in k_resize (identical output); the
// chain of 7 dependent launches becomes one.
// ===========================================================================
constexpr int kRgnThreads = 1024;
constexpr int kRgnCols = 4;   // computed rectangles are at most 64 * kRgnCols wide (plan_pyr_regions)
constexpr int kRgnTapRows = 64 * kRgnCols;   // and at most this tall
// LDS of the taps of levels 1.. (columns then rows of each)
constexpr int rgn_tap_bytes(int nlevels) { return (int)sizeof(ResizeTap) * 2 * kRgnTapRows * (nlevels - 1); }

// A workgroup barrier that orders LDS only: the kernel's global stores are
// read by later launches, so waiting for them at every level (as
// __syncthreads' release does) would only add their write latency.
__device__ inline void lds_barrier() { __asm__ volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__global__ __launch_bounds__(kRgnThreads) void k_pyramid_rgn(DevPlan p, FrameBufs fb) {
    extern __shared__ __align__(16) uint8_t lds[];
    const int r = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63;
    constexpr int kWaves = kRgnThreads / 64;
    const int4 *T = p.pyr_rgn + (int64_t)r * 2 * kMaxLevels;   // [l] = R_l, [kMaxLevels + l] = O_l
    uint8_t *cur = lds, *nxt = lds + p.pyr_rgn_half;
    // every level's taps for this region's columns and rows, staged with R_0 so
    // the level loop issues no global loads (on gfx9 a wait for a load also
    // waits for the level's earlier global stores)
    ResizeTap *sxt = reinterpret_cast<ResizeTap *>(lds + 2 * p.pyr_rgn_half);
    ResizeTap *syt = sxt + kRgnTapRows * (p.nlevels - 1);
    for (int i = tid; i < 2 * kRgnTapRows * (p.nlevels - 1); i += kRgnThreads) {
        const int ly = i >= kRgnTapRows * (p.nlevels - 1);
        const int j = i - ly * kRgnTapRows * (p.nlevels - 1);
        const int l = 1 + j / kRgnTapRows, k = j - (l - 1) * kRgnTapRows;
        const int4 Rl = T[l];
        const LevelGeom &g = p.lv[l];
        if (!ly && k <= Rl.z - Rl.x) sxt[j] = p.xtaps[g.xtab_off + Rl.x + k];
        if (ly && k <= Rl.w - Rl.y) syt[j] = p.ytaps[g.ytab_off + Rl.y + k];
    }
    // R_0 from level 0, dword-aligned rows (level 0's base and pitch are dword multiples)
    int4 R = T[0];
    int ox = R.x & ~3, oy = R.y;
    int stride;
    {
        int sp;
        const uint8_t *src = level_ptr(p, fb, 0, b, sp);
        const int ndw = ((R.z - ox) >> 2) + 1, nrows = R.w - R.y + 1;
        stride = 4 * ndw + 4;
        for (int row = wave; row < nrows; row += kWaves) {
            const uint32_t *s32 = reinterpret_cast<const uint32_t *>(src + (int64_t)(oy + row) * sp + ox);
            uint32_t *d32 = reinterpret_cast<uint32_t *>(cur + row * stride);
            for (int d = lane; d < ndw; d += 64) d32[d] = s32[d];
        }
    }
    lds_barrier();
    for (int l = 1; l < p.nlevels; ++l) {
        const int4 Rl = T[l], Ol = T[kMaxLevels + l];
        const LevelArgs g = p.la[l];
        const int gsh = p.la[l - 1].h;
        const ResizeTap *xt = sxt + kRgnTapRows * (l - 1);
        const ResizeTap *yt = syt + kRgnTapRows * (l - 1);
        const int w = Rl.z - Rl.x + 1, h = Rl.w - Rl.y + 1;
        const int dstride = (w + 4 + 3) & ~3;
        uint8_t *dst = fb.pyr + (int64_t)b * p.pyr_bytes + g.pyr_off;
        // this lane's columns lane + 64 k (k < kRgnCols: the plan bounds the
        // widths) and their taps, read once for all rows
        ResizeTap tx[kRgnCols];
#pragma unroll
        for (int k = 0; k < kRgnCols; ++k) tx[k] = xt[min(lane + 64 * k, w - 1)];
        for (int row = wave; row < h; row += kWaves) {
            const int y = Rl.y + row;
            const ResizeTap ty = yt[row];
            const int s0 = min(max((int)ty.src, 0), gsh - 1) - oy, s1 = min(max((int)ty.src + 1, 0), gsh - 1) - oy;
            const uint8_t *S0 = cur + s0 * stride - ox, *S1 = cur + s1 * stride - ox;
            const int b0 = ty.a0, b1 = ty.a1;
            const bool own_row = y >= Ol.y && y <= Ol.w;
#pragma unroll
            for (int k = 0; k < kRgnCols; ++k) {
                const int col = lane + 64 * k;
                if (col >= w) break;
                const int x = Rl.x + col;
                const int sx = tx[k].src;
                const int h0 = mul24u(S0[sx], tx[k].a0) + mul24u(S0[sx + 1], tx[k].a1);
                const int h1 = mul24u(S1[sx], tx[k].a0) + mul24u(S1[sx + 1], tx[k].a1);
                const int v_simd = ((mul24u(h0 >> 4, b0) >> 16) + (mul24u(h1 >> 4, b1) >> 16) + 2) >> 2;
                const int v_tail = (mul24u(h0, b0) + mul24u(h1, b1) + (1 << 21)) >> 22;
                const uint8_t v = (uint8_t)min(max((tx[k].mode & 2) ? v_simd : v_tail, 0), 255);
                nxt[row * dstride + col] = v;
                if (own_row && x >= Ol.x && x <= Ol.z) dst[(int64_t)y * g.pitch + x] = v;
            }
        }
        lds_barrier();
        uint8_t *t = cur; cur = nxt; nxt = t;
        stride = dstride; ox = Rl.x; oy = Rl.y;
    }
}

// ===========================================================================
// K2: Gaussian 7x7, sigma 2, BORDER_REFLECT_101 on each level (OpenCV 3.2
// fixed-point separable filter).  The SSE2 column pass accumulates exactly in
// float and rounds half-to-even; the scalar tail adds 2^15 and shifts: both are
// reproduced here in integers (exact: the float sums are < 2^24 whenever the
// result is < 256).  Tile = 64 x 16 outputs, 70 x 22 inputs in LDS.
// ===========================================================================
constexpr int kBlurTW = 64, kBlurTH = 16;

__global__ __launch_bounds__(kThreads) void k_blur(DevPlan p, FrameBufs fb) {
    const int4 t = p.blur_tiles[blockIdx.x];
    const int l = t.x, x0 = t.y, y0 = t.z, b = blockIdx.y;
    const LevelGeom g = p.lv[l];
    int spitch;
    const uint8_t *src = level_ptr(p, fb, g, l, b, spitch);
    uint8_t *dst = fb.blur + (int64_t)b * p.blur_bytes + g.blur_off;
    __shared__ uint8_t tin[kBlurTH + 6][kBlurTW + 8];
    __shared__ int rowp[kBlurTH + 6][kBlurTW];
    const int tid = threadIdx.x;
    for (int i = tid; i < (kBlurTH + 6) * (kBlurTW + 6); i += kThreads) {
        const int r = i / (kBlurTW + 6), c = i - r * (kBlurTW + 6);
        const int yy = reflect101(min(y0 + r - 3, g.h + 2), g.h);
        const int xx = reflect101(min(x0 + c - 3, g.w + 2), g.w);
        tin[r][c] = src[(int64_t)yy * spitch + xx];
    }
    __syncthreads();
    const int k0 = p.gauss[0], k1 = p.gauss[1], k2 = p.gauss[2], k3 = p.gauss[3];
    for (int i = tid; i < (kBlurTH + 6) * kBlurTW; i += kThreads) {
        const int r = i / kBlurTW, c = i - r * kBlurTW;
        const uint8_t *q = &tin[r][c];
        rowp[r][c] = k0 * (q[0] + q[6]) + k1 * (q[1] + q[5]) + k2 * (q[2] + q[4]) + k3 * q[3];
    }
    __syncthreads();
    const int xs = g.w & ~3;
    for (int i = tid; i < kBlurTH * kBlurTW; i += kThreads) {
        const int r = i / kBlurTW, c = i - r * kBlurTW;
        const int x = x0 + c, y = y0 + r;
        if (x >= g.w || y >= g.h) continue;
        const int s = k3 * rowp[r + 3][c] + k2 * (rowp[r + 2][c] + rowp[r + 4][c]) +
                      k1 * (rowp[r + 1][c] + rowp[r + 5][c]) + k0 * (rowp[r][c] + rowp[r + 6][c]);
        int q = s >> 16;
        if (x < xs) {
            const int rem = s & 0xFFFF;
            q += (rem > 0x8000) | ((rem == 0x8000) & (q & 1));
        } else {
            q = (s + (1 << 15)) >> 16;
        }
        dst[(int64_t)y * g.pitch + x] = (uint8_t)min(q, 255);
    }
}

// ===========================================================================
// K3: per-cell FAST-9 with the reference's cell semantics, one wave per cell
// (no workgroup barriers: each wave owns its cell's LDS slice).
// For each interior pixel the arc score S = max over the 16 nine-pixel arcs of
// max(min(v - p), min(p - v)); the pixel is a corner at threshold t iff S > t
// and cv::FAST's cornerScore is S - 1.  S is evaluated only
// for pixels that pass a compass pre-test at the pass's threshold.  NMS is the
// strict 3x3 test inside the cell (outside neighbours count 0, as FAST on the
// cell sub-image sees them).  As the reference, a pass at iniThFAST comes
// first and a pass at minThFAST only for a cell it left empty (27 % of the
// level-0 cells of the bench frames); the count word says which list the cell uses (bit 31 =
// minThFAST, ORBextractor.cc:846-850).
// Output: keypoints in row-major order, packed (x | y<<12 | s<<24).
// ===========================================================================
// max over the 16 arcs of 9 of max(min(p) - v, v - max(p)) for circle bytes p.
// Lane pair (p, 255 - p): the minimum of the second half is 255 - max(p).
// Equal to OpenCV's cornerScore<16> arc order (its even-anchored pairs of
// arcs cover all 16 starts); min / max are exact, so any order agrees.
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

__device__ inline u16x2 as_u16x2(uint32_t v) { return __builtin_bit_cast(u16x2, v); }

// The 16 arcs in pairs sharing 8 points (as OpenCV's cornerScore<16> walks
// them): for even k, arcs k..k+8 and k+1..k+9 are the block B = k+1..k+8 plus
// point k or point k+9.  The eight blocks (odd starts j) come from minima of
// pairs and quads at odd starts only: 24 + 24 packed ops (the 16 arcs' minima
// folded per block) instead of the 48 + 16 + 15 of all sixteen sliding windows.
#ifndef ORBX_ARC_DIST
#define ORBX_ARC_DIST 1
#endif
// ORBX_ARC_F16=1: the pairs offset by K = 0x3C00 (both halves normal positive
// f16 numbers, 1.0 .. 1.25, ordered as their bit patterns), so gfx950's packed
// three-input v_pk_minimum3_f16 / v_pk_maximum3_f16 apply: block i's value is
// min3(m4[i], m4[i+2], max(e[2i], e[2i+9])) (no m8 stage) and the eight block
// values fold by max3 -- 8 + 8 + 16 + 4 packed ops against 8 + 8 + 8 + 24.
#ifndef ORBX_ARC_F16
#define ORBX_ARC_F16 1
#endif
#if ORBX_ARC_F16
__device__ inline u16x2 pk_min3_h(u16x2 a, u16x2 b, u16x2 c) {
    uint32_t r;
    asm("v_pk_minimum3_f16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return as_u16x2(r);
}
__device__ inline u16x2 pk_max3_h(u16x2 a, u16x2 b, u16x2 c) {
    uint32_t r;
    asm("v_pk_maximum3_f16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return as_u16x2(r);
}
__device__ inline int arc_score_bytes(const int p[16], int v) {
    constexpr uint32_t K = 0x3C00u, C = ((255u + K) << 16) + K;   // (p, 255 - p) + (K, K)
    u16x2 e[16], m2[8], m4[8], x[8];
#pragma unroll
    for (int k = 0; k < 16; ++k) e[k] = as_u16x2(C - (uint32_t)p[k] * 65535u);
#pragma unroll
    for (int i = 0; i < 8; ++i) m2[i] = __builtin_elementwise_min(e[2 * i + 1], e[(2 * i + 2) & 15]);   // j, j+1
#pragma unroll
    for (int i = 0; i < 8; ++i) m4[i] = __builtin_elementwise_min(m2[i], m2[(i + 1) & 7]);              // j..j+3
#pragma unroll
    for (int i = 0; i < 8; ++i)
        x[i] = pk_min3_h(m4[i], m4[(i + 2) & 7], __builtin_elementwise_max(e[2 * i], e[(2 * i + 9) & 15]));
    const u16x2 best = __builtin_elementwise_max(pk_max3_h(pk_max3_h(pk_max3_h(x[0], x[1], x[2]), x[3], x[4]), x[5], x[6]), x[7]);
    return max((int)best.x - (int)K - v, v - (255 + (int)K - (int)best.y));
}
#else
__device__ inline int arc_score_bytes(const int p[16], int v) {
    u16x2 e[16], m2[8], m4[8], m8[8];
#pragma unroll
    for (int k = 0; k < 16; ++k) e[k] = as_u16x2((uint32_t)p[k] + ((uint32_t)(255 - p[k]) << 16));
#pragma unroll
    for (int i = 0; i < 8; ++i) m2[i] = __builtin_elementwise_min(e[2 * i + 1], e[(2 * i + 2) & 15]);   // j, j+1
#pragma unroll
    for (int i = 0; i < 8; ++i) m4[i] = __builtin_elementwise_min(m2[i], m2[(i + 1) & 7]);              // j..j+3
#pragma unroll
    for (int i = 0; i < 8; ++i) m8[i] = __builtin_elementwise_min(m4[i], m4[(i + 2) & 7]);              // j..j+7
    // block i = points 2i+1 .. 2i+8: arcs starting at 2i and 2i+1, whose
    // minima max together as min(m8, e[2i]) v min(m8, e[2i+9]) =
    // min(m8, max(e[2i], e[2i+9])) (min distributes over max): three packed
    // ops a block instead of four (ORBX_ARC_DIST=0: the four)
    u16x2 best;
#if ORBX_ARC_DIST
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const u16x2 x = __builtin_elementwise_min(m8[i], __builtin_elementwise_max(e[2 * i], e[(2 * i + 9) & 15]));
        best = i ? __builtin_elementwise_max(best, x) : x;
    }
#else
    best = __builtin_elementwise_min(m8[0], e[0]);
    best = __builtin_elementwise_max(best, __builtin_elementwise_min(m8[0], e[9]));
#pragma unroll
    for (int i = 1; i < 8; ++i) {
        best = __builtin_elementwise_max(best, __builtin_elementwise_min(m8[i], e[2 * i]));
        best = __builtin_elementwise_max(best, __builtin_elementwise_min(m8[i], e[(2 * i + 9) & 15]));
    }
#endif
    return max((int)best.x - v, v - (255 - (int)best.y));
}
#endif

// k_fast's cell + ring (ORBX_FAST_STAGE): nr rows of nd dwords from column
// x0 - 1, so that column x0 lands at patch column 1 (interior column 0 at
// column 4).  R rows a pass (lanes rl < R, R = 64 / nd from a table: no
// division), 8 passes: every load is issued (the buffer's range ends at the
// rectangle, so rows past nr read zeros -- raw buffers check the lane offset,
// which holds the whole row offset here) and the stores of passes starting at
// or past nr are skipped by uniform branches.  The generic loop's per-load
// and per-store exec masks (~3 scalar instructions and a compare each) go.
// Rows in [nr, nr + R) of the last pass land below the patch, in its spare
// rows or the score map, which each FAST pass zeroes before use; the caller
// checks that 8 R >= nr and that nr + R - 1 rows fit the patch + score map.
__device__ inline int fast_stage_rows(int nd) {   // 64 / nd for nd in [1, 12], 0 past (selects, no division)
    return nd <= 1 ? 64 : nd == 2 ? 32 : nd == 3 ? 21 : nd == 4 ? 16 : nd == 5 ? 12 : nd == 6 ? 10 : nd == 7 ? 9
         : nd == 8 ? 8 : nd == 9 ? 7 : nd == 10 ? 6 : nd <= 12 ? 5 : 0;
}
__device__ inline void stage_fast_patch(uint8_t *dst, int ps, const uint8_t *img, int pitch, int y0, int x0, int nr,
                                        int nd, int R, int lane) {
    const int xs = x0 - 1, xa = xs & ~3, sh = xs - xa;
    const uint64_t a = reinterpret_cast<uint64_t>(img + (int64_t)y0 * pitch + xa);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    const __amdgpu_buffer_rsrc_t src = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void *>(((uint64_t)hi << 32) | lo), (short)0, nr * pitch, 0x00020000);
    const int rl = div_small(lane, nd), k = lane - mul24u(rl, nd);
    const int voff = mul24u(rl, pitch) + 4 * k + sh, loff = mul24u(rl, ps) + 4 * k;
    const int Rp = R * pitch, Rs = R * ps;   // (scalar)
    typedef __attribute__((address_space(3))) uint32_t lds_u32;
    if (rl < R) {
        uint32_t v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = __builtin_amdgcn_raw_buffer_load_b32(src, voff + j * Rp, 0, 0);
#pragma unroll
        for (int j = 0; j < 8; ++j) asm volatile("" : "+v"(v[j]));   // (all eight issued before any store)
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (j * R < nr) *(lds_u32 *)(dst + loff + j * Rs) = v[j];
    }
}

#ifndef ORBX_FAST_STAGE
#define ORBX_FAST_STAGE 1   // 0: the generic wave_stage_rows
#endif
#ifndef ORBX_FAST_EVEN8
#define ORBX_FAST_EVEN8 0   // 1: the 8-even-point pre-test before the arc score (A/B, slower)
#endif

// PIPE: a level's cells in a level-pipelined step (a distinct instantiation so
// profiles tell per-level launches from whole-batch ones).
// PSC: the patch / score-map row stride as a compile-time constant (48 or 64:
// every circle, ring and NMS neighbour offset becomes an LDS immediate), or 0
// for the launch's runtime stride.
#ifndef ORBX_FAST_ALIGN
#define ORBX_FAST_ALIGN 1
#endif
constexpr bool kFastAlign = ORBX_FAST_ALIGN != 0;

template <bool PIPE, int PSC>
__global__ __launch_bounds__(kThreads) void k_fast(DevPlan p, FrameBufs fb, int c0, int nc, FastLds fl,
                                                   uint32_t gmagic) {
    extern __shared__ __align__(16) uint8_t lds[];
    PHASE_START();
    const int wave = wave_id(), lane = threadIdx.x & 63;
    int bx, b;
    xcd_block_2d(bx, b, gmagic);
    if (bx * 4 + wave >= nc) return;
    const int ci = c0 + bx * 4 + wave;
    // the cell as five dwords: scalar loads (a 16-bit field would take a
    // vector load, and a vector round trip, ahead of the staging)
    static_assert(sizeof(Cell) == 20, "five dwords");
    Cell c;
    {
        const uint32_t *cp = reinterpret_cast<const uint32_t *>(p.cells) + 5 * ci;
        const uint32_t w0 = cp[0], w1 = cp[1], w2 = cp[2];
        c.level = (int16_t)(w0 & 0xFFFFu);
        c.pad = 0;
        c.x0 = (int16_t)(w1 & 0xFFFFu);
        c.y0 = (int16_t)(w1 >> 16);
        c.x1 = (int16_t)(w2 & 0xFFFFu);
        c.y1 = (int16_t)(w2 >> 16);
        c.slot = (int32_t)cp[3];
        c.cap = (int32_t)cp[4];
    }
    int32_t *count_out = fb.cell_count + (int64_t)b * p.ncells + ci;
    const int cw = c.x1 - c.x0, ch = c.y1 - c.y0;
    if (cw <= 0 || ch <= 0) {
        if (lane == 0) *count_out = 0;
        return;
    }
    // the patch and the score map share the row stride (fast_lds)
    const int PS = PSC ? PSC : fl.ps;
    const int pmag = PSC ? (int)(((1u << 24) + PSC - 1) / (PSC ? PSC : 1)) : fl.pmag;
    const int kxy0 = c.x0 + (c.y0 << 12);   // pack_key of interior pixel (0, 0), score 0
    uint8_t *patch = lds + (size_t)wave * fl.per_wave;
    uint8_t *scm = patch + fl.patch_bytes;   // S-1 of the pass's corners, 0 elsewhere
    // survivors and corners as patch offsets yy * PS + xx from interior pixel
    // (0, 0) (the score map's index of the pixel is the same + PS + 1), row-major
    uint16_t *list = reinterpret_cast<uint16_t *>(scm + fl.score_bytes);
    int spitch;
    const uint8_t *img = level_ptr(p, fb, c.level, b, spitch);
    // (ORBX_FAST_ALIGN: the cell is staged so that interior column 0 lands on
    // a dword boundary (patch column 4, loads unaligned): a 31-pixel cell row
    // is then 8 quads, 4 lane groups, 16 rows per compass step, where a
    // misaligned one took 9 quads, 5 groups, 12 rows: 2.66 -> 2.06 compass
    // steps per VGA cell)
    int o;
    {
        const int sp = __builtin_amdgcn_readfirstlane(spitch), nr = ch + 6;
        const int nd = (1 + cw + 6 + 3) >> 2;
        const int R = fast_stage_rows(nd);
        if (ORBX_FAST_STAGE && kFastAlign && R && 8 * R >= nr &&
            (nr + R - 1) * PS <= fl.patch_bytes + fl.score_bytes) {
            stage_fast_patch(patch, PS, img, sp, c.y0 - 3, c.x0 - 3, nr, nd, R, lane);
            o = 1;
        } else {
            o = wave_stage_rows<8, true, false, kFastAlign ? 1 : -1>(patch, PS, img, spitch, c.y0 - 3, c.x0 - 3,
                                                                    nr, cw + 6, lane);
        }
    }
    const uint8_t *pc = patch + 3 * PS + o + 3;         // interior pixel (0, 0)
    PHASE_MARK(0, 0);   // prologue + staging
    if constexpr (kStopFast == 1) {
        if (lane == 0) *count_out = 0;
        return;
    }
    uint32_t *out_i = fb.cand + (int64_t)b * p.cand_cap + c.slot;
    uint32_t *out_m = fb.cand2 + (int64_t)b * p.cand_cap + c.slot;
    // The compass pass's lane geometry (both passes): lane = (row in pass,
    // quad of the row), 64 / nq rows per pass; a lane keeps its quad column,
    // so its interior mask is fixed.
    const int qc0 = (o + 3) & ~3;                           // patch column of the first quad
    const int nq = ((o + 2 + cw) >> 2) - (qc0 >> 2) + 1;   // quads per row
    // a lane takes kFQ adjacent quads (4 kFQ pixels) of one row: the loads,
    // the loop and the compaction scan are shared by that many pixels
    constexpr int kFQ = 2, kFP = 4 * kFQ;   // (3: 706 VALU per wave against 698, same time)
    const int np = kFQ == 2 ? (nq + 1) >> 1 : div_small(nq + kFQ - 1, kFQ);   // quad groups per row
    const int R = __builtin_amdgcn_readfirstlane(div_small(64, np));
    const int rl = div_small(lane, np), pi = lane - mul24u(rl, np);
    const int xx0 = qc0 - o - 3 + kFP * pi;   // interior x of the group's byte 0
    // candidate bits: bit j = pixel j of the group; the interior pixels
    // [lo, hi) of the group as one bit field
    const int vlo = min(max(-xx0, 0), kFP), vhi = min(max(cw - xx0, 0), kFP);
    uint32_t vmask = __builtin_amdgcn_ubfe(((1u << kFP) - 1u) << vlo, 0, (uint32_t)vhi);   // bits [lo, hi)
    if (rl >= R) vmask = 0;   // (tail lanes: rows of the next pass)
    // the lane's group in LDS, 3 rows up (every load a non-negative offset
    // from it; 32-bit address arithmetic), and its row limit
    const lds_u8 *qb0 = (const lds_u8 *)(patch + mul24u(rl, PS) + qc0 + kFP * pi);
    const int rlim = mul24u(max(ch - rl, 0), PS);   // (row offsets in bytes: the loop runs on scalars)

    // One FAST pass at threshold th: returns the keypoints kept after NMS,
    // written to out.  The reference runs iniThFAST first and minThFAST only
    // for a cell where that found nothing (ORBextractor.cc:842-850).
    auto pass = [&](int th, uint32_t *out, int ph) -> int {
        {
            uint4 *z0 = reinterpret_cast<uint4 *>(scm);   // (16-B aligned; score_bytes a multiple of 16)
            const int nz = fl.score_bytes >> 4;
            for (int i = lane; i < nz; i += 64) z0[i] = make_uint4(0u, 0u, 0u, 0u);
        }
        wave_lds_fence();
        // The list holds, in row-major order, the corners still waiting for
        // their NMS (list[0, npend): the last scored row's) and then the
        // compass survivors of the rows since (list[npend, npend + nsurv)).
        // It has room for fl.list_cap entries (8 workgroups per CU at VGA,
        // 6 with a list for every pixel of the cell); before a compass step
        // could overflow it, the survivors so far are scored and the corners
        // of every finished row are suppressed and written (flush).
        int npend = 0, nsurv = 0, base = 0;
        // B + C for the survivors in list[npend, npend + nsurv), rows [0, ydone)
        // compass-tested; final: every remaining corner is decided.
        auto flush = [&](int ydone, bool final) {
            // B. arc score of every survivor: S = max(M1 - v, v - M2), M1 = max over
            //    the 16 nine-pixel arcs of the arc's minimum, M2 = min over arcs of the
            //    arc's maximum, side by side as packed u16 lanes (p, 255 - p) through
            //    sliding-window minima (2, 4, 8, 9).  A corner at th iff S > th; its
            //    FAST score S - 1 goes to the map, corners compacted in place.
            // (wave-uniform counts, kept in scalars: loops on scalar compares)
            npend = __builtin_amdgcn_readfirstlane(npend);
            nsurv = __builtin_amdgcn_readfirstlane(nsurv);
            int ncorner = npend;
#if ORBX_FAST_EVEN8
            // (A/B candidate, off) a second pre-test on the 8 even circle points:
            // any 9-arc holds >= 4 cyclically consecutive even points, all
            // brighter or all darker; survivors that fail it are dropped before
            // the 16-point score (compacted in place, as the corners below)
            {
                int npass = npend;
                for (int i0 = 0; i0 < nsurv; i0 += 64) {
                    const bool live = i0 + lane < nsurv;
                    const int e = live ? (int)list[npend + i0 + lane] : 0;
                    const uint8_t *q = pc + e;
                    const int v = q[0];
                    const uint32_t pe[8] = {q[3 * PS], q[2 * PS + 2], q[3], q[-2 * PS + 2],
                                            q[-3 * PS], q[-2 * PS - 2], q[-3], q[2 * PS - 2]};
                    u16x2 ev[8], m2[8];
#pragma unroll
                    for (int k = 0; k < 8; ++k) ev[k] = as_u16x2(pe[k] + ((255u - pe[k]) << 16));
#pragma unroll
                    for (int k = 0; k < 8; ++k) m2[k] = __builtin_elementwise_min(ev[k], ev[(k + 1) & 7]);
                    u16x2 best = __builtin_elementwise_min(m2[0], m2[2]);
#pragma unroll
                    for (int k = 1; k < 8; ++k) best = __builtin_elementwise_max(best, __builtin_elementwise_min(m2[k], m2[(k + 2) & 7]));
                    const bool pass = live & (max((int)best.x - v, v - (255 - (int)best.y)) > th);
                    const uint64_t m = __ballot(pass);
                    wave_lds_fence();
                    if (pass) list[npass + mbcnt64(m)] = (uint16_t)e;
                    npass += __popcll(m);
                }
                nsurv = __builtin_amdgcn_readfirstlane(npass - npend);
                wave_lds_fence();
            }
#endif
            for (int i0 = 0; i0 < nsurv; i0 += 64) {
                // every lane scores (no exec region): a lane past the survivors
                // reads a stale entry, or LDS past the list, clamped to entry 0
                // (pixel (0, 0)) so that its circle reads stay inside the patch;
                // it is masked after
                const bool live = i0 + lane < nsurv;
                const int e = live ? (int)list[npend + i0 + lane] : 0;
                const uint8_t *q = pc + e;
                const int v = q[0];
                const uint32_t pr[16] = {q[3 * PS],  q[3 * PS + 1],  q[2 * PS + 2],  q[PS + 3],
                                         q[3],       q[-PS + 3],     q[-2 * PS + 2], q[-3 * PS + 1],
                                         q[-3 * PS], q[-3 * PS - 1], q[-2 * PS - 2], q[-PS - 3],
                                         q[-3],      q[PS - 3],      q[2 * PS - 2],  q[3 * PS - 1]};
                const int S = arc_score_bytes(reinterpret_cast<const int *>(pr), v);
                const bool corner = live & (S > th);
                const uint64_t m = lanes_lt(i0 + lane, nsurv) & lanes_gt(S, th);   // (the ballot of corner)
                if (corner) scm[e + PS + 1] = (uint8_t)(S - 1);
                wave_lds_fence();   // all survivor reads of this chunk precede the in-place writes
                if (corner) list[ncorner + mbcnt64(m)] = (uint16_t)e;
                ncorner += __popcll(m);
            }
            nsurv = 0;
            wave_lds_fence();
            PHASE_MARK(0, ph + 1);   // arc scores
            if constexpr (kStopFast == 3) { npend = 0; return; }
            // C. strict 3x3 NMS inside the cell (outside neighbours and non-corners
            //    score 0), compacted in row-major order; a corner of row ydone - 1
            //    waits for the next rows' scores unless final.
            // (entries are patch offsets ey * PS + ex: row ey is final below ylast * PS)
            const int ylast = final ? INT_MAX : (ydone - 1) * PS;
            int nfin = 0;
            for (int i0 = 0; i0 < ncorner; i0 += 64) {
                // every lane reads (as in B: a lane past the corners clamped to
                // entry 0, inside the score map), masked after
                const bool live = i0 + lane < ncorner;
                const int e = live ? (int)list[i0 + lane] : 0;
                const bool fin = live & (e < ylast);
                const int si = e + PS + 1;
                // the centre and its 8 neighbours read together, compared
                // with their maximum (no short-circuit chain of dependent reads)
                const int sv = scm[si];
                const int n0 = scm[si - 1], n1 = scm[si + 1], n2 = scm[si - PS - 1], n3 = scm[si - PS],
                          n4 = scm[si - PS + 1], n5 = scm[si + PS - 1], n6 = scm[si + PS], n7 = scm[si + PS + 1];
                const int mx = max(max(max(n0, n1), max(n2, n3)), max(max(n4, n5), max(n6, n7)));
                const bool keep = fin & (sv > mx);
                const uint64_t mf = lanes_lt(i0 + lane, ncorner) & lanes_lt(e, ylast);   // (the ballots of fin, keep)
                const uint64_t mk = mf & lanes_gt(sv, mx);
                const int pk = base + mbcnt64(mk);
                // the key from the offset: ey by the 24-bit reciprocal, then
                // x | y << 12 = x0 + (y0 << 12) + e + ey (4096 - PS)
                const int ey = (int)(__umul24((uint32_t)e, (uint32_t)pmag) >> 24);
                if (keep && pk < c.cap) out[pk] = (uint32_t)(kxy0 + e + mul24u(ey, 4096 - PS)) | ((uint32_t)sv << 24);
                base += __popcll(mk);
                nfin += __popcll(mf);
            }
            // the waiting corners (one row: < 64) to the front
            npend = ncorner - nfin;
            if (npend) {
                const int e = lane < npend ? list[nfin + lane] : 0;
                wave_lds_fence();
                if (lane < npend) list[lane] = (uint16_t)e;
                wave_lds_fence();
            }
            PHASE_MARK(0, ph + 2);   // NMS + output
        };
        // A. compass pre-test: an arc of 9 covers two cyclically adjacent points
        //    of {0, 4, 8, 12}, so a pixel is a corner candidate only if some
        //    adjacent pair is all brighter (min of the pair > v + th) or all
        //    darker (max of the pair < v - th).  A lane tests a dword-aligned
        //    quad of 4 pixels from 5 aligned LDS dwords (the +-3 column
        //    neighbours by byte alignment), as two packed u16 pairs (even and
        //    odd pixels); survivors are compacted in row-major order.
        {
            const u16x2 thv = {(unsigned short)th, (unsigned short)th};
            const u16x2 thv8 = {(unsigned short)(th << 8), (unsigned short)(th << 8)};
            typedef __attribute__((address_space(3))) const uint32_t lds_u32c;
            const int e = mul24u(rl, PS) + xx0;   // the list entry of the group's byte 0 at yo = 0
            const int RPS = __builtin_amdgcn_readfirstlane(R * PS);
            const int chps = __builtin_amdgcn_readfirstlane(ch * PS);
            for (int yo = 0, ys = 0; yo < chps; yo += RPS, ys += R) {
                // survivors this step can add: its rows' pixels (wave-uniform)
                if (npend + nsurv + min(R, ch - ys) * cw > fl.list_cap) {
                    if constexpr (kStopFast == 2) nsurv = 0;
                    else flush(ys, false);
                }
                uint32_t cand = 0;
                if (yo < rlim) {
                    const lds_u8 *qb = qb0 + yo;
                    // the group's dwords c[0..kFQ), their row neighbours c[-1] and
                    // c[kFQ], and the rows 3 up / down
                    uint32_t c[kFQ + 2], up[kFQ], dn[kFQ];
#pragma unroll
                    for (int k = 0; k < kFQ + 2; ++k) c[k] = *reinterpret_cast<lds_u32c *>(qb + 3 * PS - 4 + 4 * k);
#pragma unroll
                    for (int k = 0; k < kFQ; ++k) {
                        up[k] = *reinterpret_cast<lds_u32c *>(qb + 4 * k);
                        dn[k] = *reinterpret_cast<lds_u32c *>(qb + 6 * PS + 4 * k);
                    }
                    // one quad: pixel pairs (0, 2) and (1, 3) as u16 halves, straight
                    // from the aligned dwords (v_perm picks the +-3 column bytes of
                    // (lo, hi) dword pairs); even pixels: bytes 0 / 2 as the low bytes
                    // of the halves (an AND for the aligned dwords); odd pixels: bytes
                    // 1 / 3 left in the high bytes, every value and the threshold
                    // scaled by 256 -- the same comparisons, without the shift
                    auto quad = [&](uint32_t c, uint32_t lft, uint32_t rgt, uint32_t up, uint32_t dn) -> uint32_t {
                        // ODD: the pixels sit in the high bytes of the halves and the low
                        // bytes are left as they come (another pixel).  Max / min then
                        // give the right high byte and some low byte h or l, and with the
                        // centre as V:FF against hi and V:00 against lo,
                        //   sat(H:h - V:FF) > th:00  <=>  H - V > th,  sat(V:00 - L:l) > th:00  <=>  V - L > th
                        // (the low-byte terms lie in [-255, 0]): one operand op fewer a half.
                        auto half = [&](auto odd, uint32_t sel4, uint32_t sel12, u16x2 thv) -> u16x2 {   // 1: candidate
                            constexpr bool kOdd = decltype(odd)::value;
                            const u16x2 vh = as_u16x2(kOdd ? (c | 0x00FF00FFu) : (c & 0x00FF00FFu));   // (v against hi)
                            const u16x2 vl = kOdd ? as_u16x2(c & 0xFF00FF00u) : vh;                  // (v against lo)
                            const u16x2 a0 = as_u16x2(kOdd ? dn : (dn & 0x00FF00FFu));
                            const u16x2 a4 = as_u16x2(__builtin_amdgcn_perm(rgt, c, sel4));    // x + 3
                            const u16x2 a8 = as_u16x2(kOdd ? up : (up & 0x00FF00FFu));
                            const u16x2 a12 = as_u16x2(__builtin_amdgcn_perm(c, lft, sel12));  // x - 3
                            // max over the cyclic pairs of the pair's min, and min of the max:
                            // max(min(a,b), min(b,c), min(c,d), min(d,a)) = min(max(a,c), max(b,d))
                            const u16x2 hi = __builtin_elementwise_min(__builtin_elementwise_max(a0, a8),
                                                                       __builtin_elementwise_max(a4, a12));
                            const u16x2 lo = __builtin_elementwise_max(__builtin_elementwise_min(a0, a8),
                                                                       __builtin_elementwise_min(a4, a12));
                            // hi > v + th  or  lo + th < v  <=>  max(hi - v, v - lo) > th (saturating)
                            const u16x2 d = __builtin_elementwise_sub_sat(
                                __builtin_elementwise_max(__builtin_elementwise_sub_sat(hi, vh),
                                                          __builtin_elementwise_sub_sat(vl, lo)),
                                thv);
                            u16x2 m;   // min(d, 1) per half, kept one packed op
                            asm("v_pk_min_u16 %0, %1, %2" : "=v"(m) : "v"(d), "s"(0x00010001u));
                            return m;
                        };
                        // pixels 0 / 2 at bits 0 / 16, 1 / 3 at bits 1 / 17
                        return __builtin_bit_cast(uint32_t, half(std::false_type{}, 0x0c050c03u, 0x0c030c01u, thv)) |
                               (__builtin_bit_cast(uint32_t, half(std::true_type{}, 0x060c040cu, 0x040c020cu, thv8)) << 1);
                    };
                    // quad k's pixels 0 / 2 at bits 4k / 4k + 16, 1 / 3 at 4k + 1 / 4k + 17,
                    // folded to bits 4k .. 4k + 3
                    uint32_t bits = 0;
#pragma unroll
                    for (int k = 0; k < kFQ; ++k) bits |= quad(c[k + 1], c[k], c[k + 2], up[k], dn[k]) << (4 * k);
                    cand = (bits | (bits >> 14)) & vmask;
                }
                // compaction in row-major order: an inclusive DPP scan of the
                // lanes' counts (0..4 kFQ) places each lane's run, then its bits
                const int cnt = __builtin_popcount(cand);
                const int incl = wave_incl_scan_i32_to(cnt);
                const int total = __builtin_amdgcn_readlane(incl, 63);
                if (total) {
                    typedef __attribute__((address_space(3))) uint16_t lds_u16;
                    lds_u16 *dst = (lds_u16 *)list + npend + nsurv + (incl - cnt);
                    const int ey = e + yo;
                    // the lane's k-th bit to dst[k] (LDS immediate offsets), while any lane has one
#pragma unroll
                    for (int k = 0; k < kFP; ++k) {
                        if (!__builtin_amdgcn_ballot_w64(cand != 0u)) break;
                        if (cand) {
                            dst[k] = (uint16_t)(ey + __builtin_ctz(cand));
                            cand &= cand - 1u;
                        }
                    }
                    nsurv += total;
                }
            }
        }
        wave_lds_fence();
        PHASE_MARK(0, ph);       // score-map zeroing + compass pre-test + compaction
        if constexpr (kStopFast == 2) return 0;
        flush(ch, true);
        return base;
    };
    const int n_ini = pass(p.ini_th, out_i, 1);
    int32_t cnt;
    if (n_ini > 0 || (kStopFast >= 2 && kStopFast <= 4)) {
        cnt = min(n_ini, c.cap);
    } else {
        wave_lds_fence();
        const int n_min = pass(p.min_th, out_m, 4);
        cnt = (int32_t)(0x80000000u | (uint32_t)min(n_min, c.cap));
    }
    if (lane == 0) *count_out = cnt;
}

// ===========================================================================
// K4: DistributeOctTree, one 256-thread workgroup per (level, frame).
// The reference's std::list is replaced by node arrays rebuilt each round in
// the exact order push_front/erase would leave them:
//   full round:  new list = reverse(children in parent order, n1..n4)
//                           ++ unsplit (single-key) nodes in list order
//   final phase: split the (size, creation) largest first; new list =
//                reverse(children in split order) ++ unsplit nodes in order.
// Keys stay in global scratch (L2-resident); each key carries its node index.
// Size ties in the final phase: later-created node first.
// ===========================================================================
struct QNode {
    int16_t x0, y0, x1, y1;
    int32_t count;
    uint32_t best;   // (score << 24) | (0xFFFFFF - key index): max = best response, first on ties
    int32_t seq;     // creation order among this round's children
};

__device__ inline QNode child_of(const QNode &n, int q) {
    const int hx = (n.x1 - n.x0 + 1) >> 1, hy = (n.y1 - n.y0 + 1) >> 1;
    const int mx = n.x0 + hx, my = n.y0 + hy;
    QNode c;
    c.x0 = (int16_t)((q & 1) ? mx : n.x0);
    c.x1 = (int16_t)((q & 1) ? n.x1 : mx);
    c.y0 = (int16_t)((q & 2) ? my : n.y0);
    c.y1 = (int16_t)((q & 2) ? n.y1 : my);
    c.count = 0;
    c.best = 0;
    c.seq = 0;
    return c;
}

__device__ inline int quadrant_of(const QNode &n, uint32_t key) {
    const int hx = (n.x1 - n.x0 + 1) >> 1, hy = (n.y1 - n.y0 + 1) >> 1;
    const int rx = (int)(key & 0xFFF) - kBorder, ry = (int)((key >> 12) & 0xFFF) - kBorder;
    return (rx < n.x0 + hx ? 0 : 1) | (ry < n.y0 + hy ? 0 : 2);
}

__device__ inline uint32_t best_pack(uint32_t key, int k) {
    return ((key >> 24) << 24) | (uint32_t)(0xFFFFFF - k);
}

struct QLds {
    QNode *cur, *nxt;
    uint32_t *ccnt, *cbest;
    int16_t *nidx_c, *nidx_s;
    uint8_t *mark;
    uint64_t *a64, *b64;
    int np2;
};

// The level's keys, each with its node index and quadrant.  R > 0: thread t
// holds keys t + 256 j (j < R) in registers for the whole distribution (the
// rounds then touch no global memory); R == 0: they stay in global scratch.
// 6 keys per thread cover the bench levels (VGA level 0: ~1300 keys) in 72
// VGPRs (7 waves per SIMD); levels up to kQuadRegKeys take 8 (with spills)
// Per workgroup size NT: register keys per thread on the narrow (R1) and wide
// (R2) paths, the key -> source map's capacity (KR) and workgroups per CU.
// NT = 1024 serves launches too small to fill the chip (a few frames: the
// drop-in call, a sharded camera set), where a level's latency is the step's.
#ifndef ORBX_QT_R4A
#define ORBX_QT_R4A 1   // (0.403 -> 0.395 ms per 3072 VGA frames, profiles/r04_ab_qt_rounds_vga.txt)
#endif
constexpr bool kQtRoundsR4 = ORBX_QT_R4A;   // (A/B: round 3's round structure on the 256-thread register path)
template <int NT> struct QCfg;
#ifndef ORBX_QT_REGROOTS
#define ORBX_QT_REGROOTS 0   // 1: the register paths count the roots in the gather too (slower:
                             // FHD 0.162 -> 0.164, EuRoC 0.069 -> 0.080 ms, profiles/r04_ab_qt_regroots.txt)
#endif
constexpr bool kQtRegRoots = ORBX_QT_REGROOTS;
#ifndef ORBX_QT_LEVEL_MAJOR
#define ORBX_QT_LEVEL_MAJOR 1   // workgroups dispatched level by level (longest first), not frame by frame
#endif
constexpr bool kQtLevelMajor = ORBX_QT_LEVEL_MAJOR;
constexpr int kQPreRoots = 16;   // roots the global-key gather counts itself (more: the roots' own pass)
#ifndef ORBX_QT_R2
#define ORBX_QT_R2 (kQuadRegKeys / 256)
#endif
#ifndef ORBX_QT_MINB
#define ORBX_QT_MINB 7
#endif
template <> struct QCfg<256> { static constexpr int R1 = 6, R2 = ORBX_QT_R2, KR = kQuadRegKeys, MINB = ORBX_QT_MINB; };
#ifndef ORBX_QT_R2_512
#define ORBX_QT_R2_512 (2 * kQuadRegKeysW / 1024)
#endif
template <> struct QCfg<512> { static constexpr int R1 = 10, R2 = ORBX_QT_R2_512, KR = kQuadRegKeysW, MINB = 4; };
template <> struct QCfg<1024> { static constexpr int R1 = 4, R2 = kQuadRegKeysW / 1024, KR = kQuadRegKeysW, MINB = 1; };
// R == 0 (keys in global scratch): a pass walks the keys kQU per thread at a
// time, the chunk's loads issued together into a register cache (key k =
// k0 + u NT + tid: every pass maps a key to the same thread, so its node
// and quadrant need no cross-thread ordering), then the chunk's node and
// quadrant written back.  A key pass is then ~n / (kQU NT) L2 round
// trips instead of n / NT (FHD level 0: ~9.6 k keys, 5 instead of 38).
#ifndef ORBX_QT_QU
#define ORBX_QT_QU 4
#endif
constexpr int kQU = ORBX_QT_QU;
#ifndef ORBX_QT_PF
#define ORBX_QT_PF 0   // (FHD quadtree 0.243 -> 0.255 ms with it, profiles/r04_ab_qt_fhd.txt)
#endif
template <int R, int NT>
struct QKeys {
    static constexpr int C = R > 0 ? R : kQU;   // registers: the keys, or the chunk cache
    uint32_t key[C];
    uint32_t nq[C];   // node | quadrant << 16
    uint32_t *gkeys;
    uint16_t *gnode;
    uint8_t *gq;
    int n;
    // the chunk at k0 into the cache (R == 0)
    __device__ inline void load(int k0) {
#pragma unroll
        for (int u = 0; u < C; ++u) {
            const int k = k0 + u * NT + (int)threadIdx.x;
            if (k < n) {
                key[u] = gkeys[k];
                // (a key's quadrant is 0..3; masked, as the scratch starts
                // unwritten and an unsplit node's keys read any of its 4 slots)
                nq[u] = (uint32_t)gnode[k] | ((uint32_t)(gq[k] & 3) << 16);
            }
        }
    }
    // the chunk at k0 into (pk, pq) without touching the cache (prefetch)
    __device__ inline void fetch(int k0, uint32_t *pk, uint32_t *pq) const {
#pragma unroll
        for (int u = 0; u < C; ++u) {
            const int k = k0 + u * NT + (int)threadIdx.x;
            if (k < n) {
                pk[u] = gkeys[k];
                pq[u] = (uint32_t)gnode[k] | ((uint32_t)(gq[k] & 3) << 16);
            }
        }
    }
    // body(k0) over every chunk, the next chunk's loads in flight while the
    // body runs (ORBX_QT_PF; the loads of a chunk precede the stores of the
    // chunk before it, and the chunks are disjoint)
    template <typename B>
    __device__ inline void chunks(B body) {
#if ORBX_QT_PF
        uint32_t pk[C], pq[C];
        fetch(0, pk, pq);
        for (int k0 = 0; k0 < n; k0 += NT * kQU) {
#pragma unroll
            for (int u = 0; u < C; ++u) { key[u] = pk[u]; nq[u] = pq[u]; }
            if (k0 + NT * kQU < n) fetch(k0 + NT * kQU, pk, pq);
            body(k0);
            store(k0);
        }
#else
        for (int k0 = 0; k0 < n; k0 += NT * kQU) {
            load(k0);
            body(k0);
            store(k0);
        }
#endif
    }
    __device__ inline void store(int k0) {
#pragma unroll
        for (int u = 0; u < C; ++u) {
            const int k = k0 + u * NT + (int)threadIdx.x;
            if (k < n) {
                gnode[k] = (uint16_t)(nq[u] & 0xFFFF);
                gq[k] = (uint8_t)(nq[u] >> 16);
            }
        }
    }
    // f(j, k) for every key this thread owns
    template <typename F>
    __device__ inline void each(F f) {
        if constexpr (R > 0) {
#pragma unroll
            for (int j = 0; j < R; ++j) {
                const int k = (int)threadIdx.x + j * NT;
                if (k < n) f(j, k);
            }
        } else {
            chunks([&](int k0) {
#pragma unroll
                for (int u = 0; u < kQU; ++u) {
                    const int k = k0 + u * NT + (int)threadIdx.x;
                    if (k < n) f(u, k);
                }
            });
        }
    }
    // f(j, k, valid) on every lane for every key slot (bodies with DPP)
    template <typename F>
    __device__ inline void each_all(F f) {
        if constexpr (R > 0) {
#pragma unroll
            for (int j = 0; j < R; ++j) {
                const int k = (int)threadIdx.x + j * NT;
                f(j, k, k < n);
            }
        } else {
            chunks([&](int k0) {
#pragma unroll
                for (int u = 0; u < kQU; ++u) {
                    const int k = k0 + u * NT + (int)threadIdx.x;
                    f(u, k, k < n);
                }
            });
        }
    }
    __device__ inline uint32_t get_key(int j, int) const { return key[j]; }
    __device__ inline int node(int j, int) const { return (int)(nq[j] & 0xFFFF); }
    __device__ inline int quad(int j, int) const { return (int)(nq[j] >> 16); }
    __device__ inline void set_node(int j, int, int nd) { nq[j] = (nq[j] & 0xFFFF0000u) | (uint32_t)nd; }
    __device__ inline void set_quad(int j, int, int q) { nq[j] = (nq[j] & 0xFFFFu) | ((uint32_t)q << 16); }
};

#ifndef ORBX_QT_AGG
#define ORBX_QT_AGG 2   // 1: lane quads only, 2: quads, then rows of 16 lanes
#endif
// Adds each lane's (slot, bp) to cnt[slot] += 1, best[slot] = max(., bp)
// (slot ~0u: nothing) with LDS atomics pre-aggregated over neighbouring
// lanes.  The quadtree's keys sit in cell order, so neighbouring lanes mostly
// hit one slot, and same-address atomics within an instruction serialise in
// the LDS (636 address-conflict cycles per wave before this, 247 after; the
// kernel 0.61 -> 0.38 ms per 3072 VGA frames).  A lane row (16 lanes) or
// quad whose lanes all carry one slot adds its count and maximum from its
// first lane.  Every lane of the wave must call it (DPP).
__device__ inline void agg_atomics(uint32_t *cnt, uint32_t *best, uint32_t slot, uint32_t bp) {
    constexpr int kQX1 = 0xB1, kQX2 = 0x4E;   // quad_perm [1,0,3,2], [2,3,0,1]
    uint32_t lo = min(slot, dpp_or<kQX1>(0u, slot)), hi = max(slot, dpp_or<kQX1>(0u, slot));
    lo = min(lo, dpp_or<kQX2>(0u, lo));
    hi = max(hi, dpp_or<kQX2>(0u, hi));
    uint32_t b4 = max(bp, dpp_or<kQX1>(0u, bp));
    b4 = max(b4, dpp_or<kQX2>(0u, b4));
    const bool quad = lo == hi && slot != ~0u;   // (a mixed quad has lo < hi)
    const int lane = (int)threadIdx.x & 63;
#if ORBX_QT_AGG >= 2
    constexpr int kRor4 = 0x124, kRor8 = 0x128;   // row_ror:4, row_ror:8
    uint32_t rlo = min(lo, dpp_or<kRor4>(0u, lo)), rhi = max(hi, dpp_or<kRor4>(0u, hi));
    rlo = min(rlo, dpp_or<kRor8>(0u, rlo));
    rhi = max(rhi, dpp_or<kRor8>(0u, rhi));
    uint32_t b16 = max(b4, dpp_or<kRor4>(0u, b4));
    b16 = max(b16, dpp_or<kRor8>(0u, b16));
    if (rlo == rhi && slot != ~0u) {
        if ((lane & 15) == 0) {
            atomicAdd(&cnt[slot], 16u);
            atomicMax(&best[slot], b16);
        }
        return;
    }
#endif
    if (quad) {
        if ((lane & 3) == 0) {
            atomicAdd(&cnt[slot], 4u);
            atomicMax(&best[slot], b4);
        }
    } else if (slot != ~0u) {
        atomicAdd(&cnt[slot], 1u);
        atomicMax(&best[slot], bp);
    }
}

// Child counts / best keys of the splittable nodes.  ccnt / cbest[0, 4S)
// were zeroed by the step that produced the current nodes (zero_children),
// ordered by that step's closing barrier.  Ends with a barrier.
template <int R, int NT>
__device__ __attribute__((always_inline)) void child_stats(const QLds &s, QKeys<R, NT> &K) {
    // every lane runs each slot's aggregation (lanes past the key count carry
    // slot ~0u)
    K.each_all([&](int j, int k, bool valid) {
        uint32_t slot = ~0u, bp = 0;
        if (valid) {
            const int nd = K.node(j, k);
            const QNode node = s.cur[nd];
            if (node.count > 1) {
                const uint32_t key = K.get_key(j, k);
                const int q = quadrant_of(node, key);
                K.set_quad(j, k, q);
                slot = 4u * (uint32_t)nd + (uint32_t)q;
                bp = best_pack(key, k);
            }
        }
        agg_atomics(s.ccnt, s.cbest, slot, bp);
    });
    __syncthreads();
}

template <int NT>
__device__ inline void zero_children(const QLds &s, int S) {
    for (int i = threadIdx.x; i < 4 * S; i += NT) { s.ccnt[i] = 0; s.cbest[i] = 0; }
}

// One key pass per round: each key moves to its node of the round just built
// (nidx_c[4 node + quadrant]) and, when that node is splittable, adds itself
// to the node's child counts (as child_stats).  Ends with a barrier.  The
// 256-thread form with register-held keys (VGA) moves the keys in a pass of
// their own and then counts (0.386 vs 0.403 ms fused per 3072 VGA frames,
// profiles/r04_ab_qt_fhd2.txt): the fused pass's dependent LDS reads queue
// behind each key's atomics; the global-key path and the wider forms gain from
// the single pass (FHD 0.298 -> 0.243 ms).  (No barrier between the two
// loops: the move touches registers only, and the counters were zeroed before
// the barrier that precedes this pass.)
template <int R, int NT>
__device__ __attribute__((always_inline)) void advance_stats(const QLds &s, QKeys<R, NT> &K) {
    if constexpr (NT == 256 && R > 0) {
        K.each([&](int j, int k) { K.set_node(j, k, s.nidx_c[4 * K.node(j, k) + K.quad(j, k)]); });
        child_stats(s, K);
        return;
    }
    K.each_all([&](int j, int k, bool valid) {
        uint32_t slot = ~0u, bp = 0;
        if (valid) {
            const int nd = s.nidx_c[4 * K.node(j, k) + K.quad(j, k)];
            K.set_node(j, k, nd);
            const QNode node = s.cur[nd];
            if (node.count > 1) {
                const uint32_t key = K.get_key(j, k);
                const int q = quadrant_of(node, key);
                K.set_quad(j, k, q);
                slot = 4u * (uint32_t)nd + (uint32_t)q;
                bp = best_pack(key, k);
            }
        }
        agg_atomics(s.ccnt, s.cbest, slot, bp);
    });
    __syncthreads();
}

// A node that keeps its keys maps all four quadrant slots to its new index,
// so a key's next node is one read, nidx_c[4 node + quadrant], split or not
// (an unsplit node's keys carry a stale quadrant; every slot agrees).
__device__ inline void set_all_quads(int16_t *nidx_c, int i, int ni) {
    const uint32_t v = ((uint32_t)ni & 0xFFFFu) * 0x10001u;
    *reinterpret_cast<uint2 *>(nidx_c + 4 * i) = make_uint2(v, v);
}

__device__ inline QNode make_child(const QLds &s, const QNode &parent, int i, int q, int seq) {
    QNode c = child_of(parent, q);
    c.count = (int32_t)s.ccnt[4 * i + q];
    c.best = s.cbest[4 * i + q];
    c.seq = seq;
    return c;
}

// Phases 2-5 of k_quadtree on the gathered keys (ORBextractor.cc:566-784).
template <int NR, int NT>
__device__ __attribute__((always_inline)) void quadtree_rounds(const DevPlan &p, const FrameBufs &fb, QLds &s, const LevelGeom &g, int b, int l,
                                QKeys<NR, NT> &K, uint64_t &phase_t_, const uint32_t *pre_cnt = nullptr,
                                const uint32_t *pre_best = nullptr) {
    const int tid = threadIdx.x;
    const int N = g.quota, NC = p.node_cap;
    const uint32_t *keys = K.gkeys;
    int32_t *level_count = fb.level_count + (int64_t)b * kMaxLevels + l;
    __shared__ uint64_t ws64[NT / 64];
    __shared__ int sh_S, sh_R, sh_nv;

    // ---- 2. root nodes (ORBextractor.cc:566-613)
    const int nini = g.nini;
    if (pre_cnt) {
        // counted in the gather (every key's node is its root index r, its
        // quadrant 0): the non-empty roots in order, and root r's four slots
        // of nidx_c map to its list position, so the first key pass moves the
        // keys as any round's does (advance_stats)
        for (int i = tid; i < 4 * nini; i += NT) { s.ccnt[i] = 0; s.cbest[i] = 0; }
        if (tid == 0) {
            int S = 0;
            for (int r = 0; r < nini; ++r) {
                if (pre_cnt[r] == 0) continue;
                QNode nd;
                nd.x0 = (int16_t)(int)__fmul_rn(g.hx, (float)r);
                nd.x1 = (int16_t)(int)__fmul_rn(g.hx, (float)(r + 1));
                nd.y0 = 0;
                nd.y1 = (int16_t)(g.h - 2 * kBorder);
                nd.count = (int32_t)pre_cnt[r];
                nd.best = pre_best[r];
                nd.seq = 0;
                s.cur[S] = nd;
                set_all_quads(s.nidx_c, r, S);
                ++S;
            }
            sh_S = S;
        }
        __syncthreads();
    } else if (nini == 1) {
        // one root (every 4:3 or squarer level): every key's node is 0, its
        // count the key count and its best key a block maximum (wave maxima
        // through LDS: no per-key atomics, no serial pass)
        __shared__ uint32_t ws_root[NT / 64];
        uint32_t bm = 0;
        K.each([&](int j, int k) {
            K.set_node(j, k, 0);
            bm = max(bm, best_pack(K.get_key(j, k), k));
        });
        bm = wave_max_u32(bm);
        if ((tid & 63) == 0) ws_root[tid >> 6] = bm;
        zero_children<NT>(s, 1);
        __syncthreads();
        if (tid == 0) {
            QNode nd;
            nd.x0 = (int16_t)(int)__fmul_rn(g.hx, 0.0f);
            nd.x1 = (int16_t)(int)__fmul_rn(g.hx, 1.0f);
            nd.y0 = 0;
            nd.y1 = (int16_t)(g.h - 2 * kBorder);
            nd.count = (int32_t)K.n;
            uint32_t best = 0;
            for (int w = 0; w < NT / 64; ++w) best = max(best, ws_root[w]);
            nd.best = best;
            nd.seq = 0;
            s.cur[0] = nd;
            sh_S = 1;
        }
        __syncthreads();
    } else {
        for (int i = tid; i < nini; i += NT) { s.ccnt[i] = 0; s.cbest[i] = 0; }
        __syncthreads();
        auto root_of = [&](uint32_t key) {
            const float rx = (float)((int)(key & 0xFFF) - kBorder);
            return min((int)__fdiv_rn(rx, g.hx), nini - 1);
        };
        K.each_all([&](int j, int k, bool valid) {
            uint32_t slot = ~0u, bp = 0;
            if (valid) {
                const uint32_t key = K.get_key(j, k);
                const int r = root_of(key);
                K.set_node(j, k, r);
                slot = (uint32_t)r;
                bp = best_pack(key, k);
            }
            agg_atomics(s.ccnt, s.cbest, slot, bp);
        });
        __syncthreads();
        if (tid == 0) {
            int S = 0;
            for (int r = 0; r < nini; ++r) {
                if (s.ccnt[r] == 0) continue;
                QNode nd;
                nd.x0 = (int16_t)(int)__fmul_rn(g.hx, (float)r);
                nd.x1 = (int16_t)(int)__fmul_rn(g.hx, (float)(r + 1));
                nd.y0 = 0;
                nd.y1 = (int16_t)(g.h - 2 * kBorder);
                nd.count = (int32_t)s.ccnt[r];
                nd.best = s.cbest[r];
                nd.seq = 0;
                s.cur[S] = nd;
                s.nidx_s[r] = (int16_t)S;
                ++S;
            }
            sh_S = S;
        }
        __syncthreads();
        K.each([&](int j, int k) { K.set_node(j, k, s.nidx_s[K.node(j, k)]); });
        zero_children<NT>(s, sh_S);   // (the roots' counts were read before the barrier above)
        __syncthreads();
    }
    PHASE_MARK(2, 1);   // roots

    if (p.dbg_stop == 2) return;
    int S;
    if constexpr (kQtRoundsR4 && NT == 256 && NR > 0) {
        // the round structure of round 3 (a stats pass at the top of each round,
        // the move and the counters' zeroing after the node phase): ORBX_QT_R4A
        // ---- 3. full rounds (ORBextractor.cc:618-696)
        bool final_phase = false;
        if (pre_cnt)   // (roots counted in the gather: the keys move to the roots' list positions)
            K.each([&](int j, int k) { K.set_node(j, k, s.nidx_c[4 * K.node(j, k)]); });
        while (true) {
            const int S = sh_S;
            child_stats(s, K);
            PHASE_MARK(2, 2);   // full rounds: child counts
            // per node: (non-empty children | single-key parents << 21 | children
            // with more than one key << 42), scanned over a contiguous node range
            // per thread, so each thread reads back only its own entries
            const int per = (S + NT - 1) / NT;
            const int i0 = min(tid * per, S), i1 = min(i0 + per, S);
            uint64_t local = 0;
            for (int i = i0; i < i1; ++i) {
                uint64_t v = 1ull << 21;
                if (s.cur[i].count > 1) {
                    uint64_t nc = 0, ex = 0;
                    for (int q = 0; q < 4; ++q) { nc += s.ccnt[4 * i + q] > 0; ex += s.ccnt[4 * i + q] > 1; }
                    v = nc | (ex << 42);
                }
                s.a64[i] = v;
                local += v;
            }
            const uint64_t incl = wave_incl_scan_u64(local);
            if ((tid & 63) == 63) ws64[tid >> 6] = incl;
            __syncthreads();
            uint64_t run = incl - local, tot = 0;
            for (int w = 0; w < NT / 64; ++w) {
                if (w < (tid >> 6)) run += ws64[w];
                tot += ws64[w];
            }
            const int C = (int)(tot & 0x1FFFFF), singles = (int)((tot >> 21) & 0x1FFFFF);
            const int nexp = (int)(tot >> 42);
            const int S2 = C + singles;
            if (S2 > NC) {  // cannot happen by the bound in make_plan; fail loudly
                if (tid == 0) *level_count = -1;
                return;
            }
            for (int i = i0; i < i1; ++i) {
                const uint64_t pre = run;
                run += s.a64[i];
                const QNode nd = s.cur[i];
                if (nd.count > 1) {
                    int pos = (int)(pre & 0x1FFFFF);
                    for (int q = 0; q < 4; ++q) {
                        if (s.ccnt[4 * i + q] == 0) continue;
                        const int ni = C - 1 - pos;
                        s.nxt[ni] = make_child(s, nd, i, q, pos);
                        s.nidx_c[4 * i + q] = (int16_t)ni;
                        ++pos;
                    }
                } else {
                    const int ni = C + (int)((pre >> 21) & 0x1FFFFF);
                    s.nxt[ni] = nd;
                    set_all_quads(s.nidx_c, i, ni);
                }
            }
            __syncthreads();
            K.each([&](int j, int k) { K.set_node(j, k, s.nidx_c[4 * K.node(j, k) + K.quad(j, k)]); });
            zero_children<NT>(s, S2);
            {
                QNode *t = s.cur; s.cur = s.nxt; s.nxt = t;
            }
            if (tid == 0) sh_S = S2;
            __syncthreads();
            PHASE_MARK(2, 3);   // full rounds: scan + children
            if (S2 >= N || S2 == S) break;
            if (S2 + nexp * 3 > N) { final_phase = true; break; }
        }

        if (p.dbg_stop == 3) return;
        // ---- 4. final phase (ORBextractor.cc:697-762)
        while (final_phase) {
            const int S = sh_S;
            if (tid == 0) sh_nv = 0;   // (ordered by child_stats' barrier)
            child_stats(s, K);
            {
                int nz = 0;
                for (int i = tid; i < s.np2; i += NT) {
                    uint64_t v = 0;
                    if (i < S && s.cur[i].count > 1)
                        v = ((uint64_t)s.cur[i].count << 40) | ((uint64_t)s.cur[i].seq << 16) | (uint64_t)i;
                    s.a64[i] = v;
                    s.b64[i] = 0;
                    nz += v != 0;
                }
                nz = wave_sum_i32(nz);
                if ((tid & 63) == 0 && nz) atomicAdd(&sh_nv, nz);
            }
            for (int i = tid; i < S; i += NT) s.mark[i] = 0;
            __syncthreads();
            PHASE_MARK(2, 4);   // final: child counts
            // descending order of the splittable nodes' (count, seq, index) keys
            // (all distinct) by rank counting: one barrier instead of a bitonic
            // network's log^2 stages; zeros (unsplittable) stay behind, in b64
            {
                // eight entries per step, their four reads issued together (one LDS
                // round trip per step instead of per pair); a64[S, np2) is 0 and np2
                // a power of two >= 8
                const int S8 = (S + 7) & ~7;
                for (int i = tid; i < S; i += NT) {
                    const uint64_t v = s.a64[i];
                    if (v == 0) continue;
                    int r = 0;
                    for (int j = 0; j < S8; j += 8) {
                        const ulonglong2 w0 = *reinterpret_cast<const ulonglong2 *>(s.a64 + j);
                        const ulonglong2 w1 = *reinterpret_cast<const ulonglong2 *>(s.a64 + j + 2);
                        const ulonglong2 w2 = *reinterpret_cast<const ulonglong2 *>(s.a64 + j + 4);
                        const ulonglong2 w3 = *reinterpret_cast<const ulonglong2 *>(s.a64 + j + 6);
                        r += (w0.x > v) + (w0.y > v) + (w1.x > v) + (w1.y > v) + (w2.x > v) + (w2.y > v) +
                             (w3.x > v) + (w3.y > v);
                    }
                    s.b64[r] = v;
                }
                __syncthreads();
                uint64_t *t = s.a64; s.a64 = s.b64; s.b64 = t;
            }
            PHASE_MARK(2, 5);   // final: sort
            // per rank: number of non-empty children (nc) and gain (nc - 1)
            for (int r = tid; r < s.np2; r += NT) {
                uint64_t v = 0;
                if (s.a64[r] != 0) {
                    const int i = (int)(s.a64[r] & 0xFFFF);
                    int nc = 0;
                    for (int q = 0; q < 4; ++q) nc += s.ccnt[4 * i + q] > 0;
                    v = (uint64_t)nc | ((uint64_t)(nc - 1) << 32);
                }
                s.b64[r] = v;
            }
            if (tid == 0) sh_R = -1;
            __syncthreads();
            const int nv = sh_nv;
            block_excl_scan_u64<NT>(s.b64, s.np2, ws64);
            for (int r = tid; r < nv; r += NT) {
                const int i = (int)(s.a64[r] & 0xFFFF);
                int nc = 0;
                for (int q = 0; q < 4; ++q) nc += s.ccnt[4 * i + q] > 0;
                const int incl = (int)(s.b64[r] >> 32) + nc - 1;
                const int prev = (int)(s.b64[r] >> 32);
                if (S + incl >= N && S + prev < N) sh_R = r + 1;
            }
            __syncthreads();
            const int R = sh_R < 0 ? nv : sh_R;
            int CC;
            {
                if (R > 0) {
                    const int i = (int)(s.a64[R - 1] & 0xFFFF);
                    int nc = 0;
                    for (int q = 0; q < 4; ++q) nc += s.ccnt[4 * i + q] > 0;
                    CC = (int)(s.b64[R - 1] & 0xFFFFFFFF) + nc;
                } else {
                    CC = 0;
                }
            }
            const int S2 = CC + (S - R);
            if (S2 > NC) {
                if (tid == 0) *level_count = -1;
                return;
            }
            for (int r = tid; r < R; r += NT) {
                const int i = (int)(s.a64[r] & 0xFFFF);
                int cs = (int)(s.b64[r] & 0xFFFFFFFF);
                const QNode nd = s.cur[i];
                for (int q = 0; q < 4; ++q) {
                    if (s.ccnt[4 * i + q] == 0) continue;
                    const int ni = CC - 1 - cs;
                    s.nxt[ni] = make_child(s, nd, i, q, cs);
                    s.nidx_c[4 * i + q] = (int16_t)ni;
                    ++cs;
                }
                s.mark[i] = 1;
            }
            __syncthreads();
            for (int i = tid; i < s.np2; i += NT) s.b64[i] = (i < S && !s.mark[i]) ? 1 : 0;
            __syncthreads();
            block_excl_scan_u64<NT>(s.b64, s.np2, ws64);
            for (int i = tid; i < S; i += NT) {
                if (s.mark[i]) continue;
                const int ni = CC + (int)s.b64[i];
                s.nxt[ni] = s.cur[i];
                set_all_quads(s.nidx_c, i, ni);
            }
            __syncthreads();
            K.each([&](int j, int k) { K.set_node(j, k, s.nidx_c[4 * K.node(j, k) + K.quad(j, k)]); });
            zero_children<NT>(s, S2);
            {
                QNode *t = s.cur; s.cur = s.nxt; s.nxt = t;
            }
            if (tid == 0) sh_S = S2;
            __syncthreads();
            PHASE_MARK(2, 6);   // final: splits
            if (S2 >= N || S2 == S) break;
        }
        S = sh_S;
    } else {
        // Each round is one key pass: the pass that moves the keys into their
        // new nodes also adds them to those nodes' child counts (advance_stats),
        // and the child counts are re-zeroed in the round's node phase (each
        // thread its own nodes' entries after it read them, plus [4 S, 4 S2)), so
        // the rounds need no pass of their own for either.  The last round's move
        // only matters to the register path's output (phase 5).
        bool final_phase = false;
        S = sh_S;
        if (pre_cnt) advance_stats(s, K);
        else child_stats(s, K);
        PHASE_MARK(2, 2);   // child counts
        // ---- 3. full rounds (ORBextractor.cc:618-696)
        while (true) {
            // per node: (non-empty children | single-key parents << 21 | children
            // with more than one key << 42), scanned over a contiguous node range
            // per thread, so each thread reads back only its own entries
            const int per = (S + NT - 1) / NT;
            const int i0 = min(tid * per, S), i1 = min(i0 + per, S);
            uint64_t local = 0;
            for (int i = i0; i < i1; ++i) {
                uint64_t v = 1ull << 21;
                if (s.cur[i].count > 1) {
                    uint64_t nc = 0, ex = 0;
                    for (int q = 0; q < 4; ++q) { nc += s.ccnt[4 * i + q] > 0; ex += s.ccnt[4 * i + q] > 1; }
                    v = nc | (ex << 42);
                }
                s.a64[i] = v;
                local += v;
            }
            const uint64_t incl = wave_incl_scan_u64(local);
            if ((tid & 63) == 63) ws64[tid >> 6] = incl;
            __syncthreads();
            uint64_t run = incl - local, tot = 0;
            for (int w = 0; w < NT / 64; ++w) {
                if (w < (tid >> 6)) run += ws64[w];
                tot += ws64[w];
            }
            const int C = (int)(tot & 0x1FFFFF), singles = (int)((tot >> 21) & 0x1FFFFF);
            const int nexp = (int)(tot >> 42);
            const int S2 = C + singles;
            if (S2 > NC) {  // cannot happen by the bound in make_plan; fail loudly
                if (tid == 0) *level_count = -1;
                return;
            }
            for (int i = i0; i < i1; ++i) {
                const uint64_t pre = run;
                run += s.a64[i];
                const QNode nd = s.cur[i];
                if (nd.count > 1) {
                    int pos = (int)(pre & 0x1FFFFF);
                    for (int q = 0; q < 4; ++q) {
                        if (s.ccnt[4 * i + q] == 0) continue;
                        const int ni = C - 1 - pos;
                        s.nxt[ni] = make_child(s, nd, i, q, pos);
                        s.nidx_c[4 * i + q] = (int16_t)ni;
                        ++pos;
                    }
                } else {
                    const int ni = C + (int)((pre >> 21) & 0x1FFFFF);
                    s.nxt[ni] = nd;
                    set_all_quads(s.nidx_c, i, ni);
                }
            }
            // (only this thread reads its nodes' child entries)
            for (int i = 4 * i0; i < 4 * i1; ++i) { s.ccnt[i] = 0; s.cbest[i] = 0; }
            for (int i = 4 * S + tid; i < 4 * S2; i += NT) { s.ccnt[i] = 0; s.cbest[i] = 0; }
            __syncthreads();
            {
                QNode *t = s.cur; s.cur = s.nxt; s.nxt = t;
            }
            PHASE_MARK(2, 3);   // full rounds: scan + children
            const bool stop = S2 >= N || S2 == S;
            final_phase = !stop && S2 + nexp * 3 > N;
            S = S2;
            if (stop) {
                if constexpr (NR > 0) K.each([&](int j, int k) { K.set_node(j, k, s.nidx_c[4 * K.node(j, k) + K.quad(j, k)]); });
                break;
            }
            if (tid == 0) sh_nv = 0;   // (the final phase's count; ordered by the pass's barrier)
            advance_stats(s, K);
            PHASE_MARK(2, 2);   // full rounds: move + child counts
            if (final_phase) break;
        }

        if (p.dbg_stop == 3) return;
        // ---- 4. final phase (ORBextractor.cc:697-762); the child counts of the
        //         S nodes are in place
        while (final_phase) {
            {
                int nz = 0;
                for (int i = tid; i < s.np2; i += NT) {
                    uint64_t v = 0;
                    if (i < S && s.cur[i].count > 1)
                        v = ((uint64_t)s.cur[i].count << 40) | ((uint64_t)s.cur[i].seq << 16) | (uint64_t)i;
                    s.a64[i] = v;
                    s.b64[i] = 0;
                    nz += v != 0;
                }
                nz = wave_sum_i32(nz);
                if ((tid & 63) == 0 && nz) atomicAdd(&sh_nv, nz);
            }
            for (int i = tid; i < S; i += NT) s.mark[i] = 0;
            __syncthreads();
            PHASE_MARK(2, 4);   // final: node keys
            // descending order of the splittable nodes' (count, seq, index) keys
            // (all distinct) by rank counting: one barrier instead of a bitonic
            // network's log^2 stages; zeros (unsplittable) stay behind, in b64
            {
                // eight entries per step, their four reads issued together (one LDS
                // round trip per step instead of per pair); a64[S, np2) is 0 and np2
                // a power of two >= 8
                const int S8 = (S + 7) & ~7;
                for (int i = tid; i < S; i += NT) {
                    const uint64_t v = s.a64[i];
                    if (v == 0) continue;
                    int r = 0;
                    for (int j = 0; j < S8; j += 8) {
                        const ulonglong2 w0 = *reinterpret_cast<const ulonglong2 *>(s.a64 + j);
                        const ulonglong2 w1 = *reinterpret_cast<const ulonglong2 *>(s.a64 + j + 2);
                        const ulonglong2 w2 = *reinterpret_cast<const ulonglong2 *>(s.a64 + j + 4);
                        const ulonglong2 w3 = *reinterpret_cast<const ulonglong2 *>(s.a64 + j + 6);
                        r += (w0.x > v) + (w0.y > v) + (w1.x > v) + (w1.y > v) + (w2.x > v) + (w2.y > v) +
                             (w3.x > v) + (w3.y > v);
                    }
                    s.b64[r] = v;
                }
                __syncthreads();
                uint64_t *t = s.a64; s.a64 = s.b64; s.b64 = t;
            }
            PHASE_MARK(2, 5);   // final: sort
            // per rank: number of non-empty children (nc) and gain (nc - 1)
            for (int r = tid; r < s.np2; r += NT) {
                uint64_t v = 0;
                if (s.a64[r] != 0) {
                    const int i = (int)(s.a64[r] & 0xFFFF);
                    int nc = 0;
                    for (int q = 0; q < 4; ++q) nc += s.ccnt[4 * i + q] > 0;
                    v = (uint64_t)nc | ((uint64_t)(nc - 1) << 32);
                }
                s.b64[r] = v;
            }
            if (tid == 0) sh_R = -1;
            __syncthreads();
            const int nv = sh_nv;
            block_excl_scan_u64<NT>(s.b64, s.np2, ws64);
            for (int r = tid; r < nv; r += NT) {
                const int i = (int)(s.a64[r] & 0xFFFF);
                int nc = 0;
                for (int q = 0; q < 4; ++q) nc += s.ccnt[4 * i + q] > 0;
                const int incl = (int)(s.b64[r] >> 32) + nc - 1;
                const int prev = (int)(s.b64[r] >> 32);
                if (S + incl >= N && S + prev < N) sh_R = r + 1;
            }
            __syncthreads();
            const int R = sh_R < 0 ? nv : sh_R;
            int CC;
            {
                if (R > 0) {
                    const int i = (int)(s.a64[R - 1] & 0xFFFF);
                    int nc = 0;
                    for (int q = 0; q < 4; ++q) nc += s.ccnt[4 * i + q] > 0;
                    CC = (int)(s.b64[R - 1] & 0xFFFFFFFF) + nc;
                } else {
                    CC = 0;
                }
            }
            const int S2 = CC + (S - R);
            if (S2 > NC) {
                if (tid == 0) *level_count = -1;
                return;
            }
            for (int r = tid; r < R; r += NT) {
                const int i = (int)(s.a64[r] & 0xFFFF);
                int cs = (int)(s.b64[r] & 0xFFFFFFFF);
                const QNode nd = s.cur[i];
                for (int q = 0; q < 4; ++q) {
                    if (s.ccnt[4 * i + q] == 0) continue;
                    const int ni = CC - 1 - cs;
                    s.nxt[ni] = make_child(s, nd, i, q, cs);
                    s.nidx_c[4 * i + q] = (int16_t)ni;
                    ++cs;
                }
                s.mark[i] = 1;
            }
            __syncthreads();
            // (the child entries are read no more this round: re-zeroed for the
            // next round's counts, S2 >= S)
            for (int i = tid; i < s.np2; i += NT) s.b64[i] = (i < S && !s.mark[i]) ? 1 : 0;
            zero_children<NT>(s, S2);
            __syncthreads();
            block_excl_scan_u64<NT>(s.b64, s.np2, ws64);
            for (int i = tid; i < S; i += NT) {
                if (s.mark[i]) continue;
                const int ni = CC + (int)s.b64[i];
                s.nxt[ni] = s.cur[i];
                set_all_quads(s.nidx_c, i, ni);
            }
            __syncthreads();
            {
                QNode *t = s.cur; s.cur = s.nxt; s.nxt = t;
            }
            PHASE_MARK(2, 6);   // final: splits
            const bool stop = S2 >= N || S2 == S;
            S = S2;
            if (stop) {
                if constexpr (NR > 0) K.each([&](int j, int k) { K.set_node(j, k, s.nidx_c[4 * K.node(j, k) + K.quad(j, k)]); });
                break;
            }
            if (tid == 0) sh_nv = 0;
            advance_stats(s, K);
            PHASE_MARK(2, 4);   // final: move + child counts
        }
    }

    // ---- 5. best key per node, in list order (ORBextractor.cc:765-784)
    uint32_t *sel = fb.sel + (int64_t)b * p.out_cap + g.out_off;
    const int S_out = min(S, g.out_cap);
    if constexpr (NR > 0) {
        // the owner of each node's best key writes it (keys live in registers)
        K.each([&](int j, int k) {
            const int nd = K.node(j, k);
            if (nd < S_out && 0xFFFFFF - (int)(s.cur[nd].best & 0xFFFFFF) == k) sel[nd] = K.key[j];
        });
    } else {
        for (int i = tid; i < S_out; i += NT) {
            const int k = 0xFFFFFF - (int)(s.cur[i].best & 0xFFFFFF);
            sel[i] = keys[k];
        }
    }
    if (tid == 0) *level_count = S <= g.out_cap ? S : -1;
    PHASE_MARK(2, 7);   // output
}

template <bool PIPE, int NT>
__global__ __launch_bounds__(NT, QCfg<NT>::MINB) void k_quadtree(DevPlan p, FrameBufs fb, int l0) {
    extern __shared__ __align__(16) uint8_t lds[];
    PHASE_START();
    // (level-major grid: every frame's level 0, the longest, goes out first)
    const int l = l0 + (kQtLevelMajor ? blockIdx.y : blockIdx.x), b = kQtLevelMajor ? blockIdx.x : blockIdx.y;
    const int tid = threadIdx.x;
    const LevelGeom g = p.lv[l];
    const int NC = p.node_cap;
    QLds s;
    s.np2 = 1;
    while (s.np2 < NC) s.np2 <<= 1;
    uint8_t *ptr = lds;
    s.a64 = reinterpret_cast<uint64_t *>(ptr); ptr += sizeof(uint64_t) * s.np2;
    s.b64 = reinterpret_cast<uint64_t *>(ptr); ptr += sizeof(uint64_t) * s.np2;
    s.cur = reinterpret_cast<QNode *>(ptr); ptr += sizeof(QNode) * NC;
    s.nxt = reinterpret_cast<QNode *>(ptr); ptr += sizeof(QNode) * NC;
    s.ccnt = reinterpret_cast<uint32_t *>(ptr); ptr += sizeof(uint32_t) * 4 * NC;
    s.cbest = reinterpret_cast<uint32_t *>(ptr); ptr += sizeof(uint32_t) * 4 * NC;
    s.nidx_c = reinterpret_cast<int16_t *>(ptr); ptr += sizeof(int16_t) * 4 * NC;
    s.nidx_s = reinterpret_cast<int16_t *>(ptr); ptr += sizeof(int16_t) * NC;
    s.mark = ptr;

    const int64_t kbase = (int64_t)b * p.cand_cap + g.cand_off;
    uint32_t *keys = fb.keys + kbase;
    uint16_t *knode = fb.key_node + kbase;
    uint8_t *kq = fb.key_q + kbase;
    int32_t *level_count = fb.level_count + (int64_t)b * kMaxLevels + l;

    // ---- 1. gather the level's candidates in cell order (the order the
    //         reference pushes them into vToDistributeKeys): per-cell start
    //         offsets and sources in LDS (the node arrays are free until phase 2)
    const int ncell = g.cell_end - g.cell_begin;
    int *cell_off = reinterpret_cast<int *>(lds);            // ncell + 1
    int *cell_src = cell_off + ncell + 1;                    // slot | bit 31: minThFAST list
    // key k's source (slot index | bit 31: minThFAST list), for the first
    // QCfg<NT>::KR keys: each cell's thread writes its keys' entries right after
    // the scan, so the keys load with one LDS read each after one barrier
    uint32_t *kaddr = reinterpret_cast<uint32_t *>(cell_src + ncell);
    __shared__ int ws2[2 * (NT / 64)];   // scan partials, alternating per chunk
    int base = 0;
    for (int c0 = 0, chunk = 0; c0 < ncell; c0 += NT, ++chunk) {
        const int c = c0 + tid;
        int word = 0, slot = 0;
        if (c < ncell) {
            word = fb.cell_count[(int64_t)b * p.ncells + g.cell_begin + c];
            slot = p.cells[g.cell_begin + c].slot;
        }
        const int cnt = word & 0x7FFFFFFF;
        int *ws = ws2 + (chunk & 1) * (NT / 64);
        const int incl = wave_incl_scan_i32(cnt);
        if ((tid & 63) == 63) ws[tid >> 6] = incl;
        __syncthreads();
        int pre = 0, tot = 0;
        for (int w = 0; w < NT / 64; ++w) {
            if (w < (tid >> 6)) pre += ws[w];
            tot += ws[w];
        }
        if (c < ncell) {
            const int off = base + pre + incl - cnt;
            const uint32_t src = (uint32_t)slot | (word < 0 ? 0x80000000u : 0u);
            cell_off[c] = off;
            cell_src[c] = (int)src;
            for (int i = 0; i < cnt && off + i < QCfg<NT>::KR; ++i) kaddr[off + i] = src + (uint32_t)i;
        }
        base += tot;
    }
    const int n = base;
    if (tid == 0) cell_off[ncell] = n;
    __syncthreads();
    if (p.dbg_stop == 1) return;
    if (n == 0 || g.nini <= 0) {
        if (tid == 0) *level_count = 0;
        return;
    }
    const uint32_t *cand = fb.cand + (int64_t)b * p.cand_cap, *cand2 = fb.cand2 + (int64_t)b * p.cand_cap;
    // the roots counted in the gather when there are few (every level but the
    // narrowest strips; one root has its own pass without atomics): count and
    // best key per root by the aggregated atomics, each key's node = its root
    // and quadrant 0 set with it (no roots pass over the keys of its own)
    __shared__ uint32_t rcnt[kQPreRoots], rbest[kQPreRoots];
    const int nini = g.nini;
    auto root_of = [&](uint32_t key) {
        const float rx = (float)((int)(key & 0xFFF) - kBorder);
        return min((int)__fdiv_rn(rx, g.hx), nini - 1);
    };
    // up to QCfg<NT>::R1 (R2) keys per thread stay in registers
    // through the rounds
    auto in_registers = [&](auto &K) {
        K.gkeys = nullptr; K.gnode = knode; K.gq = kq; K.n = n;
        const bool pre = kQtRegRoots && nini > 1 && nini <= kQPreRoots;
        if (pre) {
            if (tid < kQPreRoots) { rcnt[tid] = 0; rbest[tid] = 0; }
            __syncthreads();
            K.each_all([&](int j, int k, bool valid) {
                uint32_t slot = ~0u, bp = 0;
                if (valid) {
                    const uint32_t a = kaddr[k];
                    const uint32_t key = ((int)a < 0 ? cand2 : cand)[a & 0x7FFFFFFFu];
                    K.key[j] = key;
                    const int r = root_of(key);
                    K.nq[j] = (uint32_t)r;
                    slot = (uint32_t)r;
                    bp = best_pack(key, k);
                }
                agg_atomics(rcnt, rbest, slot, bp);   // (every lane: DPP)
            });
        } else {
            K.each([&](int j, int k) {
                const uint32_t a = kaddr[k];
                K.key[j] = ((int)a < 0 ? cand2 : cand)[a & 0x7FFFFFFFu];
                K.nq[j] = 0;
            });
        }
        __syncthreads();   // the cell tables are dead from here
        PHASE_MARK(2, 0);   // gather
        quadtree_rounds(p, fb, s, g, b, l, K, phase_t_, pre ? rcnt : nullptr, pre ? rbest : nullptr);
    };
    if (n <= QCfg<NT>::R1 * NT) {
        QKeys<QCfg<NT>::R1, NT> K;
        in_registers(K);
    } else if (n <= QCfg<NT>::R2 * NT) {
        QKeys<QCfg<NT>::R2, NT> K;
        in_registers(K);
    } else {
        QKeys<0, NT> K;
        K.gkeys = keys; K.gnode = knode; K.gq = kq; K.n = n;
        // the cell of key 64 m for every m (in the key-source map's LDS,
        // unused on this path): a wave's 64 keys (k0 is a multiple of 64)
        // then bisect only the cells between two of them
        const int nco = (n + 63) >> 6;
        int *coarse = reinterpret_cast<int *>(kaddr);
        const bool use_co = nco < QCfg<NT>::KR;
        if (use_co) {
            for (int c = tid; c < ncell; c += NT) {
                const int o = cell_off[c], e = cell_off[c + 1];
                for (int m = (o + 63) >> 6; (m << 6) < e; ++m) coarse[m] = c;
            }
            if (tid == 0) coarse[nco] = ncell - 1;
        }
        // the roots counted here when there are few (rcnt / rbest above)
        const bool pre = nini <= kQPreRoots;
        if (tid < kQPreRoots) { rcnt[tid] = 0; rbest[tid] = 0; }
        __syncthreads();
        // kQU keys per thread at a time (the chunk mapping of QKeys<0>): their
        // bisections interleave, and their candidate loads go out together
        for (int k0 = 0; k0 < n; k0 += NT * kQU) {
            int lo[kQU], hi[kQU];
#pragma unroll
            for (int u = 0; u < kQU; ++u) {
                const int m = (k0 + u * NT + tid) >> 6;   // (wave-uniform)
                lo[u] = use_co && m < nco ? coarse[m] : 0;
                hi[u] = use_co && m < nco ? coarse[m + 1] : ncell - 1;
            }
            for (bool more = true; more;) {
                more = false;
#pragma unroll
                for (int u = 0; u < kQU; ++u) {
                    const int k = k0 + u * NT + tid;
                    if (lo[u] < hi[u]) {
                        const int mid = (lo[u] + hi[u] + 1) >> 1;
                        if (cell_off[mid] <= k) lo[u] = mid; else hi[u] = mid - 1;
                        more |= lo[u] < hi[u];
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < kQU; ++u) {
                const int k = k0 + u * NT + tid;
                uint32_t slot = ~0u, bp = 0;
                if (k < n) {
                    const int src = cell_src[lo[u]];
                    const uint32_t key = ((src < 0) ? cand2 : cand)[(src & 0x7FFFFFFF) + (k - cell_off[lo[u]])];
                    keys[k] = key;
                    if (pre) {
                        int r = 0;
                        if (nini > 1) r = root_of(key);
                        knode[k] = (uint16_t)r;
                        kq[k] = 0;
                        slot = (uint32_t)r;
                        bp = best_pack(key, k);
                    }
                }
                if (pre) agg_atomics(rcnt, rbest, slot, bp);   // (every lane: DPP)
            }
        }
        __syncthreads();
        PHASE_MARK(2, 0);
        if (pre) quadtree_rounds(p, fb, s, g, b, l, K, phase_t_, rcnt, rbest);
        else quadtree_rounds(p, fb, s, g, b, l, K, phase_t_);
    }
}

// ===========================================================================
// K5: orientation + rBRIEF + keypoint record, one wave per selected key.
// The wave stages the 43x43 neighbourhood of its keypoint (radius 21, with the
// level's reflect-101 at the borders) in LDS once; from it come the integer
// IC moments (radius-15 disc, unblurred), the horizontal pass of the 7x7 s=2
// Gaussian over the window the rotated pattern can reach (|offset| <= 18), and
// each of the 512 samples as the vertical pass at that pixel.  Identical to
// sampling the blurred level (same taps, same per-column rounding); no
// blurred pyramid is written to HBM.
// ===========================================================================
constexpr int kDescR = 21;                  // patch radius = 18 (samples) + 3 (blur taps)
constexpr int kDescP = 2 * kDescR + 1;      // 43
constexpr int kDescPS = 48;                 // patch row stride (bytes): 43 + align offset, 8-aligned rows
constexpr int kBlurR = 18;
constexpr int kRowCols = 40;                // row-pass outputs at patch columns 0..39
constexpr int kColS = 44;                   // column-major row-pass buffer: stride (u16) of a column, rows 0..43
// The row-pass buffer is column-major: a sample's seven column-pass inputs
// (rows r..r+6 of one column) are 14 contiguous bytes, one unaligned
// ds_read_b128 (row 43 is padding the read may cover).
// The MFMA row pass reads 48 rows x 64 columns at the patch stride (rows
// 43..47, and columns past 45 that wrap into the next row, are either
// multiplied by zero taps or feed outputs that are never stored), all of it
// into registers before its first store: the patch is dead by then, so the
// row buffer overlays it (ORBX_DESC_OVERLAY; 3.5 KB a wave instead of 5.5:
// LDS no longer caps the occupancy).  Without the overlay the buffer follows
// the patch and the row pass's reads may run into it (they still precede
// the wave's stores).
#ifndef ORBX_DESC_OVERLAY
#define ORBX_DESC_OVERLAY 1
#endif
#ifndef ORBX_DESC_WAVES
#define ORBX_DESC_WAVES 8   // waves per SIMD the launch bounds ask for (VGPR budget 512 / this)
#endif
constexpr int kDescRowOff = ORBX_DESC_OVERLAY ? 0 : (kDescP * kDescPS + 15) & ~15;   // 0 or 2064
constexpr int kDescWaveLds = std::max(kDescRowOff + kRowCols * kColS * 2 + 8,    // (+ 8: the row pass's spill, below)
                                      47 * kDescPS + 64);                         // 3528 or 5592 B
static_assert((kDescR - 3 + kBlurR) + 7 < kColS, "a sample's 16-byte read stays in its column");
#ifndef ORBX_DESC_PAD
#define ORBX_DESC_PAD 0   // (occupancy probe: extra LDS bytes a wave)
#endif
constexpr int kDescWaveStride = (kDescWaveLds + ORBX_DESC_PAD + 15) & ~15;
static_assert(47 * kDescPS + 63 < kDescWaveLds, "MFMA row-pass reads stay inside the wave's LDS");
// LDS is allocated per workgroup in 512-byte granules: 4 waves + 48 B of
// shared angle records must fit ORBX_DESC_WAVES workgroups in a CU's 160 KB
static_assert(ORBX_DESC_WAVES * ((4 * kDescWaveStride + 48 + 511) & ~511) <= 160 * 1024,
              "k_describe: LDS for the occupancy the launch bounds ask");

// The row pass as an int8 matrix product (v_mfma_i32_16x16x32_i8): outputs
// j = 0..15 of a 16-column tile from the tile's 32 input columns,
//   R[r][16 t + j] = sum_c T[j][c] P[r][16 t + c],  T[j][c] = w[c - j] (0 <= c - j <= 6).
// T is the A operand, lane l holds T[l & 15][8 (l >> 4) + 0..7] (8 bytes, i8:
// the taps are <= 55).  The pixels go in as P - 128 (xor 0x80), so the
// accumulator starts at 128 * sum(w) = 128 * 257 = 32896, and the exact i32
// result is the reference's integer row sum (<= 65535).
struct RowTaps {
    uint64_t t[64];
    constexpr RowTaps() : t() {
        for (int l = 0; l < 64; ++l) {
            uint64_t v = 0;
            for (int jj = 0; jj < 8; ++jj) {
                const int d = 8 * (l >> 4) + jj - (l & 15);
                if (d >= 0 && d <= 6) v |= (uint64_t)kGaussTaps[d] << (8 * jj);
            }
            t[l] = v;
        }
    }
};
// k_describe's three per-lane tables in one constant block: one buffer
// resource (one s_getpc / add / addc) serves every table load at immediate offsets
struct DescTables {
    MomTables mom;   // 3072 B
    PatternQ pat;    // 1024 B
    RowTaps taps;    // 512 B
};
static_assert(offsetof(DescTables, pat) == 3072 && offsetof(DescTables, taps) == 4096, "immediate offsets below");
__constant__ __attribute__((aligned(16))) DescTables c_desc = DescTables();
typedef int i32x4 __attribute__((ext_vector_type(4)));

#ifndef ORBX_DESC_NOTAB
#define ORBX_DESC_NOTAB 0   // timing probe only (wrong descriptors): no pattern / moment table loads
#endif
#ifndef ORBX_DESC_STAGE
#define ORBX_DESC_STAGE 1   // 0: the generic wave_stage_rows
#endif
#ifndef ORBX_DESC_PKF32
#define ORBX_DESC_PKF32 1   // 0: the sample offsets as eight unpacked VOP2 f32 ops (fewer issue cycles, more instructions; time neutral, profiles/r06_ab_desc_f32.txt)
#endif
// k_describe's 43 x 43 patch inside the level, staged with its column 0 at
// patch column 2 (the keypoint at kDescKpCol = 23: the orientation disc in one
// 32-column MFMA window): a row is 12 dwords from x0 - 2, unaligned loads
// (the buffer base stays 4-aligned, the misalignment in the lane offset),
// so 5 rows a pass (lanes (rl, k), rl < 5) and 9 passes cover rows rl + 5 j;
// every row lane has j < 8, rows 40..42 (j = 8) only rl < 3.  One exec region
// for the nine loads and stores (the generic loop guards each with its own
// compare and exec save / restore: ~70 scalar instructions a wave), row
// offsets as scalar multiples of the pitch, LDS offsets as immediates.
// Stored XOR 0x80 (the int8 MFMAs' I - 128).  Needs x0 >= 2, x0 + 46 <= pitch.
constexpr int kDescCol0 = kDescKpCol - kDescR;   // 2: the patch column of the window's column 0
__device__ inline void stage_desc_patch(uint8_t *dst, const uint8_t *img, int pitch, int y0, int x0, int lane) {
    static_assert(kDescP == 43 && kDescPS == 48 && kDescCol0 == 2, "5 rows of 12 dwords a pass");
    pitch = __builtin_amdgcn_readfirstlane(pitch);
    const int xs = x0 - kDescCol0, xa = xs & ~3, sh = xs - xa;
    constexpr int nd = kDescPS / 4;
    const __amdgpu_buffer_rsrc_t src = wave_rsrc(img + (int64_t)y0 * pitch + xa);
    const int rl = lane / nd, k = lane - mul24u(rl, nd);
    const int voff = mul24u(rl, pitch) + 4 * k + sh;
    const int p5 = __builtin_amdgcn_readfirstlane(5 * pitch);
    typedef __attribute__((address_space(3))) uint32_t lds_u32;
    lds_u32 *d = (lds_u32 *)(dst + mul24u(rl, kDescPS) + 4 * k);
    if (rl < 5) {
        uint32_t v[9];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = buf_ld32(src, voff, j * p5);
        const bool last = rl < 3;
        if (last) v[8] = buf_ld32(src, voff, 8 * p5);
#pragma unroll
        for (int j = 0; j < 8; ++j) d[j * 5 * kDescPS / 4] = v[j] ^ 0x80808080u;
        if (last) d[8 * 5 * kDescPS / 4] = v[8] ^ 0x80808080u;
    }
}

template <bool PIPE>
__global__ __launch_bounds__(kThreads, ORBX_DESC_WAVES) void k_describe(DevPlan p, FrameBufs fb, int s0, int ns, int write_total,
                                                           uint32_t gmagic) {
    __shared__ __align__(16) uint8_t lds[4 * kDescWaveStride];
    __shared__ int s_mom[4][2];      // each wave's (m01, m10)
    __shared__ float s_ang[4][3];    // each wave's (angle, sin, cos), computed by wave 0
    PHASE_START();
    const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
    int bx, b;
    xcd_block_2d(bx, b, gmagic);
    const int slot = s0 + bx * 4 + wave;
    const bool in_range = slot < p.out_cap && bx * 4 + wave < ns;
    // level of this slot (plan table) and the selected key: scalar loads
    const int l = in_range ? (int)p.slot_level[slot] : 0;
    // (32-bit index: the plan bounds max_batch * out_cap below 2^31, orbx_runtime.hip)
    const uint32_t key = in_range ? __builtin_amdgcn_readfirstlane(fb.sel[(uint32_t)(b * p.out_cap + slot)]) : 0u;
    // the frame's level counts: lane q < nlevels holds count q; the slot's
    // output offset is the prefix below its level (16-lane DPP scan)
    const int32_t *lc = fb.level_count + (uint32_t)(b * kMaxLevels);
    const int lq = lane & (kMaxLevels - 1);
    const int lcv = lc[lq];   // (every lane: a frame holds kMaxLevels counts)
    // the tables after the level counts: the scan below waits for the
    // counts alone (vector loads complete in order), not for the tables
    // this lane's 4 pattern pairs (pairs 64 g + lane, g = 0..3, as fp8 bytes
    // x0 y0 x1 y1 in word g), fetched first so the load overlaps the staging;
    // one buffer resource over each table, the loads at immediate offsets (the
    // compiler otherwise rebuilds a symbol's address, s_getpc + add + addc, per load)
    const __amdgpu_buffer_rsrc_t tab_rsrc = wave_rsrc(&c_desc);
    const long row_taps = __builtin_bit_cast(long, __builtin_amdgcn_raw_buffer_load_b64(tab_rsrc, 8 * lane, 4096, 0));
    const uint4 patq = ORBX_DESC_NOTAB ? make_uint4(0x38u * lane, 0x40u, 0x48u, 0xC4u)
                                       : __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(tab_rsrc, 16 * lane, 3072, 0));
    // the moment products' operand tables (the same for every keypoint: the
    // patch is staged with the keypoint at a fixed column), ahead of the
    // key's chain of scalar loads and the staging, whose latency they hide under
    typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
    u64x2 mom[3];
    {
#pragma unroll
        for (int t = 0; t < 3; ++t)
            mom[t] = ORBX_DESC_NOTAB ? u64x2{0x00FFFF00FF00FFFFull * (uint64_t)(lane + t), 0x0102030405060708ull + t}
                                     : __builtin_bit_cast(u64x2, __builtin_amdgcn_raw_buffer_load_b128(tab_rsrc, 16 * lane + 1024 * t, 0, 0));
    }
    const int cq = lane < p.nlevels ? max(lcv, 0) : 0;
    static_assert(kMaxLevels == 16, "one DPP row");
    uint32_t scan = (uint32_t)cq;
    scan += dpp_or<kRowShr1>(0u, scan);
    scan += dpp_or<kRowShr2>(0u, scan);
    scan += dpp_or<kRowShr4>(0u, scan);
    scan += dpp_or<kRowShr8>(0u, scan);
    const int cl = __builtin_amdgcn_readlane(cq, l);
    const int off = __builtin_amdgcn_readlane((int)scan, l) - cl;
    if (write_total && bx == 0 && tid == 0) fb.nkps[b] = __builtin_amdgcn_readlane((int)scan, kMaxLevels - 1);
    // (no early exit: every wave reaches the block's two barriers)
    const LevelArgs g = p.la[l];
    const int i = slot - g.out_off;
    const bool valid = in_range && i < cl;
    const int x = (int)(key & 0xFFF), y = (int)((key >> 12) & 0xFFF), score = (int)(key >> 24);

    uint8_t *lbase = lds + wave * kDescWaveStride;
    uint16_t *rowp = reinterpret_cast<uint16_t *>(lbase + kDescRowOff);
    // taps of getGaussianKernel(7, 2) x256 (checked against the plan on the host)
    constexpr int k0 = kGaussTaps[0], k1 = kGaussTaps[1], k2 = kGaussTaps[2], k3 = kGaussTaps[3];
    // column-pass taps as u16 pairs for v_dot2_u32_u16 over rows (r, r+1), (r+2, r+3), (r+4, r+5), (r+6, r+7)
    constexpr u16x2 kK01 = {(unsigned short)k0, (unsigned short)k1}, kK23 = {(unsigned short)k2, (unsigned short)k3},
                    kK21 = {(unsigned short)k2, (unsigned short)k1}, kK0z = {(unsigned short)k0, 0};
    if (valid) {

    // 1. stage the 43x43 unblurred neighbourhood at patch columns 2..44: dword
    //    loads when it lies inside the level, else byte loads with reflect-101
    //    at the borders
    int spitch;
    const uint8_t *img = level_ptr(p, fb, l, b, spitch);
    const int px0 = x - kDescR, py0 = y - kDescR;
    // (every term >= 0 <=> their OR is: one scalar compare instead of five compare / select / and)
    const bool inside = ((px0 - kDescCol0) | py0 | (g.w - 1 - kDescR - x) | (g.h - 1 - kDescR - y) |
                         (spitch - (px0 - kDescCol0 + kDescPS))) >= 0;
    if (inside) {
        if constexpr (ORBX_DESC_STAGE) stage_desc_patch(lbase, img, spitch, py0, px0, lane);
        else wave_stage_rows<(kDescP + 4) / 5, true, true, kDescCol0>(lbase, kDescPS, img, spitch, py0, px0, kDescP, kDescP, lane);   // 5 rows a pass
    } else {
        // near a level border: lane = patch column (its reflect-101 column fixed),
        // the rows in turn (the row's reflection is wave-uniform); columns
        // outside the window are not needed (multiplied by zero taps or feeding
        // unread outputs) and stay as they are
        const int c = min(max(lane, kDescCol0), kDescCol0 + kDescP - 1);
        const int xx = reflect101(px0 - kDescCol0 + c, g.w);
        const int sp = __builtin_amdgcn_readfirstlane(spitch);
        const bool col = lane >= kDescCol0 && lane < kDescCol0 + kDescP;
#pragma unroll 11
        for (int r = 0; r < kDescP; ++r) {
            const int yy = reflect101(py0 + r, g.h);
            const uint8_t v = img[(int64_t)yy * sp + xx];
            if (col) lbase[r * kDescPS + lane] = v ^ 0x80;
        }
    }
    wave_lds_fence();
    PHASE_MARK(1, 0);   // prologue + staging

    if constexpr (kStopDesc == 0 || kStopDesc >= 2) {
    // 2. IC_Angle's moments (ORBextractor.cc:77-104) and the horizontal pass of
    //    the 7x7 Gaussian, both as int8 MFMAs on the same pixel tiles.  The patch
    //    was staged as I - 128 (XOR 0x80); the moments over the disc do not see
    //    that bias (sum u = sum v = 0 over the symmetric disc) and the row pass's
    //    accumulator starts at 128 * sum(w) to undo it.
    {
        const int rl = lane & 15, q = lane >> 4;
        const uint8_t *bsrc = lbase + rl * kDescPS + 8 * q;
        uint64_t px[3][3];
#pragma unroll
        for (int rt = 0; rt < 3; ++rt)
#pragma unroll
            for (int ct = 0; ct < 3; ++ct)
                px[rt][ct] = *reinterpret_cast<const uint64_t *>(bsrc + 16 * rt * kDescPS + 16 * ct);
        // moments: A = the disc's pixels of the window tiles (rows 16 rt..,
        // columns 8..39), B = c_desc.mom's b; D[i][15] = sum of u I over row i,
        // D[i][12 + rt] = sum of I over row 16 rt + i, summed over the three
        // products (lane l: D[4 (l >> 4) + ii][l & 15])
        {
            static_assert(kDescKpCol - 15 == 8, "the disc's columns start the 8-aligned window");
            i32x4 acc = {0, 0, 0, 0};
#pragma unroll
            for (int rt = 0; rt < 3; ++rt) {
                const uint64_t pw = *reinterpret_cast<const uint64_t *>(bsrc + 16 * rt * kDescPS + 8);
                acc = __builtin_amdgcn_mfma_i32_16x16x32_i8((long)(pw & mom[rt].x), (long)mom[rt].y, acc, 0, 0, 0);
            }
            // m10: lane 15 of each row, S; m01: lanes 12..14, v-weighted rows
            // (v = 16 (j - 12) + 4 (l >> 4) + ii - 21), folded into lane 15
            const int j = rl;
            const int S = acc[0] + acc[1] + acc[2] + acc[3];
            const int T = acc[1] + 2 * acc[2] + 3 * acc[3];
            const bool rows = j >= 12 && j <= 14;
            int y = rows ? __mul24(16 * (j - 12) + 4 * q - 21, S) + T : 0;
            int x = S;
            asm volatile(
                "s_nop 1\n\t"
                "v_add_u32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                "s_nop 1\n\t"
                "v_add_u32_dpp %0, %0, %0 row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                "s_nop 1\n\t"
                "v_add_u32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
                "v_add_u32_dpp %1, %1, %1 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
                "s_nop 1\n\t"
                "v_add_u32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf\n\t"
                "v_add_u32_dpp %1, %1, %1 row_bcast:31 row_mask:0xc bank_mask:0xf\n\t"
                "s_nop 1"
                : "+v"(y), "+v"(x));
            if (lane == 0) {
                s_mom[wave][0] = __builtin_amdgcn_readlane(y, 63);
                s_mom[wave][1] = __builtin_amdgcn_readlane(x, 63);
            }
        }
        PHASE_MARK(1, 1);   // moments
        // row pass: nine 16 x 16 output tiles (rows 16 rt.., patch columns
        // 16 ct..; window column = patch column - o), D = P T: A operand, lane
        // l holds P[16 rt + (l & 15)][16 ct + 8 (l >> 4) + 0..7] - 128 (one
        // ds_read_b64); B = the Toeplitz taps.  D's lane l holds rows
        // 16 rt + 4 (l >> 4) + 0..3 of output column 16 ct + (l & 15): one
        // 8-byte store into the column-major buffer.  Only columns < 40 and
        // rows < 44 are stored (row 43 is padding).
        const i32x4 bias = {128 * 257, 128 * 257, 128 * 257, 128 * 257};
        static_assert(kGaussTaps[0] + kGaussTaps[1] + kGaussTaps[2] + kGaussTaps[3] + kGaussTaps[4] +
                          kGaussTaps[5] + kGaussTaps[6] == 257, "bias = 128 * sum of the taps");
        // Every lane stores (no exec regions): the outputs outside the buffer
        // land where a later store of the same wave rewrites them (LDS stores
        // of a wave complete in order; compiler barriers keep that order):
        //  - rows 44..47 (rt = 2, q = 3) are rows 0..3 of the next column,
        //    rewritten by the rt = 0 tiles, stored last (the last column's
        //    go to the buffer's 8 spare bytes);
        //  - columns 40..47 (ct = 2, rl >= 8) are sent to columns 0..7 of the
        //    same rows, rewritten by the ct = 0 tile stored after it.
        static_assert(kRowCols == 40 && kColS == 44, "the spill targets above");
        uint16_t *dst = rowp + rl * kColS + 4 * q;
        uint16_t *dst2 = rowp + (rl < kRowCols - 32 ? rl + 32 : rl - 8) * kColS + 4 * q;   // tile ct = 2
        auto store = [&](int rt, int ct) {
            const i32x4 d = __builtin_amdgcn_mfma_i32_16x16x32_i8((long)px[rt][ct], row_taps, bias, 0, 0, 0);
            uint2 w;
            w.x = __builtin_amdgcn_perm((uint32_t)d[1], (uint32_t)d[0], 0x05040100u);   // (d0, d1) as u16 halves
            w.y = __builtin_amdgcn_perm((uint32_t)d[3], (uint32_t)d[2], 0x05040100u);
            *reinterpret_cast<uint2 *>((ct == 2 ? dst2 : dst + 16 * ct * kColS) + 16 * rt) = w;
            asm volatile("" ::: "memory");
        };
#pragma unroll
        for (int rt = 2; rt >= 0; --rt) {
            store(rt, 2);
            store(rt, 0);
            store(rt, 1);
        }
    }
    PHASE_MARK(1, 2);   // row pass
    }   // kStopDesc
    }   // valid
    // The orientation (fastAtan2) and its sincosf are wave-uniform scalar
    // chains of ~90 VALU each: wave 0 evaluates the block's four at once (lane
    // = wave), instead of every wave issuing the chain for one value.
    __syncthreads();
    if (wave == 0 && lane < 4) {
        const float a = fast_atan2_deg((float)s_mom[lane][0], (float)s_mom[lane][1]);
        float sa, ca;
        glibc_sincosf(__fmul_rn(a, (float)(3.14159265358979323846 / 180.f)), &sa, &ca);
        s_ang[lane][0] = a;
        s_ang[lane][1] = sa;
        s_ang[lane][2] = ca;
    }
    __syncthreads();
    if (!valid) return;
    const float angle = s_ang[wave][0], sa = s_ang[wave][1], ca = s_ang[wave][2];
    const int64_t kp_index = (int64_t)b * p.max_kps + off + i;
    // the keypoint record (the matchers downstream index their grids with it)
    auto write_record = [&]() {
        if (lane == 0) {
            orbx_keypoint kp;
            float fx = (float)x, fy = (float)y;
            if (l != 0) { fx = __fmul_rn(fx, g.scale); fy = __fmul_rn(fy, g.scale); }
            kp.x = fx;
            kp.y = fy;
            kp.size = g.patch_size;
            kp.angle = angle;
            kp.response = (float)score;
            kp.octave = l;
            kp.class_id = -1;
            fb.kps[kp_index] = kp;
        }
    };
    if constexpr (kStopDesc != 0 && kStopDesc < 4) {
        write_record();
        return;
    }

    // 4. computeOrbDescriptor (ORBextractor.cc:106-147) on the blurred level:
    //    each sample's blurred value is the column pass evaluated at that pixel
    //    from the row-pass buffer, with OpenCV 3.2's per-column rounding
    //    (half-even below w & ~3, else half-up).
    const int xs = g.w & ~3;
    // whole sample window left of w & ~3 (almost every keypoint): half-even
    // rounding everywhere, (s + 0x7FFF + bit16) >> 16, no per-column test
    const bool all_even = x + kBlurR < xs;
    // all 8 of the lane's samples: offsets, then every column-pass read in
    // flight at once, then the rounding
    // A sample at window offset (r, c) reads column c + kBlurR + kDescCol0, rows
    // r + kBlurR .. +6 of the column-major buffer: byte offset
    // 2 kColS (c + kBlurR + kDescCol0) + 2 (r + kBlurR), from the cvRound'ed float
    // bits (0x4B400000 + n, below) as one 24-bit multiply-add and one
    // shift-add; the constant folds the bias bits away (mod 2^32).  The read
    // is the four dwords from the one holding row r down (two ds_read2_b32;
    // unaligned ds_read_b128 measured 470 stall cycles a wave), and an odd
    // row's pairs are realigned by 16 bits (v_alignbit by a per-lane shift).
    const uint32_t kOff = (uint32_t)(kDescRowOff + 2 * kColS * (kBlurR + kDescCol0) + 2 * kBlurR) -
                          (uint32_t)(2 * kColS) * 0x400000u - 2u * 0x4B400000u;
    static_assert((kDescRowOff & 3) == 0 && (kColS & 1) == 0, "dword-aligned column starts");
    typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(4)));
    typedef __attribute__((address_space(3))) const u32x4a lds_u32x4a;
    // the LDS address of the wave's buffer folded into the constant: the
    // address is then one v_lshl_add and one v_mad_u32_u24 from the bits
    const uint32_t kOffL = __builtin_amdgcn_readfirstlane(kOff + (uint32_t)(uintptr_t)(const lds_u8 *)lbase);
    int sums[8], cbs[8];
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    // cvRound by the 1.5 * 2^23 bias: the float add rounds to the nearest
    // integer, ties to even, and the bits are then 0x4B400000 + n (|n| < 2^22)
    constexpr float kRndBias = 12582912.f;
#if ORBX_DESC_PKF32
    const f32x2 sc = {sa, ca}, rnd2 = {kRndBias, kRndBias};
#else
    // (wave-uniform, moved into VGPRs once: a VOP2 f32 op with an SGPR operand issues at half rate)
    float sav, cav, rndv;
    asm volatile("v_mov_b32 %0, %1" : "=v"(sav) : "v"(sa));
    asm volatile("v_mov_b32 %0, %1" : "=v"(cav) : "v"(ca));
    asm volatile("v_mov_b32 %0, %1" : "=v"(rndv) : "v"(kRndBias));
#endif
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint32_t pw = (k >> 1) == 0 ? patq.x : (k >> 1) == 1 ? patq.y : (k >> 1) == 2 ? patq.z : patq.w;
        // (rb, cb) side by side as packed f32 pairs (v_pk_mul / v_pk_add:
        // the same IEEE products and sums, two per instruction):
        //   rb = (px sa + py ca) + bias,  cb = (px ca - py sa) + bias
        // (written out: the compiler's own packing negates and moves pairs around)
        const f32x2 pxy = (k & 1) ? __builtin_amdgcn_cvt_pk_f32_fp8((int)pw, true)      // (x, y) of point k
                                  : __builtin_amdgcn_cvt_pk_f32_fp8((int)pw, false);
        f32x2 rc;
#if ORBX_DESC_PKF32
        f32x2 py2;
        asm("v_pk_mul_f32 %0, %2, %3 op_sel_hi:[0,1]\n\t"               // (px sa, px ca)
            "v_pk_mul_f32 %1, %2, %3 op_sel:[1,1] op_sel_hi:[1,0]\n\t"  // (py ca, py sa)
            "v_pk_add_f32 %0, %0, %1 neg_hi:[0,1]\n\t"                  // (px sa + py ca, px ca - py sa)
            "v_pk_add_f32 %0, %0, %4"                                   // + (bias, bias)
            : "=&v"(rc), "=&v"(py2)
            : "v"(pxy), "v"(sc), "s"(rnd2));
#else
        // the same eight IEEE steps as unpacked VOP2 f32 ops on VGPR operands
        // only (sa, ca and the bias held in VGPRs): ~2.2 cycles each where a
        // packed f32 op takes ~8.4 and an SGPR operand makes any op ~4.2
        {
            float t0, t1, t2, t3;
            asm("v_mul_f32 %0, %1, %2" : "=v"(t0) : "v"(pxy.x), "v"(sav));
            asm("v_mul_f32 %0, %1, %2" : "=v"(t1) : "v"(pxy.y), "v"(cav));
            asm("v_mul_f32 %0, %1, %2" : "=v"(t2) : "v"(pxy.x), "v"(cav));
            asm("v_mul_f32 %0, %1, %2" : "=v"(t3) : "v"(pxy.y), "v"(sav));
            asm("v_add_f32 %0, %1, %2" : "=v"(t0) : "v"(t0), "v"(t1));
            asm("v_sub_f32 %0, %1, %2" : "=v"(t2) : "v"(t2), "v"(t3));
            asm("v_add_f32 %0, %1, %2" : "=v"(rc.x) : "v"(t0), "v"(rndv));
            asm("v_add_f32 %0, %1, %2" : "=v"(rc.y) : "v"(t2), "v"(rndv));
        }
#endif
        const uint32_t rb = __float_as_uint(rc.x), cb = __float_as_uint(rc.y);
        cbs[k] = (int)cb;
        // (__umul24 reads the low 24 bits of cb: 0x400000 + c, c in [-18, 18])
        uint32_t t, off;
        asm("v_lshl_add_u32 %0, %1, 1, %2" : "=v"(t) : "v"(rb), "s"(kOffL));
        asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(off) : "v"(cb), "s"(2u * kColS), "v"(t));
        const u32x4a v = *reinterpret_cast<lds_u32x4a *>((uintptr_t)(off & ~3u));
        // odd row (the low bit of rb): shift 16; v_alignbit reads its shift's low 5 bits
        const uint32_t sh = rb << 4;
        // k0 R0 + k1 R1 + k2 R2 + k3 R3 + k2 R4 + k1 R5 + k0 R6 as four u16-pair dot products
        const uint32_t e0 = __builtin_amdgcn_alignbit(v.y, v.x, sh), e1 = __builtin_amdgcn_alignbit(v.z, v.y, sh),
                       e2 = __builtin_amdgcn_alignbit(v.w, v.z, sh), e3 = __builtin_amdgcn_alignbit(v.w, v.w, sh);
        sums[k] = (int)__builtin_amdgcn_udot2(
            as_u16x2(e0), kK01,
            __builtin_amdgcn_udot2(as_u16x2(e1), kK23,
                                   __builtin_amdgcn_udot2(as_u16x2(e2), kK21,
                                                          __builtin_amdgcn_udot2(as_u16x2(e3), kK0z, 0u, false),
                                                          false),
                                   false),
            false);
    }
    PHASE_MARK(1, 3);   // sincos + sample offsets + column pass
    if constexpr (kStopDesc == 4) {   // keep the column pass: its sums reach LDS
        int acc = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) acc ^= sums[k] + cbs[k];
        if (acc == 0x7FFFFFFF) lbase[0] = 1;
        write_record();
        return;
    }
    int val[8];
    if (all_even) {
#pragma unroll
        for (int k = 0; k < 8; ++k) val[k] = min((sums[k] + 0x7FFF + ((sums[k] >> 16) & 1)) >> 16, 255);
    } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int sum = sums[k];
            int qv;
            if (x + (cbs[k] - 0x4B400000) < xs) {
                qv = sum >> 16;
                const int rem = sum & 0xFFFF;
                qv += (rem > 0x8000) | ((rem == 0x8000) & (qv & 1));
            } else {
                qv = (sum + (1 << 15)) >> 16;
            }
            val[k] = min(qv, 255);
        }
    }
    uint64_t m[4];
#pragma unroll
    for (int grp = 0; grp < 4; ++grp) m[grp] = lanes_lt(val[2 * grp], val[2 * grp + 1]);
    if (lane == 0) {
        ulonglong2 *dout = reinterpret_cast<ulonglong2 *>(fb.desc + kp_index * 32);
        dout[0] = make_ulonglong2(m[0], m[1]);
        dout[1] = make_ulonglong2(m[2], m[3]);
    }
    write_record();
    PHASE_MARK(1, 4);   // rounding + ballots + records
}

__global__ void k_trig(const float *in, float *so, float *co, int n, const float *ay, const float *ax,
                       float *at, int m) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) glibc_sincosf(in[i], &so[i], &co[i]);
    if (i < m) at[i] = fast_atan2_deg(ay[i], ax[i]);
}

}  // namespace

// ---------------------------------------------------------------------------
hipError_t launch_resize_level(const DevPlan &p, const Plan &hp, const FrameBufs &fb, int B, hipStream_t st, int l) {
    if (!hp.rw.empty()) {
        const ResizeWave &a = hp.rw[l];
        const int waves = a.ntiles * B;
        if (a.direct) {
            hipLaunchKernelGGL(k_resize_d, dim3((waves + 3) / 4), dim3(kThreads), 0, st, p, fb, l, a, B);
            return hipGetLastError();
        }
        // one global round trip for the whole window: NB >= the staging's row passes
        if (a.stage_passes <= 9)
            hipLaunchKernelGGL(k_resize_w<9>, dim3((waves + 3) / 4), dim3(kThreads), 4 * a.win_bytes, st, p, fb, l, a, B);
        else if (a.stage_passes <= 16)
            hipLaunchKernelGGL(k_resize_w<16>, dim3((waves + 3) / 4), dim3(kThreads), 4 * a.win_bytes, st, p, fb, l, a, B);
        else
            hipLaunchKernelGGL(k_resize_w<24>, dim3((waves + 3) / 4), dim3(kThreads), 4 * a.win_bytes, st, p, fb, l, a, B);
        return hipGetLastError();
    }
    const LevelGeom &g = hp.lv[l];
    dim3 grid((g.w + kResTW - 1) / kResTW, (g.h + kResTH - 1) / kResTH, B);
    hipLaunchKernelGGL(k_resize, grid, dim3(kThreads), 0, st, p, fb, l);
    return hipGetLastError();
}

hipError_t launch_resize(const DevPlan &p, const Plan &hp, const FrameBufs &fb, int B, hipStream_t st) {
    if (use_pyr_regions(hp, B)) {
        static bool lds_set = false;   // (one attribute per process; the size bound is the plan check's)
        if (!lds_set) {
            if (hipFuncSetAttribute(reinterpret_cast<const void *>(k_pyramid_rgn),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess)
                return hipErrorInvalidValue;
            lds_set = true;
        }
        hipLaunchKernelGGL(k_pyramid_rgn, dim3(hp.rgn_n, B), dim3(kRgnThreads), 2 * hp.rgn_half + rgn_tap_bytes(hp.nlevels), st,
                           p, fb);
        return hipGetLastError();
    }
    for (int l = 1; l < hp.nlevels; ++l)
        if (launch_resize_level(p, hp, fb, B, st, l) != hipSuccess) return hipErrorLaunchFailure;
    return hipSuccess;
}

hipError_t launch_blur(const DevPlan &p, const FrameBufs &fb, int B, hipStream_t st) {
    hipLaunchKernelGGL(k_blur, dim3(p.nblur_tiles, B), dim3(kThreads), 0, st, p, fb);
    return hipGetLastError();
}

namespace {
// Magic for xcd_block_2d(bx, by, magic): ceil(2^32 / gx), exact for every
// block index L with L * gx < 2^32; 0 (divide) when that does not hold.
uint32_t grid_magic(uint32_t gx, uint32_t gy) {
    if (gx <= 1 || (uint64_t)gx * gy * gx >= (1ull << 32)) return 0;
    return (uint32_t)(((1ull << 32) + gx - 1) / gx);
}
}  // namespace

#ifndef ORBX_FAST_LIST_CAP
#define ORBX_FAST_LIST_CAP 640   // (survivor-list entries, at least what a compass step needs)
#endif
FastLds fast_lds(int mw, int mh) {
    FastLds f;
    // survivor-list capacity: every pixel of the largest cell, or 640.  It
    // must hold a row of waiting corners plus what one compass step can add,
    // R rows of cw pixels (k_fast flushes before a step could overflow it):
    // R = 64 / the lane groups of a row, (quads + 1) / 2 for the aligned
    // staging's (cw + 3) / 4 quads (the unaligned fallback has more groups,
    // fewer rows); 527 at VGA.  (Sized to that, 528, the launch fits 9
    // workgroups per CU instead of 8 and measured slower: 2.61 -> 2.70 ms;
    // 7 and 6 workgroups 2.71 and 2.88, profiles/r05_ab_fast_occupancy.txt.)
    int need = 0;
    for (int cw = 1; cw <= mw; ++cw) {
        const int nq = (cw + 3) >> 2, np = (nq + 1) >> 1, R = 64 / np;
        need = std::max(need, (R + 1) * cw);
    }
    f.list_cap = std::min(mw * mh, std::max(ORBX_FAST_LIST_CAP, (need + 7) & ~7));
    f.ps = (mw + 6 + 3 + 3) & ~3;   // + alignment offset, dword rows
    // the compass's last lane group reads up to column 4 + 8 ceil(mw / 8) + 3
    // (interior column 0 at patch column 4, ORBX_FAST_ALIGN)
    f.ps = std::max(f.ps, 8 * ((mw + 7) / 8) + 8);
    if (f.ps <= 64) f.ps = f.ps <= 48 ? 48 : 64;   // k_fast's constant-stride instantiations
    // the score map at the patch's stride: a survivor's list entry, its patch
    // offset ey * ps + ex from interior pixel (0, 0), also indexes the map
    // (cells are under 60 px a side, ORBextractor.cc:796-817: offsets < 2^13)
    f.sw = f.ps;
    f.pmag = (int)(((1u << 24) + f.ps - 1) / f.ps);
    f.patch_bytes = (f.ps * (mh + 6) + 15) & ~15;
    f.score_bytes = (f.sw * (mh + 2) + 15) & ~15;
    f.per_wave = f.patch_bytes + f.score_bytes + ((2 * f.list_cap + 15) & ~15);
    return f;
}

namespace {
// The levels [l0, l1)'s cells with LDS sized by their largest cell.
template <bool PIPE>
hipError_t launch_fast_range(const DevPlan &p, const Plan &hp, const FrameBufs &fb, int B, hipStream_t st, int l0,
                             int l1) {
    const int c0 = hp.lv[l0].cell_begin, nc = hp.lv[l1 - 1].cell_end - c0;
    if (nc <= 0) return hipSuccess;
    int mw = 1, mh = 1;
    for (int c = c0; c < c0 + nc; ++c) {
        mw = std::max(mw, hp.cells[c].x1 - hp.cells[c].x0);
        mh = std::max(mh, hp.cells[c].y1 - hp.cells[c].y0);
    }
    const FastLds fl = fast_lds(mw, mh);
    const dim3 grid((nc + 3) / 4, B);
    const uint32_t gm = grid_magic(grid.x, grid.y);
    if (fl.ps == 48 && fl.sw == 48)
        hipLaunchKernelGGL((k_fast<PIPE, 48>), grid, dim3(kThreads), 4 * fl.per_wave, st, p, fb, c0, nc, fl, gm);
    else if (fl.ps == 64 && fl.sw == 64)
        hipLaunchKernelGGL((k_fast<PIPE, 64>), grid, dim3(kThreads), 4 * fl.per_wave, st, p, fb, c0, nc, fl, gm);
    else
        hipLaunchKernelGGL((k_fast<PIPE, 0>), grid, dim3(kThreads), 4 * fl.per_wave, st, p, fb, c0, nc, fl, gm);
    return hipGetLastError();
}

}  // namespace

// All cells of all levels in one launch (one dispatch per stage keeps the
// per-launch roofline figure clean; splitting by cell size measured +1 %).
hipError_t launch_fast(const DevPlan &p, const Plan &hp, const FrameBufs &fb, int B, hipStream_t st) {
    return launch_fast_range<false>(p, hp, fb, B, st, 0, hp.nlevels);
}

hipError_t launch_fast_level(const DevPlan &p, const Plan &hp, const FrameBufs &fb, int B, hipStream_t st, int l,
                             int l_end) {
    return launch_fast_range<true>(p, hp, fb, B, st, l, l_end);
}

// Dynamic LDS above 64 KiB must be opted into per kernel.
template <typename K>
hipError_t allow_lds(K kernel, int bytes) {
    if (bytes <= 64 * 1024) return hipSuccess;
    return hipFuncSetAttribute(reinterpret_cast<const void *>(kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

// Workgroup size of k_quadtree for a launch of `blocks` (level, frame)
// blocks: 1024 threads when the launch is too small to fill the chip with
// 256-thread workgroups (a few frames: the drop-in call, a sharded camera
// set); 512 for images of more than 0.6 MP (HD, FHD: thousands of keys on
// every level, up to 20 per thread in registers, two workgroups per CU);
// else 256 (VGA: <= 8 register keys per thread, 7 workgroups per CU).
// ORBX_QT_NT=256 / 512 / 1024 forces one (where its LDS fits); ORBX_QT_WIDE=0
// never takes 1024, =1 always (read per launch: tests switch them per extractor).
int quadtree_nt(const DevPlan &p, int blocks) {
    const bool wide_fits = p.node_lds_bytes_w <= 160 * 1024;
    if (const char *e = std::getenv("ORBX_QT_NT")) {
        const int nt = std::atoi(e);
        if ((nt == 512 || nt == 1024) && wide_fits) return nt;
        if (nt == 256) return 256;
    }
    const char *w = std::getenv("ORBX_QT_WIDE");
    const int mode = w ? std::atoi(w) : -1;
    if (!wide_fits) return 256;
    if (mode == 1 || (mode != 0 && blocks <= 256)) return 1024;
    return (int64_t)p.lv[0].w * p.lv[0].h > 600 * 1000 ? 512 : 256;
}

template <bool PIPE>
hipError_t launch_quadtree_range(const DevPlan &p, const FrameBufs &fb, int B, hipStream_t st, int l, int l_end) {
    const dim3 grid = kQtLevelMajor ? dim3(B, l_end - l) : dim3(l_end - l, B);
    switch (quadtree_nt(p, (l_end - l) * B)) {
        case 1024:
            if (allow_lds(k_quadtree<PIPE, 1024>, p.node_lds_bytes_w) != hipSuccess) return hipErrorInvalidValue;
            hipLaunchKernelGGL((k_quadtree<PIPE, 1024>), grid, dim3(1024), p.node_lds_bytes_w, st, p, fb, l);
            break;
        case 512:
            if (allow_lds(k_quadtree<PIPE, 512>, p.node_lds_bytes_w) != hipSuccess) return hipErrorInvalidValue;
            hipLaunchKernelGGL((k_quadtree<PIPE, 512>), grid, dim3(512), p.node_lds_bytes_w, st, p, fb, l);
            break;
        default:
            if (allow_lds(k_quadtree<PIPE, kThreads>, p.node_lds_bytes) != hipSuccess) return hipErrorInvalidValue;
            hipLaunchKernelGGL((k_quadtree<PIPE, kThreads>), grid, dim3(kThreads), p.node_lds_bytes, st, p, fb, l);
    }
    return hipGetLastError();
}

hipError_t launch_quadtree(const DevPlan &p, const FrameBufs &fb, int B, hipStream_t st) {
    return launch_quadtree_range<false>(p, fb, B, st, 0, p.nlevels);
}

hipError_t launch_quadtree_level(const DevPlan &p, const FrameBufs &fb, int B, hipStream_t st, int l, int l_end) {
    return launch_quadtree_range<true>(p, fb, B, st, l, l_end);
}

hipError_t launch_describe(const DevPlan &p, const FrameBufs &fb, int B, hipStream_t st) {
    const uint32_t gx = (p.out_cap + 3) / 4;
    hipLaunchKernelGGL(k_describe<false>, dim3(gx, B), dim3(kThreads), 0, st, p, fb, 0, p.out_cap, 1,
                       grid_magic(gx, B));
    return hipGetLastError();
}

// Levels [l, l_end)'s keypoints; the launch with the last level also writes each
// frame's keypoint total (every level's count is final by then).
hipError_t launch_describe_level(const DevPlan &p, const Plan &hp, const FrameBufs &fb, int B, hipStream_t st, int l,
                                 int l_end) {
    const int s0 = hp.lv[l].out_off, ns = hp.lv[l_end - 1].out_off + hp.lv[l_end - 1].out_cap - s0;
    const uint32_t gx = (ns + 3) / 4;
    hipLaunchKernelGGL(k_describe<true>, dim3(gx, B), dim3(kThreads), 0, st, p, fb, s0, ns,
                       l_end == hp.nlevels ? 1 : 0, grid_magic(gx, B));
    return hipGetLastError();
}

hipError_t launch_trig_check(const float *in, float *s, float *c, float *atan_out, const float *ay,
                             const float *ax, int n, int m, hipStream_t st) {
    const int total = n > m ? n : m;
    if (total <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_trig, dim3((total + 255) / 256), dim3(256), 0, st, in, s, c, n, ay, ax, atan_out, m);
    return hipGetLastError();
}

// Region pyramid plan (k_pyramid_rgn): level 1 cut into ~96 x 96 owned
// rectangles, every level cut at the same fractions; each region's computed
// rectangles grow from the coarsest level down by what the next level reads.
// False (rgn_n = 0) when a region's level buffers exceed the LDS.
bool plan_pyr_regions(Plan &hp) {
    hp.rgn.clear();
    hp.rgn_n = 0;
    hp.rgn_half = 0;
    const int n = hp.nlevels;
    if (n < 2 || n > kMaxLevels) return false;
    const int gx = std::max(1, (hp.lv[1].w + 95) / 96), gy = std::max(1, (hp.lv[1].h + 95) / 96);
    // the source rectangle of level-l output rectangle q (as k_resize reads it)
    auto src_of = [&](int l, const RgnRect &q) {
        const LevelGeom &g = hp.lv[l], &gs = hp.lv[l - 1];
        const ResizeTap *xt = hp.xtaps.data() + g.xtab_off;
        const ResizeTap *yt = hp.ytaps.data() + g.ytab_off;
        RgnRect s{INT_MAX, INT_MAX, -1, -1};
        for (int x = q.x0; x <= q.x1; ++x) {
            s.x0 = std::min(s.x0, (int)xt[x].src);
            s.x1 = std::max(s.x1, std::min((int)xt[x].src + 1, gs.w - 1));
        }
        for (int y = q.y0; y <= q.y1; ++y) {
            s.y0 = std::min(s.y0, std::min(std::max((int)yt[y].src, 0), gs.h - 1));
            s.y1 = std::max(s.y1, std::min(std::max((int)yt[y].src + 1, 0), gs.h - 1));
        }
        return s;
    };
    auto unite = [](const RgnRect &a, const RgnRect &b) {
        return RgnRect{std::min(a.x0, b.x0), std::min(a.y0, b.y0), std::max(a.x1, b.x1), std::max(a.y1, b.y1)};
    };
    std::vector<RgnRect> out((size_t)gx * gy * 2 * kMaxLevels, RgnRect{0, 0, -1, -1});
    size_t half = 0;
    for (int ry = 0; ry < gy; ++ry)
        for (int rx = 0; rx < gx; ++rx) {
            RgnRect *T = out.data() + ((size_t)ry * gx + rx) * 2 * kMaxLevels;
            for (int l = 1; l < n; ++l) {
                const LevelGeom &g = hp.lv[l];
                T[kMaxLevels + l] = RgnRect{(int)((int64_t)rx * g.w / gx), (int)((int64_t)ry * g.h / gy),
                                            (int)((int64_t)(rx + 1) * g.w / gx) - 1,
                                            (int)((int64_t)(ry + 1) * g.h / gy) - 1};
                const RgnRect &o = T[kMaxLevels + l];
                if (o.x1 < o.x0 || o.y1 < o.y0) return false;   // a level narrower than the cut
            }
            T[n - 1] = T[kMaxLevels + n - 1];
            for (int l = n - 2; l >= 1; --l) T[l] = unite(T[kMaxLevels + l], src_of(l + 1, T[l + 1]));
            T[0] = src_of(1, T[1]);
            for (int l = 0; l < n; ++l) {
                const RgnRect &q = T[l];
                if (l > 0 && (q.x1 - q.x0 + 1 > 64 * kRgnCols || q.y1 - q.y0 + 1 > kRgnTapRows)) return false;
                const size_t stride = l == 0 ? 4 * (size_t)(((q.x1 - (q.x0 & ~3)) >> 2) + 1) + 4
                                             : (size_t)((q.x1 - q.x0 + 1 + 4 + 3) & ~3);
                half = std::max(half, stride * (q.y1 - q.y0 + 1));
            }
        }
    half = (half + 15) & ~size_t(15);
    if (2 * half + rgn_tap_bytes(n) > 160 * 1024) return false;
    hp.rgn = std::move(out);
    hp.rgn_n = gx * gy;
    hp.rgn_half = (int)half;
    return true;
}

// The region pyramid while one block per region and frame still leaves the
// chip short of a block per CU.
#ifndef ORBX_RGN_MAX
#define ORBX_RGN_MAX 256   // (region blocks a launch may take before the per-level kernels win)
#endif
bool use_pyr_regions(const Plan &hp, int B) { return hp.rgn_n > 0 && (int64_t)B * hp.rgn_n <= ORBX_RGN_MAX; }

// Wave-tile geometry of every level (ResizeWave).  False when some level does
// not fit the wave kernel (a column group spanning more than 7 source bytes,
// i.e. scale factors above ~2.3, or a window over the LDS budget); the block
// kernel k_resize then runs instead.
bool plan_resize_waves(Plan &hp) {
    hp.rw.assign(hp.nlevels, ResizeWave{});
    for (int l = 1; l < hp.nlevels; ++l) {
        bool direct = ORBX_RS_DIRECT && hp.lv[l - 1].w >= 8 && !std::getenv("ORBX_RESIZE_LDS");   // =1: windows in LDS
        if (l == 1) {
            hp.rcols.clear();
            hp.rrows.assign(hp.ytaps.size(), ResizeRow{});
        }
        const LevelGeom &g = hp.lv[l], &gs = hp.lv[l - 1];
        const ResizeTap *xt = hp.xtaps.data() + g.xtab_off;
        const ResizeTap *yt = hp.ytaps.data() + g.ytab_off;
        ResizeWave a;
        a.xtab_off = g.xtab_off;
        a.ytab_off = g.ytab_off;
        a.sx = 1. / ((double)g.w / gs.w);
        a.sy = 1. / ((double)g.h / gs.h);
        int best = -1;
        for (int sh = 6; sh >= 4; --sh) {
            const int cols = 4 << sh, n = (g.w + cols - 1) / cols;
            if (best < 0 || n * cols < best) { best = n * cols; a.twg_shift = sh; }
        }
        if (const char *e = std::getenv("ORBX_RS_TWG")) {   // (A/B probe: one column-group width for every level)
            const int t = std::atoi(e);
            if (t == 16 || t == 32 || t == 64) a.twg_shift = t == 16 ? 4 : t == 32 ? 5 : 6;
        }
        a.twg = 1 << a.twg_shift;
        const int TW = 4 * a.twg, TH = (64 >> a.twg_shift) * kResizeK;
        a.ntx = (g.w + TW - 1) / TW;
        const int nty = (g.h + TH - 1) / TH;
        a.ntiles = a.ntx * nty;
        int nd_max = 0, nd_win = 0;
        a.col_off = (int)hp.rcols.size();   // one ResizeCol per 4 columns, x / 4
        for (int tx = 0; tx < a.ntx; ++tx) {
            const int x0 = tx * TW, xl = std::min(x0 + TW, g.w) - 1;
            const int c_lo = std::min(std::max(resize_src_raw(x0, a.sx), 0), gs.w - 1);
            const int c_hi = std::min(std::max(resize_src_raw(xl, a.sx), 0) + 1, gs.w - 1);
            // the kernel's arithmetic bounds must be the tables' (and cover them)
            if (c_lo != xt[x0].src || c_hi < std::min((int)xt[xl].src + 1, gs.w - 1)) return false;
            nd_win = std::max(nd_win, ((c_lo & 3) + c_hi - c_lo + 1 + 3) >> 2);
            nd_max = std::max(nd_max, nd_win);
            for (int xb = x0; xb <= xl; xb += 4) {
                const int s0 = xt[xb].src, s3 = xt[std::min(xb + 3, g.w - 1)].src;
                if (s3 - s0 + 1 > 7) return false;   // pair bytes within the 8 realigned ones
                nd_max = std::max(nd_max, ((s0 - (c_lo & ~3)) >> 2) + 3);
                // k_resize_d: the 8 bytes from cs = min(s0, w_src - 8) hold every
                // pair byte whose coefficient is not 0 (resize_tile_direct)
                const int cs = std::min(s0, gs.w - 8);
                ResizeCol rc{};
                rc.c = cs & ~3;
                rc.o = cs & 3;
                for (int k = 0; k < 4; ++k) {
                    const ResizeTap &t = xt[std::min(xb + k, g.w - 1)];
                    const int r = t.src - cs;
                    if (r < 0 || r > 7 || (r == 7 && t.a1 != 0)) direct = false;
                    rc.sel[k] = (uint32_t)(r & 7) | 0x0C00u | ((uint32_t)(r < 7 ? r + 1 : 0x0C) << 16) | 0x0C000000u;
                    rc.coef[k] = (uint32_t)(uint16_t)t.a0 | ((uint32_t)(uint16_t)t.a1 << 16);
                    rc.smask |= (t.mode & 2) ? 1 << k : 0;
                }
                hp.rcols.push_back(rc);
            }
        }
        for (int y = 0; y < g.h; ++y) {
            ResizeRow &rr = hp.rrows[g.ytab_off + y];
            rr.s01 = (uint32_t)std::min(std::max((int)yt[y].src, 0), gs.h - 1) |
                     (uint32_t)std::min(std::max((int)yt[y].src + 1, 0), gs.h - 1) << 16;
            rr.b01 = ((uint32_t)yt[y].a0 & 0xFFFu) | ((uint32_t)yt[y].a1 & 0xFFFu) << 16;
        }
        int nr_max = 0;
        for (int ty = 0; ty < nty; ++ty) {
            const int y0 = ty * TH, yl = std::min(y0 + TH, g.h) - 1;
            const int r_lo = std::min(std::max(resize_src_raw(y0, a.sy), 0), gs.h - 1);
            const int r_hi = std::min(std::max(resize_src_raw(yl, a.sy) + 1, 0), gs.h - 1);
            for (int y = y0; y <= yl; ++y) {
                const int s0 = std::min(std::max((int)yt[y].src, 0), gs.h - 1);
                const int s1 = std::min(std::max((int)yt[y].src + 1, 0), gs.h - 1);
                if (s0 < r_lo || s1 > r_hi) return false;
            }
            nr_max = std::max(nr_max, r_hi - r_lo + 1);
        }
        a.win_stride = 4 * nd_max;
        a.win_dwords = nr_max * nd_win;
        a.stage_passes = nd_win <= 64 ? (nr_max + 64 / nd_win - 1) / (64 / nd_win) : nr_max;
        a.win_bytes = (nr_max * a.win_stride + 15) & ~15;
        if (4 * a.win_bytes > 64 * 1024) return false;
        a.direct = direct;
        hp.rw[l] = a;
    }
    return true;
}

bool resize_window_fits(const Plan &hp) {
    for (int l = 1; l < hp.nlevels; ++l) {
        const LevelGeom &g = hp.lv[l];
        for (int x0 = 0; x0 < g.w; x0 += kResTW) {
            const int xl = std::min(x0 + kResTW, g.w) - 1;
            if (hp.xtaps[g.xtab_off + xl].src + 8 - hp.xtaps[g.xtab_off + x0].src > kResCols) return false;
        }
        for (int y0 = 0; y0 < g.h; y0 += kResTH) {
            const int yl = std::min(y0 + kResTH, g.h) - 1;
            if (hp.ytaps[g.ytab_off + yl].src + 2 - hp.ytaps[g.ytab_off + y0].src > kResRows) return false;
        }
    }
    return true;
}

#ifdef ORBX_PHASE_PROF
extern "C" int orbx_debug_phase_cycles(unsigned long long *out, int cap, int reset) {
    static unsigned long long h[24 * 256];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_phase), sizeof(h)) != hipSuccess) return -5;
    for (int i = 0; i < 24 && i < cap; ++i) {
        unsigned long long t = 0;
        for (int j = 0; j < 256; ++j) t += h[256 * i + j];
        out[i] = t;
    }
    if (reset) {
        static unsigned long long z[24 * 256];
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_phase), z, sizeof(z)) != hipSuccess) return -5;
    }
    return 24;
}
#endif

int quadtree_lds_bytes(int node_cap) {
    int np2 = 1;
    while (np2 < node_cap) np2 <<= 1;
    return (int)(2 * sizeof(uint64_t) * np2 + 2 * sizeof(QNode) * node_cap +
                 2 * sizeof(uint32_t) * 4 * node_cap + sizeof(int16_t) * 5 * node_cap + node_cap + 64);
}

}  // namespace orbx
