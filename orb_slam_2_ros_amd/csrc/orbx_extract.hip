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
// All of this is integer / byte work bound by HBM or by latency; no MFMA.
#include <hip/hip_runtime.h>

#include "orbx_device.h"
#include "orbx_math.h"

namespace orbx {

__constant__ int8_t c_pattern[512][2] = {
#define ORBX_PATTERN_BEGIN
#define ORBX_PATTERN_END
#include "orb_pattern.inc"
#undef ORBX_PATTERN_BEGIN
#undef ORBX_PATTERN_END
};

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

__device__ inline int reflect101(int v, int n) {
    // BORDER_REFLECT_101 for the 3-px halo of a >= 4 px image.
    v = v < 0 ? -v : v;
    return v >= n ? 2 * n - v - 2 : v;
}

__device__ inline uint32_t pack_key(int x, int y, int score) {
    return (uint32_t)x | ((uint32_t)y << 12) | ((uint32_t)score << 24);
}

// ---- wave / block helpers (wave64) ----------------------------------------
__device__ inline uint64_t shfl_up_u64(uint64_t v, int d) {
    const int lo = __shfl_up((int)(uint32_t)v, d, 64);
    const int hi = __shfl_up((int)(uint32_t)(v >> 32), d, 64);
    return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}

__device__ inline uint64_t wave_incl_scan_u64(uint64_t v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t o = shfl_up_u64(v, d);
        if (lane >= d) v += o;
    }
    return v;
}

__device__ inline int wave_sum_i32(int v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

// Exclusive scan of a[0..m) (uint64) in LDS by the whole 256-thread block.
// ws: 4 uint64 of LDS scratch.  Returns the total.  Ends with a barrier.
__device__ uint64_t block_excl_scan_u64(uint64_t *a, int m, uint64_t *ws) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int per = (m + kThreads - 1) / kThreads;
    const int s = min(tid * per, m), e = min(s + per, m);
    uint64_t local = 0;
    for (int i = s; i < e; ++i) local += a[i];
    const uint64_t incl = wave_incl_scan_u64(local);
    if (lane == 63) ws[wave] = incl;
    __syncthreads();
    uint64_t base = 0, total = 0;
    for (int w = 0; w < kThreads / 64; ++w) {
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
    int incl = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int o = __shfl_up(incl, d, 64);
        if (lane >= d) incl += o;
    }
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

// ===========================================================================
// K1: bilinear level l from level l-1 (cv::resize INTER_LINEAR 8U, OpenCV 3.2
// fixed point; SSE2 vertical rounding on the leading columns, scalar tail).
// Thread = 4 consecutive output pixels; block = 256 x 4 pixels.
// ===========================================================================
__global__ __launch_bounds__(kThreads) void k_resize(DevPlan p, FrameBufs fb, int l) {
    const LevelGeom g = p.lv[l];
    const LevelGeom gs = p.lv[l - 1];
    const int b = blockIdx.z;
    const int x4 = (blockIdx.x * 64 + (threadIdx.x & 63)) * 4;
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (y >= g.h || x4 >= g.w) return;
    int spitch;
    const uint8_t *src = level_ptr(p, fb, gs, l - 1, b, spitch);
    uint8_t *dst = fb.pyr + (int64_t)b * p.pyr_bytes + g.pyr_off;
    const ResizeTap ty = p.ytaps[g.ytab_off + y];
    const int r0 = min(max((int)ty.src, 0), gs.h - 1);
    const int r1 = min(max((int)ty.src + 1, 0), gs.h - 1);
    const uint8_t *S0 = src + (int64_t)r0 * spitch;
    const uint8_t *S1 = src + (int64_t)r1 * spitch;
    const int b0 = ty.a0, b1 = ty.a1;
    uint32_t packed = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int x = x4 + k;
        if (x >= g.w) break;
        const ResizeTap tx = p.xtaps[g.xtab_off + x];
        int h0, h1;
        if (tx.mode & 1) {
            h0 = S0[tx.src] * tx.a0 + S0[tx.src + 1] * tx.a1;
            h1 = S1[tx.src] * tx.a0 + S1[tx.src + 1] * tx.a1;
        } else {
            h0 = S0[tx.src] * 2048;
            h1 = S1[tx.src] * 2048;
        }
        int v;
        if (tx.mode & 2) {
            // _mm_packs_epi32(h>>4) ; _mm_mulhi_epi16 ; _mm_adds_epi16 ; +2 ; >>2 ; packus
            v = ((((h0 >> 4) * b0) >> 16) + (((h1 >> 4) * b1) >> 16) + 2) >> 2;
        } else {
            v = (h0 * b0 + h1 * b1 + (1 << 21)) >> 22;
        }
        v = min(max(v, 0), 255);
        packed |= (uint32_t)v << (8 * k);
    }
    *reinterpret_cast<uint32_t *>(dst + (int64_t)y * g.pitch + x4) = packed;
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
// K3: per-cell FAST-9 with the reference's cell semantics.  For each interior
// pixel the arc score S = max over the 16 nine-pixel arcs of
// max(min(v - p), min(p - v)); the pixel is a corner at threshold t iff S > t
// and cv::FAST's cornerScore is S - 1.  NMS is the strict 3x3 test inside the
// cell (outside neighbours count 0, as FAST on the cell sub-image sees them).
// If no keypoint survives at iniThFAST the cell is redone at minThFAST.
// Output: the cell's keypoints in row-major order, packed (x | y<<12 | s<<24).
// ===========================================================================
constexpr int kCellMax = 64;                 // wCell/hCell < 60 by construction
constexpr int kPatchW = kCellMax + 6;
constexpr int kScoreW = kCellMax + 2;

__device__ inline int arc_score(const uint8_t *c, int stride) {
    const int v = c[0];
    int d[16];
    d[0] = v - c[3 * stride];      d[1] = v - c[3 * stride + 1];
    d[2] = v - c[2 * stride + 2];  d[3] = v - c[stride + 3];
    d[4] = v - c[3];               d[5] = v - c[-stride + 3];
    d[6] = v - c[-2 * stride + 2]; d[7] = v - c[-3 * stride + 1];
    d[8] = v - c[-3 * stride];     d[9] = v - c[-3 * stride - 1];
    d[10] = v - c[-2 * stride - 2]; d[11] = v - c[-stride - 3];
    d[12] = v - c[-3];             d[13] = v - c[stride - 3];
    d[14] = v - c[2 * stride - 2]; d[15] = v - c[3 * stride - 1];
    int mn[16], mx[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) { mn[k] = min(d[k], d[(k + 1) & 15]); mx[k] = max(d[k], d[(k + 1) & 15]); }
    int mn4[16], mx4[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) { mn4[k] = min(mn[k], mn[(k + 2) & 15]); mx4[k] = max(mx[k], mx[(k + 2) & 15]); }
    int dark = -1024, bright = 1024;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int a8 = min(mn4[k], mn4[(k + 4) & 15]);
        const int b8 = max(mx4[k], mx4[(k + 4) & 15]);
        dark = max(dark, min(a8, d[(k + 8) & 15]));
        bright = min(bright, max(b8, d[(k + 8) & 15]));
    }
    return max(dark, -bright);
}

__device__ inline bool nms_keep(const uint8_t *sc, int idx) {
    const int s = sc[idx];
    return s > sc[idx - 1] && s > sc[idx + 1] &&
           s > sc[idx - kScoreW - 1] && s > sc[idx - kScoreW] && s > sc[idx - kScoreW + 1] &&
           s > sc[idx + kScoreW - 1] && s > sc[idx + kScoreW] && s > sc[idx + kScoreW + 1];
}

__global__ __launch_bounds__(kThreads) void k_fast(DevPlan p, FrameBufs fb) {
    const int ci = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
    const Cell c = p.cells[ci];
    int32_t *count_out = fb.cell_count + (int64_t)b * p.ncells + ci;
    const int cw = c.x1 - c.x0, ch = c.y1 - c.y0;
    if (cw <= 0 || ch <= 0) {
        if (tid == 0) *count_out = 0;
        return;
    }
    const LevelGeom g = p.lv[c.level];
    int spitch;
    const uint8_t *src = level_ptr(p, fb, g, c.level, b, spitch);
    __shared__ uint8_t patch[(kCellMax + 6) * kPatchW];
    __shared__ uint8_t sc_ini[(kCellMax + 2) * kScoreW];
    __shared__ uint8_t sc_min[(kCellMax + 2) * kScoreW];
    __shared__ int ws[4];
    __shared__ int any_ini;
    const int pw = cw + 6, ph = ch + 6;
    for (int i = tid; i < pw * ph; i += kThreads) {
        const int r = i / pw, col = i - r * pw;
        patch[r * kPatchW + col] = src[(int64_t)(c.y0 - 3 + r) * spitch + (c.x0 - 3 + col)];
    }
    for (int i = tid; i < (ch + 2) * kScoreW; i += kThreads) { sc_ini[i] = 0; sc_min[i] = 0; }
    if (tid == 0) any_ini = 0;
    __syncthreads();
    const int npx = cw * ch;
    for (int i = tid; i < npx; i += kThreads) {
        const int yy = i / cw, xx = i - yy * cw;
        const int s = arc_score(&patch[(yy + 3) * kPatchW + xx + 3], kPatchW);
        const int si = (yy + 1) * kScoreW + xx + 1;
        sc_ini[si] = s > p.ini_th ? (uint8_t)(s - 1) : 0;
        sc_min[si] = s > p.min_th ? (uint8_t)(s - 1) : 0;
    }
    __syncthreads();
    int found = 0;
    for (int i = tid; i < npx; i += kThreads) {
        const int yy = i / cw, xx = i - yy * cw;
        found |= nms_keep(sc_ini, (yy + 1) * kScoreW + xx + 1);
    }
    if (found) any_ini = 1;
    __syncthreads();
    const uint8_t *sc = any_ini ? sc_ini : sc_min;
    uint32_t *out = fb.cand + (int64_t)b * p.cand_cap + c.slot;
    int base = 0;
    for (int r0 = 0; r0 < npx; r0 += kThreads) {
        const int i = r0 + tid;
        int keep = 0, yy = 0, xx = 0;
        if (i < npx) {
            yy = i / cw;
            xx = i - yy * cw;
            keep = nms_keep(sc, (yy + 1) * kScoreW + xx + 1);
        }
        int total;
        const int pos = base + block_excl_scan_i32(keep, &total, ws);
        if (keep && pos < c.cap)
            out[pos] = pack_key(c.x0 + xx, c.y0 + yy, sc[(yy + 1) * kScoreW + xx + 1]);
        base += total;
    }
    if (tid == 0) *count_out = min(base, c.cap);
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

__device__ void child_stats(const QLds &s, int S, const uint32_t *keys, const uint16_t *knode,
                            uint8_t *kq, int n) {
    const int tid = threadIdx.x;
    for (int i = tid; i < 4 * S; i += kThreads) { s.ccnt[i] = 0; s.cbest[i] = 0; }
    __syncthreads();
    for (int k = tid; k < n; k += kThreads) {
        const int nd = knode[k];
        const QNode node = s.cur[nd];
        if (node.count > 1) {
            const uint32_t key = keys[k];
            const int q = quadrant_of(node, key);
            kq[k] = (uint8_t)q;
            atomicAdd(&s.ccnt[4 * nd + q], 1u);
            atomicMax(&s.cbest[4 * nd + q], best_pack(key, k));
        }
    }
    __syncthreads();
}

__device__ inline QNode make_child(const QLds &s, const QNode &parent, int i, int q, int seq) {
    QNode c = child_of(parent, q);
    c.count = (int32_t)s.ccnt[4 * i + q];
    c.best = s.cbest[4 * i + q];
    c.seq = seq;
    return c;
}

__device__ void bitonic_desc(uint64_t *a, int np2) {
    for (int size = 2; size <= np2; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int i = threadIdx.x; i < (np2 >> 1); i += kThreads) {
                const int lo = 2 * stride * (i / stride) + (i % stride);
                const int hi = lo + stride;
                const bool up = (lo & size) == 0;
                const uint64_t x = a[lo], y = a[hi];
                if (up ? (x < y) : (x > y)) { a[lo] = y; a[hi] = x; }
            }
            __syncthreads();
        }
    }
}

__global__ __launch_bounds__(kThreads) void k_quadtree(DevPlan p, FrameBufs fb) {
    extern __shared__ __align__(16) uint8_t lds[];
    const int l = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
    const LevelGeom g = p.lv[l];
    const int N = g.quota, NC = p.node_cap;
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
    __shared__ uint64_t ws64[4];
    __shared__ int ws32[4];
    __shared__ int sh_S, sh_R;

    const int64_t kbase = (int64_t)b * p.cand_cap + g.cand_off;
    uint32_t *keys = fb.keys + kbase;
    uint16_t *knode = fb.key_node + kbase;
    uint8_t *kq = fb.key_q + kbase;
    int32_t *level_count = fb.level_count + (int64_t)b * kMaxLevels + l;

    // ---- 1. gather the level's candidates in cell order (the order the
    //         reference pushes them into vToDistributeKeys)
    const int ncell = g.cell_end - g.cell_begin;
    int base = 0;
    for (int c0 = 0; c0 < ncell; c0 += kThreads) {
        const int c = c0 + tid;
        const int cnt = c < ncell ? fb.cell_count[(int64_t)b * p.ncells + g.cell_begin + c] : 0;
        int tot;
        const int ex = block_excl_scan_i32(cnt, &tot, ws32);
        if (cnt > 0) {
            const uint32_t *src = fb.cand + (int64_t)b * p.cand_cap + p.cells[g.cell_begin + c].slot;
            for (int k = 0; k < cnt; ++k) keys[base + ex + k] = src[k];
        }
        base += tot;
    }
    const int n = base;
    __syncthreads();
    if (n == 0 || g.nini <= 0) {
        if (tid == 0) *level_count = 0;
        return;
    }

    // ---- 2. root nodes (ORBextractor.cc:566-613)
    const int nini = g.nini;
    for (int i = tid; i < nini; i += kThreads) { s.ccnt[i] = 0; s.cbest[i] = 0; }
    __syncthreads();
    for (int k = tid; k < n; k += kThreads) {
        const uint32_t key = keys[k];
        const float rx = (float)((int)(key & 0xFFF) - kBorder);
        int r = (int)__fdiv_rn(rx, g.hx);
        r = min(r, nini - 1);
        knode[k] = (uint16_t)r;
        atomicAdd(&s.ccnt[r], 1u);
        atomicMax(&s.cbest[r], best_pack(key, k));
    }
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
    for (int k = tid; k < n; k += kThreads) knode[k] = (uint16_t)s.nidx_s[knode[k]];
    __syncthreads();

    // ---- 3. full rounds (ORBextractor.cc:618-696)
    bool final_phase = false;
    while (true) {
        const int S = sh_S;
        child_stats(s, S, keys, knode, kq, n);
        for (int i = tid; i < S; i += kThreads) {
            uint64_t v = 0;
            if (s.cur[i].count > 1) {
                uint64_t nc = 0, ex = 0;
                for (int q = 0; q < 4; ++q) { nc += s.ccnt[4 * i + q] > 0; ex += s.ccnt[4 * i + q] > 1; }
                v = nc | (ex << 42);
            } else {
                v = 1ull << 21;
            }
            s.a64[i] = v;
        }
        __syncthreads();
        const uint64_t tot = block_excl_scan_u64(s.a64, S, ws64);
        const int C = (int)(tot & 0x1FFFFF), singles = (int)((tot >> 21) & 0x1FFFFF);
        const int nexp = (int)(tot >> 42);
        const int S2 = C + singles;
        if (S2 > NC) {  // cannot happen by the bound in make_plan; fail loudly
            if (tid == 0) *level_count = -1;
            return;
        }
        for (int i = tid; i < S; i += kThreads) {
            const uint64_t pre = s.a64[i];
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
                s.nidx_s[i] = (int16_t)ni;
            }
        }
        __syncthreads();
        for (int k = tid; k < n; k += kThreads) {
            const int nd = knode[k];
            knode[k] = (uint16_t)(s.cur[nd].count > 1 ? s.nidx_c[4 * nd + kq[k]] : s.nidx_s[nd]);
        }
        {
            QNode *t = s.cur; s.cur = s.nxt; s.nxt = t;
        }
        if (tid == 0) sh_S = S2;
        __syncthreads();
        if (S2 >= N || S2 == S) break;
        if (S2 + nexp * 3 > N) { final_phase = true; break; }
    }

    // ---- 4. final phase (ORBextractor.cc:697-762)
    while (final_phase) {
        const int S = sh_S;
        child_stats(s, S, keys, knode, kq, n);
        for (int i = tid; i < s.np2; i += kThreads) {
            uint64_t v = 0;
            if (i < S && s.cur[i].count > 1)
                v = ((uint64_t)s.cur[i].count << 40) | ((uint64_t)s.cur[i].seq << 16) | (uint64_t)i;
            s.a64[i] = v;
        }
        for (int i = tid; i < S; i += kThreads) s.mark[i] = 0;
        __syncthreads();
        bitonic_desc(s.a64, s.np2);
        // per rank: number of non-empty children (nc) and gain (nc - 1)
        for (int r = tid; r < s.np2; r += kThreads) {
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
        int nv = 0;
        for (int r = 0; r < s.np2; ++r) nv += s.a64[r] != 0;   // uniform, small
        block_excl_scan_u64(s.b64, s.np2, ws64);
        for (int r = tid; r < nv; r += kThreads) {
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
        for (int r = tid; r < R; r += kThreads) {
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
        for (int i = tid; i < s.np2; i += kThreads) s.b64[i] = (i < S && !s.mark[i]) ? 1 : 0;
        __syncthreads();
        block_excl_scan_u64(s.b64, s.np2, ws64);
        for (int i = tid; i < S; i += kThreads) {
            if (s.mark[i]) continue;
            const int ni = CC + (int)s.b64[i];
            s.nxt[ni] = s.cur[i];
            s.nidx_s[i] = (int16_t)ni;
        }
        __syncthreads();
        for (int k = tid; k < n; k += kThreads) {
            const int nd = knode[k];
            knode[k] = (uint16_t)(s.mark[nd] ? s.nidx_c[4 * nd + kq[k]] : s.nidx_s[nd]);
        }
        {
            QNode *t = s.cur; s.cur = s.nxt; s.nxt = t;
        }
        if (tid == 0) sh_S = S2;
        __syncthreads();
        if (S2 >= N || S2 == S) break;
    }

    // ---- 5. best key per node, in list order (ORBextractor.cc:765-784)
    const int S = sh_S;
    uint32_t *sel = fb.sel + (int64_t)b * p.out_cap + g.out_off;
    const int S_out = min(S, g.out_cap);
    for (int i = tid; i < S_out; i += kThreads) {
        const int k = 0xFFFFFF - (int)(s.cur[i].best & 0xFFFFFF);
        sel[i] = keys[k];
    }
    if (tid == 0) *level_count = S <= g.out_cap ? S : -1;
}

// ===========================================================================
// K5: orientation + rBRIEF + keypoint record, one wave per selected key.
// ===========================================================================
__global__ __launch_bounds__(kThreads) void k_describe(DevPlan p, FrameBufs fb) {
    const int b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int32_t *lc = fb.level_count + (int64_t)b * kMaxLevels;
    if (blockIdx.x == 0 && tid == 0) {
        int total = 0;
        for (int l = 0; l < p.nlevels; ++l) total += max(lc[l], 0);
        fb.nkps[b] = total;
    }
    const int slot = blockIdx.x * 4 + wave;
    if (slot >= p.out_cap) return;
    int l = 0;
    while (l + 1 < p.nlevels && slot >= p.lv[l + 1].out_off) ++l;
    const LevelGeom g = p.lv[l];
    const int i = slot - g.out_off;
    if (i >= lc[l]) return;
    int off = 0;
    for (int q = 0; q < l; ++q) off += max(lc[q], 0);
    const uint32_t key = fb.sel[(int64_t)b * p.out_cap + slot];
    const int x = (int)(key & 0xFFF), y = (int)((key >> 12) & 0xFFF), score = (int)(key >> 24);

    // IC_Angle on the unblurred level (ORBextractor.cc:77-104): exact integer moments.
    int spitch;
    const uint8_t *img = level_ptr(p, fb, g, l, b, spitch);
    const uint8_t *center = img + (int64_t)y * spitch + x;
    const int u = (lane & 31) - 15;
    const int half = lane >> 5;
    int m10 = 0, m01 = 0;
    if (u <= 15) {
        for (int v = 0; v <= 15; ++v) {
            if (half == 1 && v == 0) continue;
            const int row = half ? -v : v;
            if (abs(u) <= p.umax[v]) {
                const int val = center[(int64_t)row * spitch + u];
                m10 += u * val;
                m01 += row * val;
            }
        }
    }
    m10 = wave_sum_i32(m10);
    m01 = wave_sum_i32(m01);
    const float angle = fast_atan2_deg((float)m01, (float)m10);

    // computeOrbDescriptor on the blurred level (ORBextractor.cc:106-147).
    const float factor_pi = (float)(3.14159265358979323846 / 180.f);
    float sa, ca;
    glibc_sincosf(__fmul_rn(angle, factor_pi), &sa, &ca);
    const uint8_t *blur = fb.blur + (int64_t)b * p.blur_bytes + g.blur_off;
    const uint8_t *bc = blur + (int64_t)y * g.pitch + x;
    const int64_t kp_index = (int64_t)b * p.max_kps + off + i;
    uint64_t *dout = reinterpret_cast<uint64_t *>(fb.desc + kp_index * 32);
#pragma unroll
    for (int grp = 0; grp < 4; ++grp) {
        const int j = grp * 64 + lane;
        int val[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const float px = (float)c_pattern[2 * j + e][0], py = (float)c_pattern[2 * j + e][1];
            const int r = __float2int_rn(__fadd_rn(__fmul_rn(px, sa), __fmul_rn(py, ca)));
            const int cc = __float2int_rn(__fsub_rn(__fmul_rn(px, ca), __fmul_rn(py, sa)));
            val[e] = bc[(int64_t)r * g.pitch + cc];
        }
        const uint64_t m = __ballot(val[0] < val[1]);
        if (lane == 0) dout[grp] = m;
    }
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
}

__global__ void k_trig(const float *in, float *so, float *co, int n, const float *ay, const float *ax,
                       float *at, int m) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) glibc_sincosf(in[i], &so[i], &co[i]);
    if (i < m) at[i] = fast_atan2_deg(ay[i], ax[i]);
}

}  // namespace

// ---------------------------------------------------------------------------
hipError_t launch_resize(const DevPlan &p, const Plan &hp, const FrameBufs &fb, int B, hipStream_t st) {
    for (int l = 1; l < hp.nlevels; ++l) {
        const LevelGeom &g = hp.lv[l];
        dim3 grid((g.w + 255) / 256, (g.h + 3) / 4, B);
        hipLaunchKernelGGL(k_resize, grid, dim3(kThreads), 0, st, p, fb, l);
    }
    return hipGetLastError();
}

hipError_t launch_blur(const DevPlan &p, const FrameBufs &fb, int B, hipStream_t st) {
    hipLaunchKernelGGL(k_blur, dim3(p.nblur_tiles, B), dim3(kThreads), 0, st, p, fb);
    return hipGetLastError();
}

hipError_t launch_fast(const DevPlan &p, const FrameBufs &fb, int B, hipStream_t st) {
    hipLaunchKernelGGL(k_fast, dim3(p.ncells, B), dim3(kThreads), 0, st, p, fb);
    return hipGetLastError();
}

hipError_t launch_quadtree(const DevPlan &p, const FrameBufs &fb, int B, hipStream_t st) {
    hipLaunchKernelGGL(k_quadtree, dim3(p.nlevels, B), dim3(kThreads), p.node_lds_bytes, st, p, fb);
    return hipGetLastError();
}

hipError_t launch_describe(const DevPlan &p, const FrameBufs &fb, int B, hipStream_t st) {
    hipLaunchKernelGGL(k_describe, dim3((p.out_cap + 3) / 4, B), dim3(kThreads), 0, st, p, fb);
    return hipGetLastError();
}

hipError_t launch_trig_check(const float *in, float *s, float *c, float *atan_out, const float *ay,
                             const float *ax, int n, int m, hipStream_t st) {
    const int total = n > m ? n : m;
    if (total <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_trig, dim3((total + 255) / 256), dim3(256), 0, st, in, s, c, n, ay, ax, atan_out, m);
    return hipGetLastError();
}

int quadtree_lds_bytes(int node_cap) {
    int np2 = 1;
    while (np2 < node_cap) np2 <<= 1;
    return (int)(2 * sizeof(uint64_t) * np2 + 2 * sizeof(QNode) * node_cap +
                 2 * sizeof(uint32_t) * 4 * node_cap + sizeof(int16_t) * 5 * node_cap + node_cap + 64);
}

}  // namespace orbx
