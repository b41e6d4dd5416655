// orbx_plan.h -- host-side geometry of one ORBextractor configuration.
//
// Everything here is computed once per (image size, extractor parameters) and
// uploaded as small device tables; the per-frame kernels only index them.
// The arithmetic follows the reference's exact float/double/int types:
//   scale tables and feature quotas   ORBextractor.cc:416-455 (+ ORBextractor.h:98:
//                                     scaleFactor is stored as double)
//   level sizes                       ORBextractor.cc:1157-1159
//   umax (orientation disc)           ORBextractor.cc:461-478
//   FAST cell grid                    ORBextractor.cc:796-863
//   quadtree root split               ORBextractor.cc:566-591
//   resize coefficient tables         cv::resize INTER_LINEAR 8U, OpenCV 3.2
//   Gaussian 7x7 integer taps         cv::getGaussianKernel(7, 2) x256, OpenCV 3.2
#pragma once

#include <algorithm>
#include <cfloat>
#include <climits>
#include <cmath>
#include <cstdint>
#include <vector>

namespace orbx {

constexpr int kMaxLevels = 16;
constexpr int kEdge = 19;          // EDGE_THRESHOLD, ORBextractor.cc:71
constexpr int kBorder = kEdge - 3; // minBorderX/Y, ORBextractor.cc:796-797
constexpr int kFastCell = 30;      // W, ORBextractor.cc:788
// cvRound(256 * getGaussianKernel(7, 2, CV_32F)) = {18, 34, 49, 55, 49, 34, 18};
// make_gauss_taps recomputes it from the OpenCV formula and the runtime checks both agree.
constexpr int kGaussTaps[7] = {18, 34, 49, 55, 49, 34, 18};
// umax of the orientation disc (HALF_PATCH_SIZE 15, ORBextractor.cc:461-478);
// make_plan recomputes it and the runtime checks both agree.
constexpr int kUmax[16] = {15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3};

// x86-64 cvRound (cvtss2si / cvtsd2si): round half to even.
inline int round_even(float v) { return (int)std::nearbyint(v); }
inline int round_even(double v) { return (int)std::nearbyint(v); }
inline int floor_i(float v) { int i = round_even(v); return i - (float(i) > v ? 1 : 0); }
inline int floor_i(double v) { int i = round_even(v); return i - (double(i) > v ? 1 : 0); }
inline int ceil_i(double v) { int i = round_even(v); return i + (double(i) < v ? 1 : 0); }
inline int16_t coef_short(float v) {
    return (int16_t)std::min(std::max(round_even(v), (int)SHRT_MIN), (int)SHRT_MAX);
}

// One FAST cell: interior rectangle [x0,x1) x [y0,y1) in level pixels, and
// where its candidates go.
struct Cell {
    int16_t level, pad;
    int16_t x0, y0, x1, y1;
    int32_t slot;   // first candidate slot of this cell in the frame's candidate array
    int32_t cap;    // candidate capacity (strict 3x3 maxima: ceil(w/2)*ceil(h/2))
};

// Per destination column / row of a bilinear level: source index and 11-bit
// coefficients; mode bit0 = "use both taps" (dx < xmax), bit1 = "SSE2 column".
struct ResizeTap {
    int16_t src, a0, a1, mode;
};

// k_resize_d's per-level tables (plan_resize_waves).  A column group (4
// destination columns, one lane): its row loads start at the dword c, the 8
// bytes it uses at c + o; sel / coef are the v_perm selectors of its 4 pixel
// pairs within those 8 bytes and their horizontal coefficients (a0 | a1 << 16);
// bit k of smask = column k is an SSE2 column.  A destination row: its two
// source rows (clamped) and vertical coefficients, two 16-bit halves each.
struct ResizeCol {
    int c, o, smask, pad;
    uint32_t sel[4], coef[4];
};
struct ResizeRow {
    uint32_t s01;   // s0 | s1 << 16
    uint32_t b01;   // b0 | b1 << 16
};

struct LevelGeom {
    int w, h;
    int pitch;            // row pitch of the device images (multiple of 64)
    int64_t pyr_off;      // byte offset inside a frame's pyramid block (levels >= 1; level 0
                          // is the caller's image and has no slot)
    int64_t blur_off;     // byte offset inside a frame's blurred-pyramid block (all levels)
    int quota;            // mnFeaturesPerLevel
    float scale, inv_scale, sigma2, inv_sigma2;
    float patch_size;     // (float)(int)(31 * scale), ORBextractor.cc:874
    int ncols, nrows, wcell, hcell;
    int cell_begin, cell_end;        // range in the plan's cell table
    int64_t cand_off;     // first candidate slot of the level (per frame)
    int cand_cap;         // candidate capacity of the level
    int out_off, out_cap; // per-frame staging slots for the level's selected keys
    int nini;             // quadtree root count
    float hx;             // quadtree root width (float), ORBextractor.cc:568
    int xtab_off, ytab_off;          // into the plan's resize tap tables (levels >= 1)
};

// Wave-tile geometry of one pyramid level's resize (k_resize): a wave owns
// 4*twg columns x (64/twg)*kResizeK rows; lane (lr, lg) writes columns
// x0 + 4 lg .. + 3 of rows y0 + lr kResizeK + j.  twg in {16, 32, 64} is chosen
// per level to waste the fewest columns at the right edge.  10 rows per lane:
// at the 1.2 scale factor the source rows advance by 6 every 5 output rows,
// so every lane group starts at the same phase and the lanes of a wave reuse
// the previous row's horizontal pass together (resize_tile).
#ifndef ORBX_RS_K
#define ORBX_RS_K 10
#endif
constexpr int kResizeK = ORBX_RS_K;
struct ResizeWave {
    double sx = 0, sy = 0;     // source / destination size ratio, as make_resize_taps
    int twg = 64, twg_shift = 6;
    int ntx = 0, ntiles = 0;   // tiles per row of tiles, per frame
    int win_stride = 0;        // LDS bytes per window row (dword multiple)
    int win_bytes = 0;         // LDS bytes per wave (16-B multiple)
    int win_dwords = 0;        // largest window, in staged dwords
    int stage_passes = 0;      // row passes of the window staging (wave_stage_rows)
    int xtab_off = 0, ytab_off = 0;   // the level's tap tables
    int direct = 0;            // k_resize_d: rows read straight from global memory (no window)
    int col_off = 0;           // the level's ResizeCol table (k_resize_d; rows: ytab_off)
};

// A pixel rectangle, inclusive bounds (an int4 on the device).
struct RgnRect {
    int x0, y0, x1, y1;
};

struct Plan {
    int width = 0, height = 0;
    int nfeatures = 0, nlevels = 0, ini_th = 0, min_th = 0;
    float scale_factor = 1.2f;
    std::vector<LevelGeom> lv;
    std::vector<Cell> cells;
    std::vector<ResizeTap> xtaps, ytaps;
    int gauss[7] = {0};
    int umax[16] = {0};
    int64_t pyr_bytes = 0;    // bytes of one frame's pyramid block (levels 1..n-1)
    int64_t blur_bytes = 0;   // bytes of one frame's blurred pyramid (levels 0..n-1)
    int64_t cand_cap = 0;     // candidate slots per frame
    int out_cap = 0;          // staging slots per frame (sum of level out_cap)
    int max_kps = 0;          // keypoint capacity per frame
    int max_quota = 0;
    std::vector<ResizeWave> rw;   // per level (index 0 unused); empty: k_resize_lds path
    std::vector<ResizeCol> rcols;   // k_resize_d tables (rw[l].col_off; rows at lv[l].ytab_off)
    std::vector<ResizeRow> rrows;
    // Region pyramid (k_pyramid_rgn, small batches): per region 2 x kMaxLevels
    // rectangles, [l] = the level-l pixels it computes (level 0: reads),
    // [kMaxLevels + l] = the ones it owns and writes.  rgn_n = 0: not used.
    std::vector<RgnRect> rgn;
    int rgn_n = 0;
    int rgn_half = 0;   // LDS bytes of one of the kernel's two level buffers
};

inline int pitch_of(int w) { return (w + 63) & ~63; }

inline void make_gauss_taps(int k[7]) {
    float cf[7];
    double sum = 0;
    const double sigma = 2.0, scale2x = -0.5 / (sigma * sigma);
    for (int i = 0; i < 7; ++i) {
        const double x = i - 3.0;
        cf[i] = (float)std::exp(scale2x * x * x);
        sum += cf[i];
    }
    sum = 1. / sum;
    for (int i = 0; i < 7; ++i) cf[i] = (float)(cf[i] * sum);
    for (int i = 0; i < 7; ++i) k[i] = round_even(cf[i] * 256.f);
}

// Bilinear coefficient table for one axis (OpenCV 3.2 resize(), INTER_LINEAR).
// For x taps, bit1 of mode marks columns handled by the SSE2 vertical pass.
inline void make_resize_taps(int ssize, int dsize, bool is_x, std::vector<ResizeTap> &out) {
    const double inv = (double)dsize / ssize;
    const double scale = 1. / inv;
    int xmax = dsize;
    std::vector<ResizeTap> t(dsize);
    for (int d = 0; d < dsize; ++d) {
        float f = (float)((d + 0.5) * scale - 0.5);
        int s = floor_i(f);
        f -= s;
        if (is_x) {
            if (s < 0) { f = 0.f; s = 0; }
            if (s + 1 >= ssize) {
                xmax = std::min(xmax, d);
                if (s >= ssize - 1) { f = 0.f; s = ssize - 1; }
            }
        }
        t[d].src = (int16_t)s;
        t[d].a0 = coef_short((1.f - f) * 2048);
        t[d].a1 = coef_short(f * 2048);
        t[d].mode = 0;
    }
    if (is_x) {
        int xs = 0;
        while (xs <= dsize - 16) xs += 16;
        while (xs < dsize - 4) xs += 4;
        for (int d = 0; d < dsize; ++d) {
            t[d].mode = (int16_t)((d < xmax ? 1 : 0) | (d < xs ? 2 : 0));
            // From xmax on, HResizeLinear stores S[sx]*2048: the same value as the
            // two-tap form with coefficients (2048, 0), which keeps the kernel branch-free.
            if (d >= xmax) { t[d].a0 = 2048; t[d].a1 = 0; }
        }
    }
    out.insert(out.end(), t.begin(), t.end());
}

inline Plan make_plan(int width, int height, int nfeatures, float scale_factor_f, int nlevels,
                      int ini_th, int min_th) {
    Plan p;
    p.width = width; p.height = height; p.nfeatures = nfeatures; p.nlevels = nlevels;
    p.ini_th = ini_th; p.min_th = min_th; p.scale_factor = scale_factor_f;
    p.lv.resize(nlevels);
    const double sf = scale_factor_f;  // double member, ORBextractor.h:98
    std::vector<float> scale(nlevels, 1.f), sig2(nlevels, 1.f);
    for (int i = 1; i < nlevels; ++i) {
        scale[i] = (float)(scale[i - 1] * sf);
        sig2[i] = scale[i] * scale[i];
    }
    const float factor = (float)(1.0f / sf);
    float ndesired = nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)nlevels));
    int sum = 0;
    for (int l = 0; l < nlevels; ++l) {
        LevelGeom &g = p.lv[l];
        g.scale = scale[l];
        g.inv_scale = 1.0f / scale[l];
        g.sigma2 = sig2[l];
        g.inv_sigma2 = 1.0f / sig2[l];
        g.patch_size = (float)(int)(31 * scale[l]);
        if (l < nlevels - 1) {
            g.quota = round_even(ndesired);
            sum += g.quota;
            ndesired *= factor;
        } else {
            g.quota = std::max(nfeatures - sum, 0);
        }
        g.w = round_even((float)width * g.inv_scale);
        g.h = round_even((float)height * g.inv_scale);
        g.pitch = pitch_of(g.w);
        p.max_quota = std::max(p.max_quota, g.quota);
    }
    // umax, ORBextractor.cc:461-478
    {
        const int hp = 15;
        int vmax = floor_i(hp * std::sqrt(2.f) / 2 + 1);
        int vmin = ceil_i(hp * std::sqrt(2.f) / 2);
        const double hp2 = hp * hp;
        for (int v = 0; v <= vmax; ++v) p.umax[v] = round_even(std::sqrt(hp2 - v * v));
        for (int v = hp, v0 = 0; v >= vmin; --v) {
            while (p.umax[v0] == p.umax[v0 + 1]) ++v0;
            p.umax[v] = v0;
            ++v0;
        }
    }
    make_gauss_taps(p.gauss);
    int64_t pyr_off = 0, blur_off = 0, cand_off = 0;
    int out_off = 0;
    for (int l = 0; l < nlevels; ++l) {
        LevelGeom &g = p.lv[l];
        g.pyr_off = l == 0 ? -1 : pyr_off;
        if (l > 0) pyr_off += (int64_t)g.pitch * g.h;
        g.blur_off = blur_off;
        blur_off += (int64_t)g.pitch * g.h;
        // FAST cell grid (ORBextractor.cc:796-817); interiors tile [19, dim-19).
        const int maxbx = g.w - kEdge + 3, maxby = g.h - kEdge + 3;
        const float width_f = (float)(maxbx - kBorder), height_f = (float)(maxby - kBorder);
        g.ncols = std::max(0, (int)(width_f / kFastCell));
        g.nrows = std::max(0, (int)(height_f / kFastCell));
        g.wcell = g.ncols > 0 ? (int)std::ceil(width_f / g.ncols) : 0;
        g.hcell = g.nrows > 0 ? (int)std::ceil(height_f / g.nrows) : 0;
        g.cell_begin = (int)p.cells.size();
        g.cand_off = cand_off;
        int64_t lvl_cap = 0;
        for (int i = 0; i < g.nrows; ++i) {
            for (int j = 0; j < g.ncols; ++j) {
                Cell c;
                c.level = (int16_t)l; c.pad = 0;
                c.x0 = (int16_t)(kEdge + j * g.wcell);
                c.y0 = (int16_t)(kEdge + i * g.hcell);
                c.x1 = (int16_t)std::min(kEdge + (j + 1) * g.wcell, g.w - kEdge);
                c.y1 = (int16_t)std::min(kEdge + (i + 1) * g.hcell, g.h - kEdge);
                const int cw = std::max(0, c.x1 - c.x0), ch = std::max(0, c.y1 - c.y0);
                c.slot = (int32_t)(cand_off + lvl_cap);
                c.cap = ((cw + 1) / 2) * ((ch + 1) / 2);
                lvl_cap += c.cap;
                p.cells.push_back(c);
            }
        }
        g.cell_end = (int)p.cells.size();
        g.cand_cap = (int)lvl_cap;
        cand_off += lvl_cap;
        // quadtree roots, ORBextractor.cc:566-568
        const int minx = kBorder, maxx = g.w - kBorder, miny = kBorder, maxy = g.h - kBorder;
        g.nini = (maxy - miny) > 0 ? (int)std::round((float)(maxx - minx) / (maxy - miny)) : 0;
        g.hx = g.nini > 0 ? (float)(maxx - minx) / g.nini : 0.f;
        // Output bound: a full round never overshoots N, a final-phase split adds <= 3,
        // and the unconditional first round yields <= 4 * nIni nodes.
        g.out_cap = std::max(g.quota, 4 * g.nini) + 3;
        g.out_off = out_off;
        out_off += g.out_cap;
        if (l >= 1) {
            g.xtab_off = (int)p.xtaps.size();
            make_resize_taps(p.lv[l - 1].w, g.w, true, p.xtaps);
            g.ytab_off = (int)p.ytaps.size();
            make_resize_taps(p.lv[l - 1].h, g.h, false, p.ytaps);
        } else {
            g.xtab_off = g.ytab_off = 0;
        }
    }
    p.pyr_bytes = pyr_off;
    p.blur_bytes = blur_off;
    p.cand_cap = cand_off;
    p.out_cap = out_off;
    p.max_kps = out_off;
    return p;
}

}  // namespace orbx
