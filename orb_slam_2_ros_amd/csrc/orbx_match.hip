// orbx_match.hip -- ORBmatcher::SearchForInitialization on gfx950.
//
// Reference: ORBmatcher.cc:406-521 (+ ComputeThreeMaxima :1603-1644,
// DescriptorDistance :1649-1665), Frame::AssignFeaturesToGrid / PosInGrid /
// GetFeaturesInArea (Frame.cc:239-256, 415-425, 354-412).
//
// One 256-thread workgroup per frame pair.  The work that carries no
// dependency -- grid build, window enumeration (a lane per query), filters,
// all Hamming distances -- runs on every wave; the reference's greedy loop
// (its vMatchedDistance / vnMatches21 state makes query i1 depend on every
// earlier one) is replayed in order by a single wave.  Each query's 4 smallest (distance, position)
// entries are found in the parallel phase; the replay only checks their
// vMatchedDistance validity, falling back to a 64-wide ballot/min scan of the
// whole list when fewer than two of the four are still valid.  Tie semantics
// are the reference's: first minimum wins; second-best is the multiset second
// minimum.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>

#include "orbx_device.h"
#include "orbx_wave.h"

namespace orbx {
namespace {

constexpr int kGridCols = 64, kGridRows = 48;  // Frame.h:37-38
// The F2 grid is kept as column buckets of kBucketRows cells: a window's
// bucket range per column holds its cells' entries in the same order (cell,
// then index), plus entries of up to kBucketRows - 1 cells above and below
// the window, which lie at least half a cell outside the window's rows and so
// fail GetFeaturesInArea's |dy| < r test like any non-candidate (the list
// positions stay monotone, which is all the tie order needs).
constexpr int kBucketRows = 8, kColBuckets = kGridRows / kBucketRows;   // 6
constexpr int kBuckets = kGridCols * kColBuckets;                        // 384
static_assert(kGridRows % kBucketRows == 0, "whole buckets per column");
constexpr int kHisto = 30;                      // ORBmatcher::HISTO_LENGTH
constexpr int kThLow = 50;                      // ORBmatcher::TH_LOW
constexpr int kSkip = 0xFFFF;
constexpr int kMT = 256;                        // threads per frame pair
constexpr int kMW = kMT / 64;                   // waves

// LDS layout of one frame pair, indexed by grid position (F2 octave-0
// keypoints, < maxc) or query rank (F1 octave-0 keypoints, < maxq) only, with
// 16-bit bucket starts, distances and indices; the query descriptors stay in
// global memory (each is read once, by its query's lane, into registers), so a
// pair needs ~19 KB at VGA and eight pairs share a CU (16-B aligned arrays
// first).
struct MLds {
    uint4 *gd;       // maxc x 2: F2 octave-0 descriptors in grid order
    float2 *gxy;     // maxc: F2 positions in grid order
    float2 *qxy;     // maxq: query centres (vbPrevMatched)
    uint32_t *top4;  // maxq x 4: (grid position << 16 | dist) of the 4 smallest (dist, list position)
    uint32_t *claim; // maxc: (replay batch << 16 | (255 - lane) << 8 | dist) of a batch's first acceptor
    uint16_t *gstart;   // kBuckets + 1 (+1 pad): first grid position of each bucket (dword-aligned pairs)
    uint16_t *gcell; // maxc: grid cell of each grid position (the in-bucket sort key)
    int16_t *mdist;  // maxc: vMatchedDistance by grid position (kNoDist: none)
    int16_t *m21;    // maxc: vnMatches21 (query rank) by grid position
    int16_t *m12;    // maxq: vnMatches12 (grid position) by query rank
    int16_t *glist;  // maxc: F2 index by grid position
    int16_t *qidx;   // maxq: F1 index of each query
    int16_t *live;   // maxq: queries that can be accepted, in order
    int16_t *acc;    // maxq: grid position accepted by each query (-1: none)
    int8_t *rbin;    // maxq: rotation bin of accepted queries (-1: none)
};

__device__ inline MLds carve(uint8_t *ptr, int maxq, int maxc) {
    MLds s;
    s.gd = reinterpret_cast<uint4 *>(ptr); ptr += sizeof(uint4) * 2 * maxc;
    s.gxy = reinterpret_cast<float2 *>(ptr); ptr += sizeof(float2) * maxc;
    s.qxy = reinterpret_cast<float2 *>(ptr); ptr += sizeof(float2) * maxq;
    ptr += 8 * ((maxc + maxq) & 1);   // top4 rows are read as uint4
    s.top4 = reinterpret_cast<uint32_t *>(ptr); ptr += sizeof(uint32_t) * 4 * maxq;
    s.claim = reinterpret_cast<uint32_t *>(ptr); ptr += sizeof(uint32_t) * maxc;
    s.gstart = reinterpret_cast<uint16_t *>(ptr); ptr += sizeof(uint16_t) * (kBuckets + 2);
    s.gcell = reinterpret_cast<uint16_t *>(ptr); ptr += sizeof(uint16_t) * ((maxc + 1) & ~1);
    s.mdist = reinterpret_cast<int16_t *>(ptr); ptr += sizeof(int16_t) * ((maxc + 1) & ~1);
    s.m21 = reinterpret_cast<int16_t *>(ptr); ptr += sizeof(int16_t) * ((maxc + 1) & ~1);
    s.m12 = reinterpret_cast<int16_t *>(ptr); ptr += sizeof(int16_t) * ((maxq + 1) & ~1);
    s.glist = reinterpret_cast<int16_t *>(ptr); ptr += sizeof(int16_t) * ((maxc + 1) & ~1);
    s.qidx = reinterpret_cast<int16_t *>(ptr); ptr += sizeof(int16_t) * ((maxq + 1) & ~1);
    s.live = reinterpret_cast<int16_t *>(ptr); ptr += sizeof(int16_t) * ((maxq + 1) & ~1);
    s.acc = reinterpret_cast<int16_t *>(ptr); ptr += sizeof(int16_t) * ((maxq + 1) & ~1);
    s.rbin = reinterpret_cast<int8_t *>(ptr);
    return s;
}

// atomicAdd on one 16-bit cell start: LDS atomics are 32-bit, so the pair
// holding it takes the add in its half (counts stay < 2^16: no carry).
// Returns the half's old value.
__device__ inline int gstart_add(uint16_t *gstart, int cell, int v) {
    uint32_t *w = reinterpret_cast<uint32_t *>(gstart) + (cell >> 1);
    const int sh = 16 * (cell & 1);
    return (int)((atomicAdd(w, (uint32_t)v << sh) >> sh) & 0xFFFFu);
}

constexpr int kNoDist = 0x7FFF;   // vMatchedDistance's INT_MAX (distances are <= 256)

__device__ inline int hamming_regs(const uint4 a0, const uint4 a1, const uint4 b0, const uint4 b1) {
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

// Exclusive scan of one int per thread over the block.
__device__ inline int block_scan_i32(int v, int *total, int *ws) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int incl = wave_incl_scan_i32(v);
    if (lane == 63) ws[wave] = incl;
    __syncthreads();
    int base = 0, tot = 0;
    for (int w = 0; w < kMW; ++w) {
        if (w < wave) base += ws[w];
        tot += ws[w];
    }
    __syncthreads();
    *total = tot;
    return base + incl - v;
}

// PosInGrid (Frame.cc:415-425) for an undistorted image: round(), cell
// ix * 48 + iy, or -1 outside the grid.
__device__ inline int bucket_of(int cell) {
    const int ix = cell / kGridRows;
    return ix * kColBuckets + (cell - ix * kGridRows) / kBucketRows;
}
__device__ inline int grid_cell(float x, float y, float minX, float minY, float invW, float invH) {
    const int px = (int)roundf(__fmul_rn(__fsub_rn(x, minX), invW));
    const int py = (int)roundf(__fmul_rn(__fsub_rn(y, minY), invH));
    return (px >= 0 && px < kGridCols && py >= 0 && py < kGridRows) ? px * kGridRows + py : -1;
}

__global__ __launch_bounds__(kMT) void k_search_init(MatchBufs mb, int maxq, int maxc) {
    extern __shared__ __align__(16) uint8_t lds[];
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const orbx_keypoint *k1 = mb.k1 + (int64_t)b * mb.k1_stride;
    const orbx_keypoint *k2 = mb.k2 + (int64_t)b * mb.k2_stride;
    const uint8_t *d1 = mb.d1 + (int64_t)b * mb.k1_stride * 32;
    const uint8_t *d2 = mb.d2 + (int64_t)b * mb.k2_stride * 32;
    const int n1 = mb.n1[b], n2 = mb.n2[b];
    float *prev = mb.prev_xy + (int64_t)b * mb.k1_stride * 2;
    int32_t *out12 = mb.matches12 + (int64_t)b * mb.k1_stride;
    const MLds s = carve(lds, maxq, maxc);
    __shared__ int hist[kHisto];
    __shared__ int ws[kMW];
    __shared__ int sh_top[3];
    __shared__ int sh_err, sh_nq;

    // Frame grid constants (Frame.cc:218-221 over ComputeImageBounds, :487-497;
    // an undistorted camera has minX = minY = 0, maxX / maxY the image size)
    const float minX = mb.min_x, minY = mb.min_y;
    const float invW = __fdiv_rn((float)kGridCols, __fsub_rn(mb.max_x, minX));
    const float invH = __fdiv_rn((float)kGridRows, __fsub_rn(mb.max_y, minY));
    const float r = (float)mb.window;
    const bool clk = mb.clocks && b == 0 && tid == 0;
    if (clk) { mb.clocks[0] = clock64(); mb.clocks[6] = 0; mb.clocks[7] = 0; }

    // ---- 0. init; every output defaults to "no match"
    for (int i = tid; i < (kBuckets + 2) / 2; i += kMT) reinterpret_cast<uint32_t *>(s.gstart)[i] = 0;
    for (int i = tid; i < maxc; i += kMT) { s.mdist[i] = kNoDist; s.m21[i] = -1; s.claim[i] = 0; }
    for (int i = tid; i < maxq; i += kMT) { s.m12[i] = -1; s.rbin[i] = -1; s.acc[i] = -1; }
    for (int i = tid; i < n1; i += kMT) {
        out12[i] = -1;
        if (mb.reset_prev) { prev[2 * i] = k1[i].x; prev[2 * i + 1] = k1[i].y; }
    }
    if (tid < kHisto) hist[tid] = 0;
    if (tid == 0) sh_err = 0;
    __syncthreads();
    if (clk) mb.clocks[1] = clock64();

    // ---- 1. F2 grid of octave-0 keypoints by bucket: counts, exclusive scan,
    //         then placement by a second atomic pass on the starts (which
    //         leaves gstart[c] at the end of bucket c, i.e. the start of c + 1)
    for (int i = tid; i < n2; i += kMT) {
        if (k2[i].octave != 0) continue;
        const int cell = grid_cell(k2[i].x, k2[i].y, minX, minY, invW, invH);
        if (cell >= 0) gstart_add(s.gstart, bucket_of(cell), 1);
    }
    __syncthreads();
    constexpr int kPer = (kBuckets + kMT - 1) / kMT;   // 2 buckets per thread, contiguous
    {
        int local = 0;
        for (int i = 0; i < kPer; ++i)
            if (tid * kPer + i < kBuckets) local += s.gstart[tid * kPer + i];
        int tot;
        int run = block_scan_i32(local, &tot, ws);
        for (int i = 0; i < kPer; ++i) {
            if (tid * kPer + i >= kBuckets) break;
            const int v = s.gstart[tid * kPer + i];
            s.gstart[tid * kPer + i] = (uint16_t)run;
            run += v;
        }
        if (tid == kMT - 1) s.gstart[kBuckets] = (uint16_t)min(tot, 0xFFFF);
        if (tid == 0 && tot > maxc) sh_err = 1;
        __syncthreads();
    }
    for (int i = tid; i < n2; i += kMT) {
        if (k2[i].octave != 0) continue;
        const int cell = grid_cell(k2[i].x, k2[i].y, minX, minY, invW, invH);
        if (cell >= 0) {
            const int pos = gstart_add(s.gstart, bucket_of(cell), 1);
            if (pos < maxc) {
                s.glist[pos] = (int16_t)i;
                s.gcell[pos] = (uint16_t)cell;
            }
        }
    }
    __syncthreads();
    {   // shift back: start(c) = end(c - 1)
        int v[kPer];
#pragma unroll
        for (int i = 0; i < kPer; ++i) {
            const int c = tid * kPer + i;
            v[i] = c == 0 || c >= kBuckets ? 0 : s.gstart[c - 1];
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < kPer; ++i)
            if (tid * kPer + i < kBuckets) s.gstart[tid * kPer + i] = (uint16_t)v[i];
        __syncthreads();
    }
    // each bucket's list in (cell, keypoint index) order: mGrid's cells in
    // window order, each in push_back (index) order
    for (int c = tid; c < kBuckets; c += kMT) {
        const int st = s.gstart[c], en = min((int)s.gstart[c + 1], maxc);
        for (int a = st + 1; a < en; ++a) {
            const int16_t v = s.glist[a];
            const uint16_t vc = s.gcell[a];
            int j = a - 1;
            while (j >= st && (s.gcell[j] > vc || (s.gcell[j] == vc && s.glist[j] > v))) {
                s.glist[j + 1] = s.glist[j];
                s.gcell[j + 1] = s.gcell[j];
                --j;
            }
            s.glist[j + 1] = v;
            s.gcell[j + 1] = vc;
        }
    }
    __syncthreads();
    const int ngrid = min((int)s.gstart[kBuckets], maxc);
    for (int pos = tid; pos < ngrid; pos += kMT) {
        const int i2 = s.glist[pos];
        s.gxy[pos] = make_float2(k2[i2].x, k2[i2].y);
        const uint4 *dp = reinterpret_cast<const uint4 *>(d2 + (int64_t)i2 * 32);
        s.gd[2 * pos] = dp[0];
        s.gd[2 * pos + 1] = dp[1];
    }
    // queries: F1 octave-0 keypoints in index order
    {
        const int per = (n1 + kMT - 1) / kMT;
        const int st = min(tid * per, n1), en = min(st + per, n1);
        int local = 0;
        for (int i = st; i < en; ++i) local += k1[i].octave == 0;
        int tot;
        int run = block_scan_i32(local, &tot, ws);
        for (int i = st; i < en; ++i) {
            if (k1[i].octave != 0) continue;
            if (run < maxq) {
                s.qidx[run] = (int16_t)i;
                s.qxy[run] = make_float2(prev[2 * i], prev[2 * i + 1]);
            }
            ++run;
        }
        if (tid == 0) { sh_nq = min(tot, maxq); if (tot > maxq) sh_err = 1; }
    }
    __syncthreads();
    const int nq = sh_nq;
    if (clk) mb.clocks[2] = clock64();

    // GetFeaturesInArea's cell window (Frame.cc:354-412) of a query centre
    auto cells_of = [&](float x, float y, int &cx0, int &cx1, int &cy0, int &cy1) {
        const float ux = __fsub_rn(x, minX), uy = __fsub_rn(y, minY);   // (x - mnMinX) -/+ r, Frame.cc:361-373
        cx0 = max(0, (int)floorf(__fmul_rn(__fsub_rn(ux, r), invW)));
        cx1 = min(kGridCols - 1, (int)ceilf(__fmul_rn(__fadd_rn(ux, r), invW)));
        cy0 = max(0, (int)floorf(__fmul_rn(__fsub_rn(uy, r), invH)));
        cy1 = min(kGridRows - 1, (int)ceilf(__fmul_rn(__fadd_rn(uy, r), invH)));
        return !(cx0 >= kGridCols || cx1 < 0 || cy0 >= kGridRows || cy1 < 0 || cx1 < cx0 || cy1 < cy0);
    };
    // distance of grid entry gp to query q's descriptor; kSkip outside the window
    auto entry_dist = [&](int gp, float x, float y, const uint4 &qa, const uint4 &qb) {
        const float2 kp = s.gxy[gp];
        const float dx = __fsub_rn(kp.x, x), dy = __fsub_rn(kp.y, y);
        return (fabsf(dx) < r && fabsf(dy) < r) ? hamming_regs(qa, qb, s.gd[2 * gp], s.gd[2 * gp + 1]) : kSkip;
    };

    // ---- 2. candidate distances, one lane per query.  GetFeaturesInArea
    //         visits ix outer, iy inner, then cell insertion order; the grid
    //         is sorted by cell = ix * 48 + iy and index, so the window's list
    //         is one contiguous grid range per column ix and a candidate's list
    //         position is a running count over the columns.  Each query keeps
    //         its 4 smallest (dist, position) entries; the rare replay that
    //         needs more walks the window again.
    for (int q = tid; q < nq; q += kMT) {
        uint32_t tk[4] = {~0u, ~0u, ~0u, ~0u};
        int tg[4] = {0, 0, 0, 0};
        int cx0, cx1, cy0, cy1;
        const float2 c = s.qxy[q];
        if (cells_of(c.x, c.y, cx0, cx1, cy0, cy1)) {
            const uint4 *qp = reinterpret_cast<const uint4 *>(d1 + (int64_t)s.qidx[q] * 32);
            const uint4 qa = qp[0], qb = qp[1];
            int pos = 0;
            for (int ix = cx0; ix <= cx1; ++ix) {
                const int col = ix * kColBuckets;
                const int st = s.gstart[col + cy0 / kBucketRows];
                const int en = min((int)s.gstart[col + cy1 / kBucketRows + 1], maxc);
                for (int gp = st; gp < en; ++gp, ++pos) {
                    const int dist = entry_dist(gp, c.x, c.y, qa, qb);
                    if (dist == kSkip || pos >= maxc) continue;
                    uint32_t k = ((uint32_t)dist << 16) | (uint32_t)pos;
                    int kg = gp;
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        if (k < tk[j]) {
                            const uint32_t t = tk[j]; tk[j] = k; k = t;
                            const int u = tg[j]; tg[j] = kg; kg = u;
                        }
                    }
                }
            }
            if (pos > maxc) sh_err = 1;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j)
            s.top4[4 * q + j] = tk[j] == ~0u ? 0xFFFFFFFFu : ((uint32_t)tg[j] << 16) | (tk[j] >> 16);
    }
    __syncthreads();
    if (clk) mb.clocks[3] = clock64();

    // ---- 3. ordered greedy replay (ORBmatcher.cc:425-491), wave 0 only.
    // The valid entries (vMatchedDistance > dist) among a query's 4 smallest
    // (dist, position) entries, in order, are the smallest valid ones of its
    // whole list: two found decide (best, best2); a list that fits in 4 is
    // decided too; otherwise the whole list is walked again.  Queries whose
    // smallest distance exceeds TH_LOW can never be accepted and change no
    // state, so only the others ("live") are replayed, 64 consecutive ones per
    // batch, one per lane, each against the state left by the committed ones.
    // A lane's decision is the in-order one unless an earlier lane of the
    // batch accepts a keypoint among the entries it examined (the only state
    // its decision reads): the batch commits up to the first such lane (or the
    // first lane that needs its whole list, which then runs alone) and the
    // next batch starts there.  Lane 0 of a batch always commits.
    if (wave == 0) {
        // the replay is the block's serial critical path: let it issue ahead
        // of the co-resident blocks' waves
        __builtin_amdgcn_s_setprio(3);
        int nlive = 0;
        for (int g0 = 0; g0 < nq; g0 += 64) {
            const int q = g0 + lane;
            const uint32_t r0 = q < nq ? s.top4[4 * q] : 0xFFFFFFFFu;
            const bool live = r0 != 0xFFFFFFFFu && (int)(r0 & 0xFFFF) <= kThLow;
            const uint64_t m = __ballot(live);
            if (live) s.live[nlive + __popcll(m & ((1ull << lane) - 1))] = (int16_t)q;
            nlive += __popcll(m);
        }
        wave_lds_fence();
        if (clk) mb.clocks[7] = nlive;
        const float nnr = mb.nnratio;
        uint32_t batch = 0;
        for (int P = 0; P < nlive;) {
            ++batch;
            const int idx = P + lane;
            const bool act = idx < nlive;
            const int q = act ? s.live[idx] : 0;
            uint32_t e4[4];
            {
                const uint4 t4 = act ? *reinterpret_cast<const uint4 *>(s.top4 + 4 * q)
                                     : make_uint4(~0u, ~0u, ~0u, ~0u);
                e4[0] = t4.x; e4[1] = t4.y; e4[2] = t4.z; e4[3] = t4.w;
            }
            int md[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) md[t] = s.mdist[e4[t] == 0xFFFFFFFFu ? 0 : (e4[t] >> 16)];
            int best = INT_MAX, best2 = INT_MAX, best_g = -1, found = 0, ne = 0;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                if (e4[t] == 0xFFFFFFFFu || found == 2) continue;
                ne = t + 1;
                const int g = (int)(e4[t] >> 16), dist = (int)(e4[t] & 0xFFFF);
                if (md[t] <= dist) continue;
                if (found == 0) { best = dist; best_g = g; }
                else best2 = dist;
                ++found;
            }
            const bool fb = act && !(found == 2 || e4[3] == 0xFFFFFFFFu);
            const bool ok = act && !fb && best <= kThLow && (float)best < __fmul_rn((float)best2, nnr);
            const uint64_t fbm = __ballot(fb);
            const int f = fbm ? (int)__builtin_ctzll(fbm) : 64;
            // claim = batch << 16 | (255 - lane) << 8 | best: the earliest
            // accepting lane of the batch and the vMatchedDistance it leaves
            if (ok && lane < f)
                atomicMax(&s.claim[best_g], (batch << 16) | ((uint32_t)(255 - lane) << 8) | (uint32_t)best);
            wave_lds_fence();
            // An entry the lane found valid (md > dist) turns invalid iff an
            // earlier lane accepts its keypoint with best <= dist; an invalid
            // one stays invalid (the acceptor saw md > best).  Accepting a
            // keypoint an earlier lane accepts (a steal within the batch) also
            // ends the commit, so each keypoint has one acceptor per batch and
            // the claim's distance is what that acceptor leaves.
            bool inval = false;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                if (t < ne && act && lane < f) {
                    const uint32_t c = s.claim[e4[t] >> 16];
                    const int dist = (int)(e4[t] & 0xFFFF);
                    const bool earlier = (c >> 16) == batch && 255 - (int)((c >> 8) & 0xFF) < lane;
                    inval |= earlier && ((md[t] > dist && (int)(c & 0xFF) <= dist) ||
                                         (ok && (int)(e4[t] >> 16) == best_g));
                }
            }
            const uint64_t im = __ballot(inval);
            const int cut = min(min(im ? (int)__builtin_ctzll(im) : 64, f), nlive - P);
            if (ok && lane < cut) {
                const int old = s.m21[best_g];
                if (old >= 0) s.m12[old] = -1;
                s.m12[q] = (int16_t)best_g;
                s.m21[best_g] = (int16_t)q;
                s.mdist[best_g] = (int16_t)best;
                s.acc[q] = (int16_t)best_g;   // binned in phase 4 (stolen pairs keep their bin)
            }
            wave_lds_fence();
            if (clk) mb.clocks[6] += 1;
            P += cut;
            if (cut == f && P < nlive) {
                // lane f's query needs its whole list: walk the window again,
                // lane = grid column; each lane keeps its column's smallest
                // valid (dist, position) key and its second distance
                const int qf = s.live[P];
                const float2 c = s.qxy[qf];
                int cx0, cx1, cy0, cy1, st = 0, cc = 0;
                if (cells_of(c.x, c.y, cx0, cx1, cy0, cy1) && lane < cx1 - cx0 + 1) {
                    const int col = (cx0 + lane) * kColBuckets;
                    st = s.gstart[col + cy0 / kBucketRows];
                    cc = max(min((int)s.gstart[col + cy1 / kBucketRows + 1], maxc) - st, 0);
                }
                const int pos0 = wave_incl_scan_i32(cc) - cc;
                const uint4 *qp = reinterpret_cast<const uint4 *>(d1 + (int64_t)s.qidx[qf] * 32);
                const uint4 qa = qp[0], qb = qp[1];
                uint32_t k1 = ~0u;
                int d2 = INT_MAX, ga = 0;
                for (int e = 0; e < cc; ++e) {
                    const int gp = st + e;
                    if (pos0 + e >= maxc) break;
                    const int dist = entry_dist(gp, c.x, c.y, qa, qb);
                    if (dist == kSkip || s.mdist[gp] <= dist) continue;
                    const uint32_t k = ((uint32_t)dist << 16) | (uint32_t)(pos0 + e);
                    if (k < k1) { d2 = k1 == ~0u ? INT_MAX : (int)(k1 >> 16); k1 = k; ga = gp; }
                    else d2 = min(d2, dist);
                }
                const uint32_t mn = wave_min_u32(k1);
                int fbest = INT_MAX, fbest2 = INT_MAX, fg = -1;
                if (mn != ~0u) {
                    const uint64_t who = __ballot(k1 == mn);
                    const int wl = (int)__builtin_ctzll(who);
                    fbest = (int)(mn >> 16);
                    fg = __builtin_amdgcn_readlane(ga, wl);
                    // multiset second: the best lane's second, every other lane's first
                    const uint32_t cand2 = lane == wl ? (uint32_t)d2 : (k1 == ~0u ? ~0u : (k1 >> 16));
                    const uint32_t m2 = wave_min_u32(cand2);
                    fbest2 = m2 >= (uint32_t)INT_MAX ? INT_MAX : (int)m2;
                }
                if (fbest <= kThLow && (float)fbest < __fmul_rn((float)fbest2, nnr) && lane == 0) {
                    const int old = s.m21[fg];
                    if (old >= 0) s.m12[old] = -1;
                    s.m12[qf] = (int16_t)fg;
                    s.m21[fg] = (int16_t)qf;
                    s.mdist[fg] = (int16_t)fbest;
                    s.acc[qf] = (int16_t)fg;
                }
                wave_lds_fence();
                ++P;
            }
        }
        __builtin_amdgcn_s_setprio(0);
    }
    __syncthreads();
    if (clk) mb.clocks[4] = clock64();

    // ---- 4. rotation histogram of every accepted pair (rotHist, ORBmatcher.cc:475-483),
    //         ComputeThreeMaxima, consistency filter and outputs (:494-520)
    if (mb.check_ori) {
        const float factor = 1.0f / kHisto;
        for (int q = tid; q < nq; q += kMT) {
            const int a = s.acc[q];
            if (a < 0) continue;
            float rot = __fsub_rn(k1[s.qidx[q]].angle, k2[s.glist[a]].angle);
            if (rot < 0.0f) rot = __fadd_rn(rot, 360.0f);
            int bin = (int)roundf(__fmul_rn(rot, factor));
            if (bin == kHisto) bin = 0;
            s.rbin[q] = (int8_t)bin;
            atomicAdd(&hist[bin], 1);
        }
    }
    __syncthreads();
    if (tid == 0) {
        if (mb.check_ori) {
            int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
            for (int i = 0; i < kHisto; ++i) {
                const int sz = hist[i];
                if (sz > max1) { max3 = max2; max2 = max1; max1 = sz; ind3 = ind2; ind2 = ind1; ind1 = i; }
                else if (sz > max2) { max3 = max2; max2 = sz; ind3 = ind2; ind2 = i; }
                else if (sz > max3) { max3 = sz; ind3 = i; }
            }
            if ((float)max2 < __fmul_rn(0.1f, (float)max1)) { ind2 = -1; ind3 = -1; }
            else if ((float)max3 < __fmul_rn(0.1f, (float)max1)) { ind3 = -1; }
            sh_top[0] = ind1; sh_top[1] = ind2; sh_top[2] = ind3;
        }
    }
    __syncthreads();
    int local = 0;
    for (int q = tid; q < nq; q += kMT) {
        const int g = s.m12[q];
        if (g < 0) continue;
        if (mb.check_ori) {
            const int bin = s.rbin[q];
            if (bin >= 0 && bin != sh_top[0] && bin != sh_top[1] && bin != sh_top[2]) continue;
        }
        const int i1 = s.qidx[q], i2 = s.glist[g];
        out12[i1] = i2;
        prev[2 * i1] = s.gxy[g].x;
        prev[2 * i1 + 1] = s.gxy[g].y;
        ++local;
    }
    int total;
    block_scan_i32(local, &total, ws);
    if (tid == 0) mb.nmatches[b] = sh_err ? -1 : total;
    if (clk) mb.clocks[5] = clock64();
    host_tail(mb.tail);
}

}  // namespace

// LDS of one frame pair (n1cap / n2cap: kept for the callers; the layout
// is indexed by query rank and grid position only).
int match_lds_bytes(int n1cap, int n2cap, int maxq, int maxc) {
    (void)n1cap; (void)n2cap;
    return (int)(40 * maxc + 8 * maxq + 8 + 16 * maxq + 4 * maxc + sizeof(uint16_t) * (kBuckets + 2) +
                 sizeof(int16_t) * (4 * ((maxc + 1) & ~1) + 4 * ((maxq + 1) & ~1)) + maxq + 64);
}

constexpr int kMatchLdsMax = 160 * 1024 - 1024;   // dynamic LDS; the kernel's static LDS needs < 1 KiB

hipError_t launch_match(const MatchBufs &mb, int B, int n1cap, int n2cap, int maxq, int maxc, hipStream_t st) {
    const int bytes = match_lds_bytes(n1cap, n2cap, maxq, maxc);
    if (bytes > kMatchLdsMax) return hipErrorInvalidValue;
    if (bytes > 64 * 1024 &&
        hipFuncSetAttribute(reinterpret_cast<const void *>(k_search_init),
                            hipFuncAttributeMaxDynamicSharedMemorySize, bytes) != hipSuccess)
        return hipErrorInvalidValue;
    if (mb.tail.flag && mb.tail.blocks != B) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_search_init, dim3(B), dim3(kMT), bytes, st, mb, maxq, maxc);
    return hipGetLastError();
}

}  // namespace orbx
