// orbx_match.hip -- ORBmatcher::SearchForInitialization on gfx950.
//
// Reference: ORBmatcher.cc:406-521 (+ ComputeThreeMaxima :1603-1644,
// DescriptorDistance :1649-1665), Frame::AssignFeaturesToGrid / PosInGrid /
// GetFeaturesInArea (Frame.cc:239-256, 415-425, 354-412).
//
// One 256-thread workgroup per frame pair.  The work that carries no
// dependency -- grid build, window enumeration, filters, all Hamming distances
// -- runs on every wave; the reference's greedy loop (its vMatchedDistance /
// vnMatches21 state makes query i1 depend on every earlier one) is replayed in
// order by a single wave that evaluates each query's candidates 64 at a time
// with ballot/min reductions, keeping the exact tie semantics (first minimum
// wins; second-best is the multiset second minimum).
#include <hip/hip_runtime.h>

#include <climits>

#include "orbx_device.h"

namespace orbx {
namespace {

constexpr int kGridCols = 64, kGridRows = 48;  // Frame.h:37-38
constexpr int kGridCells = kGridCols * kGridRows;
constexpr int kHisto = 30;                      // ORBmatcher::HISTO_LENGTH
constexpr int kThLow = 50;                      // ORBmatcher::TH_LOW
constexpr int kSkip = 0xFFFF;

__device__ inline int hamming(const uint8_t *a, const uint8_t *b) {
    const uint4 *pa = reinterpret_cast<const uint4 *>(a);
    const uint4 *pb = reinterpret_cast<const uint4 *>(b);
    const uint4 x0 = pa[0], x1 = pa[1], y0 = pb[0], y1 = pb[1];
    return __popc(x0.x ^ y0.x) + __popc(x0.y ^ y0.y) + __popc(x0.z ^ y0.z) + __popc(x0.w ^ y0.w) +
           __popc(x1.x ^ y1.x) + __popc(x1.y ^ y1.y) + __popc(x1.z ^ y1.z) + __popc(x1.w ^ y1.w);
}

__device__ inline int wave_incl_scan_i32(int v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int o = __shfl_up(v, d, 64);
        if (lane >= d) v += o;
    }
    return v;
}

__device__ inline uint64_t wave_min_u64(uint64_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, d, 64);
        const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), d, 64);
        const uint64_t o = ((uint64_t)hi << 32) | lo;
        v = o < v ? o : v;
    }
    return v;
}

struct MLds {
    int *gstart;    // kGridCells + 1
    int *gfill;     // kGridCells
    int16_t *glist; // n2cap
    int16_t *kcell_or_rank;
    int *mdist;     // n2cap
    int *m21;       // n2cap
    int *m12;       // n1cap
    int8_t *rbin;   // n1cap
    int *qrank;     // n1cap (rank among octave-0 queries, or -1)
    int *qcount;    // n1cap
};

__global__ __launch_bounds__(256) void k_search_init(MatchBufs mb, int n1cap, int n2cap, int maxq, int maxc) {
    extern __shared__ __align__(16) uint8_t lds[];
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const orbx_keypoint *k1 = mb.k1 + (int64_t)b * mb.k1_stride;
    const orbx_keypoint *k2 = mb.k2 + (int64_t)b * mb.k2_stride;
    const uint8_t *d1 = mb.d1 + (int64_t)b * mb.k1_stride * 32;
    const uint8_t *d2 = mb.d2 + (int64_t)b * mb.k2_stride * 32;
    const int n1 = min(mb.n1[b], n1cap), n2 = min(mb.n2[b], n2cap);
    float *prev = mb.prev_xy + (int64_t)b * mb.k1_stride * 2;
    int32_t *out12 = mb.matches12 + (int64_t)b * mb.k1_stride;
    uint32_t *scratch = mb.scratch + (int64_t)b * mb.scratch_stride;

    MLds s;
    uint8_t *ptr = lds;
    s.gstart = reinterpret_cast<int *>(ptr); ptr += sizeof(int) * (kGridCells + 1);
    s.gfill = reinterpret_cast<int *>(ptr); ptr += sizeof(int) * kGridCells;
    s.mdist = reinterpret_cast<int *>(ptr); ptr += sizeof(int) * n2cap;
    s.m21 = reinterpret_cast<int *>(ptr); ptr += sizeof(int) * n2cap;
    s.m12 = reinterpret_cast<int *>(ptr); ptr += sizeof(int) * n1cap;
    s.qrank = reinterpret_cast<int *>(ptr); ptr += sizeof(int) * n1cap;
    s.qcount = reinterpret_cast<int *>(ptr); ptr += sizeof(int) * n1cap;
    s.glist = reinterpret_cast<int16_t *>(ptr); ptr += sizeof(int16_t) * n2cap;
    s.kcell_or_rank = reinterpret_cast<int16_t *>(ptr); ptr += sizeof(int16_t) * n2cap;
    s.rbin = reinterpret_cast<int8_t *>(ptr); ptr += n1cap;
    __shared__ int hist[kHisto];
    __shared__ int ws[4];
    __shared__ int sh_top[3];
    __shared__ int sh_err;

    // Frame grid constants for an undistorted img_w x img_h image
    // (Frame.cc:218-220, ComputeImageBounds with k1 == 0).
    const float minX = 0.f, maxX = (float)mb.img_w, minY = 0.f, maxY = (float)mb.img_h;
    const float invW = __fdiv_rn((float)kGridCols, __fsub_rn(maxX, minX));
    const float invH = __fdiv_rn((float)kGridRows, __fsub_rn(maxY, minY));
    const float r = (float)mb.window;

    // ---- 0. init
    for (int i = tid; i <= kGridCells; i += 256) s.gstart[i] = 0;
    for (int i = tid; i < kGridCells; i += 256) s.gfill[i] = 0;
    for (int i = tid; i < n2; i += 256) { s.mdist[i] = INT_MAX; s.m21[i] = -1; }
    for (int i = tid; i < n1; i += 256) { s.m12[i] = -1; s.rbin[i] = -1; s.qcount[i] = 0; }
    if (tid < kHisto) hist[tid] = 0;
    if (tid == 0) sh_err = 0;
    if (mb.reset_prev) {
        for (int i = tid; i < n1; i += 256) { prev[2 * i] = k1[i].x; prev[2 * i + 1] = k1[i].y; }
    }
    __syncthreads();

    // ---- 1. grid of F2's octave-0 keypoints (PosInGrid uses round(), Frame.cc:417-418)
    for (int i = tid; i < n2; i += 256) {
        int cell = -1;
        if (k2[i].octave == 0) {
            const int px = (int)roundf(__fmul_rn(__fsub_rn(k2[i].x, minX), invW));
            const int py = (int)roundf(__fmul_rn(__fsub_rn(k2[i].y, minY), invH));
            if (px >= 0 && px < kGridCols && py >= 0 && py < kGridRows) {
                cell = px * kGridRows + py;
                atomicAdd(&s.gstart[cell], 1);
            }
        }
        s.kcell_or_rank[i] = (int16_t)cell;
    }
    __syncthreads();
    {
        // exclusive scan of the 3072 counts (12 per thread, contiguous)
        const int per = kGridCells / 256;
        int local = 0;
        for (int i = 0; i < per; ++i) local += s.gstart[tid * per + i];
        const int incl = wave_incl_scan_i32(local);
        if (lane == 63) ws[wave] = incl;
        __syncthreads();
        int base = 0;
        for (int w = 0; w < wave; ++w) base += ws[w];
        int run = base + incl - local;
        for (int i = 0; i < per; ++i) {
            const int v = s.gstart[tid * per + i];
            s.gstart[tid * per + i] = run;
            run += v;
        }
        if (tid == 255) s.gstart[kGridCells] = run;
        __syncthreads();
    }
    for (int i = tid; i < n2; i += 256) {
        const int cell = s.kcell_or_rank[i];
        if (cell >= 0) {
            const int pos = atomicAdd(&s.gfill[cell], 1);
            s.glist[s.gstart[cell] + pos] = (int16_t)i;
        }
    }
    __syncthreads();
    // keep each cell's list in keypoint-index order (mGrid push_back order)
    for (int c = tid; c < kGridCells; c += 256) {
        const int st = s.gstart[c], en = s.gstart[c + 1];
        for (int a = st + 1; a < en; ++a) {
            const int16_t v = s.glist[a];
            int j = a - 1;
            while (j >= st && s.glist[j] > v) { s.glist[j + 1] = s.glist[j]; --j; }
            s.glist[j + 1] = v;
        }
    }
    // rank of each octave-0 query in F1 (scratch row index)
    {
        const int per = (n1 + 255) / 256;
        const int st = min(tid * per, n1), en = min(st + per, n1);
        int local = 0;
        for (int i = st; i < en; ++i) local += k1[i].octave == 0;
        const int incl = wave_incl_scan_i32(local);
        if (lane == 63) ws[wave] = incl;
        __syncthreads();
        int base = 0;
        for (int w = 0; w < wave; ++w) base += ws[w];
        int run = base + incl - local;
        for (int i = st; i < en; ++i) {
            s.qrank[i] = k1[i].octave == 0 ? run : -1;
            run += k1[i].octave == 0;
        }
        __syncthreads();
    }

    // ---- 2. candidate lists + distances (GetFeaturesInArea order: ix outer,
    //         iy inner, cell insertion order; |dx| < r and |dy| < r).
    for (int i1 = wave; i1 < n1; i1 += 4) {
        const int q = s.qrank[i1];
        if (q < 0) continue;
        if (q >= maxq) { if (lane == 0) sh_err = 1; continue; }
        const float x = prev[2 * i1], y = prev[2 * i1 + 1];
        const int cx0 = max(0, (int)floorf(__fmul_rn(__fsub_rn(__fsub_rn(x, minX), r), invW)));
        const int cx1 = min(kGridCols - 1, (int)ceilf(__fmul_rn(__fadd_rn(__fsub_rn(x, minX), r), invW)));
        const int cy0 = max(0, (int)floorf(__fmul_rn(__fsub_rn(__fsub_rn(y, minY), r), invH)));
        const int cy1 = min(kGridRows - 1, (int)ceilf(__fmul_rn(__fadd_rn(__fsub_rn(y, minY), r), invH)));
        if (cx0 >= kGridCols || cx1 < 0 || cy0 >= kGridRows || cy1 < 0 || cx1 < cx0 || cy1 < cy0) continue;
        const int ncy = cy1 - cy0 + 1;
        const int ncells = (cx1 - cx0 + 1) * ncy;
        const uint8_t *q1 = d1 + (int64_t)i1 * 32;
        uint32_t *list = scratch + (int64_t)q * maxc;
        int written = 0;
        for (int c0 = 0; c0 < ncells; c0 += 64) {
            const int cidx = c0 + lane;
            int st = 0, cnt = 0;
            if (cidx < ncells) {
                const int ix = cx0 + cidx / ncy, iy = cy0 + cidx % ncy;
                const int cell = ix * kGridRows + iy;
                st = s.gstart[cell];
                cnt = s.gstart[cell + 1] - st;
            }
            const int incl = wave_incl_scan_i32(cnt);
            const int tot = __shfl(incl, 63, 64);
            const int pos0 = written + incl - cnt;
            for (int e = 0; e < cnt; ++e) {
                const int i2 = s.glist[st + e];
                const float dx = __fsub_rn(k2[i2].x, x), dy = __fsub_rn(k2[i2].y, y);
                int dist = kSkip;
                if (fabsf(dx) < r && fabsf(dy) < r) dist = hamming(q1, d2 + (int64_t)i2 * 32);
                if (pos0 + e < maxc) list[pos0 + e] = ((uint32_t)i2 << 16) | (uint32_t)dist;
            }
            written += tot;
        }
        if (written > maxc) { if (lane == 0) sh_err = 1; written = maxc; }
        if (lane == 0) s.qcount[i1] = written;
    }
    __syncthreads();

    // ---- 3. ordered greedy replay (ORBmatcher.cc:425-491), wave 0 only
    if (wave == 0) {
        const float factor = 1.0f / kHisto;
        for (int i1 = 0; i1 < n1; ++i1) {
            const int q = s.qrank[i1];
            if (q < 0 || q >= maxq) continue;
            const int cnt = s.qcount[i1];
            if (cnt == 0) continue;
            const uint32_t *list = scratch + (int64_t)q * maxc;
            int best = INT_MAX, best2 = INT_MAX, best_i2 = -1;
            for (int c0 = 0; c0 < cnt; c0 += 64) {
                const int e = c0 + lane;
                uint64_t key = ~0ull;
                int dist = INT_MAX, i2 = -1;
                if (e < cnt) {
                    const uint32_t v = list[e];
                    i2 = (int)(v >> 16);
                    dist = (int)(v & 0xFFFF);
                    if (dist == kSkip || s.mdist[i2] <= dist) dist = INT_MAX;
                    else key = ((uint64_t)dist << 32) | (uint32_t)e;
                }
                const uint64_t mn = wave_min_u64(key);
                if (mn == ~0ull) continue;
                const int cb = (int)(mn >> 32);
                const int cb_lane = (int)(mn & 0xFFFFFFFF) - c0;
                const int cb_i2 = __shfl(i2, cb_lane, 64);
                // second smallest of this chunk's valid distances (multiset)
                const uint64_t key2 = (lane == cb_lane || dist == INT_MAX) ? ~0ull : (uint64_t)dist;
                const uint64_t mn2 = wave_min_u64(key2);
                const int cs = mn2 == ~0ull ? INT_MAX : (int)mn2;
                // merge (running result precedes this chunk)
                const int nb = best <= cb ? best : cb;
                const int hi = best <= cb ? cb : best;
                best2 = min(hi, min(best2, cs));
                if (cb < best) best_i2 = cb_i2;
                best = nb;
            }
            if (best <= kThLow && (float)best < __fmul_rn((float)best2, mb.nnratio)) {
                if (lane == 0) {
                    const int old = s.m21[best_i2];
                    if (old >= 0) s.m12[old] = -1;
                    s.m12[i1] = best_i2;
                    s.m21[best_i2] = i1;
                    s.mdist[best_i2] = best;
                    if (mb.check_ori) {
                        float rot = __fsub_rn(k1[i1].angle, k2[best_i2].angle);
                        if (rot < 0.0f) rot = __fadd_rn(rot, 360.0f);
                        int bin = (int)roundf(__fmul_rn(rot, factor));
                        if (bin == kHisto) bin = 0;
                        s.rbin[i1] = (int8_t)bin;
                        hist[bin] += 1;
                    }
                }
                __builtin_amdgcn_s_waitcnt(0);
                __builtin_amdgcn_wave_barrier();
            }
        }
        if (lane == 0 && mb.check_ori) {
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

    // ---- 4. rotation-consistency filter and outputs (ORBmatcher.cc:494-520)
    int local = 0;
    for (int i1 = tid; i1 < n1; i1 += 256) {
        int m = s.m12[i1];
        if (mb.check_ori && m >= 0) {
            const int bin = s.rbin[i1];
            if (bin >= 0 && bin != sh_top[0] && bin != sh_top[1] && bin != sh_top[2]) m = -1;
        }
        out12[i1] = m;
        if (m >= 0) {
            prev[2 * i1] = k2[m].x;
            prev[2 * i1 + 1] = k2[m].y;
            ++local;
        }
    }
    local = wave_incl_scan_i32(local);
    if (lane == 63) ws[wave] = local;
    __syncthreads();
    if (tid == 0) mb.nmatches[b] = sh_err ? -1 : ws[0] + ws[1] + ws[2] + ws[3];
}

}  // namespace

int match_lds_bytes(int n1cap, int n2cap) {
    return (int)(sizeof(int) * (2 * kGridCells + 1) + sizeof(int) * 2 * n2cap + sizeof(int) * 3 * n1cap +
                 sizeof(int16_t) * 2 * n2cap + n1cap + 64);
}

hipError_t launch_match(const MatchBufs &mb, int B, int n1cap, int n2cap, int maxq, int maxc, hipStream_t st) {
    const int bytes = match_lds_bytes(n1cap, n2cap);
    hipLaunchKernelGGL(k_search_init, dim3(B), dim3(256), bytes, st, mb, n1cap, n2cap, maxq, maxc);
    return hipGetLastError();
}

}  // namespace orbx
