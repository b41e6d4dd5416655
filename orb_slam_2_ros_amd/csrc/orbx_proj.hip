// orbx_proj.hip -- ORBmatcher's projection searches on gfx950:
// SearchByProjection x4 and the candidate search of Fuse x2
// (ORBmatcher.cc:45-129, 291-404, 827-1102, 1330-1601; GetFeaturesInArea
// Frame.cc:354-412 / KeyFrame.cc:700-739; ComputeThreeMaxima :1603-1644).
//
// One 1024-thread workgroup per call.  The frame's 64x48 grid (positions,
// octaves, mvuRight, map-point state) is built in LDS.  Every wave then takes
// queries in turn and expands the query's window into candidate entries, one
// lane per entry.  The static filters (level range, window, stereo gate, Fuse's
// reprojection test) and the Hamming distances are evaluated here, and the
// query's 4 smallest (distance, candidate position) entries are kept.
//
// The reference assigns keypoints greedily in query order: a keypoint taken by
// an earlier point is skipped by later ones.  That dependency is replayed by
// wave 0 in query order; each query needs only its first one (best-only
// variants) or two (SearchByProjection(Frame&, vector<MapPoint*>&)) still-free
// entries in (distance, position) order.  Those come from the 4 kept entries,
// or from a 64-wide scan of the query's full list when too few are free.
// Fuse has no such dependency (its map edits stay with the caller), so its
// queries finish in the parallel phase.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>

#include "orbx_device.h"
#include "orbx_wave.h"

namespace orbx {
namespace {

constexpr int kPT = 1024, kPW = kPT / 64;
constexpr int kGC = 64, kGR = 48, kCells = kGC * kGR;
constexpr int kHist = 30;
constexpr int kEnt = 512;                 // per-wave entry map (candidate -> grid column)
constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr int kBadDist = 0x1FF;           // entry failed a static filter

// list entry: keypoint index | octave << 16 | distance << 20
__device__ inline uint32_t entry(int idx, int oct, int dist) {
    return (uint32_t)idx | ((uint32_t)(oct & 0xF) << 16) | ((uint32_t)dist << 20);
}
__device__ inline int e_idx(uint32_t e) { return (int)(e & 0xFFFF); }
__device__ inline int e_oct(uint32_t e) { return (int)((e >> 16) & 0xF); }
__device__ inline int e_dist(uint32_t e) { return (int)(e >> 20); }

struct PLds {
    int *gstart;      // kCells + 1
    int *gfill;       // kCells
    float2 *gxy;      // n, by grid position
    float *gur;       // n, mvuRight by grid position
    int16_t *glist;   // n, keypoint index by grid position
    int16_t *kcell;   // n
    int8_t *goct;     // n, octave by grid position
    uint8_t *state;   // n, by keypoint index: bit0 has a point, bit1 it blocks
    uint8_t *entmap;  // kPW x kEnt
    uint32_t *pool;   // pool_cap list entries
};

__device__ inline PLds carve(uint8_t *p, int n, int pool_cap) {
    PLds s;
    auto take = [&](size_t bytes) { uint8_t *r = p; p += (bytes + 15) & ~size_t(15); return r; };
    s.gstart = reinterpret_cast<int *>(take(4 * (kCells + 1)));
    s.gfill = reinterpret_cast<int *>(take(4 * kCells));
    s.gxy = reinterpret_cast<float2 *>(take(8 * (size_t)n));
    s.gur = reinterpret_cast<float *>(take(4 * (size_t)n));
    s.glist = reinterpret_cast<int16_t *>(take(2 * (size_t)n));
    s.kcell = reinterpret_cast<int16_t *>(take(2 * (size_t)n));
    s.goct = reinterpret_cast<int8_t *>(take((size_t)n));
    s.state = reinterpret_cast<uint8_t *>(take((size_t)n));
    s.entmap = take((size_t)kPW * kEnt);
    s.pool = reinterpret_cast<uint32_t *>(take(4 * (size_t)pool_cap));
    return s;
}

__device__ inline int hamming_q(const uint4 a0, const uint4 a1, const uint8_t *d) {
    const uint4 b0 = *reinterpret_cast<const uint4 *>(d);
    const uint4 b1 = *reinterpret_cast<const uint4 *>(d + 16);
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

__device__ inline int block_scan(int v, int *total, int *ws) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int incl = wave_incl_scan_i32(v);
    if (lane == 63) ws[wave] = incl;
    __syncthreads();
    int base = 0, tot = 0;
    for (int w = 0; w < kPW; ++w) {
        if (w < wave) base += ws[w];
        tot += ws[w];
    }
    __syncthreads();
    *total = tot;
    return base + incl - v;
}

__global__ __launch_bounds__(kPT) void k_proj_match(ProjBufs a) {
    extern __shared__ __align__(16) uint8_t lds[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int n = a.n, nq = a.nq;
    const PLds s = carve(lds, n, a.pool_cap);
    __shared__ int ws[kPW];
    __shared__ int hist[kHist];
    __shared__ int sh_pool, sh_acc, sh_removed, sh_top[3];
    const int V = a.variant;
    const bool fuse = V == ORBX_PROJ_FUSE || V == ORBX_PROJ_FUSE_SIM3;
    const bool occ_obs = V == ORBX_PROJ_LOCALMAP || V == ORBX_PROJ_LASTFRAME;   // skip: has && Observations() > 0
    const bool ratio = V == ORBX_PROJ_LOCALMAP;
    const bool use_ori = a.check_ori && (V == ORBX_PROJ_LASTFRAME || V == ORBX_PROJ_KEYFRAME);
    const float invW = __fdiv_rn((float)kGC, __fsub_rn(a.max_x, a.min_x));
    const float invH = __fdiv_rn((float)kGR, __fsub_rn(a.max_y, a.min_y));

    // ---- 0. init
    for (int i = tid; i <= kCells; i += kPT) s.gstart[i] = 0;
    for (int i = tid; i < kCells; i += kPT) s.gfill[i] = 0;
    for (int i = tid; i < n; i += kPT) {
        s.state[i] = a.mp_state ? (a.mp_state[i] & 3) : 0;
        a.kp_final[i] = -1;
    }
    for (int i = tid; i < nq; i += kPT) {
        a.q_idx[i] = -1;
        a.q_dist[i] = -1;
        a.qlen[i] = 0;   // queries with an empty window never reach phase 2's stores
        a.qbase[i] = -1;
        reinterpret_cast<uint4 *>(a.qtop)[i] = make_uint4(kNone, kNone, kNone, kNone);
    }
    if (tid < kHist) hist[tid] = 0;
    if (tid == 0) { sh_pool = 0; sh_acc = 0; sh_removed = 0; }
    __syncthreads();

    // ---- 1. grid: counting sort by cell, then index order inside each cell
    for (int i = tid; i < n; i += kPT) {
        const orbx_keypoint k = a.keys[i];
        const int px = (int)roundf(__fmul_rn(__fsub_rn(k.x, a.min_x), invW));
        const int py = (int)roundf(__fmul_rn(__fsub_rn(k.y, a.min_y), invH));
        int cell = -1;
        if (px >= 0 && px < kGC && py >= 0 && py < kGR) {
            cell = px * kGR + py;
            atomicAdd(&s.gstart[cell], 1);
        }
        s.kcell[i] = (int16_t)cell;
    }
    __syncthreads();
    {
        constexpr int per = kCells / kPT;
        int local = 0;
        for (int i = 0; i < per; ++i) local += s.gstart[tid * per + i];
        int tot;
        int run = block_scan(local, &tot, ws);
        for (int i = 0; i < per; ++i) {
            const int v = s.gstart[tid * per + i];
            s.gstart[tid * per + i] = run;
            run += v;
        }
        if (tid == kPT - 1) s.gstart[kCells] = run;
        __syncthreads();
    }
    for (int i = tid; i < n; i += kPT) {
        const int cell = s.kcell[i];
        if (cell >= 0) s.glist[s.gstart[cell] + atomicAdd(&s.gfill[cell], 1)] = (int16_t)i;
    }
    __syncthreads();
    for (int c = tid; c < kCells; c += kPT) {
        const int st = s.gstart[c], en = s.gstart[c + 1];
        for (int x = st + 1; x < en; ++x) {
            const int16_t v = s.glist[x];
            int j = x - 1;
            while (j >= st && s.glist[j] > v) { s.glist[j + 1] = s.glist[j]; --j; }
            s.glist[j + 1] = v;
        }
    }
    __syncthreads();
    const int ngrid = s.gstart[kCells];
    for (int g = tid; g < ngrid; g += kPT) {
        const int i = s.glist[g];
        const orbx_keypoint k = a.keys[i];
        s.gxy[g] = make_float2(k.x, k.y);
        s.goct[g] = (int8_t)k.octave;
        s.gur[g] = a.uright ? a.uright[i] : -1.0f;
    }
    __syncthreads();

    // ---- 2. window expansion, static filters, distances, 4 smallest per query
    uint8_t *emap = s.entmap + wave * kEnt;
    for (int q = wave; q < nq; q += kPW) {
        const orbx_proj_query Q = a.q[q];
        if (!(Q.flags & ORBX_QUERY_ACTIVE)) continue;
        const float x = Q.u, y = Q.v, r = Q.radius;
        // Frame::GetFeaturesInArea cell range (float, as the reference)
        const int cx0 = max(0, (int)floorf(__fmul_rn(__fsub_rn(__fsub_rn(x, a.min_x), r), invW)));
        const int cx1 = min(kGC - 1, (int)ceilf(__fmul_rn(__fadd_rn(__fsub_rn(x, a.min_x), r), invW)));
        const int cy0 = max(0, (int)floorf(__fmul_rn(__fsub_rn(__fsub_rn(y, a.min_y), r), invH)));
        const int cy1 = min(kGR - 1, (int)ceilf(__fmul_rn(__fadd_rn(__fsub_rn(y, a.min_y), r), invH)));
        if (cx0 >= kGC || cx1 < 0 || cy0 >= kGR || cy1 < 0 || cx1 < cx0 || cy1 < cy0) continue;
        const int ncx = cx1 - cx0 + 1;   // <= 64
        int st = 0, cnt = 0;
        if (lane < ncx) {
            const int col = (cx0 + lane) * kGR;
            st = s.gstart[col + cy0];
            cnt = s.gstart[col + cy1 + 1] - st;
        }
        const int incl = wave_incl_scan_i32(cnt);
        const int pos0 = incl - cnt;
        const int T = __builtin_amdgcn_readlane(incl, 63);
        if (T == 0) continue;
        int base = -1;
        if (lane == 0) {
            base = atomicAdd(&sh_pool, T);
            if (base + T > a.pool_cap) base = -1;
        }
        base = __builtin_amdgcn_readfirstlane(base);
        uint32_t *list = base >= 0 ? s.pool + base : a.spill + (int64_t)q * a.spill_stride;
        const uint4 qa = *reinterpret_cast<const uint4 *>(a.qdesc + 32 * (int64_t)q);
        const uint4 qb = *reinterpret_cast<const uint4 *>(a.qdesc + 32 * (int64_t)q + 16);
        const bool check_lv = Q.min_level > 0 || Q.max_level >= 0;
        uint32_t tk[4] = {kNone, kNone, kNone, kNone};   // (dist << 16 | position) of this lane's 4 smallest
        uint32_t te[4] = {0, 0, 0, 0};                   // their entries
        for (int E0 = 0; E0 < T; E0 += kEnt) {
            // entry -> column map of this piece of the list
            const int lo = max(pos0, E0), hi = min(pos0 + cnt, E0 + kEnt);
            for (int t = lo; t < hi; ++t) emap[t - E0] = (uint8_t)lane;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const int pend = min(T, E0 + kEnt);
            for (int t0 = E0; t0 < pend; t0 += 64) {
                const int t = t0 + lane;
                const int c = t < pend ? emap[t - E0] : 0;
                const int cst = __shfl(st, c, 64), cp0 = __shfl(pos0, c, 64);
                uint32_t ent = kNone;
                if (t < pend) {
                    const int gp = cst + (t - cp0);
                    const int i2 = s.glist[gp];
                    const float2 kp = s.gxy[gp];
                    const int oct = s.goct[gp];
                    bool ok = true;
                    if (check_lv) {
                        if (oct < Q.min_level) ok = false;
                        if (Q.max_level >= 0 && oct > Q.max_level) ok = false;
                    }
                    const float dx = __fsub_rn(kp.x, x), dy = __fsub_rn(kp.y, y);
                    if (!(fabsf(dx) < r && fabsf(dy) < r)) ok = false;
                    if (ok && (V == ORBX_PROJ_LOCALMAP || V == ORBX_PROJ_LASTFRAME)) {
                        const float ur = s.gur[gp];
                        if (ur > 0.0f && fabsf(__fsub_rn(Q.ur, ur)) > Q.ur_tol) ok = false;
                    } else if (ok && V == ORBX_PROJ_FUSE) {
                        // ORBmatcher.cc:903-932: chi-square gate on the reprojection error
                        const float ur = s.gur[gp];
                        const float ex = __fsub_rn(x, kp.x), ey = __fsub_rn(y, kp.y);
                        const float isg = oct >= 0 && oct < a.nlevels ? a.inv_sigma2[oct] : 0.0f;
                        if (ur >= 0.0f) {
                            const float er = __fsub_rn(Q.ur, ur);
                            const float e2 = __fadd_rn(__fadd_rn(__fmul_rn(ex, ex), __fmul_rn(ey, ey)), __fmul_rn(er, er));
                            if ((double)__fmul_rn(e2, isg) > 7.8) ok = false;
                        } else {
                            const float e2 = __fadd_rn(__fmul_rn(ex, ex), __fmul_rn(ey, ey));
                            if ((double)__fmul_rn(e2, isg) > 5.99) ok = false;
                        }
                    }
                    const int dist = ok ? hamming_q(qa, qb, a.desc + 32 * (int64_t)i2) : kBadDist;
                    ent = entry(i2, oct, dist);
                    list[t] = ent;
                    if (ok) {
                        uint32_t k = ((uint32_t)dist << 16) | (uint32_t)t;
                        uint32_t ke = ent;
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            if (k < tk[j]) {
                                const uint32_t t1 = tk[j]; tk[j] = k; k = t1;
                                const uint32_t t2 = te[j]; te[j] = ke; ke = t2;
                            }
                        }
                    }
                }
                (void)ent;
            }
            __builtin_amdgcn_wave_barrier();
        }
        uint32_t top[4];
        for (int j = 0; j < 4; ++j) {
            const uint32_t mn = wave_min_u32(tk[0]);
            const bool mine = tk[0] == mn && mn != kNone;
            const uint64_t who = __ballot(mine);
            uint32_t e = kNone;
            if (who) e = (uint32_t)__builtin_amdgcn_readlane((int)te[0], (int)__builtin_ctzll(who));
            if (mine) { tk[0] = tk[1]; tk[1] = tk[2]; tk[2] = tk[3]; tk[3] = kNone; te[0] = te[1]; te[1] = te[2]; te[2] = te[3]; }
            top[j] = e;
        }
        if (fuse) {
            // best only, no keypoint state: decided here (INT_MAX / 256 start both
            // reject a 256 distance against TH_LOW)
            if (lane == 0 && top[0] != kNone && e_dist(top[0]) <= a.th_dist) {
                a.q_idx[q] = e_idx(top[0]);
                a.q_dist[q] = e_dist(top[0]);
            }
        } else if (lane == 0) {
            uint4 t4;
            t4.x = top[0]; t4.y = top[1]; t4.z = top[2]; t4.w = top[3];
            reinterpret_cast<uint4 *>(a.qtop)[q] = t4;
            a.qlen[q] = T;
            a.qbase[q] = base;
        }
    }
    __syncthreads();

    // ---- 3. greedy assignment in query order (wave 0)
    if (!fuse && wave == 0) {
        int accepted = 0;
        for (int g0 = 0; g0 < nq; g0 += 64) {
            const int gq = g0 + lane;
            uint4 t4 = make_uint4(kNone, kNone, kNone, kNone);
            int len = 0, qb = -1, qblk = 0;
            bool live = false;
            if (gq < nq) {
                const orbx_proj_query Q = a.q[gq];
                qblk = (Q.flags & ORBX_QUERY_BLOCKS) ? 2 : 0;
                if (Q.flags & ORBX_QUERY_ACTIVE) {
                    t4 = reinterpret_cast<const uint4 *>(a.qtop)[gq];
                    len = a.qlen[gq];
                    qb = a.qbase[gq];
                    // nothing at or under th_dist: no state change possible
                    live = len > 0 && t4.x != kNone && e_dist(t4.x) <= a.th_dist;
                }
            }
            uint64_t todo = __ballot(live);
            while (todo) {
                const int j = (int)__builtin_ctzll(todo);
                todo &= todo - 1;
                const int q = g0 + j;
                const uint32_t e4[4] = {(uint32_t)__builtin_amdgcn_readlane((int)t4.x, j),
                                        (uint32_t)__builtin_amdgcn_readlane((int)t4.y, j),
                                        (uint32_t)__builtin_amdgcn_readlane((int)t4.z, j),
                                        (uint32_t)__builtin_amdgcn_readlane((int)t4.w, j)};
                const int blocks = __builtin_amdgcn_readlane(qblk, j);
                int st4[4];
#pragma unroll
                for (int t = 0; t < 4; ++t) st4[t] = e4[t] == kNone ? 0 : s.state[e_idx(e4[t])];
                const int need = ratio ? 2 : 1;
                uint32_t got[2] = {kNone, kNone};
                int found = 0;
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    if (e4[t] == kNone || found == need) continue;
                    const bool taken = occ_obs ? (st4[t] == 3) : (st4[t] & 1);
                    if (taken) continue;
                    got[found++] = e4[t];
                }
                if (found < need && e4[3] != kNone) {
                    // more entries than the 4 kept: scan the whole list
                    const int cnt = __builtin_amdgcn_readlane(len, j);
                    const int lb = __builtin_amdgcn_readlane(qb, j);
                    const uint32_t *list = lb >= 0 ? s.pool + lb : a.spill + (int64_t)q * a.spill_stride;
                    uint32_t k1 = kNone, k2 = kNone;   // (dist << 16 | position), two smallest free
                    uint32_t x1 = kNone, x2 = kNone;
                    for (int c0 = 0; c0 < cnt; c0 += 64) {
                        const int e = c0 + lane;
                        uint32_t key = kNone, ent = kNone;
                        if (e < cnt) {
                            ent = list[e];
                            const int d = e_dist(ent);
                            const int stt = s.state[e_idx(ent)];
                            const bool taken = occ_obs ? (stt == 3) : (stt & 1);
                            if (d != kBadDist && !taken) key = ((uint32_t)d << 16) | (uint32_t)e;
                        }
                        const uint32_t m1 = wave_min_u32(key);
                        if (m1 == kNone) continue;
                        const int l1 = (int)(m1 & 0xFFFF) - c0;
                        const uint32_t ent1 = (uint32_t)__builtin_amdgcn_readlane((int)ent, l1);
                        const uint32_t m2 = wave_min_u32(lane == l1 ? kNone : key);
                        uint32_t ent2 = kNone;
                        if (m2 != kNone) ent2 = (uint32_t)__builtin_amdgcn_readlane((int)ent, (int)(m2 & 0xFFFF) - c0);
                        // merge (m1, m2) into the running two smallest
                        if (m1 < k1) {
                            if (m2 < k1) { k2 = m2; x2 = ent2; } else { k2 = k1; x2 = x1; }
                            k1 = m1; x1 = ent1;
                        } else if (m1 < k2) {
                            k2 = m1; x2 = ent1;
                        }
                    }
                    got[0] = x1;
                    got[1] = x2;
                    found = (x1 != kNone) + (x2 != kNone);
                }
                if (got[0] == kNone) continue;
                const int bestDist = e_dist(got[0]);
                // bestDist starts at 256 and only strictly smaller distances replace it
                if (bestDist > a.th_dist || bestDist >= 256) continue;
                if (ratio) {
                    // best and second of ORBmatcher.cc:98-112: the first two free
                    // entries in (distance, position) order, with their octaves; a
                    // 256 never becomes second (bestDist2 = 256, bestLevel2 = -1)
                    const bool has2 = got[1] != kNone && e_dist(got[1]) < 256;
                    const int bestDist2 = has2 ? e_dist(got[1]) : 256;
                    const int lv1 = e_oct(got[0]), lv2 = has2 ? e_oct(got[1]) : -1;
                    if (lv1 == lv2 && (float)bestDist > __fmul_rn(a.nnratio, (float)bestDist2)) continue;
                }
                const int idx = e_idx(got[0]);
                if (lane == 0) {
                    s.state[idx] = (uint8_t)(1 | blocks);
                    a.kp_final[idx] = q;
                    a.q_idx[q] = idx;
                    a.q_dist[q] = bestDist;
                }
                ++accepted;
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                __builtin_amdgcn_wave_barrier();
            }
        }
        if (lane == 0) sh_acc = accepted;
    }
    __syncthreads();

    // ---- 4. rotation consistency (ORBmatcher.cc:1434-1469, 1568-1598)
    if (use_ori) {
        const float factor = 1.0f / kHist;
        for (int q = tid; q < nq; q += kPT) {
            const int idx = a.q_idx[q];
            if (idx < 0) continue;
            float rot = __fsub_rn(a.q[q].angle, a.keys[idx].angle);
            if (rot < 0.0f) rot = __fadd_rn(rot, 360.0f);
            int bin = (int)roundf(__fmul_rn(rot, factor));
            if (bin == kHist) bin = 0;
            atomicAdd(&hist[bin], 1);
        }
        __syncthreads();
        if (tid == 0) {
            int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
            for (int i = 0; i < kHist; ++i) {
                const int sz = hist[i];
                if (sz > max1) { max3 = max2; max2 = max1; max1 = sz; ind3 = ind2; ind2 = ind1; ind1 = i; }
                else if (sz > max2) { max3 = max2; max2 = sz; ind3 = ind2; ind2 = i; }
                else if (sz > max3) { max3 = sz; ind3 = i; }
            }
            if ((float)max2 < __fmul_rn(0.1f, (float)max1)) { ind2 = -1; ind3 = -1; }
            else if ((float)max3 < __fmul_rn(0.1f, (float)max1)) { ind3 = -1; }
            sh_top[0] = ind1; sh_top[1] = ind2; sh_top[2] = ind3;
        }
        __syncthreads();
        int removed = 0;
        for (int q = tid; q < nq; q += kPT) {
            const int idx = a.q_idx[q];
            if (idx < 0) continue;
            float rot = __fsub_rn(a.q[q].angle, a.keys[idx].angle);
            if (rot < 0.0f) rot = __fadd_rn(rot, 360.0f);
            int bin = (int)roundf(__fmul_rn(rot, factor));
            if (bin == kHist) bin = 0;
            if (bin != sh_top[0] && bin != sh_top[1] && bin != sh_top[2]) {
                a.kp_final[idx] = -2;
                a.q_idx[q] = -1;
                ++removed;
            }
        }
        if (removed) atomicAdd(&sh_removed, removed);
    }
    __syncthreads();

    // ---- 5. count
    if (fuse) {
        int local = 0;
        for (int q = tid; q < nq; q += kPT) local += a.q_idx[q] >= 0;
        int tot;
        block_scan(local, &tot, ws);
        if (tid == 0) *a.nmatches = tot;
    } else if (tid == 0) {
        *a.nmatches = sh_acc - sh_removed;
    }
}

}  // namespace

int proj_lds_bytes(int n, int pool_cap) {
    auto al = [](size_t b) { return (int)((b + 15) & ~size_t(15)); };
    return al(4 * (kCells + 1)) + al(4 * kCells) + al(8 * (size_t)n) + al(4 * (size_t)n) + al(2 * (size_t)n) +
           al(2 * (size_t)n) + al((size_t)n) + al((size_t)n) + al((size_t)kPW * kEnt) + al(4 * (size_t)pool_cap);
}

constexpr int kProjLdsMax = 160 * 1024 - 1024;   // dynamic LDS; the static part needs < 1 KiB

int proj_pool_cap(int n, int nq) {
    const int fixed = proj_lds_bytes(n, 0);
    if (fixed > kProjLdsMax) return -1;
    return (int)std::min<int64_t>((int64_t)std::max(nq, 1) * std::max(n, 1), (kProjLdsMax - fixed) / 4);
}

hipError_t launch_proj(const ProjBufs &a, hipStream_t st) {
    const int bytes = proj_lds_bytes(a.n, a.pool_cap);
    if (bytes > kProjLdsMax) return hipErrorInvalidValue;
    if (bytes > 64 * 1024 &&
        hipFuncSetAttribute(reinterpret_cast<const void *>(k_proj_match), hipFuncAttributeMaxDynamicSharedMemorySize,
                            bytes) != hipSuccess)
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_proj_match, dim3(1), dim3(kPT), bytes, st, a);
    return hipGetLastError();
}

}  // namespace orbx
