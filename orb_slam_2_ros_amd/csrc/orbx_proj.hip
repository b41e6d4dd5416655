// orbx_proj.hip -- ORBmatcher's projection searches on gfx950:
// SearchByProjection x4 and the candidate search of Fuse x2
// (ORBmatcher.cc:45-129, 291-404, 827-1102, 1330-1601; GetFeaturesInArea
// Frame.cc:354-412 / KeyFrame.cc:700-739; ComputeThreeMaxima :1603-1644).
//
// k_proj_search: many 1024-thread workgroups; each builds the frame's 64x48
// grid (positions, octaves, mvuRight) in its LDS and takes a slice of the
// queries, one wave per query, expanding the query's window into candidate
// entries, one lane per entry.  The static filters (level range, window, stereo gate, Fuse's
// reprojection test) and the Hamming distances are evaluated here, and the
// query's 4 smallest (distance, candidate position) entries are kept; the full
// list goes to a global pool.
//
// The reference assigns keypoints greedily in query order: a keypoint taken by
// an earlier point is skipped by later ones.  Each query needs only its first
// one (best-only variants) or two (SearchByProjection(Frame&,
// vector<MapPoint*>&)) still-free entries in (distance, position) order.
// k_proj_replay (one workgroup) decides the queries in rounds: an open query
// none of whose examined entries can still be taken by an earlier open query
// sees what the in-order loop would see, and is decided in parallel.  What the
// rounds leave (chains of contention, or more than the 4 kept entries needed)
// is replayed by wave 0 in query order, from the 4 kept entries or a 64-wide
// scan of the full list.
// Fuse has no such dependency (its map edits stay with the caller), so its
// queries finish in the parallel phase.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include <algorithm>
#include <climits>

#include "orbx_device.h"
#include "orbx_wave.h"

namespace orbx {
namespace {

constexpr int kPT = 1024, kPW = kPT / 64;
constexpr int kGC = 64, kGR = 48, kCells = kGC * kGR;
constexpr int kHist = 30;
constexpr int kKPer = 8;                  // keypoints per thread in the grid build (n <= 8192)
constexpr int kEnt = 512;                 // per-wave entry map (candidate -> grid column)
constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr int kBadDist = 0x1FF;           // entry failed a static filter
constexpr int kProjLdsMax = 160 * 1024 - 1024;   // dynamic LDS; the static part needs < 1 KiB

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
    int16_t *gtmp;    // n, keypoint index by grid position, unordered inside a cell
    int8_t *goct;     // n, octave by grid position
    uint8_t *entmap;  // kPW x kEnt
};

__device__ inline PLds carve(uint8_t *p, int n) {
    PLds s;
    auto take = [&](size_t bytes) { uint8_t *r = p; p += (bytes + 15) & ~size_t(15); return r; };
    s.gstart = reinterpret_cast<int *>(take(4 * (kCells + 1)));
    s.gfill = reinterpret_cast<int *>(take(4 * kCells));
    s.gxy = reinterpret_cast<float2 *>(take(8 * (size_t)n));
    s.gur = reinterpret_cast<float *>(take(4 * (size_t)n));
    s.glist = reinterpret_cast<int16_t *>(take(2 * (size_t)n));
    s.gtmp = reinterpret_cast<int16_t *>(take(2 * (size_t)n));
    s.goct = reinterpret_cast<int8_t *>(take((size_t)n));
    s.entmap = take((size_t)kPW * kEnt);
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

// Grid (max nblk, problems): problem blockIdx.y, its first a.nblk blocks.
__device__ __attribute__((always_inline)) void proj_search(const ProjBufs *pa, uint8_t *lds) {
    const ProjBufs a = pa[blockIdx.y];
    if ((int)blockIdx.x >= a.nblk) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int n = a.n, nq = a.nq;
    const PLds s = carve(lds, n);
    __shared__ int ws[kPW];
    const int V = a.variant;
    const bool fuse = V == ORBX_PROJ_FUSE || V == ORBX_PROJ_FUSE_SIM3;
    const float invW = __fdiv_rn((float)kGC, __fsub_rn(a.max_x, a.min_x));
    const float invH = __fdiv_rn((float)kGR, __fsub_rn(a.max_y, a.min_y));

    // ---- 0. init
    for (int i = tid; i <= kCells; i += kPT) s.gstart[i] = 0;
    for (int i = tid; i < kCells; i += kPT) s.gfill[i] = 0;
    __syncthreads();

    // ---- 1. grid: counting sort by cell, index order inside each cell.  Each
    // thread keeps its keypoints in registers and places them by rank.
    float kx[kKPer], ky[kKPer], kur[kKPer];
    int koc[kKPer], kc[kKPer];
#pragma unroll
    for (int r = 0; r < kKPer; ++r) {
        const int i = tid + r * kPT;
        kc[r] = -1;
        if (i < n) {
            const orbx_keypoint k = a.keys[i];
            kx[r] = k.x; ky[r] = k.y; koc[r] = k.octave;
            kur[r] = a.uright ? a.uright[i] : -1.0f;
            const int px = (int)roundf(__fmul_rn(__fsub_rn(k.x, a.min_x), invW));
            const int py = (int)roundf(__fmul_rn(__fsub_rn(k.y, a.min_y), invH));
            if (px >= 0 && px < kGC && py >= 0 && py < kGR) {
                kc[r] = px * kGR + py;
                atomicAdd(&s.gstart[kc[r]], 1);
            }
        }
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
#pragma unroll
    for (int r = 0; r < kKPer; ++r)
        if (kc[r] >= 0) s.gtmp[s.gstart[kc[r]] + atomicAdd(&s.gfill[kc[r]], 1)] = (int16_t)(tid + r * kPT);
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kKPer; ++r) {
        if (kc[r] < 0) continue;
        const int i = tid + r * kPT;
        const int st = s.gstart[kc[r]], en = s.gstart[kc[r] + 1];
        int pos = st;
        for (int x = st; x < en; ++x) pos += s.gtmp[x] < i;
        s.glist[pos] = (int16_t)i;
        s.gxy[pos] = make_float2(kx[r], ky[r]);
        s.goct[pos] = (int8_t)koc[r];
        s.gur[pos] = kur[r];
    }
    __syncthreads();

    for (int i = blockIdx.x * kPT + tid; i < n; i += a.nblk * kPT) a.kp_final[i] = -1;

    // ---- 2. window expansion, static filters, distances, 4 smallest per query
    uint8_t *emap = s.entmap + wave * kEnt;
    const bool occ_obs = V == ORBX_PROJ_LOCALMAP || V == ORBX_PROJ_LASTFRAME;
    __shared__ int sh_T[kPW], sh_base;
    // uniform trip count: the waves of a block allocate their lists together
    for (int q0 = blockIdx.x * kPW; q0 < nq; q0 += a.nblk * kPW) {
        const int q = q0 + wave;
        orbx_proj_query Q{};
        int T = 0, st = 0, cnt = 0, pos0 = 0;
        float x = 0.f, y = 0.f, r = 0.f;
        if (q < nq) {
            if (lane == 0) {   // this wave owns query q: default results
                a.qlen[q] = 0;
                a.qbase[q] = -1;
                reinterpret_cast<uint4 *>(a.qtop)[q] = make_uint4(kNone, kNone, kNone, kNone);
                a.q_idx[q] = -1;
                a.q_dist[q] = -1;
            }
            Q = a.q[q];
            x = Q.u; y = Q.v; r = Q.radius;
            // Frame::GetFeaturesInArea cell range (float, as the reference)
            const int cx0 = max(0, (int)floorf(__fmul_rn(__fsub_rn(__fsub_rn(x, a.min_x), r), invW)));
            const int cx1 = min(kGC - 1, (int)ceilf(__fmul_rn(__fadd_rn(__fsub_rn(x, a.min_x), r), invW)));
            const int cy0 = max(0, (int)floorf(__fmul_rn(__fsub_rn(__fsub_rn(y, a.min_y), r), invH)));
            const int cy1 = min(kGR - 1, (int)ceilf(__fmul_rn(__fadd_rn(__fsub_rn(y, a.min_y), r), invH)));
            const bool win = (Q.flags & ORBX_QUERY_ACTIVE) && !(cx0 >= kGC || cx1 < 0 || cy0 >= kGR || cy1 < 0 ||
                                                                 cx1 < cx0 || cy1 < cy0);
            const int ncx = cx1 - cx0 + 1;   // <= 64
            if (win && lane < ncx) {
                const int col = (cx0 + lane) * kGR;
                st = s.gstart[col + cy0];
                cnt = s.gstart[col + cy1 + 1] - st;
            }
            const int incl = wave_incl_scan_i32(cnt);
            pos0 = incl - cnt;
            T = __builtin_amdgcn_readlane(incl, 63);
        }
        // the replay kernel needs the whole lists: one slice of the global
        // pool per block and pass (Fuse decides from the 4 smallest alone)
        if (lane == 0) sh_T[wave] = fuse ? 0 : T;
        __syncthreads();
        if (tid == 0) {
            int tot = 0;
            for (int w = 0; w < kPW; ++w) { const int t = sh_T[w]; sh_T[w] = tot; tot += t; }
            int b = -1;
            if (tot > 0) {
                const unsigned long long g = atomicAdd(a.pool_top, (unsigned long long)tot);
                if (g + tot <= (unsigned long long)a.pool_cap) b = (int)g;   // overflow: the host reruns larger
            }
            sh_base = b;
        }
        __syncthreads();
        const int base = fuse || sh_base < 0 ? -1 : sh_base + sh_T[wave];
        __syncthreads();   // sh_T / sh_base are rewritten by the next pass
        if (T == 0) continue;
        uint32_t *list = base >= 0 ? a.pool + base : nullptr;
        const uint4 qa = *reinterpret_cast<const uint4 *>(a.qdesc + 32 * (int64_t)q);
        const uint4 qb = *reinterpret_cast<const uint4 *>(a.qdesc + 32 * (int64_t)q + 16);
        const bool check_lv = Q.min_level > 0 || Q.max_level >= 0;
        // a keypoint q takes is closed to later queries when q blocks it
        const bool claims = !fuse && (!occ_obs || (Q.flags & ORBX_QUERY_BLOCKS));
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
                    if (list) list[t] = ent;
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
        } else {
            if (claims && top[3] != kNone && e_dist(top[3]) <= a.th_dist && list) {
                // more possible takes than the 4 kept: register them all (rare)
                __threadfence();
                for (int t = lane; t < T; t += 64) {
                    const uint32_t ent = __hip_atomic_load(list + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (e_dist(ent) <= a.th_dist) {
                        const uint32_t h = atomicAdd(a.hard_cnt, 1u);
                        if (h < (uint32_t)a.hard_cap) a.hard[h] = make_uint2((uint32_t)e_idx(ent), (uint32_t)q);
                    }
                }
            }
            if (lane != 0) continue;
            uint4 t4;
            t4.x = top[0]; t4.y = top[1]; t4.z = top[2]; t4.w = top[3];
            reinterpret_cast<uint4 *>(a.qtop)[q] = t4;
            a.qlen[q] = T;
            a.qbase[q] = base;
        }
    }
}

__global__ __launch_bounds__(kPT) void k_proj_search(const ProjBufs *pa) {
    extern __shared__ __align__(16) uint8_t lds[];
    proj_search(pa, lds);
}

__device__ inline bool taken_static(int st, bool occ_obs) { return occ_obs ? st == 3 : (st & 1); }

constexpr int kFQ = 512;   // full-list queries a round hands to the waves

// Keypoint state seen by query q in the replay.
struct RState {
    const uint8_t *state;   // initial map-point state
    uint32_t *blk;          // first blocking taker so far
    const uint32_t *opn;    // first open claimer this round
    const uint32_t *hard;   // first claimer with claims past its 4 kept entries
    bool occ_obs;
    __device__ bool taken(int k, uint32_t q) const { return taken_static(state[k], occ_obs) || blk[k] < q; }
    // an earlier query that is still open may take it
    __device__ bool contended(int k, uint32_t q) const { return opn[k] < q || hard[k] < q; }
};

// The two smallest not-taken entries of a query's full candidate list, by
// (distance, position in the list); wave-uniform arguments and results.
__device__ inline void wave_two_free(const uint32_t *list, int cnt, uint32_t q, const RState &r, int lane,
                                     uint32_t &x1, uint32_t &x2) {
    uint32_t k1 = kNone, k2 = kNone;
    x1 = x2 = kNone;
    for (int c0 = 0; c0 < cnt; c0 += 64) {
        const int e = c0 + lane;
        uint32_t key = kNone, ent = kNone;
        if (e < cnt) {
            ent = list[e];
            if (e_dist(ent) != kBadDist && !r.taken(e_idx(ent), q)) key = ((uint32_t)e_dist(ent) << 16) | (uint32_t)e;
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
}

// ORBmatcher's acceptance of the best (and, with the ratio test, second)
// free entry; records the take.  True when q takes a keypoint.
__device__ inline bool accept(const ProjBufs &a, bool ratio, int q, const uint32_t got[2], bool blocks, uint32_t *blk) {
    if (got[0] == kNone) return false;
    const int bestDist = e_dist(got[0]);
    // bestDist starts at 256 and only strictly smaller distances replace it
    if (bestDist > a.th_dist || bestDist >= 256) return false;
    if (ratio) {
        // best and second of ORBmatcher.cc:98-112, with their octaves; a 256
        // never becomes second (bestDist2 = 256, bestLevel2 = -1)
        const bool has2 = got[1] != kNone && e_dist(got[1]) < 256;
        const int bestDist2 = has2 ? e_dist(got[1]) : 256;
        const int lv1 = e_oct(got[0]), lv2 = has2 ? e_oct(got[1]) : -1;
        if (lv1 == lv2 && (float)bestDist > __fmul_rn(a.nnratio, (float)bestDist2)) return false;
    }
    const int idx = e_idx(got[0]);
    a.q_idx[q] = idx;
    a.q_dist[q] = bestDist;
    atomicMax(&a.kp_final[idx], q);   // a non-blocking take leaves it to later queries
    if (blocks) atomicMin(&blk[idx], (uint32_t)q);
    return true;
}

// The greedy assignment (ORBmatcher.cc:45-129, 1330-1601), then the rotation
// check and the count.  One block.
//
// A query examines its entries in (distance, position) order until it has the
// one (two, with the ratio test) not yet taken.  An entry is taken at query q
// when its initial state says so or a blocking take by a query < q made it
// so; only entries within th_dist of a query ("claims", all among its 4 kept
// entries unless `hard` has them) can ever be taken by it.  Rounds: every open
// query registers its claims (minimum open claimer per keypoint); an open
// query none of whose examined entries has an open claimer < q sees exactly
// what the in-order loop would, and is decided (by a thread from its 4 kept
// entries, or by a wave from its full list when those are not enough).  The
// rounds stop when none progresses; what is left (contention chains through
// `hard` claims) is replayed by wave 0 in query order.
template <bool QL>   // per-query data in LDS (else global; one instantiation each keeps ds_* loads ds_*)
__device__ __attribute__((always_inline)) void proj_replay(const ProjBufs &a, uint8_t *lds) {
    const uint64_t c0 = wall_clock64();
    const int n = a.n, nq = a.nq;
    const int V = a.variant;
    const bool fuse = V == ORBX_PROJ_FUSE || V == ORBX_PROJ_FUSE_SIM3;
    const bool occ_obs = V == ORBX_PROJ_LOCALMAP || V == ORBX_PROJ_LASTFRAME;   // skip: has && Observations() > 0
    const bool ratio = V == ORBX_PROJ_LOCALMAP;
    const bool use_ori = a.check_ori && (V == ORBX_PROJ_LASTFRAME || V == ORBX_PROJ_KEYFRAME);
    const int need = ratio ? 2 : 1;
    // LDS: per keypoint blk / opn / hard (u32) and state (u8), the full-list
    // queue; per query the 4 kept entries and a status byte, in LDS when they
    // fit (else in global memory)
    constexpr bool q_in_lds = QL;
    uint32_t *blk = reinterpret_cast<uint32_t *>(lds);
    uint32_t *opn = blk + n;
    uint32_t *hard = opn + n;
    int32_t *fq = reinterpret_cast<int32_t *>(hard + n);
    uint8_t *p8 = lds + ((12 * (size_t)n + 12 * kFQ + 15) & ~size_t(15));
    uint4 *qt = q_in_lds ? reinterpret_cast<uint4 *>(p8) : reinterpret_cast<uint4 *>(a.qtop);
    if (q_in_lds) p8 += 16 * (size_t)nq;
    uint8_t *state = p8;
    // per query: bits 0-1 status (0 decided, 1 open), bit 2 blocks
    uint8_t *qs = q_in_lds ? p8 + n : a.und;
    const RState rs{state, blk, opn, hard, occ_obs};
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    __shared__ int ws[kPW];
    __shared__ int hist[kHist];
    __shared__ int sh_acc, sh_removed, sh_top[3], sh_prog[2], sh_fq;
    if (!fuse) {
        for (int i = tid; i < n; i += kPT) {
            state[i] = a.mp_state ? (a.mp_state[i] & 3) : 0;
            blk[i] = kNone;
            hard[i] = kNone;
        }
        for (int q = tid; q < nq; q += kPT) {
            const uint4 t4 = reinterpret_cast<const uint4 *>(a.qtop)[q];
            const int fl = a.q[q].flags;
            if (q_in_lds) qt[q] = t4;
            // open: some entry within th_dist (else no take is possible)
            const bool open = (fl & ORBX_QUERY_ACTIVE) && t4.x != kNone && e_dist(t4.x) <= a.th_dist;
            const bool blocks = !occ_obs || (fl & ORBX_QUERY_BLOCKS);
            qs[q] = (uint8_t)((open ? 1 : 0) | (blocks ? 4 : 0));
        }
    }
    if (tid < kHist) hist[tid] = 0;
    if (tid == 0) { sh_acc = 0; sh_removed = 0; }
    __syncthreads();
    const uint32_t nhard = fuse ? 0 : *a.hard_cnt;
    for (uint32_t h = tid; h < min(nhard, (uint32_t)a.hard_cap); h += kPT) {
        const uint2 c = a.hard[h];
        atomicMin(&hard[c.x], c.y);
    }
    __syncthreads();
    if (a.stats && tid == 0) a.stats[2] = (int)(wall_clock64() - c0);

    // ---- 3a. rounds of order-independent decisions
    // (claims lost to a full `hard` list: everything goes in order)
    if (!fuse && nhard <= (uint32_t)a.hard_cap) {
        int accepted = 0;
        for (int round = 0; round < 64; ++round) {
            for (int i = tid; i < n; i += kPT) opn[i] = kNone;
            if (tid == 0) { sh_prog[round & 1] = 0; sh_fq = 0; }
            int any_open = 0;
            for (int q = tid; q < nq && !any_open; q += kPT) any_open = (qs[q] & 3) == 1;
            if (!__syncthreads_or(any_open)) {
                if (a.stats && tid == 0) a.stats[0] = round;
                break;
            }
            for (int q = tid; q < nq; q += kPT) {
                if (qs[q] != (1 | 4)) continue;   // open and blocking (other takes close nothing)
                const uint4 t4 = qt[q];
                const uint32_t e4[4] = {t4.x, t4.y, t4.z, t4.w};
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    if (e4[t] == kNone || e_dist(e4[t]) > a.th_dist) break;
                    const int k = e_idx(e4[t]);
                    if (!taken_static(state[k], occ_obs)) atomicMin(&opn[k], (uint32_t)q);
                }
            }
            __syncthreads();
            int prog = 0;
            for (int q = tid; q < nq; q += kPT) {
                const int st = qs[q];
                if ((st & 3) != 1) continue;
                const uint4 t4 = qt[q];
                const uint32_t e4[4] = {t4.x, t4.y, t4.z, t4.w};
                // all four entries' state at once (independent LDS reads)
                bool tk[4], ct[4];
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const int k = e4[t] == kNone ? 0 : e_idx(e4[t]);
                    tk[t] = rs.taken(k, q);
                    ct[t] = rs.contended(k, q);
                }
                uint32_t got[2] = {kNone, kNone};
                int found = 0;
                bool stuck = false;
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    if (found == need || stuck || e4[t] == kNone) continue;
                    if (tk[t]) continue;
                    if (ct[t]) { stuck = true; continue; }
                    got[found++] = e4[t];
                }
                if (stuck) continue;
                if (found < need && e4[3] != kNone) {
                    // past the 4 kept entries: a wave scans the full list below
                    const int slot = atomicAdd(&sh_fq, 1);
                    if (slot < kFQ) {   // (a full queue leaves q open for the next round)
                        fq[3 * slot] = q;
                        fq[3 * slot + 1] = a.qbase[q];
                        fq[3 * slot + 2] = a.qlen[q];
                    }
                    continue;
                }
                qs[q] = (uint8_t)(st & 4);
                prog = 1;
                accepted += accept(a, ratio, q, got, st & 4, blk);
            }
            __syncthreads();
            const int nfq = min(sh_fq, kFQ);
            for (int i = wave; i < nfq; i += kPW) {
                const int q = fq[3 * i], qb = fq[3 * i + 1], len = fq[3 * i + 2];
                const int st = qs[q];
                prog = 1;
                if (qb < 0) {   // the pool overflowed: the host runs the call again
                    if (lane == 0) qs[q] = (uint8_t)(st & 4);
                    continue;
                }
                uint32_t got[2];
                wave_two_free(a.pool + qb, len, q, rs, lane, got[0], got[1]);
                if (need == 1) got[1] = kNone;
                bool stuck = false;
                for (int t = 0; t < 2; ++t)
                    if (got[t] != kNone && rs.contended(e_idx(got[t]), q)) stuck = true;
                if (stuck) continue;
                if (lane == 0) {
                    qs[q] = (uint8_t)(st & 4);
                    accepted += accept(a, ratio, q, got, st & 4, blk);
                }
            }
            if (prog) sh_prog[round & 1] = 1;
            __syncthreads();
            if (!sh_prog[round & 1]) {   // (the next round resets the other flag)
                if (a.stats && tid == 0) a.stats[0] = round + 1;
                break;
            }
        }
        const int tot = wave_sum_i32(accepted);
        if (lane == 0 && tot) atomicAdd(&sh_acc, tot);
        __syncthreads();
    }
    if (a.stats && tid == 0) a.stats[3] = (int)(wall_clock64() - c0);

    // ---- 3b. what is left, in query order (wave 0)
    int left = 0;
    if (!fuse)
        for (int q = tid; q < nq && !left; q += kPT) left = (qs[q] & 3) != 0;
    if (__syncthreads_or(left) && wave == 0) {
        int accepted = 0, nserial = 0;
        for (int g0 = 0; g0 < nq; g0 += 64) {
            const int gq = g0 + lane;
            const int st = gq < nq ? qs[gq] : 0;
            uint64_t todo = __ballot((st & 3) != 0);
            if (!todo) continue;
            nserial += __popcll(todo);
            const uint4 t4 = (st & 3) ? qt[gq] : make_uint4(kNone, kNone, kNone, kNone);
            while (todo) {
                const int j = (int)__builtin_ctzll(todo);
                todo &= todo - 1;
                const int q = g0 + j;
                const uint32_t e4[4] = {(uint32_t)__builtin_amdgcn_readlane((int)t4.x, j),
                                        (uint32_t)__builtin_amdgcn_readlane((int)t4.y, j),
                                        (uint32_t)__builtin_amdgcn_readlane((int)t4.z, j),
                                        (uint32_t)__builtin_amdgcn_readlane((int)t4.w, j)};
                const bool blocks = __builtin_amdgcn_readlane(st, j) & 4;
                uint32_t got[2] = {kNone, kNone};
                int found = 0;
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    if (e4[t] == kNone || found == need) continue;
                    if (rs.taken(e_idx(e4[t]), q)) continue;
                    got[found++] = e4[t];
                }
                if (found < need && e4[3] != kNone) {
                    // more entries than the 4 kept: scan the whole list
                    const int qb = a.qbase[q];
                    if (qb < 0) continue;   // the pool overflowed: the host runs the call again
                    wave_two_free(a.pool + qb, a.qlen[q], q, rs, lane, got[0], got[1]);
                    if (need == 1) got[1] = kNone;
                }
                bool took = false;
                if (lane == 0) took = accept(a, ratio, q, got, blocks, blk);
                accepted += __builtin_amdgcn_readfirstlane((int)took);
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront", "local");
                __builtin_amdgcn_wave_barrier();
            }
        }
        if (lane == 0) sh_acc += accepted;
        if (a.stats && lane == 0) a.stats[1] = nserial;
    }
    __syncthreads();
    if (a.stats && tid == 0) a.stats[5] = (int)(wall_clock64() - c0);

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
    __syncthreads();
}

template <bool QL>
__global__ __launch_bounds__(kPT) void k_proj_replay(const ProjBufs *pa, HostTail tail) {   // one block per problem
    extern __shared__ __align__(16) uint8_t lds[];
    const ProjBufs a = pa[blockIdx.x];   // (a copy: the fields in registers)
    proj_replay<QL>(a, lds);
    host_tail(tail);
}

// The single-problem host call in one launch: the search, then its last
// workgroup to finish runs the replay and copies the outputs to the host
// (dynamic LDS: the larger of the two layouts).
template <bool QL>
__global__ __launch_bounds__(kPT) void k_proj_search_replay(const ProjBufs *pa, HostTail tail) {
    extern __shared__ __align__(16) uint8_t lds[];
    proj_search(pa, lds);
    __shared__ int s_last;
    __threadfence();   // this workgroup's lists and entries before its count
    __syncthreads();
    if (threadIdx.x == 0) s_last = atomicAdd(tail.done, 1u) == (uint32_t)(tail.blocks - 1);
    __syncthreads();
    if (!s_last) return;
    __threadfence();   // (acquire: every workgroup's results)
    const ProjBufs a = pa[0];
    proj_replay<QL>(a, lds);
    tail_copy(tail);
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(tail.flag, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace

int proj_lds_bytes(int n) {
    auto al = [](size_t b) { return (int)((b + 15) & ~size_t(15)); };
    return al(4 * (kCells + 1)) + al(4 * kCells) + al(8 * (size_t)n) + al(4 * (size_t)n) + al(2 * (size_t)n) +
           al(2 * (size_t)n) + al((size_t)n) + al((size_t)kPW * kEnt);
}


int proj_replay_lds_bytes(int n, int nq, bool q_in_lds) {
    return 13 * n + 12 * kFQ + (q_in_lds ? 17 * nq : 0) + 64;
}

bool proj_fits(int n) { return n <= kKPer * kPT && proj_lds_bytes(n) <= kProjLdsMax && proj_replay_lds_bytes(n, 0, false) <= kProjLdsMax; }

int proj_blocks(int nq) { return std::max(1, std::min(512, (nq + kPW - 1) / kPW)); }

// The one-launch form of the single host call (k_proj_search_replay) measured
// slower than the two launches (SearchByProjection localmap 0.115 -> 0.148 ms:
// the search then runs with the replay's LDS and registers): off unless
// ORBX_PROJ_ONE_LAUNCH=1.
bool proj_one_launch() {
    const char *e = std::getenv("ORBX_PROJ_ONE_LAUNCH");
    return e && e[0] == '1';
}

int proj_tail_blocks(const ProjBufs *h, int np) { return np == 1 && proj_one_launch() ? h[0].nblk : np; }

// h: the problems' buffers on the host, d: the same array in device memory.
hipError_t launch_proj(const ProjBufs *h, const ProjBufs *d, int np, const HostTail &tail, hipStream_t st) {
    if (np <= 0) return hipSuccess;
    if (tail.flag && tail.blocks != proj_tail_blocks(h, np)) return hipErrorInvalidValue;
    int bytes = 0, nblk = 1;
    bool q_in_lds = true;
    for (int k = 0; k < np; ++k) {
        bytes = std::max(bytes, proj_lds_bytes(h[k].n));
        nblk = std::max(nblk, h[k].nblk);
        q_in_lds = q_in_lds && proj_replay_lds_bytes(h[k].n, h[k].nq, true) <= kProjLdsMax;
    }
    if (bytes > kProjLdsMax) return hipErrorInvalidValue;
    int rbytes = 0;
    for (int k = 0; k < np; ++k) rbytes = std::max(rbytes, proj_replay_lds_bytes(h[k].n, h[k].nq, q_in_lds));
    if (rbytes > kProjLdsMax) return hipErrorInvalidValue;
    if (np == 1 && tail.flag && proj_one_launch()) {   // the host call: one launch
        const int fb = std::max(bytes, rbytes);
        const void *fk = q_in_lds ? reinterpret_cast<const void *>(k_proj_search_replay<true>)
                                  : reinterpret_cast<const void *>(k_proj_search_replay<false>);
        if (fb > 64 * 1024 && hipFuncSetAttribute(fk, hipFuncAttributeMaxDynamicSharedMemorySize, fb) != hipSuccess)
            return hipErrorInvalidValue;
        if (q_in_lds)
            hipLaunchKernelGGL(k_proj_search_replay<true>, dim3(nblk, 1), dim3(kPT), fb, st, d, tail);
        else
            hipLaunchKernelGGL(k_proj_search_replay<false>, dim3(nblk, 1), dim3(kPT), fb, st, d, tail);
        return hipGetLastError();
    }
    if (bytes > 64 * 1024 &&
        hipFuncSetAttribute(reinterpret_cast<const void *>(k_proj_search), hipFuncAttributeMaxDynamicSharedMemorySize,
                            bytes) != hipSuccess)
        return hipErrorInvalidValue;
    // each problem's queries spread over up to 512 blocks, one query per wave
    hipLaunchKernelGGL(k_proj_search, dim3(nblk, np), dim3(kPT), bytes, st, d);
    const void *rk = q_in_lds ? reinterpret_cast<const void *>(k_proj_replay<true>)
                              : reinterpret_cast<const void *>(k_proj_replay<false>);
    if (rbytes > 64 * 1024 && hipFuncSetAttribute(rk, hipFuncAttributeMaxDynamicSharedMemorySize, rbytes) != hipSuccess)
        return hipErrorInvalidValue;
    if (q_in_lds)
        hipLaunchKernelGGL(k_proj_replay<true>, dim3(np), dim3(kPT), rbytes, st, d, tail);
    else
        hipLaunchKernelGGL(k_proj_replay<false>, dim3(np), dim3(kPT), rbytes, st, d, tail);
    return hipGetLastError();
}

}  // namespace orbx
