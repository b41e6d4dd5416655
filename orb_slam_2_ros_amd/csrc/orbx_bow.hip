// orbx_bow.hip -- ORBmatcher's vocabulary-node matchers on gfx950:
// SearchByBoW(KeyFrame*, Frame&) (ORBmatcher.cc:160-289), SearchByBoW(KeyFrame*,
// KeyFrame*) (:524-657) and SearchForTriangulation (:659-825, epipolar test
// CheckDistEpipolarLine :140-157).
//
// The reference merge-joins the two FeatureVectors (node id -> feature
// indices) and compares only features that share a node.  A feature belongs
// to exactly one node, so the greedy "already matched" state of the two
// SearchByBoW variants never crosses nodes: nodes are independent.  One wave
// takes one node of side A, finds it in side B (binary search over the
// ascending ids) and walks A's features in order; for each, the lanes hold
// B's features of the node, compute the distances and reduce (distance,
// position) minima with DPP.  Accepted B positions are flagged in the wave's
// LDS.  SearchForTriangulation never sets its vbMatched2 (the reference
// leaves it false), so there every A feature is independent; its update rule
// (dist <= bestDist, after the epipolar tests) keeps the LAST minimum.
// The rotation-consistency pass runs in a second single-block kernel.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "orbx_device.h"
#include "orbx_wave.h"

namespace orbx {
namespace {

constexpr int kBT = 256;
constexpr int kHist = 30;
constexpr int kThLow = 50;
constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr int kRepairs = kHist + 1;   // count slot of the repair passes (after the match count)
#ifndef ORBX_BOW_LANES_A
#define ORBX_BOW_LANES_A 1   // nodes of <= 64 B features: lanes take A's features (0: one A feature at a time)
#endif
constexpr bool kBowLanesA = ORBX_BOW_LANES_A;

__device__ inline int hamming_rr(const uint4 a0, const uint4 a1, const uint4 b0, const uint4 b1) {
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

__device__ inline int rot_bin(float a1, float a2) {
    float rot = __fsub_rn(a1, a2);
    if (rot < 0.0f) rot = __fadd_rn(rot, 360.0f);
    int bin = (int)roundf(__fmul_rn(rot, 1.0f / kHist));
    return bin == kHist ? 0 : bin;
}

// CheckDistEpipolarLine (ORBmatcher.cc:140-157); F row-major.
__device__ inline bool epipolar_ok(float x1, float y1, float x2, float y2, const float *F, float sigma2) {
    const float a = __fadd_rn(__fadd_rn(__fmul_rn(x1, F[0]), __fmul_rn(y1, F[3])), F[6]);
    const float b = __fadd_rn(__fadd_rn(__fmul_rn(x1, F[1]), __fmul_rn(y1, F[4])), F[7]);
    const float c = __fadd_rn(__fadd_rn(__fmul_rn(x1, F[2]), __fmul_rn(y1, F[5])), F[8]);
    const float num = __fadd_rn(__fadd_rn(__fmul_rn(a, x2), __fmul_rn(b, y2)), c);
    const float den = __fadd_rn(__fmul_rn(a, a), __fmul_rn(b, b));
    if (den == 0.0f) return false;
    const float dsqr = __fdiv_rn(__fmul_rn(num, num), den);
    return (double)dsqr < __dmul_rn(3.84, (double)sigma2);
}

// Position of id in the ascending, distinct ids[0, n), or -1, by the whole
// wave: 64 pivots per round narrow the range 64-fold, so a side of up to 4096
// nodes takes two rounds of loads where a binary search takes twelve
// dependent ones (the single drop-in call waits on every round trip).
__device__ inline int wave_find_u32(const uint32_t *ids, int n, uint32_t id, int lane) {
    int lo = 0, hi = n;
    while (hi - lo > 64) {
        const int step = (hi - lo + 63) >> 6;
        const int p = lo + lane * step;
        const bool le = p < hi && ids[p] <= id;   // a prefix of the lanes
        const int c = __popcll(__ballot(le));
        if (c == 0) return -1;
        lo += (c - 1) * step;
        hi = min(hi, lo + step);
    }
    const int p = lo + lane;
    const uint64_t eq = __ballot(p < hi && ids[p] == id);
    return eq ? lo + __ffsll((unsigned long long)eq) - 1 : -1;
}

// One wave: node na_node of side A against its node in side B.
// Accepted matches are counted in the workgroup's LDS (cnt[0, 30): rotation
// bins, cnt[30]: matches, cnt[31]: features that took the in-order repair
// pass, a diagnostic the host reports through orbx_debug_counter); each workgroup stores its counts to its own slot
// of a.part and the finish sums the slots.  (Device atomics on the problem's
// counters -- one per match, or even one per bin per workgroup -- all land on
// one cache line and serialise at its L2 channel: 43 -> 31 us of kernel time
// in the drop-in call, profiles/r04_bow_call_phases3.txt.)
__device__ __attribute__((always_inline)) void bow_match_node(const BowBufs &a, int na_node, int lane,
                                                              uint8_t *mflag, int *cnt) {
    int a0, a1, b0, nbk, ia0;
    if (a.span) {   // the host's merge join of the two node lists: one load
        const int4 sp = a.span[na_node];
        a0 = sp.x; a1 = sp.y; b0 = sp.z; nbk = sp.w - sp.z;
        if (nbk <= 0) return;
        ia0 = lane < a1 - a0 ? a.A.node_features[a0 + lane] : -1;
    } else {
        const uint32_t id = a.A.node_ids[na_node];
        a0 = a.A.node_offsets[na_node]; a1 = a.A.node_offsets[na_node + 1];
        // A's first 64 feature indices, in flight with the search below
        ia0 = lane < a1 - a0 ? a.A.node_features[a0 + lane] : -1;
        // the node in side B
        const int nb_node = wave_find_u32(a.B.node_ids, a.B.nnodes, id, lane);
        if (nb_node < 0) return;
        b0 = a.B.node_offsets[nb_node]; nbk = a.B.node_offsets[nb_node + 1] - b0;
    }
    const bool tri = a.variant == ORBX_BOW_TRIANGULATION;
    for (int p = lane; p < nbk; p += 64) mflag[p] = 0;
    // the first 64 B features stay in registers
    int i2r = -1, fbr = 0, octr = 0;
    uint4 d0r = make_uint4(0, 0, 0, 0), d1r = d0r;
    float xr = 0.f, yr = 0.f, angr = 0.f;
    if (lane < nbk) {
        i2r = a.B.node_features[b0 + lane];
        fbr = a.B.flags[i2r];
        const uint4 *dp = reinterpret_cast<const uint4 *>(a.B.desc + 32 * (int64_t)i2r);
        d0r = dp[0]; d1r = dp[1];
        if (tri) {
            const orbx_keypoint k = a.B.keys[i2r];
            xr = k.x; yr = k.y; octr = k.octave;
        }
        angr = a.B.ang[i2r];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const float *F = a.tri;
    if (nbk <= 64 && kBowLanesA) {
        // The lanes take A's features (64 at a time) and B's features are
        // broadcast one at a time from the registers above: every A feature's
        // two best keys over all of B, with no cross-lane reduction per
        // feature.  SearchByBoW's greedy pass then walks the features in
        // order; a feature's two keys stand unless an earlier feature took one
        // of their B features (then its exact pass over the untaken ones runs,
        // the lanes holding B again).  Triangulation's features are
        // independent: each lane writes its own.
        uint64_t taken = 0;   // B positions matched by earlier A features (wave-uniform)
        for (int pa = a0; pa < a1; pa += 64) {
            const int np = min(64, a1 - pa);
            int i1l = -1, fal = 0;
            uint4 qal = make_uint4(0, 0, 0, 0), qbl = qal;
            float x1l = 0.f, y1l = 0.f, an1l = 0.f;
            if (lane < np) {
                i1l = pa == a0 ? ia0 : a.A.node_features[pa + lane];
                fal = a.A.flags[i1l];
                const uint4 *ap = reinterpret_cast<const uint4 *>(a.A.desc + 32 * (int64_t)i1l);
                qal = ap[0]; qbl = ap[1];
                if (tri) {
                    const orbx_keypoint k = a.A.keys[i1l];
                    x1l = k.x; y1l = k.y;
                }
                an1l = a.A.ang[i1l];
            }
            const bool st1 = (fal >> 1) & 1;
            uint32_t k1 = kNone, k2 = kNone;   // the lane's smallest two (dist << 16 | position) keys
            for (int p = 0; p < nbk; ++p) {
                const int fb = __builtin_amdgcn_readlane(fbr, p);
                if (!(a.variant == ORBX_BOW_KF_FRAME || (fb & 1))) continue;
                const uint4 e0 = make_uint4(__builtin_amdgcn_readlane(d0r.x, p), __builtin_amdgcn_readlane(d0r.y, p),
                                            __builtin_amdgcn_readlane(d0r.z, p), __builtin_amdgcn_readlane(d0r.w, p));
                const uint4 e1 = make_uint4(__builtin_amdgcn_readlane(d1r.x, p), __builtin_amdgcn_readlane(d1r.y, p),
                                            __builtin_amdgcn_readlane(d1r.z, p), __builtin_amdgcn_readlane(d1r.w, p));
                const int dist = hamming_rr(qal, qbl, e0, e1);
                uint32_t key = kNone;
                if (!tri) {
                    key = ((uint32_t)dist << 16) | (uint32_t)p;
                } else if (dist <= kThLow) {
                    const float x2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, xr), p));
                    const float y2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, yr), p));
                    const int oct = __builtin_amdgcn_readlane(octr, p);
                    const bool st2 = (fb >> 1) & 1;
                    const bool lv = oct >= 0 && oct < a.nlevels;
                    bool ok = true;
                    if (!st1 && !st2) {
                        const float dx = __fsub_rn(a.ex, x2), dy = __fsub_rn(a.ey, y2);
                        const float sc = lv ? F[11 + oct] : 0.0f;
                        if (__fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)) < __fmul_rn(100.0f, sc)) ok = false;
                    }
                    if (ok && epipolar_ok(x1l, y1l, x2, y2, F, lv ? F[11 + a.nlevels + oct] : 0.0f))
                        key = ((uint32_t)dist << 16) | (uint32_t)(0xFFFF - p);   // last minimum wins
                }
                if (key < k1) { k2 = k1; k1 = key; }
                else if (key < k2) { k2 = key; }
            }
            if (tri) {
                const int p1 = k1 == kNone ? 0 : 0xFFFF - (int)(k1 & 0xFFFF);
                const int x_1 = __shfl(i2r, p1);   // (every lane active)
                const float an2 = __shfl(angr, p1);
                if (lane < np && (fal & 1) && k1 != kNone) {
                    a.match_a[i1l] = x_1;
                    if (a.check_ori) {
                        const int bin = rot_bin(an1l, an2);
                        a.bin_a[i1l] = (int8_t)bin;
                        atomicAdd(&cnt[bin], 1);
                    }
                    atomicAdd(&cnt[kHist], 1);
                }
                continue;
            }
            for (int q = 0; q < np; ++q) {
                const int fa = __builtin_amdgcn_readlane(fal, q);
                if (!(fa & 1)) continue;
                uint32_t c1 = (uint32_t)__builtin_amdgcn_readlane((int)k1, q);
                uint32_t c2 = (uint32_t)__builtin_amdgcn_readlane((int)k2, q);
                if (c1 == kNone) continue;
                if (((taken >> (c1 & 63)) & 1) || (c2 != kNone && ((taken >> (c2 & 63)) & 1))) {
                    if (lane == 0) atomicAdd(&cnt[kRepairs], 1);
                    const uint4 qa = make_uint4(__builtin_amdgcn_readlane(qal.x, q), __builtin_amdgcn_readlane(qal.y, q),
                                                __builtin_amdgcn_readlane(qal.z, q), __builtin_amdgcn_readlane(qal.w, q));
                    const uint4 qb = make_uint4(__builtin_amdgcn_readlane(qbl.x, q), __builtin_amdgcn_readlane(qbl.y, q),
                                                __builtin_amdgcn_readlane(qbl.z, q), __builtin_amdgcn_readlane(qbl.w, q));
                    uint32_t key = kNone;
                    if (lane < nbk && (a.variant == ORBX_BOW_KF_FRAME || (fbr & 1)) && !((taken >> lane) & 1))
                        key = ((uint32_t)hamming_rr(qa, qb, d0r, d1r) << 16) | (uint32_t)lane;
                    c1 = wave_min_u32(key);
                    if (c1 == kNone) continue;
                    c2 = wave_min_u32(lane == (int)(c1 & 0xFFFF) ? kNone : key);
                }
                const int best1 = (int)(c1 >> 16), best2 = c2 == kNone ? 256 : (int)(c2 >> 16);
                const bool pass = a.variant == ORBX_BOW_KF_FRAME ? best1 <= kThLow : best1 < kThLow;
                if (!(pass && (float)best1 < __fmul_rn(a.nnratio, (float)best2))) continue;
                const int p1 = (int)(c1 & 0xFFFF);
                taken |= 1ull << p1;
                const int x_1 = __builtin_amdgcn_readlane(i2r, p1), i1 = __builtin_amdgcn_readlane(i1l, q);
                float an1 = 0.f, an2 = 0.f;
                if (a.check_ori) {
                    an1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, an1l), q));
                    an2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, angr), p1));
                }
                if (lane == 0) {
                    a.match_a[i1] = x_1;
                    a.match_b[x_1] = i1;
                    if (a.check_ori) {
                        const int bin = rot_bin(an1, an2);
                        a.bin_a[i1] = (int8_t)bin;
                        atomicAdd(&cnt[bin], 1);
                    }
                    atomicAdd(&cnt[kHist], 1);
                }
            }
        }
        return;
    }
    // A's features walked in order, 64 at a time: lane q holds feature
    // a0 + q's index, flags, descriptor and keypoint (one round of loads for
    // the run instead of a dependent chain per feature), read back by readlane
    for (int pa = a0; pa < a1; pa += 64) {
        const int np = min(64, a1 - pa);
        int i1l = -1, fal = 0;
        uint4 qal = make_uint4(0, 0, 0, 0), qbl = qal;
        float x1l = 0.f, y1l = 0.f, an1l = 0.f;
        if (lane < np) {
            i1l = pa == a0 ? ia0 : a.A.node_features[pa + lane];
            fal = a.A.flags[i1l];
            const uint4 *ap = reinterpret_cast<const uint4 *>(a.A.desc + 32 * (int64_t)i1l);
            qal = ap[0]; qbl = ap[1];
            if (tri) {
                const orbx_keypoint k = a.A.keys[i1l];
                x1l = k.x; y1l = k.y;
            }
            an1l = a.A.ang[i1l];
        }
        for (int q = 0; q < np; ++q) {
            const int fa = __builtin_amdgcn_readlane(fal, q);
            if (!(fa & 1)) continue;
            const int i1 = __builtin_amdgcn_readlane(i1l, q);
            const uint4 qa = make_uint4(__builtin_amdgcn_readlane(qal.x, q), __builtin_amdgcn_readlane(qal.y, q),
                                        __builtin_amdgcn_readlane(qal.z, q), __builtin_amdgcn_readlane(qal.w, q));
            const uint4 qb = make_uint4(__builtin_amdgcn_readlane(qbl.x, q), __builtin_amdgcn_readlane(qbl.y, q),
                                        __builtin_amdgcn_readlane(qbl.z, q), __builtin_amdgcn_readlane(qbl.w, q));
            const float k1x = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x1l), q));
            const float k1y = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, y1l), q));
            const bool st1 = (fa >> 1) & 1;
            uint32_t k_1 = kNone, k_2 = kNone;   // running (dist << 16 | position) smallest two
            int x_1 = -1, p_1 = -1;               // B feature of k_1 and its position in the node
            for (int c0 = 0; c0 < nbk; c0 += 64) {
                const int pos = c0 + lane;
                int i2 = -1, fb = 0, oct = 0;
                uint4 e0, e1;
                float x2 = 0.f, y2 = 0.f;
                if (c0 == 0) {
                    i2 = i2r; fb = fbr; e0 = d0r; e1 = d1r; x2 = xr; y2 = yr; oct = octr;
                } else if (pos < nbk) {
                    i2 = a.B.node_features[b0 + pos];
                    fb = a.B.flags[i2];
                    const uint4 *dp = reinterpret_cast<const uint4 *>(a.B.desc + 32 * (int64_t)i2);
                    e0 = dp[0]; e1 = dp[1];
                    if (tri) {
                        const orbx_keypoint k = a.B.keys[i2];
                        x2 = k.x; y2 = k.y; oct = k.octave;
                    }
                }
                uint32_t key = kNone;
                if (pos < nbk) {
                    const bool usable = a.variant == ORBX_BOW_KF_FRAME ? true : (fb & 1);
                    if (usable && !(tri ? false : mflag[pos])) {
                        const int dist = hamming_rr(qa, qb, e0, e1);
                        if (!tri) {
                            key = ((uint32_t)dist << 16) | (uint32_t)pos;
                        } else if (dist <= kThLow) {
                            bool ok = true;
                            const bool st2 = (fb >> 1) & 1;
                            const bool lv = oct >= 0 && oct < a.nlevels;
                            if (!st1 && !st2) {
                                const float dx = __fsub_rn(a.ex, x2), dy = __fsub_rn(a.ey, y2);
                                const float sc = lv ? F[11 + oct] : 0.0f;
                                if (__fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)) < __fmul_rn(100.0f, sc)) ok = false;
                            }
                            if (ok && epipolar_ok(k1x, k1y, x2, y2, F, lv ? F[11 + a.nlevels + oct] : 0.0f))
                                key = ((uint32_t)dist << 16) | (uint32_t)(0xFFFF - pos);   // last minimum wins
                        }
                    }
                }
                const uint32_t m1 = wave_min_u32(key);
                if (m1 == kNone) continue;
                const int pm = tri ? (int)(0xFFFF - (m1 & 0xFFFF)) : (int)(m1 & 0xFFFF);
                const int w1 = __builtin_amdgcn_readlane(i2, pm - c0);
                if (tri) {
                    if (m1 < k_1) { k_1 = m1; x_1 = w1; p_1 = pm; }
                    continue;
                }
                const uint32_t m2 = wave_min_u32(lane == pm - c0 ? kNone : key);
                if (m1 < k_1) {
                    k_2 = m2 < k_1 ? m2 : k_1;
                    k_1 = m1;
                    x_1 = w1;
                    p_1 = pm;
                } else if (m1 < k_2) {
                    k_2 = m1;
                }
            }
            if (k_1 == kNone) continue;
            const int best1 = (int)(k_1 >> 16);
            if (!tri) {
                const int best2 = k_2 == kNone ? 256 : (int)(k_2 >> 16);
                const bool pass = a.variant == ORBX_BOW_KF_FRAME ? best1 <= kThLow : best1 < kThLow;
                if (!(pass && (float)best1 < __fmul_rn(a.nnratio, (float)best2))) continue;
                if (lane == 0) mflag[k_1 & 0xFFFF] = 1;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
            // the matched B feature's angle: from its lane's registers when it is
            // one of the node's first 64 (wave-uniform position)
            float an1 = 0.f, an2 = 0.f;
            if (a.check_ori) {
                an1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, an1l), q));
                if (p_1 < 64) an2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, angr), p_1));
                else an2 = a.B.ang[x_1];
            }
            if (lane == 0) {
                a.match_a[i1] = x_1;
                if (!tri) a.match_b[x_1] = i1;
                if (a.check_ori) {
                    const int bin = rot_bin(an1, an2);
                    a.bin_a[i1] = (int8_t)bin;
                    atomicAdd(&cnt[bin], 1);
                }
                atomicAdd(&cnt[kHist], 1);
            }
        }
    }
}

// ComputeThreeMaxima + removal of the matches outside the three main bins,
// by one workgroup (any size); ends with a barrier.
__device__ __attribute__((always_inline)) void bow_finish_problem(const BowBufs &a) {
    __shared__ int top[3];
    __shared__ int hist[32];
    __shared__ int removed;
    const int tid = threadIdx.x, bd = blockDim.x;
    if (tid < 32) hist[tid] = 0;
    __syncthreads();
    {   // the match workgroups' partial counts, eight loads in flight per thread
        const int ne = 32 * a.nparts;
        for (int base = tid; base < ne; base += 8 * bd) {
            int v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = base + j * bd < ne ? a.part[base + j * bd] : 0;
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (v[j]) atomicAdd(&hist[(base + j * bd) & 31], v[j]);
        }
    }
    __syncthreads();
    if (tid < 32) a.hist[tid] = hist[tid];
    if (tid == 0) {
        a.counts[0] = hist[kHist];
        removed = 0;
        int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
        for (int i = 0; i < kHist; ++i) {
            const int sz = hist[i];
            if (sz > max1) { max3 = max2; max2 = max1; max1 = sz; ind3 = ind2; ind2 = ind1; ind1 = i; }
            else if (sz > max2) { max3 = max2; max2 = sz; ind3 = ind2; ind2 = i; }
            else if (sz > max3) { max3 = sz; ind3 = i; }
        }
        if ((float)max2 < __fmul_rn(0.1f, (float)max1)) { ind2 = -1; ind3 = -1; }
        else if ((float)max3 < __fmul_rn(0.1f, (float)max1)) { ind3 = -1; }
        top[0] = ind1; top[1] = ind2; top[2] = ind3;
    }
    __syncthreads();
    if (a.check_ori) {
        // eight features per thread with their loads in flight together
        int local = 0;
        const int n = a.A.n;
        for (int base = tid; base < n; base += 8 * bd) {
            int m[8], bin[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int i1 = base + j * bd;
                m[j] = i1 < n ? a.match_a[i1] : -1;
                bin[j] = i1 < n ? a.bin_a[i1] : 0;
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if (m[j] < 0 || bin[j] == top[0] || bin[j] == top[1] || bin[j] == top[2]) continue;
                a.match_a[base + j * bd] = -1;
                if (a.variant != ORBX_BOW_TRIANGULATION) a.match_b[m[j]] = -1;
                ++local;
            }
        }
        if (local) atomicAdd(&removed, local);
    }
    __syncthreads();
    if (tid == 0) a.counts[1] = hist[kHist] - removed;
    __syncthreads();
}

// Grid (nodes of the largest side A / 4, problems).  With a host tail (one
// problem: the drop-in call) the last workgroup to finish also runs the
// rotation pass and copies the outputs to the host, so the call is one launch.
__global__ __launch_bounds__(kBT) void k_bow_match(const BowBufs *pa, HostTail tail) {
    __shared__ uint8_t matched[kBT / 64][kBowNodeCap];
    const BowBufs a = pa[blockIdx.y];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int na_node = blockIdx.x * (kBT / 64) + wave;
    const long long t0 = a.clk ? (long long)wall_clock64() : 0;
    __shared__ int cnt[32];
    if (threadIdx.x < 32) cnt[threadIdx.x] = 0;
    __syncthreads();
    if (na_node < a.A.nnodes) bow_match_node(a, na_node, lane, matched[wave], cnt);
    __syncthreads();
    if (threadIdx.x < 32) a.part[32 * blockIdx.x + threadIdx.x] = cnt[threadIdx.x];
    if (a.clk && threadIdx.x == 0) {   // first start, last match end, longest workgroup
        const long long t1 = (long long)wall_clock64();
        atomicMin(&a.clk[0], t0);
        atomicMax(&a.clk[1], t1);
        atomicMax(&a.clk[5], t1 - t0);
    }
    if (!tail.flag) return;
    __shared__ int s_last;
    __threadfence();   // this workgroup's matches before its count
    __syncthreads();
    if (threadIdx.x == 0) s_last = atomicAdd(tail.done, 1u) == (uint32_t)(tail.blocks - 1);
    __syncthreads();
    if (!s_last) return;
    __threadfence();   // (acquire: every workgroup's matches)
    if (a.clk && threadIdx.x == 0) a.clk[2] = (long long)wall_clock64();
    bow_finish_problem(a);
    if (a.clk && threadIdx.x == 0) a.clk[3] = (long long)wall_clock64();
    tail_copy(tail);
    __threadfence_system();
    __syncthreads();
    if (a.clk && threadIdx.x == 0) a.clk[4] = (long long)wall_clock64();
    if (threadIdx.x == 0) __hip_atomic_store(tail.flag, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(1024) void k_bow_finish(const BowBufs *pa, HostTail tail) {   // one block per problem
    const BowBufs a = pa[blockIdx.x];
    bow_finish_problem(a);
    host_tail(tail);
}

}  // namespace

int bow_tail_blocks(const BowBufs *h, int np) {
    if (np != 1) return np;   // k_bow_finish, a workgroup per problem
    return (h[0].A.nnodes + kBT / 64 - 1) / (kBT / 64);   // k_bow_match's workgroups
}

hipError_t launch_bow(const BowBufs *h, const BowBufs *d, int np, const HostTail &tail, hipStream_t st) {
    if (np <= 0) return hipSuccess;
    if (tail.flag && tail.blocks != bow_tail_blocks(h, np)) return hipErrorInvalidValue;
    int nodes = 0;
    for (int k = 0; k < np; ++k) nodes = std::max(nodes, h[k].A.nnodes);
    const dim3 grid((nodes + kBT / 64 - 1) / (kBT / 64), np);
    for (int k = 0; k < np; ++k)
        if (h[k].nparts != (int)grid.x || (grid.x && !h[k].part)) return hipErrorInvalidValue;
    if (np == 1 && tail.flag && nodes > 0) {   // one launch: matching, rotation pass, outputs
        hipLaunchKernelGGL(k_bow_match, grid, dim3(kBT), 0, st, d, tail);
        return hipGetLastError();
    }
    if (tail.flag && np == 1) return hipErrorInvalidValue;   // (no nodes: nothing to elect a last workgroup)
    if (nodes > 0) hipLaunchKernelGGL(k_bow_match, grid, dim3(kBT), 0, st, d, HostTail{});
    hipLaunchKernelGGL(k_bow_finish, dim3(np), dim3(1024), 0, st, d, tail);
    return hipGetLastError();
}

}  // namespace orbx
