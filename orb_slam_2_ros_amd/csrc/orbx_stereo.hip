// orbx_stereo.hip -- depth for stereo and RGB-D frames, per keypoint:
//
//   k_stereo_band    Frame::ComputeStereoMatches (Frame.cc:502-660): row-band
//                    Hamming search over the right keypoints, 11x11 SAD over 11
//                    offsets on the unblurred pyramid level, parabola fit.
//   k_stereo_cut     the median cut of Frame.cc:662-675.
//   k_rgbd_depth     Frame::ComputeStereoFromRGBD (Frame.cc:679-701).
//
// One block of k_stereo_band covers 256 left keypoints of one stereo pair
// (k_stereo_band_g: 16, a group of 16 lanes per keypoint, for launches too
// small to fill the chip, e.g. the single pair of the host-array call).  It
// first counting-sorts the pair's right keypoints by the first row of their
// band (vRowIndices of Frame.cc:512-529 without the per-row copies) into LDS,
// then every thread walks the bands that can contain its keypoint's row.  The
// reference keeps the first strictly smaller distance in candidate (= right
// index) order, i.e. the lexicographic minimum of (distance, index), which is
// what the walk computes in any order.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "orbx_device.h"
#include "orbx_wave.h"

namespace orbx {
namespace {

constexpr int kST = 256;
constexpr int kThOrbDist = (100 + 50) / 2;   // (TH_HIGH + TH_LOW) / 2, Frame.cc:507
constexpr int kSadW = 5, kSadL = 5;          // Frame.cc:597, 607

__device__ inline const uint8_t *view_level(const PyrView &v, const LevelGeom &g, int l, int f, int &pitch) {
    if (l == 0) {
        pitch = v.img0_pitch;
        return v.img0 + (int64_t)f * v.img0_stride;
    }
    pitch = g.pitch;
    return v.pyr + (int64_t)f * v.pyr_bytes + g.pyr_off;
}

__device__ inline int hamming(const uint32_t a[8], const uint8_t *d) {
    const uint4 q0 = *reinterpret_cast<const uint4 *>(d);
    const uint4 q1 = *reinterpret_cast<const uint4 *>(d + 16);
    return __popc(a[0] ^ q0.x) + __popc(a[1] ^ q0.y) + __popc(a[2] ^ q0.z) + __popc(a[3] ^ q0.w) +
           __popc(a[4] ^ q1.x) + __popc(a[5] ^ q1.y) + __popc(a[6] ^ q1.z) + __popc(a[7] ^ q1.w);
}

// In-place exclusive scan of n ints in LDS by the whole block; returns the total.
__device__ int block_scan_lds(int *a, int n, int *ws) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int per = (n + kST - 1) / kST;
    const int lo = min(n, tid * per), hi = min(n, lo + per);
    int s = 0;
    for (int i = lo; i < hi; ++i) s += a[i];
    int incl = s;
    for (int d = 1; d < 64; d <<= 1) {
        const int t = __shfl_up(incl, d);
        if (lane >= d) incl += t;
    }
    if (lane == 63) ws[wv] = incl;
    __syncthreads();
    int base = 0;
    for (int w = 0; w < wv; ++w) base += ws[w];
    const int total = ws[0] + ws[1] + ws[2] + ws[3];
    int run = base + incl - s;
    for (int i = lo; i < hi; ++i) {
        const int v = a[i];
        a[i] = run;
        run += v;
    }
    __syncthreads();
    return total;
}

// Bytes [o, o + 4*N) of the dwords d[] as N dwords (v_alignbyte).
template <int N>
__device__ inline void realign(const uint32_t *d, uint32_t o, uint32_t *e) {
#pragma unroll
    for (int k = 0; k < N; ++k) e[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], o);
}

__device__ inline int byte_of(const uint32_t *e, int j) { return (e[j >> 2] >> (8 * (j & 3))) & 0xFF; }

// Left row (11 px from column c0) and right row (21 px from column c0r) of
// one SAD window row, from dword-aligned loads.
__device__ inline void load_rows(const uint8_t *lrow, int c0, const uint8_t *rrow, int c0r, int l[11], int r[21]) {
    {
        const uint32_t o = (uint32_t)(reinterpret_cast<uintptr_t>(lrow + c0) & 3);
        const uint32_t *p = reinterpret_cast<const uint32_t *>(lrow + c0 - o);
        uint32_t d[4], e[3];
        d[0] = p[0]; d[1] = p[1]; d[2] = p[2];
        d[3] = o >= 2 ? p[3] : 0u;   // byte o + 10 lies in dword 3 only then
        realign<3>(d, o, e);
#pragma unroll
        for (int j = 0; j < 11; ++j) l[j] = byte_of(e, j);
    }
    {
        const uint32_t o = (uint32_t)(reinterpret_cast<uintptr_t>(rrow + c0r) & 3);
        const uint32_t *p = reinterpret_cast<const uint32_t *>(rrow + c0r - o);
        uint32_t d[7], e[6];
#pragma unroll
        for (int k = 0; k < 6; ++k) d[k] = p[k];
        d[6] = 0u;                   // byte o + 20 always lies in dword 5
        realign<6>(d, o, e);
#pragma unroll
        for (int j = 0; j < 21; ++j) r[j] = byte_of(e, j);
    }
}

// 11 pixels of a row from column c0, from dword-aligned loads.
__device__ inline void load_row11(const uint8_t *row, int c0, int px[11]) {
    const uint32_t o = (uint32_t)(reinterpret_cast<uintptr_t>(row + c0) & 3);
    const uint32_t *p = reinterpret_cast<const uint32_t *>(row + c0 - o);
    uint32_t d[4], e[3];
    d[0] = p[0]; d[1] = p[1]; d[2] = p[2];
    d[3] = o >= 2 ? p[3] : 0u;   // byte o + 10 lies in dword 3 only then
    realign<3>(d, o, e);
#pragma unroll
    for (int j = 0; j < 11; ++j) px[j] = byte_of(e, j);
}

// The pair's right keypoints counting-sorted by the first row of their band
// (vRowIndices, Frame.cc:512-529) into LDS; returns the widest band - 1.
struct Bands {
    int *rend;        // H + 1 counters, then bucket ends
    float *sx;        // right u, in band order
    int16_t *smaxr;   // last row of the band
    uint16_t *sidx;
    int8_t *soct;
};

__host__ __device__ inline int band_bytes(int rows, int nr_cap) {
    return ((rows + 1) * 4 + nr_cap * (4 + 2 + 2 + 1) + 15) & ~15;
}

__device__ inline Bands bands_in(uint8_t *lds, const StereoBufs &a) {
    Bands d;
    d.rend = reinterpret_cast<int *>(lds);
    d.sx = reinterpret_cast<float *>(d.rend + a.rows + 1);
    d.smaxr = reinterpret_cast<int16_t *>(d.sx + a.nr_cap);
    d.sidx = reinterpret_cast<uint16_t *>(d.smaxr + a.nr_cap);
    d.soct = reinterpret_cast<int8_t *>(d.sidx + a.nr_cap);
    return d;
}

__device__ int band_sort(const StereoBufs &a, int b, const Bands &d, int *ws, int *s_span) {
    const int tid = threadIdx.x;
    const int nr = min(a.nr[(int64_t)b * a.nstride], a.nr_cap);
    const int H = a.rows;
    const orbx_keypoint *kr = a.kr + (int64_t)b * a.kstride;
    // Rows outside the image (undefined behaviour in the reference) are dropped.
    for (int i = tid; i <= H; i += kST) d.rend[i] = 0;
    if (tid == 0) *s_span = 0;
    __syncthreads();
    int span = 0;
    for (int iR = tid; iR < nr; iR += kST) {
        const orbx_keypoint k = kr[iR];
        if (k.octave < 0 || k.octave >= a.nlevels) continue;
        const float r = __fmul_rn(2.0f, a.lv[k.octave].scale);
        const int maxr = (int)ceilf(__fadd_rn(k.y, r)), minr = (int)floorf(__fsub_rn(k.y, r));
        const int lo = max(minr, 0), hi = min(maxr, H - 1);
        if (lo > hi) continue;
        atomicAdd(&d.rend[lo], 1);
        span = max(span, hi - lo);
    }
    atomicMax(s_span, span);
    __syncthreads();
    block_scan_lds(d.rend, H + 1, ws);
    for (int iR = tid; iR < nr; iR += kST) {
        const orbx_keypoint k = kr[iR];
        if (k.octave < 0 || k.octave >= a.nlevels) continue;
        const float r = __fmul_rn(2.0f, a.lv[k.octave].scale);
        const int maxr = (int)ceilf(__fadd_rn(k.y, r)), minr = (int)floorf(__fsub_rn(k.y, r));
        const int lo = max(minr, 0), hi = min(maxr, H - 1);
        if (lo > hi) continue;
        const int pos = atomicAdd(&d.rend[lo], 1);   // afterwards rend[m] = end of band m
        d.sx[pos] = k.x;
        d.smaxr[pos] = (int16_t)hi;
        d.sidx[pos] = (uint16_t)iR;
        d.soct[pos] = (int8_t)k.octave;
    }
    __syncthreads();
    return *s_span;
}

#ifndef ORBX_STEREO_WALK
#define ORBX_STEREO_WALK 4
#endif
constexpr int kWalk = ORBX_STEREO_WALK;   // band positions per batch of descriptor loads

// SCR: the pair's bands sorted once by k_band_sort into its scratch (read
// from L2), instead of every block sorting them into its LDS.
template <bool SCR>
__device__ __attribute__((always_inline)) void stereo_band_body(const StereoBufs &a, uint8_t *lds) {
    __shared__ int ws[4];
    __shared__ int s_span;
    const int b = blockIdx.y, tid = threadIdx.x;
    const int nl = a.nl[(int64_t)b * a.nstride];
    const int i0 = blockIdx.x * kST;
    if (i0 >= nl) return;
    const int H = a.rows;
    const orbx_keypoint *kl = a.kl + (int64_t)b * a.kstride;
    const orbx_keypoint *kr = a.kr + (int64_t)b * a.kstride;
    const uint8_t *dl = a.dl + (int64_t)b * a.kstride * 32;
    const uint8_t *dr = a.dr + (int64_t)b * a.kstride * 32;
    // 1. vRowIndices (Frame.cc:517-529): right keypoint iR lies in rows
    //    [floor(y - r), ceil(y + r)], r = 2 * scale[octave].
    Bands bd;
    int span;
    if constexpr (SCR) {
        uint8_t *scr = a.bands + (int64_t)b * a.band_stride;
        bd = bands_in(scr, a);
        span = reinterpret_cast<const int *>(scr + band_bytes(a.rows, a.nr_cap))[0];
    } else {
        bd = bands_in(lds, a);
        span = band_sort(a, b, bd, ws, &s_span);
    }
    const int *rend = bd.rend;
    const float *sx = bd.sx;
    const int16_t *smaxr = bd.smaxr;
    const uint16_t *sidx = bd.sidx;
    const int8_t *soct = bd.soct;

    const int iL = i0 + tid;
    if (iL >= nl) return;
    float *ur_out = a.ur + (int64_t)b * a.ostride;
    float *dp_out = a.depth + (int64_t)b * a.ostride;
    int32_t *sad_out = a.sad + (int64_t)b * a.ostride;
    ur_out[iL] = -1.0f;
    dp_out[iL] = -1.0f;
    sad_out[iL] = -1;
    const orbx_keypoint kL = kl[iL];
    const float vL = kL.y, uL = kL.x;
    const int levelL = kL.octave;
    if (!(vL >= 0.0f) || vL >= (float)H || levelL < 0 || levelL >= a.nlevels) return;
    const int v = (int)vL;
    const float minU = __fsub_rn(uL, a.maxd), maxU = uL;   // uL - minD, minD = 0
    if (maxU < 0.0f) return;

    // 2. best Hamming distance over the band (Frame.cc:556-585)
    uint32_t q[8];
    {
        const uint4 q0 = *reinterpret_cast<const uint4 *>(dl + 32 * (int64_t)iL);
        const uint4 q1 = *reinterpret_cast<const uint4 *>(dl + 32 * (int64_t)iL + 16);
        q[0] = q0.x; q[1] = q0.y; q[2] = q0.z; q[3] = q0.w;
        q[4] = q1.x; q[5] = q1.y; q[6] = q1.z; q[7] = q1.w;
    }
    // the bands starting in rows [v - span, v] are one contiguous range of the
    // sort; kWalk positions at a time, their descriptor loads issued together
    // (the (distance, index) minimum does not depend on the visiting order)
    const int m0 = max(0, v - span);
    const int p0 = m0 ? rend[m0 - 1] : 0, p1 = rend[v];
    uint32_t bk = 100u << 16;   // (distance << 16) | index; TH_HIGH, index 0
    for (int pos = p0; pos < p1; pos += kWalk) {
        bool ok[kWalk];
        int iR[kWalk];
#pragma unroll
        for (int j = 0; j < kWalk; ++j) {
            const int pj = pos + j;
            ok[j] = false;
            iR[j] = 0;
            if (pj < p1 && smaxr[pj] >= v) {
                const int o = soct[pj];
                const float uR = sx[pj];
                if (o >= levelL - 1 && o <= levelL + 1 && uR >= minU && uR <= maxU) {
                    ok[j] = true;
                    iR[j] = sidx[pj];
                }
            }
        }
        uint4 e0[kWalk], e1[kWalk];
#pragma unroll
        for (int j = 0; j < kWalk; ++j) {
            if (ok[j]) {
                const uint4 *dp = reinterpret_cast<const uint4 *>(dr + 32 * (int64_t)iR[j]);
                e0[j] = dp[0];
                e1[j] = dp[1];
            }
        }
#pragma unroll
        for (int j = 0; j < kWalk; ++j) {
            if (ok[j]) {
                const int dist = __popc(q[0] ^ e0[j].x) + __popc(q[1] ^ e0[j].y) + __popc(q[2] ^ e0[j].z) +
                                 __popc(q[3] ^ e0[j].w) + __popc(q[4] ^ e1[j].x) + __popc(q[5] ^ e1[j].y) +
                                 __popc(q[6] ^ e1[j].z) + __popc(q[7] ^ e1[j].w);
                bk = min(bk, ((uint32_t)dist << 16) | (uint32_t)iR[j]);
            }
        }
    }
    const int best = (int)(bk >> 16), bidx = (int)(bk & 0xFFFF);
    if (best >= kThOrbDist) return;

    // 3. SAD over 11 offsets (Frame.cc:587-629).  Windows the reference's
    //    Mat::rowRange / colRange would assert on are reported as no match.
    const LevelGeom g = a.lv[levelL];
    const float sf = g.inv_scale;
    const float suL = roundf(__fmul_rn(uL, sf)), svL = roundf(__fmul_rn(vL, sf));
    const float suR0 = roundf(__fmul_rn(kr[bidx].x, sf));
    if (svL - kSadW < 0.0f || svL + kSadW + 1 > (float)g.h || suL - kSadW < 0.0f || suL + kSadW + 1 > (float)g.w)
        return;
    const float iniu = suR0 + kSadL - kSadW, endu = suR0 + kSadL + kSadW + 1;
    if (iniu < 0.0f || endu >= (float)g.w) return;
    if (suR0 - kSadL - kSadW < 0.0f) return;
    int lp, rp;
    const uint8_t *IL = view_level(a.left, g, levelL, a.left_f0 + b * a.fstep, lp);
    const uint8_t *IR = view_level(a.right, g, levelL, a.right_f0 + b * a.fstep, rp);
    const int r0 = (int)svL - kSadW, cl0 = (int)suL - kSadW, cr0 = (int)suR0 - kSadL - kSadW;
    int l[11], r[21];
    load_rows(IL + (int64_t)(r0 + kSadW) * lp, cl0, IR + (int64_t)(r0 + kSadW) * rp, cr0, l, r);
    int kc[11];   // center difference IL(w,w) - IR(w,w) per offset
#pragma unroll
    for (int i = 0; i < 11; ++i) kc[i] = l[kSadW] - r[i + kSadW];
    int sad[11];
#pragma unroll
    for (int i = 0; i < 11; ++i) sad[i] = 0;
    for (int rr = 0; rr < 2 * kSadW + 1; ++rr) {
        load_rows(IL + (int64_t)(r0 + rr) * lp, cl0, IR + (int64_t)(r0 + rr) * rp, cr0, l, r);
#pragma unroll
        for (int i = 0; i < 11; ++i)
#pragma unroll
            for (int c = 0; c < 11; ++c) sad[i] += abs(l[c] - r[c + i] - kc[i]);
    }
    int bestSad = sad[0], bestInc = 0;   // first strict minimum (exact integer floats)
#pragma unroll
    for (int i = 1; i < 11; ++i)
        if (sad[i] < bestSad) { bestSad = sad[i]; bestInc = i; }
    if (bestInc == 0 || bestInc == 2 * kSadL) return;
    float d1 = 0.f, d2 = 0.f, d3 = 0.f;
#pragma unroll
    for (int i = 1; i < 10; ++i)
        if (i == bestInc) { d1 = (float)sad[i - 1]; d2 = (float)sad[i]; d3 = (float)sad[i + 1]; }
    // 4. parabola fit and depth (Frame.cc:631-657)
    const float deltaR = __fdiv_rn(__fsub_rn(d1, d3), __fmul_rn(2.0f, __fsub_rn(__fadd_rn(d1, d3), __fmul_rn(2.0f, d2))));
    if (deltaR < -1.0f || deltaR > 1.0f) return;
    float bestuR = __fmul_rn(g.scale, __fadd_rn(__fadd_rn(suR0, (float)(bestInc - kSadL)), deltaR));
    float disparity = __fsub_rn(uL, bestuR);
    if (disparity >= 0.0f && disparity < a.maxd) {
        if (disparity <= 0.0f) {
            disparity = 0.01f;                         // (float)0.01
            bestuR = (float)__dsub_rn((double)uL, 0.01);   // uL - 0.01 in double
        }
        dp_out[iL] = __fdiv_rn(a.mbf, disparity);
        ur_out[iL] = bestuR;
        sad_out[iL] = bestSad;
    }
}


// With a.pair_done (batched steps) the last of a pair's workgroups to finish
// also runs the pair's median cut (no k_stereo_cut launch); it resets the
// pair's counter for the next step.  Defined after stereo_cut_pair.
template <bool SCR>
__global__ __launch_bounds__(kST) void k_stereo_band(StereoBufs a);

// The same search with a group of kG lanes per left keypoint (kST / kG
// keypoints per block): the lanes stride over the keypoint's band range and
// reduce (distance, index) to its lexicographic minimum; lane i < 11 of the
// group sums the SAD of offset i.  For launches of few pairs, where one lane
// per keypoint leaves the chip idle and each lane's serial search is the
// latency.
constexpr int kG = 16;

__device__ inline uint32_t group_min_u32(uint32_t v) {
#pragma unroll
    for (int o = kG / 2; o > 0; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o));
    return v;
}

// Steps 2-4 for the kPer left keypoints of this block, a group of kG lanes
// each, over the pair's sorted bands (LDS or the pair's scratch).
__device__ __forceinline__ void group_search(const StereoBufs &a, int b, const Bands &bd, int span) {
    const int tid = threadIdx.x;
    const int nl = a.nl[(int64_t)b * a.nstride];
    const int i0 = blockIdx.x * (kST / kG);
    const int H = a.rows;
    const orbx_keypoint *kl = a.kl + (int64_t)b * a.kstride;
    const orbx_keypoint *kr = a.kr + (int64_t)b * a.kstride;
    const uint8_t *dl = a.dl + (int64_t)b * a.kstride * 32;
    const uint8_t *dr = a.dr + (int64_t)b * a.kstride * 32;
    const int g = tid & (kG - 1);
    const int iL = i0 + tid / kG;
    if (iL >= nl) return;   // (whole groups leave together)
    float *ur_out = a.ur + (int64_t)b * a.ostride;
    float *dp_out = a.depth + (int64_t)b * a.ostride;
    int32_t *sad_out = a.sad + (int64_t)b * a.ostride;
    if (g == 0) {
        ur_out[iL] = -1.0f;
        dp_out[iL] = -1.0f;
        sad_out[iL] = -1;
    }
    const orbx_keypoint kL = kl[iL];
    const float vL = kL.y, uL = kL.x;
    const int levelL = kL.octave;
    if (!(vL >= 0.0f) || vL >= (float)H || levelL < 0 || levelL >= a.nlevels) return;
    const int v = (int)vL;
    const float minU = __fsub_rn(uL, a.maxd), maxU = uL;
    if (maxU < 0.0f) return;

    // 2. best Hamming distance over the band (Frame.cc:556-585): the bands
    //    starting in rows [v - span, v] are one contiguous range of the sort
    uint32_t q[8];
    {
        const uint4 q0 = *reinterpret_cast<const uint4 *>(dl + 32 * (int64_t)iL);
        const uint4 q1 = *reinterpret_cast<const uint4 *>(dl + 32 * (int64_t)iL + 16);
        q[0] = q0.x; q[1] = q0.y; q[2] = q0.z; q[3] = q0.w;
        q[4] = q1.x; q[5] = q1.y; q[6] = q1.z; q[7] = q1.w;
    }
    const int m0 = max(0, v - span);
    const int p0 = m0 ? bd.rend[m0 - 1] : 0, p1 = bd.rend[v];
    uint32_t bk = 100u << 16;   // (distance << 16) | index; TH_HIGH, index 0
    for (int pos = p0 + g; pos < p1; pos += kG) {
        if (bd.smaxr[pos] < v) continue;
        const int o = bd.soct[pos];
        if (o < levelL - 1 || o > levelL + 1) continue;
        const float uR = bd.sx[pos];
        if (!(uR >= minU && uR <= maxU)) continue;
        const int iR = bd.sidx[pos];
        bk = min(bk, ((uint32_t)hamming(q, dr + 32 * (int64_t)iR) << 16) | (uint32_t)iR);
    }
    bk = group_min_u32(bk);
    const int best = (int)(bk >> 16), bidx = (int)(bk & 0xFFFF);
    if (best >= kThOrbDist) return;

    // 3. SAD over 11 offsets (Frame.cc:587-629), offset g on lane g
    const LevelGeom lg = a.lv[levelL];
    const float sf = lg.inv_scale;
    const float suL = roundf(__fmul_rn(uL, sf)), svL = roundf(__fmul_rn(vL, sf));
    const float suR0 = roundf(__fmul_rn(kr[bidx].x, sf));
    if (svL - kSadW < 0.0f || svL + kSadW + 1 > (float)lg.h || suL - kSadW < 0.0f || suL + kSadW + 1 > (float)lg.w)
        return;
    const float iniu = suR0 + kSadL - kSadW, endu = suR0 + kSadL + kSadW + 1;
    if (iniu < 0.0f || endu >= (float)lg.w) return;
    if (suR0 - kSadL - kSadW < 0.0f) return;
    int lp, rp;
    const uint8_t *IL = view_level(a.left, lg, levelL, a.left_f0 + b * a.fstep, lp);
    const uint8_t *IR = view_level(a.right, lg, levelL, a.right_f0 + b * a.fstep, rp);
    const int r0 = (int)svL - kSadW, cl0 = (int)suL - kSadW, cr0 = (int)suR0 - kSadL - kSadW;
    // this lane's offset: the right window starts i columns further (lanes
    // 11..15 repeat offset 10 and drop out of the minimum)
    const int i = min(g, 2 * kSadL);
    int l[11], r[11];
    load_row11(IL + (int64_t)(r0 + kSadW) * lp, cl0, l);
    load_row11(IR + (int64_t)(r0 + kSadW) * rp, cr0 + i, r);
    const int kc = l[kSadW] - r[kSadW];   // IL(w,w) - IR(w,w) at this offset
    int sad = 0;
    for (int rr = 0; rr < 2 * kSadW + 1; ++rr) {
        load_row11(IL + (int64_t)(r0 + rr) * lp, cl0, l);
        load_row11(IR + (int64_t)(r0 + rr) * rp, cr0 + i, r);
#pragma unroll
        for (int c = 0; c < 11; ++c) sad += abs(l[c] - r[c] - kc);
    }
    // first strict minimum over the 11 offsets
    const uint32_t sk = group_min_u32(g <= 2 * kSadL ? ((uint32_t)sad << 4) | (uint32_t)g : 0xFFFFFFFFu);
    const int bestSad = (int)(sk >> 4), bestInc = (int)(sk & 15);
    const int gb = tid & ~(kG - 1) & 63;   // the group's first lane in the wave
    const int s1 = __shfl(sad, gb + max(bestInc - 1, 0)), s3 = __shfl(sad, gb + min(bestInc + 1, 2 * kSadL));
    if (g != 0 || bestInc == 0 || bestInc == 2 * kSadL) return;
    const float d1 = (float)s1, d2 = (float)bestSad, d3 = (float)s3;
    // 4. parabola fit and depth (Frame.cc:631-657)
    const float deltaR = __fdiv_rn(__fsub_rn(d1, d3), __fmul_rn(2.0f, __fsub_rn(__fadd_rn(d1, d3), __fmul_rn(2.0f, d2))));
    if (deltaR < -1.0f || deltaR > 1.0f) return;
    float bestuR = __fmul_rn(lg.scale, __fadd_rn(__fadd_rn(suR0, (float)(bestInc - kSadL)), deltaR));
    float disparity = __fsub_rn(uL, bestuR);
    if (disparity >= 0.0f && disparity < a.maxd) {
        if (disparity <= 0.0f) {
            disparity = 0.01f;
            bestuR = (float)__dsub_rn((double)uL, 0.01);
        }
        dp_out[iL] = __fdiv_rn(a.mbf, disparity);
        ur_out[iL] = bestuR;
        sad_out[iL] = bestSad;
    }
}

__global__ __launch_bounds__(kST) void k_stereo_band_g(StereoBufs a) {
    extern __shared__ __align__(16) uint8_t lds[];
    __shared__ int ws[4];
    __shared__ int s_span;
    const int b = blockIdx.y;
    if (blockIdx.x * (kST / kG) >= a.nl[(int64_t)b * a.nstride]) return;
    const Bands bd = bands_in(lds, a);
    const int span = band_sort(a, b, bd, ws, &s_span);
    group_search(a, b, bd, span);
}

// The bands of each pair sorted once (k_band_sort: the LDS image of band_sort
// copied to the pair's scratch, span in its last dword), then the grouped
// search over the scratch (k_stereo_band_gs), so a batch of pairs runs the
// 16-lane search on thousands of small blocks without every block re-sorting
// its pair's right keypoints.  Measured no faster than k_stereo_band at the
// bench's batches (EuRoC 123.6 -> 122.5 k, KITTI 77.1 -> 75.4 k pairs/s,
// profiles/r04_ab_stereo_sort_once.txt): off unless ORBX_STEREO_SORT_ONCE=1.
__global__ __launch_bounds__(kST) void k_band_sort(StereoBufs a) {
    extern __shared__ __align__(16) uint8_t lds[];
    __shared__ int ws[4];
    __shared__ int s_span;
    const int b = blockIdx.x;
    const Bands bd = bands_in(lds, a);
    const int span = band_sort(a, b, bd, ws, &s_span);
    const int bytes = band_bytes(a.rows, a.nr_cap);
    uint4 *dst = reinterpret_cast<uint4 *>(a.bands + (int64_t)b * a.band_stride);
    const uint4 *src = reinterpret_cast<const uint4 *>(lds);
    for (int i = threadIdx.x; i < bytes / 16; i += kST) dst[i] = src[i];
    if (threadIdx.x == 0) reinterpret_cast<int *>(a.bands + (int64_t)b * a.band_stride + bytes)[0] = span;
}

__global__ __launch_bounds__(kST) void k_stereo_band_gs(StereoBufs a) {
    const int b = blockIdx.y;
    if (blockIdx.x * (kST / kG) >= a.nl[(int64_t)b * a.nstride]) return;
    uint8_t *scr = a.bands + (int64_t)b * a.band_stride;
    const int span = reinterpret_cast<const int *>(scr + band_bytes(a.rows, a.nr_cap))[0];
    group_search(a, b, bands_in(scr, a), span);
}

// Median cut (Frame.cc:662-675): entries with SAD >= 1.5f*1.4f*median are
// dropped; the median is element size/2 of the ascending SAD order.  SADs are
// < 2^16 (121 * 510), so the median is a two-pass 8-bit radix select; each
// pass finds its bucket by a block scan of the 256-bin histogram (thread t
// owns bin t).  With `hout` set (one pair, the host-array call) the block also
// writes the results into that host-visible buffer: uRight at [0, nl), depth
// at [hcap, hcap + nl), the kept count at 2 * hcap.
__device__ inline int hist_select(const int *hist, int k, int *ws, int *s_sel, int *s_rank) {
    const int tid = threadIdx.x;
    const int h = hist[tid];
    const int incl = wave_incl_scan_i32(h);
    if ((tid & 63) == 63) ws[tid >> 6] = incl;
    if (tid == 0) *s_sel = -1;
    __syncthreads();
    int base = 0;
    for (int w = 0; w < (tid >> 6); ++w) base += ws[w];
    const int ex = base + incl - h;   // bins before t
    if (h > 0 && ex <= k && k < ex + h) { *s_sel = tid; *s_rank = k - ex; }
    const int total = ws[0] + ws[1] + ws[2] + ws[3];
    __syncthreads();
    return total;
}

__device__ __attribute__((always_inline)) void stereo_cut_pair(const StereoBufs &a, int b) {
    __shared__ int hist[256];
    __shared__ int ws[4];
    __shared__ int s_sel, s_rank, s_kept;
    const int tid = threadIdx.x;
    const int nl = a.nl[(int64_t)b * a.nstride];
    float *ur = a.ur + (int64_t)b * a.ostride;
    float *dp = a.depth + (int64_t)b * a.ostride;
    const int32_t *sad = a.sad + (int64_t)b * a.ostride;
    hist[tid] = 0;
    __syncthreads();
    for (int i = tid; i < nl; i += kST) {
        const int s = sad[i];
        if (s >= 0) atomicAdd(&hist[s >> 8], 1);
    }
    __syncthreads();
    // (with nothing to cut, k = 0 finds no bin: the reference reads an empty vector)
    int total = 0;
    {
        int probe = hist[tid];
        probe = wave_sum_i32(probe);
        if ((tid & 63) == 0) ws[tid >> 6] = probe;
        __syncthreads();
        total = ws[0] + ws[1] + ws[2] + ws[3];
        __syncthreads();
    }
    int kept = total;
    if (total > 0) {
        (void)hist_select(hist, total / 2, ws, &s_sel, &s_rank);
        const int hi = s_sel, rank = s_rank;
        hist[tid] = 0;
        __syncthreads();
        for (int i = tid; i < nl; i += kST) {
            const int s = sad[i];
            if (s >= 0 && (s >> 8) == hi) atomicAdd(&hist[s & 0xFF], 1);
        }
        __syncthreads();
        (void)hist_select(hist, rank, ws, &s_sel, &s_rank);
        const int med = (hi << 8) | s_sel;
        constexpr float kCut = 1.5f * 1.4f;   // folded in float, as the reference's constant product
        const float thDist = __fmul_rn(kCut, (float)med);
        if (tid == 0) s_kept = total;
        __syncthreads();
        int dropped = 0;
        for (int i = tid; i < nl; i += kST) {
            const int s = sad[i];
            if (s >= 0 && !((float)s < thDist)) {
                ur[i] = -1.0f;
                dp[i] = -1.0f;
                ++dropped;
            }
        }
        if (dropped) atomicSub(&s_kept, dropped);
        __syncthreads();
        kept = s_kept;
    }
    if (tid == 0) a.nkept[b] = kept;
    if (a.hout) {
        for (int i = tid; i < nl; i += kST) {   // (each thread rereads only its own entries)
            a.hout[i] = ur[i];
            a.hout[a.hcap + i] = dp[i];
        }
        if (tid == 0) reinterpret_cast<int32_t *>(a.hout)[2 * a.hcap] = kept;
    }
}

__global__ __launch_bounds__(kST) void k_stereo_cut(StereoBufs a) { stereo_cut_pair(a, blockIdx.x); }

template <bool SCR>
__global__ __launch_bounds__(kST) void k_stereo_band(StereoBufs a) {
    extern __shared__ __align__(16) uint8_t lds[];
    stereo_band_body<SCR>(a, lds);
    if (!a.pair_done) return;
    const int b = blockIdx.y;
    const int nl = a.nl[(int64_t)b * a.nstride];
    const int nact = (nl + kST - 1) / kST;   // the pair's workgroups that searched
    if (nl <= 0) {
        if (blockIdx.x != 0) return;   // (an empty pair: its first workgroup cuts)
    } else {
        if ((int)blockIdx.x >= nact) return;
        __shared__ int s_last;
        __threadfence();   // this workgroup's depths before its count
        __syncthreads();
        if (threadIdx.x == 0) s_last = atomicAdd(&a.pair_done[b], 1) == nact - 1;
        __syncthreads();
        if (!s_last) return;
        __threadfence();   // (acquire: the pair's other workgroups' depths)
        if (threadIdx.x == 0) a.pair_done[b] = 0;   // ready for the next step (stream order)
    }
    stereo_cut_pair(a, b);
}

// Frame::ComputeStereoFromRGBD (Frame.cc:679-701) for undistorted frames
// (mvKeysUn == mvKeys when k1 == 0, Frame.cc:440-444).
__global__ __launch_bounds__(kST) void k_rgbd_depth(const orbx_keypoint *kps, const orbx_keypoint *kun,
                                                    const int32_t *nkps, int64_t kstride, const float *dmap,
                                                    int64_t dstride, int dpitch, int w, int h, float mbf, float *ur,
                                                    float *depth, int64_t ostride, int32_t *nkept) {
    const int b = blockIdx.y, i = blockIdx.x * kST + threadIdx.x;
    const bool live = i < nkps[b];
    bool got = false;
    if (live) {
    const orbx_keypoint k = kps[(int64_t)b * kstride + i];
    float u_out = -1.0f, d_out = -1.0f;
    const int v = (int)k.y, u = (int)k.x;
    if (v >= 0 && v < h && u >= 0 && u < w) {
        const float d = *reinterpret_cast<const float *>(reinterpret_cast<const uint8_t *>(dmap) + (int64_t)b * dstride +
                                                         (int64_t)v * dpitch + 4 * (int64_t)u);
        if (d > 0.0f) {
            d_out = d;
            u_out = __fsub_rn(kun[(int64_t)b * kstride + i].x, __fdiv_rn(mbf, d));
            got = true;
        }
    }
    ur[(int64_t)b * ostride + i] = u_out;
    depth[(int64_t)b * ostride + i] = d_out;
    }
    const uint64_t m = __ballot(got);
    if ((threadIdx.x & 63) == 0 && m) atomicAdd(&nkept[b], __popcll(m));
}

// The host call's form: the depth samples at the keypoints (imDepth.at<float>(v, u),
// gathered by the host so the map itself never crosses PCIe: 4 B per keypoint
// instead of the whole CV_32F image), then the same arithmetic as k_rgbd_depth.
__global__ __launch_bounds__(kST) void k_rgbd_samples(const float *dsample, const orbx_keypoint *kun, int n, float mbf,
                                                      float *ur, float *depth, int32_t *nkept, HostTail tail) {
    const int i = blockIdx.x * kST + threadIdx.x;
    bool got = false;
    if (i < n) {
        const float d = dsample[i];
        float u_out = -1.0f, d_out = -1.0f;
        if (d > 0.0f) {
            d_out = d;
            u_out = __fsub_rn(kun[i].x, __fdiv_rn(mbf, d));
            got = true;
        }
        ur[i] = u_out;
        depth[i] = d_out;
    }
    const uint64_t m = __ballot(got);
    if ((threadIdx.x & 63) == 0 && m) atomicAdd(nkept, __popcll(m));
    host_tail(tail);
}

}  // namespace

int stereo_lds_bytes(int rows, int nr_cap) { return band_bytes(rows, nr_cap); }

int64_t stereo_band_stride(int rows, int nr_cap) { return ((int64_t)stereo_lds_bytes(rows, nr_cap) + 16 + 255) & ~255; }

hipError_t launch_stereo(const StereoBufs &a, int pairs, int nl_cap, hipStream_t st) {
    if (pairs <= 0) return hipSuccess;
    const int bytes = stereo_lds_bytes(a.rows, a.nr_cap);
    if (a.bands && pairs > 1) {
        if (bytes > 64 * 1024 &&
            hipFuncSetAttribute(reinterpret_cast<const void *>(k_band_sort), hipFuncAttributeMaxDynamicSharedMemorySize,
                                bytes) != hipSuccess)
            return hipErrorInvalidValue;
        hipLaunchKernelGGL(k_band_sort, dim3(pairs), dim3(kST), bytes, st, a);
        static const bool grouped_scr = [] {
            const char *e = std::getenv("ORBX_STEREO_SORT_ONCE");
            return e && e[0] == '1' && e[1] == 'g';   // "1g": the 16-lane search over the scratch
        }();
        if (grouped_scr)
            hipLaunchKernelGGL(k_stereo_band_gs, dim3((nl_cap + kST / kG - 1) / (kST / kG), pairs), dim3(kST), 0, st, a);
        else {
            StereoBufs g = a;
            g.pair_done = nullptr;
            hipLaunchKernelGGL(k_stereo_band<true>, dim3((nl_cap + kST - 1) / kST, pairs), dim3(kST), 0, st, g);
        }
        hipLaunchKernelGGL(k_stereo_cut, dim3(pairs), dim3(kST), 0, st, a);
        return hipGetLastError();
    }
    // a lane per keypoint while that fills the chip, else a group of kG lanes
    const bool grouped = (int64_t)pairs * ((nl_cap + kST - 1) / kST) < 256;
    const void *fn = grouped ? reinterpret_cast<const void *>(k_stereo_band_g)
                             : reinterpret_cast<const void *>(k_stereo_band<false>);
    if (bytes > 64 * 1024 && hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes) != hipSuccess)
        return hipErrorInvalidValue;
    if (grouped) {
        StereoBufs g = a;
        g.pair_done = nullptr;
        hipLaunchKernelGGL(k_stereo_band_g, dim3((nl_cap + kST / kG - 1) / (kST / kG), pairs), dim3(kST), bytes, st, g);
    } else {
        hipLaunchKernelGGL(k_stereo_band<false>, dim3((nl_cap + kST - 1) / kST, pairs), dim3(kST), bytes, st, a);
        if (a.pair_done) return hipGetLastError();   // (the cut ran in the search's last workgroups)
    }
    hipLaunchKernelGGL(k_stereo_cut, dim3(pairs), dim3(kST), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_rgbd_samples(const float *dsample, const orbx_keypoint *kun, int n, float mbf, float *ur, float *depth,
                               int32_t *nkept, const HostTail &tail, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    if (tail.flag && tail.blocks != (n + kST - 1) / kST) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_rgbd_samples, dim3((n + kST - 1) / kST), dim3(kST), 0, st, dsample, kun, n, mbf, ur, depth,
                       nkept, tail);
    return hipGetLastError();
}

hipError_t launch_rgbd(const orbx_keypoint *kps, const orbx_keypoint *kun, const int32_t *nkps, int64_t kstride,
                       int kcap, const float *dmap, int64_t dstride, int dpitch, int w, int h, float mbf, float *ur,
                       float *depth, int64_t ostride, int32_t *nkept, int B, hipStream_t st) {
    if (B <= 0) return hipSuccess;
    if (hipMemsetAsync(nkept, 0, sizeof(int32_t) * B, st) != hipSuccess) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_rgbd_depth, dim3((kcap + kST - 1) / kST, B), dim3(kST), 0, st, kps, kun ? kun : kps, nkps,
                       kstride, dmap, dstride, dpitch, w, h, mbf, ur, depth, ostride, nkept);
    return hipGetLastError();
}

}  // namespace orbx
