// orbx_device.h -- device-side buffers and kernel launchers (internal).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "orbx_plan.h"
#include "../../include/orbx.h"

namespace orbx {

// The per-level fields the per-keypoint / per-cell kernels need first, as a
// kernel-argument copy: they come from the scalar cache with the other
// arguments instead of a dependent load from the device tables.
struct LevelArgs {
    int w, h, pitch, out_off;
    int64_t pyr_off;
    float scale, patch_size;
};

// LDS layout of one k_fast launch (per wave), sized by the largest cell of the
// levels it covers.
struct FastLds {
    int ps;            // patch row stride (dword multiple)
    int patch_bytes, score_bytes, per_wave;
    int sw;            // score-map row stride (= ps: a survivor's patch offset indexes both)
    int list_cap;      // survivor-list entries (k_fast flushes before overflowing it)
    int pmag;          // ceil(2^24 / ps): row = (offset * pmag) >> 24 for offsets < 2^16
};
FastLds fast_lds(int mw, int mh);

// Plan tables resident in device memory (one copy per extractor plan).
struct DevPlan {
    LevelArgs la[kMaxLevels];
    const LevelGeom *lv;
    const Cell *cells;
    const ResizeTap *xtaps;
    const ResizeTap *ytaps;
    const ResizeCol *rcols;   // k_resize_d column groups / rows (Plan::rcols, rrows)
    const ResizeRow *rrows;
    const int4 *blur_tiles;   // (level, x0, y0, 0) per 64x16 output tile
    const uint32_t *slot_level;  // level of each output slot (out_cap entries): k_describe's one scalar load
    int nlevels, ncells, nblur_tiles;
    int gauss[7];
    int umax[16];
    int ini_th, min_th;
    int64_t pyr_bytes, blur_bytes, cand_cap;
    int out_cap, max_kps;
    int node_cap;             // quadtree node capacity (max over levels)
    int node_lds_bytes;       // dynamic LDS of the quadtree kernel
    int node_lds_bytes_w;     // ... of its 1024-thread form (launches of few frames; > 160 KB: not used)
    int dbg_stop;             // diagnostics only (ORBX_DBG_STOP): end k_quadtree after phase n (0 = off)
    const int4 *pyr_rgn;      // Plan::rgn (k_pyramid_rgn)
    int pyr_rgn_half;
};

// Per-batch device buffers.  Frame b of a batch uses the b-th slice of each.
struct FrameBufs {
    const uint8_t *img0;      // level 0 = caller's images
    int64_t img0_stride;      // bytes between frames
    int img0_pitch;           // bytes between rows
    uint8_t *pyr;             // levels >= 1, B * pyr_bytes
    uint8_t *blur;            // blurred levels, B * blur_bytes
    uint32_t *cand;           // per-cell candidate slots (iniThFAST lists), B * cand_cap
    uint32_t *cand2;          // same slots for the minThFAST lists
    int32_t *cell_count;      // B * ncells
    uint32_t *keys;           // per-level compacted candidates, B * cand_cap
    uint16_t *key_node;       // quadtree scratch, B * cand_cap
    uint8_t *key_q;           // quadtree scratch, B * cand_cap
    uint32_t *sel;            // selected keys per level slot, B * out_cap
    int32_t *level_count;     // B * kMaxLevels
    orbx_keypoint *kps;       // B * max_kps
    uint8_t *desc;            // B * max_kps * 32
    int32_t *nkps;            // B
};

// Matcher inputs/outputs for a batch of frame pairs (F1[b] -> F2[b]).
// The copy of a synchronous call's outputs into the pinned arena, done by the
// last workgroup of the call's last kernel instead of a kernel of its own
// (orbx_ws.h ws_tail): flag == nullptr means no tail.
struct HostTail {
    const uint4 *src; uint4 *dst; int n16;
    uint32_t *flag;   // pinned, raised after the copy (system scope)
    uint32_t *done;   // device counter of finished workgroups, zero before the kernel
    int blocks;       // workgroups of the kernel
};

#ifdef __HIPCC__
// The copy itself, eight loads in flight per thread before their stores (a
// loop of load -> store pairs is one memory round trip per element a thread
// copies, and the synchronous calls wait on every one of them).
__device__ inline void tail_copy(const HostTail &t) {
    const int bd = blockDim.x;
    for (int base = threadIdx.x; base < t.n16; base += 8 * bd) {
        uint4 v0 = t.src[base], v1, v2, v3, v4, v5, v6, v7;
        const int last = t.n16 - 1;   // (the tail of the range re-reads its last element)
        v1 = t.src[min(base + bd, last)];
        v2 = t.src[min(base + 2 * bd, last)];
        v3 = t.src[min(base + 3 * bd, last)];
        v4 = t.src[min(base + 4 * bd, last)];
        v5 = t.src[min(base + 5 * bd, last)];
        v6 = t.src[min(base + 6 * bd, last)];
        v7 = t.src[min(base + 7 * bd, last)];
        t.dst[base] = v0;
        if (base + bd < t.n16) t.dst[base + bd] = v1;
        if (base + 2 * bd < t.n16) t.dst[base + 2 * bd] = v2;
        if (base + 3 * bd < t.n16) t.dst[base + 3 * bd] = v3;
        if (base + 4 * bd < t.n16) t.dst[base + 4 * bd] = v4;
        if (base + 5 * bd < t.n16) t.dst[base + 5 * bd] = v5;
        if (base + 6 * bd < t.n16) t.dst[base + 6 * bd] = v6;
        if (base + 7 * bd < t.n16) t.dst[base + 7 * bd] = v7;
    }
}

// Every thread of every workgroup of the kernel calls this last.
__device__ inline void host_tail(const HostTail &t) {
    if (!t.flag) return;
    __shared__ int s_last;
    __threadfence();   // this workgroup's results before its count
    __syncthreads();
    if (threadIdx.x == 0) s_last = atomicAdd(t.done, 1u) == (uint32_t)(t.blocks - 1);
    __syncthreads();
    if (!s_last) return;
    __threadfence();   // (acquire: the other workgroups' results)
    tail_copy(t);
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(t.flag, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
#endif

struct MatchBufs {
    const orbx_keypoint *k1; const uint8_t *d1; const int32_t *n1; int64_t k1_stride;
    const orbx_keypoint *k2; const uint8_t *d2; const int32_t *n2; int64_t k2_stride;
    float *prev_xy;           // B * k1_stride * 2, in/out
    int32_t *matches12;       // B * k1_stride
    int32_t *nmatches;        // B
    float min_x, max_x, min_y, max_y;   // mnMinX, mnMaxX, mnMinY, mnMaxY: the 64 x 48 grid
    int window;
    float nnratio;
    int check_ori;
    int reset_prev;           // 1: prev_xy := F1 keypoint positions before matching
    long long *clocks;        // debug: phase timestamps of pair 0 (nullptr = off)
    HostTail tail;            // the synchronous host call's output copy (flag nullptr: none)
};

// Where a frame's pyramid lives: level 0 is the caller's image, levels >= 1
// are in the extractor's pyramid block (frame f at pyr + f * pyr_bytes).
struct PyrView {
    const uint8_t *img0; int64_t img0_stride; int img0_pitch;
    const uint8_t *pyr; int64_t pyr_bytes;
};

// Stereo matching of a batch of rectified pairs (Frame::ComputeStereoMatches).
// Pair b: left frame left_f0 + b*fstep of `left`, right frame right_f0 + b*fstep
// of `right`; keypoints kl/kr + b*kstride (descriptors likewise, 32 B each),
// counts nl/nr[b*nstride]; outputs ur/depth/sad + b*ostride, nkept[b].
struct StereoBufs {
    const LevelGeom *lv; int nlevels; int rows;   // rows: level-0 height (nRows)
    PyrView left, right; int left_f0, right_f0, fstep;
    const orbx_keypoint *kl; const uint8_t *dl; const int32_t *nl;
    const orbx_keypoint *kr; const uint8_t *dr; const int32_t *nr;
    int64_t kstride; int64_t nstride;
    int nr_cap;               // right keypoints indexed per pair (LDS capacity)
    float mbf, maxd;          // maxD = mbf / mb (Frame.cc:532-534)
    float *ur, *depth; int32_t *sad; int64_t ostride; int32_t *nkept;
    float *hout; int64_t hcap;   // optional host-visible copy of one pair's results (k_stereo_cut)
    uint8_t *bands; int64_t band_stride;   // optional per-pair band scratch (sorted once per pair), or nullptr
    int32_t *pair_done;          // optional per-pair workgroup counters (zero): the median cut fused into the search
};

// Projection searches (ORBmatcher SearchByProjection x4, Fuse x2): one frame
// per launch, query table in reference loop order.
struct ProjBufs {
    const orbx_keypoint *keys; const uint8_t *desc; const float *uright; const uint8_t *mp_state;
    const float *inv_sigma2;
    int n, nlevels;
    float min_x, max_x, min_y, max_y;
    const orbx_proj_query *q; const uint8_t *qdesc; int nq;
    int variant, th_dist; float nnratio; int check_ori;
    int32_t *q_idx, *q_dist, *kp_final, *nmatches;
    uint32_t *qtop; int32_t *qlen, *qbase;   // per query: 4 kept entries (16-B aligned), list length, pool base
    uint32_t *pool; int64_t pool_cap;        // candidate lists of all queries (global)
    // zeroed by the caller before a launch: list-pool counter (> pool_cap:
    // rerun with more) and count of `hard` claims
    unsigned long long *pool_top; uint32_t *hard_cnt;
    uint2 *hard; int hard_cap;               // (keypoint, query) claims past a query's 4 kept entries
    uint8_t *und;                            // nq: 0 decided, 1 open, 2 left to the in-order replay
    int32_t *stats;                          // optional: rounds, queries replayed in order
    int nblk;                                // search blocks of this problem (proj_blocks(nq))
};

// Vocabulary-node matchers (SearchByBoW x2, SearchForTriangulation).
constexpr int kBowNodeCap = 2048;   // largest side-B node (features) a wave handles
struct BowSideDev {
    const orbx_keypoint *keys; const uint8_t *desc; const uint8_t *flags; int n;
    const uint32_t *node_ids; const int32_t *node_offsets; const int32_t *node_features; int nnodes;
    const float *ang;   // keypoint angles (keys: triangulation only, nullptr otherwise)
};
struct BowBufs {
    BowSideDev A, B;
    int variant; float nnratio; int check_ori;
    const float *tri;   // F12[9], ex, ey, scale2[nlevels], sigma2[nlevels] (triangulation)
    float ex, ey; int nlevels;
    int32_t *match_a, *match_b;
    int8_t *bin_a;      // rotation bin per accepted A feature
    int32_t *hist;      // 30 bins
    int32_t *counts;    // [0] accepted, [1] nmatches after the rotation check
    const int4 *span;   // per side-A node: A's features [x, y), its side-B node's [z, w) (z == w: none)
    int32_t *part;      // per k_bow_match workgroup: 32 partial counts (30 bins, accepted, 0)
    int nparts;         // k_bow_match's workgroups per problem (its grid's x)
    long long *clk;     // debug (ORBX_BOW_CLOCKS): wall-clock marks of problem 0's one-launch call
};

enum Stage { kStageResize = 0, kStageBlur, kStageFast, kStageQuadtree, kStageDescribe, kStageMatch, kNumStages };

hipError_t launch_resize(const DevPlan &p, const Plan &hp, const FrameBufs &fb, int B, hipStream_t s);
// Per-level launches of the level-pipelined step (orbx_extractor_pipeline).
hipError_t launch_resize_level(const DevPlan &p, const Plan &hp, const FrameBufs &fb, int B, hipStream_t s, int l);
// (levels [l, l_end))
hipError_t launch_fast_level(const DevPlan &p, const Plan &hp, const FrameBufs &fb, int B, hipStream_t s, int l, int l_end);
hipError_t launch_quadtree_level(const DevPlan &p, const FrameBufs &fb, int B, hipStream_t s, int l, int l_end);
hipError_t launch_describe_level(const DevPlan &p, const Plan &hp, const FrameBufs &fb, int B, hipStream_t s, int l,
                                 int l_end);
hipError_t launch_blur(const DevPlan &p, const FrameBufs &fb, int B, hipStream_t s);
hipError_t launch_fast(const DevPlan &p, const Plan &hp, const FrameBufs &fb, int B, hipStream_t s);
hipError_t launch_quadtree(const DevPlan &p, const FrameBufs &fb, int B, hipStream_t s);
hipError_t launch_describe(const DevPlan &p, const FrameBufs &fb, int B, hipStream_t s);
hipError_t launch_match(const MatchBufs &mb, int B, int n1cap, int n2cap, int maxq, int maxc, hipStream_t s);
// sincosf restatement and fastAtan2 evaluated on the device over an array
// (exhaustive-check hook used by the GPU tests).
hipError_t launch_trig_check(const float *in, float *s, float *c, float *atan_out,
                             const float *ay, const float *ax, int n, int m, hipStream_t st);
hipError_t launch_stereo(const StereoBufs &a, int pairs, int nl_cap, hipStream_t s);
int stereo_lds_bytes(int rows, int nr_cap);
int64_t stereo_band_stride(int rows, int nr_cap);   // per-pair band scratch (StereoBufs::bands)
hipError_t launch_rgbd_samples(const float *dsample, const orbx_keypoint *kun, int n, float mbf, float *ur, float *depth,
                               int32_t *nkept, const HostTail &tail, hipStream_t st);
hipError_t launch_rgbd(const orbx_keypoint *kps, const orbx_keypoint *kun, const int32_t *nkps, int64_t kstride,
                       int kcap, const float *dmap, int64_t dstride, int dpitch, int w, int h, float mbf, float *ur,
                       float *depth, int64_t ostride, int32_t *nkept, int B, hipStream_t s);
// A batch of independent problems: h on the host, d the same array on the device.
hipError_t launch_proj(const ProjBufs *h, const ProjBufs *d, int np, const HostTail &tail, hipStream_t s);
int proj_tail_blocks(const ProjBufs *h, int np);   // the workgroups the host tail of launch_proj counts
int proj_blocks(int nq);
bool proj_fits(int n);   // the frame's grid fits the search kernel's LDS
hipError_t launch_bow(const BowBufs *h, const BowBufs *d, int np, const HostTail &tail, hipStream_t s);
int bow_tail_blocks(const BowBufs *h, int np);   // the workgroups the host tail of launch_bow counts

// DBoW2 vocabulary in slot order: the children of a node occupy consecutive
// slots (root = slot 0).  16 B per slot + 32-B descriptor + weight.
struct VocabNode {
    int32_t first;    // slot of the first child
    int32_t nchild;   // 0: a leaf (DBoW2's isLeaf() = children.empty())
    uint32_t word;    // word id (0 for a node without the file's leaf flag, as Node())
    uint32_t id;      // node id (file order)
};
struct VocabDev {
    const VocabNode *nodes; const uint8_t *desc; const double *weight;
    int k;            // largest child count
};
hipError_t launch_vocab_transform(const VocabDev &v, const uint8_t *feat, int n, int nid_level, uint32_t *o_word,
                                  double *o_weight, uint32_t *o_node, hipStream_t s);
int match_lds_bytes(int n1cap, int n2cap, int maxq, int maxc);
int quadtree_lds_bytes(int node_cap);
constexpr int kQuadRegKeys = 8 * 256;     // keys k_quadtree can keep in registers (6 or 8 per thread)
constexpr int kQuadRegKeysW = 10 * 1024;  // the same for its 1024-thread form (4 or 10 per thread)
bool resize_window_fits(const Plan &hp);
bool plan_resize_waves(Plan &hp);   // fills hp.rw, or leaves it empty (block kernel)
bool plan_pyr_regions(Plan &hp);   // fills hp.rgn, or leaves rgn_n = 0
bool use_pyr_regions(const Plan &hp, int B);

}  // namespace orbx
