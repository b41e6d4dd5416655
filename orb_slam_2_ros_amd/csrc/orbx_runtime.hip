// orbx_runtime.hip -- extractor object, device buffers, streams and the C ABI
// declared in include/orbx.h.
//
// Memory layout per extractor (HBM, all frames of a batch side by side):
//   pyramid   B x pyr_bytes    levels 1..7, rows padded to 64 B (level 0 is the
//                              caller's image, read in place)
//   blurred   B x blur_bytes   levels 0..7
//   cand      B x cand_cap     per-cell FAST slots (u32 packed x|y<<12|s<<24)
//   keys etc. B x cand_cap     quadtree scratch (compacted keys, node ids)
//   results   2 slots x B x kp_stride x (28 + 32) B  keypoints + descriptors
// The two result slots ping-pong so a mono step can match the previous frame
// of every stream against the current one without a copy.
#include <hip/hip_runtime.h>

#include <chrono>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <atomic>
#include <cstring>
#include <mutex>
#include <new>
#include <vector>

#include "orbx_device.h"
#include "orbx_ws.h"

using namespace orbx;

namespace {

template <typename T>
hipError_t dalloc(T **p, size_t count) {
    *p = nullptr;
    if (count == 0) return hipSuccess;
    return hipMalloc(reinterpret_cast<void **>(p), sizeof(T) * count);
}

template <typename T>
void dfree(T *&p) {
    if (p) (void)hipFree(p);
    p = nullptr;
}

int popcount32(uint32_t v) {
    v = v - ((v >> 1) & 0x55555555u);
    v = (v & 0x33333333u) + ((v >> 2) & 0x33333333u);
    return (int)((((v + (v >> 4)) & 0xF0F0F0Fu) * 0x1010101u) >> 24);
}

}  // namespace

struct orbx_extractor {
    int device = 0;
    int nfeatures = 0, nlevels = 0, ini_th = 0, min_th = 0;
    float scale_factor = 1.2f;
    Plan plan;
    bool planned = false;
    int max_batch = 0;

    DevPlan dp{};
    uint8_t *d_tables = nullptr;

    uint8_t *d_pyr = nullptr, *d_blur = nullptr;
    uint32_t *d_cand = nullptr, *d_cand2 = nullptr, *d_keys = nullptr, *d_sel = nullptr;
    int32_t *d_cell_count = nullptr, *d_level_count = nullptr;
    uint16_t *d_key_node = nullptr;
    uint8_t *d_key_q = nullptr;

    struct Slot {
        orbx_keypoint *kps = nullptr;
        uint8_t *desc = nullptr;
        int32_t *nkps = nullptr;
        int batch = 0;
        const uint8_t *img0 = nullptr;
        int64_t img0_stride = 0;
        int img0_pitch = 0;
    } slot[2];
    int cur = 0;
    int steps = 0;

    // matcher state (results of the last mono step)
    float *d_prev = nullptr;
    int32_t *d_m12 = nullptr, *d_nmatch = nullptr;
    int match_batch = 0;
    int l0cap = 0;

    // depth results of the last stereo / RGB-D step (per pair or per frame)
    float *d_ur = nullptr, *d_depth = nullptr;
    int32_t *d_sad = nullptr, *d_nkept = nullptr;
    uint8_t *d_bands = nullptr;   // per stereo pair: the right image's sorted bands (StereoBufs::bands)
    int32_t *d_pair_done = nullptr;   // per stereo pair: workgroup counter of the fused median cut
    int depth_mode = 0;         // 0 none, 1 stereo (index = pair), 2 RGB-D (index = frame)
    int depth_count = 0;

    uint8_t *d_img = nullptr;   // staging for the host API
    size_t d_img_bytes = 0;

    // Host-API fast path (orbx_extract, one frame per call as Frame::ExtractORB
    // makes it): the upload, the extraction and the result downloads captured
    // once per plan as a hipGraph on `stream`, replayed per call from pinned
    // staging buffers -- one launch and one synchronisation instead of ~15
    // launches and four blocking copies.  ORBX_HOST_GRAPH=0 turns it off.
    hipGraphExec_t host_graph = nullptr;
    int graph_w = 0, graph_h = 0;
    uint8_t *h_img = nullptr, *h_out = nullptr;   // pinned
    size_t h_img_bytes = 0, h_out_bytes = 0;
    bool host_result_valid = false;   // slot 0 still holds what h_out holds (no extraction since)

    // orbx_compute_stereo_matches workspace (this extractor as the left one),
    // kept across calls: uploads of host keypoints that are not the right /
    // left extractor's own last results, the outputs, a pinned readback.
    struct StereoWs {
        orbx_keypoint *kl = nullptr, *kr = nullptr;
        uint8_t *dl = nullptr, *dr = nullptr;
        int32_t *n = nullptr, *sad = nullptr, *nk = nullptr;
        float *ur = nullptr, *depth = nullptr;
        int cap_l = 0, cap_r = 0;
        uint8_t *h_res = nullptr;   // pinned: ur[cap_l], depth[cap_l], nkept
        size_t h_bytes = 0;
        void free_dev() {
            dfree(kl); dfree(kr); dfree(dl); dfree(dr); dfree(n); dfree(sad); dfree(nk); dfree(ur); dfree(depth);
            cap_l = cap_r = 0;
        }
    } sws;

    hipStream_t stream = nullptr;
    // The current results' completion: recorded on the launch stream at the end
    // of every device step (the caller's stream, or `stream`), so the download
    // calls wait for exactly that work -- no device-wide synchronisation, which
    // would also wait for (and serialise with) other extractors' streams, e.g.
    // the two extraction threads of Frame's stereo constructor.
    hipEvent_t res_ev = nullptr;
    bool res_pending = false;
    // pinned staging of the host pyramid copy (orbx_extractor_pyramid_host)
    uint8_t *h_pyr = nullptr;
    size_t h_pyr_bytes = 0;

    // Batch split: a large batch runs as `split` interleaved sub-batches on
    // their own streams (forked from / joined to the launch stream), so the
    // latency-bound kernels of one half overlap the other half's work.
    static constexpr int kMaxParts = 2;

    // Level pipeline (orbx_extractor_pipeline, default off): level 0's FAST,
    // quadtree and describe run on a second stream beside the resize chain and
    // levels 1.. (run_extract_pipe).  Per part of a split.  Measured on MI355X:
    // VGA x512 +2.5 %, EuRoC x256 +-0, KITTI x192 -25 %.
    int pipeline = 0;
    struct PipeSet {
        hipStream_t s[2] = {};
        hipEvent_t fork = nullptr, level0 = nullptr, done[2] = {};
        hipEvent_t resized = nullptr, early = nullptr;   // (pipeline 2: levels 1..E resized / their quadtree done)
    } pipe[kMaxParts];
    // pipeline 2: the levels FAST / quadtree take on the side stream once the
    // resize chain has produced them (ORBX_PIPE_EARLY, 1..nlevels - 2), and
    // whether their describe runs there too (ORBX_PIPE_DESC=1) rather than
    // with the other levels' at the end of the main stream
    // (E = 2 with their describe there: VGA 467.9 k -> 484.5 k, FHD stereo 47.66 k -> 49.80 k on one box;
    // E = 1 / 3 and the describe at the end measured lower, profiles/r06_ab_deep_pipeline.txt)
    int pipe_early = 2;
    int pipe_desc = 1;
    bool pipe_ready = false;
    int split = 1;   // orbx_extractor_split / ORBX_SPLIT=2 turn it on
    hipStream_t part_stream[kMaxParts] = {};
    hipEvent_t fork_ev = nullptr, done_ev[kMaxParts] = {};
    // Stagger (ORBX_STAGGER=s, s in 1..3): part 1 starts after part 0's first
    // s stages (resize, FAST, quadtree), so the parts' latency-bound kernels
    // meet the other part's VALU-bound ones instead of each other.
    int stagger = 0;
    hipEvent_t stag_ev = nullptr;
    // Serial chunks (ORBX_CHUNKS=c, diagnostic): an unsplit batch runs as c
    // chunks one after another on the launch stream, each chunk's resize,
    // FAST, quadtree and describe back to back, so a chunk's pyramid is still
    // in the 256 MB MALL when its describe re-reads it.
    int chunks = 1;

    // Matcher overlap (orbx_extractor_overlap_match, default off): a mono
    // step's SearchForInitialization runs on match_stream, which the launch
    // stream does not wait for, so it overlaps the next step's resize / FAST /
    // quadtree.  The next extraction's k_describe launches (the only writers of
    // a result slot, which the matcher reads) wait for match_ev (match_gate);
    // res_ev is recorded after the matcher, so downloads wait for it.
    int overlap_match = 0;
    hipStream_t match_stream = nullptr;
    hipEvent_t ext_ev = nullptr, match_ev = nullptr;
    bool match_gate = false;

    // Stage profiling: a ring of event sets, one set per step, folded into
    // per-stage sums lazily so the timed loop never waits on the host.
    static constexpr int kRing = 64;
    bool profiling = false;
    hipEvent_t ev[kRing][kNumStages + 1] = {};
    bool pending[kRing] = {false};
    bool valid[kRing][kNumStages] = {};
    int ring_pos = 0;
    double stage_sum[kNumStages] = {0};
    long stage_cnt[kNumStages] = {0};
    hipEvent_t *cur_ev = nullptr;
    bool *cur_valid = nullptr;

    ~orbx_extractor() {
        release();
        if (h_img) (void)hipHostFree(h_img);
        if (h_out) (void)hipHostFree(h_out);
        if (h_pyr) (void)hipHostFree(h_pyr);
        if (res_ev) (void)hipEventDestroy(res_ev);
        sws.free_dev();
        if (sws.h_res) (void)hipHostFree(sws.h_res);
        if (stream) (void)hipStreamDestroy(stream);
        for (auto &ps : part_stream)
            if (ps) (void)hipStreamDestroy(ps);
        if (fork_ev) (void)hipEventDestroy(fork_ev);
        if (stag_ev) (void)hipEventDestroy(stag_ev);
        if (match_stream) (void)hipStreamDestroy(match_stream);
        if (ext_ev) (void)hipEventDestroy(ext_ev);
        if (match_ev) (void)hipEventDestroy(match_ev);
        for (auto &e : done_ev)
            if (e) (void)hipEventDestroy(e);
        for (auto &set : ev)
            for (auto &e : set)
                if (e) (void)hipEventDestroy(e);
        for (auto &ps : pipe) {
            for (auto &x : ps.s)
                if (x) (void)hipStreamDestroy(x);
            for (hipEvent_t e : {ps.fork, ps.level0, ps.done[0], ps.done[1], ps.resized, ps.early})
                if (e) (void)hipEventDestroy(e);
        }
    }

    void release() {
        if (match_gate && match_ev) (void)hipEventSynchronize(match_ev);   // (the matcher reads the slots freed below)
        match_gate = false;
        if (host_graph) (void)hipGraphExecDestroy(host_graph);
        host_graph = nullptr;
        host_result_valid = false;   // the result slots are freed: h_out no longer mirrors slot 0
        res_pending = false;
        graph_w = graph_h = 0;
        dfree(d_tables); dfree(d_pyr); dfree(d_blur); dfree(d_cand); dfree(d_cand2); dfree(d_keys); dfree(d_sel);
        dfree(d_cell_count); dfree(d_level_count); dfree(d_key_node); dfree(d_key_q);
        for (auto &s : slot) { dfree(s.kps); dfree(s.desc); dfree(s.nkps); s.batch = 0; }
        dfree(d_prev); dfree(d_m12); dfree(d_nmatch); dfree(d_img);
        dfree(d_ur); dfree(d_depth); dfree(d_sad); dfree(d_nkept); dfree(d_bands); dfree(d_pair_done);
        depth_mode = 0;
        depth_count = 0;
        d_img_bytes = 0;
        planned = false;
        max_batch = 0;
        match_batch = 0;
    }
};

namespace {

int check(hipError_t e) { return e == hipSuccess ? ORBX_OK : ORBX_EIO; }

hipStream_t stream_of(orbx_extractor *ex, void *s) {
    return s ? reinterpret_cast<hipStream_t>(s) : ex->stream;
}

// End of a device step on st: its results are complete when res_ev is.
void note_results(orbx_extractor *ex, hipStream_t st) {
    if (!ex->res_ev && hipEventCreateWithFlags(&ex->res_ev, hipEventDisableTiming) != hipSuccess) {
        ex->res_ev = nullptr;
        (void)hipStreamSynchronize(st);   // (no event: wait here instead)
        ex->res_pending = false;
        return;
    }
    ex->res_pending = hipEventRecord(ex->res_ev, st) == hipSuccess;
    if (!ex->res_pending) (void)hipStreamSynchronize(st);
}

// Waits for the current results; the copies that follow go on ex->stream.
int sync_results(orbx_extractor *ex) {
    if (ex->res_pending) {
        if (hipEventSynchronize(ex->res_ev) != hipSuccess) return ORBX_EIO;
        ex->res_pending = false;
    }
    return ORBX_OK;
}

// Device -> host copies on the extractor's stream, then one wait for them.
struct D2H {
    orbx_extractor *ex;
    bool ok = true;
    void operator()(void *dst, const void *src, size_t n) {
        if (ok && n) ok = hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, ex->stream) == hipSuccess;
    }
    bool wait() { return ok && hipStreamSynchronize(ex->stream) == hipSuccess; }
};

int upload_plan(orbx_extractor *ex) {
    Plan &p = ex->plan;
    // blur tile table
    std::vector<int4> tiles;
    for (int l = 0; l < p.nlevels; ++l)
        for (int y = 0; y < p.lv[l].h; y += 16)
            for (int x = 0; x < p.lv[l].w; x += 64) tiles.push_back(make_int4(l, x, y, 0));
    const size_t b_lv = sizeof(LevelGeom) * p.lv.size();
    const size_t b_cells = sizeof(Cell) * p.cells.size();
    const size_t b_xt = sizeof(ResizeTap) * p.xtaps.size();
    const size_t b_yt = sizeof(ResizeTap) * p.ytaps.size();
    const size_t b_rc = sizeof(ResizeCol) * p.rcols.size();
    const size_t b_rr = sizeof(ResizeRow) * p.rrows.size();
    const size_t b_tiles = sizeof(int4) * tiles.size();
    // level of every output slot (the last level whose range starts at or before it)
    std::vector<uint32_t> slot_level((size_t)std::max(p.out_cap, 0) + 4, 0);
    for (int s = 0; s < p.out_cap; ++s) {
        int l = 0;
        for (int q = 1; q < p.nlevels; ++q)
            if (s >= p.lv[q].out_off) l = q;
        slot_level[s] = (uint32_t)l;
    }
    const size_t b_sl = sizeof(uint32_t) * slot_level.size();
    const size_t b_rgn = sizeof(RgnRect) * p.rgn.size();
    auto al = [](size_t v) { return (v + 255) & ~size_t(255); };
    const size_t total = al(b_lv) + al(b_cells) + al(b_xt) + al(b_yt) + al(b_rc) + al(b_rr) + al(b_tiles) + al(b_sl) + al(b_rgn) + 256;
    std::vector<uint8_t> host(total, 0);
    size_t o = 0;
    const size_t o_lv = o; std::memcpy(&host[o], p.lv.data(), b_lv); o += al(b_lv);
    const size_t o_cells = o; if (b_cells) std::memcpy(&host[o], p.cells.data(), b_cells); o += al(b_cells);
    const size_t o_xt = o; if (b_xt) std::memcpy(&host[o], p.xtaps.data(), b_xt); o += al(b_xt);
    const size_t o_yt = o; if (b_yt) std::memcpy(&host[o], p.ytaps.data(), b_yt); o += al(b_yt);
    const size_t o_rc = o; if (b_rc) std::memcpy(&host[o], p.rcols.data(), b_rc); o += al(b_rc);
    const size_t o_rr = o; if (b_rr) std::memcpy(&host[o], p.rrows.data(), b_rr); o += al(b_rr);
    const size_t o_tiles = o; if (b_tiles) std::memcpy(&host[o], tiles.data(), b_tiles); o += al(b_tiles);
    const size_t o_sl = o; std::memcpy(&host[o], slot_level.data(), b_sl); o += al(b_sl);
    const size_t o_rgn = o; if (b_rgn) std::memcpy(&host[o], p.rgn.data(), b_rgn); o += al(b_rgn);
    if (dalloc(&ex->d_tables, total) != hipSuccess) return ORBX_ENOMEM;
    if (hipMemcpy(ex->d_tables, host.data(), total, hipMemcpyHostToDevice) != hipSuccess) return ORBX_EIO;
    DevPlan &d = ex->dp;
    d.lv = reinterpret_cast<const LevelGeom *>(ex->d_tables + o_lv);
    d.cells = reinterpret_cast<const Cell *>(ex->d_tables + o_cells);
    d.xtaps = reinterpret_cast<const ResizeTap *>(ex->d_tables + o_xt);
    d.ytaps = reinterpret_cast<const ResizeTap *>(ex->d_tables + o_yt);
    d.rcols = reinterpret_cast<const ResizeCol *>(ex->d_tables + o_rc);
    d.rrows = reinterpret_cast<const ResizeRow *>(ex->d_tables + o_rr);
    d.blur_tiles = reinterpret_cast<const int4 *>(ex->d_tables + o_tiles);
    d.slot_level = reinterpret_cast<const uint32_t *>(ex->d_tables + o_sl);
    d.pyr_rgn = reinterpret_cast<const int4 *>(ex->d_tables + o_rgn);
    d.pyr_rgn_half = p.rgn_half;
    d.nlevels = p.nlevels;
    for (int l = 0; l < kMaxLevels; ++l) {
        LevelArgs &a = d.la[l];
        a = LevelArgs{};
        if (l >= p.nlevels) continue;
        const LevelGeom &g = p.lv[l];
        a.w = g.w; a.h = g.h; a.pitch = g.pitch; a.out_off = g.out_off;
        a.pyr_off = g.pyr_off; a.scale = g.scale; a.patch_size = g.patch_size;
    }
    d.ncells = (int)p.cells.size();
    d.nblur_tiles = (int)tiles.size();
    for (int i = 0; i < 7; ++i) {
        d.gauss[i] = p.gauss[i];
        if (p.gauss[i] != kGaussTaps[i]) return ORBX_EINVAL;   // kernels use the constant taps
    }
    for (int i = 0; i < 16; ++i) d.umax[i] = p.umax[i];
    for (int i = 0; i < 16; ++i)
        if (p.umax[i] != kUmax[i]) return ORBX_EINVAL;   // k_describe's disc masks are built from kUmax
    d.ini_th = std::min(std::max(p.ini_th, 0), 255);
    d.min_th = std::min(std::max(p.min_th, 0), 255);
    d.pyr_bytes = p.pyr_bytes;
    d.blur_bytes = p.blur_bytes;
    d.cand_cap = p.cand_cap;
    d.out_cap = p.out_cap;
    d.max_kps = p.max_kps;
    int node_cap = 8;
    for (const LevelGeom &g : p.lv) node_cap = std::max(node_cap, std::max(g.quota, 4 * g.nini) + 4);
    d.node_cap = node_cap;
    int mw = 1, mh = 1;
    for (const Cell &c : p.cells) { mw = std::max(mw, c.x1 - c.x0); mh = std::max(mh, c.y1 - c.y0); }
    if (mw > 255 || mh > 255) return ORBX_EINVAL;   // survivor list packs (y << 8 | x)
    if (4 * fast_lds(mw, mh).per_wave > 64 * 1024) return ORBX_EINVAL;   // k_fast's LDS for the largest cell
    d.node_lds_bytes = quadtree_lds_bytes(node_cap);
    // phase 1 of k_quadtree keeps two ints per cell of a level and a u32 key
    // source per register-held key (kQuadRegKeys in all) in the same LDS
    d.node_lds_bytes_w = d.node_lds_bytes;   // (the 1024-thread form's map holds kQuadRegKeysW sources)
    for (const LevelGeom &g : p.lv) {
        d.node_lds_bytes = std::max(d.node_lds_bytes, (int)(8 * (g.cell_end - g.cell_begin) + 16 + 4 * kQuadRegKeys));
        d.node_lds_bytes_w = std::max(d.node_lds_bytes_w, (int)(8 * (g.cell_end - g.cell_begin) + 16 + 4 * kQuadRegKeysW));
    }
    d.dbg_stop = std::getenv("ORBX_DBG_STOP") ? std::atoi(std::getenv("ORBX_DBG_STOP")) : 0;
    if (d.node_lds_bytes > 160 * 1024) return ORBX_EINVAL;
    return ORBX_OK;
}

int reserve(orbx_extractor *ex, int w, int h, int max_batch) {
    if (w < 8 || h < 8 || w > 4095 || h > 4095 || max_batch <= 0) return ORBX_EINVAL;
    if (ex->planned && ex->plan.width == w && ex->plan.height == h && ex->max_batch >= max_batch) return ORBX_OK;
    if (hipSetDevice(ex->device) != hipSuccess) return ORBX_ENODEV;
    (void)hipStreamSynchronize(ex->stream);
    ex->release();
    ex->plan = make_plan(w, h, ex->nfeatures, ex->scale_factor, ex->nlevels, ex->ini_th, ex->min_th);
    // Levels too small for a FAST cell grid yield no keypoints, as in the reference
    // (nCols or nRows == 0 skips its cell loop).  Rejected: levels under 4 px (the
    // blur's reflect-101 halo needs them) and a quadtree with cells but nIni == 0
    // (w/h < 0.5: the reference divides by zero at ORBextractor.cc:568).
    for (const LevelGeom &g : ex->plan.lv) {
        if (g.w < 4 || g.h < 4 || g.wcell >= 60 || g.hcell >= 60) return ORBX_EINVAL;
        if (g.ncols > 0 && g.nrows > 0 && g.nini <= 0) return ORBX_EINVAL;
    }
    if (!resize_window_fits(ex->plan)) return ORBX_EINVAL;
    if (!plan_resize_waves(ex->plan) || std::getenv("ORBX_RESIZE_BLOCKS")) ex->plan.rw.clear();
    const char *rg = std::getenv("ORBX_PYR_RGN");   // =0: the per-level resize kernels at every batch
    if (!(rg && rg[0] == '0')) (void)plan_pyr_regions(ex->plan);
    int rc = upload_plan(ex);
    if (rc) return rc;
    const Plan &p = ex->plan;
    const size_t B = (size_t)max_batch;
    if (B * (size_t)std::max(p.out_cap, 1) >= (size_t(1) << 31)) return ORBX_EINVAL;   // (k_describe's 32-bit slot index)
    bool ok = true;
    ok &= dalloc(&ex->d_pyr, B * p.pyr_bytes) == hipSuccess;
    ok &= dalloc(&ex->d_blur, B * p.blur_bytes) == hipSuccess;
    ok &= dalloc(&ex->d_cand, B * p.cand_cap) == hipSuccess;
    ok &= dalloc(&ex->d_cand2, B * p.cand_cap) == hipSuccess;
    ok &= dalloc(&ex->d_keys, B * p.cand_cap) == hipSuccess;
    ok &= dalloc(&ex->d_key_node, B * p.cand_cap) == hipSuccess;
    ok &= dalloc(&ex->d_key_q, B * p.cand_cap) == hipSuccess;
    ok &= dalloc(&ex->d_cell_count, B * p.cells.size()) == hipSuccess;
    ok &= dalloc(&ex->d_sel, B * p.out_cap) == hipSuccess;
    ok &= dalloc(&ex->d_level_count, B * kMaxLevels) == hipSuccess;
    for (auto &s : ex->slot) {
        ok &= dalloc(&s.kps, B * p.max_kps) == hipSuccess;
        ok &= dalloc(&s.desc, B * p.max_kps * 32) == hipSuccess;
        ok &= dalloc(&s.nkps, B) == hipSuccess;
        s.batch = 0;
    }
    ex->l0cap = p.lv[0].out_cap;
    ok &= dalloc(&ex->d_prev, B * p.max_kps * 2) == hipSuccess;
    ok &= dalloc(&ex->d_m12, B * p.max_kps) == hipSuccess;
    ok &= dalloc(&ex->d_nmatch, B) == hipSuccess;
    ok &= dalloc(&ex->d_ur, B * p.max_kps) == hipSuccess;
    ok &= dalloc(&ex->d_depth, B * p.max_kps) == hipSuccess;
    ok &= dalloc(&ex->d_sad, B * p.max_kps) == hipSuccess;
    ok &= dalloc(&ex->d_nkept, B) == hipSuccess;
    const char *so = std::getenv("ORBX_STEREO_SORT_ONCE");   // (k_band_sort + k_stereo_band_gs, orbx_stereo.hip)
    if (so && so[0] == '1' && B >= 4 && p.max_kps <= 65535)
        ok &= dalloc(&ex->d_bands, (size_t)(B / 2) * stereo_band_stride(p.height, p.max_kps)) == hipSuccess;
    if (B >= 2) {   // (zero; the fused cut's last workgroup resets its pair's counter)
        ok &= dalloc(&ex->d_pair_done, B / 2) == hipSuccess;   // (zeroed before each fused launch)
    }
    if (!ok) { ex->release(); return ORBX_ENOMEM; }
    ex->planned = true;
    ex->max_batch = max_batch;
    ex->cur = 0;
    return ORBX_OK;
}

FrameBufs frame_bufs(orbx_extractor *ex, int slot) {
    FrameBufs fb;
    const auto &s = ex->slot[slot];
    fb.img0 = s.img0;
    fb.img0_stride = s.img0_stride;
    fb.img0_pitch = s.img0_pitch;
    fb.pyr = ex->d_pyr;
    fb.blur = ex->d_blur;
    fb.cand = ex->d_cand;
    fb.cand2 = ex->d_cand2;
    fb.cell_count = ex->d_cell_count;
    fb.keys = ex->d_keys;
    fb.key_node = ex->d_key_node;
    fb.key_q = ex->d_key_q;
    fb.sel = ex->d_sel;
    fb.level_count = ex->d_level_count;
    fb.kps = s.kps;
    fb.desc = s.desc;
    fb.nkps = s.nkps;
    return fb;
}

PyrView pyr_view(const orbx_extractor *ex, int slot) {
    const auto &s = ex->slot[slot];
    return PyrView{s.img0, s.img0_stride, s.img0_pitch, ex->d_pyr, ex->plan.pyr_bytes};
}

bool same_geometry(const Plan &a, const Plan &b) {
    if (a.width != b.width || a.height != b.height || a.nlevels != b.nlevels) return false;
    for (int l = 0; l < a.nlevels; ++l)
        if (a.lv[l].w != b.lv[l].w || a.lv[l].h != b.lv[l].h || a.lv[l].scale != b.lv[l].scale ||
            a.lv[l].inv_scale != b.lv[l].inv_scale)
            return false;
    return true;
}

// The same buffers seen from frame b0 on.
FrameBufs offset_frames(const orbx_extractor *ex, FrameBufs fb, int b0) {
    const Plan &p = ex->plan;
    fb.img0 += (int64_t)b0 * fb.img0_stride;
    fb.pyr += (int64_t)b0 * p.pyr_bytes;
    fb.blur += (int64_t)b0 * p.blur_bytes;
    fb.cand += (int64_t)b0 * p.cand_cap;
    fb.cand2 += (int64_t)b0 * p.cand_cap;
    fb.cell_count += (int64_t)b0 * p.cells.size();
    fb.keys += (int64_t)b0 * p.cand_cap;
    fb.key_node += (int64_t)b0 * p.cand_cap;
    fb.key_q += (int64_t)b0 * p.cand_cap;
    fb.sel += (int64_t)b0 * p.out_cap;
    fb.level_count += (int64_t)b0 * kMaxLevels;
    fb.kps += (int64_t)b0 * p.max_kps;
    fb.desc += (int64_t)b0 * p.max_kps * 32;
    fb.nkps += b0;
    return fb;
}

MatchBufs offset_pairs(MatchBufs mb, int b0) {
    mb.k1 += b0 * mb.k1_stride; mb.d1 += b0 * mb.k1_stride * 32; mb.n1 += b0;
    mb.k2 += b0 * mb.k2_stride; mb.d2 += b0 * mb.k2_stride * 32; mb.n2 += b0;
    mb.prev_xy += b0 * mb.k1_stride * 2;
    mb.matches12 += b0 * mb.k1_stride;
    mb.nmatches += b0;
    return mb;
}

struct Parts {
    int n = 1;
    int b0[orbx_extractor::kMaxParts] = {0, 0};
    int nb[orbx_extractor::kMaxParts] = {0, 0};
    hipStream_t s[orbx_extractor::kMaxParts] = {};
};

// A stream for the extractor's own forks (batch parts, level pipeline).
// ORBX_QUEUES=dedicated: one made by hipExtStreamCreateWithCUMask (every CU),
// which the runtime gives a hardware queue of its own, so two forks never
// share one of the process's pooled queues (GPU_MAX_HW_QUEUES) and serialise.
hipError_t fork_stream(hipStream_t *s) {
    static const bool dedicated = [] {
        const char *q = std::getenv("ORBX_QUEUES");
        return q && std::strcmp(q, "dedicated") == 0;
    }();
    if (!dedicated) return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
    int dev = 0, ncu = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
        return hipErrorInvalidValue;
    std::vector<uint32_t> mask((ncu + 31) / 32, 0xFFFFFFFFu);
    return hipExtStreamCreateWithCUMask(s, (uint32_t)mask.size(), mask.data());
}

// Splits `batch` into sub-batches on the part streams (forked from st), or a
// single part on st itself.
Parts fork_parts(orbx_extractor *ex, hipStream_t st, int batch) {
    Parts P;
    P.nb[0] = batch;
    P.s[0] = st;
    constexpr int kMinPart = 32;   // orbx.h: batches under 64 frames are never split
    if (ex->split < 2 || batch < 2 * kMinPart) return P;
    if (!ex->fork_ev) {
        bool ok = hipEventCreateWithFlags(&ex->fork_ev, hipEventDisableTiming) == hipSuccess;
        for (int k = 0; k < orbx_extractor::kMaxParts && ok; ++k)
            ok = fork_stream(&ex->part_stream[k]) == hipSuccess &&
                 hipEventCreateWithFlags(&ex->done_ev[k], hipEventDisableTiming) == hipSuccess;
        if (!ok) { ex->split = 1; return P; }
    }
    if (hipEventRecord(ex->fork_ev, st) != hipSuccess) return P;
    P.n = orbx_extractor::kMaxParts;
    for (int k = 0; k < P.n; ++k) {
        P.b0[k] = batch * k / P.n;
        P.nb[k] = batch * (k + 1) / P.n - P.b0[k];
        P.s[k] = ex->part_stream[k];
        (void)hipStreamWaitEvent(P.s[k], ex->fork_ev, 0);
    }
    return P;
}

int join_parts(orbx_extractor *ex, hipStream_t st, const Parts &P) {
    if (P.n < 2) return ORBX_OK;
    for (int k = 0; k < P.n; ++k)
        if (hipEventRecord(ex->done_ev[k], P.s[k]) != hipSuccess || hipStreamWaitEvent(st, ex->done_ev[k], 0) != hipSuccess)
            return ORBX_EIO;
    return ORBX_OK;
}

// Before a k_describe launch on `st` (it writes the result slot): wait for a
// matcher still reading that slot on match_stream (orbx_extractor_overlap_match).
bool gate_describe(orbx_extractor *ex, hipStream_t st) {
    return !ex->match_gate || hipStreamWaitEvent(st, ex->match_ev, 0) == hipSuccess;
}

void fold(orbx_extractor *ex, int set) {
    if (!ex->pending[set]) return;
    (void)hipEventSynchronize(ex->ev[set][kNumStages]);
    for (int i = 0; i < kNumStages; ++i) {
        if (!ex->valid[set][i]) continue;
        float t = 0.f;
        if (hipEventElapsedTime(&t, ex->ev[set][i], ex->ev[set][i + 1]) == hipSuccess) {
            ex->stage_sum[i] += t;
            ex->stage_cnt[i] += 1;
        } else {
            (void)hipGetLastError();   // (not the next launch's error)
        }
    }
    ex->pending[set] = false;
}

// Starts a profiled step: picks the next event set (folding it first if it
// still holds an unread step).
void prof_begin(orbx_extractor *ex) {
    ex->cur_ev = nullptr;
    ex->cur_valid = nullptr;
    if (!ex->profiling) return;
    const int set = ex->ring_pos;
    ex->ring_pos = (ex->ring_pos + 1) % orbx_extractor::kRing;
    fold(ex, set);
    for (auto &e : ex->ev[set])
        if (!e && hipEventCreate(&e) != hipSuccess) return;
    for (int i = 0; i < kNumStages; ++i) ex->valid[set][i] = false;
    ex->cur_ev = ex->ev[set];
    ex->cur_valid = ex->valid[set];
    ex->pending[set] = true;
}

void mark(orbx_extractor *ex, int i, hipStream_t st) {
    if (ex->cur_ev) (void)hipEventRecord(ex->cur_ev[i], st);
}

void mark_valid(orbx_extractor *ex, int stage) {
    if (ex->cur_valid) ex->cur_valid[stage] = true;
}

bool make_pipe(orbx_extractor *ex) {
    if (ex->pipe_ready) return true;
    const unsigned f = hipEventDisableTiming;
    bool ok = true;
    for (auto &ps : ex->pipe) {
        for (auto &x : ps.s) ok = ok && fork_stream(&x) == hipSuccess;
        ok = ok && hipEventCreateWithFlags(&ps.fork, f) == hipSuccess && hipEventCreateWithFlags(&ps.level0, f) == hipSuccess;
        ok = ok && hipEventCreateWithFlags(&ps.resized, f) == hipSuccess && hipEventCreateWithFlags(&ps.early, f) == hipSuccess;
        for (auto &e : ps.done) ok = ok && hipEventCreateWithFlags(&e, f) == hipSuccess;
    }
    ex->pipe_ready = ok;
    return ok;
}

// One part's extraction in two level groups, forked from / joined to `st`:
//   stream 1: FAST + quadtree of level 0 (event level0), describe of level 0
//   stream 0: the resize chain, FAST + quadtree of levels 1.., then (after
//             level0: the output offsets need level 0's count) their describe
// so level 0's work overlaps the latency-bound resize chain.
int run_extract_pipe(orbx_extractor *ex, const FrameBufs &fb, int nb, hipStream_t st, orbx_extractor::PipeSet &ps) {
    const Plan &hp = ex->plan;
    const DevPlan &dp = ex->dp;
    const int n = hp.nlevels;
    if (hipEventRecord(ps.fork, st) != hipSuccess) return ORBX_EIO;
    for (auto &x : ps.s)
        if (hipStreamWaitEvent(x, ps.fork, 0) != hipSuccess) return ORBX_EIO;
    if (launch_fast_level(dp, hp, fb, nb, ps.s[1], 0, 1) != hipSuccess ||
        launch_quadtree_level(dp, fb, nb, ps.s[1], 0, 1) != hipSuccess)
        return ORBX_EIO;
    if (hipEventRecord(ps.level0, ps.s[1]) != hipSuccess) return ORBX_EIO;
    if (!gate_describe(ex, ps.s[1]) || launch_describe_level(dp, hp, fb, nb, ps.s[1], 0, 1) != hipSuccess) return ORBX_EIO;
    if (n > 1) {
        if (launch_resize(dp, hp, fb, nb, ps.s[0]) != hipSuccess ||
            launch_fast_level(dp, hp, fb, nb, ps.s[0], 1, n) != hipSuccess ||
            launch_quadtree_level(dp, fb, nb, ps.s[0], 1, n) != hipSuccess)
            return ORBX_EIO;
        if (hipStreamWaitEvent(ps.s[0], ps.level0, 0) != hipSuccess) return ORBX_EIO;
        if (!gate_describe(ex, ps.s[0]) || launch_describe_level(dp, hp, fb, nb, ps.s[0], 1, n) != hipSuccess) return ORBX_EIO;
    }
    for (int i = 0; i < 2; ++i)
        if (hipEventRecord(ps.done[i], ps.s[i]) != hipSuccess || hipStreamWaitEvent(st, ps.done[i], 0) != hipSuccess)
            return ORBX_EIO;
    return ORBX_OK;
}

// The deep level pipeline (pipeline 2): the side stream also takes levels
// 1..E once the resize chain has produced them, so the rest of the chain
// (latency- and memory-bound) runs beside their FAST (VALU-bound):
//   stream 1: FAST + quadtree of level 0, describe of level 0, then (after
//             `resized`) FAST + quadtree of levels 1..E (event `early`), and
//             with ORBX_PIPE_DESC=1 their describe
//   stream 0: resize of levels 1..E (event `resized`), resize of E+1..,
//             FAST + quadtree of levels E+1.., then (after `early`: every
//             count below a level is final) describe of levels 1.. (E+1..)
// Each describe launch needs the counts of the levels below it (its output
// offsets), which `early` covers.  Same kernels, same outputs.
int run_extract_pipe2(orbx_extractor *ex, const FrameBufs &fb, int nb, hipStream_t st, orbx_extractor::PipeSet &ps) {
    const Plan &hp = ex->plan;
    const DevPlan &dp = ex->dp;
    const int n = hp.nlevels, E = std::max(1, std::min(ex->pipe_early, n - 2));
    if (hipEventRecord(ps.fork, st) != hipSuccess) return ORBX_EIO;
    for (auto &x : ps.s)
        if (hipStreamWaitEvent(x, ps.fork, 0) != hipSuccess) return ORBX_EIO;
    if (launch_fast_level(dp, hp, fb, nb, ps.s[1], 0, 1) != hipSuccess ||
        launch_quadtree_level(dp, fb, nb, ps.s[1], 0, 1) != hipSuccess)
        return ORBX_EIO;
    if (!gate_describe(ex, ps.s[1]) || launch_describe_level(dp, hp, fb, nb, ps.s[1], 0, 1) != hipSuccess) return ORBX_EIO;
    for (int l = 1; l <= E; ++l)
        if (launch_resize_level(dp, hp, fb, nb, ps.s[0], l) != hipSuccess) return ORBX_EIO;
    if (hipEventRecord(ps.resized, ps.s[0]) != hipSuccess || hipStreamWaitEvent(ps.s[1], ps.resized, 0) != hipSuccess)
        return ORBX_EIO;
    if (launch_fast_level(dp, hp, fb, nb, ps.s[1], 1, E + 1) != hipSuccess ||
        launch_quadtree_level(dp, fb, nb, ps.s[1], 1, E + 1) != hipSuccess)
        return ORBX_EIO;
    if (hipEventRecord(ps.early, ps.s[1]) != hipSuccess) return ORBX_EIO;
    const int d0 = ex->pipe_desc ? E + 1 : 1;   // the main stream's describe levels [d0, n)
    if (ex->pipe_desc &&
        (!gate_describe(ex, ps.s[1]) || launch_describe_level(dp, hp, fb, nb, ps.s[1], 1, E + 1) != hipSuccess))
        return ORBX_EIO;
    for (int l = E + 1; l < n; ++l)
        if (launch_resize_level(dp, hp, fb, nb, ps.s[0], l) != hipSuccess) return ORBX_EIO;
    if (launch_fast_level(dp, hp, fb, nb, ps.s[0], E + 1, n) != hipSuccess ||
        launch_quadtree_level(dp, fb, nb, ps.s[0], E + 1, n) != hipSuccess)
        return ORBX_EIO;
    if (hipStreamWaitEvent(ps.s[0], ps.early, 0) != hipSuccess) return ORBX_EIO;
    if (!gate_describe(ex, ps.s[0]) || launch_describe_level(dp, hp, fb, nb, ps.s[0], d0, n) != hipSuccess) return ORBX_EIO;
    for (int i = 0; i < 2; ++i)
        if (hipEventRecord(ps.done[i], ps.s[i]) != hipSuccess || hipStreamWaitEvent(st, ps.done[i], 0) != hipSuccess)
            return ORBX_EIO;
    return ORBX_OK;
}

// Runs the five extractor stages for `batch` frames into result slot `si`,
// stage by stage across the parts (profiling marks on part 0's stream), or as
// a level pipeline per part (stage marks then cover only the match).
int run_extract(orbx_extractor *ex, int si, const uint8_t *d_images, int64_t stride, int pitch, int batch,
                const Parts &P) {
    ex->host_result_valid = false;
    auto &s = ex->slot[si];
    s.img0 = d_images;
    s.img0_stride = stride;
    s.img0_pitch = pitch;
    s.batch = batch;
    const FrameBufs fb = frame_bufs(ex, si);
    FrameBufs pf[orbx_extractor::kMaxParts];
    for (int k = 0; k < P.n; ++k) pf[k] = offset_frames(ex, fb, P.b0[k]);
    const hipStream_t m = P.s[0];
    if (ex->chunks > 1 && P.n == 1 && !ex->pipeline) {
        mark(ex, 0, m);   // (one span for the whole extraction, no per-stage times)
        const int nc = std::min(ex->chunks, batch);
        for (int k = 0; k < nc; ++k) {
            const int c0 = batch * k / nc, cn = batch * (k + 1) / nc - c0;
            const FrameBufs fc = offset_frames(ex, fb, c0);
            if (launch_resize(ex->dp, ex->plan, fc, cn, m) != hipSuccess ||
                launch_fast(ex->dp, ex->plan, fc, cn, m) != hipSuccess ||
                launch_quadtree(ex->dp, fc, cn, m) != hipSuccess || !gate_describe(ex, m) ||
                launch_describe(ex->dp, fc, cn, m) != hipSuccess)
                return ORBX_EIO;
        }
        for (int i = 1; i <= kStageMatch; ++i) mark(ex, i, m);
        return ORBX_OK;   // (no stage marks: stage times come from unchunked runs)
    }
    if (ex->pipeline && make_pipe(ex)) {
        for (int k = 0; k < P.n; ++k) {
            // (the deep form needs the per-level resize kernels: not the
            // small-batch region pyramid, and at least three levels)
            const bool deep = ex->pipeline == 2 && ex->plan.nlevels >= 3 && !use_pyr_regions(ex->plan, P.nb[k]);
            const int rc = deep ? run_extract_pipe2(ex, pf[k], P.nb[k], P.s[k], ex->pipe[k])
                                : run_extract_pipe(ex, pf[k], P.nb[k], P.s[k], ex->pipe[k]);
            if (rc) return rc;
        }
        return ORBX_OK;
    }
    auto stage = [&](int k, int st) -> bool {
        switch (st) {
            case 0: return launch_resize(ex->dp, ex->plan, pf[k], P.nb[k], P.s[k]) == hipSuccess;
            case 1: return launch_fast(ex->dp, ex->plan, pf[k], P.nb[k], P.s[k]) == hipSuccess;
            case 2: return launch_quadtree(ex->dp, pf[k], P.nb[k], P.s[k]) == hipSuccess;
            default: return gate_describe(ex, P.s[k]) && launch_describe(ex->dp, pf[k], P.nb[k], P.s[k]) == hipSuccess;
        }
    };
    if (P.n == 2 && ex->stagger > 0 &&
        (ex->stag_ev || hipEventCreateWithFlags(&ex->stag_ev, hipEventDisableTiming) == hipSuccess)) {
        const int sg = std::min(ex->stagger, 3);
        for (int st = 0; st < 4; ++st) {
            if (!stage(0, st)) return ORBX_EIO;
            if (st == sg - 1 && (hipEventRecord(ex->stag_ev, P.s[0]) != hipSuccess ||
                                 hipStreamWaitEvent(P.s[1], ex->stag_ev, 0) != hipSuccess))
                return ORBX_EIO;
        }
        for (int st = 0; st < 4; ++st)
            if (!stage(1, st)) return ORBX_EIO;
        return ORBX_OK;   // (no stage marks: stage times come from unsplit runs)
    }
    mark(ex, 0, m);
    for (int k = 0; k < P.n; ++k)
        if (launch_resize(ex->dp, ex->plan, pf[k], P.nb[k], P.s[k]) != hipSuccess) return ORBX_EIO;
    mark(ex, 1, m);
    mark(ex, 2, m);   // the blur is fused into k_describe (patch-local); stage 1 stays empty
    for (int k = 0; k < P.n; ++k)
        if (launch_fast(ex->dp, ex->plan, pf[k], P.nb[k], P.s[k]) != hipSuccess) return ORBX_EIO;
    mark(ex, 3, m);
    for (int k = 0; k < P.n; ++k)
        if (launch_quadtree(ex->dp, pf[k], P.nb[k], P.s[k]) != hipSuccess) return ORBX_EIO;
    mark(ex, 4, m);
    for (int k = 0; k < P.n; ++k)
        if (!gate_describe(ex, P.s[k]) || launch_describe(ex->dp, pf[k], P.nb[k], P.s[k]) != hipSuccess) return ORBX_EIO;
    mark(ex, 5, m);
    for (int i = 0; i < kStageMatch; ++i)
        if (i != kStageBlur) mark_valid(ex, i);
    return ORBX_OK;
}

int run_extract(orbx_extractor *ex, int si, const uint8_t *d_images, int64_t stride, int pitch, int batch,
                hipStream_t st) {
    Parts P;
    P.nb[0] = batch;
    P.s[0] = st;
    return run_extract(ex, si, d_images, stride, pitch, batch, P);
}

int validate_batch(orbx_extractor *ex, const uint8_t *d_images, int pitch, int batch) {
    if (!ex || !ex->planned || !d_images || batch <= 0 || batch > ex->max_batch) return ORBX_EINVAL;
    if (pitch < ex->plan.width) return ORBX_EINVAL;
    return ORBX_OK;
}

// The kernels stage level 0 with aligned dword loads: base, pitch and frame
// stride must be multiples of 4.  Other layouts are first copied (on the
// stream) into an aligned staging buffer.
// Level 0 repacked to a 4-aligned pitch, all frames in one launch: a
// workgroup per (row, frame), a thread per destination dword (the source row
// may start at any byte: four byte loads, one dword store).
__global__ __launch_bounds__(256) void k_align_rows(const uint8_t *src, int64_t stride, int pitch, uint8_t *dst,
                                                    int64_t fs, int dp, int w, int h) {
    const int y = blockIdx.x, b = blockIdx.y;
    const uint8_t *s = src + stride * b + (int64_t)pitch * y;
    uint32_t *d = reinterpret_cast<uint32_t *>(dst + fs * b + (int64_t)dp * y);
    for (int q = threadIdx.x; 4 * q < w; q += blockDim.x) {
        const int x = 4 * q;
        uint32_t v = s[x];
        if (x + 1 < w) v |= (uint32_t)s[x + 1] << 8;
        if (x + 2 < w) v |= (uint32_t)s[x + 2] << 16;
        if (x + 3 < w) v |= (uint32_t)s[x + 3] << 24;
        d[q] = v;
    }
}

int align_level0(orbx_extractor *ex, const uint8_t **d_images, int64_t *stride, int *pitch, int batch,
                 hipStream_t st) {
    if ((((uintptr_t)*d_images) | (uintptr_t)*stride | (uintptr_t)*pitch) % 4 == 0) return ORBX_OK;
    const int w = ex->plan.width, h = ex->plan.height;
    const size_t dp = (size_t)pitch_of(w), fs = dp * h, need = fs * batch;
    if (ex->d_img_bytes < need) {
        (void)hipStreamSynchronize(st);
        dfree(ex->d_img);
        if (dalloc(&ex->d_img, need) != hipSuccess) return ORBX_ENOMEM;
        ex->d_img_bytes = need;
    }
    hipLaunchKernelGGL(k_align_rows, dim3(h, batch), dim3(256), 0, st, *d_images, *stride, *pitch, ex->d_img,
                       (int64_t)fs, (int)dp, w, h);
    if (hipGetLastError() != hipSuccess) return ORBX_EIO;
    *d_images = ex->d_img;
    *stride = (int64_t)fs;
    *pitch = (int)dp;
    return ORBX_OK;
}

}  // namespace

// =============================================================================
namespace orbx {

namespace {
bool ws_direct(const CallWs &ws, size_t off, size_t bytes) {
    const size_t n16 = (bytes + 15) / 16;
    return bytes && ws.host_d && ws.flag_d && (off & 15) == 0 && n16 * 16 + off <= ws.cap && bytes <= (256u << 10);
}

int ws_copy_sync(CallWs &ws, size_t off, size_t bytes) {
    if (bytes && hipMemcpyAsync(ws.host + off, ws.dev + off, bytes, hipMemcpyDeviceToHost, ws.st) != hipSuccess)
        return ORBX_EIO;
    return hipStreamSynchronize(ws.st) == hipSuccess ? ORBX_OK : ORBX_EIO;
}

// The same copy, its completion polled (hipStreamQuery) instead of waited for.
int ws_copy_spin(CallWs &ws, size_t off, size_t bytes) {
    if (bytes && hipMemcpyAsync(ws.host + off, ws.dev + off, bytes, hipMemcpyDeviceToHost, ws.st) != hipSuccess)
        return ORBX_EIO;
    hipError_t e;
    while ((e = hipStreamQuery(ws.st)) == hipErrorNotReady) __builtin_ia32_pause();
    return e == hipSuccess ? ORBX_OK : ORBX_EIO;
}

void ws_arm(CallWs &ws) {
    *reinterpret_cast<volatile uint32_t *>(ws.flag) = 0;
    std::atomic_thread_fence(std::memory_order_seq_cst);
}

// Polls the pinned flag; the stream's state ends the wait on an error.
int ws_poll(CallWs &ws) {
    volatile uint32_t *flag = ws.flag;
    for (uint32_t i = 1; !*flag; ++i) {
        if ((i & 255) == 0 && hipStreamQuery(ws.st) != hipErrorNotReady) break;
        __builtin_ia32_pause();
    }
    if (!*flag) {
        if (hipStreamSynchronize(ws.st) != hipSuccess) return ORBX_EIO;
        for (int i = 0; i < (1 << 20) && !*flag; ++i) __builtin_ia32_pause();
        if (!*flag) return ORBX_EIO;
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    return ORBX_OK;
}
}  // namespace

void ws_tail(CallWs &ws, size_t off, size_t bytes, uint32_t *done_d, int blocks, HostTail &t) {
    t = HostTail{};
    if (!ws_direct(ws, off, bytes) || !done_d || blocks <= 0) return;
    ws_arm(ws);
    t.src = reinterpret_cast<const uint4 *>(ws.dev + off);
    t.dst = reinterpret_cast<uint4 *>(ws.host_d + off);
    t.n16 = (int)((bytes + 15) / 16);
    t.flag = ws.flag_d;
    t.done = done_d;
    t.blocks = blocks;
}

int ws_wait(CallWs &ws, const HostTail &t, size_t off, size_t bytes) {
    return t.flag ? ws_poll(ws) : ws_copy_sync(ws, off, bytes);
}

}  // namespace orbx

extern "C" {

const char *orbx_strerror(int code) {
    switch (code) {
        case ORBX_OK: return "ok";
        case ORBX_EIO: return "HIP runtime or kernel failure";
        case ORBX_ENOMEM: return "allocation failed";
        case ORBX_EINVAL: return "invalid argument";
        case ORBX_ERANGE: return "output capacity too small";
        case ORBX_ENODEV: return "no usable device";
        default: return "unknown error";
    }
}

int orbx_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

orbx_extractor *orbx_extractor_create(int device, int nfeatures, float scaleFactor, int nlevels,
                                      int iniThFAST, int minThFAST) {
    if (nfeatures < 0 || nlevels < 1 || nlevels > kMaxLevels || !(scaleFactor > 1.0f)) return nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return nullptr;
    if (hipSetDevice(device) != hipSuccess) return nullptr;
    orbx_extractor *ex = new (std::nothrow) orbx_extractor();
    if (!ex) return nullptr;
    ex->device = device;
    ex->nfeatures = nfeatures;
    ex->nlevels = nlevels;
    ex->scale_factor = scaleFactor;
    ex->ini_th = iniThFAST;
    ex->min_th = minThFAST;
    if (hipStreamCreateWithFlags(&ex->stream, hipStreamNonBlocking) != hipSuccess) { delete ex; return nullptr; }
    if (const char *sp = std::getenv("ORBX_SPLIT")) ex->split = std::max(1, std::min(std::atoi(sp), orbx_extractor::kMaxParts));
    if (const char *pp = std::getenv("ORBX_PIPELINE")) ex->pipeline = std::max(0, std::min(std::atoi(pp), 2));
    if (const char *pe = std::getenv("ORBX_PIPE_EARLY")) ex->pipe_early = std::max(1, std::atoi(pe));
    if (const char *pd = std::getenv("ORBX_PIPE_DESC")) ex->pipe_desc = std::atoi(pd) != 0;
    if (const char *om = std::getenv("ORBX_OVERLAP_MATCH")) ex->overlap_match = std::atoi(om) != 0;
    if (const char *sg = std::getenv("ORBX_STAGGER")) ex->stagger = std::max(0, std::min(std::atoi(sg), 3));
    if (const char *ck = std::getenv("ORBX_CHUNKS")) ex->chunks = std::max(1, std::min(std::atoi(ck), 64));
    // geometry tables for the getters are size independent; plan a nominal size
    ex->plan = make_plan(640, 480, nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST);
    return ex;
}

void orbx_extractor_destroy(orbx_extractor *ex) {
    if (!ex) return;
    (void)hipSetDevice(ex->device);
    if (ex->stream) (void)hipStreamSynchronize(ex->stream);
    delete ex;
}

int orbx_extractor_get_levels(const orbx_extractor *ex) { return ex ? ex->nlevels : ORBX_EINVAL; }
float orbx_extractor_get_scale_factor(const orbx_extractor *ex) {
    return ex ? (float)(double)ex->scale_factor : 0.f;
}

int orbx_extractor_get_scale_table(const orbx_extractor *ex, int which, float *out, int cap) {
    if (!ex || which < 0 || which > 3 || (cap > 0 && !out)) return ORBX_EINVAL;
    for (int l = 0; l < ex->nlevels && l < cap; ++l) {
        const LevelGeom &g = ex->plan.lv[l];
        out[l] = which == 0 ? g.scale : which == 1 ? g.inv_scale : which == 2 ? g.sigma2 : g.inv_sigma2;
    }
    return ex->nlevels;
}

int orbx_extractor_get_level_quotas(const orbx_extractor *ex, int32_t *out, int cap) {
    if (!ex || (cap > 0 && !out)) return ORBX_EINVAL;
    for (int l = 0; l < ex->nlevels && l < cap; ++l) out[l] = ex->plan.lv[l].quota;
    return ex->nlevels;
}

int orbx_extractor_reserve(orbx_extractor *ex, int width, int height, int max_batch) {
    if (!ex) return ORBX_EINVAL;
    if (hipSetDevice(ex->device) != hipSuccess) return ORBX_ENODEV;
    return reserve(ex, width, height, max_batch);
}

int orbx_extractor_kp_stride(const orbx_extractor *ex) {
    return ex && ex->planned ? ex->plan.max_kps : ORBX_EINVAL;
}

int orbx_extract_batch_device(orbx_extractor *ex, const uint8_t *d_images, int64_t frame_stride, int pitch,
                              int batch, void *stream) {
    int rc = validate_batch(ex, d_images, pitch, batch);
    if (rc) return rc;
    if (hipSetDevice(ex->device) != hipSuccess) return ORBX_ENODEV;
    const int next = ex->cur ^ 1;
    hipStream_t st = stream_of(ex, stream);
    rc = align_level0(ex, &d_images, &frame_stride, &pitch, batch, st);
    if (rc) return rc;
    prof_begin(ex);
    rc = run_extract(ex, next, d_images, frame_stride, pitch, batch, st);
    if (rc) return rc;
    mark(ex, kNumStages, st);
    note_results(ex, st);
    ex->cur = next;
    ex->match_batch = 0;
    return ORBX_OK;
}

int orbx_batch_results_device(orbx_extractor *ex, const orbx_keypoint **d_kps, const uint8_t **d_desc,
                              const int32_t **d_counts) {
    if (!ex || !ex->planned) return ORBX_EINVAL;
    const auto &s = ex->slot[ex->cur];
    if (d_kps) *d_kps = s.kps;
    if (d_desc) *d_desc = s.desc;
    if (d_counts) *d_counts = s.nkps;
    return ORBX_OK;
}

int orbx_batch_pack_device(orbx_extractor *ex, void *d_out, int64_t cap, int64_t *bytes, void *stream) {
    if (!ex || !ex->planned || !bytes) return ORBX_EINVAL;
    const auto &s = ex->slot[ex->cur];
    const int64_t B = s.batch, K = ex->plan.max_kps;
    const int64_t head = (4 * B + 63) / 64 * 64;
    const int64_t need = head + B * K * (int64_t)sizeof(orbx_keypoint) + B * K * 32;
    *bytes = need;
    if (B <= 0) return ORBX_EINVAL;
    if (!d_out) return ORBX_OK;
    if (cap < need) return ORBX_ERANGE;
    if (hipSetDevice(ex->device) != hipSuccess) return ORBX_ENODEV;
    hipStream_t st = stream_of(ex, stream);
    auto *o = static_cast<uint8_t *>(d_out);
    if (hipMemcpyAsync(o, s.nkps, 4 * B, hipMemcpyDeviceToDevice, st) != hipSuccess ||
        hipMemcpyAsync(o + head, s.kps, B * K * sizeof(orbx_keypoint), hipMemcpyDeviceToDevice, st) != hipSuccess ||
        hipMemcpyAsync(o + head + B * K * (int64_t)sizeof(orbx_keypoint), s.desc, B * K * 32,
                       hipMemcpyDeviceToDevice, st) != hipSuccess)
        return ORBX_EIO;
    return ORBX_OK;
}

int orbx_batch_download(orbx_extractor *ex, int frame, orbx_keypoint *kps, uint8_t *desc, int cap, int *n) {
    if (!ex || !ex->planned || !n) return ORBX_EINVAL;
    const auto &s = ex->slot[ex->cur];
    if (frame < 0 || frame >= s.batch) return ORBX_EINVAL;
    if (hipSetDevice(ex->device) != hipSuccess) return ORBX_ENODEV;
    if (sync_results(ex)) return ORBX_EIO;
    int32_t cnt = 0;
    int32_t lc[kMaxLevels];
    D2H copy{ex};
    copy(&cnt, s.nkps + frame, sizeof(int32_t));
    copy(lc, ex->d_level_count + (size_t)frame * kMaxLevels, sizeof(lc));
    if (!copy.wait()) return ORBX_EIO;
    for (int l = 0; l < ex->nlevels; ++l)
        if (lc[l] < 0) return ORBX_EIO;   // quadtree capacity guard tripped
    *n = cnt;
    if (cnt > cap) return ORBX_ERANGE;
    const size_t base = (size_t)frame * ex->plan.max_kps;
    if (cnt > 0 && kps) copy(kps, s.kps + base, sizeof(orbx_keypoint) * cnt);
    if (cnt > 0 && desc) copy(desc, s.desc + base * 32, 32 * (size_t)cnt);
    return copy.wait() ? ORBX_OK : ORBX_EIO;
}

namespace {

// Layout of the host graph's pinned download: [0] keypoint count, [16..80) the
// level counts, then max_kps keypoint records and max_kps descriptors.
constexpr size_t kOutKps = 128;

// Frame 0's results written straight into the pinned (device-visible) host
// buffer: one small kernel instead of four blit copies (~5 us each at B = 1).
// Dwords: [0] count, [2] done flag, [4..20) level counts, then the first
// `count` keypoint records and descriptors (the host reads no further).  One
// workgroup: after its writes are visible system-wide it raises the flag, so
// the host can poll it instead of sleeping in a stream synchronisation (~10
// us of wake-up at B = 1).
constexpr int kOutFlag = 2, kPackThreads = 1024;
__global__ __launch_bounds__(kPackThreads) void k_pack_host(const int32_t *nkps, const int32_t *lc,
                                                            const uint32_t *kps, const uint32_t *desc, int nlevels,
                                                            int kdesc_dw, uint32_t *out) {
    const int n = max(nkps[0], 0);
    const int t = threadIdx.x;
    if (t == 0) out[0] = (uint32_t)nkps[0];
    if (t < kMaxLevels) out[4 + t] = t < nlevels ? (uint32_t)lc[t] : 0u;
    const int nk = n * (int)(sizeof(orbx_keypoint) / 4), nd = n * 8;
    for (int i = t; i < nk; i += kPackThreads) out[kOutKps / 4 + i] = kps[i];
    for (int i = t; i < nd; i += kPackThreads) out[kdesc_dw + i] = desc[i];
    __threadfence_system();
    __syncthreads();
    if (t == 0) __hip_atomic_store(out + kOutFlag, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
size_t out_desc_off(const orbx_extractor *ex) {
    return kOutKps + sizeof(orbx_keypoint) * (size_t)ex->plan.max_kps;
}

bool host_graph_enabled() {
    static const bool on = [] {
        const char *e = std::getenv("ORBX_HOST_GRAPH");
        return !(e && e[0] == '0');
    }();
    return on;
}

// Captures upload + extraction (result slot 0, unsplit, no level pipeline, no
// stage marks) + downloads for a width x height frame.
int build_host_graph(orbx_extractor *ex, int width, int height) {
    if (ex->host_graph) (void)hipGraphExecDestroy(ex->host_graph);
    ex->host_graph = nullptr;
    const size_t dp = (size_t)pitch_of(width), need = dp * height;
    const size_t out_bytes = out_desc_off(ex) + 32 * (size_t)ex->plan.max_kps;
    if (ex->h_img_bytes < need) {
        if (ex->h_img) (void)hipHostFree(ex->h_img);
        ex->h_img = nullptr;
        ex->h_img_bytes = 0;
        if (hipHostMalloc(reinterpret_cast<void **>(&ex->h_img), need, hipHostMallocDefault) != hipSuccess)
            return ORBX_ENOMEM;
        ex->h_img_bytes = need;
    }
    if (ex->h_out_bytes < out_bytes) {
        if (ex->h_out) (void)hipHostFree(ex->h_out);
        ex->h_out = nullptr;
        ex->h_out_bytes = 0;
        if (hipHostMalloc(reinterpret_cast<void **>(&ex->h_out), out_bytes, hipHostMallocDefault) != hipSuccess)
            return ORBX_ENOMEM;
        ex->h_out_bytes = out_bytes;
    }
    hipStream_t st = ex->stream;
    // An overlapped matcher (orbx_extractor_overlap_match) may still read the
    // result slots on match_stream; gate_describe would then wait on match_ev
    // inside the capture, an event recorded outside it (a cross-capture wait
    // invalidates the capture).  Drain it here: the capture then has no gate,
    // and the graph's launch site gates later overlapped steps itself.
    if (ex->match_gate) {
        if (hipEventSynchronize(ex->match_ev) != hipSuccess) return ORBX_EIO;
        ex->match_gate = false;
    }
    const int pipe = ex->pipeline;
    hipEvent_t *ev = ex->cur_ev;
    bool *valid = ex->cur_valid;
    // one linear chain: a graph with the level pipeline's forked branch
    // (ORBX_HOST_PIPE=1) replays its cross-queue joins at ~10-20 us each and
    // measured slower at B = 1 (VGA 0.159 vs 0.141 ms)
    static const bool host_pipe = [] {
        const char *e = std::getenv("ORBX_HOST_PIPE");
        return e && e[0] == '1';
    }();
    ex->pipeline = host_pipe && make_pipe(ex) ? 1 : 0;
    ex->cur_ev = nullptr;
    ex->cur_valid = nullptr;
    auto restore = [&] { ex->pipeline = pipe; ex->cur_ev = ev; ex->cur_valid = valid; };
    // one eager run first: lazy attributes (LDS limits) are set outside the capture
    int rc = run_extract(ex, 0, ex->d_img, (int64_t)need, (int)dp, 1, st);
    if (rc || hipStreamSynchronize(st) != hipSuccess) { restore(); return rc ? rc : ORBX_EIO; }
    hipGraph_t g = nullptr;
    if (hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal) != hipSuccess) { restore(); return ORBX_EIO; }
    const auto &s0 = ex->slot[0];
    bool ok = hipMemcpyAsync(ex->d_img, ex->h_img, need, hipMemcpyHostToDevice, st) == hipSuccess;
    ok = ok && run_extract(ex, 0, ex->d_img, (int64_t)need, (int)dp, 1, st) == ORBX_OK;
    void *dout = nullptr;   // the pinned buffer's device address
    ok = ok && hipHostGetDevicePointer(&dout, ex->h_out, 0) == hipSuccess;
    if (ok) {
        hipLaunchKernelGGL(k_pack_host, dim3(1), dim3(kPackThreads), 0, st, s0.nkps, ex->d_level_count,
                           reinterpret_cast<const uint32_t *>(s0.kps), reinterpret_cast<const uint32_t *>(s0.desc),
                           ex->nlevels, (int)(out_desc_off(ex) / 4), reinterpret_cast<uint32_t *>(dout));
        ok = hipGetLastError() == hipSuccess;
    }
    const bool ended = hipStreamEndCapture(st, &g) == hipSuccess;
    restore();
    if (!ok || !ended || !g) {
        if (g) (void)hipGraphDestroy(g);
        (void)hipGetLastError();
        return ORBX_EIO;
    }
    const bool inst = hipGraphInstantiate(&ex->host_graph, g, nullptr, nullptr, 0) == hipSuccess;
    (void)hipGraphDestroy(g);
    if (!inst) { ex->host_graph = nullptr; return ORBX_EIO; }
    ex->graph_w = width;
    ex->graph_h = height;
    return ORBX_OK;
}

}  // namespace

int orbx_extract(orbx_extractor *ex, const uint8_t *image, int width, int height, size_t pitch,
                 orbx_keypoint *kps, uint8_t *desc, int cap, int *n) {
    if (!ex || !n) return ORBX_EINVAL;
    if (!image || width <= 0 || height <= 0) { *n = -1; return ORBX_OK; }  // ORBextractor.cc:1086-1087
    if (pitch < (size_t)width) return ORBX_EINVAL;
    if (hipSetDevice(ex->device) != hipSuccess) return ORBX_ENODEV;
    const size_t dp = (size_t)pitch_of(width);
    const size_t need = dp * height;
    const bool graph = host_graph_enabled();
    {
        // Setup (plan upload, allocations, graph capture) under one process-wide
        // lock: extractors driven from several threads (Frame's stereo
        // constructor runs two) must not make a synchronous runtime call while
        // another thread's stream is being captured.
        static std::mutex setup_mu;
        std::unique_lock<std::mutex> lk(setup_mu, std::defer_lock);
        const bool ready = ex->planned && ex->plan.width == width && ex->plan.height == height &&
                           ex->d_img_bytes >= need &&
                           (!graph || (ex->host_graph && ex->graph_w == width && ex->graph_h == height));
        if (!ready) lk.lock();
        int rc = reserve(ex, width, height, std::max(1, ex->max_batch));
        if (rc) return rc;
        if (ex->d_img_bytes < need) {
            if (ex->host_graph) (void)hipGraphExecDestroy(ex->host_graph);
            ex->host_graph = nullptr;
            dfree(ex->d_img);
            if (dalloc(&ex->d_img, need) != hipSuccess) return ORBX_ENOMEM;
            ex->d_img_bytes = need;
        }
        if (graph && (!ex->host_graph || ex->graph_w != width || ex->graph_h != height)) {
            rc = build_host_graph(ex, width, height);
            if (rc) return rc;
        }
    }
    int rc = ORBX_OK;
    if (graph) {
        for (int r = 0; r < height; ++r) std::memcpy(ex->h_img + r * dp, image + r * pitch, (size_t)width);
        volatile uint32_t *flag = reinterpret_cast<volatile uint32_t *>(ex->h_out) + kOutFlag;
        *flag = 0;
        std::atomic_thread_fence(std::memory_order_seq_cst);
        if (!gate_describe(ex, ex->stream) || hipGraphLaunch(ex->host_graph, ex->stream) != hipSuccess) return ORBX_EIO;
        // poll the pack kernel's flag; the stream's state ends the wait on an error
        for (uint32_t i = 1; !*flag; ++i) {
            if ((i & 255) == 0 && hipStreamQuery(ex->stream) != hipErrorNotReady) break;
            __builtin_ia32_pause();
        }
        if (!*flag) {   // the stream has ended: a failure, or the flag's write still in flight
            if (hipStreamSynchronize(ex->stream) != hipSuccess) return ORBX_EIO;
            for (int i = 0; i < (1 << 20) && !*flag; ++i) __builtin_ia32_pause();
            if (!*flag) return ORBX_EIO;
        }
        std::atomic_thread_fence(std::memory_order_acquire);
        ex->cur = 0;
        ex->res_pending = false;   // (the graph's work is complete: its last kernel raised the flag)
        ex->match_batch = 0;
        ex->host_result_valid = true;
        int32_t cnt, lc[kMaxLevels];
        std::memcpy(&cnt, ex->h_out, sizeof(cnt));
        std::memcpy(lc, ex->h_out + 16, sizeof(lc));
        for (int l = 0; l < ex->nlevels; ++l)
            if (lc[l] < 0) return ORBX_EIO;   // quadtree capacity guard tripped
        *n = cnt;
        if (cnt > cap) return ORBX_ERANGE;
        if (cnt > 0 && kps) std::memcpy(kps, ex->h_out + kOutKps, sizeof(orbx_keypoint) * (size_t)cnt);
        if (cnt > 0 && desc) std::memcpy(desc, ex->h_out + out_desc_off(ex), 32 * (size_t)cnt);
        return ORBX_OK;
    }
    if (hipMemcpy2DAsync(ex->d_img, dp, image, pitch, width, height, hipMemcpyHostToDevice, ex->stream) != hipSuccess)
        return ORBX_EIO;
    rc = orbx_extract_batch_device(ex, ex->d_img, (int64_t)need, (int)dp, 1, nullptr);
    if (rc) return rc;
    return orbx_batch_download(ex, 0, kps, desc, cap, n);
}

int orbx_extractor_pyramid_level(orbx_extractor *ex, int level, uint8_t *out, size_t out_pitch, int *w, int *h) {
    if (!ex || !ex->planned || level < 0 || level >= ex->nlevels) return ORBX_EINVAL;
    const LevelGeom &g = ex->plan.lv[level];
    if (w) *w = g.w;
    if (h) *h = g.h;
    if (!out) return ORBX_OK;
    if (out_pitch < (size_t)g.w) return ORBX_EINVAL;
    const auto &s = ex->slot[ex->cur];
    if (s.batch <= 0) return ORBX_EINVAL;
    if (hipSetDevice(ex->device) != hipSuccess) return ORBX_ENODEV;
    if (sync_results(ex)) return ORBX_EIO;
    const uint8_t *src = level == 0 ? s.img0 : ex->d_pyr + g.pyr_off;
    const size_t sp = level == 0 ? (size_t)s.img0_pitch : (size_t)g.pitch;
    if (hipMemcpy2DAsync(out, out_pitch, src, sp, g.w, g.h, hipMemcpyDeviceToHost, ex->stream) != hipSuccess)
        return ORBX_EIO;
    return check(hipStreamSynchronize(ex->stream));
}

int orbx_extractor_pyramid_host(orbx_extractor *ex, uint8_t *const *out, const size_t *out_pitch, int nlevels) {
    if (!ex || !ex->planned || !out || !out_pitch || nlevels < 1 || nlevels > ex->nlevels) return ORBX_EINVAL;
    const auto &s = ex->slot[ex->cur];
    if (s.batch <= 0) return ORBX_EINVAL;
    for (int l = 0; l < nlevels; ++l)
        if (!out[l] || out_pitch[l] < (size_t)ex->plan.lv[l].w) return ORBX_EINVAL;
    // two linear spans, pitches included (a 2-D copy of narrow rows runs row by
    // row): level 0 where the last call read it, levels 1.. of frame 0 (one
    // contiguous block of the pyramid)
    const LevelGeom &g0 = ex->plan.lv[0], &gl = ex->plan.lv[nlevels - 1];
    const size_t p0 = (size_t)s.img0_pitch;
    const size_t span0 = p0 * (g0.h - 1) + g0.w;
    const size_t base1 = nlevels > 1 ? (size_t)ex->plan.lv[1].pyr_off : 0;
    const size_t span1 = nlevels > 1 ? (size_t)gl.pyr_off + (size_t)gl.pitch * (gl.h - 1) + gl.w - base1 : 0;
    const size_t off1 = (span0 + 255) & ~size_t(255), total = off1 + span1;
    if (hipSetDevice(ex->device) != hipSuccess) return ORBX_ENODEV;
    if (ex->h_pyr_bytes < total) {
        if (ex->h_pyr) (void)hipHostFree(ex->h_pyr);
        ex->h_pyr = nullptr;
        ex->h_pyr_bytes = 0;
        if (hipHostMalloc(reinterpret_cast<void **>(&ex->h_pyr), total, hipHostMallocDefault) != hipSuccess)
            return ORBX_ENOMEM;
        ex->h_pyr_bytes = total;
    }
    if (sync_results(ex)) return ORBX_EIO;
    if (hipMemcpyAsync(ex->h_pyr, s.img0, span0, hipMemcpyDeviceToHost, ex->stream) != hipSuccess ||
        (span1 && hipMemcpyAsync(ex->h_pyr + off1, ex->d_pyr + base1, span1, hipMemcpyDeviceToHost, ex->stream) !=
                      hipSuccess) ||
        hipStreamSynchronize(ex->stream) != hipSuccess)
        return ORBX_EIO;
    for (int l = 0; l < nlevels; ++l) {
        const LevelGeom &g = ex->plan.lv[l];
        const uint8_t *src = l == 0 ? ex->h_pyr : ex->h_pyr + off1 + ((size_t)g.pyr_off - base1);
        const size_t sp = l == 0 ? p0 : (size_t)g.pitch;
        for (int r = 0; r < g.h; ++r) std::memcpy(out[l] + (size_t)r * out_pitch[l], src + (size_t)r * sp, g.w);
    }
    return ORBX_OK;
}

int orbx_extractor_debug_fetch(orbx_extractor *ex, int frame, int level, int what, void *out, int64_t cap) {
    if (!ex || !ex->planned || level < 0 || level >= ex->nlevels || !out) return ORBX_EINVAL;
    const auto &s = ex->slot[ex->cur];
    if (frame < 0 || frame >= s.batch) return ORBX_EINVAL;
    if (hipSetDevice(ex->device) != hipSuccess) return ORBX_ENODEV;
    if (sync_results(ex)) return ORBX_EIO;
    const Plan &p = ex->plan;
    const LevelGeom &g = p.lv[level];
    if (what == 0 || what == 1) {
        if (cap < (int64_t)g.w * g.h) return ORBX_ERANGE;
        const uint8_t *src;
        size_t sp;
        if (what == 0) {
            src = level == 0 ? s.img0 + (int64_t)frame * s.img0_stride
                             : ex->d_pyr + (int64_t)frame * p.pyr_bytes + g.pyr_off;
            sp = level == 0 ? (size_t)s.img0_pitch : (size_t)g.pitch;
        } else {
            // the hot path blurs patch-locally inside k_describe; materialise the
            // full blurred pyramid on demand with the standalone kernel
            if (launch_blur(ex->dp, frame_bufs(ex, ex->cur), s.batch, ex->stream) != hipSuccess ||
                hipStreamSynchronize(ex->stream) != hipSuccess)
                return ORBX_EIO;
            src = ex->d_blur + (int64_t)frame * p.blur_bytes + g.blur_off;
            sp = (size_t)g.pitch;
        }
        if (hipMemcpy2D(out, g.w, src, sp, g.w, g.h, hipMemcpyDeviceToHost) != hipSuccess) return ORBX_EIO;
        return g.w * g.h;
    }
    int32_t *o = static_cast<int32_t *>(out);
    if (what == 2) {
        const int nc = g.cell_end - g.cell_begin;
        std::vector<int32_t> counts(nc);
        if (nc && hipMemcpy(counts.data(), ex->d_cell_count + (size_t)frame * p.cells.size() + g.cell_begin,
                            sizeof(int32_t) * nc, hipMemcpyDeviceToHost) != hipSuccess)
            return ORBX_EIO;
        std::vector<uint32_t> cand(g.cand_cap), cand2(g.cand_cap);
        if (g.cand_cap && (hipMemcpy(cand.data(), ex->d_cand + (size_t)frame * p.cand_cap + g.cand_off,
                                     sizeof(uint32_t) * g.cand_cap, hipMemcpyDeviceToHost) != hipSuccess ||
                           hipMemcpy(cand2.data(), ex->d_cand2 + (size_t)frame * p.cand_cap + g.cand_off,
                                     sizeof(uint32_t) * g.cand_cap, hipMemcpyDeviceToHost) != hipSuccess))
            return ORBX_EIO;
        int64_t k = 0;
        for (int c = 0; c < nc; ++c) {
            const Cell &cell = p.cells[g.cell_begin + c];
            const std::vector<uint32_t> &src = counts[c] < 0 ? cand2 : cand;
            const int cnt = counts[c] & 0x7FFFFFFF;
            for (int i = 0; i < cnt; ++i, ++k) {
                if (3 * (k + 1) > cap) return ORBX_ERANGE;
                const uint32_t v = src[cell.slot - g.cand_off + i];
                o[3 * k] = (int32_t)(v & 0xFFF);
                o[3 * k + 1] = (int32_t)((v >> 12) & 0xFFF);
                o[3 * k + 2] = (int32_t)(v >> 24);
            }
        }
        return (int)k;
    }
    if (what == 3) {
        int32_t cnt = 0;
        if (hipMemcpy(&cnt, ex->d_level_count + (size_t)frame * kMaxLevels + level, sizeof(int32_t),
                      hipMemcpyDeviceToHost) != hipSuccess)
            return ORBX_EIO;
        if (cnt < 0) return ORBX_EIO;
        if (3 * (int64_t)cnt > cap) return ORBX_ERANGE;
        std::vector<uint32_t> sel(cnt);
        if (cnt && hipMemcpy(sel.data(), ex->d_sel + (size_t)frame * p.out_cap + g.out_off, sizeof(uint32_t) * cnt,
                             hipMemcpyDeviceToHost) != hipSuccess)
            return ORBX_EIO;
        for (int i = 0; i < cnt; ++i) {
            o[3 * i] = (int32_t)(sel[i] & 0xFFF);
            o[3 * i + 1] = (int32_t)((sel[i] >> 12) & 0xFFF);
            o[3 * i + 2] = (int32_t)(sel[i] >> 24);
        }
        return cnt;
    }
    return ORBX_EINVAL;
}

int orbx_mono_step_device(orbx_extractor *ex, const uint8_t *d_images, int64_t frame_stride, int pitch, int batch,
                          int window, float nnratio, int check_ori, void *stream) {
    int rc = validate_batch(ex, d_images, pitch, batch);
    if (rc) return rc;
    if (hipSetDevice(ex->device) != hipSuccess) return ORBX_ENODEV;
    hipStream_t st = stream_of(ex, stream);
    rc = align_level0(ex, &d_images, &frame_stride, &pitch, batch, st);
    if (rc) return rc;
    const int prev = ex->cur, next = ex->cur ^ 1;
    const bool have_prev = ex->slot[prev].batch == batch && ex->steps > 0;
    prof_begin(ex);
    const Parts P = fork_parts(ex, st, batch);
    rc = run_extract(ex, next, d_images, frame_stride, pitch, batch, P);
    if (rc) return rc;
    ex->cur = next;
    ++ex->steps;
    ex->match_batch = 0;
    if (!have_prev) {
        if ((rc = join_parts(ex, st, P))) return rc;
        mark(ex, kNumStages, st);
        note_results(ex, st);
        return ORBX_OK;
    }
    MatchBufs mb{};
    const auto &s1 = ex->slot[prev];
    const auto &s2 = ex->slot[next];
    mb.k1 = s1.kps; mb.d1 = s1.desc; mb.n1 = s1.nkps; mb.k1_stride = ex->plan.max_kps;
    mb.k2 = s2.kps; mb.d2 = s2.desc; mb.n2 = s2.nkps; mb.k2_stride = ex->plan.max_kps;
    mb.prev_xy = ex->d_prev;
    mb.matches12 = ex->d_m12;
    mb.nmatches = ex->d_nmatch;
    mb.min_x = 0.f; mb.max_x = (float)ex->plan.width;    // undistorted frames (Frame.cc:495-497)
    mb.min_y = 0.f; mb.max_y = (float)ex->plan.height;
    mb.window = window;
    mb.nnratio = nnratio;
    mb.check_ori = check_ori;
    mb.reset_prev = 1;
    mb.clocks = nullptr;
    if (ex->overlap_match && !ex->profiling) {
        // the matcher for the whole batch on match_stream, after the extraction
        if ((rc = join_parts(ex, st, P))) return rc;
        if (!ex->match_stream) {
            if (fork_stream(&ex->match_stream) != hipSuccess ||
                hipEventCreateWithFlags(&ex->ext_ev, hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&ex->match_ev, hipEventDisableTiming) != hipSuccess)
                return ORBX_EIO;
        }
        if (hipEventRecord(ex->ext_ev, st) != hipSuccess || hipStreamWaitEvent(ex->match_stream, ex->ext_ev, 0) != hipSuccess)
            return ORBX_EIO;
        if (launch_match(mb, batch, ex->plan.max_kps, ex->plan.max_kps, ex->l0cap, ex->l0cap, ex->match_stream) != hipSuccess ||
            hipEventRecord(ex->match_ev, ex->match_stream) != hipSuccess)
            return ORBX_EIO;
        ex->match_gate = true;
        note_results(ex, ex->match_stream);
        ex->match_batch = batch;
        return ORBX_OK;
    }
    static const bool dbg_clocks = std::getenv("ORBX_MATCH_CLOCKS") != nullptr;
    long long *dclk = nullptr;
    if (dbg_clocks && hipMalloc(reinterpret_cast<void **>(&dclk), 8 * sizeof(long long)) == hipSuccess)
        mb.clocks = dclk;
    if (ex->match_gate) {   // (overlap just turned off: the last overlapped matcher writes the same state)
        for (int k = 0; k < P.n; ++k)
            if (hipStreamWaitEvent(P.s[k], ex->match_ev, 0) != hipSuccess) return ORBX_EIO;
        ex->match_gate = false;
    }
    for (int k = 0; k < P.n; ++k) {
        MatchBufs pm = offset_pairs(mb, P.b0[k]);
        if (k > 0) pm.clocks = nullptr;
        if (launch_match(pm, P.nb[k], ex->plan.max_kps, ex->plan.max_kps, ex->l0cap, ex->l0cap, P.s[k]) != hipSuccess)
            return ORBX_EIO;
    }
    if ((rc = join_parts(ex, st, P))) return rc;
    if (dclk) {   // debug: phase cycle counts of pair 0
        long long c[8] = {};
        if (hipStreamSynchronize(st) == hipSuccess &&
            hipMemcpy(c, dclk, sizeof(c), hipMemcpyDeviceToHost) == hipSuccess)
            std::fprintf(stderr, "match phases (cycles): init %lld grid+queries %lld lists %lld replay %lld tail %lld; "
                         "live queries %lld replay batches %lld\n",
                         c[1] - c[0], c[2] - c[1], c[3] - c[2], c[4] - c[3], c[5] - c[4], c[7], c[6]);
        (void)hipFree(dclk);
    }
    mark(ex, kNumStages, st);
    note_results(ex, st);
    mark_valid(ex, kStageMatch);
    ex->match_batch = batch;
    return ORBX_OK;
}

int orbx_mono_matches_download(orbx_extractor *ex, int frame, int32_t *matches12, int cap, int *n1, int *nmatches) {
    if (!ex || !ex->planned || frame < 0 || frame >= ex->match_batch) return ORBX_EINVAL;
    if (hipSetDevice(ex->device) != hipSuccess) return ORBX_ENODEV;
    if (sync_results(ex)) return ORBX_EIO;
    const int prev = ex->cur ^ 1;
    int32_t cnt = 0, nm = 0;
    D2H copy{ex};
    copy(&cnt, ex->slot[prev].nkps + frame, sizeof(int32_t));
    copy(&nm, ex->d_nmatch + frame, sizeof(int32_t));
    if (!copy.wait()) return ORBX_EIO;
    if (nm < 0) return ORBX_EIO;
    if (n1) *n1 = cnt;
    if (nmatches) *nmatches = nm;
    if (cnt > cap) return ORBX_ERANGE;
    if (cnt > 0 && matches12) copy(matches12, ex->d_m12 + (size_t)frame * ex->plan.max_kps, sizeof(int32_t) * cnt);
    return copy.wait() ? ORBX_OK : ORBX_EIO;
}

int orbx_extractor_overlap_match(orbx_extractor *ex, int on) {
    if (!ex || on < -1 || on > 1) return ORBX_EINVAL;
    if (on >= 0) ex->overlap_match = on != 0;
    return ex->overlap_match;
}

int orbx_extractor_pipeline(orbx_extractor *ex, int on) {
    if (!ex || on < -1 || on > 2) return ORBX_EINVAL;
    if (on >= 0) ex->pipeline = on;
    return ex->pipeline;
}

int orbx_extractor_split(orbx_extractor *ex, int parts) {
    if (!ex || parts < 0 || parts > orbx_extractor::kMaxParts) return ORBX_EINVAL;
    if (parts > 0) ex->split = parts;
    return ex->split;
}

int orbx_extractor_set_profiling(orbx_extractor *ex, int on) {
    if (!ex) return ORBX_EINVAL;
    if (hipSetDevice(ex->device) != hipSuccess) return ORBX_ENODEV;
    for (int s = 0; s < orbx_extractor::kRing; ++s) fold(ex, s);
    for (int i = 0; i < kNumStages; ++i) { ex->stage_sum[i] = 0; ex->stage_cnt[i] = 0; }
    ex->profiling = on != 0;
    return ORBX_OK;
}

int orbx_extractor_stage_times(orbx_extractor *ex, float *ms, int cap) {
    if (!ex || (cap > 0 && !ms)) return ORBX_EINVAL;
    if (hipSetDevice(ex->device) != hipSuccess) return ORBX_ENODEV;
    for (int s = 0; s < orbx_extractor::kRing; ++s) fold(ex, s);
    int nw = 0;
    for (int i = 0; i < kNumStages && i < cap; ++i) {
        ms[i] = ex->stage_cnt[i] ? (float)(ex->stage_sum[i] / ex->stage_cnt[i]) : -1.f;
        ++nw;
    }
    return nw;
}

namespace {
// The host arrays are the extractor's own last host-API result (Frame passes
// the mvKeys / mDescriptors ExtractORB just returned): its device copies serve.
bool same_as_last_host_result(const orbx_extractor *ex, const orbx_keypoint *k, const uint8_t *d, int n) {
    if (!ex->host_result_valid || ex->cur != 0 || !ex->h_out) return false;
    int32_t cnt;
    std::memcpy(&cnt, ex->h_out, sizeof(cnt));
    return cnt == n && (n == 0 || (std::memcmp(k, ex->h_out + kOutKps, sizeof(orbx_keypoint) * (size_t)n) == 0 &&
                                   std::memcmp(d, ex->h_out + out_desc_off(ex), 32 * (size_t)n) == 0));
}
}  // namespace

int orbx_compute_stereo_matches(orbx_extractor *left, orbx_extractor *right, const orbx_keypoint *kl,
                                const uint8_t *dl, int nl, const orbx_keypoint *kr, const uint8_t *dr, int nr,
                                float mbf, float mb, float *uright, float *depth, int *nkept) {
    if (!left || !right || !left->planned || !right->planned || !nkept) return ORBX_EINVAL;
    if (nl < 0 || nr < 0 || nr > 65535 || (nl && (!kl || !dl || !uright || !depth)) || (nr && (!kr || !dr)))
        return ORBX_EINVAL;
    if (left->device != right->device || !same_geometry(left->plan, right->plan)) return ORBX_EINVAL;
    if (left->slot[left->cur].batch <= 0 || right->slot[right->cur].batch <= 0) return ORBX_EINVAL;
    *nkept = 0;
    if (nl == 0) return ORBX_OK;
    const int rows = left->plan.height;
    const int ncap = std::max(nr, 1);
    if (stereo_lds_bytes(rows, ncap) > 160 * 1024) return ORBX_EINVAL;
    if (hipSetDevice(left->device) != hipSuccess) return ORBX_ENODEV;
    if (hipStreamSynchronize(right->stream) != hipSuccess || hipStreamSynchronize(left->stream) != hipSuccess)
        return ORBX_EIO;
    auto &w = left->sws;
    if (nl > w.cap_l || ncap > w.cap_r) {
        w.free_dev();
        const int cl = std::max(nl, left->plan.max_kps), cr = std::max(ncap, left->plan.max_kps);
        if (dalloc(&w.kl, cl) != hipSuccess || dalloc(&w.dl, 32 * (size_t)cl) != hipSuccess ||
            dalloc(&w.kr, cr) != hipSuccess || dalloc(&w.dr, 32 * (size_t)cr) != hipSuccess ||
            dalloc(&w.n, 2) != hipSuccess || dalloc(&w.sad, cl) != hipSuccess || dalloc(&w.nk, 1) != hipSuccess ||
            dalloc(&w.ur, cl) != hipSuccess || dalloc(&w.depth, cl) != hipSuccess) {
            w.free_dev();
            return ORBX_ENOMEM;
        }
        w.cap_l = cl;
        w.cap_r = cr;
    }
    const size_t hb = 8 * (size_t)w.cap_l + 16;
    if (w.h_bytes < hb) {
        if (w.h_res) (void)hipHostFree(w.h_res);
        w.h_res = nullptr;
        w.h_bytes = 0;
        if (hipHostMalloc(reinterpret_cast<void **>(&w.h_res), hb, hipHostMallocDefault) != hipSuccess)
            return ORBX_ENOMEM;
        w.h_bytes = hb;
    }
    hipStream_t st = left->stream;
    StereoBufs a{};
    a.lv = left->dp.lv; a.nlevels = left->nlevels; a.rows = rows;
    a.left = pyr_view(left, left->cur); a.right = pyr_view(right, right->cur);
    a.left_f0 = 0; a.right_f0 = 0; a.fstep = 0;
    a.kstride = 0; a.nstride = 0; a.nr_cap = ncap;
    // each side: the extractor's resident result when the host arrays are it,
    // else an upload (with the counts in the workspace)
    const bool lhit = same_as_last_host_result(left, kl, dl, nl), rhit = same_as_last_host_result(right, kr, dr, nr);
    const int32_t ns[2] = {nl, nr};
    bool ok = true;
    if (!lhit || !rhit) ok = hipMemcpyAsync(w.n, ns, sizeof(ns), hipMemcpyHostToDevice, st) == hipSuccess;
    if (lhit) {
        a.kl = left->slot[0].kps; a.dl = left->slot[0].desc; a.nl = left->slot[0].nkps;
    } else {
        ok = ok && hipMemcpyAsync(w.kl, kl, sizeof(orbx_keypoint) * nl, hipMemcpyHostToDevice, st) == hipSuccess &&
             hipMemcpyAsync(w.dl, dl, 32 * (size_t)nl, hipMemcpyHostToDevice, st) == hipSuccess;
        a.kl = w.kl; a.dl = w.dl; a.nl = w.n;
    }
    if (rhit) {
        a.kr = right->slot[0].kps; a.dr = right->slot[0].desc; a.nr = right->slot[0].nkps;
    } else {
        ok = ok && (nr == 0 || (hipMemcpyAsync(w.kr, kr, sizeof(orbx_keypoint) * nr, hipMemcpyHostToDevice, st) ==
                                    hipSuccess &&
                                hipMemcpyAsync(w.dr, dr, 32 * (size_t)nr, hipMemcpyHostToDevice, st) == hipSuccess));
        a.kr = w.kr; a.dr = w.dr; a.nr = w.n + 1;
    }
    a.mbf = mbf; a.maxd = mbf / mb;
    a.ur = w.ur; a.depth = w.depth; a.sad = w.sad; a.ostride = 0; a.nkept = w.nk;
    // k_stereo_cut writes the results straight into the pinned buffer
    void *hdev = nullptr;
    ok = ok && hipHostGetDevicePointer(&hdev, w.h_res, 0) == hipSuccess;
    a.hout = static_cast<float *>(hdev);
    a.hcap = w.cap_l;
    ok = ok && launch_stereo(a, 1, nl, st) == hipSuccess && hipStreamSynchronize(st) == hipSuccess;
    if (!ok) return ORBX_EIO;
    std::memcpy(uright, w.h_res, 4 * (size_t)nl);
    std::memcpy(depth, w.h_res + 4 * (size_t)w.cap_l, 4 * (size_t)nl);
    std::memcpy(nkept, w.h_res + 8 * (size_t)w.cap_l, sizeof(int32_t));
    return ORBX_OK;
}

int orbx_stereo_step_device(orbx_extractor *ex, const uint8_t *d_images, int64_t frame_stride, int pitch, int pairs,
                            float mbf, float mb, void *stream) {
    if (pairs <= 0) return ORBX_EINVAL;
    int rc = validate_batch(ex, d_images, pitch, 2 * pairs);
    if (rc) return rc;
    const int kcap = ex->plan.max_kps;
    if (kcap > 65535 || stereo_lds_bytes(ex->plan.height, kcap) > 160 * 1024) return ORBX_EINVAL;
    if (hipSetDevice(ex->device) != hipSuccess) return ORBX_ENODEV;
    hipStream_t st = stream_of(ex, stream);
    rc = align_level0(ex, &d_images, &frame_stride, &pitch, 2 * pairs, st);
    if (rc) return rc;
    const int next = ex->cur ^ 1;
    prof_begin(ex);
    {   // (a split batch joins before the pairs are matched: a part boundary may cut a pair)
        const Parts P = fork_parts(ex, st, 2 * pairs);
        rc = run_extract(ex, next, d_images, frame_stride, pitch, 2 * pairs, P);
        if (!rc) rc = join_parts(ex, st, P);
    }
    if (rc) return rc;
    ex->cur = next;
    ++ex->steps;
    ex->match_batch = 0;
    const auto &s = ex->slot[next];
    StereoBufs a{};
    a.lv = ex->dp.lv; a.nlevels = ex->nlevels; a.rows = ex->plan.height;
    a.left = a.right = pyr_view(ex, next);
    a.left_f0 = 0; a.right_f0 = 1; a.fstep = 2;
    a.kl = s.kps; a.dl = s.desc; a.nl = s.nkps;
    a.kr = s.kps + kcap; a.dr = s.desc + (size_t)kcap * 32; a.nr = s.nkps + 1;
    a.kstride = 2 * (int64_t)kcap; a.nstride = 2; a.nr_cap = kcap;
    a.mbf = mbf; a.maxd = mbf / mb;
    a.ur = ex->d_ur; a.depth = ex->d_depth; a.sad = ex->d_sad; a.ostride = kcap; a.nkept = ex->d_nkept;
    a.bands = ex->d_bands; a.band_stride = stereo_band_stride(a.rows, kcap);
    {   // the median cut fused into the search's last workgroups: measured slower
        // (EuRoC depth 0.106 -> 0.23 ms, profiles/r04_ab_stereo_fused_cut.txt), so
        // only with ORBX_STEREO_FUSED_CUT=1
        const char *e = std::getenv("ORBX_STEREO_FUSED_CUT");
        a.pair_done = (e && e[0] == '1') ? ex->d_pair_done : nullptr;
        // each launch starts from zeroed counters (a failed launch cannot leave
        // them counting for the next one)
        if (a.pair_done && hipMemsetAsync(a.pair_done, 0, sizeof(int32_t) * (size_t)pairs, st) != hipSuccess)
            return ORBX_EIO;
    }
    if (launch_stereo(a, pairs, kcap, st) != hipSuccess) return ORBX_EIO;
    mark(ex, kNumStages, st);
    note_results(ex, st);
    mark_valid(ex, kStageMatch);
    ex->depth_mode = 1;
    ex->depth_count = pairs;
    return ORBX_OK;
}

int orbx_rgbd_step_device(orbx_extractor *ex, const uint8_t *d_images, int64_t frame_stride, int pitch, int batch,
                          const float *d_depth, int64_t depth_stride, int depth_pitch, float mbf, void *stream) {
    int rc = validate_batch(ex, d_images, pitch, batch);
    if (rc) return rc;
    if (!d_depth || depth_pitch < 4 * ex->plan.width || (depth_pitch & 3) || (depth_stride & 3) ||
        (reinterpret_cast<uintptr_t>(d_depth) & 3))
        return ORBX_EINVAL;
    if (hipSetDevice(ex->device) != hipSuccess) return ORBX_ENODEV;
    hipStream_t st = stream_of(ex, stream);
    rc = align_level0(ex, &d_images, &frame_stride, &pitch, batch, st);
    if (rc) return rc;
    const int next = ex->cur ^ 1;
    prof_begin(ex);
    {
        const Parts P = fork_parts(ex, st, batch);
        rc = run_extract(ex, next, d_images, frame_stride, pitch, batch, P);
        if (!rc) rc = join_parts(ex, st, P);
    }
    if (rc) return rc;
    ex->cur = next;
    ++ex->steps;
    ex->match_batch = 0;
    const auto &s = ex->slot[next];
    const int kcap = ex->plan.max_kps;
    if (launch_rgbd(s.kps, nullptr, s.nkps, kcap, kcap, d_depth, depth_stride, depth_pitch, ex->plan.width,
                    ex->plan.height, mbf, ex->d_ur, ex->d_depth, kcap, ex->d_nkept, batch, st) != hipSuccess)
        return ORBX_EIO;
    mark(ex, kNumStages, st);
    note_results(ex, st);
    mark_valid(ex, kStageMatch);
    ex->depth_mode = 2;
    ex->depth_count = batch;
    return ORBX_OK;
}

int orbx_depth_download(orbx_extractor *ex, int index, float *uright, float *depth, int cap, int *n, int *nkept) {
    if (!ex || !ex->planned || !n || ex->depth_mode == 0 || index < 0 || index >= ex->depth_count) return ORBX_EINVAL;
    if (hipSetDevice(ex->device) != hipSuccess) return ORBX_ENODEV;
    if (sync_results(ex)) return ORBX_EIO;
    const int frame = ex->depth_mode == 1 ? 2 * index : index;
    int32_t cnt = 0, nk = 0;
    D2H copy{ex};
    copy(&cnt, ex->slot[ex->cur].nkps + frame, sizeof(int32_t));
    copy(&nk, ex->d_nkept + index, sizeof(int32_t));
    if (!copy.wait()) return ORBX_EIO;
    *n = cnt;
    if (nkept) *nkept = nk;
    if (cnt > cap) return ORBX_ERANGE;
    const size_t base = (size_t)index * ex->plan.max_kps;
    if (cnt > 0 && uright) copy(uright, ex->d_ur + base, 4 * (size_t)cnt);
    if (cnt > 0 && depth) copy(depth, ex->d_depth + base, 4 * (size_t)cnt);
    return copy.wait() ? ORBX_OK : ORBX_EIO;
}

int orbx_stereo_from_rgbd(int device, const orbx_keypoint *kps, const orbx_keypoint *kps_un, int n,
                          const float *depth_map, int width, int height, size_t pitch, float mbf, float *uright,
                          float *depth, int *nkept) {
    if (n < 0 || width <= 0 || height <= 0 || pitch < 4 * (size_t)width || (pitch & 3) || !depth_map || !nkept)
        return ORBX_EINVAL;
    if (n && (!kps || !uright || !depth)) return ORBX_EINVAL;
    *nkept = 0;
    if (n == 0) return ORBX_OK;
    if (hipSetDevice(device) != hipSuccess) return ORBX_ENODEV;
    // the per-call workspace (no allocation per call); inputs: mvKeysUn and the
    // depth samples imDepth.at<float>(v, u) at the mvKeys positions (an
    // out-of-image keypoint, undefined in the reference, gets 0: no depth)
    Layout L;
    const size_t o_k = L.add(sizeof(orbx_keypoint) * (size_t)n), o_s = L.add(4 * (size_t)n);
    const size_t o_nk = L.add(16), in_end = L.size;   // nkept, then the HostTail counter
    const size_t o_ur = L.add(4 * (size_t)n), o_d = L.add(4 * (size_t)n), out_end = L.size;
    CallWs &ws = call_ws(device);
    std::lock_guard<std::mutex> lock(ws.mu);
    int rc = ws_reserve(ws, L.size);
    if (rc) return rc;
    put(ws, o_k, kps_un ? kps_un : kps, sizeof(orbx_keypoint) * (size_t)n);
    float *samp = reinterpret_cast<float *>(ws.host + o_s);
    const size_t pf = pitch / 4;
    for (int i = 0; i < n; ++i) {
        const int v = (int)kps[i].y, u = (int)kps[i].x;
        samp[i] = (v >= 0 && v < height && u >= 0 && u < width) ? depth_map[(size_t)v * pf + u] : 0.0f;
    }
    std::memset(ws.host + o_nk, 0, 16);
    uint8_t *D = ws.dev;
    // (the count sits just before the outputs: one contiguous run back, by
    // the kernel's last workgroup)
    HostTail tail;
    ws_tail(ws, o_nk, out_end - o_nk, at<uint32_t>(D, o_nk + 4), (n + 255) / 256, tail);
    if (hipMemcpyAsync(D, ws.host, in_end, hipMemcpyHostToDevice, ws.st) != hipSuccess ||
        launch_rgbd_samples(at<float>(D, o_s), at<orbx_keypoint>(D, o_k), n, mbf, at<float>(D, o_ur),
                            at<float>(D, o_d), at<int32_t>(D, o_nk), tail, ws.st) != hipSuccess)
        return ORBX_EIO;
    if (ws_wait(ws, tail, o_nk, out_end - o_nk)) return ORBX_EIO;
    get(ws, o_ur, uright, 4 * (size_t)n);
    get(ws, o_d, depth, 4 * (size_t)n);
    get(ws, o_nk, nkept, 4);
    return ORBX_OK;
}

int orbx_descriptor_distance(const uint8_t *a, const uint8_t *b) {
    if (!a || !b) return ORBX_EINVAL;
    int dist = 0;
    for (int i = 0; i < 8; ++i) {
        uint32_t pa, pb;
        std::memcpy(&pa, a + 4 * i, 4);
        std::memcpy(&pb, b + 4 * i, 4);
        dist += popcount32(pa ^ pb);
    }
    return dist;
}

int orbx_search_for_initialization(int device, const orbx_keypoint *k1, const uint8_t *d1, int n1,
                                   const orbx_keypoint *k2, const uint8_t *d2, int n2, int img_w, int img_h,
                                   float *prev_xy, int32_t *matches12, int window, float nnratio, int check_ori,
                                   int *nmatches) {
    if (img_w <= 0 || img_h <= 0) return ORBX_EINVAL;
    return orbx_search_for_initialization_bounds(device, k1, d1, n1, k2, d2, n2, 0.f, (float)img_w, 0.f,
                                                 (float)img_h, prev_xy, matches12, window, nnratio, check_ori,
                                                 nmatches);
}

int orbx_search_for_initialization_bounds(int device, const orbx_keypoint *k1, const uint8_t *d1, int n1,
                                          const orbx_keypoint *k2, const uint8_t *d2, int n2, float min_x,
                                          float max_x, float min_y, float max_y, float *prev_xy, int32_t *matches12,
                                          int window, float nnratio, int check_ori, int *nmatches) {
    if (n1 < 0 || n2 < 0 || n1 > 32767 || n2 > 32767 || !nmatches) return ORBX_EINVAL;
    if (!(max_x > min_x) || !(max_y > min_y) || !std::isfinite(min_x) || !std::isfinite(max_x) ||
        !std::isfinite(min_y) || !std::isfinite(max_y))
        return ORBX_EINVAL;
    if ((n1 && (!k1 || !d1 || !prev_xy || !matches12)) || (n2 && (!k2 || !d2))) return ORBX_EINVAL;
    if (hipSetDevice(device) != hipSuccess) return ORBX_ENODEV;
    int q = 0, c = 0;
    for (int i = 0; i < n1; ++i) q += k1[i].octave == 0;
    for (int i = 0; i < n2; ++i) c += k2[i].octave == 0;
    q = std::max(q, 1);
    c = std::max(c, 1);
    if (match_lds_bytes(std::max(n1, 1), std::max(n2, 1), q, c) > 160 * 1024) return ORBX_EINVAL;
    const int n1c = std::max(n1, 1), n2c = std::max(n2, 1);
    Layout L;
    const size_t o_k1 = L.add(sizeof(orbx_keypoint) * n1c), o_d1 = L.add(32 * (size_t)n1c),
                 o_k2 = L.add(sizeof(orbx_keypoint) * n2c), o_d2 = L.add(32 * (size_t)n2c), o_ns = L.add(8);
    const size_t o_prev = L.add(8 * (size_t)n1c);   // in / out
    // outputs (uploaded with the inputs: the HostTail counter goes up as 0)
    const size_t o_m = L.add(4 * (size_t)n1c), o_nm = L.add(16);   // nmatches, then the HostTail counter
    const size_t out_end = L.size;
    CallWs &ws = call_ws(device);
    std::lock_guard<std::mutex> lock(ws.mu);
    int rc = ws_reserve(ws, L.size);
    if (rc) return rc;
    const int32_t ns[2] = {n1, n2};
    put(ws, o_k1, k1, sizeof(orbx_keypoint) * n1);
    put(ws, o_d1, d1, 32 * (size_t)n1);
    put(ws, o_k2, k2, sizeof(orbx_keypoint) * n2);
    put(ws, o_d2, d2, 32 * (size_t)n2);
    put(ws, o_ns, ns, sizeof(ns));
    put(ws, o_prev, prev_xy, 8 * (size_t)n1);
    std::memset(ws.host + o_nm + 4, 0, 4);
    uint8_t *D = ws.dev;
    if (hipMemcpyAsync(D, ws.host, out_end, hipMemcpyHostToDevice, ws.st) != hipSuccess) return ORBX_EIO;
    MatchBufs mb{};
    mb.k1 = at<orbx_keypoint>(D, o_k1); mb.d1 = D + o_d1; mb.n1 = at<int32_t>(D, o_ns); mb.k1_stride = n1c;
    mb.k2 = at<orbx_keypoint>(D, o_k2); mb.d2 = D + o_d2; mb.n2 = at<int32_t>(D, o_ns) + 1; mb.k2_stride = n2c;
    mb.prev_xy = at<float>(D, o_prev); mb.matches12 = at<int32_t>(D, o_m); mb.nmatches = at<int32_t>(D, o_nm);
    mb.min_x = min_x; mb.max_x = max_x; mb.min_y = min_y; mb.max_y = max_y;
    mb.window = window; mb.nnratio = nnratio;
    mb.check_ori = check_ori; mb.reset_prev = 0; mb.clocks = nullptr;
    ws_tail(ws, o_prev, out_end - o_prev, at<uint32_t>(D, o_nm + 4), 1, mb.tail);
    if (launch_match(mb, 1, n1c, n2c, q, c, ws.st) != hipSuccess) return ORBX_EIO;
    if (ws_wait(ws, mb.tail, o_prev, out_end - o_prev)) return ORBX_EIO;
    int32_t nm = 0;
    get(ws, o_nm, &nm, 4);
    if (nm < 0) return ORBX_EIO;
    get(ws, o_m, matches12, 4 * (size_t)n1);
    get(ws, o_prev, prev_xy, 8 * (size_t)n1);
    *nmatches = nm;
    return ORBX_OK;
}

namespace {

// Checks one projection problem; 1 = nothing to search (outputs filled here).
int proj_check(int variant, const orbx_match_frame *F, const orbx_proj_query *queries, const uint8_t *qdesc, int nq,
               int th_dist, int32_t *q_idx, int32_t *q_dist, int32_t *kp_final, int *nmatches) {
    if (!F || !nmatches || variant < ORBX_PROJ_LOCALMAP || variant > ORBX_PROJ_FUSE_SIM3) return ORBX_EINVAL;
    const int n = F->n;
    if (n < 0 || n > 32767 || nq < 0 || th_dist < 0 || th_dist > 255) return ORBX_EINVAL;
    if ((n && (!F->keys || !F->desc || !kp_final)) || (nq && (!queries || !qdesc || !q_idx || !q_dist)))
        return ORBX_EINVAL;
    if (variant == ORBX_PROJ_FUSE && (!F->inv_sigma2 || F->nlevels <= 0 || F->nlevels > kMaxLevels)) return ORBX_EINVAL;
    if (!(F->max_x > F->min_x) || !(F->max_y > F->min_y)) return ORBX_EINVAL;
    *nmatches = 0;
    if (n == 0 || nq == 0) {
        for (int i = 0; i < nq; ++i) { q_idx[i] = -1; q_dist[i] = -1; }
        for (int i = 0; i < n; ++i) kp_final[i] = -1;
        return 1;
    }
    return proj_fits(n) ? ORBX_OK : ORBX_EINVAL;
}

// Host arrays several problems share (a frame searched with several query
// sets) go up once: offsets by (pointer, bytes).
struct Dedup {
    struct E { const void *p; size_t bytes, off; };
    std::vector<E> v;
    size_t add(Layout &L, const void *p, size_t bytes, bool &fresh) {
        for (const E &e : v)
            if (e.p == p && e.bytes == bytes) { fresh = false; return e.off; }
        fresh = true;
        v.push_back({p, bytes, L.add(bytes)});
        return v.back().off;
    }
};

// Runs the problems (all of one variant) in one pair of launches.
// ORBX_CALL_TIMING=1: a synchronous call's host phases (checks, staging,
// enqueue, wait, readback) in microseconds on stderr (diagnostics).
struct CallClock {
    bool on;
    std::chrono::steady_clock::time_point t0;
    double us[6] = {};
    int n = 0;
    CallClock() : on(std::getenv("ORBX_CALL_TIMING") != nullptr), t0(std::chrono::steady_clock::now()) {}
    void mark() {
        if (!on || n >= 6) return;
        const auto t = std::chrono::steady_clock::now();
        us[n++] = std::chrono::duration<double, std::micro>(t - t0).count();
        t0 = t;
    }
    void print(const char *what) const {
        if (!on) return;
        std::fprintf(stderr, "orbx %s us:", what);
        for (int i = 0; i < n; ++i) std::fprintf(stderr, " %.1f", us[i]);
        std::fprintf(stderr, "\n");
    }
};

int proj_run(int device, int variant, orbx_proj_problem *P, int np, int th_dist, float nnratio, int check_ori) {
    if (np < 0 || (np && !P)) return ORBX_EINVAL;
    CallClock clk;   // (ORBX_CALL_TIMING: checks / staging / enqueue / wait / readback)
    std::vector<int> live;
    for (int k = 0; k < np; ++k) {
        const int rc = proj_check(variant, &P[k].frame, P[k].queries, P[k].qdesc, P[k].nq, th_dist, P[k].q_idx,
                                  P[k].q_dist, P[k].kp_final, &P[k].nmatches);
        if (rc < 0) return rc;
        if (rc == 0) live.push_back(k);
    }
    if (live.empty()) return ORBX_OK;
    if (hipSetDevice(device) != hipSuccess) return ORBX_ENODEV;
    clk.mark();
    const bool fuse = variant == ORBX_PROJ_FUSE || variant == ORBX_PROJ_FUSE_SIM3;
    const int nl = (int)live.size();
    int64_t nq_tot = 0;
    for (int k : live) nq_tot += P[k].nq;
    CallWs &ws = call_ws(device);
    std::lock_guard<std::mutex> lock(ws.mu);
    // candidate lists of all queries share one pool; its size is learnt: a
    // call that overflows it reports the total it needed and runs again
    int64_t pool = fuse ? 1 : std::max<int64_t>({ws.proj_pool, 64 * nq_tot, 1 << 16});
    static const bool dbg_stats = std::getenv("ORBX_PROJ_STATS") != nullptr;
    for (int attempt = 0; attempt < 2; ++attempt) {
        Layout L;   // inputs, then outputs, then device-only scratch
        Dedup dd;
        struct Off { size_t k, d, ur, ms, isg, q, qd, qi, qdist, kf, nm, top, len, base, hard, und; int nlev, hard_cap; };
        std::vector<Off> o(nl);
        std::vector<bool> up(5 * nl);
        for (int t = 0; t < nl; ++t) {
            const orbx_proj_problem &pr = P[live[t]];
            const orbx_match_frame *F = &pr.frame;
            const int n = F->n;
            bool f;
            o[t].nlev = F->inv_sigma2 ? std::max(F->nlevels, 0) : 0;
            o[t].k = dd.add(L, F->keys, sizeof(orbx_keypoint) * n, f); up[5 * t] = f;
            o[t].d = dd.add(L, F->desc, 32 * (size_t)n, f); up[5 * t + 1] = f;
            o[t].ur = F->uright ? dd.add(L, F->uright, 4 * (size_t)n, f) : 0; up[5 * t + 2] = F->uright && f;
            o[t].ms = F->mp_state ? dd.add(L, F->mp_state, (size_t)n, f) : 0; up[5 * t + 3] = F->mp_state && f;
            o[t].isg = o[t].nlev ? dd.add(L, F->inv_sigma2, 4 * (size_t)o[t].nlev, f) : 0; up[5 * t + 4] = o[t].nlev && f;
            o[t].q = L.add(sizeof(orbx_proj_query) * pr.nq);
            o[t].qd = L.add(32 * (size_t)pr.nq);
        }
        const size_t o_pa = L.add(sizeof(ProjBufs) * nl);
        // pool_top, then hard_cnt per problem, then the HostTail counter: zeros from the host
        const size_t o_cnt = L.add(16 + 8 * (size_t)nl);
        const size_t in_bytes = L.size;
        for (int t = 0; t < nl; ++t) {
            const int n = P[live[t]].frame.n, nq = P[live[t]].nq;
            o[t].qi = L.add(4 * (size_t)nq); o[t].qdist = L.add(4 * (size_t)nq);
            o[t].kf = L.add(4 * (size_t)n); o[t].nm = L.add(4);
        }
        const size_t out_end = L.size;
        for (int t = 0; t < nl; ++t) {
            const int nq = P[live[t]].nq;
            o[t].hard_cap = 4 * nq + 4096;
            o[t].top = L.add(16 * (size_t)nq); o[t].len = L.add(4 * (size_t)nq); o[t].base = L.add(4 * (size_t)nq);
            o[t].hard = L.add(8 * (size_t)o[t].hard_cap); o[t].und = L.add((size_t)nq);
        }
        const size_t o_pool = L.add(4 * (size_t)pool), o_stats = L.add(64);
        int rc = ws_reserve(ws, L.size);
        if (rc) return rc;
        uint8_t *D = ws.dev;
        std::vector<ProjBufs> hb(nl);
        for (int t = 0; t < nl; ++t) {
            const orbx_proj_problem &pr = P[live[t]];
            const orbx_match_frame *F = &pr.frame;
            const int n = F->n, nq = pr.nq;
            if (up[5 * t]) put(ws, o[t].k, F->keys, sizeof(orbx_keypoint) * n);
            if (up[5 * t + 1]) put(ws, o[t].d, F->desc, 32 * (size_t)n);
            if (up[5 * t + 2]) put(ws, o[t].ur, F->uright, 4 * (size_t)n);
            if (up[5 * t + 3]) put(ws, o[t].ms, F->mp_state, (size_t)n);
            if (up[5 * t + 4]) put(ws, o[t].isg, F->inv_sigma2, 4 * (size_t)o[t].nlev);
            put(ws, o[t].q, pr.queries, sizeof(orbx_proj_query) * nq);
            put(ws, o[t].qd, pr.qdesc, 32 * (size_t)nq);
            ProjBufs &a = hb[t];
            a = ProjBufs{};
            a.keys = at<orbx_keypoint>(D, o[t].k); a.desc = D + o[t].d;
            a.uright = F->uright ? at<float>(D, o[t].ur) : nullptr;
            a.mp_state = F->mp_state ? D + o[t].ms : nullptr;
            a.inv_sigma2 = o[t].nlev ? at<float>(D, o[t].isg) : nullptr;
            a.n = n; a.nlevels = o[t].nlev;
            a.min_x = F->min_x; a.max_x = F->max_x; a.min_y = F->min_y; a.max_y = F->max_y;
            a.q = at<orbx_proj_query>(D, o[t].q); a.qdesc = D + o[t].qd; a.nq = nq;
            a.variant = variant; a.th_dist = th_dist; a.nnratio = nnratio; a.check_ori = check_ori;
            a.q_idx = at<int32_t>(D, o[t].qi); a.q_dist = at<int32_t>(D, o[t].qdist);
            a.kp_final = at<int32_t>(D, o[t].kf); a.nmatches = at<int32_t>(D, o[t].nm);
            a.qtop = at<uint32_t>(D, o[t].top); a.qlen = at<int32_t>(D, o[t].len); a.qbase = at<int32_t>(D, o[t].base);
            a.pool = at<uint32_t>(D, o_pool); a.pool_cap = pool;
            a.pool_top = at<unsigned long long>(D, o_cnt); a.hard_cnt = at<uint32_t>(D, o_cnt + 8 + 8 * (size_t)t);
            a.hard = at<uint2>(D, o[t].hard); a.hard_cap = o[t].hard_cap; a.und = D + o[t].und;
            a.stats = dbg_stats && t == 0 ? at<int32_t>(D, o_stats) : nullptr;
            a.nblk = proj_blocks(nq);
        }
        put(ws, o_pa, hb.data(), sizeof(ProjBufs) * nl);
        std::memset(ws.host + o_cnt, 0, 16 + 8 * (size_t)nl);
        clk.mark();
        if (hipMemcpyAsync(D, ws.host, in_bytes, hipMemcpyHostToDevice, ws.st) != hipSuccess) return ORBX_EIO;
        // Outputs: one copy whose completion the host polls (ORBX_PROJ_TAIL=2,
        // the default).  The replay's workgroup writing them into pinned
        // memory itself (1) measured 7-10 us slower a call, the copy waited
        // for by a stream synchronisation (0) 1-3 us (profiles/r05_ab_proj_call.txt).
        HostTail tail{};
        static const int tail_mode = std::getenv("ORBX_PROJ_TAIL") ? std::atoi(std::getenv("ORBX_PROJ_TAIL")) : 2;
        if (tail_mode == 1)
            ws_tail(ws, o_cnt, out_end - o_cnt, at<uint32_t>(D, o_cnt + 8 + 8 * (size_t)nl),
                    proj_tail_blocks(hb.data(), nl), tail);
        if (launch_proj(hb.data(), at<ProjBufs>(D, o_pa), nl, tail, ws.st) != hipSuccess) return ORBX_EIO;
        clk.mark();
        if (tail_mode == 1 ? ws_wait(ws, tail, o_cnt, out_end - o_cnt)
                           : tail_mode == 2 ? ws_copy_spin(ws, o_cnt, out_end - o_cnt)
                                            : ws_copy_sync(ws, o_cnt, out_end - o_cnt))
            return ORBX_EIO;
        clk.mark();
        unsigned long long used = 0;
        get(ws, o_cnt, &used, 8);
        if (dbg_stats) {
            int32_t st2[6] = {};
            if (hipMemcpy(st2, D + o_stats, sizeof(st2), hipMemcpyDeviceToHost) == hipSuccess)
                std::fprintf(stderr, "orbx proj: variant %d problems %d rounds %d in-order %d pool %llu | 10ns: init %d rounds %d end %d\n",
                             variant, nl, st2[0], st2[1], used, st2[2], st2[3], st2[5]);
        }
        if (!fuse) ws.proj_pool = std::max<int64_t>(ws.proj_pool, (int64_t)used);
        if (!fuse && (int64_t)used > pool) {
            if (used > (unsigned long long)INT32_MAX) return ORBX_ENOMEM;
            pool = (int64_t)used;
            continue;
        }
        for (int t = 0; t < nl; ++t) {
            orbx_proj_problem &pr = P[live[t]];
            get(ws, o[t].qi, pr.q_idx, 4 * (size_t)pr.nq);
            get(ws, o[t].qdist, pr.q_dist, 4 * (size_t)pr.nq);
            get(ws, o[t].kf, pr.kp_final, 4 * (size_t)pr.frame.n);
            get(ws, o[t].nm, &pr.nmatches, 4);
        }
        clk.mark();
        clk.print("proj");
        return ORBX_OK;
    }
    return ORBX_EIO;
}

}  // namespace

int orbx_search_by_projection(int device, int variant, const orbx_match_frame *F, const orbx_proj_query *queries,
                              const uint8_t *qdesc, int nq, int th_dist, float nnratio, int check_ori,
                              int32_t *q_idx, int32_t *q_dist, int32_t *kp_final, int *nmatches) {
    if (!F || !nmatches) return ORBX_EINVAL;
    orbx_proj_problem pr{};
    pr.frame = *F;
    pr.queries = queries; pr.qdesc = qdesc; pr.nq = nq;
    pr.q_idx = q_idx; pr.q_dist = q_dist; pr.kp_final = kp_final;
    const int rc = proj_run(device, variant, &pr, 1, th_dist, nnratio, check_ori);
    *nmatches = rc == ORBX_OK ? pr.nmatches : 0;
    return rc;
}

int orbx_search_by_projection_batch(int device, int variant, orbx_proj_problem *problems, int nproblems, int th_dist,
                                    float nnratio, int check_ori) {
    return proj_run(device, variant, problems, nproblems, th_dist, nnratio, check_ori);
}

namespace {

// Checks one vocabulary-node problem; 1 = nothing to search (outputs filled).
int bow_check(int variant, const orbx_bow_side *A, const orbx_bow_side *B, const float *tri, int nlevels,
              int32_t *match_a, int32_t *match_b, int *nmatches) {
    if (!A || !B || !nmatches || variant < ORBX_BOW_KF_FRAME || variant > ORBX_BOW_TRIANGULATION) return ORBX_EINVAL;
    if (A->n < 0 || B->n < 0 || A->nnodes < 0 || B->nnodes < 0 || (A->n && !match_a) || (B->n && !match_b))
        return ORBX_EINVAL;
    if (variant == ORBX_BOW_TRIANGULATION && (!tri || nlevels <= 0 || nlevels > kMaxLevels)) return ORBX_EINVAL;
    for (const orbx_bow_side *S : {A, B}) {
        if (S->n && (!S->keys || !S->desc || !S->flags)) return ORBX_EINVAL;
        if (S->nnodes && (!S->node_ids || !S->node_offsets || !S->node_features)) return ORBX_EINVAL;
        for (int k = 0; k < S->nnodes; ++k) {   // ascending ids, sane offsets, indices in range
            if (k > 0 && S->node_ids[k] <= S->node_ids[k - 1]) return ORBX_EINVAL;
            if (S->node_offsets[k + 1] < S->node_offsets[k]) return ORBX_EINVAL;
        }
        const int nf = S->nnodes ? S->node_offsets[S->nnodes] : 0;
        if (S->nnodes && S->node_offsets[0] != 0) return ORBX_EINVAL;
        for (int k = 0; k < nf; ++k)
            if (S->node_features[k] < 0 || S->node_features[k] >= S->n) return ORBX_EINVAL;
    }
    for (int k = 0; k < B->nnodes; ++k)
        if (B->node_offsets[k + 1] - B->node_offsets[k] > kBowNodeCap) return ORBX_EINVAL;
    *nmatches = 0;
    for (int i = 0; i < A->n; ++i) match_a[i] = -1;
    for (int i = 0; i < B->n; ++i) match_b[i] = -1;
    return (A->n == 0 || B->n == 0 || A->nnodes == 0 || B->nnodes == 0) ? 1 : ORBX_OK;
}

// Diagnostics of the calling thread's last host call (orbx_debug_counter).
struct DebugCounters {
    int64_t bow_repairs = 0;   // SearchByBoW features that took the in-order repair pass (orbx_bow.hip)
};
thread_local DebugCounters g_debug;

int bow_run(int device, int variant, orbx_bow_problem *P, int np, float nnratio, int check_ori, int nlevels) {
    g_debug.bow_repairs = 0;
    if (np < 0 || (np && !P)) return ORBX_EINVAL;
    CallClock clk;
    std::vector<int> live;
    for (int k = 0; k < np; ++k) {
        const int rc = bow_check(variant, &P[k].a, &P[k].b, P[k].tri, nlevels, P[k].match_a, P[k].match_b,
                                 &P[k].nmatches);
        if (rc < 0) return rc;
        if (rc == 0) live.push_back(k);
    }
    if (live.empty()) return ORBX_OK;
    if (hipSetDevice(device) != hipSuccess) return ORBX_ENODEV;
    clk.mark();   // checks
    const int nl = (int)live.size();
    const int ntri = variant == ORBX_BOW_TRIANGULATION ? 11 + 2 * nlevels : 0;
    Layout L;
    Dedup dd;
    struct Off { size_t side[2][7]; size_t tri, span, ma, mb, cnt, bin; };
    std::vector<Off> o(nl);
    std::vector<uint8_t> up(14 * nl);
    // the keypoints go up whole for triangulation only; the SearchByBoW
    // variants read just their angles (4 of 28 bytes: a third of the call's
    // upload)
    const bool whole_keys = variant == ORBX_BOW_TRIANGULATION;
    for (int t = 0; t < nl; ++t) {
        const orbx_bow_problem &pr = P[live[t]];
        for (int k = 0; k < 2; ++k) {
            const orbx_bow_side *S = k ? &pr.b : &pr.a;
            const int nf = S->node_offsets[S->nnodes];
            bool f;
            uint8_t *u = &up[14 * t + 7 * k];
            o[t].side[k][0] = 0; u[0] = 0;
            if (whole_keys) { o[t].side[k][0] = dd.add(L, S->keys, sizeof(orbx_keypoint) * S->n, f); u[0] = f; }
            o[t].side[k][1] = dd.add(L, S->desc, 32 * (size_t)S->n, f); u[1] = f;
            o[t].side[k][2] = dd.add(L, S->flags, (size_t)S->n, f); u[2] = f;
            o[t].side[k][3] = dd.add(L, S->node_ids, 4 * (size_t)S->nnodes, f); u[3] = f;
            o[t].side[k][4] = dd.add(L, S->node_offsets, 4 * (size_t)(S->nnodes + 1), f); u[4] = f;
            o[t].side[k][5] = dd.add(L, S->node_features, 4 * (size_t)std::max(nf, 1), f); u[5] = f;
            o[t].side[k][6] = dd.add(L, S->keys, 4 * (size_t)std::max(S->n, 1), f); u[6] = f;   // (angles)
        }
        o[t].tri = ntri ? L.add(4 * (size_t)ntri) : 0;
        o[t].span = L.add(sizeof(int4) * (size_t)std::max(pr.a.nnodes, 1));
    }
    const size_t o_pa = L.add(sizeof(BowBufs) * nl);
    for (int t = 0; t < nl; ++t) {   // match arrays start as -1 (host copies), counters zeroed on the device
        o[t].ma = L.add(4 * (size_t)P[live[t]].a.n);
        o[t].mb = L.add(4 * (size_t)P[live[t]].b.n);
    }
    const size_t in_bytes = L.size;
    for (int t = 0; t < nl; ++t) o[t].cnt = L.add(4 * 34);   // hist[32] + counts[2]
    const size_t o_done = L.add(16);   // k_bow_finish's workgroup counter (HostTail)
    const size_t cnt_end = L.size;
    for (int t = 0; t < nl; ++t) o[t].bin = L.add((size_t)P[live[t]].a.n);
    int nparts = 0;   // k_bow_match's workgroups per problem (4 side-A nodes each)
    for (int t = 0; t < nl; ++t) nparts = std::max(nparts, (P[live[t]].a.nnodes + 3) / 4);
    const size_t o_part = L.add(4 * 32 * (size_t)nparts * nl);
    CallWs &ws = call_ws(device);
    std::lock_guard<std::mutex> lock(ws.mu);
    int rc = ws_reserve(ws, L.size);
    if (rc) return rc;
    uint8_t *D = ws.dev;
    std::vector<BowBufs> hb(nl);
    for (int t = 0; t < nl; ++t) {
        const orbx_bow_problem &pr = P[live[t]];
        BowBufs &a = hb[t];
        a = BowBufs{};
        for (int k = 0; k < 2; ++k) {
            const orbx_bow_side *S = k ? &pr.b : &pr.a;
            const int nf = S->node_offsets[S->nnodes];
            const size_t *so = o[t].side[k];
            const uint8_t *u = &up[14 * t + 7 * k];
            if (u[0]) put(ws, so[0], S->keys, sizeof(orbx_keypoint) * S->n);
            if (u[6]) {
                float *ang = at<float>(ws.host, so[6]);
                for (int i = 0; i < S->n; ++i) ang[i] = S->keys[i].angle;
            }
            if (u[1]) put(ws, so[1], S->desc, 32 * (size_t)S->n);
            if (u[2]) put(ws, so[2], S->flags, (size_t)S->n);
            if (u[3]) put(ws, so[3], S->node_ids, 4 * (size_t)S->nnodes);
            if (u[4]) put(ws, so[4], S->node_offsets, 4 * (size_t)(S->nnodes + 1));
            if (u[5]) put(ws, so[5], S->node_features, 4 * (size_t)nf);
            BowSideDev &d = k ? a.B : a.A;
            d = BowSideDev{whole_keys ? at<orbx_keypoint>(D, so[0]) : nullptr, D + so[1], D + so[2], S->n,
                           at<uint32_t>(D, so[3]), at<int32_t>(D, so[4]), at<int32_t>(D, so[5]), S->nnodes,
                           at<float>(D, so[6])};
        }
        if (ntri) put(ws, o[t].tri, pr.tri, 4 * (size_t)ntri);
        {   // merge join of the ascending node ids: each A node's features and its B node's
            int4 *sp = at<int4>(ws.host, o[t].span);
            const orbx_bow_side &A = pr.a, &Bs = pr.b;
            int j = 0;
            for (int i = 0; i < A.nnodes; ++i) {
                const uint32_t id = A.node_ids[i];
                while (j < Bs.nnodes && Bs.node_ids[j] < id) ++j;
                const bool hit = j < Bs.nnodes && Bs.node_ids[j] == id;
                sp[i] = make_int4(A.node_offsets[i], A.node_offsets[i + 1], hit ? Bs.node_offsets[j] : 0,
                                  hit ? Bs.node_offsets[j + 1] : 0);
            }
            a.span = at<int4>(D, o[t].span);
        }
        put(ws, o[t].ma, pr.match_a, 4 * (size_t)pr.a.n);
        put(ws, o[t].mb, pr.match_b, 4 * (size_t)pr.b.n);
        a.variant = variant; a.nnratio = nnratio; a.check_ori = check_ori;
        a.tri = ntri ? at<float>(D, o[t].tri) : nullptr;
        a.ex = ntri ? pr.tri[9] : 0.f; a.ey = ntri ? pr.tri[10] : 0.f;
        a.nlevels = nlevels;
        a.match_a = at<int32_t>(D, o[t].ma); a.match_b = at<int32_t>(D, o[t].mb); a.bin_a = at<int8_t>(D, o[t].bin);
        a.hist = at<int32_t>(D, o[t].cnt); a.counts = at<int32_t>(D, o[t].cnt) + 32;
        a.part = at<int32_t>(D, o_part) + 32 * (size_t)nparts * t; a.nparts = nparts;
    }
    static const bool dbg_clk = std::getenv("ORBX_BOW_CLOCKS") != nullptr;   // diagnostic
    struct DbgClk {   // this call's clock buffer, on the call's device, freed when the call returns
        long long *p = nullptr;
        ~DbgClk() { if (p) (void)hipFree(p); }
    } dclk;
    if (dbg_clk && nl == 1 && hipMalloc(reinterpret_cast<void **>(&dclk.p), 8 * sizeof(long long)) == hipSuccess) {
        const long long init[8] = {INT64_MAX, 0, 0, 0, 0, 0, 0, 0};
        if (hipMemcpy(dclk.p, init, sizeof(init), hipMemcpyHostToDevice) == hipSuccess) hb[0].clk = dclk.p;
    }
    put(ws, o_pa, hb.data(), sizeof(BowBufs) * nl);
    std::memset(ws.host + in_bytes, 0, cnt_end - in_bytes);   // the counters go up as zeros with the inputs
    clk.mark();   // layout + staging copies
    if (hipMemcpyAsync(D, ws.host, cnt_end, hipMemcpyHostToDevice, ws.st) != hipSuccess) return ORBX_EIO;
    const size_t o_out = o[0].ma;   // match arrays and counters are one contiguous run
    HostTail tail{};
    // 1: the match kernel's last workgroup runs the rotation pass and copies
    // the outputs into pinned memory (one launch); 2: match + finish launches,
    // then one copy whose completion the host polls
    static const int tail_mode = std::getenv("ORBX_BOW_TAIL") ? std::atoi(std::getenv("ORBX_BOW_TAIL")) : 1;
    if (tail_mode == 1)
        ws_tail(ws, o_out, cnt_end - o_out, at<uint32_t>(D, o_done), bow_tail_blocks(hb.data(), nl), tail);
    if (launch_bow(hb.data(), at<BowBufs>(D, o_pa), nl, tail, ws.st) != hipSuccess) return ORBX_EIO;
    clk.mark();   // enqueue
    if (tail_mode == 1 ? ws_wait(ws, tail, o_out, cnt_end - o_out) : ws_copy_spin(ws, o_out, cnt_end - o_out))
        return ORBX_EIO;
    clk.mark();   // wait
    for (int t = 0; t < nl; ++t) {
        orbx_bow_problem &pr = P[live[t]];
        get(ws, o[t].ma, pr.match_a, 4 * (size_t)pr.a.n);
        get(ws, o[t].mb, pr.match_b, 4 * (size_t)pr.b.n);
        int32_t counts[2], repairs = 0;
        get(ws, o[t].cnt + 4 * 32, counts, sizeof(counts));
        get(ws, o[t].cnt + 4 * 31, &repairs, sizeof(repairs));
        pr.nmatches = counts[1];
        g_debug.bow_repairs += repairs;
    }
    clk.mark();   // readback
    clk.print("bow");
    if (hb[0].clk) {
        long long c[8];
        if (hipMemcpy(c, hb[0].clk, sizeof(c), hipMemcpyDeviceToHost) == hipSuccess)   // 100 MHz ticks
            std::fprintf(stderr, "orbx bow clocks us: matched %.2f elected %.2f finished %.2f copied %.2f longest wg %.2f\n",
                         (c[1] - c[0]) / 100.0, (c[2] - c[0]) / 100.0, (c[3] - c[0]) / 100.0, (c[4] - c[0]) / 100.0,
                         c[5] / 100.0);
    }
    return ORBX_OK;
}

}  // namespace

int orbx_search_by_bow(int device, int variant, const orbx_bow_side *A, const orbx_bow_side *B, float nnratio,
                       int check_ori, const float *tri, int nlevels, int32_t *match_a, int32_t *match_b,
                       int *nmatches) {
    if (!A || !B || !nmatches) return ORBX_EINVAL;
    orbx_bow_problem pr{};
    pr.a = *A; pr.b = *B; pr.tri = tri; pr.match_a = match_a; pr.match_b = match_b;
    const int rc = bow_run(device, variant, &pr, 1, nnratio, check_ori, nlevels);
    *nmatches = rc == ORBX_OK ? pr.nmatches : 0;
    return rc;
}

int orbx_search_by_bow_batch(int device, int variant, orbx_bow_problem *problems, int nproblems, float nnratio,
                             int check_ori, int nlevels) {
    return bow_run(device, variant, problems, nproblems, nnratio, check_ori, nlevels);
}

int orbx_debug_counter(const char *name, int64_t *value) {
    if (!name || !value) return ORBX_EINVAL;
    if (!std::strcmp(name, "bow_repairs")) { *value = g_debug.bow_repairs; return ORBX_OK; }
    return ORBX_EINVAL;
}

int orbx_rotation_filter(const orbx_keypoint *ka, const orbx_keypoint *kb, int32_t *match_a, int na,
                         const uint8_t *exclude, int *nmatches) {
    if (na < 0 || !nmatches || (na && (!ka || !kb || !match_a))) return ORBX_EINVAL;
    constexpr int kHist = 30;
    std::vector<int> bins(na, -1);
    int hist[kHist] = {};
    const float factor = 1.0f / kHist;
    for (int i = 0; i < na; ++i) {
        if (match_a[i] < 0) continue;
        if (exclude && exclude[i]) { match_a[i] = -1; continue; }
        float rot = ka[i].angle - kb[match_a[i]].angle;
        if (rot < 0.0f) rot += 360.0f;
        int bin = (int)std::round(rot * factor);
        if (bin == kHist) bin = 0;
        if (bin < 0 || bin >= kHist) return ORBX_EINVAL;   // angles outside [0, 360)
        bins[i] = bin;
        ++hist[bin];
    }
    // ComputeThreeMaxima (ORBmatcher.cc:1603-1644)
    int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
    for (int b = 0; b < kHist; ++b) {
        const int sz = hist[b];
        if (sz > max1) { max3 = max2; max2 = max1; max1 = sz; ind3 = ind2; ind2 = ind1; ind1 = b; }
        else if (sz > max2) { max3 = max2; max2 = sz; ind3 = ind2; ind2 = b; }
        else if (sz > max3) { max3 = sz; ind3 = b; }
    }
    if (max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
    else if (max3 < 0.1f * (float)max1) { ind3 = -1; }
    int kept = 0;
    for (int i = 0; i < na; ++i) {
        if (match_a[i] < 0) continue;
        if (bins[i] != ind1 && bins[i] != ind2 && bins[i] != ind3) { match_a[i] = -1; continue; }
        ++kept;
    }
    *nmatches = kept;
    return ORBX_OK;
}

int orbx_search_by_sim3(int device, const orbx_match_frame *kf1, const orbx_match_frame *kf2,
                        const orbx_proj_query *q1, const uint8_t *qdesc1, const orbx_proj_query *q2,
                        const uint8_t *qdesc2, int th_dist, int32_t *matches12, int *nfound) {
    if (!kf1 || !kf2 || !nfound || kf1->n < 0 || kf2->n < 0 || (kf1->n && !matches12)) return ORBX_EINVAL;
    const int n1 = kf1->n, n2 = kf2->n;
    std::vector<int32_t> m1(n1), d1(n1), m2(n2), d2(n2), f1(n1), f2(n2);
    // pKF1's points into pKF2 and pKF2's into pKF1 (ORBmatcher.cc:1147-1219,
    // 1222-1294), one batch of two problems
    orbx_proj_problem pr[2] = {};
    pr[0].frame = *kf2; pr[0].queries = q1; pr[0].qdesc = qdesc1; pr[0].nq = n1;
    pr[0].q_idx = m1.data(); pr[0].q_dist = d1.data(); pr[0].kp_final = f2.data();
    pr[1].frame = *kf1; pr[1].queries = q2; pr[1].qdesc = qdesc2; pr[1].nq = n2;
    pr[1].q_idx = m2.data(); pr[1].q_dist = d2.data(); pr[1].kp_final = f1.data();
    const int rc = proj_run(device, ORBX_PROJ_FUSE_SIM3, pr, 2, th_dist, 1.0f, 0);
    if (rc) return rc;
    // agreement check (:1297-1315)
    int found = 0;
    for (int i1 = 0; i1 < n1; ++i1) {
        const int idx2 = m1[i1];
        matches12[i1] = -1;
        if (idx2 >= 0 && idx2 < n2 && m2[idx2] == i1) { matches12[i1] = idx2; ++found; }
    }
    *nfound = found;
    return ORBX_OK;
}

int orbx_debug_trig(int device, const float *angles, float *s, float *c, int n, const float *ys, const float *xs,
                    float *atan_deg, int m) {
    if (n < 0 || m < 0) return ORBX_EINVAL;
    if (hipSetDevice(device) != hipSuccess) return ORBX_ENODEV;
    float *da = nullptr, *ds = nullptr, *dc = nullptr, *dy = nullptr, *dx = nullptr, *dt = nullptr;
    const size_t nn = std::max(n, 1), mm = std::max(m, 1);
    int rc = ORBX_OK;
    if (dalloc(&da, nn) || dalloc(&ds, nn) || dalloc(&dc, nn) || dalloc(&dy, mm) || dalloc(&dx, mm) || dalloc(&dt, mm))
        rc = ORBX_ENOMEM;
    if (!rc && n && hipMemcpy(da, angles, 4 * (size_t)n, hipMemcpyHostToDevice) != hipSuccess) rc = ORBX_EIO;
    if (!rc && m && (hipMemcpy(dy, ys, 4 * (size_t)m, hipMemcpyHostToDevice) != hipSuccess ||
                     hipMemcpy(dx, xs, 4 * (size_t)m, hipMemcpyHostToDevice) != hipSuccess))
        rc = ORBX_EIO;
    if (!rc && (launch_trig_check(da, ds, dc, dt, dy, dx, n, m, nullptr) != hipSuccess ||
                hipDeviceSynchronize() != hipSuccess))
        rc = ORBX_EIO;
    if (!rc && n && (hipMemcpy(s, ds, 4 * (size_t)n, hipMemcpyDeviceToHost) != hipSuccess ||
                     hipMemcpy(c, dc, 4 * (size_t)n, hipMemcpyDeviceToHost) != hipSuccess))
        rc = ORBX_EIO;
    if (!rc && m && hipMemcpy(atan_deg, dt, 4 * (size_t)m, hipMemcpyDeviceToHost) != hipSuccess) rc = ORBX_EIO;
    dfree(da); dfree(ds); dfree(dc); dfree(dy); dfree(dx); dfree(dt);
    return rc;
}

}  // extern "C"
