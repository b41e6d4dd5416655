// orbx_kfdb.hip -- KeyFrameDatabase (KeyFrameDatabase.cc:31-236) with its
// two queries, DetectLoopCandidates and DetectRelocalizationCandidates, and
// L1Scoring::score (ScoringObject.cpp:23-66), for SURVEY.md §8 f3.
//
// The reference walks an inverted file (one std::list per word, keyframes in
// add order) to count, per keyframe, the query words it shares, and scores
// the keyframes with the most.  Here the keyframes' BowVectors sit in one
// device arena in add order, and the counting is a brute-force pass: a wave
// per keyframe looks its words up in the query's (sorted, in LDS).  The
// inverted file's visiting order -- which fixes the candidate order -- is
// recovered exactly: a keyframe is first met at its first shared query word,
// and among keyframes first met at the same word, in add order.  So the key
// (rank of that word, add sequence) sorts them as the reference lists them.
// The per-keyframe query state (mnLoopQuery, mnLoopWords, mLoopScore and the
// reloc trio) lives on the device beside the arena, one record per slot, and
// is updated by the counting pass exactly as the walk updates it; the same
// pass lists the keyframes the walk would add to lKFsSharingWords.  The L1
// scores of the retained ones are a second pass (a wave per keyframe; the
// common-word terms are summed in ascending word order, as the reference's
// merge adds them), which also appends the survivors of the score threshold.
// Only those come back to the host, in a fixed-size buffer, with the state of
// the covisible neighbours the accumulation reads (KeyFrameDatabase.cc:151-185
// / 287-318: the covisibility graph is the caller's, through a callback).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <list>
#include <mutex>
#include <set>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "orbx_device.h"
#include "orbx_wave.h"
#include "orbx_ws.h"

namespace orbx {
namespace {

constexpr int kKT = 256;
constexpr int kQLds = 8192;   // query words (and values) staged in LDS; more: read from global
constexpr int kScoreChunk = 1024;   // keyframe words scored per wave step (16 per lane)

struct SlotDev {
    int64_t off;   // first word in the arena
    int32_t n;     // words
    int32_t alive;
};

__device__ inline int find_word(const uint32_t *qw, int nq, uint32_t w) {
    int lo = 0, hi = nq - 1;
    while (lo <= hi) {
        const int mid = (lo + hi) >> 1;
        const uint32_t v = qw[mid];
        if (v == w) return mid;
        if (v < w) lo = mid + 1; else hi = mid - 1;
    }
    return -1;
}

// Per-keyframe query state (KeyFrame.h: mnLoopQuery, mnLoopWords,
// mLoopScore, mnRelocQuery, mnRelocWords, mRelocScore), by slot.
struct KState {
    uint64_t loop_query, reloc_query;
    int32_t loop_words, reloc_words;
    float loop_score, reloc_score;
};

// A keyframe the walk lists (lKFsSharingWords), for the scoring pass.
struct Listed {
    uint32_t first;   // rank of its first shared query word: the walk's order
    int32_t slot;
    float score;
};

struct QueryDev {
    uint64_t qid;
    int reloc;
    int nconn;           // connected keyframes (slots, ascending)
    float min_score;
    int32_t *max_words;  // [0] maxCommonWords over the listed ones, [1] survivors
    int list_cap;        // survivors past list_cap go to over[]
    Listed *over;
    uint32_t stamp;      // this query's number
    int4 *rec;           // per slot, written for the keyframes met: (stamp, words, score bits, query == qid)
};

// ---- the inverted file on the device
// Postings of the keyframes added before the last build, as CSR over word
// ids (csr_off[V + 1], csr_slot[]): a query walks only its words' lists, as
// the reference walks mvInvertedFile.  Keyframes added since (the "delta",
// kept small by rebuilding) are counted by brute force against the query.
// The order inside a list does not matter: a keyframe's count and first
// shared word, and its state update, do not depend on it.

// build: postings per word, then their placement (wave per slot)
__global__ __launch_bounds__(kKT) void k_csr_count(const SlotDev *slots, int nslots, const uint32_t *words,
                                                   uint32_t *counts) {
    const int s = blockIdx.x * (kKT / 64) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (s >= nslots) return;
    const SlotDev sl = slots[s];
    for (int i = lane; i < sl.n; i += 64) atomicAdd(&counts[words[sl.off + i]], 1u);
}

__global__ __launch_bounds__(kKT) void k_csr_fill(const SlotDev *slots, int nslots, const uint32_t *words,
                                                  const uint32_t *off, uint32_t *fill, int32_t *post) {
    const int s = blockIdx.x * (kKT / 64) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (s >= nslots) return;
    const SlotDev sl = slots[s];
    for (int i = lane; i < sl.n; i += 64) {
        const uint32_t w = words[sl.off + i];
        post[off[w] + atomicAdd(&fill[w], 1u)] = s;
    }
}

// Exclusive prefix sum of the posting counts (n = V + 1 words, up to ~1 M for
// ORBvoc), in three launches: tile sums (1024 threads x 4 counts a tile),
// one workgroup scanning the tile sums, then each tile's own scan offset by
// its tile's prefix.  Runs once per rebuild of the inverted file.
constexpr int kScanT = 1024, kScanTile = 4 * kScanT;

// exclusive scan of v over the workgroup; *total = the workgroup's sum
__device__ inline uint32_t block_excl_scan_u32(uint32_t v, uint32_t *total, uint32_t *ws) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t incl = (uint32_t)wave_incl_scan_i32((int)v);
    if (lane == 63) ws[w] = incl;
    __syncthreads();
    uint32_t base = 0, all = 0;
    for (int k = 0; k < kScanT / 64; ++k) {
        const uint32_t t = ws[k];
        base += k < w ? t : 0u;
        all += t;
    }
    __syncthreads();   // (ws reusable)
    *total = all;
    return base + incl - v;
}

__device__ inline uint4 scan_load4(const uint32_t *in, int n, int i) {
    if (i + 3 < n) return *reinterpret_cast<const uint4 *>(in + i);
    return make_uint4(i < n ? in[i] : 0u, i + 1 < n ? in[i + 1] : 0u, i + 2 < n ? in[i + 2] : 0u, 0u);
}

__global__ __launch_bounds__(kScanT) void k_scan_tiles(const uint32_t *in, int n, uint32_t *tsum) {
    __shared__ uint32_t ws[kScanT / 64];
    const uint4 v = scan_load4(in, n, blockIdx.x * kScanTile + 4 * threadIdx.x);
    uint32_t total;
    (void)block_excl_scan_u32(v.x + v.y + v.z + v.w, &total, ws);
    if (threadIdx.x == 0) tsum[blockIdx.x] = total;
}

__global__ __launch_bounds__(kScanT) void k_scan_top(uint32_t *tsum, int nt) {
    __shared__ uint32_t ws[kScanT / 64];
    uint32_t carry = 0;
    for (int b = 0; b < nt; b += kScanT) {
        const int i = b + threadIdx.x;
        const uint32_t v = i < nt ? tsum[i] : 0u;
        uint32_t total;
        const uint32_t ex = block_excl_scan_u32(v, &total, ws);
        if (i < nt) tsum[i] = carry + ex;
        carry += total;
    }
}

__global__ __launch_bounds__(kScanT) void k_scan_apply(const uint32_t *in, int n, const uint32_t *tsum, uint32_t *out) {
    __shared__ uint32_t ws[kScanT / 64];
    const int i = blockIdx.x * kScanTile + 4 * threadIdx.x;
    const uint4 v = scan_load4(in, n, i);
    uint32_t total;
    const uint32_t e0 = tsum[blockIdx.x] + block_excl_scan_u32(v.x + v.y + v.z + v.w, &total, ws);
    const uint32_t e1 = e0 + v.x, e2 = e1 + v.y, e3 = e2 + v.z;
    if (i + 3 < n) {
        *reinterpret_cast<uint4 *>(out + i) = make_uint4(e0, e1, e2, e3);
    } else {
        if (i < n) out[i] = e0;
        if (i + 1 < n) out[i + 1] = e1;
        if (i + 2 < n) out[i + 2] = e2;
    }
}

struct TouchDev {
    const uint32_t *csr_off; const int32_t *csr_slot; uint32_t V;
    int delta0, nslots;          // brute-force slots [delta0, nslots)
    int32_t *qcnt; uint32_t *qfirst;   // per slot, 0 / ~0 between queries
};

// Shared words of a keyframe with the query and the rank of the first one
// (both lists ascend: each lane merges a contiguous run of the keyframe's
// words with the query's, from the run's lower bound).
__device__ inline void count_slot(const SlotDev &sl, const uint32_t *words, const uint32_t *qw, int nq, int lane,
                                  int &cnt, uint32_t &first) {
    cnt = 0;
    first = ~0u;
    if (sl.alive && sl.n > 0) {
        const int per = (sl.n + 63) >> 6;
        const int i0 = min(lane * per, sl.n), i1 = min(i0 + per, sl.n);
        if (i0 < i1) {
            const uint32_t *kw = words + sl.off;
            uint32_t w = kw[i0];
            int lo = 0, hi = nq;   // lower_bound(qw, w)
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (qw[mid] < w) lo = mid + 1; else hi = mid;
            }
            int i = i0, r = lo;
            while (r < nq) {
                const uint32_t q = qw[r];
                while (w < q && ++i < i1) w = kw[i];
                if (i >= i1) break;
                if (w == q) {
                    ++cnt;
                    first = min(first, (uint32_t)r);
                    if (++i >= i1) break;
                    w = kw[i];
                }
                ++r;
            }
        }
    }
    cnt = wave_sum_i32(cnt);
    first = wave_min_u32(first);
}

// Pass 1 (persistent grid, wave per work item): items [0, nq) walk the
// posting list of query word r; items past nq count one delta keyframe.
// The per-slot counts are fire-and-forget atomics (no return value waited on).
__global__ __launch_bounds__(kKT) void k_kfdb_touch(const SlotDev *slots, const uint32_t *words, const uint32_t *qw_g,
                                                    int nq, TouchDev t, int32_t *counters) {
    extern __shared__ uint32_t qs[];
    if (blockIdx.x == 0 && threadIdx.x == 0) {   // the list / score passes' counters (they run after this pass)
        counters[0] = 0;
        counters[1] = 0;
    }
    // (only the delta keyframes' merges read the whole query: staged for them)
    const int items = nq + (t.nslots - t.delta0);
    const bool staged = nq <= kQLds && items > nq;
    if (staged) {
        for (int i = threadIdx.x; i < nq; i += kKT) qs[i] = qw_g[i];
        __syncthreads();
    }
    const uint32_t *qw = staged ? qs : qw_g;
    const int lane = threadIdx.x & 63;
    const int nw = gridDim.x * (kKT / 64);
    for (int it = blockIdx.x * (kKT / 64) + (threadIdx.x >> 6); it < items; it += nw) {
        if (it < nq) {
            const uint32_t w = qw[it];
            if (w >= t.V) continue;
            const uint32_t b = t.csr_off[w], e = t.csr_off[w + 1];
            for (uint32_t i = b + lane; i < e; i += 64) {
                const int s = t.csr_slot[i];
                if (!slots[s].alive) continue;
                atomicMin(&t.qfirst[s], (uint32_t)it);
                atomicAdd(&t.qcnt[s], 1);
            }
        } else {
            const int s = t.delta0 + (it - nq);
            int c;
            uint32_t f;
            count_slot(slots[s], words, qw, nq, lane, c, f);
            if (lane == 0 && c > 0) {
                t.qcnt[s] = c;
                t.qfirst[s] = f;
            }
        }
    }
}

// Pass 2 (thread per slot; the keyframes the query met: count > 0): the walk's state update
// (KeyFrameDatabase.cc:95-119 / 234-251):
//   loop:  not met by this query yet -> connected: words = 1 (it is reset at
//          every meeting and ends at 1); else query = qid, words = count, listed;
//          met before (same query id) -> words += count;
//   reloc: not met -> query = qid, words = count, listed; else words += count.
// Resets the per-slot scratch for the next query.
__global__ __launch_bounds__(kKT) void k_kfdb_list(TouchDev t, const int32_t *conn, QueryDev qd, KState *state,
                                                   int4 *listed) {
    for (int s = blockIdx.x * kKT + threadIdx.x; s < t.nslots; s += gridDim.x * kKT) {
        const int cnt = t.qcnt[s];
        if (cnt == 0) {
            listed[s] = make_int4(0, 0, s, 0);
            continue;
        }
        const uint32_t first = t.qfirst[s];
        t.qcnt[s] = 0;
        t.qfirst[s] = ~0u;
        int lst = 0;
        KState &st = state[s];
        if (!qd.reloc) {
            if (st.loop_query != qd.qid) {
                int lo = 0, hi = qd.nconn - 1;
                bool connected = false;
                while (lo <= hi) {
                    const int mid = (lo + hi) >> 1;
                    if (conn[mid] == s) { connected = true; break; }
                    if (conn[mid] < s) lo = mid + 1; else hi = mid - 1;
                }
                if (connected) {
                    st.loop_words = 1;
                } else {
                    st.loop_query = qd.qid;
                    st.loop_words = cnt;
                    lst = 1;
                }
            } else {
                st.loop_words += cnt;
            }
        } else {
            if (st.reloc_query != qd.qid) {
                st.reloc_query = qd.qid;
                st.reloc_words = cnt;
                lst = 1;
            } else {
                st.reloc_words += cnt;
            }
        }
        if (lst) atomicMax(qd.max_words, cnt);
        listed[s] = make_int4(lst ? cnt : 0, (int)first, s, 0);
        // what the accumulation may read of this keyframe as a neighbour
        qd.rec[s] = qd.reloc ? make_int4((int)qd.stamp, st.reloc_words, __float_as_int(st.reloc_score),
                                         st.reloc_query == qd.qid)
                             : make_int4((int)qd.stamp, st.loop_words, __float_as_int(st.loop_score),
                                         st.loop_query == qd.qid);
    }
}

// Pass 3 (persistent grid, a wave per 64 slots): L1Scoring::score of
// the listed keyframes above minCommonWords = maxCommonWords * 0.8f
// (KeyFrameDatabase.cc:124-149 / 259-284), in double; the score goes to the
// keyframe's state and the keyframes the reference keeps (loop: score >=
// minScore; reloc: all) are appended to the output.
__global__ __launch_bounds__(kKT) void k_kfdb_score(const SlotDev *slots, int n, const int4 *listed,
                                                    const uint32_t *words, const double *values, const uint32_t *qw_g,
                                                    const double *qv_g, int nq, QueryDev qd, KState *state,
                                                    Listed *list) {
    __shared__ double tbuf[kKT / 64][kScoreChunk];   // per wave: a chunk's terms
    extern __shared__ uint32_t qs[];   // the query's words (nq <= kQLds), else read from global
    const bool staged = nq <= kQLds;
    if (staged)
        for (int i = threadIdx.x; i < nq; i += kKT) qs[i] = qw_g[i];
    __syncthreads();
    const uint32_t *qw = staged ? qs : qw_g;
    double *trow = tbuf[threadIdx.x >> 6];
    const int min_words = (int)((float)*qd.max_words * 0.8f);
    const int lane = threadIdx.x & 63;
    const int nw = gridDim.x * (kKT / 64);
    // the wave reads 64 list entries at once and scores the ones above the
    // threshold one after another
    for (int k0 = (blockIdx.x * (kKT / 64) + (threadIdx.x >> 6)) * 64; k0 < n; k0 += nw * 64) {
        const int4 Lk = k0 + lane < n ? listed[k0 + lane] : make_int4(0, 0, 0, 0);
        for (uint64_t pass = __ballot(Lk.x > min_words); pass; pass &= pass - 1) {   // not listed (0) or too few words
            const int j = (int)__builtin_ctzll(pass);
            const int s = __shfl(Lk.z, j), first = __shfl(Lk.y, j);
            const SlotDev sl = slots[s];
            // 1024 words at a time: every lane loads and looks up 16 words at
            // once (branch-free searches in lock step), the common words'
            // terms go to the wave's LDS row in word order, then lane 0 adds
            // them in order
            double acc = 0;
            for (int c0 = 0; c0 < sl.n; c0 += kScoreChunk) {
                uint32_t w[16];
                int pos[16];
#pragma unroll
                for (int u = 0; u < 16; ++u) {
                    const int i = c0 + u * 64 + lane;
                    w[u] = i < sl.n ? words[sl.off + i] : 0u;
                    pos[u] = 0;
                }
                for (int len = nq; len > 1;) {
                    const int half = len >> 1;
#pragma unroll
                    for (int u = 0; u < 16; ++u) pos[u] = qw[pos[u] + half] <= w[u] ? pos[u] + half : pos[u];
                    len -= half;
                }
                int m = 0;   // the common words' terms, compacted in word order
#pragma unroll
                for (int u = 0; u < 16; ++u) {
                    const int i = c0 + u * 64 + lane;
                    const bool hit = i < sl.n && qw[pos[u]] == w[u];
                    const uint64_t hm = __ballot(hit);
                    if (hit) {
                        const double vi = qv_g[pos[u]], wi = values[sl.off + i];
                        const int at = m + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(hm >> 32),
                                                                          __builtin_amdgcn_mbcnt_lo((uint32_t)hm, 0u));
                        trow[at] = __dsub_rn(__dsub_rn(fabs(__dsub_rn(vi, wi)), fabs(vi)), fabs(wi));
                    }
                    m += __popcll(hm);
                }
                wave_lds_fence();
                if (lane == 0) {
                    int q = 0;
                    for (; q + 8 <= m; q += 8) {
                        double x[8];
#pragma unroll
                        for (int u = 0; u < 8; ++u) x[u] = trow[q + u];
#pragma unroll
                        for (int u = 0; u < 8; ++u) acc = __dadd_rn(acc, x[u]);
                    }
                    for (; q < m; ++q) acc = __dadd_rn(acc, trow[q]);
                }
                wave_lds_fence();
            }
            if (lane == 0) {
                const float si = (float)(-acc / 2.0);
                if (qd.reloc) state[s].reloc_score = si; else state[s].loop_score = si;
                qd.rec[s].z = __float_as_int(si);
                if (qd.reloc || si >= qd.min_score) {
                    const int at = atomicAdd(qd.max_words + 1, 1);
                    if (at < qd.list_cap) list[at] = Listed{(uint32_t)first, s, si};
                    else qd.over[at - qd.list_cap] = Listed{(uint32_t)first, s, si};
                }
            }
        }
    }
}

// New slots: a re-added keyframe keeps its query state (the reference's
// KeyFrame object keeps its members), a new one starts at zero.
__global__ void k_kfdb_seed(KState *state, int first, int count, const int32_t *src) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const int p = src[i];
    state[first + i] = p >= 0 ? state[p] : KState{0, 0, 0, 0, 0.f, 0.f};
}

__global__ void k_kfdb_gather(const KState *state, const int32_t *slots, int n, KState *out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = state[slots[i]];
}

}  // namespace
}  // namespace orbx

using namespace orbx;

namespace {
struct Slot {
    uint64_t id;
    int64_t off;
    int n;
    bool alive;
};
}  // namespace

struct orbx_kfdb {
    int device = 0;
    std::mutex mu;
    hipStream_t st = nullptr;
    std::vector<Slot> slots;                      // add order
    std::unordered_map<uint64_t, int> live;       // id -> alive slot
    std::unordered_map<uint64_t, int> last_slot;  // id -> its newest slot (its query state), erased or not
    std::vector<int32_t> seed_src;                // per slot not yet on the device: slot whose state it inherits, or -1
    std::vector<uint32_t> h_words;                // host mirror of the arena (compaction)
    std::vector<double> h_values;
    uint32_t *d_words = nullptr;
    double *d_values = nullptr;
    SlotDev *d_slots = nullptr;
    KState *d_state = nullptr;
    int32_t *d_qcnt = nullptr;   // per-slot query scratch
    uint32_t *d_qfirst = nullptr;
    // the device inverted file over slots [0, csr_ns): postings by word id
    uint32_t *d_csr_off = nullptr, *d_csr_cnt = nullptr, *d_csr_tsum = nullptr;   // (tsum: the scan's tile sums)
    int32_t *d_csr_slot = nullptr;
    uint32_t csr_V = 0;
    int csr_ns = 0;
    int64_t csr_cap_post = 0, csr_cap_V = 0;
    uint32_t max_word = 0;
    // one buffer per database, brought back by one copy per query: the
    // counters (16 B), the first kListCap survivors, the per-slot records
    // (what the last query met, QueryDev::rec); then the survivors past
    // kListCap (rarely copied)
    uint8_t *d_qbuf = nullptr;
    int4 *d_rec = nullptr;
    Listed *d_over = nullptr;
    uint32_t stamp = 0;
    std::unordered_set<uint64_t> loop_qids, reloc_qids;   // query ids used so far
    int64_t cap_words = 0, dev_words = 0;        // arena capacity / words on the device
    int cap_slots = 0, dev_slots = 0;             // slot table capacity / rows on the device
    bool slots_dirty = false;
};

namespace {

constexpr int kListCap = 1024;   // scored keyframes brought back with the first copy
constexpr size_t kQHdr = (16 + sizeof(Listed) * kListCap + 255) & ~size_t(255);   // counters + first survivors

int kfdb_sync(orbx_kfdb *db) {
    // grow-and-upload the arena tail and the slot table; seed new slots' state
    const int64_t need_w = (int64_t)db->h_words.size();
    if (need_w > db->cap_words) {
        const int64_t cap = std::max<int64_t>(need_w * 2, 1 << 16);
        uint32_t *w = nullptr;
        double *v = nullptr;
        if (hipMalloc(reinterpret_cast<void **>(&w), 4 * cap) != hipSuccess ||
            hipMalloc(reinterpret_cast<void **>(&v), 8 * cap) != hipSuccess)
            return ORBX_ENOMEM;
        if (db->dev_words && (hipMemcpyAsync(w, db->d_words, 4 * db->dev_words, hipMemcpyDeviceToDevice, db->st) !=
                                  hipSuccess ||
                              hipMemcpyAsync(v, db->d_values, 8 * db->dev_words, hipMemcpyDeviceToDevice, db->st) !=
                                  hipSuccess))
            return ORBX_EIO;
        (void)hipStreamSynchronize(db->st);
        if (db->d_words) (void)hipFree(db->d_words);
        if (db->d_values) (void)hipFree(db->d_values);
        db->d_words = w;
        db->d_values = v;
        db->cap_words = cap;
    }
    if (need_w > db->dev_words) {
        const int64_t a = db->dev_words, m = need_w - a;
        if (hipMemcpyAsync(db->d_words + a, db->h_words.data() + a, 4 * m, hipMemcpyHostToDevice, db->st) !=
                hipSuccess ||
            hipMemcpyAsync(db->d_values + a, db->h_values.data() + a, 8 * m, hipMemcpyHostToDevice, db->st) !=
                hipSuccess)
            return ORBX_EIO;
        db->dev_words = need_w;
    }
    const int ns = (int)db->slots.size();
    if (ns > db->cap_slots) {
        const int cap = std::max(ns * 2, 1024);
        SlotDev *d = nullptr;
        KState *k = nullptr;
        if (hipMalloc(reinterpret_cast<void **>(&d), sizeof(SlotDev) * cap) != hipSuccess ||
            hipMalloc(reinterpret_cast<void **>(&k), sizeof(KState) * cap) != hipSuccess)
            return ORBX_ENOMEM;
        if (db->dev_slots &&
            hipMemcpyAsync(k, db->d_state, sizeof(KState) * db->dev_slots, hipMemcpyDeviceToDevice, db->st) != hipSuccess)
            return ORBX_EIO;
        (void)hipStreamSynchronize(db->st);
        if (db->d_slots) (void)hipFree(db->d_slots);
        if (db->d_state) (void)hipFree(db->d_state);
        for (void *x : {(void *)db->d_qcnt, (void *)db->d_qfirst, (void *)db->d_qbuf})
            if (x) (void)hipFree(x);
        db->d_slots = d;
        db->d_state = k;
        db->d_qcnt = nullptr;
        db->d_qfirst = nullptr;
        db->d_qbuf = nullptr;
        db->d_rec = nullptr;
        db->d_over = nullptr;
        if (hipMalloc(reinterpret_cast<void **>(&db->d_qbuf), kQHdr + (sizeof(int4) + sizeof(Listed)) * (size_t)cap) !=
                hipSuccess)
            return ORBX_ENOMEM;
        db->d_rec = reinterpret_cast<int4 *>(db->d_qbuf + kQHdr);
        db->d_over = reinterpret_cast<Listed *>(db->d_qbuf + kQHdr + sizeof(int4) * (size_t)cap);
        if (hipMemsetAsync(db->d_rec, 0, sizeof(int4) * (size_t)cap, db->st) != hipSuccess) return ORBX_ENOMEM;
        if (hipMalloc(reinterpret_cast<void **>(&db->d_qcnt), 4 * (size_t)cap) != hipSuccess ||
            hipMalloc(reinterpret_cast<void **>(&db->d_qfirst), 4 * (size_t)cap) != hipSuccess)
            return ORBX_ENOMEM;
        if (hipMemsetAsync(db->d_qcnt, 0, 4 * (size_t)cap, db->st) != hipSuccess ||
            hipMemsetAsync(db->d_qfirst, 0xFF, 4 * (size_t)cap, db->st) != hipSuccess)
            return ORBX_EIO;
        db->cap_slots = cap;
        db->slots_dirty = true;
    }
    if (db->slots_dirty || ns > db->dev_slots) {
        std::vector<SlotDev> t(ns);
        for (int i = 0; i < ns; ++i) t[i] = {db->slots[i].off, db->slots[i].n, db->slots[i].alive ? 1 : 0};
        const int fresh = ns - db->dev_slots;
        if (ns && hipMemcpyAsync(db->d_slots, t.data(), sizeof(SlotDev) * ns, hipMemcpyHostToDevice, db->st) !=
                      hipSuccess)
            return ORBX_EIO;
        int32_t *d_src = nullptr;
        if (fresh > 0) {
            if (hipMalloc(reinterpret_cast<void **>(&d_src), 4 * (size_t)fresh) != hipSuccess) return ORBX_ENOMEM;
            if (hipMemcpyAsync(d_src, db->seed_src.data(), 4 * (size_t)fresh, hipMemcpyHostToDevice, db->st) !=
                hipSuccess)
                return ORBX_EIO;
            hipLaunchKernelGGL(k_kfdb_seed, dim3((fresh + 255) / 256), dim3(256), 0, db->st, db->d_state,
                               db->dev_slots, fresh, d_src);
            if (hipGetLastError() != hipSuccess) return ORBX_EIO;
        }
        (void)hipStreamSynchronize(db->st);   // (t and seed_src are host temporaries)
        if (d_src) (void)hipFree(d_src);
        db->seed_src.clear();
        db->dev_slots = ns;
        db->slots_dirty = false;
    }
    // rebuild the inverted file once the brute-force delta has grown
    if (ns - db->csr_ns > std::max(256, db->csr_ns / 8)) {
        const int64_t V = (int64_t)db->max_word + 1, P = std::max<int64_t>(db->dev_words, 1);
        if (V + 1 > db->csr_cap_V) {
            const int64_t cap = (V + 1) * 2;
            for (uint32_t **x : {&db->d_csr_off, &db->d_csr_cnt, &db->d_csr_tsum})
                if (*x) { (void)hipStreamSynchronize(db->st); (void)hipFree(*x); *x = nullptr; }
            if (hipMalloc(reinterpret_cast<void **>(&db->d_csr_off), 4 * cap) != hipSuccess ||
                hipMalloc(reinterpret_cast<void **>(&db->d_csr_cnt), 4 * cap) != hipSuccess ||
                hipMalloc(reinterpret_cast<void **>(&db->d_csr_tsum), 4 * (cap / kScanTile + 1)) != hipSuccess)
                return ORBX_ENOMEM;
            db->csr_cap_V = cap;
        }
        if (P > db->csr_cap_post) {
            const int64_t cap = P * 2;
            if (db->d_csr_slot) { (void)hipStreamSynchronize(db->st); (void)hipFree(db->d_csr_slot); }
            if (hipMalloc(reinterpret_cast<void **>(&db->d_csr_slot), 4 * cap) != hipSuccess) return ORBX_ENOMEM;
            db->csr_cap_post = cap;
        }
        const dim3 grid((ns + kKT / 64 - 1) / (kKT / 64));
        if (hipMemsetAsync(db->d_csr_cnt, 0, 4 * (size_t)(V + 1), db->st) != hipSuccess) return ORBX_EIO;
        hipLaunchKernelGGL(k_csr_count, grid, dim3(kKT), 0, db->st, db->d_slots, ns, db->d_words, db->d_csr_cnt);
        const int nscan = (int)(V + 1), ntile = (nscan + kScanTile - 1) / kScanTile;
        hipLaunchKernelGGL(k_scan_tiles, dim3(ntile), dim3(kScanT), 0, db->st, db->d_csr_cnt, nscan, db->d_csr_tsum);
        hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(kScanT), 0, db->st, db->d_csr_tsum, ntile);
        hipLaunchKernelGGL(k_scan_apply, dim3(ntile), dim3(kScanT), 0, db->st, db->d_csr_cnt, nscan, db->d_csr_tsum,
                           db->d_csr_off);
        const bool ok = hipMemsetAsync(db->d_csr_cnt, 0, 4 * (size_t)(V + 1), db->st) == hipSuccess;
        if (ok)
            hipLaunchKernelGGL(k_csr_fill, grid, dim3(kKT), 0, db->st, db->d_slots, ns, db->d_words, db->d_csr_off,
                               db->d_csr_cnt, db->d_csr_slot);
        (void)hipStreamSynchronize(db->st);
        if (!ok || hipGetLastError() != hipSuccess) return ORBX_EIO;
        db->csr_ns = ns;
        db->csr_V = (uint32_t)V;
    }
    return ORBX_OK;
}

double l1_host(const uint32_t *w1, const double *v1, int n1, const uint32_t *w2, const double *v2, int n2) {
    int i = 0, j = 0;
    double score = 0;
    while (i < n1 && j < n2) {
        if (w1[i] == w2[j]) {
            score += std::fabs(v1[i] - v2[j]) - std::fabs(v1[i]) - std::fabs(v2[j]);
            ++i;
            ++j;
        } else if (w1[i] < w2[j]) {
            i = (int)(std::lower_bound(w1, w1 + n1, w2[j]) - w1);
        } else {
            j = (int)(std::lower_bound(w2, w2 + n2, w1[i]) - w2);
        }
    }
    return -score / 2.0;
}

bool sorted_unique(const uint32_t *w, int n) {
    for (int i = 1; i < n; ++i)
        if (w[i] <= w[i - 1]) return false;
    return true;
}

int detect(orbx_kfdb *db, bool reloc, uint64_t qid, const uint32_t *words, const double *values, int n,
           const uint64_t *connected, int n_connected, float minScore, orbx_covis_fn covis, void *ctx,
           uint64_t *out, int cap, int *n_out) {
    if (!db || n < 0 || !n_out || (n && (!words || !values)) || !covis || (n_connected > 0 && !connected) ||
        (cap > 0 && !out) || !sorted_unique(words, n))
        return ORBX_EINVAL;
    *n_out = 0;
    // ORBX_KFDB_TIMING: phase times of this query on stderr (diagnostics)
    static const bool timing = std::getenv("ORBX_KFDB_TIMING") != nullptr;
    auto tms = [] { return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    const double t_a = timing ? tms() : 0;
    std::lock_guard<std::mutex> lock(db->mu);
    const int ns = (int)db->slots.size();
    if (n == 0 || ns == 0) return ORBX_OK;
    if (hipSetDevice(db->device) != hipSuccess) return ORBX_ENODEV;
    if (!db->st && hipStreamCreateWithFlags(&db->st, hipStreamNonBlocking) != hipSuccess) return ORBX_EIO;
    int rc = kfdb_sync(db);
    if (rc) return rc;
    // connected keyframes the walk can meet: their alive slots, ascending
    std::vector<int32_t> conn;
    if (!reloc)
        for (int i = 0; i < n_connected; ++i) {
            auto it = db->live.find(connected[i]);
            if (it != db->live.end()) conn.push_back(it->second);
        }
    std::sort(conn.begin(), conn.end());
    conn.erase(std::unique(conn.begin(), conn.end()), conn.end());
    Layout L;
    const size_t o_qw = L.add(4 * (size_t)n), o_qv = L.add(8 * (size_t)n), o_conn = L.add(4 * (conn.size() + 1));
    const size_t in_bytes = L.size;
    const size_t o_lst = L.add(16 * (size_t)ns);                          // the walk's list (device only)
    const size_t o_rb = L.add(kQHdr + sizeof(int4) * (size_t)ns);          // the readback (host only)
    const size_t o_ov = L.add(sizeof(Listed) * (size_t)std::max(ns - kListCap, 0));
    // a keyframe never queried has query id 0 (KeyFrame.cc's initialiser), so
    // a query with id 0 matches every such neighbour, as a repeated id would
    const bool repeated = !(reloc ? db->reloc_qids : db->loop_qids).insert(qid).second || qid == 0;
    if (++db->stamp == 0) ++db->stamp;   // (0: never written)
    CallWs &ws = call_ws(db->device);
    std::lock_guard<std::mutex> wl(ws.mu);
    rc = ws_reserve(ws, L.size);
    if (rc) return rc;
    put(ws, o_qw, words, 4 * (size_t)n);
    put(ws, o_qv, values, 8 * (size_t)n);
    put(ws, o_conn, conn.data(), 4 * conn.size());
    uint8_t *D = ws.dev;
    QueryDev qd;
    qd.qid = qid;
    qd.reloc = reloc;
    qd.nconn = (int)conn.size();
    qd.min_score = minScore;
    qd.max_words = reinterpret_cast<int32_t *>(db->d_qbuf);   // [0] maxCommonWords, [1] kept (zeroed by touch)
    qd.list_cap = kListCap;
    qd.over = db->d_over;
    qd.stamp = db->stamp;
    qd.rec = db->d_rec;
    TouchDev t;
    t.csr_off = db->d_csr_off; t.csr_slot = db->d_csr_slot; t.V = db->csr_ns ? db->csr_V : 0;
    t.delta0 = db->csr_ns; t.nslots = ns;
    t.qcnt = db->d_qcnt; t.qfirst = db->d_qfirst;
    // pass 1: the query words' posting lists + the delta keyframes; pass 2:
    // state update and the walk's list; pass 3: scores above minCommonWords
    const size_t qlds = n <= kQLds ? 4 * (size_t)n : 0;
    const int items = n + (ns - db->csr_ns);
    if (hipStreamSynchronize(db->st) != hipSuccess ||
        hipMemcpyAsync(D, ws.host, in_bytes, hipMemcpyHostToDevice, ws.st) != hipSuccess)
        return ORBX_EIO;
    hipLaunchKernelGGL(k_kfdb_touch, dim3(std::min(1024, (items + 3) / 4)), dim3(kKT), qlds, ws.st, db->d_slots,
                       db->d_words, at<uint32_t>(D, o_qw), n, t, qd.max_words);
    hipLaunchKernelGGL(k_kfdb_list, dim3(std::min(256, (ns + kKT - 1) / kKT)), dim3(kKT), 0, ws.st, t,
                       at<int32_t>(D, o_conn), qd, db->d_state, at<int4>(D, o_lst));
    // few keyframes pass minCommonWords: a small persistent grid, each block
    // with the query words in LDS
    hipLaunchKernelGGL(k_kfdb_score, dim3(std::min(64, (ns + 3) / 4)), dim3(kKT), qlds, ws.st, db->d_slots,
                       ns, at<int4>(D, o_lst), db->d_words, db->d_values, at<uint32_t>(D, o_qw),
                       at<double>(D, o_qv), n, qd, db->d_state, reinterpret_cast<Listed *>(db->d_qbuf + 16));
    // k_kfdb_list clears the per-slot scratch k_kfdb_touch filled; a query that
    // fails in between clears it here, so later queries start from zero counts
    auto fail_scratch = [&]() {
        (void)hipGetLastError();
        (void)hipStreamSynchronize(ws.st);
        // (on the query's own stream: no legacy-stream or device-wide sync that
        // could break another thread's graph capture)
        (void)hipMemsetAsync(db->d_qcnt, 0, sizeof(*db->d_qcnt) * (size_t)ns, ws.st);
        (void)hipMemsetAsync(db->d_qfirst, 0xFF, sizeof(*db->d_qfirst) * (size_t)ns, ws.st);
        (void)hipStreamSynchronize(ws.st);
        return ORBX_EIO;
    };
    if (hipGetLastError() != hipSuccess ||
        hipMemcpyAsync(ws.host + o_rb, db->d_qbuf, kQHdr + sizeof(int4) * (size_t)ns, hipMemcpyDeviceToHost, ws.st) !=
            hipSuccess ||
        hipStreamSynchronize(ws.st) != hipSuccess)
        return fail_scratch();
    const double t_b = timing ? tms() : 0;
    const int4 *rec = at<int4>(ws.host, o_rb + kQHdr);
    int32_t mw[2];
    get(ws, o_rb, mw, 8);
    const int nsc = mw[1];
    if (nsc > kListCap &&
        (hipMemcpyAsync(ws.host + o_ov, db->d_over, sizeof(Listed) * (size_t)(nsc - kListCap), hipMemcpyDeviceToHost,
                        ws.st) != hipSuccess ||
         hipStreamSynchronize(ws.st) != hipSuccess))
        return ORBX_EIO;
    if (nsc == 0) return ORBX_OK;
    // the kept keyframes in the walk's order: (first shared word, add order)
    const Listed *first = at<Listed>(ws.host, o_rb + 16);
    std::vector<Listed> scored(first, first + std::min(nsc, kListCap));
    if (nsc > kListCap)
        scored.insert(scored.end(), at<Listed>(ws.host, o_ov), at<Listed>(ws.host, o_ov) + (nsc - kListCap));
    std::sort(scored.begin(), scored.end(), [](const Listed &a, const Listed &b) {
        return a.first != b.first ? a.first < b.first : a.slot < b.slot;
    });
    const int minCommonWords = mw[0] * 0.8f;
    // covisible neighbours (KeyFrameDatabase.cc:151-185 / 287-318).  The
    // state the accumulation reads came back with the query for every
    // keyframe this query met; one that it did not meet matches the query id
    // only if an earlier query used the same id -- then it is gathered.
    struct NState { bool match; int words; float score; };
    std::vector<uint64_t> nid;
    std::vector<int> nfirst(nsc + 1, 0);
    std::vector<NState> nst;
    std::vector<int32_t> gslot;
    std::vector<int> gpos;
    uint64_t neigh[64];
    for (int i = 0; i < nsc; ++i) {
        const int nn = std::min(covis(ctx, db->slots[scored[i].slot].id, neigh, 10), 10);
        for (int t = 0; t < nn; ++t) {
            auto it = db->last_slot.find(neigh[t]);
            const int sl = it == db->last_slot.end() ? -1 : it->second;   // never in the database: no state
            NState x{false, 0, 0.f};
            if (sl >= 0 && (uint32_t)rec[sl].x == db->stamp) {
                float sc;
                std::memcpy(&sc, &rec[sl].z, 4);
                x = NState{rec[sl].w != 0, rec[sl].y, sc};
            } else if (sl >= 0 && repeated) {
                gslot.push_back(sl);
                gpos.push_back((int)nst.size());
            }
            nid.push_back(neigh[t]);
            nst.push_back(x);
        }
        nfirst[i + 1] = (int)nid.size();
    }
    const double t_c = timing ? tms() : 0;
    if (!gslot.empty()) {
        std::vector<KState> gst(gslot.size());
        Layout G;
        const size_t o_gs = G.add(4 * gslot.size()), o_go = G.add(sizeof(KState) * gslot.size());
        rc = ws_reserve(ws, G.size);
        if (rc) return rc;
        D = ws.dev;
        put(ws, o_gs, gslot.data(), 4 * gslot.size());
        if (hipMemcpyAsync(D + o_gs, ws.host + o_gs, 4 * gslot.size(), hipMemcpyHostToDevice, ws.st) != hipSuccess)
            return ORBX_EIO;
        hipLaunchKernelGGL(k_kfdb_gather, dim3(((int)gslot.size() + 255) / 256), dim3(256), 0, ws.st, db->d_state,
                           at<int32_t>(D, o_gs), (int)gslot.size(), at<KState>(D, o_go));
        if (hipGetLastError() != hipSuccess ||
            hipMemcpyAsync(ws.host + o_go, D + o_go, sizeof(KState) * gslot.size(), hipMemcpyDeviceToHost, ws.st) !=
                hipSuccess ||
            hipStreamSynchronize(ws.st) != hipSuccess)
            return ORBX_EIO;
        get(ws, o_go, gst.data(), sizeof(KState) * gslot.size());
        for (size_t g = 0; g < gslot.size(); ++g) {
            const KState &k = gst[g];
            nst[gpos[g]] = reloc ? NState{k.reloc_query == qid, k.reloc_words, k.reloc_score}
                                 : NState{k.loop_query == qid, k.loop_words, k.loop_score};
        }
    }
    std::vector<std::pair<float, uint64_t>> acc;
    float bestAccScore = reloc ? 0 : minScore;
    for (int i = 0; i < nsc; ++i) {
        const uint64_t kid = db->slots[scored[i].slot].id;
        float bestScore = scored[i].score, accScore = scored[i].score;
        uint64_t best = kid;
        for (int t = nfirst[i]; t < nfirst[i + 1]; ++t) {
            const NState &k2 = nst[t];
            if (!k2.match || (!reloc && k2.words <= minCommonWords)) continue;
            accScore += k2.score;
            if (k2.score > bestScore) { best = nid[t]; bestScore = k2.score; }
        }
        acc.emplace_back(accScore, best);
        if (accScore > bestAccScore) bestAccScore = accScore;
    }
    const float minScoreToRetain = 0.75f * bestAccScore;
    std::set<uint64_t> added;
    int m = 0;
    for (auto &a : acc) {
        if (a.first > minScoreToRetain && !added.count(a.second)) {
            if (m < cap) out[m] = a.second;
            ++m;
            added.insert(a.second);
        }
    }
    *n_out = m;
    if (timing)
        std::fprintf(stderr, "kfdb query us: pre+gpu %.1f covis(%d kept) %.1f post %.1f\n", t_b - t_a, nsc, t_c - t_b,
                     tms() - t_c);
    return m > cap ? ORBX_ERANGE : ORBX_OK;
}

}  // namespace

extern "C" {

int orbx_kfdb_create(int device, orbx_kfdb **out) {
    if (!out) return ORBX_EINVAL;
    orbx_kfdb *db = new orbx_kfdb;
    db->device = device;
    *out = db;
    return ORBX_OK;
}

void orbx_kfdb_destroy(orbx_kfdb *db) {
    if (!db) return;
    if (db->st || db->d_words || db->d_slots) (void)hipSetDevice(db->device);
    if (db->st) (void)hipStreamSynchronize(db->st);
    if (db->d_words) (void)hipFree(db->d_words);
    if (db->d_values) (void)hipFree(db->d_values);
    if (db->d_slots) (void)hipFree(db->d_slots);
    if (db->d_state) (void)hipFree(db->d_state);
    for (void *x : {(void *)db->d_qcnt, (void *)db->d_qfirst, (void *)db->d_qbuf, (void *)db->d_csr_off,
                    (void *)db->d_csr_cnt, (void *)db->d_csr_tsum, (void *)db->d_csr_slot})
        if (x) (void)hipFree(x);
    if (db->st) (void)hipStreamDestroy(db->st);
    delete db;
}

int orbx_kfdb_add(orbx_kfdb *db, uint64_t kf_id, const uint32_t *words, const double *values, int n) {
    if (!db || n < 0 || (n && (!words || !values)) || !sorted_unique(words, n)) return ORBX_EINVAL;
    // the inverted file is indexed by word id: bounded (ORBvoc has 10^6 words)
    if (n && words[n - 1] >= ORBX_KFDB_MAX_WORDS) return ORBX_EINVAL;
    std::lock_guard<std::mutex> lock(db->mu);
    if (db->live.count(kf_id)) return ORBX_EINVAL;   // the reference would list it twice per word
    Slot s{kf_id, (int64_t)db->h_words.size(), n, true};
    if (n) db->max_word = std::max(db->max_word, words[n - 1]);
    db->h_words.insert(db->h_words.end(), words, words + n);
    db->h_values.insert(db->h_values.end(), values, values + n);
    const int slot = (int)db->slots.size();
    // a re-added keyframe keeps its query state: the state of its previous
    // slot, or of that slot's own source while it is not on the device yet
    auto prev = db->last_slot.find(kf_id);
    int src = prev == db->last_slot.end() ? -1 : prev->second;
    if (src >= db->dev_slots) src = db->seed_src[src - db->dev_slots];
    db->seed_src.push_back(src);
    db->live[kf_id] = slot;
    db->last_slot[kf_id] = slot;
    db->slots.push_back(s);
    return ORBX_OK;
}

int orbx_kfdb_erase(orbx_kfdb *db, uint64_t kf_id) {
    if (!db) return ORBX_EINVAL;
    std::lock_guard<std::mutex> lock(db->mu);
    auto it = db->live.find(kf_id);
    if (it == db->live.end()) return ORBX_OK;   // not in the database: nothing to remove
    db->slots[it->second].alive = false;
    db->live.erase(it);
    db->slots_dirty = true;
    return ORBX_OK;
}

int orbx_kfdb_clear(orbx_kfdb *db) {
    if (!db) return ORBX_EINVAL;
    std::lock_guard<std::mutex> lock(db->mu);
    for (auto &s : db->slots) s.alive = false;
    db->live.clear();
    db->slots_dirty = true;
    return ORBX_OK;
}

int orbx_kfdb_size(const orbx_kfdb *db) { return db ? (int)db->live.size() : ORBX_EINVAL; }

int orbx_kfdb_detect_loop_candidates(orbx_kfdb *db, uint64_t query_id, const uint32_t *words, const double *values,
                                     int n, const uint64_t *connected, int n_connected, float min_score,
                                     orbx_covis_fn covis, void *ctx, uint64_t *out, int cap, int *n_out) {
    return detect(db, false, query_id, words, values, n, connected, n_connected, min_score, covis, ctx, out, cap,
                  n_out);
}

int orbx_kfdb_detect_relocalization_candidates(orbx_kfdb *db, uint64_t frame_id, const uint32_t *words,
                                               const double *values, int n, orbx_covis_fn covis, void *ctx,
                                               uint64_t *out, int cap, int *n_out) {
    return detect(db, true, frame_id, words, values, n, nullptr, 0, 0.f, covis, ctx, out, cap, n_out);
}

int orbx_bow_score_l1(const uint32_t *w1, const double *v1, int n1, const uint32_t *w2, const double *v2, int n2,
                      double *score) {
    if (!score || n1 < 0 || n2 < 0 || (n1 && (!w1 || !v1)) || (n2 && (!w2 || !v2))) return ORBX_EINVAL;
    *score = l1_host(w1, v1, n1, w2, v2, n2);
    return ORBX_OK;
}

}  // extern "C"
