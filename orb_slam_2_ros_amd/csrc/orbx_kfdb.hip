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
// The L1 scores of the retained keyframes are a second pass (a wave per
// keyframe; the common-word terms are summed in ascending word order, as the
// reference's merge adds them).  The per-keyframe query state (mnLoopQuery,
// mnLoopWords, mLoopScore and the reloc trio) persists across queries on the
// host exactly as in the reference, and the covisibility accumulation and the
// retention run there too (a few hundred scalars).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <list>
#include <mutex>
#include <set>
#include <unordered_map>
#include <vector>

#include "orbx_device.h"
#include "orbx_wave.h"
#include "orbx_ws.h"

namespace orbx {
namespace {

constexpr int kKT = 256;
constexpr int kQLds = 8192;   // query words (and values) staged in LDS; more: read from global

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

// Per keyframe: the number of query words it contains and the rank of the
// first one (the query word at which the inverted-file walk first meets it).
__global__ __launch_bounds__(kKT) void k_kfdb_count(const SlotDev *slots, int nslots, const uint32_t *words,
                                                    const uint32_t *qw_g, int nq, int2 *out) {
    __shared__ uint32_t qs[kQLds];
    const bool staged = nq <= kQLds;
    if (staged)
        for (int i = threadIdx.x; i < nq; i += kKT) qs[i] = qw_g[i];
    __syncthreads();
    const uint32_t *qw = staged ? qs : qw_g;
    const int lane = threadIdx.x & 63;
    const int s = blockIdx.x * (kKT / 64) + (threadIdx.x >> 6);
    if (s >= nslots) return;
    const SlotDev sl = slots[s];
    int cnt = 0;
    uint32_t first = ~0u;
    if (sl.alive) {
        for (int i = lane; i < sl.n; i += 64) {
            const int r = find_word(qw, nq, words[sl.off + i]);
            if (r >= 0) { ++cnt; first = min(first, (uint32_t)r); }
        }
    }
    cnt = wave_sum_i32(cnt);
    first = wave_min_u32(first);
    if (lane == 0) out[s] = make_int2(cnt, (int)first);
}

// L1Scoring::score(query, keyframe) for the listed slots, in double.
__global__ __launch_bounds__(kKT) void k_kfdb_score(const SlotDev *slots, const int32_t *list, int nlist,
                                                    const uint32_t *words, const double *values, const uint32_t *qw_g,
                                                    const double *qv_g, int nq, double *score) {
    __shared__ uint32_t qs[kQLds];
    const bool staged = nq <= kQLds;
    if (staged)
        for (int i = threadIdx.x; i < nq; i += kKT) qs[i] = qw_g[i];
    __syncthreads();
    const uint32_t *qw = staged ? qs : qw_g;
    const int lane = threadIdx.x & 63;
    const int li = blockIdx.x * (kKT / 64) + (threadIdx.x >> 6);
    if (li >= nlist) return;
    const SlotDev sl = slots[list[li]];
    double acc = 0;
    for (int c0 = 0; c0 < sl.n; c0 += 64) {
        const int i = c0 + lane;
        double term = 0;
        bool hit = false;
        if (i < sl.n) {
            const int r = find_word(qw, nq, words[sl.off + i]);
            if (r >= 0) {
                const double vi = qv_g[r], wi = values[sl.off + i];
                term = __dsub_rn(__dsub_rn(fabs(__dsub_rn(vi, wi)), fabs(vi)), fabs(wi));
                hit = true;
            }
        }
        // add the terms in ascending word order (the keyframe's words are sorted)
        for (uint64_t b = __ballot(hit); b; b &= b - 1) {
            const int j = (int)__builtin_ctzll(b);
            const uint64_t bits = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)__double_as_longlong(term), j) |
                                  ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(
                                       (int)(uint32_t)((uint64_t)__double_as_longlong(term) >> 32), j)
                                   << 32);
            acc = __dadd_rn(acc, __longlong_as_double((long long)bits));
        }
    }
    if (lane == 0) score[li] = -acc / 2.0;
}

}  // namespace
}  // namespace orbx

using namespace orbx;

namespace {
struct KFState {
    uint64_t loop_query = 0, reloc_query = 0;   // KeyFrame.cc:41
    int loop_words = 0, reloc_words = 0;
    float loop_score = 0, reloc_score = 0;      // uninitialised in the reference
};
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
    std::unordered_map<uint64_t, KFState> state;  // persists across erase / re-add
    std::vector<uint32_t> h_words;                // host mirror of the arena (compaction)
    std::vector<double> h_values;
    uint32_t *d_words = nullptr;
    double *d_values = nullptr;
    SlotDev *d_slots = nullptr;
    int64_t cap_words = 0, dev_words = 0;        // arena capacity / words on the device
    int cap_slots = 0, dev_slots = 0;             // slot table capacity / rows on the device
    bool slots_dirty = false;
};

namespace {

int kfdb_sync(orbx_kfdb *db) {
    // grow-and-upload the arena tail and the slot table
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
        if (hipMalloc(reinterpret_cast<void **>(&d), sizeof(SlotDev) * cap) != hipSuccess) return ORBX_ENOMEM;
        (void)hipStreamSynchronize(db->st);
        if (db->d_slots) (void)hipFree(db->d_slots);
        db->d_slots = d;
        db->cap_slots = cap;
        db->slots_dirty = true;
    }
    if (db->slots_dirty || ns > db->dev_slots) {
        std::vector<SlotDev> t(ns);
        for (int i = 0; i < ns; ++i) t[i] = {db->slots[i].off, db->slots[i].n, db->slots[i].alive ? 1 : 0};
        if (ns && hipMemcpyAsync(db->d_slots, t.data(), sizeof(SlotDev) * ns, hipMemcpyHostToDevice, db->st) !=
                      hipSuccess)
            return ORBX_EIO;
        (void)hipStreamSynchronize(db->st);   // (t is a host temporary)
        db->dev_slots = ns;
        db->slots_dirty = false;
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
    std::lock_guard<std::mutex> lock(db->mu);
    const int ns = (int)db->slots.size();
    if (n == 0 || ns == 0) return ORBX_OK;
    if (hipSetDevice(db->device) != hipSuccess) return ORBX_ENODEV;
    if (!db->st && hipStreamCreateWithFlags(&db->st, hipStreamNonBlocking) != hipSuccess) return ORBX_EIO;
    int rc = kfdb_sync(db);
    if (rc) return rc;
    // pass 1: shared-word counts and first shared word of every keyframe
    Layout L;
    const size_t o_qw = L.add(4 * (size_t)n), o_qv = L.add(8 * (size_t)n), o_cnt = L.add(8 * (size_t)ns);
    const size_t o_list = L.add(4 * (size_t)ns), o_sc = L.add(8 * (size_t)ns);
    CallWs &ws = call_ws(db->device);
    std::lock_guard<std::mutex> wl(ws.mu);
    rc = ws_reserve(ws, L.size);
    if (rc) return rc;
    put(ws, o_qw, words, 4 * (size_t)n);
    put(ws, o_qv, values, 8 * (size_t)n);
    uint8_t *D = ws.dev;
    if (hipStreamSynchronize(db->st) != hipSuccess ||
        hipMemcpyAsync(D, ws.host, o_cnt, hipMemcpyHostToDevice, ws.st) != hipSuccess)
        return ORBX_EIO;
    hipLaunchKernelGGL(k_kfdb_count, dim3((ns + kKT / 64 - 1) / (kKT / 64)), dim3(kKT), 0, ws.st, db->d_slots, ns,
                       db->d_words, at<uint32_t>(D, o_qw), n, at<int2>(D, o_cnt));
    if (hipGetLastError() != hipSuccess ||
        hipMemcpyAsync(ws.host + o_cnt, D + o_cnt, 8 * (size_t)ns, hipMemcpyDeviceToHost, ws.st) != hipSuccess ||
        hipStreamSynchronize(ws.st) != hipSuccess)
        return ORBX_EIO;
    const int2 *cnt = at<int2>(ws.host, o_cnt);
    // the inverted-file walk's visiting order: (first shared query word, add order)
    std::vector<int> met;
    for (int s = 0; s < ns; ++s)
        if (cnt[s].x > 0) met.push_back(s);
    std::stable_sort(met.begin(), met.end(), [&](int a, int b) { return cnt[a].y < cnt[b].y; });
    std::set<uint64_t> conn;
    if (!reloc) conn.insert(connected, connected + n_connected);
    std::vector<int> sharing;   // slots in lKFsSharingWords order
    for (int s : met) {
        KFState &k = db->state[db->slots[s].id];
        const int c = cnt[s].x;
        if (!reloc) {
            // the walk meets the keyframe c times: the first meeting resets the
            // count (unless already met by this query id) and lists it unless
            // connected; a connected keyframe is reset at every meeting
            if (k.loop_query != qid) {
                if (!conn.count(db->slots[s].id)) {
                    k.loop_query = qid;
                    k.loop_words = c;
                    sharing.push_back(s);
                } else {
                    k.loop_words = 1;
                }
            } else {
                k.loop_words += c;
            }
        } else {
            if (k.reloc_query != qid) {
                k.reloc_query = qid;
                k.reloc_words = c;
                sharing.push_back(s);
            } else {
                k.reloc_words += c;
            }
        }
    }
    if (sharing.empty()) return ORBX_OK;
    int maxCommonWords = 0;
    for (int s : sharing) {
        const KFState &k = db->state[db->slots[s].id];
        maxCommonWords = std::max(maxCommonWords, reloc ? k.reloc_words : k.loop_words);
    }
    const int minCommonWords = maxCommonWords * 0.8f;
    // pass 2: L1 scores of the keyframes above minCommonWords
    std::vector<int> to_score;
    for (int s : sharing) {
        const KFState &k = db->state[db->slots[s].id];
        if ((reloc ? k.reloc_words : k.loop_words) > minCommonWords) to_score.push_back(s);
    }
    const int nsc = (int)to_score.size();
    put(ws, o_list, to_score.data(), 4 * (size_t)nsc);
    if (hipMemcpyAsync(D + o_list, ws.host + o_list, 4 * (size_t)nsc, hipMemcpyHostToDevice, ws.st) != hipSuccess)
        return ORBX_EIO;
    hipLaunchKernelGGL(k_kfdb_score, dim3((nsc + kKT / 64 - 1) / (kKT / 64)), dim3(kKT), 0, ws.st, db->d_slots,
                       at<int32_t>(D, o_list), nsc, db->d_words, db->d_values, at<uint32_t>(D, o_qw),
                       at<double>(D, o_qv), n, at<double>(D, o_sc));
    if (hipGetLastError() != hipSuccess ||
        hipMemcpyAsync(ws.host + o_sc, D + o_sc, 8 * (size_t)nsc, hipMemcpyDeviceToHost, ws.st) != hipSuccess ||
        hipStreamSynchronize(ws.st) != hipSuccess)
        return ORBX_EIO;
    const double *sc = at<double>(ws.host, o_sc);
    std::vector<std::pair<float, int>> scored;
    for (int i = 0; i < nsc; ++i) {
        KFState &k = db->state[db->slots[to_score[i]].id];
        const float si = (float)sc[i];
        if (reloc) {
            k.reloc_score = si;
            scored.emplace_back(si, to_score[i]);
        } else {
            k.loop_score = si;
            if (si >= minScore) scored.emplace_back(si, to_score[i]);
        }
    }
    if (scored.empty()) return ORBX_OK;
    // covisibility accumulation (KeyFrameDatabase.cc:151-185 / 287-318)
    std::vector<std::pair<float, uint64_t>> acc;
    float bestAccScore = reloc ? 0 : minScore;
    uint64_t neigh[64];
    for (auto &sm : scored) {
        const uint64_t kid = db->slots[sm.second].id;
        const int nn = std::min(covis(ctx, kid, neigh, 10), 10);
        float bestScore = sm.first, accScore = sm.first;
        uint64_t best = kid;
        for (int t = 0; t < nn; ++t) {
            auto it = db->state.find(neigh[t]);
            if (it == db->state.end()) continue;   // never in the database: no query state
            const KFState &k2 = it->second;
            if (!reloc) {
                if (k2.loop_query == qid && k2.loop_words > minCommonWords) {
                    accScore += k2.loop_score;
                    if (k2.loop_score > bestScore) { best = neigh[t]; bestScore = k2.loop_score; }
                }
            } else {
                if (k2.reloc_query != qid) continue;
                accScore += k2.reloc_score;
                if (k2.reloc_score > bestScore) { best = neigh[t]; bestScore = k2.reloc_score; }
            }
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
    if (db->st) (void)hipStreamDestroy(db->st);
    delete db;
}

int orbx_kfdb_add(orbx_kfdb *db, uint64_t kf_id, const uint32_t *words, const double *values, int n) {
    if (!db || n < 0 || (n && (!words || !values)) || !sorted_unique(words, n)) return ORBX_EINVAL;
    std::lock_guard<std::mutex> lock(db->mu);
    if (db->live.count(kf_id)) return ORBX_EINVAL;   // the reference would list it twice per word
    Slot s{kf_id, (int64_t)db->h_words.size(), n, true};
    db->h_words.insert(db->h_words.end(), words, words + n);
    db->h_values.insert(db->h_values.end(), values, values + n);
    db->live[kf_id] = (int)db->slots.size();
    db->slots.push_back(s);
    db->state.emplace(kf_id, KFState());
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
