// orbx_vocab_api.hip -- host side of the DBoW2 vocabulary (include/orbx.h):
// the two file loaders, the slot layout the descent kernel reads, and the
// assembly of BowVector / FeatureVector from the per-feature results.
//
// Loaders: TemplatedVocabulary::loadFromTextFile (TemplatedVocabulary.h:
// 1351-1425) and loadFromBinFile (:1473-1547).  Assembly: the two loops of
// transform(features, v, fv, levelsup) (:1140-1207) -- addWeight (TF, TF_IDF)
// or addIfNotExist (IDF, BINARY) in feature order, FeatureVector::addFeature,
// then BowVector::normalize (BowVector.cpp) with the scoring object's norm, or
// the division by the word count when the scoring does not normalise.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <fstream>
#include <map>
#include <mutex>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/orbx.h"
#include "orbx_device.h"

using namespace orbx;

struct orbx_vocab {
    int device = 0, k = 0, L = 0, scoring = 0, weighting = 0, n_nodes = 0, n_words = 0;
    std::vector<int32_t> parent;   // file order
    std::vector<uint8_t> leaf, desc;
    std::vector<double> weight;
    // slot layout (children of a node in consecutive slots)
    std::vector<VocabNode> nodes;
    std::vector<uint8_t> sdesc;
    std::vector<double> sweight;
    int kmax = 0;
    std::mutex mu;
    bool uploaded = false;
    VocabNode *d_nodes = nullptr;
    uint8_t *d_desc = nullptr;
    double *d_weight = nullptr;
    hipStream_t st = nullptr;
    uint8_t *d_buf = nullptr, *h_buf = nullptr;
    size_t buf_cap = 0;
};

namespace {

int build_slots(orbx_vocab *v) {
    const int n = v->n_nodes;
    std::vector<int> cnt(n, 0), start(n + 1, 0);
    for (int i = 1; i < n; ++i) {
        if (v->parent[i] < 0 || v->parent[i] >= i) return ORBX_EINVAL;
        ++cnt[v->parent[i]];
    }
    for (int i = 0; i < n; ++i) start[i + 1] = start[i] + cnt[i];
    std::vector<int> kids(std::max(n - 1, 1)), fill(start.begin(), start.end() - 1);
    for (int i = 1; i < n; ++i) kids[fill[v->parent[i]]++] = i;   // file order
    v->kmax = 0;
    for (int i = 0; i < n; ++i) v->kmax = std::max(v->kmax, cnt[i]);
    if (v->kmax > 64) return ORBX_EINVAL;
    std::vector<uint32_t> word(n, 0);
    int nw = 0;
    for (int i = 1; i < n; ++i)
        if (v->leaf[i]) word[i] = (uint32_t)nw++;
    v->n_words = nw;
    // breadth-first slots: node order[s] sits in slot s
    std::vector<int> order(n), slot_of(n);
    order[0] = 0;
    slot_of[0] = 0;
    int next = 1;
    for (int s = 0; s < n; ++s) {
        const int u = order[s];
        for (int j = start[u]; j < start[u + 1]; ++j) {
            order[next] = kids[j];
            slot_of[kids[j]] = next;
            ++next;
        }
    }
    if (next != n) return ORBX_EINVAL;
    v->nodes.resize(n);
    v->sdesc.assign(32 * (size_t)n, 0);
    v->sweight.resize(n);
    for (int s = 0; s < n; ++s) {
        const int u = order[s];
        VocabNode &nd = v->nodes[s];
        nd.nchild = cnt[u];
        nd.first = cnt[u] ? slot_of[kids[start[u]]] : 0;
        nd.word = word[u];
        nd.id = (uint32_t)u;
        std::memcpy(&v->sdesc[32 * (size_t)s], &v->desc[32 * (size_t)u], 32);
        v->sweight[s] = v->weight[u];
    }
    return ORBX_OK;
}

bool header_ok(int k, int L, int n1, int n2) {
    // TemplatedVocabulary.h:1381 / :1497
    return !(k < 0 || k > 20 || L < 1 || L > 10 || n1 < 0 || n1 > 5 || n2 < 0 || n2 > 3);
}

int finish(orbx_vocab *v, orbx_vocab **out) {
    const int rc = build_slots(v);
    if (rc) { delete v; return rc; }
    *out = v;
    return ORBX_OK;
}

int ensure_device(orbx_vocab *v, size_t scratch) {
    if (hipSetDevice(v->device) != hipSuccess) return ORBX_ENODEV;
    if (!v->st && hipStreamCreateWithFlags(&v->st, hipStreamNonBlocking) != hipSuccess) return ORBX_EIO;
    if (!v->uploaded) {
        const size_t n = (size_t)v->n_nodes;
        if (hipMalloc(reinterpret_cast<void **>(&v->d_nodes), sizeof(VocabNode) * n) != hipSuccess ||
            hipMalloc(reinterpret_cast<void **>(&v->d_desc), 32 * n) != hipSuccess ||
            hipMalloc(reinterpret_cast<void **>(&v->d_weight), 8 * n) != hipSuccess)
            return ORBX_ENOMEM;
        if (hipMemcpy(v->d_nodes, v->nodes.data(), sizeof(VocabNode) * n, hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy(v->d_desc, v->sdesc.data(), 32 * n, hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy(v->d_weight, v->sweight.data(), 8 * n, hipMemcpyHostToDevice) != hipSuccess)
            return ORBX_EIO;
        v->uploaded = true;
    }
    if (scratch > v->buf_cap) {
        (void)hipStreamSynchronize(v->st);
        if (v->d_buf) (void)hipFree(v->d_buf);
        if (v->h_buf) (void)hipHostFree(v->h_buf);
        v->d_buf = v->h_buf = nullptr;
        v->buf_cap = 0;
        const size_t cap = std::max(scratch, size_t(1) << 16) * 3 / 2;
        if (hipMalloc(reinterpret_cast<void **>(&v->d_buf), cap) != hipSuccess) return ORBX_ENOMEM;
        if (hipHostMalloc(reinterpret_cast<void **>(&v->h_buf), cap, hipHostMallocDefault) != hipSuccess)
            return ORBX_ENOMEM;
        v->buf_cap = cap;
    }
    return ORBX_OK;
}

VocabDev dev_view(const orbx_vocab *v) {
    VocabDev d;
    d.nodes = v->d_nodes;
    d.desc = v->d_desc;
    d.weight = v->d_weight;
    d.k = std::max(v->kmax, 1);
    return d;
}

}  // namespace

extern "C" {

int orbx_vocab_create(int device, int k, int L, int scoring, int weighting, int n_nodes, const int32_t *parent,
                      const uint8_t *is_leaf, const uint8_t *desc, const double *weight, orbx_vocab **out) {
    if (!out || n_nodes < 1 || !header_ok(k, L, scoring, weighting)) return ORBX_EINVAL;
    if (n_nodes > 1 && (!parent || !is_leaf || !desc || !weight)) return ORBX_EINVAL;
    orbx_vocab *v = new orbx_vocab;
    v->device = device; v->k = k; v->L = L; v->scoring = scoring; v->weighting = weighting; v->n_nodes = n_nodes;
    v->parent.assign(n_nodes, 0);
    v->leaf.assign(n_nodes, 0);
    v->desc.assign(32 * (size_t)n_nodes, 0);
    v->weight.assign(n_nodes, 0.0);
    if (n_nodes > 1) {
        std::copy(parent + 1, parent + n_nodes, v->parent.begin() + 1);
        std::copy(is_leaf + 1, is_leaf + n_nodes, v->leaf.begin() + 1);
        std::copy(desc + 32, desc + 32 * (size_t)n_nodes, v->desc.begin() + 32);
        std::copy(weight + 1, weight + n_nodes, v->weight.begin() + 1);
    }
    return finish(v, out);
}

int orbx_vocab_load(int device, const char *path, int format, orbx_vocab **out) {
    if (!path || !out || (format != 0 && format != 1)) return ORBX_EINVAL;
    std::ifstream f(path, format ? std::ios::in | std::ios::binary : std::ios::in);
    if (!f.is_open()) return ORBX_EINVAL;
    orbx_vocab *v = new orbx_vocab;
    v->device = device;
    int k = 0, L = 0, n1 = 0, n2 = 0;
    if (format == 0) {
        std::string line;
        std::getline(f, line);
        std::stringstream hs(line);
        hs >> k >> L >> n1 >> n2;
        if (hs.fail() || !header_ok(k, L, n1, n2)) { delete v; return ORBX_EINVAL; }
    } else {
        int32_t h[4];
        f.read(reinterpret_cast<char *>(h), sizeof(h));
        if (!f || !header_ok(h[0], h[1], h[2], h[3]) || h[0] < 2) { delete v; return ORBX_EINVAL; }
        k = h[0]; L = h[1]; n1 = h[2]; n2 = h[3];
    }
    v->k = k; v->L = L; v->scoring = n1; v->weighting = n2;
    v->parent.push_back(0);   // root
    v->leaf.push_back(0);
    v->desc.resize(32, 0);
    v->weight.push_back(0.0);
    if (format == 0) {
        std::string line;
        while (std::getline(f, line)) {
            if (line.find_first_not_of(" \t\r\n") == std::string::npos) continue;
            std::stringstream ss(line);
            int pid = 0, isleaf = 0;
            ss >> pid >> isleaf;
            uint8_t d[32];
            for (int i = 0; i < 32; ++i) {
                int x = 0;
                ss >> x;
                d[i] = (uint8_t)x;
            }
            double w = 0.0;
            ss >> w;
            const int nid = (int)v->parent.size();
            if (ss.fail() || pid < 0 || pid >= nid) { delete v; return ORBX_EINVAL; }
            v->parent.push_back(pid);
            v->leaf.push_back(isleaf > 0);
            v->desc.insert(v->desc.end(), d, d + 32);
            v->weight.push_back(w);
        }
    } else {
        const int expected = (int)((std::pow((double)k, (double)L + 1) - 1) / (k - 1));
        while ((int)v->parent.size() < expected) {
            int32_t pid;
            uint8_t isleaf, d[32];
            double w;
            f.read(reinterpret_cast<char *>(&pid), 4);
            f.read(reinterpret_cast<char *>(&isleaf), 1);
            f.read(reinterpret_cast<char *>(d), 32);
            f.read(reinterpret_cast<char *>(&w), 8);
            if (!f) break;   // the last complete record
            const int nid = (int)v->parent.size();
            if (pid < 0 || pid >= nid) { delete v; return ORBX_EINVAL; }
            v->parent.push_back(pid);
            v->leaf.push_back(isleaf > 0);
            v->desc.insert(v->desc.end(), d, d + 32);
            v->weight.push_back(w);
        }
    }
    v->n_nodes = (int)v->parent.size();
    return finish(v, out);
}

void orbx_vocab_destroy(orbx_vocab *v) {
    if (!v) return;
    if (v->uploaded || v->st || v->d_buf) (void)hipSetDevice(v->device);
    if (v->st) (void)hipStreamSynchronize(v->st);
    if (v->d_nodes) (void)hipFree(v->d_nodes);
    if (v->d_desc) (void)hipFree(v->d_desc);
    if (v->d_weight) (void)hipFree(v->d_weight);
    if (v->d_buf) (void)hipFree(v->d_buf);
    if (v->h_buf) (void)hipHostFree(v->h_buf);
    if (v->st) (void)hipStreamDestroy(v->st);
    delete v;
}

int orbx_vocab_info(const orbx_vocab *v, int *k, int *L, int *scoring, int *weighting, int *n_nodes, int *n_words) {
    if (!v) return ORBX_EINVAL;
    if (k) *k = v->k;
    if (L) *L = v->L;
    if (scoring) *scoring = v->scoring;
    if (weighting) *weighting = v->weighting;
    if (n_nodes) *n_nodes = v->n_nodes;
    if (n_words) *n_words = v->n_words;
    return ORBX_OK;
}

int orbx_vocab_export(const orbx_vocab *v, int32_t *parent, uint8_t *is_leaf, uint8_t *desc, double *weight, int cap) {
    if (!v) return ORBX_EINVAL;
    if (cap < v->n_nodes) return ORBX_ERANGE;
    const size_t n = (size_t)v->n_nodes;
    if (parent) std::copy(v->parent.begin(), v->parent.end(), parent);
    if (is_leaf) std::copy(v->leaf.begin(), v->leaf.end(), is_leaf);
    if (desc) std::memcpy(desc, v->desc.data(), 32 * n);
    if (weight) std::copy(v->weight.begin(), v->weight.end(), weight);
    return ORBX_OK;
}

int orbx_vocab_transform_device(orbx_vocab *v, const uint8_t *d_desc, int n, int levelsup, uint32_t *d_word,
                                double *d_weight, uint32_t *d_node, void *stream) {
    if (!v || n < 0 || (n && (!d_desc || !d_word || !d_weight || !d_node))) return ORBX_EINVAL;
    if (n == 0 || v->n_words == 0) return ORBX_OK;
    std::lock_guard<std::mutex> lock(v->mu);
    int rc = ensure_device(v, 0);
    if (rc) return rc;
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : v->st;   // NULL: the vocabulary's own stream
    if (launch_vocab_transform(dev_view(v), d_desc, n, v->L - levelsup, d_word, d_weight, d_node, st) != hipSuccess)
        return ORBX_EIO;
    return ORBX_OK;
}

int orbx_vocab_transform(orbx_vocab *v, const uint8_t *desc, int n, int levelsup, uint32_t *bow_words,
                         double *bow_values, int *n_bow, uint32_t *fv_nodes, int32_t *fv_offsets,
                         int32_t *fv_features, int *n_fv) {
    if (!v || n < 0 || !n_bow || !n_fv || !fv_offsets) return ORBX_EINVAL;
    if (n && (!desc || !bow_words || !bow_values || !fv_nodes || !fv_features)) return ORBX_EINVAL;
    *n_bow = 0;
    *n_fv = 0;
    fv_offsets[0] = 0;
    if (n == 0 || v->n_words == 0) return ORBX_OK;   // transform on empty(): cleared
    std::vector<uint32_t> word(n), node(n);
    std::vector<double> w(n);
    {
        std::lock_guard<std::mutex> lock(v->mu);
        const size_t o_w = 32 * (size_t)n, o_wt = o_w + ((4 * (size_t)n + 7) & ~size_t(7)),
                     o_nd = o_wt + 8 * (size_t)n, total = o_nd + 4 * (size_t)n;
        int rc = ensure_device(v, total);
        if (rc) return rc;
        std::memcpy(v->h_buf, desc, 32 * (size_t)n);
        uint8_t *D = v->d_buf;
        if (hipMemcpyAsync(D, v->h_buf, 32 * (size_t)n, hipMemcpyHostToDevice, v->st) != hipSuccess ||
            launch_vocab_transform(dev_view(v), D, n, v->L - levelsup, reinterpret_cast<uint32_t *>(D + o_w),
                                   reinterpret_cast<double *>(D + o_wt), reinterpret_cast<uint32_t *>(D + o_nd),
                                   v->st) != hipSuccess ||
            hipMemcpyAsync(v->h_buf + o_w, D + o_w, total - o_w, hipMemcpyDeviceToHost, v->st) != hipSuccess ||
            hipStreamSynchronize(v->st) != hipSuccess)
            return ORBX_EIO;
        std::memcpy(word.data(), v->h_buf + o_w, 4 * (size_t)n);
        std::memcpy(w.data(), v->h_buf + o_wt, 8 * (size_t)n);
        std::memcpy(node.data(), v->h_buf + o_nd, 4 * (size_t)n);
    }
    // BowVector / FeatureVector in the reference's order of operations
    const bool tf = v->weighting == 0 || v->weighting == 1;
    const bool must = v->scoring != 5, l2 = v->scoring == 1;
    std::map<uint32_t, double> bow;
    std::map<uint32_t, std::vector<int32_t>> fv;
    for (int f = 0; f < n; ++f) {
        if (!(w[f] > 0)) continue;   // stopped word
        auto it = bow.find(word[f]);
        if (it == bow.end()) bow.emplace(word[f], w[f]);
        else if (tf) it->second += w[f];
        fv[node[f]].push_back(f);
    }
    if (tf && !bow.empty() && !must) {
        const double nd = (double)bow.size();
        for (auto &kv : bow) kv.second /= nd;
    }
    if (must) {
        double norm = 0.0;
        if (!l2) {
            for (auto &kv : bow) norm += std::fabs(kv.second);
        } else {
            for (auto &kv : bow) norm += kv.second * kv.second;
            norm = std::sqrt(norm);
        }
        if (norm > 0.0)
            for (auto &kv : bow) kv.second /= norm;
    }
    int i = 0;
    for (auto &kv : bow) { bow_words[i] = kv.first; bow_values[i] = kv.second; ++i; }
    *n_bow = i;
    int j = 0, t = 0;
    for (auto &kv : fv) {
        fv_nodes[j] = kv.first;
        for (int32_t x : kv.second) fv_features[t++] = x;
        fv_offsets[++j] = t;
    }
    *n_fv = j;
    return ORBX_OK;
}

}  // extern "C"
