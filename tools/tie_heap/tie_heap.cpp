// tie_heap -- diagnostic for DESIGN.md §3.4 (CPU only; not linked by the
// product or the tests).
//
// DistributeOctTree (ORBextractor.cc:561-787) sorts pair<int, ExtractorNode*>
// (:705-708), so quadtree nodes holding equally many keypoints are split in
// heap-address order.  The restatement (oracle + kernels) replaces that by
// creation order.  This program measures how often a real glibc heap agrees:
// it replays the allocation sequence of ORBextractor::operator() up to the
// last level's tree -- the level buffers of ComputePyramid, per level the
// vToDistributeKeys reserve, one vector<KeyPoint> per visited cell grown by
// push_back to the cell's corner count and freed, the level's keypoints
// reserve, then the tree itself with ExtractorNode's shape (a std::list node of
// a 72-byte object: vector<28-byte key>, four int points, a list iterator, a
// bool), the children's reserve(parent size) in DivideNode order, the list
// copies, erase, the locals' destruction, the (size, pointer) vectors and
// their copy in the final phase -- and sorts by the REAL addresses.
//
// Input (binary file, argv[1]): int32 nlevels, nfeatures, frames, then per
// frame per level: w, h, quota, ncand, ncells, ncand x (x, y, score), ncells
// counts.  Output (stdout, text): per frame per level the selected candidate
// indices in output order, one line "f l n i0 i1 ...".
// frames: the frames run back to back in ONE thread that the program starts
// (a fresh thread: its own arena and an empty tcache), each frame's level
// buffers and outputs kept until the next frame replaces them, as the
// extractor and the Frame hold them.
//
//   g++ -O2 -std=c++17 -pthread tools/tie_heap/tie_heap.cpp -o tools/tie_heap/tie_heap
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <list>
#include <thread>
#include <utility>
#include <vector>

#ifdef TIE_SIM
#include <map>
#include <unordered_map>
#endif

namespace {

#ifdef TIE_SIM
// -DTIE_SIM: a deterministic model of glibc's small-chunk reuse instead of the
// real heap -- every allocation gets a virtual address from a simulated arena:
// chunk = (n + 8) rounded up to 16 (min 32); malloc takes the newest chunk of
// its size from the tcache (7 per size, LIFO), then a fastbin (<= 128 B,
// LIFO), then an exact-size free list (larger chunks, LIFO), else the top
// (addresses ascending); requests >= the mmap threshold (128 KiB, raised to a
// freed mapping's size as glibc does) never touch the arena.  No coalescing.
struct SimHeap {
    std::map<size_t, std::vector<uint64_t>> tc, fb, big;
    uint64_t top = 0x10000;
    size_t mmap_th = 128 * 1024;
    std::unordered_map<const void *, std::pair<uint64_t, size_t>> live;   // real -> (virtual, chunk; 0 = mapped)
    static size_t chunk(size_t n) { return std::max<size_t>(32, (n + 8 + 15) & ~(size_t)15); }
    uint64_t take(size_t c) {
        auto grab = [&](std::map<size_t, std::vector<uint64_t>> &m) -> uint64_t {
            auto it = m.find(c);
            if (it == m.end() || it->second.empty()) return 0;
            const uint64_t a = it->second.back();
            it->second.pop_back();
            return a;
        };
        uint64_t a = grab(tc);
        if (!a && c <= 128) a = grab(fb);
        if (!a && c > 128) a = grab(big);
        if (!a) { a = top; top += c; }
        return a;
    }
    void give(uint64_t a, size_t c) {
        std::vector<uint64_t> &t = tc[c];
        if (t.size() < 7) t.push_back(a);
        else if (c <= 128) fb[c].push_back(a);
        else big[c].push_back(a);
    }
    void *alloc(size_t n) {
        void *p = std::malloc(n ? n : 1);
        if (n >= mmap_th) live[p] = {0x7f0000000000ull + (uint64_t)(uintptr_t)p, 0};
        else { const size_t c = chunk(n); live[p] = {take(c), c}; }
        return p;
    }
    void release(void *p) {
        if (!p) return;
        auto it = live.find(p);
        if (it != live.end()) {
            if (it->second.second) give(it->second.first, it->second.second);
            live.erase(it);
        }
        std::free(p);
    }
    uint64_t vaddr(const void *node_payload) const {   // a std::list node's payload sits 16 B in
        auto it = live.find(static_cast<const char *>(node_payload) - 16);
        return it == live.end() ? 0 : it->second.first + 16;
    }
};
SimHeap g_sim;
template <class T>
struct SimAlloc {
    typedef T value_type;
    SimAlloc() = default;
    template <class U>
    SimAlloc(const SimAlloc<U> &) {}
    T *allocate(size_t n) { return static_cast<T *>(g_sim.alloc(n * sizeof(T))); }
    void deallocate(T *p, size_t) { g_sim.release(p); }
    template <class U>
    bool operator==(const SimAlloc<U> &) const { return true; }
    template <class U>
    bool operator!=(const SimAlloc<U> &) const { return false; }
};
template <class T> using Vec = std::vector<T, SimAlloc<T>>;
template <class T> using Lst = std::list<T, SimAlloc<T>>;
void *raw_alloc(size_t n) { return g_sim.alloc(n); }
void raw_free(void *p) { g_sim.release(p); }
#else
template <class T> using Vec = std::vector<T>;
template <class T> using Lst = std::list<T>;
void *raw_alloc(size_t n) { return std::malloc(n); }
void raw_free(void *p) { std::free(p); }
#endif

struct Key {   // cv::KeyPoint's 28 bytes; class_id carries the candidate index
    float x, y, size, angle, response;
    int octave, class_id;
};
static_assert(sizeof(Key) == 28, "cv::KeyPoint is 28 bytes");

struct Pt {
    int x, y;
};

// -DTIE_CREATION: a check build that sorts by creation number instead of the
// address (the restatement's rule; it must reproduce orbo_distribute exactly).
struct Node {   // ExtractorNode (ORBextractor.h:32-43)
    Node() : done(false) {}
    Vec<Key> keys;
    Pt ul, ur, bl, br;
    typename Lst<Node>::iterator self;
    bool done;
#ifdef TIE_CREATION
    long seq = 0;
#endif
};
#ifndef TIE_CREATION
static_assert(sizeof(Node) == 72, "ExtractorNode is 72 bytes");
#else
long g_seq = 0;
#endif

// DivideNode (ORBextractor.cc:498-554): each child reserves the parent's key
// count, in child order, then takes its quadrant's keys.
void divide(const Node &p, Node &a, Node &b, Node &c, Node &d) {
    const int hx = (int)std::ceil((float)(p.ur.x - p.ul.x) / 2);
    const int hy = (int)std::ceil((float)(p.br.y - p.ul.y) / 2);
    a.ul = p.ul;
    a.ur = {p.ul.x + hx, p.ul.y};
    a.bl = {p.ul.x, p.ul.y + hy};
    a.br = {p.ul.x + hx, p.ul.y + hy};
    a.keys.reserve(p.keys.size());
    b.ul = a.ur;
    b.ur = p.ur;
    b.bl = a.br;
    b.br = {p.ur.x, p.ul.y + hy};
    b.keys.reserve(p.keys.size());
    c.ul = a.bl;
    c.ur = a.br;
    c.bl = p.bl;
    c.br = {a.br.x, p.bl.y};
    c.keys.reserve(p.keys.size());
    d.ul = c.ur;
    d.ur = b.br;
    d.bl = c.br;
    d.br = p.br;
    d.keys.reserve(p.keys.size());
    for (const Key &k : p.keys) {
        if (k.x < a.ur.x) (k.y < a.br.y ? a : c).keys.push_back(k);
        else (k.y < a.br.y ? b : d).keys.push_back(k);
    }
    for (Node *n : {&a, &b, &c, &d})
        if (n->keys.size() == 1) n->done = true;
}

typedef Vec<std::pair<int, Node *>> SizePtr;

// Children into the list (push_front copies: a list node, then the key
// vector's copy), the splittable ones recorded with their address.
void push_children(Lst<Node> &L, Node *ch[4], SizePtr &v, int *nexpand) {
    for (int q = 0; q < 4; ++q) {
        if (ch[q]->keys.empty()) continue;
#ifdef TIE_CREATION
        ch[q]->seq = g_seq++;
#endif
        L.push_front(*ch[q]);
        if (ch[q]->keys.size() > 1) {
            if (nexpand) ++*nexpand;
            v.push_back(std::make_pair((int)ch[q]->keys.size(), &L.front()));
            L.front().self = L.begin();
        }
    }
}

Vec<Key> tree(const Vec<Key> &in, int minX, int maxX, int minY, int maxY, int N, int nfeatures) {
    const int nIni = (int)std::round((float)(maxX - minX) / (maxY - minY));
    const float hX = (float)(maxX - minX) / nIni;
    Lst<Node> L;
    Vec<Node *> ini;
    ini.resize(nIni);
    for (int i = 0; i < nIni; ++i) {
        Node n;
        n.ul = {(int)(hX * (float)i), 0};
        n.ur = {(int)(hX * (float)(i + 1)), 0};
        n.bl = {n.ul.x, maxY - minY};
        n.br = {n.ur.x, maxY - minY};
        n.keys.reserve(in.size());
#ifdef TIE_CREATION
        n.seq = g_seq++;
#endif
        L.push_back(n);
        ini[i] = &L.back();
    }
    for (const Key &k : in) ini[(size_t)(k.x / hX)]->keys.push_back(k);
    for (auto it = L.begin(); it != L.end();) {
        if (it->keys.size() == 1) { it->done = true; ++it; }
        else if (it->keys.empty()) it = L.erase(it);
        else ++it;
    }
    bool finish = false;
    SizePtr cur;
    cur.reserve(L.size() * 4);
    while (!finish) {
        int prev = (int)L.size();
        int nexpand = 0;
        cur.clear();
        for (auto it = L.begin(); it != L.end();) {
            if (it->done) { ++it; continue; }
            Node a, b, c, d;
            divide(*it, a, b, c, d);
            Node *ch[4] = {&a, &b, &c, &d};
            push_children(L, ch, cur, &nexpand);
            it = L.erase(it);
        }
        if ((int)L.size() >= N || (int)L.size() == prev) {
            finish = true;
        } else if ((int)L.size() + nexpand * 3 > N) {
            while (!finish) {
                prev = (int)L.size();
                SizePtr todo = cur;
                cur.clear();
#ifdef TIE_CREATION
                std::sort(todo.begin(), todo.end(), [](const std::pair<int, Node *> &a, const std::pair<int, Node *> &b) {
                    return a.first != b.first ? a.first < b.first : a.second->seq < b.second->seq;
                });
#elif defined(TIE_SIM)
                std::sort(todo.begin(), todo.end(), [](const std::pair<int, Node *> &a, const std::pair<int, Node *> &b) {
                    return a.first != b.first ? a.first < b.first : g_sim.vaddr(a.second) < g_sim.vaddr(b.second);
                });
#else
                std::sort(todo.begin(), todo.end());   // (size, real address)
#endif
                for (int j = (int)todo.size() - 1; j >= 0; --j) {
                    Node a, b, c, d;
                    divide(*todo[j].second, a, b, c, d);
                    Node *ch[4] = {&a, &b, &c, &d};
                    push_children(L, ch, cur, nullptr);
                    L.erase(todo[j].second->self);
                    if ((int)L.size() >= N) break;
                }
                if ((int)L.size() >= N || (int)L.size() == prev) finish = true;
            }
        }
    }
    Vec<Key> out;
    out.reserve(nfeatures);
    for (const Node &n : L) {
        const Key *best = &n.keys[0];
        for (size_t k = 1; k < n.keys.size(); ++k)
            if (n.keys[k].response > best->response) best = &n.keys[k];
        out.push_back(*best);
    }
    return out;
}

struct Level {
    int w, h, quota;
    std::vector<Key> cand;     // candidate index in class_id
    std::vector<int> cells;    // corners per visited cell, in cell order
};

struct Frame {
    std::vector<Level> lv;
};

int g_nlevels, g_nfeatures;

// One frame of operator() up to the trees; out[l] = the selected candidates.
void run_frame(const Frame &f, std::vector<void *> &pyr, std::vector<std::vector<int>> &out) {
    const int E = 19;
    // Frame's scale tables (Frame.cc: four vector<float> copies) and
    // ComputePyramid's level buffers (ORBextractor.cc:1152-1185): each level a
    // new (w + 2E) x (h + 2E) buffer that replaces (frees) the previous
    // frame's, plus the resize's coefficient buffer for levels >= 1
    Vec<Vec<float>> tables(4, Vec<float>(g_nlevels, 1.f));
    for (int l = 0; l < g_nlevels; ++l) {
        void *m = raw_alloc((size_t)(f.lv[l].w + 2 * E) * (f.lv[l].h + 2 * E) + 64);
        raw_free(pyr[l]);
        pyr[l] = m;
        if (l > 0) {
            void *tmp = raw_alloc((size_t)(f.lv[l].w + f.lv[l].h) * 8 + 64);
            raw_free(tmp);
        }
    }
    Vec<Vec<Key>> all;
    all.resize(g_nlevels);
    out.assign(g_nlevels, {});
    for (int l = 0; l < g_nlevels; ++l) {
        const Level &L = f.lv[l];
        Vec<Key> todo;
        todo.reserve((size_t)g_nfeatures * 10);
        size_t k = 0;
        for (int cnt : L.cells) {
            Vec<Key> cell;   // cv::FAST's push_back per corner
            for (int i = 0; i < cnt; ++i) cell.push_back(L.cand[k + i]);
            for (const Key &c : cell) todo.push_back(c);
            k += cnt;
        }
        Vec<Key> &kps = all[l];
        kps.reserve(g_nfeatures);
        kps = tree(todo, E - 3, L.w - E + 3, E - 3, L.h - E + 3, L.quota, g_nfeatures);
        for (const Key &c : kps) out[l].push_back(c.class_id);
    }
}

bool rd(FILE *fp, void *p, size_t n) { return std::fread(p, 1, n, fp) == n; }

}  // namespace

int main(int argc, char **argv) {
    if (argc < 2) return 2;
    FILE *fp = std::fopen(argv[1], "rb");
    if (!fp) return 2;
    int32_t hdr[3];
    if (!rd(fp, hdr, sizeof hdr)) return 2;
    g_nlevels = hdr[0];
    g_nfeatures = hdr[1];
    const int nframes = hdr[2];
    std::vector<Frame> frames(nframes);
    for (Frame &f : frames) {
        f.lv.resize(g_nlevels);
        for (Level &L : f.lv) {
            int32_t h5[5];
            if (!rd(fp, h5, sizeof h5)) return 2;
            L.w = h5[0]; L.h = h5[1]; L.quota = h5[2];
            std::vector<int32_t> xys(3 * (size_t)h5[3]);
            L.cells.resize(h5[4]);
            if (!rd(fp, xys.data(), 4 * xys.size()) || !rd(fp, L.cells.data(), 4 * L.cells.size())) return 2;
            L.cand.resize(h5[3]);
            for (int i = 0; i < h5[3]; ++i)
                // (cell coordinates shifted as ComputeKeyPointsOctTree leaves
                // them: relative to minBorderX = minBorderY = 16)
                L.cand[i] = {(float)(xys[3 * i] - 16), (float)(xys[3 * i + 1] - 16), 7.f, -1.f, (float)xys[3 * i + 2],
                             0, i};
        }
    }
    std::fclose(fp);
    std::vector<std::vector<std::vector<int>>> res(nframes);
    // (the input sits in the main arena; the replay runs in a fresh thread)
    std::thread t([&] {
        std::vector<void *> pyr(g_nlevels, nullptr);
        for (int i = 0; i < nframes; ++i) run_frame(frames[i], pyr, res[i]);
        for (void *p : pyr) raw_free(p);
    });
    t.join();
    for (int i = 0; i < nframes; ++i)
        for (int l = 0; l < g_nlevels; ++l) {
            std::printf("%d %d %zu", i, l, res[i][l].size());
            for (int s : res[i][l]) std::printf(" %d", s);
            std::printf("\n");
        }
    return 0;
}
