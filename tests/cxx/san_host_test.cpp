// ASan + UBSan driver for the host side of the C ABI (include/orbx.h): the
// library's objects are compiled with -Xarch_host -fsanitize=address,undefined
// (device code unchanged) and linked into this executable, which runs without
// a GPU: argument validation of every entry point that checks before touching
// the device, DescriptorDistance, the error strings, and the two DBoW2
// vocabulary loaders (TemplatedVocabulary.h:1351-1425 text, :1473-1547 binary)
// on valid and malformed files -- the host code that parses untrusted input.
//   san_host_test TMPDIR      (tests/test_sanitizers.py)
#include "orbx.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

static int failures = 0;
#define EXPECT(c)                                                              \
    do {                                                                       \
        if (!(c)) { std::fprintf(stderr, "FAILED %s:%d %s\n", __FILE__, __LINE__, #c); ++failures; } \
    } while (0)

static uint32_t st = 12345;
static uint32_t rnd() { st = st * 1664525u + 1013904223u; return st >> 8; }

struct Tree { int k, L; std::vector<int> parent; std::vector<int> leaf; std::vector<uint8_t> desc; std::vector<double> w; };

static Tree make_tree(int k, int L) {
    Tree t{k, L, {0}, {0}, std::vector<uint8_t>(32, 0), {0.0}};
    std::vector<int> level{0};
    for (int d = 1; d <= L; ++d) {
        std::vector<int> next;
        for (int p : level)
            for (int c = 0; c < k; ++c) {
                next.push_back((int)t.parent.size());
                t.parent.push_back(p);
                t.leaf.push_back(d == L);
                for (int i = 0; i < 32; ++i) t.desc.push_back((uint8_t)rnd());
                t.w.push_back(d == L ? 0.25 + (rnd() % 1000) / 997.0 : 0.0);
            }
        level = next;
    }
    return t;
}

static void write_text(const std::string &p, const Tree &t, const char *extra = "") {
    FILE *f = std::fopen(p.c_str(), "w");
    std::fprintf(f, "%d %d 0 0\n", t.k, t.L);
    for (size_t n = 1; n < t.parent.size(); ++n) {
        std::fprintf(f, "%d %d", t.parent[n], t.leaf[n]);
        for (int i = 0; i < 32; ++i) std::fprintf(f, " %d", t.desc[32 * n + i]);
        std::fprintf(f, " %.17g\n", t.w[n]);
    }
    std::fputs(extra, f);
    std::fclose(f);
}

static void write_bin(const std::string &p, const Tree &t, size_t truncate = 0) {
    std::vector<uint8_t> b;
    const int32_t h[4] = {t.k, t.L, 0, 0};
    b.insert(b.end(), (const uint8_t *)h, (const uint8_t *)h + 16);
    for (size_t n = 1; n < t.parent.size(); ++n) {
        const int32_t pid = t.parent[n];
        const uint8_t lf = (uint8_t)t.leaf[n];
        b.insert(b.end(), (const uint8_t *)&pid, (const uint8_t *)&pid + 4);
        b.push_back(lf);
        b.insert(b.end(), &t.desc[32 * n], &t.desc[32 * n] + 32);
        b.insert(b.end(), (const uint8_t *)&t.w[n], (const uint8_t *)&t.w[n] + 8);
    }
    if (truncate) b.resize(b.size() - truncate);
    FILE *f = std::fopen(p.c_str(), "wb");
    std::fwrite(b.data(), 1, b.size(), f);
    std::fclose(f);
}

static void write_raw(const std::string &p, const std::string &s) {
    FILE *f = std::fopen(p.c_str(), "wb");
    std::fwrite(s.data(), 1, s.size(), f);
    std::fclose(f);
}

static int load_and_check(const std::string &p, int fmt, const Tree *want) {
    orbx_vocab *v = nullptr;
    const int rc = orbx_vocab_load(0, p.c_str(), fmt, &v);
    if (rc != ORBX_OK) return rc;
    int k = 0, L = 0, sc = 0, wt = 0, nn = 0, nw = 0;
    EXPECT(orbx_vocab_info(v, &k, &L, &sc, &wt, &nn, &nw) == ORBX_OK);
    if (want) {
        EXPECT(k == want->k && L == want->L && nn == (int)want->parent.size());
        std::vector<int32_t> par(nn);
        std::vector<uint8_t> lf(nn), d(32 * (size_t)nn);
        std::vector<double> w(nn);
        EXPECT(orbx_vocab_export(v, par.data(), lf.data(), d.data(), w.data(), nn - 1) == ORBX_ERANGE);
        EXPECT(orbx_vocab_export(v, par.data(), lf.data(), d.data(), w.data(), nn) == ORBX_OK);
        for (int n = 1; n < nn; ++n) {
            EXPECT(par[n] == want->parent[n] && (lf[n] != 0) == (want->leaf[n] != 0));
            EXPECT(std::memcmp(&d[32 * (size_t)n], &want->desc[32 * (size_t)n], 32) == 0);
            EXPECT(w[n] == want->w[n]);
        }
    }
    orbx_vocab_destroy(v);
    return rc;
}

int main(int argc, char **argv) {
    if (argc < 2) return 2;
    const std::string dir = argv[1];
    // error strings and plain host entry points
    for (int c : {ORBX_OK, ORBX_EIO, ORBX_ENOMEM, ORBX_EINVAL, ORBX_ERANGE, ORBX_ENODEV, -999, 7})
        EXPECT(orbx_strerror(c) != nullptr);
    uint8_t a[32], b[32];
    for (int t = 0; t < 1000; ++t) {
        int ref = 0;
        for (int i = 0; i < 32; ++i) { a[i] = (uint8_t)rnd(); b[i] = (uint8_t)rnd(); ref += __builtin_popcount(a[i] ^ b[i]); }
        EXPECT(orbx_descriptor_distance(a, b) == ref);
    }
    // argument validation before any device work
    EXPECT(orbx_extractor_create(0, 0, 1.2f, 8, 20, 7) == nullptr);
    EXPECT(orbx_extractor_create(0, 1000, 1.2f, 0, 20, 7) == nullptr);
    EXPECT(orbx_extractor_create(0, 1000, 0.5f, 8, 20, 7) == nullptr);
    int n = 0;
    EXPECT(orbx_extract(nullptr, nullptr, 0, 0, 0, nullptr, nullptr, 0, &n) == ORBX_EINVAL);
    EXPECT(orbx_extractor_reserve(nullptr, 640, 480, 1) == ORBX_EINVAL);
    EXPECT(orbx_extractor_kp_stride(nullptr) == ORBX_EINVAL);
    int64_t nb = 0;
    EXPECT(orbx_batch_pack_device(nullptr, nullptr, 0, &nb, nullptr) == ORBX_EINVAL);
    EXPECT(orbx_vocab_load(0, nullptr, 0, nullptr) == ORBX_EINVAL);
    orbx_vocab *v = nullptr;
    EXPECT(orbx_vocab_load(0, (dir + "/does_not_exist").c_str(), 0, &v) == ORBX_EINVAL);
    EXPECT(orbx_vocab_load(0, (dir + "/does_not_exist").c_str(), 2, &v) == ORBX_EINVAL);
    // vocabulary loaders: valid trees round-trip through export
    for (auto kl : {std::pair<int, int>{2, 1}, {3, 2}, {10, 2}, {5, 4}}) {
        const Tree t = make_tree(kl.first, kl.second);
        write_text(dir + "/v.txt", t);
        EXPECT(load_and_check(dir + "/v.txt", 0, &t) == ORBX_OK);
        write_text(dir + "/v2.txt", t, "\n\n   \n");          // trailing blank lines are skipped
        EXPECT(load_and_check(dir + "/v2.txt", 0, &t) == ORBX_OK);
        write_bin(dir + "/v.bin", t);
        EXPECT(load_and_check(dir + "/v.bin", 1, &t) == ORBX_OK);
        write_bin(dir + "/vt.bin", t, 3);                   // truncated last record: ends the file
        EXPECT(load_and_check(dir + "/vt.bin", 1, nullptr) == ORBX_OK);
    }
    // malformed input
    const char *bad_text[] = {"", "x y z w\n", "3 2 0\n", "30 2 0 0\n", "3 0 0 0\n", "3 2 9 0\n", "3 2 0 9\n",
                              "-3 2 0 0\n",
                              "3 2 0 0\n5 0 1 2 3\n",                       // parent out of range
                              "3 2 0 0\n0 1 1 2 3\n",                       // truncated record
                              "3 2 0 0\n-1 1 0 0 0 0 0 0 0 0 0 0 0 0 0 0 0 0 0 0 0 0 0 0 0 0 0 0 0 0 0 0 0 0 1.0\n",
                              "3 2 0 0\n0 1 99999999999999999999 0\n"};
    for (const char *s : bad_text) {
        write_raw(dir + "/bad.txt", s);
        const int rc = load_and_check(dir + "/bad.txt", 0, nullptr);
        EXPECT(rc == ORBX_EINVAL || rc == ORBX_OK);
    }
    std::string hdr(16, '\0');
    const int32_t h1[4] = {1, 2, 0, 0}, h2[4] = {3, 2, 0, 0}, h3[4] = {3, 11, 0, 0};
    write_raw(dir + "/bad.bin", std::string((const char *)h1, 16));
    EXPECT(load_and_check(dir + "/bad.bin", 1, nullptr) == ORBX_EINVAL);      // k < 2
    write_raw(dir + "/bad.bin", std::string((const char *)h3, 16));
    EXPECT(load_and_check(dir + "/bad.bin", 1, nullptr) == ORBX_EINVAL);      // L > 10
    write_raw(dir + "/bad.bin", std::string((const char *)h2, 12));
    EXPECT(load_and_check(dir + "/bad.bin", 1, nullptr) == ORBX_EINVAL);      // short header
    std::string rec((const char *)h2, 16);
    const int32_t badpid = 7;
    rec.append((const char *)&badpid, 4);
    rec.append(41, '\1');
    write_raw(dir + "/bad.bin", rec);
    EXPECT(load_and_check(dir + "/bad.bin", 1, nullptr) == ORBX_EINVAL);      // parent out of range
    for (int t = 0; t < 50; ++t) {                                            // random bytes after a valid header
        std::string r((const char *)h2, 16);
        const int len = (int)(rnd() % 400);
        for (int i = 0; i < len; ++i) r.push_back((char)(rnd() & 0xff));
        write_raw(dir + "/rnd.bin", r);
        const int rc = load_and_check(dir + "/rnd.bin", 1, nullptr);
        EXPECT(rc == ORBX_EINVAL || rc == ORBX_OK);
        write_raw(dir + "/rnd.txt", "3 2 0 0\n" + r.substr(16));
        const int rc2 = load_and_check(dir + "/rnd.txt", 0, nullptr);
        EXPECT(rc2 == ORBX_EINVAL || rc2 == ORBX_OK);
    }
    if (failures) return 1;
    std::printf("sanitize host ok\n");
    return 0;
}
