// orbx_oracle_shim.cpp -- TEST INFRASTRUCTURE ONLY.  The orbx_* entry points
// the reference-side forwarders (integration/) call, answered by the CPU
// oracle (oracle/orbx_oracle.h), so tests/cxx/forwarders_test.cpp can check
// the forwarders' own work (table construction, result application, map
// edits) on a machine without a GPU.  It never ships: the product links
// liborbx.so, whose device results the GPU run of the same test compares.
#include <cstring>
#include <set>
#include <vector>

#include "orbx.h"
#include "orbx_oracle.h"

static_assert(sizeof(orbx_keypoint) == sizeof(orbo_keypoint), "keypoint layouts");
static_assert(sizeof(orbx_proj_query) == sizeof(orbo_proj_query), "query layouts");
static_assert(sizeof(orbx_ba_edge) == sizeof(orbo_ba_edge), "edge layouts");

namespace {
const orbo_keypoint *K(const orbx_keypoint *k) { return reinterpret_cast<const orbo_keypoint *>(k); }
const orbo_proj_query *Q(const orbx_proj_query *q) { return reinterpret_cast<const orbo_proj_query *>(q); }
}  // namespace

extern "C" {

const char *orbx_strerror(int code) { return code == ORBX_OK ? "ok" : "error (oracle shim)"; }

int orbx_descriptor_distance(const uint8_t *a, const uint8_t *b) { return orbo_descriptor_distance(a, b); }

int orbx_search_for_initialization(int, const orbx_keypoint *k1, const uint8_t *d1, int n1, const orbx_keypoint *k2,
                                   const uint8_t *d2, int n2, int img_w, int img_h, float *prev_xy,
                                   int32_t *matches12, int window, float nnratio, int check_ori, int *nmatches) {
    *nmatches = orbo_search_for_initialization(K(k1), d1, n1, K(k2), d2, n2, img_w, img_h, prev_xy, matches12, window,
                                               nnratio, check_ori);
    return ORBX_OK;
}

int orbx_search_for_initialization_bounds(int, const orbx_keypoint *k1, const uint8_t *d1, int n1,
                                          const orbx_keypoint *k2, const uint8_t *d2, int n2, float min_x,
                                          float max_x, float min_y, float max_y, float *prev_xy, int32_t *matches12,
                                          int window, float nnratio, int check_ori, int *nmatches) {
    *nmatches = orbo_search_for_initialization_bounds(K(k1), d1, n1, K(k2), d2, n2, min_x, max_x, min_y, max_y,
                                                      prev_xy, matches12, window, nnratio, check_ori);
    return ORBX_OK;
}

int orbx_search_by_projection(int, int variant, const orbx_match_frame *f, const orbx_proj_query *q,
                              const uint8_t *qdesc, int nq, int th_dist, float nnratio, int check_ori, int32_t *q_idx,
                              int32_t *q_dist, int32_t *kp_final, int *nmatches) {
    *nmatches = orbo_search_by_projection(variant, K(f->keys), f->desc, f->uright, f->mp_state, f->inv_sigma2, f->n,
                                          f->min_x, f->max_x, f->min_y, f->max_y, Q(q), qdesc, nq, th_dist, nnratio,
                                          check_ori, q_idx, q_dist, kp_final);
    return ORBX_OK;
}

int orbx_search_by_sim3(int, const orbx_match_frame *a, const orbx_match_frame *b, const orbx_proj_query *q1,
                        const uint8_t *qd1, const orbx_proj_query *q2, const uint8_t *qd2, int th_dist,
                        int32_t *matches12, int *nfound) {
    *nfound = orbo_search_by_sim3(K(a->keys), a->desc, a->n, K(b->keys), b->desc, b->n, a->min_x, a->max_x, a->min_y,
                                  a->max_y, b->min_x, b->max_x, b->min_y, b->max_y, Q(q1), qd1, Q(q2), qd2, th_dist,
                                  matches12);
    return ORBX_OK;
}

int orbx_search_by_bow(int, int variant, const orbx_bow_side *a, const orbx_bow_side *b, float nnratio,
                       int check_ori, const float *tri, int nlevels, int32_t *match_a, int32_t *match_b,
                       int *nmatches) {
    *nmatches = orbo_search_by_bow(variant, K(a->keys), a->desc, a->flags, a->n, a->node_ids, a->node_offsets,
                                   a->node_features, a->nnodes, K(b->keys), b->desc, b->flags, b->n, b->node_ids,
                                   b->node_offsets, b->node_features, b->nnodes, nnratio, check_ori, tri, nlevels,
                                   match_a, match_b);
    return ORBX_OK;
}

int orbx_search_by_projection_batch(int dev, int variant, orbx_proj_problem *pr, int np, int th_dist, float nnratio,
                                    int check_ori) {
    for (int k = 0; k < np; ++k)
        orbx_search_by_projection(dev, variant, &pr[k].frame, pr[k].queries, pr[k].qdesc, pr[k].nq, th_dist, nnratio,
                                  check_ori, pr[k].q_idx, pr[k].q_dist, pr[k].kp_final, &pr[k].nmatches);
    return ORBX_OK;
}

int orbx_search_by_bow_batch(int dev, int variant, orbx_bow_problem *pr, int np, float nnratio, int check_ori,
                             int nlevels) {
    for (int k = 0; k < np; ++k)
        orbx_search_by_bow(dev, variant, &pr[k].a, &pr[k].b, nnratio, check_ori, pr[k].tri, nlevels, pr[k].match_a,
                           pr[k].match_b, &pr[k].nmatches);
    return ORBX_OK;
}

int orbx_local_ba(int, const float *Tcw, const uint8_t *fixed, int ncam, const float *Xw, int npt,
                  const orbx_ba_edge *edges, int ne, int iters1, int iters2, float *Tcw_out, float *Xw_out,
                  uint8_t *outlier, int *iterations) {
    orbo_local_ba(Tcw, fixed, ncam, Xw, npt, reinterpret_cast<const orbo_ba_edge *>(edges), ne, iters1, iters2,
                  Tcw_out, Xw_out, outlier, iterations);
    return ORBX_OK;
}

// the database: the oracle's literal KeyFrameDatabase plus the id checks of orbx_kfdb_add
struct orbx_kfdb {
    void *db;
    std::set<uint64_t> ids;
};

int orbx_kfdb_create(int, orbx_kfdb **out) {
    *out = new orbx_kfdb{orbo_kfdb_create(1 << 16), {}};
    return ORBX_OK;
}
void orbx_kfdb_destroy(orbx_kfdb *d) {
    if (!d) return;
    orbo_kfdb_destroy(d->db);
    delete d;
}
int orbx_kfdb_add(orbx_kfdb *d, uint64_t id, const uint32_t *w, const double *v, int n) {
    for (int i = 0; i < n; ++i)
        if (w[i] >= (1u << 16)) return ORBX_EINVAL;
    if (!d->ids.insert(id).second) return ORBX_EINVAL;
    orbo_kfdb_add(d->db, id, w, v, n);
    return ORBX_OK;
}
int orbx_kfdb_erase(orbx_kfdb *d, uint64_t id) {
    if (!d->ids.erase(id)) return ORBX_OK;
    orbo_kfdb_erase(d->db, id);
    return ORBX_OK;
}
int orbx_kfdb_clear(orbx_kfdb *d) {
    d->ids.clear();
    orbo_kfdb_clear(d->db);
    return ORBX_OK;
}
int orbx_kfdb_size(const orbx_kfdb *d) { return (int)d->ids.size(); }
static int detect(orbx_kfdb *d, int reloc, uint64_t qid, const uint32_t *w, const double *v, int n,
                  const uint64_t *conn, int nconn, float ms, orbx_covis_fn covis, void *ctx, uint64_t *out, int cap,
                  int *n_out) {
    std::vector<uint64_t> all(d->ids.size() + 1);
    const int k = orbo_kfdb_detect(d->db, reloc, qid, w, v, n, conn, nconn, ms, covis, ctx, all.data(),
                                   (int)all.size());
    *n_out = k;
    if (k > cap) return ORBX_ERANGE;
    std::memcpy(out, all.data(), sizeof(uint64_t) * (size_t)k);
    return ORBX_OK;
}
int orbx_kfdb_detect_loop_candidates(orbx_kfdb *d, uint64_t qid, const uint32_t *w, const double *v, int n,
                                     const uint64_t *conn, int nconn, float ms, orbx_covis_fn covis, void *ctx,
                                     uint64_t *out, int cap, int *n_out) {
    return detect(d, 0, qid, w, v, n, conn, nconn, ms, covis, ctx, out, cap, n_out);
}
int orbx_kfdb_detect_relocalization_candidates(orbx_kfdb *d, uint64_t qid, const uint32_t *w, const double *v,
                                               int n, orbx_covis_fn covis, void *ctx, uint64_t *out, int cap,
                                               int *n_out) {
    return detect(d, 1, qid, w, v, n, nullptr, 0, 0.f, covis, ctx, out, cap, n_out);
}

void orbx_vocab_destroy(orbx_vocab *) {}

int orbx_undistort_keypoints(int, const orbx_keypoint *kps, int n, const float *K_, const float *dist, int ncoef,
                             orbx_keypoint *kps_un) {
    std::vector<float> in(2 * (size_t)n), out(2 * (size_t)n);
    for (int i = 0; i < n; ++i) { in[2 * i] = kps[i].x; in[2 * i + 1] = kps[i].y; }
    orbo_undistort_points(in.data(), n, K_, dist, ncoef, out.data());
    for (int i = 0; i < n; ++i) { kps_un[i] = kps[i]; kps_un[i].x = out[2 * i]; kps_un[i].y = out[2 * i + 1]; }
    return ORBX_OK;
}

int orbx_stereo_from_rgbd(int, const orbx_keypoint *k, const orbx_keypoint *ku, int n, const float *dmap, int w,
                          int h, size_t pitch, float mbf, float *uright, float *depth, int *kept) {
    orbo_stereo_from_rgbd(K(k), K(ku), n, dmap, w, h, pitch, mbf, uright, depth);
    *kept = 0;
    for (int i = 0; i < n; ++i) *kept += depth[i] > 0;
    return ORBX_OK;
}

// needs the extractors' device pyramids: not answerable on the CPU
int orbx_compute_stereo_matches(orbx_extractor *, orbx_extractor *, const orbx_keypoint *, const uint8_t *, int,
                                const orbx_keypoint *, const uint8_t *, int, float, float, float *, float *, int *) {
    return ORBX_ENODEV;
}

}  // extern "C"
