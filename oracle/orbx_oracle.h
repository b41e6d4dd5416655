/*
 * orbx_oracle.h -- CPU restatement of the ORB-SLAM2 feature hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (orb_slam_2_ros_amd/,
 * include/) links or calls this library; only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg load it, as the checker / CPU baseline.
 *
 * PARITY STATUS: UNPINNED against the reference binary.  The reference
 * (wjjcdy/orb_slam_2_ros) ships no tests, fixtures or golden vectors, and its
 * extractor needs OpenCV (not vendored, absent here), so it cannot be built in
 * this container.  This file restates (a) the reference's own logic from its
 * sources (file:line cited per function) and (b) the OpenCV 3.2.0 primitives it
 * calls (x86-64 SSE2 code paths, IPP off: the Ubuntu 18.04 / ROS Melodic build
 * named by reference docker/melodic/Dockerfile:1), spelled out in DESIGN.md §3.
 * sinf/cosf are taken from glibc directly, as the reference does.
 */
#ifndef ORBX_ORACLE_H
#define ORBX_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Same 28-byte layout as cv::KeyPoint (pt.x, pt.y, size, angle, response,
 * octave, class_id) and as orbx_keypoint in include/orbx.h. */
typedef struct {
    float x, y, size, angle, response;
    int32_t octave, class_id;
} orbo_keypoint;

/* ---- primitives (KAT targets) ---- */
int   orbo_cv_round(float v);
float orbo_fast_atan2(float y, float x);
void  orbo_sincosf(float a, float *s, float *c);
int   orbo_descriptor_distance(const uint8_t *a, const uint8_t *b);
/* cv::resize(INTER_LINEAR, 8U) restated (OpenCV 3.2 SSE2). */
void  orbo_resize_linear(const uint8_t *src, int sw, int sh, size_t sstep,
                         uint8_t *dst, int dw, int dh, size_t dstep);
/* cv::GaussianBlur(7x7, sigma 2, BORDER_REFLECT_101) on a borderless image. */
void  orbo_gauss7(const uint8_t *src, int w, int h, size_t sstep,
                  uint8_t *dst, size_t dstep);
/* cv::FAST(TYPE_9_16, nonmax=true) on a sub-image; returns #keypoints written
 * as (x, y, score) triples (row-major order), up to cap. */
int   orbo_fast(const uint8_t *img, int w, int h, size_t step, int threshold,
                int32_t *xys, int cap);

/* ---- extractor (ORBextractor) ---- */
/* Level geometry of ORBextractor(nfeat, scale, nlev, ...): per level the
 * width, height, feature quota and scale factor (ORBextractor.cc:416-455,
 * 1157-1159). Arrays have nlevels entries. */
void  orbo_levels(int w, int h, int nfeatures, float scaleFactor, int nlevels,
                  int *lw, int *lh, int *quota, float *scale);
/* ComputePyramid: writes all levels contiguously (level l at sum of previous
 * w*h, rows packed).  Returns total bytes. */
size_t orbo_pyramid(const uint8_t *img, int w, int h, size_t step,
                    float scaleFactor, int nlevels, uint8_t *out);
/* FAST candidates of one level, cell loop of ComputeKeyPointsOctTree
 * (ORBextractor.cc:796-863): (x, y, score) in level pixel coordinates, in the
 * order the reference pushes them.  Returns the count (or -needed if > cap). */
int   orbo_level_candidates(const uint8_t *lvl, int w, int h, int iniTh, int minTh,
                            int32_t *xys, int cap);
/* The same plus each visited cell's corner count, in cell order (diagnostic:
 * tools/tie_heap replays the per-cell vector<KeyPoint> allocations). */
int   orbo_level_candidates_cells(const uint8_t *lvl, int w, int h, int iniTh, int minTh,
                                  int32_t *xys, int cap, int32_t *cell_counts, int cell_cap, int *ncells);
/* DistributeOctTree on a candidate list (ORBextractor.cc:561-787): writes the
 * selected candidate indices in output order; returns the count. */
void  orbo_tie_stats(int64_t out[9], int reset);   /* diagnostic, see orbx_oracle.cpp */
void  orbo_set_tie_mode(int mode);                  /* diagnostic: 0 = the restatement's rule */
int   orbo_distribute(const int32_t *xys, int n, int w, int h, int N, int32_t *sel);
/* Full operator() (ORBextractor.cc:1083-1149).  Returns 0, or -1 if cap is
 * too small (then *n_out holds the required count). */
int   orbo_extract(const uint8_t *img, int w, int h, size_t step,
                   int nfeatures, float scaleFactor, int nlevels,
                   int iniThFAST, int minThFAST,
                   orbo_keypoint *kps, uint8_t *desc, int cap, int *n_out);

/* ---- matcher (ORBmatcher::SearchForInitialization, ORBmatcher.cc:406-521) ----
 * Frames are described by keypoints (undistorted == distorted, k1 = 0) and
 * descriptors; the 64x48 grid is built from (img_w, img_h) as
 * Frame::AssignFeaturesToGrid does (Frame.cc:239-256, 415-425).
 * prev_xy (2*n1 floats) is read and updated like vbPrevMatched; matches12
 * (n1 ints) receives vnMatches12.  Returns nmatches. */
int   orbo_search_for_initialization(const orbo_keypoint *k1, const uint8_t *d1, int n1,
                                     const orbo_keypoint *k2, const uint8_t *d2, int n2,
                                     int img_w, int img_h,
                                     float *prev_xy, int32_t *matches12,
                                     int window, float nnratio, int check_ori);
/* The same over explicit bounds (mnMinX, mnMaxX, mnMinY, mnMaxY; a distorted
 * camera's, Frame::ComputeImageBounds, Frame.cc:475-499). */
int   orbo_search_for_initialization_bounds(const orbo_keypoint *k1, const uint8_t *d1, int n1,
                                            const orbo_keypoint *k2, const uint8_t *d2, int n2,
                                            float min_x, float max_x, float min_y, float max_y,
                                            float *prev_xy, int32_t *matches12,
                                            int window, float nnratio, int check_ori);

/* ---- stereo (Frame::ComputeStereoMatches, Frame.cc:502-676) ----
 * pyrL / pyrR: all levels packed as orbo_pyramid writes them, level sizes
 * lw/lh; scale / inv_scale = mvScaleFactors / mvInvScaleFactors.  uright and
 * depth (nl floats) receive mvuRight / mvDepth.  Returns the count kept. */
int   orbo_compute_stereo_matches(const uint8_t *pyrL, const uint8_t *pyrR, const int *lw, const int *lh,
                                  int nlevels, const float *scale, const float *inv_scale,
                                  const orbo_keypoint *kl, const uint8_t *dl, int nl,
                                  const orbo_keypoint *kr, const uint8_t *dr, int nr,
                                  float mbf, float mb, float *uright, float *depth);
/* Frame::ComputeStereoFromRGBD (Frame.cc:679-701); dmap is CV_32F. */
void  orbo_stereo_from_rgbd(const orbo_keypoint *kps, const orbo_keypoint *kps_un, int n,
                            const float *dmap, int w, int h, size_t pitch_bytes, float mbf,
                            float *uright, float *depth);

/* ---- projection matchers (ORBmatcher.cc:45-129, 291-404, 827-1102, 1330-1601) ----
 * Queries carry the projection the reference computes in the caller or at
 * the top of each loop body (u, v, window radius, stereo u, level range of
 * GetFeaturesInArea, the query keypoint's angle).  flags: bit0 = query taken
 * (the reference's own skip tests passed), bit1 = assigning it blocks the
 * keypoint for later queries (its Observations() > 0).  mp_state per
 * keypoint: bit0 = mvpMapPoints[i] / vpMatched[i] non-NULL, bit1 = that point's
 * Observations() > 0.  Outputs: q_idx / q_dist per query (the keypoint it was
 * assigned, -1 if none or if the rotation check dropped its bin), kp_final per
 * keypoint (query whose point it holds at the end, -1 untouched, -2 cleared
 * by the rotation check; untouched by the Fuse variants, whose map updates
 * stay with the caller).  Returns nmatches / nFused as the reference counts. */
typedef struct {
    float u, v, radius, ur, ur_tol;
    int32_t min_level, max_level;
    float angle;
    int32_t flags;
} orbo_proj_query;
enum { ORBO_PROJ_LOCALMAP = 0, ORBO_PROJ_LASTFRAME = 1, ORBO_PROJ_KEYFRAME = 2, ORBO_PROJ_SIM3 = 3,
       ORBO_PROJ_FUSE = 4, ORBO_PROJ_FUSE_SIM3 = 5 };
int   orbo_search_by_projection(int variant, const orbo_keypoint *keys, const uint8_t *desc, const float *uright,
                                const uint8_t *mp_state, const float *inv_sigma2, int n, float min_x, float max_x,
                                float min_y, float max_y, const orbo_proj_query *q, const uint8_t *qdesc, int nq,
                                int th_dist, float nnratio, int check_ori, int32_t *q_idx, int32_t *q_dist,
                                int32_t *kp_final);

/* SearchBySim3 (ORBmatcher.cc:1104-1328): q1 has one row per KF1 map-point
 * slot (its projection into KF2), q2 one per KF2 slot (into KF1); the query's
 * level window is [min_level, max_level] = [pred-1, pred].  matches12[n1] = the
 * agreed KF2 index (-1 none).  Returns nFound. */
int   orbo_search_by_sim3(const orbo_keypoint *k1, const uint8_t *dsc1, int n1, const orbo_keypoint *k2,
                          const uint8_t *dsc2, int n2, float minx1, float maxx1, float miny1, float maxy1,
                          float minx2, float maxx2, float miny2, float maxy2, const orbo_proj_query *q1,
                          const uint8_t *qd1, const orbo_proj_query *q2, const uint8_t *qd2, int th_dist,
                          int32_t *matches12);

/* ---- BoW matchers (ORBmatcher.cc:160-289, 524-657, 659-825) ----
 * Side A = pKF / pKF1 (the outer loop), side B = F / pKF2.  Each side: keys,
 * descriptors, per-feature flags (bit0 usable: A of the SearchByBoW variants =
 * has a good map point; B of KF_FRAME = 1; B of KF_KF = has a good map point;
 * triangulation = no map point yet [and stereo when bOnlyStereo]; bit1 =
 * mvuRight >= 0), and the FeatureVector as CSR (ascending node ids, offsets,
 * feature indices).  tri (triangulation only): F12 row-major [9], epipole
 * ex, ey, then pKF2->mvScaleFactors[nlevels], pKF2->mvLevelSigma2[nlevels].
 * match_a[na] / match_b[nb] receive the pairs (-1 none); returns nmatches. */
enum { ORBO_BOW_KF_FRAME = 0, ORBO_BOW_KF_KF = 1, ORBO_BOW_TRIANGULATION = 2 };
int   orbo_search_by_bow(int variant, const orbo_keypoint *ka, const uint8_t *da, const uint8_t *fa, int na,
                         const uint32_t *ida, const int32_t *offa, const int32_t *feata, int nna,
                         const orbo_keypoint *kb, const uint8_t *db, const uint8_t *fb, int nb,
                         const uint32_t *idb, const int32_t *offb, const int32_t *featb, int nnb,
                         float nnratio, int check_ori, const float *tri, int nlevels,
                         int32_t *match_a, int32_t *match_b);

/* DBoW2 TemplatedVocabulary<FORB>::transform(features, BowVector&,
 * FeatureVector&, levelsup) (TemplatedVocabulary.h:1140-1207, per feature
 * :1231-1272; BowVector::addWeight / addIfNotExist / normalize
 * BowVector.cpp; FeatureVector::addFeature FeatureVector.cpp:31-45).  The
 * vocabulary is given as loadFromTextFile / loadFromBinFile build it
 * (TemplatedVocabulary.h:1351-1425, 1473-1547): node 0 is the root, nodes
 * 1..n_nodes-1 in file order with parent (< own index), file leaf flag,
 * 32-B descriptor (row 0 unused) and weight; children in file order; word ids
 * in order of the leaf flags.  scoring / weighting are DBoW2's ScoringType /
 * WeightingType values.  Outputs: the BowVector as ascending (word, value);
 * the FeatureVector as ascending node ids with per-node feature lists (CSR,
 * fv_offsets[n_fv] = total).  Optional per-feature word / weight / node
 * (nullable).  A leaf shallower than L - levelsup leaves the reference's nid
 * unset (undefined); here it is the leaf.  Returns the number of words
 * (0 for an empty vocabulary: outputs cleared). */
int   orbo_vocab_transform(int L, int scoring, int weighting, int n_nodes, const int32_t *parent,
                           const uint8_t *is_leaf, const uint8_t *desc, const double *weight,
                           const uint8_t *features, int n, int levelsup,
                           uint32_t *bow_words, double *bow_values, int *n_bow,
                           uint32_t *fv_nodes, int32_t *fv_offsets, int32_t *fv_features, int *n_fv,
                           uint32_t *f_word, double *f_weight, uint32_t *f_node);
/* The same with the tree built once (CPU-baseline timing). */
void *orbo_vocab_prepare(int n_nodes, const int32_t *parent, const uint8_t *is_leaf);
void  orbo_vocab_release(void *tree);
int   orbo_vocab_transform_prepared(void *tree, int L, int scoring, int weighting, const uint8_t *desc,
                                    const double *weight, const uint8_t *features, int n, int levelsup,
                                    uint32_t *bow_words, double *bow_values, int *n_bow,
                                    uint32_t *fv_nodes, int32_t *fv_offsets, int32_t *fv_features, int *n_fv,
                                    uint32_t *f_word, double *f_weight, uint32_t *f_node);

/* ---- per-frame neighbours ---- */
/* MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:288-361) for np
 * points: point p's observation descriptors are rows offsets[p] ..
 * offsets[p+1]-1 of desc.  best[p] = the index (within the point's rows) of
 * the descriptor with the least median distance to the others (first on
 * ties), -1 for a point without descriptors. */
void  orbo_distinctive_descriptors(const uint8_t *desc, const int32_t *offsets, int np, int32_t *best);
/* Frame::UndistortKeyPoints (Frame.cc:438-469): cv::undistortPoints(K, D,
 * R = I, P = K) as OpenCV 3.2 computes it in double (5 fixed iterations;
 * coefficients k1 k2 p1 p2 [k3], ncoef 4 or 5).  k1 == 0: a plain copy.
 * xy in / out: n (x, y) float pairs. */
void  orbo_undistort_points(const float *xy_in, int n, const float *K /* row-major 3x3 */,
                            const float *dist, int ncoef, float *xy_out);
/* cv::cvtColor(CV_RGB2GRAY / BGR2GRAY / RGBA2GRAY / BGRA2GRAY) for 8U
 * (Tracking.cc:179-264): 14-bit fixed point, coefficients 4899 (R), 9617 (G),
 * 1868 (B), rounding 1 << 13.  channels 3 or 4; rgb 1 = R first. */
void  orbo_cvt_gray(const uint8_t *src, int w, int h, size_t spitch, int channels, int rgb,
                    uint8_t *dst, size_t dpitch);
/* Mat::convertTo(CV_32F, scale) of a 16U depth image (Tracking.cc:228-229):
 * dst = (float)src * scale in float. */
void  orbo_depth_to_float(const uint16_t *src, int w, int h, size_t spitch, float scale, float *dst,
                          size_t dpitch);

/* ---- keyframe database: KeyFrameDatabase.cc:31-236 restated
 * literally -- inverted file of std::lists in add order, the per-keyframe
 * query state (mnLoopQuery / mnLoopWords / mLoopScore and the reloc trio)
 * persisting across queries, L1Scoring::score (ScoringObject.cpp:23-66).
 * Keyframes are named by 64-bit ids; covisibility (GetBestCovisibilityKeyFrames
 * (10)) comes from a callback.  Scores the reference leaves uninitialised
 * start at 0 here. */
typedef int (*orbo_covis_fn)(void *ctx, uint64_t kf_id, uint64_t *out, int cap);
void *orbo_kfdb_create(int n_words);
void  orbo_kfdb_destroy(void *db);
void  orbo_kfdb_add(void *db, uint64_t kf_id, const uint32_t *words, const double *values, int n);
void  orbo_kfdb_erase(void *db, uint64_t kf_id);
void  orbo_kfdb_clear(void *db);
int   orbo_kfdb_detect(void *db, int reloc, uint64_t query_id, const uint32_t *words, const double *values, int n,
                       const uint64_t *connected, int n_connected, float min_score, orbo_covis_fn covis, void *ctx,
                       uint64_t *out, int cap);
double orbo_bow_score_l1(const uint32_t *w1, const double *v1, int n1, const uint32_t *w2, const double *v2, int n2);

/* ---- local bundle adjustment ----
 * Optimizer::LocalBundleAdjustment's optimisation (Optimizer.cc:517-900)
 * restated over g2o's Levenberg (optimization_algorithm_levenberg.cpp:60-160),
 * BlockSolver_6_3 with the Schur complement (block_solver.hpp:354-484), the
 * two projection edges (types_six_dof_expmap.cpp:109-230), Huber
 * (robust_kernel_impl.cpp:65-91) and SE3Quat (se3quat.h).  The sums follow a
 * fixed order (edge order per vertex, ascending point per camera pair, a dense
 * Cholesky of the reduced system with k-ascending dot products, the
 * forward solve's terms k-ascending and the backward solve's k-descending):
 * g2o's own order is unspecified (it sorts
 * edges of equal ids) and Eigen's sparse LDLT differs, so parity with g2o is
 * to rounding -- unpinned.  Edge layout as orbx_ba_edge in include/orbx.h. */
typedef struct {
    int32_t cam, point;
    float u, v, ur, inv_sigma2, fx, fy, cx, cy, bf;
} orbo_ba_edge;
int   orbo_local_ba(const float *Tcw, const uint8_t *fixed, int ncam, const float *Xw, int npt,
                    const orbo_ba_edge *edges, int ne, int iters1, int iters2, float *Tcw_out, float *Xw_out,
                    uint8_t *outlier, int *iterations);
int   orbo_ba_debug_step(const float *Tcw, const uint8_t *fixed, int ncam, const float *Xw, int npt,
                         const orbo_ba_edge *edges, int ne, int robust, double lambda, double *x_out,
                         double *chi2_out);

#ifdef __cplusplus
}
#endif
#endif
