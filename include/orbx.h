/*
 * orbx.h -- C ABI of liborbx.so, the MI355X (gfx950) ORB front end that stands
 * in for ORB-SLAM2's ORBextractor / ORBmatcher hot path
 * (reference: wjjcdy/orb_slam_2_ros, orb_slam2/include/ORBextractor.h and
 * orb_slam2/include/ORBmatcher.h).
 *
 * Plain C types only: pointers, sizes, status codes.  HIP streams are passed
 * as `void *` (a hipStream_t, or NULL for the library's own stream).  Every
 * function returns ORBX_OK (0) or a negative errno-style code; the reference
 * itself has no error channel, so its silent cases are
 * mapped explicitly and documented per function.
 *
 * The C++ drop-in adapters that re-expose ORB_SLAM2::ORBextractor /
 * ORB_SLAM2::ORBmatcher over these calls are shown in INTEGRATION.md.
 */
#ifndef ORBX_H
#define ORBX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORBX_OK 0
#define ORBX_EIO (-5)      /* HIP runtime / kernel failure */
#define ORBX_ENOMEM (-12)  /* device or host allocation failed */
#define ORBX_EINVAL (-22)  /* bad argument */
#define ORBX_ERANGE (-34)  /* output capacity too small (count still reported) */
#define ORBX_ENODEV (-19)  /* no usable gfx950 device */

/* Same layout and field order as cv::KeyPoint (28 bytes):
 * pt.x, pt.y, size, angle, response, octave, class_id. */
typedef struct orbx_keypoint {
    float x, y, size, angle, response;
    int32_t octave, class_id;
} orbx_keypoint;

typedef struct orbx_extractor orbx_extractor;

const char *orbx_strerror(int code);
int orbx_device_count(void);

/* Diagnostic counters of the calling thread's last host call, for tests (no
 * reference counterpart): "bow_repairs" -- in the last orbx_search_by_bow(_batch)
 * call, the A features whose two best B features (of a node of <= 64 B
 * features) included one an earlier A feature had taken, so that the exact
 * in-order pass over the untaken ones ran.  ORBX_EINVAL for an unknown name. */
int orbx_debug_counter(const char *name, int64_t *value);

/* ---- ORB_SLAM2::ORBextractor ------------------------------------------ */

/* ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST,
 *              int minThFAST)                         ORBextractor.h:51-52
 * Returns NULL on bad arguments or when no device is usable. */
orbx_extractor *orbx_extractor_create(int device, int nfeatures, float scaleFactor,
                                      int nlevels, int iniThFAST, int minThFAST);
void orbx_extractor_destroy(orbx_extractor *ex);

/* GetLevels / GetScaleFactor                          ORBextractor.h:63-67 */
int orbx_extractor_get_levels(const orbx_extractor *ex);
float orbx_extractor_get_scale_factor(const orbx_extractor *ex);
/* GetScaleFactors / GetInverseScaleFactors / GetScaleSigmaSquares /
 * GetInverseScaleSigmaSquares                          ORBextractor.h:69-83
 * which: 0 = mvScaleFactor, 1 = mvInvScaleFactor, 2 = mvLevelSigma2,
 * 3 = mvInvLevelSigma2.  Writes min(cap, nlevels) floats, returns nlevels. */
int orbx_extractor_get_scale_table(const orbx_extractor *ex, int which, float *out, int cap);
/* mnFeaturesPerLevel (protected in the reference; exposed for tests). */
int orbx_extractor_get_level_quotas(const orbx_extractor *ex, int32_t *out, int cap);

/* void operator()(InputArray image, InputArray mask, vector<KeyPoint>& kps,
 *                 OutputArray descriptors)           ORBextractor.h:59-61,
 *                                                    ORBextractor.cc:1083-1149
 * Host image in, host keypoints/descriptors out; synchronous.  The mask is
 * ignored by the reference and is therefore not a parameter.
 * An empty image (NULL, width or height 0) returns ORBX_OK with *n = -1 and
 * leaves kps/desc untouched, as the reference does (ORBextractor.cc:1086-1087).
 * If cap < the keypoint count, returns ORBX_ERANGE with *n = the count. */
int orbx_extract(orbx_extractor *ex, const uint8_t *image, int width, int height,
                 size_t pitch, orbx_keypoint *kps, uint8_t *desc, int cap, int *n);

/* std::vector<cv::Mat> mvImagePyramid (public member, ORBextractor.h:85):
 * host copy of level `level` of the last orbx_extract call (the 19-px border
 * of the reference's buffers is not materialised).  Writes rows of `w` bytes
 * at `out_pitch` stride when out != NULL; always reports w, h. */
int orbx_extractor_pyramid_level(orbx_extractor *ex, int level, uint8_t *out,
                                 size_t out_pitch, int *w, int *h);
/* The same for levels 0 .. nlevels-1 at once (out[l] rows of level l's width
 * at out_pitch[l]): one stream-ordered copy of every level into pinned
 * staging and one wait -- what an mvImagePyramid read costs after a call. */
int orbx_extractor_pyramid_host(orbx_extractor *ex, uint8_t *const *out, const size_t *out_pitch,
                                int nlevels);

/* ---- batched device API (many cameras / frames per launch) ------------- */

/* Plan buffers for width x height frames, up to max_batch per call. */
int orbx_extractor_reserve(orbx_extractor *ex, int width, int height, int max_batch);
/* Keypoint capacity per frame of the current plan (stride of the result arrays). */
int orbx_extractor_kp_stride(const orbx_extractor *ex);
/* Extract `batch` device-resident frames (frame b at d_images + b*frame_stride,
 * rows `pitch` bytes apart) on `stream`; asynchronous.  Results stay on the
 * device in the current result slot (see orbx_batch_results_device). */
int orbx_extract_batch_device(orbx_extractor *ex, const uint8_t *d_images,
                              int64_t frame_stride, int pitch, int batch, void *stream);
/* Device pointers of the current result slot: frame b's keypoints are
 * d_kps[b*kp_stride ...], descriptors d_desc[(b*kp_stride + i)*32 ...],
 * counts d_counts[b]. */
int orbx_batch_results_device(orbx_extractor *ex, const orbx_keypoint **d_kps,
                              const uint8_t **d_desc, const int32_t **d_counts);
/* Keyframe publication for the cross-stream exchange (config C5; the
 * reference's analogue is KeyFrameDatabase::add, KeyFrameDatabase.cc:41-48,
 * fed by LoopClosing::InsertKeyFrame, LoopClosing.cc:96): copies the current result slot into
 * one contiguous device buffer, ready for an RCCL all-gather --
 *   int32 counts[B] (padded to 64 B) | orbx_keypoint [B][kp_stride] |
 *   uint8 desc [B][kp_stride][32]
 * *bytes = the size of that layout (d_out may be NULL to query it).
 * Asynchronous on `stream`; ORBX_ERANGE if cap < *bytes. */
int orbx_batch_pack_device(orbx_extractor *ex, void *d_out, int64_t cap, int64_t *bytes, void *stream);
/* Synchronous host copy of frame b of the current result slot. */
int orbx_batch_download(orbx_extractor *ex, int frame, orbx_keypoint *kps, uint8_t *desc,
                        int cap, int *n);

/* Mono front-end step (the benchmark unit): extract the batch
 * into the next result slot, then, if the previous slot holds a batch of the
 * same size, run SearchForInitialization(F1 = previous frame b,
 * F2 = current frame b, vbPrevMatched = F1 keypoint positions) for every b.
 * Asynchronous on `stream`. */
int orbx_mono_step_device(orbx_extractor *ex, const uint8_t *d_images, int64_t frame_stride,
                          int pitch, int batch, int window, float nnratio, int check_ori,
                          void *stream);
/* Host copy of frame b's last match result: matches12 (n1 entries, F1 index ->
 * F2 index or -1), n1, nmatches. */
int orbx_mono_matches_download(orbx_extractor *ex, int frame, int32_t *matches12, int cap,
                               int *n1, int *nmatches);

/* Batch split: a step's batch runs as up to `parts` interleaved sub-batches
 * on internal streams forked from and joined to the launch stream (latency-
 * bound kernels of one part overlap the other's).  parts 1 or 2; 0 queries.
 * Returns the current setting.  Batches under 64 frames are never split. */
int orbx_extractor_split(orbx_extractor *ex, int parts);

/* Level pipeline (default off): a step's extraction runs in two level groups
 * on internal streams forked from and joined to the launch stream -- level 0's
 * FAST, quadtree and describe beside the resize chain and levels 1.. -- so
 * level 0's work overlaps the latency-bound resize chain.  on = 2, the deep
 * form: the side stream also takes FAST, quadtree and describe of levels 1..E
 * as soon as the resize chain has produced them (E: environment
 * ORBX_PIPE_EARLY, default 2; ORBX_PIPE_DESC=0 leaves their describe with the
 * other levels'), so the rest of the chain runs beside them.  Outputs are identical in
 * every form.  on: 2 / 1 / 0 sets, -1 queries; returns the current setting.
 * Stage times (orbx_extractor_stage_times) cover the extractor stages only
 * with the pipeline off. */
int orbx_extractor_pipeline(orbx_extractor *ex, int on);

/* Matcher overlap (default off): orbx_mono_step_device's SearchForInitialization
 * runs on an internal stream that the launch stream does not wait for, so it
 * overlaps the next step's resize / FAST / quadtree; the next extraction's
 * descriptor stage (the only writer of the result slot the matcher reads)
 * waits for it.  The step's matches are complete when the device is idle or a
 * download call (orbx_mono_matches_download) returns, not when the launch
 * stream is; the extraction results are complete with the launch stream as
 * before.  Outputs are identical either way.  No reference counterpart (a
 * scheduling option of the batched step, like the split and the pipeline).
 * on: 1 / 0 sets, -1 queries; returns the current setting. */
int orbx_extractor_overlap_match(orbx_extractor *ex, int on);

/* Per-stage device time of the last batch (HIP events on the launch stream),
 * in ms, when profiling is enabled: resize, blur, fast, quadtree, describe,
 * match.  Returns the number of stages written. */
int orbx_extractor_set_profiling(orbx_extractor *ex, int on);
int orbx_extractor_stage_times(orbx_extractor *ex, float *ms, int cap);

/* Debug hooks for stage-level parity tests (current result slot, frame b):
 * what: 0 = pyramid level, 1 = blurred level (out: w*h bytes, packed rows);
 *       2 = FAST candidates of the level (out: int32 triples x,y,score in
 *           reference push order), 3 = quadtree selection of the level (int32
 *           triples in output order).  Returns element count (bytes for 0/1,
 *           triples for 2/3) or a negative code; ORBX_ERANGE if cap too small. */
int orbx_extractor_debug_fetch(orbx_extractor *ex, int frame, int level, int what,
                               void *out, int64_t cap);

/* ---- ORB_SLAM2::Frame depth: stereo and RGB-D ------------------------- */

/* void Frame::ComputeStereoMatches()                      Frame.cc:502-676
 * For the rectified pair last extracted by `left` and `right` (orbx_extract on
 * each, or frame 0 of each one's current batch): kl/dl/nl are mvKeys /
 * mDescriptors and kr/dr/nr mvKeysRight / mDescriptorsRight as those calls
 * returned them; mbf and mb as the Frame holds them (maxD = mbf / mb).
 * uright / depth (nl floats) receive mvuRight / mvDepth, -1 where there is no
 * match; *nkept = the number of depths kept after the median cut.  Both
 * extractors must share parameters and image size.  Synchronous.
 * Where the reference has undefined behaviour or raises cv::Exception (a band
 * row outside the image, an SAD window outside the level) the keypoint gets
 * no match. */
int orbx_compute_stereo_matches(orbx_extractor *left, orbx_extractor *right,
                                const orbx_keypoint *kl, const uint8_t *dl, int nl,
                                const orbx_keypoint *kr, const uint8_t *dr, int nr,
                                float mbf, float mb, float *uright, float *depth, int *nkept);

/* Stereo front-end step (config C3/C4 unit): frames 2p (left) and 2p+1
 * (right) of d_images, p < pairs, are extracted, then ComputeStereoMatches
 * runs for every pair on the device.  Needs max_batch >= 2 * pairs.
 * Asynchronous on `stream`; results via orbx_depth_download. */
int orbx_stereo_step_device(orbx_extractor *ex, const uint8_t *d_images, int64_t frame_stride,
                            int pitch, int pairs, float mbf, float mb, void *stream);

/* RGB-D front-end step: extract `batch` frames, then
 * Frame::ComputeStereoFromRGBD (Frame.cc:679-701) against float32 depth maps
 * (frame b at d_depth + b * depth_stride bytes, rows depth_pitch bytes apart;
 * undistorted cameras, mvKeysUn == mvKeys).  Asynchronous. */
int orbx_rgbd_step_device(orbx_extractor *ex, const uint8_t *d_images, int64_t frame_stride,
                          int pitch, int batch, const float *d_depth, int64_t depth_stride,
                          int depth_pitch, float mbf, void *stream);

/* Host copy of the last stereo (index = pair) or RGB-D (index = frame) step:
 * mvuRight / mvDepth of the left frame's n keypoints, and the kept count. */
int orbx_depth_download(orbx_extractor *ex, int index, float *uright, float *depth, int cap,
                        int *n, int *nkept);

/* void Frame::ComputeStereoFromRGBD(const cv::Mat &imDepth) Frame.cc:679-701
 * Host keypoints (mvKeys; mvKeysUn = kps_un, or kps when NULL) and CV_32F
 * depth image in, mvuRight / mvDepth out; computed on `device`. */
int orbx_stereo_from_rgbd(int device, const orbx_keypoint *kps, const orbx_keypoint *kps_un, int n,
                          const float *depth_map, int width, int height, size_t pitch, float mbf,
                          float *uright, float *depth, int *nkept);

/* ---- ORB_SLAM2::ORBmatcher -------------------------------------------- */

/* static int DescriptorDistance(const cv::Mat &a, const cv::Mat &b)
 *                                                     ORBmatcher.cc:1649-1665
 * 32-byte descriptors; host computation (no device round trip). */
int orbx_descriptor_distance(const uint8_t *a, const uint8_t *b);

/* int SearchForInitialization(Frame &F1, Frame &F2, vector<Point2f>
 *     &vbPrevMatched, vector<int> &vnMatches12, int windowSize)
 *                                                     ORBmatcher.cc:406-521
 * with ORBmatcher(nnratio, checkOri).  Frames are given by their (undistorted)
 * keypoints and descriptors; the 64x48 grid follows Frame::AssignFeaturesToGrid
 * for an img_w x img_h image without distortion (Frame.cc:239-256).
 * prev_xy (2*n1 floats) is vbPrevMatched (read and updated); matches12 (n1)
 * receives vnMatches12; *nmatches the return value.  Runs on `device`. */
int orbx_search_for_initialization(int device, const orbx_keypoint *k1, const uint8_t *d1,
                                   int n1, const orbx_keypoint *k2, const uint8_t *d2, int n2,
                                   int img_w, int img_h, float *prev_xy, int32_t *matches12,
                                   int window, float nnratio, int check_ori, int *nmatches);
/* The same over the Frame's image bounds (mnMinX, mnMaxX, mnMinY, mnMaxY,
 * Frame::ComputeImageBounds, Frame.cc:475-499): a distorted camera's bounds
 * are non-zero and non-integer, and the grid is PosInGrid's
 * round((x - mnMinX) * mfGridElementWidthInv) (Frame.cc:415-425) with
 * GetFeaturesInArea's floor / ceil((x - mnMinX -/+ r) * inv) windows
 * (:361-373).  orbx_search_for_initialization is this with (0, img_w, 0, img_h).
 * ORBX_EINVAL unless max > min on both axes. */
int orbx_search_for_initialization_bounds(int device, const orbx_keypoint *k1, const uint8_t *d1, int n1,
                                          const orbx_keypoint *k2, const uint8_t *d2, int n2, float min_x,
                                          float max_x, float min_y, float max_y, float *prev_xy,
                                          int32_t *matches12, int window, float nnratio, int check_ori,
                                          int *nmatches);

/* ORBmatcher projection searches: SearchByProjection x4 and the candidate
 * search of Fuse x2 (ORBmatcher.cc:45-129, 291-404, 827-1102, 1330-1601).
 * The caller projects its map points (the pose algebra stays in the host, on
 * the caller's cv::Mat types) and passes one row per point, in the
 * reference's loop order; the device runs the window search, the Hamming
 * distances, the reference's greedy keypoint assignment and the rotation
 * check. */
typedef struct orbx_match_frame {
    const orbx_keypoint *keys;  /* mvKeysUn (grid position, octave, angle) */
    const uint8_t *desc;        /* mDescriptors, 32-byte rows */
    const float *uright;        /* mvuRight, or NULL (monocular) */
    const uint8_t *mp_state;    /* mvpMapPoints / vpMatched per keypoint: bit0 non-NULL,
                                   bit1 its Observations() > 0; NULL = all NULL */
    const float *inv_sigma2;    /* mvInvLevelSigma2 (Fuse's reprojection test) or NULL */
    int n;
    int nlevels;                /* entries of inv_sigma2 */
    float min_x, max_x, min_y, max_y;   /* mnMinX, mnMaxX, mnMinY, mnMaxY: the 64 x 48 grid */
} orbx_match_frame;

typedef struct orbx_proj_query {
    float u, v;          /* projection */
    float radius;        /* GetFeaturesInArea half-size */
    float ur;            /* projected right u (mTrackProjXR, u - mbf * invz) */
    float ur_tol;        /* stereo gate |ur - mvuRight| > ur_tol (SearchByProjection) */
    int32_t min_level;   /* GetFeaturesInArea level arguments, reference semantics */
    int32_t max_level;
    float angle;         /* the query keypoint's angle (rotation check) */
    int32_t flags;       /* ORBX_QUERY_ACTIVE | ORBX_QUERY_BLOCKS */
} orbx_proj_query;

#define ORBX_QUERY_ACTIVE 1   /* the reference's per-point skip tests passed */
#define ORBX_QUERY_BLOCKS 2   /* its map point has Observations() > 0 */

#define ORBX_PROJ_LOCALMAP 0  /* SearchByProjection(Frame&, const vector<MapPoint*>&, th)       :45  */
#define ORBX_PROJ_LASTFRAME 1 /* SearchByProjection(Frame&, const Frame&, th, bMono)            :1330 */
#define ORBX_PROJ_KEYFRAME 2  /* SearchByProjection(Frame&, KeyFrame*, set, th, ORBdist)        :1474 */
#define ORBX_PROJ_SIM3 3      /* SearchByProjection(KeyFrame*, Scw, vpPoints, vpMatched, th)    :291 */
#define ORBX_PROJ_FUSE 4      /* Fuse(KeyFrame*, vpMapPoints, th): candidate search             :827 */
#define ORBX_PROJ_FUSE_SIM3 5 /* Fuse(KeyFrame*, Scw, vpPoints, th, vpReplacePoint): search     :979 */

/* th_dist: TH_HIGH / ORBdist / TH_LOW as the variant's reference uses;
 * nnratio and check_ori: the ORBmatcher's.  Outputs (host arrays):
 *   q_idx[nq]   keypoint assigned to the query (the variant's bestIdx when it
 *               passes), -1 none or dropped by the rotation check;
 *   q_dist[nq]  its distance (-1 none);
 *   kp_final[n] query whose point the keypoint holds afterwards, -1 untouched,
 *               -2 cleared by the rotation check (search variants only);
 *   *nmatches   the reference's return value (nmatches / nFused).
 * Synchronous. */
int orbx_search_by_projection(int device, int variant, const orbx_match_frame *frame,
                              const orbx_proj_query *queries, const uint8_t *qdesc, int nq,
                              int th_dist, float nnratio, int check_ori, int32_t *q_idx,
                              int32_t *q_dist, int32_t *kp_final, int *nmatches);

/* Several independent projection searches of one variant in one pair of
 * launches and one round trip -- the reference's per-keyframe loops:
 *   LocalMapping::SearchInNeighbors, Fuse(pKFi, vpMapPointMatches) for every
 *     neighbour (LocalMapping.cc:537-548; ORBX_PROJ_FUSE);
 *   Tracking::Relocalization, SearchByProjection(mCurrentFrame,
 *     vpCandidateKFs[i], sFound, 10, 100) for every candidate that reached it
 *     (Tracking.cc:1667, 1685; ORBX_PROJ_KEYFRAME).
 * Each problem is exactly one orbx_search_by_projection call (same inputs,
 * same outputs, filled in place including nmatches); problems may share a
 * frame's arrays (uploaded once).  Fuse's candidate search reads one piece
 * of map state: the query point's descriptor (pMP->GetDescriptor(),
 * ORBmatcher.cc:901).  A Replace in an earlier neighbour (or earlier in the
 * same one) recomputes the surviving point's descriptor (MapPoint.cc:254),
 * and the sequential reference searches later neighbours with the new one.
 * So the caller applies the edits neighbour by neighbour in query order,
 * re-checks pMP->isBad() / IsInKeyFrame() before each edit (as Fuse does at
 * the top of its loop), and for a point whose descriptor changed since the
 * batch ran, re-runs that one row (orbx_search_by_projection, nq = 1,
 * current descriptor) instead of using the batch's result.  Position, normal
 * and scale are untouched by Replace, so the query rows stay valid
 * (tests/test_gpu_batch_match.py::test_fuse_neighbours_batched_with_research).
 * Synchronous. */
typedef struct orbx_proj_problem {
    orbx_match_frame frame;
    const orbx_proj_query *queries;
    const uint8_t *qdesc;
    int nq;
    int32_t *q_idx;      /* [nq] */
    int32_t *q_dist;     /* [nq] */
    int32_t *kp_final;   /* [frame.n] */
    int nmatches;        /* out */
} orbx_proj_problem;

int orbx_search_by_projection_batch(int device, int variant, orbx_proj_problem *problems, int nproblems,
                                    int th_dist, float nnratio, int check_ori);

/* int SearchBySim3(KeyFrame *pKF1, KeyFrame *pKF2, vector<MapPoint*> &vpMatches12,
 *                  const float &s12, const cv::Mat &R12, const cv::Mat &t12, th)
 *                                                     ORBmatcher.cc:1104-1328
 * q1: one row per pKF1 map-point slot, its projection into pKF2 (inactive for
 * NULL / bad / already matched / rejected points); q2 likewise for pKF2 into
 * pKF1; each row's level window is [pred - 1, pred].  Two independent window
 * searches (best only, TH_HIGH = th_dist) on the device, then the agreement
 * check: matches12[kf1->n] = the KF2 index of each newly agreed pair (-1
 * none; the caller sets vpMatches12[i1] = vpMapPoints2[matches12[i1]]).
 * *nfound = the reference's return value.  Synchronous. */
int orbx_search_by_sim3(int device, const orbx_match_frame *kf1, const orbx_match_frame *kf2,
                        const orbx_proj_query *q1, const uint8_t *qdesc1, const orbx_proj_query *q2,
                        const uint8_t *qdesc2, int th_dist, int32_t *matches12, int *nfound);

/* ORBmatcher vocabulary-node searches (ORBmatcher.cc:160-289, 524-657,
 * 659-825).  Each side is a keyframe / frame with its DBoW2::FeatureVector
 * given as CSR: ascending node ids, offsets (nnodes + 1), and the feature
 * indices of every node in the vector's order.  flags per feature: bit0 =
 * usable as the reference tests it (side A of SearchByBoW: has a map point
 * that is not bad; side B of the KF-KF search: the same; both sides of
 * SearchForTriangulation: no map point yet, and stereo if bOnlyStereo;
 * side B of the KF-Frame search: ignored), bit1 = mvuRight >= 0. */
typedef struct orbx_bow_side {
    const orbx_keypoint *keys;   /* mvKeysUn (angles; positions for triangulation) */
    const uint8_t *desc;
    const uint8_t *flags;
    int n;
    const uint32_t *node_ids;
    const int32_t *node_offsets;
    const int32_t *node_features;
    int nnodes;
} orbx_bow_side;

#define ORBX_BOW_KF_FRAME 0      /* SearchByBoW(KeyFrame* A, Frame& B, vpMapPointMatches)      :160 */
#define ORBX_BOW_KF_KF 1         /* SearchByBoW(KeyFrame* A, KeyFrame* B, vpMatches12)         :524 */
#define ORBX_BOW_TRIANGULATION 2 /* SearchForTriangulation(KeyFrame* A, KeyFrame* B, F12, ...)  :659 */

/* tri (triangulation only): F12 row-major [9], the epipole (ex, ey) in B,
 * then B's mvScaleFactors[nlevels] and mvLevelSigma2[nlevels].
 * match_a[a.n] / match_b[b.n]: the pairs (-1 none; match_b unused by
 * triangulation, whose pairs are (i, match_a[i]) in index order);
 * *nmatches: the reference's return value.  Synchronous. */
int orbx_search_by_bow(int device, int variant, const orbx_bow_side *a, const orbx_bow_side *b,
                       float nnratio, int check_ori, const float *tri, int nlevels,
                       int32_t *match_a, int32_t *match_b, int *nmatches);

/* Several vocabulary-node searches of one variant in one pair of launches
 * and one round trip: LocalMapping::CreateNewMapPoints' SearchForTriangulation
 * of the new keyframe against each covisible neighbour (LocalMapping.cc:
 * 276-315), or any set of SearchByBoW calls.  Each problem is exactly one
 * orbx_search_by_bow call with the same inputs (tri: its own 11 + 2 nlevels
 * floats; match arrays and nmatches filled in place).
 * The reference runs the neighbours in order and each one's triangulations
 * give keyframe A new map points, which bar those features from the next
 * neighbour's search (side A flags).  A feature's search never depends on the
 * other A features (SearchForTriangulation sets no vbMatched2), so a batch
 * run with the flags at the start stays exact: the caller drops, neighbour by
 * neighbour, the pairs whose A feature got a map point from an earlier
 * neighbour -- with check_ori = 0, as LocalMapping's ORBmatcher(0.6, false)
 * has it; with check_ori = 1 run orbx_rotation_filter over the survivors
 * (pass check_ori = 0 to the batch and keep its raw pairs).
 * Synchronous. */
typedef struct orbx_bow_problem {
    orbx_bow_side a, b;
    const float *tri;    /* triangulation only */
    int32_t *match_a;    /* [a.n] */
    int32_t *match_b;    /* [b.n] (unused by triangulation) */
    int nmatches;        /* out */
} orbx_bow_problem;

int orbx_search_by_bow_batch(int device, int variant, orbx_bow_problem *problems, int nproblems,
                             float nnratio, int check_ori, int nlevels);

/* The reference's rotation-consistency pass (rotHist + ComputeThreeMaxima +
 * removal, ORBmatcher.cc:1603-1644 and e.g. :800-818) over pairs
 * (i, match_a[i] >= 0) of keypoints ka / kb, skipping A features with
 * exclude[i] != 0 (NULL: none), in place; *nmatches = the pairs kept.  Host
 * only. */
int orbx_rotation_filter(const orbx_keypoint *ka, const orbx_keypoint *kb, int32_t *match_a, int na,
                         const uint8_t *exclude, int *nmatches);

/* ---- DBoW2 vocabulary ----
 * ORBVocabulary = DBoW2::TemplatedVocabulary<FORB::TDescriptor, FORB>
 * (ORBVocabulary.h).  The tree is held as loadFromTextFile /
 * loadFromBinFile build it (TemplatedVocabulary.h:1351-1425 / 1473-1547):
 * node 0 the root, nodes 1..n_nodes-1 in file order with parent (< own
 * index), the file's leaf flag, a 32-byte descriptor and a weight (double);
 * children in file order, word ids in the order of the leaf flags.
 * scoring / weighting are DBoW2's ScoringType (L1_NORM 0 .. DOT_PRODUCT 5) /
 * WeightingType (TF_IDF 0, TF 1, IDF 2, BINARY 3).  Creation and loading are
 * host-only; the first transform uploads the tree to `device`. */
typedef struct orbx_vocab orbx_vocab;

/* From arrays (row 0 of desc / weight / parent / is_leaf is the root's and
 * ignored).  k = the header's branching factor (informational; the tree's
 * own child counts are used, up to 64). */
int orbx_vocab_create(int device, int k, int L, int scoring, int weighting, int n_nodes,
                      const int32_t *parent, const uint8_t *is_leaf, const uint8_t *desc,
                      const double *weight, orbx_vocab **out);
/* loadFromTextFile (format 0: "k L scoring weighting" then one
 * "parent isLeaf d0 .. d31 weight" line per node; blank lines skipped) or
 * loadFromBinFile (format 1: int32 k, L, scoring, weighting, then per node
 * int32 parent, u8 isLeaf, 32 B, f64 weight, up to (k^(L+1)-1)/(k-1) nodes).
 * Header checks as the reference: 0<=k<=20, 1<=L<=10, scoring 0..5,
 * weighting 0..3, else ORBX_EINVAL. */
int orbx_vocab_load(int device, const char *path, int format, orbx_vocab **out);
void orbx_vocab_destroy(orbx_vocab *v);
/* header and sizes; any pointer may be NULL. */
int orbx_vocab_info(const orbx_vocab *v, int *k, int *L, int *scoring, int *weighting, int *n_nodes,
                    int *n_words);
/* The tree back as arrays of n_nodes (cap >= n_nodes, else ORBX_ERANGE). */
int orbx_vocab_export(const orbx_vocab *v, int32_t *parent, uint8_t *is_leaf, uint8_t *desc,
                      double *weight, int cap);

/* TemplatedVocabulary::transform(features, BowVector&, FeatureVector&,
 * levelsup) (TemplatedVocabulary.h:1140-1207), as Frame::ComputeBoW
 * (Frame.cc:428-435) and KeyFrame::ComputeBoW (KeyFrame.cc:68-77, levelsup 4)
 * call it.  desc: n rows of 32 B.  BowVector out as ascending (word, value)
 * pairs (capacity n); FeatureVector out as ascending node ids with per-node
 * feature lists: fv_offsets[n_fv + 1] (capacity n + 1), fv_features
 * (capacity n) -- the layout orbx_bow_side takes.  A leaf above level
 * L - levelsup (the reference leaves its node unset) files the feature under
 * the leaf.  An empty vocabulary clears both.  Synchronous. */
int orbx_vocab_transform(orbx_vocab *v, const uint8_t *desc, int n, int levelsup,
                         uint32_t *bow_words, double *bow_values, int *n_bow,
                         uint32_t *fv_nodes, int32_t *fv_offsets, int32_t *fv_features, int *n_fv);
/* Per-feature descent on device buffers, ordered on `stream` (NULL: the
 * vocabulary's own stream, as the extractor's): word id, weight (0: a
 * stopped word the vectors skip) and FeatureVector node of each row. */
int orbx_vocab_transform_device(orbx_vocab *v, const uint8_t *d_desc, int n, int levelsup,
                                uint32_t *d_word, double *d_weight, uint32_t *d_node, void *stream);

/* ---- per-frame neighbours ----
 * The *_device forms run on `stream` (a hipStream_t; NULL = the current
 * device's default stream) over device buffers; the others are synchronous
 * over host buffers. */

/* MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:288-361) for a batch of
 * map points: point p's usable observation descriptors (the reference skips
 * bad keyframes) are rows offsets[p] .. offsets[p+1]-1 of desc (32 B each,
 * in the observation map's order; at most 65535 per point).  best[p] = the
 * row (relative to offsets[p]) with the least median Hamming distance to the
 * point's rows, the first on ties -- mDescriptor = that row; -1 when the
 * point has none (the reference returns without change). */
int orbx_distinctive_descriptors(int device, const uint8_t *desc, const int32_t *offsets, int npoints,
                                 int32_t *best);
int orbx_distinctive_descriptors_device(const uint8_t *d_desc, const int32_t *d_offsets, int npoints,
                                        int32_t *d_best, void *stream);

/* Frame::UndistortKeyPoints (Frame.cc:438-469): cv::undistortPoints(mK,
 * mDistCoef, R = I, P = mK).  K: row-major 3x3 (mK, CV_32F); dist: k1 k2 p1
 * p2 [k3 ...] (ncoef 4..8).  dist[0] == 0: a copy, as the reference.  Only
 * pt.x / pt.y change. */
int orbx_undistort_keypoints(int device, const orbx_keypoint *kps, int n, const float *K, const float *dist,
                             int ncoef, orbx_keypoint *kps_un);
/* The same on device (x, y) float pairs. */
int orbx_undistort_points_device(const float *d_xy, int n, const float *K, const float *dist, int ncoef,
                                 float *d_xy_un, void *stream);

/* cv::cvtColor(CV_RGB2GRAY / CV_BGR2GRAY / CV_RGBA2GRAY / CV_BGRA2GRAY) of
 * 8-bit images (Tracking.cc:179-264): channels 3 or 4, rgb 1 when the first
 * channel is red (mbRGB). */
int orbx_cvt_gray(int device, const uint8_t *src, int width, int height, size_t pitch, int channels, int rgb,
                  uint8_t *dst, size_t dst_pitch);
int orbx_cvt_gray_device(const uint8_t *d_src, int64_t src_frame_stride, int src_pitch, int channels, int rgb,
                         int width, int height, int batch, uint8_t *d_dst, int64_t dst_frame_stride,
                         int dst_pitch, void *stream);
/* imDepth.convertTo(imDepth, CV_32F, mDepthMapFactor) of 16-bit depth
 * (Tracking.cc:228-229): dst = (float)src * scale. */
int orbx_depth_to_float_device(const uint16_t *d_src, int64_t src_frame_stride, int src_pitch, int width,
                               int height, int batch, float scale, float *d_dst, int64_t dst_frame_stride,
                               int dst_pitch, void *stream);

/* ---- keyframe database ----
 * KeyFrameDatabase (KeyFrameDatabase.cc:31-236) over keyframes named by 64-bit
 * ids, BowVectors as ascending (word, value) arrays (orbx_vocab_transform's
 * output).  The per-keyframe query state of the reference (mnLoopQuery,
 * mnLoopWords, mLoopScore, mnRelocQuery, mnRelocWords, mRelocScore) lives in
 * the database and persists across queries, erase and re-add; the scores the
 * reference leaves uninitialised start at 0.  Scoring is L1 (ORBvoc's
 * L1_NORM).  Covisibility (KeyFrame::GetBestCovisibilityKeyFrames(10)) comes
 * from the caller's callback, which writes up to cap ids and returns the
 * count. */
typedef struct orbx_kfdb orbx_kfdb;
typedef int (*orbx_covis_fn)(void *ctx, uint64_t kf_id, uint64_t *out, int cap);
int orbx_kfdb_create(int device, orbx_kfdb **out);
void orbx_kfdb_destroy(orbx_kfdb *db);
/* add (:37-44) / erase (:46-67) / clear (:69-73).  Adding an id that is in the
 * database is ORBX_EINVAL (the reference would list it twice), and so is a
 * word id >= ORBX_KFDB_MAX_WORDS (the inverted file is indexed by word id;
 * ORBvoc has 10^6 words).  A query id of 0 matches every keyframe never
 * queried (the reference's mnLoopQuery / mnRelocQuery start at 0). */
#define ORBX_KFDB_MAX_WORDS (1u << 26)
int orbx_kfdb_add(orbx_kfdb *db, uint64_t kf_id, const uint32_t *words, const double *values, int n);
int orbx_kfdb_erase(orbx_kfdb *db, uint64_t kf_id);
int orbx_kfdb_clear(orbx_kfdb *db);
int orbx_kfdb_size(const orbx_kfdb *db);
/* DetectLoopCandidates(pKF, minScore) (:76-236): query = pKF's id and
 * BowVector, connected = pKF->GetConnectedKeyFrames().  out: candidate ids in
 * the reference's order; ORBX_ERANGE (with *n_out) if cap is too small. */
int orbx_kfdb_detect_loop_candidates(orbx_kfdb *db, uint64_t query_id, const uint32_t *words,
                                     const double *values, int n, const uint64_t *connected, int n_connected,
                                     float min_score, orbx_covis_fn covis, void *ctx, uint64_t *out, int cap,
                                     int *n_out);
/* DetectRelocalizationCandidates(F) (:238-330): frame id and BowVector. */
int orbx_kfdb_detect_relocalization_candidates(orbx_kfdb *db, uint64_t frame_id, const uint32_t *words,
                                               const double *values, int n, orbx_covis_fn covis, void *ctx,
                                               uint64_t *out, int cap, int *n_out);
/* L1Scoring::score (ScoringObject.cpp:23-66), host. */
int orbx_bow_score_l1(const uint32_t *w1, const double *v1, int n1, const uint32_t *w2, const double *v2, int n2,
                      double *score);

/* ---- local bundle adjustment ----
 * Optimizer::LocalBundleAdjustment (Optimizer.cc:517-900) on the graph the
 * caller collected: cameras (local keyframes + fixed cameras) and local map
 * points, one edge per observation.  Runs g2o's Levenberg-Marquardt over a
 * 6/3 block solver with the Schur complement: iters1 iterations with Huber
 * kernels (delta sqrt(5.991) mono, sqrt(7.815) stereo), then the outliers
 * (chi2 > 5.991 / 7.815 or point behind the camera) leave, the kernels are
 * dropped and iters2 more iterations run (the reference: 5 and 10). */
typedef struct orbx_ba_edge {
    int32_t cam, point;       /* indices into the camera / point arrays */
    float u, v;               /* mvKeysUn[idx].pt */
    float ur;                 /* mvuRight[idx]; < 0: monocular edge */
    float inv_sigma2;         /* mvInvLevelSigma2[octave] */
    float fx, fy, cx, cy, bf; /* the keyframe's intrinsics (bf stereo only) */
} orbx_ba_edge;

/* Tcw: ncam row-major 3x4 float poses (KeyFrame::GetPose()), fixed[c] != 0
 * for fixed vertices (mnId == 0 and the fixed cameras); Xw: npt x 3 float
 * (MapPoint::GetWorldPos()).  Out: Tcw_out / Xw_out as Converter::toCvMat
 * casts them back; outlier[e] = the reference's final check (chi2 over the
 * threshold or depth not positive: the observation is erased);
 * iterations[2] (nullable) = LM iterations run per pass.  At most 170 free
 * cameras.  Synchronous. */
int orbx_local_ba(int device, const float *Tcw, const uint8_t *fixed, int ncam, const float *Xw, int npt,
                  const orbx_ba_edge *edges, int ne, int iters1, int iters2, float *Tcw_out, float *Xw_out,
                  uint8_t *outlier, int *iterations);
/* The same optimisation in a fast mode: the per-vertex sums as parallel
 * reductions instead of sequential chains in edge / point order, the Schur
 * complement and reduced right-hand side as one dense FP64 matrix-core
 * product (S = Hpp + lambda I - W^T W, W_p = L_p^-1 B_p^T with D_p = L_p L_p^T),
 * the reduced system factored as an augmented matrix with its trailing tiles
 * on the matrix cores, the trial's acceptance decided on the device.  Same
 * algorithm, another floating-point order: outputs equal orbx_local_ba's to
 * rounding (tolerances in tests/test_gpu_ba.py), not bit for bit; the LM
 * iteration counts and outlier flags came out equal on every test problem.
 * No reference counterpart beyond LocalBundleAdjustment itself, whose g2o
 * sums are unordered too. */
int orbx_local_ba_fast(int device, const float *Tcw, const uint8_t *fixed, int ncam, const float *Xw, int npt,
                       const orbx_ba_edge *edges, int ne, int iters1, int iters2, float *Tcw_out, float *Xw_out,
                       uint8_t *outlier, int *iterations);
/* One LM linear system of the first pass at the given lambda: x (6 per free
 * camera, then 3 per point) and the robust chi2; *solved = 0 when the
 * reduced system is not positive definite.  Test hook. */
int orbx_ba_debug_step(int device, const float *Tcw, const uint8_t *fixed, int ncam, const float *Xw, int npt,
                       const orbx_ba_edge *edges, int ne, int robust, double lambda, double *x_out,
                       double *chi2_out, int *solved);

/* Device evaluation of the restated sincosf / fastAtan2 (test hook). */
int orbx_debug_trig(int device, const float *angles, float *s, float *c, int n,
                    const float *ys, const float *xs, float *atan_deg, int m);

#ifdef __cplusplus
}
#endif
#endif /* ORBX_H */
