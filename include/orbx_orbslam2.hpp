// orbx_orbslam2.hpp -- header-only drop-in for ORB_SLAM2::ORBextractor and
// ORB_SLAM2::ORBmatcher::{DescriptorDistance, SearchForInitialization} over
// liborbx.so (include/orbx.h).
//
// Reference interfaces reproduced (wjjcdy/orb_slam_2_ros):
//   orb_slam2/include/ORBextractor.h:45-111  (class ORBextractor)
//   orb_slam2/include/ORBmatcher.h:46,65     (DescriptorDistance, SearchForInitialization)
//   orb_slam2/src/Frame.cc:502-676,679-701   (ComputeStereoMatches, ComputeStereoFromRGBD)
//
// Use: replace `#include "ORBextractor.h"` by this header in Frame.h /
// Tracking.h (or add the GPU class beside the CPU one) and
// link liborbx.so.  The types are OpenCV's; nothing here includes HIP.
#pragma once

#include <algorithm>
#include <cassert>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include <opencv2/core/core.hpp>

#include "orbx.h"

namespace ORB_SLAM2 {

namespace orbx_detail {
inline int device_index() {
    const char *s = std::getenv("ORBX_DEVICE");
    return s ? std::atoi(s) : 0;
}
inline void check(int rc, const char *what) {
    if (rc < 0) throw std::runtime_error(std::string(what) + ": " + orbx_strerror(rc));
}
inline std::vector<orbx_keypoint> pack(const std::vector<cv::KeyPoint> &ks) {
    std::vector<orbx_keypoint> out(ks.size());
    for (size_t i = 0; i < ks.size(); ++i)
        out[i] = {ks[i].pt.x, ks[i].pt.y, ks[i].size, ks[i].angle, ks[i].response, ks[i].octave, ks[i].class_id};
    return out;
}
}  // namespace orbx_detail

// mvImagePyramid (ORBextractor.h:85) as a lazily filled container: each level
// an ROI of a buffer with a 19-px reflect-101 border, as ComputePyramid builds
// it (ORBextractor.cc:1152-1185), copied from the device on the first access
// after an extraction (orbx_extractor_pyramid_host: one stream-ordered copy of
// every level).  The reference reads it only in Frame::ComputeStereoMatches
// (Frame.cc:509, 599-616), which Frame_orbx.cc forwards to the device
// pyramids, so with the forwarder in place no call pays for it.  operator[],
// size(), begin()/end() read as std::vector<cv::Mat> does.  Each refill
// allocates new level buffers, as ComputePyramid's fresh `temp` does, so a
// cv::Mat a caller kept from an earlier frame keeps that frame's pixels.  The
// fill is guarded by a mutex, so concurrent const reads are safe; as with
// the reference's vector, reading while the extractor runs is not.
class OrbxPyramid {
public:
    cv::Mat &operator[](size_t l) { fill(); return lv_[l]; }
    const cv::Mat &operator[](size_t l) const { fill(); return lv_[l]; }
    size_t size() const { return lv_.size(); }
    bool empty() const { return lv_.empty(); }
    std::vector<cv::Mat>::iterator begin() { fill(); return lv_.begin(); }
    std::vector<cv::Mat>::iterator end() { fill(); return lv_.end(); }
    std::vector<cv::Mat>::const_iterator begin() const { fill(); return lv_.begin(); }
    std::vector<cv::Mat>::const_iterator end() const { fill(); return lv_.end(); }
    void resize(size_t n) { lv_.resize(n); whole_.resize(n); }

private:
    friend class ORBextractor;
    void fill() const {
        std::lock_guard<std::mutex> lock(mu_);
        if (!stale_) return;
        const int E = 19;   // EDGE_THRESHOLD
        const int n = (int)lv_.size();
        std::vector<uint8_t *> ptr(n);
        std::vector<size_t> pitch(n);
        for (int l = 0; l < n; ++l) {
            int w = 0, h = 0;
            orbx_detail::check(orbx_extractor_pyramid_level(h_, l, nullptr, 0, &w, &h), "pyramid level");
            whole_[l] = cv::Mat(h + 2 * E, w + 2 * E, CV_8U);   // new buffer: old ROIs keep their data
            lv_[l] = whole_[l](cv::Rect(E, E, w, h));
            ptr[l] = lv_[l].data;
            pitch[l] = lv_[l].step;
        }
        orbx_detail::check(orbx_extractor_pyramid_host(h_, ptr.data(), pitch.data(), n), "pyramid");
        for (int l = 0; l < n; ++l)
            cv::copyMakeBorder(lv_[l], whole_[l], E, E, E, E, cv::BORDER_REFLECT_101 + cv::BORDER_ISOLATED);
        stale_ = false;
    }
    orbx_extractor *h_ = nullptr;
    mutable std::vector<cv::Mat> lv_, whole_;
    mutable bool stale_ = false;
    mutable std::mutex mu_;
};

class ORBextractor {
public:
    enum { HARRIS_SCORE = 0, FAST_SCORE = 1 };

    ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST)
        : nfeatures_(nfeatures), nlevels_(nlevels) {
        h_ = orbx_extractor_create(orbx_detail::device_index(), nfeatures, scaleFactor, nlevels, iniThFAST,
                                   minThFAST);
        if (!h_) throw std::runtime_error("orbx_extractor_create failed (no gfx950 device or bad parameters)");
        scaleFactor_ = orbx_extractor_get_scale_factor(h_);
        mvScaleFactor = table(0);
        mvInvScaleFactor = table(1);
        mvLevelSigma2 = table(2);
        mvInvLevelSigma2 = table(3);
        mvImagePyramid.h_ = h_;
        mvImagePyramid.resize(nlevels);
    }
    ~ORBextractor() { orbx_extractor_destroy(h_); }
    ORBextractor(const ORBextractor &) = delete;
    ORBextractor &operator=(const ORBextractor &) = delete;

    // ORBextractor.cc:1083-1149.  The mask is ignored, as in the reference.
    void operator()(cv::InputArray _image, cv::InputArray /*mask*/, std::vector<cv::KeyPoint> &_keypoints,
                    cv::OutputArray _descriptors) {
        if (_image.empty()) return;   // outputs untouched (ORBextractor.cc:1086-1087)
        cv::Mat image = _image.getMat();
        assert(image.type() == CV_8UC1);
        int cap = nfeatures_ + 16 * nlevels_ + 64;
        std::vector<orbx_keypoint> kps;
        cv::Mat desc;
        int n = 0;
        for (;;) {
            kps.resize(cap);
            desc.create(cap, 32, CV_8U);
            const int rc = orbx_extract(h_, image.data, image.cols, image.rows, image.step, kps.data(), desc.data,
                                        cap, &n);
            if (rc == ORBX_ERANGE) { cap = n; continue; }
            orbx_detail::check(rc, "ORBextractor::operator()");
            break;
        }
        _keypoints.clear();
        _keypoints.reserve(n);
        for (int i = 0; i < n; ++i) {
            const orbx_keypoint &k = kps[i];
            _keypoints.push_back(cv::KeyPoint(cv::Point2f(k.x, k.y), k.size, k.angle, k.response, k.octave,
                                              k.class_id));
        }
        if (n == 0) {
            _descriptors.release();
        } else {
            _descriptors.create(n, 32, CV_8U);
            desc.rowRange(0, n).copyTo(_descriptors.getMat());
        }
        {
            std::lock_guard<std::mutex> lock(mvImagePyramid.mu_);
            mvImagePyramid.stale_ = true;   // filled from the device when read
        }
    }

    int inline GetLevels() { return nlevels_; }
    // The liborbx handle (device pyramid of the last call), for OrbxFrame.
    orbx_extractor *handle() const { return h_; }
    float inline GetScaleFactor() { return scaleFactor_; }
    std::vector<float> inline GetScaleFactors() { return mvScaleFactor; }
    std::vector<float> inline GetInverseScaleFactors() { return mvInvScaleFactor; }
    std::vector<float> inline GetScaleSigmaSquares() { return mvLevelSigma2; }
    std::vector<float> inline GetInverseScaleSigmaSquares() { return mvInvLevelSigma2; }

    // ORBextractor.h:85 (see OrbxPyramid)
    OrbxPyramid mvImagePyramid;

protected:
    std::vector<float> table(int which) {
        std::vector<float> v(nlevels_);
        orbx_detail::check(orbx_extractor_get_scale_table(h_, which, v.data(), nlevels_), "scale table");
        return v;
    }

    orbx_extractor *h_ = nullptr;
    int nfeatures_;
    int nlevels_;
    float scaleFactor_ = 1.2f;
    std::vector<float> mvScaleFactor, mvInvScaleFactor, mvLevelSigma2, mvInvLevelSigma2;
};

// Free-function forms of the ORBmatcher members this tier accelerates; the
// reference class keeps its signatures and forwards to these.
struct OrbxMatcher {
    // ORBmatcher.cc:1649-1665
    static int DescriptorDistance(const cv::Mat &a, const cv::Mat &b) {
        return orbx_descriptor_distance(a.ptr<uint8_t>(), b.ptr<uint8_t>());
    }

    // ORBmatcher.cc:406-521 for frames given by (mvKeysUn, mDescriptors) and the
    // undistorted image size that sizes Frame's 64x48 grid (mnMinX = mnMinY = 0).
    static int SearchForInitialization(const std::vector<cv::KeyPoint> &keys1, const cv::Mat &desc1,
                                       const std::vector<cv::KeyPoint> &keys2, const cv::Mat &desc2, int img_w,
                                       int img_h, std::vector<cv::Point2f> &vbPrevMatched,
                                       std::vector<int> &vnMatches12, int windowSize, float nnratio,
                                       bool checkOri) {
        return SearchForInitialization(keys1, desc1, keys2, desc2, 0.f, (float)img_w, 0.f, (float)img_h,
                                       vbPrevMatched, vnMatches12, windowSize, nnratio, checkOri);
    }

    // The same over the Frame's grid bounds mnMinX, mnMaxX, mnMinY, mnMaxY
    // (Frame::ComputeImageBounds, Frame.cc:475-499: non-zero and non-integer
    // for a distorted camera).
    static int SearchForInitialization(const std::vector<cv::KeyPoint> &keys1, const cv::Mat &desc1,
                                       const std::vector<cv::KeyPoint> &keys2, const cv::Mat &desc2, float min_x,
                                       float max_x, float min_y, float max_y, std::vector<cv::Point2f> &vbPrevMatched,
                                       std::vector<int> &vnMatches12, int windowSize, float nnratio,
                                       bool checkOri) {
        const std::vector<orbx_keypoint> k1 = orbx_detail::pack(keys1), k2 = orbx_detail::pack(keys2);
        const cv::Mat d1 = desc1.isContinuous() ? desc1 : desc1.clone();
        const cv::Mat d2 = desc2.isContinuous() ? desc2 : desc2.clone();
        std::vector<float> prev(2 * keys1.size());
        for (size_t i = 0; i < keys1.size(); ++i) { prev[2 * i] = vbPrevMatched[i].x; prev[2 * i + 1] = vbPrevMatched[i].y; }
        vnMatches12.assign(keys1.size(), -1);
        int nm = 0;
        orbx_detail::check(orbx_search_for_initialization_bounds(orbx_detail::device_index(), k1.data(), d1.data,
                                                                 (int)k1.size(), k2.data(), d2.data, (int)k2.size(),
                                                                 min_x, max_x, min_y, max_y, prev.data(),
                                                                 vnMatches12.data(), windowSize, nnratio,
                                                                 checkOri ? 1 : 0, &nm),
                           "SearchForInitialization");
        for (size_t i = 0; i < keys1.size(); ++i) vbPrevMatched[i] = cv::Point2f(prev[2 * i], prev[2 * i + 1]);
        return nm;
    }

    // The searched frame / keyframe of a projection search: mvKeysUn,
    // mDescriptors, mvuRight (may be empty), the current mvpMapPoints /
    // vpMatched as per-keypoint flags (bit0 non-NULL, bit1 Observations() > 0),
    // mvInvLevelSigma2 (Fuse) and the grid bounds mnMinX..mnMaxY.
    struct ProjFrame {
        const std::vector<cv::KeyPoint> *keys = nullptr;
        const cv::Mat *desc = nullptr;
        const std::vector<float> *uright = nullptr;
        const std::vector<uint8_t> *mp_state = nullptr;
        const std::vector<float> *inv_sigma2 = nullptr;
        float min_x = 0, max_x = 0, min_y = 0, max_y = 0;
    };

    // SearchByProjection x4 / Fuse x2 (search part), ORBmatcher.cc:45-129,
    // 291-404, 827-1102, 1330-1601: one query row per point in the reference's
    // loop order (orbx_proj_query), descriptors as an nq x 32 Mat.  Returns the
    // reference's count; q_idx / kp_final as in include/orbx.h.
    static int SearchByProjectionTable(int variant, const ProjFrame &F, const std::vector<orbx_proj_query> &q,
                                       const cv::Mat &qdesc, int th_dist, float nnratio, bool checkOri,
                                       std::vector<int> &q_idx, std::vector<int> &q_dist,
                                       std::vector<int> &kp_final) {
        const std::vector<orbx_keypoint> k = orbx_detail::pack(*F.keys);
        const cv::Mat d = F.desc->isContinuous() ? *F.desc : F.desc->clone();
        const cv::Mat qd = qdesc.isContinuous() ? qdesc : qdesc.clone();
        orbx_match_frame mf{};
        mf.keys = k.data();
        mf.desc = d.data;
        mf.uright = F.uright && !F.uright->empty() ? F.uright->data() : nullptr;
        mf.mp_state = F.mp_state && !F.mp_state->empty() ? F.mp_state->data() : nullptr;
        mf.inv_sigma2 = F.inv_sigma2 ? F.inv_sigma2->data() : nullptr;
        mf.n = (int)k.size();
        mf.nlevels = F.inv_sigma2 ? (int)F.inv_sigma2->size() : 0;
        mf.min_x = F.min_x; mf.max_x = F.max_x; mf.min_y = F.min_y; mf.max_y = F.max_y;
        q_idx.assign(q.size(), -1);
        q_dist.assign(q.size(), -1);
        kp_final.assign(k.size(), -1);
        int nm = 0;
        orbx_detail::check(orbx_search_by_projection(orbx_detail::device_index(), variant, &mf, q.data(), qd.data,
                                                     (int)q.size(), th_dist, nnratio, checkOri ? 1 : 0, q_idx.data(),
                                                     q_dist.data(), kp_final.data(), &nm),
                           "SearchByProjection");
        return nm;
    }

    // One row of a projection search with the point's current descriptor: the
    // re-search the batched Fuse recipe needs for a point whose descriptor a
    // Replace changed after the batch ran (include/orbx.h).  idx / dist as
    // q_idx[0] / q_dist[0] of SearchByProjectionTable.
    static void SearchOneRow(int variant, const ProjFrame &F, const orbx_proj_query &q, const cv::Mat &desc,
                             int th_dist, float nnratio, int &idx, int &dist) {
        std::vector<int> qi, qdist, kf;
        SearchByProjectionTable(variant, F, std::vector<orbx_proj_query>(1, q), desc, th_dist, nnratio, false, qi,
                                qdist, kf);
        idx = qi[0];
        dist = qdist[0];
    }

    // The per-keyframe loops in one launch pair: problem k searches frame
    // F[k] with queries q[k] / qdesc[k], exactly as SearchByProjectionTable
    // would (Fuse over LocalMapping's neighbours, relocalisation's candidates;
    // include/orbx.h orbx_search_by_projection_batch).  Returns each problem's
    // count.
    static std::vector<int> SearchByProjectionBatch(int variant, const std::vector<ProjFrame> &F,
                                                    const std::vector<std::vector<orbx_proj_query>> &q,
                                                    const std::vector<cv::Mat> &qdesc, int th_dist, float nnratio,
                                                    bool checkOri, std::vector<std::vector<int>> &q_idx,
                                                    std::vector<std::vector<int>> &q_dist,
                                                    std::vector<std::vector<int>> &kp_final) {
        const size_t np = F.size();
        // one packed copy per distinct frame: problems that search the same
        // frame (relocalisation: one current frame, many candidates) pass the
        // same host pointers, which the runtime uploads once
        std::vector<std::vector<orbx_keypoint>> k(np);
        std::vector<const std::vector<orbx_keypoint> *> kp(np);
        std::vector<cv::Mat> d(np), qd(np);
        std::vector<orbx_proj_problem> pr(np);
        q_idx.assign(np, {});
        q_dist.assign(np, {});
        kp_final.assign(np, {});
        for (size_t i = 0; i < np; ++i) {
            size_t src = i;
            for (size_t j = 0; j < i; ++j)
                if (F[j].keys == F[i].keys && F[j].desc == F[i].desc) { src = j; break; }
            if (src == i) {
                k[i] = orbx_detail::pack(*F[i].keys);
                d[i] = F[i].desc->isContinuous() ? *F[i].desc : F[i].desc->clone();
            } else {
                d[i] = d[src];   // shares the same buffer (cv::Mat header copy)
            }
            kp[i] = src == i ? &k[i] : kp[src];
            qd[i] = qdesc[i].isContinuous() ? qdesc[i] : qdesc[i].clone();
            orbx_match_frame &mf = pr[i].frame;
            mf = orbx_match_frame{};
            mf.keys = kp[i]->data();
            mf.desc = d[i].data;
            mf.uright = F[i].uright && !F[i].uright->empty() ? F[i].uright->data() : nullptr;
            mf.mp_state = F[i].mp_state && !F[i].mp_state->empty() ? F[i].mp_state->data() : nullptr;
            mf.inv_sigma2 = F[i].inv_sigma2 ? F[i].inv_sigma2->data() : nullptr;
            mf.n = (int)kp[i]->size();
            mf.nlevels = F[i].inv_sigma2 ? (int)F[i].inv_sigma2->size() : 0;
            mf.min_x = F[i].min_x; mf.max_x = F[i].max_x; mf.min_y = F[i].min_y; mf.max_y = F[i].max_y;
            q_idx[i].assign(q[i].size(), -1);
            q_dist[i].assign(q[i].size(), -1);
            kp_final[i].assign(kp[i]->size(), -1);
            pr[i].queries = q[i].data();
            pr[i].qdesc = qd[i].data;
            pr[i].nq = (int)q[i].size();
            pr[i].q_idx = q_idx[i].data();
            pr[i].q_dist = q_dist[i].data();
            pr[i].kp_final = kp_final[i].data();
        }
        orbx_detail::check(orbx_search_by_projection_batch(orbx_detail::device_index(), variant, pr.data(), (int)np,
                                                           th_dist, nnratio, checkOri ? 1 : 0),
                           "SearchByProjection batch");
        std::vector<int> nm(np);
        for (size_t i = 0; i < np; ++i) nm[i] = pr[i].nmatches;
        return nm;
    }

    // SearchByBoW x2 / SearchForTriangulation (ORBmatcher.cc:160-289, 524-825)
    // on two sides given as orbx_bow_side (FeatureVector as CSR).
    static int SearchByBoWTable(int variant, const orbx_bow_side &A, const orbx_bow_side &B, float nnratio,
                                bool checkOri, const std::vector<float> &tri, int nlevels,
                                std::vector<int> &match_a, std::vector<int> &match_b) {
        match_a.assign(A.n, -1);
        match_b.assign(B.n, -1);
        int nm = 0;
        orbx_detail::check(orbx_search_by_bow(orbx_detail::device_index(), variant, &A, &B, nnratio, checkOri ? 1 : 0,
                                              tri.empty() ? nullptr : tri.data(), nlevels, match_a.data(),
                                              match_b.data(), &nm),
                           "SearchByBoW");
        return nm;
    }

    // SearchForTriangulation of one keyframe against its neighbours (or any
    // set of SearchByBoW calls) in one launch pair: problem k = (A[k], B[k],
    // tri[k]); include/orbx.h orbx_search_by_bow_batch for the neighbour-order
    // rule LocalMapping::CreateNewMapPoints needs.  Returns each count.
    static std::vector<int> SearchByBoWBatch(int variant, const std::vector<orbx_bow_side> &A,
                                             const std::vector<orbx_bow_side> &B,
                                             const std::vector<std::vector<float>> &tri, int nlevels, float nnratio,
                                             bool checkOri, std::vector<std::vector<int>> &match_a,
                                             std::vector<std::vector<int>> &match_b) {
        const size_t np = A.size();
        std::vector<orbx_bow_problem> pr(np);
        match_a.assign(np, {});
        match_b.assign(np, {});
        for (size_t i = 0; i < np; ++i) {
            match_a[i].assign(A[i].n, -1);
            match_b[i].assign(B[i].n, -1);
            pr[i].a = A[i];
            pr[i].b = B[i];
            pr[i].tri = i < tri.size() && !tri[i].empty() ? tri[i].data() : nullptr;
            pr[i].match_a = match_a[i].data();
            pr[i].match_b = match_b[i].data();
        }
        orbx_detail::check(orbx_search_by_bow_batch(orbx_detail::device_index(), variant, pr.data(), (int)np, nnratio,
                                                    checkOri ? 1 : 0, nlevels),
                           "SearchByBoW batch");
        std::vector<int> nm(np);
        for (size_t i = 0; i < np; ++i) nm[i] = pr[i].nmatches;
        return nm;
    }
};

// The two Frame depth steps this tier accelerates, as free functions over the
// Frame members they read and write (see INTEGRATION.md for the Frame.cc patch).
struct OrbxFrame {
    // Frame::ComputeStereoMatches (Frame.cc:502-676): left / right are the
    // extractors that produced mvKeys / mvKeysRight in this frame (their device
    // pyramids are the mvImagePyramid the reference reads).  Returns the number
    // of depths kept.
    static int ComputeStereoMatches(ORBextractor &left, ORBextractor &right, const std::vector<cv::KeyPoint> &mvKeys,
                                    const cv::Mat &mDescriptors, const std::vector<cv::KeyPoint> &mvKeysRight,
                                    const cv::Mat &mDescriptorsRight, float mbf, float mb,
                                    std::vector<float> &mvuRight, std::vector<float> &mvDepth) {
        const std::vector<orbx_keypoint> kl = orbx_detail::pack(mvKeys), kr = orbx_detail::pack(mvKeysRight);
        const cv::Mat dl = mDescriptors.isContinuous() ? mDescriptors : mDescriptors.clone();
        const cv::Mat dr = mDescriptorsRight.isContinuous() ? mDescriptorsRight : mDescriptorsRight.clone();
        mvuRight.assign(kl.size(), -1.0f);
        mvDepth.assign(kl.size(), -1.0f);
        int kept = 0;
        orbx_detail::check(orbx_compute_stereo_matches(left.handle(), right.handle(), kl.data(), dl.data, (int)kl.size(),
                                                       kr.data(), dr.data, (int)kr.size(), mbf, mb, mvuRight.data(),
                                                       mvDepth.data(), &kept),
                           "ComputeStereoMatches");
        return kept;
    }

    // Frame::ComputeStereoFromRGBD (Frame.cc:679-701); imDepth is CV_32F.
    static void ComputeStereoFromRGBD(const std::vector<cv::KeyPoint> &mvKeys,
                                      const std::vector<cv::KeyPoint> &mvKeysUn, const cv::Mat &imDepth, float mbf,
                                      std::vector<float> &mvuRight, std::vector<float> &mvDepth) {
        assert(imDepth.type() == CV_32F);
        const std::vector<orbx_keypoint> k = orbx_detail::pack(mvKeys), ku = orbx_detail::pack(mvKeysUn);
        mvuRight.assign(k.size(), -1.0f);
        mvDepth.assign(k.size(), -1.0f);
        int kept = 0;
        orbx_detail::check(orbx_stereo_from_rgbd(orbx_detail::device_index(), k.data(), ku.data(), (int)k.size(),
                                                 imDepth.ptr<float>(), imDepth.cols, imDepth.rows, imDepth.step,
                                                 mbf, mvuRight.data(), mvDepth.data(), &kept),
                           "ComputeStereoFromRGBD");
    }
};

// The per-frame neighbours as free functions over the members
// they read and write (INTEGRATION.md shows the one-line forwarders).
struct OrbxFrameAux {
    // Frame::UndistortKeyPoints (Frame.cc:438-469); mK CV_32F 3x3, mDistCoef
    // CV_32F 4x1 or 5x1.
    static void UndistortKeyPoints(const std::vector<cv::KeyPoint> &mvKeys, const cv::Mat &mK,
                                   const cv::Mat &mDistCoef, std::vector<cv::KeyPoint> &mvKeysUn) {
        assert(mK.type() == CV_32F && mDistCoef.type() == CV_32F);
        const std::vector<orbx_keypoint> k = orbx_detail::pack(mvKeys);
        std::vector<orbx_keypoint> ku(k.size());
        float K[9], D[8];
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) K[3 * r + c] = mK.at<float>(r, c);
        const int nc = std::min(mDistCoef.rows * mDistCoef.cols, 8);
        for (int i = 0; i < nc; ++i) D[i] = mDistCoef.ptr<float>(0)[i];
        orbx_detail::check(orbx_undistort_keypoints(orbx_detail::device_index(), k.data(), (int)k.size(), K, D, nc,
                                                    ku.data()),
                           "UndistortKeyPoints");
        mvKeysUn = mvKeys;
        for (size_t i = 0; i < ku.size(); ++i) { mvKeysUn[i].pt.x = ku[i].x; mvKeysUn[i].pt.y = ku[i].y; }
    }

    // MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:288-361) for a batch
    // of map points: vvDescriptors[p] = point p's usable observation rows (1x32
    // CV_8U), in its observation order.  Returns each point's chosen row (-1:
    // none, mDescriptor unchanged).
    static std::vector<int> DistinctiveDescriptors(const std::vector<std::vector<cv::Mat>> &vvDescriptors) {
        std::vector<int32_t> off(vvDescriptors.size() + 1, 0);
        for (size_t p = 0; p < vvDescriptors.size(); ++p) off[p + 1] = off[p] + (int32_t)vvDescriptors[p].size();
        std::vector<uint8_t> desc(32 * (size_t)off.back());
        size_t r = 0;
        for (const auto &v : vvDescriptors)
            for (const cv::Mat &d : v) std::memcpy(&desc[32 * r++], d.ptr<uint8_t>(), 32);
        std::vector<int32_t> best(vvDescriptors.size(), -1);
        orbx_detail::check(orbx_distinctive_descriptors(orbx_detail::device_index(), desc.data(), off.data(),
                                                        (int)vvDescriptors.size(), best.data()),
                           "ComputeDistinctiveDescriptors");
        return std::vector<int>(best.begin(), best.end());
    }

    // Tracking::GrabImage* colour conversion (Tracking.cc:179-264): 3- or
    // 4-channel 8-bit input to gray in place; other input is left as is.
    static void ToGray(cv::Mat &im, bool mbRGB) {
        const int cn = im.channels();
        if (cn != 3 && cn != 4) return;
        cv::Mat gray(im.rows, im.cols, CV_8U);
        orbx_detail::check(orbx_cvt_gray(orbx_detail::device_index(), im.data, im.cols, im.rows, im.step, cn,
                                         mbRGB ? 1 : 0, gray.data, gray.step),
                           "cvtColor");
        im = gray;
    }
};

// ORBVocabulary = DBoW2::TemplatedVocabulary<FORB::TDescriptor, FORB> for the
// parts the per-frame path uses: the two loaders and transform(features, v,
// fv, levelsup) (TemplatedVocabulary.h:1140-1207, 1351-1547).  BowVector /
// FeatureVector are DBoW2's (std::map<WordId, WordValue> and
// std::map<NodeId, std::vector<unsigned int>>); any map-like types with
// clear() / operator[] work, so this header needs no DBoW2 include.
class OrbxVocabulary {
public:
    OrbxVocabulary() = default;
    OrbxVocabulary(const OrbxVocabulary &) = delete;
    OrbxVocabulary &operator=(const OrbxVocabulary &) = delete;
    ~OrbxVocabulary() { orbx_vocab_destroy(v_); }

    bool loadFromTextFile(const std::string &filename) { return load(filename, 0); }
    bool loadFromBinFile(const std::string &filename) { return load(filename, 1); }

    bool empty() const { return size() == 0; }
    unsigned int size() const {
        int nw = 0;
        if (v_) orbx_vocab_info(v_, nullptr, nullptr, nullptr, nullptr, nullptr, &nw);
        return (unsigned int)nw;
    }

    template <class BowVector, class FeatureVector>
    void transform(const std::vector<cv::Mat> &features, BowVector &v, FeatureVector &fv, int levelsup) const {
        v.clear();
        fv.clear();
        if (!v_ || features.empty()) return;
        const int n = (int)features.size();
        std::vector<uint8_t> desc(32 * (size_t)n);
        for (int i = 0; i < n; ++i) std::memcpy(&desc[32 * (size_t)i], features[i].ptr<uint8_t>(), 32);
        std::vector<uint32_t> bw(n), fn(n);
        std::vector<double> bv(n);
        std::vector<int32_t> fo(n + 1), ff(n);
        int nb = 0, nf = 0;
        orbx_detail::check(orbx_vocab_transform(v_, desc.data(), n, levelsup, bw.data(), bv.data(), &nb, fn.data(),
                                                fo.data(), ff.data(), &nf),
                           "ORBVocabulary::transform");
        for (int i = 0; i < nb; ++i) v[bw[i]] = bv[i];
        for (int j = 0; j < nf; ++j)
            for (int t = fo[j]; t < fo[j + 1]; ++t) fv[fn[j]].push_back((unsigned int)ff[t]);
    }

    orbx_vocab *handle() const { return v_; }

private:
    bool load(const std::string &filename, int format) {
        orbx_vocab_destroy(v_);
        v_ = nullptr;
        return orbx_vocab_load(orbx_detail::device_index(), filename.c_str(), format, &v_) == ORBX_OK;
    }
    orbx_vocab *v_ = nullptr;
};

}  // namespace ORB_SLAM2
