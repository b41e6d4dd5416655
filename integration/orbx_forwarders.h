// orbx_forwarders.h -- helpers the forwarders in integration/ share: the
// device tables (query rows, match frames, CSR FeatureVectors) built from the
// reference's Frame / KeyFrame / MapPoint members, and the batched forms of
// LocalMapping's per-keyframe search loops (LocalMapping_orbx.cc).  Include
// after the reference headers.
#pragma once
#include <cmath>
#include <cstring>
#include <set>
#include <vector>

#include "Frame.h"
#include "KeyFrame.h"
#include "MapPoint.h"
#include "orbx_orbslam2.hpp"

namespace ORB_SLAM2 {
namespace orbx_fwd {

// mvpMapPoints / vpMatched as the device's per-keypoint occupancy bits.
inline std::vector<uint8_t> occupancy(const std::vector<MapPoint *> &mps) {
    std::vector<uint8_t> s(mps.size(), 0);
    for (size_t i = 0; i < mps.size(); ++i)
        if (mps[i]) s[i] = (uint8_t)(1 | (mps[i]->Observations() > 0 ? 2 : 0));
    return s;
}

// The searched frame or keyframe: keypoints, descriptors, grid bounds.
template <class F>
OrbxMatcher::ProjFrame proj_frame(const F &f, const std::vector<uint8_t> *state, bool stereo, bool sigma) {
    OrbxMatcher::ProjFrame p;
    p.keys = &f.mvKeysUn;
    p.desc = &f.mDescriptors;
    p.uright = stereo ? &f.mvuRight : nullptr;
    p.mp_state = state;
    p.inv_sigma2 = sigma ? &f.mvInvLevelSigma2 : nullptr;
    p.min_x = f.mnMinX; p.max_x = f.mnMaxX; p.min_y = f.mnMinY; p.max_y = f.mnMaxY;
    return p;
}

inline orbx_proj_query row(float u, float v, float radius, int lmin, int lmax, float ur = -1.f, float ur_tol = 0.f,
                    float angle = 0.f, int flags = ORBX_QUERY_ACTIVE) {
    orbx_proj_query q;
    q.u = u; q.v = v; q.radius = radius; q.ur = ur; q.ur_tol = ur_tol;
    q.min_level = lmin; q.max_level = lmax; q.angle = angle; q.flags = flags;
    return q;
}

// Query descriptors as an n x 32 Mat, rows filled for the active points.
struct QueryTable {
    std::vector<orbx_proj_query> q;
    cv::Mat desc;
    explicit QueryTable(size_t n) : q(n, orbx_proj_query{}), desc((int)n, 32, CV_8U) {
        if (n) std::memset(desc.data, 0, n * 32);
    }
    void set(size_t i, const orbx_proj_query &r, const cv::Mat &d) {
        q[i] = r;
        std::memcpy(desc.ptr<uint8_t>((int)i), d.data, 32);
    }
};

// A point's projection through (R, t) and the keyframe's intrinsics, with the
// distance / viewing-angle / scale gates of the keyframe searches
// (ORBmatcher.cc:318-356, 850-885, 1010-1052).  Returns false when a gate
// rejects the point.
struct Projected { float u, v, invz; int level; };
inline bool project_kf(MapPoint *pMP, const cv::Mat &Rcw, const cv::Mat &tcw, const cv::Mat &Ow, KeyFrame *pKF,
                bool check_normal, Projected &o) {
    cv::Mat p3Dw = pMP->GetWorldPos();
    cv::Mat p3Dc = Rcw * p3Dw + tcw;
    if (p3Dc.at<float>(2) < 0.0f) return false;
    const float invz = 1 / p3Dc.at<float>(2);
    const float u = pKF->fx * (p3Dc.at<float>(0) * invz) + pKF->cx;
    const float v = pKF->fy * (p3Dc.at<float>(1) * invz) + pKF->cy;
    if (!pKF->IsInImage(u, v)) return false;
    const float maxD = pMP->GetMaxDistanceInvariance(), minD = pMP->GetMinDistanceInvariance();
    cv::Mat PO = p3Dw - Ow;
    const float dist = cv::norm(PO);
    if (dist < minD || dist > maxD) return false;
    if (check_normal && PO.dot(pMP->GetNormal()) < 0.5 * dist) return false;
    o.u = u; o.v = v; o.invz = invz; o.level = pMP->PredictScale(dist, pKF);
    return true;
}

// Scw = [sR t] -> (R, t / s, camera centre), ORBmatcher.cc:299-305.
inline void split_sim3(const cv::Mat &Scw, cv::Mat &Rcw, cv::Mat &tcw, cv::Mat &Ow) {
    cv::Mat sRcw = Scw.rowRange(0, 3).colRange(0, 3);
    const float scw = std::sqrt(sRcw.row(0).dot(sRcw.row(0)));
    Rcw = sRcw / scw;
    tcw = Scw.rowRange(0, 3).col(3) / scw;
    Ow = -Rcw.t() * tcw;
}

// DBoW2::FeatureVector (std::map<NodeId, vector<unsigned>>) as CSR arrays.
struct BowSide {
    std::vector<orbx_keypoint> keys;
    cv::Mat desc;
    std::vector<uint8_t> flags;
    std::vector<uint32_t> ids;
    std::vector<int32_t> off{0}, feat;
    template <class F>
    BowSide(const F &f, std::vector<uint8_t> fl) : keys(orbx_detail::pack(f.mvKeysUn)), flags(std::move(fl)) {
        desc = f.mDescriptors.isContinuous() ? f.mDescriptors : f.mDescriptors.clone();
        for (const auto &node : f.mFeatVec) {
            ids.push_back(node.first);
            feat.insert(feat.end(), node.second.begin(), node.second.end());
            off.push_back((int32_t)feat.size());
        }
    }
    orbx_bow_side side() const {
        orbx_bow_side s;
        s.keys = keys.data(); s.desc = desc.data; s.flags = flags.data(); s.n = (int)keys.size();
        s.node_ids = ids.data(); s.node_offsets = off.data(); s.node_features = feat.data(); s.nnodes = (int)ids.size();
        return s;
    }
};

// flags of a BoW side: bit0 = a usable feature, bit1 = mvuRight >= 0
template <class F, class Use>
std::vector<uint8_t> bow_flags(const F &f, Use use) {
    std::vector<uint8_t> fl(f.N, 0);
    for (int i = 0; i < f.N; ++i) fl[i] = (uint8_t)((use(i) ? 1 : 0) | (f.mvuRight[i] >= 0 ? 2 : 0));
    return fl;
}

inline bool good(const MapPoint *p) { return p && !p->isBad(); }

// SearchForTriangulation's geometry (ORBmatcher.cc:665-672): F12 row-major,
// the epipole of pKF1's centre in pKF2, then pKF2's mvScaleFactors and
// mvLevelSigma2.
inline std::vector<float> tri_row(KeyFrame *pKF1, KeyFrame *pKF2, const cv::Mat &F12) {
    cv::Mat C2 = pKF2->GetRotation() * pKF1->GetCameraCenter() + pKF2->GetTranslation();
    const float invz = 1.0f / C2.at<float>(2);
    std::vector<float> tri(11);
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) tri[3 * r + c] = F12.at<float>(r, c);
    tri[9] = pKF2->fx * C2.at<float>(0) * invz + pKF2->cx;
    tri[10] = pKF2->fy * C2.at<float>(1) * invz + pKF2->cy;
    tri.insert(tri.end(), pKF2->mvScaleFactors.begin(), pKF2->mvScaleFactors.end());
    tri.insert(tri.end(), pKF2->mvLevelSigma2.begin(), pKF2->mvLevelSigma2.end());
    return tri;
}

// SearchForTriangulation's usable features: no map point yet (and stereo when bOnlyStereo)
inline std::vector<uint8_t> tri_flags(KeyFrame *k, bool bOnlyStereo) {
    return bow_flags(*k, [k, bOnlyStereo](int i) { return !k->GetMapPoint(i) && (!bOnlyStereo || k->mvuRight[i] >= 0); });
}

}  // namespace orbx_fwd

// LocalMapping::SearchInNeighbors (LocalMapping.cc:531-538): the loop
//   for (pKFi : vpTargetKFs) matcher.Fuse(pKFi, vpMapPointMatches);
// of ORBmatcher(nnratio) as one device batch, with the same map edits.
int OrbxFuseIntoKeyFrames(const std::vector<KeyFrame *> &vpTargetKFs, const std::vector<MapPoint *> &vpMapPoints,
                          float th = 3.0f, float nnratio = 0.6f);

// LocalMapping::CreateNewMapPoints (LocalMapping.cc:276-315): the
// SearchForTriangulation(pKF1, vpNeighKFs[i], vF12[i], pairs, bOnlyStereo)
// of every neighbour (ORBmatcher(nnratio, false)) as one device batch, from
// pKF1's map points as they are now.  A feature of pKF1 that gets a map point
// from an earlier neighbour's triangulation is skipped by the reference's
// later searches: drop pairs with pKF1->GetMapPoint(idx1) != NULL when walking
// neighbour i.
std::vector<std::vector<std::pair<size_t, size_t>>> OrbxSearchForTriangulationBatch(
    KeyFrame *pKF1, const std::vector<KeyFrame *> &vpNeighKFs, const std::vector<cv::Mat> &vF12, bool bOnlyStereo,
    float nnratio = 0.6f);

}  // namespace ORB_SLAM2
