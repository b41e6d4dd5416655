// LocalMapping_orbx.cc -- the two per-keyframe search loops of
// orb_slam2/src/LocalMapping.cc as one device batch each (declared in
// orbx_forwarders.h).  Every problem of a batch is exactly the single call
// the reference makes; what the reference's loop changes between calls is
// replayed here (Fuse) or left to the caller's loop (triangulation), so the
// map ends as the sequential reference leaves it.
//
// tests/cxx/forwarders_test.cpp runs both against the sequential reference
// loop on the GPU (and on the oracle).
#include <memory>

#include "ORBmatcher.h"
#include "orbx_forwarders.h"

namespace ORB_SLAM2 {

using namespace orbx_fwd;

int OrbxFuseIntoKeyFrames(const std::vector<KeyFrame *> &vpTargetKFs, const std::vector<MapPoint *> &vpMapPoints,
                          float th, float nnratio) {
    const size_t nk = vpTargetKFs.size(), np = vpMapPoints.size();
    // the points' descriptors as the batch searches them
    std::vector<cv::Mat> desc0(np);
    for (size_t i = 0; i < np; ++i)
        if (vpMapPoints[i] && !vpMapPoints[i]->isBad()) desc0[i] = vpMapPoints[i]->GetDescriptor();
    // one problem per keyframe: the rows of Fuse(pKF, vpMapPoints, th)
    std::vector<OrbxMatcher::ProjFrame> frames;
    std::vector<std::vector<orbx_proj_query>> rows;
    std::vector<cv::Mat> descs;
    for (KeyFrame *pKF : vpTargetKFs) {
        const cv::Mat Rcw = pKF->GetRotation(), tcw = pKF->GetTranslation(), Ow = pKF->GetCameraCenter();
        QueryTable t(np);
        for (size_t i = 0; i < np; ++i) {
            MapPoint *pMP = vpMapPoints[i];
            Projected p;
            if (desc0[i].empty() || !project_kf(pMP, Rcw, tcw, Ow, pKF, true, p)) continue;
            t.set(i, row(p.u, p.v, th * pKF->mvScaleFactors[p.level], p.level - 1, p.level, p.u - pKF->mbf * p.invz),
                  desc0[i]);
        }
        frames.push_back(proj_frame(*pKF, nullptr, true, true));
        rows.push_back(t.q);
        descs.push_back(t.desc);
    }
    std::vector<std::vector<int>> qi, qd, kfinal;
    OrbxMatcher::SearchByProjectionBatch(ORBX_PROJ_FUSE, frames, rows, descs, ORBmatcher::TH_LOW, nnratio, false, qi,
                                         qd, kfinal);
    // the edits keyframe by keyframe, point by point, as the sequential calls
    // make them (ORBmatcher.cc:844-974)
    int nFused = 0;
    for (size_t k = 0; k < nk; ++k) {
        KeyFrame *pKF = vpTargetKFs[k];
        for (size_t i = 0; i < np; ++i) {
            MapPoint *pMP = vpMapPoints[i];
            if (!(rows[k][i].flags & ORBX_QUERY_ACTIVE) || pMP->isBad() || pMP->IsInKeyFrame(pKF)) continue;
            int idx = qi[k][i], dist = qd[k][i];
            // a Replace in an earlier keyframe that this point survived
            // recomputed its descriptor (MapPoint.cc:254): the reference
            // searches this keyframe with the new one
            const cv::Mat d = pMP->GetDescriptor();
            if (ORBmatcher::DescriptorDistance(d, desc0[i]) != 0)
                OrbxMatcher::SearchOneRow(ORBX_PROJ_FUSE, frames[k], rows[k][i], d, ORBmatcher::TH_LOW, nnratio, idx,
                                          dist);
            if (idx < 0 || dist > ORBmatcher::TH_LOW) continue;
            MapPoint *pMPinKF = pKF->GetMapPoint(idx);
            if (pMPinKF) {
                if (!pMPinKF->isBad()) {
                    if (pMPinKF->Observations() > pMP->Observations()) pMP->Replace(pMPinKF);
                    else pMPinKF->Replace(pMP);
                }
            } else {
                pMP->AddObservation(pKF, idx);
                pKF->AddMapPoint(pMP, idx);
            }
            nFused++;
        }
    }
    return nFused;
}

std::vector<std::vector<std::pair<size_t, size_t>>> OrbxSearchForTriangulationBatch(
    KeyFrame *pKF1, const std::vector<KeyFrame *> &vpNeighKFs, const std::vector<cv::Mat> &vF12, bool bOnlyStereo,
    float nnratio) {
    const size_t nk = vpNeighKFs.size();
    std::vector<std::vector<std::pair<size_t, size_t>>> pairs(nk);
    if (nk == 0) return pairs;
    const BowSide a(*pKF1, tri_flags(pKF1, bOnlyStereo));
    std::vector<std::unique_ptr<BowSide>> b;   // the sides' arrays must stay put
    std::vector<orbx_bow_side> A(nk, a.side()), B;
    std::vector<std::vector<float>> tri;
    for (size_t i = 0; i < nk; ++i) {
        b.emplace_back(new BowSide(*vpNeighKFs[i], tri_flags(vpNeighKFs[i], bOnlyStereo)));
        B.push_back(b.back()->side());
        tri.push_back(tri_row(pKF1, vpNeighKFs[i], vF12[i]));
    }
    std::vector<std::vector<int>> ma, mb;
    OrbxMatcher::SearchByBoWBatch(ORBX_BOW_TRIANGULATION, A, B, tri, vpNeighKFs[0]->mnScaleLevels, nnratio, false, ma,
                                  mb);
    for (size_t i = 0; i < nk; ++i)
        for (int idx1 = 0; idx1 < pKF1->N; ++idx1)
            if (ma[i][idx1] >= 0) pairs[i].push_back(std::make_pair((size_t)idx1, (size_t)ma[i][idx1]));
    return pairs;
}

}  // namespace ORB_SLAM2
