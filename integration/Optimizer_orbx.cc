// Optimizer_orbx.cc -- Optimizer::LocalBundleAdjustment (orb_slam2/src/
// Optimizer.cc:517-890) for a reference tree that links liborbx.so.  The
// collection of the local window and the tail that applies the result are the
// reference's; the g2o graph becomes the arrays orbx_local_ba takes, in the
// same order (cameras: local keyframes then fixed cameras; points in
// lLocalMapPoints order; one edge per usable observation), and the
// optimisation runs on the device.  The other Optimizer functions stay as
// they are: replace only this function's body in Optimizer.cc.
//
// tests/cxx/forwarders_test.cpp compiles this file against test stand-ins of
// the reference headers and checks it on the GPU against the same steps over
// the CPU oracle's solver.
#include <cstring>
#include <list>
#include <map>
#include <mutex>
#include <vector>

#include "Optimizer.h"
#include "orbx_orbslam2.hpp"

namespace ORB_SLAM2 {

void Optimizer::LocalBundleAdjustment(KeyFrame *pKF, bool *pbStopFlag, Map *pMap) {
    // the local window, exactly as :521-590
    std::list<KeyFrame *> lLocalKeyFrames{pKF};
    pKF->mnBALocalForKF = pKF->mnId;
    for (KeyFrame *pKFi : pKF->GetVectorCovisibleKeyFrames()) {
        pKFi->mnBALocalForKF = pKF->mnId;
        if (!pKFi->isBad()) lLocalKeyFrames.push_back(pKFi);
    }
    std::list<MapPoint *> lLocalMapPoints;
    for (KeyFrame *pKFi : lLocalKeyFrames)
        for (MapPoint *pMP : pKFi->GetMapPointMatches())
            if (pMP && !pMP->isBad() && pMP->mnBALocalForKF != pKF->mnId) {
                lLocalMapPoints.push_back(pMP);
                pMP->mnBALocalForKF = pKF->mnId;
            }
    std::list<KeyFrame *> lFixedCameras;
    for (MapPoint *pMP : lLocalMapPoints)
        for (const auto &obs : pMP->GetObservations()) {
            KeyFrame *pKFi = obs.first;
            if (pKFi->mnBALocalForKF != pKF->mnId && pKFi->mnBAFixedForKF != pKF->mnId) {
                pKFi->mnBAFixedForKF = pKF->mnId;
                if (!pKFi->isBad()) lFixedCameras.push_back(pKFi);
            }
        }

    // the graph as arrays (:608-757)
    std::vector<KeyFrame *> cams(lLocalKeyFrames.begin(), lLocalKeyFrames.end());
    cams.insert(cams.end(), lFixedCameras.begin(), lFixedCameras.end());
    std::map<KeyFrame *, int> camIndex;
    std::vector<float> Tcw(12 * cams.size());
    std::vector<uint8_t> fixed(cams.size());
    for (size_t c = 0; c < cams.size(); ++c) {
        camIndex[cams[c]] = (int)c;
        const cv::Mat T = cams[c]->GetPose();
        for (int r = 0; r < 3; ++r) std::memcpy(&Tcw[12 * c + 4 * r], T.ptr<float>(r), 4 * sizeof(float));
        fixed[c] = c >= lLocalKeyFrames.size() || cams[c]->mnId == 0;
    }
    std::vector<MapPoint *> points(lLocalMapPoints.begin(), lLocalMapPoints.end());
    std::vector<float> Xw(3 * points.size());
    std::vector<orbx_ba_edge> edges;
    std::vector<std::pair<KeyFrame *, MapPoint *>> edgeOwner;
    for (size_t p = 0; p < points.size(); ++p) {
        MapPoint *pMP = points[p];
        const cv::Mat X = pMP->GetWorldPos();
        for (int k = 0; k < 3; ++k) Xw[3 * p + k] = X.at<float>(k);
        for (const auto &obs : pMP->GetObservations()) {
            KeyFrame *pKFi = obs.first;
            if (pKFi->isBad()) continue;
            const cv::KeyPoint &kpUn = pKFi->mvKeysUn[obs.second];
            orbx_ba_edge e;
            e.cam = camIndex.at(pKFi);
            e.point = (int32_t)p;
            e.u = kpUn.pt.x;
            e.v = kpUn.pt.y;
            e.ur = pKFi->mvuRight[obs.second];
            e.inv_sigma2 = pKFi->mvInvLevelSigma2[kpUn.octave];
            e.fx = pKFi->fx; e.fy = pKFi->fy; e.cx = pKFi->cx; e.cy = pKFi->cy; e.bf = pKFi->mbf;
            edges.push_back(e);
            edgeOwner.push_back(std::make_pair(pKFi, pMP));
        }
    }
    if (pbStopFlag && *pbStopFlag) return;   // :759-761

    // 5 robust iterations, outlier removal, 10 more (:764-813).  The device
    // runs both passes in one call, so a stop request (another thread) raised
    // after the check above is honoured at the launch: the second pass is
    // skipped (iters2 = 0), as :769-771 would skip it
    std::vector<float> Tout(Tcw.size()), Xout(Xw.size());
    std::vector<uint8_t> outlier(edges.size(), 0);
    const int iters2 = pbStopFlag && *pbStopFlag ? 0 : 10;
    orbx_detail::check(orbx_local_ba(orbx_detail::device_index(), Tcw.data(), fixed.data(), (int)cams.size(),
                                     Xw.data(), (int)points.size(), edges.data(), (int)edges.size(), 5, iters2,
                                     Tout.data(), Xout.data(), outlier.data(), nullptr),
                       "LocalBundleAdjustment");

    // :818-852: the mono edges' outliers, then the stereo edges'
    std::vector<std::pair<KeyFrame *, MapPoint *>> vToErase;
    for (int stereo = 0; stereo < 2; ++stereo)
        for (size_t e = 0; e < edges.size(); ++e)
            if ((edges[e].ur >= 0) == (stereo == 1) && outlier[e] && !edgeOwner[e].second->isBad())
                vToErase.push_back(edgeOwner[e]);

    std::unique_lock<std::mutex> lock(pMap->mMutexMapUpdate);
    for (auto &kp : vToErase) {
        kp.first->EraseMapPointMatch(kp.second);
        kp.second->EraseObservation(kp.first);
    }
    for (size_t c = 0; c < lLocalKeyFrames.size(); ++c) {   // :873-879
        cv::Mat T = cv::Mat::eye(4, 4, CV_32F);
        for (int r = 0; r < 3; ++r) std::memcpy(T.ptr<float>(r), &Tout[12 * c + 4 * r], 4 * sizeof(float));
        cams[c]->SetPose(T);
    }
    for (size_t p = 0; p < points.size(); ++p) {   // :883-889
        cv::Mat X(3, 1, CV_32F);
        for (int k = 0; k < 3; ++k) X.at<float>(k) = Xout[3 * p + k];
        points[p]->SetWorldPos(X);
        points[p]->UpdateNormalAndDepth();
    }
}

}  // namespace ORB_SLAM2
