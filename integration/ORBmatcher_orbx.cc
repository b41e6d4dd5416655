// ORBmatcher_orbx.cc -- the body of orb_slam2/src/ORBmatcher.cc for a
// reference tree that links liborbx.so: the same class and signatures
// (ORBmatcher.h:41-89), each search a forwarder.  The per-point pose algebra
// and the reference's skip tests stay here, on the caller's cv::Mat types;
// the device runs the grid windows, the Hamming distances, the greedy
// assignment and the rotation check (include/orbx.h).  Fuse's map edits stay
// here too, in query order.
//
// Build: replace ORBmatcher.cc by this file and add include/ of this repo and
// liborbx.so.  tests/cxx/forwarders_test.cpp compiles it
// against test stand-ins of the reference headers and checks every method on
// the GPU against a CPU restatement of the reference method.
#include <cmath>
#include <cstring>
#include <set>
#include <vector>

#include "ORBmatcher.h"
#include "orbx_forwarders.h"

namespace ORB_SLAM2 {

const int ORBmatcher::TH_HIGH = 100;
const int ORBmatcher::TH_LOW = 50;
const int ORBmatcher::HISTO_LENGTH = 30;

ORBmatcher::ORBmatcher(float nnratio, bool checkOri) : mfNNratio(nnratio), mbCheckOrientation(checkOri) {}

int ORBmatcher::DescriptorDistance(const cv::Mat &a, const cv::Mat &b) { return OrbxMatcher::DescriptorDistance(a, b); }

float ORBmatcher::RadiusByViewingCos(const float &viewCos) { return viewCos > 0.998 ? 2.5 : 4.0; }

using namespace orbx_fwd;

// ---- SearchByProjection(Frame&, const vector<MapPoint*>&, th)  ORBmatcher.cc:45-129
int ORBmatcher::SearchByProjection(Frame &F, const std::vector<MapPoint *> &vpMapPoints, const float th) {
    QueryTable t(vpMapPoints.size());
    for (size_t i = 0; i < vpMapPoints.size(); ++i) {
        MapPoint *pMP = vpMapPoints[i];
        if (!pMP->mbTrackInView || pMP->isBad()) continue;
        const int lvl = pMP->mnTrackScaleLevel;
        float r = RadiusByViewingCos(pMP->mTrackViewCos);
        if (th != 1.0) r *= th;
        const float rs = r * F.mvScaleFactors[lvl];
        t.set(i, row(pMP->mTrackProjX, pMP->mTrackProjY, rs, lvl - 1, lvl, pMP->mTrackProjXR, rs, 0.f,
                     ORBX_QUERY_ACTIVE | (pMP->Observations() > 0 ? ORBX_QUERY_BLOCKS : 0)),
              pMP->GetDescriptor());
    }
    const std::vector<uint8_t> st = occupancy(F.mvpMapPoints);
    std::vector<int> qi, qd, kfinal;
    const int n = OrbxMatcher::SearchByProjectionTable(ORBX_PROJ_LOCALMAP, proj_frame(F, &st, true, false), t.q,
                                                       t.desc, TH_HIGH, mfNNratio, false, qi, qd, kfinal);
    for (int i = 0; i < F.N; ++i)
        if (kfinal[i] >= 0) F.mvpMapPoints[i] = vpMapPoints[kfinal[i]];
    return n;
}

// ---- SearchByProjection(Frame&, const Frame&, th, bMono)  ORBmatcher.cc:1330-1472
int ORBmatcher::SearchByProjection(Frame &CurrentFrame, const Frame &LastFrame, const float th, const bool bMono) {
    const cv::Mat Rcw = CurrentFrame.mTcw.rowRange(0, 3).colRange(0, 3);
    const cv::Mat tcw = CurrentFrame.mTcw.rowRange(0, 3).col(3);
    const cv::Mat twc = -Rcw.t() * tcw;
    const cv::Mat Rlw = LastFrame.mTcw.rowRange(0, 3).colRange(0, 3);
    const cv::Mat tlw = LastFrame.mTcw.rowRange(0, 3).col(3);
    const cv::Mat tlc = Rlw * twc + tlw;
    const bool bForward = tlc.at<float>(2) > CurrentFrame.mb && !bMono;
    const bool bBackward = -tlc.at<float>(2) > CurrentFrame.mb && !bMono;
    QueryTable t(LastFrame.N);
    for (int i = 0; i < LastFrame.N; ++i) {
        MapPoint *pMP = LastFrame.mvpMapPoints[i];
        if (!pMP || LastFrame.mvbOutlier[i]) continue;
        cv::Mat x3Dc = Rcw * pMP->GetWorldPos() + tcw;
        const float xc = x3Dc.at<float>(0), yc = x3Dc.at<float>(1);
        const float invzc = 1.0 / x3Dc.at<float>(2);
        if (invzc < 0) continue;
        const float u = CurrentFrame.fx * xc * invzc + CurrentFrame.cx;
        const float v = CurrentFrame.fy * yc * invzc + CurrentFrame.cy;
        if (u < CurrentFrame.mnMinX || u > CurrentFrame.mnMaxX || v < CurrentFrame.mnMinY || v > CurrentFrame.mnMaxY)
            continue;
        const int o = LastFrame.mvKeys[i].octave;
        const float radius = th * CurrentFrame.mvScaleFactors[o];
        const int lmin = bForward ? o : (bBackward ? 0 : o - 1), lmax = bForward ? -1 : (bBackward ? o : o + 1);
        t.set(i, row(u, v, radius, lmin, lmax, u - CurrentFrame.mbf * invzc, radius, LastFrame.mvKeysUn[i].angle,
                     ORBX_QUERY_ACTIVE | (pMP->Observations() > 0 ? ORBX_QUERY_BLOCKS : 0)),
              pMP->GetDescriptor());
    }
    const std::vector<uint8_t> st = occupancy(CurrentFrame.mvpMapPoints);
    std::vector<int> qi, qd, kfinal;
    const int n = OrbxMatcher::SearchByProjectionTable(ORBX_PROJ_LASTFRAME, proj_frame(CurrentFrame, &st, true, false),
                                                       t.q, t.desc, TH_HIGH, mfNNratio, mbCheckOrientation, qi, qd,
                                                       kfinal);
    for (int i = 0; i < CurrentFrame.N; ++i) {
        if (kfinal[i] >= 0) CurrentFrame.mvpMapPoints[i] = LastFrame.mvpMapPoints[kfinal[i]];
        else if (kfinal[i] == -2) CurrentFrame.mvpMapPoints[i] = static_cast<MapPoint *>(NULL);
    }
    return n;
}

// ---- SearchByProjection(Frame&, KeyFrame*, set, th, ORBdist)  ORBmatcher.cc:1474-1601
int ORBmatcher::SearchByProjection(Frame &CurrentFrame, KeyFrame *pKF, const std::set<MapPoint *> &sAlreadyFound,
                                   const float th, const int ORBdist) {
    const cv::Mat Rcw = CurrentFrame.mTcw.rowRange(0, 3).colRange(0, 3);
    const cv::Mat tcw = CurrentFrame.mTcw.rowRange(0, 3).col(3);
    const cv::Mat Ow = -Rcw.t() * tcw;
    const std::vector<MapPoint *> vpMPs = pKF->GetMapPointMatches();
    QueryTable t(vpMPs.size());
    for (size_t i = 0; i < vpMPs.size(); ++i) {
        MapPoint *pMP = vpMPs[i];
        if (!good(pMP) || sAlreadyFound.count(pMP)) continue;
        cv::Mat x3Dw = pMP->GetWorldPos();
        cv::Mat x3Dc = Rcw * x3Dw + tcw;
        const float invzc = 1.0 / x3Dc.at<float>(2);
        const float u = CurrentFrame.fx * x3Dc.at<float>(0) * invzc + CurrentFrame.cx;
        const float v = CurrentFrame.fy * x3Dc.at<float>(1) * invzc + CurrentFrame.cy;
        if (u < CurrentFrame.mnMinX || u > CurrentFrame.mnMaxX || v < CurrentFrame.mnMinY || v > CurrentFrame.mnMaxY)
            continue;
        cv::Mat PO = x3Dw - Ow;
        const float dist3D = cv::norm(PO);
        if (dist3D < pMP->GetMinDistanceInvariance() || dist3D > pMP->GetMaxDistanceInvariance()) continue;
        const int lvl = pMP->PredictScale(dist3D, &CurrentFrame);
        const float radius = th * CurrentFrame.mvScaleFactors[lvl];
        t.set(i, row(u, v, radius, lvl - 1, lvl + 1, -1.f, 0.f, pKF->mvKeysUn[i].angle), pMP->GetDescriptor());
    }
    const std::vector<uint8_t> st = occupancy(CurrentFrame.mvpMapPoints);
    std::vector<int> qi, qd, kfinal;
    const int n = OrbxMatcher::SearchByProjectionTable(ORBX_PROJ_KEYFRAME, proj_frame(CurrentFrame, &st, false, false),
                                                       t.q, t.desc, ORBdist, mfNNratio, mbCheckOrientation, qi, qd,
                                                       kfinal);
    for (int i = 0; i < CurrentFrame.N; ++i) {
        if (kfinal[i] >= 0) CurrentFrame.mvpMapPoints[i] = vpMPs[kfinal[i]];
        else if (kfinal[i] == -2) CurrentFrame.mvpMapPoints[i] = NULL;
    }
    return n;
}

// ---- SearchByProjection(KeyFrame*, Scw, vpPoints, vpMatched, th)  ORBmatcher.cc:291-404
int ORBmatcher::SearchByProjection(KeyFrame *pKF, cv::Mat Scw, const std::vector<MapPoint *> &vpPoints,
                                   std::vector<MapPoint *> &vpMatched, int th) {
    cv::Mat Rcw, tcw, Ow;
    split_sim3(Scw, Rcw, tcw, Ow);
    std::set<MapPoint *> found(vpMatched.begin(), vpMatched.end());
    found.erase(static_cast<MapPoint *>(NULL));
    QueryTable t(vpPoints.size());
    for (size_t i = 0; i < vpPoints.size(); ++i) {
        MapPoint *pMP = vpPoints[i];
        Projected p;
        if (pMP->isBad() || found.count(pMP) || !project_kf(pMP, Rcw, tcw, Ow, pKF, true, p)) continue;
        t.set(i, row(p.u, p.v, th * pKF->mvScaleFactors[p.level], p.level - 1, p.level), pMP->GetDescriptor());
    }
    std::vector<uint8_t> st(vpMatched.size(), 0);
    for (size_t i = 0; i < vpMatched.size(); ++i) st[i] = vpMatched[i] ? 1 : 0;
    std::vector<int> qi, qd, kfinal;
    const int n = OrbxMatcher::SearchByProjectionTable(ORBX_PROJ_SIM3, proj_frame(*pKF, &st, false, false), t.q,
                                                       t.desc, TH_LOW, mfNNratio, false, qi, qd, kfinal);
    for (size_t i = 0; i < vpMatched.size(); ++i)
        if (kfinal[i] >= 0) vpMatched[i] = vpPoints[kfinal[i]];
    return n;
}

// ---- SearchByBoW(KeyFrame*, Frame&, vpMapPointMatches)  ORBmatcher.cc:160-289
int ORBmatcher::SearchByBoW(KeyFrame *pKF, Frame &F, std::vector<MapPoint *> &vpMapPointMatches) {
    const std::vector<MapPoint *> vpMapPointsKF = pKF->GetMapPointMatches();
    const BowSide A(*pKF, bow_flags(*pKF, [&](int i) { return good(vpMapPointsKF[i]); }));
    const BowSide B(F, bow_flags(F, [](int) { return true; }));
    std::vector<int> ma, mb;
    const int n = OrbxMatcher::SearchByBoWTable(ORBX_BOW_KF_FRAME, A.side(), B.side(), mfNNratio, mbCheckOrientation,
                                                {}, 0, ma, mb);
    vpMapPointMatches.assign(F.N, static_cast<MapPoint *>(NULL));
    for (int j = 0; j < F.N; ++j)
        if (mb[j] >= 0) vpMapPointMatches[j] = vpMapPointsKF[mb[j]];
    return n;
}

// ---- SearchByBoW(KeyFrame*, KeyFrame*, vpMatches12)  ORBmatcher.cc:524-657
int ORBmatcher::SearchByBoW(KeyFrame *pKF1, KeyFrame *pKF2, std::vector<MapPoint *> &vpMatches12) {
    const std::vector<MapPoint *> vpMapPoints1 = pKF1->GetMapPointMatches();
    const std::vector<MapPoint *> vpMapPoints2 = pKF2->GetMapPointMatches();
    const BowSide A(*pKF1, bow_flags(*pKF1, [&](int i) { return good(vpMapPoints1[i]); }));
    const BowSide B(*pKF2, bow_flags(*pKF2, [&](int i) { return good(vpMapPoints2[i]); }));
    std::vector<int> ma, mb;
    const int n = OrbxMatcher::SearchByBoWTable(ORBX_BOW_KF_KF, A.side(), B.side(), mfNNratio, mbCheckOrientation, {},
                                                0, ma, mb);
    vpMatches12.assign(vpMapPoints1.size(), static_cast<MapPoint *>(NULL));
    for (size_t i = 0; i < vpMapPoints1.size(); ++i)
        if (ma[i] >= 0) vpMatches12[i] = vpMapPoints2[ma[i]];
    return n;
}

// ---- SearchForInitialization  ORBmatcher.cc:406-521 (F2's grid: its bounds mnMinX..mnMaxY, Frame.cc:475-499)
int ORBmatcher::SearchForInitialization(Frame &F1, Frame &F2, std::vector<cv::Point2f> &vbPrevMatched,
                                        std::vector<int> &vnMatches12, int windowSize) {
    return OrbxMatcher::SearchForInitialization(F1.mvKeysUn, F1.mDescriptors, F2.mvKeysUn, F2.mDescriptors,
                                                F2.mnMinX, F2.mnMaxX, F2.mnMinY, F2.mnMaxY, vbPrevMatched,
                                                vnMatches12, windowSize, mfNNratio, mbCheckOrientation);
}

// ---- SearchForTriangulation  ORBmatcher.cc:659-825
int ORBmatcher::SearchForTriangulation(KeyFrame *pKF1, KeyFrame *pKF2, cv::Mat F12,
                                       std::vector<pair<size_t, size_t>> &vMatchedPairs, const bool bOnlyStereo) {
    const BowSide A(*pKF1, tri_flags(pKF1, bOnlyStereo)), B(*pKF2, tri_flags(pKF2, bOnlyStereo));
    const std::vector<float> tri = tri_row(pKF1, pKF2, F12);
    std::vector<int> ma, mb;
    const int n = OrbxMatcher::SearchByBoWTable(ORBX_BOW_TRIANGULATION, A.side(), B.side(), mfNNratio,
                                                mbCheckOrientation, tri, pKF2->mnScaleLevels, ma, mb);
    vMatchedPairs.clear();
    for (int i = 0; i < pKF1->N; ++i)
        if (ma[i] >= 0) vMatchedPairs.push_back(std::make_pair((size_t)i, (size_t)ma[i]));
    return n;
}

// ---- SearchBySim3  ORBmatcher.cc:1104-1328
int ORBmatcher::SearchBySim3(KeyFrame *pKF1, KeyFrame *pKF2, std::vector<MapPoint *> &vpMatches12, const float &s12,
                             const cv::Mat &R12, const cv::Mat &t12, const float th) {
    const float fx = pKF1->fx, fy = pKF1->fy, cx = pKF1->cx, cy = pKF1->cy;
    const cv::Mat R1w = pKF1->GetRotation(), t1w = pKF1->GetTranslation();
    const cv::Mat R2w = pKF2->GetRotation(), t2w = pKF2->GetTranslation();
    const cv::Mat sR12 = s12 * R12, sR21 = (1.0 / s12) * R12.t(), t21 = -sR21 * t12;
    const std::vector<MapPoint *> vpMapPoints1 = pKF1->GetMapPointMatches(), vpMapPoints2 = pKF2->GetMapPointMatches();
    const int N1 = (int)vpMapPoints1.size(), N2 = (int)vpMapPoints2.size();
    std::vector<bool> matched1(N1, false), matched2(N2, false);
    for (int i = 0; i < N1; ++i)
        if (MapPoint *pMP = vpMatches12[i]) {
            matched1[i] = true;
            const int idx2 = pMP->GetIndexInKeyFrame(pKF2);
            if (idx2 >= 0 && idx2 < N2) matched2[idx2] = true;
        }
    // one side's rows: its points through (R, t) then (sR, t') into the other keyframe
    auto side = [&](const std::vector<MapPoint *> &mps, const std::vector<bool> &done, const cv::Mat &Rw,
                    const cv::Mat &tw, const cv::Mat &sR, const cv::Mat &tt, KeyFrame *other) {
        QueryTable t(mps.size());
        for (size_t i = 0; i < mps.size(); ++i) {
            MapPoint *pMP = mps[i];
            if (!pMP || done[i] || pMP->isBad()) continue;
            cv::Mat p3Dc = sR * (Rw * pMP->GetWorldPos() + tw) + tt;
            if (p3Dc.at<float>(2) < 0.0) continue;
            const float invz = 1.0 / p3Dc.at<float>(2);
            const float u = fx * (p3Dc.at<float>(0) * invz) + cx, v = fy * (p3Dc.at<float>(1) * invz) + cy;
            if (!other->IsInImage(u, v)) continue;
            const float dist3D = cv::norm(p3Dc);
            if (dist3D < pMP->GetMinDistanceInvariance() || dist3D > pMP->GetMaxDistanceInvariance()) continue;
            const int lvl = pMP->PredictScale(dist3D, other);
            t.set(i, row(u, v, th * other->mvScaleFactors[lvl], lvl - 1, lvl), pMP->GetDescriptor());
        }
        return t;
    };
    const QueryTable q1 = side(vpMapPoints1, matched1, R1w, t1w, sR21, t21, pKF2);
    const QueryTable q2 = side(vpMapPoints2, matched2, R2w, t2w, sR12, t12, pKF1);
    const std::vector<orbx_keypoint> k1 = orbx_detail::pack(pKF1->mvKeysUn), k2 = orbx_detail::pack(pKF2->mvKeysUn);
    const cv::Mat d1 = pKF1->mDescriptors.isContinuous() ? pKF1->mDescriptors : pKF1->mDescriptors.clone();
    const cv::Mat d2 = pKF2->mDescriptors.isContinuous() ? pKF2->mDescriptors : pKF2->mDescriptors.clone();
    auto mframe = [](const std::vector<orbx_keypoint> &k, const cv::Mat &d, const KeyFrame *f) {
        orbx_match_frame m{};
        m.keys = k.data(); m.desc = d.data; m.n = (int)k.size();
        m.min_x = f->mnMinX; m.max_x = f->mnMaxX; m.min_y = f->mnMinY; m.max_y = f->mnMaxY;
        return m;
    };
    const orbx_match_frame f1 = mframe(k1, d1, pKF1), f2 = mframe(k2, d2, pKF2);
    std::vector<int32_t> m12(N1, -1);
    int nFound = 0;
    orbx_detail::check(orbx_search_by_sim3(orbx_detail::device_index(), &f1, &f2, q1.q.data(), q1.desc.data,
                                           q2.q.data(), q2.desc.data, TH_HIGH, m12.data(), &nFound),
                       "SearchBySim3");
    for (int i = 0; i < N1; ++i)
        if (m12[i] >= 0) vpMatches12[i] = vpMapPoints2[m12[i]];
    return nFound;
}

// ---- Fuse(KeyFrame*, vpMapPoints, th)  ORBmatcher.cc:827-977
int ORBmatcher::Fuse(KeyFrame *pKF, const vector<MapPoint *> &vpMapPoints, const float th) {
    const cv::Mat Rcw = pKF->GetRotation(), tcw = pKF->GetTranslation(), Ow = pKF->GetCameraCenter();
    // rows for every point the geometry admits; isBad() / IsInKeyFrame() are
    // tested at each point's turn below, after the edits of the points before
    // it, as the reference tests them.  (No point's descriptor changes before
    // its own turn within one call: a Replace recomputes only the survivor,
    // which is the current point or one already in pKF.  The batched form
    // over several keyframes does need the re-search, INTEGRATION.md.)
    QueryTable t(vpMapPoints.size());
    for (size_t i = 0; i < vpMapPoints.size(); ++i) {
        MapPoint *pMP = vpMapPoints[i];
        Projected p;
        if (!pMP || pMP->isBad() || !project_kf(pMP, Rcw, tcw, Ow, pKF, true, p)) continue;
        const float radius = th * pKF->mvScaleFactors[p.level];
        t.set(i, row(p.u, p.v, radius, p.level - 1, p.level, p.u - pKF->mbf * p.invz), pMP->GetDescriptor());
    }
    std::vector<int> qi, qd, kfinal;
    OrbxMatcher::SearchByProjectionTable(ORBX_PROJ_FUSE, proj_frame(*pKF, nullptr, true, true), t.q, t.desc, TH_LOW,
                                         mfNNratio, false, qi, qd, kfinal);
    int nFused = 0;
    for (size_t i = 0; i < vpMapPoints.size(); ++i) {
        MapPoint *pMP = vpMapPoints[i];
        if (qi[i] < 0 || pMP->isBad() || pMP->IsInKeyFrame(pKF)) continue;
        MapPoint *pMPinKF = pKF->GetMapPoint(qi[i]);
        if (pMPinKF) {
            if (!pMPinKF->isBad()) {
                if (pMPinKF->Observations() > pMP->Observations()) pMP->Replace(pMPinKF);
                else pMPinKF->Replace(pMP);
            }
        } else {
            pMP->AddObservation(pKF, qi[i]);
            pKF->AddMapPoint(pMP, qi[i]);
        }
        nFused++;
    }
    return nFused;
}

// ---- Fuse(KeyFrame*, Scw, vpPoints, th, vpReplacePoint)  ORBmatcher.cc:979-1102
int ORBmatcher::Fuse(KeyFrame *pKF, cv::Mat Scw, const std::vector<MapPoint *> &vpPoints, float th,
                     vector<MapPoint *> &vpReplacePoint) {
    cv::Mat Rcw, tcw, Ow;
    split_sim3(Scw, Rcw, tcw, Ow);
    const std::set<MapPoint *> spAlreadyFound = pKF->GetMapPoints();
    QueryTable t(vpPoints.size());
    for (size_t i = 0; i < vpPoints.size(); ++i) {
        MapPoint *pMP = vpPoints[i];
        Projected p;
        if (pMP->isBad() || spAlreadyFound.count(pMP) || !project_kf(pMP, Rcw, tcw, Ow, pKF, true, p)) continue;
        t.set(i, row(p.u, p.v, th * pKF->mvScaleFactors[p.level], p.level - 1, p.level), pMP->GetDescriptor());
    }
    std::vector<int> qi, qd, kfinal;
    OrbxMatcher::SearchByProjectionTable(ORBX_PROJ_FUSE_SIM3, proj_frame(*pKF, nullptr, false, false), t.q, t.desc,
                                         TH_LOW, mfNNratio, false, qi, qd, kfinal);
    int nFused = 0;
    for (size_t i = 0; i < vpPoints.size(); ++i) {
        if (qi[i] < 0) continue;
        MapPoint *pMP = vpPoints[i];
        MapPoint *pMPinKF = pKF->GetMapPoint(qi[i]);
        if (pMPinKF) {
            if (!pMPinKF->isBad()) vpReplacePoint[i] = pMPinKF;
        } else {
            pMP->AddObservation(pKF, qi[i]);
            pKF->AddMapPoint(pMP, qi[i]);
        }
        nFused++;
    }
    return nFused;
}

}  // namespace ORB_SLAM2
