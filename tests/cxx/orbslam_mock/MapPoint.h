// Test stand-in for ORB_SLAM2::MapPoint (orb_slam2/include/MapPoint.h): the
// members and methods the ORBmatcher / Optimizer / KeyFrameDatabase forwarders
// (integration/) and the test's restated reference read, over the cv mock.
// Test scaffolding only: a real build uses the reference's own headers.
#pragma once
#include <map>
#include <vector>

#include <opencv2/core/core.hpp>

namespace ORB_SLAM2 {

class KeyFrame;
class Frame;
class Map;

// Observations ordered by keyframe id: the reference's std::map<KeyFrame*,
// size_t> is ordered by heap address; the test runs two copies of a world
// (forwarder / restated reference) that must iterate alike.
struct KFIdLess {
    bool operator()(const KeyFrame *a, const KeyFrame *b) const;
};
typedef std::map<KeyFrame *, size_t, KFIdLess> ObsMap;

class MapPoint {
public:
    long unsigned int mnId = 0;
    // tracking (set by Frame::isInFrustum before SearchByProjection, MapPoint.h:100-106)
    float mTrackProjX = 0, mTrackProjY = 0, mTrackProjXR = 0;
    bool mbTrackInView = false;
    int mnTrackScaleLevel = 0;
    float mTrackViewCos = 1.f;

    cv::Mat mWorldPos, mNormalVector, mDescriptor;   // 3x1, 3x1 float; 1x32 u8
    float mfMinDistance = 0, mfMaxDistance = 0;
    bool mbBad = false;
    MapPoint *mpReplaced = nullptr;
    ObsMap mObservations;
    int nObs = 0;
    int mnVisible = 1, mnFound = 1;
    long unsigned int mnBALocalForKF = 0;
    KeyFrame *mpRefKF = nullptr;

    cv::Mat GetWorldPos() const { return mWorldPos.clone(); }
    cv::Mat GetNormal() const { return mNormalVector.clone(); }
    cv::Mat GetDescriptor() const { return mDescriptor.clone(); }
    bool isBad() const { return mbBad; }
    int Observations() const { return nObs; }
    ObsMap GetObservations() const { return mObservations; }
    bool IsInKeyFrame(KeyFrame *pKF) const { return mObservations.count(pKF) > 0; }
    int GetIndexInKeyFrame(KeyFrame *pKF) const {
        auto it = mObservations.find(pKF);
        return it == mObservations.end() ? -1 : (int)it->second;
    }
    float GetMinDistanceInvariance() const { return 0.8f * mfMinDistance; }
    float GetMaxDistanceInvariance() const { return 1.2f * mfMaxDistance; }
    int PredictScale(const float &currentDist, KeyFrame *pKF);   // MapPoint.cc:455-471
    int PredictScale(const float &currentDist, Frame *pF);       // MapPoint.cc:473-488
    void AddObservation(KeyFrame *pKF, size_t idx);              // MapPoint.cc:90-104 (monocular count)
    void EraseObservation(KeyFrame *pKF);
    void Replace(MapPoint *pMP);                                 // MapPoint.cc:198-256
    void ComputeDistinctiveDescriptors();                        // MapPoint.cc:288-361
    void SetWorldPos(const cv::Mat &Pos) { mWorldPos = Pos.clone(); }
    void UpdateNormalAndDepth();                                 // MapPoint.cc:363-400
    void SetBadFlag();                                           // MapPoint.cc:149-172
    void IncreaseFound(int n = 1) { mnFound += n; }
    void IncreaseVisible(int n = 1) { mnVisible += n; }
};

}  // namespace ORB_SLAM2
