// Test stand-in for ORB_SLAM2::Frame / KeyFrame (orb_slam2/include/Frame.h,
// KeyFrame.h): the members the forwarders (integration/) and the test's
// restated reference read.  The grid and GetFeaturesInArea follow
// Frame.cc:239-256, 354-425 (a KeyFrame copies its frame's grid).
// Test scaffolding only: a real build uses the reference's own headers.
#pragma once
#include <cmath>
#include <map>
#include <mutex>
#include <set>
#include <vector>

#include <opencv2/core/core.hpp>

#include "BoostArchiver.h"
#include "MapPoint.h"
#include "orbx_orbslam2.hpp"
#include "Thirdparty/DBoW2/DBoW2/BowVector.h"
#include "Thirdparty/DBoW2/DBoW2/FeatureVector.h"

#define FRAME_GRID_ROWS 48
#define FRAME_GRID_COLS 64

namespace ORB_SLAM2 {

class KeyFrameDatabase;

// The members Frame and KeyFrame share (calibration, features, scale tables, grid).
struct FeatureSet {
    int N = 0;
    std::vector<cv::KeyPoint> mvKeys, mvKeysUn;
    std::vector<float> mvuRight, mvDepth;
    cv::Mat mDescriptors;   // N x 32 u8
    DBoW2::BowVector mBowVec;
    DBoW2::FeatureVector mFeatVec;
    float fx = 0, fy = 0, cx = 0, cy = 0, invfx = 0, invfy = 0, mbf = 0, mb = 0;
    int mnScaleLevels = 8;
    float mfScaleFactor = 1.2f, mfLogScaleFactor = 0;
    std::vector<float> mvScaleFactors, mvInvScaleFactors, mvLevelSigma2, mvInvLevelSigma2;
    float mnMinX = 0, mnMaxX = 0, mnMinY = 0, mnMaxY = 0;
    float mfGridElementWidthInv = 0, mfGridElementHeightInv = 0;
    std::vector<size_t> mGrid[FRAME_GRID_COLS][FRAME_GRID_ROWS];

    void SetScales(int levels, float scale);
    void AssignFeaturesToGrid();
    bool PosInGrid(const cv::KeyPoint &kp, int &posX, int &posY) const;
    std::vector<size_t> GetFeaturesInArea(const float &x, const float &y, const float &r, const int minLevel = -1,
                                          const int maxLevel = -1) const;
    bool IsInImage(const float &x, const float &y) const { return x >= mnMinX && x < mnMaxX && y >= mnMinY && y < mnMaxY; }
};

class Frame : public FeatureSet {
public:
    long unsigned int mnId = 0;
    std::vector<MapPoint *> mvpMapPoints;
    std::vector<bool> mvbOutlier;
    cv::Mat mTcw, mRcw, mtcw, mOw;   // 4x4, 3x3, 3x1, 3x1
    ORBextractor *mpORBextractorLeft = nullptr, *mpORBextractorRight = nullptr;
    std::vector<cv::KeyPoint> mvKeysRight;
    cv::Mat mDescriptorsRight, mK, mDistCoef;   // mK 3x3, mDistCoef 4x1 or 5x1 (CV_32F)
    void SetPose(const cv::Mat &Tcw);
    void ComputeStereoMatches();                          // integration/Frame_orbx.cc
    void ComputeStereoFromRGBD(const cv::Mat &imDepth);
    void UndistortKeyPoints();
};

class KeyFrame : public FeatureSet {
public:
    long unsigned int mnId = 0;
    long unsigned int mnBALocalForKF = 0, mnBAFixedForKF = 0;
    bool mbBad = false;
    std::vector<MapPoint *> mvpMapPoints;
    cv::Mat Tcw, Ow;
    std::vector<KeyFrame *> mvpOrderedConnectedKeyFrames;

    bool isBad() const { return mbBad; }
    cv::Mat GetPose() const { return Tcw.clone(); }
    cv::Mat GetRotation() const { return Tcw.rowRange(0, 3).colRange(0, 3).clone(); }
    cv::Mat GetTranslation() const { return Tcw.rowRange(0, 3).col(3).clone(); }
    cv::Mat GetCameraCenter() const { return Ow.clone(); }
    void SetPose(const cv::Mat &Tcw_);
    MapPoint *GetMapPoint(const size_t &idx) const { return mvpMapPoints[idx]; }
    std::vector<MapPoint *> GetMapPointMatches() const { return mvpMapPoints; }
    std::set<MapPoint *> GetMapPoints() const {
        std::set<MapPoint *> s;
        for (MapPoint *p : mvpMapPoints)
            if (p && !p->isBad()) s.insert(p);
        return s;
    }
    void AddMapPoint(MapPoint *pMP, const size_t &idx) { mvpMapPoints[idx] = pMP; }
    void EraseMapPointMatch(const size_t &idx) { mvpMapPoints[idx] = nullptr; }
    void EraseMapPointMatch(MapPoint *pMP) {
        const int idx = pMP->GetIndexInKeyFrame(this);
        if (idx >= 0) mvpMapPoints[idx] = nullptr;
    }
    void ReplaceMapPointMatch(const size_t &idx, MapPoint *pMP) { mvpMapPoints[idx] = pMP; }
    std::vector<KeyFrame *> GetVectorCovisibleKeyFrames() const { return mvpOrderedConnectedKeyFrames; }
    std::vector<KeyFrame *> GetBestCovisibilityKeyFrames(const int &N) const {
        return std::vector<KeyFrame *>(mvpOrderedConnectedKeyFrames.begin(),
                                       mvpOrderedConnectedKeyFrames.begin() +
                                           std::min<size_t>(N, mvpOrderedConnectedKeyFrames.size()));
    }
    std::set<KeyFrame *> GetConnectedKeyFrames() const {
        return std::set<KeyFrame *>(mvpOrderedConnectedKeyFrames.begin(), mvpOrderedConnectedKeyFrames.end());
    }

    // map serialisation (KeyFrame.cc:823-893): the members the keyframe
    // database's queries read, and the database pointer as the fork archives
    // it (`ar & mpKeyFrameDB`, KeyFrame.cc:877, after mBowVec)
    KeyFrameDatabase *mpKeyFrameDB = nullptr;
    template <class Archive> void serialize(Archive &ar, const unsigned int version);
};

class Map {
public:
    std::vector<KeyFrame *> keyframes;
    std::mutex mMutexMapUpdate;
    template <class Archive> void serialize(Archive &ar, const unsigned int version);   // (Map.cc: the keyframes)
    KeyFrame *KeyFrameById(unsigned long id) const {
        for (KeyFrame *k : keyframes)
            if (k->mnId == id) return k;
        return nullptr;
    }
};

}  // namespace ORB_SLAM2
