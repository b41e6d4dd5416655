// Method bodies of the test stand-ins (MapPoint.h, Frame.h), restated from
// the reference: MapPoint.cc:90-104, 198-256, 288-361, 455-488; Frame.cc:
// 239-256, 354-425; KeyFrame.cc (grid copy, IsInImage).  Test scaffolding.
#include <algorithm>
#include <climits>

#include "Frame.h"
#include "KeyFrameDatabase.h"
#include "MapPoint.h"
#include "orbx.h"

namespace ORB_SLAM2 {

bool KFIdLess::operator()(const KeyFrame *a, const KeyFrame *b) const { return a->mnId < b->mnId; }

void FeatureSet::SetScales(int levels, float scale) {
    mnScaleLevels = levels;
    mfScaleFactor = scale;
    mfLogScaleFactor = std::log(scale);
    mvScaleFactors.assign(levels, 1.f);
    mvLevelSigma2.assign(levels, 1.f);
    for (int i = 1; i < levels; ++i) {
        mvScaleFactors[i] = (float)((double)mvScaleFactors[i - 1] * (double)scale);
        mvLevelSigma2[i] = mvScaleFactors[i] * mvScaleFactors[i];
    }
    mvInvScaleFactors.resize(levels);
    mvInvLevelSigma2.resize(levels);
    for (int i = 0; i < levels; ++i) {
        mvInvScaleFactors[i] = 1.0f / mvScaleFactors[i];
        mvInvLevelSigma2[i] = 1.0f / mvLevelSigma2[i];
    }
}

bool FeatureSet::PosInGrid(const cv::KeyPoint &kp, int &posX, int &posY) const {
    posX = (int)std::round((kp.pt.x - mnMinX) * mfGridElementWidthInv);
    posY = (int)std::round((kp.pt.y - mnMinY) * mfGridElementHeightInv);
    return !(posX < 0 || posX >= FRAME_GRID_COLS || posY < 0 || posY >= FRAME_GRID_ROWS);
}

void FeatureSet::AssignFeaturesToGrid() {
    mfGridElementWidthInv = (float)FRAME_GRID_COLS / (mnMaxX - mnMinX);
    mfGridElementHeightInv = (float)FRAME_GRID_ROWS / (mnMaxY - mnMinY);
    for (auto &col : mGrid)
        for (auto &cell : col) cell.clear();
    for (int i = 0; i < N; ++i) {
        int x, y;
        if (PosInGrid(mvKeysUn[i], x, y)) mGrid[x][y].push_back(i);
    }
}

std::vector<size_t> FeatureSet::GetFeaturesInArea(const float &x, const float &y, const float &r, const int minLevel,
                                                  const int maxLevel) const {
    std::vector<size_t> out;
    const int x0 = std::max(0, (int)std::floor((x - mnMinX - r) * mfGridElementWidthInv));
    if (x0 >= FRAME_GRID_COLS) return out;
    const int x1 = std::min(FRAME_GRID_COLS - 1, (int)std::ceil((x - mnMinX + r) * mfGridElementWidthInv));
    if (x1 < 0) return out;
    const int y0 = std::max(0, (int)std::floor((y - mnMinY - r) * mfGridElementHeightInv));
    if (y0 >= FRAME_GRID_ROWS) return out;
    const int y1 = std::min(FRAME_GRID_ROWS - 1, (int)std::ceil((y - mnMinY + r) * mfGridElementHeightInv));
    if (y1 < 0) return out;
    const bool levels = minLevel > 0 || maxLevel >= 0;
    for (int ix = x0; ix <= x1; ++ix)
        for (int iy = y0; iy <= y1; ++iy)
            for (size_t j : mGrid[ix][iy]) {
                const cv::KeyPoint &k = mvKeysUn[j];
                if (levels && (k.octave < minLevel || (maxLevel >= 0 && k.octave > maxLevel))) continue;
                if (std::fabs(k.pt.x - x) < r && std::fabs(k.pt.y - y) < r) out.push_back(j);
            }
    return out;
}

void Frame::SetPose(const cv::Mat &Tcw) {
    mTcw = Tcw.clone();
    mRcw = mTcw.rowRange(0, 3).colRange(0, 3).clone();
    mtcw = mTcw.rowRange(0, 3).col(3).clone();
    mOw = -mRcw.t() * mtcw;
}

void KeyFrame::SetPose(const cv::Mat &Tcw_) {
    Tcw = Tcw_.clone();
    cv::Mat R = Tcw.rowRange(0, 3).colRange(0, 3).clone(), t = Tcw.rowRange(0, 3).col(3).clone();
    Ow = -R.t() * t;
}

int MapPoint::PredictScale(const float &currentDist, KeyFrame *pKF) {
    int s = (int)std::ceil(std::log(mfMaxDistance / currentDist) / pKF->mfLogScaleFactor);
    return s < 0 ? 0 : (s >= pKF->mnScaleLevels ? pKF->mnScaleLevels - 1 : s);
}

int MapPoint::PredictScale(const float &currentDist, Frame *pF) {
    int s = (int)std::ceil(std::log(mfMaxDistance / currentDist) / pF->mfLogScaleFactor);
    return s < 0 ? 0 : (s >= pF->mnScaleLevels ? pF->mnScaleLevels - 1 : s);
}

void MapPoint::AddObservation(KeyFrame *pKF, size_t idx) {
    if (mObservations.count(pKF)) return;
    mObservations[pKF] = idx;
    nObs += (pKF->mvuRight[idx] >= 0) ? 2 : 1;
}

void MapPoint::EraseObservation(KeyFrame *pKF) {
    auto it = mObservations.find(pKF);
    if (it == mObservations.end()) return;
    nObs -= (pKF->mvuRight[it->second] >= 0) ? 2 : 1;
    mObservations.erase(it);
    if (mpRefKF == pKF && !mObservations.empty()) mpRefKF = mObservations.begin()->first;
    if (nObs <= 2) SetBadFlag();
}

void MapPoint::SetBadFlag() {
    mbBad = true;
    ObsMap obs;
    obs.swap(mObservations);
    for (auto &o : obs) o.first->EraseMapPointMatch(o.second);
}

void MapPoint::UpdateNormalAndDepth() {
    if (mbBad || mObservations.empty() || !mpRefKF) return;
    cv::Mat normal = cv::Mat::zeros(3, 1, CV_32F);
    int n = 0;
    for (auto &o : mObservations) {
        cv::Mat d = mWorldPos - o.first->GetCameraCenter();
        normal = normal + d / (float)cv::norm(d);
        n++;
    }
    const float dist = cv::norm(mWorldPos - mpRefKF->GetCameraCenter());
    auto it = mObservations.find(mpRefKF);
    const int level = it == mObservations.end() ? 0 : mpRefKF->mvKeysUn[it->second].octave;
    mfMaxDistance = dist * mpRefKF->mvScaleFactors[level];
    mfMinDistance = mfMaxDistance / mpRefKF->mvScaleFactors[mpRefKF->mnScaleLevels - 1];
    mNormalVector = normal / (float)n;
}

void MapPoint::Replace(MapPoint *pMP) {
    if (pMP->mnId == mnId) return;
    ObsMap obs = mObservations;
    mObservations.clear();
    mbBad = true;
    const int nvis = mnVisible, nfound = mnFound;
    mpReplaced = pMP;
    for (auto &o : obs) {
        KeyFrame *pKF = o.first;
        if (!pMP->IsInKeyFrame(pKF)) {
            pKF->ReplaceMapPointMatch(o.second, pMP);
            pMP->AddObservation(pKF, o.second);
        } else {
            pKF->EraseMapPointMatch(o.second);
        }
    }
    pMP->IncreaseFound(nfound);
    pMP->IncreaseVisible(nvis);
    pMP->ComputeDistinctiveDescriptors();
}

void MapPoint::ComputeDistinctiveDescriptors() {
    if (mbBad || mObservations.empty()) return;
    std::vector<const uint8_t *> d;
    for (auto &o : mObservations)
        if (!o.first->isBad()) d.push_back(o.first->mDescriptors.ptr<uint8_t>((int)o.second));
    if (d.empty()) return;
    const size_t n = d.size();
    int best = INT_MAX;
    size_t bi = 0;
    for (size_t i = 0; i < n; ++i) {
        std::vector<int> row(n);
        for (size_t j = 0; j < n; ++j) row[j] = i == j ? 0 : orbx_descriptor_distance(d[i], d[j]);
        std::sort(row.begin(), row.end());
        const int med = row[(size_t)(0.5 * (n - 1))];
        if (med < best) { best = med; bi = i; }
    }
    mDescriptor = cv::Mat(1, 32, CV_8U);
    std::memcpy(mDescriptor.data, d[bi], 32);
}

// KeyFrame.cc:823-893 (the fields the database queries read, in the fork's
// order: mnId, mBowVec, then mpKeyFrameDB at :877) and Map.cc's keyframe set
template <class Archive>
void KeyFrame::serialize(Archive &ar, const unsigned int) {
    ar & mnId;
    ar & mbBad;
    ar & mBowVec;
    ar & mvpOrderedConnectedKeyFrames;
    ar & mpKeyFrameDB;
}
template void KeyFrame::serialize(boost::archive::binary_iarchive &, const unsigned int);
template void KeyFrame::serialize(boost::archive::binary_oarchive &, const unsigned int);

template <class Archive>
void Map::serialize(Archive &ar, const unsigned int) {
    ar & keyframes;
}
template void Map::serialize(boost::archive::binary_iarchive &, const unsigned int);
template void Map::serialize(boost::archive::binary_oarchive &, const unsigned int);

}  // namespace ORB_SLAM2
