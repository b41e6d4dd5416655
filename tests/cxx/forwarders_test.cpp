// forwarders_test.cpp -- runs the reference-side forwarders of integration/
// (the 11 ORBmatcher searches, Optimizer::LocalBundleAdjustment, the
// KeyFrameDatabase methods) on the GPU, each on one copy of a synthetic map,
// and checks it against the CPU on a second, identical copy:
//   - ORBmatcher: a restatement of the reference method (ORBmatcher.cc, cited
//     per function) over the same test stand-ins, walking the Frame grid;
//   - LocalBundleAdjustment: the reference's collection / tail restated, with
//     the CPU oracle's solver (orbo_local_ba) in place of g2o;
//   - KeyFrameDatabase: the CPU oracle's literal database (orbo_kfdb_*).
// After each case the whole map (every keyframe slot, observation, flag,
// descriptor, position and pose) of the two copies must be identical, and so
// must the method's outputs.
//   forwarders_test            run every case; one line per case; exit 1 on a mismatch
// Test scaffolding; built by tests/cxx_build.py::build_forwarders_test.
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <functional>
#include <list>
#include <memory>
#include <set>
#include <sstream>
#include <string>
#include <vector>

#include "KeyFrameDatabase.h"
#include "ORBmatcher.h"
#include "Optimizer.h"
#include "orbx_forwarders.h"
#include "orbx_oracle.h"

using namespace ORB_SLAM2;

// ---------------------------------------------------------------- the map
namespace {

struct Rng {   // xorshift64: the same stream on every platform
    uint64_t s;
    explicit Rng(uint64_t seed) : s(seed * 0x9E3779B97F4A7C15ull + 0x2545F4914F6CDD1Dull) {}
    uint32_t next() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return (uint32_t)(s >> 32); }
    float uni(float a, float b) { return a + (b - a) * (float)(next() >> 8) * (1.0f / 16777216.0f); }
    bool p(float q) { return uni(0.f, 1.f) < q; }
    int below(int n) { return (int)(next() % (uint32_t)n); }
};

constexpr float kFx = 458.f, kCx = 320.f, kCy = 240.f, kBf = 50.38f, kW = 640.f, kH = 480.f;
constexpr int kPoints = 700, kKFs = 6;

cv::Mat pose(float yaw, float pitch, float x, float y, float z) {
    const float cy = std::cos(yaw), sy = std::sin(yaw), cp = std::cos(pitch), sp = std::sin(pitch);
    const float R[9] = {cy, sy * sp, sy * cp, 0.f, cp, -sp, -sy, cy * sp, cy * cp};   // Ry(yaw) Rx(pitch)
    cv::Mat T = cv::Mat::eye(4, 4, CV_32F);
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) T.at<float>(r, c) = R[3 * r + c];
        T.at<float>(r, 3) = -(R[3 * r] * x + R[3 * r + 1] * y + R[3 * r + 2] * z);
    }
    return T;
}

struct World {
    std::vector<std::unique_ptr<MapPoint>> mps;
    std::vector<std::unique_ptr<KeyFrame>> kfs;
    std::unique_ptr<Frame> cur, last;
    std::vector<cv::Mat> truth;   // each point's generating descriptor
    std::vector<cv::Mat> alt;     // duplicated points: the descriptor family keyframes 3-5 see
    std::vector<float> angle;     // each point's base keypoint angle
    Map map;
};

void flip(cv::Mat &d, Rng &g, int n) {
    for (int i = 0; i < n; ++i) {
        const int b = g.below(256);
        d.data[b >> 3] ^= (uint8_t)(1u << (b & 7));
    }
}

// Keypoints of `f` (pose T): the visible points with noise plus distractors,
// ordered by level as the extractor returns them.  Returns each keypoint's
// point (-1: distractor).
template <class FS>
std::vector<int> observe(World &w, FS &f, const cv::Mat &T, Rng &g, bool alt_view = false) {
    f.fx = f.fy = kFx; f.cx = kCx; f.cy = kCy; f.invfx = f.invfy = 1.f / kFx;
    f.mbf = kBf; f.mb = kBf / kFx;
    f.SetScales(8, 1.2f);
    f.mnMinX = 0.f; f.mnMaxX = kW; f.mnMinY = 0.f; f.mnMaxY = kH;
    const cv::Mat R = T.rowRange(0, 3).colRange(0, 3), t = T.rowRange(0, 3).col(3);
    const cv::Mat C = -R.t() * t;
    struct Cand { cv::KeyPoint kp; cv::Mat d; int p; float ur; };
    std::vector<Cand> c;
    for (int p = 0; p < (int)w.mps.size(); ++p) {
        MapPoint *mp = w.mps[p].get();
        if (p >= (int)w.truth.size() || !g.p(0.9f)) continue;
        const cv::Mat Xc = R * mp->GetWorldPos() + t;
        const float z = Xc.at<float>(2);
        if (z < 0.5f) continue;
        const float u = kFx * Xc.at<float>(0) / z + kCx, v = kFx * Xc.at<float>(1) / z + kCy;
        if (u < 8 || u > kW - 8 || v < 8 || v > kH - 8) continue;
        const float dist = cv::norm(mp->GetWorldPos() - C);
        int lvl = mp->PredictScale(dist, &f);
        if (g.p(0.15f)) lvl = std::min(lvl + 1, 7);
        const float s = f.mvScaleFactors[lvl];
        cv::KeyPoint kp(cv::Point2f(u + g.uni(-1.f, 1.f) * s, v + g.uni(-1.f, 1.f) * s), 31.f * s,
                        std::fmod(w.angle[p] + 3.f * (float)f.mnScaleLevels + g.uni(-4.f, 4.f) + 360.f, 360.f),
                        g.uni(0.f, 1.f), lvl);
        cv::Mat d = (alt_view && !w.alt[p].empty() ? w.alt[p] : w.truth[p]).clone();
        flip(d, g, g.p(0.1f) ? 20 + g.below(20) : g.below(7));
        // duplicated points: stereo in the views of their own family, mono in the other
        const bool dp = !w.alt[p].empty(), stereo = dp ? !alt_view : g.p(0.5f);
        const float ur = stereo ? kp.pt.x - kBf / z + g.uni(-0.3f, 0.3f) : -1.f;
        c.push_back({kp, d, p, ur >= 0 ? ur : -1.f});
    }
    for (int i = 0; i < 120; ++i) {
        const int lvl = g.below(8);
        cv::KeyPoint kp(cv::Point2f(g.uni(2.f, kW - 2), g.uni(2.f, kH - 2)), 31.f * f.mvScaleFactors[lvl],
                        g.uni(0.f, 359.9f), g.uni(0.f, 1.f), lvl);
        cv::Mat d(1, 32, CV_8U);
        if (g.p(0.3f)) {
            d = w.truth[g.below((int)w.truth.size())].clone();
            flip(d, g, 8 + g.below(12));
        } else {
            for (int b = 0; b < 32; ++b) d.data[b] = (uint8_t)g.next();
        }
        const float ur = g.p(0.3f) ? kp.pt.x - g.uni(2.f, 15.f) : -1.f;
        c.push_back({kp, d, -1, ur >= 0 ? ur : -1.f});
    }
    std::stable_sort(c.begin(), c.end(), [](const Cand &a, const Cand &b) { return a.kp.octave < b.kp.octave; });
    f.N = (int)c.size();
    f.mvKeys.clear(); f.mvuRight.clear(); f.mvDepth.clear();
    f.mDescriptors = cv::Mat(f.N, 32, CV_8U);
    std::vector<int> pt;
    std::map<unsigned, double> bow;
    for (int i = 0; i < f.N; ++i) {
        f.mvKeys.push_back(c[i].kp);
        std::memcpy(f.mDescriptors.template ptr<uint8_t>(i), c[i].d.data, 32);
        f.mvuRight.push_back(c[i].ur);
        f.mvDepth.push_back(c[i].ur >= 0 ? kBf / (c[i].kp.pt.x - c[i].ur) : -1.f);
        pt.push_back(c[i].p);
        const unsigned h = c[i].p >= 0 ? (unsigned)c[i].p * 2654435761u : g.next();
        const unsigned node = g.p(0.1f) ? (unsigned)g.below(64) : (h >> 8) % 64;
        f.mFeatVec[node].push_back((unsigned)i);
        bow[c[i].p >= 0 && !g.p(0.1f) ? (unsigned)c[i].p % 409 : (unsigned)g.below(409)] += 1.0;
    }
    for (auto &kv : bow) f.mBowVec[kv.first] = kv.second / f.N;
    f.mvKeysUn = f.mvKeys;
    f.AssignFeaturesToGrid();
    return pt;
}

// The map: kPoints points, kKFs keyframes along a short arc, the current and
// last frames.  Keyframes 3 and 4 see some points through duplicates (for
// Fuse's Replace); a few points are bad, a few have no observations.
std::unique_ptr<World> make_world(uint64_t seed, float cur_dz = 0.f) {
    auto w = std::make_unique<World>();
    Rng g(seed);
    for (int p = 0; p < kPoints; ++p) {
        auto mp = std::make_unique<MapPoint>();
        mp->mnId = p;
        mp->mWorldPos = cv::Mat(3, 1, CV_32F);
        mp->mWorldPos.at<float>(0) = g.uni(-7.f, 7.f);
        mp->mWorldPos.at<float>(1) = g.uni(-5.f, 5.f);
        mp->mWorldPos.at<float>(2) = g.uni(4.f, 14.f);
        const float d0 = cv::norm(mp->mWorldPos);
        mp->mfMaxDistance = 0.95f * d0 * std::pow(1.2f, (float)g.below(3));
        mp->mfMinDistance = mp->mfMaxDistance / std::pow(1.2f, 7.f);
        mp->mNormalVector = mp->mWorldPos / d0;
        cv::Mat d(1, 32, CV_8U);
        for (int b = 0; b < 32; ++b) d.data[b] = (uint8_t)g.next();
        w->truth.push_back(d);
        mp->mDescriptor = d.clone();
        w->angle.push_back(g.uni(0.f, 360.f));
        w->mps.push_back(std::move(mp));
    }
    // duplicates: keyframes 2-4 see some points through a second MapPoint,
    // and keyframes 2-5 see those points with a descriptor ~48 bits away
    // (mono there, stereo in keyframes 0-1).  Fusing a point into keyframe 3
    // then makes the duplicate Replace into it (fewer observations), its
    // descriptor moves to the other family, and keyframe 5's search -- where
    // the point has no slot -- gives another answer with the new descriptor
    // (LocalMapping's batched Fuse must search that row again)
    std::vector<int> dup(kPoints, -1);   // point -> its duplicate
    w->alt.resize(kPoints);
    for (int p = 0; p < kPoints; ++p)
        if (g.p(0.08f)) {
            w->alt[p] = w->truth[p].clone();
            flip(w->alt[p], g, 52);
            auto q = std::make_unique<MapPoint>(*w->mps[p]);
            q->mnId = (long unsigned)w->mps.size();
            q->mDescriptor = w->alt[p].clone();
            flip(q->mDescriptor, g, 3);
            dup[p] = (int)w->mps.size();
            w->mps.push_back(std::move(q));
        }
    for (int k = 0; k < kKFs; ++k) {
        auto kf = std::make_unique<KeyFrame>();
        kf->mnId = (long unsigned)k + 1;
        kf->SetPose(pose(0.03f * k, 0.01f * k, 0.25f * k - 0.6f, 0.05f * std::sin((float)k), 0.1f * k));
        const std::vector<int> pt = observe(*w, *kf, kf->Tcw, g, k >= 2);
        kf->mvpMapPoints.assign(kf->N, nullptr);
        for (int i = 0; i < kf->N; ++i) {
            if (pt[i] < 0 || !g.p(0.85f) || (k == 5 && dup[pt[i]] >= 0)) continue;
            MapPoint *mp = w->mps[k >= 2 && k <= 4 && dup[pt[i]] >= 0 ? dup[pt[i]] : pt[i]].get();
            kf->mvpMapPoints[i] = mp;
            mp->AddObservation(kf.get(), i);
            if (!mp->mpRefKF) mp->mpRefKF = kf.get();
        }
        w->map.keyframes.push_back(kf.get());
        w->kfs.push_back(std::move(kf));
    }
    for (auto &a : w->kfs) {   // covisibility: shared points, then id
        std::vector<std::pair<int, KeyFrame *>> v;
        for (auto &b : w->kfs) {
            if (a == b) continue;
            int n = 0;
            for (MapPoint *mp : a->mvpMapPoints)
                if (mp && mp->IsInKeyFrame(b.get())) ++n;
            if (n > 0) v.push_back({n, b.get()});
        }
        std::stable_sort(v.begin(), v.end(), [](auto &x, auto &y) { return x.first > y.first; });
        for (auto &x : v) a->mvpOrderedConnectedKeyFrames.push_back(x.second);
    }
    for (auto &mp : w->mps) {
        mp->ComputeDistinctiveDescriptors();
        if (g.p(0.03f)) mp->mbBad = true;
    }
    for (int i = 0; i < 10; ++i) {   // points with no observations (fresh tracking points)
        auto mp = std::make_unique<MapPoint>(*w->mps[g.below(kPoints)]);
        mp->mnId = (long unsigned)w->mps.size();
        mp->mObservations.clear();
        mp->nObs = 0;
        mp->mbBad = false;
        mp->mpRefKF = nullptr;
        w->mps.push_back(std::move(mp));
    }
    w->last = std::make_unique<Frame>();
    w->last->mnId = 99;
    w->last->SetPose(pose(0.04f, 0.012f, 0.2f, 0.1f, 0.2f));
    const std::vector<int> lpt = observe(*w, *w->last, w->last->mTcw, g);
    w->last->mvpMapPoints.assign(w->last->N, nullptr);
    w->last->mvbOutlier.assign(w->last->N, false);
    for (int i = 0; i < w->last->N; ++i)
        if (lpt[i] >= 0 && g.p(0.9f)) {
            w->last->mvpMapPoints[i] = w->mps[lpt[i]].get();
            w->last->mvbOutlier[i] = g.p(0.1f);
        }
    w->cur = std::make_unique<Frame>();
    w->cur->mnId = 100;
    w->cur->SetPose(pose(0.05f, 0.015f, 0.27f, 0.12f, 0.25f + cur_dz));
    observe(*w, *w->cur, w->cur->mTcw, g);
    w->cur->mvpMapPoints.assign(w->cur->N, nullptr);
    w->cur->mvbOutlier.assign(w->cur->N, false);
    for (int i = 0; i < w->cur->N; ++i)
        if (g.p(0.05f)) w->cur->mvpMapPoints[i] = w->mps[g.below((int)w->mps.size())].get();
    return w;
}

// Everything the searches, BA and the database can change, as one vector.
std::vector<int64_t> snapshot(const World &w) {
    std::vector<int64_t> s;
    auto id = [](const MapPoint *p) { return p ? (int64_t)p->mnId : -1; };
    auto bits = [&s](const cv::Mat &m) {
        for (int r = 0; r < m.rows; ++r)
            for (int c = 0; c < m.cols; ++c) {
                float v = m.at<float>(r, c);
                int32_t b;
                std::memcpy(&b, &v, 4);
                s.push_back(b);
            }
    };
    for (const auto &kf : w.kfs) {
        s.push_back((int64_t)kf->mnId);
        s.push_back(kf->mbBad);
        for (MapPoint *p : kf->mvpMapPoints) s.push_back(id(p));
        bits(kf->Tcw);
    }
    for (const Frame *f : {w.cur.get(), w.last.get()})
        for (MapPoint *p : f->mvpMapPoints) s.push_back(id(p));
    for (const auto &mp : w.mps) {
        s.push_back((int64_t)mp->mnId);
        s.push_back(mp->mbBad);
        s.push_back(id(mp->mpReplaced));
        s.push_back(mp->nObs);
        s.push_back(mp->mnFound);
        s.push_back(mp->mnVisible);
        for (auto &o : mp->mObservations) {
            s.push_back((int64_t)o.first->mnId);
            s.push_back((int64_t)o.second);
        }
        for (int b = 0; b < 32; ++b) s.push_back(mp->mDescriptor.data[b]);
        bits(mp->mWorldPos);
        bits(mp->mNormalVector);
        float md[2] = {mp->mfMinDistance, mp->mfMaxDistance};
        int32_t mb[2];
        std::memcpy(mb, md, 8);
        s.push_back(mb[0]);
        s.push_back(mb[1]);
    }
    return s;
}

// ------------------------------------------------- the reference, restated
// ORBmatcher.cc restated over the stand-ins: the grid walk of
// Frame::GetFeaturesInArea, the best / second-best bookkeeping, the rotation
// histogram.  Written for the check, in the reference's loop order.
namespace ref {

constexpr int TH_HIGH = 100, TH_LOW = 50, HISTO = 30;

int dist(const cv::Mat &a, const cv::Mat &b) { return orbo_descriptor_distance(a.ptr<uint8_t>(), b.ptr<uint8_t>()); }

// the rotation histogram and ComputeThreeMaxima (:1603-1644)
struct RotHist {
    std::vector<int> h[HISTO];
    void add(float a1, float a2, int v) {
        float rot = a1 - a2;
        if (rot < 0.0) rot += 360.0f;
        int bin = (int)std::round(rot * (1.0f / HISTO));
        if (bin == HISTO) bin = 0;
        h[bin].push_back(v);
    }
    // calls drop(v) for every entry outside the three largest bins
    void filter(const std::function<void(int)> &drop) const {
        int m[3] = {0, 0, 0}, ind[3] = {-1, -1, -1};
        for (int i = 0; i < HISTO; ++i) {
            const int s = (int)h[i].size();
            int slot = s > m[0] ? 0 : s > m[1] ? 1 : s > m[2] ? 2 : 3;
            if (slot == 3) continue;
            for (int j = 2; j > slot; --j) { m[j] = m[j - 1]; ind[j] = ind[j - 1]; }
            m[slot] = s;
            ind[slot] = i;
        }
        if (m[1] < 0.1f * (float)m[0]) ind[1] = ind[2] = -1;
        else if (m[2] < 0.1f * (float)m[0]) ind[2] = -1;
        for (int i = 0; i < HISTO; ++i)
            if (i != ind[0] && i != ind[1] && i != ind[2])
                for (int v : h[i]) drop(v);
    }
};

struct Best2 {   // best and second-best distance, with the levels of both
    int d1 = 256, d2 = 256, l1 = -1, l2 = -1, idx = -1;
    void offer(int d, int idx_, int lvl) {
        if (d < d1) { d2 = d1; l2 = l1; d1 = d; l1 = lvl; idx = idx_; }
        else if (d < d2) { d2 = d; l2 = lvl; }
    }
};

// :45-129
int ByProjectionLocal(float nn, Frame &F, const std::vector<MapPoint *> &pts, float th) {
    int n = 0;
    for (MapPoint *mp : pts) {
        if (!mp->mbTrackInView || mp->isBad()) continue;
        const int lvl = mp->mnTrackScaleLevel;
        float r = mp->mTrackViewCos > 0.998 ? 2.5f : 4.0f;
        if (th != 1.0) r *= th;
        const float win = r * F.mvScaleFactors[lvl];
        const cv::Mat d = mp->GetDescriptor();
        Best2 b;
        bool any = false;
        for (size_t i : F.GetFeaturesInArea(mp->mTrackProjX, mp->mTrackProjY, win, lvl - 1, lvl)) {
            any = true;
            if (F.mvpMapPoints[i] && F.mvpMapPoints[i]->Observations() > 0) continue;
            if (F.mvuRight[i] > 0 && std::fabs(mp->mTrackProjXR - F.mvuRight[i]) > win) continue;
            b.offer(dist(d, F.mDescriptors.row((int)i)), (int)i, F.mvKeysUn[i].octave);
        }
        if (!any || b.d1 > TH_HIGH) continue;
        if (b.l1 == b.l2 && b.d1 > nn * b.d2) continue;
        F.mvpMapPoints[b.idx] = mp;
        ++n;
    }
    return n;
}

// :1330-1472
int ByProjectionLast(bool ori, Frame &C, const Frame &L, float th, bool mono) {
    const cv::Mat Rcw = C.mTcw.rowRange(0, 3).colRange(0, 3), tcw = C.mTcw.rowRange(0, 3).col(3);
    const cv::Mat tlc = L.mTcw.rowRange(0, 3).colRange(0, 3) * (-Rcw.t() * tcw) + L.mTcw.rowRange(0, 3).col(3);
    const bool fwd = tlc.at<float>(2) > C.mb && !mono, bwd = -tlc.at<float>(2) > C.mb && !mono;
    RotHist rh;
    int n = 0;
    for (int i = 0; i < L.N; ++i) {
        MapPoint *mp = L.mvpMapPoints[i];
        if (!mp || L.mvbOutlier[i]) continue;
        const cv::Mat x = Rcw * mp->GetWorldPos() + tcw;
        const float iz = 1.0 / x.at<float>(2);
        if (iz < 0) continue;
        const float u = C.fx * x.at<float>(0) * iz + C.cx, v = C.fy * x.at<float>(1) * iz + C.cy;
        if (u < C.mnMinX || u > C.mnMaxX || v < C.mnMinY || v > C.mnMaxY) continue;
        const int o = L.mvKeys[i].octave;
        const float rad = th * C.mvScaleFactors[o];
        const std::vector<size_t> cand = fwd ? C.GetFeaturesInArea(u, v, rad, o)
                                       : bwd ? C.GetFeaturesInArea(u, v, rad, 0, o)
                                             : C.GetFeaturesInArea(u, v, rad, o - 1, o + 1);
        const cv::Mat d = mp->GetDescriptor();
        int bd = 256, bi = -1;
        for (size_t j : cand) {
            if (C.mvpMapPoints[j] && C.mvpMapPoints[j]->Observations() > 0) continue;
            if (C.mvuRight[j] > 0 && std::fabs(u - C.mbf * iz - C.mvuRight[j]) > rad) continue;
            const int dd = dist(d, C.mDescriptors.row((int)j));
            if (dd < bd) { bd = dd; bi = (int)j; }
        }
        if (bd > TH_HIGH) continue;
        C.mvpMapPoints[bi] = mp;
        ++n;
        if (ori) rh.add(L.mvKeysUn[i].angle, C.mvKeysUn[bi].angle, bi);
    }
    if (ori) rh.filter([&](int j) { C.mvpMapPoints[j] = nullptr; --n; });
    return n;
}

// :1474-1601
int ByProjectionKF(bool ori, Frame &C, KeyFrame *K, const std::set<MapPoint *> &found, float th, int orbdist) {
    const cv::Mat Rcw = C.mTcw.rowRange(0, 3).colRange(0, 3), tcw = C.mTcw.rowRange(0, 3).col(3);
    const cv::Mat Ow = -Rcw.t() * tcw;
    const std::vector<MapPoint *> mps = K->GetMapPointMatches();
    RotHist rh;
    int n = 0;
    for (size_t i = 0; i < mps.size(); ++i) {
        MapPoint *mp = mps[i];
        if (!mp || mp->isBad() || found.count(mp)) continue;
        const cv::Mat X = mp->GetWorldPos(), x = Rcw * X + tcw;
        const float iz = 1.0 / x.at<float>(2);
        const float u = C.fx * x.at<float>(0) * iz + C.cx, v = C.fy * x.at<float>(1) * iz + C.cy;
        if (u < C.mnMinX || u > C.mnMaxX || v < C.mnMinY || v > C.mnMaxY) continue;
        const float d3 = cv::norm(X - Ow);
        if (d3 < mp->GetMinDistanceInvariance() || d3 > mp->GetMaxDistanceInvariance()) continue;
        const int lvl = mp->PredictScale(d3, &C);
        const float rad = th * C.mvScaleFactors[lvl];
        const cv::Mat d = mp->GetDescriptor();
        int bd = 256, bi = -1;
        for (size_t j : C.GetFeaturesInArea(u, v, rad, lvl - 1, lvl + 1)) {
            if (C.mvpMapPoints[j]) continue;
            const int dd = dist(d, C.mDescriptors.row((int)j));
            if (dd < bd) { bd = dd; bi = (int)j; }
        }
        if (bd > orbdist) continue;
        C.mvpMapPoints[bi] = mp;
        ++n;
        if (ori) rh.add(K->mvKeysUn[i].angle, C.mvKeysUn[bi].angle, bi);
    }
    if (ori) rh.filter([&](int j) { C.mvpMapPoints[j] = nullptr; --n; });
    return n;
}

// The checks the keyframe projections share (:318-363, :850-894, :1010-1053):
// returns the predicted level, or -1.
int project(MapPoint *mp, const cv::Mat &R, const cv::Mat &t, const cv::Mat &O, KeyFrame *K, float &u, float &v,
            float &iz) {
    const cv::Mat X = mp->GetWorldPos(), x = R * X + t;
    if (x.at<float>(2) < 0.0f) return -1;
    iz = 1 / x.at<float>(2);
    u = K->fx * (x.at<float>(0) * iz) + K->cx;
    v = K->fy * (x.at<float>(1) * iz) + K->cy;
    if (!K->IsInImage(u, v)) return -1;
    const cv::Mat PO = X - O;
    const float d3 = cv::norm(PO);
    if (d3 < mp->GetMinDistanceInvariance() || d3 > mp->GetMaxDistanceInvariance()) return -1;
    if (PO.dot(mp->GetNormal()) < 0.5 * d3) return -1;
    return mp->PredictScale(d3, K);
}

void sim3_split(const cv::Mat &S, cv::Mat &R, cv::Mat &t, cv::Mat &O) {
    const cv::Mat sR = S.rowRange(0, 3).colRange(0, 3);
    const float s = std::sqrt(sR.row(0).dot(sR.row(0)));
    R = sR / s;
    t = S.rowRange(0, 3).col(3) / s;
    O = -R.t() * t;
}

// :291-404
int ByProjectionSim3(KeyFrame *K, const cv::Mat &S, const std::vector<MapPoint *> &pts,
                     std::vector<MapPoint *> &matched, int th) {
    cv::Mat R, t, O;
    sim3_split(S, R, t, O);
    std::set<MapPoint *> found(matched.begin(), matched.end());
    found.erase(nullptr);
    int n = 0;
    for (MapPoint *mp : pts) {
        if (mp->isBad() || found.count(mp)) continue;
        float u, v, iz;
        const int lvl = project(mp, R, t, O, K, u, v, iz);
        if (lvl < 0) continue;
        const cv::Mat d = mp->GetDescriptor();
        int bd = 256, bi = -1;
        for (size_t j : K->GetFeaturesInArea(u, v, th * K->mvScaleFactors[lvl])) {
            if (matched[j]) continue;
            const int o = K->mvKeysUn[j].octave;
            if (o < lvl - 1 || o > lvl) continue;
            const int dd = dist(d, K->mDescriptors.row((int)j));
            if (dd < bd) { bd = dd; bi = (int)j; }
        }
        if (bd > TH_LOW) continue;
        matched[bi] = mp;
        ++n;
    }
    return n;
}

// the FeatureVector walk shared by the BoW searches (:176-265, :547-634, :688-791)
template <class Body>
void bow_walk(const DBoW2::FeatureVector &A, const DBoW2::FeatureVector &B, Body body) {
    auto a = A.begin();
    auto b = B.begin();
    while (a != A.end() && b != B.end()) {
        if (a->first == b->first) { body(a->second, b->second); ++a; ++b; }
        else if (a->first < b->first) a = A.lower_bound(b->first);
        else b = B.lower_bound(a->first);
    }
}

// :160-289
int BoWFrame(float nn, bool ori, KeyFrame *K, Frame &F, std::vector<MapPoint *> &out) {
    const std::vector<MapPoint *> mk = K->GetMapPointMatches();
    out.assign(F.N, nullptr);
    RotHist rh;
    int n = 0;
    bow_walk(K->mFeatVec, F.mFeatVec, [&](const std::vector<unsigned> &ik, const std::vector<unsigned> &jf) {
        for (unsigned i : ik) {
            MapPoint *mp = mk[i];
            if (!mp || mp->isBad()) continue;
            Best2 b;
            for (unsigned j : jf)
                if (!out[j]) b.offer(dist(K->mDescriptors.row((int)i), F.mDescriptors.row((int)j)), (int)j, 0);
            if (b.d1 > TH_LOW || !((float)b.d1 < nn * (float)b.d2)) continue;
            out[b.idx] = mp;
            if (ori) rh.add(K->mvKeysUn[i].angle, F.mvKeys[b.idx].angle, b.idx);
            ++n;
        }
    });
    if (ori) rh.filter([&](int j) { out[j] = nullptr; --n; });
    return n;
}

// :524-657
int BoWKF(float nn, bool ori, KeyFrame *K1, KeyFrame *K2, std::vector<MapPoint *> &m12) {
    const std::vector<MapPoint *> p1 = K1->GetMapPointMatches(), p2 = K2->GetMapPointMatches();
    m12.assign(p1.size(), nullptr);
    std::vector<bool> used2(p2.size(), false);
    RotHist rh;
    int n = 0;
    bow_walk(K1->mFeatVec, K2->mFeatVec, [&](const std::vector<unsigned> &i1, const std::vector<unsigned> &i2) {
        for (unsigned a : i1) {
            if (!p1[a] || p1[a]->isBad()) continue;
            Best2 b;
            for (unsigned c : i2)
                if (!used2[c] && p2[c] && !p2[c]->isBad())
                    b.offer(dist(K1->mDescriptors.row((int)a), K2->mDescriptors.row((int)c)), (int)c, 0);
            if (b.d1 >= TH_LOW || !((float)b.d1 < nn * (float)b.d2)) continue;
            m12[a] = p2[b.idx];
            used2[b.idx] = true;
            if (ori) rh.add(K1->mvKeysUn[a].angle, K2->mvKeysUn[b.idx].angle, (int)a);
            ++n;
        }
    });
    if (ori) rh.filter([&](int a) { m12[a] = nullptr; --n; });
    return n;
}

// :406-521
int Init(float nn, bool ori, Frame &F1, Frame &F2, std::vector<cv::Point2f> &prev, std::vector<int> &m12, int win) {
    m12.assign(F1.mvKeysUn.size(), -1);
    std::vector<int> best21(F2.mvKeysUn.size(), INT_MAX), m21(F2.mvKeysUn.size(), -1);
    RotHist rh;
    int n = 0;
    for (size_t i = 0; i < F1.mvKeysUn.size(); ++i) {
        if (F1.mvKeysUn[i].octave > 0) continue;
        int d1 = INT_MAX, d2 = INT_MAX, bi = -1;
        for (size_t j : F2.GetFeaturesInArea(prev[i].x, prev[i].y, win, 0, 0)) {
            const int d = dist(F1.mDescriptors.row((int)i), F2.mDescriptors.row((int)j));
            if (best21[j] <= d) continue;
            if (d < d1) { d2 = d1; d1 = d; bi = (int)j; }
            else if (d < d2) d2 = d;
        }
        if (d1 > TH_LOW || !(d1 < (float)d2 * nn)) continue;
        if (m21[bi] >= 0) { m12[m21[bi]] = -1; --n; }
        m12[i] = bi;
        m21[bi] = (int)i;
        best21[bi] = d1;
        ++n;
        if (ori) rh.add(F1.mvKeysUn[i].angle, F2.mvKeysUn[bi].angle, (int)i);
    }
    if (ori) rh.filter([&](int i) { if (m12[i] >= 0) { m12[i] = -1; --n; } });
    for (size_t i = 0; i < m12.size(); ++i)
        if (m12[i] >= 0) prev[i] = F2.mvKeysUn[m12[i]].pt;
    return n;
}

// :659-825 (with CheckDistEpipolarLine, :140-157)
int Triangulation(bool ori, KeyFrame *K1, KeyFrame *K2, const cv::Mat &F12,
                  std::vector<std::pair<size_t, size_t>> &pairs, bool only_stereo) {
    const cv::Mat C2 = K2->GetRotation() * K1->GetCameraCenter() + K2->GetTranslation();
    const float iz = 1.0f / C2.at<float>(2);
    const float ex = K2->fx * C2.at<float>(0) * iz + K2->cx, ey = K2->fy * C2.at<float>(1) * iz + K2->cy;
    std::vector<bool> used2(K2->N, false);
    std::vector<int> m12(K1->N, -1);
    RotHist rh;
    int n = 0;
    auto epi_ok = [&](const cv::KeyPoint &k1, const cv::KeyPoint &k2) {
        const float a = k1.pt.x * F12.at<float>(0, 0) + k1.pt.y * F12.at<float>(1, 0) + F12.at<float>(2, 0);
        const float b = k1.pt.x * F12.at<float>(0, 1) + k1.pt.y * F12.at<float>(1, 1) + F12.at<float>(2, 1);
        const float c = k1.pt.x * F12.at<float>(0, 2) + k1.pt.y * F12.at<float>(1, 2) + F12.at<float>(2, 2);
        const float num = a * k2.pt.x + b * k2.pt.y + c, den = a * a + b * b;
        return den != 0 && num * num / den < 3.84 * K2->mvLevelSigma2[k2.octave];
    };
    bow_walk(K1->mFeatVec, K2->mFeatVec, [&](const std::vector<unsigned> &i1, const std::vector<unsigned> &i2) {
        for (unsigned a : i1) {
            if (K1->GetMapPoint(a)) continue;
            const bool st1 = K1->mvuRight[a] >= 0;
            if (only_stereo && !st1) continue;
            const cv::KeyPoint &k1 = K1->mvKeysUn[a];
            int bd = TH_LOW, bi = -1;
            for (unsigned c : i2) {
                if (used2[c] || K2->GetMapPoint(c)) continue;
                const bool st2 = K2->mvuRight[c] >= 0;
                if (only_stereo && !st2) continue;
                const int d = dist(K1->mDescriptors.row((int)a), K2->mDescriptors.row((int)c));
                if (d > TH_LOW || d > bd) continue;
                const cv::KeyPoint &k2 = K2->mvKeysUn[c];
                if (!st1 && !st2) {
                    const float dx = ex - k2.pt.x, dy = ey - k2.pt.y;
                    if (dx * dx + dy * dy < 100 * K2->mvScaleFactors[k2.octave]) continue;
                }
                if (epi_ok(k1, k2)) { bi = (int)c; bd = d; }
            }
            if (bi < 0) continue;
            m12[a] = bi;
            ++n;
            if (ori) rh.add(k1.angle, K2->mvKeysUn[bi].angle, (int)a);
        }
    });
    if (ori) rh.filter([&](int a) { m12[a] = -1; --n; });
    pairs.clear();
    for (size_t i = 0; i < m12.size(); ++i)
        if (m12[i] >= 0) pairs.push_back({i, (size_t)m12[i]});
    return n;
}

// :1104-1328
int Sim3(KeyFrame *K1, KeyFrame *K2, std::vector<MapPoint *> &m12, float s12, const cv::Mat &R12,
         const cv::Mat &t12, float th) {
    const cv::Mat sR12 = s12 * R12, sR21 = (1.0 / s12) * R12.t(), t21 = -sR21 * t12;
    const std::vector<MapPoint *> p1 = K1->GetMapPointMatches(), p2 = K2->GetMapPointMatches();
    std::vector<bool> done1(p1.size(), false), done2(p2.size(), false);
    for (size_t i = 0; i < p1.size(); ++i)
        if (m12[i]) {
            done1[i] = true;
            const int j = m12[i]->GetIndexInKeyFrame(K2);
            if (j >= 0 && j < (int)p2.size()) done2[j] = true;
        }
    // one direction: points of A through (Rw, tw) then (sR, tt) into B
    auto search = [&](const std::vector<MapPoint *> &pa, const std::vector<bool> &done, KeyFrame *A, KeyFrame *B,
                      const cv::Mat &sR, const cv::Mat &tt) {
        std::vector<int> m(pa.size(), -1);
        for (size_t i = 0; i < pa.size(); ++i) {
            MapPoint *mp = pa[i];
            if (!mp || done[i] || mp->isBad()) continue;
            const cv::Mat x = sR * (A->GetRotation() * mp->GetWorldPos() + A->GetTranslation()) + tt;
            if (x.at<float>(2) < 0.0) continue;
            const float iz = 1.0 / x.at<float>(2);
            const float u = K1->fx * (x.at<float>(0) * iz) + K1->cx, v = K1->fy * (x.at<float>(1) * iz) + K1->cy;
            if (!B->IsInImage(u, v)) continue;
            const float d3 = cv::norm(x);
            if (d3 < mp->GetMinDistanceInvariance() || d3 > mp->GetMaxDistanceInvariance()) continue;
            const int lvl = mp->PredictScale(d3, B);
            int bd = INT_MAX, bi = -1;
            for (size_t j : B->GetFeaturesInArea(u, v, th * B->mvScaleFactors[lvl])) {
                const int o = B->mvKeysUn[j].octave;
                if (o < lvl - 1 || o > lvl) continue;
                const int d = dist(mp->GetDescriptor(), B->mDescriptors.row((int)j));
                if (d < bd) { bd = d; bi = (int)j; }
            }
            if (bd <= TH_HIGH) m[i] = bi;
        }
        return m;
    };
    const std::vector<int> a = search(p1, done1, K1, K2, sR21, t21), b = search(p2, done2, K2, K1, sR12, t12);
    int n = 0;
    for (size_t i = 0; i < a.size(); ++i)
        if (a[i] >= 0 && b[a[i]] == (int)i) { m12[i] = p2[a[i]]; ++n; }
    return n;
}

// :827-977
int Fuse(KeyFrame *K, const std::vector<MapPoint *> &pts, float th) {
    const cv::Mat R = K->GetRotation(), t = K->GetTranslation(), O = K->GetCameraCenter();
    int n = 0;
    for (MapPoint *mp : pts) {
        if (!mp || mp->isBad() || mp->IsInKeyFrame(K)) continue;
        float u, v, iz;
        const int lvl = project(mp, R, t, O, K, u, v, iz);
        if (lvl < 0) continue;
        const float ur = u - K->mbf * iz;
        const cv::Mat d = mp->GetDescriptor();
        int bd = 256, bi = -1;
        for (size_t j : K->GetFeaturesInArea(u, v, th * K->mvScaleFactors[lvl])) {
            const cv::KeyPoint &kp = K->mvKeysUn[j];
            if (kp.octave < lvl - 1 || kp.octave > lvl) continue;
            const float dx = u - kp.pt.x, dy = v - kp.pt.y;
            if (K->mvuRight[j] >= 0) {
                const float dr = ur - K->mvuRight[j];
                if ((dx * dx + dy * dy + dr * dr) * K->mvInvLevelSigma2[kp.octave] > 7.8) continue;
            } else if ((dx * dx + dy * dy) * K->mvInvLevelSigma2[kp.octave] > 5.99) {
                continue;
            }
            const int dd = dist(d, K->mDescriptors.row((int)j));
            if (dd < bd) { bd = dd; bi = (int)j; }
        }
        if (bd > TH_LOW) continue;
        if (MapPoint *in = K->GetMapPoint(bi)) {
            if (!in->isBad()) {
                if (in->Observations() > mp->Observations()) mp->Replace(in);
                else in->Replace(mp);
            }
        } else {
            mp->AddObservation(K, bi);
            K->AddMapPoint(mp, bi);
        }
        ++n;
    }
    return n;
}

// :979-1102
int FuseSim3(KeyFrame *K, const cv::Mat &S, const std::vector<MapPoint *> &pts, float th,
             std::vector<MapPoint *> &repl) {
    cv::Mat R, t, O;
    sim3_split(S, R, t, O);
    const std::set<MapPoint *> found = K->GetMapPoints();
    int n = 0;
    for (size_t i = 0; i < pts.size(); ++i) {
        MapPoint *mp = pts[i];
        if (mp->isBad() || found.count(mp)) continue;
        float u, v, iz;
        const int lvl = project(mp, R, t, O, K, u, v, iz);
        if (lvl < 0) continue;
        int bd = INT_MAX, bi = -1;
        for (size_t j : K->GetFeaturesInArea(u, v, th * K->mvScaleFactors[lvl])) {
            const int o = K->mvKeysUn[j].octave;
            if (o < lvl - 1 || o > lvl) continue;
            const int d = dist(mp->GetDescriptor(), K->mDescriptors.row((int)j));
            if (d < bd) { bd = d; bi = (int)j; }
        }
        if (bd > TH_LOW) continue;
        if (MapPoint *in = K->GetMapPoint(bi)) {
            if (!in->isBad()) repl[i] = in;
        } else {
            mp->AddObservation(K, bi);
            K->AddMapPoint(mp, bi);
        }
        ++n;
    }
    return n;
}

// Optimizer.cc:517-890 with the oracle's solver in place of g2o
void LocalBA(KeyFrame *K, Map *map) {
    std::vector<KeyFrame *> local{K}, fixedc;
    K->mnBALocalForKF = K->mnId;
    for (KeyFrame *k : K->GetVectorCovisibleKeyFrames()) {
        k->mnBALocalForKF = K->mnId;
        if (!k->isBad()) local.push_back(k);
    }
    std::vector<MapPoint *> pts;
    for (KeyFrame *k : local)
        for (MapPoint *mp : k->GetMapPointMatches())
            if (mp && !mp->isBad() && mp->mnBALocalForKF != K->mnId) { pts.push_back(mp); mp->mnBALocalForKF = K->mnId; }
    for (MapPoint *mp : pts)
        for (auto &o : mp->GetObservations())
            if (o.first->mnBALocalForKF != K->mnId && o.first->mnBAFixedForKF != K->mnId) {
                o.first->mnBAFixedForKF = K->mnId;
                if (!o.first->isBad()) fixedc.push_back(o.first);
            }
    std::vector<KeyFrame *> cams = local;
    cams.insert(cams.end(), fixedc.begin(), fixedc.end());
    std::vector<float> T(12 * cams.size()), X(3 * pts.size());
    std::vector<uint8_t> fx(cams.size());
    for (size_t c = 0; c < cams.size(); ++c) {
        for (int r = 0; r < 3; ++r)
            for (int q = 0; q < 4; ++q) T[12 * c + 4 * r + q] = cams[c]->Tcw.at<float>(r, q);
        fx[c] = c >= local.size() || cams[c]->mnId == 0;
    }
    std::vector<orbo_ba_edge> E;
    std::vector<std::pair<KeyFrame *, MapPoint *>> own;
    for (size_t p = 0; p < pts.size(); ++p) {
        for (int q = 0; q < 3; ++q) X[3 * p + q] = pts[p]->mWorldPos.at<float>(q);
        for (auto &o : pts[p]->GetObservations()) {
            KeyFrame *k = o.first;
            if (k->isBad()) continue;
            const int c = (int)(std::find(cams.begin(), cams.end(), k) - cams.begin());
            const cv::KeyPoint &kp = k->mvKeysUn[o.second];
            E.push_back({c, (int32_t)p, kp.pt.x, kp.pt.y, k->mvuRight[o.second], k->mvInvLevelSigma2[kp.octave],
                         k->fx, k->fy, k->cx, k->cy, k->mbf});
            own.push_back({k, pts[p]});
        }
    }
    std::vector<float> To(T.size()), Xo(X.size());
    std::vector<uint8_t> out(E.size());
    orbo_local_ba(T.data(), fx.data(), (int)cams.size(), X.data(), (int)pts.size(), E.data(), (int)E.size(), 5, 10,
                  To.data(), Xo.data(), out.data(), nullptr);
    std::vector<std::pair<KeyFrame *, MapPoint *>> erase;
    for (size_t e = 0; e < E.size(); ++e)
        if (E[e].ur < 0 && out[e] && !own[e].second->isBad()) erase.push_back(own[e]);
    for (size_t e = 0; e < E.size(); ++e)
        if (E[e].ur >= 0 && out[e] && !own[e].second->isBad()) erase.push_back(own[e]);
    std::unique_lock<std::mutex> lock(map->mMutexMapUpdate);
    for (auto &x : erase) { x.first->EraseMapPointMatch(x.second); x.second->EraseObservation(x.first); }
    for (size_t c = 0; c < local.size(); ++c) {
        cv::Mat P = cv::Mat::eye(4, 4, CV_32F);
        for (int r = 0; r < 3; ++r)
            for (int q = 0; q < 4; ++q) P.at<float>(r, q) = To[12 * c + 4 * r + q];
        local[c]->SetPose(P);
    }
    for (size_t p = 0; p < pts.size(); ++p) {
        cv::Mat P(3, 1, CV_32F);
        for (int q = 0; q < 3; ++q) P.at<float>(q) = Xo[3 * p + q];
        pts[p]->SetWorldPos(P);
        pts[p]->UpdateNormalAndDepth();
    }
}

}  // namespace ref

// Frame::isInFrustum (Frame.cc:284-350): the tracking fields the local-map
// search reads (test setup, the same on both copies).
void in_frustum(Frame &F, MapPoint *mp, float cos_limit) {
    mp->mbTrackInView = false;
    const cv::Mat P = mp->GetWorldPos(), Pc = F.mRcw * P + F.mtcw;
    if (Pc.at<float>(2) < 0.0f) return;
    const float iz = 1.0f / Pc.at<float>(2);
    const float u = F.fx * Pc.at<float>(0) * iz + F.cx, v = F.fy * Pc.at<float>(1) * iz + F.cy;
    if (u < F.mnMinX || u > F.mnMaxX || v < F.mnMinY || v > F.mnMaxY) return;
    const cv::Mat PO = P - F.mOw;
    const float d = cv::norm(PO);
    if (d < mp->GetMinDistanceInvariance() || d > mp->GetMaxDistanceInvariance()) return;
    const float vc = PO.dot(mp->GetNormal()) / d;
    if (vc < cos_limit) return;
    mp->mbTrackInView = true;
    mp->mTrackProjX = u;
    mp->mTrackProjXR = u - F.mbf * iz;
    mp->mTrackProjY = v;
    mp->mnTrackScaleLevel = mp->PredictScale(d, &F);
    mp->mTrackViewCos = vc;
}

std::vector<MapPoint *> all_points(World &w) {
    std::vector<MapPoint *> v;
    for (auto &m : w.mps) v.push_back(m.get());
    return v;
}

std::vector<int64_t> ids(const std::vector<MapPoint *> &v) {
    std::vector<int64_t> s;
    for (MapPoint *p : v) s.push_back(p ? (int64_t)p->mnId : -1);
    return s;
}

cv::Mat scaled(const cv::Mat &T, float s) {   // Scw = [sR st; 0 1]
    cv::Mat S = T.clone();
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 4; ++c) S.at<float>(r, c) *= s;
    return S;
}

int failures = 0;

// Runs gpu(world A) and cpu(world B) on two copies of the map made by `mk`;
// the methods return their outputs as int vectors.
void check_case(const std::string &name, const std::function<std::unique_ptr<World>()> &mk,
                const std::function<std::vector<int64_t>(World &)> &gpu,
                const std::function<std::vector<int64_t>(World &)> &cpu) {
    std::unique_ptr<World> a = mk(), b = mk();
    if (snapshot(*a) != snapshot(*b)) {
        std::printf("%-40s SETUP: the two copies differ\n", name.c_str());
        ++failures;
        return;
    }
    const std::vector<int64_t> ra = gpu(*a), rb = cpu(*b);
    const std::vector<int64_t> sa = snapshot(*a), sb = snapshot(*b);
    const bool ok = ra == rb && sa == sb;
    int64_t nres = ra.empty() ? 0 : ra[0];
    std::printf("%-40s %s (result[0] %lld, outputs %zu, map %zu)\n", name.c_str(), ok ? "ok" : "MISMATCH", (long long)nres,
                ra.size(), sa.size());
    if (!ok) {
        ++failures;
        if (ra != rb)
            for (size_t i = 0; i < std::min(ra.size(), rb.size()); ++i)
                if (ra[i] != rb[i]) { std::printf("  output %zu: gpu %lld cpu %lld\n", i, (long long)ra[i], (long long)rb[i]); break; }
        if (sa != sb)
            for (size_t i = 0; i < std::min(sa.size(), sb.size()); ++i)
                if (sa[i] != sb[i]) { std::printf("  map word %zu: gpu %lld cpu %lld\n", i, (long long)sa[i], (long long)sb[i]); break; }
    }
}

int covis_cb(void *ctx, uint64_t id, uint64_t *out, int cap) {
    World *w = static_cast<World *>(ctx);
    KeyFrame *k = w->map.KeyFrameById(id);
    if (!k) return 0;
    const std::vector<KeyFrame *> v = k->GetBestCovisibilityKeyFrames(10);
    const int n = std::min<int>((int)v.size(), cap);
    for (int i = 0; i < n; ++i) out[i] = v[i]->mnId;
    return n;
}

}  // namespace

int main() {
    const float nn = 0.75f;
    for (uint64_t seed : {11ull, 12ull}) {
        auto mk = [seed] { return make_world(seed); };
        auto name = [seed](const char *s) { return std::string(s) + "/" + std::to_string(seed); };

        for (float th : {3.f, 1.f}) {
            auto setup = [&](World &w) { for (auto &m : w.mps) in_frustum(*w.cur, m.get(), 0.5f); };
            check_case(name(th == 1.f ? "SearchByProjection(local,th1)" : "SearchByProjection(local)"), mk,
                       [&](World &w) { setup(w); return std::vector<int64_t>{ORBmatcher(nn, true).SearchByProjection(*w.cur, all_points(w), th)}; },
                       [&](World &w) { setup(w); return std::vector<int64_t>{ref::ByProjectionLocal(nn, *w.cur, all_points(w), th)}; });
        }
        for (float dz : {0.f, 0.3f, -0.3f})
            for (bool mono : {false, true}) {
                char tag[64];
                std::snprintf(tag, sizeof tag, "SearchByProjection(last,dz%+.1f%s)", dz, mono ? ",mono" : "");
                check_case(name(tag), [seed, dz] { return make_world(seed, dz); },
                           [&](World &w) { return std::vector<int64_t>{ORBmatcher(0.9f, true).SearchByProjection(*w.cur, *w.last, 7.f, mono)}; },
                           [&](World &w) { return std::vector<int64_t>{ref::ByProjectionLast(true, *w.cur, *w.last, 7.f, mono)}; });
            }
        auto found = [](World &w) {
            std::set<MapPoint *> s;
            for (MapPoint *p : w.cur->mvpMapPoints) if (p) s.insert(p);
            return s;
        };
        check_case(name("SearchByProjection(keyframe)"), mk,
                   [&](World &w) { return std::vector<int64_t>{ORBmatcher(0.9f, true).SearchByProjection(*w.cur, w.kfs[2].get(), found(w), 10.f, 100)}; },
                   [&](World &w) { return std::vector<int64_t>{ref::ByProjectionKF(true, *w.cur, w.kfs[2].get(), found(w), 10.f, 100)}; });
        auto sim3_args = [](World &w, std::vector<MapPoint *> &pts, std::vector<MapPoint *> &matched) {
            for (MapPoint *p : w.kfs[0]->mvpMapPoints) if (p) pts.push_back(p);
            matched.assign(w.kfs[2]->N, nullptr);
            for (int i = 0; i < w.kfs[2]->N; i += 3) matched[i] = w.kfs[2]->mvpMapPoints[i];
        };
        check_case(name("SearchByProjection(sim3)"), mk,
                   [&](World &w) { std::vector<MapPoint *> p, m; sim3_args(w, p, m);
                                   int n = ORBmatcher(0.75f, true).SearchByProjection(w.kfs[2].get(), scaled(w.kfs[2]->Tcw, 1.7f), p, m, 10);
                                   std::vector<int64_t> r{n}; for (auto x : ids(m)) r.push_back(x); return r; },
                   [&](World &w) { std::vector<MapPoint *> p, m; sim3_args(w, p, m);
                                   int n = ref::ByProjectionSim3(w.kfs[2].get(), scaled(w.kfs[2]->Tcw, 1.7f), p, m, 10);
                                   std::vector<int64_t> r{n}; for (auto x : ids(m)) r.push_back(x); return r; });
        check_case(name("SearchByBoW(keyframe,frame)"), mk,
                   [&](World &w) { std::vector<MapPoint *> m; int n = ORBmatcher(nn, true).SearchByBoW(w.kfs[1].get(), *w.cur, m);
                                   std::vector<int64_t> r{n}; for (auto x : ids(m)) r.push_back(x); return r; },
                   [&](World &w) { std::vector<MapPoint *> m; int n = ref::BoWFrame(nn, true, w.kfs[1].get(), *w.cur, m);
                                   std::vector<int64_t> r{n}; for (auto x : ids(m)) r.push_back(x); return r; });
        check_case(name("SearchByBoW(keyframe,keyframe)"), mk,
                   [&](World &w) { std::vector<MapPoint *> m; int n = ORBmatcher(nn, true).SearchByBoW(w.kfs[0].get(), w.kfs[2].get(), m);
                                   std::vector<int64_t> r{n}; for (auto x : ids(m)) r.push_back(x); return r; },
                   [&](World &w) { std::vector<MapPoint *> m; int n = ref::BoWKF(nn, true, w.kfs[0].get(), w.kfs[2].get(), m);
                                   std::vector<int64_t> r{n}; for (auto x : ids(m)) r.push_back(x); return r; });
        for (int variant : {0, 1, 2}) {
            const bool ori = variant != 1, distorted = variant == 2;
            auto init = [ori, distorted](World &w, bool gpu) {
                if (distorted)   // a distorted camera's ComputeImageBounds (Frame.cc:475-499): non-zero, non-integer
                    for (Frame *f : {w.last.get(), w.cur.get()}) {
                        f->mnMinX = -13.37f; f->mnMaxX = kW + 21.61f; f->mnMinY = 7.25f; f->mnMaxY = kH - 3.83f;
                        f->AssignFeaturesToGrid();
                    }
                std::vector<cv::Point2f> prev;
                for (auto &k : w.last->mvKeysUn) prev.push_back(k.pt);
                std::vector<int> m;
                const int n = gpu ? ORBmatcher(0.9f, ori).SearchForInitialization(*w.last, *w.cur, prev, m, 100)
                                  : ref::Init(0.9f, ori, *w.last, *w.cur, prev, m, 100);
                std::vector<int64_t> r{n};
                for (int x : m) r.push_back(x);
                for (auto &p : prev) { int32_t b[2]; std::memcpy(b, &p, 8); r.push_back(b[0]); r.push_back(b[1]); }
                return r;
            };
            check_case(name(distorted ? "SearchForInitialization(bounds)"
                                      : ori ? "SearchForInitialization" : "SearchForInitialization(noori)"), mk,
                       [&](World &w) { return init(w, true); }, [&](World &w) { return init(w, false); });
        }
        auto f12 = [](KeyFrame *k1, KeyFrame *k2) {
            const cv::Mat R1 = k1->GetRotation(), t1 = k1->GetTranslation(), R2 = k2->GetRotation(), t2 = k2->GetTranslation();
            const cv::Mat R12 = R1 * R2.t(), t12 = -R1 * R2.t() * t2 + t1;
            cv::Mat tx = cv::Mat::zeros(3, 3, CV_32F);
            tx.at<float>(0, 1) = -t12.at<float>(2); tx.at<float>(0, 2) = t12.at<float>(1);
            tx.at<float>(1, 0) = t12.at<float>(2);  tx.at<float>(1, 2) = -t12.at<float>(0);
            tx.at<float>(2, 0) = -t12.at<float>(1); tx.at<float>(2, 1) = t12.at<float>(0);
            cv::Mat Ki = cv::Mat::eye(3, 3, CV_32F);
            Ki.at<float>(0, 0) = Ki.at<float>(1, 1) = 1.f / kFx;
            Ki.at<float>(0, 2) = -kCx / kFx; Ki.at<float>(1, 2) = -kCy / kFx;
            return Ki.t() * tx * R12 * Ki;
        };
        for (bool stereo : {false, true})
            for (bool ori : {false, true}) {
                auto tri = [&, stereo, ori](World &w, bool gpu) {
                    // free the slots of some keypoints so there is something to triangulate
                    for (int k : {1, 2})
                        for (int i = 0; i < w.kfs[k]->N; i += 2)
                            if (MapPoint *p = w.kfs[k]->mvpMapPoints[i]) { w.kfs[k]->EraseMapPointMatch((size_t)i); p->EraseObservation(w.kfs[k].get()); }
                    std::vector<std::pair<size_t, size_t>> pr;
                    const cv::Mat F = f12(w.kfs[1].get(), w.kfs[2].get());
                    const int n = gpu ? ORBmatcher(0.6f, ori).SearchForTriangulation(w.kfs[1].get(), w.kfs[2].get(), F, pr, stereo)
                                      : ref::Triangulation(ori, w.kfs[1].get(), w.kfs[2].get(), F, pr, stereo);
                    std::vector<int64_t> r{n};
                    for (auto &x : pr) { r.push_back((int64_t)x.first); r.push_back((int64_t)x.second); }
                    return r;
                };
                char tag[64];
                std::snprintf(tag, sizeof tag, "SearchForTriangulation(%s%s)", stereo ? "stereo" : "all", ori ? ",ori" : "");
                check_case(name(tag), mk, [&](World &w) { return tri(w, true); }, [&](World &w) { return tri(w, false); });
            }
        auto sim3 = [](World &w, bool gpu) {
            KeyFrame *k1 = w.kfs[0].get(), *k2 = w.kfs[3].get();
            const cv::Mat R12 = k1->GetRotation() * k2->GetRotation().t();
            const cv::Mat t12 = -R12 * k2->GetTranslation() + k1->GetTranslation();
            std::vector<MapPoint *> m(k1->N, nullptr);
            for (int i = 0; i < k1->N; i += 5)
                if (MapPoint *p = k1->mvpMapPoints[i]) if (p->IsInKeyFrame(k2)) m[i] = p;
            const float s = 1.f;
            const int n = gpu ? ORBmatcher(0.75f, true).SearchBySim3(k1, k2, m, s, R12, t12, 7.5f)
                              : ref::Sim3(k1, k2, m, s, R12, t12, 7.5f);
            std::vector<int64_t> r{n};
            for (auto x : ids(m)) r.push_back(x);
            return r;
        };
        check_case(name("SearchBySim3"), mk, [&](World &w) { return sim3(w, true); }, [&](World &w) { return sim3(w, false); });
        for (int target : {3, 4}) {
            auto fuse = [target](World &w, bool gpu) {
                const std::vector<MapPoint *> pts = w.kfs[0]->GetMapPointMatches();
                const int n = gpu ? ORBmatcher(0.6f, true).Fuse(w.kfs[target].get(), pts, 3.f) : ref::Fuse(w.kfs[target].get(), pts, 3.f);
                return std::vector<int64_t>{n};
            };
            char tag[64];
            std::snprintf(tag, sizeof tag, "Fuse(kf%d)", target);
            check_case(name(tag), mk, [&](World &w) { return fuse(w, true); }, [&](World &w) { return fuse(w, false); });
        }
        auto fuse_sim3 = [](World &w, bool gpu) {
            std::vector<MapPoint *> pts;
            for (MapPoint *p : w.kfs[1]->mvpMapPoints) if (p) pts.push_back(p);
            std::vector<MapPoint *> repl(pts.size(), nullptr);
            KeyFrame *k = w.kfs[4].get();
            const cv::Mat S = scaled(k->Tcw, 1.3f);
            const int n = gpu ? ORBmatcher(0.6f, true).Fuse(k, S, pts, 4.f, repl) : ref::FuseSim3(k, S, pts, 4.f, repl);
            std::vector<int64_t> r{n};
            for (auto x : ids(repl)) r.push_back(x);
            return r;
        };
        check_case(name("Fuse(sim3)"), mk, [&](World &w) { return fuse_sim3(w, true); }, [&](World &w) { return fuse_sim3(w, false); });

        // LocalMapping::SearchInNeighbors' fusion loop (LocalMapping.cc:531-538)
        // as one batch: keyframe 3 first, so that Replaces change descriptors
        // before the later keyframes' searches
        auto fuse_nb = [](World &w, bool gpu) {
            const std::vector<MapPoint *> pts = w.kfs[0]->GetMapPointMatches();
            const std::vector<KeyFrame *> targets{w.kfs[3].get(), w.kfs[5].get(), w.kfs[4].get(), w.kfs[2].get()};
            int n = 0;
            if (gpu) n = OrbxFuseIntoKeyFrames(targets, pts, 3.f, 0.6f);
            else for (KeyFrame *k : targets) n += ref::Fuse(k, pts, 3.f);
            return std::vector<int64_t>{n};
        };
        check_case(name("LocalMapping:Fuse(neighbours,batched)"), mk, [&](World &w) { return fuse_nb(w, true); },
                   [&](World &w) { return fuse_nb(w, false); });
        // LocalMapping::CreateNewMapPoints' searches (LocalMapping.cc:276-315)
        // as one batch, with a stand-in triangulation that accepts 3 of 4
        // pairs and gives keyframe 1 new map points between neighbours
        auto create = [&](World &w, bool gpu) {
            KeyFrame *k1 = w.kfs[1].get();
            const std::vector<KeyFrame *> nb{w.kfs[0].get(), w.kfs[2].get(), w.kfs[3].get()};
            for (KeyFrame *k : {k1, nb[0], nb[1], nb[2]})
                for (int i = 0; i < k->N; i += (k == k1 ? 2 : 3))
                    if (MapPoint *p = k->mvpMapPoints[i]) { k->EraseMapPointMatch((size_t)i); p->EraseObservation(k); }
            std::vector<cv::Mat> F;
            for (KeyFrame *k : nb) F.push_back(f12(k1, k));
            std::vector<std::vector<std::pair<size_t, size_t>>> all;
            if (gpu) all = OrbxSearchForTriangulationBatch(k1, nb, F, false, 0.6f);
            int made = 0;
            for (size_t i = 0; i < nb.size(); ++i) {
                std::vector<std::pair<size_t, size_t>> pairs;
                if (gpu) {
                    for (auto &pr : all[i])
                        if (!k1->GetMapPoint(pr.first)) pairs.push_back(pr);
                } else {
                    ref::Triangulation(false, k1, nb[i], F[i], pairs, false);
                }
                for (auto &pr : pairs) {
                    if ((pr.first + 3 * pr.second) % 4 == 0) continue;
                    auto mp = std::make_unique<MapPoint>(*w.mps[(pr.first * 7 + pr.second) % kPoints]);
                    mp->mnId = (long unsigned)w.mps.size();
                    mp->mObservations.clear();
                    mp->nObs = 0;
                    mp->mbBad = false;
                    mp->mpRefKF = k1;
                    mp->AddObservation(k1, pr.first);
                    mp->AddObservation(nb[i], pr.second);
                    k1->AddMapPoint(mp.get(), pr.first);
                    nb[i]->AddMapPoint(mp.get(), pr.second);
                    mp->ComputeDistinctiveDescriptors();
                    w.mps.push_back(std::move(mp));
                    ++made;
                }
            }
            return std::vector<int64_t>{made};
        };
        check_case(name("LocalMapping:CreateNewMapPoints(batched)"), mk, [&](World &w) { return create(w, true); },
                   [&](World &w) { return create(w, false); });
        // Frame::UndistortKeyPoints (Frame.cc:438-469) and
        // ComputeStereoFromRGBD (Frame.cc:679-701) on the current frame
        auto fbits = [](std::vector<int64_t> &r, float v) { int32_t b; std::memcpy(&b, &v, 4); r.push_back(b); };
        for (float k1 : {-0.28f, 0.f}) {
            auto undist = [&, k1](World &w, bool gpu) {
                Frame &F = *w.cur;
                F.mK = cv::Mat::eye(3, 3, CV_32F);
                F.mK.at<float>(0, 0) = F.mK.at<float>(1, 1) = kFx;
                F.mK.at<float>(0, 2) = kCx;
                F.mK.at<float>(1, 2) = kCy;
                const float D[5] = {k1, 0.07f, 2e-4f, 1.7e-5f, 0.01f};
                F.mDistCoef = cv::Mat(5, 1, CV_32F);
                for (int i = 0; i < 5; ++i) F.mDistCoef.at<float>(i) = D[i];
                for (auto &k : F.mvKeysUn) k.pt.x = -1.f;   // overwritten by both
                if (gpu) {
                    F.UndistortKeyPoints();
                } else if (F.mDistCoef.at<float>(0) == 0.0) {
                    F.mvKeysUn = F.mvKeys;
                } else {
                    std::vector<float> in, out(2 * F.mvKeys.size());
                    for (auto &k : F.mvKeys) { in.push_back(k.pt.x); in.push_back(k.pt.y); }
                    orbo_undistort_points(in.data(), (int)F.mvKeys.size(), F.mK.ptr<float>(0), D, 5, out.data());
                    F.mvKeysUn = F.mvKeys;
                    for (size_t i = 0; i < F.mvKeysUn.size(); ++i) { F.mvKeysUn[i].pt.x = out[2 * i]; F.mvKeysUn[i].pt.y = out[2 * i + 1]; }
                }
                std::vector<int64_t> r{(int64_t)F.mvKeysUn.size()};
                for (auto &k : F.mvKeysUn) { fbits(r, k.pt.x); fbits(r, k.pt.y); fbits(r, k.angle); r.push_back(k.octave); }
                return r;
            };
            check_case(name(k1 == 0.f ? "Frame::UndistortKeyPoints(k1=0)" : "Frame::UndistortKeyPoints"), mk,
                       [&](World &w) { return undist(w, true); }, [&](World &w) { return undist(w, false); });
        }
        auto rgbd = [&](World &w, bool gpu) {
            Frame &F = *w.cur;
            cv::Mat D(480, 640, CV_32F);
            for (int y = 0; y < 480; ++y)
                for (int x = 0; x < 640; ++x)
                    D.at<float>(y, x) = (x * 7 + y * 13) % 61 == 0 ? 0.f
                                      : (x + y) % 97 == 0       ? -1.f
                                                                : 0.5f + (float)((x * 31 + y * 17) % 97) * 0.05f;
            if (gpu) {
                F.ComputeStereoFromRGBD(D);
            } else {   // Frame.cc:679-701
                F.mvuRight.assign(F.N, -1);
                F.mvDepth.assign(F.N, -1);
                for (int i = 0; i < F.N; ++i) {
                    const float d = D.at<float>((int)F.mvKeys[i].pt.y, (int)F.mvKeys[i].pt.x);
                    if (d > 0) { F.mvDepth[i] = d; F.mvuRight[i] = F.mvKeysUn[i].pt.x - F.mbf / d; }
                }
            }
            std::vector<int64_t> r{(int64_t)F.mvDepth.size()};
            for (int i = 0; i < F.N; ++i) { fbits(r, F.mvuRight[i]); fbits(r, F.mvDepth[i]); }
            return r;
        };
        check_case(name("Frame::ComputeStereoFromRGBD"), mk, [&](World &w) { return rgbd(w, true); }, [&](World &w) { return rgbd(w, false); });

        // Optimizer::LocalBundleAdjustment: keyframe 4's window is itself and
        // its two best neighbours (one of them bad), the other observers fixed;
        // some observations pushed far off to make outliers
        auto ba = [](World &w, bool gpu) {
            KeyFrame *k = w.kfs[4].get();
            k->mvpOrderedConnectedKeyFrames.resize(3);
            k->mvpOrderedConnectedKeyFrames[2]->mbBad = true;
            for (auto &kf : w.kfs)
                for (int i = 0; i < kf->N; i += 17) kf->mvKeysUn[i].pt.x += 25.f;
            bool stop = false;
            if (gpu) Optimizer::LocalBundleAdjustment(k, &stop, &w.map);
            else ref::LocalBA(k, &w.map);
            int64_t bad = 0;
            for (auto &m : w.mps) bad += m->isBad();
            return std::vector<int64_t>{bad};
        };
        check_case(name("LocalBundleAdjustment"), mk, [&](World &w) { return ba(w, true); }, [&](World &w) { return ba(w, false); });

        // KeyFrameDatabase: add every keyframe, loop and relocalisation
        // queries, erase one, query again, clear
        auto kfdb = [](World &w, bool gpu) {
            std::vector<int64_t> r;
            for (auto &kf : w.kfs) kf->mvpOrderedConnectedKeyFrames.resize(std::min<size_t>(2, kf->mvpOrderedConnectedKeyFrames.size()));
            auto push = [&r](const std::vector<uint64_t> &v) { r.push_back((int64_t)v.size()); for (auto x : v) r.push_back((int64_t)x); };
            auto bowv = [](const DBoW2::BowVector &b, std::vector<uint32_t> &wd, std::vector<double> &vl) {
                for (auto &kv : b) { wd.push_back(kv.first); vl.push_back(kv.second); }
            };
            if (gpu) {
                ORBVocabulary voc;
                KeyFrameDatabase db(voc);
                for (auto &kf : w.kfs) db.add(kf.get());
                auto as_ids = [](const std::vector<KeyFrame *> &v) { std::vector<uint64_t> o; for (auto *k : v) o.push_back(k->mnId); return o; };
                for (int q : {0, 5, 3}) push(as_ids(db.DetectLoopCandidates(w.kfs[q].get(), 0.001f)));
                push(as_ids(db.DetectRelocalizationCandidates(w.cur.get())));
                db.erase(w.kfs[1].get());
                push(as_ids(db.DetectLoopCandidates(w.kfs[5].get(), 0.001f)));
                push(as_ids(db.DetectRelocalizationCandidates(w.last.get())));
                db.clear();
                push(as_ids(db.DetectRelocalizationCandidates(w.cur.get())));
            } else {
                void *db = orbo_kfdb_create(409);
                for (auto &kf : w.kfs) {
                    std::vector<uint32_t> wd; std::vector<double> vl; bowv(kf->mBowVec, wd, vl);
                    orbo_kfdb_add(db, kf->mnId, wd.data(), vl.data(), (int)wd.size());
                }
                auto det = [&](int reloc, uint64_t qid, const DBoW2::BowVector &b, const std::set<KeyFrame *> &conn, float ms) {
                    std::vector<uint32_t> wd; std::vector<double> vl; bowv(b, wd, vl);
                    std::vector<uint64_t> c;
                    for (auto *k : conn) c.push_back(k->mnId);
                    std::vector<uint64_t> out(64);
                    const int n = orbo_kfdb_detect(db, reloc, qid, wd.data(), vl.data(), (int)wd.size(), c.data(), (int)c.size(), ms,
                                                   covis_cb, &w, out.data(), (int)out.size());
                    out.resize(n);
                    return out;
                };
                for (int q : {0, 5, 3}) push(det(0, w.kfs[q]->mnId, w.kfs[q]->mBowVec, w.kfs[q]->GetConnectedKeyFrames(), 0.001f));
                push(det(1, w.cur->mnId, w.cur->mBowVec, {}, 0.f));
                orbo_kfdb_erase(db, w.kfs[1]->mnId);
                push(det(0, w.kfs[5]->mnId, w.kfs[5]->mBowVec, w.kfs[5]->GetConnectedKeyFrames(), 0.001f));
                push(det(1, w.last->mnId, w.last->mBowVec, {}, 0.f));
                orbo_kfdb_clear(db);
                push(det(1, w.cur->mnId, w.cur->mBowVec, {}, 0.f));
                orbo_kfdb_destroy(db);
            }
            return r;
        };
        check_case(name("KeyFrameDatabase"), mk, [&](World &w) { return kfdb(w, true); }, [&](World &w) { return kfdb(w, false); });

        // KeyFrameDatabase map save / load (KeyFrameDatabase.h:72-81): the
        // database with one keyframe erased is archived with the map as
        // System::SaveMap does (System.cc:629: the map, then the database;
        // each keyframe archives mpKeyFrameDB, KeyFrame.cc:877), loaded into
        // new objects as LoadMap does (System.cc:665-667, SetORBvocabulary
        // after the load), and queried through the loaded keyframes; the
        // reference side queries the database that was saved
        auto kfdb_io = [](World &w, bool gpu) {
            std::vector<int64_t> r;
            for (auto &kf : w.kfs) kf->mvpOrderedConnectedKeyFrames.resize(std::min<size_t>(2, kf->mvpOrderedConnectedKeyFrames.size()));
            auto push = [&r](const std::vector<uint64_t> &v) { r.push_back((int64_t)v.size()); for (auto x : v) r.push_back((int64_t)x); };
            if (gpu) {
                ORBVocabulary voc;
                std::stringstream ss;
                {
                    KeyFrameDatabase db(voc);
                    for (auto &kf : w.kfs) { db.add(kf.get()); kf->mpKeyFrameDB = &db; }
                    db.erase(w.kfs[1].get());
                    Map *mpMap = &w.map;
                    KeyFrameDatabase *mpKeyFrameDatabase = &db;
                    boost::archive::binary_oarchive oa(ss, boost::archive::no_header);
                    oa << mpMap;
                    oa << mpKeyFrameDatabase;
                }   // (the saved database is gone before the load)
                Map *mpMap = nullptr;
                KeyFrameDatabase *mpKeyFrameDatabase = nullptr;
                boost::archive::binary_iarchive ia(ss, boost::archive::no_header);
                ia >> mpMap;
                ia >> mpKeyFrameDatabase;
                mpKeyFrameDatabase->SetORBvocabulary(&voc);
                auto as_ids = [](const std::vector<KeyFrame *> &v) { std::vector<uint64_t> o; for (auto *k : v) o.push_back(k->mnId); return o; };
                bool same_db = true;
                for (KeyFrame *k : mpMap->keyframes) same_db = same_db && k->mpKeyFrameDB == mpKeyFrameDatabase;
                r.push_back(same_db && mpMap->keyframes.size() == w.kfs.size());
                for (int q : {0, 5, 3}) push(as_ids(mpKeyFrameDatabase->DetectLoopCandidates(mpMap->KeyFrameById(w.kfs[q]->mnId), 0.001f)));
                push(as_ids(mpKeyFrameDatabase->DetectRelocalizationCandidates(w.cur.get())));
                push(as_ids(mpKeyFrameDatabase->DetectRelocalizationCandidates(w.last.get())));
                // the loaded database stays live: erase, add back, query
                mpKeyFrameDatabase->erase(mpMap->KeyFrameById(w.kfs[2]->mnId));
                mpKeyFrameDatabase->add(mpMap->KeyFrameById(w.kfs[2]->mnId));
                push(as_ids(mpKeyFrameDatabase->DetectLoopCandidates(mpMap->KeyFrameById(w.kfs[5]->mnId), 0.001f)));
                for (KeyFrame *k : mpMap->keyframes) delete k;
                delete mpKeyFrameDatabase;
                delete mpMap;
                for (auto &kf : w.kfs) kf->mpKeyFrameDB = nullptr;
            } else {
                auto bowv = [](const DBoW2::BowVector &b, std::vector<uint32_t> &wd, std::vector<double> &vl) {
                    for (auto &kv : b) { wd.push_back(kv.first); vl.push_back(kv.second); }
                };
                void *db = orbo_kfdb_create(409);
                auto add = [&](KeyFrame *kf) {
                    std::vector<uint32_t> wd; std::vector<double> vl; bowv(kf->mBowVec, wd, vl);
                    orbo_kfdb_add(db, kf->mnId, wd.data(), vl.data(), (int)wd.size());
                };
                for (auto &kf : w.kfs) add(kf.get());
                orbo_kfdb_erase(db, w.kfs[1]->mnId);
                auto det = [&](int reloc, uint64_t qid, const DBoW2::BowVector &b, const std::set<KeyFrame *> &conn, float ms) {
                    std::vector<uint32_t> wd; std::vector<double> vl; bowv(b, wd, vl);
                    std::vector<uint64_t> c;
                    for (auto *k : conn) c.push_back(k->mnId);
                    std::vector<uint64_t> out(64);
                    const int n = orbo_kfdb_detect(db, reloc, qid, wd.data(), vl.data(), (int)wd.size(), c.data(), (int)c.size(), ms,
                                                   covis_cb, &w, out.data(), (int)out.size());
                    out.resize(n);
                    return out;
                };
                r.push_back(1);
                for (int q : {0, 5, 3}) push(det(0, w.kfs[q]->mnId, w.kfs[q]->mBowVec, w.kfs[q]->GetConnectedKeyFrames(), 0.001f));
                push(det(1, w.cur->mnId, w.cur->mBowVec, {}, 0.f));
                push(det(1, w.last->mnId, w.last->mBowVec, {}, 0.f));
                orbo_kfdb_erase(db, w.kfs[2]->mnId);
                add(w.kfs[2].get());
                push(det(0, w.kfs[5]->mnId, w.kfs[5]->mBowVec, w.kfs[5]->GetConnectedKeyFrames(), 0.001f));
                orbo_kfdb_destroy(db);
            }
            return r;
        };
        check_case(name("KeyFrameDatabase(save/load)"), mk, [&](World &w) { return kfdb_io(w, true); }, [&](World &w) { return kfdb_io(w, false); });
    }
    std::printf("%s: %d mismatching case(s)\n", failures ? "FAIL" : "PASS", failures);
    return failures ? 1 : 0;
}
