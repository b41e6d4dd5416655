// KeyFrameDatabase_orbx.cc -- orb_slam2/src/KeyFrameDatabase.cc for a
// reference tree that links liborbx.so (with integration/KeyFrameDatabase.h).
// Each method forwards to the device database by keyframe id; the candidate
// lists come back in the reference's order (KeyFrameDatabase.cc:76-330).
//
// tests/cxx/forwarders_test.cpp compiles this file against test stand-ins of
// the reference headers and checks it on the GPU against the CPU oracle's
// literal restatement of KeyFrameDatabase.cc.
#include <algorithm>
#include <set>

#include "KeyFrameDatabase.h"
#include "orbx_orbslam2.hpp"

namespace ORB_SLAM2 {

namespace {
void bow_arrays(const DBoW2::BowVector &bow, std::vector<uint32_t> &w, std::vector<double> &v) {
    w.clear();
    v.clear();
    for (const auto &kv : bow) {   // a std::map: ascending word ids
        w.push_back(kv.first);
        v.push_back(kv.second);
    }
}
}  // namespace

KeyFrameDatabase::KeyFrameDatabase(const ORBVocabulary &voc) : mpVoc(&voc) {
    orbx_detail::check(orbx_kfdb_create(orbx_detail::device_index(), &mDb), "KeyFrameDatabase");
}

// (KeyFrameDatabase.h:75, the archive's constructor)
KeyFrameDatabase::KeyFrameDatabase() {
    orbx_detail::check(orbx_kfdb_create(orbx_detail::device_index(), &mDb), "KeyFrameDatabase");
}

KeyFrameDatabase::~KeyFrameDatabase() { orbx_kfdb_destroy(mDb); }

void KeyFrameDatabase::AddLocked(KeyFrame *pKF) {
    std::vector<uint32_t> w;
    std::vector<double> v;
    bow_arrays(pKF->mBowVec, w, v);
    orbx_detail::check(orbx_kfdb_add(mDb, pKF->mnId, w.data(), v.data(), (int)w.size()), "KeyFrameDatabase::add");
    mKFs[pKF->mnId] = pKF;
}

// :37-44
void KeyFrameDatabase::add(KeyFrame *pKF) {
    std::unique_lock<std::mutex> lock(mMutex);
    AddLocked(pKF);
    mvpKFs.push_back(pKF);
}

// :46-67
void KeyFrameDatabase::erase(KeyFrame *pKF) {
    std::unique_lock<std::mutex> lock(mMutex);
    if (!mKFs.erase(pKF->mnId)) return;   // not in the database: nothing to remove, as the reference
    orbx_detail::check(orbx_kfdb_erase(mDb, pKF->mnId), "KeyFrameDatabase::erase");
    mvpKFs.erase(std::find(mvpKFs.begin(), mvpKFs.end(), pKF));
}

// :69-73
void KeyFrameDatabase::clear() {
    std::unique_lock<std::mutex> lock(mMutex);
    orbx_detail::check(orbx_kfdb_clear(mDb), "KeyFrameDatabase::clear");
    mKFs.clear();
    mvpKFs.clear();
}

// Map serialisation (KeyFrameDatabase.cc:371-384).  The reference archives its
// inverted file, mvInvertedFile's KeyFrame* lists, each in insertion order.
// Here the archived state is the database's keyframes in insertion order; each
// keyframe archives its own mBowVec (KeyFrame.cc:858), so the inverted file is
// determined by them: adding them again in that order gives every word's
// posting list the same keyframes in the same order.  The vocabulary is not
// archived, as in the reference.
template <class Archive>
void KeyFrameDatabase::serialize(Archive &ar, const unsigned int) {
    std::unique_lock<std::mutex> lock(mMutex);
    ar & mvpKFs;
}
template void KeyFrameDatabase::serialize(boost::archive::binary_iarchive &, const unsigned int);
template void KeyFrameDatabase::serialize(boost::archive::binary_oarchive &, const unsigned int);

// (KeyFrameDatabase.h:76) System::LoadMap calls this once the map and the
// database are loaded (System.cc:666-667): every archived keyframe is then
// complete, and the device database is rebuilt from them.  On a live database
// it rebuilds the same state.
void KeyFrameDatabase::SetORBvocabulary(ORBVocabulary *porbv) {
    std::unique_lock<std::mutex> lock(mMutex);
    mpVoc = porbv;
    orbx_detail::check(orbx_kfdb_clear(mDb), "KeyFrameDatabase::SetORBvocabulary");
    mKFs.clear();
    for (KeyFrame *pKF : mvpKFs) AddLocked(pKF);
}

// GetBestCovisibilityKeyFrames(10) of a candidate, by id (:129, :279)
int KeyFrameDatabase::Covisible(void *ctx, uint64_t id, uint64_t *out, int cap) {
    KeyFrameDatabase *db = static_cast<KeyFrameDatabase *>(ctx);
    auto it = db->mKFs.find(id);
    if (it == db->mKFs.end()) return 0;
    const std::vector<KeyFrame *> v = it->second->GetBestCovisibilityKeyFrames(10);
    const int n = std::min<int>((int)v.size(), cap);
    for (int i = 0; i < n; ++i) out[i] = v[i]->mnId;
    return n;
}

std::vector<KeyFrame *> KeyFrameDatabase::Detect(int reloc, uint64_t qid, const DBoW2::BowVector &bow,
                                                 const std::vector<uint64_t> &connected, float minScore) {
    std::vector<uint32_t> w;
    std::vector<double> v;
    bow_arrays(bow, w, v);
    std::unique_lock<std::mutex> lock(mMutex);
    std::vector<uint64_t> ids(std::max<size_t>(mKFs.size(), 1));
    int n = 0;
    const int rc = reloc ? orbx_kfdb_detect_relocalization_candidates(mDb, qid, w.data(), v.data(), (int)w.size(),
                                                                       Covisible, this, ids.data(),
                                                                       (int)ids.size(), &n)
                         : orbx_kfdb_detect_loop_candidates(mDb, qid, w.data(), v.data(), (int)w.size(),
                                                            connected.data(), (int)connected.size(), minScore,
                                                            Covisible, this, ids.data(), (int)ids.size(), &n);
    orbx_detail::check(rc, reloc ? "DetectRelocalizationCandidates" : "DetectLoopCandidates");
    std::vector<KeyFrame *> out;
    out.reserve(n);
    for (int i = 0; i < n; ++i) out.push_back(mKFs.at(ids[i]));
    return out;
}

// :76-236
std::vector<KeyFrame *> KeyFrameDatabase::DetectLoopCandidates(KeyFrame *pKF, float minScore) {
    std::vector<uint64_t> connected;
    for (KeyFrame *k : pKF->GetConnectedKeyFrames()) connected.push_back(k->mnId);
    return Detect(0, pKF->mnId, pKF->mBowVec, connected, minScore);
}

// :238-330
std::vector<KeyFrame *> KeyFrameDatabase::DetectRelocalizationCandidates(Frame *F) {
    return Detect(1, F->mnId, F->mBowVec, {}, 0.f);
}

}  // namespace ORB_SLAM2
