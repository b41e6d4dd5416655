// KeyFrameDatabase.h -- replacement for orb_slam2/include/KeyFrameDatabase.h
// in a reference tree that links liborbx.so.  The public interface is the
// reference's (KeyFrameDatabase.h:43-60); the inverted file
// (mvInvertedFile) and the per-keyframe query state the reference keeps in
// KeyFrame (mnLoopQuery, mnLoopWords, mLoopScore and the reloc trio) live in
// the device database (include/orbx.h orbx_kfdb_*).  Keyframes are named by
// mnId; the id -> KeyFrame* table maps results back and serves the
// covisibility callback.  Map serialisation keeps the fork's members
// (KeyFrameDatabase.h:72-81: the default constructor, SetORBvocabulary, the
// private serialize reached through boost::serialization::access), so
// KeyFrame.cc:877 (`ar & mpKeyFrameDB`) and System::SaveMap / LoadMap
// (System.cc:629, 666-667) compile unchanged: the archive holds the
// database's keyframes in insertion order, and SetORBvocabulary -- which
// LoadMap calls once the map is loaded -- rebuilds the device database from
// them (KeyFrameDatabase_orbx.cc).
#ifndef KEYFRAMEDATABASE_H
#define KEYFRAMEDATABASE_H

#include <mutex>
#include <unordered_map>
#include <vector>

#include "BoostArchiver.h"
#include "Frame.h"
#include "KeyFrame.h"
#include "ORBVocabulary.h"
#include "orbx.h"

namespace ORB_SLAM2 {

class KeyFrameDatabase {
public:
    explicit KeyFrameDatabase(const ORBVocabulary &voc);
    ~KeyFrameDatabase();
    KeyFrameDatabase(const KeyFrameDatabase &) = delete;
    KeyFrameDatabase &operator=(const KeyFrameDatabase &) = delete;

    void add(KeyFrame *pKF);
    void erase(KeyFrame *pKF);
    void clear();

    // Loop Detection
    std::vector<KeyFrame *> DetectLoopCandidates(KeyFrame *pKF, float minScore);

    // Relocalization
    std::vector<KeyFrame *> DetectRelocalizationCandidates(Frame *F);

protected:
    const ORBVocabulary *mpVoc = nullptr;
    orbx_kfdb *mDb = nullptr;
    std::unordered_map<uint64_t, KeyFrame *> mKFs;   // the keyframes in the database, by mnId
    std::vector<KeyFrame *> mvpKFs;                  // the same keyframes in insertion order (archived)
    std::mutex mMutex;

    static int Covisible(void *ctx, uint64_t id, uint64_t *out, int cap);
    std::vector<KeyFrame *> Detect(int reloc, uint64_t qid, const DBoW2::BowVector &bow,
                                   const std::vector<uint64_t> &connected, float minScore);
    void AddLocked(KeyFrame *pKF);

// map serialization addition (KeyFrameDatabase.h:72-81)
public:
    // for serialization: an empty database; SetORBvocabulary fills it from the
    // archived keyframes
    KeyFrameDatabase();
    void SetORBvocabulary(ORBVocabulary *porbv);

private:
    friend class boost::serialization::access;
    template <class Archive>
    void serialize(Archive &ar, const unsigned int version);
};

}  // namespace ORB_SLAM2

#endif
