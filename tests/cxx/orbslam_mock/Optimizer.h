// Test stand-in for orb_slam2/include/Optimizer.h: the one function
// integration/Optimizer_orbx.cc replaces (Optimizer.h:45).
#pragma once
#include "Frame.h"

namespace ORB_SLAM2 {
class Optimizer {
public:
    void static LocalBundleAdjustment(KeyFrame *pKF, bool *pbStopFlag, Map *pMap);
};
}  // namespace ORB_SLAM2
