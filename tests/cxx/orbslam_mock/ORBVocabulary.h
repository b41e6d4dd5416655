// Test stand-in for orb_slam2/include/ORBVocabulary.h, typedef'd to the
// adapter's vocabulary as INTEGRATION.md §2 shows.
#pragma once
#include "orbx_orbslam2.hpp"

namespace ORB_SLAM2 {
typedef OrbxVocabulary ORBVocabulary;
}  // namespace ORB_SLAM2
