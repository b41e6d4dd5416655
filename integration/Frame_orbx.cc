// Frame_orbx.cc -- the three Frame member functions of orb_slam2/src/Frame.cc
// that become forwarders in a reference tree linking liborbx.so (replace
// their bodies in Frame.cc; the rest of Frame.cc is unchanged).  The
// extractors that produced mvKeys / mvKeysRight hold the device pyramids that
// the reference reads from mvImagePyramid.
//
// tests/cxx/forwarders_test.cpp compiles this file against test stand-ins of
// the reference headers and checks UndistortKeyPoints / ComputeStereoFromRGBD
// against the CPU oracle; ComputeStereoMatches runs through the same
// OrbxFrame call in tests/cxx/adapter_test.cpp (stereo mode).
#include "Frame.h"
#include "orbx_orbslam2.hpp"

namespace ORB_SLAM2 {

// Frame.cc:502-676.  mb = mbf / fx from this frame's own mK: the reference
// reads the member mb before Frame.cc:115 assigns it.
void Frame::ComputeStereoMatches() {
    OrbxFrame::ComputeStereoMatches(*mpORBextractorLeft, *mpORBextractorRight, mvKeys, mDescriptors, mvKeysRight,
                                    mDescriptorsRight, mbf, mbf / mK.at<float>(0, 0), mvuRight, mvDepth);
}

// Frame.cc:679-701
void Frame::ComputeStereoFromRGBD(const cv::Mat &imDepth) {
    OrbxFrame::ComputeStereoFromRGBD(mvKeys, mvKeysUn, imDepth, mbf, mvuRight, mvDepth);
}

// Frame.cc:438-469 (a zero k1 copies mvKeys, as the reference)
void Frame::UndistortKeyPoints() { OrbxFrameAux::UndistortKeyPoints(mvKeys, mK, mDistCoef, mvKeysUn); }

}  // namespace ORB_SLAM2
