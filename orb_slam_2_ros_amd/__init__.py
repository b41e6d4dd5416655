"""orb_slam_2_ros_amd -- MI355X-native ORB front end for ORB-SLAM2.

The hot path of wjjcdy/orb_slam_2_ros (ORBextractor: pyramid, per-cell FAST-9,
quadtree distribution, orientation, rBRIEF; ORBmatcher::SearchForInitialization;
Frame's stereo / RGB-D depth association; the other ORBmatcher searches; the
DBoW2 vocabulary transform)
as hand-written HIP kernels for gfx950 behind a C ABI (include/orbx.h,
liborbx.so), with host mirrors of the reference's classes.
"""
from ._lib import KEYPOINT_DTYPE, OrbxError, load  # noqa: F401
from .extractor import ORBextractor  # noqa: F401
from .matcher import Frame, ORBmatcher  # noqa: F401
from .depth import compute_stereo_matches, stereo_from_rgbd  # noqa: F401
from .vocabulary import ORBVocabulary  # noqa: F401
from .frame_aux import compute_distinctive_descriptors, cvt_gray, undistort_keypoints  # noqa: F401
from .keyframe_db import KeyFrameDatabase  # noqa: F401
from .optimizer import local_bundle_adjustment  # noqa: F401

__all__ = ["KEYPOINT_DTYPE", "OrbxError", "load", "ORBextractor", "ORBmatcher", "Frame",
           "compute_stereo_matches", "stereo_from_rgbd", "ORBVocabulary",
           "compute_distinctive_descriptors", "cvt_gray", "undistort_keypoints", "KeyFrameDatabase",
           "local_bundle_adjustment"]
