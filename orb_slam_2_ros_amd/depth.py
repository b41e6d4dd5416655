"""Host mirror of ORB_SLAM2::Frame's depth association for stereo and RGB-D
frames, over liborbx.so.

Reference: orb_slam2/src/Frame.cc:502-676 (ComputeStereoMatches) and
:679-701 (ComputeStereoFromRGBD).  Both run on the GPU; there is no CPU path.

``compute_stereo_matches`` works on the pair the two extractors extracted
last (their device-resident pyramids are the mvImagePyramid the reference
reads), with that call's keypoints and descriptors, exactly the inputs
Frame::ComputeStereoMatches reads from the Frame.  ``mb`` is the Frame's
baseline (mbf / fx); the reference reads it before Frame.cc:115 assigns it,
so callers pass it explicitly.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import KEYPOINT_DTYPE, check, ptr


def compute_stereo_matches(left, right, mvKeys, mDescriptors, mvKeysRight, mDescriptorsRight,
                           mbf: float, mb: float):
    """Returns (mvuRight, mvDepth, nkept) -- float32 arrays of len(mvKeys)."""
    lib = _lib.load()
    kl = np.ascontiguousarray(mvKeys, KEYPOINT_DTYPE)
    kr = np.ascontiguousarray(mvKeysRight, KEYPOINT_DTYPE)
    dl = np.ascontiguousarray(mDescriptors, np.uint8).reshape(-1, 32)
    dr = np.ascontiguousarray(mDescriptorsRight, np.uint8).reshape(-1, 32)
    if len(kl) != len(dl) or len(kr) != len(dr):
        raise ValueError("keypoints and descriptors differ in length")
    ur = np.full(max(len(kl), 1), -1, np.float32)
    dp = np.full(max(len(kl), 1), -1, np.float32)
    nk = ctypes.c_int(0)
    check(lib.orbx_compute_stereo_matches(left._h, right._h, ptr(kl), ptr(dl), len(kl), ptr(kr), ptr(dr),
                                          len(kr), ctypes.c_float(mbf), ctypes.c_float(mb), ptr(ur), ptr(dp),
                                          ctypes.byref(nk)), "ComputeStereoMatches")
    return ur[:len(kl)].copy(), dp[:len(kl)].copy(), nk.value


def stereo_from_rgbd(mvKeys, imDepth: np.ndarray, mbf: float, mvKeysUn=None, device: int = 0):
    """Frame::ComputeStereoFromRGBD: returns (mvuRight, mvDepth, nkept)."""
    lib = _lib.load()
    k = np.ascontiguousarray(mvKeys, KEYPOINT_DTYPE)
    ku = None if mvKeysUn is None else np.ascontiguousarray(mvKeysUn, KEYPOINT_DTYPE)
    d = np.ascontiguousarray(imDepth, np.float32)
    if d.ndim != 2:
        raise ValueError("imDepth must be a 2-D float32 (CV_32F) image")
    ur = np.full(max(len(k), 1), -1, np.float32)
    dp = np.full(max(len(k), 1), -1, np.float32)
    nk = ctypes.c_int(0)
    check(lib.orbx_stereo_from_rgbd(device, ptr(k), ptr(ku), len(k), ptr(d), d.shape[1], d.shape[0],
                                    d.strides[0], ctypes.c_float(mbf), ptr(ur), ptr(dp), ctypes.byref(nk)),
          "ComputeStereoFromRGBD")
    return ur[:len(k)].copy(), dp[:len(k)].copy(), nk.value
