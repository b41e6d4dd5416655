"""Host mirrors of the per-frame neighbours of the front end (SURVEY.md §8
f4) over liborbx (include/orbx.h): MapPoint::ComputeDistinctiveDescriptors
(MapPoint.cc:288-361), Frame::UndistortKeyPoints (Frame.cc:438-469) and the
Tracking::Grab* colour conversion (Tracking.cc:179-264).  GPU only; no host
fallback."""
from __future__ import annotations

import numpy as np

from ._lib import KEYPOINT_DTYPE, check, load, ptr


def compute_distinctive_descriptors(descs, device: int = 0) -> np.ndarray:
    """Batch form of MapPoint::ComputeDistinctiveDescriptors.  descs: a list
    (one entry per map point) of (N_i, 32) u8 observation descriptors, or a
    pair (desc (total, 32), offsets (np + 1)).  Returns best[np]: the row of
    each point's list that becomes mDescriptor (-1: no descriptors)."""
    if isinstance(descs, tuple):
        desc, offsets = descs
        desc = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        offsets = np.ascontiguousarray(offsets, np.int32)
    else:
        sizes = [len(d) for d in descs]
        offsets = np.zeros(len(descs) + 1, np.int32)
        offsets[1:] = np.cumsum(sizes)
        desc = (np.concatenate([np.asarray(d, np.uint8).reshape(-1, 32) for d in descs])
                if offsets[-1] else np.zeros((0, 32), np.uint8))
    npts = len(offsets) - 1
    best = np.full(max(npts, 1), -1, np.int32)
    check(load().orbx_distinctive_descriptors(device, ptr(desc), ptr(offsets), npts, ptr(best)),
          "orbx_distinctive_descriptors")
    return best[:npts]


def undistort_keypoints(kps: np.ndarray, K, dist, device: int = 0) -> np.ndarray:
    """Frame::UndistortKeyPoints: mvKeysUn from mvKeys, mK (3x3) and
    mDistCoef (k1 k2 p1 p2 [k3])."""
    kps = np.ascontiguousarray(kps, KEYPOINT_DTYPE)
    K = np.ascontiguousarray(K, np.float32).reshape(9)
    dist = np.ascontiguousarray(dist, np.float32).reshape(-1)
    out = np.empty_like(kps)
    check(load().orbx_undistort_keypoints(device, ptr(kps), len(kps), ptr(K), ptr(dist), len(dist), ptr(out)),
          "orbx_undistort_keypoints")
    return out


def cvt_gray(img: np.ndarray, rgb: bool = True, device: int = 0) -> np.ndarray:
    """cvtColor(..., CV_RGB2GRAY / CV_BGR2GRAY / CV_RGBA2GRAY / CV_BGRA2GRAY)
    of an (h, w, 3|4) u8 image; a 2-D image is returned as is (the
    reference converts only 3- and 4-channel input)."""
    img = np.asarray(img)
    if img.ndim == 2:
        return img
    img = np.ascontiguousarray(img, np.uint8)
    h, w, cn = img.shape
    out = np.empty((h, w), np.uint8)
    check(load().orbx_cvt_gray(device, ptr(img), w, h, w * cn, cn, int(bool(rgb)), ptr(out), w), "orbx_cvt_gray")
    return out
