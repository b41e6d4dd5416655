"""Host mirror of ``ORB_SLAM2::ORBextractor`` over liborbx.so.

Reference interface: orb_slam2/include/ORBextractor.h:45-111.

    ex = ORBextractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST)
    keypoints, descriptors = ex(image, mask)          # operator()
    ex.GetLevels(), ex.GetScaleFactor(), ex.GetScaleFactors(), ...
    ex.mvImagePyramid                                  # levels of the last call

``keypoints`` is a structured array with cv::KeyPoint's fields
(x, y, size, angle, response, octave, class_id); ``descriptors`` is N x 32 u8.
Every call runs on the GPU; there is no CPU path.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import KEYPOINT_DTYPE, check, ptr


class ORBextractor:
    HARRIS_SCORE = 0
    FAST_SCORE = 1

    def __init__(self, nfeatures: int, scaleFactor: float, nlevels: int, iniThFAST: int,
                 minThFAST: int, device: int = 0):
        lib = _lib.load()
        self._lib = lib
        h = lib.orbx_extractor_create(device, int(nfeatures), ctypes.c_float(scaleFactor),
                                      int(nlevels), int(iniThFAST), int(minThFAST))
        if not h:
            raise _lib.OrbxError(_lib.ORBX_ENODEV if lib.orbx_device_count() == 0 else _lib.ORBX_EINVAL,
                                 "ORBextractor")
        self._h = ctypes.c_void_p(h)
        self.nfeatures = int(nfeatures)
        self.nlevels = int(nlevels)
        self.device = device
        self._last_shape = None

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.orbx_extractor_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- getters (ORBextractor.h:63-83) ------------------------------------
    def GetLevels(self) -> int:
        return int(self._lib.orbx_extractor_get_levels(self._h))

    def GetScaleFactor(self) -> float:
        return float(self._lib.orbx_extractor_get_scale_factor(self._h))

    def _table(self, which: int) -> list:
        out = np.zeros(self.nlevels, dtype=np.float32)
        check(self._lib.orbx_extractor_get_scale_table(self._h, which, ptr(out), self.nlevels), "scale table")
        return [float(v) for v in out]

    def GetScaleFactors(self) -> list:
        return self._table(0)

    def GetInverseScaleFactors(self) -> list:
        return self._table(1)

    def GetScaleSigmaSquares(self) -> list:
        return self._table(2)

    def GetInverseScaleSigmaSquares(self) -> list:
        return self._table(3)

    def level_quotas(self) -> list:
        out = np.zeros(self.nlevels, dtype=np.int32)
        check(self._lib.orbx_extractor_get_level_quotas(self._h, ptr(out), self.nlevels), "quotas")
        return [int(v) for v in out]

    # -- operator() (ORBextractor.cc:1083-1149) ----------------------------
    def __call__(self, image, mask=None):
        """Returns (keypoints, descriptors).  An empty image returns (None, None),
        mirroring the reference leaving its outputs untouched."""
        if image is None or getattr(image, "size", 0) == 0:
            return None, None
        img = np.asarray(image)
        if img.dtype != np.uint8 or img.ndim != 2:
            raise ValueError("ORBextractor expects a 2-D uint8 (CV_8UC1) image")
        img = np.ascontiguousarray(img)
        h, w = img.shape
        cap = self.nfeatures + 16 * self.nlevels + 64
        while True:
            kps = np.empty(cap, dtype=KEYPOINT_DTYPE)
            desc = np.empty((cap, 32), dtype=np.uint8)
            n = ctypes.c_int(0)
            rc = self._lib.orbx_extract(self._h, ptr(img), w, h, img.strides[0], ptr(kps), ptr(desc), cap,
                                        ctypes.byref(n))
            if rc == _lib.ORBX_ERANGE:
                cap = n.value
                continue
            check(rc, "ORBextractor()")
            break
        self._last_shape = (h, w)
        nk = n.value
        return kps[:nk], desc[:nk]   # (views of this call's own arrays)

    @property
    def mvImagePyramid(self) -> list:
        """The last call's pyramid (ORBextractor::mvImagePyramid without the
        EDGE_THRESHOLD border), all levels in one orbx_extractor_pyramid_host
        call (one stream-ordered wait)."""
        levels = []
        for l in range(self.nlevels):
            w, h = ctypes.c_int(0), ctypes.c_int(0)
            check(self._lib.orbx_extractor_pyramid_level(self._h, l, None, 0, ctypes.byref(w), ctypes.byref(h)),
                  "pyramid level")
            levels.append(np.zeros((h.value, w.value), dtype=np.uint8))
        outs = (ctypes.c_void_p * len(levels))(*[a.ctypes.data for a in levels])
        pitches = (ctypes.c_size_t * len(levels))(*[a.strides[0] for a in levels])
        check(self._lib.orbx_extractor_pyramid_host(self._h, outs, pitches, len(levels)), "pyramid")
        return levels

    # -- batched device API -------------------------------------------------
    def reserve(self, width: int, height: int, max_batch: int) -> None:
        check(self._lib.orbx_extractor_reserve(self._h, width, height, max_batch), "reserve")

    def kp_stride(self) -> int:
        return check(self._lib.orbx_extractor_kp_stride(self._h), "kp_stride")

    def extract_batch_device(self, d_images: int, frame_stride: int, pitch: int, batch: int,
                             stream: int | None = None) -> None:
        check(self._lib.orbx_extract_batch_device(self._h, ctypes.c_void_p(d_images), frame_stride, pitch,
                                                  batch, ctypes.c_void_p(stream or 0)), "extract_batch_device")

    def mono_step_device(self, d_images: int, frame_stride: int, pitch: int, batch: int, window: int = 100,
                         nnratio: float = 0.9, check_ori: bool = True, stream: int | None = None) -> None:
        check(self._lib.orbx_mono_step_device(self._h, ctypes.c_void_p(d_images), frame_stride, pitch, batch,
                                              window, ctypes.c_float(nnratio), int(check_ori),
                                              ctypes.c_void_p(stream or 0)), "mono_step_device")

    def stereo_step_device(self, d_images: int, frame_stride: int, pitch: int, pairs: int, mbf: float,
                           mb: float, stream: int | None = None) -> None:
        """Frames 2p / 2p+1 are the left / right images of pair p."""
        check(self._lib.orbx_stereo_step_device(self._h, ctypes.c_void_p(d_images), frame_stride, pitch, pairs,
                                                ctypes.c_float(mbf), ctypes.c_float(mb),
                                                ctypes.c_void_p(stream or 0)), "stereo_step_device")

    def rgbd_step_device(self, d_images: int, frame_stride: int, pitch: int, batch: int, d_depth: int,
                         depth_stride: int, depth_pitch: int, mbf: float, stream: int | None = None) -> None:
        check(self._lib.orbx_rgbd_step_device(self._h, ctypes.c_void_p(d_images), frame_stride, pitch, batch,
                                              ctypes.c_void_p(d_depth), depth_stride, depth_pitch,
                                              ctypes.c_float(mbf), ctypes.c_void_p(stream or 0)),
              "rgbd_step_device")

    def depth_download(self, index: int):
        """(mvuRight, mvDepth, nkept) of pair / frame `index` of the last stereo / RGB-D step."""
        cap = self.kp_stride()
        ur = np.zeros(cap, dtype=np.float32)
        dp = np.zeros(cap, dtype=np.float32)
        n, nk = ctypes.c_int(0), ctypes.c_int(0)
        check(self._lib.orbx_depth_download(self._h, index, ptr(ur), ptr(dp), cap, ctypes.byref(n),
                                            ctypes.byref(nk)), "depth_download")
        return ur[:n.value].copy(), dp[:n.value].copy(), nk.value

    def pack_bytes(self) -> int:
        """Size of the orbx_batch_pack_device layout for the current batch."""
        nb = ctypes.c_int64(0)
        check(self._lib.orbx_batch_pack_device(self._h, None, 0, ctypes.byref(nb), None), "pack size")
        return nb.value

    def pack_device(self, d_out: int, cap: int, stream: int | None = None) -> int:
        """Copy the current results (counts | keypoints | descriptors) into a
        device buffer for the keyframe all-gather; returns the bytes written."""
        nb = ctypes.c_int64(0)
        check(self._lib.orbx_batch_pack_device(self._h, ctypes.c_void_p(d_out), cap, ctypes.byref(nb),
                                               ctypes.c_void_p(stream or 0)), "pack_device")
        return nb.value

    def batch_download(self, frame: int):
        cap = self.kp_stride()
        kps = np.zeros(cap, dtype=KEYPOINT_DTYPE)
        desc = np.zeros((cap, 32), dtype=np.uint8)
        n = ctypes.c_int(0)
        check(self._lib.orbx_batch_download(self._h, frame, ptr(kps), ptr(desc), cap, ctypes.byref(n)),
              "batch_download")
        return kps[:n.value].copy(), desc[:n.value].copy()

    def mono_matches_download(self, frame: int):
        cap = self.kp_stride()
        m = np.full(cap, -1, dtype=np.int32)
        n1, nm = ctypes.c_int(0), ctypes.c_int(0)
        check(self._lib.orbx_mono_matches_download(self._h, frame, ptr(m), cap, ctypes.byref(n1),
                                                   ctypes.byref(nm)), "mono_matches_download")
        return m[:n1.value].copy(), nm.value

    def split(self, parts: int = 0) -> int:
        """Batch split into sub-batches on internal streams (0 = query)."""
        return check(self._lib.orbx_extractor_split(self._h, int(parts)), "split")

    def pipeline(self, on: int = -1) -> int:
        """Level-pipelined extraction on internal streams (2 deep, 1 on, 0 off, -1 query)."""
        return check(self._lib.orbx_extractor_pipeline(self._h, int(on)), "pipeline")

    def overlap_match(self, on: int = -1) -> int:
        """Mono-step matcher on an internal stream, overlapping the next step's
        extraction (1 on, 0 off, -1 query; include/orbx.h)."""
        return check(self._lib.orbx_extractor_overlap_match(self._h, int(on)), "overlap_match")

    def set_profiling(self, on: bool) -> None:
        check(self._lib.orbx_extractor_set_profiling(self._h, int(on)), "set_profiling")

    def stage_times(self) -> list:
        out = np.zeros(8, dtype=np.float32)
        n = check(self._lib.orbx_extractor_stage_times(self._h, ptr(out), 8), "stage_times")
        return [float(v) for v in out[:n]]

    def debug_fetch(self, frame: int, level: int, what: int) -> np.ndarray:
        """what: 0 pyramid level, 1 blurred level, 2 FAST candidates, 3 quadtree selection."""
        if what in (0, 1):
            w, h = ctypes.c_int(0), ctypes.c_int(0)
            check(self._lib.orbx_extractor_pyramid_level(self._h, level, None, 0, ctypes.byref(w),
                                                         ctypes.byref(h)), "level size")
            out = np.zeros((h.value, w.value), dtype=np.uint8)
            check(self._lib.orbx_extractor_debug_fetch(self._h, frame, level, what, ptr(out), out.size),
                  "debug_fetch")
            return out
        cap = 1 << 16
        while True:
            out = np.zeros(3 * cap, dtype=np.int32)
            rc = self._lib.orbx_extractor_debug_fetch(self._h, frame, level, what, ptr(out), out.size)
            if rc == _lib.ORBX_ERANGE:
                cap *= 4
                continue
            n = check(rc, "debug_fetch")
            return out[:3 * n].reshape(n, 3).copy()
