"""Host mirror of ``ORB_SLAM2::ORBmatcher`` (and the Frame data it reads).

Reference interface: orb_slam2/include/ORBmatcher.h:36-106,
orb_slam2/src/ORBmatcher.cc:37-43 (constants, constructor), :406-521
(SearchForInitialization), :1649-1665 (DescriptorDistance).

``Frame`` carries what the matcher reads from ORB_SLAM2::Frame: the undistorted
keypoints (mvKeysUn; distortion-free cameras, so equal to mvKeys), the
descriptors (mDescriptors) and the image bounds that size the 64x48 grid
(Frame.cc:218-220).  SearchForInitialization runs on the GPU through
liborbx.so; DescriptorDistance is a host popcount (no device round trip).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import KEYPOINT_DTYPE, PROJ_QUERY_DTYPE, BowProblem, BowSide, MatchFrame, ProjProblem, check, load, ptr

# orbx_search_by_projection variants (include/orbx.h)
PROJ_VARIANTS = {"localmap": 0, "lastframe": 1, "keyframe": 2, "sim3": 3, "fuse": 4, "fuse_sim3": 5}
# orbx_search_by_bow variants
BOW_VARIANTS = {"kf_frame": 0, "kf_kf": 1, "triangulation": 2}


class Frame:
    """bounds: (mnMinX, mnMaxX, mnMinY, mnMaxY) as Frame::ComputeImageBounds
    leaves them (Frame.cc:475-499); None = an undistorted camera's
    (0, width, 0, height)."""

    def __init__(self, keypoints: np.ndarray, descriptors: np.ndarray, width: int, height: int, bounds=None):
        self.mvKeysUn = np.ascontiguousarray(keypoints, dtype=KEYPOINT_DTYPE)
        self.mvKeys = self.mvKeysUn
        self.mDescriptors = np.ascontiguousarray(descriptors, dtype=np.uint8).reshape(-1, 32)
        if len(self.mvKeysUn) != len(self.mDescriptors):
            raise ValueError("keypoints and descriptors differ in length")
        self.N = len(self.mvKeysUn)
        self.width, self.height = int(width), int(height)
        b = (0.0, float(width), 0.0, float(height)) if bounds is None else tuple(float(v) for v in bounds)
        self.mnMinX, self.mnMaxX, self.mnMinY, self.mnMaxY = (float(np.float32(v)) for v in b)


class ORBmatcher:
    TH_HIGH = 100
    TH_LOW = 50
    HISTO_LENGTH = 30

    def __init__(self, nnratio: float = 0.6, checkOri: bool = True, device: int = 0):
        self._lib = _lib.load()
        self.mfNNratio = float(nnratio)
        self.mbCheckOrientation = bool(checkOri)
        self.device = device

    @staticmethod
    def DescriptorDistance(a: np.ndarray, b: np.ndarray) -> int:
        a = np.ascontiguousarray(a, dtype=np.uint8).reshape(32)
        b = np.ascontiguousarray(b, dtype=np.uint8).reshape(32)
        return int(_lib.load().orbx_descriptor_distance(ptr(a), ptr(b)))

    def SearchForInitialization(self, F1: Frame, F2: Frame, vbPrevMatched: np.ndarray,
                                windowSize: int = 10):
        """Returns (nmatches, vnMatches12); vbPrevMatched (N1 x 2 float32) is
        updated in place like the reference's vector<cv::Point2f>&."""
        if vbPrevMatched.dtype != np.float32 or vbPrevMatched.shape != (F1.N, 2) or \
                not vbPrevMatched.flags.c_contiguous:
            raise ValueError("vbPrevMatched must be a C-contiguous (N1, 2) float32 array")
        m12 = np.full(max(F1.N, 1), -1, dtype=np.int32)
        nm = ctypes.c_int(0)
        # the grid is F2's (the reference's bounds are static Frame members)
        check(self._lib.orbx_search_for_initialization_bounds(
            self.device, ptr(F1.mvKeysUn), ptr(F1.mDescriptors), F1.N,
            ptr(F2.mvKeysUn), ptr(F2.mDescriptors), F2.N, ctypes.c_float(F2.mnMinX), ctypes.c_float(F2.mnMaxX),
            ctypes.c_float(F2.mnMinY), ctypes.c_float(F2.mnMaxY),
            ptr(vbPrevMatched), ptr(m12), int(windowSize), ctypes.c_float(self.mfNNratio),
            int(self.mbCheckOrientation), ctypes.byref(nm)), "SearchForInitialization")
        return nm.value, m12[:F1.N].copy()

    # -- projection searches (ORBmatcher.cc:45-129, 291-404, 827-1102, 1330-1601) --
    def search_by_projection(self, variant, keys, desc, queries, qdesc, bounds, uright=None, mp_state=None,
                             inv_sigma2=None, th_dist=None):
        """One of SearchByProjection x4 / Fuse x2 (search part) on a query table
        (PROJ_QUERY_DTYPE rows in the reference's loop order; the caller
        projects its map points).  variant: "localmap" (Frame&, vector<MapPoint*>&),
        "lastframe" (Frame&, const Frame&), "keyframe" (Frame&, KeyFrame*, set),
        "sim3" (KeyFrame*, Scw, ...), "fuse", "fuse_sim3".  th_dist defaults to
        the reference's constant (TH_HIGH for localmap/lastframe, TH_LOW else).
        Returns (nmatches, q_idx, q_dist, kp_final), see include/orbx.h."""
        v = PROJ_VARIANTS[variant] if isinstance(variant, str) else int(variant)
        if th_dist is None:
            th_dist = self.TH_HIGH if v in (0, 1) else self.TH_LOW
        keys = np.ascontiguousarray(keys, KEYPOINT_DTYPE)
        desc = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        q = np.ascontiguousarray(queries, PROJ_QUERY_DTYPE)
        qd = np.ascontiguousarray(qdesc, np.uint8).reshape(-1, 32)
        if len(keys) != len(desc) or len(q) != len(qd):
            raise ValueError("rows of keys/desc or queries/qdesc differ")
        ur = None if uright is None else np.ascontiguousarray(uright, np.float32)
        ms = None if mp_state is None else np.ascontiguousarray(mp_state, np.uint8)
        isg = None if inv_sigma2 is None else np.ascontiguousarray(inv_sigma2, np.float32)
        f = MatchFrame(ptr(keys), ptr(desc), ptr(ur), ptr(ms), ptr(isg), len(keys),
                       0 if isg is None else len(isg), *[float(b) for b in bounds])
        qi = np.full(max(len(q), 1), -1, np.int32)
        qdist = np.full(max(len(q), 1), -1, np.int32)
        kf = np.full(max(len(keys), 1), -1, np.int32)
        nm = ctypes.c_int(0)
        check(self._lib.orbx_search_by_projection(self.device, v, ctypes.byref(f), ptr(q), ptr(qd), len(q),
                                                  int(th_dist), ctypes.c_float(self.mfNNratio),
                                                  int(self.mbCheckOrientation), ptr(qi), ptr(qdist), ptr(kf),
                                                  ctypes.byref(nm)), "SearchByProjection")
        return nm.value, qi[:len(q)].copy(), qdist[:len(q)].copy(), kf[:len(keys)].copy()

    def search_by_projection_batch(self, variant, problems, th_dist=None):
        """Several search_by_projection calls of one variant in one launch pair
        (orbx_search_by_projection_batch): Fuse over a keyframe's neighbours
        (LocalMapping.cc:537), relocalisation's SearchByProjection over the
        candidates (Tracking.cc:1667).  problems: dicts with the keyword
        arguments of search_by_projection (keys, desc, queries, qdesc, bounds,
        uright, mp_state, inv_sigma2); arrays that are the same object are
        uploaded once.  Returns one (nmatches, q_idx, q_dist, kp_final) per problem."""
        v = PROJ_VARIANTS[variant] if isinstance(variant, str) else int(variant)
        if th_dist is None:
            th_dist = self.TH_HIGH if v in (0, 1) else self.TH_LOW
        arr = (ProjProblem * max(len(problems), 1))()
        keep, outs, conv = [], [], {}

        def c(a, dt, shape=None):   # same source object -> same converted array (uploaded once)
            if a is None:
                return None
            key = (id(a), dt)
            if key not in conv:
                x = np.ascontiguousarray(a, dt)
                conv[key] = (a, x.reshape(shape) if shape else x)
            return conv[key][1]
        for k, P in enumerate(problems):
            keys = c(P["keys"], KEYPOINT_DTYPE)
            desc = c(P["desc"], np.uint8, (-1, 32))
            q = c(P["queries"], PROJ_QUERY_DTYPE)
            qd = c(P["qdesc"], np.uint8, (-1, 32))
            if len(keys) != len(desc) or len(q) != len(qd):
                raise ValueError("rows of keys/desc or queries/qdesc differ")
            ur, ms, isg = c(P.get("uright"), np.float32), c(P.get("mp_state"), np.uint8), c(P.get("inv_sigma2"), np.float32)
            qi = np.full(max(len(q), 1), -1, np.int32)
            qdist = np.full(max(len(q), 1), -1, np.int32)
            kf = np.full(max(len(keys), 1), -1, np.int32)
            keep.extend([keys, desc, q, qd, ur, ms, isg])
            outs.append((qi, qdist, kf, len(q), len(keys)))
            f = MatchFrame(ptr(keys), ptr(desc), ptr(ur), ptr(ms), ptr(isg), len(keys),
                           0 if isg is None else len(isg), *[float(b) for b in P["bounds"]])
            arr[k] = ProjProblem(f, ptr(q), ptr(qd), len(q), ptr(qi), ptr(qdist), ptr(kf), 0)
        check(self._lib.orbx_search_by_projection_batch(self.device, v, arr, len(problems), int(th_dist),
                                                        ctypes.c_float(self.mfNNratio), int(self.mbCheckOrientation)),
              "SearchByProjection batch")
        return [(arr[k].nmatches, qi[:nq].copy(), qd[:nq].copy(), kf[:n].copy())
                for k, (qi, qd, kf, nq, n) in enumerate(outs)]

    # -- vocabulary-node searches (ORBmatcher.cc:160-289, 524-657, 659-825) --
    _BOW_FIELDS = (("keys", KEYPOINT_DTYPE), ("desc", np.uint8), ("flags", np.uint8), ("ids", np.uint32),
                   ("off", np.int32), ("feat", np.int32))
    _side_cache: list = []   # (source arrays, BowSide): sides whose arrays went in unconverted

    @classmethod
    def _bow_side(cls, S, keep):
        src = tuple(S[f] for f, _ in cls._BOW_FIELDS)
        for c_src, side in cls._side_cache:   # the same array objects as a recent call: same addresses
            if all(a is b for a, b in zip(c_src, src)) and side.n == len(src[0]) and side.nnodes == len(src[3]):
                keep.append(c_src)
                return side
        arrs = tuple(np.ascontiguousarray(a, dt) for a, (_, dt) in zip(src, cls._BOW_FIELDS))
        keep.append(arrs)
        k, d, f, i, o, e = arrs
        side = BowSide(ptr(k), ptr(d), ptr(f), len(k), ptr(i), ptr(o), ptr(e), len(i))
        if all(a is b for a, b in zip(arrs, src)):   # (a converted copy could go stale: not cached)
            cls._side_cache = ([(src, side)] + cls._side_cache)[:8]
        return side

    def search_by_bow_batch(self, variant, problems, nlevels=8):
        """Several search_by_bow calls of one variant in one launch pair
        (orbx_search_by_bow_batch), e.g. SearchForTriangulation of a new
        keyframe against its covisible neighbours (LocalMapping.cc:276-315).
        problems: dicts with A, B (as search_by_bow) and tri.  A side dict that
        is the same object in several problems is uploaded once.  Returns one
        (nmatches, match_a, match_b) per problem."""
        v = BOW_VARIANTS[variant] if isinstance(variant, str) else int(variant)
        arr = (BowProblem * max(len(problems), 1))()
        keep, outs, sides = [], [], {}
        for k, P in enumerate(problems):
            for S in (P["A"], P["B"]):
                if id(S) not in sides:
                    sides[id(S)] = (S, self._bow_side(S, keep), len(keep) - 1)
            sa, ia = sides[id(P["A"])][1:]
            sb, ib = sides[id(P["B"])][1:]
            na, nb = len(keep[ia][0]), len(keep[ib][0])
            t = None if P.get("tri") is None else np.ascontiguousarray(P["tri"], np.float32)
            ma = np.full(max(na, 1), -1, np.int32)
            mb = np.full(max(nb, 1), -1, np.int32)
            keep.append((t,))
            outs.append((ma, mb, na, nb))
            arr[k] = BowProblem(sa, sb, ptr(t), ptr(ma), ptr(mb), 0)
        check(self._lib.orbx_search_by_bow_batch(self.device, v, arr, len(problems), ctypes.c_float(self.mfNNratio),
                                                 int(self.mbCheckOrientation), int(nlevels)), "SearchByBoW batch")
        return [(arr[k].nmatches, ma[:na].copy(), mb[:nb].copy()) for k, (ma, mb, na, nb) in enumerate(outs)]

    @staticmethod
    def rotation_filter(ka, kb, match_a, exclude=None):
        """orbx_rotation_filter: the reference's rotation-consistency pass over
        the pairs (i, match_a[i]), skipping A features flagged in exclude.
        Returns (nmatches, filtered match_a)."""
        ka = np.ascontiguousarray(ka, KEYPOINT_DTYPE)
        kb = np.ascontiguousarray(kb, KEYPOINT_DTYPE)
        m = np.array(match_a, np.int32, copy=True)
        ex = None if exclude is None else np.ascontiguousarray(exclude, np.uint8)
        nm = ctypes.c_int(0)
        check(load().orbx_rotation_filter(ptr(ka), ptr(kb), ptr(m), len(m), ptr(ex), ctypes.byref(nm)),
              "rotation filter")
        return nm.value, m
    def search_by_bow(self, variant, A, B, tri=None, nlevels=8):
        """SearchByBoW(KF, F) ("kf_frame"), SearchByBoW(KF1, KF2) ("kf_kf") or
        SearchForTriangulation ("triangulation").  A, B: dicts with keys, desc,
        flags (see include/orbx.h), ids / off / feat (the FeatureVector as CSR).
        tri: F12[9], ex, ey, B's scale factors and sigma2 (triangulation).
        Returns (nmatches, match_a, match_b)."""
        v = BOW_VARIANTS[variant] if isinstance(variant, str) else int(variant)
        keep = []
        sa, sb = self._bow_side(A, keep), self._bow_side(B, keep)
        t = None if tri is None else np.ascontiguousarray(tri, np.float32)
        na, nb = len(keep[0][0]), len(keep[1][0])
        ma = np.full(max(na, 1), -1, np.int32)
        mb = np.full(max(nb, 1), -1, np.int32)
        nm = ctypes.c_int(0)
        check(self._lib.orbx_search_by_bow(self.device, v, ctypes.byref(sa), ctypes.byref(sb),
                                           ctypes.c_float(self.mfNNratio), int(self.mbCheckOrientation), ptr(t),
                                           int(nlevels), ptr(ma), ptr(mb), ctypes.byref(nm)), "SearchByBoW")
        return nm.value, ma[:na].copy(), mb[:nb].copy()

    def search_by_sim3(self, kf1, kf2, q1, qdesc1, q2, qdesc2, th_dist=None):
        """SearchBySim3 (ORBmatcher.cc:1104-1328) on per-slot query tables.
        kf1 / kf2: dicts with keys, desc, bounds.  Returns (nfound, matches12)."""
        th_dist = self.TH_HIGH if th_dist is None else th_dist
        arrs = []

        def frame(K):
            k = np.ascontiguousarray(K["keys"], KEYPOINT_DTYPE)
            d = np.ascontiguousarray(K["desc"], np.uint8).reshape(-1, 32)
            arrs.extend([k, d])
            return MatchFrame(ptr(k), ptr(d), None, None, None, len(k), 0, *[float(b) for b in K["bounds"]])
        f1, f2 = frame(kf1), frame(kf2)
        a1 = np.ascontiguousarray(q1, PROJ_QUERY_DTYPE); a2 = np.ascontiguousarray(q2, PROJ_QUERY_DTYPE)
        b1 = np.ascontiguousarray(qdesc1, np.uint8).reshape(-1, 32)
        b2 = np.ascontiguousarray(qdesc2, np.uint8).reshape(-1, 32)
        if len(a1) != f1.n or len(a2) != f2.n:
            raise ValueError("one query row per keyframe map-point slot")
        m = np.full(max(f1.n, 1), -1, np.int32)
        nf = ctypes.c_int(0)
        check(self._lib.orbx_search_by_sim3(self.device, ctypes.byref(f1), ctypes.byref(f2), ptr(a1), ptr(b1),
                                            ptr(a2), ptr(b2), int(th_dist), ptr(m), ctypes.byref(nf)),
              "SearchBySim3")
        return nf.value, m[:f1.n].copy()
