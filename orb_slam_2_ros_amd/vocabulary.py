"""Host mirror of ORB_SLAM2::ORBVocabulary = DBoW2::TemplatedVocabulary<FORB>
(Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h) over liborbx's vocabulary
(include/orbx.h).

Method names follow the reference: loadFromTextFile / loadFromBinFile
(:1351 / :1473), transform(features, levelsup) -> (BowVector, FeatureVector)
(:1140), empty(), size(), getBranchingFactor(), getDepthLevels(),
getScoringType(), getWeightingType().  BowVector is a dict word -> value
and FeatureVector a dict node -> [feature indices], both in ascending key
order like the reference's std::maps.  The descent runs on the GPU; there is
no host fallback.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import check, load, ptr

TEXT, BINARY = 0, 1
# DBoW2 enums (BowVector.h:36-53)
TF_IDF, TF, IDF, BINARY_W = 0, 1, 2, 3
L1_NORM, L2_NORM, CHI_SQUARE, KL, BHATTACHARYYA, DOT_PRODUCT = range(6)


class ORBVocabulary:
    """DBoW2::TemplatedVocabulary<FORB::TDescriptor, FORB> on liborbx."""

    def __init__(self, device: int = 0):
        self.device = int(device)
        self._h = ctypes.c_void_p()

    # --- construction -----------------------------------------------------
    @classmethod
    def from_arrays(cls, k, L, scoring, weighting, parent, is_leaf, desc, weight, device: int = 0):
        """The tree as the loaders build it (row 0 = root, ignored)."""
        v = cls(device)
        parent = np.ascontiguousarray(parent, np.int32)
        is_leaf = np.ascontiguousarray(is_leaf, np.uint8)
        desc = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        weight = np.ascontiguousarray(weight, np.float64)
        n = len(parent)
        if not (len(is_leaf) == n and len(desc) == n and len(weight) == n):
            raise ValueError("parent / is_leaf / desc / weight lengths differ")
        check(load().orbx_vocab_create(v.device, int(k), int(L), int(scoring), int(weighting), n, ptr(parent),
                                       ptr(is_leaf), ptr(desc), ptr(weight), ctypes.byref(v._h)),
              "orbx_vocab_create")
        return v

    def _load(self, path, fmt) -> bool:
        self._release()
        rc = load().orbx_vocab_load(self.device, str(path).encode(), fmt, ctypes.byref(self._h))
        if rc < 0:
            self._h = ctypes.c_void_p()
            return False   # the reference prints and returns false
        return True

    def loadFromTextFile(self, path) -> bool:
        return self._load(path, TEXT)

    def loadFromBinFile(self, path) -> bool:
        return self._load(path, BINARY)

    def _release(self):
        if self._h:
            load().orbx_vocab_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self._release()
        except Exception:
            pass

    # --- queries ------------------------------------------------------------
    def _info(self):
        if not self._h:
            raise RuntimeError("vocabulary not loaded")
        vals = [ctypes.c_int(0) for _ in range(6)]
        check(load().orbx_vocab_info(self._h, *[ctypes.byref(x) for x in vals]), "orbx_vocab_info")
        return [x.value for x in vals]

    def getBranchingFactor(self) -> int:
        return self._info()[0]

    def getDepthLevels(self) -> int:
        return self._info()[1]

    def getScoringType(self) -> int:
        return self._info()[2]

    def getWeightingType(self) -> int:
        return self._info()[3]

    def size(self) -> int:
        """Number of words."""
        return self._info()[5] if self._h else 0

    def empty(self) -> bool:
        return self.size() == 0

    def n_nodes(self) -> int:
        return self._info()[4]

    def export(self):
        """(parent, is_leaf, desc, weight) in file order."""
        n = self.n_nodes()
        parent = np.zeros(n, np.int32)
        leaf = np.zeros(n, np.uint8)
        desc = np.zeros((n, 32), np.uint8)
        weight = np.zeros(n, np.float64)
        check(load().orbx_vocab_export(self._h, ptr(parent), ptr(leaf), ptr(desc), ptr(weight), n),
              "orbx_vocab_export")
        return parent, leaf, desc, weight

    # --- transform ----------------------------------------------------------
    def transform_arrays(self, features: np.ndarray, levelsup: int = 4):
        """(bow_words u32, bow_values f64, fv_nodes u32, fv_offsets i32,
        fv_features i32): the BowVector and FeatureVector as ascending arrays
        (the FeatureVector in orbx_bow_side's node layout)."""
        if not self._h:
            return (np.zeros(0, np.uint32), np.zeros(0, np.float64), np.zeros(0, np.uint32),
                    np.zeros(1, np.int32), np.zeros(0, np.int32))
        f = np.ascontiguousarray(features, np.uint8).reshape(-1, 32)
        n = len(f)
        m = max(n, 1)
        bw = np.zeros(m, np.uint32)
        bv = np.zeros(m, np.float64)
        fn = np.zeros(m, np.uint32)
        fo = np.zeros(m + 1, np.int32)
        ff = np.zeros(m, np.int32)
        nb, nf = ctypes.c_int(0), ctypes.c_int(0)
        check(load().orbx_vocab_transform(self._h, ptr(f), n, int(levelsup), ptr(bw), ptr(bv), ctypes.byref(nb),
                                          ptr(fn), ptr(fo), ptr(ff), ctypes.byref(nf)), "orbx_vocab_transform")
        return bw[:nb.value], bv[:nb.value], fn[:nf.value], fo[:nf.value + 1], ff[:fo[nf.value]]

    def transform(self, features: np.ndarray, levelsup: int = 4):
        """TemplatedVocabulary::transform(features, BowVector&, FeatureVector&,
        levelsup) -> (BowVector dict, FeatureVector dict)."""
        bw, bv, fn, fo, ff = self.transform_arrays(features, levelsup)
        bow = {int(w): float(x) for w, x in zip(bw, bv)}
        fv = {int(fn[j]): [int(x) for x in ff[fo[j]:fo[j + 1]]] for j in range(len(fn))}
        return bow, fv

    def transform_device(self, d_desc: int, n: int, levelsup: int, d_word: int, d_weight: int, d_node: int,
                         stream: int | None = None):
        """Per-feature descent on device pointers (e.g. torch tensors'
        data_ptr()), stream-ordered."""
        check(load().orbx_vocab_transform_device(self._h, ctypes.c_void_p(d_desc), int(n), int(levelsup),
                                                 ctypes.c_void_p(d_word), ctypes.c_void_p(d_weight),
                                                 ctypes.c_void_p(d_node),
                                                 None if stream is None else ctypes.c_void_p(stream)),
              "orbx_vocab_transform_device")
