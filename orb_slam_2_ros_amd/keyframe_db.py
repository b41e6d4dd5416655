"""Host mirror of ORB_SLAM2::KeyFrameDatabase (KeyFrameDatabase.cc:31-236)
over liborbx's GPU keyframe database (include/orbx.h), and
the cross-stream keyframe exchange: every rank's new keyframes (BowVector,
keypoints, descriptors) are all-gathered over torch.distributed (RCCL on
GPUs, gloo on CPU), so each rank holds the same database of every stream's
keyframes and answers loop / relocalisation queries against all of them.

Keyframes are named by 64-bit ids (a multi-stream deployment makes them
unique across streams, e.g. stream << 40 | mnId).  BowVectors are ascending
(word, value) arrays as ORBVocabulary.transform_arrays returns them.
Covisibility -- KeyFrame::GetBestCovisibilityKeyFrames(10) -- is a callable
kf_id -> iterable of ids.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import COVIS_FN, KEYPOINT_DTYPE, check, load, ptr


def _bow(words, values):
    w = np.ascontiguousarray(words, np.uint32)
    v = np.ascontiguousarray(values, np.float64)
    if len(w) != len(v):
        raise ValueError("words / values lengths differ")
    return w, v


def _covis_cb(covis):
    def cb(_ctx, kf_id, out, cap):
        ids = list(covis(int(kf_id)))[:cap]
        for i, k in enumerate(ids):
            out[i] = int(k)
        return len(ids)
    return COVIS_FN(cb)


class KeyFrameDatabase:
    """KeyFrameDatabase: add / erase / clear / DetectLoopCandidates /
    DetectRelocalizationCandidates.  GPU only."""

    def __init__(self, device: int = 0):
        self._h = ctypes.c_void_p()
        check(load().orbx_kfdb_create(int(device), ctypes.byref(self._h)), "orbx_kfdb_create")
        self._out = np.empty(64, np.uint64)   # candidates (grown with the database, reused)
        self._cb_for = None                   # the last covisibility callable and its C callback
        self._cb = None
        self._n = ctypes.c_int(0)

    def __del__(self):
        try:
            if self._h:
                load().orbx_kfdb_destroy(self._h)
        except Exception:
            pass

    def add(self, kf_id: int, words, values):
        w, v = _bow(words, values)
        check(load().orbx_kfdb_add(self._h, int(kf_id), ptr(w), ptr(v), len(w)), "orbx_kfdb_add")

    def erase(self, kf_id: int):
        check(load().orbx_kfdb_erase(self._h, int(kf_id)), "orbx_kfdb_erase")

    def clear(self):
        check(load().orbx_kfdb_clear(self._h), "orbx_kfdb_clear")

    def size(self) -> int:
        return check(load().orbx_kfdb_size(self._h), "orbx_kfdb_size")

    def _detect(self, reloc, qid, words, values, connected, min_score, covis):
        w, v = _bow(words, values)
        conn = np.ascontiguousarray(sorted(connected or []), np.uint64)
        if covis is not self._cb_for:   # (one C callback per covisibility callable)
            self._cb_for, self._cb = covis, _covis_cb(covis)
        cb = self._cb
        cap = max(self.size(), 1)   # every live keyframe could be a candidate
        if len(self._out) < cap:
            self._out = np.empty(max(cap, 2 * len(self._out)), np.uint64)
        out, cap = self._out, len(self._out)
        n = self._n
        if reloc:
            rc = load().orbx_kfdb_detect_relocalization_candidates(self._h, int(qid), ptr(w), ptr(v), len(w), cb,
                                                                   None, ptr(out), cap, ctypes.byref(n))
        else:
            rc = load().orbx_kfdb_detect_loop_candidates(self._h, int(qid), ptr(w), ptr(v), len(w), ptr(conn),
                                                         len(conn), float(min_score), cb, None, ptr(out), cap,
                                                         ctypes.byref(n))
        check(rc, "DetectCandidates")
        return [int(x) for x in out[:n.value]]

    def DetectLoopCandidates(self, kf_id, words, values, connected, min_score, covis):
        return self._detect(False, kf_id, words, values, connected, min_score, covis)

    def DetectRelocalizationCandidates(self, frame_id, words, values, covis):
        return self._detect(True, frame_id, words, values, None, 0.0, covis)


def bow_score_l1(w1, v1, w2, v2) -> float:
    """L1Scoring::score (ScoringObject.cpp:23-66)."""
    a, b = _bow(w1, v1)
    c, d = _bow(w2, v2)
    out = ctypes.c_double(0)
    check(load().orbx_bow_score_l1(ptr(a), ptr(b), len(a), ptr(c), ptr(d), len(c), ctypes.byref(out)),
          "orbx_bow_score_l1")
    return out.value


# ---- cross-stream keyframe exchange ----------------------------------------
_HDR = np.dtype([("kf_id", "<u8"), ("n_words", "<i4"), ("n_kps", "<i4")])


def pack_keyframes(records) -> np.ndarray:
    """records: iterable of dicts (kf_id, words u32, values f64, keys
    KEYPOINT_DTYPE, desc (n, 32) u8) -> one u8 buffer."""
    parts = [np.array([len(records)], "<i8").view(np.uint8)]
    for r in records:
        w, v = _bow(r["words"], r["values"])
        k = np.ascontiguousarray(r.get("keys", np.zeros(0, KEYPOINT_DTYPE)), KEYPOINT_DTYPE)
        d = np.ascontiguousarray(r.get("desc", np.zeros((0, 32), np.uint8)), np.uint8).reshape(-1, 32)
        if len(d) != len(k):
            raise ValueError("keys / desc lengths differ")
        h = np.zeros(1, _HDR)
        h["kf_id"], h["n_words"], h["n_kps"] = r["kf_id"], len(w), len(k)
        parts += [h.view(np.uint8), w.view(np.uint8), v.view(np.uint8), k.view(np.uint8), d.reshape(-1)]
    return np.concatenate(parts)


def unpack_keyframes(buf: np.ndarray):
    buf = np.ascontiguousarray(buf, np.uint8)
    n = int(buf[:8].view("<i8")[0])
    off, out = 8, []
    for _ in range(n):
        h = buf[off:off + _HDR.itemsize].view(_HDR)[0]
        off += _HDR.itemsize
        nw, nk = int(h["n_words"]), int(h["n_kps"])
        w = buf[off:off + 4 * nw].view(np.uint32).copy(); off += 4 * nw
        v = buf[off:off + 8 * nw].view(np.float64).copy(); off += 8 * nw
        k = buf[off:off + 28 * nk].view(KEYPOINT_DTYPE).copy(); off += 28 * nk
        d = buf[off:off + 32 * nk].reshape(-1, 32).copy(); off += 32 * nk
        out.append({"kf_id": int(h["kf_id"]), "words": w, "values": v, "keys": k, "desc": d})
    return out


def all_gather_keyframes(records, dist, device=None):
    """Exchange this rank's new keyframes with every rank: returns all ranks'
    records, rank-major (rank 0's first), identical on every rank.  One
    all_gather of the buffer lengths, one of the padded buffers -- RCCL over
    xGMI when the process group is "nccl" (pass the rank's cuda device), gloo
    otherwise."""
    import torch
    buf = pack_keyframes(records)
    dev = torch.device("cpu") if device is None else torch.device(device)
    world = dist.get_world_size()
    ln = torch.tensor([len(buf)], dtype=torch.int64, device=dev)
    lens = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(lens, ln)
    sizes = [int(x.item()) for x in lens]
    m = max(sizes)
    mine = torch.zeros(m, dtype=torch.uint8, device=dev)
    mine[:len(buf)] = torch.from_numpy(buf).to(dev)
    allb = torch.zeros(world * m, dtype=torch.uint8, device=dev)
    dist.all_gather_into_tensor(allb, mine)
    allb = allb.cpu().numpy()
    out = []
    for r in range(world):
        out += unpack_keyframes(allb[r * m:r * m + sizes[r]])
    return out
