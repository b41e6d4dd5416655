"""ctypes binding of liborbx.so (the C ABI in include/orbx.h).

The library is built in-tree (``orb_slam_2_ros_amd/liborbx.so``) by
``__graft_entry__.build()`` / ``make -C orb_slam_2_ros_amd/csrc``.  There is no
fallback: if the library or a gfx950 device is missing, the calls raise.
"""
from __future__ import annotations

import ctypes
import os
import sys
from pathlib import Path

import numpy as np

LIB_PATH = Path(__file__).resolve().parent / "liborbx.so"

ORBX_OK = 0
ORBX_EIO = -5
ORBX_ENOMEM = -12
ORBX_EINVAL = -22
ORBX_ERANGE = -34
ORBX_ENODEV = -19

# cv::KeyPoint field order (orbx_keypoint, 28 bytes).
KEYPOINT_DTYPE = np.dtype([
    ("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
    ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4"),
])
assert KEYPOINT_DTYPE.itemsize == 28

# orbx_proj_query (36 bytes)
PROJ_QUERY_DTYPE = np.dtype([
    ("u", "<f4"), ("v", "<f4"), ("radius", "<f4"), ("ur", "<f4"), ("ur_tol", "<f4"),
    ("min_level", "<i4"), ("max_level", "<i4"), ("angle", "<f4"), ("flags", "<i4"),
])
assert PROJ_QUERY_DTYPE.itemsize == 36


class BowSide(ctypes.Structure):
    """orbx_bow_side"""
    _fields_ = [("keys", ctypes.c_void_p), ("desc", ctypes.c_void_p), ("flags", ctypes.c_void_p),
                ("n", ctypes.c_int), ("node_ids", ctypes.c_void_p), ("node_offsets", ctypes.c_void_p),
                ("node_features", ctypes.c_void_p), ("nnodes", ctypes.c_int)]


class MatchFrame(ctypes.Structure):
    """orbx_match_frame"""
    _fields_ = [("keys", ctypes.c_void_p), ("desc", ctypes.c_void_p), ("uright", ctypes.c_void_p),
                ("mp_state", ctypes.c_void_p), ("inv_sigma2", ctypes.c_void_p), ("n", ctypes.c_int),
                ("nlevels", ctypes.c_int), ("min_x", ctypes.c_float), ("max_x", ctypes.c_float),
                ("min_y", ctypes.c_float), ("max_y", ctypes.c_float)]


class ProjProblem(ctypes.Structure):
    """orbx_proj_problem"""
    _fields_ = [("frame", MatchFrame), ("queries", ctypes.c_void_p), ("qdesc", ctypes.c_void_p),
                ("nq", ctypes.c_int), ("q_idx", ctypes.c_void_p), ("q_dist", ctypes.c_void_p),
                ("kp_final", ctypes.c_void_p), ("nmatches", ctypes.c_int)]


class BowProblem(ctypes.Structure):
    """orbx_bow_problem"""
    _fields_ = [("a", BowSide), ("b", BowSide), ("tri", ctypes.c_void_p), ("match_a", ctypes.c_void_p),
                ("match_b", ctypes.c_void_p), ("nmatches", ctypes.c_int)]


class OrbxError(RuntimeError):
    def __init__(self, code: int, what: str):
        self.code = code
        msg = _strerror(code) if _LIB is not None else str(code)
        super().__init__(f"{what}: {msg} ({code})")


_LIB = None

P = ctypes.c_void_p
I32 = ctypes.c_int
I64 = ctypes.c_int64
F32 = ctypes.c_float
SZ = ctypes.c_size_t

_SIGNATURES = {
    "orbx_strerror": (ctypes.c_char_p, [I32]),
    "orbx_device_count": (I32, []),
    "orbx_debug_counter": (I32, [ctypes.c_char_p, P]),
    "orbx_extractor_create": (P, [I32, I32, F32, I32, I32, I32]),
    "orbx_extractor_destroy": (None, [P]),
    "orbx_extractor_get_levels": (I32, [P]),
    "orbx_extractor_get_scale_factor": (F32, [P]),
    "orbx_extractor_get_scale_table": (I32, [P, I32, P, I32]),
    "orbx_extractor_get_level_quotas": (I32, [P, P, I32]),
    "orbx_extract": (I32, [P, P, I32, I32, SZ, P, P, I32, P]),
    "orbx_extractor_pyramid_level": (I32, [P, I32, P, SZ, P, P]),
    "orbx_extractor_pyramid_host": (I32, [P, P, P, I32]),
    "orbx_extractor_reserve": (I32, [P, I32, I32, I32]),
    "orbx_extractor_kp_stride": (I32, [P]),
    "orbx_extract_batch_device": (I32, [P, P, I64, I32, I32, P]),
    "orbx_batch_results_device": (I32, [P, P, P, P]),
    "orbx_batch_pack_device": (I32, [P, P, I64, P, P]),
    "orbx_batch_download": (I32, [P, I32, P, P, I32, P]),
    "orbx_mono_step_device": (I32, [P, P, I64, I32, I32, I32, F32, I32, P]),
    "orbx_mono_matches_download": (I32, [P, I32, P, I32, P, P]),
    "orbx_extractor_split": (I32, [P, I32]),
    "orbx_extractor_pipeline": (I32, [P, I32]),
    "orbx_extractor_overlap_match": (I32, [P, I32]),
    "orbx_extractor_set_profiling": (I32, [P, I32]),
    "orbx_extractor_stage_times": (I32, [P, P, I32]),
    "orbx_extractor_debug_fetch": (I32, [P, I32, I32, I32, P, I64]),
    "orbx_compute_stereo_matches": (I32, [P, P, P, P, I32, P, P, I32, F32, F32, P, P, P]),
    "orbx_stereo_step_device": (I32, [P, P, I64, I32, I32, F32, F32, P]),
    "orbx_rgbd_step_device": (I32, [P, P, I64, I32, I32, P, I64, I32, F32, P]),
    "orbx_depth_download": (I32, [P, I32, P, P, I32, P, P]),
    "orbx_stereo_from_rgbd": (I32, [I32, P, P, I32, P, I32, I32, SZ, F32, P, P, P]),
    "orbx_search_by_projection": (I32, [I32, I32, P, P, P, I32, I32, F32, I32, P, P, P, P]),
    "orbx_search_by_projection_batch": (I32, [I32, I32, P, I32, I32, F32, I32]),
    "orbx_search_by_sim3": (I32, [I32, P, P, P, P, P, P, I32, P, P]),
    "orbx_search_by_bow_batch": (I32, [I32, I32, P, I32, F32, I32, I32]),
    "orbx_rotation_filter": (I32, [P, P, P, I32, P, P]),
    "orbx_search_by_bow": (I32, [I32, I32, P, P, F32, I32, P, I32, P, P, P]),
    "orbx_descriptor_distance": (I32, [P, P]),
    "orbx_search_for_initialization": (I32, [I32, P, P, I32, P, P, I32, I32, I32, P, P, I32, F32, I32, P]),
    "orbx_search_for_initialization_bounds": (I32, [I32, P, P, I32, P, P, I32, F32, F32, F32, F32, P, P, I32, F32,
                                                    I32, P]),
    "orbx_debug_trig": (I32, [I32, P, P, P, I32, P, P, P, I32]),
    "orbx_vocab_create": (I32, [I32, I32, I32, I32, I32, I32, P, P, P, P, P]),
    "orbx_vocab_load": (I32, [I32, ctypes.c_char_p, I32, P]),
    "orbx_vocab_destroy": (None, [P]),
    "orbx_vocab_info": (I32, [P, P, P, P, P, P, P]),
    "orbx_vocab_export": (I32, [P, P, P, P, P, I32]),
    "orbx_vocab_transform": (I32, [P, P, I32, I32, P, P, P, P, P, P, P]),
    "orbx_vocab_transform_device": (I32, [P, P, I32, I32, P, P, P, P]),
    "orbx_distinctive_descriptors": (I32, [I32, P, P, I32, P]),
    "orbx_distinctive_descriptors_device": (I32, [P, P, I32, P, P]),
    "orbx_undistort_keypoints": (I32, [I32, P, I32, P, P, I32, P]),
    "orbx_undistort_points_device": (I32, [P, I32, P, P, I32, P, P]),
    "orbx_cvt_gray": (I32, [I32, P, I32, I32, SZ, I32, I32, P, SZ]),
    "orbx_cvt_gray_device": (I32, [P, I64, I32, I32, I32, I32, I32, I32, P, I64, I32, P]),
    "orbx_depth_to_float_device": (I32, [P, I64, I32, I32, I32, I32, F32, P, I64, I32, P]),
    "orbx_kfdb_create": (I32, [I32, P]),
    "orbx_kfdb_destroy": (None, [P]),
    "orbx_kfdb_add": (I32, [P, ctypes.c_uint64, P, P, I32]),
    "orbx_kfdb_erase": (I32, [P, ctypes.c_uint64]),
    "orbx_kfdb_clear": (I32, [P]),
    "orbx_kfdb_size": (I32, [P]),
    "orbx_kfdb_detect_loop_candidates": (I32, [P, ctypes.c_uint64, P, P, I32, P, I32, F32, P, P, P, I32, P]),
    "orbx_kfdb_detect_relocalization_candidates": (I32, [P, ctypes.c_uint64, P, P, I32, P, P, P, I32, P]),
    "orbx_bow_score_l1": (I32, [P, P, I32, P, P, I32, P]),
    "orbx_local_ba": (I32, [I32, P, P, I32, P, I32, P, I32, I32, I32, P, P, P, P]),
    "orbx_local_ba_fast": (I32, [I32, P, P, I32, P, I32, P, I32, I32, I32, P, P, P, P]),
    "orbx_ba_debug_step": (I32, [I32, P, P, I32, P, I32, P, I32, I32, ctypes.c_double, P, P, P]),
}

# orbx_covis_fn
COVIS_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64),
                            ctypes.c_int)

EXPORTED = tuple(_SIGNATURES)


def load(path: os.PathLike | str | None = None) -> ctypes.CDLL:
    """Load liborbx.so once; raises OSError if it has not been built."""
    global _LIB
    if _LIB is not None and path is None:
        return _LIB
    # ORBX_LIB: an alternative build of the same ABI (the phase-profiling
    # diagnostic build, tools/phase_prof.py); never set by tests or the bench
    p = Path(path) if path is not None else Path(os.environ.get("ORBX_LIB", LIB_PATH))
    if not p.exists():
        raise OSError(f"{p} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
    # torch-ROCm bundles its own libamdhip64.so.7 (same SONAME as /opt/rocm's).
    # Loading torch first makes liborbx bind to that one copy, so a process that
    # uses both has a single HIP runtime (the other order leaves torch without
    # devices).  Without torch, liborbx uses /opt/rocm's runtime via its RUNPATH.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(str(p))
    # ORBX_LIB_ALLOW_MISSING=1 (A/B timing of an older build that predates an
    # entry point): skip the missing symbols, listed on stderr.  Otherwise a
    # stale or mismatched library fails here, with the ABI names it lacks.
    allow = os.environ.get("ORBX_LIB_ALLOW_MISSING") == "1"
    missing = [name for name in _SIGNATURES if not hasattr(lib, name)]
    if missing and not allow:
        raise OSError(f"{p}: missing entry points {missing} (stale or mismatched build; "
                      "ORBX_LIB_ALLOW_MISSING=1 skips them for A/B timing)")
    if missing:
        print(f"orbx: {p} lacks {missing}; skipped (ORBX_LIB_ALLOW_MISSING=1)", file=sys.stderr)
    for name, (res, args) in _SIGNATURES.items():
        if name in missing:
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _LIB = lib
    return lib


def _strerror(code: int) -> str:
    s = load().orbx_strerror(code)
    return s.decode() if s else str(code)


def check(code: int, what: str) -> int:
    if code < 0:
        raise OrbxError(code, what)
    return code


def ptr(a: np.ndarray | None) -> int | None:
    """The array's data address (an int: ctypes passes it as void*)."""
    if a is None:
        return None
    return a.__array_interface__["data"][0]


def debug_counter(name: str) -> int:
    """orbx_debug_counter: a diagnostic of this thread's last host call (tests)."""
    v = ctypes.c_int64(0)
    check(load().orbx_debug_counter(name.encode(), ctypes.byref(v)), f"orbx_debug_counter({name})")
    return v.value
