"""Host mirror of Optimizer::LocalBundleAdjustment (Optimizer.cc:517-900)
over liborbx's GPU bundle adjustment (include/orbx.h).  The
caller collects the graph (local keyframes, fixed cameras, local map points
and their observations) exactly as the reference does; this runs the two LM
passes and returns the optimised poses and points and the observations to
erase.  GPU only."""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import check, load, ptr
from .synth_ba import BA_EDGE_DTYPE


def local_bundle_adjustment(Tcw, fixed, Xw, edges, iters=(5, 10), device: int = 0, fast: bool = False):
    """Tcw (ncam, 3, 4) f32, fixed (ncam,) bool, Xw (npt, 3) f32, edges
    BA_EDGE_DTYPE.  Returns (Tcw_out, Xw_out, outlier (ne,) bool,
    (iterations pass 1, pass 2)).  fast: orbx_local_ba_fast (the sums as
    parallel reductions; equal to the ordered mode to rounding)."""
    T = np.ascontiguousarray(Tcw, np.float32).reshape(-1, 3, 4)
    F = np.ascontiguousarray(fixed, np.uint8)
    X = np.ascontiguousarray(Xw, np.float32).reshape(-1, 3)
    E = np.ascontiguousarray(edges, BA_EDGE_DTYPE)
    To, Xo = np.empty_like(T), np.empty_like(X)
    out = np.zeros(max(len(E), 1), np.uint8)
    its = np.zeros(2, np.int32)
    fn = load().orbx_local_ba_fast if fast else load().orbx_local_ba
    check(fn(device, ptr(T), ptr(F), len(T), ptr(X), len(X), ptr(E), len(E), int(iters[0]),
             int(iters[1]), ptr(To), ptr(Xo), ptr(out), ptr(its)), "orbx_local_ba")
    return To, Xo, out[:len(E)].astype(bool), (int(its[0]), int(its[1]))


def debug_step(Tcw, fixed, Xw, edges, robust=True, lam=1e-3, device: int = 0):
    """One LM linear system of the first pass (test hook): (x, chi2, solved)."""
    T = np.ascontiguousarray(Tcw, np.float32).reshape(-1, 3, 4)
    F = np.ascontiguousarray(fixed, np.uint8)
    X = np.ascontiguousarray(Xw, np.float32).reshape(-1, 3)
    E = np.ascontiguousarray(edges, BA_EDGE_DTYPE)
    n = 6 * int((F == 0).sum()) + 3 * len(X)
    x = np.zeros(max(n, 1), np.float64)
    chi2 = ctypes.c_double(0)
    ok = ctypes.c_int(0)
    check(load().orbx_ba_debug_step(device, ptr(T), ptr(F), len(T), ptr(X), len(X), ptr(E), len(E), int(robust),
                                    float(lam), ptr(x), ctypes.byref(chi2), ctypes.byref(ok)), "orbx_ba_debug_step")
    return x[:n], chi2.value, bool(ok.value)
