"""Synthetic local bundle-adjustment problems:
KITTI-like stereo keyframes along a forward trajectory, map points in front
of them, mono and stereo observations with octave-scaled pixel noise and a
few gross outliers; the estimates start perturbed from the truth."""
from __future__ import annotations

import numpy as np

BA_EDGE_DTYPE = np.dtype([("cam", "<i4"), ("point", "<i4"), ("u", "<f4"), ("v", "<f4"), ("ur", "<f4"),
                          ("inv_sigma2", "<f4"), ("fx", "<f4"), ("fy", "<f4"), ("cx", "<f4"), ("cy", "<f4"),
                          ("bf", "<f4")])
assert BA_EDGE_DTYPE.itemsize == 44


def _rot(axis_angle):
    a = np.asarray(axis_angle, np.float64)
    th = np.linalg.norm(a)
    if th < 1e-12:
        return np.eye(3)
    k = a / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K


def make_ba_problem(n_local=10, n_fixed=4, n_points=1500, seed=0, stereo_frac=0.5, outlier_frac=0.03,
                    w=1241, h=376, fx=718.856, fy=718.856, cx=607.1928, cy=185.2157, bf=386.1448,
                    pose_noise=(0.004, 0.05), point_noise=0.05):
    """Returns dict: Tcw (ncam, 3, 4) f32 (perturbed), fixed u8, Xw (npt, 3)
    f32 (perturbed), edges BA_EDGE_DTYPE, and the truth (Tcw_true, Xw_true)."""
    rng = np.random.default_rng(seed)
    ncam = n_local + n_fixed
    sf = 1.2 ** np.arange(8)
    inv_sigma2 = (1.0 / (sf * sf)).astype(np.float32)
    Tt = []
    for c in range(ncam):                       # fixed cameras first along the path, then the local ones
        Rwc = _rot([0, 0.02 * c + rng.normal(0, 0.01), 0])
        twc = np.array([0.1 * rng.normal(), 0.05 * rng.normal(), 1.0 * c])
        Rcw = Rwc.T
        Tt.append(np.hstack([Rcw, (-Rcw @ twc)[:, None]]))
    Tt = np.array(Tt)
    Xt = np.stack([rng.uniform(-15, 15, n_points), rng.uniform(-3, 3, n_points),
                   rng.uniform(6, 45, n_points) + ncam * rng.random(n_points)], 1)
    edges = []
    for p in range(n_points):
        for c in range(ncam):
            Xc = Tt[c, :, :3] @ Xt[p] + Tt[c, :, 3]
            if Xc[2] <= 0.5:
                continue
            u, v = fx * Xc[0] / Xc[2] + cx, fy * Xc[1] / Xc[2] + cy
            if not (0 <= u < w and 0 <= v < h) or rng.random() < 0.3:
                continue
            oct_ = int(rng.choice(8, p=[0.3, 0.2, 0.15, 0.12, 0.09, 0.07, 0.04, 0.03]))
            s = sf[oct_]
            un, vn = u + rng.normal(0, s), v + rng.normal(0, s)
            ur = -1.0
            if rng.random() < stereo_frac:
                ur = u - bf / Xc[2] + rng.normal(0, s)
            if rng.random() < outlier_frac:
                un += rng.choice([-1, 1]) * rng.uniform(15, 60)
            edges.append((c, p, un, vn, ur, inv_sigma2[oct_], fx, fy, cx, cy, bf))
    E = np.array(edges, BA_EDGE_DTYPE)
    fixed = np.zeros(ncam, np.uint8)
    fixed[:n_fixed] = 1
    fixed[n_fixed] = 1                          # the first local keyframe plays mnId == 0
    T = Tt.copy()
    for c in range(ncam):
        if fixed[c]:
            continue
        dR = _rot(rng.normal(0, pose_noise[0], 3))
        T[c, :, :3] = dR @ T[c, :, :3]
        T[c, :, 3] = dR @ T[c, :, 3] + rng.normal(0, pose_noise[1], 3)
    X = Xt + rng.normal(0, point_noise, Xt.shape)
    return {"Tcw": T.astype(np.float32), "fixed": fixed, "Xw": X.astype(np.float32), "edges": E,
            "Tcw_true": Tt, "Xw_true": Xt}
