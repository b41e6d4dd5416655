"""Seeded synthetic inputs for the ORBmatcher searches (tests and bench.py).

Projection searches (SearchByProjection x4, Fuse x2, SearchBySim3): a frame's
keypoints / descriptors / mvuRight / map-point state and a query table of
projected map points.  Most queries are perturbed copies of a keypoint (a true
match nearby, descriptor with bit noise, similar angle); the rest are random.
Duplicated descriptors force exact distance ties, and already-assigned
keypoints, non-blocking (Observations() == 0) points, stereo and off-grid
projections exercise every skip rule.

Vocabulary searches (SearchByBoW x2, SearchForTriangulation): two views with
FeatureVectors over a shared pool of vocabulary nodes; a fraction of B's
features are noisy copies of A's in the same node, and for triangulation the
copies sit near their epipolar line under a synthetic F12.
"""

import numpy as np

from ._lib import KEYPOINT_DTYPE, PROJ_QUERY_DTYPE
from .synth import scale_tables


def make_proj_case(seed, variant, n=1500, nq=1200, w=640, h=480, stereo=False, th=1.0):
    rng = np.random.default_rng(seed)
    sf, _ = scale_tables(1.2, 8)
    inv_sigma2 = (np.float32(1) / (sf * sf)).astype(np.float32)
    keys = np.zeros(n, KEYPOINT_DTYPE)
    keys["octave"] = rng.choice(8, n, p=[0.25, 0.2, 0.15, 0.12, 0.1, 0.08, 0.06, 0.04])
    keys["x"] = rng.uniform(-3, w + 3, n).astype(np.float32)
    keys["y"] = rng.uniform(-3, h + 3, n).astype(np.float32)
    keys["angle"] = rng.uniform(0, 360, n).astype(np.float32)
    keys["size"] = 31
    keys["class_id"] = -1
    desc = rng.integers(0, 256, (n, 32)).astype(np.uint8)
    dup = rng.integers(0, n, n // 20)
    desc[dup] = desc[rng.integers(0, n, len(dup))]        # exact ties
    uright = None
    if stereo:
        uright = np.full(n, -1.0, np.float32)
        st = rng.random(n) < 0.6
        uright[st] = (keys["x"][st] - rng.uniform(2, 40, st.sum())).astype(np.float32)
        uright[rng.random(n) < 0.05] = 0.0                 # mvuRight == 0: '>0' vs '>=0' rules differ
    mp_state = np.zeros(n, np.uint8)
    occ = rng.random(n) < 0.12
    mp_state[occ] = 1 | (2 * (rng.random(occ.sum()) < 0.5)).astype(np.uint8)

    q = np.zeros(nq, PROJ_QUERY_DTYPE)
    qdesc = rng.integers(0, 256, (nq, 32)).astype(np.uint8)
    true_kp = rng.integers(0, n, nq)
    real = rng.random(nq) < 0.75
    lvl = np.where(real, keys["octave"][true_kp], rng.integers(0, 8, nq)).astype(np.int32)
    jitter = rng.normal(0, 1.5, (nq, 2)).astype(np.float32)
    q["u"] = np.where(real, keys["x"][true_kp] + jitter[:, 0], rng.uniform(-20, w + 20, nq)).astype(np.float32)
    q["v"] = np.where(real, keys["y"][true_kp] + jitter[:, 1], rng.uniform(-20, h + 20, nq)).astype(np.float32)
    nbits = rng.integers(0, 60, nq)
    for i in np.nonzero(real)[0]:
        d = desc[true_kp[i]].copy()
        bits = rng.choice(256, nbits[i], replace=False)
        for b in bits:
            d[b >> 3] ^= np.uint8(1 << (b & 7))
        qdesc[i] = d
    q["angle"] = np.where(real, keys["angle"][true_kp] + rng.normal(0, 8, nq),
                          rng.uniform(0, 360, nq)).astype(np.float32) % np.float32(360)
    if variant == "localmap":
        view = rng.random(nq) < 0.5
        r = np.where(view, np.float32(2.5), np.float32(4.0)).astype(np.float32)
        if th != 1.0:
            r = (r * np.float32(th)).astype(np.float32)
        q["radius"] = (r * sf[lvl]).astype(np.float32)
        q["min_level"], q["max_level"] = lvl - 1, lvl
        q["ur_tol"] = q["radius"]
    elif variant == "lastframe":
        q["radius"] = (np.float32(th) * sf[lvl]).astype(np.float32)
        mode = rng.integers(0, 3, nq)          # forward / backward / neither (ORBmatcher.cc:1382-1389)
        q["min_level"] = np.where(mode == 0, lvl, np.where(mode == 1, 0, lvl - 1))
        q["max_level"] = np.where(mode == 0, -1, np.where(mode == 1, lvl, lvl + 1))
        q["ur_tol"] = q["radius"]
    elif variant == "keyframe":
        q["radius"] = (np.float32(th) * sf[lvl]).astype(np.float32)
        q["min_level"], q["max_level"] = lvl - 1, lvl + 1
    else:                                      # sim3, fuse, fuse_sim3: KeyFrame window + level filter
        q["radius"] = (np.float32(th) * sf[lvl]).astype(np.float32)
        q["min_level"], q["max_level"] = lvl - 1, lvl
    disp = rng.uniform(2, 40, nq).astype(np.float32)
    q["ur"] = (q["u"] - disp).astype(np.float32)
    q["flags"] = (rng.random(nq) < 0.9).astype(np.int32) | (2 * (rng.random(nq) < 0.8)).astype(np.int32)
    return dict(keys=keys, desc=desc, queries=q, qdesc=qdesc, bounds=(0.0, float(w), 0.0, float(h)),
                uright=uright, mp_state=mp_state, inv_sigma2=inv_sigma2)


# reference call sites per variant: (th_dist, nnratio, check_ori, window th)
PROJ_VARIANT_ARGS = {
    "localmap": (100, 0.8, False, 3.0),    # Tracking::SearchLocalPoints: ORBmatcher(0.8), th 1 or 3
    "lastframe": (100, 0.9, True, 15.0),   # TrackWithMotionModel: ORBmatcher(0.9, true), th 15 (mono)
    "keyframe": (64, 0.9, True, 10.0),     # Relocalization: th 10, ORBdist 100 / 64
    "sim3": (50, 0.75, False, 10.0),       # LoopClosing::ComputeSim3: th 10, TH_LOW
    "fuse": (50, 0.6, False, 3.0),         # LocalMapping::SearchInNeighbors: th 3, TH_LOW
    "fuse_sim3": (50, 0.8, False, 4.0),    # LoopClosing::SearchAndFuse: th 4, TH_LOW
}


def make_sim3_case(seed, n1=900, n2=850, w=640, h=480, th=7.5):
    """Two keyframes that see overlapping points: slot i of KF1 projects near
    its partner's keypoint in KF2 and vice versa (plus random slots)."""
    rng = np.random.default_rng(seed)
    sf, _ = scale_tables(1.2, 8)
    c1 = make_proj_case(seed, "sim3", n=n1, nq=n2, th=th)      # KF1's frame data, queries = KF2 slots -> KF1
    c2 = make_proj_case(seed + 1, "sim3", n=n2, nq=n1, th=th)  # KF2's frame data, queries = KF1 slots -> KF2
    # tie the two tables: KF1 slot i's descriptor matches KF2 keypoint partner[i] and vice versa
    partner = rng.permutation(n2)[:min(n1, n2)]
    for i1, i2 in enumerate(partner[:n1]):
        if rng.random() < 0.7:
            c2["qdesc"][i1] = c2["desc"][i2]
            c2["queries"]["u"][i1] = c2["keys"]["x"][i2] + np.float32(rng.normal(0, 1))
            c2["queries"]["v"][i1] = c2["keys"]["y"][i2] + np.float32(rng.normal(0, 1))
            lv = int(c2["keys"]["octave"][i2])
            c2["queries"]["min_level"][i1], c2["queries"]["max_level"][i1] = lv - 1, lv
            c2["queries"]["radius"][i1] = np.float32(th) * sf[lv]
            c1["qdesc"][i2] = c1["desc"][i1]
            c1["queries"]["u"][i2] = c1["keys"]["x"][i1] + np.float32(rng.normal(0, 1))
            c1["queries"]["v"][i2] = c1["keys"]["y"][i1] + np.float32(rng.normal(0, 1))
            lv1 = int(c1["keys"]["octave"][i1])
            c1["queries"]["min_level"][i2], c1["queries"]["max_level"][i2] = lv1 - 1, lv1
            c1["queries"]["radius"][i2] = np.float32(th) * sf[lv1]
    kf1 = dict(keys=c1["keys"], desc=c1["desc"], bounds=c1["bounds"])
    kf2 = dict(keys=c2["keys"], desc=c2["desc"], bounds=c2["bounds"])
    return kf1, kf2, c2["queries"], c2["qdesc"], c1["queries"], c1["qdesc"]


def _bow_csr(node_of, n):
    ids = np.unique(node_of).astype(np.uint32)
    off = np.zeros(len(ids) + 1, np.int32)
    feat = []
    for k, nid in enumerate(ids):
        members = np.nonzero(node_of == nid)[0]          # ascending feature index, as addFeature
        feat.extend(members.tolist())
        off[k + 1] = len(feat)
    return ids, off, np.array(feat, np.int32)


def make_bow_case(seed, variant, na=1000, nb=1000, nodes=120, w=640, h=480):
    rng = np.random.default_rng(seed)
    sf, _ = scale_tables(1.2, 8)
    sigma2 = (sf * sf).astype(np.float32)
    pool = np.sort(rng.choice(10 ** 6, nodes, replace=False)).astype(np.uint32)

    def keys(n):
        k = np.zeros(n, KEYPOINT_DTYPE)
        k["x"] = rng.uniform(0, w, n).astype(np.float32)
        k["y"] = rng.uniform(0, h, n).astype(np.float32)
        k["octave"] = rng.choice(8, n, p=[0.3, 0.2, 0.15, 0.1, 0.1, 0.06, 0.05, 0.04])
        k["angle"] = rng.uniform(0, 360, n).astype(np.float32)
        k["class_id"] = -1
        return k
    ka, kb = keys(na), keys(nb)
    da = rng.integers(0, 256, (na, 32)).astype(np.uint8)
    db = rng.integers(0, 256, (nb, 32)).astype(np.uint8)
    node_a = pool[rng.integers(0, nodes, na)]
    node_b = pool[rng.integers(0, nodes, nb)]
    # true pairs: b copies a (same node, bit noise, similar angle)
    pairs = rng.choice(min(na, nb), min(na, nb) * 2 // 3, replace=False)
    src = rng.permutation(na)[:len(pairs)]
    F12 = np.array([[0.0, -2e-6, 1e-3], [2e-6, 0.0, -2e-3], [-1.2e-3, 2.1e-3, 0.05]], np.float32)
    for b, a in zip(pairs, src):
        node_b[b] = node_a[a]
        d = da[a].copy()
        for bit in rng.choice(256, rng.integers(0, 50), replace=False):
            d[bit >> 3] ^= np.uint8(1 << (bit & 7))
        db[b] = d
        kb["angle"][b] = np.float32((ka["angle"][a] + rng.normal(0, 6)) % 360)
        kb["octave"][b] = ka["octave"][a]
        if variant == "triangulation":
            # move kb onto the epipolar line of ka (+ noise)
            x1, y1 = float(ka["x"][a]), float(ka["y"][a])
            la = x1 * F12[0, 0] + y1 * F12[1, 0] + F12[2, 0]
            lb = x1 * F12[0, 1] + y1 * F12[1, 1] + F12[2, 1]
            lc = x1 * F12[0, 2] + y1 * F12[1, 2] + F12[2, 2]
            px, py = float(kb["x"][b]), float(kb["y"][b])
            t = (la * px + lb * py + lc) / (la * la + lb * lb)
            kb["x"][b] = np.float32(px - la * t + rng.normal(0, 1.0))
            kb["y"][b] = np.float32(py - lb * t + rng.normal(0, 1.0))
    dup = rng.integers(0, nb, nb // 25)
    db[dup] = db[rng.integers(0, nb, len(dup))]          # exact ties
    fa = np.ones(na, np.uint8)
    fb = np.ones(nb, np.uint8)
    if variant in ("kf_frame", "kf_kf"):
        fa[rng.random(na) < 0.2] = 0                      # no (good) map point
    if variant == "kf_kf":
        fb[rng.random(nb) < 0.2] = 0
    if variant == "triangulation":
        fa[rng.random(na) < 0.3] = 0                      # already has a map point
        fb[rng.random(nb) < 0.3] = 0
        fa |= (2 * (rng.random(na) < 0.4)).astype(np.uint8)   # stereo
        fb |= (2 * (rng.random(nb) < 0.4)).astype(np.uint8)
    ia, oa, fea = _bow_csr(node_a, na)
    ib, ob, feb = _bow_csr(node_b, nb)
    A = dict(keys=ka, desc=da, flags=fa, ids=ia, off=oa, feat=fea)
    B = dict(keys=kb, desc=db, flags=fb, ids=ib, off=ob, feat=feb)
    tri = None
    if variant == "triangulation":
        ex, ey = np.float32(w * 0.5), np.float32(h * 0.5)
        tri = np.concatenate([F12.ravel(), [ex, ey], sf, sigma2]).astype(np.float32)
    return A, B, tri


def make_bow_contention_case(seed, variant, nb_node, na_node, nodes=12, hubs=3, w=640, h=480):
    """Tiny descriptor pools: in each of `nodes` nodes, nb_node B features are
    noisy copies of a few hub descriptors and na_node A features are noisy
    copies of the same hubs, so many A features share their best and second
    B features and the greedy "already matched" state of SearchByBoW decides
    most of them (ORBmatcher.cc:200-250, 577-625).  Exact ties included."""
    rng = np.random.default_rng(seed)
    sf, _ = scale_tables(1.2, 8)
    sigma2 = (sf * sf).astype(np.float32)
    pool = np.sort(rng.choice(10 ** 6, nodes, replace=False)).astype(np.uint32)
    na, nb = nodes * na_node, nodes * nb_node

    def noisy(d, nbits):
        d = d.copy()
        for bit in rng.choice(256, nbits, replace=False):
            d[bit >> 3] ^= np.uint8(1 << (bit & 7))
        return d

    def keys(n):
        k = np.zeros(n, KEYPOINT_DTYPE)
        k["x"] = rng.uniform(0, w, n).astype(np.float32)
        k["y"] = rng.uniform(0, h, n).astype(np.float32)
        k["octave"] = rng.choice(8, n, p=[0.3, 0.2, 0.15, 0.1, 0.1, 0.06, 0.05, 0.04])
        k["angle"] = rng.uniform(0, 30, n).astype(np.float32)   # mostly one rotation bin
        k["class_id"] = -1
        return k
    ka, kb = keys(na), keys(nb)
    da = np.zeros((na, 32), np.uint8)
    db = np.zeros((nb, 32), np.uint8)
    node_a = np.repeat(pool, na_node)
    node_b = np.repeat(pool, nb_node)
    for t in range(nodes):
        hub = rng.integers(0, 256, (hubs, 32)).astype(np.uint8)
        for j in range(nb_node):
            db[t * nb_node + j] = noisy(hub[rng.integers(hubs)], int(rng.integers(0, 24)))
        for j in range(na_node):
            da[t * na_node + j] = noisy(hub[rng.integers(hubs)], int(rng.integers(0, 16)))
    dup = rng.integers(0, nb, nb // 10)
    db[dup] = db[rng.integers(0, nb, len(dup))]          # exact ties
    # shuffle so a node's features are not contiguous indices
    pa, pb = rng.permutation(na), rng.permutation(nb)
    ka, da, node_a = ka[pa], da[pa], node_a[pa]
    kb, db, node_b = kb[pb], db[pb], node_b[pb]
    fa = (rng.random(na) > 0.1).astype(np.uint8)
    fb = np.ones(nb, np.uint8) if variant == "kf_frame" else (rng.random(nb) > 0.1).astype(np.uint8)
    tri = None
    if variant == "triangulation":
        fa |= (2 * (rng.random(na) < 0.4)).astype(np.uint8)
        fb |= (2 * (rng.random(nb) < 0.4)).astype(np.uint8)
        F12 = np.array([[0.0, -2e-6, 1e-3], [2e-6, 0.0, -2e-3], [-1.2e-3, 2.1e-3, 0.05]], np.float32)
        tri = np.concatenate([F12.ravel(), [np.float32(w * 0.5), np.float32(h * 0.5)], sf, sigma2]).astype(np.float32)
    ia, oa, fea = _bow_csr(node_a, na)
    ib, ob, feb = _bow_csr(node_b, nb)
    A = dict(keys=ka, desc=da, flags=fa, ids=ia, off=oa, feat=fea)
    B = dict(keys=kb, desc=db, flags=fb, ids=ib, off=ob, feat=feb)
    return A, B, tri


BOW_VARIANT_ARGS = {   # (nnratio, check_ori) at the reference's call sites
    "kf_frame": (0.75, True),        # Tracking::TrackReferenceKeyFrame / Relocalization
    "kf_kf": (0.75, True),           # LoopClosing::ComputeSim3
    "triangulation": (0.6, False),   # LocalMapping::CreateNewMapPoints: ORBmatcher(0.6, false)
}
