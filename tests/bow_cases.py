"""Seeded synthetic inputs for the BoW matchers (SearchByBoW x2,
SearchForTriangulation): two views with FeatureVectors over a shared pool of
vocabulary nodes.  A fraction of B's features are noisy copies of A's in the
same node (true matches, similar angle); for triangulation the copies are
placed near their epipolar line under a synthetic F12 so that
CheckDistEpipolarLine passes for many of them."""
import numpy as np

from oracle.oracle import KEYPOINT_DTYPE, scale_tables


def _bow(node_of, n):
    ids = np.unique(node_of).astype(np.uint32)
    off = np.zeros(len(ids) + 1, np.int32)
    feat = []
    for k, nid in enumerate(ids):
        members = np.nonzero(node_of == nid)[0]          # ascending feature index, as addFeature
        feat.extend(members.tolist())
        off[k + 1] = len(feat)
    return ids, off, np.array(feat, np.int32)


def make_case(seed, variant, na=1000, nb=1000, nodes=120, w=640, h=480):
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
    ia, oa, fea = _bow(node_a, na)
    ib, ob, feb = _bow(node_b, nb)
    A = dict(keys=ka, desc=da, flags=fa, ids=ia, off=oa, feat=fea)
    B = dict(keys=kb, desc=db, flags=fb, ids=ib, off=ob, feat=feb)
    tri = None
    if variant == "triangulation":
        ex, ey = np.float32(w * 0.5), np.float32(h * 0.5)
        tri = np.concatenate([F12.ravel(), [ex, ey], sf, sigma2]).astype(np.float32)
    return A, B, tri


VARIANT_ARGS = {   # (nnratio, check_ori) at the reference's call sites
    "kf_frame": (0.75, True),        # Tracking::TrackReferenceKeyFrame / Relocalization
    "kf_kf": (0.75, True),           # LoopClosing::ComputeSim3
    "triangulation": (0.6, False),   # LocalMapping::CreateNewMapPoints: ORBmatcher(0.6, false)
}
