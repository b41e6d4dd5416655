"""Known-answer tests for the primitives the oracle restates (OpenCV 3.2
semantics) and cross-checks of the C++ oracle against the
independent pure-Python restatement in tests/pyref.py on small seeded inputs.

The reference ships no golden vectors, so these pins are
hand-derived from the published algorithms: parity vs the reference binary
itself stays unpinned."""
import math

import numpy as np
import pytest

import pyref
from orb_slam_2_ros_amd import synth


def test_cv_round_half_even(oracle_mod):
    for v, want in [(0.5, 0), (1.5, 2), (2.5, 2), (-0.5, 0), (-1.5, -2), (2.4999, 2), (3.5000002, 4)]:
        assert oracle_mod.cv_round(v) == want


def test_fast_atan2_axes_and_accuracy(oracle_mod):
    assert oracle_mod.fast_atan2(0.0, 1.0) == 0.0
    assert oracle_mod.fast_atan2(1.0, 0.0) == 90.0
    assert oracle_mod.fast_atan2(0.0, -1.0) == 180.0
    assert oracle_mod.fast_atan2(-1.0, 0.0) == 270.0
    assert oracle_mod.fast_atan2(0.0, 0.0) == 0.0
    rng = np.random.default_rng(1)
    for y, x in rng.integers(-10 ** 5, 10 ** 5, size=(500, 2)):
        a = oracle_mod.fast_atan2(float(y), float(x))
        ref = math.degrees(math.atan2(y, x)) % 360.0
        d = abs(a - ref)
        assert min(d, 360 - d) < 0.01  # OpenCV's polynomial: ~0.0065 deg max error


def test_sincosf_is_glibc(oracle_mod):
    for a in [0.0, 1e-5, 0.5, 1.0, 3.0, 6.2]:
        s, c = oracle_mod.sincosf(a)
        assert abs(s - math.sin(a)) <= 1e-6 and abs(c - math.cos(a)) <= 1e-6


def test_descriptor_distance(oracle_mod):
    a = np.zeros(32, np.uint8)
    b = np.zeros(32, np.uint8)
    assert oracle_mod.descriptor_distance(a, b) == 0
    b[:] = 0xFF
    assert oracle_mod.descriptor_distance(a, b) == 256
    b[:] = 0
    b[5] = 0b1011
    b[31] = 0x80
    assert oracle_mod.descriptor_distance(a, b) == 4
    rng = np.random.default_rng(2)
    for _ in range(50):
        x, y = rng.integers(0, 256, (2, 32)).astype(np.uint8)
        assert oracle_mod.descriptor_distance(x, y) == pyref.hamming(x, y)


def test_gauss_taps():
    # getGaussianKernel(7, 2, CV_32F) scaled by 256 and rounded: the taps sum to
    # 257, so OpenCV 3.2's 8U blur brightens flat areas by 257^2/2^16.
    assert pyref.gauss_taps() == [18, 34, 49, 55, 49, 34, 18]


def test_gauss_constant_and_impulse(oracle_mod):
    flat = np.full((20, 23), 100, np.uint8)
    out = oracle_mod.gauss7(flat)
    assert (out == 101).all()          # 100 * 66049 / 65536 = 100.78
    imp = np.zeros((21, 21), np.uint8)
    imp[10, 10] = 255
    out = oracle_mod.gauss7(imp)
    assert out[10, 10] == 12           # 255 * 55 * 55 / 65536 = 11.77
    assert out[10, 7] == 4 and out[7, 10] == 4   # 255 * 18 * 55 / 65536 = 3.85


@pytest.mark.parametrize("shape", [(17, 13), (31, 45), (24, 37)])
def test_gauss_vs_python(shape, oracle_mod):
    rng = np.random.default_rng(shape[0])
    img = rng.integers(0, 256, shape).astype(np.uint8)
    assert np.array_equal(oracle_mod.gauss7(img), pyref.gauss7(img))


def test_resize_constant_and_ramp(oracle_mod):
    flat = np.full((40, 50), 77, np.uint8)
    assert (oracle_mod.resize_linear(flat, 42, 33) == 77).all()
    ramp = np.tile(np.arange(0, 250, 5, dtype=np.uint8), (12, 1))   # 50 wide
    out = oracle_mod.resize_linear(ramp, 42, 10)
    assert np.array_equal(out, pyref.resize_linear(ramp, 42, 10))
    assert (np.diff(out[0].astype(int)) >= 0).all()


@pytest.mark.parametrize("src,dst", [((48, 64), (40, 53)), ((100, 133), (83, 111)), ((33, 21), (28, 18))])
def test_resize_vs_python(src, dst, oracle_mod):
    rng = np.random.default_rng(src[0])
    img = rng.integers(0, 256, src).astype(np.uint8)
    assert np.array_equal(oracle_mod.resize_linear(img, dst[1], dst[0]),
                          pyref.resize_linear(img, dst[1], dst[0]))


def _fast_patch(arc_len, arc_val=150, center=100, start=0):
    img = np.full((9, 9), center, np.uint8)
    for i in range(arc_len):
        dx, dy = pyref.CIRCLE[(start + i) % 16]
        img[4 + dy, 4 + dx] = arc_val
    return img


def test_fast_known_answers(oracle_mod):
    # 9 contiguous brighter pixels by 50: corner for every threshold < 50, score 49.
    img = _fast_patch(9, start=5)
    for th in (7, 20, 49):
        got = oracle_mod.fast(img, th)
        assert got.tolist() == [[4, 4, 49]]
    assert oracle_mod.fast(img, 50).size == 0
    # 8 contiguous pixels: never a corner.
    assert oracle_mod.fast(_fast_patch(8), 7).size == 0
    # darker arc of 12 pixels by 30: score 29.
    img = _fast_patch(12, arc_val=70, start=11)
    assert oracle_mod.fast(img, 20).tolist() == [[4, 4, 29]]


@pytest.mark.parametrize("seed", range(4))
def test_fast_vs_python(seed, oracle_mod):
    rng = np.random.default_rng(seed)
    img = synth.frame(40, 37, 900 + seed)
    img = np.clip(img.astype(int) + rng.integers(-40, 40, img.shape), 0, 255).astype(np.uint8)
    for th in (7, 20):
        got = [tuple(r) for r in oracle_mod.fast(img, th).tolist()]
        assert got == pyref.fast_cell(img, th)


@pytest.mark.parametrize("seed,N", [(0, 5), (1, 17), (2, 40), (3, 60), (4, 3), (5, 100)])
def test_distribute_vs_python(seed, N, oracle_mod):
    rng = np.random.default_rng(seed)
    w, h = 160 + 37 * seed, 120 + 11 * seed
    n = int(rng.integers(30, 300))
    xs = rng.integers(19, w - 19, n)
    ys = rng.integers(19, h - 19, n)
    pts = sorted(set(zip(ys.tolist(), xs.tolist())))  # unique pixels, row-major
    cands = [(x, y, int(rng.integers(7, 120))) for y, x in pts]
    sel = oracle_mod.distribute(np.array(cands, np.int32), w, h, N).tolist()
    assert sel == pyref.distribute(cands, w, h, N)
    assert len(sel) <= max(N + 2, 4 * 4)


def test_level_geometry_matches_survey(oracle_mod):
    # SURVEY.md Appendix A (level sizes) and §8(a) a1 (quotas)
    lw, lh, q, s = oracle_mod.levels(640, 480, 1000)
    assert list(zip(lw.tolist(), lh.tolist())) == [(640, 480), (533, 400), (444, 333), (370, 278),
                                                   (309, 231), (257, 193), (214, 161), (179, 134)]
    assert q.tolist() == [217, 181, 151, 126, 105, 87, 73, 60]
    lw, lh, q, _ = oracle_mod.levels(1920, 1080, 1000)
    assert list(zip(lw.tolist(), lh.tolist()))[-1] == (536, 301)
    assert int((lw.astype(np.int64) * lh).sum()) == 6419321
    _, _, q, _ = oracle_mod.levels(752, 480, 1200)
    assert q.tolist() == [261, 217, 181, 151, 126, 105, 87, 72]
    _, _, q, _ = oracle_mod.levels(1241, 376, 2000)
    assert q.tolist() == [434, 362, 302, 251, 209, 175, 145, 122]


@pytest.mark.parametrize("seed", range(3))
def test_matcher_vs_python(seed, oracle_mod):
    w, h = 320, 240
    fr = synth.frames(w, h, 300 + seed, 2)
    k1, d1 = oracle_mod.extract(fr[0], 500)
    k2, d2 = oracle_mod.extract(fr[1], 500)
    prev = np.ascontiguousarray(np.stack([k1["x"], k1["y"]], 1).astype(np.float32))
    for window, ratio, ori in [(100, 0.9, True), (30, 0.6, True), (60, 0.9, False)]:
        nm, m12, p2 = oracle_mod.search_for_initialization(k1, d1, k2, d2, w, h, prev, window, ratio, ori)
        nm_p, m12_p, p2_p = pyref.search_for_initialization(k1, d1, k2, d2, w, h, prev, window, ratio, ori)
        assert nm == nm_p and np.array_equal(m12, m12_p) and np.array_equal(p2, p2_p)
    assert nm > 0


def _stereo_inputs(oracle_mod, w, h, nf, seed, disparity):
    L, R = synth.stereo_pair(w, h, seed, 0, disparity)
    kl, dl = oracle_mod.extract(L, nf)
    kr, dr = oracle_mod.extract(R, nf)
    return oracle_mod.pyramid(L), oracle_mod.pyramid(R), kl, dl, kr, dr


def _edge_keypoints(pyr, n, rng, nlev=8):
    """Random keypoints anywhere on random levels (incl. the borders the
    reference would assert on), in level-0 coordinates like the extractor's."""
    sf, _ = __import__("oracle.oracle", fromlist=["x"]).scale_tables(1.2, nlev)
    k = np.zeros(n, dtype=[("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                           ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
    oc = rng.integers(0, nlev, n)
    for i in range(n):
        hh, ww = pyr[oc[i]].shape
        k["x"][i] = np.float32(rng.integers(0, ww)) * sf[oc[i]]
        k["y"][i] = np.float32(rng.integers(0, hh)) * sf[oc[i]]
    k["octave"] = oc
    k["class_id"] = -1
    return k


@pytest.mark.parametrize("w,h,nf,seed,disp", [(320, 240, 500, 41, 12), (400, 200, 400, 42, 3)])
def test_stereo_vs_python(w, h, nf, seed, disp, oracle_mod):
    pl, pr, kl, dl, kr, dr = _stereo_inputs(oracle_mod, w, h, nf, seed, disp)
    sf, inv = oracle_mod.scale_tables()
    mbf, mb = 40.0, float(np.float32(40.0) / np.float32(300.0))
    ur, dp, kept = oracle_mod.compute_stereo_matches(pl, pr, kl, dl, kr, dr, mbf, mb)
    pur, pdp, pkept = pyref.compute_stereo_matches(pl, pr, sf, inv, kl, dl, kr, dr, mbf, mb)
    assert kept == pkept and kept > 0.3 * len(kl)
    assert np.array_equal(ur, pur) and np.array_equal(dp, pdp)
    v = ur >= 0
    assert abs(np.median(kl["x"][v] - ur[v]) - disp) < 0.5


def test_stereo_edge_keypoints_vs_python(oracle_mod):
    rng = np.random.default_rng(43)
    pl, pr, _, _, _, _ = _stereo_inputs(oracle_mod, 320, 240, 300, 43, 8)
    kl = _edge_keypoints(pl, 300, rng)
    kr = kl.copy()
    kr["x"] -= np.float32(8.0)
    dl = rng.integers(0, 256, (300, 32)).astype(np.uint8)
    dr = dl.copy()
    flips = rng.integers(0, 256, (300, 32)).astype(np.uint8) & rng.integers(0, 256, (300, 32)).astype(np.uint8) \
        & rng.integers(0, 256, (300, 32)).astype(np.uint8)
    dr ^= flips   # ~1/8 of the bits differ: some pairs pass TH 75, some do not
    sf, inv = oracle_mod.scale_tables()
    for mbf, mb in [(40.0, 0.1), (40.0, 1e9), (1e6, 0.5)]:
        ur, dp, kept = oracle_mod.compute_stereo_matches(pl, pr, kl, dl, kr, dr, mbf, mb)
        pur, pdp, pkept = pyref.compute_stereo_matches(pl, pr, sf, inv, kl, dl, kr, dr, mbf, mb)
        assert kept == pkept and np.array_equal(ur, pur) and np.array_equal(dp, pdp)


def test_stereo_from_rgbd_oracle(oracle_mod):
    rng = np.random.default_rng(44)
    d = synth.depth_map(160, 120, 44)
    k = np.zeros(500, oracle_mod.KEYPOINT_DTYPE)
    k["x"] = rng.uniform(-2, 162, 500).astype(np.float32)
    k["y"] = rng.uniform(-2, 122, 500).astype(np.float32)
    ur, dp = oracle_mod.stereo_from_rgbd(k, d, 40.0)
    for i in range(500):
        u, v = int(k["x"][i]), int(k["y"][i])
        z = d[v, u] if (0 <= u < 160 and 0 <= v < 120) else np.float32(np.nan)
        if z > 0:
            assert dp[i] == z and ur[i] == np.float32(k["x"][i] - np.float32(np.float32(40.0) / z))
        else:
            assert dp[i] == -1 and ur[i] == -1


@pytest.mark.parametrize("variant", ["localmap", "lastframe", "keyframe", "sim3", "fuse", "fuse_sim3"])
@pytest.mark.parametrize("seed,stereo", [(81, False), (82, True)])
def test_projection_matchers_vs_python(variant, seed, stereo, oracle_mod):
    from orb_slam_2_ros_amd.synth_match import PROJ_VARIANT_ARGS as VARIANT_ARGS, make_proj_case as make_case
    th, ratio, ori, wth = VARIANT_ARGS[variant]
    c = make_case(seed, variant, n=900, nq=700, stereo=stereo, th=wth)
    a = oracle_mod.search_by_projection(variant, c["keys"], c["desc"], c["queries"], c["qdesc"], c["bounds"],
                                        c["uright"], c["mp_state"], c["inv_sigma2"], th, ratio, ori)
    b = pyref.search_by_projection(variant, c["keys"], c["desc"], c["queries"], c["qdesc"], c["bounds"],
                                   c["uright"], c["mp_state"], c["inv_sigma2"], th, ratio, ori)
    assert a[0] == b[0] and a[0] > 20
    for x, y in zip(a[1:], b[1:]):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("variant", ["kf_frame", "kf_kf", "triangulation"])
@pytest.mark.parametrize("seed,ori", [(101, True), (102, False)])
def test_bow_matchers_vs_python(variant, seed, ori, oracle_mod):
    from orb_slam_2_ros_amd.synth_match import BOW_VARIANT_ARGS as VARIANT_ARGS, make_bow_case as make_case
    A, B, tri = make_case(seed, variant, na=700, nb=650)
    ratio, _ = VARIANT_ARGS[variant]
    a = oracle_mod.search_by_bow(variant, A, B, ratio, ori, tri)
    b = pyref.search_by_bow(variant, A, B, ratio, ori, tri)
    assert a[0] == b[0] and a[0] > 20
    assert np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2])


def test_search_by_sim3_vs_python(oracle_mod):
    from orb_slam_2_ros_amd.synth_match import make_sim3_case
    kf1, kf2, q1, qd1, q2, qd2 = make_sim3_case(97, n1=500, n2=480)
    nf, m = oracle_mod.search_by_sim3(kf1["keys"], kf1["desc"], kf1["bounds"], kf2["keys"], kf2["desc"],
                                      kf2["bounds"], q1, qd1, q2, qd2, 100)
    # two best-only searches (INT_MAX start, TH_HIGH) + agreement, from the pure-Python restatement
    _, m1, _, _ = pyref.search_by_projection("fuse_sim3", kf2["keys"], kf2["desc"], q1, qd1, kf2["bounds"],
                                             th_dist=100)
    _, m2, _, _ = pyref.search_by_projection("fuse_sim3", kf1["keys"], kf1["desc"], q2, qd2, kf1["bounds"],
                                             th_dist=100)
    want = np.array([i2 if i2 >= 0 and m2[i2] == i1 else -1 for i1, i2 in enumerate(m1)], np.int32)
    assert nf == int((want >= 0).sum()) and nf > 30
    assert np.array_equal(m, want)


@pytest.mark.parametrize("irregular", [False, True])
@pytest.mark.parametrize("scoring,weighting", [(0, 0), (1, 1), (5, 0), (5, 2), (0, 3), (2, 1)])
@pytest.mark.parametrize("levelsup", [0, 2, 4, 9])
def test_vocab_transform_vs_python(irregular, scoring, weighting, levelsup, oracle_mod):
    """DBoW2 transform: the oracle against an independent restatement, on
    small synthetic trees (regular and with early leaves), every weighting and
    normalisation path, FeatureVector levels from the root to the leaves."""
    from orb_slam_2_ros_amd.synth_vocab import features_near_leaves, make_vocab
    voc = make_vocab(k=6 if irregular else 5, L=4, seed=3 + irregular, irregular=irregular, stop_frac=0.1,
                     scoring=scoring, weighting=weighting)
    feats = features_near_leaves(voc, 300, seed=7)
    feats[5] = feats[4]                                  # repeated words
    bow, fv, _ = oracle_mod.vocab_transform(voc, feats, levelsup)
    pbow, pfv = pyref.vocab_transform(voc, feats, levelsup)
    assert list(bow) == list(pbow) and list(fv) == list(pfv)
    assert all(bow[k] == pbow[k] for k in bow)           # bit-exact doubles
    assert fv == pfv
    assert len(bow) > 10


def test_vocab_transform_empty_oracle(oracle_mod):
    from orb_slam_2_ros_amd.synth_vocab import make_vocab
    voc = make_vocab(k=4, L=2, seed=1)
    bow, fv, _ = oracle_mod.vocab_transform(voc, np.zeros((0, 32), np.uint8), 1)
    assert bow == {} and fv == {}
    voc["is_leaf"][:] = 0                                # no words: empty()
    bow, fv, _ = oracle_mod.vocab_transform(voc, np.ones((3, 32), np.uint8), 1)
    assert bow == {} and fv == {}


def _obs_descs(seed, npts, maxn):
    rng = np.random.default_rng(seed)
    sizes = rng.integers(0, maxn + 1, npts)
    sizes[0] = 0
    sizes[1] = 1
    offsets = np.zeros(npts + 1, np.int32)
    offsets[1:] = np.cumsum(sizes)
    base = rng.integers(0, 256, (npts, 32)).astype(np.uint8)
    desc = np.repeat(base, sizes, axis=0)
    noise = (rng.integers(0, 256, desc.shape) & rng.integers(0, 256, desc.shape)
             & rng.integers(0, 256, desc.shape)).astype(np.uint8)
    desc ^= noise
    dup = rng.random(len(desc)) < 0.1                       # repeated rows: median ties
    desc[dup] = desc[np.maximum(np.nonzero(dup)[0] - 1, 0)]
    return desc, offsets


def test_distinctive_descriptors_vs_python(oracle_mod):
    desc, offsets = _obs_descs(3, 60, 25)
    assert np.array_equal(oracle_mod.distinctive_descriptors(desc, offsets),
                          pyref.distinctive_descriptors(desc, offsets))


CAMERAS = {   # fx fy cx cy, k1 k2 p1 p2 [k3]: TUM1 / EuRoC / KITTI-like settings files
    "tum1": ((517.306408, 516.469215, 318.643040, 255.313989), (0.262383, -0.953104, -0.005358, 0.002628, 1.163314)),
    "euroc": ((458.654, 457.296, 367.215, 248.375), (-0.28340811, 0.07395907, 0.00019359, 1.76187114e-05)),
    "none": ((718.856, 718.856, 607.1928, 185.2157), (0.0, 0.0, 0.0, 0.0)),
}


def _K(c):
    fx, fy, cx, cy = c
    return np.array([[fx, 0, cx], [0, fy, cy], [0, 0, 1]], np.float32)


@pytest.mark.parametrize("cam", sorted(CAMERAS))
def test_undistort_vs_python(cam, oracle_mod):
    c, d = CAMERAS[cam]
    rng = np.random.default_rng(4)
    xy = np.stack([rng.uniform(0, 752, 400), rng.uniform(0, 480, 400)], 1).astype(np.float32)
    o = oracle_mod.undistort_points(xy, _K(c), d)
    p = pyref.undistort_points(xy, _K(c), d)
    assert np.array_equal(o.view(np.uint32), p.view(np.uint32))
    if cam == "none":
        assert np.array_equal(o, xy)
    else:
        assert np.abs(o - xy).max() > 1.0


def test_cvt_gray_and_depth_oracle(oracle_mod):
    rng = np.random.default_rng(5)
    img = rng.integers(0, 256, (37, 53, 4)).astype(np.uint8)
    i32 = img.astype(np.int64)
    for cn in (3, 4):
        for rgb in (True, False):
            r, b = (i32[..., 0], i32[..., 2]) if rgb else (i32[..., 2], i32[..., 0])
            ref = ((r * 4899 + i32[..., 1] * 9617 + b * 1868 + 8192) >> 14).astype(np.uint8)
            assert np.array_equal(oracle_mod.cvt_gray(img[..., :cn], rgb), ref)
    d16 = rng.integers(0, 65536, (21, 33)).astype(np.uint16)
    scale = np.float32(1.0) / np.float32(5000.0)
    assert np.array_equal(oracle_mod.depth_to_float(d16, scale), d16.astype(np.float32) * scale)


def _kfdb_script():
    """A query script over synthetic keyframes: add along the trajectory,
    loop queries (connected = covisible neighbours), relocalisation queries,
    an erase + re-add, and a repeated query id."""
    from orb_slam_2_ros_amd.synth_vocab import make_keyframe_bows
    bows, covis = make_keyframe_bows(n_kf=240, n_words=20000, words_per_kf=300, seed=5, loop_every=50)
    ops = []
    for i, (w, v) in enumerate(bows):
        if i >= 20 and i % 7 == 0:
            ops.append(("loop", i, w, v, covis[i], 0.01))
        if i >= 20 and i % 11 == 0:
            ops.append(("reloc", 10000 + i, w, v, None, 0.0))
        ops.append(("add", i, w, v))
        if i == 120:
            ops.append(("erase", 60))
        if i == 160:
            ops.append(("add", 60, *bows[60]))
        if i == 200:
            ops.append(("loop", 196, w, v, covis[196], 0.005))   # a query id met before
    return ops, covis


def _run_kfdb(db, ops, covis, detect):
    out = []
    for op in ops:
        if op[0] == "add":
            db.add(op[1], op[2], op[3])
        elif op[0] == "erase":
            db.erase(op[1])
        else:
            kind, qid, w, v, conn, ms = op
            out.append(detect(db, kind == "reloc", qid, w, v, conn, ms, lambda k: covis.get(k, [])))
    return out


def test_kfdb_oracle_vs_python(oracle_mod):
    ops, covis = _kfdb_script()
    o = _run_kfdb(oracle_mod.KeyFrameDB(20000), ops, covis,
                  lambda db, r, q, w, v, c, m, cv: db.detect(r, q, w, v, c, m, cv))
    p = _run_kfdb(pyref.KeyFrameDB(), ops, covis,
                  lambda db, r, q, w, v, c, m, cv: db.detect(r, q, w, v, c, m, cv))
    assert o == p
    assert sum(len(x) > 0 for x in o) > 10


def test_bow_score_l1_oracle(oracle_mod):
    from orb_slam_2_ros_amd.synth_vocab import make_keyframe_bows
    bows, _ = make_keyframe_bows(n_kf=30, n_words=3000, words_per_kf=200, seed=2)
    for a in range(0, 30, 3):
        for b in range(1, 30, 4):
            assert oracle_mod.bow_score_l1(*bows[a], *bows[b]) == pyref.l1_score(*bows[a], *bows[b])


def _reproj_median(T, X, E):
    Xc = np.einsum("eij,ej->ei", T[E["cam"], :, :3].astype(np.float64), X[E["point"]].astype(np.float64)) \
        + T[E["cam"], :, 3]
    u = E["fx"] * Xc[:, 0] / Xc[:, 2] + E["cx"]
    v = E["fy"] * Xc[:, 1] / Xc[:, 2] + E["cy"]
    return float(np.median(np.hypot(u - E["u"], v - E["v"])))


def test_local_ba_oracle_converges_and_flags_outliers(oracle_mod):
    """The restated LocalBundleAdjustment reduces the reprojection error,
    brings the free poses toward the truth, keeps the fixed ones, and marks
    the injected gross outliers for erasure."""
    from orb_slam_2_ros_amd.synth_ba import make_ba_problem
    P = make_ba_problem(n_local=6, n_fixed=2, n_points=600, seed=3, outlier_frac=0.04)
    To, Xo, out, its = oracle_mod.local_ba(P["Tcw"], P["fixed"], P["Xw"], P["edges"])
    assert its[0] >= 1 and its[1] >= 1
    assert _reproj_median(To, Xo, P["edges"]) < 0.6 * _reproj_median(P["Tcw"], P["Xw"], P["edges"])
    free = P["fixed"] == 0
    assert np.abs(To[free] - P["Tcw_true"][free]).max() < 0.5 * np.abs(P["Tcw"][free] - P["Tcw_true"][free]).max()
    assert np.array_equal(To[~free], P["Tcw"][~free])
    E = P["edges"]
    Xc = np.einsum("eij,ej->ei", P["Tcw_true"][E["cam"], :, :3], P["Xw_true"][E["point"]]) + P["Tcw_true"][E["cam"], :, 3]
    gross = np.hypot(E["fx"] * Xc[:, 0] / Xc[:, 2] + E["cx"] - E["u"], E["fy"] * Xc[:, 1] / Xc[:, 2] + E["cy"] - E["v"]) > 14
    assert out[gross].mean() > 0.95


def test_local_ba_step_solves_the_normal_equations(oracle_mod):
    """The Schur-reduced step equals the solution of the full damped normal
    equations (H + lambda I) x = b built from numerical Jacobians of the
    reprojection error under g2o's left SE3 / additive point perturbations."""
    from orb_slam_2_ros_amd.synth_ba import make_ba_problem
    P = make_ba_problem(n_local=3, n_fixed=1, n_points=40, seed=4, outlier_frac=0.0, stereo_frac=0.5)
    T, F, X, E = P["Tcw"].astype(np.float64), P["fixed"], P["Xw"].astype(np.float64), P["edges"]
    lam = 1e-2
    x, chi2, ok = oracle_mod.ba_debug_step(P["Tcw"], F, P["Xw"], E, robust=False, lam=lam)
    assert ok
    free = np.nonzero(F == 0)[0]
    nf, npt = len(free), len(X)
    fidx = {c: i for i, c in enumerate(free)}

    def expm(w6):
        R = pyref_rot(w6[:3])
        return R, w6[3:]

    def pyref_rot(w):
        th = np.linalg.norm(w)
        K = np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]])
        if th < 1e-12:
            return np.eye(3) + K
        return np.eye(3) + np.sin(th) / th * K + (1 - np.cos(th)) / th ** 2 * K @ K

    def resid(Tc, Xp, e):
        Xc = Tc[:, :3] @ Xp + Tc[:, 3]
        u = e["fx"] * Xc[0] / Xc[2] + e["cx"]
        v = e["fy"] * Xc[1] / Xc[2] + e["cy"]
        r = [e["u"] - u, e["v"] - v]
        if e["ur"] >= 0:
            r.append(e["ur"] - (u - e["bf"] / Xc[2]))
        return np.array(r)

    n = 6 * nf + 3 * npt
    H, b = np.zeros((n, n)), np.zeros(n)
    for e in E:
        c, p = int(e["cam"]), int(e["point"])
        r0 = resid(T[c], X[p], e)
        cols, J = [], []
        if c in fidx:
            for k in range(6):
                d = np.zeros(6); d[k] = 1e-6
                R, t = expm(d)
                Tn = np.hstack([R @ T[c][:, :3], (R @ T[c][:, 3] + t)[:, None]])
                J.append((resid(Tn, X[p], e) - r0) / 1e-6)
                cols.append(6 * fidx[c] + k)
        for k in range(3):
            d = np.zeros(3); d[k] = 1e-6
            J.append((resid(T[c], X[p] + d, e) - r0) / 1e-6)
            cols.append(6 * nf + 3 * p + k)
        J = np.array(J).T
        w = float(e["inv_sigma2"])
        H[np.ix_(cols, cols)] += w * J.T @ J
        b[cols] += -w * J.T @ r0
    xr = np.linalg.solve(H + lam * np.eye(n), b)
    assert np.allclose(x, xr, rtol=2e-3, atol=2e-5 * np.abs(xr).max())
