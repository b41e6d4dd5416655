"""GPU parity for the depth association rows (SURVEY.md §8 a20 + RGB-D):
Frame::ComputeStereoMatches and Frame::ComputeStereoFromRGBD on liborbx.so vs
the CPU oracle, bit-exact (mvuRight / mvDepth are float32; both sides evaluate
the same IEEE-single sequence of Frame.cc:631-657, so the tolerance is 0 ulp).
"""
import numpy as np
import pytest

from orb_slam_2_ros_amd import ORBextractor, compute_stereo_matches, stereo_from_rgbd, synth

pytestmark = pytest.mark.gpu

STEREO = [
    # (w, h, nfeatures, seed, disparity, fx, bf)   C3 EuRoC, C4 KITTI + small/odd
    (752, 480, 1200, 51, 20, 435.2, 47.9),
    (1241, 376, 2000, 52, 20, 718.856, 386.1448),
    (1920, 1080, 1000, 57, 20, 1050.0, 126.0),      # north_star FHD stereo (largest bands / SAD levels)
    (1920, 1080, 2000, 58, 41, 1050.0, 126.0),
    (640, 480, 1000, 53, 7, 517.3, 40.0),
    (333, 250, 500, 54, 13, 300.0, 30.0),
]


def _mb(bf, fx):
    return float(np.float32(bf) / np.float32(fx))   # Frame.cc:115, mb = mbf / fx


@pytest.fixture(scope="module")
def pairs_of_extractors():
    cache = {}

    def get(nfeat):
        if nfeat not in cache:
            cache[nfeat] = (ORBextractor(nfeat, 1.2, 8, 20, 7), ORBextractor(nfeat, 1.2, 8, 20, 7))
        return cache[nfeat]
    return get


@pytest.mark.parametrize("w,h,nf,seed,disp,fx,bf", STEREO)
def test_compute_stereo_matches_bit_exact(w, h, nf, seed, disp, fx, bf, pairs_of_extractors, oracle_mod):
    L, R = synth.stereo_pair(w, h, seed, 0, disp)
    exl, exr = pairs_of_extractors(nf)
    kl, dl = exl(L)
    kr, dr = exr(R)
    ko, do = oracle_mod.extract(L, nf)
    assert len(kl) == len(ko) and (kl == ko).all() and np.array_equal(dl, do)
    ur, dp, kept = compute_stereo_matches(exl, exr, kl, dl, kr, dr, bf, _mb(bf, fx))
    our, odp, okept = oracle_mod.compute_stereo_matches(oracle_mod.pyramid(L), oracle_mod.pyramid(R), kl, dl, kr, dr,
                                                        bf, _mb(bf, fx))
    assert kept == okept and kept > 0.3 * len(kl)
    i = np.nonzero(ur.view(np.uint32) != our.view(np.uint32))[0]
    assert len(i) == 0, f"mvuRight differs at {i[:5]}: {ur[i[:5]]} vs {our[i[:5]]}"
    assert np.array_equal(dp.view(np.uint32), odp.view(np.uint32))


def _random_keypoints(levels, n, rng):
    from oracle.oracle import KEYPOINT_DTYPE, scale_tables
    sf, _ = scale_tables(1.2, len(levels))
    k = np.zeros(n, KEYPOINT_DTYPE)
    oc = rng.integers(0, len(levels), n)
    for i in range(n):
        hh, ww = levels[oc[i]].shape
        k["x"][i] = np.float32(rng.integers(0, ww)) * sf[oc[i]]
        k["y"][i] = np.float32(rng.integers(0, hh)) * sf[oc[i]]
    k["octave"] = oc
    k["class_id"] = -1
    return k


@pytest.mark.parametrize("shift", [8.0, 0.0, 31.5])
def test_stereo_edge_keypoints(shift, pairs_of_extractors, oracle_mod):
    """Keypoints on every level incl. image borders (the reference's
    assert / UB cases), descriptors with controlled bit noise, and ties."""
    rng = np.random.default_rng(int(shift * 10) + 7)
    w, h = 640, 480
    L, R = synth.stereo_pair(w, h, 55, 0, 8)
    exl, exr = pairs_of_extractors(1000)
    exl(L)
    exr(R)
    pl, pr = oracle_mod.pyramid(L), oracle_mod.pyramid(R)
    n = 1500
    kl = _random_keypoints(pl, n, rng)
    kr = kl.copy()
    kr["x"] -= np.float32(shift)
    dl = rng.integers(0, 256, (n, 32)).astype(np.uint8)
    noise = (rng.integers(0, 256, dl.shape) & rng.integers(0, 256, dl.shape) & rng.integers(0, 256, dl.shape))
    dr = dl ^ noise.astype(np.uint8)
    kr = np.concatenate([kr, kr[:200]])   # duplicated right keypoints: exact distance ties
    dr = np.concatenate([dr, dr[:200]])
    for bf, mb in [(40.0, 0.1), (1e6, 0.5), (40.0, 1e9)]:
        ur, dp, kept = compute_stereo_matches(exl, exr, kl, dl, kr, dr, bf, mb)
        our, odp, okept = oracle_mod.compute_stereo_matches(pl, pr, kl, dl, kr, dr, bf, mb)
        assert kept == okept
        assert np.array_equal(ur.view(np.uint32), our.view(np.uint32))
        assert np.array_equal(dp.view(np.uint32), odp.view(np.uint32))


def test_stereo_empty_sides(pairs_of_extractors, oracle_mod):
    L, R = synth.stereo_pair(320, 240, 56, 0, 10)
    exl, exr = pairs_of_extractors(500)
    kl, dl = exl(L)
    kr, dr = exr(R)
    ur, dp, kept = compute_stereo_matches(exl, exr, kl, dl, kr[:0], dr[:0], 40.0, 0.1)
    assert kept == 0 and (ur == -1).all() and (dp == -1).all()
    ur, dp, kept = compute_stereo_matches(exl, exr, kl[:0], dl[:0], kr, dr, 40.0, 0.1)
    assert kept == 0 and len(ur) == 0


def test_stereo_step_device_matches_host(pairs_of_extractors, oracle_mod):
    import torch
    w, h, P, nf = 752, 480, 3, 1200
    bf, fx = 47.9, 435.2
    pairs = [synth.stereo_pair(w, h, 60 + p, 0, 20) for p in range(P)]
    ex = ORBextractor(nf, 1.2, 8, 20, 7)
    ex.reserve(w, h, 2 * P)
    dev = torch.device("cuda:0")
    imgs = torch.from_numpy(np.stack([im for pr in pairs for im in pr])).to(dev)
    torch.cuda.synchronize()
    ex.stereo_step_device(imgs.data_ptr(), w * h, w, P, bf, _mb(bf, fx))
    for p, (L, R) in enumerate(pairs):
        kl, dl = ex.batch_download(2 * p)
        kr, dr = ex.batch_download(2 * p + 1)
        ko, do = oracle_mod.extract(L, nf)
        assert len(kl) == len(ko) and (kl == ko).all()
        ur, dp, kept = ex.depth_download(p)
        our, odp, okept = oracle_mod.compute_stereo_matches(oracle_mod.pyramid(L), oracle_mod.pyramid(R), kl, dl, kr,
                                                            dr, bf, _mb(bf, fx))
        assert kept == okept and kept > 0
        assert np.array_equal(ur.view(np.uint32), our.view(np.uint32))
        assert np.array_equal(dp.view(np.uint32), odp.view(np.uint32))


def test_stereo_from_rgbd_host_and_batch(oracle_mod):
    import torch
    w, h, B = 640, 480, 3
    bf = 40.0
    frames = [synth.frame(w, h, 70 + b) for b in range(B)]
    depths = [synth.depth_map(w, h, 70 + b) for b in range(B)]
    ex = ORBextractor(1000, 1.2, 8, 20, 7)
    # host API on the extractor's keypoints, plus out-of-image keypoints
    k, _ = ex(frames[0])
    rng = np.random.default_rng(71)
    ko = k.copy()
    ko["x"][:50] = rng.uniform(-5, w + 5, 50).astype(np.float32)
    ko["y"][:50] = rng.uniform(-5, h + 5, 50).astype(np.float32)
    ur, dp, kept = stereo_from_rgbd(ko, depths[0], bf)
    our, odp = oracle_mod.stereo_from_rgbd(ko, depths[0], bf)
    assert np.array_equal(ur.view(np.uint32), our.view(np.uint32))
    assert np.array_equal(dp.view(np.uint32), odp.view(np.uint32))
    assert kept == int((odp > 0).sum())
    # batched device step
    ex.reserve(w, h, B)
    dev = torch.device("cuda:0")
    ti = torch.from_numpy(np.stack(frames)).to(dev)
    td = torch.from_numpy(np.stack(depths)).to(dev)
    torch.cuda.synchronize()
    ex.rgbd_step_device(ti.data_ptr(), w * h, w, B, td.data_ptr(), 4 * w * h, 4 * w, bf)
    for b in range(B):
        kg, _ = ex.batch_download(b)
        ur, dp, kept = ex.depth_download(b)
        our, odp = oracle_mod.stereo_from_rgbd(kg, depths[b], bf)
        assert np.array_equal(ur.view(np.uint32), our.view(np.uint32))
        assert np.array_equal(dp.view(np.uint32), odp.view(np.uint32))
        assert kept == int((odp > 0).sum())


def _read_kps(buf, off):
    from orb_slam_2_ros_amd import KEYPOINT_DTYPE
    n = int(np.frombuffer(buf, np.int32, 1, off)[0])
    off += 4
    k = np.frombuffer(buf, KEYPOINT_DTYPE, n, off)
    off += 28 * n
    d = np.frombuffer(buf, np.uint8, 32 * n, off).reshape(n, 32)
    return k, d, off + 32 * n


def test_cpp_adapter_stereo_and_rgbd(tmp_path, oracle_mod):
    """OrbxFrame::ComputeStereoMatches / ComputeStereoFromRGBD of the C++
    drop-in (include/orbx_orbslam2.hpp) vs the oracle."""
    import subprocess
    from cxx_build import build_adapter_test
    exe = build_adapter_test()
    w, h, bf, fx = 752, 480, 47.9, 435.2
    L, R = synth.stereo_pair(w, h, 80, 0, 20)
    (tmp_path / "l.raw").write_bytes(L.tobytes())
    (tmp_path / "r.raw").write_bytes(R.tobytes())
    mb = _mb(bf, fx)
    subprocess.run([str(exe), "stereo", str(w), str(h), str(tmp_path / "l.raw"), str(tmp_path / "r.raw"), repr(bf),
                    repr(mb), str(tmp_path / "s.bin")], check=True)
    buf = (tmp_path / "s.bin").read_bytes()
    kl, dl, off = _read_kps(buf, 0)
    kr, dr, off = _read_kps(buf, off)
    kept = int(np.frombuffer(buf, np.int32, 1, off)[0])
    ur = np.frombuffer(buf, np.float32, len(kl), off + 4)
    dp = np.frombuffer(buf, np.float32, len(kl), off + 4 + 4 * len(kl))
    # the adapter parses mbf / mb with atof -> float, as the test does
    our, odp, okept = oracle_mod.compute_stereo_matches(oracle_mod.pyramid(L), oracle_mod.pyramid(R), kl, dl, kr, dr,
                                                        float(np.float32(bf)), float(np.float32(mb)))
    assert kept == okept and kept > 0
    assert np.array_equal(ur.view(np.uint32), our.view(np.uint32))
    assert np.array_equal(dp.view(np.uint32), odp.view(np.uint32))

    img = synth.frame(w, h, 81)
    dm = synth.depth_map(w, h, 81)
    (tmp_path / "i.raw").write_bytes(img.tobytes())
    (tmp_path / "d.raw").write_bytes(dm.tobytes())
    subprocess.run([str(exe), "rgbd", str(w), str(h), str(tmp_path / "i.raw"), str(tmp_path / "d.raw"), repr(bf),
                    str(tmp_path / "g.bin")], check=True)
    buf = (tmp_path / "g.bin").read_bytes()
    k, _, off = _read_kps(buf, 0)
    ur = np.frombuffer(buf, np.float32, len(k), off)
    dp = np.frombuffer(buf, np.float32, len(k), off + 4 * len(k))
    our, odp = oracle_mod.stereo_from_rgbd(k, dm, float(np.float32(bf)))
    assert np.array_equal(ur.view(np.uint32), our.view(np.uint32))
    assert np.array_equal(dp.view(np.uint32), odp.view(np.uint32))


def test_stereo_pair_on_two_threads(oracle_mod):
    """Frame's stereo constructor extracts left and right on two threads
    (Frame.cc:79-82): two fresh extractors whose first calls (plan upload,
    graph capture) run concurrently, then repeated concurrent calls; every
    result is the oracle's."""
    import threading
    w, h, nf = 752, 480, 1200
    L, R = synth.stereo_pair(w, h, 61, 0, 20)
    ko_l, do_l = oracle_mod.extract(L, nf)
    ko_r, do_r = oracle_mod.extract(R, nf)
    for rep in range(3):
        exl, exr = ORBextractor(nf, 1.2, 8, 20, 7), ORBextractor(nf, 1.2, 8, 20, 7)
        out = {}
        go = threading.Barrier(2)

        def run(name, ex, img):
            go.wait()
            out[name] = [ex(img) for _ in range(4)]
        ts = [threading.Thread(target=run, args=("l", exl, L)), threading.Thread(target=run, args=("r", exr, R))]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        for (k, d) in out["l"]:
            assert len(k) == len(ko_l) and (k == ko_l).all() and np.array_equal(d, do_l)
        for (k, d) in out["r"]:
            assert len(k) == len(ko_r) and (k == ko_r).all() and np.array_equal(d, do_r)
        bf, fx = 47.9, 435.2
        kl, dl = out["l"][-1]
        kr, dr = out["r"][-1]
        ur, dp, kept = compute_stereo_matches(exl, exr, kl, dl, kr, dr, bf, _mb(bf, fx))
        our, odp, okept = oracle_mod.compute_stereo_matches(oracle_mod.pyramid(L), oracle_mod.pyramid(R), kl, dl, kr,
                                                            dr, bf, _mb(bf, fx))
        assert kept == okept and np.array_equal(ur.view(np.uint32), our.view(np.uint32))
        exl.close()
        exr.close()
