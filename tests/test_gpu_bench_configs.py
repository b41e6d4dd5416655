"""The timed kernels are the tested kernels: bench.py's own configurations,
at the batch sizes it times, checked against the oracle on
sampled streams -- first, last, both sides of the split boundary and one
stream in each XCD's frame range -- plus two size-independent properties:
every stream's output equals that of the stream showing the same scene (the
bench's 32 unique scenes), and sharding a stream set over ranks changes no
stream's output (SURVEY.md §8(e) scaling check, 1x16 vs 2x8).

Reference: ORBextractor.cc:1083-1149, ORBmatcher.cc:406-521,
Frame.cc:502-676 (stereo), Frame.cc:679-701 (RGB-D)."""
import sys
from pathlib import Path

import numpy as np
import pytest

from orb_slam_2_ros_amd import ORBextractor

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402

pytestmark = pytest.mark.gpu

BF, FX = 47.9, 435.2                               # bench.py's rig
MB = float(np.float32(BF) / np.float32(FX))


def _samples(n):
    """First, last, the split-2 boundary, and the first/last frame of every
    eighth of the batch (the XCD-contiguous frame ranges of the remap)."""
    s = {0, 1, n - 1, n // 2 - 1, n // 2}
    for x in range(8):
        s.add(x * n // 8)
        s.add(max(0, (x + 1) * n // 8 - 1))
    return sorted(i for i in s if 0 <= i < n)


def _kp_equal(a, b):
    return len(a) == len(b) and all(np.array_equal(a[f], b[f]) for f in a.dtype.names)


def _frames(torch, mode, w, h, streams):
    host, depth = bench._resident_frames(mode, w, h, streams)
    dev = torch.device("cuda:0")
    fr = torch.from_numpy(host).to(dev)
    dm = torch.from_numpy(depth).to(dev) if depth is not None else None
    torch.cuda.synchronize()
    return host, depth, fr, dm


def test_mono_bench_config_b3072(oracle_mod):
    """The headline timed region: 3072 VGA streams, split and level pipeline as
    bench.py runs them, two steps (the second matches against the first)."""
    import torch
    w, h, B = 640, 480, 3072
    streams = list(range(B))
    host, _, fr, _ = _frames(torch, "mono", w, h, streams)
    ex = ORBextractor(1000, 1.2, 8, 20, 7)
    ex.reserve(w, h, B)
    ex.split(bench.HEADLINE_SPLIT)
    ex.pipeline(bench.HEADLINE_PIPE)   # (as bench.py times it)
    ex.overlap_match(bench.MONO_OVERLAP)
    assert ex.split() == bench.HEADLINE_SPLIT
    for t in range(2):
        ex.mono_step_device(fr[t].data_ptr(), w * h, w, B, 100, 0.9, True)
    torch.cuda.synchronize()
    outs = [ex.batch_download(b) for b in range(B)]
    matches = [ex.mono_matches_download(b) for b in range(B)]
    # every stream equals the stream that shows the same scene
    for b in range(B):
        r = bench.stream_scene(b)
        assert _kp_equal(outs[b][0], outs[r][0]) and np.array_equal(outs[b][1], outs[r][1]), f"stream {b}"
        assert matches[b][1] == matches[r][1] and np.array_equal(matches[b][0], matches[r][0]), f"stream {b}"
    for b in _samples(B):
        k1, d1 = oracle_mod.extract(host[0, b])
        k2, d2 = oracle_mod.extract(host[1, b])
        assert _kp_equal(outs[b][0], k2) and np.array_equal(outs[b][1], d2), f"stream {b} extract"
        prev = np.ascontiguousarray(np.stack([k1["x"], k1["y"]], 1).astype(np.float32))
        nm, m12, _ = oracle_mod.search_for_initialization(k1, d1, k2, d2, w, h, prev, 100, 0.9, True)
        assert matches[b][1] == nm and np.array_equal(matches[b][0], m12), f"stream {b} matches"
        assert nm > 0
    ex.close()


def test_mono_overlap_match_steps(oracle_mod):
    """Matcher overlap (orbx_extractor_overlap_match): four mono steps issued
    back to back, each step's matcher on the internal stream beside the next
    step's extraction (whose descriptor stage waits for it); the last step's
    matches and keypoints equal the oracle's on sampled streams, and the same
    extractor without the overlap gives the same matches for every stream."""
    import torch
    w, h, B = 640, 480, 3072
    host, _, fr, _ = _frames(torch, "mono", w, h, list(range(B)))
    res = []
    for ovl in (1, 0):
        ex = ORBextractor(1000, 1.2, 8, 20, 7)
        ex.reserve(w, h, B)
        ex.split(bench.HEADLINE_SPLIT)
        ex.pipeline(bench.HEADLINE_PIPE)
        assert ex.overlap_match(ovl) == ovl and ex.overlap_match() == ovl
        for t in range(4):
            ex.mono_step_device(fr[t].data_ptr(), w * h, w, B, 100, 0.9, True)
        torch.cuda.synchronize()
        res.append(([ex.mono_matches_download(b) for b in range(B)], [ex.batch_download(b) for b in _samples(B)]))
        ex.close()
    (m_ovl, o_ovl), (m_ref, o_ref) = res
    for b in range(B):
        assert m_ovl[b][1] == m_ref[b][1] and np.array_equal(m_ovl[b][0], m_ref[b][0]), f"stream {b}"
    for j, b in enumerate(_samples(B)):
        k1, d1 = oracle_mod.extract(host[2, b])
        k2, d2 = oracle_mod.extract(host[3, b])
        assert _kp_equal(o_ovl[j][0], k2) and np.array_equal(o_ovl[j][1], d2), f"stream {b} extract"
        prev = np.ascontiguousarray(np.stack([k1["x"], k1["y"]], 1).astype(np.float32))
        nm, m12, _ = oracle_mod.search_for_initialization(k1, d1, k2, d2, w, h, prev, 100, 0.9, True)
        assert m_ovl[b][1] == nm and np.array_equal(m_ovl[b][0], m12), f"stream {b} matches"
        assert nm > 0


def test_mono_overlap_transitions(oracle_mod):
    """The matcher overlap's state changes on one extractor, each phase checked
    against the oracle: overlapped steps, then overlap off (the matcher waits on
    the last overlapped one), profiling on mid-sequence (falls back to the
    non-overlapped path), overlap on again, the host-image call on the same
    handle right after an overlapped step (its graph capture must not wait on
    the overlapped matcher's event), then a reserve at a new batch size (frees
    the slots the matcher reads)."""
    import torch
    w, h, B = 640, 480, 64
    # 2 B resident streams (the last phase's batch); the earlier phases use the first B
    host, _, fr, _ = _frames(torch, "mono", w, h, list(range(2 * B)))
    ex = ORBextractor(1000, 1.2, 8, 20, 7)
    ex.reserve(w, h, B)
    ex.split(2)
    smp = [0, 31, 32, 63, 64, 127]

    def step_and_check(t, nb=B, tag=""):
        ex.mono_step_device(fr[t % 4].data_ptr(), w * h, w, nb, 100, 0.9, True)
        torch.cuda.synchronize()
        for b in smp:
            if b >= nb:
                continue
            kp, de = ex.batch_download(b)
            m12, nm = ex.mono_matches_download(b)
            k1, d1 = oracle_mod.extract(host[(t - 1) % 4, b])
            k2, d2 = oracle_mod.extract(host[t % 4, b])
            assert _kp_equal(kp, k2) and np.array_equal(de, d2), f"{tag} step {t} stream {b} extract"
            prev = np.ascontiguousarray(np.stack([k1["x"], k1["y"]], 1).astype(np.float32))
            onm, om12, _ = oracle_mod.search_for_initialization(k1, d1, k2, d2, w, h, prev, 100, 0.9, True)
            assert nm == onm and np.array_equal(m12, om12), f"{tag} step {t} stream {b} matches"

    ex.overlap_match(1)
    for t in range(3):
        ex.mono_step_device(fr[t].data_ptr(), w * h, w, B, 100, 0.9, True)
    step_and_check(3, tag="overlap")
    ex.overlap_match(0)
    step_and_check(4, tag="overlap->off")
    ex.overlap_match(1)
    ex.mono_step_device(fr[1].data_ptr(), w * h, w, B, 100, 0.9, True)
    ex.set_profiling(True)
    step_and_check(6, tag="profiling")
    assert all(x >= 0 for x in ex.stage_times()[:1])
    ex.set_profiling(False)
    step_and_check(7, tag="overlap again")
    # the deep level pipeline on the same handle (and through the host call below, whose
    # graph is captured with the pipeline off and must leave the setting as it was)
    assert ex.pipeline(2) == 2
    step_and_check(8, tag="deep pipeline")
    # the host-image call right after an overlapped step (no synchronisation between)
    ex.mono_step_device(fr[0].data_ptr(), w * h, w, B, 100, 0.9, True)
    img = np.ascontiguousarray(host[2, 5])
    kp, de = ex(img)
    ok, od = oracle_mod.extract(img)
    assert _kp_equal(kp, ok) and np.array_equal(de, od), "host call after an overlapped step"
    assert ex.pipeline() == 2
    # and back to the device path, then a reserve at another batch size
    ex.mono_step_device(fr[0].data_ptr(), w * h, w, B, 100, 0.9, True)
    step_and_check(1, tag="after host call")
    ex.mono_step_device(fr[2].data_ptr(), w * h, w, B, 100, 0.9, True)
    ex.reserve(w, h, 2 * B)
    ex.mono_step_device(fr[2].data_ptr(), w * h, w, 2 * B, 100, 0.9, True)
    step_and_check(3, nb=2 * B, tag="reserve")
    ex.close()


@pytest.mark.parametrize("mode,w,h,nf,B", [("mono", 640, 480, 1000, 256), ("stereo", 1920, 1080, 1000, 32),
                                            ("mono", 1241, 376, 2000, 64)])
def test_deep_level_pipeline(mode, w, h, nf, B, oracle_mod):
    """The deep level pipeline (orbx_extractor_pipeline(2): FAST / quadtree of
    levels 1..E on the side stream as the resize chain produces them, E =
    ORBX_PIPE_EARLY; their describe there too with ORBX_PIPE_DESC=1) gives
    byte-identical keypoints, descriptors and matches / depths to the
    unpipelined step for every stream and E in 1..3, and the oracle's on
    sampled streams; split 2 as well (each part pipelined)."""
    import os
    import torch
    host, _, fr, _ = _frames(torch, mode, w, h, list(range(B)))
    frames = 2 * B if mode == "stereo" else B

    def run(pipe, early, split, desc=0):
        saved = {k: os.environ.get(k) for k in ("ORBX_PIPE_EARLY", "ORBX_PIPE_DESC")}
        os.environ["ORBX_PIPE_EARLY"] = str(early)   # (read at extractor creation)
        os.environ["ORBX_PIPE_DESC"] = str(desc)
        try:
            ex = ORBextractor(nf, 1.2, 8, 20, 7)
        finally:
            for k, v in saved.items():
                if v is None:
                    del os.environ[k]
                else:
                    os.environ[k] = v
        ex.reserve(w, h, frames)
        ex.split(split)
        assert ex.pipeline(pipe) == pipe
        for t in range(2):
            if mode == "mono":
                ex.mono_step_device(fr[t].data_ptr(), w * h, w, B, 100, 0.9, True)
            else:
                ex.stereo_step_device(fr[t].data_ptr(), w * h, w, B, BF, MB)
        torch.cuda.synchronize()
        kd = [ex.batch_download(b) for b in range(frames)]
        extra = [ex.mono_matches_download(b) if mode == "mono" else ex.depth_download(b) for b in range(B)]
        ex.close()
        return kd, extra

    ref_kd, ref_x = run(0, 2, 1)
    for pipe, early, split, desc in [(2, 1, 1, 0), (2, 2, 1, 0), (2, 3, 1, 0), (2, 2, 2, 0), (2, 2, 1, 1), (2, 3, 2, 1)]:
        kd, x = run(pipe, early, split, desc)
        for b in range(frames):
            assert _kp_equal(kd[b][0], ref_kd[b][0]) and np.array_equal(kd[b][1], ref_kd[b][1]), \
                f"pipe {pipe} E {early} split {split} frame {b}"
        for b in range(B):
            assert all(np.array_equal(np.asarray(u), np.asarray(v)) for u, v in zip(x[b], ref_x[b])), \
                f"pipe {pipe} E {early} split {split} stream {b}"
    for b in (0, B - 1):
        k2, d2 = oracle_mod.extract(host[1, b], nf) if mode == "mono" else oracle_mod.extract(host[1, 2 * b], nf)
        f = b if mode == "mono" else 2 * b
        assert _kp_equal(ref_kd[f][0], k2) and np.array_equal(ref_kd[f][1], d2), f"frame {f} vs oracle"


MONO_EXTRAS = [(w, h, nf, B) for key, mode, w, h, nf, B, _ in bench.EXTRAS if mode == "mono"]


@pytest.mark.parametrize("w,h,nf,B", MONO_EXTRAS)
def test_mono_extra_bench_configs(w, h, nf, B, oracle_mod):
    """The mono extras at the batches and split / pipeline settings bench.py
    times them (HD 1280x720 at 384 streams, FHD at 192, both unsplit): two
    steps, every stream equal to its scene's, sampled streams vs the oracle."""
    import torch
    key = next(k for k, m, ww, hh, _, _, _ in bench.EXTRAS if m == "mono" and (ww, hh) == (w, h))
    streams = list(range(B))
    host, _, fr, _ = _frames(torch, "mono", w, h, streams)
    ex = ORBextractor(nf, 1.2, 8, 20, 7)
    ex.reserve(w, h, B)
    ex.split(bench.EXTRA_SPLIT.get(key, 2))   # (as bench.py times it)
    ex.pipeline(bench.EXTRA_PIPE.get(key, 0))
    ex.overlap_match(bench.MONO_OVERLAP)
    for t in range(2):
        ex.mono_step_device(fr[t].data_ptr(), w * h, w, B, 100, 0.9, True)
    torch.cuda.synchronize()
    outs = [ex.batch_download(b) for b in range(B)]
    matches = [ex.mono_matches_download(b) for b in range(B)]
    for b in range(B):
        r = bench.stream_scene(b)
        assert _kp_equal(outs[b][0], outs[r][0]) and np.array_equal(outs[b][1], outs[r][1]), f"stream {b}"
        assert matches[b][1] == matches[r][1] and np.array_equal(matches[b][0], matches[r][0]), f"stream {b}"
    for b in [0, 1, B // 2 - 1, B // 2, B - 1]:
        k1, d1 = oracle_mod.extract(host[0, b], nf)
        k2, d2 = oracle_mod.extract(host[1, b], nf)
        assert _kp_equal(outs[b][0], k2) and np.array_equal(outs[b][1], d2), f"stream {b} extract"
        prev = np.ascontiguousarray(np.stack([k1["x"], k1["y"]], 1).astype(np.float32))
        nm, m12, _ = oracle_mod.search_for_initialization(k1, d1, k2, d2, w, h, prev, 100, 0.9, True)
        assert matches[b][1] == nm and np.array_equal(matches[b][0], m12), f"stream {b} matches"
        assert nm > 0
    ex.close()


STEREO_CONFIGS = [   # bench.py EXTRAS: (w, h, nfeatures, pairs, split, level pipeline as bench.py runs it)
    (752, 480, 1200, 256, 2, 0),
    (1241, 376, 2000, 144, 2, 0),
    (1920, 1080, 1000, 192, 1, 1),
    (752, 480, 1200, 32, 2, 1),   # (the level pipeline on a small split stereo step)
]


@pytest.mark.parametrize("w,h,nf,P,split,pipe", STEREO_CONFIGS)
def test_stereo_bench_configs(w, h, nf, P, split, pipe, oracle_mod):
    import torch
    streams = list(range(P))
    host, _, fr, _ = _frames(torch, "stereo", w, h, streams)
    ex = ORBextractor(nf, 1.2, 8, 20, 7)
    ex.reserve(w, h, 2 * P)
    ex.split(split)   # (as bench.py times it)
    ex.pipeline(pipe)
    ex.stereo_step_device(fr[1].data_ptr(), w * h, w, P, BF, MB)
    torch.cuda.synchronize()
    deps = [ex.depth_download(p) for p in range(P)]
    for p in range(P):
        r = bench.stream_scene(p)
        assert np.array_equal(deps[p][0], deps[r][0]) and deps[p][2] == deps[r][2]
    samples = _samples(P) if w < 1920 else [0, 1, P // 2, P - 1]
    for p in samples:
        L, R = host[1, 2 * p], host[1, 2 * p + 1]
        kl, dl = ex.batch_download(2 * p)
        kr, dr = ex.batch_download(2 * p + 1)
        ko, do = oracle_mod.extract(L, nf)
        kro, dro = oracle_mod.extract(R, nf)
        assert _kp_equal(kl, ko) and np.array_equal(dl, do), f"pair {p} left"
        assert _kp_equal(kr, kro) and np.array_equal(dr, dro), f"pair {p} right"
        our, odp, okept = oracle_mod.compute_stereo_matches(oracle_mod.pyramid(L), oracle_mod.pyramid(R), ko, do,
                                                            kro, dro, BF, MB)
        ur, dp, kept = deps[p]
        assert kept == okept and kept > 0, f"pair {p}"
        assert np.array_equal(ur.view(np.uint32), our.view(np.uint32)), f"pair {p} mvuRight"
        assert np.array_equal(dp.view(np.uint32), odp.view(np.uint32)), f"pair {p} mvDepth"
    ex.close()


@pytest.mark.parametrize("B", [192, 64])
def test_rgbd_fhd_bench_configs(B, oracle_mod):
    """RGB-D FHD at the bench's 192 streams per GPU, and C5's 64 streams as
    one GPU runs them."""
    import torch
    w, h = 1920, 1080
    streams = list(range(B))
    host, depth, fr, dm = _frames(torch, "rgbd", w, h, streams)
    ex = ORBextractor(1000, 1.2, 8, 20, 7)
    ex.reserve(w, h, B)
    ex.split(bench.EXTRA_SPLIT.get("rgbd_fhd_1920x1080", 2) if B == 192 else 2)   # (as bench.py times it)
    ex.pipeline(bench.EXTRA_PIPE.get("rgbd_fhd_1920x1080", 0) if B == 192 else 0)
    ex.rgbd_step_device(fr[2].data_ptr(), w * h, w, B, dm.data_ptr(), 4 * w * h, 4 * w, BF)
    torch.cuda.synchronize()
    for b in [0, 1, B // 2 - 1, B // 2, B - 1]:
        kg, dg = ex.batch_download(b)
        ko, do = oracle_mod.extract(host[2, b])
        assert _kp_equal(kg, ko) and np.array_equal(dg, do), f"frame {b}"
        ur, dp, kept = ex.depth_download(b)
        our, odp = oracle_mod.stereo_from_rgbd(ko, depth[b], BF)
        assert np.array_equal(ur.view(np.uint32), our.view(np.uint32))
        assert np.array_equal(dp.view(np.uint32), odp.view(np.uint32))
        assert kept == int((odp > 0).sum()) and kept > 0
    ex.close()


def _run_streams(torch, mode, w, h, nf, streams, steps):
    """One extractor (one 'rank') stepping its streams; per-stream outputs."""
    host, depth, fr, dm = _frames(torch, mode, w, h, streams)
    n = len(streams)
    ex = ORBextractor(nf, 1.2, 8, 20, 7)
    ex.reserve(w, h, 2 * n if mode == "stereo" else n)
    for t in range(steps):
        if mode == "mono":
            ex.mono_step_device(fr[t].data_ptr(), w * h, w, n, 100, 0.9, True)
        elif mode == "rgbd":
            ex.rgbd_step_device(fr[t].data_ptr(), w * h, w, n, dm.data_ptr(), 4 * w * h, 4 * w, BF)
        else:
            ex.stereo_step_device(fr[t].data_ptr(), w * h, w, n, BF, MB)
    torch.cuda.synchronize()
    out = {}
    for b, s in enumerate(streams):
        if mode == "mono":
            k, d = ex.batch_download(b)
            m, nm = ex.mono_matches_download(b)
            out[s] = (k.tobytes(), d.tobytes(), m.tobytes(), nm)
        elif mode == "rgbd":
            k, d = ex.batch_download(b)
            ur, dp, kept = ex.depth_download(b)
            out[s] = (k.tobytes(), d.tobytes(), ur.tobytes(), dp.tobytes(), kept)
        else:
            k, d = ex.batch_download(2 * b)
            ur, dp, kept = ex.depth_download(b)
            out[s] = (k.tobytes(), d.tobytes(), ur.tobytes(), dp.tobytes(), kept)
    ex.close()
    return out


@pytest.mark.parametrize("mode,w,h,nf,total,world", [("mono", 640, 480, 1000, 16, 2),
                                                      ("mono", 640, 480, 1000, 16, 4),
                                                      ("stereo", 752, 480, 1200, 8, 2),
                                                      ("rgbd", 1920, 1080, 1000, 64, 8)])
def test_sharding_changes_no_stream(mode, w, h, nf, total, world):
    """per-frame outputs at G ranks are byte-identical to
    G = 1.  Each rank's share (stream s -> rank s mod G, bench.stream_partition)
    runs as its own batch, as bench.py's ranks run it.  The RGB-D case is C5's
    64 FHD streams as 1 x 64 against 8 x 8 (streams past the 32 scenes repeat
    them)."""
    import torch
    whole = _run_streams(torch, mode, w, h, nf, list(range(total)), 3)
    for r in range(world):
        part = bench.stream_partition(total, world, r)
        got = _run_streams(torch, mode, w, h, nf, part, 3)
        for s in part:
            assert got[s] == whole[s], f"stream {s} differs on rank {r} of {world}"
    # the streams really are distinct (up to the scene count)
    assert len({v[0] for v in whole.values()}) == min(total, bench.UNIQUE_SCENES)


def test_pack_device_equals_download():
    """orbx_batch_pack_device (the keyframe exchange's send buffer, config C5)
    holds exactly what orbx_batch_download returns for every stream: counts,
    then keypoint records and descriptors at kp_stride per stream."""
    import torch
    w, h, B = 1920, 1080, 8
    host, depth, fr, dm = _frames(torch, "rgbd", w, h, list(range(B)))
    ex = ORBextractor(1000, 1.2, 8, 20, 7)
    ex.reserve(w, h, B)
    ex.rgbd_step_device(fr[0].data_ptr(), w * h, w, B, dm.data_ptr(), 4 * w * h, 4 * w, BF)
    nbytes = ex.pack_bytes()
    buf = torch.full((nbytes + 256,), 0xAB, dtype=torch.uint8, device="cuda:0")
    assert ex.pack_device(buf.data_ptr(), nbytes) == nbytes
    torch.cuda.synchronize()
    raw = buf.cpu().numpy()
    assert (raw[nbytes:] == 0xAB).all()                 # nothing past the reported size
    K = ex.kp_stride()
    from orb_slam_2_ros_amd._lib import KEYPOINT_DTYPE
    coff = ((4 * B + 63) // 64) * 64
    counts = raw[:4 * B].view(np.int32)
    kps = raw[coff:coff + B * K * KEYPOINT_DTYPE.itemsize].view(KEYPOINT_DTYPE).reshape(B, K)
    desc = raw[coff + B * K * KEYPOINT_DTYPE.itemsize:nbytes].reshape(B, K, 32)
    assert nbytes == coff + B * K * (KEYPOINT_DTYPE.itemsize + 32)
    for b in range(B):
        k, d = ex.batch_download(b)
        assert counts[b] == len(k) > 0, f"stream {b}"
        assert kps[b, :len(k)].tobytes() == k.tobytes(), f"stream {b} keypoints"
        assert np.array_equal(desc[b, :len(k)], d), f"stream {b} descriptors"
    ex.close()
