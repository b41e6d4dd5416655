"""GPU parity of the per-frame neighbours against the CPU
oracle: MapPoint::ComputeDistinctiveDescriptors (index-exact, incl. median
ties and points past the LDS-staged size), Frame::UndistortKeyPoints
(bit-exact floats through OpenCV 3.2's double iteration), cvtColor *2GRAY and
the 16U depth conversion (byte / bit exact)."""
import numpy as np
import pytest

from orb_slam_2_ros_amd import KEYPOINT_DTYPE, compute_distinctive_descriptors, cvt_gray, undistort_keypoints
from orb_slam_2_ros_amd._lib import check, load

pytestmark = pytest.mark.gpu


def test_distinctive_descriptors_bit_exact(oracle_mod):
    from test_oracle_kat import _obs_descs
    for seed, npts, maxn in ((1, 500, 40), (2, 40, 300)):     # (300 > the 128 rows staged in LDS)
        desc, offsets = _obs_descs(seed, npts, maxn)
        g = compute_distinctive_descriptors((desc, offsets))
        o = oracle_mod.distinctive_descriptors(desc, offsets)
        assert np.array_equal(g, o)
        assert g[0] == -1 and g[1] == 0


def test_distinctive_descriptors_list_form(oracle_mod):
    rng = np.random.default_rng(9)
    descs = [rng.integers(0, 256, (n, 32)).astype(np.uint8) for n in (3, 0, 7, 64, 65, 129)]
    g = compute_distinctive_descriptors(descs)
    offsets = np.concatenate([[0], np.cumsum([len(d) for d in descs])]).astype(np.int32)
    assert np.array_equal(g, oracle_mod.distinctive_descriptors(np.concatenate(descs), offsets))


@pytest.mark.parametrize("cam", ["tum1", "euroc", "none"])
def test_undistort_keypoints_bit_exact(cam, oracle_mod):
    from test_oracle_kat import CAMERAS, _K
    c, d = CAMERAS[cam]
    rng = np.random.default_rng(11)
    kps = np.zeros(3000, KEYPOINT_DTYPE)
    kps["x"] = rng.uniform(-5, 757, 3000)
    kps["y"] = rng.uniform(-5, 485, 3000)
    kps["angle"] = rng.uniform(0, 360, 3000)
    kps["octave"] = rng.integers(0, 8, 3000)
    un = undistort_keypoints(kps, _K(c), d)
    o = oracle_mod.undistort_points(np.stack([kps["x"], kps["y"]], 1), _K(c), d)
    assert np.array_equal(un["x"].view(np.uint32), o[:, 0].view(np.uint32))
    assert np.array_equal(un["y"].view(np.uint32), o[:, 1].view(np.uint32))
    for f in ("angle", "octave", "size", "response", "class_id"):
        assert np.array_equal(un[f], kps[f])


def test_cvt_gray_host_and_batch(oracle_mod):
    import torch
    rng = np.random.default_rng(12)
    for cn in (3, 4):
        for rgb in (True, False):
            img = rng.integers(0, 256, (97, 131, cn)).astype(np.uint8)
            assert np.array_equal(cvt_gray(img, rgb), oracle_mod.cvt_gray(img, rgb))
    # batch of 5 BGRA frames (odd width, padded pitches) on device
    B, h, w, cn = 5, 61, 77, 4
    src = torch.from_numpy(rng.integers(0, 256, (B, h, 320), dtype=np.uint8)).cuda()
    dst = torch.zeros((B, h, 96), dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream()
    check(load().orbx_cvt_gray_device(src.data_ptr(), h * 320, 320, cn, 0, w, h, B, dst.data_ptr(), h * 96, 96,
                                      st.cuda_stream), "orbx_cvt_gray_device")
    torch.cuda.synchronize()
    s, d = src.cpu().numpy(), dst.cpu().numpy()
    for b in range(B):
        ref = oracle_mod.cvt_gray(s[b, :, :w * cn].reshape(h, w, cn), False)
        assert np.array_equal(d[b, :, :w], ref)
        assert not d[b, :, w:].any()                          # nothing past the row


def test_depth_to_float_batch(oracle_mod):
    import torch
    rng = np.random.default_rng(13)
    B, h, w = 3, 45, 67
    d16 = torch.from_numpy(rng.integers(0, 65536, (B, h, 72), dtype=np.uint16)).cuda()
    out = torch.zeros((B, h, 68), dtype=torch.float32, device="cuda")
    scale = np.float32(1.0) / np.float32(5000.0)
    check(load().orbx_depth_to_float_device(d16.data_ptr(), h * 72 * 2, 144, w, h, B, float(scale), out.data_ptr(),
                                            h * 68 * 4, 272, torch.cuda.current_stream().cuda_stream),
          "orbx_depth_to_float_device")
    torch.cuda.synchronize()
    s, o = d16.cpu().numpy(), out.cpu().numpy()
    for b in range(B):
        ref = oracle_mod.depth_to_float(s[b, :, :w], scale)
        assert np.array_equal(o[b, :, :w].view(np.uint32), ref.view(np.uint32))


def test_cpp_adapter_frame_aux(tmp_path, oracle_mod):
    """OrbxFrameAux::ToGray / UndistortKeyPoints through the C++ drop-in's
    cv-typed signatures."""
    import subprocess
    from cxx_build import build_adapter_test
    from test_oracle_kat import CAMERAS, _K
    rng = np.random.default_rng(21)
    w, h = 75, 41
    img = rng.integers(0, 256, (h, w, 3)).astype(np.uint8)
    kps = np.zeros(500, KEYPOINT_DTYPE)
    kps["x"] = rng.uniform(0, 640, 500)
    kps["y"] = rng.uniform(0, 480, 500)
    (tmp_path / "i.raw").write_bytes(img.tobytes())
    (tmp_path / "k.bin").write_bytes(np.int32(500).tobytes() + kps.tobytes())
    exe = build_adapter_test()
    subprocess.run([str(exe), "aux", str(w), str(h), str(tmp_path / "i.raw"), str(tmp_path / "k.bin"),
                    str(tmp_path / "o.bin")], check=True)
    buf = (tmp_path / "o.bin").read_bytes()
    gray = np.frombuffer(buf, np.uint8, w * h).reshape(h, w)
    xy = np.frombuffer(buf, np.float32, 1000, w * h).reshape(-1, 2)
    assert np.array_equal(gray, oracle_mod.cvt_gray(img, True))
    c, d = CAMERAS["tum1"]
    o = oracle_mod.undistort_points(np.stack([kps["x"], kps["y"]], 1), _K(c), np.array(d, np.float32))
    assert np.array_equal(xy.view(np.uint32), o.view(np.uint32))
