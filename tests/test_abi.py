"""C-ABI checks that need no GPU: liborbx.so builds, loads and exports every
function include/orbx.h declares; host-only entry points behave; the product
fails loudly (no CPU fallback) when no device is present."""
import re
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]


def _declared():
    text = (ROOT / "include" / "orbx.h").read_text()
    return sorted(set(re.findall(r"\b(orbx_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_what_binding_uses():
    from orb_slam_2_ros_amd import _lib
    assert sorted(_lib.EXPORTED) == _declared()


def test_library_exports_every_declared_symbol():
    import ctypes
    from orb_slam_2_ros_amd import _lib
    lib = ctypes.CDLL(str(_lib.LIB_PATH))
    missing = [s for s in _declared() if not hasattr(lib, s)]
    assert not missing, missing


def test_descriptor_distance_host_path(oracle_mod):
    from orb_slam_2_ros_amd import ORBmatcher
    rng = np.random.default_rng(5)
    for _ in range(100):
        a, b = rng.integers(0, 256, (2, 32)).astype(np.uint8)
        assert ORBmatcher.DescriptorDistance(a, b) == oracle_mod.descriptor_distance(a, b)


def test_strerror_codes():
    from orb_slam_2_ros_amd import _lib
    lib = _lib.load()
    assert lib.orbx_strerror(0) == b"ok"
    assert b"capacity" in lib.orbx_strerror(_lib.ORBX_ERANGE)
    assert b"invalid" in lib.orbx_strerror(_lib.ORBX_EINVAL)


def test_keypoint_layout_is_cv_keypoint():
    from orb_slam_2_ros_amd import KEYPOINT_DTYPE
    assert KEYPOINT_DTYPE.itemsize == 28
    assert KEYPOINT_DTYPE.names == ("x", "y", "size", "angle", "response", "octave", "class_id")


def test_no_device_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("device present")
    from orb_slam_2_ros_amd import ORBextractor, OrbxError
    with pytest.raises(OrbxError):
        ORBextractor(1000, 1.2, 8, 20, 7)


def test_cpp_dropin_adapter_compiles_and_links():
    """include/orbx_orbslam2.hpp keeps ORB_SLAM2::ORBextractor's signatures; it
    must compile, link against liborbx.so and, without a device, fail loudly."""
    import subprocess
    import torch
    from cxx_build import build_adapter_test
    exe = build_adapter_test()
    out = subprocess.run([str(exe), "probe"], capture_output=True, text=True, check=True).stdout
    if not torch.cuda.is_available():
        assert out.strip() == "nodevice"
    else:
        assert out.startswith("levels 8")


def test_pattern_stays_inside_blur_window():
    """k_describe blurs only the 37x37 window (|offset| <= 18) around a key:
    every rotated sample cvRound(x*b + y*a) must land inside it for every angle,
    i.e. every pattern point lies strictly within radius 18.5."""
    import re as _re
    txt = (ROOT / "orb_slam_2_ros_amd" / "csrc" / "orb_pattern.inc").read_text()
    pts = np.array([[int(a), int(b)] for a, b in _re.findall(r"\{\s*(-?\d+),\s*(-?\d+)\}", txt)])
    assert pts.shape == (512, 2)
    assert float(np.sqrt((pts.astype(float) ** 2).sum(1)).max()) < 18.5 - 1e-3
