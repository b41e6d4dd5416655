"""SearchForInitialization over a distorted camera's grid bounds.

Frame::ComputeImageBounds (Frame.cc:475-499) leaves mnMinX .. mnMaxY non-zero
and non-integer when the camera has distortion; PosInGrid rounds
(x - mnMinX) * inv (Frame.cc:415-425) and GetFeaturesInArea floors / ceils
(x - mnMinX -/+ r) * inv (:361-373).  The oracle restates that arithmetic; the
GPU test holds liborbx to it bit for bit.
"""
import numpy as np
import pytest

from orb_slam_2_ros_amd import KEYPOINT_DTYPE

W, H = 640, 480
BOUNDS = [(-13.37, 661.61, 7.25, 476.17), (-0.5, 639.5, -2.75, 481.3), (21.9, 603.3, 11.1, 455.6)]


def _frames(seed, n1=700, n2=760, pool=24):
    rng = np.random.default_rng(seed)
    base = rng.integers(0, 256, (pool, 32)).astype(np.uint8)

    def frame(n):
        k = np.zeros(n, KEYPOINT_DTYPE)
        # undistorted keypoints spill past the image on every side
        k["x"] = rng.uniform(-20, W + 25, n).astype(np.float32)
        k["y"] = rng.uniform(-10, H + 12, n).astype(np.float32)
        k["octave"] = rng.choice([0, 0, 0, 1], n)
        k["angle"] = rng.uniform(0, 360, n).astype(np.float32)
        k["class_id"] = -1
        d = base[rng.integers(0, pool, n)].copy()
        d[np.arange(n), rng.integers(0, 32, n)] ^= rng.integers(0, 8, n).astype(np.uint8)
        return k, d
    return frame(n1), frame(n2)


def _prev(k1):
    return np.ascontiguousarray(np.stack([k1["x"], k1["y"]], 1).astype(np.float32))


def test_oracle_bounds_default_equals_image_size(oracle_mod):
    (k1, d1), (k2, d2) = _frames(3)
    a = oracle_mod.search_for_initialization(k1, d1, k2, d2, W, H, _prev(k1), 100, 0.9, True)
    b = oracle_mod.search_for_initialization(k1, d1, k2, d2, W, H, _prev(k1), 100, 0.9, True,
                                             bounds=(0.0, W, 0.0, H))
    assert a[0] == b[0] and np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2])


def test_oracle_bounds_change_the_grid(oracle_mod):
    """The bounds are not cosmetic: on these frames they change the matches
    (grid membership of the spilled keypoints and the window cells)."""
    (k1, d1), (k2, d2) = _frames(4)
    base = oracle_mod.search_for_initialization(k1, d1, k2, d2, W, H, _prev(k1), 30, 0.9, True)
    differs = 0
    for bnd in BOUNDS:
        r = oracle_mod.search_for_initialization(k1, d1, k2, d2, W, H, _prev(k1), 30, 0.9, True, bounds=bnd)
        differs += not np.array_equal(r[1], base[1])
    assert differs >= 2


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [5, 6])
@pytest.mark.parametrize("bounds", BOUNDS)
def test_search_for_initialization_bounds_gpu(seed, bounds, oracle_mod):
    from orb_slam_2_ros_amd import Frame, ORBmatcher
    (k1, d1), (k2, d2) = _frames(seed)
    for window, ratio, ori in [(100, 0.9, True), (30, 0.9, True), (60, 0.7, False)]:
        prev = _prev(k1)
        nm_o, m_o, prev_o = oracle_mod.search_for_initialization(k1, d1, k2, d2, W, H, prev, window, ratio, ori,
                                                                 bounds=bounds)
        nm_g, m_g = ORBmatcher(ratio, ori).SearchForInitialization(
            Frame(k1, d1, W, H, bounds=bounds), Frame(k2, d2, W, H, bounds=bounds), prev, window)
        assert nm_g == nm_o and np.array_equal(m_g, m_o) and np.array_equal(prev, prev_o)
