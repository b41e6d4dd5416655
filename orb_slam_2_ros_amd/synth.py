"""Seeded synthetic grayscale scenes for parity tests and the benchmark.

There are no images in the reference tree, so every test and
bench input is generated here (SURVEY.md §8(d) "Synthetic inputs"):

* background: value noise on a 16-px lattice, intensities U[40, 215], bilinear
  upsampled, then a 3x3 box blur;
* W*H/2000 axis-aligned rectangles and discs with intensity U[0, 255];
* i.i.d. noise U{-3..3} per frame, clamped to [0, 255].

A *stream* is a fixed scene canvas; frame t is the W x H crop at offset
(3t, 2t) (mod the canvas margin) with fresh noise, so consecutive frames
overlap with a (-3, -2) px motion and real matches exist.  A stereo right
image is the left crop shifted by a 20-px disparity.
"""
from __future__ import annotations

import numpy as np

MARGIN = 64


def _scene(width: int, height: int, seed: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    lat = 16
    gh, gw = height // lat + 2, width // lat + 2
    grid = rng.uniform(40.0, 215.0, size=(gh, gw))
    ys = np.arange(height) / lat
    xs = np.arange(width) / lat
    y0 = np.floor(ys).astype(np.int64)
    x0 = np.floor(xs).astype(np.int64)
    fy = (ys - y0)[:, None]
    fx = (xs - x0)[None, :]
    g00 = grid[y0][:, x0]
    g01 = grid[y0][:, x0 + 1]
    g10 = grid[y0 + 1][:, x0]
    g11 = grid[y0 + 1][:, x0 + 1]
    img = (g00 * (1 - fx) + g01 * fx) * (1 - fy) + (g10 * (1 - fx) + g11 * fx) * fy
    pad = np.pad(img, 1, mode="edge")
    img = sum(pad[dy:dy + height, dx:dx + width] for dy in range(3) for dx in range(3)) / 9.0
    nshapes = max(1, (width * height) // 2000)
    yy, xx = np.mgrid[0:height, 0:width]
    for _ in range(nshapes):
        val = rng.uniform(0.0, 255.0)
        cx, cy = rng.integers(0, width), rng.integers(0, height)
        if rng.random() < 0.5:
            hw, hh = rng.integers(3, 40), rng.integers(3, 40)
            img[max(cy - hh, 0):cy + hh, max(cx - hw, 0):cx + hw] = val
        else:
            r = int(rng.integers(3, 30))
            y_lo, y_hi = max(cy - r, 0), min(cy + r + 1, height)
            x_lo, x_hi = max(cx - r, 0), min(cx + r + 1, width)
            sub_y, sub_x = yy[y_lo:y_hi, x_lo:x_hi], xx[y_lo:y_hi, x_lo:x_hi]
            m = (sub_y - cy) ** 2 + (sub_x - cx) ** 2 <= r * r
            img[y_lo:y_hi, x_lo:x_hi][m] = val
    return img


def stream_canvas(width: int, height: int, seed: int) -> np.ndarray:
    """Float scene canvas of (height + MARGIN, width + MARGIN) for one stream."""
    return _scene(width + MARGIN, height + MARGIN, seed)


def frame_from_canvas(canvas: np.ndarray, width: int, height: int, t: int, noise_seed: int,
                      disparity: int = 0) -> np.ndarray:
    ox = (3 * t) % (MARGIN - 24) + disparity
    oy = (2 * t) % (MARGIN - 24)
    crop = canvas[oy:oy + height, ox:ox + width]
    rng = np.random.default_rng(noise_seed)
    noise = rng.integers(-3, 4, size=crop.shape)
    return np.clip(np.rint(crop) + noise, 0, 255).astype(np.uint8)


def frame(width: int, height: int, seed: int, t: int = 0) -> np.ndarray:
    """Frame t of stream `seed` (u8, C-contiguous)."""
    canvas = stream_canvas(width, height, seed)
    return np.ascontiguousarray(frame_from_canvas(canvas, width, height, t, seed * 7919 + t))


def frames(width: int, height: int, seed: int, count: int) -> np.ndarray:
    """`count` consecutive frames of one stream, shape (count, height, width)."""
    canvas = stream_canvas(width, height, seed)
    out = np.empty((count, height, width), dtype=np.uint8)
    for t in range(count):
        out[t] = frame_from_canvas(canvas, width, height, t, seed * 7919 + t)
    return out


def stereo_pair(width: int, height: int, seed: int, t: int = 0, disparity: int = 20):
    """Rectified (left, right) pair of stream `seed` at time t: the right image
    is the left crop shifted by `disparity` px (u_R = u_L - disparity), with
    its own noise."""
    canvas = stream_canvas(width, height, seed)
    left = frame_from_canvas(canvas, width, height, t, seed * 7919 + t)
    right = frame_from_canvas(canvas, width, height, t, seed * 7919 + t + 500009, disparity=disparity)
    return np.ascontiguousarray(left), np.ascontiguousarray(right)


def depth_map(width: int, height: int, seed: int, z: float = 1.5) -> np.ndarray:
    """float32 depth image: a plane at z metres with a tilted patch and a few
    invalid (0 / NaN) pixels, as an RGB-D sensor delivers."""
    rng = np.random.default_rng(seed)
    d = np.full((height, width), z, np.float32)
    yy, xx = np.mgrid[0:height, 0:width]
    d += (0.0005 * (xx - width / 2) + 0.0003 * (yy - height / 2)).astype(np.float32)
    holes = rng.random((height, width)) < 0.02
    d[holes] = 0.0
    d[rng.random((height, width)) < 0.005] = np.nan
    return d


def scale_tables(scale=1.2, nlevels=8):
    """mvScaleFactor / mvInvScaleFactor (ORBextractor.cc:424-438): float
    products computed in double (the member scaleFactor is a double)."""
    sf = np.zeros(nlevels, np.float32)
    sf[0] = 1.0
    for i in range(1, nlevels):
        sf[i] = np.float32(float(sf[i - 1]) * float(np.float32(scale)))
    inv = (np.float32(1.0) / sf).astype(np.float32)
    return sf, inv
