#!/usr/bin/env python3
"""Writes tests/golden/*.npz: oracle outputs on seeded synthetic frames.

These are REGRESSION fixtures of this project's CPU restatement (oracle/),
not reference-produced vectors: the reference has none and cannot be built
here (parity unpinned).  They freeze the oracle's behaviour so
any later change to it -- or to the GPU path -- is caught without re-deriving.
Inputs are regenerated from (w, h, seed) by orb_slam_2_ros_amd.synth; the
input's SHA-256 is stored to detect generator drift.
"""
import hashlib
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from orb_slam_2_ros_amd import synth  # noqa: E402
from oracle import oracle  # noqa: E402

CASES = [
    # name, w, h, nfeatures, seed
    ("vga_1000", 640, 480, 1000, 21),
    ("euroc_1200", 752, 480, 1200, 22),
    ("kitti_2000", 1241, 376, 2000, 23),
    ("qvga_500", 320, 240, 500, 24),
]


def main():
    out = Path(__file__).resolve().parent
    for name, w, h, nf, seed in CASES:
        f0 = synth.frame(w, h, seed, 0)
        f1 = synth.frame(w, h, seed, 1)
        k0, d0 = oracle.extract(f0, nf)
        k1, d1 = oracle.extract(f1, nf)
        prev = np.ascontiguousarray(np.stack([k0["x"], k0["y"]], 1).astype(np.float32))
        nm, m12, prev2 = oracle.search_for_initialization(k0, d0, k1, d1, w, h, prev, 100, 0.9, True)
        np.savez_compressed(out / f"{name}.npz", w=w, h=h, nfeatures=nf, seed=seed,
                            sha0=hashlib.sha256(f0.tobytes()).hexdigest(),
                            sha1=hashlib.sha256(f1.tobytes()).hexdigest(),
                            kps0=k0, desc0=d0, kps1=k1, desc1=d1, nmatches=nm, matches12=m12, prev_after=prev2)
        print(name, len(k0), len(k1), nm)


if __name__ == "__main__":
    main()
