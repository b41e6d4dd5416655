"""Regression fixtures (tests/golden/, made by make_golden.py from the oracle):
the CPU restatement must keep reproducing them, and so must the GPU path."""
import hashlib
from pathlib import Path

import numpy as np
import pytest

from orb_slam_2_ros_amd import synth

GOLD = sorted((Path(__file__).resolve().parent / "golden").glob("*.npz"))


def _load(p):
    z = np.load(p, allow_pickle=False)
    return {k: z[k] for k in z.files}


def _frames(g):
    w, h, seed = int(g["w"]), int(g["h"]), int(g["seed"])
    f0, f1 = synth.frame(w, h, seed, 0), synth.frame(w, h, seed, 1)
    assert hashlib.sha256(f0.tobytes()).hexdigest() == str(g["sha0"]), "synthetic generator drifted"
    assert hashlib.sha256(f1.tobytes()).hexdigest() == str(g["sha1"]), "synthetic generator drifted"
    return w, h, f0, f1


@pytest.mark.parametrize("path", GOLD, ids=[p.stem for p in GOLD])
def test_oracle_reproduces_golden(path, oracle_mod):
    g = _load(path)
    w, h, f0, f1 = _frames(g)
    nf = int(g["nfeatures"])
    k0, d0 = oracle_mod.extract(f0, nf)
    k1, d1 = oracle_mod.extract(f1, nf)
    assert (k0 == g["kps0"]).all() and np.array_equal(d0, g["desc0"])
    assert (k1 == g["kps1"]).all() and np.array_equal(d1, g["desc1"])
    prev = np.ascontiguousarray(np.stack([k0["x"], k0["y"]], 1).astype(np.float32))
    nm, m12, prev2 = oracle_mod.search_for_initialization(k0, d0, k1, d1, w, h, prev, 100, 0.9, True)
    assert nm == int(g["nmatches"]) and np.array_equal(m12, g["matches12"])
    assert np.array_equal(prev2, g["prev_after"])


@pytest.mark.gpu
@pytest.mark.parametrize("path", GOLD, ids=[p.stem for p in GOLD])
def test_gpu_reproduces_golden(path):
    from orb_slam_2_ros_amd import ORBextractor, ORBmatcher, Frame
    g = _load(path)
    w, h, f0, f1 = _frames(g)
    ex = ORBextractor(int(g["nfeatures"]), 1.2, 8, 20, 7)
    k0, d0 = ex(f0)
    k1, d1 = ex(f1)
    assert len(k0) == len(g["kps0"]) and (k0 == g["kps0"]).all() and np.array_equal(d0, g["desc0"])
    assert len(k1) == len(g["kps1"]) and (k1 == g["kps1"]).all() and np.array_equal(d1, g["desc1"])
    prev = np.ascontiguousarray(np.stack([k0["x"], k0["y"]], 1).astype(np.float32))
    nm, m12 = ORBmatcher(0.9, True).SearchForInitialization(Frame(k0, d0, w, h), Frame(k1, d1, w, h), prev, 100)
    assert nm == int(g["nmatches"]) and np.array_equal(m12, g["matches12"])
    assert np.array_equal(prev, g["prev_after"])
