"""Cross-stream keyframe exchange: packing round trip, and
a world_size-2 gloo all-gather in which every rank ends with the same,
rank-major list of all ranks' keyframes.  CPU only."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from orb_slam_2_ros_amd import KEYPOINT_DTYPE
from orb_slam_2_ros_amd.keyframe_db import pack_keyframes, unpack_keyframes


def _records(rank, n):
    rng = np.random.default_rng(100 + rank)
    out = []
    for i in range(n):
        nw, nk = int(rng.integers(0, 50)), int(rng.integers(0, 30))
        k = np.zeros(nk, KEYPOINT_DTYPE)
        k["x"] = rng.uniform(0, 640, nk)
        k["octave"] = rng.integers(0, 8, nk)
        out.append({"kf_id": (rank << 40) | i, "words": np.sort(rng.choice(1000, nw, replace=False)).astype(np.uint32),
                    "values": rng.random(nw), "keys": k, "desc": rng.integers(0, 256, (nk, 32)).astype(np.uint8)})
    return out


def _same(a, b):
    assert len(a) == len(b)
    for x, y in zip(a, b):
        assert x["kf_id"] == y["kf_id"]
        for f in ("words", "values", "keys", "desc"):
            assert np.array_equal(x[f], y[f])


def test_pack_round_trip():
    r = _records(3, 7)
    _same(unpack_keyframes(pack_keyframes(r)), r)
    _same(unpack_keyframes(pack_keyframes([])), [])


def _worker(rank, world, port, q):
    import torch.distributed as dist
    from orb_slam_2_ros_amd.keyframe_db import all_gather_keyframes
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    got = all_gather_keyframes(_records(rank, 3 + 2 * rank), dist)
    q.put((rank, pack_keyframes(got)))
    dist.destroy_process_group()


def test_all_gather_keyframes_gloo():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = _records(0, 3) + _records(1, 5)
    for r in range(2):
        _same(unpack_keyframes(res[r]), want)
