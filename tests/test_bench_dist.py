"""The multi-rank bench harness (bench.timed_region / max_over_ranks) on the
CPU with gloo, world_size 2: barriers bracket the timed region on every rank,
and the reported time is the slowest rank's (replicas, no
collective on the data path)."""
import os
import socket
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out):
    import time
    import torch
    import torch.distributed as dist
    sys.path.insert(0, str(ROOT))
    import bench
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    calls = []

    def step(k):
        calls.append(k)
        time.sleep(0.01 * (rank + 1))   # rank 1 is the slow replica

    el = bench.timed_region(step, 6, 2, lambda: None, dist, world)
    mx = bench.max_over_ranks(torch, dist, world, el, torch.device("cpu"))
    gathered = [None] * world
    dist.all_gather_object(gathered, el)
    dist.destroy_process_group()
    out.put((rank, el, mx, gathered, calls))


def test_timed_region_two_ranks_gloo():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    for rank, el, mx, gathered, calls in res:
        assert calls == list(range(8))               # 2 warmup + exactly 6 timed steps
        assert mx == pytest.approx(max(gathered))    # max over ranks, identical on both
        assert mx >= 6 * 0.02 * 0.9                  # bounded below by the slow rank's work
    assert res[0][2] == res[1][2]


def _exchange_worker(rank, world, port, out):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, str(ROOT))
    import bench
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    r = bench.keyframe_exchange(torch, dist, world, None, kfs_per_rank=2, nkp=50, reps=2)
    dist.destroy_process_group()
    out.put((rank, r))


def test_keyframe_exchange_two_ranks_gloo():
    """bench.keyframe_exchange (the C5 keyframe all-gather extra) runs on every
    rank and each receives world x keyframes_per_rank keyframes."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_exchange_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(2):
        assert res[r]["ranks"] == 2 and res[r]["keyframes_per_rank"] == 2 and res[r]["ms"] > 0
