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


def test_stream_partition_covers_every_stream_once():
    """s -> rank s mod G for the C5 stream count and the
    headline weak-scaling sets, at every world size the driver runs."""
    sys.path.insert(0, str(ROOT))
    import bench
    for world in (1, 2, 3, 4, 8):
        for total in (bench.C5_STREAMS, 16 * world, 1024 * world):
            parts = [bench.stream_partition(total, world, r) for r in range(world)]
            flat = sorted(s for p in parts for s in p)
            assert flat == list(range(total))
            assert max(map(len, parts)) - min(map(len, parts)) <= 1
            for r, p in enumerate(parts):
                assert all(s % world == r for s in p)


def test_bench_launcher_two_ranks_stub():
    """`bench.py --gpus 2` started WITHOUT a launcher spawns the two ranks
    itself (torch.distributed.run, gloo under --stub) and the JSON line
    reports the whole job: n_gpus 2, each rank's exact batch shape, every
    global stream exactly once, and each stream's frames are the ones its
    global id names (so a stream's content does not depend on G)."""
    import json
    import subprocess
    import numpy as np
    sys.path.insert(0, str(ROOT))
    import bench
    B, steps, warmup, w, h = 6, 3, 1, 64, 48
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--stub", "--width", str(w),
                        "--height", str(h), "--batch", str(B), "--steps", str(steps), "--warmup", str(warmup),
                        "--cpu-seconds", "0"], capture_output=True, text=True, timeout=300, env=env, cwd=str(ROOT))
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["config"]["global_batch"] == 2 * B
    assert line["config"]["streams_per_gpu"] == B and line["scaling"] == "weak"
    ranks = sorted(line["stub"], key=lambda d: d["rank"])
    assert [d["rank"] for d in ranks] == [0, 1]
    seen = []
    for d in ranks:
        assert d["batches"] == [B]                        # every step hands the library B frames
        assert d["calls"] == max(warmup, 2) + steps       # warmup (at least 2: the match needs a previous frame) + timed
        assert d["streams"] == bench.stream_partition(2 * B, 2, d["rank"])
        for s, cs in zip(d["streams"], d["checksums"]):
            ref = bench.scene_frames("mono", w, h, bench.stream_scene(s))[0]
            assert cs == int(ref.astype(np.uint64).sum())
        seen += d["streams"]
    assert sorted(seen) == list(range(2 * B))
    c5 = line["extras"]["c5_rgbd_fhd_64_streams"]
    assert c5["streams_total"] == 64 and c5["streams_per_gpu"] == 32
    assert c5["keyframe_all_gather"]["ranks"] == 2


def test_bench_rejects_world_mismatch():
    """Under a launcher, --gpus must equal WORLD_SIZE."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "1", "--stub", "--cpu-seconds", "0",
                        "--no-extras"], capture_output=True, text=True, timeout=120, env=env, cwd=str(ROOT))
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr
