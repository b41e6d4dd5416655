"""KFDB loop-query latency probe: bench.kfdb_latency, then the same GPU
queries back to back (no oracle in between), for profiling."""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402

import bench  # noqa: E402
from orb_slam_2_ros_amd.keyframe_db import KeyFrameDatabase  # noqa: E402
from orb_slam_2_ros_amd.synth_vocab import make_keyframe_bows  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
print(json.dumps(bench.kfdb_latency(reps=reps)))
n_kf = 10000
bows, covis = make_keyframe_bows(n_kf=n_kf + reps, n_words=1000000, words_per_kf=1000, seed=11, loop_every=500)
g = KeyFrameDatabase()
for i in range(n_kf):
    g.add(i, *bows[i])
cv = lambda k: covis.get(k, [])   # noqa: E731
for r in range(3):
    g.DetectLoopCandidates(n_kf + r, *bows[n_kf + r], covis[n_kf + r], 0.01, cv)
ts = []
for k in range(5 * reps):
    q = n_kf + k % reps
    t0 = time.perf_counter()
    g.DetectLoopCandidates(100000 + k, *bows[q], covis[q], 0.01, cv)
    ts.append(time.perf_counter() - t0)
print(json.dumps({"back_to_back_gpu_ms": round(1e3 * float(np.median(ts)), 4)}))
