"""Local BA fast mode alone (config C4, as bench.local_ba_latency), for a
kernel trace: REPS calls after one warm-up."""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from orb_slam_2_ros_amd.optimizer import local_bundle_adjustment  # noqa: E402
from orb_slam_2_ros_amd.synth_ba import make_ba_problem  # noqa: E402

P = make_ba_problem(n_local=20, n_fixed=4, n_points=3000, seed=2)
args = (P["Tcw"], P["fixed"], P["Xw"], P["edges"])
local_bundle_adjustment(*args, fast=True)
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
for _ in range(reps):
    t0 = time.perf_counter()
    local_bundle_adjustment(*args, fast=True)
    print("fast local BA ms", round(1e3 * (time.perf_counter() - t0), 3), flush=True)
