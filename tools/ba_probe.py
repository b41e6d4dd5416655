"""Local BA latency probe (bench.local_ba_latency alone), for profiling."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402

print(json.dumps(bench.local_ba_latency(reps=int(sys.argv[1]) if len(sys.argv) > 1 else 3)))
