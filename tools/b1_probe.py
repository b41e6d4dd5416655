"""One-frame host-API extraction (the drop-in call Frame::ExtractORB makes) run
repeatedly, for a kernel trace of the B = 1 chain:
    rocprofv3 --kernel-trace --stats -d gpurun_out/b1 -- python tools/b1_probe.py [W H N]"""
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402,F401  (one HIP runtime for torch and liborbx)

from orb_slam_2_ros_amd import ORBextractor, synth  # noqa: E402

w, h, n = (int(a) for a in sys.argv[1:4]) if len(sys.argv) >= 4 else (640, 480, 200)
img = synth.frame(w, h, 4242)
ex = ORBextractor(1000, 1.2, 8, 20, 7)
for _ in range(5):
    ex(img)
ts = []
for _ in range(n):
    t0 = time.perf_counter()
    ex(img)
    ts.append(time.perf_counter() - t0)
print(f"{w}x{h}: median {1e3 * np.median(ts):.4f} ms, min {1e3 * np.min(ts):.4f} ms over {n} calls")
