"""One-frame host-API extraction (the drop-in call Frame::ExtractORB makes) run
repeatedly, for a trace of the B = 1 chain:
    rocprofv3 --kernel-trace --hip-runtime-trace --stats -d gpurun_out/b1 -- python tools/b1_probe.py [MODE W H N]
MODE: mono (one extractor), pair (EuRoC-style stereo pair, the two
extractions one after the other + ComputeStereoMatches), pair2 (the two
extractions on two host threads, as Frame.cc:79-82 runs them)."""
import sys
import threading
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402,F401  (one HIP runtime for torch and liborbx)

from orb_slam_2_ros_amd import ORBextractor, synth  # noqa: E402
from orb_slam_2_ros_amd.depth import compute_stereo_matches  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "mono"
w, h, n = (int(a) for a in sys.argv[2:5]) if len(sys.argv) >= 5 else (640, 480, 200)


class Worker:
    """A persistent second host thread (the reference starts one per frame)."""

    def __init__(self):
        self.go, self.done = threading.Event(), threading.Event()
        self.fn = None
        threading.Thread(target=self._run, daemon=True).start()

    def _run(self):
        while True:
            self.go.wait()
            self.go.clear()
            self.out = self.fn()
            self.done.set()

    def submit(self, fn):
        self.fn = fn
        self.done.clear()
        self.go.set()

    def result(self):
        self.done.wait()
        return self.out


if mode == "mono":
    img = synth.frame(w, h, 4242)
    ex = ORBextractor(1000, 1.2, 8, 20, 7)

    def call():
        ex(img)
else:
    L, R = synth.stereo_pair(w, h, 4243)
    exl, exr = ORBextractor(1200, 1.2, 8, 20, 7), ORBextractor(1200, 1.2, 8, 20, 7)
    bf, fx = 47.9, 435.2
    mb = float(np.float32(bf) / np.float32(fx))
    wk = Worker()

    def call():
        if mode == "pair2":
            wk.submit(lambda: exr(R))
            kl, dl = exl(L)
            kr, dr = wk.result()
        else:
            kl, dl = exl(L)
            kr, dr = exr(R)
        return compute_stereo_matches(exl, exr, kl, dl, kr, dr, bf, mb)

for _ in range(5):
    call()
ts = []
for _ in range(n):
    t0 = time.perf_counter()
    call()
    ts.append(time.perf_counter() - t0)
print(f"{mode} {w}x{h}: median {1e3 * np.median(ts):.4f} ms, min {1e3 * np.min(ts):.4f} ms over {n} calls")
