"""Per-phase cycle breakdown of k_fast, k_describe and k_quadtree (diagnostic build with
s_memtime marks, -DORBX_PHASE_PROF):
    make -C orb_slam_2_ros_amd/csrc prof
    ORBX_LIB=orb_slam_2_ros_amd/liborbx_prof.so python tools/phase_prof.py [W H B]
Runs the bench's mono step (unsplit) and prints, per phase, the summed wave
cycles per launch and their share of the kernel's wave cycles."""
import ctypes
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
assert "liborbx_prof" in os.environ.get("ORBX_LIB", ""), "set ORBX_LIB to the phase-profiling build"
import torch  # noqa: E402

import bench  # noqa: E402
from orb_slam_2_ros_amd import ORBextractor, _lib  # noqa: E402

w, h, B = (int(a) for a in sys.argv[1:4]) if len(sys.argv) >= 4 else (640, 480, 1024)
lib = _lib.load()
fn = lib.orbx_debug_phase_cycles
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
buf = np.zeros(24, np.uint64)
host, _ = bench._resident_frames("mono", w, h, list(range(B)))
fr = torch.from_numpy(host).cuda()
ex = ORBextractor(1000, 1.2, 8, 20, 7)
ex.reserve(w, h, B)
ex.split(1)
for t in range(3):
    ex.mono_step_device(fr[t % 4].data_ptr(), w * h, w, B, 100, 0.9, True)
torch.cuda.synchronize()
fn(buf.ctypes.data, 24, 1)
reps = 5
for t in range(reps):
    ex.mono_step_device(fr[t % 4].data_ptr(), w * h, w, B, 100, 0.9, True)
torch.cuda.synchronize()
fn(buf.ctypes.data, 24, 1)
names = {0: ["prologue+stage", "ini: zero+compass+compact", "ini: arc scores", "ini: NMS+out",
             "min: zero+compass+compact", "min: arc scores", "min: NMS+out", "-"],
         1: ["prologue+stage", "moments+atan", "row pass", "sincos+offsets+column pass", "round+ballot+write",
             "-", "-", "-"],
         2: ["gather", "roots", "full: child counts", "full: scan+children", "final: child counts",
             "final: sort", "final: splits", "output"]}
for k, kname in ((0, "k_fast"), (1, "k_describe"), (2, "k_quadtree")):
    v = buf[8 * k:8 * k + 8].astype(np.float64) / reps
    tot = v.sum()
    print(f"{kname} ({w}x{h}, B={B}): {tot / 1e9:.3f} G wave-cycles per launch")
    for i in range(8):
        if v[i] > 0:
            print(f"  {names[k][i]:<30s} {v[i] / 1e6:10.1f} M  {100 * v[i] / tot:5.1f} %")
