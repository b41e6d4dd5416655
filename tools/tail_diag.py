"""Stage times of one front-end configuration, unsplit, from the library's HIP
event ring (the bench's profiling pass, alone).  Environment knobs of liborbx
(ORBX_DBG_STOP, ORBX_MATCH_CLOCKS, ORBX_SPLIT) pass through, so phase costs
come from differences between runs:
    tools/tail_diag.py MODE W H NFEAT BATCH [STEPS]
MODE mono | stereo | rgbd; BATCH = streams (stereo: pairs)."""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np
import torch

from orb_slam_2_ros_amd import ORBextractor, synth

mode, w, h, nf, batch = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
steps = int(sys.argv[6]) if len(sys.argv) > 6 else 20
dev = torch.device("cuda", 0)
nfr = 2 * batch if mode == "stereo" else batch
scenes = [synth.frames(w, h, seed=7000 + s, count=2) for s in range(8)]
host = np.stack([np.stack([scenes[b % 8][t] for b in range(nfr)]) for t in range(2)])
frames = torch.from_numpy(host).to(dev)
dmap = torch.from_numpy(np.stack([synth.depth_map(w, h, 7000 + b % 8) for b in range(batch)])).to(dev) \
    if mode == "rgbd" else None
ex = ORBextractor(nf, 1.2, 8, 20, 7, device=0)
ex.reserve(w, h, nfr)
sp = torch.cuda.current_stream(dev).cuda_stream
fs = w * h


def step(k):
    f = frames[k % 2].data_ptr()
    if mode == "mono":
        ex.mono_step_device(f, fs, w, batch, 100, 0.9, True, sp)
    elif mode == "stereo":
        ex.stereo_step_device(f, fs, w, batch, 47.9, float(np.float32(47.9) / np.float32(435.2)), sp)
    else:
        ex.rgbd_step_device(f, fs, w, batch, dmap.data_ptr(), 4 * fs, 4 * w, 47.9, sp)


for k in range(3):
    step(k)
torch.cuda.synchronize()
t0 = time.perf_counter()
for k in range(steps):
    step(k)
torch.cuda.synchronize()
el = time.perf_counter() - t0
ex.set_profiling(True)
for k in range(steps):
    step(k)
torch.cuda.synchronize()
st = ex.stage_times()
unit = batch / (el / steps)
print(f"{mode} {w}x{h} nf={nf} batch={batch}: {unit:,.0f} units/s ({1e3 * el / steps:.3f} ms/step); "
      "stages ms resize/blur/fast/quadtree/describe/match|depth: " + " ".join(f"{x:.4f}" for x in st))
