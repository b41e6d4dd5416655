"""Host-fed rate vs the hardware queues of its streams (bench.py's full run
read lower than the standalone extra): the host_fed VGA step repeatedly,
with more torch streams created in between; streams from torch's pool or
from hipExtStreamCreateWithCUMask (HF_STREAMS=pool|cumask), level pipeline
HF_PIPE.  (The dedicated streams are made once and reused: destroying them
after a run segfaulted the process.)"""
import json
import os
import sys

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402

dev = torch.device("cuda:0")
w, h, nf, ns, split, pipe = bench.HOST_FED["host_fed_vga"]
pipe = int(os.environ.get("HF_PIPE", pipe))
bench.HOST_FED_STREAMS = os.environ.get("HF_STREAMS", "cumask")
keep = []
for n in range(int(os.environ.get("HF_RUNS", "4"))):
    r = bench.host_fed(torch, dev, w, h, nf, ns, split, pipe, 20, 3)
    print(json.dumps([bench.HOST_FED_STREAMS, pipe, f"after {len(keep)} more streams", r["value"], r["h2d_GBs"]]),
          flush=True)
    keep.append(torch.cuda.Stream(dev))
