"""Repeated drop-in matcher calls on the bench's synthetic cases, for
`rocprofv3 --kernel-trace --stats` per-kernel times of the matcher kernels."""
import sys
import time

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from orb_slam_2_ros_amd import ORBmatcher  # noqa: E402
from orb_slam_2_ros_amd.synth_match import PROJ_VARIANT_ARGS, make_proj_case  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
for variant, n, nq in [("localmap", 2000, 2500), ("lastframe", 2000, 1500), ("keyframe", 2000, 1000)]:
    th, ratio, ori, wth = PROJ_VARIANT_ARGS[variant]
    c = make_proj_case(1234, variant, n=n, nq=nq, stereo=variant != "keyframe", th=wth)
    m = ORBmatcher(ratio, ori)
    args = (variant, c["keys"], c["desc"], c["queries"], c["qdesc"], c["bounds"], c["uright"], c["mp_state"],
            c["inv_sigma2"])
    m.search_by_projection(*args, th)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        r = m.search_by_projection(*args, th)
        ts.append(time.perf_counter() - t0)
    print(variant, "matches", r[0], "median ms", round(1e3 * float(np.median(ts)), 4), flush=True)
