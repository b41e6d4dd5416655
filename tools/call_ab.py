"""A/B of the per-call matchers (SearchByProjection keyframe and last-frame
variants, SearchByBoW(KF, F) and SearchForTriangulation: bench.py
matcher_latencies' cases) across liborbx builds: each library is dlopen'ed on
its own (only the two calls bound), median of `reps` calls per turn.  Several
libraries in one process have failed their first calls on the box; run one
library per process and alternate the processes (tools/gpu/r5d.sh).
    python tools/call_ab.py ROUNDS REPS lib1.so[:VAR=VALUE] [lib2.so ...]
A VAR=VALUE is in the environment for that library's first call (the
library reads its switches once); copies of one build under other names
compare its runtime switches."""
import ctypes
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from orb_slam_2_ros_amd import _lib  # noqa: E402
from orb_slam_2_ros_amd.matcher import ORBmatcher  # noqa: E402
from orb_slam_2_ros_amd.synth_match import BOW_VARIANT_ARGS, PROJ_VARIANT_ARGS, make_bow_case, make_proj_case  # noqa: E402


def _M(lib, ratio, ori):
    """An ORBmatcher bound to another library's handle."""
    m = ORBmatcher.__new__(ORBmatcher)
    m._lib, m.device, m.mfNNratio, m.mbCheckOrientation = lib, 0, ratio, ori
    return m


def main():
    rounds, reps, specs = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3:]
    libs = [x.split(":")[0] for x in specs]
    envs = [dict(kv.split("=", 1) for kv in x.split(":")[1:]) for x in specs]
    handles = []
    for p in libs:
        lib = ctypes.CDLL(str(Path(p).resolve()))
        for name in ("orbx_search_by_projection", "orbx_search_by_bow"):
            res, args = _lib._SIGNATURES[name]
            getattr(lib, name).restype = res
            getattr(lib, name).argtypes = args
        handles.append(lib)
    cases = {}   # name -> (call, ratio, ori)
    for variant, n, nq in [("lastframe", 2000, 1500), ("keyframe", 2000, 1000)]:
        th, ratio, ori, wth = PROJ_VARIANT_ARGS[variant]
        c = make_proj_case(1234, variant, n=n, nq=nq, stereo=variant != "keyframe", th=wth)
        args = (variant, c["keys"], c["desc"], c["queries"], c["qdesc"], c["bounds"], c["uright"], c["mp_state"],
                c["inv_sigma2"], th)
        cases[variant] = (lambda m, a=args: ORBmatcher.search_by_projection(m, *a), ratio, ori)
    for variant in ("kf_frame", "triangulation"):
        ratio, ori = BOW_VARIANT_ARGS[variant]
        A, B, tri = make_bow_case(4321, variant, na=2000, nb=2000, nodes=200)
        cases[variant] = (lambda m, v=variant, a=A, b=B, t=tri: ORBmatcher.search_by_bow(m, v, a, b, t), ratio, ori)
    ref = {}
    for p, lib, env in zip(specs, handles, envs):   # first calls with the library's switches set
        os.environ.update(env)
        for variant, (call, ratio, ori) in cases.items():
            call(_M(lib, ratio, ori))
        for k in env:
            del os.environ[k]
    for r in range(rounds):
        for p, lib in zip(specs, handles):
            row = []
            for variant, (call, ratio, ori) in cases.items():
                m = _M(lib, ratio, ori)
                out = call(m)
                key = variant
                if key in ref:
                    assert out[0] == ref[key][0] and all(np.array_equal(a, b) for a, b in zip(out[1:], ref[key][1:]))
                else:
                    ref[key] = out
                ts = []
                for _ in range(reps):
                    t0 = time.perf_counter()
                    call(m)
                    ts.append(time.perf_counter() - t0)
                row.append(f"{variant} {1e3 * float(np.median(ts)):.4f} ms")
            print(f"round {r} {Path(p).name}: " + ", ".join(row), flush=True)


if __name__ == "__main__":
    main()
