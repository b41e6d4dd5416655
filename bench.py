#!/usr/bin/env python3
"""Benchmark: frames/s of the ORB front end (extract + SearchForInitialization
against the previous frame of the same stream), 1000 kp, 8 levels, VGA mono
(BASELINE.json configs[1]) on N MI355X GPUs, one process per GPU.

Unit of work: one frame = ORBextractor::operator() on a
640x480 u8 image + ORBmatcher::SearchForInitialization(F1 = that stream's
previous frame, F2 = this frame, vbPrevMatched = F1 keypoints, window 100,
nnratio 0.9, checkOri).  A step processes one new frame for each of the B = 512
streams a GPU owns (streams are independent: weak scaling, no collective on
the data path; RCCL is used only for the barrier / max-time reduction).

Secondary configurations (reported under "extras", not the headline value):
FHD mono, and the stereo / RGB-D units of SURVEY.md §8(d) -- a stereo pair =
extract left + right + Frame::ComputeStereoMatches (C3 EuRoC 752x480 1200 kp,
C4 KITTI 1241x376 2000 kp, FHD); an RGB-D frame = extract + ComputeStereoFromRGBD.

Inputs are synthetic (orb_slam_2_ros_amd.synth) and resident in HBM before
the timed region.  Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "frames/sec ORB extract+match (1000 kp, 8 lvl) @640x480 & 1920x1080, 1-GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)
FRAMES_PER_STREAM = 4  # resident frames per stream, stepped cyclically
UNIQUE_SCENES = 32


def level_geometry(w: int, h: int, nfeatures: int):
    """Level sizes / quotas exactly as the extractor computes them (host copy of
    ORBextractor.cc:416-455,1157-1159 semantics via the library's getters)."""
    from orb_slam_2_ros_amd import ORBextractor
    ex = ORBextractor(nfeatures, 1.2, 8, 20, 7)
    inv = ex.GetInverseScaleFactors()
    sizes = [(int(np.rint(np.float32(w) * np.float32(s))), int(np.rint(np.float32(h) * np.float32(s)))) for s in inv]
    ex.close()
    return sizes


def algorithmic_bytes(sizes, nkp: float, stage: str) -> float:
    """Compulsory HBM bytes per frame of one stage."""
    p0 = sizes[0][0] * sizes[0][1]
    p = sum(a * b for a, b in sizes)
    if stage == "resize":      # read levels 0..6, write levels 1..7
        return float(p - sizes[-1][0] * sizes[-1][1]) + float(p - p0)
    if stage == "blur":        # read every level, write its blurred copy
        return 2.0 * p
    if stage == "fast":        # read every level once
        return float(p)
    if stage == "describe":    # 60 B per keypoint out; its patch reads re-read what k_fast streamed (L2)
        return nkp * 60
    if stage == "match":       # both frames' descriptors + keypoints read, matches written
        return nkp * (2 * 32 + 2 * 28 + 4)
    if stage == "stereo":      # per pair: both images' keypoints + descriptors read, uR / depth / SAD written
        return nkp * (2 * 60 + 12)
    if stage == "rgbd":        # per frame: keypoints read, one depth sample each, uR / depth written
        return nkp * (28 + 4 + 8)
    if stage == "quadtree":    # candidates in, selection out (counted in the kernel)
        return 0.0
    if stage == "frame":       # SURVEY.md §8(d) compulsory figure
        return float(p0 + 2 * (p - p0)) + nkp * 60 + nkp * (2 * 32 + 4)
    raise ValueError(stage)


TRAFFIC_FILE = ROOT / "profiles" / "traffic_vga.json"
# per-workload PMC summaries (tools/profile.sh + tools/prof_summary.py --json) for the extras' rooflines
TRAFFIC_FILES = {"fhd_1920x1080": ROOT / "profiles" / "traffic_fhd.json",
                 "stereo_fhd_1920x1080": ROOT / "profiles" / "traffic_fhd_stereo.json"}
STAGE_KERNEL = {"resize": "k_resize", "fast": "k_fast", "quadtree": "k_quadtree", "describe": "k_describe",
                "match": "k_search_init"}


def measured_traffic(stage: str, frames_per_launch: float, path=None):
    """HBM bytes per launch of the stage's kernel from the committed rocprofv3
    PMC passes (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE, MI355X_MICROARCH.md),
    scaled from the profiled dispatch's frame count; (None, None) if absent."""
    path = path or TRAFFIC_FILE
    try:
        prof = json.loads(path.read_text())
        name = STAGE_KERNEL[stage]
        # template instantiations are listed as k_name<args>; the whole-batch
        # launch is the <false> one
        keys = [k for k in prof["kernels"] if k == name or k.startswith(name + "<") or k.startswith(name + "_w<")]
        keys.sort(key=lambda k: "<false" not in k)
        k = prof["kernels"][keys[0]]
        per_frame = k["hbm_bytes_per_dispatch"] / prof["frames_per_dispatch"]
        return round(per_frame * frames_per_launch), str(path.relative_to(ROOT))
    except (OSError, KeyError, ValueError, ZeroDivisionError, IndexError):
        return None, None


# VALU issue ceilings measured on MI355X with the clock each launch held
# (s_memtime / s_memrealtime; profiles/r02_valu_rate_clock.txt, r02_valu_ops.txt):
# - full rate: v_add/sub/and/or/xor/lshrrev_b32, 16-bit VOP2 min/max/sub, f32
#   add/mul/fma, mov -- 0.908 ns per wave-instruction per SIMD at 16 waves/SIMD
#   (2.14 cycles at 2.36 GHz): 1024 SIMDs / 0.908 ns = 1128 G wave-instr/s;
# - half rate: u32 min/max, every 3-operand integer op, v_perm / alignbyte /
#   bfe, packed 16-bit, dot2/dot4, DPP, cvt, any op with an SGPR operand --
#   1.727 ns (4.15 cycles): 593 G wave-instr/s.
VALU_PEAK_GINST = 1127.8
VALU_HALF_RATE_GINST = 592.9
VALU_PEAK_SOURCE = "profiles/r02_valu_rate_clock.txt, profiles/r02_valu_ops.txt"


def measured_valu(stage: str, frames_per_launch: float, path=None):
    """VALU wave-instructions per launch of the stage's kernel (SQ_INSTS_VALU
    from the committed PMC pass, scaled from the profiled dispatch's frame
    count); None if absent."""
    path = path or TRAFFIC_FILE
    try:
        prof = json.loads(path.read_text())
        name = STAGE_KERNEL[stage]
        keys = [k for k in prof["kernels"] if k == name or k.startswith(name + "<") or k.startswith(name + "_w<")]
        keys.sort(key=lambda k: "<false" not in k)
        k = prof["kernels"][keys[0]]
        return round(k["valu_insts_per_dispatch"] / prof["frames_per_dispatch"] * frames_per_launch)
    except (OSError, KeyError, ValueError, ZeroDivisionError, IndexError):
        return None


STAGE_NAMES = ["resize", "blur", "fast", "quadtree", "describe", "match"]


def roofline_block(sizes, nkp, stages, frames_per_launch, units_per_s_gpu, mode="mono", traffic_path=None):
    """The `roofline` object for one workload: the dominant HBM-streaming
    kernel (by time among the stages that move a tenth or more of the frame's
    compulsory bytes) with its algorithmic bytes per launch
    over its measured launch time (stage times: HIP events on the launch
    stream, a separate unsplit, unpipelined pass, one whole-batch launch per
    stage), its PMC traffic and VALU issue rate from the workload's committed
    profile, the time-dominant stage beside it, and the whole unit's
    compulsory bytes at the measured throughput (`pipeline_frac`).
    frames_per_launch counts images (2 per stereo pair); units_per_s_gpu is
    the workload's own unit (frames or stereo pairs) per second per GPU.
    Returns (roofline, stage_ms)."""
    if not stages:
        return None, None
    stage_ms = dict(zip(STAGE_NAMES, [round(s, 4) for s in stages]))
    if mode == "stereo":
        stage_ms["stereo"] = stage_ms.pop("match")
    elif mode == "rgbd":
        stage_ms["rgbd"] = stage_ms.pop("match")
    fb = algorithmic_bytes(sizes, nkp, "frame")
    # (per launch: frames for the extraction stages, pairs / frames for the last)
    per_launch = {n: frames_per_launch / 2 if n == "stereo" else frames_per_launch for n in stage_ms}
    cand = {n: t for n, t in stage_ms.items()
            if t and t > 0 and algorithmic_bytes(sizes, nkp, n) >= 0.1 * fb}
    if not cand:
        return None, stage_ms
    dom = max(cand, key=cand.get)
    bytes_launch = algorithmic_bytes(sizes, nkp, dom) * per_launch[dom]
    achieved = bytes_launch / (cand[dom] * 1e-3) / 1e9
    traffic, tsrc = measured_traffic(dom, per_launch[dom], traffic_path)
    roof = {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
            "traffic_source": tsrc, "bytes_per_launch": bytes_launch, "frames_per_launch": frames_per_launch,
            "launch_ms": cand[dom]}
    valu = measured_valu(dom, per_launch[dom], traffic_path)
    if valu:
        # the same kernel against the VALU issue rate (its actual bound)
        ach = valu / (cand[dom] * 1e-3) / 1e9
        roof["issue"] = {"bound": "valu", "achieved": round(ach, 1), "peak": VALU_PEAK_GINST,
                         "unit": "G wave-instr/s", "frac": round(ach / VALU_PEAK_GINST, 4),
                         "half_rate_peak": VALU_HALF_RATE_GINST,
                         "frac_of_half_rate": round(ach / VALU_HALF_RATE_GINST, 4),
                         "insts_per_launch": valu, "source": tsrc, "peak_source": VALU_PEAK_SOURCE}
    tdom = max((n for n, t in stage_ms.items() if t and t > 0), key=lambda n: stage_ms[n])
    if tdom != dom:
        tb = algorithmic_bytes(sizes, nkp, tdom) * per_launch[tdom]
        tach = tb / (stage_ms[tdom] * 1e-3) / 1e9
        tv = measured_valu(tdom, per_launch[tdom], traffic_path)
        roof["dominant_by_time"] = {
            "kernel": tdom, "ms": stage_ms[tdom], "bytes_per_launch": tb, "achieved": round(tach, 2),
            "frac": round(tach / HBM_PEAK_GBS, 5),
            "traffic": measured_traffic(tdom, per_launch[tdom], traffic_path)[0],
            "issue_frac_of_half_rate": round(tv / (stage_ms[tdom] * 1e-3) / 1e9 / VALU_HALF_RATE_GINST, 4)
            if tv else None}
    # the unit's compulsory bytes: a frame, or a stereo pair =
    # two frames' extraction + the pair's stereo search
    if mode == "stereo":
        unit_bytes = 2 * algorithmic_bytes(sizes, nkp, "frame") - 2 * nkp * (2 * 32 + 4) \
            + algorithmic_bytes(sizes, nkp, "stereo")
    elif mode == "rgbd":
        unit_bytes = fb - nkp * (2 * 32 + 4) + algorithmic_bytes(sizes, nkp, "rgbd")
    else:
        unit_bytes = fb
    roof["unit_bytes"] = round(unit_bytes)
    roof["pipeline_GBs"] = round(unit_bytes * units_per_s_gpu / 1e9, 2)
    roof["pipeline_frac"] = round(unit_bytes * units_per_s_gpu / 1e9 / HBM_PEAK_GBS, 5)
    return roof, stage_ms



def cpu_model() -> str:
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(w: int, h: int, nfeatures: int, budget_s: float):
    """The oracle (C++ restatement of the reference, scalar primitives as
    written -- not OpenCV-SIMD/IPP) on the same workload, 1 thread: extract +
    SearchForInitialization vs the previous frame.  Timed on the oracle's
    -O3 -march=native build (oracle.use_timing_build)."""
    from oracle import oracle
    from orb_slam_2_ros_amd import synth
    build = oracle.use_timing_build()
    frames = synth.frames(w, h, 4242, 8)
    prev = oracle.extract(frames[0], nfeatures)
    n = 0
    t0 = time.perf_counter()
    while True:
        img = frames[(n + 1) % len(frames)]
        k2, d2 = oracle.extract(img, nfeatures)
        k1, d1 = prev
        pxy = np.ascontiguousarray(np.stack([k1["x"], k1["y"]], 1).astype(np.float32))
        oracle.search_for_initialization(k1, d1, k2, d2, w, h, pxy, 100, 0.9, True)
        prev = (k2, d2)
        n += 1
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    return {"value": n / el, "unit": "frames/s", "cores": 1, "kind": "port",
            "cpu_model": cpu_model(), "host_cpus": os.cpu_count(), "build": build,
            "sample": f"{n} consecutive {w}x{h} synthetic frames ({el:.1f} s), oracle timing build, 1 thread; "
                      "restated reference, scalar primitives (not OpenCV-SIMD/IPP)"}


def cpu_baseline_threads(w: int, h: int, nfeatures: int, budget_s: float, threads: int):
    """The same oracle workload on `threads` host threads at once, one stream
    per thread (ORB-SLAM2 runs one extraction per std::thread, Frame.cc:79-82);
    ctypes drops the GIL inside each call.  Whole-host frames/s."""
    import threading
    from oracle import oracle
    from orb_slam_2_ros_amd import synth
    frames = synth.frames(w, h, 4242, 8)
    counts = [0] * threads
    stop = time.perf_counter() + budget_s

    def worker(t):
        prev = oracle.extract(frames[t % len(frames)], nfeatures)
        n = 0
        while time.perf_counter() < stop:
            img = frames[(t + n + 1) % len(frames)]
            k2, d2 = oracle.extract(img, nfeatures)
            k1, d1 = prev
            pxy = np.ascontiguousarray(np.stack([k1["x"], k1["y"]], 1).astype(np.float32))
            oracle.search_for_initialization(k1, d1, k2, d2, w, h, pxy, 100, 0.9, True)
            prev = (k2, d2)
            n += 1
        counts[t] = n

    t0 = time.perf_counter()
    ths = [threading.Thread(target=worker, args=(t,)) for t in range(threads)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    el = time.perf_counter() - t0
    return {"value": sum(counts) / el, "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"{sum(counts)} {w}x{h} synthetic frames on {threads} threads ({el:.1f} s)"}


def timed_region(step, steps, warmup, sync, dist, world, on_start=None):
    """W untimed warmup steps, then EXACTLY `steps` timed steps bracketed by a
    barrier + device sync on both sides.  Returns this rank's elapsed seconds."""
    k = 0
    for _ in range(warmup):
        step(k); k += 1
    sync()
    if world > 1:
        dist.barrier()
    if on_start is not None:
        on_start()
    sync()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step(k); k += 1
    sync()
    if world > 1:
        dist.barrier()
    return time.perf_counter() - t0


def max_over_ranks(torch, dist, world, el, device):
    """The slowest rank's elapsed time (whole-job throughput divides by it)."""
    t = torch.tensor([el], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def write_bow_case(path, variant: int, A, B, tri, nnratio: float, check_ori: bool, nlevels: int = 8):
    """One SearchByBoW problem as adapter_test time_bow reads it."""
    from orb_slam_2_ros_amd._lib import KEYPOINT_DTYPE
    t = np.zeros(0, np.float32) if tri is None else np.ascontiguousarray(tri, np.float32)
    with open(path, "wb") as f:
        f.write(np.array([variant, nlevels, int(check_ori), len(t), 0], np.int32).tobytes())
        f.write(np.float32(nnratio).tobytes())
        f.write(t.tobytes())
        for S in (A, B):
            k = np.ascontiguousarray(S["keys"], KEYPOINT_DTYPE)
            ids = np.ascontiguousarray(S["ids"], np.uint32)
            feat = np.ascontiguousarray(S["feat"], np.int32)
            f.write(np.array([len(k), len(ids), len(feat)], np.int32).tobytes())
            f.write(k.tobytes())
            f.write(np.ascontiguousarray(S["desc"], np.uint8).tobytes())
            f.write(np.ascontiguousarray(S["flags"], np.uint8).tobytes())
            f.write(ids.tobytes())
            f.write(np.ascontiguousarray(S["off"], np.int32).tobytes())
            f.write(feat.tobytes())


def matcher_latencies(reps: int = 20):
    """Per-call latency of the drop-in ORBmatcher searches (host arrays in and
    out, as Tracking / LocalMapping / LoopClosing call them) next to the
    oracle's single-thread time on the same inputs."""
    from oracle import oracle
    from orb_slam_2_ros_amd import ORBmatcher
    from orb_slam_2_ros_amd.matcher import BOW_VARIANTS, PROJ_VARIANTS
    from orb_slam_2_ros_amd.synth_match import (BOW_VARIANT_ARGS, PROJ_VARIANT_ARGS, make_bow_case,
                                                make_proj_case)

    def timed(fn, k):
        ts = []
        for _ in range(k):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return 1e3 * float(np.median(ts))

    out = {}
    for variant, n, nq in [("localmap", 2000, 2500), ("lastframe", 2000, 1500), ("keyframe", 2000, 1000),
                           ("fuse", 2000, 2000)]:
        th, ratio, ori, wth = PROJ_VARIANT_ARGS[variant]
        c = make_proj_case(1234, variant, n=n, nq=nq, stereo=variant != "keyframe", th=wth)
        m = ORBmatcher(ratio, ori)
        args = (variant, c["keys"], c["desc"], c["queries"], c["qdesc"], c["bounds"], c["uright"], c["mp_state"],
                c["inv_sigma2"])
        m.search_by_projection(*args, th)
        out[f"SearchByProjection_{variant}" if "fuse" not in variant else "Fuse"] = {
            "keypoints": n, "points": nq,
            "gpu_ms": round(timed(lambda: m.search_by_projection(*args, th), reps), 4),
            **cxx_proj_latency(PROJ_VARIANTS[variant], c, th, ratio, ori),
            "cpu_ms": round(timed(lambda: oracle.search_by_projection(*args, th, ratio, ori), 5), 4)}
    for variant, na in [("kf_frame", 2000), ("triangulation", 2000)]:
        ratio, ori = BOW_VARIANT_ARGS[variant]
        A, B, tri = make_bow_case(4321, variant, na=na, nb=na, nodes=200)
        m = ORBmatcher(ratio, ori)
        m.search_by_bow(variant, A, B, tri)
        name = "SearchByBoW_kf_frame" if variant == "kf_frame" else "SearchForTriangulation"
        out[name] = {"features": na,
                     "gpu_ms": round(timed(lambda: m.search_by_bow(variant, A, B, tri), reps), 4),
                     "cxx_ms": cxx_bow_latency(BOW_VARIANTS[variant], A, B, tri, ratio, ori, 100),
                     "cpu_ms": round(timed(lambda: oracle.search_by_bow(variant, A, B, ratio, ori, tri), 5), 4)}
    out["local_mapping_20_neighbours"] = local_mapping_matchers(reps)
    return out


def local_mapping_matchers(reps: int = 10, nn: int = 20):
    """The matcher work LocalMapping does per new keyframe over its nn = 20
    covisible neighbours: SearchForTriangulation against each
    (CreateNewMapPoints, LocalMapping.cc:276-315, ORBmatcher(0.6, false)) and
    Fuse of its map points into each (SearchInNeighbors, :537-548), plus
    relocalisation's SearchByProjection over 10 candidates (Tracking.cc:1667).
    Batched (one launch pair per loop) vs one drop-in call per neighbour vs
    the oracle's single thread."""
    from oracle import oracle
    from orb_slam_2_ros_amd import ORBmatcher
    from orb_slam_2_ros_amd.synth_match import (BOW_VARIANT_ARGS, PROJ_VARIANT_ARGS, make_bow_case,
                                                make_proj_case)

    def timed(fn, k):
        ts = []
        for _ in range(k):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return 1e3 * float(np.median(ts))

    out = {}
    ratio, ori = BOW_VARIANT_ARGS["triangulation"]
    A, B, tri = make_bow_case(777, "triangulation", na=2000, nb=2000, nodes=200)
    rng = np.random.default_rng(778)
    probs = []
    for _ in range(nn):
        d = B["desc"].copy()
        flip = rng.random(d.shape) < 0.03
        d[flip] ^= (1 << rng.integers(0, 8, flip.sum())).astype(np.uint8)
        probs.append({"A": A, "B": dict(B, desc=d), "tri": tri})
    m = ORBmatcher(ratio, ori)
    m.search_by_bow_batch("triangulation", probs)
    out["SearchForTriangulation"] = {
        "features": 2000, "neighbours": nn,
        "gpu_batched_ms": round(timed(lambda: m.search_by_bow_batch("triangulation", probs), reps), 4),
        "gpu_per_call_ms": round(timed(lambda: [m.search_by_bow("triangulation", P["A"], P["B"], P["tri"])
                                                for P in probs], max(3, reps // 3)), 4),
        "cpu_ms": round(timed(lambda: [oracle.search_by_bow("triangulation", P["A"], P["B"], ratio, ori, P["tri"])
                                       for P in probs], 3), 4)}
    for variant, key, count, n, nq in [("fuse", "Fuse", nn, 2000, 1500), ("keyframe", "reloc_SearchByProjection", 10,
                                                                          2000, 1000)]:
        th, ratio, ori, wth = PROJ_VARIANT_ARGS[variant]
        cases = [make_proj_case(900 + k, variant, n=n, nq=nq, stereo=variant == "fuse", th=wth) for k in range(count)]
        if variant == "keyframe":   # one current frame, each candidate's points
            cases = [dict(cases[0], queries=c["queries"], qdesc=c["qdesc"]) for c in cases]
        m = ORBmatcher(ratio, ori)
        m.search_by_projection_batch(variant, cases, th)

        def per_call(cs=cases, mm=m, v=variant, t=th):
            for c in cs:
                mm.search_by_projection(v, c["keys"], c["desc"], c["queries"], c["qdesc"], c["bounds"], c["uright"],
                                        c["mp_state"], c["inv_sigma2"], t)

        def cpu(cs=cases, v=variant, t=th, r=ratio, o=ori):
            for c in cs:
                oracle.search_by_projection(v, c["keys"], c["desc"], c["queries"], c["qdesc"], c["bounds"],
                                            c["uright"], c["mp_state"], c["inv_sigma2"], t, r, o)
        out[key] = {"keypoints": n, "points": nq, "problems": count,
                    "gpu_batched_ms": round(timed(lambda: m.search_by_projection_batch(variant, cases, th), reps), 4),
                    "gpu_per_call_ms": round(timed(per_call, max(3, reps // 3)), 4),
                    "cpu_ms": round(timed(cpu, 3), 4)}
    return out


def bow_transform_throughput(torch, frames=512, nfeat=1000, reps=20):
    """DBoW2 transform of `frames` x `nfeat` device-resident
    descriptors through a synthetic ORBvoc-shaped vocabulary (k=10, L=6,
    1.1M nodes; ORBvoc.txt itself is not in the repository), levelsup 4 as
    Frame::ComputeBoW.  The per-feature descent only (word, weight, node per
    descriptor); the CPU oracle is timed on 20 frames with its tree prebuilt."""
    from oracle import oracle
    from orb_slam_2_ros_amd.synth_vocab import features_near_leaves, make_vocab
    from orb_slam_2_ros_amd.vocabulary import ORBVocabulary
    voc = make_vocab(k=10, L=6, seed=5)
    v = ORBVocabulary.from_arrays(10, 6, 0, 0, voc["parent"], voc["is_leaf"], voc["desc"], voc["weight"])
    n = frames * nfeat
    feats = features_near_leaves(voc, n, seed=9, noise=30)
    d = torch.from_numpy(feats).cuda()
    word = torch.empty(n, dtype=torch.int32, device="cuda")
    wt = torch.empty(n, dtype=torch.float64, device="cuda")
    node = torch.empty(n, dtype=torch.int32, device="cuda")
    st = torch.cuda.Stream()   # a real stream handle (NULL would mean the library's own stream)
    st.wait_stream(torch.cuda.current_stream())

    def run():
        v.transform_device(d.data_ptr(), n, 4, word.data_ptr(), wt.data_ptr(), node.data_ptr(), st.cuda_stream)
    for _ in range(3):
        run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(st)
    for _ in range(reps):
        run()
    e1.record(st)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    pv = oracle.PreparedVocab(voc)
    sample = feats[:20 * nfeat]
    pv.transform(sample[:nfeat])
    t0 = time.perf_counter()
    for f in range(20):
        pv.transform(sample[f * nfeat:(f + 1) * nfeat])
    cpu_ms = 1e3 * (time.perf_counter() - t0) / 20
    # L2/MALL-resident tree: per feature L levels x (k x 32 B child rows + 16 B node)
    return {"value": round(n / (ms * 1e-3), 1), "unit": "features/s", "frames_per_launch": frames,
            "features_per_frame": nfeat, "ms_per_launch": round(ms, 4), "frame_equiv_per_s": round(frames / (ms * 1e-3), 1),
            "bytes_per_feature_from_cache": 6 * (10 * 32 + 16),
            "cpu_ms_per_frame": round(cpu_ms, 4), "cpu_kind": "port, 1 thread, tree prebuilt"}


def kfdb_latency(n_kf=10000, words=1000, reps=10):
    """KeyFrameDatabase::DetectLoopCandidates over a 10,000-keyframe database
    (64 streams x ~150 keyframes; synthetic BowVectors of 1,000 words of a
    1M-word vocabulary), GPU vs the oracle's literal inverted-file walk."""
    from oracle import oracle
    from orb_slam_2_ros_amd.keyframe_db import KeyFrameDatabase
    from orb_slam_2_ros_amd.synth_vocab import make_keyframe_bows
    bows, covis = make_keyframe_bows(n_kf=n_kf + reps, n_words=1000000, words_per_kf=words, seed=11, loop_every=500)
    g, o = KeyFrameDatabase(), oracle.KeyFrameDB(1000000)
    for i in range(n_kf):
        g.add(i, *bows[i])
        o.add(i, *bows[i])
    cv = lambda k: covis.get(k, [])   # noqa: E731
    tg, to = [], []
    for r in range(reps):
        q = n_kf + r
        t0 = time.perf_counter()
        a = g.DetectLoopCandidates(q, *bows[q], covis[q], 0.01, cv)
        tg.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        b = o.detect(False, q, *bows[q], covis[q], 0.01, cv)
        to.append(time.perf_counter() - t0)
        assert a == b
    # steady state: each side's queries back to back (fresh query ids, the
    # same sequence on both; the answers are compared too)
    tgb, tob, ga, oa = [], [], [], []
    for k in range(3 * reps):
        q = n_kf + k % reps
        t0 = time.perf_counter()
        ga.append(g.DetectLoopCandidates(200000 + k, *bows[q], covis[q], 0.01, cv))
        tgb.append(time.perf_counter() - t0)
    for k in range(3 * reps):
        q = n_kf + k % reps
        t0 = time.perf_counter()
        oa.append(o.detect(False, 200000 + k, *bows[q], covis[q], 0.01, cv))
        tob.append(time.perf_counter() - t0)
    assert ga == oa
    return {"keyframes": n_kf, "words_per_keyframe": words, "gpu_ms": round(1e3 * float(np.median(tg)), 4),
            "cpu_ms": round(1e3 * float(np.median(to)), 4), "gpu_ms_back_to_back": round(1e3 * float(np.median(tgb)), 4),
            "cpu_ms_back_to_back": round(1e3 * float(np.median(tob)), 4), "cpu_kind": "port, 1 thread, inverted file"}


def local_ba_latency(reps=3):
    """Optimizer::LocalBundleAdjustment (config C4, KITTI-like stereo: 20
    local + 4 fixed keyframes, 3,000 map points, ~25k observations; 5 + 10 LM
    iterations), GPU vs the oracle's single-thread restatement."""
    from oracle import oracle
    from orb_slam_2_ros_amd.optimizer import local_bundle_adjustment
    from orb_slam_2_ros_amd.synth_ba import make_ba_problem
    P = make_ba_problem(n_local=20, n_fixed=4, n_points=3000, seed=2)
    args = (P["Tcw"], P["fixed"], P["Xw"], P["edges"])
    local_bundle_adjustment(*args)
    local_bundle_adjustment(*args, fast=True)
    tg, tf, to = [], [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        g = local_bundle_adjustment(*args)
        tg.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        f = local_bundle_adjustment(*args, fast=True)
        tf.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        o = oracle.local_ba(*args)
        to.append(time.perf_counter() - t0)
    assert np.array_equal(g[0], o[0]) and np.array_equal(g[2], o[2])
    return {"keyframes": 24, "points": 3000, "observations": int(len(P["edges"])), "lm_iterations": list(g[3]),
            "gpu_ms": round(1e3 * float(np.median(tg)), 3), "cpu_ms": round(1e3 * float(np.median(to)), 3),
            "cpu_kind": "port, 1 thread, same summation order",
            "fast_mode": {"gpu_ms": round(1e3 * float(np.median(tf)), 3), "lm_iterations": list(f[3]),
                          "outliers_identical": bool(np.array_equal(f[2], o[2])),
                          "max_abs_pose_diff": float(np.abs(f[0] - o[0]).max()),
                          "max_rel_point_diff": float(np.abs(f[1] - o[1]).max() / np.abs(o[1]).max())}}


def keyframe_exchange(torch, dist, world, dev, kfs_per_rank=8, nkp=1000, reps=10):
    """The C5 cross-stream keyframe all-gather: every
    rank publishes kfs_per_rank new keyframes (BowVector of ~nkp words,
    nkp keypoints + descriptors) and receives everyone's, over RCCL."""
    from orb_slam_2_ros_amd import KEYPOINT_DTYPE
    from orb_slam_2_ros_amd.keyframe_db import all_gather_keyframes
    rng = np.random.default_rng(dist.get_rank() if world > 1 else 0)
    recs = []
    for i in range(kfs_per_rank):
        recs.append({"kf_id": i, "words": np.sort(rng.choice(1000000, nkp, replace=False)).astype(np.uint32),
                     "values": rng.random(nkp), "keys": np.zeros(nkp, KEYPOINT_DTYPE),
                     "desc": rng.integers(0, 256, (nkp, 32)).astype(np.uint8)})
    all_gather_keyframes(recs, dist, dev)
    ts = []
    for _ in range(reps):
        dist.barrier()
        t0 = time.perf_counter()
        got = all_gather_keyframes(recs, dist, dev)
        ts.append(time.perf_counter() - t0)
    assert len(got) == world * kfs_per_rank
    return {"ranks": world, "keyframes_per_rank": kfs_per_rank, "bytes_per_rank": int(sum(
        12 * len(r["words"]) + 60 * len(r["keys"]) + 16 for r in recs)), "ms": round(1e3 * float(np.median(ts)), 4)}


def stream_partition(total: int, world: int, rank: int) -> list:
    """Global stream ids a rank owns: stream s -> rank s mod G (SURVEY.md §8(e),
    stream-affine; a stereo pair is one stream and stays on one GPU)."""
    return list(range(rank, total, world))


def stream_scene(s: int) -> int:
    """Synthetic scene of global stream s: the content is a function of the
    stream id alone, so a stream's frames (and outputs) do not depend on how
    many ranks share the job.  UNIQUE_SCENES distinct scenes keep the set-up
    cheap at 3072 streams per GPU."""
    return s % UNIQUE_SCENES


def scene_frames(mode, w, h, scene):
    """The FRAMES_PER_STREAM resident frames of one scene: [T, h, w] (mono /
    RGB-D) or [T, 2, h, w] (stereo L/R, 20-px disparity)."""
    from orb_slam_2_ros_amd import synth
    seed = 7000 + scene
    if mode == "stereo":
        canvas = synth.stream_canvas(w, h, seed)
        out = np.empty((FRAMES_PER_STREAM, 2, h, w), np.uint8)
        for t in range(FRAMES_PER_STREAM):
            out[t, 0] = synth.frame_from_canvas(canvas, w, h, t, seed * 7919 + t)
            out[t, 1] = synth.frame_from_canvas(canvas, w, h, t, seed * 7919 + t + 500009, disparity=20)
        return out
    return synth.frames(w, h, seed, FRAMES_PER_STREAM)


class _Worker:
    """A second host thread that runs one call at a time (the library's host
    calls release the GIL, so the two extractions overlap on the device)."""

    def __init__(self):
        import threading
        self.go, self.done = threading.Event(), threading.Event()
        self.fn = self.out = None
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


def dropin_latency(torch, dev, reps=100):
    """The drop-in path as ORB-SLAM2 drives it, one frame per call:
    - `ORBextractor::operator()` on a host image (Frame::ExtractORB,
      Frame.cc:259-265, from Tracking::GrabImage*, Tracking.cc:247-276),
      host keypoints/descriptors out, synchronous -- VGA, HD and FHD;
    - a stereo pair: two extractors on two host threads, as Frame.cc:79-82
      runs them, + Frame::ComputeStereoMatches (Frame.cc:502-676), EuRoC size;
    - the batched device step at B in {1, 8, 64, 256} VGA frames per launch;
    next to the oracle's single-thread latency on the same frames."""
    from oracle import oracle
    from orb_slam_2_ros_amd import ORBextractor, synth
    from orb_slam_2_ros_amd.depth import compute_stereo_matches

    def med(fn, k):
        ts = []
        for _ in range(k):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return 1e3 * float(np.median(ts))

    out = {}
    for key, w, h in (("vga", 640, 480), ("hd", 1280, 720), ("fhd", 1920, 1080)):
        img = synth.frame(w, h, 4242)
        ex = ORBextractor(1000, 1.2, 8, 20, 7, device=dev.index)
        ex(img)
        out[f"extract_host_{key}"] = {"gpu_ms": round(med(lambda: ex(img), reps), 4),
                                      "cpu_ms": round(med(lambda: oracle.extract(img), 3), 3)}
        ex.close()
    w, h = 752, 480
    L, R = synth.stereo_pair(w, h, 4243)
    exl, exr = ORBextractor(1200, 1.2, 8, 20, 7, device=dev.index), ORBextractor(1200, 1.2, 8, 20, 7, device=dev.index)
    bf, fx = 47.9, 435.2
    mb = float(np.float32(bf) / np.float32(fx))

    # Frame's stereo constructor extracts the two images on two threads
    # (Frame.cc:79-82): the right one goes to a second (persistent) thread
    right = _Worker()

    def pair():
        right.submit(lambda: exr(R))
        kl, dl = exl(L)
        kr, dr = right.result()
        return compute_stereo_matches(exl, exr, kl, dl, kr, dr, bf, mb)

    def pair_cpu():
        kl, dl = oracle.extract(L, 1200)
        kr, dr = oracle.extract(R, 1200)
        return oracle.compute_stereo_matches(oracle.pyramid(L), oracle.pyramid(R), kl, dl, kr, dr, bf, mb)

    pair()
    out["stereo_pair_host_euroc"] = {"gpu_ms": round(med(pair, reps), 4), "cpu_ms": round(med(pair_cpu, 3), 3)}
    exl.close()
    exr.close()
    out.update(cxx_dropin_latency(L, R, bf, mb, reps))
    # batched device step, VGA mono (extract + SearchForInitialization)
    w, h = 640, 480
    base = synth.frames(w, h, 4244, FRAMES_PER_STREAM)
    sweep = {}
    sp = torch.cuda.current_stream(dev).cuda_stream
    for B in (1, 8, 64, 256):
        ex = ORBextractor(1000, 1.2, 8, 20, 7, device=dev.index)
        ex.reserve(w, h, B)
        fr = torch.from_numpy(np.ascontiguousarray(np.repeat(base[:, None], B, axis=1))).to(dev)
        k = [0]

        def step():
            ex.mono_step_device(fr[k[0] % FRAMES_PER_STREAM].data_ptr(), w * h, w, B, 100, 0.9, True, sp)
            k[0] += 1
        for _ in range(3):
            step()
        torch.cuda.synchronize(dev)
        n = 20
        t0 = time.perf_counter()
        for _ in range(n):
            step()
        torch.cuda.synchronize(dev)
        ms = 1e3 * (time.perf_counter() - t0) / n
        sweep[str(B)] = {"ms_per_step": round(ms, 4), "frames_per_s": round(B / (ms * 1e-3), 1),
                         "us_per_frame": round(1e3 * ms / B, 3)}
        ex.close()
        del fr
    out["mono_step_device_vga_batch_sweep"] = sweep
    return out


def _adapter_exe():
    exe = Path(__file__).resolve().parent / "orb_slam_2_ros_amd" / "bin" / "adapter_test"
    if not exe.exists():
        sys.path.insert(0, str(Path(__file__).resolve().parent / "tests"))
        from cxx_build import build_adapter_test
        build_adapter_test(exe)
    return exe


def cxx_bow_latency(variant: int, A, B, tri, nnratio, check_ori, reps):
    """A SearchByBoW call through the C++ forwarder's entry
    (OrbxMatcher::SearchByBoWTable), as ORBmatcher_orbx.cc makes it: ms."""
    import subprocess
    import tempfile
    with tempfile.TemporaryDirectory() as td:
        p = Path(td) / "bow.bin"
        write_bow_case(p, variant, A, B, tri, nnratio, check_ori)
        r = subprocess.run([str(_adapter_exe()), "time_bow", str(p), str(reps)], capture_output=True, text=True,
                           timeout=120, check=True)
    return float(r.stdout.split("bow_ms")[1].split()[0])


def write_proj_case(d: Path, c):
    """One SearchByProjection problem as adapter_test proj / time_proj read it
    (frame.bin, queries.bin in d)."""
    n, nq = len(c["keys"]), len(c["queries"])
    with open(d / "f.bin", "wb") as f:
        f.write(np.int32(n).tobytes()); f.write(np.array(c["bounds"], np.float32).tobytes())
        f.write(np.ascontiguousarray(c["keys"]).tobytes()); f.write(np.ascontiguousarray(c["desc"]).tobytes())
        ur = c["uright"] if c["uright"] is not None else np.full(n, -1, np.float32)
        f.write(np.ascontiguousarray(ur, np.float32).tobytes())
        ms = c["mp_state"] if c["mp_state"] is not None else np.zeros(n, np.uint8)
        f.write(np.ascontiguousarray(ms, np.uint8).tobytes())
        isg = c["inv_sigma2"] if c["inv_sigma2"] is not None else np.zeros(0, np.float32)
        f.write(np.int32(len(isg)).tobytes()); f.write(np.ascontiguousarray(isg, np.float32).tobytes())
    with open(d / "q.bin", "wb") as f:
        f.write(np.int32(nq).tobytes()); f.write(np.ascontiguousarray(c["queries"]).tobytes())
        f.write(np.ascontiguousarray(c["qdesc"]).tobytes())


def cxx_proj_latency(variant: int, c, th, ratio, ori, reps=1000, phase_reps=200):
    """A SearchByProjection / Fuse call through the C++ forwarder's entry
    (OrbxMatcher::SearchByProjectionTable, ORBmatcher_orbx.cc), host tables in
    and out: median and minimum over `reps` calls, then the host call's phases
    (ORBX_CALL_TIMING: checks, staging, enqueue, wait for the outputs, readback;
    medians over `phase_reps` calls, in microseconds)."""
    import subprocess
    import tempfile
    with tempfile.TemporaryDirectory() as td:
        d = Path(td)
        write_proj_case(d, c)
        args = [str(_adapter_exe()), "time_proj", str(variant), str(th), repr(float(ratio)), str(int(ori)),
                str(d / "f.bin"), str(d / "q.bin")]
        r = subprocess.run(args + [str(reps)], capture_output=True, text=True, timeout=300, check=True)
        rp = subprocess.run(args + [str(phase_reps)], capture_output=True, text=True, timeout=300, check=True,
                            env=dict(os.environ, ORBX_CALL_TIMING="1"))
    val = {k: float(r.stdout.split(k + " ")[1].split()[0]) for k in ("proj_ms", "proj_min_ms")}
    ph = [[float(x) for x in ln.split(":", 1)[1].split()] for ln in rp.stderr.splitlines()
          if ln.startswith("orbx proj us:")]
    ph = [p for p in ph if len(p) == 5][-phase_reps:]
    med = [round(float(np.median([p[i] for p in ph])), 2) for i in range(5)] if ph else None
    return {"cxx_ms": val["proj_ms"], "cxx_min_ms": val["proj_min_ms"], "calls": reps,
            "phases_us": dict(zip(["checks", "staging", "enqueue", "wait", "readback"], med)) if med else None}


def cxx_dropin_latency(L, R, bf, mb, reps):
    """The C++ drop-in (include/orbx_orbslam2.hpp) as a reference tree would
    link it, timed by orb_slam_2_ros_amd/bin/adapter_test (built by
    __graft_entry__.build()): ORBextractor::operator() at VGA / FHD (and the
    first mvImagePyramid read after a call), Frame's stereo constructor (two
    threads started per frame, Frame.cc:79-82, + ComputeStereoMatches through
    OrbxFrame) at EuRoC size, and the RGB-D frame (extract +
    ComputeStereoFromRGBD) at FHD."""
    import subprocess
    import tempfile
    from orb_slam_2_ros_amd import synth
    exe = _adapter_exe()

    def run(*args):
        r = subprocess.run([str(exe), *map(str, args)], capture_output=True, text=True, timeout=300, check=True)
        return {ln.split()[0]: float(ln.split()[1]) for ln in r.stdout.splitlines() if ln.endswith(tuple("0123456789")) and
                ln.split()[0].endswith("_ms")}

    out = {}
    with tempfile.TemporaryDirectory() as td:
        td = Path(td)
        for key, w, h in (("vga", 640, 480), ("fhd", 1920, 1080)):
            p = td / f"{key}.raw"
            synth.frame(w, h, 4242).tofile(p)
            t = run("time", w, h, p, 1000, reps)
            out[f"cxx_extract_{key}"] = {"gpu_ms": t["extract_ms"], "pyramid_read_ms": t["pyramid_read_ms"]}
        pl, pr = td / "l.raw", td / "r.raw"
        np.ascontiguousarray(L).tofile(pl)
        np.ascontiguousarray(R).tofile(pr)
        t = run("time_stereo", L.shape[1], L.shape[0], pl, pr, 1200, bf, mb, reps)
        out["cxx_stereo_pair_euroc"] = {"gpu_ms": t["pair_ms"]}
        w, h = 1920, 1080
        img = synth.frame(w, h, 4245)
        rng = np.random.default_rng(5)
        dmap = rng.uniform(0.5, 8.0, (h, w)).astype(np.float32)
        dmap[rng.random((h, w)) < 0.2] = 0.0
        pi, pd = td / "rgbd.raw", td / "depth.raw"
        img.tofile(pi)
        dmap.tofile(pd)
        t = run("time_rgbd", w, h, pi, pd, 40.0, reps)
        out["cxx_rgbd_fhd"] = {"frame_ms": t["rgbd_frame_ms"], "depth_ms": t["rgbd_depth_ms"]}
    return out


def _resident_frames(mode, w, h, streams):
    """Host array [FRAMES_PER_STREAM, frames_per_step, h, w] for this rank's
    global stream ids (+ float32 depth maps for RGB-D): local slot b holds
    stream streams[b] (stereo: slots 2b / 2b+1 its left / right image)."""
    from orb_slam_2_ros_amd import synth
    batch = len(streams)
    cache = {}
    depth = None
    if mode == "stereo":
        host = np.empty((FRAMES_PER_STREAM, 2 * batch, h, w), np.uint8)
    else:
        host = np.empty((FRAMES_PER_STREAM, batch, h, w), np.uint8)
    for b, s in enumerate(streams):
        sc = stream_scene(s)
        if sc not in cache:
            cache[sc] = scene_frames(mode, w, h, sc)
        if mode == "stereo":
            host[:, 2 * b], host[:, 2 * b + 1] = cache[sc][:, 0], cache[sc][:, 1]
        else:
            host[:, b] = cache[sc]
    if mode == "rgbd":
        dm = {}
        for s in streams:
            dm.setdefault(stream_scene(s) % 8, None)
        dm = {k: synth.depth_map(w, h, 7000 + k) for k in dm}
        depth = np.stack([dm[stream_scene(s) % 8] for s in streams])
    return host, depth


class StubExtractor:
    """Stands in for ORBextractor under `bench.py --stub` (CPU, gloo): records
    what each step hands the library -- batch size and a checksum of every
    frame of the batch -- so the launcher, the stream partition and the batch
    shapes are testable without a GPU (tests/test_bench_dist.py)."""

    def __init__(self, w, h):
        self.w, self.h = w, h
        self.batches = []
        self.checksums = None
        self._t = 0

    def _record(self, ptr, fstride, batch):
        import ctypes
        buf = np.ctypeslib.as_array((ctypes.c_uint8 * (fstride * batch)).from_address(ptr))
        sums = [int(buf[i * fstride:(i + 1) * fstride].astype(np.uint64).sum()) for i in range(batch)]
        if self.checksums is None:
            self.checksums = sums
        self.batches.append(batch)

    def reserve(self, w, h, b):
        pass

    def split(self, parts=0):
        return 1

    def pipeline(self, on=-1):
        return 0

    def mono_step_device(self, ptr, fstride, pitch, batch, *a):
        self._record(ptr, fstride, batch)

    def stereo_step_device(self, ptr, fstride, pitch, pairs, *a):
        self._record(ptr, fstride, 2 * pairs)

    def rgbd_step_device(self, ptr, fstride, pitch, batch, *a):
        self._record(ptr, fstride, batch)

    def set_profiling(self, on):
        pass

    def stage_times(self):
        return [0.0] * 6

    def batch_download(self, b):
        return np.zeros(1), None

    def mono_matches_download(self, b):
        return None, 0

    def depth_download(self, b):
        return None, None, 0

    def pack_bytes(self):
        return 64

    def close(self):
        pass


def run_config(torch, dist, rank, world, dev, w, h, nfeatures, streams, steps, warmup, profile, mode="mono",
               stub=None, split=2, pipeline=0, kframes=1, overlap=None):
    """Times `steps` front-end steps of this rank's `streams` (global stream
    ids: mono / RGB-D frames or stereo pairs, one per stream per step); returns
    (max-over-ranks seconds, stage ms, kps, sanity, frames per launch, extractor).
    kframes (RGB-D only): K consecutive frames of every stream in one launch
    (a step is then K frames per stream; RGB-D frames are independent, the
    depth lookup reads only the frame's own depth map)."""
    assert kframes == 1 or mode == "rgbd"
    nstreams = len(streams)
    batch = nstreams * kframes
    if stub is not None:
        ex = stub
    else:
        from orb_slam_2_ros_amd import ORBextractor
        ex = ORBextractor(nfeatures, 1.2, 8, 20, 7, device=dev.index)
    ex.reserve(w, h, 2 * batch if mode == "stereo" else batch)
    if batch >= 64 and "ORBX_SPLIT" not in os.environ:
        # two half-batches on forked streams: one half's latency-bound quadtree /
        # matcher launches overlap the other half's VALU-bound ones
        ex.split(split)
    if pipeline and stub is None and "ORBX_PIPELINE" not in os.environ:
        ex.pipeline(pipeline)   # level pipeline (2: the deep form): on where it measured faster
    if overlap is None:
        overlap = MONO_OVERLAP
    if overlap and mode == "mono" and stub is None and "ORBX_OVERLAP_MATCH" not in os.environ:
        # each step's matcher beside the next step's extraction (orbx_extractor_overlap_match;
        # the timed region ends with a device-wide synchronisation, which covers it)
        ex.overlap_match(1)
    host, depth = _resident_frames(mode, w, h, streams)
    if kframes > 1:
        # launch u holds times u K .. u K + K - 1 (mod the resident frames) of
        # every stream, time-major; each frame keeps its stream's depth map
        host = np.stack([np.concatenate([host[(u * kframes + j) % FRAMES_PER_STREAM] for j in range(kframes)])
                         for u in range(FRAMES_PER_STREAM)])
        depth = np.concatenate([depth] * kframes)
    frames = torch.from_numpy(host).to(dev)
    dmaps = torch.from_numpy(depth).to(dev) if depth is not None else None
    del host, depth
    on_gpu = dev.type == "cuda"
    stream = torch.cuda.current_stream(dev) if on_gpu else None
    sp = stream.cuda_stream if on_gpu else 0
    fstride = h * w
    bf, fx = 47.9, 435.2                       # EuRoC-like rig: mbf, fx (mb = mbf / fx)
    mb = float(np.float32(bf) / np.float32(fx))

    def step(k):
        t = k % FRAMES_PER_STREAM
        if mode == "mono":
            ex.mono_step_device(frames[t].data_ptr(), fstride, w, batch, 100, 0.9, True, sp)
        elif mode == "stereo":
            ex.stereo_step_device(frames[t].data_ptr(), fstride, w, batch, bf, mb, sp)
        else:
            ex.rgbd_step_device(frames[t].data_ptr(), fstride, w, batch, dmaps.data_ptr(), 4 * fstride, 4 * w, bf, sp)

    sync = (lambda: torch.cuda.synchronize(dev)) if on_gpu else (lambda: None)
    el = timed_region(step, steps, max(warmup, 2), sync, dist, world)
    stages = None
    if profile and stub is None:
        # per-stage launch durations (HIP events on the launch stream) from a
        # separate untimed pass with the level pipeline off (if it was on), so
        # each stage is one whole-batch launch that overlaps nothing
        piped, parts = ex.pipeline(), ex.split()
        ex.pipeline(0)
        ex.split(1)
        step(steps)
        sync()
        ex.set_profiling(True)
        for k in range(max(5, steps // 5)):
            step(steps + 1 + k)
        sync()
        stages = ex.stage_times()
        ex.set_profiling(False)
        ex.pipeline(piped)
        ex.split(parts)
    # sanity: the last step produced keypoints and matches / depths on stream 0
    kp, _ = ex.batch_download(0)
    if mode == "mono":
        _, sane = ex.mono_matches_download(0)
    else:
        _, _, sane = ex.depth_download(0)
    el = max_over_ranks(torch, dist, world, el, dev)
    return el, stages, len(kp), sane, float(batch), ex   # the profiled launches cover the whole batch


HOST_FED_STREAMS = "cumask"   # (tools/host_fed_probe.py: "pool" = torch's stream pool)
_hip_rt = None


def dedicated_stream(torch, dev):
    """A stream on a hardware queue of its own: hipExtStreamCreateWithCUMask
    (every CU enabled) makes the runtime create a new queue for it rather
    than share one of the process's pooled queues."""
    global _hip_rt
    if HOST_FED_STREAMS == "pool":
        return torch.cuda.Stream(dev)
    import ctypes
    if _hip_rt is None:
        _hip_rt = ctypes.CDLL("libamdhip64.so")
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    words = (ncu + 31) // 32
    mask = (ctypes.c_uint32 * words)(*([0xFFFFFFFF] * words))
    s = ctypes.c_void_p()
    torch.cuda.set_device(dev)
    rc = _hip_rt.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(words), mask)
    if rc != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask: {rc}")
    return torch.cuda.ExternalStream(s.value, device=dev)


_hf_streams = {}


def host_fed_streams(torch, dev):
    """The host-fed runs' compute / upload / download streams, made once per
    process and reused (torch keeps referring to external streams it has
    run work on, so they are never destroyed: destroying them crashed the
    process on exit)."""
    key = (HOST_FED_STREAMS, dev.index)
    if key not in _hf_streams:
        _hf_streams[key] = tuple(dedicated_stream(torch, dev) for _ in range(3))
    return _hf_streams[key]


def host_fed(torch, dev, w, h, nfeatures, nstreams, split, pipeline, steps, warmup):
    """The mono step fed from host memory, as a camera-fed node sees it
    (ros/src/MonoNode.cc:38-50 -> Frame.cc:259-265: each frame arrives in a host
    cv::Mat).  Frames sit in pinned host memory (two per stream, alternating);
    step k's batch goes up on its own copy stream while step k - 1 computes
    (two device input buffers), and step k's keypoints + descriptors
    (orbx_batch_pack_device) come back on a third stream while step k + 1
    computes.  Reports frames/s with both PCIe directions inside the timed
    region, the host->device and device->host rates achieved, and a
    copy-only host->device rate over the same buffers: the bound PCIe puts on
    a host-fed front end (frames/s <= that rate / frame bytes)."""
    from orb_slam_2_ros_amd import ORBextractor
    streams = list(range(nstreams))
    host, _ = _resident_frames("mono", w, h, streams)
    src = torch.empty((2, nstreams, h, w), dtype=torch.uint8, pin_memory=True)
    src.copy_(torch.from_numpy(host[:2]))
    del host
    ex = ORBextractor(nfeatures, 1.2, 8, 20, 7, device=dev.index)
    ex.reserve(w, h, nstreams)
    ex.split(split)
    ex.pipeline(pipeline)
    dbuf = torch.empty((2, nstreams, h, w), dtype=torch.uint8, device=dev)
    # compute, upload and download on three streams of their own hardware
    # queues: HIP spreads a process's streams over its few queues
    # (GPU_MAX_HW_QUEUES), and a copy stream that shares the compute stream's
    # queue waits behind its kernels (180 k -> 124 k frames/s,
    # tools/host_fed_probe.py)
    s_comp, s_up, s_down = host_fed_streams(torch, dev)
    # the pack layout's size (known once a batch of this size has run)
    ex.mono_step_device(dbuf[0].data_ptr(), h * w, w, nstreams, 100, 0.9, True, s_comp.cuda_stream)
    torch.cuda.synchronize(dev)
    nb = ex.pack_bytes()
    pbuf = torch.empty((2, nb), dtype=torch.uint8, device=dev)
    hout = torch.empty((2, nb), dtype=torch.uint8, pin_memory=True)
    up_done = [torch.cuda.Event() for _ in range(2)]
    comp_done = [torch.cuda.Event() for _ in range(2)]
    down_done = [torch.cuda.Event() for _ in range(2)]
    recorded = [False, False]

    def step(k):
        i = k % 2
        if recorded[i]:
            s_up.wait_event(comp_done[i])     # step k - 2 has read dbuf[i]
        with torch.cuda.stream(s_up):
            dbuf[i].copy_(src[i], non_blocking=True)
            up_done[i].record(s_up)
        s_comp.wait_event(up_done[i])
        if recorded[i]:
            s_comp.wait_event(down_done[i])   # pbuf[i] of step k - 2 is on the host
        ex.mono_step_device(dbuf[i].data_ptr(), h * w, w, nstreams, 100, 0.9, True, s_comp.cuda_stream)
        ex.pack_device(pbuf[i].data_ptr(), nb, s_comp.cuda_stream)
        comp_done[i].record(s_comp)
        s_down.wait_event(comp_done[i])
        with torch.cuda.stream(s_down):
            hout[i].copy_(pbuf[i], non_blocking=True)
            down_done[i].record(s_down)
        recorded[i] = True

    sync = lambda: torch.cuda.synchronize(dev)   # noqa: E731
    el = timed_region(step, steps, warmup, sync, None, 1)
    # the copies alone over the same buffers: PCIe's own rate
    sync()
    t0 = time.perf_counter()
    for k in range(steps):
        with torch.cuda.stream(s_up):
            dbuf[k % 2].copy_(src[k % 2], non_blocking=True)
    sync()
    el_up = time.perf_counter() - t0
    t0 = time.perf_counter()
    for k in range(steps):
        with torch.cuda.stream(s_down):
            hout[k % 2].copy_(pbuf[k % 2], non_blocking=True)
    sync()
    el_down = time.perf_counter() - t0
    counts = hout[(steps - 1) % 2][:4 * nstreams].view(torch.int32)
    ok = int(counts.min().item()) > 0
    ex.close()
    fb = w * h
    up_rate = nstreams * fb * steps / el_up / 1e9
    return {"value": round(nstreams * steps / el, 2), "unit": "frames/s", "streams_per_gpu": nstreams,
            "ms_per_step": round(1e3 * el / steps, 4),
            "h2d_GBs": round(nstreams * fb * steps / el / 1e9, 2), "d2h_GBs": round(nb * steps / el / 1e9, 2),
            "d2h_bytes_per_frame": round(nb / nstreams, 1),
            "copy_only_h2d_GBs": round(up_rate, 2), "copy_only_d2h_GBs": round(nb * steps / el_down / 1e9, 2),
            "pcie_bound_frames_per_s": round(up_rate * 1e9 / fb, 1), "results_on_host": ok}


EXTRAS = [
    # key, mode, w, h, nfeatures, streams per GPU, unit
    # frames per GPU swept (round 4, profiles/r04_sweep_mono_streams.txt): FHD 128 / 192 / 256:
    # 70.7k / 74.1k / 74.7k frames/s; HD 256 / 384: 144.4k / 151.1k; FHD RGB-D 128 / 192: 72.3k / 75.2k
    ("fhd_1920x1080", "mono", 1920, 1080, 1000, 192, "frames/s"),
    ("hd_1280x720", "mono", 1280, 720, 1000, 384, "frames/s"),
    # EuRoC pairs per GPU swept 128 / 192 / 256: 129.6k / 135.8k / 140.8k pairs/s; KITTI 96 / 144 / 192:
    # 80.6k / 84.4k / 84.9k (round 4, profiles/r04_sweep_stereo_streams.txt)
    ("stereo_euroc_752x480", "stereo", 752, 480, 1200, 256, "stereo pairs/s"),
    ("stereo_kitti_1241x376", "stereo", 1241, 376, 2000, 144, "stereo pairs/s"),
    # FHD stereo pairs per GPU swept 32 / 64 / 128 / 192 / 256: 23.9k / 27.3k / 28.2k / 28.6k / 28.4k pairs/s
    ("stereo_fhd_1920x1080", "stereo", 1920, 1080, 1000, 192, "stereo pairs/s"),
    ("rgbd_fhd_1920x1080", "rgbd", 1920, 1080, 1000, 192, "frames/s"),
]

# Batch split per extra (2 unless listed): every extra gains from the split or
# is neutral (KITTI stereo 65.6 / 67.2 k unsplit / split, EuRoC 106.4 / 107.8 k,
# FHD stereo 28.1 / 29.8 k, FHD RGB-D 56.2 / 58.6 k pairs or frames/s).
# Round 4, after the level-major quadtree grid (profiles/r04_ab_split.txt), unsplit measured faster for
# FHD mono 75.1 / 75.5-75.7 k, FHD RGB-D 76.1-76.2 / 76.8-77.0 k, FHD stereo 37.7-38.0 / 38.1 k
# (split / unsplit), HD 152.3 / 152.8-153.7 k; EuRoC and KITTI within noise, kept split
EXTRA_SPLIT = {"fhd_1920x1080": 1, "hd_1280x720": 1, "rgbd_fhd_1920x1080": 1, "stereo_fhd_1920x1080": 1}
# Level pipeline per config (off unless listed), on / off measured on one box:
# VGA 1536 streams 318.0 / 314.5 k, FHD stereo 31.2 / 29.9 k pairs/s -- and
# off elsewhere: FHD 53.1 / 57.4 k, HD 116.0 / 123.9 k, FHD RGB-D 54.2 / 58.3 k,
# EuRoC 98.5 / 108.2 k, KITTI 62.0 / 67.3 k.  Round 4, after the level-major quadtree grid: FHD
# stereo on / off 37.2-37.3 / 37.9-38.0 k, so off there too (profiles/r04_ab_pipeline.txt)
# Round 5, after the LDS-free resize (k_resize_d), on / off on one box: FHD mono 89.5-90.8 / 88.2-88.5 k,
# HD 184.0 / 180.5-180.6 k, FHD stereo 45.6-45.7 / 44.0-44.1 k, FHD RGB-D 90.8-90.9 / 89.0-89.3 k; EuRoC
# 148.0 / 161.0-162.3 k and KITTI 87.8-88.2 / 95.2-95.3 k stay off (profiles/r05_ab_pipeline_extras.txt)
# Round 6, the deep form (2) on one box (profiles/r06_ab_pipe_extras.txt), pipeline 0 / 1 / 2: FHD mono 92.3 / 94.9 /
# 99.5 k, HD 188.2 / 192.3 / 197.9 k, FHD RGB-D 92.5 / 94.7 / 98.1 k frames/s; EuRoC 166.9 / 153.3 / 161.0 k and
# KITTI 97.6 / 89.6 / 95.1 k pairs/s stay unpipelined
EXTRA_PIPE = {"fhd_1920x1080": 2, "hd_1280x720": 2, "stereo_fhd_1920x1080": 2, "rgbd_fhd_1920x1080": 2}
# Round 6, the deep level pipeline (2: the side stream also takes levels 1..2 as the resize chain
# produces them, and their describe): VGA 467.9 k -> 484.5 k, FHD stereo 47.66 k -> 49.80 k pairs/s on
# one box (profiles/r06_ab_deep_pipeline.txt)
HEADLINE_PIPE = 2
# Matcher overlap of the mono steps (orbx_extractor_overlap_match): each step's
# SearchForInitialization on an internal stream beside the next step's resize /
# FAST / quadtree: VGA 449.1 k -> 454.1 k frames/s on one box (profiles/r05_ab_overlap_match.txt)
MONO_OVERLAP = 1
# Batch split of the VGA headline: with the quadtree's child counts aggregated
# (0.61 -> 0.38 ms) there is less latency-bound work to hide behind the other
# half, and one launch per stage measured faster on one box over two rounds
# (split / pipeline 1/1: 375.8-376.3 k, 2/1: 373.7-374.2 k, 2/0: 372.2-373.1 k,
# 1/0: 369.0-370.4 k frames/s; profiles/r03_split_sweep.txt)
HEADLINE_SPLIT = 1

# Host-fed runs of the mono step (frames from pinned host memory, both PCIe
# directions in the timed region): (w, h, nfeatures, streams per GPU, split, level pipeline)
HOST_FED = {"host_fed_vga": (640, 480, 1000, 3072, HEADLINE_SPLIT, HEADLINE_PIPE),
            "host_fed_fhd": (1920, 1080, 1000, 192, 1, 0)}

# Config C5 (BASELINE.json configs[4]): 64 FHD RGB-D streams over the job's
# GPUs (stream s -> rank s mod G), plus the cross-stream keyframe exchange.
C5_STREAMS = 64


def keyframe_publish(torch, dist, world, dev, ex, reps=10):
    """C5's one collective (reference analogue
    KeyFrameDatabase::add / DetectLoopCandidates, KeyFrameDatabase.cc:41,82):
    every rank packs its streams' newest keypoints + descriptors on the device
    (orbx_batch_pack_device) and all-gathers them over RCCL, so every GPU
    holds every stream's keyframe.  Times pack + all-gather, median of reps."""
    nb = ex.pack_bytes()
    sizes = [nb] * world
    if world > 1:
        t = torch.tensor([nb], dtype=torch.int64, device=dev)
        g = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(g, t)
        sizes = [int(x.item()) for x in g]
    cap = max(sizes)
    buf = torch.zeros(cap, dtype=torch.uint8, device=dev)
    out = torch.empty(world * cap, dtype=torch.uint8, device=dev)
    on_gpu = dev.type == "cuda"
    sp = torch.cuda.current_stream(dev).cuda_stream if on_gpu else 0

    def once():
        if on_gpu:
            ex.pack_device(buf.data_ptr(), cap, sp)
        if world > 1 and on_gpu:
            dist.all_gather_into_tensor(out, buf)
        elif world > 1:                      # gloo (CPU tests): list form
            dist.all_gather(list(out.view(world, cap).unbind(0)), buf)
        else:
            out.copy_(buf)
        if on_gpu:
            torch.cuda.synchronize(dev)

    once()
    ts = []
    for _ in range(reps):
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        once()
        ts.append(time.perf_counter() - t0)
    ms = 1e3 * float(np.median(ts))
    if world > 1:
        m = torch.tensor([ms], dtype=torch.float64, device=dev)
        dist.all_reduce(m, op=dist.ReduceOp.MAX)
        ms = float(m.item())
    # every gathered block carries its rank's per-stream keypoint counts
    counts = []
    if on_gpu:
        for r in range(world):
            nst = len(stream_partition(C5_STREAMS, world, r))
            counts += out[r * cap:r * cap + 4 * nst].view(torch.int32).tolist()
    return {"ranks": world, "bytes_per_rank": int(nb), "bytes_gathered": int(world * cap), "ms": round(ms, 4),
            "GB_per_s_received": round(world * cap / (ms * 1e-3) / 1e9, 2) if ms > 0 else None,
            "streams_received": len(counts), "min_keypoints_per_stream": min(counts) if counts else None}


def c5_config(torch, dist, rank, world, dev, steps, warmup, profile, stub=None, w=1920, h=1080, total=None,
              kframes=None, exchange=True):
    """C5 as configured: 64 FHD RGB-D streams in total, s -> rank s mod G, one
    extract + ComputeStereoFromRGBD per stream per frame (strong scaling inside
    the config: the stream count is fixed); then the keyframe all-gather.
    Each launch takes K consecutive frames of every stream of the rank, K =
    64 / streams per rank by default (1 on one GPU, 8 at eight: a rank's launch
    stays 64 frames, which a GPU needs to fill)."""
    total = total or C5_STREAMS
    streams = stream_partition(total, world, rank)
    k = kframes or max(1, C5_STREAMS // max(1, len(streams)))
    el, st, nk, sane, _, ex = run_config(torch, dist, rank, world, dev, w, h, 1000, streams, steps, warmup,
                                         profile, "rgbd", stub, kframes=k)
    xchg = keyframe_publish(torch, dist, world, dev, ex) if exchange else None
    ex.close()
    return {"value": round(total * k * steps / el, 2), "unit": "frames/s", "mode": "rgbd", "streams_total": total,
            "streams_per_gpu": len(streams), "frames_per_stream_per_launch": k, "frames_per_launch": len(streams) * k,
            "workload": f"rgbd {w}x{h}", "scaling": "strong", "stage_ms": st, "kps_last_frame": nk,
            "depths_last_frame": sane, "keyframe_all_gather": xchg}


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv: list) -> int:
    """`bench.py --gpus N` outside a launcher: start N ranks (one process per
    GPU) under torch.distributed.run and return its exit code.  This parent
    never touches HIP -- it runs before torch is imported -- and the ranks are
    child processes, not an exec of this one."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", str(Path(__file__).resolve())] + argv
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    # VGA streams per GPU swept (split 2, level pipeline on): 1536 -> 315.1-316.6k, 2048 -> 318.5-319.5k,
    # 2560 -> 319.5-320.3k, 3072 -> 321.5-322.3k, 4096 -> 323.7-324.2k frames/s (split 2, pipeline off:
    # 1024 -> 306k, 1536 -> 312k); 3072 keeps the resident frames at 3.8 GB per rank
    ap.add_argument("--batch", type=int, default=3072, help="streams (frames per step) per GPU")
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--height", type=int, default=480)
    ap.add_argument("--nfeatures", type=int, default=1000)
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the secondary FHD / stereo / RGB-D / C5 configurations")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--extra", default=None,
                    help="time only this EXTRAS config, 'c5' or 'dropin' (diagnostics; prints its dict)")
    ap.add_argument("--stub", action="store_true",
                    help="CPU / gloo dry run of the launcher, stream partition and batch shapes (tests)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(args.gpus, sys.argv[1:])

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        return 2
    if args.stub:
        dev = torch.device("cpu")
        if world > 1:
            dist.init_process_group("gloo")
    else:
        if world > 1:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        dev = torch.device("cuda", local)
        torch.cuda.set_device(dev)
    profile = not args.no_profile and not args.stub
    stub = (lambda w, h: StubExtractor(w, h)) if args.stub else (lambda w, h: None)
    # the stub keeps C5's stream count but not its frame size
    c5_args = (stub(args.width, args.height), args.width, args.height) if args.stub else (None,)

    if args.extra:
        res = None
        if args.extra == "c5":
            res = c5_config(torch, dist, rank, world, dev, args.steps, args.warmup, profile, *c5_args)
        if args.extra == "dropin":
            res = dropin_latency(torch, dev)
        if args.extra == "matchers":   # the drop-in ORBmatcher calls (host arrays), per call
            res = matcher_latencies()
        if args.extra in ("host_fed_vga", "host_fed_fhd"):
            res = host_fed(torch, dev, *HOST_FED[args.extra], args.steps, args.warmup)
        if args.extra in ("c5_rank8", "c5_rank8_k8"):   # one rank's share of C5 at 8 GPUs
            res = c5_config(torch, dist, rank, world, dev, args.steps, args.warmup, profile, *c5_args, total=8,
                            kframes=8 if args.extra == "c5_rank8_k8" else 1, exchange=False)
        for key, mode, ew, eh, enf, eb, unit in EXTRAS:
            if key == args.extra:
                streams = stream_partition(eb * world, world, rank)
                el2, st2, nk2, sane2, _, ex2 = run_config(torch, dist, rank, world, dev, ew, eh, enf, streams,
                                                          args.steps, args.warmup, profile, mode, stub(ew, eh),
                                                          EXTRA_SPLIT.get(key, 2), EXTRA_PIPE.get(key, 0))
                ex2.close()
                res = {"value": round(world * eb * args.steps / el2, 2), "unit": unit, "stage_ms": st2,
                       "kps_last_frame": nk2}
                if rank == 0 and st2 and not args.stub:
                    res["roofline"], _ = roofline_block(
                        level_geometry(ew, eh, enf), nk2, st2, (2 if mode == "stereo" else 1) * eb,
                        eb * args.steps / el2, mode, TRAFFIC_FILES.get(key))
        if rank == 0:
            print(json.dumps({"extra": args.extra, **(res or {"error": "unknown extra"})}), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return 0

    w, h, nf, B = args.width, args.height, args.nfeatures, args.batch
    streams = stream_partition(B * world, world, rank)          # weak scaling: B streams per GPU
    el, stages, nkp_last, nm_last, frames_per_launch, ex = run_config(
        torch, dist, rank, world, dev, w, h, nf, streams, args.steps, args.warmup, profile, "mono", stub(w, h),
        HEADLINE_SPLIT, HEADLINE_PIPE)
    ex.close()
    frames_total = world * B * args.steps
    value = frames_total / el
    ms_per_step = 1000.0 * el / args.steps
    stub_report = None
    if args.stub:
        mine = {"rank": rank, "streams": streams, "batches": sorted(set(ex.batches)), "calls": len(ex.batches),
                "checksums": ex.checksums}
        allr = [None] * world
        if world > 1:
            dist.all_gather_object(allr, mine)
        else:
            allr = [mine]
        stub_report = allr

    extras = {}
    if not args.no_extras:
        for key, mode, ew, eh, enf, eb, unit in EXTRAS:
            if args.stub:
                continue
            es = max(5, args.steps // 4)
            est = stream_partition(eb * world, world, rank)
            el2, st2, nk2, sane2, _, ex2 = run_config(torch, dist, rank, world, dev, ew, eh, enf, est, es, 2, profile,
                                                      mode, None, EXTRA_SPLIT.get(key, 2), EXTRA_PIPE.get(key, 0))
            ex2.close()
            extras[key] = {"value": round(world * eb * es / el2, 2), "unit": unit, "mode": mode,
                           "streams_per_gpu": eb, "nfeatures": enf, "stage_ms": st2,
                           "kps_last_frame": nk2, ("matches" if mode == "mono" else "depths") + "_last_frame": sane2}
            if rank == 0 and st2:
                extras[key]["roofline"], _ = roofline_block(
                    level_geometry(ew, eh, enf), nk2, st2, (2 if mode == "stereo" else 1) * eb, eb * es / el2, mode,
                    TRAFFIC_FILES.get(key))
        c5 = c5_config(torch, dist, rank, world, dev, max(5, args.steps // 4), 2, profile, *c5_args)
        extras["c5_rgbd_fhd_64_streams"] = c5
        if world > 1 and not args.stub:
            extras["keyframe_bow_all_gather"] = keyframe_exchange(torch, dist, world, dev)

    if rank == 0:
        sizes = level_geometry(w, h, nf) if not args.stub else [(w, h)]
        roof, stage_ms = roofline_block(sizes, nkp_last, stages, frames_per_launch, value / world, "mono")
        run_cpu = world == 1 and args.cpu_seconds > 0 and not args.stub
        cpu = cpu_baseline(w, h, nf, args.cpu_seconds) if run_cpu else None
        if cpu is not None:
            # the host's share of cores, all at once: the CPUs this process may
            # run on (its affinity set), capped by OMP_NUM_THREADS where the
            # box sets its share that way (16 of 256 on the GPU box)
            aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
            omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
            nthr = max(1, min(aff, omp or aff, 64))
            cpu["all_cores"] = cpu_baseline_threads(w, h, nf, max(2.0, args.cpu_seconds / 2), nthr)
            cpu["all_cores"]["threads_from"] = {"affinity_cpus": aff, "OMP_NUM_THREADS": omp or None}
            # the timing build stays selected: every CPU time in extras uses it too
        full = world == 1 and not args.no_extras and not args.stub
        matchers = matcher_latencies() if full else None
        if full:
            # one rank's share of C5 at 8 GPUs (8 streams), one frame per stream
            # per launch and K = 8 consecutive frames per stream per launch
            for kk in (1, 8):
                extras[f"c5_rank_share_8_streams_k{kk}"] = c5_config(
                    torch, dist, rank, world, dev, max(5, args.steps // 4), 2, profile, total=8, kframes=kk,
                    exchange=False)
            for key, cfg in HOST_FED.items():
                extras[key] = host_fed(torch, dev, *cfg, max(20, args.steps // 2), 3)
            extras["dropin_latency"] = dropin_latency(torch, dev)
            extras["bow_transform_orbvoc"] = bow_transform_throughput(torch)
            extras["keyframe_db_loop_query"] = kfdb_latency()
            extras["local_ba_kitti"] = local_ba_latency()
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (orb_slam_2_ros_amd.synth: value-noise + shapes, 4 resident frames per stream)",
            "config": {"workload": f"mono {w}x{h}, {nf} kp, 8 lvl, scale 1.2, FAST 20/7: ORBextractor + "
                                   "SearchForInitialization(prev frame, window 100, nnratio 0.9, checkOri)",
                       "streams_per_gpu": B, "global_batch": B * world, "parallelism": f"replicas x{world}",
                       "stream_partition": "global stream s -> rank s mod G",
                       "kps_last_frame": nkp_last, "matches_last_frame": nm_last},
            "roofline": roof,
            "stage_ms_per_step": stage_ms,
            "cpu_baseline": cpu,
            "extras": extras,
            "matchers_per_call": matchers,
        }
        if stub_report is not None:
            line["stub"] = stub_report
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
