"""Does the creation-order tie rule agree with the reference on a real heap?
(CPU only, the oracle is the candidate source.)

DistributeOctTree sorts (size, ExtractorNode*) pairs (ORBextractor.cc:705-708),
so equal-size nodes split in heap-address order.  tools/tie_heap/tie_heap
replays operator()'s allocation sequence up to the last level's tree in a fresh
thread under this host's glibc and sorts by the real addresses; this script
feeds it the oracle's per-level FAST candidates (with the per-cell counts the
cell vectors are grown to) of the bench's scenes and compares each level's
selection with the oracle's creation-order rule (orbo_distribute) and with
reverse creation order.

Two heap states per camera: frame 0 (the first extraction in a fresh thread)
and frame 1 of the same scene, extracted after frame 0 in the same thread (the
extractor's level buffers and the previous frame's outputs replaced as the
reference replaces them).

    python tools/tie_heap.py [--scenes 32] [--out profiles/r04_tie_heap.txt]
"""
import argparse
import ctypes
import subprocess
import sys
import tempfile
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402
from oracle import oracle  # noqa: E402

EXE = ROOT / "tools" / "tie_heap" / "tie_heap"
EXE_CHECK = ROOT / "tools" / "tie_heap" / "tie_heap_creation"   # -DTIE_CREATION: must equal the oracle
EXE_SIM = ROOT / "tools" / "tie_heap" / "tie_heap_sim"   # -DTIE_SIM: a deterministic tcache/fastbin LIFO model
CONFIGS = [  # (name, w, h, nfeatures, mode)
    ("C2 VGA mono", 640, 480, 1000, "mono"),
    ("C3 EuRoC stereo", 752, 480, 1200, "stereo"),
    ("C4 KITTI stereo", 1241, 376, 2000, "stereo"),
    ("FHD stereo", 1920, 1080, 1000, "stereo"),
]


def build():
    src = EXE.parent / "tie_heap.cpp"
    for exe, flags in ((EXE, []), (EXE_CHECK, ["-DTIE_CREATION"]), (EXE_SIM, ["-DTIE_SIM"])):
        if not exe.exists() or exe.stat().st_mtime < src.stat().st_mtime:
            subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", *flags, str(src), "-o", str(exe)], check=True)


def set_mode(m):
    f = oracle.lib().orbo_set_tie_mode
    f.restype = None
    f.argtypes = [ctypes.c_int]
    f(m)


def levels_of(img, nf):
    """Per level (w, h, quota, candidates, cell counts) of one image."""
    h, w = img.shape
    lw = np.zeros(8, np.int32); lh = np.zeros(8, np.int32); q = np.zeros(8, np.int32); sc = np.zeros(8, np.float32)
    p = lambda a: ctypes.c_void_p(a.ctypes.data)
    oracle.lib().orbo_levels(w, h, nf, ctypes.c_float(1.2), 8, p(lw), p(lh), p(q), p(sc))
    pyr = oracle.pyramid(np.ascontiguousarray(img)) if hasattr(oracle, "pyramid") else None
    out = []
    for l in range(8):
        lvl = pyr[l]
        cands, cells = oracle.level_candidates_cells(lvl)
        out.append((int(lw[l]), int(lh[l]), int(q[l]), cands, cells))
    return out


def run_heap(frames, nf, exe=EXE):
    """frames: list of levels_of() results, run back to back in one fresh thread."""
    with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as fp:
        fp.write(np.array([8, nf, len(frames)], np.int32).tobytes())
        for lv in frames:
            for (w, h, q, c, cells) in lv:
                fp.write(np.array([w, h, q, len(c), len(cells)], np.int32).tobytes())
                fp.write(np.ascontiguousarray(c, np.int32).tobytes())
                fp.write(np.ascontiguousarray(cells, np.int32).tobytes())
        name = fp.name
    r = subprocess.run([str(exe), name], capture_output=True, text=True, check=True)
    Path(name).unlink()
    res = {}
    for line in r.stdout.splitlines():
        v = [int(t) for t in line.split()]
        res[(v[0], v[1])] = v[3:3 + v[2]]
    return res


def compare(a, b):
    """(identical, same set, keypoints selected differently, at another position)"""
    same = a == b
    sa, sb = set(a), set(b)
    diff = len(sa - sb)
    moved = sum(1 for x, y in zip(a, b) if x != y) + abs(len(a) - len(b))
    return same, sa == sb, diff, moved


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenes", type=int, default=bench.UNIQUE_SCENES)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    build()
    lines = [__doc__.strip().splitlines()[0], ""]
    import platform
    glibc = " ".join(platform.libc_ver())
    lines.append(f"host glibc: {glibc}; replay: tools/tie_heap/tie_heap.cpp (fresh thread per camera stream)")
    lines.append("")
    for name, w, h, nf, mode in CONFIGS:
        # per heap state: [images, identical to creation, same set as creation, identical to reverse, kp differing (sum),
        #                  kp moved (sum), keypoints]
        st = {0: np.zeros(7, np.int64), 1: np.zeros(7, np.int64)}
        lvl_stats = np.zeros(3, np.int64)   # levels, levels identical (creation), identical (reverse)
        rep = np.zeros(4, np.int64)         # images, identical, same set, keypoints differing
        sm = {0: np.zeros(5, np.int64), 1: np.zeros(5, np.int64)}   # the LIFO model vs the real heap
        for sc in range(args.scenes):
            frs = bench.scene_frames(mode, w, h, sc)
            cams = [0, 1] if mode == "stereo" else [0]
            for cam in cams:
                imgs = [np.ascontiguousarray(frs[t][cam] if mode == "stereo" else frs[t]) for t in (0, 1)]
                lvs = [levels_of(im, nf) for im in imgs]
                heap = run_heap(lvs, nf)
                check = run_heap(lvs, nf, EXE_CHECK)
                # the reference's own repeatability: frame 0's image extracted
                # again in the same thread, after frame 1 (another heap state)
                again = run_heap([lvs[0], lvs[1], lvs[0]], nf)
                r0 = [(l, i) for l in range(8) for i in heap[(0, l)]]
                r2 = [(l, i) for l in range(8) for i in again[(2, l)]]
                rep += [1, r0 == r2, set(r0) == set(r2), len(set(r0) - set(r2))]
                sim = run_heap(lvs, nf, EXE_SIM)
                for t in (0, 1):
                    sel_c, sel_r, sel_h, sel_s = [], [], [], []
                    for l, (lw, lh, q, c, cells) in enumerate(lvs[t]):
                        set_mode(0)
                        a = list(oracle.distribute(c, lw, lh, q))
                        set_mode(1)
                        r = list(oracle.distribute(c, lw, lh, q))
                        set_mode(0)
                        hh = heap[(t, l)]
                        if check[(t, l)] != a:
                            raise SystemExit(f"replica check failed: {name} scene {sc} cam {cam} t {t} level {l}")
                        lvl_stats += [1, a == hh, r == hh]
                        sel_c += [(l, i) for i in a]
                        sel_r += [(l, i) for i in r]
                        sel_h += [(l, i) for i in hh]
                        sel_s += [(l, i) for i in sim[(t, l)]]
                    same, sset, diff, moved = compare(sel_c, sel_h)
                    st[t] += [1, same, sset, sel_r == sel_h, diff, moved, len(sel_h)]
                    same, sset, diff, moved = compare(sel_s, sel_h)
                    sm[t] += [1, same, sset, diff, moved]
        lines.append(f"{name} {w}x{h}, {nf} kp, {args.scenes} scenes")
        for t, tag in ((0, "frame 0 (fresh thread)"), (1, "frame 1 (after frame 0, same thread)")):
            s = st[t]
            n = max(1, s[0])
            lines.append(f"  {tag}: {s[0]} images")
            lines.append(f"    identical to creation order (set and order)  {s[1]} of {s[0]}")
            lines.append(f"    same keypoint set as creation order          {s[2]} of {s[0]}")
            lines.append(f"    identical to reverse creation order          {s[3]} of {s[0]}")
            lines.append(f"    keypoints selected differently               {s[4] / n:.2f} per image "
                         f"({100 * s[4] / max(1, s[6]):.2f} %)")
            lines.append(f"    keypoints at another output position         {s[5] / n:.1f} per image "
                         f"({100 * s[5] / max(1, s[6]):.1f} %)")
            m = sm[t]
            lines.append(f"    the deterministic LIFO model (tie_heap_sim) vs the real heap: identical {m[1]} of {m[0]}, "
                         f"same set {m[2]} of {m[0]}, {m[3] / n:.2f} keypoints selected differently, "
                         f"{m[4] / n:.1f} at another position per image")
        lines.append(f"  levels identical to creation / reverse order: {lvl_stats[1]} / {lvl_stats[2]} of {lvl_stats[0]}")
        lines.append(f"  the same image on the real heap, fresh thread vs after two other extractions: identical "
                     f"{rep[1]} of {rep[0]}, same set {rep[2]} of {rep[0]}, {rep[3] / max(1, rep[0]):.2f} keypoints "
                     f"selected differently per image")
        lines.append("")
        print("\n".join(lines[-17:]), flush=True)
    text = "\n".join(lines)
    if args.out:
        Path(args.out).write_text(text + "\n")


if __name__ == "__main__":
    main()
