"""How much of the extractor's output depends on the reference's pointer tie rule
(DistributeOctTree sorts (size, ExtractorNode*) pairs, ORBextractor.cc:705-708:
nodes of equal key count are ordered by heap address, which the restatement
replaces by creation order).  CPU only: runs the oracle's
extraction over the bench's frames and reads its tie counters
(orbo_tie_stats, oracle/orbx_oracle.cpp).

    python tools/tie_exposure.py [--out profiles/r03_tie_exposure.txt]

Per config: levels run, levels with a final phase, and two exposures --
"order": a final round splits >= 2 nodes of equal size, so the list order of
their children (the output order of those keypoints) follows the tie rule;
"set": the round's cutoff falls inside a group of equal-size nodes, so WHICH of
them are split (and so which keypoints are selected) follows the tie rule.
"""
import argparse
import ctypes
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402
from oracle import oracle  # noqa: E402

CONFIGS = [  # (name, w, h, nfeatures, mode)
    ("C2 VGA mono", 640, 480, 1000, "mono"),
    ("C3 EuRoC stereo", 752, 480, 1200, "stereo"),
    ("C4 KITTI stereo", 1241, 376, 2000, "stereo"),
    ("FHD stereo", 1920, 1080, 1000, "stereo"),
]
ALT_MODES = (1, 2, 3, 4)
NAMES = ["levels", "final-phase levels", "final rounds", "rounds w/ order exposure", "nodes in order groups",
         "rounds w/ set exposure", "nodes in set groups", "levels w/ any exposure", "levels w/ set exposure"]


def stats(reset=True):
    f = oracle.lib().orbo_tie_stats
    f.restype = None
    f.argtypes = [ctypes.c_void_p, ctypes.c_int]
    out = np.zeros(9, np.int64)
    f(out.ctypes.data, int(reset))
    return out


def set_mode(m):
    f = oracle.lib().orbo_set_tie_mode
    f.restype = None
    f.argtypes = [ctypes.c_int]
    f(m)


def kp_keys(k):
    return [(round(float(p[0]), 3), round(float(p[1]), 3), int(p[5])) for p in k]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--scenes", type=int, default=bench.UNIQUE_SCENES)
    args = ap.parse_args()
    lines = [__doc__.strip().splitlines()[0], ""]
    stats(True)
    for name, w, h, nf, mode in CONFIGS:
        tot = np.zeros(9, np.int64)
        nimg = nkp = 0
        kp_set = 0
        alt_changed = alt_moved = alt_imgs_diff = 0
        alt_max = 0
        for sc in range(args.scenes):
            fr = bench.scene_frames(mode, w, h, sc)[0]   # frame t = 0 of the scene
            for img in (fr if mode == "stereo" else [fr]):
                before = tot.copy()
                k, _ = oracle.extract(np.ascontiguousarray(img), nf)
                tot += stats(True)
                after = tot
                nimg += 1
                nkp += len(k)
                if after[5] > before[5]:
                    kp_set += 1
                # the same image under other tie orders: keypoints selected
                # differently (set) and keypoints at another output position
                base = kp_keys(k)
                for m in ALT_MODES:
                    set_mode(m)
                    ka, _ = oracle.extract(np.ascontiguousarray(img), nf)
                    set_mode(0)
                    alt = kp_keys(ka)
                    ch = len(set(base) - set(alt))
                    mv = sum(1 for a, b in zip(base, alt) if a != b) + abs(len(base) - len(alt))
                    alt_changed += ch
                    alt_moved += mv
                    alt_max = max(alt_max, ch)
                    alt_imgs_diff += int(ch > 0)
                stats(True)
        s = tot
        lines.append(f"{name} {w}x{h}, {nf} kp, {nimg} images ({args.scenes} scenes, frame 0), {nkp} keypoints")
        for n, v in zip(NAMES, s):
            lines.append(f"    {n:28s} {v}")
        lines.append(f"    images with a set exposure   {kp_set} of {nimg}")
        na = nimg * len(ALT_MODES)
        lines.append(f"    under {len(ALT_MODES)} other tie orders (reverse creation + {len(ALT_MODES) - 1} seeded random), "
                     f"{na} extractions:")
        lines.append(f"      extractions whose keypoint set differs   {alt_imgs_diff} of {na}")
        lines.append(f"      keypoints selected differently           {alt_changed / na:.2f} per image "
                     f"({100 * alt_changed / max(1, nkp * len(ALT_MODES)):.2f} %), max {alt_max}")
        lines.append(f"      keypoints at another output position     {alt_moved / na:.1f} per image "
                     f"({100 * alt_moved / max(1, nkp * len(ALT_MODES)):.1f} %)")
        lines.append("")
    text = "\n".join(lines)
    print(text)
    if args.out:
        Path(args.out).write_text(text + "\n")


if __name__ == "__main__":
    main()
