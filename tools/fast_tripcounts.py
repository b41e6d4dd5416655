"""Trip counts of k_fast's loops on the bench's VGA frames (CPU, numpy):
per cell, the compass passes (R = 64 / quads-per-row rows each), the
compaction iterations (the largest survivor count of a lane in the pass), the
arc-score chunks (64 survivors each) and the NMS chunks, for the iniThFAST
pass and for the minThFAST pass the reference runs on a cell left empty
(ORBextractor.cc:842-850).  Multiplied by the per-iteration VALU counts of
the kernel's assembly (tools/isa_mix.py) this is k_fast's dynamic VALU split.

    python tools/fast_tripcounts.py [scenes]
"""
import math
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402
from oracle import oracle  # noqa: E402

CIRC = [(3, 0), (3, 1), (2, 2), (1, 3), (0, 3), (-1, 3), (-2, 2), (-3, 1), (-3, 0), (-3, -1), (-2, -2), (-1, -3),
        (0, -3), (1, -3), (2, -2), (3, -1)]


def level_maps(img):
    """Compass pre-test margin d and arc score S for every pixel >= 3 px from the border."""
    im = img.astype(np.int32)
    H, W = im.shape
    v = im[3:H - 3, 3:W - 3]
    P = np.stack([im[3 + dy:H - 3 + dy, 3 + dx:W - 3 + dx] for dy, dx in CIRC])
    a0, a4, a8, a12 = P[0], P[4], P[8], P[12]
    hi = np.minimum(np.maximum(a0, a8), np.maximum(a4, a12))
    lo = np.maximum(np.minimum(a0, a8), np.minimum(a4, a12))
    d = np.maximum(np.maximum(hi - v, 0), np.maximum(v - lo, 0))
    S = np.full(v.shape, -10 ** 6)
    for s in range(16):
        idx = [(s + k) % 16 for k in range(9)]
        S = np.maximum(S, np.maximum(P[idx].min(0) - v, v - P[idx].max(0)))
    dm = np.zeros((H, W), np.int32)
    Sm = np.full((H, W), -1, np.int32)
    dm[3:H - 3, 3:W - 3] = d
    Sm[3:H - 3, 3:W - 3] = S
    return dm, Sm


def cells(w, h):
    minB, maxBX, maxBY = 16, w - 16, h - 16
    width, height = maxBX - minB, maxBY - minB
    nC, nR = int(width / 30), int(height / 30)
    wC, hC = math.ceil(width / nC), math.ceil(height / nR)
    for i in range(nR):
        y0 = minB + i * hC
        y1 = min(y0 + hC + 6, maxBY)
        if y0 >= maxBY - 3:
            continue
        for j in range(nC):
            x0 = minB + j * wC
            x1 = min(x0 + wC + 6, maxBX)
            if x0 >= maxBX - 6:
                continue
            yield x0 + 3, y0 + 3, x1 - 3, y1 - 3   # FAST's evaluated interior


def one_pass(dm, Sm, cx0, cy0, cx1, cy1, th):
    cw, ch = cx1 - cx0, cy1 - cy0
    o = (cx0 - 3) & 3
    qc0 = (o + 3) & ~3
    nq = ((o + 2 + cw) >> 2) - (qc0 >> 2) + 1
    R = 64 // nq
    passes = math.ceil(ch / R)
    d = dm[cy0:cy1, cx0:cx1]
    surv = d > th
    # per pass: the largest per-lane (quad) survivor count
    comp_it = 0
    xs = np.arange(cw)
    quad = (xs + (o + 3) - qc0) // 4   # quad index of interior column x
    for p in range(passes):
        rows = surv[p * R:(p + 1) * R]
        if rows.size == 0:
            continue
        cnt = np.zeros((rows.shape[0], nq), np.int32)
        for q in range(nq):
            cnt[:, q] = rows[:, quad == q].sum(1)
        comp_it += int(cnt.max())
    ns = int(surv.sum())
    S = Sm[cy0:cy1, cx0:cx1]
    corner = surv & (S > th)
    nc = int(corner.sum())
    # strict 3x3 NMS on S-1 inside the cell
    sc = np.where(corner, S - 1, 0)
    pad = np.pad(sc, 1)
    keep = corner.copy()
    for dy in (-1, 0, 1):
        for dx in (-1, 0, 1):
            if dy or dx:
                keep &= sc > pad[1 + dy:1 + dy + ch, 1 + dx:1 + dx + cw]
    return dict(passes=passes, comp_it=comp_it, arc_chunks=math.ceil(ns / 64), nms_chunks=math.ceil(nc / 64),
                surv=ns, corners=nc, kept=int(keep.sum()))


def main():
    scenes = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    tot = {}
    ncells = nmin = 0
    for sc in range(scenes):
        img = bench.scene_frames("mono", 640, 480, sc)[0]
        for lvl in oracle.pyramid(np.ascontiguousarray(img)):
            dm, Sm = level_maps(lvl)
            h, w = lvl.shape
            for c in cells(w, h):
                ncells += 1
                r = one_pass(dm, Sm, *c, 20)
                for k, v in r.items():
                    tot["ini_" + k] = tot.get("ini_" + k, 0) + v
                if r["kept"] == 0:
                    nmin += 1
                    r = one_pass(dm, Sm, *c, 7)
                    for k, v in r.items():
                        tot["min_" + k] = tot.get("min_" + k, 0) + v
    print(f"{scenes} VGA frames, {ncells} cells ({ncells / scenes:.0f} per frame), "
          f"minThFAST pass in {nmin} ({100 * nmin / ncells:.1f} %)")
    for k in sorted(tot):
        print(f"  {k:18s} {tot[k] / ncells:8.2f} per cell")


if __name__ == "__main__":
    main()
