"""Pure-Python restatements of the reference hot path for SMALL inputs.

A third, independent formulation next to the C++ oracle (oracle/) and the HIP
kernels, written straight from the reference sources and the OpenCV 3.2
semantics in DESIGN.md §3; used only to cross-check the oracle on small
seeded cases (the reference itself ships no test vectors: SURVEY.md §4).
numpy float32 scalars are used wherever the reference computes in float.
"""
from __future__ import annotations

import math

import numpy as np

f32 = np.float32


def cv_round(v) -> int:
    return int(np.rint(v))  # half-to-even, as x86 cvRound


def cv_floor(v) -> int:
    return int(math.floor(float(v)))


# ---- cv::resize INTER_LINEAR 8U, OpenCV 3.2 (ORBextractor.cc:1171) -----------
def resize_linear(src: np.ndarray, dw: int, dh: int) -> np.ndarray:
    sh, sw = src.shape
    scale_x, scale_y = 1.0 / (dw / sw), 1.0 / (dh / sh)

    def taps(ssize, dsize, scale, is_x):
        out, xmax = [], dsize
        for d in range(dsize):
            f = f32((d + 0.5) * scale - 0.5)
            s = cv_floor(f)
            f = f32(f - f32(s))
            if is_x:
                if s < 0:
                    f, s = f32(0), 0
                if s + 1 >= ssize:
                    xmax = min(xmax, d)
                    if s >= ssize - 1:
                        f, s = f32(0), ssize - 1
            a0 = max(-32768, min(32767, cv_round(f32(f32(1) - f) * f32(2048))))
            a1 = max(-32768, min(32767, cv_round(f * f32(2048))))
            out.append((s, a0, a1))
        return out, xmax

    xt, xmax = taps(sw, dw, scale_x, True)
    yt, _ = taps(sh, dh, scale_y, False)
    xs = 0
    while xs <= dw - 16:
        xs += 16
    while xs < dw - 4:
        xs += 4
    dst = np.zeros((dh, dw), np.uint8)
    src = src.astype(np.int64)
    for dy, (sy, b0, b1) in enumerate(yt):
        r0, r1 = min(max(sy, 0), sh - 1), min(max(sy + 1, 0), sh - 1)
        for dx, (sx, a0, a1) in enumerate(xt):
            if dx < xmax:
                h0 = src[r0, sx] * a0 + src[r0, sx + 1] * a1
                h1 = src[r1, sx] * a0 + src[r1, sx + 1] * a1
            else:
                h0, h1 = src[r0, sx] * 2048, src[r1, sx] * 2048
            if dx < xs:
                v = ((((h0 >> 4) * b0) >> 16) + (((h1 >> 4) * b1) >> 16) + 2) >> 2
            else:
                v = (h0 * b0 + h1 * b1 + (1 << 21)) >> 22
            dst[dy, dx] = min(max(v, 0), 255)
    return dst


# ---- GaussianBlur 7x7 sigma 2 REFLECT_101, OpenCV 3.2 (ORBextractor.cc:1130) --
def gauss_taps() -> list:
    cf = [f32(math.exp(-0.5 / 4.0 * (i - 3) ** 2)) for i in range(7)]
    s = 0.0
    for c in cf:
        s += float(c)
    s = 1.0 / s
    cf = [f32(float(c) * s) for c in cf]
    return [cv_round(f32(c) * f32(256)) for c in cf]


def gauss7(img: np.ndarray) -> np.ndarray:
    h, w = img.shape
    k = gauss_taps()

    def r101(p, n):
        while p < 0 or p >= n:
            p = -p if p < 0 else 2 * n - p - 2
        return p

    src = img.astype(np.int64)
    rows = np.zeros((h, w), np.int64)
    for y in range(h):
        for x in range(w):
            rows[y, x] = sum(k[t] * src[y, r101(x + t - 3, w)] for t in range(7))
    xs = w & ~3
    kf = [f32(f32(k[3 + i]) * f32(1.0 / 65536.0)) for i in range(4)]
    out = np.zeros((h, w), np.uint8)
    for y in range(h):
        R = [rows[r101(y + t - 3, h)] for t in range(7)]
        for x in range(w):
            if x < xs:
                s = f32(f32(R[3][x]) * kf[0]) + f32(0)
                for t in range(1, 4):
                    s = f32(s + f32(f32(R[3 + t][x] + R[3 - t][x]) * kf[t]))
                v = cv_round(s)
                out[y, x] = min(max(v, 0), 255)
            else:
                s = k[3] * R[3][x] + sum(k[3 + t] * (R[3 + t][x] + R[3 - t][x]) for t in range(1, 4))
                out[y, x] = min(max((s + (1 << 15)) >> 16, 0), 255)
    return out


# ---- FAST-9 arc score (cv::FAST TYPE_9_16 + cornerScore<16>) ----------------
CIRCLE = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3),
          (0, -3), (-1, -3), (-2, -2), (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]


def arc_score(img: np.ndarray, x: int, y: int) -> int:
    v = int(img[y, x])
    d = [v - int(img[y + dy, x + dx]) for dx, dy in CIRCLE]
    best = -10 ** 9
    for k in range(16):
        arc = [d[(k + i) % 16] for i in range(9)]
        best = max(best, min(arc), min(-a for a in arc))
    return best


def fast_cell(img: np.ndarray, threshold: int) -> list:
    """cv::FAST(img, kps, threshold, nonmax=true) on a whole (sub)image."""
    h, w = img.shape
    sc = np.zeros((h, w), np.int64)
    for y in range(3, h - 3):
        for x in range(3, w - 3):
            s = arc_score(img, x, y)
            if s > threshold:
                sc[y, x] = s - 1
    out = []
    for y in range(3, h - 3):
        for x in range(3, w - 3):
            s = sc[y, x]
            if s and all(s > sc[y + dy, x + dx] for dy in (-1, 0, 1) for dx in (-1, 0, 1) if dx or dy):
                out.append((x, y, int(s)))
    return out


# ---- DistributeOctTree (ORBextractor.cc:561-787), literal list semantics -----
class _Node:
    __slots__ = ("x0", "y0", "x1", "y1", "keys", "no_more", "seq")

    def __init__(self, x0, y0, x1, y1, seq=0):
        self.x0, self.y0, self.x1, self.y1 = x0, y0, x1, y1
        self.keys, self.no_more, self.seq = [], False, seq


def distribute(cands, w: int, h: int, N: int) -> list:
    """cands: list of (x, y, score) in level coordinates; returns indices."""
    if not cands:
        return []
    minx, maxx, miny, maxy = 16, w - 16, 16, h - 16
    nini = round_half_away(f32(f32(maxx - minx) / f32(maxy - miny)))
    hx = f32(f32(maxx - minx) / f32(nini))
    seq = [0]
    nodes = []
    for i in range(nini):
        nodes.append(_Node(int(f32(hx * f32(i))), 0, int(f32(hx * f32(i + 1))), maxy - miny))
    for k, (x, y, _) in enumerate(cands):
        nodes[int(f32(f32(x - 16) / hx))].keys.append(k)
    lst = [n for n in nodes if n.keys]
    for n in lst:
        n.no_more = len(n.keys) == 1

    def divide(n):
        hxx = int(math.ceil((n.x1 - n.x0) / 2))
        hyy = int(math.ceil((n.y1 - n.y0) / 2))
        mx, my = n.x0 + hxx, n.y0 + hyy
        ch = [_Node(n.x0, n.y0, mx, my), _Node(mx, n.y0, n.x1, my),
              _Node(n.x0, my, mx, n.y1), _Node(mx, my, n.x1, n.y1)]
        for k in n.keys:
            x, y = cands[k][0] - 16, cands[k][1] - 16
            q = (0 if y < my else 2) if x < mx else (1 if y < my else 3)
            ch[q].keys.append(k)
        for c in ch:
            c.no_more = len(c.keys) == 1
        return ch

    finish = False
    expand = []
    while not finish:
        prev = len(lst)
        n_to_expand = 0
        expand = []
        i = 0
        while i < len(lst):
            n = lst[i]
            if n.no_more:
                i += 1
                continue
            for c in divide(n):
                if c.keys:
                    c.seq = seq[0]
                    seq[0] += 1
                    lst.insert(0, c)
                    i += 1
                    if len(c.keys) > 1:
                        n_to_expand += 1
                        expand.append(c)
            del lst[i]
        if len(lst) >= N or len(lst) == prev:
            finish = True
        elif len(lst) + n_to_expand * 3 > N:
            while not finish:
                prev = len(lst)
                todo = sorted(expand, key=lambda n: (len(n.keys), n.seq))
                expand = []
                for n in reversed(todo):
                    for c in divide(n):
                        if c.keys:
                            c.seq = seq[0]
                            seq[0] += 1
                            lst.insert(0, c)
                            if len(c.keys) > 1:
                                expand.append(c)
                    lst.remove(n)
                    if len(lst) >= N:
                        break
                if len(lst) >= N or len(lst) == prev:
                    finish = True
    res = []
    for n in lst:
        best = n.keys[0]
        for k in n.keys[1:]:
            if cands[k][2] > cands[best][2]:
                best = k
        res.append(best)
    return res


# ---- SearchForInitialization (ORBmatcher.cc:406-521) ------------------------
def hamming(a: np.ndarray, b: np.ndarray) -> int:
    return int(np.unpackbits(np.bitwise_xor(a, b)).sum())


def search_for_initialization(k1, d1, k2, d2, w, h, prev, window, nnratio, check_ori):
    GC, GR, HL = 64, 48, 30
    invw, invh = f32(f32(GC) / f32(w)), f32(f32(GR) / f32(h))
    grid = {}
    for i, kp in enumerate(k2):
        px = int(round_half_away(f32(kp["x"] * invw)))
        py = int(round_half_away(f32(kp["y"] * invh)))
        if 0 <= px < GC and 0 <= py < GR:
            grid.setdefault((px, py), []).append(i)
    m12 = [-1] * len(k1)
    m21 = [-1] * len(k2)
    mdist = [2 ** 31 - 1] * len(k2)
    rot = [[] for _ in range(HL)]
    r = f32(window)
    factor = f32(f32(1.0) / f32(HL))
    for i1 in range(len(k1)):
        if k1[i1]["octave"] > 0:
            continue
        x, y = f32(prev[i1, 0]), f32(prev[i1, 1])
        cx0 = max(0, math.floor(f32(f32(x - r) * invw)))
        cx1 = min(GC - 1, math.ceil(f32(f32(x + r) * invw)))
        cy0 = max(0, math.floor(f32(f32(y - r) * invh)))
        cy1 = min(GR - 1, math.ceil(f32(f32(y + r) * invh)))
        cand = []
        if cx0 < GC and cx1 >= 0 and cy0 < GR and cy1 >= 0:
            for ix in range(cx0, cx1 + 1):
                for iy in range(cy0, cy1 + 1):
                    for j in grid.get((ix, iy), []):
                        if k2[j]["octave"] != 0:
                            continue
                        if abs(f32(k2[j]["x"] - x)) < r and abs(f32(k2[j]["y"] - y)) < r:
                            cand.append(j)
        if not cand:
            continue
        best, best2, bi = 2 ** 31 - 1, 2 ** 31 - 1, -1
        for i2 in cand:
            dist = hamming(d1[i1], d2[i2])
            if mdist[i2] <= dist:
                continue
            if dist < best:
                best2, best, bi = best, dist, i2
            elif dist < best2:
                best2 = dist
        if best <= 50 and f32(best) < f32(f32(best2) * f32(nnratio)):
            if m21[bi] >= 0:
                m12[m21[bi]] = -1
            m12[i1], m21[bi], mdist[bi] = bi, i1, best
            if check_ori:
                rv = f32(k1[i1]["angle"] - k2[bi]["angle"])
                if rv < 0.0:
                    rv = f32(rv + f32(360.0))
                b = int(round_half_away(f32(rv * factor)))
                if b == HL:
                    b = 0
                rot[b].append(i1)
    if check_ori:
        sizes = [len(b) for b in rot]
        m1 = m2 = m3 = 0
        i1_ = i2_ = i3_ = -1
        for i, s in enumerate(sizes):
            if s > m1:
                m3, m2, m1, i3_, i2_, i1_ = m2, m1, s, i2_, i1_, i
            elif s > m2:
                m3, m2, i3_, i2_ = m2, s, i2_, i
            elif s > m3:
                m3, i3_ = s, i
        if f32(m2) < f32(f32(0.1) * f32(m1)):
            i2_ = i3_ = -1
        elif f32(m3) < f32(f32(0.1) * f32(m1)):
            i3_ = -1
        for i, b in enumerate(rot):
            if i in (i1_, i2_, i3_):
                continue
            for idx in b:
                m12[idx] = -1
    prev = prev.copy()
    for i1, m in enumerate(m12):
        if m >= 0:
            prev[i1, 0], prev[i1, 1] = k2[m]["x"], k2[m]["y"]
    return sum(1 for m in m12 if m >= 0), np.array(m12, np.int32), prev


def round_half_away(v) -> int:
    v = float(v)
    return int(math.floor(v + 0.5)) if v >= 0 else -int(math.floor(-v + 0.5))


# ---- Frame::ComputeStereoMatches (Frame.cc:502-676) --------------------------
def compute_stereo_matches(pyr_l, pyr_r, scale, inv_scale, kl, dl, kr, dr, mbf, mb):
    """Straight transcription of the reference loop (vRowIndices as lists,
    candidates in right-index order); returns (uright, depth, kept)."""
    n = len(kl)
    ur = np.full(n, -1, np.float32)
    dp = np.full(n, -1, np.float32)
    nrows = pyr_l[0].shape[0]
    rows = [[] for _ in range(nrows)]
    for iR in range(len(kr)):
        y = f32(kr["y"][iR])
        r = f32(f32(2.0) * f32(scale[kr["octave"][iR]]))
        maxr, minr = int(math.ceil(f32(y + r))), int(math.floor(f32(y - r)))
        for yi in range(minr, maxr + 1):
            if 0 <= yi < nrows:
                rows[yi].append(iR)
    mbf, mb = f32(mbf), f32(mb)
    maxD = f32(mbf / mb)
    dist_idx = []
    for iL in range(n):
        uL, vL, lvl = f32(kl["x"][iL]), f32(kl["y"][iL]), int(kl["octave"][iL])
        if not (0 <= vL < nrows):
            continue
        cands = rows[int(vL)]
        if not cands:
            continue
        minU, maxU = f32(uL - maxD), uL
        if maxU < 0:
            continue
        best, bidx = 100, 0
        for iR in cands:
            if kr["octave"][iR] < lvl - 1 or kr["octave"][iR] > lvl + 1:
                continue
            uR = f32(kr["x"][iR])
            if minU <= uR <= maxU:
                d = hamming(dl[iL], dr[iR])
                if d < best:
                    best, bidx = d, iR
        if best >= 75:
            continue
        sf = f32(inv_scale[lvl])
        suL = f32(round_half_away(f32(uL * sf)))
        svL = f32(round_half_away(f32(vL * sf)))
        suR0 = f32(round_half_away(f32(f32(kr["x"][bidx]) * sf)))
        IL, IR = pyr_l[lvl].astype(np.int64), pyr_r[lvl].astype(np.int64)
        h, w = IL.shape
        if svL - 5 < 0 or svL + 6 > h or suL - 5 < 0 or suL + 6 > w:
            continue
        if suR0 < 0 or suR0 + 11 >= w or suR0 - 10 < 0:
            continue
        r0, c0 = int(svL) - 5, int(suL) - 5
        wl = IL[r0:r0 + 11, c0:c0 + 11]
        wl = wl - wl[5, 5]
        sads = []
        for inc in range(-5, 6):
            cr = int(suR0) + inc - 5
            wr = IR[r0:r0 + 11, cr:cr + 11]
            sads.append(int(np.abs(wl - (wr - wr[5, 5])).sum()))
        bi = int(np.argmin(sads))     # first minimum
        if bi in (0, 10):
            continue
        d1, d2, d3 = f32(sads[bi - 1]), f32(sads[bi]), f32(sads[bi + 1])
        delta = f32(f32(d1 - d3) / f32(f32(2.0) * f32(f32(d1 + d3) - f32(f32(2.0) * d2))))
        if delta < -1 or delta > 1:
            continue
        bestuR = f32(f32(scale[lvl]) * f32(f32(suR0 + f32(bi - 5)) + delta))
        disp = f32(uL - bestuR)
        if 0 <= disp < maxD:
            if disp <= 0:
                disp = f32(0.01)
                bestuR = f32(float(uL) - 0.01)
            dp[iL] = f32(mbf / disp)
            ur[iL] = bestuR
            dist_idx.append((sads[bi], iL))
    if not dist_idx:
        return ur, dp, 0
    dist_idx.sort()
    median = f32(dist_idx[len(dist_idx) // 2][0])
    th = f32(f32(f32(1.5) * f32(1.4)) * median)
    kept = len(dist_idx)
    for d, i in reversed(dist_idx):
        if f32(d) < th:
            break
        ur[i] = dp[i] = -1
        kept -= 1
    return ur, dp, kept


# ---- ORBmatcher::SearchByProjection x4 / Fuse x2 search (ORBmatcher.cc) -------
def _grid(keys, bounds):
    minX, maxX, minY, maxY = [f32(b) for b in bounds]
    invW, invH = f32(f32(64) / f32(maxX - minX)), f32(f32(48) / f32(maxY - minY))
    cells = {}
    for i in range(len(keys)):
        px = round_half_away(f32(f32(f32(keys["x"][i]) - minX) * invW))
        py = round_half_away(f32(f32(f32(keys["y"][i]) - minY) * invH))
        if 0 <= px < 64 and 0 <= py < 48:
            cells.setdefault((px, py), []).append(i)
    return minX, minY, invW, invH, cells


def _area(keys, g, x, y, r, min_level, max_level):
    minX, minY, invW, invH, cells = g
    x, y, r = f32(x), f32(y), f32(r)
    c0 = max(0, math.floor(f32(f32(f32(x - minX) - r) * invW)))
    if c0 >= 64:
        return []
    c1 = min(63, math.ceil(f32(f32(f32(x - minX) + r) * invW)))
    if c1 < 0:
        return []
    r0 = max(0, math.floor(f32(f32(f32(y - minY) - r) * invH)))
    if r0 >= 48:
        return []
    r1 = min(47, math.ceil(f32(f32(f32(y - minY) + r) * invH)))
    if r1 < 0:
        return []
    check = min_level > 0 or max_level >= 0
    out = []
    for ix in range(c0, c1 + 1):
        for iy in range(r0, r1 + 1):
            for j in cells.get((ix, iy), []):
                if check and (keys["octave"][j] < min_level or (max_level >= 0 and keys["octave"][j] > max_level)):
                    continue
                if abs(f32(f32(keys["x"][j]) - x)) < r and abs(f32(f32(keys["y"][j]) - y)) < r:
                    out.append(j)
    return out


def search_by_projection(variant, keys, desc, q, qdesc, bounds, uright=None, mp_state=None, inv_sigma2=None,
                         th_dist=100, nnratio=0.6, check_ori=True):
    g = _grid(keys, bounds)
    n = len(keys)
    has = [bool(mp_state[i] & 1) if mp_state is not None else False for i in range(n)]
    obs = [bool(mp_state[i] & 2) if mp_state is not None else False for i in range(n)]
    q_idx, q_dist, kp_final = [-1] * len(q), [-1] * len(q), [-1] * n
    hist = [[] for _ in range(30)]
    nm = 0
    use_ori = check_ori and variant in ("lastframe", "keyframe")
    for iq in range(len(q)):
        Q = q[iq]
        if not (Q["flags"] & 1):
            continue
        cand = _area(keys, g, Q["u"], Q["v"], Q["radius"], int(Q["min_level"]), int(Q["max_level"]))
        if not cand:
            continue
        if variant == "localmap":                      # ORBmatcher.cc:45-129
            bd, bl, bd2, bl2, bi = 256, -1, 256, -1, -1
            for idx in cand:
                if has[idx] and obs[idx]:
                    continue
                if uright is not None and uright[idx] > 0 and abs(f32(Q["ur"] - uright[idx])) > Q["ur_tol"]:
                    continue
                d = hamming(qdesc[iq], desc[idx])
                if d < bd:
                    bd2, bd, bl2, bl, bi = bd, d, bl, int(keys["octave"][idx]), idx
                elif d < bd2:
                    bl2, bd2 = int(keys["octave"][idx]), d
            if bd <= th_dist:
                if bl == bl2 and f32(bd) > f32(f32(nnratio) * f32(bd2)):
                    continue
                has[bi], obs[bi] = True, bool(Q["flags"] & 2)
                kp_final[bi], q_idx[iq], q_dist[iq] = iq, bi, bd
                nm += 1
            continue
        bd, bi = (2 ** 31 - 1 if variant == "fuse_sim3" else 256), -1
        for idx in cand:
            if variant == "lastframe":                 # :1403-1413
                if has[idx] and obs[idx]:
                    continue
                if uright is not None and uright[idx] > 0 and abs(f32(Q["ur"] - uright[idx])) > Q["ur_tol"]:
                    continue
            elif variant in ("keyframe", "sim3"):      # :1546-1548, :371-372
                if has[idx]:
                    continue
            elif variant == "fuse":                    # :903-932
                lvl = int(keys["octave"][idx])
                ex = f32(Q["u"] - keys["x"][idx])
                ey = f32(Q["v"] - keys["y"][idx])
                if uright is not None and uright[idx] >= 0:
                    er = f32(Q["ur"] - uright[idx])
                    e2 = f32(f32(f32(ex * ex) + f32(ey * ey)) + f32(er * er))
                    if float(f32(e2 * inv_sigma2[lvl])) > 7.8:
                        continue
                else:
                    e2 = f32(f32(ex * ex) + f32(ey * ey))
                    if float(f32(e2 * inv_sigma2[lvl])) > 5.99:
                        continue
            d = hamming(qdesc[iq], desc[idx])
            if d < bd:
                bd, bi = d, idx
        if bd <= th_dist:
            q_idx[iq], q_dist[iq] = bi, bd
            nm += 1
            if variant in ("fuse", "fuse_sim3"):
                continue
            has[bi], obs[bi] = True, bool(Q["flags"] & 2)
            kp_final[bi] = iq
            if use_ori:
                rot = f32(Q["angle"] - keys["angle"][bi])
                if rot < 0:
                    rot = f32(rot + f32(360))
                b = round_half_away(f32(rot * f32(f32(1) / f32(30))))
                hist[0 if b == 30 else b].append(iq)
    if use_ori:
        sizes = [len(h) for h in hist]
        m1 = m2 = m3 = 0
        i1 = i2 = i3 = -1
        for i, s in enumerate(sizes):
            if s > m1:
                m3, m2, m1, i3, i2, i1 = m2, m1, s, i2, i1, i
            elif s > m2:
                m3, m2, i3, i2 = m2, s, i2, i
            elif s > m3:
                m3, i3 = s, i
        if m2 < f32(0.1) * f32(m1):
            i2 = i3 = -1
        elif m3 < f32(0.1) * f32(m1):
            i3 = -1
        for i in range(30):
            if i in (i1, i2, i3):
                continue
            for iq in hist[i]:
                kp_final[q_idx[iq]] = -2
                q_idx[iq] = -1
                nm -= 1
    return nm, np.array(q_idx, np.int32), np.array(q_dist, np.int32), np.array(kp_final, np.int32)


# ---- SearchByBoW x2 / SearchForTriangulation (ORBmatcher.cc:160-289, 524-825) ----
def search_by_bow(variant, A, B, nnratio=0.6, check_ori=True, tri=None, nlevels=8):
    na, nb = len(A["keys"]), len(B["keys"])
    ma, mb = [-1] * na, [-1] * nb
    hist = [[] for _ in range(30)]
    nm = 0
    idsB = {int(x): j for j, x in enumerate(B["ids"])}
    if tri is not None:
        F = [f32(x) for x in tri[:9]]
        ex, ey = f32(tri[9]), f32(tri[10])
        scale2, sigma2 = tri[11:11 + nlevels], tri[11 + nlevels:11 + 2 * nlevels]

    def epi_ok(k1, k2):
        x1, y1 = f32(k1["x"]), f32(k1["y"])
        a = f32(f32(f32(x1 * F[0]) + f32(y1 * F[3])) + F[6])
        b = f32(f32(f32(x1 * F[1]) + f32(y1 * F[4])) + F[7])
        c = f32(f32(f32(x1 * F[2]) + f32(y1 * F[5])) + F[8])
        num = f32(f32(f32(a * f32(k2["x"])) + f32(b * f32(k2["y"]))) + c)
        den = f32(f32(a * a) + f32(b * b))
        if den == 0:
            return False
        dsqr = f32(f32(num * num) / den)
        return float(dsqr) < 3.84 * float(f32(sigma2[k2["octave"]]))

    for i, nid in enumerate(A["ids"]):
        j = idsB.get(int(nid))
        if j is None:
            continue
        for p in range(A["off"][i], A["off"][i + 1]):
            i1 = int(A["feat"][p])
            if not (A["flags"][i1] & 1):
                continue
            if variant == "triangulation":
                st1 = bool(A["flags"][i1] & 2)
                bd, bi = 50, -1
                for q in range(B["off"][j], B["off"][j + 1]):
                    i2 = int(B["feat"][q])
                    if not (B["flags"][i2] & 1):
                        continue
                    st2 = bool(B["flags"][i2] & 2)
                    d = hamming(A["desc"][i1], B["desc"][i2])
                    if d > 50 or d > bd:
                        continue
                    k2 = B["keys"][i2]
                    if not st1 and not st2:
                        dx, dy = f32(ex - f32(k2["x"])), f32(ey - f32(k2["y"]))
                        if f32(f32(dx * dx) + f32(dy * dy)) < f32(f32(100) * f32(scale2[k2["octave"]])):
                            continue
                    if epi_ok(A["keys"][i1], k2):
                        bi, bd = i2, d
                if bi >= 0:
                    ma[i1] = bi
                    nm += 1
                    if check_ori:
                        rot = f32(f32(A["keys"]["angle"][i1]) - f32(B["keys"]["angle"][bi]))
                        if rot < 0:
                            rot = f32(rot + f32(360))
                        b_ = round_half_away(f32(rot * f32(f32(1) / f32(30))))
                        hist[0 if b_ == 30 else b_].append(i1)
                continue
            bd1, bi, bd2 = 256, -1, 256
            for q in range(B["off"][j], B["off"][j + 1]):
                i2 = int(B["feat"][q])
                if variant == "kf_frame":
                    if mb[i2] >= 0:
                        continue
                elif mb[i2] >= 0 or not (B["flags"][i2] & 1):
                    continue
                d = hamming(A["desc"][i1], B["desc"][i2])
                if d < bd1:
                    bd2, bd1, bi = bd1, d, i2
                elif d < bd2:
                    bd2 = d
            ok = bd1 <= 50 if variant == "kf_frame" else bd1 < 50
            if ok and f32(bd1) < f32(f32(nnratio) * f32(bd2)):
                ma[i1], mb[bi] = bi, i1
                nm += 1
                if check_ori:
                    rot = f32(f32(A["keys"]["angle"][i1]) - f32(B["keys"]["angle"][bi]))
                    if rot < 0:
                        rot = f32(rot + f32(360))
                    b_ = round_half_away(f32(rot * f32(f32(1) / f32(30))))
                    hist[0 if b_ == 30 else b_].append(i1)
    if check_ori:
        sizes = [len(h) for h in hist]
        m1 = m2 = m3 = 0
        i1_ = i2_ = i3_ = -1
        for i, s in enumerate(sizes):
            if s > m1:
                m3, m2, m1, i3_, i2_, i1_ = m2, m1, s, i2_, i1_, i
            elif s > m2:
                m3, m2, i3_, i2_ = m2, s, i2_, i
            elif s > m3:
                m3, i3_ = s, i
        if m2 < f32(0.1) * f32(m1):
            i2_ = i3_ = -1
        elif m3 < f32(0.1) * f32(m1):
            i3_ = -1
        for i in range(30):
            if i in (i1_, i2_, i3_):
                continue
            for a in hist[i]:
                if ma[a] >= 0 and variant != "triangulation":
                    mb[ma[a]] = -1
                ma[a] = -1
                nm -= 1
    return nm, np.array(ma, np.int32), np.array(mb, np.int32)


def vocab_transform(voc, features, levelsup=4):
    """TemplatedVocabulary::transform (TemplatedVocabulary.h:1140-1272) with
    the loaders' tree (children in file order, word ids in leaf-flag order),
    restated independently for the oracle's KAT: (bow dict, fv dict)."""
    n_nodes = len(voc["parent"])
    children = [[] for _ in range(n_nodes)]
    word_id = [0] * n_nodes
    nw = 0
    for i in range(1, n_nodes):
        children[int(voc["parent"][i])].append(i)
        if voc["is_leaf"][i]:
            word_id[i] = nw
            nw += 1
    if nw == 0:
        return {}, {}
    scoring, weighting = int(voc["scoring"]), int(voc["weighting"])
    must = scoring != 5
    nid_level = int(voc["L"]) - levelsup
    bow, fv = {}, {}
    for f, fd in enumerate(np.asarray(features, np.uint8).reshape(-1, 32)):
        nid = 0 if nid_level <= 0 else None
        node, level = 0, 0
        while children[node]:
            level += 1
            kids = children[node]
            best, best_d = kids[0], hamming(fd, voc["desc"][kids[0]])
            for c in kids[1:]:
                d = hamming(fd, voc["desc"][c])
                if d < best_d:
                    best, best_d = c, d
            node = best
            if level == nid_level:
                nid = node
        if nid is None:
            nid = node
        w = float(voc["weight"][node])
        if w > 0:
            wid = word_id[node]
            if weighting in (0, 1):
                bow[wid] = bow[wid] + w if wid in bow else w
            elif wid not in bow:
                bow[wid] = w
            fv.setdefault(nid, []).append(f)
    bow = dict(sorted(bow.items()))
    if weighting in (0, 1) and bow and not must:
        nd = float(len(bow))
        bow = {k: v / nd for k, v in bow.items()}
    if must:
        if scoring == 1:
            norm = math.sqrt(sum(v * v for v in bow.values()))
        else:
            norm = 0.0
            for v in bow.values():
                norm += abs(v)
        if norm > 0:
            bow = {k: v / norm for k, v in bow.items()}
    return bow, dict(sorted(fv.items()))


def distinctive_descriptors(desc, offsets):
    """MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:288-361) per point."""
    out = []
    for p in range(len(offsets) - 1):
        rows = desc[offsets[p]:offsets[p + 1]]
        N = len(rows)
        if N == 0:
            out.append(-1)
            continue
        D = [[0] * N for _ in range(N)]
        for i in range(N):
            for j in range(i + 1, N):
                D[i][j] = D[j][i] = hamming(rows[i], rows[j])
        best_med, best_idx = 2 ** 31 - 1, 0
        for i in range(N):
            med = sorted(D[i])[int(0.5 * (N - 1))]
            if med < best_med:
                best_med, best_idx = med, i
        out.append(best_idx)
    return np.array(out, np.int32)


def undistort_points(xy, K, dist):
    """cv::undistortPoints(K, D, R=I, P=K) in Python doubles, OpenCV 3.2 order."""
    K = [float(v) for v in np.asarray(K, np.float32).reshape(9)]
    d = [float(v) for v in np.asarray(dist, np.float32).reshape(-1)]
    if d[0] == 0.0:
        return np.asarray(xy, np.float32).copy()
    k = (d + [0.0] * 8)[:8]
    fx, fy, cx, cy = K[0], K[4], K[2], K[5]
    ifx, ify = 1.0 / fx, 1.0 / fy
    out = np.empty((len(xy), 2), np.float32)
    for i, (u, v) in enumerate(np.asarray(xy, np.float32)):
        x = x0 = (float(u) - cx) * ifx
        y = y0 = (float(v) - cy) * ify
        for _ in range(5):
            r2 = x * x + y * y
            icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2)
            dx = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x)
            dy = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y
            x = (x0 - dx) * icdist
            y = (y0 - dy) * icdist
        xx = K[0] * x + K[1] * y + K[2]
        yy = K[3] * x + K[4] * y + K[5]
        ww = 1.0 / (K[6] * x + K[7] * y + K[8])
        out[i] = (np.float32(xx * ww), np.float32(yy * ww))
    return out


def l1_score(w1, v1, w2, v2):
    """L1Scoring::score (ScoringObject.cpp:23-66)."""
    d2 = dict(zip((int(x) for x in w2), (float(x) for x in v2)))
    s = 0.0
    for w, vi in zip(w1, v1):
        wi = d2.get(int(w))
        if wi is not None:
            vi = float(vi)
            s += abs(vi - wi) - abs(vi) - abs(wi)
    return -s / 2.0


class KeyFrameDB:
    """KeyFrameDatabase (KeyFrameDatabase.cc:31-330) restated literally in
    Python: inverted lists in add order, per-keyframe query state."""

    def __init__(self):
        self.inv = {}
        self.bow = {}
        self.st = {}

    def add(self, k, words, values):
        self.bow[k] = (np.asarray(words), np.asarray(values))
        self.st.setdefault(k, dict(lq=0, lw=0, ls=np.float32(0), rq=0, rw=0, rs=np.float32(0)))
        for w in words:
            self.inv.setdefault(int(w), []).append(k)

    def erase(self, k):
        for w in self.bow.get(k, ([], []))[0]:
            lst = self.inv.get(int(w), [])
            if k in lst:
                lst.remove(k)

    def detect(self, reloc, qid, words, values, connected, min_score, covis):
        conn = set(connected or [])
        sharing = []
        q, wk, sk = ("rq", "rw", "rs") if reloc else ("lq", "lw", "ls")
        for w in words:
            for k in self.inv.get(int(w), []):
                s = self.st[k]
                if s[q] != qid:
                    s[wk] = 0
                    if reloc or k not in conn:
                        s[q] = qid
                        sharing.append(k)
                s[wk] += 1
        if not sharing:
            return []
        max_common = max(self.st[k][wk] for k in sharing)
        min_common = int(np.float32(max_common) * np.float32(0.8))
        scored = []
        for k in sharing:
            if self.st[k][wk] > min_common:
                si = np.float32(l1_score(words, values, *self.bow[k]))
                self.st[k][sk] = si
                if reloc or si >= np.float32(min_score):
                    scored.append((si, k))
        if not scored:
            return []
        acc = []
        best_acc = np.float32(0) if reloc else np.float32(min_score)
        for si, k in scored:
            best_s, acc_s, best_k = si, si, k
            for k2 in list(covis(k))[:10]:
                s2 = self.st.get(k2)
                if s2 is None:
                    continue
                if reloc:
                    if s2[q] != qid:
                        continue
                elif not (s2[q] == qid and s2[wk] > min_common):
                    continue
                acc_s = np.float32(acc_s + s2[sk])
                if s2[sk] > best_s:
                    best_k, best_s = k2, s2[sk]
            acc.append((acc_s, best_k))
            if acc_s > best_acc:
                best_acc = acc_s
        keep = np.float32(np.float32(0.75) * best_acc)
        out, seen = [], set()
        for a, k in acc:
            if a > keep and k not in seen:
                out.append(k)
                seen.add(k)
        return out
