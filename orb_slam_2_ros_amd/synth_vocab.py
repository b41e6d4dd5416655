"""Synthetic DBoW2 vocabularies (the reference's ORBvoc.txt is not in the
repository: `.MISSING_LARGE_BLOBS`) and writers for the two
file formats TemplatedVocabulary loads (text :1351-1425, binary :1473-1547).

A tree is built breadth first (siblings in consecutive ids, parents before
children, as DBoW2's HKmeansStep creates them).  A child's descriptor is its
parent's with `flip` random bits flipped, so descriptors drawn near a leaf
descend to it most of the time and ties / near ties also occur.
"""
from __future__ import annotations

import struct

import numpy as np


def make_vocab(k=10, L=4, seed=0, flip=24, stop_frac=0.02, irregular=False, scoring=0, weighting=0):
    """Returns a dict (k, L, scoring, weighting, parent i32, is_leaf u8,
    desc (n, 32) u8, weight f64) with node 0 the root.  irregular: child
    counts 1..k and early leaves (not every path reaches depth L)."""
    rng = np.random.default_rng(seed)
    if not irregular:
        return _make_regular(k, L, rng, flip, stop_frac, scoring, weighting)
    parent, leaf, depth = [0], [0], [0]
    desc = [np.zeros(32, np.uint8)]
    frontier = [0]
    for lvl in range(1, L + 1):
        nxt = []
        for p in frontier:
            nk = int(rng.integers(1, k + 1)) if irregular else k
            for _ in range(nk):
                if lvl == 1:
                    d = rng.integers(0, 256, 32).astype(np.uint8)
                else:
                    d = desc[p].copy()
                    bits = rng.choice(256, flip, replace=False)
                    for b in bits:
                        d[b >> 3] ^= np.uint8(1 << (b & 7))
                nid = len(parent)
                parent.append(p)
                desc.append(d)
                depth.append(lvl)
                early = irregular and lvl < L and rng.random() < 0.15
                leaf.append(1 if (lvl == L or early) else 0)
                if not leaf[-1]:
                    nxt.append(nid)
        frontier = nxt
    n = len(parent)
    leaf = np.array(leaf, np.uint8)
    weight = np.zeros(n, np.float64)
    nl = int(leaf.sum())
    w = rng.uniform(0.3, 9.0, nl)
    w[rng.random(nl) < stop_frac] = 0.0          # stopped words (transform skips them)
    weight[leaf == 1] = w
    return {"k": k, "L": L, "scoring": scoring, "weighting": weighting,
            "parent": np.array(parent, np.int32), "is_leaf": leaf,
            "desc": np.stack(desc).astype(np.uint8), "weight": weight}


def _make_regular(k, L, rng, flip, stop_frac, scoring, weighting):
    """Full k-ary tree of depth L, level by level (vectorised; ORBvoc's
    k=10, L=6 has 1,111,111 nodes).  Bit flips are Bernoulli(flip/256)."""
    parents = [np.zeros(1, np.int32)]
    descs = [np.zeros((1, 32), np.uint8)]
    first = 1
    prev = np.zeros(1, np.int64)          # node ids of the previous level
    prev_desc = descs[0]
    for lvl in range(1, L + 1):
        par = np.repeat(prev, k)
        if lvl == 1:
            d = rng.integers(0, 256, (len(par), 32)).astype(np.uint8)
        else:
            bits = rng.random((len(par), 256)) < flip / 256.0
            mask = np.packbits(bits, axis=1, bitorder="little")
            d = np.repeat(prev_desc, k, axis=0) ^ mask
        ids = np.arange(first, first + len(par))
        first += len(par)
        parents.append(par.astype(np.int32))
        descs.append(d)
        prev, prev_desc = ids, d
    parent = np.concatenate(parents)
    desc = np.concatenate(descs)
    n = len(parent)
    leaf = np.zeros(n, np.uint8)
    leaf[n - k ** L:] = 1
    weight = np.zeros(n, np.float64)
    w = rng.uniform(0.3, 9.0, k ** L)
    w[rng.random(k ** L) < stop_frac] = 0.0
    weight[leaf == 1] = w
    return {"k": k, "L": L, "scoring": scoring, "weighting": weighting, "parent": parent, "is_leaf": leaf,
            "desc": desc, "weight": weight}


def features_near_leaves(voc, n, seed=1, noise=12, random_frac=0.1):
    """Descriptors drawn around random leaves, each with Bernoulli bit flips
    (about noise/2 bits on average), plus some uniform noise rows."""
    rng = np.random.default_rng(seed)
    leaves = np.nonzero(voc["is_leaf"])[0]
    out = voc["desc"][rng.choice(leaves, n)].copy()
    p = rng.uniform(0, noise / 256.0, (n, 1))
    out ^= np.packbits(rng.random((n, 256)) < p, axis=1, bitorder="little")
    rnd = rng.random(n) < random_frac
    out[rnd] = rng.integers(0, 256, (int(rnd.sum()), 32)).astype(np.uint8)
    return out


def write_text(voc, path):
    """ORBvoc.txt layout: "k L scoring weighting", then per node 1..n-1
    "parent isLeaf d0 .. d31 weight" (weights printed to round-trip)."""
    with open(path, "w") as f:
        f.write(f"{voc['k']} {voc['L']}  {voc['scoring']} {voc['weighting']}\n")
        for i in range(1, len(voc["parent"])):
            d = " ".join(str(int(x)) for x in voc["desc"][i])
            f.write(f"{int(voc['parent'][i])} {int(voc['is_leaf'][i])} {d} {float(voc['weight'][i])!r}\n")


def write_binary(voc, path):
    """loadFromBinFile layout: 4 x int32 header, then per node int32 parent,
    u8 isLeaf, 32 B descriptor, f64 weight."""
    with open(path, "wb") as f:
        f.write(struct.pack("<4i", voc["k"], voc["L"], voc["scoring"], voc["weighting"]))
        for i in range(1, len(voc["parent"])):
            f.write(struct.pack("<iB", int(voc["parent"][i]), int(voc["is_leaf"][i])))
            f.write(voc["desc"][i].tobytes())
            f.write(struct.pack("<d", float(voc["weight"][i])))


def make_keyframe_bows(n_kf=300, n_words=100000, words_per_kf=500, seed=0, loop_every=60):
    """Synthetic keyframe BowVectors along a trajectory with revisits: a
    keyframe keeps ~70% of the previous one's words; every `loop_every`
    keyframes the trajectory returns near an earlier place (a loop).  Values
    are positive and L1-normalised (TF-IDF with L1 scoring).  Returns a list of
    (words u32 ascending, values f64) and the covisibility order (each
    keyframe's up-to-10 neighbours, nearest first)."""
    rng = np.random.default_rng(seed)
    bows = []
    cur = np.sort(rng.choice(n_words, words_per_kf, replace=False))
    for i in range(n_kf):
        if i and i % loop_every == 0 and i > 2 * loop_every // 3:
            j = int(rng.integers(0, i - loop_every // 2))
            cur = bows[j][0].copy()                                # back at keyframe j's place
        keep = cur[rng.random(len(cur)) < 0.7]
        new = rng.choice(n_words, words_per_kf - len(keep), replace=False)
        cur = np.unique(np.concatenate([keep, new]).astype(np.uint32))
        vals = rng.uniform(0.1, 5.0, len(cur))
        vals /= np.abs(vals).sum()
        bows.append((cur.astype(np.uint32), vals))
    covis = {i: [j for j in sorted(range(max(0, i - 5), min(n_kf, i + 6)), key=lambda j: (abs(j - i), j))
                 if j != i][:10] for i in range(n_kf)}
    return bows, covis
