"""A small map for LocalMapping::SearchInNeighbors' first fusion loop
(LocalMapping.cc:537-548: Fuse(pKFi, vpMapPointMatches) for every target
keyframe), with the map edits Fuse makes (ORBmatcher.cc:827-977) and
MapPoint::Replace (MapPoint.cc:198-256), which recomputes the survivor's
descriptor (ComputeDistinctiveDescriptors, MapPoint.cc:288-361).

A later neighbour's search reads that new descriptor, so the batched recipe
(one orbx_search_by_projection_batch over all neighbours with the starting
descriptors) must re-run a one-row search for a point whose descriptor changed
before its turn (include/orbx.h).  `run` plays a schedule:
  search(j, i, desc) -> (q_idx, q_dist) of point i against neighbour j;
  recipe="sequential": every search with the current descriptor (the reference);
  recipe="batched": the batch's result unless the descriptor changed since
                    the batch, then a one-row search (the documented recipe);
  recipe="naive": always the batch's result (the round-2 contract; wrong).
"""
import numpy as np

from orb_slam_2_ros_amd.synth_match import KEYPOINT_DTYPE, PROJ_QUERY_DTYPE, scale_tables

TH_LOW = 50


def _flip(rng, d, k):
    d = d.copy()
    for b in rng.choice(256, k, replace=False):
        d[b >> 3] ^= np.uint8(1 << (b & 7))
    return d


def make_world(seed, n_true=600, n_cur=420, n_neigh=8, w=640, h=480, kp_flips=(2, 12), row_flips=(1, 6)):
    """kp_flips / row_flips: bit-flip ranges of keypoint and observation rows
    against the true point's descriptor (wider ranges put distances near TH_LOW)."""
    rng = np.random.default_rng(seed)
    sf, _ = scale_tables(1.2, 8)
    inv_sigma2 = (np.float32(1) / (sf * sf)).astype(np.float32)
    base = rng.integers(0, 256, (n_true, 32)).astype(np.uint8)
    rows = {}                     # (kf, idx) -> descriptor row
    obs = {}                      # point id -> {kf: idx}
    mp = {}                       # kf -> array of point ids (-1 none)
    # the current keyframe (kf 0) sees points 0..n_cur-1 (true points 0..n_cur-1)
    mp[0] = np.arange(n_cur)
    for i in range(n_cur):
        rows[(0, i)] = _flip(rng, base[i], int(rng.integers(*row_flips)))
        obs[i] = {0: i}
        for e in range(int(rng.integers(0, 4))):   # other observers (kf 1000 + ...)
            kf = 1000 + int(rng.integers(0, 40))
            if kf in obs[i]:
                continue
            idx = 10000 + i
            rows[(kf, idx)] = _flip(rng, base[i], int(rng.integers(*row_flips)))
            obs[i][kf] = idx
    frames = []
    for j in range(1, n_neigh + 1):
        vis = np.nonzero(rng.random(n_true) < 0.6)[0]
        n_clutter = 120
        n = len(vis) + n_clutter
        keys = np.zeros(n, KEYPOINT_DTYPE)
        keys["x"] = rng.uniform(20, w - 20, n).astype(np.float32)
        keys["y"] = rng.uniform(20, h - 20, n).astype(np.float32)
        keys["octave"] = rng.choice(8, n, p=[0.3, 0.2, 0.15, 0.12, 0.09, 0.07, 0.04, 0.03])
        keys["size"] = 31
        keys["angle"] = rng.uniform(0, 360, n).astype(np.float32)
        keys["class_id"] = -1
        desc = rng.integers(0, 256, (n, 32)).astype(np.uint8)
        tkp = {}
        for k, t in enumerate(vis):
            desc[k] = _flip(rng, base[t], int(rng.integers(*kp_flips)))
            tkp[int(t)] = k
        m = np.full(n, -1, np.int64)
        for k, t in enumerate(vis):
            if rng.random() < 0.55:          # a duplicate of true point t already mapped here
                pid = n_cur + int(t)
                m[k] = pid
                obs.setdefault(pid, {})[j] = k
        for k in range(n):
            rows[(j, k)] = desc[k]
        mp[j] = m
        frames.append(dict(keys=keys, desc=desc, tkp=tkp))
    # duplicates: a few more observers so either side of Replace can win
    for pid in range(n_cur, n_cur + n_true):
        if pid not in obs:
            continue
        t = pid - n_cur
        for e in range(int(rng.integers(0, 3))):
            kf = 2000 + int(rng.integers(0, 40))
            if kf in obs[pid]:
                continue
            rows[(kf, 20000 + t)] = _flip(rng, base[t], int(rng.integers(*row_flips)))
            obs[pid][kf] = 20000 + t
    # query rows of point i against neighbour j (the caller's projection)
    queries = []
    for j, F in enumerate(frames, start=1):
        q = np.zeros(n_cur, PROJ_QUERY_DTYPE)
        for i in range(n_cur):
            k = F["tkp"].get(i)
            if k is not None:
                lvl = int(F["keys"]["octave"][k])
                q[i]["u"] = F["keys"]["x"][k] + np.float32(rng.normal(0, 0.6))
                q[i]["v"] = F["keys"]["y"][k] + np.float32(rng.normal(0, 0.6))
            else:
                lvl = int(rng.integers(0, 8))
                q[i]["u"] = rng.uniform(0, w)
                q[i]["v"] = rng.uniform(0, h)
            q[i]["radius"] = np.float32(3.0) * sf[lvl]
            q[i]["min_level"], q[i]["max_level"] = lvl - 1, lvl
            q[i]["ur"] = -1.0
            q[i]["flags"] = 1
        queries.append(q)
    return dict(n_cur=n_cur, frames=frames, queries=queries, rows=rows, obs=obs, mp=mp,
                bounds=(0.0, float(w), 0.0, float(h)), inv_sigma2=inv_sigma2)


def distinctive(rows_of, oracle_mod):
    """MapPoint::ComputeDistinctiveDescriptors over the rows in observation order."""
    if not rows_of:
        return None
    d = np.stack(rows_of)
    best = oracle_mod.distinctive_descriptors(d, np.array([0, len(d)], np.int32))[0]
    return d[best].copy() if best >= 0 else None


def run(world, recipe, search, batch=None, oracle_mod=None):
    """Plays the first SearchInNeighbors loop; returns the final map state and
    the number of one-row re-searches the batched recipe made."""
    obs = {p: dict(o) for p, o in world["obs"].items()}
    mp = {k: v.copy() for k, v in world["mp"].items()}
    rows = world["rows"]
    bad = set()
    D = {p: distinctive([rows[(kf, obs[p][kf])] for kf in sorted(obs[p])], oracle_mod) for p in obs}
    D0 = {p: (None if d is None else d.copy()) for p, d in D.items()}
    research = 0

    def replace(x, y):                       # x->Replace(y), MapPoint.cc:198-256
        if x == y:
            return
        ox = obs.pop(x)
        obs[x] = {}
        bad.add(x)
        for kf, idx in ox.items():
            if kf not in obs[y]:
                if kf in mp:
                    mp[kf][idx] = y
                obs[y][kf] = idx
            elif kf in mp:
                mp[kf][idx] = -1
        D[y] = distinctive([rows[(kf, obs[y][kf])] for kf in sorted(obs[y])], oracle_mod)

    for j in range(1, len(world["frames"]) + 1):
        for i in range(world["n_cur"]):
            p = i
            if p in bad or j in obs[p]:
                continue
            if recipe == "sequential":
                qi, qd = search(j, i, D[p])
            elif recipe == "batched" and not np.array_equal(D[p], D0[p]):
                qi, qd = search(j, i, D[p])
                research += 1
            else:
                qi, qd = int(batch[j - 1][1][i]), int(batch[j - 1][2][i])
            if qi < 0 or qd > TH_LOW:
                continue
            other = int(mp[j][qi])
            if other >= 0:
                if other not in bad:
                    if len(obs[other]) > len(obs[p]):
                        replace(p, other)
                    else:
                        replace(other, p)
            else:
                obs[p][j] = qi
                mp[j][qi] = p
    state = dict(bad=sorted(bad), mp={k: v.tolist() for k, v in mp.items()},
                 obs={p: sorted(o.items()) for p, o in obs.items()},
                 D={p: (None if d is None else bytes(d)) for p, d in D.items()})
    return state, research


def problems(world, descs=None):
    """One Fuse problem per neighbour, every point's row with its starting descriptor."""
    out = []
    for j, F in enumerate(world["frames"], start=1):
        qd = np.stack([descs[i] for i in range(world["n_cur"])])
        out.append(dict(keys=F["keys"], desc=F["desc"], queries=world["queries"][j - 1], qdesc=qd,
                        bounds=world["bounds"], uright=None, mp_state=None, inv_sigma2=world["inv_sigma2"]))
    return out
