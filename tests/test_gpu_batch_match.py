"""GPU parity of the batched matcher entry points (VERDICT r1 "next" #7): one
launch pair for the reference's per-keyframe loops --
  Fuse over a keyframe's neighbours (LocalMapping.cc:537-548),
  relocalisation's SearchByProjection over candidates (Tracking.cc:1667),
  SearchForTriangulation over covisible neighbours (LocalMapping.cc:276-315).
Every problem of a batch must equal the oracle's single call on the same
inputs, including problems that share a frame (uploaded once) and trivial
problems (no keypoints / no queries) inside a batch."""
import numpy as np
import pytest

from orb_slam_2_ros_amd import ORBmatcher

pytestmark = pytest.mark.gpu


def _proj_oracle(oracle_mod, variant, c, th, ratio, ori):
    return oracle_mod.search_by_projection(variant, c["keys"], c["desc"], c["queries"], c["qdesc"], c["bounds"],
                                           c["uright"], c["mp_state"], c["inv_sigma2"], th, ratio, ori)


def _same(g, o, names):
    assert g[0] == o[0], f"nmatches {g[0]} vs {o[0]}"
    for name, x, y in zip(names, g[1:], o[1:]):
        bad = np.nonzero(x != y)[0]
        assert len(bad) == 0, f"{name} differs at {bad[:5]}: {x[bad[:5]]} vs {y[bad[:5]]}"


@pytest.mark.parametrize("variant", ["fuse", "keyframe", "localmap", "fuse_sim3"])
def test_projection_batch_equals_single_calls(variant, oracle_mod):
    from orb_slam_2_ros_amd.synth_match import PROJ_VARIANT_ARGS as VARIANT_ARGS, make_proj_case as make_case
    th, ratio, ori, win = VARIANT_ARGS[variant]
    cases = [make_case(300 + k, variant, n=600 + 150 * k, nq=400 + 90 * k, stereo=k % 2 == 1, th=win)
             for k in range(6)]
    # a frame searched with two query sets (relocalisation: one current frame,
    # several candidates' points): the second problem shares its arrays
    shared = dict(cases[0])
    other = make_case(399, variant, n=600, nq=350, stereo=False, th=win)
    shared["queries"], shared["qdesc"] = other["queries"], other["qdesc"]
    cases.append(shared)
    g = ORBmatcher(ratio, ori).search_by_projection_batch(variant, cases, th)
    assert len(g) == len(cases)
    for k, c in enumerate(cases):
        _same(g[k], _proj_oracle(oracle_mod, variant, c, th, ratio, ori), ("q_idx", "q_dist", "kp_final"))
    assert sum(x[0] for x in g) > 0


def test_projection_batch_with_empty_problems(oracle_mod):
    from orb_slam_2_ros_amd.synth_match import PROJ_VARIANT_ARGS as VARIANT_ARGS, make_proj_case as make_case
    th, ratio, ori, win = VARIANT_ARGS["fuse"]
    a = make_case(311, "fuse", n=800, nq=500, th=win)
    b = make_case(312, "fuse", n=700, nq=400, th=win)
    no_q = dict(b, queries=b["queries"][:0], qdesc=b["qdesc"][:0])
    no_kp = dict(b, keys=b["keys"][:0], desc=b["desc"][:0], uright=None, mp_state=None)
    g = ORBmatcher(ratio, ori).search_by_projection_batch("fuse", [a, no_q, b, no_kp], th)
    _same(g[0], _proj_oracle(oracle_mod, "fuse", a, th, ratio, ori), ("q_idx", "q_dist", "kp_final"))
    _same(g[2], _proj_oracle(oracle_mod, "fuse", b, th, ratio, ori), ("q_idx", "q_dist", "kp_final"))
    assert g[1][0] == 0 and len(g[1][1]) == 0 and (g[1][3] == -1).all()
    assert g[3][0] == 0 and (g[3][1] == -1).all() and (g[3][2] == -1).all()


def _neighbours(B, count, seed):
    """count variants of side B over the same vocabulary nodes (each one a
    different covisible keyframe of the same A): sparse descriptor bit flips,
    jittered angles, fresh usability flags."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(count):
        d = B["desc"].copy()
        flip = rng.random(d.shape) < 0.03
        d[flip] ^= (1 << rng.integers(0, 8, flip.sum())).astype(np.uint8)
        k = B["keys"].copy()
        k["angle"] = ((k["angle"] + rng.normal(0, 4, len(k))) % 360).astype(np.float32)
        f = B["flags"].copy()
        f[rng.random(len(f)) < 0.15] ^= 1
        out.append(dict(B, desc=d, keys=k, flags=f))
    return out


@pytest.mark.parametrize("variant,ori", [("triangulation", False), ("triangulation", True), ("kf_kf", True),
                                         ("kf_frame", False)])
def test_bow_batch_equals_single_calls(variant, ori, oracle_mod):
    from orb_slam_2_ros_amd.synth_match import BOW_VARIANT_ARGS as VARIANT_ARGS, make_bow_case as make_case
    ratio, _ = VARIANT_ARGS[variant]
    A, B, tri = make_case(400, variant, na=1200, nb=1300, nodes=90)
    # one keyframe A against 8 neighbours (the same A object: uploaded once),
    # plus an unrelated pair in the same batch
    probs = [{"A": A, "B": Bk, "tri": tri} for Bk in _neighbours(B, 8, 401)]
    A2, B2, tri2 = make_case(402, variant, na=700, nb=800, nodes=50)
    probs.append({"A": A2, "B": B2, "tri": tri2})
    g = ORBmatcher(ratio, ori).search_by_bow_batch(variant, probs)
    for k, P in enumerate(probs):
        o = oracle_mod.search_by_bow(variant, P["A"], P["B"], ratio, ori, P["tri"])
        _same(g[k], o, ("match_a", "match_b"))
        assert o[0] > 0


def test_triangulation_batch_sequential_exclusion(oracle_mod):
    """LocalMapping's order dependency: neighbour i's search sees A features
    mapped by neighbours < i as unusable.  Batch once with the initial flags,
    then drop the excluded features and run the rotation pass
    (orbx_rotation_filter): equal to the oracle run with the updated flags."""
    from orb_slam_2_ros_amd.synth_match import BOW_VARIANT_ARGS as VARIANT_ARGS, make_bow_case as make_case
    ratio, _ = VARIANT_ARGS["triangulation"]
    A, B, tri = make_case(420, "triangulation", na=1500, nb=1500, nodes=80)
    probs = [{"A": A, "B": Bk, "tri": tri} for Bk in _neighbours(B, 5, 421)]
    raw = ORBmatcher(ratio, False).search_by_bow_batch("triangulation", probs)
    for ori in (False, True):
        flags = A["flags"].copy()
        for k, P in enumerate(probs):
            excl = (flags & 1) == 0
            mine = raw[k][1].copy()
            if ori:
                nm, mine = ORBmatcher.rotation_filter(A["keys"], P["B"]["keys"], mine, excl)
            else:
                mine[excl] = -1
                nm = int((mine >= 0).sum())
            o = oracle_mod.search_by_bow("triangulation", dict(A, flags=flags), P["B"], ratio, ori, P["tri"])
            assert nm == o[0] and o[0] > 0
            assert np.array_equal(mine, o[1])
            # this neighbour's new map points bar their A features from the next
            flags = flags.copy()
            flags[np.nonzero(mine >= 0)[0][::2]] &= 0xFE


def test_fuse_neighbours_batched_with_research(oracle_mod):
    """Fuse over the neighbours as ONE device batch with the
    starting descriptors, then the edits neighbour by neighbour, re-searching
    (one-row device call) every point whose descriptor a Replace changed
    before its turn -- the final map state equals the sequential reference
    (oracle, one query at a time with the current descriptor)."""
    from fuse_world import TH_LOW, distinctive, make_world, problems, run
    from orb_slam_2_ros_amd.synth_match import PROJ_VARIANT_ARGS as VARIANT_ARGS
    th, ratio, ori, _ = VARIANT_ARGS["fuse"]
    w = make_world(7, kp_flips=(20, 40), row_flips=(10, 25))

    def oracle_search(j, i, d):
        F = w["frames"][j - 1]
        _, qi, qd, _ = oracle_mod.search_by_projection("fuse", F["keys"], F["desc"], w["queries"][j - 1][i:i + 1],
                                                       d.reshape(1, 32), w["bounds"], None, None, w["inv_sigma2"],
                                                       TH_LOW, ratio, ori)
        return int(qi[0]), int(qd[0])
    m = ORBmatcher(ratio, ori)

    def gpu_search(j, i, d):
        F = w["frames"][j - 1]
        _, qi, qd, _ = m.search_by_projection("fuse", F["keys"], F["desc"], w["queries"][j - 1][i:i + 1],
                                              d.reshape(1, 32), w["bounds"], None, None, w["inv_sigma2"], TH_LOW)
        return int(qi[0]), int(qd[0])
    seq, _ = run(w, "sequential", oracle_search, oracle_mod=oracle_mod)
    starts = {i: distinctive([w["rows"][(kf, w["obs"][i][kf])] for kf in sorted(w["obs"][i])], oracle_mod)
              for i in range(w["n_cur"])}
    batch = m.search_by_projection_batch("fuse", problems(w, starts), TH_LOW)
    got, nre = run(w, "batched", gpu_search, batch, oracle_mod=oracle_mod)
    naive, _ = run(w, "naive", gpu_search, batch, oracle_mod=oracle_mod)
    assert nre > 0
    assert got == seq
    assert naive != seq
