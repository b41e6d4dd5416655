"""GPU parity of the vocabulary-node matchers (SURVEY.md §8 a16 SearchByBoW x2,
a17 SearchForTriangulation) against the CPU oracle: identical pairs in both
directions and identical nmatches, with and without the rotation check."""
import numpy as np
import pytest

from orb_slam_2_ros_amd import ORBmatcher

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("variant", ["kf_frame", "kf_kf", "triangulation"])
@pytest.mark.parametrize("seed,na,nb,nodes,ori", [(111, 1000, 1100, 120, True), (112, 2500, 2400, 40, False),
                                                 (113, 3000, 3000, 15, True)])
def test_bow_matchers_bit_exact(variant, seed, na, nb, nodes, ori, oracle_mod):
    from orb_slam_2_ros_amd.synth_match import BOW_VARIANT_ARGS as VARIANT_ARGS, make_bow_case as make_case
    A, B, tri = make_case(seed, variant, na=na, nb=nb, nodes=nodes)
    ratio, _ = VARIANT_ARGS[variant]
    g = ORBmatcher(ratio, ori).search_by_bow(variant, A, B, tri)
    o = oracle_mod.search_by_bow(variant, A, B, ratio, ori, tri)
    assert g[0] == o[0] and o[0] > 0
    for name, x, y in zip(("match_a", "match_b"), g[1:], o[1:]):
        bad = np.nonzero(x != y)[0]
        assert len(bad) == 0, f"{name} differs at {bad[:5]}: {x[bad[:5]]} vs {y[bad[:5]]}"


def test_bow_disjoint_and_empty(oracle_mod):
    from orb_slam_2_ros_amd.synth_match import make_bow_case as make_case
    A, B, _ = make_case(114, "kf_frame", na=300, nb=300, nodes=30)
    B2 = dict(B, ids=(B["ids"] + np.uint32(2_000_000)).astype(np.uint32))   # no common node
    nm, ma, mb = ORBmatcher(0.75, True).search_by_bow("kf_frame", A, B2)
    assert nm == 0 and (ma == -1).all() and (mb == -1).all()
    E = dict(A, ids=A["ids"][:0], off=A["off"][:1], feat=A["feat"][:0])
    nm, ma, mb = ORBmatcher(0.75, True).search_by_bow("kf_frame", E, B)
    assert nm == 0


@pytest.mark.parametrize("variant", ["kf_frame", "kf_kf", "triangulation"])
@pytest.mark.parametrize("nb_node,na_node,seed", [(6, 40, 121), (24, 90, 122), (64, 150, 123), (100, 160, 124),
                                                  (300, 64, 125)])
def test_bow_tiny_pool_contention(variant, nb_node, na_node, seed, oracle_mod):
    """Many A features of a node competing for a few B features: nodes of <= 64
    B features run the lanes-take-A path, whose in-order repair pass must fire
    (counted by the kernel, orbx_debug_counter "bow_repairs"); larger nodes run
    the sequential path.  Both bit-exact against the oracle's in-order loop."""
    from orb_slam_2_ros_amd._lib import debug_counter
    from orb_slam_2_ros_amd.synth_match import BOW_VARIANT_ARGS, make_bow_contention_case
    A, B, tri = make_bow_contention_case(seed, variant, nb_node, na_node)
    ratio, _ = BOW_VARIANT_ARGS[variant]
    for ori in (True, False):
        g = ORBmatcher(ratio, ori).search_by_bow(variant, A, B, tri)
        repairs = debug_counter("bow_repairs")
        o = oracle_mod.search_by_bow(variant, A, B, ratio, ori, tri)
        assert g[0] == o[0] and o[0] > 0
        for name, x, y in zip(("match_a", "match_b"), g[1:], o[1:]):
            bad = np.nonzero(x != y)[0]
            assert len(bad) == 0, f"{name} differs at {bad[:5]}: {x[bad[:5]]} vs {y[bad[:5]]}"
        if variant != "triangulation" and nb_node <= 64:
            assert repairs > 0, "the repair pass never ran"
        else:
            assert repairs == 0
