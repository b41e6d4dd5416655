"""GPU parity of the projection matchers (SURVEY.md §8 a15 SearchByProjection
x4, a18 Fuse x2 search) against the CPU oracle on the same query tables:
nmatches, per-query assignment and distance, and the final keypoint
ownership must agree exactly."""
import numpy as np
import pytest

from orb_slam_2_ros_amd import ORBmatcher

pytestmark = pytest.mark.gpu

VARIANTS = ["localmap", "lastframe", "keyframe", "sim3", "fuse", "fuse_sim3"]


def _check(c, variant, oracle_mod, th=None):
    from orb_slam_2_ros_amd.synth_match import PROJ_VARIANT_ARGS as VARIANT_ARGS
    th_dist, ratio, ori, _ = VARIANT_ARGS[variant]
    if th is not None:
        th_dist = th
    g = ORBmatcher(ratio, ori).search_by_projection(variant, c["keys"], c["desc"], c["queries"], c["qdesc"],
                                                    c["bounds"], c["uright"], c["mp_state"], c["inv_sigma2"],
                                                    th_dist)
    o = oracle_mod.search_by_projection(variant, c["keys"], c["desc"], c["queries"], c["qdesc"], c["bounds"],
                                        c["uright"], c["mp_state"], c["inv_sigma2"], th_dist, ratio, ori)
    assert g[0] == o[0], f"nmatches {g[0]} vs {o[0]}"
    for name, x, y in zip(("q_idx", "q_dist", "kp_final"), g[1:], o[1:]):
        bad = np.nonzero(x != y)[0]
        assert len(bad) == 0, f"{name} differs at {bad[:5]}: {x[bad[:5]]} vs {y[bad[:5]]}"
    return o[0]


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("seed,n,nq,stereo", [(91, 1000, 800, False), (92, 2500, 2000, True)])
def test_projection_matchers_bit_exact(variant, seed, n, nq, stereo, oracle_mod):
    from orb_slam_2_ros_amd.synth_match import PROJ_VARIANT_ARGS as VARIANT_ARGS, make_proj_case as make_case
    c = make_case(seed, variant, n=n, nq=nq, stereo=stereo, th=VARIANT_ARGS[variant][3])
    assert _check(c, variant, oracle_mod) > 0


@pytest.mark.parametrize("variant", ["localmap", "lastframe", "keyframe"])
def test_projection_matchers_contention(variant, oracle_mod):
    """Wide windows over a dense frame with many near-duplicate descriptors:
    long candidate lists (LDS pool overflow into global scratch), frequent
    keypoint contention and full-list fallbacks in the greedy replay."""
    from orb_slam_2_ros_amd.synth_match import make_proj_case as make_case
    c = make_case(93, variant, n=6000, nq=3000, stereo=True, th=40.0)
    rng = np.random.default_rng(5)
    base = c["desc"][:40].copy()
    c["desc"][:] = base[rng.integers(0, 40, len(c["desc"]))]
    c["desc"] ^= (rng.integers(0, 256, c["desc"].shape) & rng.integers(0, 256, c["desc"].shape)
                  & rng.integers(0, 256, c["desc"].shape) & rng.integers(0, 256, c["desc"].shape)).astype(np.uint8)
    c["qdesc"][:] = base[rng.integers(0, 40, len(c["qdesc"]))]
    _check(c, variant, oracle_mod)


def test_projection_matchers_empty_and_edges(oracle_mod):
    from orb_slam_2_ros_amd.synth_match import make_proj_case as make_case
    c = make_case(94, "localmap", n=300, nq=200)
    m = ORBmatcher(0.8, False)
    nm, qi, qd, kf = m.search_by_projection("localmap", c["keys"][:0], c["desc"][:0], c["queries"], c["qdesc"],
                                            c["bounds"])
    assert nm == 0 and (qi == -1).all()
    nm, qi, qd, kf = m.search_by_projection("localmap", c["keys"], c["desc"], c["queries"][:0], c["qdesc"][:0],
                                            c["bounds"])
    assert nm == 0 and (kf == -1).all()
    q = c["queries"].copy()
    q["flags"] = 0                      # every point skipped by the caller's own tests
    assert _check(dict(c, queries=q), "localmap", oracle_mod) == 0


@pytest.mark.parametrize("seed", [95, 96])
def test_search_by_sim3_bit_exact(seed, oracle_mod):
    from orb_slam_2_ros_amd.synth_match import make_sim3_case
    kf1, kf2, q1, qd1, q2, qd2 = make_sim3_case(seed)
    nf, m = ORBmatcher(0.75, False).search_by_sim3(kf1, kf2, q1, qd1, q2, qd2)
    onf, om = oracle_mod.search_by_sim3(kf1["keys"], kf1["desc"], kf1["bounds"], kf2["keys"], kf2["desc"],
                                        kf2["bounds"], q1, qd1, q2, qd2, 100)
    assert nf == onf and onf > 50
    assert np.array_equal(m, om)


def test_cpp_adapter_projection_table(tmp_path, oracle_mod):
    """OrbxMatcher::SearchByProjectionTable of the C++ drop-in header driven
    through its cv-typed signature (local-map variant, stereo) vs the oracle."""
    import subprocess
    from cxx_build import build_adapter_test
    from orb_slam_2_ros_amd.synth_match import PROJ_VARIANT_ARGS as VARIANT_ARGS, make_proj_case as make_case
    c = make_case(98, "localmap", n=1200, nq=900, stereo=True, th=3.0)
    th, ratio, ori, _ = VARIANT_ARGS["localmap"]
    n, nq = len(c["keys"]), len(c["queries"])
    with open(tmp_path / "f.bin", "wb") as f:
        f.write(np.int32(n).tobytes()); f.write(np.array(c["bounds"], np.float32).tobytes())
        f.write(c["keys"].tobytes()); f.write(c["desc"].tobytes()); f.write(c["uright"].astype(np.float32).tobytes())
        f.write(c["mp_state"].tobytes()); f.write(np.int32(len(c["inv_sigma2"])).tobytes())
        f.write(c["inv_sigma2"].tobytes())
    with open(tmp_path / "q.bin", "wb") as f:
        f.write(np.int32(nq).tobytes()); f.write(c["queries"].tobytes()); f.write(c["qdesc"].tobytes())
    exe = build_adapter_test()
    subprocess.run([str(exe), "proj", "0", str(th), repr(ratio), str(int(ori)), str(tmp_path / "f.bin"),
                    str(tmp_path / "q.bin"), str(tmp_path / "o.bin")], check=True)
    buf = (tmp_path / "o.bin").read_bytes()
    nm = int(np.frombuffer(buf, np.int32, 1, 0)[0])
    qi = np.frombuffer(buf, np.int32, nq, 4)
    qd = np.frombuffer(buf, np.int32, nq, 4 + 4 * nq)
    kf = np.frombuffer(buf, np.int32, n, 4 + 8 * nq)
    o = oracle_mod.search_by_projection("localmap", c["keys"], c["desc"], c["queries"], c["qdesc"], c["bounds"],
                                        c["uright"], c["mp_state"], c["inv_sigma2"], th, np.float32(ratio), ori)
    assert nm == o[0] and nm > 0
    assert np.array_equal(qi, o[1]) and np.array_equal(qd, o[2]) and np.array_equal(kf, o[3])


def test_projection_pool_growth(oracle_mod):
    """Very wide windows over the largest frame the grid LDS holds: the
    candidate lists total millions of entries, more than the pool the earlier
    calls sized, so the call overflows it, learns the size and runs again."""
    from orb_slam_2_ros_amd.synth_match import make_proj_case as make_case
    c = make_case(97, "localmap", n=7000, nq=600, stereo=False, th=60.0)
    assert _check(c, "localmap", oracle_mod) > 0
    assert _check(c, "lastframe", oracle_mod, th=255) > 0


@pytest.mark.parametrize("variant", ["localmap", "keyframe"])
def test_projection_many_points(variant, oracle_mod):
    """More map points than the replay keeps in LDS (their kept entries and
    status stay in global memory)."""
    from orb_slam_2_ros_amd.synth_match import PROJ_VARIANT_ARGS as VARIANT_ARGS, make_proj_case as make_case
    c = make_case(98, variant, n=3000, nq=9000, stereo=True, th=VARIANT_ARGS[variant][3])
    assert _check(c, variant, oracle_mod) > 0
