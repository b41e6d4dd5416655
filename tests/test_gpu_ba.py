"""GPU local bundle adjustment against the
oracle's CPU restatement: the LM linear system's step (same summation order
on both sides), and whole LocalBundleAdjustment runs (two passes, outlier
removal) on KITTI-like stereo problems.  FP64; the step is compared to 1e-12
relative, the final float estimates, outlier flags and iteration counts
exactly (measured identical on these problems; the SE3 exponentials use the
device's sin/cos, so an ulp there could in principle show)."""
import numpy as np
import pytest

from orb_slam_2_ros_amd.optimizer import debug_step, local_bundle_adjustment
from orb_slam_2_ros_amd.synth_ba import make_ba_problem

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("robust,lam", [(True, 1e-3), (False, 10.0)])
def test_ba_step_matches_oracle(robust, lam, oracle_mod):
    P = make_ba_problem(n_local=8, n_fixed=3, n_points=1200, seed=6)
    xg, cg, okg = debug_step(P["Tcw"], P["fixed"], P["Xw"], P["edges"], robust, lam)
    xo, co, oko = oracle_mod.ba_debug_step(P["Tcw"], P["fixed"], P["Xw"], P["edges"], robust, lam)
    assert okg and oko
    assert cg == co                                       # robust chi2 sums: bit-exact
    scale = np.abs(xo).max()
    assert np.abs(xg - xo).max() <= 1e-12 * scale, np.abs(xg - xo).max() / scale


# (the reduced camera system: n <= 128 unknowns is factored in LDS, 30 local
# keyframes take the global-memory Cholesky)
@pytest.mark.parametrize("seed,n_local,n_points", [(1, 10, 1500), (2, 20, 3000), (3, 4, 300), (4, 30, 2500)])
def test_local_ba_matches_oracle(seed, n_local, n_points, oracle_mod):
    P = make_ba_problem(n_local=n_local, n_fixed=4, n_points=n_points, seed=seed)
    Tg, Xg, og, ig = local_bundle_adjustment(P["Tcw"], P["fixed"], P["Xw"], P["edges"])
    To, Xo, oo, io = oracle_mod.local_ba(P["Tcw"], P["fixed"], P["Xw"], P["edges"])
    assert ig == io
    assert np.array_equal(og, oo)
    assert np.array_equal(Tg, To) and np.array_equal(Xg, Xo)
    free = P["fixed"] == 0
    assert np.array_equal(Tg[~free], P["Tcw"][~free])     # fixed cameras untouched


def test_local_ba_mono_only_and_empty(oracle_mod):
    P = make_ba_problem(n_local=5, n_fixed=2, n_points=500, seed=8, stereo_frac=0.0)
    Tg, Xg, og, ig = local_bundle_adjustment(P["Tcw"], P["fixed"], P["Xw"], P["edges"])
    To, Xo, oo, io = oracle_mod.local_ba(P["Tcw"], P["fixed"], P["Xw"], P["edges"])
    assert ig == io and np.array_equal(og, oo)
    assert np.array_equal(Tg, To) and np.array_equal(Xg, Xo)
    e = P["edges"][:0]
    Tg, Xg, og, ig = local_bundle_adjustment(P["Tcw"], P["fixed"], P["Xw"], e)
    assert len(og) == 0


def test_local_ba_repeated_observation(oracle_mod):
    """A (camera, point) pair observed twice: the Schur pairs leave the
    per-camera point maps for the merge walk, still identical to the oracle."""
    P = make_ba_problem(n_local=6, n_fixed=2, n_points=600, seed=9)
    e = np.concatenate([P["edges"], P["edges"][5:6], P["edges"][40:41]])
    Tg, Xg, og, ig = local_bundle_adjustment(P["Tcw"], P["fixed"], P["Xw"], e)
    To, Xo, oo, io = oracle_mod.local_ba(P["Tcw"], P["fixed"], P["Xw"], e)
    assert ig == io and np.array_equal(og, oo)
    assert np.array_equal(Tg, To) and np.array_equal(Xg, Xo)


def test_local_ba_workspace_reuse(oracle_mod):
    """The per-device workspace across calls: problems that grow, shrink and
    cross the LDS / global-memory Cholesky boundary (21 and 22 free
    keyframes: 126 / 132 unknowns) in turn, a repeated observation in
    between; every call identical to the oracle."""
    seq = [(22, 2000, 31), (5, 400, 32), (21, 1800, 33), (6, 600, 9), (22, 2000, 34), (21, 1800, 33)]
    for k, (n_local, n_points, seed) in enumerate(seq):
        P = make_ba_problem(n_local=n_local, n_fixed=3, n_points=n_points, seed=seed)
        e = P["edges"]
        if k == 3:
            e = np.concatenate([e, e[7:8]])
        Tg, Xg, og, ig = local_bundle_adjustment(P["Tcw"], P["fixed"], P["Xw"], e)
        To, Xo, oo, io = oracle_mod.local_ba(P["Tcw"], P["fixed"], P["Xw"], e)
        assert ig == io and np.array_equal(og, oo), k
        assert np.array_equal(Tg, To) and np.array_equal(Xg, Xo), k


@pytest.mark.parametrize("seed,n_local,n_points", [(1, 10, 1500), (2, 20, 3000), (3, 4, 300), (5, 21, 3000),
                                                   (4, 30, 2500)])
def test_local_ba_fast_mode_within_tolerance(seed, n_local, n_points, oracle_mod):
    """orbx_local_ba_fast (the per-vertex and per-pair sums as parallel
    reductions) against the ordered oracle: identical outlier flags, poses and
    points equal to 1e-4 relative (float outputs; the double-precision LM
    differs by rounding only)."""
    P = make_ba_problem(n_local=n_local, n_fixed=4, n_points=n_points, seed=seed)
    Tg, Xg, og, ig = local_bundle_adjustment(P["Tcw"], P["fixed"], P["Xw"], P["edges"], fast=True)
    To, Xo, oo, io = oracle_mod.local_ba(P["Tcw"], P["fixed"], P["Xw"], P["edges"])
    assert np.array_equal(og, oo), f"outlier flags differ at {np.nonzero(og != oo)[0][:8]}"
    assert np.abs(Tg - To).max() <= 1e-4 * max(1.0, np.abs(To).max()), np.abs(Tg - To).max()
    assert np.abs(Xg - Xo).max() <= 1e-4 * np.abs(Xo).max(), np.abs(Xg - Xo).max()
    free = P["fixed"] == 0
    assert np.array_equal(Tg[~free], P["Tcw"][~free])
    assert abs(ig[0] - io[0]) <= 1 and abs(ig[1] - io[1]) <= 2, (ig, io)


def _fast_close(P, e, oracle_mod, tag):
    Tg, Xg, og, ig = local_bundle_adjustment(P["Tcw"], P["fixed"], P["Xw"], e, fast=True)
    To, Xo, oo, io = oracle_mod.local_ba(P["Tcw"], P["fixed"], P["Xw"], e)
    assert np.array_equal(og, oo), (tag, np.nonzero(og != oo)[0][:8])
    assert np.abs(Tg - To).max() <= 1e-4 * max(1.0, np.abs(To).max()), (tag, np.abs(Tg - To).max())
    assert np.abs(Xg - Xo).max() <= 1e-4 * np.abs(Xo).max(), (tag, np.abs(Xg - Xo).max())
    assert abs(ig[0] - io[0]) <= 1 and abs(ig[1] - io[1]) <= 2, (tag, ig, io)


def test_local_ba_fast_mode_paths_and_reuse(oracle_mod):
    """The fast mode's paths across one workspace: the dense Schur product
    and the augmented-system Cholesky (<= 126 unknowns), the global-memory
    Cholesky past them (22 free keyframes: 132 unknowns), a repeated (camera,
    point) observation (no point maps: the merge-walk pairs and the ordered
    right-hand side), growing and shrinking problems, and an ordered-mode call
    in between (its workspace has no dense operand); every call against the
    ordered oracle within the fast mode's tolerance."""
    seq = [(20, 3000, 2, False), (22, 2000, 34, False), (5, 400, 32, False), (6, 600, 9, True),
           (21, 1800, 33, False), (10, 1500, 1, False)]
    for k, (n_local, n_points, seed, dup) in enumerate(seq):
        P = make_ba_problem(n_local=n_local, n_fixed=3 if n_local != 20 else 4, n_points=n_points, seed=seed)
        e = P["edges"]
        if dup:
            e = np.concatenate([e, e[7:8]])
        _fast_close(P, e, oracle_mod, k)
        if k == 2:   # an ordered call on the same workspace, bit-exact
            Tg, Xg, og, ig = local_bundle_adjustment(P["Tcw"], P["fixed"], P["Xw"], e)
            To, Xo, oo, io = oracle_mod.local_ba(P["Tcw"], P["fixed"], P["Xw"], e)
            assert ig == io and np.array_equal(og, oo) and np.array_equal(Tg, To) and np.array_equal(Xg, Xo)


def test_local_ba_fast_mode_mono_only_and_empty(oracle_mod):
    """The fast mode on a monocular-only problem (2-row edges throughout) and
    with no edges at all (nothing to optimise: the estimate comes back as
    given, up to the float round trip)."""
    P = make_ba_problem(n_local=5, n_fixed=2, n_points=500, seed=8, stereo_frac=0.0)
    _fast_close(P, P["edges"], oracle_mod, "mono")
    e = P["edges"][:0]
    Tg, Xg, og, ig = local_bundle_adjustment(P["Tcw"], P["fixed"], P["Xw"], e, fast=True)
    assert len(og) == 0
    assert np.abs(Tg - P["Tcw"]).max() <= 1e-6 and np.abs(Xg - P["Xw"]).max() <= 1e-6 * np.abs(P["Xw"]).max()
