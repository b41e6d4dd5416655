import sys; sys.path.insert(0, "."); sys.path.insert(0, "tests")
import numpy as np
from orb_slam_2_ros_amd.optimizer import local_bundle_adjustment
from orb_slam_2_ros_amd.synth_ba import make_ba_problem
from oracle import oracle
for seed, nl, npnt in [(1, 10, 1500), (2, 20, 3000), (3, 4, 300)]:
    P = make_ba_problem(n_local=nl, n_fixed=4, n_points=npnt, seed=seed)
    for iters in [(1, 0), (5, 0), (5, 1), (5, 10)]:
        Tg, Xg, og, ig = local_bundle_adjustment(P["Tcw"], P["fixed"], P["Xw"], P["edges"], iters)
        To, Xo, oo, io = oracle.local_ba(P["Tcw"], P["fixed"], P["Xw"], P["edges"], iters)
        d = np.nonzero(og != oo)[0]
        print(seed, iters, ig, io, "flag diffs", len(d), d[:5], "T", np.abs(Tg - To).max(), "X", np.abs(Xg - Xo).max(), flush=True)
