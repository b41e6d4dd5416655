"""CPU emulation of the fast local BA dense path's index logic (set_active on the device, then the
k_ba_schur_ops map reads): every map entry it reads is -1 or an edge, with and without edges.
    python tools/ba_index_check.py"""
import sys, numpy as np
sys.path.insert(0, str(__import__('pathlib').Path(__file__).resolve().parents[1]))
from orb_slam_2_ros_amd.synth_ba import make_ba_problem

def emulate(Tcw, fixed, Xw, edges, act=None):
    ncam, npt, ne = len(Tcw), len(Xw), len(edges)
    free_idx = np.full(ncam, -1); nf = 0
    for c in range(ncam):
        if not fixed[c]: free_idx[c] = nf; nf += 1
    cam = np.array([int(e['cam']) for e in edges], dtype=np.int64) if ne else np.zeros(0, np.int64)
    pt = np.array([int(e['point']) for e in edges], dtype=np.int64) if ne else np.zeros(0, np.int64)
    efree = free_idx[cam] if ne else np.zeros(0, np.int64)
    # uniqueness (alloc)
    unique = True
    for p in range(npt):
        fs = efree[(pt == p) & (efree >= 0)]
        if len(fs) != len(set(fs.tolist())): unique = False; break
    active = np.ones(ne, np.uint8) if act is None else act
    # set_active device path: memset -1 (before the ne check), then the map
    cmap = np.full(max(nf, 1) * max(npt, 1), 0x7ead, np.int64)   # garbage
    if nf and npt: cmap[: nf * npt] = -1
    if ne:
        for e in range(ne):
            f = efree[e]
            if active[e] and f >= 0: cmap[f * npt + pt[e]] = e
    # k_ba_schur_ops reads for p < npt, f < nf
    for p in range(npt):
        for f in range(nf):
            ed = cmap[f * npt + p]
            assert ed == -1 or 0 <= ed < ne, (p, f, ed)
    return unique, nf, npt, ne

P = make_ba_problem(n_local=5, n_fixed=2, n_points=500, seed=8, stereo_frac=0.0)
E = P['edges']
print('mono', emulate(P['Tcw'], P['fixed'], P['Xw'], E))
print('empty', emulate(P['Tcw'], P['fixed'], P['Xw'], E[:0]))
P = make_ba_problem(n_local=20, n_fixed=4, n_points=3000, seed=2)
print('bench', emulate(P['Tcw'], P['fixed'], P['Xw'], P['edges'][:4000]))
# the second pass's set (set_active_pass2): a subset active, the map cleared first
rng = np.random.default_rng(0)
print('pass2', emulate(P['Tcw'], P['fixed'], P['Xw'], P['edges'], act=(rng.random(len(P['edges'])) > 0.1).astype(np.uint8)))
print('index logic ok')
