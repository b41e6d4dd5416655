"""Ad-hoc GPU diagnostic: per-stage parity summary for a few configs."""
import sys, time
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np
from orb_slam_2_ros_amd import ORBextractor, synth
from oracle import oracle

for (w, h, nf, seed) in [(640, 480, 1000, 11), (1920, 1080, 1000, 14), (160, 120, 300, 15)]:
    img = synth.frame(w, h, seed)
    ex = ORBextractor(nf, 1.2, 8, 20, 7)
    t = time.time(); kg, dg = ex(img); t = time.time() - t
    pyr = oracle.pyramid(img)
    _, _, q, _ = oracle.levels(w, h, nf)
    print(f"== {w}x{h} nf={nf}: gpu {len(kg)} kps in {t*1e3:.1f} ms (first call)")
    for l in range(8):
        gp = ex.debug_fetch(0, l, 0); gb = ex.debug_fetch(0, l, 1)
        ob = oracle.gauss7(pyr[l])
        gc = ex.debug_fetch(0, l, 2); oc = oracle.level_candidates(pyr[l])
        gs = ex.debug_fetch(0, l, 3)
        osel = oc[oracle.distribute(oc, pyr[l].shape[1], pyr[l].shape[0], int(q[l]))]
        pe = np.count_nonzero(gp != pyr[l]); be = np.count_nonzero(gb != ob)
        ce = (len(gc) == len(oc)) and np.array_equal(gc, oc)
        se = (len(gs) == len(osel)) and np.array_equal(gs, osel)
        print(f"  L{l}: pyr diff {pe}, blur diff {be}, cand {len(gc)}/{len(oc)} eq={ce}, sel {len(gs)}/{len(osel)} eq={se}")
    ko, do = oracle.extract(img, nf)
    eqk = len(kg) == len(ko) and all(np.array_equal(kg[f], ko[f]) for f in ko.dtype.names)
    print(f"  kps {len(kg)}/{len(ko)} eq={eqk} desc eq={len(dg)==len(do) and np.array_equal(dg, do)}")
    if len(kg) == len(ko) and not eqk:
        for f in ko.dtype.names:
            bad = np.nonzero(kg[f] != ko[f])[0]
            if len(bad): print(f"   field {f}: {len(bad)} diffs, first {bad[:5]} gpu {kg[f][bad[:3]]} ora {ko[f][bad[:3]]}")
