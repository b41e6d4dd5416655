"""The heap-tie diagnostic's replica (tools/tie_heap) is the
reference's DistributeOctTree: built to sort by creation number
(-DTIE_CREATION) it must select exactly what the oracle selects, level by level,
so the real-address build differs from the oracle only by the tie rule.  CPU only."""
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]


@pytest.mark.parametrize("w,h,nf,mode", [(640, 480, 1000, "mono"), (1241, 376, 2000, "stereo")])
def test_tie_heap_replica_matches_oracle(w, h, nf, mode, oracle_mod):
    sys.path.insert(0, str(ROOT / "tools"))
    import bench
    import tie_heap
    tie_heap.build()
    frs = bench.scene_frames(mode, w, h, 3)
    imgs = [np.ascontiguousarray(frs[t][0] if mode == "stereo" else frs[t]) for t in (0, 1)]
    lvs = [tie_heap.levels_of(im, nf) for im in imgs]
    check = tie_heap.run_heap(lvs, nf, tie_heap.EXE_CHECK)
    heap = tie_heap.run_heap(lvs, nf)
    tie_heap.set_mode(0)
    for t in (0, 1):
        for l, (lw, lh, q, c, cells) in enumerate(lvs[t]):
            assert sum(cells) == len(c)
            assert check[(t, l)] == list(oracle_mod.distribute(c, lw, lh, q)), (t, l)
            assert len(heap[(t, l)]) > 0
