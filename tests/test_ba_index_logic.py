"""The fast local BA dense path's index invariant, on the CPU (no GPU): the
device-built active sets (set_active's device path, set_active_pass2) clear
the camera x point map before anything else, so every entry k_ba_schur_ops
reads is -1 or an edge index, with or without edges (the r7k GPU fault was an
uncleared map on a call with no edges).  tools/ba_index_check.py replays the
index logic of orbx_ba.hip on the bench-sized problems."""
import runpy
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def test_dense_path_index_logic(capsys):
    runpy.run_path(str(ROOT / "tools" / "ba_index_check.py"), run_name="__main__")
    assert "index logic ok" in capsys.readouterr().out
