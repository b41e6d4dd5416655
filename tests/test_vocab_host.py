"""Host side of the vocabulary: the two file loaders of
TemplatedVocabulary (text :1351-1425, binary :1473-1547) read back exactly
what the synthetic writers wrote, reject what the reference rejects, and an
empty transform needs no device.  CPU only."""
import numpy as np
import pytest

from orb_slam_2_ros_amd.synth_vocab import make_vocab, write_binary, write_text
from orb_slam_2_ros_amd.vocabulary import ORBVocabulary


@pytest.mark.parametrize("fmt", ["text", "binary"])
@pytest.mark.parametrize("irregular", [False, True])
def test_loader_round_trip(fmt, irregular, tmp_path):
    voc = make_vocab(k=5, L=3, seed=11, irregular=irregular, scoring=1, weighting=2)
    path = tmp_path / f"voc.{fmt}"
    (write_text if fmt == "text" else write_binary)(voc, path)
    v = ORBVocabulary()
    assert (v.loadFromTextFile(path) if fmt == "text" else v.loadFromBinFile(path))
    assert (v.getBranchingFactor(), v.getDepthLevels(), v.getScoringType(), v.getWeightingType()) == (5, 3, 1, 2)
    assert v.size() == int(voc["is_leaf"].sum()) and v.n_nodes() == len(voc["parent"])
    parent, leaf, desc, weight = v.export()
    assert np.array_equal(parent[1:], voc["parent"][1:])
    assert np.array_equal(leaf[1:], voc["is_leaf"][1:])
    assert np.array_equal(desc[1:], voc["desc"][1:])
    assert np.array_equal(weight[1:], voc["weight"][1:])     # doubles round-trip exactly


def test_loader_rejects_bad_headers_and_parents(tmp_path):
    v = ORBVocabulary()
    p = tmp_path / "bad.txt"
    p.write_text("21 3 0 0\n")                              # k > 20
    assert not v.loadFromTextFile(p)
    p.write_text("10 0 0 0\n")                              # L < 1
    assert not v.loadFromTextFile(p)
    p.write_text("10 3 6 0\n")                              # scoring > 5
    assert not v.loadFromTextFile(p)
    p.write_text("10 3 0 4\n")                              # weighting > 3
    assert not v.loadFromTextFile(p)
    p.write_text("4 2 0 0\n" + "5 1 " + " ".join(["0"] * 32) + " 1.0\n")   # parent after the node
    assert not v.loadFromTextFile(p)
    assert not v.loadFromTextFile(tmp_path / "missing.txt")
    assert v.empty()


def test_binary_loader_stops_at_expected_nodes(tmp_path):
    voc = make_vocab(k=3, L=2, seed=2)                       # (3^3-1)/2 = 13 nodes
    p = tmp_path / "voc.bin"
    write_binary(voc, p)
    with open(p, "ab") as f:                                 # trailing records past the expected count
        f.write(b"\x00" * 45 * 3)
    v = ORBVocabulary()
    assert v.loadFromBinFile(p) and v.n_nodes() == 13
    with open(p, "r+b") as f:                                # truncated: the last complete record
        f.truncate(16 + 45 * 7 + 20)
    assert v.loadFromBinFile(p) and v.n_nodes() == 8


def test_text_loader_blank_lines(tmp_path):
    voc = make_vocab(k=3, L=2, seed=4)
    p = tmp_path / "voc.txt"
    write_text(voc, p)
    p.write_text(p.read_text() + "\n\n")
    v = ORBVocabulary()
    assert v.loadFromTextFile(p) and v.n_nodes() == len(voc["parent"])


def test_transform_empty_needs_no_device():
    voc = make_vocab(k=3, L=2, seed=5)
    v = ORBVocabulary.from_arrays(voc["k"], voc["L"], 0, 0, voc["parent"], voc["is_leaf"], voc["desc"],
                                  voc["weight"])
    bow, fv = v.transform(np.zeros((0, 32), np.uint8))
    assert bow == {} and fv == {}
