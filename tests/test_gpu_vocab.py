"""GPU parity of the DBoW2 transform against the CPU
oracle: BowVector words and values (doubles, bit-exact), FeatureVector nodes
and feature lists, and the per-feature (word, weight, node) of the device
entry point, on synthetic vocabularies including ORBvoc's size (k=10, L=6,
1.1M nodes)."""
import numpy as np
import pytest

from orb_slam_2_ros_amd.synth_vocab import features_near_leaves, make_vocab
from orb_slam_2_ros_amd.vocabulary import ORBVocabulary

pytestmark = pytest.mark.gpu


def _vocab(voc):
    # (the header's k is informational and capped at 20 as the loaders check;
    # the descent follows the tree's own child counts)
    return ORBVocabulary.from_arrays(min(voc["k"], 20), voc["L"], voc["scoring"], voc["weighting"], voc["parent"],
                                     voc["is_leaf"], voc["desc"], voc["weight"])


def _check(v, voc, feats, levelsup, oracle_mod):
    bow, fv = v.transform(feats, levelsup)
    obow, ofv, _ = oracle_mod.vocab_transform(voc, feats, levelsup)
    assert list(bow) == list(obow), "BowVector words differ"
    bad = [w for w in bow if bow[w] != obow[w]]
    assert not bad, f"BowVector values differ at {bad[:5]}"
    assert fv == ofv, "FeatureVector differs"
    return len(bow)


@pytest.mark.parametrize("irregular", [False, True])
@pytest.mark.parametrize("scoring,weighting", [(0, 0), (1, 1), (5, 0), (0, 2)])
def test_transform_bit_exact(irregular, scoring, weighting, oracle_mod):
    voc = make_vocab(k=10 if not irregular else 14, L=4, seed=21 + irregular, irregular=irregular,
                     scoring=scoring, weighting=weighting, stop_frac=0.05)
    v = _vocab(voc)
    feats = features_near_leaves(voc, 1500, seed=3)
    for levelsup in (0, 1, 4, 7):
        assert _check(v, voc, feats, levelsup, oracle_mod) > 50


def test_transform_orbvoc_size(oracle_mod):
    """k=10, L=6 (ORBvoc.txt's shape), 2000 features, levelsup 4 as
    Frame::ComputeBoW / KeyFrame::ComputeBoW call it."""
    voc = make_vocab(k=10, L=6, seed=5)
    v = _vocab(voc)
    feats = features_near_leaves(voc, 2000, seed=9, noise=30)
    assert _check(v, voc, feats, 4, oracle_mod) > 1000


def test_transform_wide_nodes(oracle_mod):
    """Branching factors past one DPP row (17..32 and 33..64 children)."""
    for k in (20, 40):
        voc = make_vocab(k=k, L=2, seed=k)
        v = _vocab(voc)
        feats = features_near_leaves(voc, 700, seed=k + 1)
        assert _check(v, voc, feats, 1, oracle_mod) > 50


def test_transform_device_per_feature(oracle_mod):
    import torch
    voc = make_vocab(k=10, L=5, seed=8, stop_frac=0.1)
    v = _vocab(voc)
    feats = features_near_leaves(voc, 4096, seed=2)
    d = torch.from_numpy(feats).cuda()
    word = torch.zeros(4096, dtype=torch.int32, device="cuda")
    wt = torch.zeros(4096, dtype=torch.float64, device="cuda")
    node = torch.zeros(4096, dtype=torch.int32, device="cuda")
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    v.transform_device(d.data_ptr(), 4096, 2, word.data_ptr(), wt.data_ptr(), node.data_ptr(), st.cuda_stream)
    st.synchronize()
    _, _, (ow, owt, ond) = oracle_mod.vocab_transform(voc, feats, 2)
    assert np.array_equal(word.cpu().numpy().view(np.uint32), ow)
    assert np.array_equal(wt.cpu().numpy(), owt)
    assert np.array_equal(node.cpu().numpy().view(np.uint32), ond)


def test_transform_file_loaded(tmp_path, oracle_mod):
    from orb_slam_2_ros_amd.synth_vocab import write_binary, write_text
    voc = make_vocab(k=8, L=4, seed=13)
    feats = features_near_leaves(voc, 800, seed=4)
    for fmt, writer in (("txt", write_text), ("bin", write_binary)):
        p = tmp_path / f"voc.{fmt}"
        writer(voc, p)
        v = ORBVocabulary()
        assert (v.loadFromTextFile(p) if fmt == "txt" else v.loadFromBinFile(p))
        assert _check(v, voc, feats, 4, oracle_mod) > 50


def test_cpp_adapter_vocabulary(tmp_path, oracle_mod):
    """OrbxVocabulary of the C++ drop-in header: loadFromTextFile, then
    transform(vector<cv::Mat>, std::map BowVector, std::map FeatureVector, 4)."""
    import struct
    import subprocess
    from cxx_build import build_adapter_test
    from orb_slam_2_ros_amd.synth_vocab import write_text
    voc = make_vocab(k=10, L=5, seed=31)
    feats = features_near_leaves(voc, 1000, seed=6)
    write_text(voc, tmp_path / "voc.txt")
    (tmp_path / "f.raw").write_bytes(feats.tobytes())
    exe = build_adapter_test()
    subprocess.run([str(exe), "vocab", str(tmp_path / "voc.txt"), str(tmp_path / "f.raw"), "1000", "4",
                    str(tmp_path / "o.bin")], check=True)
    buf = (tmp_path / "o.bin").read_bytes()
    nb = struct.unpack_from("<i", buf, 0)[0]
    off = 4
    bow = {}
    for _ in range(nb):
        w, x = struct.unpack_from("<Id", buf, off)
        bow[w] = x
        off += 12
    nf = struct.unpack_from("<i", buf, off)[0]
    off += 4
    fv = {}
    for _ in range(nf):
        node, c = struct.unpack_from("<Ii", buf, off)
        off += 8
        fv[node] = list(struct.unpack_from(f"<{c}i", buf, off))
        off += 4 * c
    obow, ofv, _ = oracle_mod.vocab_transform(voc, feats, 4)
    assert bow == obow and fv == ofv and nb > 100
