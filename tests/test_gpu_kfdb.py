"""GPU keyframe database against the oracle's literal
KeyFrameDatabase over a query script: loop and relocalisation candidates in
the reference's order, with the per-keyframe query state carried across
queries, an erase / re-add and a repeated query id."""
import numpy as np
import pytest

from orb_slam_2_ros_amd.keyframe_db import KeyFrameDatabase, bow_score_l1

pytestmark = pytest.mark.gpu


def test_kfdb_bit_exact_vs_oracle(oracle_mod):
    from test_oracle_kat import _kfdb_script, _run_kfdb
    ops, covis = _kfdb_script()
    o = _run_kfdb(oracle_mod.KeyFrameDB(20000), ops, covis,
                  lambda db, r, q, w, v, c, m, cv: db.detect(r, q, w, v, c, m, cv))

    def gdetect(db, r, q, w, v, c, m, cv):
        return db.DetectRelocalizationCandidates(q, w, v, cv) if r else db.DetectLoopCandidates(q, w, v, c, m, cv)
    g = _run_kfdb(KeyFrameDatabase(), ops, covis, gdetect)
    assert g == o
    assert sum(len(x) > 0 for x in g) > 10


def test_kfdb_large_database(oracle_mod):
    """2,000 keyframes of 1,000 words (past the LDS-staged query size only
    for the query side cases below), a loop query per 100 keyframes."""
    from orb_slam_2_ros_amd.synth_vocab import make_keyframe_bows
    bows, covis = make_keyframe_bows(n_kf=2000, n_words=100000, words_per_kf=1000, seed=9, loop_every=150)
    g, o = KeyFrameDatabase(), oracle_mod.KeyFrameDB(100000)
    cv = lambda k: covis.get(k, [])   # noqa: E731
    for i, (w, v) in enumerate(bows):
        if i and i % 100 == 0:
            a = g.DetectLoopCandidates(i, w, v, covis[i], 0.01, cv)
            b = o.detect(False, i, w, v, covis[i], 0.01, cv)
            assert a == b
        g.add(i, w, v)
        o.add(i, w, v)
    # a query with more words than the kernels stage in LDS
    w = np.unique(np.concatenate([bows[5][0], np.arange(50000, 60000, dtype=np.uint32)]))
    v = np.full(len(w), 1.0 / len(w))
    assert g.DetectRelocalizationCandidates(777777, w, v, cv) == o.detect(True, 777777, w, v, None, 0.0, cv)


def test_bow_score_l1_host(oracle_mod):
    from orb_slam_2_ros_amd.synth_vocab import make_keyframe_bows
    bows, _ = make_keyframe_bows(n_kf=10, n_words=3000, words_per_kf=200, seed=3)
    assert bow_score_l1(*bows[1], *bows[2]) == oracle_mod.bow_score_l1(*bows[1], *bows[2])


def test_kfdb_add_rejects_duplicates():
    from orb_slam_2_ros_amd import OrbxError
    db = KeyFrameDatabase()
    db.add(7, np.array([1, 5, 9], np.uint32), np.array([0.2, 0.3, 0.5]))
    with pytest.raises(OrbxError):
        db.add(7, np.array([1], np.uint32), np.array([1.0]))
    with pytest.raises(OrbxError):   # words must ascend
        db.add(8, np.array([5, 1], np.uint32), np.array([0.5, 0.5]))
    db.erase(7)
    db.add(7, np.array([2], np.uint32), np.array([1.0]))
    assert db.size() == 1


def test_kfdb_state_across_readd_chains(oracle_mod):
    """Device-resident query state: keyframes queried, then erased and re-added
    twice with no query in between (the new slots inherit the state through a
    slot that never reached the device), then queried again with the same and
    with new query ids -- candidate lists equal the oracle's."""
    from orb_slam_2_ros_amd.synth_vocab import make_keyframe_bows
    bows, covis = make_keyframe_bows(n_kf=300, n_words=20000, words_per_kf=300, seed=17, loop_every=40)
    g, o = KeyFrameDatabase(), oracle_mod.KeyFrameDB(20000)
    cv = lambda k: covis.get(k, [])   # noqa: E731
    res_g, res_o = [], []

    def both(kind, qid, i, ms=0.01):
        w, v = bows[i]
        if kind == "loop":
            res_g.append(g.DetectLoopCandidates(qid, w, v, covis[i], ms, cv))
            res_o.append(o.detect(False, qid, w, v, covis[i], ms, cv))
        else:
            res_g.append(g.DetectRelocalizationCandidates(qid, w, v, cv))
            res_o.append(o.detect(True, qid, w, v, None, 0.0, cv))
    for i in range(200):
        g.add(i, *bows[i]); o.add(i, *bows[i])
    for i in range(40, 200, 9):
        both("loop", i, i)
        both("reloc", 5000 + i, i)
    for k in range(30, 90, 3):   # erase, re-add, erase, re-add: no query in between
        for _ in range(2):
            g.erase(k); o.erase(k)
            g.add(k, *bows[k]); o.add(k, *bows[k])
    for i in range(200, 300):
        g.add(i, *bows[i]); o.add(i, *bows[i])
    for i in range(45, 300, 7):
        both("loop", i, i, 0.005)                  # some ids repeat earlier queries
        both("reloc", 5000 + (i // 2) * 2, i)
    assert res_g == res_o
    assert sum(len(x) > 0 for x in res_o) > 20


def test_kfdb_long_keyframes_and_many_slots(oracle_mod):
    """The scoring kernel's edges: keyframes of 2,500 words (three 1,024-word
    score steps each), and a 20,000-keyframe database over a small vocabulary
    (every query meets most slots, the slot scan takes two passes of the
    grid, and a wave scores several keyframes in turn)."""
    from orb_slam_2_ros_amd.synth_vocab import make_keyframe_bows
    cases = [dict(n_kf=300, n_words=60000, words_per_kf=2500, seed=23, loop_every=40),
             dict(n_kf=20000, n_words=3000, words_per_kf=60, seed=29, loop_every=500)]
    for c in cases:
        bows, covis = make_keyframe_bows(**c)
        g, o = KeyFrameDatabase(), oracle_mod.KeyFrameDB(c["n_words"])
        cv = lambda k: covis.get(k, [])   # noqa: E731
        n, step = c["n_kf"], max(c["n_kf"] // 6, 1)
        res_g, res_o = [], []
        for i in range(n):
            if i and i % step == 0:
                w, v = bows[i]
                res_g.append(g.DetectLoopCandidates(i, w, v, covis[i], 0.005, cv))
                res_o.append(o.detect(False, i, w, v, covis[i], 0.005, cv))
                res_g.append(g.DetectRelocalizationCandidates(900000 + i, w, v, cv))
                res_o.append(o.detect(True, 900000 + i, w, v, None, 0.0, cv))
            g.add(i, *bows[i])
            o.add(i, *bows[i])
        assert res_g == res_o
        assert sum(len(x) > 0 for x in res_o) > 3


def test_kfdb_more_candidates_than_the_first_copy(oracle_mod):
    """More than 1,024 scored keyframes (the list the first copy brings back):
    1,500 keyframes sharing most of their words with the query, so the
    relocalisation query scores and keeps all of them."""
    rng = np.random.default_rng(41)
    base = np.sort(rng.choice(5000, 300, replace=False)).astype(np.uint32)
    g, o = KeyFrameDatabase(), oracle_mod.KeyFrameDB(5000)
    covis = {}
    for i in range(1500):
        w = np.unique(np.concatenate([base[rng.random(len(base)) < 0.95], rng.choice(5000, 20).astype(np.uint32)]))
        v = rng.random(len(w)) + 0.1
        v /= v.sum()
        g.add(i, w, v)
        o.add(i, w, v)
        covis[i] = [j for j in (i - 1, i + 1, i + 7) if 0 <= j < 1500]
    cv = lambda k: covis.get(k, [])   # noqa: E731
    v = np.full(len(base), 1.0 / len(base))
    a = g.DetectRelocalizationCandidates(99999, base, v, cv)
    b = o.detect(True, 99999, base, v, None, 0.0, cv)
    assert a == b and len(b) > 0
    a = g.DetectLoopCandidates(99998, base, v, [3, 5], 0.0, cv)
    b = o.detect(False, 99998, base, v, [3, 5], 0.0, cv)
    assert a == b and len(b) > 0


def test_kfdb_query_id_zero_matches_never_queried(oracle_mod):
    """A query whose id is 0 matches every keyframe that was never queried
    (KeyFrame.cc initialises mnLoopQuery / mnRelocQuery to 0), including
    covisible neighbours the query's own walk did not meet: the candidate
    lists equal the oracle's (the device path used to gather those
    neighbours' state only for an id used before)."""
    from orb_slam_2_ros_amd.synth_vocab import make_keyframe_bows
    bows, covis = make_keyframe_bows(n_kf=300, n_words=4000, words_per_kf=150, seed=21, loop_every=40)
    # every keyframe's covisibility also names far keyframes that share few words
    cov = {k: list(covis.get(k, [])) + [(k + 97) % 300, (k + 151) % 300] for k in range(300)}
    cv = lambda k: cov.get(k, [])   # noqa: E731
    g, o = KeyFrameDatabase(), oracle_mod.KeyFrameDB(4000)
    for i, (w, v) in enumerate(bows[:250]):
        g.add(i, w, v)
        o.add(i, w, v)
    for qi in (250, 260, 280):
        w, v = bows[qi]
        assert g.DetectLoopCandidates(0, w, v, cov[qi][:3], 0.0, cv) == o.detect(False, 0, w, v, cov[qi][:3], 0.0, cv)
        assert g.DetectRelocalizationCandidates(0, w, v, cv) == o.detect(True, 0, w, v, None, 0.0, cv)


def test_kfdb_rejects_word_ids_past_the_bound():
    from orb_slam_2_ros_amd import OrbxError
    db = KeyFrameDatabase()
    db.add(1, np.array([3, (1 << 26) - 1], np.uint32), np.array([0.5, 0.5]))
    with pytest.raises(OrbxError):
        db.add(2, np.array([3, 1 << 26], np.uint32), np.array([0.5, 0.5]))
    with pytest.raises(OrbxError):
        db.add(3, np.array([0xFFFFFFFF], np.uint32), np.array([1.0]))
    assert db.size() == 1


def test_kfdb_orbvoc_sized_word_ids(oracle_mod):
    """Word ids over ORBvoc's whole range (10^6 words): the inverted file's
    count scan spans ~245 tiles of the three-launch scan; rebuilt several
    times as keyframes arrive."""
    from orb_slam_2_ros_amd.synth_vocab import make_keyframe_bows
    bows, covis = make_keyframe_bows(n_kf=900, n_words=1_000_000, words_per_kf=800, seed=21, loop_every=90)
    g, o = KeyFrameDatabase(), oracle_mod.KeyFrameDB(1_000_000)
    cv = lambda k: covis.get(k, [])   # noqa: E731
    hits = 0
    for i, (w, v) in enumerate(bows):
        if i and i % 60 == 0:
            a = g.DetectLoopCandidates(i, w, v, covis[i], 0.01, cv)
            assert a == o.detect(False, i, w, v, covis[i], 0.01, cv)
            r = g.DetectRelocalizationCandidates(10_000 + i, w, v, cv)
            assert r == o.detect(True, 10_000 + i, w, v, None, 0.0, cv)
            hits += len(a) > 0
        g.add(i, w, v)
        o.add(i, w, v)
    assert hits > 0
