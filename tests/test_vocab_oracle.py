"""Known-answer tests of the DBoW2 restatement (oracle/dbow2_oracle.cc) on hand-built trees,
against TemplatedVocabulary::transform / loadFromTextFile semantics
(ORB_SLAM2/Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1127-1259, 1338-1424;
BowVector.cpp:38-98; FeatureVector.cpp:31-45).  CPU only."""
import math

import numpy as np
import pytest

from ar_orbslam2_amd.vocabulary import complete_tree
from oracle import oracle as O

from vocabdata import kat_features, kat_tree, random_tree, write_text


def _voc(scoring=0, weighting=0, L=2):
    return O.Vocabulary.from_nodes(2, L, scoring, weighting, *kat_tree())


def _fv(r):
    return {int(i): r["fv_feats"][r["fv_off"][j]:r["fv_off"][j + 1]].tolist()
            for j, i in enumerate(r["fv_ids"])}


def test_kat_descent_weights_and_l1_tfidf():
    r = _voc().transform(kat_features(), levelsup=1)
    # f0 Z -> A -> leaf 3 (word 0); f1 F -> B -> leaf 5 (word 2, weight 0: stopped);
    # f2 HI ties A/B at 128 -> first child A -> leaf 4 (word 1); f3 = f0; f4 LO -> A -> 3
    assert r["word_of"].tolist() == [0, 0xFFFFFFFF, 1, 0, 0]
    assert r["bow_words"].tolist() == [0, 1]
    # TF-IDF: word 0 = 0.5+0.5+0.5, word 1 = 1.5; L1 normalised by 3.0
    assert r["bow_values"].tolist() == [0.5, 0.5]
    assert _fv(r) == {1: [0, 2, 3, 4]}  # nid level L - levelsup = 1


@pytest.mark.parametrize("levelsup,fv", [(0, {3: [0, 3, 4], 4: [2]}), (2, {0: [0, 2, 3, 4]}),
                                         (5, {0: [0, 2, 3, 4]})])
def test_kat_feature_vector_levels(levelsup, fv):
    assert _fv(_voc().transform(kat_features(), levelsup=levelsup)) == fv


def test_kat_leaf_above_nid_level_is_the_leaf():
    # declared L=4, levelsup=1 -> nid level 3, but the tree ends at depth 2
    assert _fv(_voc(L=4).transform(kat_features(), levelsup=1)) == {3: [0, 3, 4], 4: [2]}


def test_kat_weighting_and_scoring_variants():
    f = kat_features()
    # IDF: addIfNotExist -> word 0 = 0.5 once, word 1 = 1.5; L1 -> 0.25, 0.75
    assert _voc(0, 2).transform(f)["bow_values"].tolist() == [0.25, 0.75]
    # DOT_PRODUCT does not normalise; TF-IDF then divides by the number of words (2)
    assert _voc(5, 0).transform(f)["bow_values"].tolist() == [0.75, 0.75]
    # L2 with TF weighting (weights as stored): sqrt(1.5^2 + 1.5^2)
    v = _voc(1, 1).transform(f)["bow_values"]
    assert v.tolist() == [1.5 / math.sqrt(4.5)] * 2
    # BINARY with KL scoring (L1): addIfNotExist as IDF
    assert _voc(3, 3).transform(f)["bow_values"].tolist() == [0.25, 0.75]


def test_empty_inputs_and_empty_vocabulary():
    r = _voc().transform(np.zeros((0, 32), np.uint8))
    assert len(r["bow_words"]) == 0 and len(r["fv_ids"]) == 0
    e = O.Vocabulary.from_nodes(10, 6, 0, 0, np.zeros(0, np.int32), np.zeros(0, np.uint8),
                                np.zeros((0, 32), np.uint8), np.zeros(0))
    r = e.transform(kat_features())
    assert len(r["bow_words"]) == 0 and (r["word_of"] == 0xFFFFFFFF).all()


def test_text_loader_roundtrip(tmp_path):
    parent, is_leaf, desc, weight = random_tree(3)
    p = tmp_path / "voc.txt"
    write_text(p, 6, 4, 0, 0, parent, is_leaf, desc, weight)
    a = O.Vocabulary.load_text(p)
    b = O.Vocabulary.from_nodes(6, 4, 0, 0, parent, is_leaf, desc, weight)
    assert a.info() == b.info() == dict(k=6, L=4, scoring=0, weighting=0,
                                        n_nodes=len(parent) + 1, n_words=int(is_leaf.sum()))
    d = np.random.default_rng(1).integers(0, 256, (300, 32), dtype=np.uint8)
    ra, rb = a.transform(d, 2), b.transform(d, 2)
    for key in ra:
        assert np.array_equal(ra[key], rb[key]), key


@pytest.mark.parametrize("header", ["21 6 0 0", "10 0 0 0", "10 6 6 0", "10 6 0 4"])
def test_text_loader_rejects_headers_the_reference_rejects(tmp_path, header):
    p = tmp_path / "bad.txt"
    p.write_text(header + "\n0 1 " + "0 " * 32 + " 1\n")
    with pytest.raises(ValueError):
        O.Vocabulary.load_text(p)


def test_complete_tree_matches_node_id_descent():
    """The breadth-first complete tree gives the same level-2 node ids as the closed-form
    descent oracle_feature_vector uses (the layout bench.py's vocabulary relies on)."""
    rng = np.random.default_rng(42)
    desc = rng.integers(0, 256, (1111, 32), dtype=np.uint8)
    voc = O.Vocabulary.from_nodes(10, 6, 0, 0, *complete_tree(10, 3, desc))
    f = rng.integers(0, 256, (500, 32), dtype=np.uint8)
    r = voc.transform(f, levelsup=4)
    assert np.array_equal(r["node_of"], O.feature_vector(desc, 10, 6, 4, f))
    # every leaf weight 1.0, TF-IDF + L1: each value = count / number of features
    counts = np.bincount(r["word_of"].astype(np.int64))
    assert np.allclose(r["bow_values"], counts[counts > 0] / len(f), rtol=0, atol=1e-15)
