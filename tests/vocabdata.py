"""Vocabulary fixtures shared by the CPU and GPU vocabulary tests.

`kat_tree()` is a hand-built k=2 tree whose transform results are worked out by hand in
tests/test_vocab_oracle.py; `random_tree()` builds irregular trees (uneven fan-out, leaves at
several depths, zero-weight "stopped" words); `write_text()` writes DBoW2's text format the
way TemplatedVocabulary::saveToTextFile does (TemplatedVocabulary.h:1428-1448).
"""
import numpy as np

Z = np.zeros(32, np.uint8)
F = np.full(32, 255, np.uint8)
HI = np.concatenate([np.full(16, 255, np.uint8), np.zeros(16, np.uint8)])
LO = np.concatenate([np.zeros(16, np.uint8), np.full(16, 255, np.uint8)])


def kat_tree():
    """k=2, L=2: nodes 1 (A=0..0) and 2 (B=1..1) under the root; 3,4 under 1; 5,6 under 2."""
    parent = np.array([0, 0, 1, 1, 2, 2], np.int32)
    is_leaf = np.array([0, 0, 1, 1, 1, 1], np.uint8)
    desc = np.stack([Z, F, Z, HI, F, LO])
    weight = np.array([0, 0, 0.5, 1.5, 0.0, 2.0])
    return parent, is_leaf, desc, weight


def kat_features():
    return np.stack([Z, F, HI, Z, LO])


def random_tree(seed, k=6, depth=4, p_stop=0.1, p_early_leaf=0.15, n_max=4000):
    """Irregular tree in breadth-first file order: every internal node gets 1..k children,
    a node becomes a leaf early with probability p_early_leaf, leaves get a random IDF-like
    weight or 0 (stopped) with probability p_stop."""
    rng = np.random.default_rng(seed)
    parent, level = [], []
    frontier = [(0, 0)]
    while frontier:
        nxt = []
        for node, lvl in frontier:
            if lvl == depth or (lvl > 0 and rng.random() < p_early_leaf) or len(parent) > n_max:
                continue
            for _ in range(int(rng.integers(1, k + 1))):
                parent.append(node)
                level.append(lvl + 1)
                nxt.append((len(parent), lvl + 1))
        frontier = nxt
    n = len(parent)
    parent = np.array(parent, np.int32)
    has_child = np.zeros(n + 1, bool)
    has_child[parent] = True
    is_leaf = (~has_child[1:]).astype(np.uint8)
    desc = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    weight = np.where(rng.random(n) < p_stop, 0.0, rng.uniform(0.01, 5.0, n))
    weight = np.where(is_leaf == 1, np.round(weight, 4), 0.0)
    return parent, is_leaf, desc, weight


def write_text(path, k, L, scoring, weighting, parent, is_leaf, desc, weight):
    with open(path, "w") as f:
        f.write(f"{k} {L}  {scoring} {weighting}\n")
        for p, lf, d, w in zip(parent, is_leaf, desc, weight):
            f.write(f"{int(p)} {int(lf)} " + "".join(f"{int(x)} " for x in d) + f" {w:g}\n")
