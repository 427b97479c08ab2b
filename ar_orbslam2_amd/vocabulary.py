"""DBoW2 vocabulary (ORB_SLAM2/Thirdparty/DBoW2) on the GPU.

`Vocabulary` mirrors TemplatedVocabulary<FORB::TDescriptor, FORB> (ORBVocabulary,
ORB_SLAM2/include/ORBVocabulary.h): `load_text` is loadFromTextFile
(TemplatedVocabulary.h:1338-1424) and `transform(desc, levelsup)` is
transform(features, BowVector&, FeatureVector&, levelsup) (:1127-1198) as
Frame::ComputeBoW calls it (ORB_SLAM2/src/Frame.cc:400-407, levelsup = 4).  The tree lives
in HBM (orbx_vocabulary_*, include/orbx.h).  `FeatureVector` is DBoW2's
std::map<NodeId, vector<unsigned>> (FeatureVector.h:21-52) in CSR form, `BowVector` its
std::map<WordId, WordValue> (BowVector.h:55-62) as two arrays in word-id order.

`Vocabulary.synthetic()` is the seeded benchmark vocabulary of SURVEY §8d: a complete
k = 10, L = 6 tree in breadth-first file order, random 256-bit node descriptors (seed 42),
every leaf weight 1.0, L1 scoring, TF-IDF weighting.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from ._ffi import check, lib, ptr

TF_IDF, TF, IDF, BINARY = 0, 1, 2, 3
L1_NORM, L2_NORM, CHI_SQUARE, KL, BHATTACHARYYA, DOT_PRODUCT = 0, 1, 2, 3, 4, 5
STOPPED = 0xFFFFFFFF


@dataclass
class FeatureVector:
    node_ids: np.ndarray      # uint32 [n_nodes], ascending
    node_offsets: np.ndarray  # int32 [n_nodes + 1]
    node_feats: np.ndarray    # int32 [n], ascending inside each node

    @staticmethod
    def from_nodes(node_of_feature):
        """FeatureVector::addFeature over features in index order (FeatureVector.cpp:31-45);
        features whose node is STOPPED are not added."""
        nodes = np.asarray(node_of_feature, np.uint32)
        keep = np.nonzero(nodes != STOPPED)[0].astype(np.int32)
        order = keep[np.argsort(nodes[keep], kind="stable")]
        ids, counts = np.unique(nodes[keep], return_counts=True)
        offs = np.zeros(len(ids) + 1, np.int32)
        np.cumsum(counts, out=offs[1:])
        return FeatureVector(ids.astype(np.uint32), offs, order.astype(np.int32))

    def as_tuple(self):
        return self.node_ids, self.node_offsets, self.node_feats

    def __len__(self):
        return len(self.node_ids)


@dataclass
class BowVector:
    word_ids: np.ndarray  # uint32, ascending
    values: np.ndarray    # float64

    def __len__(self):
        return len(self.word_ids)


def complete_tree(k, depth, node_desc, leaf_weight=1.0):
    """Breadth-first arrays (parent, is_leaf, desc, weight) of a complete k-ary tree of the
    given depth, nodes 1..n in DBoW2 file order (what saveToTextFile writes for it)."""
    node_desc = np.ascontiguousarray(node_desc, np.uint8).reshape(-1, 32)
    sizes = [k ** l for l in range(depth + 1)]
    n = sum(sizes) - 1
    if node_desc.shape[0] < n + 1:
        raise ValueError(f"complete k={k} depth={depth} tree needs {n + 1} node descriptors")
    parent = np.empty(n, np.int32)
    first = 1
    for l in range(1, depth + 1):
        ids = np.arange(first, first + sizes[l])
        prev_first = first - sizes[l - 1]
        parent[ids - 1] = prev_first + (ids - first) // k
        first += sizes[l]
    is_leaf = np.zeros(n, np.uint8)
    is_leaf[n - sizes[depth]:] = 1
    weight = np.where(is_leaf == 1, leaf_weight, 0.0).astype(np.float64)
    return parent, is_leaf, node_desc[1:n + 1], weight


class Vocabulary:
    """TemplatedVocabulary<FORB::TDescriptor, FORB>, resident on one GPU."""

    def __init__(self, handle, device=0):
        self._h = handle
        self.device = device
        k, L, sc, wt, nn, nw = (C.c_int32() for _ in range(6))
        check("orbx_vocabulary_info",
              lib().orbx_vocabulary_info(self._h, C.byref(k), C.byref(L), C.byref(sc),
                                         C.byref(wt), C.byref(nn), C.byref(nw)))
        self.k, self.L, self.scoring, self.weighting = k.value, L.value, sc.value, wt.value
        self.n_nodes, self.n_words = nn.value, nw.value

    # -------------------------------------------------------------- construction
    @classmethod
    def from_nodes(cls, k, L, scoring, weighting, parent, is_leaf, desc, weight, device=0):
        parent = np.ascontiguousarray(parent, np.int32)
        is_leaf = np.ascontiguousarray(is_leaf, np.uint8)
        desc = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        weight = np.ascontiguousarray(weight, np.float64)
        h = C.c_void_p()
        check("orbx_vocabulary_create",
              lib().orbx_vocabulary_create(C.c_int32(k), C.c_int32(L), C.c_int32(scoring),
                                           C.c_int32(weighting), C.c_int32(len(parent)),
                                           ptr(parent), ptr(is_leaf), ptr(desc), ptr(weight),
                                           C.c_int32(device), C.byref(h)))
        return cls(h, device)

    @classmethod
    def load_text(cls, path, device=0):
        """TemplatedVocabulary::loadFromTextFile (e.g. Vocabulary/ORBvoc.txt)."""
        h = C.c_void_p()
        check("orbx_vocabulary_load_text",
              lib().orbx_vocabulary_load_text(str(path).encode(), C.c_int32(device),
                                              C.byref(h)))
        return cls(h, device)

    @classmethod
    def complete(cls, k, L, node_desc, depth=None, scoring=L1_NORM, weighting=TF_IDF,
                 leaf_weight=1.0, device=0):
        """Complete k-ary tree from breadth-first node descriptors (row 0 = root, unused).
        `depth` defaults to the deepest level the descriptors fill; L is the declared m_L."""
        node_desc = np.ascontiguousarray(node_desc, np.uint8).reshape(-1, 32)
        if depth is None:
            depth, total = 0, 1
            while total + k ** (depth + 1) <= node_desc.shape[0]:
                depth += 1
                total += k ** depth
        parent, is_leaf, desc, weight = complete_tree(k, depth, node_desc, leaf_weight)
        return cls.from_nodes(k, L, scoring, weighting, parent, is_leaf, desc, weight, device)

    @classmethod
    def synthetic(cls, k=10, L=6, seed=42, device=0):
        n = sum(k ** l for l in range(L + 1))
        desc = np.random.default_rng(seed).integers(0, 256, (n, 32), dtype=np.uint8)
        return cls.complete(k, L, desc, depth=L, device=device)

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            lib().orbx_vocabulary_destroy(self._h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    # -------------------------------------------------------------- transform
    def transform_full(self, descriptors, levelsup=4):
        """All outputs of transform: dict(word_of, node_of, bow, fv)."""
        d = np.ascontiguousarray(descriptors, np.uint8).reshape(-1, 32)
        n = d.shape[0]
        m = max(n, 1)
        word_of = np.zeros(m, np.uint32)
        node_of = np.zeros(m, np.uint32)
        bw = np.zeros(m, np.uint32)
        bv = np.zeros(m, np.float64)
        fi = np.zeros(m + 1, np.uint32)
        fo = np.zeros(m + 2, np.int32)
        ff = np.zeros(m, np.int32)
        bn, fn = C.c_int32(), C.c_int32()
        check("orbx_vocabulary_transform",
              lib().orbx_vocabulary_transform(self._h, ptr(d), C.c_int32(n), C.c_int32(levelsup),
                                              ptr(word_of), ptr(node_of), ptr(bw), ptr(bv),
                                              C.byref(bn), ptr(fi), ptr(fo), ptr(ff),
                                              C.byref(fn)))
        nf = fn.value
        fv = FeatureVector(fi[:nf].copy(), fo[:nf + 1].copy(), ff[:fo[nf]].copy())
        return dict(word_of=word_of[:n], node_of=node_of[:n],
                    bow=BowVector(bw[:bn.value].copy(), bv[:bn.value].copy()), fv=fv)

    def transform(self, descriptors, levelsup=4):
        """(BowVector, FeatureVector) — Frame::ComputeBoW's mBowVec, mFeatVec."""
        r = self.transform_full(descriptors, levelsup)
        return r["bow"], r["fv"]

    def node_ids(self, descriptors, levelsup=4):
        """FeatureVector node id of every feature (STOPPED for zero-weight words)."""
        return self.transform_full(descriptors, levelsup)["node_of"]

    def word_ids(self, descriptors):
        return self.transform_full(descriptors)["word_of"]
