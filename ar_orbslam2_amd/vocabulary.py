"""DBoW2 vocabulary node ids for the matchers (ORB_SLAM2/Thirdparty/DBoW2).

`FeatureVector` is DBoW2's std::map<NodeId, vector<unsigned>> (FeatureVector.h:21-52) in CSR
form.  `Vocabulary` holds a complete k-ary tree laid out breadth first (root id 0, then level 1
ids 1..k, ...), the layout orbx_feature_vector() descends on the GPU
(TemplatedVocabulary::transform, TemplatedVocabulary.h:1218-1259, levelsup=4 as
Frame::ComputeBoW uses, ORB_SLAM2/src/Frame.cc:400-407).  `Vocabulary.synthetic()` is the
seeded benchmark vocabulary of SURVEY §8d (k=10, L=6, seed 42, random 256-bit nodes); only the
levels the node-id descent visits are materialised.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from ._ffi import check, lib, ptr


@dataclass
class FeatureVector:
    node_ids: np.ndarray      # uint32 [n_nodes], ascending
    node_offsets: np.ndarray  # int32 [n_nodes + 1]
    node_feats: np.ndarray    # int32 [n], ascending inside each node

    @staticmethod
    def from_nodes(node_of_feature):
        """FeatureVector::addFeature over features in index order (FeatureVector.cpp:31-45)."""
        nodes = np.asarray(node_of_feature, np.uint32)
        order = np.argsort(nodes, kind="stable").astype(np.int32)
        ids, counts = np.unique(nodes, return_counts=True)
        offs = np.zeros(len(ids) + 1, np.int32)
        np.cumsum(counts, out=offs[1:])
        return FeatureVector(ids.astype(np.uint32), offs, order)

    def as_tuple(self):
        return self.node_ids, self.node_offsets, self.node_feats

    def __len__(self):
        return len(self.node_ids)


class Vocabulary:
    def __init__(self, k, L, node_desc, levelsup=4):
        self.k, self.L, self.levelsup = int(k), int(L), int(levelsup)
        self.node_desc = np.ascontiguousarray(node_desc, np.uint8)
        need = self.nodes_needed()
        if self.node_desc.shape[0] < need:
            raise ValueError(f"vocabulary needs {need} node descriptors for levelsup={levelsup}")

    def nodes_needed(self):
        lvl = max(self.L - self.levelsup, 0)
        return sum(self.k ** l for l in range(lvl + 1))

    @property
    def nid_level(self):
        return self.L - self.levelsup

    def first_node_id(self):
        """Smallest node id at level L - levelsup (the FeatureVector key range)."""
        return sum(self.k ** l for l in range(max(self.nid_level, 0))) if self.nid_level > 0 else 0

    @staticmethod
    def synthetic(k=10, L=6, seed=42, levelsup=4):
        rng = np.random.default_rng(seed)
        n = sum(k ** l for l in range(max(L - levelsup, 0) + 1))
        return Vocabulary(k, L, rng.integers(0, 256, (n, 32), dtype=np.uint8), levelsup)

    def node_ids(self, descriptors):
        d = np.ascontiguousarray(descriptors, np.uint8).reshape(-1, 32)
        out = np.zeros(d.shape[0], np.uint32)
        if d.shape[0]:
            check("orbx_feature_vector",
                  lib().orbx_feature_vector(ptr(self.node_desc), C.c_int32(self.k),
                                            C.c_int32(self.L), C.c_int32(self.levelsup), ptr(d),
                                            C.c_int32(d.shape[0]), ptr(out)))
        return out

    def transform(self, descriptors):
        """FeatureVector of a descriptor set (the `fv` output of transform)."""
        return FeatureVector.from_nodes(self.node_ids(descriptors))
