"""Shared synthetic matcher inputs: two consecutive frames of one stream,
extracted by the CPU oracle, FeatureVectors from the seeded synthetic vocabulary, seeded
map-point masks, and the F12 / epipole of a fixed pose (R = I, t = (0.10, 0.02, 0.05), TUM1 K).
Test infrastructure only."""
from __future__ import annotations

from types import SimpleNamespace

import numpy as np

from ar_orbslam2_amd import synth
from oracle import oracle as O

TUM1_K = (517.306408, 516.469215, 318.643040, 255.313989)


def vocab_desc(k=10, L=6, seed=42, levelsup=4):
    rng = np.random.default_rng(seed)
    n = sum(k ** l for l in range(max(L - levelsup, 0) + 1))
    return rng.integers(0, 256, (n, 32), dtype=np.uint8)


def featvec(nodes):
    nodes = np.asarray(nodes, np.uint32)
    order = np.argsort(nodes, kind="stable").astype(np.int32)
    ids, counts = np.unique(nodes, return_counts=True)
    offs = np.zeros(len(ids) + 1, np.int32)
    np.cumsum(counts, out=offs[1:])
    return ids.astype(np.uint32), offs, order


def fundamental(K=TUM1_K, t=(0.10, 0.02, 0.05)):
    fx, fy, cx, cy = K
    Km = np.array([[fx, 0, cx], [0, fy, cy], [0, 0, 1]], np.float32)
    tx = np.array([[0, -t[2], t[1]], [t[2], 0, -t[0]], [-t[1], t[0], 0]], np.float32)
    Kinv = np.linalg.inv(Km).astype(np.float32)
    return (Kinv.T @ tx @ Kinv).astype(np.float32)


def keyframe(img, p, voc, seed, mp_frac):
    kps, desc = O.extract(img, p)
    nodes = O.feature_vector(voc, 10, 6, 4, desc)
    t = O.tables(p, img.shape[1], img.shape[0])
    rng = np.random.default_rng(seed)
    n = len(kps)
    return SimpleNamespace(
        mDescriptors=desc, mvKeys=kps, mvKeysUn=kps, nodes=nodes, mFeatVec=featvec(nodes),
        valid=(rng.random(n) < 0.6).astype(np.uint8),
        has_mp=(rng.random(n) < mp_frac).astype(np.uint8),
        mvuRight=np.full(n, -1.0, np.float32), mvScaleFactors=t["scale"], mvLevelSigma2=t["sigma2"])


def pair(w=640, h=480, nfeat=1000, t=3, stream=0):
    p = O.params(nfeat)
    voc = vocab_desc()
    base = synth.canvas(w, h, stream)
    a = keyframe(synth.frame(w, h, t, stream, base), p, voc, t, 0.4)
    b = keyframe(synth.frame(w, h, t + 1, stream, base), p, voc, t + 1, 0.4)
    return a, b, voc
