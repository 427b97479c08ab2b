"""Regenerate the committed golden vectors with the CPU oracle (test infrastructure).

For each committed gray fixture (tests/golden/*.pgm, see make_fixtures.py) at the TUM1 ORB
configuration (1000 features, 1.2, 8 levels, FAST 20/7): keypoints (cv::KeyPoint layout, .npy)
and descriptors.  For the matchers: the `tmp` frame and the same frame rolled by (1, 1) px,
node ids from the seeded synthetic vocabulary (vocab_k10_L6_s42.npy), deterministic map-point
masks, and the SearchByBoW / SearchForTriangulation outputs.  The reference has no golden
vectors of its own: these pin the GPU path and the oracle against regressions;
they do not pin the oracle against OpenCV 2.4, which is unavailable.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from ar_orbslam2_amd import synth  # noqa: E402
from oracle import oracle as O  # noqa: E402

FIXTURES = ["tmp", "book1", "target"]
F_SHIFT = np.array([[0, 0, -1], [0, 0, 1], [1, -1, 0]], np.float32)


def featvec(nodes):
    order = np.argsort(nodes, kind="stable").astype(np.int32)
    ids, counts = np.unique(nodes, return_counts=True)
    offs = np.zeros(len(ids) + 1, np.int32)
    np.cumsum(counts, out=offs[1:])
    return ids.astype(np.uint32), offs, order


def match_inputs():
    img = synth.read_pgm(os.path.join(HERE, "tmp.pgm"))
    voc = np.load(os.path.join(HERE, "vocab_k10_L6_s42.npy"))
    p = O.params(1000)
    t = O.tables(p, img.shape[1], img.shape[0])
    sides = []
    for im in (img, np.roll(img, (1, 1), axis=(0, 1))):
        kps, desc = O.extract(im, p)
        nodes = O.feature_vector(voc, 10, 6, 4, desc)
        i = np.arange(len(kps))
        sides.append(dict(desc=desc, angle=kps["angle"], keys=kps, nodes=nodes, fv=featvec(nodes),
                          valid=(i % 5 != 0).astype(np.uint8), has_mp=(i % 3 == 0).astype(np.uint8),
                          u_right=None, scale_factors=t["scale"], level_sigma2=t["sigma2"]))
    return sides, voc


if __name__ == "__main__":
    rng = np.random.default_rng(42)
    np.save(os.path.join(HERE, "vocab_k10_L6_s42.npy"), rng.integers(0, 256, (111, 32), dtype=np.uint8))
    for name in FIXTURES:
        img = synth.read_pgm(os.path.join(HERE, name + ".pgm"))
        kps, desc = O.extract(img, O.params(1000))
        np.save(os.path.join(HERE, f"{name}_kps.npy"), kps)
        np.save(os.path.join(HERE, f"{name}_desc.npy"), desc)
        print(name, len(kps))
    (a, b), voc = match_inputs()
    np.save(os.path.join(HERE, "match_nodes_a.npy"), a["nodes"])
    np.save(os.path.join(HERE, "match_nodes_b.npy"), b["nodes"])
    n1, m1 = O.search_by_bow_kf_f(a, dict(b, valid=None), 0.7, True)
    n2, m2 = O.search_by_bow_kf_kf(a, b, 0.75, True)
    n3, p3 = O.search_for_triangulation(a, b, F_SHIFT, 1e6, 1e6, False, 0.6, False)
    np.save(os.path.join(HERE, "match_bow_kf_f.npy"), m1)
    np.save(os.path.join(HERE, "match_bow_kf_kf.npy"), m2)
    np.save(os.path.join(HERE, "match_tri_pairs.npy"), p3)
    print("bow kf-f", n1, "bow kf-kf", n2, "tri", n3)
