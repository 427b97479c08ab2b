"""The reference's threading contract on the drop-in path, checked against single-thread oracle
outputs.

* Stereo: Frame's stereo constructor extracts the left and right images on two std::threads,
  each with its own ORBextractor, joins them, then runs ComputeStereoMatches
  (ORB_SLAM2/src/Frame.cc:83-86, 100).
* ORBmatcher is stateless and called at the same time from the Tracking, LocalMapping and
  LoopClosing threads (ORB_SLAM2/src/System.cc:90-95): SearchByBoW(KF, F) (Tracking.cc:1135),
  SearchForTriangulation (LocalMapping.cc:240), SearchByBoW(KF, KF) (LoopClosing.cc:278), and
  Frame::ComputeBoW's vocabulary transform in Tracking.

ctypes releases the GIL inside every liborbx call, so Python threads run the C ABI
concurrently, as the reference's threads would: every result of every iteration must equal
the oracle's.
"""
import threading

import numpy as np
import pytest

from ar_orbslam2_amd import ORBextractor, ORBmatcher, Vocabulary, epipole, synth
from ar_orbslam2_amd.stereo import ComputeStereoMatches, stereo_params
from oracle import oracle as O

from matchdata import TUM1_K, fundamental, pair

pytestmark = pytest.mark.gpu

EUROC = stereo_params(47.90639384423901, 435.2046959714599)
ITERS = 200


def _run_threads(targets, timeout=300, barriers=()):
    errors = []

    def wrap(fn):
        def run():
            try:
                fn()
            except BaseException as e:  # noqa: BLE001 - reported below
                errors.append(repr(e))
                for b in barriers:  # release the partner thread at once
                    b.abort()
        return run

    ths = [threading.Thread(target=wrap(fn), daemon=True) for fn in targets]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout)
    assert not any(t.is_alive() for t in ths), "a thread did not finish"
    assert not errors, errors[:5]


@pytest.mark.timeout(600)
def test_stereo_extractors_and_matchers_concurrently():
    w, h, nf = 752, 480, 1200
    p = O.params(nf)
    pairs = [synth.stereo_pair(w, h, t, 6, (10 + 3 * t, 24)) for t in range(4)]
    tb = O.tables(p, w, h)
    ref_stereo = []
    for l, r in pairs:
        kl, dl, pl, _ = O.extract(l, p, want_pyramid=True)
        kr, dr, pr, _ = O.extract(r, p, want_pyramid=True)
        ur, dp, _ = O.stereo_matches(kl, dl, kr, dr, pl, pr, tb["scale"], tb["inv_scale"], *EUROC)
        ref_stereo.append((kl, dl, kr, dr, ur, dp))

    # matcher inputs (tests/matchdata.py) and their single-thread oracle results
    kf, f, vdesc = pair()
    F = fundamental()
    ex, ey = epipole(np.eye(3), [0.10, 0.02, 0.05], [0, 0, 0], *TUM1_K)
    side = lambda k, valid=True: dict(desc=k.mDescriptors, angle=k.mvKeysUn["angle"],  # noqa: E731
                                      valid=k.valid if valid else None, fv=k.mFeatVec)
    ref_kf_f = O.search_by_bow_kf_f(side(kf), side(f, False), 0.7, True)
    ref_kf_kf = O.search_by_bow_kf_kf(side(kf), side(f), 0.75, True)
    tri = lambda k: dict(desc=k.mDescriptors, keys=k.mvKeysUn, u_right=k.mvuRight,  # noqa: E731
                         has_mp=k.has_mp, fv=k.mFeatVec, scale_factors=k.mvScaleFactors,
                         level_sigma2=k.mvLevelSigma2)
    ref_tri = O.search_for_triangulation(tri(kf), tri(f), F, ex, ey, False, 0.6, False)
    assert ref_kf_f[0] > 20 and ref_kf_kf[0] > 10 and ref_tri[0] > 10

    # Frame::ComputeBoW on the full bench vocabulary
    n = sum(10 ** lv for lv in range(7))
    voc_desc = np.random.default_rng(42).integers(0, 256, (n, 32), dtype=np.uint8)
    from ar_orbslam2_amd.vocabulary import complete_tree
    arrays = complete_tree(10, 6, voc_desc)
    voc = Vocabulary.from_nodes(10, 6, 0, 0, *arrays)
    ovoc = O.Vocabulary.from_nodes(10, 6, 0, 0, *arrays)
    ref_bow = [ovoc.transform(ref_stereo[i][1], 4) for i in range(len(pairs))]

    exl, exr = ORBextractor(nf), ORBextractor(nf)
    join = threading.Barrier(2)     # threadLeft.join(); threadRight.join()
    stereo_done = threading.Barrier(2)
    results = {"stereo": 0, "kf_f": 0, "kf_kf": 0, "tri": 0, "bow": 0}

    def extract_side(exr_, side_idx):
        def run():
            for it in range(ITERS):
                i = it % len(pairs)
                k, d = exr_(pairs[i][side_idx])
                rk, rd = ref_stereo[i][2 * side_idx], ref_stereo[i][2 * side_idx + 1]
                assert np.array_equal(k, rk), ("keypoints", side_idx, it)
                assert np.array_equal(d, rd), ("descriptors", side_idx, it)
                join.wait(60)
                if side_idx == 0:  # the Frame constructor's thread, after the join
                    ur, dp = ComputeStereoMatches(exl, exr, *EUROC)
                    assert ur.tobytes() == ref_stereo[i][4].tobytes(), ("mvuRight", it)
                    assert dp.tobytes() == ref_stereo[i][5].tobytes(), ("mvDepth", it)
                    results["stereo"] += 1
                stereo_done.wait(60)
        return run

    fr = type("F", (), {})()
    fr.mDescriptors, fr.mvKeys, fr.mFeatVec = f.mDescriptors, f.mvKeys, f.mFeatVec
    f_kf = type("KF", (), {})()
    f_kf.mDescriptors, f_kf.mvKeysUn, f_kf.mFeatVec = f.mDescriptors, f.mvKeysUn, f.mFeatVec
    f_kf.valid, f_kf.is_keyframe = f.valid, True

    def tracking():  # SearchByBoW(KF, F)
        m = ORBmatcher(0.7, True)
        for it in range(ITERS):
            nm, match = m.SearchByBoW(kf, fr)
            assert nm == ref_kf_f[0] and np.array_equal(match, ref_kf_f[1]), ("kf_f", it)
            results["kf_f"] += 1

    def loop_closing():  # SearchByBoW(KF, KF)
        m = ORBmatcher(0.75, True)
        for it in range(ITERS):
            nm, match = m.SearchByBoW(kf, f_kf)
            assert nm == ref_kf_kf[0] and np.array_equal(match, ref_kf_kf[1]), ("kf_kf", it)
            results["kf_kf"] += 1

    def local_mapping():  # SearchForTriangulation
        m = ORBmatcher(0.6, False)
        for it in range(ITERS):
            nm, pr = m.SearchForTriangulation(kf, f, F, False, (ex, ey))
            assert nm == ref_tri[0] and np.array_equal(pr, ref_tri[1]), ("tri", it)
            results["tri"] += 1

    def compute_bow():  # Frame::ComputeBoW
        for it in range(ITERS):
            i = it % len(pairs)
            r = voc.transform_full(ref_stereo[i][1], 4)
            o = ref_bow[i]
            assert np.array_equal(r["word_of"], o["word_of"]), ("word_of", it)
            assert np.array_equal(r["node_of"], o["node_of"]), ("node_of", it)
            assert r["bow"].values.tobytes() == o["bow_values"].tobytes(), ("bow", it)
            results["bow"] += 1

    _run_threads([extract_side(exl, 0), extract_side(exr, 1), tracking, loop_closing,
                  local_mapping, compute_bow], barriers=(join, stereo_done))
    assert results == {"stereo": ITERS, "kf_f": ITERS, "kf_kf": ITERS, "tri": ITERS,
                       "bow": ITERS}, results


@pytest.mark.timeout(600)
def test_mono_extractors_on_many_threads():
    """Several cameras, one ORBextractor each, extracting concurrently (per-thread streams,
    graph captures and pinned staging under the process-wide resource lock)."""
    w, h, nf = 640, 480, 1000
    frames = [synth.frame(w, h, t, 9) for t in range(3)]
    refs = [O.extract(img, O.params(nf)) for img in frames]

    def cam(k):
        def run():
            ex = ORBextractor(nf)  # created inside the thread, as a Tracking thread would
            for it in range(60):
                i = (it + k) % len(frames)
                kp, d = ex(frames[i])
                assert np.array_equal(kp, refs[i][0]) and np.array_equal(d, refs[i][1]), (k, it)
        return run

    _run_threads([cam(k) for k in range(8)])
