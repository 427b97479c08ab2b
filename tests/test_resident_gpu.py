"""GPU: the frame cache behind the per-frame drop-in calls (orbx_match.h, "resident frames").

orbx_vocabulary_transform, orbx_search_by_bow_kf_* and orbx_search_for_triangulation keep a
frame's descriptors, FeatureVector and keypoints in HBM between calls, found again by content.
Every result must equal the oracle's whichever way a side got there: found resident, uploaded
on first sight, found with another FeatureVector or other keypoints than the entry holds, or
evicted by more frames than the cache holds and uploaded again.  The reference's call chain is
Frame::ComputeBoW -> SearchByBoW(reference KF, F) -> SearchForTriangulation
(ORB_SLAM2/src/Tracking.cc:1127-1136, LocalMapping.cc:238-241)."""
from types import SimpleNamespace

import numpy as np
import pytest

from ar_orbslam2_amd import ORBmatcher, Vocabulary, synth
from oracle import oracle as O

from matchdata import featvec, vocab_desc

pytestmark = pytest.mark.gpu

SHIFT_F = np.array([[0, 0, -1], [0, 0, 1], [1, -1, 0]], np.float32)
N_ENTRIES = 16  # kResEntries


def _chain():
    p = O.params(1000)
    voc = vocab_desc()
    v = Vocabulary.complete(10, 6, voc)
    base = synth.canvas(640, 480, 0)
    t = O.tables(p, 640, 480)
    frames = []
    for i in range(N_ENTRIES + 10):
        kps, desc = O.extract(synth.frame(640, 480, i, 0, base), p)
        rng = np.random.default_rng(100 + i)
        n = len(kps)
        frames.append(SimpleNamespace(
            mDescriptors=desc, mvKeys=kps, mvKeysUn=kps, nodes=O.feature_vector(voc, 10, 6, 4, desc),
            valid=(rng.random(n) < 0.6).astype(np.uint8), has_mp=(rng.random(n) < 0.4).astype(np.uint8),
            mvuRight=np.full(n, -1.0, np.float32), mvScaleFactors=t["scale"], mvLevelSigma2=t["sigma2"]))
    return frames, v


@pytest.fixture(scope="module")
def chain():
    return _chain()


def _bow_side(kf, valid=True):
    return dict(desc=kf.mDescriptors, angle=kf.mvKeysUn["angle"], valid=kf.valid if valid else None,
                fv=kf.mFeatVec)


def _tri_side(k):
    return dict(desc=k.mDescriptors, keys=k.mvKeysUn, u_right=k.mvuRight, has_mp=k.has_mp,
                fv=k.mFeatVec, scale_factors=k.mvScaleFactors, level_sigma2=k.mvLevelSigma2)


def _bow(kf, f):
    n_ref, m_ref = O.search_by_bow_kf_f(_bow_side(kf), _bow_side(f, False), 0.7, True)
    fr = SimpleNamespace(mDescriptors=f.mDescriptors.copy(), mvKeys=f.mvKeys, mFeatVec=f.mFeatVec)
    n, m = ORBmatcher(0.7, True).SearchByBoW(kf, fr)  # a fresh host buffer: found by content
    assert n == n_ref and np.array_equal(m, m_ref)
    return n


def _tri(k1, k2, F=SHIFT_F, e=(1e6, 1e6)):
    n_ref, p_ref = O.search_for_triangulation(_tri_side(k1), _tri_side(k2), F, e[0], e[1], False,
                                              0.6, False)
    n, p = ORBmatcher(0.6, False).SearchForTriangulation(k1, k2, F, False, e)
    assert n == n_ref and np.array_equal(p, p_ref)
    return n


def test_chain_with_reference_keyframes_and_evictions(chain):
    """ComputeBoW (GPU transform, FeatureVector checked against the oracle's), SearchByBoW with a
    reference keyframe kept for six frames and, from frame 18 on, one more than the cache holds
    frames back (evicted, uploaded again), SearchForTriangulation with the previous frame."""
    frames, v = chain
    total = 0
    for i, f in enumerate(frames):
        _, fv = v.transform(f.mDescriptors)
        ref = featvec(f.nodes)
        for x, y in zip(fv.as_tuple(), ref):
            assert np.array_equal(x, y)
        f.mFeatVec = fv.as_tuple()
        if i == 0:
            continue
        total += _bow(frames[(i // 6) * 6 if i % 6 else i - 6], f)
        total += _tri(frames[i - 1], f)
        if i >= N_ENTRIES + 2:
            total += _bow(frames[i - N_ENTRIES - 2], f)
    assert total > 1000


def test_same_call_twice_and_content_changed_in_place(chain):
    frames, v = chain
    for f in frames[:3]:
        if not hasattr(f, "mFeatVec"):
            f.mFeatVec = v.transform(f.mDescriptors)[1].as_tuple()
    a, b = frames[1], frames[2]
    n1 = _bow(a, b)
    assert _bow(a, b) == n1
    # the same host buffers, other bytes: a different frame for the cache
    saved = b.mDescriptors.copy()
    b.mDescriptors[::7, 3] ^= 0x5A
    try:
        _bow(a, b)
        _tri(a, b)
    finally:
        b.mDescriptors[:] = saved
    _bow(a, b)


def test_other_featurevector_and_keypoints_for_resident_descriptors(chain):
    frames, v = chain
    for f in frames[:4]:
        if not hasattr(f, "mFeatVec"):
            f.mFeatVec = v.transform(f.mDescriptors)[1].as_tuple()
    a, b = frames[2], frames[3]
    _bow(a, b)
    _tri(a, b)
    # the keyframe's descriptors with another FeatureVector (levelsup 5): re-uploaded
    a2 = SimpleNamespace(**vars(a))
    a2.mFeatVec = v.transform(a.mDescriptors, levelsup=5)[1].as_tuple()
    b2 = SimpleNamespace(**vars(b))
    b2.mFeatVec = v.transform(b.mDescriptors, levelsup=5)[1].as_tuple()
    _bow(a2, b2)
    # other keypoints (undistorted elsewhere) for resident descriptors
    k = a.mvKeysUn.copy()
    k["x"] += np.float32(0.75)
    a3 = SimpleNamespace(**vars(a))
    a3.mvKeysUn = k
    _tri(a3, b)
    _tri(a, b)  # and back


def test_kf_kf_and_stereo_on_resident_frames(chain):
    frames, v = chain
    for f in frames[:6]:
        if not hasattr(f, "mFeatVec"):
            f.mFeatVec = v.transform(f.mDescriptors)[1].as_tuple()
    k1, k2 = frames[4], frames[5]
    n_ref, m_ref = O.search_by_bow_kf_kf(_bow_side(k1), _bow_side(k2), 0.75, True)
    k2b = SimpleNamespace(**vars(k2))
    k2b.is_keyframe = True
    n, m = ORBmatcher(0.75, True).SearchByBoW(k1, k2b)
    assert n == n_ref and np.array_equal(m, m_ref)
    rng = np.random.default_rng(3)
    s1, s2 = SimpleNamespace(**vars(k1)), SimpleNamespace(**vars(k2))
    s1.mvuRight = np.where(rng.random(len(k1.mvKeys)) < 0.5, 100.0, -1.0).astype(np.float32)
    s2.mvuRight = np.where(rng.random(len(k2.mvKeys)) < 0.5, 100.0, -1.0).astype(np.float32)
    n_ref, p_ref = O.search_for_triangulation(_tri_side(s1), _tri_side(s2), SHIFT_F, 320.0, 240.0,
                                              True, 0.6, False)
    n, p = ORBmatcher(0.6, False).SearchForTriangulation(s1, s2, SHIFT_F, True, (320.0, 240.0))
    assert n == n_ref and np.array_equal(p, p_ref) and n > 10


def test_threads_share_keyframes(chain):
    """Several host threads (Tracking, LocalMapping) matching against the same resident
    keyframes at once: every result equals the oracle's."""
    import threading
    frames, v = chain
    for f in frames[:8]:
        if not hasattr(f, "mFeatVec"):
            f.mFeatVec = v.transform(f.mDescriptors)[1].as_tuple()
    errs = []

    def work(j):
        try:
            for r in range(6):
                kf, f = frames[(j + r) % 3], frames[3 + (j + 2 * r) % 5]
                _bow(kf, f)
                _tri(kf, f)
        except Exception as e:  # noqa: BLE001 - reported below
            errs.append(e)
    ts = [threading.Thread(target=work, args=(j,)) for j in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs, errs[0]
