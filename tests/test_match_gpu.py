"""GPU parity of ORBmatcher (SearchByBoW x2, SearchForTriangulation, DescriptorDistance) and
the vocabulary node ids against the CPU oracle — identical match arrays and counts."""
import numpy as np
import pytest

from ar_orbslam2_amd import FeatureVector, ORBmatcher, Vocabulary, epipole
from oracle import oracle as O

from matchdata import TUM1_K, fundamental, pair, vocab_desc

pytestmark = pytest.mark.gpu

SHIFT_F = np.array([[0, 0, -1], [0, 0, 1], [1, -1, 0]], np.float32)


@pytest.fixture(scope="module")
def frames():
    return pair()


def _oracle_bow_side(kf, valid=True):
    return dict(desc=kf.mDescriptors, angle=kf.mvKeysUn["angle"],
                valid=kf.valid if valid else None, fv=kf.mFeatVec)


def test_vocabulary_node_ids(frames):
    a, b, voc = frames
    v = Vocabulary.complete(10, 6, voc)  # the 111-node tree: levels 0..2
    for kf in (a, b):
        got = v.node_ids(kf.mDescriptors)
        assert np.array_equal(got, kf.nodes)
        _, fv = v.transform(kf.mDescriptors)
        for x, y in zip(fv.as_tuple(), kf.mFeatVec):
            assert np.array_equal(x, y)


def test_descriptor_distance(frames):
    a, b, _ = frames
    n = min(len(a.mDescriptors), len(b.mDescriptors))
    got = ORBmatcher.DescriptorDistance(a.mDescriptors[:n], b.mDescriptors[:n])
    ref = [O.descriptor_distance(a.mDescriptors[i], b.mDescriptors[i]) for i in range(n)]
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("ratio,ori", [(0.7, True), (0.75, True), (0.9, False), (0.6, True)])
def test_search_by_bow_kf_frame(frames, ratio, ori):
    kf, f, _ = frames
    n_ref, m_ref = O.search_by_bow_kf_f(_oracle_bow_side(kf), _oracle_bow_side(f, False), ratio,
                                        ori)
    fr = type("F", (), {})()
    fr.mDescriptors, fr.mvKeys, fr.mFeatVec = f.mDescriptors, f.mvKeys, f.mFeatVec
    n, m = ORBmatcher(ratio, ori).SearchByBoW(kf, fr)
    assert n == n_ref and n > 20
    assert np.array_equal(m, m_ref)


@pytest.mark.parametrize("ratio,ori", [(0.75, True), (0.9, False)])
def test_search_by_bow_kf_kf(frames, ratio, ori):
    k1, k2, _ = frames
    k2.is_keyframe = True
    n_ref, m_ref = O.search_by_bow_kf_kf(_oracle_bow_side(k1), _oracle_bow_side(k2), ratio, ori)
    n, m = ORBmatcher(ratio, ori).SearchByBoW(k1, k2)
    assert n == n_ref and n > 10
    assert np.array_equal(m, m_ref)


def _tri(k1, k2, F, ex, ey, only_stereo, ori):
    d = lambda k: dict(desc=k.mDescriptors, keys=k.mvKeysUn, u_right=k.mvuRight, has_mp=k.has_mp,
                       fv=k.mFeatVec, scale_factors=k.mvScaleFactors, level_sigma2=k.mvLevelSigma2)
    n_ref, p_ref = O.search_for_triangulation(d(k1), d(k2), F, ex, ey, only_stereo, 0.6, ori)
    n, p = ORBmatcher(0.6, ori).SearchForTriangulation(k1, k2, F, only_stereo, (ex, ey))
    assert n == n_ref
    assert np.array_equal(p, p_ref)
    return n


def test_triangulation_realistic_pose(frames):
    k1, k2, _ = frames
    fx, fy, cx, cy = TUM1_K
    ex, ey = epipole(np.eye(3), [0.10, 0.02, 0.05], [0, 0, 0], fx, fy, cx, cy)
    assert (ex, ey) == O.epipole(np.eye(3), [0.10, 0.02, 0.05], [0, 0, 0], fx, fy, cx, cy)
    _tri(k1, k2, fundamental(), ex, ey, False, False)


def test_triangulation_permissive_geometry(frames):
    # consecutive synthetic frames differ by a (-1,-1) pixel shift: F = [(dx,dy,0)]x makes the
    # epipolar line of each point pass through its true match, so many candidates survive and
    # the distance / last-wins rules are exercised; an epipole inside the image exercises the
    # epipole rejection
    k1, k2, _ = frames
    F = SHIFT_F
    n = _tri(k1, k2, F, 1e6, 1e6, False, False)
    assert n > 50
    n2 = _tri(k1, k2, F, 1e6, 1e6, False, True)
    assert n2 <= n
    n3 = _tri(k1, k2, F, 320.0, 240.0, False, False)
    assert n3 <= n


def test_triangulation_stereo(frames):
    k1, k2, _ = frames
    rng = np.random.default_rng(9)
    k1.mvuRight = np.where(rng.random(len(k1.mvKeys)) < 0.5, 100.0, -1.0).astype(np.float32)
    k2.mvuRight = np.where(rng.random(len(k2.mvKeys)) < 0.5, 100.0, -1.0).astype(np.float32)
    assert _tri(k1, k2, SHIFT_F, 320.0, 240.0, True, False) > 10
    _tri(k1, k2, SHIFT_F, 320.0, 240.0, False, False)


def test_empty_sides():
    m = ORBmatcher(0.7, True)
    e = type("E", (), {})()
    e.mDescriptors = np.zeros((0, 32), np.uint8)
    e.mvKeys = e.mvKeysUn = np.zeros(0, O.KEYPOINT_DTYPE)
    e.mFeatVec = FeatureVector.from_nodes(np.zeros(0, np.uint32))
    n, match = m.SearchByBoW(e, e)
    assert n == 0 and match.shape == (0,)


def test_committed_match_goldens(golden_dir):
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location(
        "make_goldens", os.path.join(golden_dir, "make_goldens.py"))
    MG = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(MG)
    (a, b), voc = MG.match_inputs()
    v = Vocabulary.complete(10, 6, voc)
    assert np.array_equal(v.node_ids(a["desc"]), np.load(os.path.join(golden_dir, "match_nodes_a.npy")))

    def ns(d, keyframe):
        s = type("S", (), {})()
        s.mDescriptors, s.mvKeys, s.mvKeysUn = d["desc"], d["keys"], d["keys"]
        s.mFeatVec, s.valid, s.has_mp = d["fv"], d["valid"], d["has_mp"]
        s.mvScaleFactors, s.mvLevelSigma2, s.mvuRight = d["scale_factors"], d["level_sigma2"], None
        s.is_keyframe = keyframe
        return s
    _, m1 = ORBmatcher(0.7, True).SearchByBoW(ns(a, True), ns(dict(b, valid=None), False))
    assert np.array_equal(m1, np.load(os.path.join(golden_dir, "match_bow_kf_f.npy")))
    _, m2 = ORBmatcher(0.75, True).SearchByBoW(ns(a, True), ns(b, True))
    assert np.array_equal(m2, np.load(os.path.join(golden_dir, "match_bow_kf_kf.npy")))
    _, p3 = ORBmatcher(0.6, False).SearchForTriangulation(ns(a, True), ns(b, True), MG.F_SHIFT,
                                                          False, (1e6, 1e6))
    assert np.array_equal(p3, np.load(os.path.join(golden_dir, "match_tri_pairs.npy")))


def _big_node_sides(n, seed):
    """n keyframe and n frame features in ONE vocabulary node (a dense, repetitive scene): frame
    descriptors are permuted keyframe descriptors with 0-8 flipped bits (70 %) or random."""
    rng = np.random.default_rng(seed)
    d1 = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    perm = rng.permutation(n)
    d2 = d1[perm].copy()
    bits = np.unpackbits(d2, axis=1)
    for i in range(n):
        k = rng.integers(0, 9)
        bits[i, rng.choice(256, k, replace=False)] ^= 1
    d2 = np.packbits(bits, axis=1)
    rand = rng.random(n) >= 0.7
    d2[rand] = rng.integers(0, 256, (int(rand.sum()), 32), dtype=np.uint8)

    def side(d, valid):
        s = type("S", (), {})()
        s.mDescriptors = d
        s.mvKeys = s.mvKeysUn = np.zeros(n, O.KEYPOINT_DTYPE)
        s.mvKeys["angle"] = rng.random(n).astype(np.float32) * 360
        s.mFeatVec = (np.array([5], np.uint32), np.array([0, n], np.int32),
                      np.arange(n, dtype=np.int32))
        s.valid = valid
        return s
    return side(d1, (rng.random(n) < 0.6).astype(np.uint8)), side(d2, (rng.random(n) < 0.8).astype(np.uint8))


@pytest.mark.parametrize("n", [1500, 5000])  # above the round-1 1024 limit; above the register bitmap
def test_search_by_bow_single_huge_node(n):
    """SearchByBoW has no node-size limit in the reference (ORBmatcher.cc:187-250, 557-622): a
    node with thousands of candidates must give the oracle's matches (vbMatched2 semantics)."""
    kf, f = _big_node_sides(n, n)
    for ratio, ori in ((0.7, True), (0.9, False)):
        n_ref, m_ref = O.search_by_bow_kf_f(_oracle_bow_side(kf), _oracle_bow_side(f, False),
                                            ratio, ori)
        fr = type("F", (), {})()
        fr.mDescriptors, fr.mvKeys, fr.mFeatVec = f.mDescriptors, f.mvKeys, f.mFeatVec
        got_n, got = ORBmatcher(ratio, ori).SearchByBoW(kf, fr)
        assert got_n == n_ref and n_ref > 50
        assert np.array_equal(got, m_ref)
        f.is_keyframe = True
        n_ref, m_ref = O.search_by_bow_kf_kf(_oracle_bow_side(kf), _oracle_bow_side(f), ratio, ori)
        got_n, got = ORBmatcher(ratio, ori).SearchByBoW(kf, f)
        del f.is_keyframe
        assert got_n == n_ref and n_ref > 50
        assert np.array_equal(got, m_ref)


def _contested_sides(n1, n2, palette, seed, chain=False):
    """n1 keyframe and n2 frame features in one vocabulary node, all descriptors a few bits away
    from one of `palette` base descriptors: many keyframe features want the same candidates,
    distances tie, and late features find their best candidates already matched."""
    rng = np.random.default_rng(seed)
    base = rng.integers(0, 256, (palette, 32), dtype=np.uint8)

    def draw(which, flips):
        bits = np.unpackbits(base[which], axis=1)
        for i in range(len(which)):
            bits[i, rng.choice(256, flips(i), replace=False)] ^= 1
        return np.packbits(bits, axis=1)

    def side(d, valid):
        n = len(d)
        s = type("S", (), {})()
        s.mDescriptors = d
        s.mvKeys = s.mvKeysUn = np.zeros(n, O.KEYPOINT_DTYPE)
        s.mvKeys["angle"] = rng.random(n).astype(np.float32) * 360
        s.mFeatVec = (np.array([5], np.uint32), np.array([0, n], np.int32),
                      np.arange(n, dtype=np.int32))
        s.valid = valid
        return s
    # frame: n2 / palette copies of every base, 0-8 bits off; keyframe: bases 0-3 bits off.
    # chain: copy c of a base is exactly c bits off and the keyframe features are the bases, so
    # successive keyframe features of a base claim its copies one after the other (past the
    # workgroup form's 8-key lists)
    if chain:
        return (side(draw(rng.integers(0, palette, n1), lambda i: 0), np.ones(n1, np.uint8)),
                side(draw(np.arange(n2) % palette, lambda i: i // palette), np.ones(n2, np.uint8)))
    return (side(draw(rng.integers(0, palette, n1), lambda i: rng.integers(0, 4)),
                 (rng.random(n1) < 0.8).astype(np.uint8)),
            side(draw(np.arange(n2) % palette, lambda i: rng.integers(0, 9)),
                 (rng.random(n2) < 0.8).astype(np.uint8)))


@pytest.mark.parametrize("n1,n2,palette,chain", [
    (100, 128, 8, False), (200, 60, 4, False), (64, 128, 128, False), (130, 100, 16, False),
    (90, 7, 2, False), (10, 128, 1, False), (40, 40, 2, True), (100, 128, 4, True),
    (70, 120, 1, True)])
def test_search_by_bow_contested_nodes(n1, n2, palette, chain):
    """Nodes of at most 128 candidates (the one-problem calls' workgroup form): more keyframe
    features than a wave, tied distances and best candidates claimed by earlier features — the
    greedy order of ORBmatcher.cc:187-250 / 557-622 must come out exactly."""
    kf, f = _contested_sides(n1, n2, palette, 1000 * n1 + n2, chain)
    for ratio, ori in ((0.7, True), (0.9, False), (1.0, False)):
        n_ref, m_ref = O.search_by_bow_kf_f(_oracle_bow_side(kf), _oracle_bow_side(f, False),
                                            ratio, ori)
        fr = type("F", (), {})()
        fr.mDescriptors, fr.mvKeys, fr.mFeatVec = f.mDescriptors, f.mvKeys, f.mFeatVec
        got_n, got = ORBmatcher(ratio, ori).SearchByBoW(kf, fr)
        assert got_n == n_ref
        assert np.array_equal(got, m_ref)
        f.is_keyframe = True
        n_ref2, m_ref = O.search_by_bow_kf_kf(_oracle_bow_side(kf), _oracle_bow_side(f), ratio, ori)
        got_n, got = ORBmatcher(ratio, ori).SearchByBoW(kf, f)
        del f.is_keyframe
        assert got_n == n_ref2
        assert np.array_equal(got, m_ref)
        if ratio == 1.0 and palette <= 16:
            assert n_ref > (8 if chain else 0)


@pytest.mark.parametrize("kind", [0, 1, 2])
def test_finish_kernels_reject_stale_indices(kind):
    """A match array holding indices outside the other side (what a stale buffer would hold)
    makes the finish kernels report ORBX_EDEVICE and drop those entries, never dereference
    them (the round-1 C5 fault was an out-of-bounds read through such an index)."""
    import ctypes as C
    from ar_orbslam2_amd._ffi import lib, ptr
    n1, n2 = 300, 200
    n = n2 if kind == 0 else n1
    other = n1 if kind == 0 else n2
    rng = np.random.default_rng(kind)
    match = np.where(rng.random(n) < 0.5, rng.integers(0, other, n), -1).astype(np.int32)
    out = np.zeros(n, np.int32)
    cnt = C.c_int32()
    rc = lib().orbx_debug_match_finish(kind, n1, n2, ptr(match), ptr(out), C.byref(cnt))
    assert rc == 0 and np.array_equal(out, match) and cnt.value == int((match >= 0).sum())
    bad = match.copy()
    bad[::7] = other + 10 ** np.arange(len(bad[::7])) % 1_000_000_007  # far out of range
    bad[3] = 2 ** 31 - 1
    rc = lib().orbx_debug_match_finish(kind, n1, n2, ptr(bad), ptr(out), C.byref(cnt))
    assert rc == -3  # ORBX_EDEVICE
    keep = np.where((bad >= 0) & (bad < other), bad, -1)
    assert np.array_equal(out, keep) and cnt.value == int((keep >= 0).sum())


@pytest.mark.parametrize("form", [1, 2, 3])
def test_search_by_bow_every_kernel_form(frames, form):
    """Every SearchByBoW node kernel on the same inputs (orbx_debug_bow_kernel forces the form the
    calls choose by problem count and features per node: 1 workgroup per node, 2 / 3 a wave with
    4 / 2 register chunks — the batches' forms, otherwise reached only through the frame
    pipeline): both overloads on real frames, contested small and large nodes (claim chains, ties,
    invalid features) and a node of 1,500 candidates (register chunks and memory reads)."""
    from ar_orbslam2_amd._ffi import check, lib
    check("orbx_debug_bow_kernel", lib().orbx_debug_bow_kernel(form))
    try:
        kf, f, _ = frames
        test_search_by_bow_kf_frame(frames, 0.7, True)
        test_search_by_bow_kf_kf(frames, 0.75, True)
        cases = [(10, 12, 2, False), (20, 30, 4, True), (90, 7, 2, False), (100, 128, 4, True),
                 (130, 100, 16, False)]
        for n1, n2, palette, chain in cases:
            test_search_by_bow_contested_nodes(n1, n2, palette, chain)
        test_search_by_bow_single_huge_node(1500)
    finally:
        lib().orbx_debug_bow_kernel(0)
