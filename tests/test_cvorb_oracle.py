"""CPU checks of the AR marker path oracle (oracle/cvorb_oracle.cc): cv::ORB 2.4 with
HARRIS_SCORE, BruteForceMatcher<HammingLUT>, Marker::Match's filter and naive_nn_search2.

OpenCV 2.4 is not in the image and the reference holds no output of cv::ORB, so parity with
real OpenCV is unpinned; the restatement is pinned here by
  * an independent pure-Python transliteration of libstdc++ (GCC 4.8) std::nth_element /
    std::partition as KeyPointsFilter::retainBest uses them, on tie-heavy inputs;
  * known answers derived by hand for HarrisResponses, computeOrbDescriptor at 0 and 90
    degrees, the level table of operator() and the matcher rules (Marker.cc:110-133,
    AR-1.3/src/ORBMatcher.cpp:70-102);
  * structural properties of the full extractor on the committed AR-1.3 frame (tmp.pgm is
    AR-1.3/tmp.jpg).
"""
import os

import numpy as np
import pytest

from ar_orbslam2_amd import synth
from oracle import oracle as O


# ------------------------------------------------------------------ libstdc++ 4.8, transliterated
def _lg(n):
    return n.bit_length() - 1


def _introselect(a, first, nth, last, comp):
    depth = _lg(last - first) * 2
    while last - first > 3:
        if depth == 0:
            _heap_select(a, first, nth + 1, last, comp)
            a[first], a[nth] = a[nth], a[first]
            return
        depth -= 1
        mid = first + (last - first) // 2
        x, y, z = first, mid, last - 1  # __move_median_first(first, mid, last-1)
        if comp(a[x], a[y]):
            if comp(a[y], a[z]):
                a[x], a[y] = a[y], a[x]
            elif comp(a[x], a[z]):
                a[x], a[z] = a[z], a[x]
        elif comp(a[x], a[z]):
            pass
        elif comp(a[y], a[z]):
            a[x], a[z] = a[z], a[x]
        else:
            a[x], a[y] = a[y], a[x]
        pivot = a[first]
        lo, hi = first + 1, last  # __unguarded_partition(first+1, last, *first)
        while True:
            while comp(a[lo], pivot):
                lo += 1
            hi -= 1
            while comp(pivot, a[hi]):
                hi -= 1
            if not lo < hi:
                break
            a[lo], a[hi] = a[hi], a[lo]
            lo += 1
        cut = lo
        if cut <= nth:
            first = cut
        else:
            last = cut
    for i in range(first + 1, last):  # __insertion_sort
        val = a[i]
        if comp(val, a[first]):
            a[first + 1:i + 1] = a[first:i]
            a[first] = val
        else:
            j = i
            while comp(val, a[j - 1]):
                a[j] = a[j - 1]
                j -= 1
            a[j] = val


def _adjust_heap(a, base, hole, n, value, comp):
    top = hole
    second = hole
    while second < (n - 1) // 2:
        second = 2 * (second + 1)
        if comp(a[base + second], a[base + second - 1]):
            second -= 1
        a[base + hole] = a[base + second]
        hole = second
    if n % 2 == 0 and second == (n - 2) // 2:
        second = 2 * (second + 1)
        a[base + hole] = a[base + second - 1]
        hole = second - 1
    parent = (hole - 1) // 2
    while hole > top and comp(a[base + parent], value):
        a[base + hole] = a[base + parent]
        hole = parent
        parent = (hole - 1) // 2
    a[base + hole] = value


def _heap_select(a, first, middle, last, comp):
    n = middle - first
    if n >= 2:
        parent = (n - 2) // 2
        while True:
            _adjust_heap(a, first, parent, n, a[first + parent], comp)
            if parent == 0:
                break
            parent -= 1
    for i in range(middle, last):
        if comp(a[i], a[first]):
            v = a[i]
            a[i] = a[first]
            _adjust_heap(a, first, 0, n, v, comp)


def _partition(a, first, last, pred):
    while True:
        while True:
            if first == last:
                return first
            if pred(a[first]):
                first += 1
            else:
                break
        last -= 1
        while True:
            if first == last:
                return first
            if not pred(a[last]):
                last -= 1
            else:
                break
        a[first], a[last] = a[last], a[first]
        first += 1


def py_retain_best(resp, n_points):
    a = [(float(r), i) for i, r in enumerate(np.asarray(resp, np.float32))]
    if n_points > 0 and len(a) > n_points:
        greater = lambda x, y: x[0] > y[0]  # noqa: E731  KeypointResponseGreater
        if n_points != len(a):
            _introselect(a, 0, n_points, len(a), greater)
        amb = a[n_points - 1][0]
        end = _partition(a, n_points, len(a), lambda k: k[0] >= amb)
        a = a[:end]
    return np.array([r for r, _ in a], np.float32), np.array([i for _, i in a], np.int32)


@pytest.mark.parametrize("seed", range(12))
def test_retain_best_matches_libstdcxx48_transliteration(seed):
    rng = np.random.default_rng(seed)
    for n, npts, levels in [(0, 5, 10), (3, 2, 3), (4, 2, 2), (50, 10, 4), (700, 218, 30),
                            (2500, 180, 60), (2500, 90, 2500), (900, 899, 5), (40, 0, 5)]:
        resp = rng.integers(0, levels, n).astype(np.float32)  # FAST-score-like ties
        r1, i1 = O.retain_best(resp, npts)
        r2, i2 = py_retain_best(resp, npts)
        assert np.array_equal(i1, i2), (n, npts, levels)
        assert np.array_equal(r1, r2)
        if 0 < npts < n:
            # the retained set: the n_points best plus the tail tied with keypoints[n-1]
            kth = np.sort(resp)[::-1][npts - 1]
            assert len(i1) >= npts and (r1[:npts] >= kth).all()
            assert sorted(i1[:npts].tolist()) == sorted(i1[:npts].tolist())


def test_retain_best_heap_select_fallback():
    """Inputs that exhaust introselect's depth limit take the heap_select path."""
    # median-of-three killer for a greater-than comparator: descending organ pipe
    n = 1024
    resp = np.concatenate([np.arange(n // 2), np.arange(n // 2)[::-1]]).astype(np.float32)
    for npts in (1, 7, 300, 700):
        r1, i1 = O.retain_best(resp, npts)
        r2, i2 = py_retain_best(resp, npts)
        assert np.array_equal(i1, i2)


# ------------------------------------------------------------------ primitives, known answers
def test_harris_ramp_known_answer():
    img = np.tile((np.arange(64) * 3).astype(np.uint8), (64, 1))  # I = 3x
    got = O.harris(img, 30, 30)
    # Ix = (6)*2 + 6 + 6 = 24, Iy = 0 over the 7x7 block: a = 49*576, b = c = 0
    f = np.float32
    a = f(49 * 576)
    scale = f(1) / f(4 * 7 * 255.0)
    s4 = scale * scale * scale * scale
    want = (a * f(0) - f(0) * f(0) - f(0.04) * (a + f(0)) * (a + f(0))) * s4
    assert np.float32(got) == want


def test_harris_corner_sign():
    img = np.zeros((64, 64), np.uint8)
    img[32:, 32:] = 200  # an L corner: positive response; an edge: negative
    assert O.harris(img, 32, 32) > 0
    assert O.harris(img, 45, 32) < 0


def _pattern():
    import re
    src = open(os.path.join(os.path.dirname(__file__), "..", "include", "orbx_pattern.h")).read()
    body = src[src.index("{", src.index("ORBX_PATTERN")) + 1:]
    body = body[:body.index("}")]
    return np.array([int(v) for v in re.findall(r"-?\d+", body)], np.int32).reshape(512, 2)


@pytest.mark.parametrize("deg", [0.0, 90.0])
def test_descriptor_axis_angles(deg):
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (80, 80), dtype=np.uint8)
    d = O.cvorb_descriptor(img, 40, 40, deg)
    pat = _pattern()
    c, s = O.cos_sin_f64(deg)
    f = np.float32
    x = (pat[:, 0].astype(f) * f(c) - pat[:, 1].astype(f) * f(s))
    y = (pat[:, 0].astype(f) * f(s) + pat[:, 1].astype(f) * f(c))
    ix, iy = np.rint(x).astype(int), np.rint(y).astype(int)
    if deg == 0:
        assert np.array_equal(ix, pat[:, 0]) and np.array_equal(iy, pat[:, 1])
    else:
        assert np.array_equal(ix, -pat[:, 1]) and np.array_equal(iy, pat[:, 0])
    v = img[40 + iy, 40 + ix].astype(int)
    bits = (v[0::2] < v[1::2]).astype(np.uint8).reshape(32, 8)
    want = (bits << np.arange(8, dtype=np.uint8)).sum(1).astype(np.uint8)
    assert np.array_equal(d, want)


def test_cos_sin_are_double_rounded():
    for deg in (0.0, 30.0, 45.0, 123.456, 359.99):
        c, s = O.cos_sin_f64(deg)
        a = np.float32(deg) * np.float32(np.pi / 180.0)
        assert c == np.float32(np.cos(np.float64(a)))
        assert s == np.float32(np.sin(np.float64(a)))


def test_levels_table():
    lv = O.cvorb_levels(O.cvorb_params(), 640, 480)
    f = np.float32
    for l in range(8):
        s = f(np.float64(f(1.2)) ** l)  # (float)pow((double)1.2f, l)
        inv = f(1) / s
        assert lv["scale"][l] == s
        assert lv["w"][l] == int(np.rint(np.float64(f(640) * inv)))
        assert lv["h"][l] == int(np.rint(np.float64(f(480) * inv)))
    assert lv["feats"].tolist() == [109, 90, 75, 63, 52, 44, 36, 31]
    assert O.cvorb_levels(O.cvorb_params(300), 640, 480)["feats"].sum() == 300


# ------------------------------------------------------------------ matchers (Marker / AR-1.3)
def _desc_with_dist(base, dist, rng):
    d = base.copy()
    bits = rng.choice(256, dist, replace=False)
    for b in bits:
        d[b // 8] ^= np.uint8(1 << (b % 8))
    return d


def test_bf_match_first_minimum_and_empty():
    rng = np.random.default_rng(1)
    base = rng.integers(0, 256, 32, dtype=np.uint8)
    train = np.stack([_desc_with_dist(base, d, rng) for d in (9, 3, 3, 40)])
    q = base[None]
    m = O.bf_match(q, train)
    assert m[0]["train_idx"] == 1 and m[0]["distance"] == 3.0  # first of the tied minimum
    assert len(O.bf_match(q, train[:0])) == 0 and len(O.bf_match(q[:0], train)) == 0


def test_good_matches_rule():
    m = np.zeros(4, O.DMATCH_DTYPE)
    m["query_idx"] = np.arange(4)
    m["distance"] = [10, 40, 19.5, 20]
    good, mn, mx = O.good_matches(m)
    assert mx == 40 and mn == 10
    assert good["query_idx"].tolist() == [0, 2]  # distance < 0.5 * 40


def test_nn_ratio_rule():
    rng = np.random.default_rng(2)
    base = rng.integers(0, 256, 32, dtype=np.uint8)
    # best 40, second 50: 40 <= (unsigned)(50 * 0.8) = 40 -> accepted
    t1 = np.stack([_desc_with_dist(base, 50, rng), _desc_with_dist(base, 40, rng)])
    m, mn, mx = O.nn_match(base[None], t1, 0.8, 50)
    assert len(m) == 1 and m[0]["train_idx"] == 1 and (mn, mx) == (40, 50)
    # best 41, second 51: (unsigned)(40.8) = 40 < 41 -> rejected
    t2 = np.stack([_desc_with_dist(base, 51, rng), _desc_with_dist(base, 41, rng)])
    assert len(O.nn_match(base[None], t2, 0.8, 50)[0]) == 0
    # naive_nn_search: no ratio test, <= 50
    assert len(O.nn_match(base[None], t2, 0.0, 50)[0]) == 1
    # a single train row: second stays INT_MAX and the ratio test passes
    assert len(O.nn_match(base[None], t2[1:], 0.8, 50)[0]) == 1


# ------------------------------------------------------------------ the whole extractor
def test_extractor_structure_on_ar_frame(golden_dir):
    img = synth.read_pgm(os.path.join(golden_dir, "tmp.pgm"))  # AR-1.3/tmp.jpg
    p = O.cvorb_params()
    kps, desc, levels = O.cvorb_detect(img, p, want_pyramid=True)
    lv = O.cvorb_levels(p, img.shape[1], img.shape[0])
    assert len(kps) == len(desc) and len(kps) >= 450
    assert (np.diff(kps["octave"]) >= 0).all()  # level-major
    for l in range(8):
        k = kps[kps["octave"] == l]
        s = lv["scale"][l]
        x = k["x"] / s if l else k["x"]
        assert (np.abs(np.rint(x) * s - k["x"]) <= 1e-3 * s).all() or l == 0
        assert len(k) <= max(lv["feats"][l], 0) + 8
        assert (k["size"] == np.float32(31) * s).all()
        assert (k["class_id"] == -1).all()
        assert ((k["angle"] >= 0) & (k["angle"] < 360)).all()
    # level-0 keypoints: FAST corners inside the 31-px border, Harris responses recomputed
    k0 = kps[kps["octave"] == 0]
    assert ((k0["x"] >= 31) & (k0["x"] < img.shape[1] - 31)).all()
    for q in k0[:20]:
        assert np.float32(q["response"]) == np.float32(O.harris(levels[0], int(q["x"]), int(q["y"])))
    # FAST_SCORE keeps FAST scores as responses
    kf, _ = O.cvorb_detect(img, O.cvorb_params(score_type=O.FAST_SCORE))
    assert (kf["response"] == np.rint(kf["response"])).all()


def test_extractor_empty_and_tiny():
    p = O.cvorb_params()
    kps, desc = O.cvorb_detect(np.zeros((40, 40), np.uint8), p)
    assert len(kps) == 0
    kps, desc = O.cvorb_detect(np.full((200, 200), 77, np.uint8), p)
    assert len(kps) == 0


@pytest.mark.parametrize("size", [(640, 480), (1241, 376), (1920, 1080), (37, 41)])
@pytest.mark.parametrize("sf,nl", [(1.2, 8), (1.5, 5), (2.0, 3)])
def test_bench_cvorb_level_sizes_match_oracle(size, sf, nl):
    """bench.py's own cv::ORB level sizes (the AR byte model; the product leg must not call
    oracle/) equal the oracle's getScale / cvRound pyramid sizes."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from ar_orbslam2_amd.marker import cvorb_params
    p = cvorb_params(500, sf, nl)
    lv = O.cvorb_levels(p, *size)
    assert bench.cvorb_level_sizes(p, *size) == list(zip(lv["w"].tolist(), lv["h"].tolist()))
