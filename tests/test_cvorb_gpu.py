"""GPU parity: the AR marker path on gfx950 (cv::ORB 2.4 HARRIS/FAST, BruteForceMatcher,
Marker::Match's filter, naive_nn_search2) vs the CPU oracle (oracle/cvorb_oracle.cc), bit for
bit: every cv::KeyPoint field (angles and Harris responses bitwise), the keypoint order that
retainBest's nth_element/partition leave, descriptors, match lists.

Parity against real OpenCV 2.4 cv::ORB is unpinned: the oracle is a
restatement of it, checked by tests/test_cvorb_oracle.py.
"""
import os

import numpy as np
import pytest
import torch  # before liborbx loads: torch must bring up its HIP runtime first

from ar_orbslam2_amd import _ffi, synth
from ar_orbslam2_amd import marker as M
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _kp_equal(kps, okps, what=""):
    assert len(kps) == len(okps), (what, len(kps), len(okps), np.bincount(kps["octave"]),
                                   np.bincount(okps["octave"]))
    for f in ("x", "y", "size", "angle", "response"):
        bad = np.nonzero(kps[f].view(np.uint32) != okps[f].view(np.uint32))[0]
        assert bad.size == 0, f"{what} field {f}: {bad.size} differ, first {bad[:5]}"
    for f in ("octave", "class_id"):
        assert (kps[f] == okps[f]).all(), (what, f)


def _compare(img, **kw):
    orb = M.ORB(**kw)
    kps, desc = orb(img)
    if img.size == 0:  # orb.cpp returns before touching the outputs
        assert kps is None and desc is None
        return None, None
    p = O.cvorb_params(kw.get("nfeatures", 500), kw.get("scaleFactor", 1.2),
                       kw.get("nlevels", 8), kw.get("edgeThreshold", 31),
                       score_type=kw.get("scoreType", M.HARRIS_SCORE))
    okps, odesc = O.cvorb_detect(img, p)
    _kp_equal(kps, okps)
    if len(kps):
        bad = np.nonzero((desc != odesc).any(1))[0]
        assert bad.size == 0, f"descriptors: {bad.size} rows differ, first {bad[:5]}"
    else:
        assert desc is None
    orb.close()
    return kps, desc


@pytest.mark.parametrize("name", ["tmp", "book1", "target"])
def test_real_frames(golden_dir, name):
    img = synth.read_pgm(os.path.join(golden_dir, name + ".pgm"))
    kps, _ = _compare(img)
    assert len(kps) >= 400


@pytest.mark.parametrize("w,h,t", [(640, 480, 0), (640, 480, 7), (752, 480, 3), (1241, 376, 1),
                                   (1920, 1080, 0)])
def test_synthetic_harris(w, h, t):
    _compare(synth.frame(w, h, t))


@pytest.mark.parametrize("w,h", [(640, 480), (1920, 1080)])
def test_synthetic_fast_score(w, h):
    _compare(synth.frame(w, h, 2), scoreType=M.FAST_SCORE)


def test_ar13_parameters(golden_dir):
    # AR-1.3/src/ORBMatcher.cpp:121-122: ORB orb(300, 1.2f, 8, 31, 0, 2, HARRIS_SCORE, 31)
    img = synth.read_pgm(os.path.join(golden_dir, "tmp.pgm"))
    kps, _ = _compare(img, nfeatures=300)
    assert len(kps) >= 250


def test_repeated_pattern_ties():
    # a tiled patch gives many keypoints with identical FAST scores and Harris responses: the
    # retained set and order come from nth_element / partition's tie handling
    rng = np.random.default_rng(5)
    patch = (rng.random((24, 24)) > 0.5).astype(np.uint8) * 200 + 20
    img = np.tile(patch, (20, 27))[:480, :640].copy()
    _compare(img)
    _compare(img, scoreType=M.FAST_SCORE)


def test_noise_many_candidates():
    # uniform noise: tens of thousands of FAST candidates at level 0 (the global-memory path of
    # k_cvselect, > 4096 keypoints)
    rng = np.random.default_rng(11)
    img = rng.integers(0, 256, (480, 640), dtype=np.uint8)
    _compare(img)
    _compare(img, nfeatures=5000, scoreType=M.FAST_SCORE)


def test_dense_corner_pattern_fills_pretest_queues():
    # every level-0 pixel passes the even-point pretest at 20 (tests/test_extract_gpu.py): the
    # per-wave candidate queues of k_cvfast run full
    img = synth.dense_corners(640, 480)
    _compare(img)
    _compare(img, scoreType=M.FAST_SCORE)


def test_small_and_degenerate():
    assert _compare(np.zeros((0, 0), np.uint8)) == (None, None)
    kps, desc = _compare(np.full((200, 200), 77, np.uint8))
    assert len(kps) == 0 and desc is None
    # levels smaller than 2 * edgeThreshold keep nothing
    _compare(synth.frame(160, 120, 0))
    _compare(synth.frame(97, 300, 1), nfeatures=200, nlevels=4)
    _compare(synth.frame(640, 480, 0), nfeatures=20)  # last level gets 0 -> retains all


def test_edge_threshold_and_levels():
    img = synth.frame(640, 480, 4)
    _compare(img, edgeThreshold=18)
    _compare(img, edgeThreshold=40, nlevels=5, scaleFactor=1.3)


def test_unsupported_parameters():
    with pytest.raises(_ffi.OrbxError):
        M.ORB(WTA_K=3)
    with pytest.raises(_ffi.OrbxError):
        M.ORB(edgeThreshold=10)


# ---------------------------------------------------------------- retainBest in isolation
def _retain_gpu(resp, n_points, force_global=False):
    import ctypes as C
    r = np.ascontiguousarray(resp, np.float32).copy()
    ids = np.arange(len(r), dtype=np.uint32)
    n = C.c_int32()
    _ffi.check("orbx_debug_retain_best",
               _ffi.lib().orbx_debug_retain_best(_ffi.ptr(r), _ffi.ptr(ids), C.c_int32(len(r)),
                                                 C.c_int32(n_points), C.c_int32(int(force_global)),
                                                 C.byref(n)))
    return r[:n.value], ids[:n.value].astype(np.int32)


@pytest.mark.parametrize("kind", ["random", "ints", "equal", "ascending", "descending", "organ",
                                  "two"])
@pytest.mark.parametrize("n,k", [(10, 3), (100, 7), (1000, 218), (3000, 109), (4096, 2000),
                                 (20000, 150)])
def test_retain_best_matches_libstdcxx(kind, n, k):
    rng = np.random.default_rng(n * 7 + k)
    if kind == "random":
        r = rng.random(n).astype(np.float32)
    elif kind == "ints":
        r = rng.integers(20, 40, n).astype(np.float32)
    elif kind == "equal":
        r = np.full(n, 3.0, np.float32)
    elif kind == "ascending":
        r = np.arange(n, dtype=np.float32)
    elif kind == "descending":
        r = np.arange(n, 0, -1).astype(np.float32)
    elif kind == "organ":  # organ pipe: stresses the median-of-three pivots (depth limit)
        h = np.arange(n // 2, dtype=np.float32)
        r = np.concatenate([h, h[::-1], np.zeros(n - 2 * len(h), np.float32)])
    else:
        r = rng.integers(0, 2, n).astype(np.float32)
    er, eid = O.retain_best(r, k)
    for fg in (False, True):
        gr, gid = _retain_gpu(r, k, fg)
        assert len(gid) == len(eid), (kind, n, k, fg)
        assert (gid == eid).all(), (kind, n, k, fg, np.nonzero(gid != eid)[0][:5])
        assert (gr.view(np.uint32) == er.view(np.uint32)).all()


def test_cos_sin_every_angle():
    """(float)cos/sin((double)angle) on the device equals the host libm for every float angle
    in [0, 360] degrees (all fastAtan2 can return)."""
    import ctypes as C
    lo = 0
    hi = int(np.array([360.0], np.float32).view(np.uint32)[0]) + 1
    chunk = 1 << 25
    bad = 0
    first = None
    for b0 in range(lo, hi, chunk):
        n = min(chunk, hi - b0)
        deg = np.arange(b0, b0 + n, dtype=np.uint32).view(np.float32)
        c = np.empty(n, np.float32)
        s = np.empty(n, np.float32)
        _ffi.check("orbx_debug_cvorb_cossin",
                   _ffi.lib().orbx_debug_cvorb_cossin(_ffi.ptr(deg), C.c_int64(n), _ffi.ptr(c),
                                                      _ffi.ptr(s)))
        oc, os_ = O.cos_sin_f64_range(b0, n, threads=16)
        m = (c.view(np.uint32) != oc.view(np.uint32)) | (s.view(np.uint32) != os_.view(np.uint32))
        if m.any():
            bad += int(m.sum())
            if first is None:
                first = deg[np.nonzero(m)[0][:5]]
    assert bad == 0, f"{bad} angles differ, first {first}"


# ---------------------------------------------------------------- matchers
def _desc_pairs(rng, nq, nt, flips=(0, 40)):
    base = rng.integers(0, 256, (nt, 32), dtype=np.uint8)
    q = base[rng.integers(0, nt, nq)].copy()
    bits = np.unpackbits(q, axis=1)
    for i in range(nq):
        k = rng.integers(flips[0], flips[1] + 1)
        idx = rng.choice(256, k, replace=False)
        bits[i, idx] ^= 1
    return np.packbits(bits, axis=1), base


@pytest.mark.parametrize("nq,nt", [(1, 1), (500, 500), (37, 1000), (1000, 300), (300, 0),
                                   (0, 10)])
def test_bf_match_and_filter(nq, nt):
    rng = np.random.default_rng(nq + 3 * nt)
    q, t = _desc_pairs(rng, nq, max(nt, 1))
    t = t[:nt]
    # duplicate train rows: ties must resolve to the first minimum
    if nt > 4:
        t[nt // 2] = t[1]
    m = M.BruteForceMatcher().match(q, t)
    om = O.bf_match(q, t)
    assert m.tobytes() == om.tobytes()
    g, mn, mx = M.good_matches(m)
    og, omn, omx = O.good_matches(om)
    assert g.tobytes() == og.tobytes() and mn == omn and mx == omx


@pytest.mark.parametrize("ratio", [0.8, 0.0])
@pytest.mark.parametrize("nq,nt", [(300, 300), (500, 37), (20, 1), (10, 0)])
def test_nn_match(ratio, nq, nt):
    rng = np.random.default_rng(nq * 5 + nt)
    q, t = _desc_pairs(rng, nq, max(nt, 1), (0, 60))
    t = t[:nt]
    m, mn, mx = M.nn_match(q, t, ratio, 50)
    om, omn, omx = O.nn_match(q, t, ratio, 50)
    assert m.tobytes() == om.tobytes() and mn == omn and mx == omx


def test_marker_match_dropin(golden_dir):
    target = synth.read_pgm(os.path.join(golden_dir, "target.pgm"))
    frame = synth.read_pgm(os.path.join(golden_dir, "tmp.pgm"))
    mk = M.Marker()
    mk.setTargetImage(target)
    ok, good, matches, kps2, d2 = mk.Match(frame)
    tk, td = O.cvorb_detect(target, O.cvorb_params())
    fk, fd = O.cvorb_detect(frame, O.cvorb_params())
    om = O.bf_match(td, fd)
    og, _, _ = O.good_matches(om)
    assert ok and matches.tobytes() == om.tobytes() and good.tobytes() == og.tobytes()


def test_marker_batch_pipeline(golden_dir):
    w, h, n = 640, 480, 12
    target = synth.read_pgm(os.path.join(golden_dir, "target.pgm"))
    tk, td = O.cvorb_detect(target, O.cvorb_params())
    imgs = synth.frames(w, h, n, stream=1)
    dev = torch.from_numpy(np.ascontiguousarray(imgs)).cuda()
    mb = M.MarkerBatch(w, h, 16)
    mb.set_target(td)
    mb.run(dev.data_ptr(), n)
    mb.sync()
    kp_counts, good_counts = mb.results(n)
    outs = mb.device_outputs()
    nq = len(td)
    matches = np.empty(n * nq, _ffi.DMATCH_DTYPE)
    good = np.empty(n * nq, np.uint8)
    _copy_d2h(outs["matches"], matches)
    _copy_d2h(outs["good"], good)
    for f in range(n):
        okps, odesc = O.cvorb_detect(imgs[f], O.cvorb_params())
        assert kp_counts[f] == len(okps), f
        om = O.bf_match(td, odesc)
        og, _, _ = O.good_matches(om)
        got = matches[f * nq:(f + 1) * nq]
        assert got.tobytes() == om.tobytes(), f
        assert good_counts[f] == len(og), f
        assert got[good[f * nq:(f + 1) * nq].astype(bool)].tobytes() == og.tobytes(), f
    mb.close()


def _copy_d2h(dptr, out):
    import ctypes as C
    hip = C.CDLL("libamdhip64.so")
    rc = hip.hipMemcpy(C.c_void_p(out.ctypes.data), C.c_void_p(dptr), C.c_size_t(out.nbytes),
                       C.c_int(2))
    assert rc == 0
