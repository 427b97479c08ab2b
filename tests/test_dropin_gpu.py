"""The drop-in per-frame path (bench.py --dropin, tools/orbx_dropin.cpp) in both of its modes:
the C ABI called directly ("capi") and the same calls wrapped in the reference-side shims'
per-call marshalling ("shim": per-call buffers, std::map BowVector / FeatureVector, MapPoint
masks, include/compat/*.cc).  Both modes see the same frames and the same seeded masks, so every
frame's keypoints and match counts agree; the shim mode's number is what Frame.cc:252-258,
Tracking.cc:1132-1136 and LocalMapping.cc:238-241 would see."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _dropin(mode, threads=1, frames=30):
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--dropin", "--dropin-mode", mode,
           "--threads", str(threads), "--dropin-frames", str(frames), "--warmup-frames", "3"]
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert res.returncode == 0, res.stderr[-3000:]
    return json.loads([ln for ln in res.stdout.splitlines() if ln.startswith("{")][-1])


@pytest.mark.timeout(300)
def test_dropin_shim_mode_same_work_as_capi():
    a, b = _dropin("capi"), _dropin("shim")
    assert a["config"]["dropin_mode"] == "capi" and b["config"]["dropin_mode"] == "shim"
    da, db = a["dropin"], b["dropin"]
    assert da["mode"] == "capi" and db["mode"] == "shim"
    assert da["frames"] == db["frames"] == 30
    for k in ("keypoints_per_frame", "bow_matches_per_frame", "triangulation_matches_per_frame"):
        assert da[k] == db[k], k
    assert da["keypoints_per_frame"] > 500 and da["bow_matches_per_frame"] > 50
    assert a["value"] > 0 and b["value"] > 0


def _read_dump(path):
    """tools/orbx_dropin.cpp's Dump layout: header, geometry, KF (previous) frame, current
    frame, masks, SearchByBoW matches (KF point indices), triangulation pairs."""
    import numpy as np
    from ar_orbslam2_amd import KEYPOINT_DTYPE
    b = open(path, "rb").read()
    pos = [0]

    def take(n, dt):
        dt = np.dtype(dt)
        a = np.frombuffer(b, dt, n, pos[0]).copy()
        pos[0] += n * dt.itemsize
        return a

    def i32():
        return int(take(1, np.int32)[0])

    assert b[:8] == b"ORBXDMP1"
    pos[0] = 8
    d = dict(frame=i32(), img=i32(), prev_img=i32(), F12=take(9, np.float32).reshape(3, 3))
    d["ex"], d["ey"] = (float(x) for x in take(2, np.float32))
    nl = i32()
    d["scale"], d["sigma2"] = take(nl, np.float32), take(nl, np.float32)

    def frame():
        n = i32()
        f = dict(n=n, keys=take(n, KEYPOINT_DTYPE), desc=take(32 * n, np.uint8).reshape(n, 32))
        nb = i32()
        f["bow_words"], f["bow_values"] = take(nb, np.uint32), take(nb, np.float64)
        nf = i32()
        f["fv_ids"] = take(nf, np.uint32)
        f["fv_off"] = take(nf + 1, np.int32)
        f["fv_feats"] = take(int(f["fv_off"][-1]), np.int32)
        return f

    d["kf"], d["cur"] = frame(), frame()
    d["kf_valid"] = take(d["kf"]["n"], np.uint8)
    d["kf_has_mp"] = take(d["kf"]["n"], np.uint8)
    d["cur_has_mp"] = take(d["cur"]["n"], np.uint8)
    d["nbow"] = i32()
    d["bow_match"] = take(d["cur"]["n"], np.int32)
    d["ntri"] = i32()
    d["tri_pairs"] = take(2 * d["ntri"], np.int32).reshape(-1, 2)
    assert pos[0] == len(b)
    return d


@pytest.mark.timeout(300)
def test_dropin_shim_outputs_match_oracle(tmp_path):
    """What the shim-shaped drop-in hands back to Frame / ORBmatcher's callers for its first and
    last timed frames — keypoints, descriptors, the std::map BowVector and FeatureVector,
    SearchByBoW's MapPoint pointers (as point indices) and SearchForTriangulation's pairs —
    equals the CPU oracle on the same images, vocabulary, masks and geometry (the
    shim mode was only compared with the capi mode's counts)."""
    import numpy as np
    from oracle import oracle as O
    d = tmp_path / "dropin"
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--dropin", "--dropin-mode", "shim",
           "--threads", "1", "--dropin-frames", "10", "--warmup-frames", "3", "--dropin-dir", str(d)]
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert res.returncode == 0, res.stderr[-3000:]
    w, h, nf = 640, 480, 1000
    frames = np.fromfile(d / "frames.u8", np.uint8).reshape(-1, h, w)
    voc = O.Vocabulary.from_nodes(10, 6, 0, 0, np.fromfile(d / "voc_parent.i32", np.int32),
                                  np.fromfile(d / "voc_leaf.u8", np.uint8),
                                  np.fromfile(d / "voc_desc.u8", np.uint8),
                                  np.fromfile(d / "voc_weight.f64", np.float64))
    p = O.params(nf)
    for name in ("dump_first.bin", "dump_last.bin"):
        D = _read_dump(d / name)
        sides = {}
        for key, img in (("kf", D["prev_img"]), ("cur", D["img"])):
            kps, desc = O.extract(frames[img], p)
            got = D[key]
            assert np.array_equal(got["keys"], kps), (name, key, "keypoints")
            assert np.array_equal(got["desc"], desc), (name, key, "descriptors")
            o = voc.transform(desc, 4)
            assert np.array_equal(got["bow_words"], o["bow_words"]), (name, key, "BowVector ids")
            assert got["bow_values"].tobytes() == o["bow_values"].tobytes(), (name, key, "BowVector")
            assert np.array_equal(got["fv_ids"], o["fv_ids"]), (name, key, "FeatureVector ids")
            assert np.array_equal(got["fv_off"], o["fv_off"]), (name, key, "FeatureVector offsets")
            assert np.array_equal(got["fv_feats"], o["fv_feats"]), (name, key, "FeatureVector")
            sides[key] = (kps, desc, (o["fv_ids"], o["fv_off"], o["fv_feats"]))
        (k1, d1, fv1), (k2, d2, fv2) = sides["kf"], sides["cur"]
        n, match = O.search_by_bow_kf_f(
            dict(desc=d1, angle=k1["angle"], valid=D["kf_valid"], fv=fv1),
            dict(desc=d2, angle=k2["angle"], fv=fv2), 0.7, True)
        assert D["nbow"] == n and np.array_equal(D["bow_match"], match), (name, "SearchByBoW")
        nt, pairs = O.search_for_triangulation(
            dict(desc=d1, keys=k1, has_mp=D["kf_has_mp"], fv=fv1, scale_factors=D["scale"],
                 level_sigma2=D["sigma2"]),
            dict(desc=d2, keys=k2, has_mp=D["cur_has_mp"], fv=fv2, scale_factors=D["scale"],
                 level_sigma2=D["sigma2"]),
            D["F12"], D["ex"], D["ey"], False, 0.6, False)
        assert D["ntri"] == nt and np.array_equal(D["tri_pairs"], pairs), (name, "triangulation")
        assert n > 50 and nt > 20
