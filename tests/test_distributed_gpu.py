"""The N>1 device path of bench.py on the one-GPU box: bench's own launcher starts two rank
processes (before anything touches the GPU), both run real frame pipelines on device 0
(`--same-device`) and meet over gloo for the barrier and the max-over-ranks time — the code the
driver's 8-GPU SCALE run executes, minus the hardware (camera stream s on rank
s mod G, no data-path collective)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def check_verify_dump(path, nf, stereo_cfg=None):
    """A rank's --verify-frames dump against the oracle: frames {0, B-1} and their keyframes —
    keypoints, descriptors, (stereo) mvuRight / mvDepth, SearchByBoW and SearchForTriangulation
    against frame (f - 1) mod B, with the rank's own masks."""
    from ar_orbslam2_amd.pipeline import fundamental_from_pose
    from oracle import oracle as O
    from matchdata import featvec
    from test_pipeline_gpu import _oracle_extract, _vocabs
    d = np.load(path)
    assert int(d["err"]) == 0
    stereo = bool(d["stereo"])
    B = int(d["batch"])
    ids = [int(x) for x in d["frame_ids"]]
    h, w = d["images"].shape[1:]
    t = O.tables(O.params(nf), w, h)
    _, oracle_voc = _vocabs()
    ref = {}
    for j, f in enumerate(ids):
        li = 2 * j if stereo else j
        if stereo:
            from ar_orbslam2_amd.stereo import stereo_params
            kps, desc, pl, _ = _oracle_extract(d["images"][li], nf, True)
            kr, dr, pr, _ = _oracle_extract(d["images"][li + 1], nf, True)
            assert np.array_equal(d["kps"][li + 1][:len(kr)], kr)
            assert np.array_equal(d["desc"][li + 1][:len(kr)], dr)
        else:
            kps, desc = _oracle_extract(d["images"][li], nf)
        k = len(kps)
        assert int(d["counts"][j]) == k > 0
        assert np.array_equal(d["kps"][li][:k], kps)
        assert np.array_equal(d["desc"][li][:k], desc)
        r = dict(desc=desc, angle=kps["angle"], keys=kps,
                 fv=featvec(oracle_voc.transform(desc, 4)["node_of"]), valid=d["valid"][j][:k],
                 has_mp=d["has_mp"][j][:k], scale_factors=t["scale"], level_sigma2=t["sigma2"])
        if stereo:
            ur, dp, _ = O.stereo_matches(kps, desc, kr, dr, pl, pr, t["scale"], t["inv_scale"],
                                         *stereo_params(*stereo_cfg))
            assert d["uright"][j][:k].tobytes() == ur.tobytes()
            assert d["depth"][j][:k].tobytes() == dp.tobytes()
            r["u_right"] = ur
        ref[f] = r
    ex, ey = (float(x) for x in d["epipole"])
    F = fundamental_from_pose()
    for j, f in enumerate([0, B - 1]):
        kf, cur = ref[(f - 1) % B], ref[f]
        nb, mb = O.search_by_bow_kf_f(kf, dict(cur, valid=None), 0.7, True)
        assert int(d["bow"][j]) == nb
        assert np.array_equal(d["match"][j][:len(cur["desc"])], mb)
        nt, pt = O.search_for_triangulation(kf, cur, F, ex, ey, False, 0.6, False)
        assert int(d["tri"][j]) == nt
        assert np.array_equal(d["pairs"][j][:nt], pt)
    return int(d["stream"])


@pytest.mark.timeout(600)
@pytest.mark.parametrize("extra,streams", [([], [[0, 2], [1, 3]]),
                                           (["--streams-total", "3"], [[0, 2], [1]])])
def test_two_ranks_same_device(extra, streams, tmp_path):
    """Two real ranks; besides the counts, rank 0's and rank 1's own outputs (frames {0, B-1} of
    their first camera stream, --verify-frames) equal the oracle."""
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "2",
           "--dist-backend", "gloo", "--same-device", "--steps", "3", "--warmup", "1",
           "--batch", "32", "--pool", "2", "--streams", "2", "--no-cpu-baseline", "--no-upload",
           "--roofline-steps", "1", "--verify-frames", str(tmp_path)] + extra
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=540, env=env, cwd=ROOT)
    assert res.returncode == 0, res.stderr[-3000:]
    lines = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, res.stdout[-2000:]  # rank 0 prints the one JSON line
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2
    assert out["config"]["streams_per_rank"] == streams
    assert out["config"]["dist_backend"] == "gloo" and out["config"]["same_device"]
    n = sum(len(s) for s in streams)
    assert out["config"]["frames_total"] == n * 32 * 3
    assert out["value"] > 0
    assert abs(out["value"] * out["ms_per_step"] * 3 / 1e3 - n * 32 * 3) < 1e-3 * n * 32 * 3
    assert out["scaling"] == ("strong" if extra else "weak")
    for r in (0, 1):
        assert check_verify_dump(os.path.join(tmp_path, f"rank{r}.npz"), 1000) == streams[r][0]


@pytest.mark.timeout(600)
def test_two_ranks_same_device_stereo(tmp_path):
    """The N > 1 path on a stereo config (C3, EuRoC geometry): rank 1's frames — both images,
    mvuRight / mvDepth and both matchers — equal the oracle."""
    import bench
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--config", "C3", "--gpus", "2",
           "--dist-backend", "gloo", "--same-device", "--steps", "2", "--warmup", "1",
           "--batch", "16", "--pool", "2", "--streams", "1", "--no-cpu-baseline", "--no-upload",
           "--roofline-steps", "1", "--verify-frames", str(tmp_path)]
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=540, env=env, cwd=ROOT)
    assert res.returncode == 0, res.stderr[-3000:]
    cfg = bench.CONFIGS["C3"]
    assert check_verify_dump(os.path.join(tmp_path, "rank1.npz"), cfg["nfeatures"],
                             cfg["stereo"]) == 1
