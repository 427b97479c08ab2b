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
