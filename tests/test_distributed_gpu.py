"""The N>1 device path of bench.py on the one-GPU box: bench's own launcher starts two rank
processes (before anything touches the GPU), both run real frame pipelines on device 0
(`--same-device`) and meet over gloo for the barrier and the max-over-ranks time — the code the
driver's 8-GPU SCALE run executes, minus the hardware (camera stream s on rank
s mod G, no data-path collective)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(600)
@pytest.mark.parametrize("extra,streams", [([], [[0, 2], [1, 3]]),
                                           (["--streams-total", "3"], [[0, 2], [1]])])
def test_two_ranks_same_device(extra, streams):
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "2",
           "--dist-backend", "gloo", "--same-device", "--steps", "3", "--warmup", "1",
           "--batch", "32", "--pool", "2", "--streams", "2", "--no-cpu-baseline", "--no-upload",
           "--roofline-steps", "1"] + extra
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
