"""The library's environment switches, each run in a process of its own and checked against the
oracle (every other kernel selector was removed in round 4: `grep getenv ar_orbslam2_amd/csrc`
lists exactly these).
  ORBX_SPIN_US      how long a one-call (drop-in) wait polls its stream before blocking; 0 blocks
                    at once (orbx_geometry.cpp wait_stream)
  ORBX_SYNC_STAGES  debugging: a frame pipeline runs eagerly (no captured graph), synchronising
                    after every stage to name the stage of an asynchronous fault
                    (orbx_frames.hip, orbx_internal.h Profiler::mark)
  ORBX_NO_RESIDENT  the per-frame drop-in calls take the staged per-call copies instead of the
                    resident frame cache (orbx_match.h; A/B runs of bench.py --dropin)"""
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_EXTRACT = r"""
import numpy as np
from ar_orbslam2_amd import ORBextractor, synth
from oracle import oracle as O
img = synth.frame(640, 480, t=3, stream=1)
ex = ORBextractor(1000)
for _ in range(3):
    kps, desc = ex(img)
okps, odesc = O.extract(img, O.params(1000))
assert np.array_equal(kps, okps) and np.array_equal(desc, odesc)
print("SWITCH-OK", len(kps))
"""

_PIPELINE = r"""
import sys
import numpy as np
import torch
sys.path.insert(0, "tests")
from ar_orbslam2_amd import synth
from ar_orbslam2_amd.pipeline import FramePipeline, fundamental_from_pose
from test_pipeline_gpu import _check_pipe_frames, _vocabs
voc, ovoc = _vocabs()
n = 6
pipe = FramePipeline(640, 480, n, voc, 1000)
pipe.masks = pipe.seeded_masks(range(n))
pipe.epipole = (321.5, 260.25)
pipe.set_matching(fundamental_from_pose(), pipe.epipole, bow_ratio=0.7, bow_check_ori=True,
                  tri_ratio=0.6, tri_check_ori=False)
frames = synth.frames(640, 480, n, stream=5)
d = torch.from_numpy(frames).cuda()
pipe.run(d.data_ptr(), n)
pipe.sync()
_check_pipe_frames(pipe, frames, list(range(n)), 1000, n, ovoc)
pipe.close()
print("SWITCH-OK", n)
"""


def _run(code, env_extra):
    env = dict(os.environ, **env_extra)
    res = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240,
                         cwd=ROOT, env=env)
    assert res.returncode == 0, res.stderr[-3000:]
    assert "SWITCH-OK" in res.stdout
    return res


def test_switch_list_is_exactly_the_tested_ones():
    found = set()
    for root, _, files in os.walk(os.path.join(ROOT, "ar_orbslam2_amd", "csrc")):
        for f in files:
            if f.endswith((".hip", ".h", ".cpp")):
                found |= set(re.findall(r'getenv\("(\w+)"\)', open(os.path.join(root, f)).read()))
    assert found == {"ORBX_SPIN_US", "ORBX_SYNC_STAGES", "ORBX_NO_RESIDENT"}


@pytest.mark.gpu
@pytest.mark.timeout(300)
@pytest.mark.parametrize("spin", ["0", "50"])
def test_spin_us_drop_in_extraction(spin):
    _run(_EXTRACT, {"ORBX_SPIN_US": spin})


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_sync_stages_pipeline():
    _run(_PIPELINE, {"ORBX_SYNC_STAGES": "1"})


_CHAIN = r"""
import sys
sys.path.insert(0, "tests")
import test_resident_gpu as T
frames, v = T._chain()
T.test_chain_with_reference_keyframes_and_evictions((frames, v))
T.test_other_featurevector_and_keypoints_for_resident_descriptors((frames, v))
print("SWITCH-OK", len(frames))
"""


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_no_resident_drop_in_chain():
    _run(_CHAIN, {"ORBX_NO_RESIDENT": "1"})
