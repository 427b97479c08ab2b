"""The reference-side shims (include/compat/: ORBextractor_orbx.cc, ORBmatcher_orbx.cc,
Frame_orbx.cc, Marker_orbx.cc) compile against ORB-SLAM2's own headers and include/orbx.h, so a
change of the C ABI that the shims do not follow fails here.  OpenCV 2.4 and DBoW2 are absent from this image:
tests/compat_stub/ stands in for the declarations those headers name, and the compiler runs with
-fsyntax-only (a compile check of this repository's shim code only; nothing is linked or run).
Every orbx_ function the shims call must be exported by liborbx.so.  CPU only."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/ORB_SLAM2"
SHIMS = ["ORBextractor_orbx.cc", "ORBmatcher_orbx.cc", "Frame_orbx.cc", "Marker_orbx.cc"]

needs_ref = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "include")),
                               reason="the reference headers are not present here")


@needs_ref
@pytest.mark.parametrize("shim", SHIMS)
def test_shim_compiles_against_reference_headers(shim):
    cxx = shutil.which("g++")
    assert cxx
    cmd = [cxx, "-std=c++11", "-fsyntax-only", "-Wall", "-Wextra", "-Werror",
           "-I", os.path.join(ROOT, "tests", "compat_stub"), "-I", os.path.join(ROOT, "include"),
           "-I", os.path.join(ROOT, "include", "compat"), "-I", os.path.join(REF, "include"),
           "-I", REF, os.path.join(ROOT, "include", "compat", shim)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]


def test_shim_calls_are_exported():
    lib = os.path.join(ROOT, "ar_orbslam2_amd", "_lib", "liborbx.so")
    if not os.path.exists(lib):
        pytest.skip("liborbx.so not built")
    nm = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True, text=True)
    exported = set(re.findall(r"\b(orbx_\w+)$", nm.stdout, re.M))
    called = set()
    for shim in SHIMS:
        src = open(os.path.join(ROOT, "include", "compat", shim)).read()
        called |= set(re.findall(r"\b(orbx_[a-z0-9_]+)\s*\(", src))
    # the shims' own helpers (defined in the shim files) are not library symbols
    own = {"orbx_context_of", "orbx_materialize_pyramid", "orbx_load_vocabulary", "orbx_compute_bow",
           "orbx_compute_stereo_matches", "orbx_marker_orb", "orbx_marker_good_matches"}
    hdr = open(os.path.join(ROOT, "include", "orbx.h")).read()
    types = set(re.findall(r"\b(orbx_\w+);", hdr))  # typedef names (sizeof(orbx_keypoint) ...)
    missing = sorted(called - own - types - exported)
    assert not missing, missing
    assert len(called - own - types) >= 12
