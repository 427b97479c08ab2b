"""The device math of the product (ar_orbslam2_amd/csrc/orbx_math.h), compiled for the host,
against the host libm sincosf — every float in [0, 2*pi*(1+eps)] — and against the oracle's
fastAtan2.  The same header is compiled for gfx950; tests/test_extract_gpu.py checks the
device build end to end."""
import os
import subprocess

import numpy as np
import pytest

from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "native", "check_math_port.cc")
BIN = os.path.join(ROOT, "oracle", "_build", "check_math_port")


@pytest.fixture(scope="module")
def checker():
    os.makedirs(os.path.dirname(BIN), exist_ok=True)
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-march=x86-64-v3", SRC,
                    "-o", BIN, "-lm", "-lpthread"], check=True)
    return BIN


def test_sincosf_port_exhaustive(checker):
    # all floats from +0 up to just past 360 deg * (float)(pi/180) = 6.2831855
    r = subprocess.run([checker, "0", "0x40C90FE0", str(min(8, os.cpu_count() or 1))],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "sincosf_mismatches 0" in r.stdout


def test_fast_atan2_port_matches_oracle(checker):
    src = os.path.join(ROOT, "oracle", "_build", "atan2_dump.cc")
    exe = os.path.join(ROOT, "oracle", "_build", "atan2_dump")
    with open(src, "w") as f:
        f.write('#include <cstdio>\n#include "%s"\nint main(){int y,x; while(scanf("%%d %%d",&y,&x)==2){'
                'float a=orbx::orbx_fast_atan2((float)y,(float)x); unsigned u; __builtin_memcpy(&u,&a,4);'
                'printf("%%u\\n",u);} }\n' % os.path.join(ROOT, "ar_orbslam2_amd", "csrc", "orbx_math.h"))
    subprocess.run(["g++", "-O2", "-ffp-contract=off", src, "-o", exe], check=True)
    rng = np.random.default_rng(0)
    pts = np.concatenate([rng.integers(-3_000_000, 3_000_000, (3000, 2)),
                          rng.integers(-50, 50, (2000, 2)), [[0, 0], [5, 5], [-5, 5], [7, -7]]])
    inp = "\n".join(f"{y} {x}" for y, x in pts)
    out = subprocess.run([exe], input=inp, capture_output=True, text=True, check=True).stdout.split()
    got = np.array([int(v) for v in out], np.uint32)
    ref = np.array([O.fast_atan2(float(y), float(x)) for y, x in pts], np.float32).view(np.uint32)
    assert np.array_equal(got, ref)
