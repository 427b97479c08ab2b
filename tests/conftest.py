import os
import sys

import pytest

# torch brings up its bundled HIP runtime first in every test process: liborbx binds to the
# libamdhip64.so.7 already loaded (same soname), so the process runs one HIP runtime.  Loaded the
# other way round (liborbx first: /opt/rocm's runtime), torch's later CUDA init finds no GPU
# ("No HIP GPUs are available"), which a -m gpu subset starting with a ctypes-only test file hit.
import torch  # noqa: E402,F401

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(ROOT, "tests", "golden")
