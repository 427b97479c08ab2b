"""The device build of the glibc sincosf port (ar_orbslam2_amd/csrc/orbx_math.h, used by
k_describe for computeOrbDescriptor, ORBextractor.cc:103-104) against the host libm for every
float in [0, 2*pi*(1+eps)] — the angles `kpt.angle * (float)(CV_PI/180.f)` can take.  The
host build is checked exhaustively in tests/test_math_port.py; this pins the gfx950 code."""
import ctypes as C

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

HI = 0x40C90FE0  # just past 360 deg * (float)(pi/180) = 6.2831855


def test_device_sincosf_exhaustive():
    from ar_orbslam2_amd._ffi import lib
    import platform
    chunk = 1 << 25
    s = np.empty(chunk, np.float32)
    c = np.empty(chunk, np.float32)
    bad = 0
    for lo in range(0, HI, chunk):
        n = min(chunk, HI - lo)
        rc = lib().orbx_debug_sincosf(C.c_uint32(lo), C.c_int64(n), C.c_void_p(s.ctypes.data),
                                      C.c_void_p(c.ctypes.data))
        assert rc == 0
        rs, rcos = O.sincosf_bits(lo, n)
        bad += int((s[:n].view(np.uint32) != rs.view(np.uint32)).sum())
        bad += int((c[:n].view(np.uint32) != rcos.view(np.uint32)).sum())
    print("glibc", platform.libc_ver())
    assert bad == 0
