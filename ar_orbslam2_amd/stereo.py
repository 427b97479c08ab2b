"""Frame::ComputeStereoMatches (ORB_SLAM2/src/Frame.cc:471-643) over two ORBextractor mirrors.

    left, right = ORBextractor(1200), ORBextractor(1200)
    kl, dl = left(imLeft); kr, dr = right(imRight)
    mvuRight, mvDepth = ComputeStereoMatches(left, right, mb, mbf)

Runs on the last extraction of each extractor, whose keypoints, descriptors and
mvImagePyramid are still resident on the GPU (orbx_stereo_matches, include/orbx.h).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._ffi import check, lib, ptr


def stereo_params(bf, fx):
    """(mb, mbf) as Tracking/Frame compute them: mbf = (float)Camera.bf, mb = mbf / fx."""
    mbf = np.float32(bf)
    mb = np.float32(mbf / np.float32(fx))
    return float(mb), float(mbf)


def ComputeStereoMatches(left, right, mb, mbf):
    cap = max(left._cap, 1)
    ur = np.zeros(cap, np.float32)
    dp = np.zeros(cap, np.float32)
    n = C.c_int32()
    check("orbx_stereo_matches",
          lib().orbx_stereo_matches(left._h, right._h, C.c_float(mb), C.c_float(mbf), ptr(ur),
                                    ptr(dp), C.byref(n)))
    return ur[:n.value].copy(), dp[:n.value].copy()
