"""ar_orbslam2_amd — MI355X-native ORB front end for ORB-SLAM2 (extract + BoW matching).

Drop-in for the reference hot path (ORB_SLAM2/src/ORBextractor.cc, ORBmatcher.cc): the
ORBextractor / ORBmatcher classes mirror the reference interfaces over the C ABI in
include/orbx.h, implemented by hand-written gfx950 HIP kernels in csrc/ (liborbx.so).
"""
from ._ffi import KEYPOINT_DTYPE, LIB_PATH, OrbxError, lib  # noqa: F401
from .extractor import ORBextractor  # noqa: F401
from .matcher import ORBmatcher, epipole  # noqa: F401
from .vocabulary import FeatureVector, Vocabulary  # noqa: F401

__all__ = ["ORBextractor", "ORBmatcher", "FeatureVector", "Vocabulary", "epipole",
           "KEYPOINT_DTYPE", "OrbxError", "lib", "LIB_PATH"]
