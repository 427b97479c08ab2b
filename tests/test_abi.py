"""The drop-in boundary: liborbx.so (HIP, gfx950) loads without a GPU and exports every
function include/orbx.h declares; host-only entry points behave without touching the device."""
import ctypes as C
import os
import re

import numpy as np
import pytest

import ar_orbslam2_amd as A
from ar_orbslam2_amd import _ffi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared():
    txt = open(os.path.join(ROOT, "include", "orbx.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(orbx_[a-z0-9_]+)\s*\(", txt)))


def test_header_lists_the_python_exports():
    assert set(_ffi.EXPORTS) <= set(declared())


def test_library_exports_every_declared_symbol():
    lib = A.lib()
    missing = [s for s in declared() if not hasattr(lib, s)]
    assert not missing, missing


def test_library_is_gfx950_code_object():
    data = open(A.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_struct_layouts():
    assert A.KEYPOINT_DTYPE.itemsize == 28  # cv::KeyPoint
    assert [A.KEYPOINT_DTYPE.fields[f][1] for f in ("x", "y", "size", "angle", "response", "octave",
                                                    "class_id")] == [0, 4, 8, 12, 16, 20, 24]
    assert C.sizeof(_ffi.Params) == 20
    assert C.sizeof(_ffi.FeatVec) == 32


def test_extractor_tables_without_gpu():
    ex = A.ORBextractor(1000, 1.2, 8, 20, 7)
    from oracle import oracle as O
    t = O.tables(O.params())
    np.testing.assert_array_equal(ex.GetScaleFactors(), t["scale"])
    np.testing.assert_array_equal(ex.GetInverseScaleFactors(), t["inv_scale"])
    np.testing.assert_array_equal(ex.GetScaleSigmaSquares(), t["sigma2"])
    np.testing.assert_array_equal(ex.GetInverseScaleSigmaSquares(), t["inv_sigma2"])
    np.testing.assert_array_equal(ex.mnFeaturesPerLevel, t["features_per_level"])
    assert ex.GetLevels() == 8 and ex.GetScaleFactor() == pytest.approx(1.2)


def test_invalid_arguments_are_reported():
    lib = A.lib()
    h = C.c_void_p()
    bad = _ffi.Params(1000, 1.2, 0, 20, 7)
    assert lib.orbx_extractor_create(C.byref(bad), 0, C.byref(h)) == -1
    assert lib.orbx_search_by_bow_kf_f(None, None, C.c_float(0.7), 1, None, None) == -1
    with pytest.raises(A.OrbxError):
        A.ORBextractor(1000, 1.2, 0)


def test_search_entry_points_reject_bad_arguments_without_a_gpu():
    """Argument checks of the projection-family entry points run before any device work
    (null structs, a predicted level outside the pyramid, SearchBySim3 point sets that are not
    one per keypoint): ORBX_EINVAL (-1)."""
    lib = A.lib()
    n = C.c_int32()
    assert lib.orbx_search_by_projection_kf(None, None, C.c_float(10), 100, 1, None, C.byref(n)) == -1
    assert lib.orbx_search_by_projection_sim3(None, None, C.c_float(10), None, C.byref(n)) == -1
    assert lib.orbx_search_by_sim3(None, None, None, None, C.c_float(7.5), None, C.byref(n)) == -1
    scale = np.ones(8, np.float32)
    kp = np.zeros(2, A.KEYPOINT_DTYPE)
    desc = np.zeros((2, 32), np.uint8)
    fr = _ffi.ProjFrame(2, kp.ctypes.data, desc.ctypes.data, None, None, 0.0, 0.0, 640.0, 480.0,
                        0.1, 0.1, scale.ctypes.data, 8)
    use = np.ones(1, np.uint8)
    u = np.zeros(1, np.float32)
    lev = np.array([9], np.int32)  # outside the 8-level pyramid
    pd = np.zeros((1, 32), np.uint8)
    pts = _ffi.FusePoints(1, use.ctypes.data, u.ctypes.data, u.ctypes.data, None, lev.ctypes.data,
                          pd.ctypes.data)
    match = np.zeros(2, np.int32)
    assert lib.orbx_search_by_projection_sim3(C.byref(fr), C.byref(pts), C.c_float(10),
                                              match.ctypes.data, C.byref(n)) == -1
    lev[0] = 0
    m12 = np.zeros(2, np.int32)
    # one point for a 2-keypoint keyframe: not one entry per keypoint
    assert lib.orbx_search_by_sim3(C.byref(fr), C.byref(fr), C.byref(pts), C.byref(pts),
                                   C.c_float(7.5), m12.ctypes.data, C.byref(n)) == -1


def test_empty_image_returns_untouched():
    ex = A.ORBextractor()
    assert ex(np.zeros((0, 0), np.uint8)) == (None, None)


def test_epipole_helper_matches_oracle():
    from oracle import oracle as O
    R = np.array([[0.99, -0.1, 0.02], [0.1, 0.99, 0.01], [-0.02, 0.0, 1.0]], np.float32)
    args = (R, [0.1, 0.02, 0.05], [0.3, -0.2, 1.5], 517.3, 516.5, 318.6, 255.3)
    assert A.epipole(*args) == O.epipole(*args)
