"""ORBextractor — host-side mirror of ORB_SLAM2::ORBextractor over the orbx C ABI.

Same constructor arguments, call signature and getters as the reference
(ORB_SLAM2/include/ORBextractor.h:52-88):

    ex = ORBextractor(nfeatures=1000, scaleFactor=1.2, nlevels=8, iniThFAST=20, minThFAST=7)
    keypoints, descriptors = ex(image, mask=None)        # operator()(image, mask, kps, desc)
    ex.GetScaleFactors(), ex.GetLevels(), ex.mvImagePyramid[l]

`keypoints` is a numpy structured array with cv::KeyPoint's fields (x, y, size, angle,
response, octave, class_id); `descriptors` is an (n, 32) uint8 array (None when there are no
keypoints, like `_descriptors.release()` at ORBextractor.cc:1005-1006).  Work runs on the GPU
through liborbx.so; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _ffi
from ._ffi import KEYPOINT_DTYPE, check, lib, ptr


class ORBextractor:
    HARRIS_SCORE = 0
    FAST_SCORE = 1

    def __init__(self, nfeatures=1000, scaleFactor=1.2, nlevels=8, iniThFAST=20, minThFAST=7,
                 device=0):
        self.params = _ffi.Params(int(nfeatures), float(scaleFactor), int(nlevels),
                                  int(iniThFAST), int(minThFAST))
        self._h = C.c_void_p()
        check("orbx_extractor_create",
              lib().orbx_extractor_create(C.byref(self.params), C.c_int(device), C.byref(self._h)))
        n = int(nlevels)
        self._scale = np.zeros(n, np.float32)
        self._inv_scale = np.zeros(n, np.float32)
        self._sigma2 = np.zeros(n, np.float32)
        self._inv_sigma2 = np.zeros(n, np.float32)
        self._fpl = np.zeros(n, np.int32)
        nl = C.c_int32()
        check("orbx_extractor_tables",
              lib().orbx_extractor_tables(self._h, C.byref(nl), ptr(self._scale),
                                          ptr(self._inv_scale), ptr(self._sigma2),
                                          ptr(self._inv_sigma2), ptr(self._fpl)))
        self.nlevels = nl.value
        self._cap = 0
        self._kps = None
        self._desc = None

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            lib().orbx_extractor_destroy(h)
            self._h = None

    # -- getters (ORBextractor.h:64-86)
    def GetLevels(self):
        return self.nlevels

    def GetScaleFactor(self):
        return float(np.float32(self.params.scale_factor))

    def GetScaleFactors(self):
        return self._scale.copy()

    def GetInverseScaleFactors(self):
        return self._inv_scale.copy()

    def GetScaleSigmaSquares(self):
        return self._sigma2.copy()

    def GetInverseScaleSigmaSquares(self):
        return self._inv_sigma2.copy()

    @property
    def mnFeaturesPerLevel(self):
        return self._fpl.copy()

    # -- operator() (ORBextractor.cc:985-1045)
    def __call__(self, image, mask=None):
        """Returns (keypoints, descriptors).  An empty image returns (None, None): the
        reference leaves its outputs untouched in that case (:987-988)."""
        img = np.asarray(image)
        if img.size == 0:
            return None, None
        if img.dtype != np.uint8 or img.ndim != 2:
            raise ValueError("ORBextractor expects a single-channel uint8 image (CV_8UC1)")
        img = np.ascontiguousarray(img)
        h, w = img.shape
        n = C.c_int32(0)
        while True:
            if self._cap == 0:
                self._grow(4 * self.params.nfeatures + 64)
            rc = lib().orbx_extract(self._h, ptr(img), C.c_int32(w), C.c_int32(h),
                                    C.c_int64(img.strides[0]), ptr(self._kps), ptr(self._desc),
                                    C.c_int32(self._cap), C.byref(n))
            if rc == -4:  # ORBX_ECAPACITY
                self._grow(n.value)
                continue
            check("orbx_extract", rc)
            break
        k = n.value
        if k <= 0:
            return np.zeros(0, KEYPOINT_DTYPE), None
        return self._kps[:k].copy(), self._desc[:k].copy()

    def _grow(self, cap):
        self._cap = int(cap)
        self._kps = np.zeros(self._cap, KEYPOINT_DTYPE)
        self._desc = np.zeros((self._cap, 32), np.uint8)

    @property
    def mvImagePyramid(self):
        """Pyramid ROIs of the last call (ORBextractor.h:88), exported lazily from HBM."""
        out = []
        for l in range(self.nlevels):
            w, h = C.c_int32(), C.c_int32()
            check("orbx_extractor_pyramid",
                  lib().orbx_extractor_pyramid(self._h, C.c_int32(l), None, C.c_int64(0),
                                               C.byref(w), C.byref(h)))
            a = np.zeros((h.value, w.value), np.uint8)
            check("orbx_extractor_pyramid",
                  lib().orbx_extractor_pyramid(self._h, C.c_int32(l), ptr(a), C.c_int64(w.value),
                                               C.byref(w), C.byref(h)))
            out.append(a)
        return out
