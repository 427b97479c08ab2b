"""The AR marker path over the orbx C ABI: cv::ORB, BruteForceMatcher<HammingLUT> and Marker.

Mirrors what the reference's AR code calls:

    orb = ORB()                                    # cv::ORB() defaults: 500, 1.2f, 8, 31, 0, 2,
    keypoints, descriptors = orb(image)            #   HARRIS_SCORE, 31 (OpenCV 2.4 orb.cpp)
    matches = BruteForceMatcher().match(d1, d2)    # Marker.cc:110-113
    good, min_dist, max_dist = good_matches(matches)        # Marker.cc:115-133
    matches, minD, maxD = naive_nn_search2(d1, d2)           # AR-1.3/src/ORBMatcher.cpp:70-102

    mk = Marker(); mk.setTargetImage(target); good = mk.Match(frame)   # Marker.cc:76-84, 98-133

and the batched, device-resident throughput path (MarkerBatch: a batch of frames in HBM
matched against one target, everything on the GPU stream).  Keypoints come back as numpy
structured arrays with cv::KeyPoint's fields, matches with cv::DMatch's; all work runs in
liborbx.so on the GPU, with no CPU fallback.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _ffi
from ._ffi import DMATCH_DTYPE, KEYPOINT_DTYPE, check, lib, ptr

HARRIS_SCORE = 0
FAST_SCORE = 1


def cvorb_params(nfeatures=500, scaleFactor=1.2, nlevels=8, edgeThreshold=31, firstLevel=0,
                 WTA_K=2, scoreType=HARRIS_SCORE, patchSize=31):
    return _ffi.CvorbParams(int(nfeatures), float(scaleFactor), int(nlevels), int(edgeThreshold),
                            int(firstLevel), int(WTA_K), int(scoreType), int(patchSize))


class ORB:
    """cv::ORB (OpenCV 2.4) with the same constructor arguments; `orb(image)` is
    `orb(image, Mat(), keypoints, descriptors)`.  An empty image returns (None, None) (orb.cpp
    returns before touching its outputs); no keypoints gives (empty, None)."""

    kBytes = 32
    HARRIS_SCORE = HARRIS_SCORE
    FAST_SCORE = FAST_SCORE

    def __init__(self, nfeatures=500, scaleFactor=1.2, nlevels=8, edgeThreshold=31, firstLevel=0,
                 WTA_K=2, scoreType=HARRIS_SCORE, patchSize=31, device=0, size=(640, 480),
                 max_batch=1):
        self.params = cvorb_params(nfeatures, scaleFactor, nlevels, edgeThreshold, firstLevel,
                                   WTA_K, scoreType, patchSize)
        self._h = C.c_void_p()
        check("orbx_cvorb_create",
              lib().orbx_cvorb_create(C.byref(self.params), C.c_int32(size[0]),
                                      C.c_int32(size[1]), C.c_int32(max_batch), C.c_int(device),
                                      C.byref(self._h)))
        self._cap = 0
        self._kps = None
        self._desc = None

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            lib().orbx_cvorb_destroy(self._h)
        self._h = None

    def __del__(self):
        self.close()

    def descriptorSize(self):
        return self.kBytes

    def __call__(self, image, mask=None):
        img = np.asarray(image)
        if img.size == 0:
            return None, None
        if img.dtype != np.uint8 or img.ndim != 2:
            raise ValueError("ORB expects a single-channel uint8 image")
        img = np.ascontiguousarray(img)
        h, w = img.shape
        n = C.c_int32(0)
        while True:
            if self._cap == 0:
                self._grow(2 * self.params.nfeatures + 256)
            rc = lib().orbx_cvorb_detect(self._h, ptr(img), C.c_int32(w), C.c_int32(h),
                                         C.c_int64(img.strides[0]), ptr(self._kps),
                                         ptr(self._desc), C.c_int32(self._cap), C.byref(n))
            if rc == -4 and n.value > self._cap:  # ORBX_ECAPACITY: grow and run again
                self._grow(n.value)
                continue
            check("orbx_cvorb_detect", rc)
            break
        k = n.value
        if k <= 0:
            return np.zeros(0, KEYPOINT_DTYPE), None
        return self._kps[:k].copy(), self._desc[:k].copy()

    def _grow(self, cap):
        self._cap = int(cap)
        self._kps = np.zeros(self._cap, KEYPOINT_DTYPE)
        self._desc = np.zeros((self._cap, 32), np.uint8)

    # -- batched device path: n dense h x w images at a device pointer
    def run(self, d_imgs_ptr, n):
        check("orbx_cvorb_run", lib().orbx_cvorb_run(self._h, C.c_void_p(d_imgs_ptr), C.c_int32(n)))

    def sync(self):
        check("orbx_cvorb_sync", lib().orbx_cvorb_sync(self._h))

    def capacity(self):
        c = C.c_int32()
        check("orbx_cvorb_capacity", lib().orbx_cvorb_capacity(self._h, C.byref(c)))
        return c.value

    def device_outputs(self):
        ptrs = [C.c_void_p() for _ in range(3)]
        check("orbx_cvorb_outputs", lib().orbx_cvorb_outputs(self._h, *[C.byref(p) for p in ptrs]))
        return {k: p.value for k, p in zip(["kps", "desc", "counts"], ptrs)}

    def stream(self):
        return lib().orbx_cvorb_stream(self._h)


def _desc(d):
    if d is None:
        return np.zeros((0, 32), np.uint8)
    d = np.ascontiguousarray(d, np.uint8)
    if d.ndim != 2 or d.shape[1] != 32:
        raise ValueError("descriptors must be (n, 32) uint8")
    return d


class BruteForceMatcher:
    """BruteForceMatcher<HammingLUT> (OpenCV 2.4 legacy = BFMatcher(NORM_HAMMING)).match."""

    def match(self, query, train):
        q, t = _desc(query), _desc(train)
        out = np.zeros(max(len(q), 1), DMATCH_DTYPE)
        n = C.c_int32()
        check("orbx_bf_match", lib().orbx_bf_match(ptr(q), C.c_int32(len(q)), ptr(t),
                                                   C.c_int32(len(t)), ptr(out), C.byref(n)))
        return out[:n.value].copy()


def good_matches(matches):
    """Marker::Match's filter (Marker.cc:115-133): (good, min_dist, max_dist)."""
    m = np.ascontiguousarray(matches, DMATCH_DTYPE)
    good = np.zeros(max(len(m), 1), DMATCH_DTYPE)
    n = C.c_int32()
    mn, mx = C.c_double(), C.c_double()
    check("orbx_good_matches", lib().orbx_good_matches(ptr(m), C.c_int32(len(m)), ptr(good),
                                                       C.byref(n), C.byref(mn), C.byref(mx)))
    return good[:n.value].copy(), mn.value, mx.value


def nn_match(query, train, ratio=0.8, max_dist=50):
    """naive_nn_search2 (ratio > 0) / naive_nn_search (ratio <= 0), AR-1.3/src/ORBMatcher.cpp:
    44-102; query = descp2 (keys2), train = descp1 (keys1).  Returns (matches, minD, maxD) with
    minD / maxD over this call's pairs merged into the reference's initial 100 / 0."""
    q, t = _desc(query), _desc(train)
    out = np.zeros(max(len(q), 1), DMATCH_DTYPE)
    n, mn, mx = C.c_int32(), C.c_int32(), C.c_int32()
    check("orbx_nn_match", lib().orbx_nn_match(ptr(q), C.c_int32(len(q)), ptr(t),
                                               C.c_int32(len(t)), C.c_double(ratio),
                                               C.c_int32(max_dist), ptr(out), C.byref(n),
                                               C.byref(mn), C.byref(mx)))
    return out[:n.value].copy(), mn.value, mx.value


def naive_nn_search2(descp1, descp2):
    return nn_match(descp2, descp1, 0.8, 50)


def naive_nn_search(descp1, descp2):
    return nn_match(descp2, descp1, 0.0, 50)


class Marker:
    """Marker::setTargetImage / Marker::Match up to the good-match list (Marker.cc:76-133).
    The homography / projection-error tail of Marker::Match (calib3d RANSAC) stays with the
    caller."""

    def __init__(self, device=0):
        self.orb = ORB(device=device)
        self.matcher = BruteForceMatcher()
        self.mvKeys1 = None
        self.mDescriptors1 = None

    def setTargetImage(self, image):
        self.mvKeys1, self.mDescriptors1 = self.orb(image)

    def Match(self, image):
        """Returns (ok, good_matches, matches, keypoints2, descriptors2)."""
        kps2, d2 = self.orb(image)
        if self.mDescriptors1 is None or d2 is None:  # "image invalid." (Marker.cc:115-118)
            return False, np.zeros(0, DMATCH_DTYPE), np.zeros(0, DMATCH_DTYPE), kps2, d2
        matches = self.matcher.match(self.mDescriptors1, d2)
        good, _, _ = good_matches(matches)
        return True, good, matches, kps2, d2


class MarkerBatch:
    """Marker::Match for a batch of frames already in HBM against one target (orbx_marker):
    cv::ORB of every frame, BruteForceMatcher match (query = target) and the good flags, all on
    the device stream."""

    def __init__(self, w, h, max_batch, nfeatures=500, scoreType=HARRIS_SCORE, device=0):
        self.w, self.h, self.max_batch = int(w), int(h), int(max_batch)
        self.params = cvorb_params(nfeatures, scoreType=scoreType)
        self._h = C.c_void_p()
        check("orbx_marker_create",
              lib().orbx_marker_create(C.byref(self.params), C.c_int32(self.w), C.c_int32(self.h),
                                       C.c_int32(self.max_batch), C.c_int(device),
                                       C.byref(self._h)))
        self.n_target = 0

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            lib().orbx_marker_destroy(self._h)
        self._h = None

    def __del__(self):
        self.close()

    def set_target(self, descriptors):
        d = _desc(descriptors)
        check("orbx_marker_set_target", lib().orbx_marker_set_target(self._h, ptr(d),
                                                                     C.c_int32(len(d))))
        self.n_target = len(d)

    def run(self, d_imgs_ptr, n):
        check("orbx_marker_run", lib().orbx_marker_run(self._h, C.c_void_p(d_imgs_ptr),
                                                       C.c_int32(n)))

    def sync(self):
        check("orbx_marker_sync", lib().orbx_marker_sync(self._h))

    def results(self, n):
        kp = np.zeros(n, np.int32)
        good = np.zeros(n, np.int32)
        check("orbx_marker_results", lib().orbx_marker_results(self._h, C.c_int32(n), ptr(kp),
                                                               ptr(good)))
        return kp, good

    def device_outputs(self):
        ptrs = [C.c_void_p() for _ in range(4)]
        check("orbx_marker_outputs", lib().orbx_marker_outputs(self._h, *[C.byref(p) for p in ptrs]))
        return {k: p.value for k, p in zip(["matches", "good", "kps", "desc"], ptrs)}

    def stream(self):
        return lib().orbx_marker_stream(self._h)

    def profile(self, enable=True):
        check("orbx_marker_profile", lib().orbx_marker_profile(self._h, C.c_int32(int(enable))))

    def profile_read(self):
        cap = 32
        names = (C.c_char * 32 * cap)()
        ms = np.zeros(cap, np.float64)
        launches = np.zeros(cap, np.int64)
        n = C.c_int32()
        check("orbx_marker_profile_read",
              lib().orbx_marker_profile_read(self._h, C.c_int32(cap), names, ptr(ms),
                                             ptr(launches), C.byref(n)))
        return {bytes(names[i]).split(b"\0")[0].decode(): (float(ms[i]), int(launches[i]))
                for i in range(n.value)}

    def profile_kernels(self):
        """{stage: kernel instances the profiled runs launched for it} (profile_read's stages)."""
        return _ffi.profile_kernels("orbx_marker_profile_kernels", self._h,
                                    list(self.profile_read()))
