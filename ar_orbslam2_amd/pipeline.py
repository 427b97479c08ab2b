"""FramePipeline — the batched, device-resident "ORB extract + match" unit of work.

Wraps orbx_frames (include/orbx.h): per batch of n frames already in HBM it runs the
extractor, Frame::ComputeBoW (vocabulary descent, BowVector, FeatureVector), SearchByBoW(prev-as-KF, cur) and
SearchForTriangulation(prev-as-KF, cur-as-KF) (SURVEY §8d unit of work), entirely on the GPU
stream of the pipeline.  Frame f is matched against frame (f-1) mod n of the same batch.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _ffi
from ._ffi import check, lib, ptr

TUM1_K = (517.306408, 516.469215, 318.643040, 255.313989)  # Examples/Monocular/TUM1.yaml


def fundamental_from_pose(K=TUM1_K, t=(0.10, 0.02, 0.05)):
    """F12 = K^-T [t]x R K^-1 for R = I (LocalMapping::ComputeF12 with a fixed synthetic pose)."""
    fx, fy, cx, cy = K
    Km = np.array([[fx, 0, cx], [0, fy, cy], [0, 0, 1]], np.float32)
    tx = np.array([[0, -t[2], t[1]], [t[2], 0, -t[0]], [-t[1], t[0], 0]], np.float32)
    Kinv = np.linalg.inv(Km).astype(np.float32)
    return (Kinv.T @ tx @ Kinv).astype(np.float32)


class FramePipeline:
    def __init__(self, w, h, max_batch, vocabulary, nfeatures=1000, scale_factor=1.2, nlevels=8,
                 ini_th_fast=20, min_th_fast=7, device=0, levelsup=4, stereo=None):
        """stereo=(mb, mbf) makes a stereo pipeline: a frame is an interleaved (left, right)
        image pair, so `run` takes 2n images for n frames."""
        self.w, self.h, self.max_batch = int(w), int(h), int(max_batch)
        self.params = _ffi.Params(int(nfeatures), float(scale_factor), int(nlevels),
                                  int(ini_th_fast), int(min_th_fast))
        self.voc = vocabulary
        self.stereo = stereo is not None
        self._h = C.c_void_p()
        if self.stereo:
            check("orbx_frames_create_stereo",
                  lib().orbx_frames_create_stereo(C.byref(self.params), C.c_int32(self.w),
                                                  C.c_int32(self.h), C.c_int32(self.max_batch),
                                                  vocabulary.handle, C.c_int32(levelsup),
                                                  C.c_float(stereo[0]), C.c_float(stereo[1]),
                                                  C.c_int(device), C.byref(self._h)))
        else:
            check("orbx_frames_create",
                  lib().orbx_frames_create(C.byref(self.params), C.c_int32(self.w),
                                           C.c_int32(self.h), C.c_int32(self.max_batch),
                                           vocabulary.handle, C.c_int32(levelsup),
                                           C.c_int(device), C.byref(self._h)))
        cap = C.c_int32()
        check("orbx_frames_capacity", lib().orbx_frames_capacity(self._h, C.byref(cap)))
        self.kp_cap = cap.value

    def close(self):
        if self._h is not None and self._h.value:
            lib().orbx_frames_destroy(self._h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_masks(self, valid=None, has_mp=None):
        shape = (self.max_batch, self.kp_cap)
        v = None if valid is None else np.ascontiguousarray(np.broadcast_to(valid, shape), np.uint8)
        m = None if has_mp is None else np.ascontiguousarray(np.broadcast_to(has_mp, shape), np.uint8)
        check("orbx_frames_set_masks", lib().orbx_frames_set_masks(self._h, ptr(v), ptr(m)))

    def seeded_masks(self, frame_ids, valid_frac=0.6, mp_frac=0.4):
        """KF-side 'valid MapPoint' on 60 % and 'has MapPoint' on 40 % of
        features, seeded by frame index."""
        valid = np.zeros((self.max_batch, self.kp_cap), np.uint8)
        has_mp = np.zeros((self.max_batch, self.kp_cap), np.uint8)
        for slot, fid in enumerate(frame_ids):
            rng = np.random.default_rng(int(fid))
            valid[slot] = rng.random(self.kp_cap) < valid_frac
            has_mp[slot] = rng.random(self.kp_cap) < mp_frac
        self.set_masks(valid, has_mp)
        return valid, has_mp

    def set_matching(self, F12, epipole, bow_ratio=0.7, bow_check_ori=True, tri_ratio=0.6,
                     tri_check_ori=False, only_stereo=False):
        F = np.ascontiguousarray(F12, np.float32).reshape(9)
        check("orbx_frames_set_matching",
              lib().orbx_frames_set_matching(self._h, C.c_float(bow_ratio),
                                             C.c_int32(int(bow_check_ori)), ptr(F),
                                             C.c_float(epipole[0]), C.c_float(epipole[1]),
                                             C.c_float(tri_ratio), C.c_int32(int(tri_check_ori)),
                                             C.c_int32(int(only_stereo))))

    def run(self, d_imgs_ptr, n):
        """Enqueue one batch of n frames; `d_imgs_ptr` is a device pointer to n dense h*w uint8
        images (2n, interleaved left/right, for a stereo pipeline)."""
        check("orbx_frames_run", lib().orbx_frames_run(self._h, C.c_void_p(d_imgs_ptr),
                                                       C.c_int32(n)))

    def sync(self):
        check("orbx_frames_sync", lib().orbx_frames_sync(self._h))

    def results(self, n):
        kp = np.zeros(n, np.int32)
        bow = np.zeros(n, np.int32)
        tri = np.zeros(n, np.int32)
        err = np.zeros(1, np.int32)
        check("orbx_frames_results",
              lib().orbx_frames_results(self._h, C.c_int32(n), ptr(kp), ptr(bow), ptr(tri),
                                        ptr(err)))
        return kp, bow, tri, int(err[0])

    def device_outputs(self):
        names = ["kps", "desc", "counts", "node_of", "bow_match", "tri_pairs"]
        ptrs = [C.c_void_p() for _ in names]
        check("orbx_frames_outputs", lib().orbx_frames_outputs(self._h, *[C.byref(p) for p in ptrs]))
        return {k: p.value for k, p in zip(names, ptrs)}

    def bow_outputs(self):
        names = ["bow_words", "bow_values", "bow_n", "word_of"]
        ptrs = [C.c_void_p() for _ in names]
        check("orbx_frames_bow", lib().orbx_frames_bow(self._h, *[C.byref(p) for p in ptrs]))
        return {k: p.value for k, p in zip(names, ptrs)}

    def stereo_outputs(self):
        ur, dp = C.c_void_p(), C.c_void_p()
        check("orbx_frames_stereo", lib().orbx_frames_stereo(self._h, C.byref(ur), C.byref(dp)))
        return {"uright": ur.value, "depth": dp.value}

    def stream(self):
        return lib().orbx_frames_stream(self._h)

    def profile(self, enable=True):
        check("orbx_frames_profile", lib().orbx_frames_profile(self._h, C.c_int32(int(enable))))

    def profile_read(self):
        cap = 32
        names = (C.c_char * 32 * cap)()
        ms = np.zeros(cap, np.float64)
        launches = np.zeros(cap, np.int64)
        n = C.c_int32()
        check("orbx_frames_profile_read",
              lib().orbx_frames_profile_read(self._h, C.c_int32(cap), names, ptr(ms), ptr(launches),
                                             C.byref(n)))
        return {bytes(names[i]).split(b"\0")[0].decode(): (float(ms[i]), int(launches[i]))
                for i in range(n.value)}

    def profile_kernels(self):
        """{stage: kernel instances the profiled runs launched for it} (profile_read's stages)."""
        return _ffi.profile_kernels("orbx_frames_profile_kernels", self._h,
                                    list(self.profile_read()))
