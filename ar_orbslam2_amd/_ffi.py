"""ctypes binding of liborbx.so (include/orbx.h).

The product path has exactly one implementation: the HIP library built from
ar_orbslam2_amd/csrc for gfx950.  If the library is missing this module raises — there is
no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_lib", "liborbx.so")
# experiments only: ORBX_LIB_DIR names another build directory (a variant built from an
# experiment copy of the sources, `make OUT=<dir>`); it needs ORBX_ALLOW_CUSTOM_BUILD=1 like any
# custom build, and such a library is not checked against the tree's sources
EXPERIMENT_LIB = bool(os.environ.get("ORBX_LIB_DIR") and os.environ.get("ORBX_ALLOW_CUSTOM_BUILD"))
if EXPERIMENT_LIB:
    LIB_PATH = os.path.join(os.environ["ORBX_LIB_DIR"], "liborbx.so")

KEYPOINT_DTYPE = np.dtype(
    [("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"), ("response", "<f4"),
     ("octave", "<i4"), ("class_id", "<i4")])

ERRORS = {-1: "ORBX_EINVAL", -2: "ORBX_ENOMEM", -3: "ORBX_EDEVICE", -4: "ORBX_ECAPACITY",
          -5: "ORBX_EUNSUPPORTED"}
ORBX_ECAPACITY = -4

EXPORTS = [
    "orbx_extractor_create", "orbx_extractor_destroy", "orbx_extractor_tables", "orbx_extract",
    "orbx_extractor_pyramid", "orbx_plan_create", "orbx_plan_destroy", "orbx_plan_capacity",
    "orbx_plan_extract", "orbx_plan_outputs", "orbx_plan_sync", "orbx_plan_stream",
    "orbx_plan_profile", "orbx_plan_profile_read", "orbx_plan_profile_kernels",
    "orbx_descriptor_distance",
    "orbx_search_by_bow_kf_f", "orbx_search_by_bow_kf_kf", "orbx_search_for_triangulation",
    "orbx_epipole", "orbx_search_by_projection", "orbx_search_by_projection_last",
    "orbx_search_for_initialization", "orbx_fuse", "orbx_fuse_sim3",
    "orbx_search_by_projection_kf", "orbx_search_by_projection_sim3", "orbx_search_by_sim3",
    "orbx_stereo_matches", "orbx_vocabulary_load_text", "orbx_vocabulary_create",
    "orbx_vocabulary_destroy", "orbx_vocabulary_info", "orbx_vocabulary_transform",
    "orbx_frames_create", "orbx_frames_create_stereo", "orbx_frames_destroy",
    "orbx_frames_capacity", "orbx_frames_set_masks", "orbx_frames_set_matching",
    "orbx_frames_run", "orbx_frames_sync", "orbx_frames_results", "orbx_frames_outputs",
    "orbx_frames_bow", "orbx_frames_stereo", "orbx_frames_stream", "orbx_frames_profile", "orbx_frames_profile_read",
    "orbx_frames_profile_kernels",
    "orbx_cvorb_create", "orbx_cvorb_destroy", "orbx_cvorb_capacity", "orbx_cvorb_detect",
    "orbx_cvorb_run", "orbx_cvorb_outputs", "orbx_cvorb_sync", "orbx_cvorb_stream",
    "orbx_bf_match", "orbx_good_matches", "orbx_nn_match", "orbx_marker_create",
    "orbx_marker_destroy", "orbx_marker_set_target", "orbx_marker_run", "orbx_marker_sync",
    "orbx_marker_results", "orbx_marker_outputs", "orbx_marker_stream", "orbx_marker_profile",
    "orbx_marker_profile_read", "orbx_marker_profile_kernels", "orbx_debug_cvorb_cossin", "orbx_debug_retain_best",
    "orbx_debug_match_finish", "orbx_debug_bow_kernel", "orbx_debug_sincosf", "orbx_debug_extractor_blur",
    "orbx_debug_plan_level",
]

# == cv::DMatch (OpenCV 2.4): queryIdx, trainIdx, imgIdx, distance
DMATCH_DTYPE = np.dtype([("query_idx", "<i4"), ("train_idx", "<i4"), ("img_idx", "<i4"),
                         ("distance", "<f4")])


class OrbxError(RuntimeError):
    def __init__(self, fn, rc):
        super().__init__(f"{fn} failed: {ERRORS.get(rc, rc)}")
        self.rc = rc


class Params(C.Structure):
    _fields_ = [("nfeatures", C.c_int32), ("scale_factor", C.c_float), ("nlevels", C.c_int32),
                ("ini_th_fast", C.c_int32), ("min_th_fast", C.c_int32)]


class CvorbParams(C.Structure):
    """cv::ORB constructor arguments (OpenCV 2.4 features2d.hpp), include/orbx.h."""
    _fields_ = [("nfeatures", C.c_int32), ("scale_factor", C.c_float), ("nlevels", C.c_int32),
                ("edge_threshold", C.c_int32), ("first_level", C.c_int32), ("wta_k", C.c_int32),
                ("score_type", C.c_int32), ("patch_size", C.c_int32)]


class FeatVec(C.Structure):
    _fields_ = [("n_nodes", C.c_int32), ("node_ids", C.c_void_p), ("node_offsets", C.c_void_p),
                ("node_feats", C.c_void_p)]


class BowSide(C.Structure):
    _fields_ = [("n", C.c_int32), ("desc", C.c_void_p), ("angle", C.c_void_p),
                ("valid", C.c_void_p), ("fv", FeatVec)]


class TriSide(C.Structure):
    _fields_ = [("n", C.c_int32), ("desc", C.c_void_p), ("keys_un", C.c_void_p),
                ("u_right", C.c_void_p), ("has_mp", C.c_void_p), ("fv", FeatVec),
                ("scale_factors", C.c_void_p), ("level_sigma2", C.c_void_p),
                ("nlevels", C.c_int32)]


class ProjFrame(C.Structure):
    _fields_ = [("n", C.c_int32), ("keys_un", C.c_void_p), ("desc", C.c_void_p),
                ("u_right", C.c_void_p), ("has_mp_obs", C.c_void_p), ("min_x", C.c_float),
                ("min_y", C.c_float), ("max_x", C.c_float), ("max_y", C.c_float),
                ("grid_w_inv", C.c_float), ("grid_h_inv", C.c_float),
                ("scale_factors", C.c_void_p), ("nlevels", C.c_int32)]


class ProjPoints(C.Structure):
    _fields_ = [("n", C.c_int32), ("track", C.c_void_p), ("proj_x", C.c_void_p),
                ("proj_y", C.c_void_p), ("proj_xr", C.c_void_p), ("pred_level", C.c_void_p),
                ("view_cos", C.c_void_p), ("desc", C.c_void_p)]


class FusePoints(C.Structure):
    _fields_ = [("n", C.c_int32), ("use", C.c_void_p), ("u", C.c_void_p), ("v", C.c_void_p),
                ("ur", C.c_void_p), ("pred_level", C.c_void_p), ("desc", C.c_void_p)]


class ProjLast(C.Structure):
    _fields_ = [("n", C.c_int32), ("valid", C.c_void_p), ("u", C.c_void_p), ("v", C.c_void_p),
                ("ur", C.c_void_p), ("octave", C.c_void_p), ("angle", C.c_void_p),
                ("desc", C.c_void_p), ("blocks", C.c_void_p)]


_lib = None


# the options __graft_entry__.build() compiles with (csrc/Makefile BUILDFLAGS)
DEFAULT_BUILDFLAGS = "ARCH=gfx950:sramecc+ EXTRA="


def source_hash():
    """(sha256 of the sources in liborbx.srclist order and of the build-option line, the hash
    the build recorded, that option line); (None, None, None) if any of them cannot be read."""
    import hashlib
    lib_dir = os.path.dirname(LIB_PATH)
    csrc = os.path.join(_HERE, "csrc")
    try:
        names = open(os.path.join(lib_dir, "liborbx.srclist")).read().split()
        built = open(os.path.join(lib_dir, "liborbx.srchash")).read().strip()
        flags_path = os.path.join(lib_dir, "liborbx.buildflags")
        h = hashlib.sha256()
        for n in names:
            with open(os.path.join(csrc, n), "rb") as f:
                h.update(f.read())
        with open(flags_path, "rb") as f:
            flags = f.read()
        h.update(flags)
    except OSError:
        return None, None, None
    return h.hexdigest(), built, flags.decode(errors="replace").strip()


def lib():
    """Load liborbx.so; raises ImportError if the HIP library has not been built (no fallback),
    was built from other sources than the ones in the tree (Makefile's liborbx.srchash), or with
    other options than the default build (set ORBX_ALLOW_CUSTOM_BUILD=1 for experiments)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} missing: build it with `python -c 'import __graft_entry__ as g; "
                "g.build()'` (hipcc, gfx950). There is no CPU fallback.")
        now, built, flags = source_hash()
        if not EXPERIMENT_LIB and (now is None or now != built):
            raise ImportError(
                f"{LIB_PATH} is stale or its sources are missing: it was built from other "
                f"sources than ar_orbslam2_amd/csrc (hash {built} vs {now}); rebuild with "
                "`python -c 'import __graft_entry__ as g; g.build()'`.")
        if flags != DEFAULT_BUILDFLAGS and not os.environ.get("ORBX_ALLOW_CUSTOM_BUILD"):
            raise ImportError(
                f"{LIB_PATH} was built with non-default options ({flags!r}, default "
                f"{DEFAULT_BUILDFLAGS!r}); rebuild with __graft_entry__.build() or set "
                "ORBX_ALLOW_CUSTOM_BUILD=1.")
        _lib = C.CDLL(LIB_PATH)
        _lib.orbx_plan_stream.restype = C.c_void_p
        _lib.orbx_frames_stream.restype = C.c_void_p
        _lib.orbx_cvorb_stream.restype = C.c_void_p
        _lib.orbx_marker_stream.restype = C.c_void_p
    return _lib


def check(fn, rc):
    if rc != 0:
        raise OrbxError(fn, rc)
    return rc


def ptr(a):
    return None if a is None else C.c_void_p(a.ctypes.data)


def profile_kernels(fn, handle, stage_names):
    """{stage: [kernel instance names]} of a profiled pipeline (orbx_*_profile_kernels: the
    instances launched for each stage, named as rocprofv3 reports them)."""
    out = {}
    cap = 4096
    for i, name in enumerate(stage_names):
        while True:  # ORBX_ECAPACITY: the list does not fit (never returned cut): a larger buffer
            buf = C.create_string_buffer(cap)
            rc = getattr(lib(), fn)(handle, C.c_int32(i), buf, C.c_int32(cap))
            if rc != ORBX_ECAPACITY or cap >= 1 << 20:
                break
            cap *= 4
        check(fn, rc)
        out[name] = [k for k in buf.value.decode().split(";") if k]
    return out
