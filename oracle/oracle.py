"""ctypes binding of the CPU oracle (oracle/orb_oracle.cc).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg as the checker.  The product package (ar_orbslam2_amd) never imports it.
Parity status: see orb_oracle.h — pinned by known-answer tests from the reference's own
tables; parity against real OpenCV 2.4 primitives is unpinned.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liborb_oracle.so")
_lib = None

KEYPOINT_DTYPE = np.dtype(
    [("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"), ("response", "<f4"),
     ("octave", "<i4"), ("class_id", "<i4")])
assert KEYPOINT_DTYPE.itemsize == 28


class Params(C.Structure):
    _fields_ = [("nfeatures", C.c_int32), ("scale_factor", C.c_float), ("nlevels", C.c_int32),
                ("ini_th_fast", C.c_int32), ("min_th_fast", C.c_int32)]


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


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = C.CDLL(_LIB_PATH)
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def params(nfeatures=1000, scale_factor=1.2, nlevels=8, ini_th_fast=20, min_th_fast=7):
    return Params(nfeatures, scale_factor, nlevels, ini_th_fast, min_th_fast)


def extract(img, p=None, tie_mode=0, cap=None, want_pyramid=False):
    """ORBextractor::operator() restated.  Returns (keypoints structured array, desc [n,32])
    or, with want_pyramid, also the list of pyramid levels and pre-octree candidate counts."""
    p = p or params()
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    cap = cap or max(4 * p.nfeatures + 64, 256)
    kps = np.zeros(cap, KEYPOINT_DTYPE)
    desc = np.zeros((cap, 32), np.uint8)
    n = C.c_int(0)
    lw = np.zeros(p.nlevels, np.int32)
    lh = np.zeros(p.nlevels, np.int32)
    ncand = np.zeros(p.nlevels, np.int32)
    pyr_cap = int(w * h * p.nlevels + 1024) if want_pyramid else 0
    pyr = np.zeros(pyr_cap, np.uint8) if want_pyramid else None
    L = lib()
    L.oracle_extract_ex.restype = C.c_int
    rc = L.oracle_extract_ex(C.byref(p), _p(img), C.c_int(w), C.c_int(h), C.c_int64(w),
                             C.c_int(tie_mode), _p(kps), _p(desc), C.c_int(cap), C.byref(n),
                             _p(pyr), C.c_int64(pyr_cap), _p(lw), _p(lh), _p(ncand))
    if rc != 0:
        raise RuntimeError(f"oracle_extract failed rc={rc}")
    k = n.value
    out = (kps[:k].copy(), desc[:k].copy())
    if not want_pyramid:
        return out
    levels, off = [], 0
    for l in range(p.nlevels):
        sz = int(lw[l]) * int(lh[l])
        levels.append(pyr[off:off + sz].reshape(int(lh[l]), int(lw[l])).copy())
        off += sz
    return out + (levels, ncand.copy())


def extract_rc(img, p=None):
    """Status code only (for edge-case tests)."""
    p = p or params()
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape if img.ndim == 2 else (0, 0)
    cap = 4 * p.nfeatures + 64
    kps = np.zeros(cap, KEYPOINT_DTYPE)
    desc = np.zeros((cap, 32), np.uint8)
    n = C.c_int(123456)
    rc = lib().oracle_extract(C.byref(p), _p(img), C.c_int(w), C.c_int(h), C.c_int64(max(w, 1)),
                              C.c_int(0), _p(kps), _p(desc), C.c_int(cap), C.byref(n))
    return rc, n.value


def tables(p=None, w=640, h=480):
    p = p or params()
    n = p.nlevels
    f = lambda: np.zeros(n, np.float32)
    scale, inv, s2, is2 = f(), f(), f(), f()
    fpl = np.zeros(n, np.int32)
    umax = np.zeros(16, np.int32)
    lw = np.zeros(n, np.int32)
    lh = np.zeros(n, np.int32)
    rc = lib().oracle_tables(C.byref(p), _p(scale), _p(inv), _p(s2), _p(is2), _p(fpl), _p(umax),
                             _p(lw), _p(lh), C.c_int(w), C.c_int(h))
    assert rc == 0
    return dict(scale=scale, inv_scale=inv, sigma2=s2, inv_sigma2=is2, features_per_level=fpl,
                umax=umax, level_w=lw, level_h=lh)


def resize_linear(src, dw, dh):
    src = np.ascontiguousarray(src, np.uint8)
    dst = np.zeros((dh, dw), np.uint8)
    lib().oracle_resize_linear(_p(src), C.c_int(src.shape[1]), C.c_int(src.shape[0]),
                               C.c_int64(src.shape[1]), _p(dst), C.c_int(dw), C.c_int(dh),
                               C.c_int64(dw))
    return dst


def gaussian7(src):
    src = np.ascontiguousarray(src, np.uint8)
    dst = np.zeros_like(src)
    lib().oracle_gaussian7(_p(src), C.c_int(src.shape[1]), C.c_int(src.shape[0]), _p(dst))
    return dst


def fast_atan2(y, x):
    f = lib().oracle_fast_atan2
    f.restype = C.c_float
    f.argtypes = [C.c_float, C.c_float]
    return f(y, x)


def sincosf(x):
    s, c = C.c_float(), C.c_float()
    lib().oracle_sincosf(C.c_float(x), C.byref(s), C.byref(c))
    return s.value, c.value


def sincosf_bits(lo, n, threads=None):
    """Host libm sincosf of the n floats with bit patterns lo, lo+1, ... -> (s, c) f32 arrays."""
    s = np.empty(n, np.float32)
    c = np.empty(n, np.float32)
    import os
    th = threads or min(16, len(os.sched_getaffinity(0)))
    lib().oracle_sincosf_bits(C.c_uint32(lo), C.c_int64(n), _p(s), _p(c), C.c_int(th))
    return s, c


def fast_roi(roi, t):
    roi = np.ascontiguousarray(roi, np.uint8)
    rows, cols = roi.shape
    cap = rows * cols
    xs = np.zeros(cap, np.int32)
    ys = np.zeros(cap, np.int32)
    sc = np.zeros(cap, np.int32)
    n = lib().oracle_fast_roi(_p(roi), C.c_int(rows), C.c_int(cols), C.c_int64(cols), C.c_int(t),
                              _p(xs), _p(ys), _p(sc), C.c_int(cap))
    return xs[:n].copy(), ys[:n].copy(), sc[:n].copy()


def fast_score(img, x, y):
    img = np.ascontiguousarray(img, np.uint8)
    ptr = img.ctypes.data + int(y) * img.shape[1] + int(x)
    return lib().oracle_fast_score(C.c_void_p(ptr), C.c_int64(img.shape[1]))


def ic_angle(img, x, y):
    img = np.ascontiguousarray(img, np.uint8)
    f = lib().oracle_ic_angle
    f.restype = C.c_float
    return f(_p(img), C.c_int64(img.shape[1]), C.c_int(x), C.c_int(y))


def orb_descriptor(blurred, x, y, angle):
    blurred = np.ascontiguousarray(blurred, np.uint8)
    d = np.zeros(32, np.uint8)
    lib().oracle_orb_descriptor(_p(blurred), C.c_int64(blurred.shape[1]), C.c_int(x), C.c_int(y),
                                C.c_float(angle), _p(d))
    return d


def descriptor_distance(a, b):
    a = np.ascontiguousarray(a, np.uint8)
    b = np.ascontiguousarray(b, np.uint8)
    return lib().oracle_descriptor_distance(_p(a), _p(b))


# ------------------------------------------------------------------ matcher sides
class _Keep:
    """Holds numpy buffers alive for the lifetime of a ctypes side struct."""

    def __init__(self, **kw):
        self.__dict__.update(kw)


def featvec_struct(fv):
    node_ids, offsets, feats = fv
    k = _Keep(node_ids=np.ascontiguousarray(node_ids, np.uint32),
              offsets=np.ascontiguousarray(offsets, np.int32),
              feats=np.ascontiguousarray(feats, np.int32))
    s = FeatVec(len(k.node_ids), _p(k.node_ids), _p(k.offsets), _p(k.feats))
    return s, k


def bow_side(desc, angle, valid, fv):
    desc = np.ascontiguousarray(desc, np.uint8)
    angle = np.ascontiguousarray(angle, np.float32)
    valid = None if valid is None else np.ascontiguousarray(valid, np.uint8)
    fvs, fk = featvec_struct(fv)
    s = BowSide(desc.shape[0], _p(desc), _p(angle), _p(valid), fvs)
    return s, _Keep(desc=desc, angle=angle, valid=valid, fk=fk)


def tri_side(desc, keys_un, u_right, has_mp, fv, scale_factors, level_sigma2):
    desc = np.ascontiguousarray(desc, np.uint8)
    keys_un = np.ascontiguousarray(keys_un, KEYPOINT_DTYPE)
    u_right = None if u_right is None else np.ascontiguousarray(u_right, np.float32)
    has_mp = None if has_mp is None else np.ascontiguousarray(has_mp, np.uint8)
    sf = np.ascontiguousarray(scale_factors, np.float32)
    s2 = np.ascontiguousarray(level_sigma2, np.float32)
    fvs, fk = featvec_struct(fv)
    s = TriSide(desc.shape[0], _p(desc), _p(keys_un), _p(u_right), _p(has_mp), fvs, _p(sf),
                _p(s2), len(sf))
    return s, _Keep(desc=desc, keys_un=keys_un, u_right=u_right, has_mp=has_mp, sf=sf, s2=s2,
                    fk=fk)


def search_by_bow_kf_f(kf, f, nnratio=0.7, check_ori=True):
    """kf, f: dicts with desc, angle, valid (kf only), fv=(node_ids, offsets, feats)."""
    ks, kk = bow_side(kf["desc"], kf["angle"], kf.get("valid"), kf["fv"])
    fs, fk = bow_side(f["desc"], f["angle"], None, f["fv"])
    match = np.full(f["desc"].shape[0], -1, np.int32)
    n = lib().oracle_search_by_bow_kf_f(C.byref(ks), C.byref(fs), C.c_float(nnratio),
                                        C.c_int(int(check_ori)), _p(match))
    return n, match


def search_by_bow_kf_kf(kf1, kf2, nnratio=0.75, check_ori=True):
    s1, k1 = bow_side(kf1["desc"], kf1["angle"], kf1.get("valid"), kf1["fv"])
    s2, k2 = bow_side(kf2["desc"], kf2["angle"], kf2.get("valid"), kf2["fv"])
    match = np.full(kf1["desc"].shape[0], -1, np.int32)
    n = lib().oracle_search_by_bow_kf_kf(C.byref(s1), C.byref(s2), C.c_float(nnratio),
                                         C.c_int(int(check_ori)), _p(match))
    return n, match


def search_for_triangulation(kf1, kf2, F12, ex, ey, only_stereo=False, nnratio=0.6,
                             check_ori=False):
    s1, k1 = tri_side(kf1["desc"], kf1["keys"], kf1.get("u_right"), kf1.get("has_mp"), kf1["fv"],
                      kf1["scale_factors"], kf1["level_sigma2"])
    s2, k2 = tri_side(kf2["desc"], kf2["keys"], kf2.get("u_right"), kf2.get("has_mp"), kf2["fv"],
                      kf2["scale_factors"], kf2["level_sigma2"])
    F = np.ascontiguousarray(F12, np.float32).reshape(9)
    pairs = np.zeros((max(1, kf1["desc"].shape[0]), 2), np.int32)
    n = lib().oracle_search_for_triangulation(C.byref(s1), C.byref(s2), _p(F), C.c_float(ex),
                                              C.c_float(ey), C.c_int(int(only_stereo)),
                                              C.c_float(nnratio), C.c_int(int(check_ori)),
                                              _p(pairs))
    return n, pairs[:n].copy()


def epipole(R2w, t2w, Cw, fx, fy, cx, cy):
    ex, ey = C.c_float(), C.c_float()
    R = np.ascontiguousarray(R2w, np.float32).reshape(9)
    t = np.ascontiguousarray(t2w, np.float32).reshape(3)
    c = np.ascontiguousarray(Cw, np.float32).reshape(3)
    lib().oracle_epipole(_p(R), _p(t), _p(c), C.c_float(fx), C.c_float(fy), C.c_float(cx),
                         C.c_float(cy), C.byref(ex), C.byref(ey))
    return ex.value, ey.value


def feature_vector(voc_desc, k, L, levelsup, desc):
    voc_desc = np.ascontiguousarray(voc_desc, np.uint8)
    desc = np.ascontiguousarray(desc, np.uint8)
    out = np.zeros(desc.shape[0], np.uint32)
    lib().oracle_feature_vector(_p(voc_desc), C.c_int(k), C.c_int(L), C.c_int(levelsup), _p(desc),
                                C.c_int(desc.shape[0]), _p(out))
    return out


# ---------------------------------------------------------------- DBoW2 (dbow2_oracle.cc)
class Vocabulary:
    """TemplatedVocabulary<FORB> restatement: nodes 1..n in file order (root 0 implicit)."""

    def __init__(self, handle):
        if not handle:
            raise ValueError("oracle vocabulary rejected")
        self._h = C.c_void_p(handle)

    @staticmethod
    def from_nodes(k, L, scoring, weighting, parent, is_leaf, desc, weight):
        parent = np.ascontiguousarray(parent, np.int32)
        is_leaf = np.ascontiguousarray(is_leaf, np.uint8)
        desc = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        weight = np.ascontiguousarray(weight, np.float64)
        L_ = lib()
        L_.oracle_voc_create.restype = C.c_void_p
        h = L_.oracle_voc_create(C.c_int(k), C.c_int(L), C.c_int(scoring), C.c_int(weighting),
                                 C.c_int(len(parent)), _p(parent), _p(is_leaf), _p(desc),
                                 _p(weight))
        return Vocabulary(h)

    @staticmethod
    def load_text(path):
        L_ = lib()
        L_.oracle_voc_load_text.restype = C.c_void_p
        return Vocabulary(L_.oracle_voc_load_text(str(path).encode()))

    def __del__(self):
        if getattr(self, "_h", None):
            lib().oracle_voc_destroy(self._h)
            self._h = None

    def info(self):
        v = [C.c_int() for _ in range(6)]
        lib().oracle_voc_info(self._h, *[C.byref(x) for x in v])
        return dict(zip(("k", "L", "scoring", "weighting", "n_nodes", "n_words"),
                        (x.value for x in v)))

    def transform(self, desc, levelsup=4):
        desc = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        n = desc.shape[0]
        word_of = np.zeros(n, np.uint32)
        node_of = np.zeros(n, np.uint32)
        bw = np.zeros(max(n, 1), np.uint32)
        bv = np.zeros(max(n, 1), np.float64)
        fi = np.zeros(max(n, 1), np.uint32)
        fo = np.zeros(n + 1, np.int32)
        ff = np.zeros(max(n, 1), np.int32)
        bn, fn = C.c_int(), C.c_int()
        lib().oracle_voc_transform(self._h, _p(desc), C.c_int(n), C.c_int(levelsup), _p(word_of),
                                   _p(node_of), _p(bw), _p(bv), C.byref(bn), _p(fi), _p(fo),
                                   _p(ff), C.byref(fn))
        return dict(word_of=word_of, node_of=node_of, bow_words=bw[:bn.value],
                    bow_values=bv[:bn.value], fv_ids=fi[:fn.value], fv_off=fo[:fn.value + 1],
                    fv_feats=ff[:fo[fn.value]])


# ---------------------------------------------------------------- stereo (stereo_oracle.cc)
def stereo_matches(kl, dl, kr, dr, pyr_left, pyr_right, scale, inv_scale, mb, mbf):
    """Frame::ComputeStereoMatches restated: (mvuRight, mvDepth, SAD or -1) per left keypoint.
    pyr_left / pyr_right: lists of 2-D uint8 level images (mvImagePyramid)."""
    kl = np.ascontiguousarray(kl, KEYPOINT_DTYPE)
    kr = np.ascontiguousarray(kr, KEYPOINT_DTYPE)
    dl = np.ascontiguousarray(dl, np.uint8).reshape(-1, 32)
    dr = np.ascontiguousarray(dr, np.uint8).reshape(-1, 32)
    L = len(pyr_left)
    pl = [np.ascontiguousarray(x, np.uint8) for x in pyr_left]
    pr = [np.ascontiguousarray(x, np.uint8) for x in pyr_right]
    for a, b in zip(pl, pr):
        assert a.shape == b.shape
    PL = (C.c_void_p * L)(*[x.ctypes.data for x in pl])
    PR = (C.c_void_p * L)(*[x.ctypes.data for x in pr])
    lw = np.array([x.shape[1] for x in pl], np.int32)
    lh = np.array([x.shape[0] for x in pl], np.int32)
    ls = np.array([x.strides[0] for x in pl], np.int64)
    sc = np.ascontiguousarray(scale, np.float32)
    isc = np.ascontiguousarray(inv_scale, np.float32)
    n = len(kl)
    ur = np.zeros(max(n, 1), np.float32)
    dp = np.zeros(max(n, 1), np.float32)
    sd = np.zeros(max(n, 1), np.int32)
    lib().oracle_stereo_matches(_p(kl), C.c_int(n), _p(dl), _p(kr), C.c_int(len(kr)), _p(dr),
                                PL, PR, _p(lw), _p(lh), _p(ls), _p(sc), _p(isc),
                                C.c_float(mb), C.c_float(mbf), _p(ur), _p(dp), _p(sd))
    return ur[:n], dp[:n], sd[:n]


# ---------------------------------------------------------------- projection searches
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


class ProjLast(C.Structure):
    _fields_ = [("n", C.c_int32), ("valid", C.c_void_p), ("u", C.c_void_p), ("v", C.c_void_p),
                ("ur", C.c_void_p), ("octave", C.c_void_p), ("angle", C.c_void_p),
                ("desc", C.c_void_p), ("blocks", C.c_void_p)]


def _arrs(d, spec):
    return {k: (None if d.get(k) is None else np.ascontiguousarray(d[k], t)) for k, t in spec}


def proj_frame(f):
    """f: dict(keys_un, desc, u_right|None, has_mp_obs|None, min_x, min_y, max_x, max_y,
    grid_w_inv, grid_h_inv, scale_factors)."""
    a = _arrs(f, [("keys_un", KEYPOINT_DTYPE), ("desc", np.uint8), ("u_right", np.float32),
                  ("has_mp_obs", np.uint8), ("scale_factors", np.float32)])
    s = ProjFrame(len(a["keys_un"]), _p(a["keys_un"]), _p(a["desc"]), _p(a["u_right"]),
                  _p(a["has_mp_obs"]), f["min_x"], f["min_y"], f["max_x"], f["max_y"],
                  f["grid_w_inv"], f["grid_h_inv"], _p(a["scale_factors"]),
                  len(a["scale_factors"]))
    return s, a


def features_in_area(f, x, y, r, min_level, max_level, cap=100000):
    s, keep = proj_frame(f)
    out = np.zeros(cap, np.int32)
    n = lib().oracle_features_in_area(C.byref(s), C.c_float(x), C.c_float(y), C.c_float(r),
                                      C.c_int(min_level), C.c_int(max_level), _p(out), C.c_int(cap))
    return out[:n].copy()


def search_by_projection(f, pts, th, nnratio):
    s, keep = proj_frame(f)
    a = _arrs(pts, [("track", np.uint8), ("proj_x", np.float32), ("proj_y", np.float32),
                    ("proj_xr", np.float32), ("pred_level", np.int32), ("view_cos", np.float32),
                    ("desc", np.uint8)])
    p = ProjPoints(len(a["track"]), *[_p(a[k]) for k in ("track", "proj_x", "proj_y", "proj_xr",
                                                          "pred_level", "view_cos", "desc")])
    match = np.zeros(max(s.n, 1), np.int32)
    n = lib().oracle_search_by_projection(C.byref(s), C.byref(p), C.c_float(th),
                                          C.c_float(nnratio), _p(match))
    return n, match[:s.n].copy()


def search_by_projection_last(f, last, th, forward, backward, check_ori):
    s, keep = proj_frame(f)
    a = _arrs(last, [("valid", np.uint8), ("u", np.float32), ("v", np.float32), ("ur", np.float32),
                     ("octave", np.int32), ("angle", np.float32), ("desc", np.uint8),
                     ("blocks", np.uint8)])
    p = ProjLast(len(a["valid"]), *[_p(a[k]) for k in ("valid", "u", "v", "ur", "octave", "angle",
                                                        "desc", "blocks")])
    match = np.zeros(max(s.n, 1), np.int32)
    n = lib().oracle_search_by_projection_last(C.byref(s), C.byref(p), C.c_float(th),
                                               C.c_int(int(forward)), C.c_int(int(backward)),
                                               C.c_int(int(check_ori)), _p(match))
    return n, match[:s.n].copy()


def search_for_initialization(f1, f2, prev, nnratio, check_ori, window):
    """ORBmatcher::SearchForInitialization (ORBmatcher.cc:405-523).  f1, f2: proj_frame dicts;
    prev: (n1, 2) float32 vbPrevMatched.  Returns (nmatches, vnMatches12, updated prev)."""
    s1, k1 = proj_frame(f1)
    s2, k2 = proj_frame(f2)
    pv = np.ascontiguousarray(prev, np.float32).reshape(-1, 2).copy()
    m12 = np.zeros(max(s1.n, 1), np.int32)
    n = lib().oracle_search_for_initialization(C.byref(s1), C.byref(s2), _p(pv), C.c_float(nnratio),
                                               C.c_int(int(check_ori)), C.c_int(int(window)), _p(m12))
    return n, m12[:s1.n].copy(), pv


class FusePoints(C.Structure):
    _fields_ = [("n", C.c_int32), ("use", C.c_void_p), ("u", C.c_void_p), ("v", C.c_void_p),
                ("ur", C.c_void_p), ("pred_level", C.c_void_p), ("desc", C.c_void_p)]


def fuse(kf, inv_sigma2, pts, th, reproj=True):
    """ORBmatcher::Fuse's per-point search (ORBmatcher.cc:828-978 / 980-1103).  Returns
    (count, best_idx, best_dist)."""
    s, keep = proj_frame(kf)
    a = _arrs(pts, [("use", np.uint8), ("u", np.float32), ("v", np.float32), ("ur", np.float32),
                    ("pred_level", np.int32), ("desc", np.uint8)])
    p = FusePoints(len(a["use"]), *[_p(a[k]) for k in ("use", "u", "v", "ur", "pred_level", "desc")])
    isg = np.ascontiguousarray(inv_sigma2, np.float32)
    bi = np.zeros(max(p.n, 1), np.int32)
    bd = np.zeros(max(p.n, 1), np.int32)
    n = lib().oracle_fuse(C.byref(s), _p(isg), C.byref(p), C.c_float(th), C.c_int(int(reproj)),
                          _p(bi), _p(bd))
    return n, bi[:p.n].copy(), bd[:p.n].copy()


def _fuse_points(pts):
    a = _arrs(pts, [("use", np.uint8), ("u", np.float32), ("v", np.float32), ("ur", np.float32),
                    ("pred_level", np.int32), ("desc", np.uint8)])
    return FusePoints(len(a["use"]), *[_p(a[k]) for k in ("use", "u", "v", "ur", "pred_level", "desc")]), a


def search_by_projection_kf(f, kf_points, th, orb_dist, check_ori):
    """ORBmatcher::SearchByProjection(Frame&, KeyFrame*, sAlreadyFound, th, ORBdist)
    (ORBmatcher.cc:1475-1602).  f: proj_frame dict whose has_mp_obs = mvpMapPoints != NULL;
    kf_points: valid, u, v, octave (predicted level), angle, desc.  Returns (n, match)."""
    s, keep = proj_frame(f)
    a = _arrs(kf_points, [("valid", np.uint8), ("u", np.float32), ("v", np.float32),
                          ("ur", np.float32), ("octave", np.int32), ("angle", np.float32),
                          ("desc", np.uint8)])
    p = ProjLast(len(a["valid"]), *[_p(a[k]) for k in ("valid", "u", "v", "ur", "octave", "angle",
                                                        "desc")])
    match = np.zeros(max(s.n, 1), np.int32)
    n = lib().oracle_search_by_projection_kf(C.byref(s), C.byref(p), C.c_float(th),
                                             C.c_int(int(orb_dist)), C.c_int(int(check_ori)),
                                             _p(match))
    return n, match[:s.n].copy()


def search_by_projection_sim3(kf, pts, th):
    """ORBmatcher::SearchByProjection(KeyFrame*, Scw, vpPoints, vpMatched, th)
    (ORBmatcher.cc:290-403).  kf: proj_frame dict whose has_mp_obs = vpMatched != NULL; pts:
    use, u, v, pred_level, desc.  Returns (n, match)."""
    s, keep = proj_frame(kf)
    p, a = _fuse_points(pts)
    match = np.zeros(max(s.n, 1), np.int32)
    n = lib().oracle_search_by_projection_sim3(C.byref(s), C.byref(p), C.c_float(th), _p(match))
    return n, match[:s.n].copy()


def search_by_sim3(kf1, kf2, pts12, pts21, th):
    """ORBmatcher::SearchBySim3 (ORBmatcher.cc:1105-1329).  pts12: KF1's points projected into
    KF2 (one per KF1 keypoint), pts21: KF2's into KF1.  Returns (nFound, m12)."""
    s1, k1 = proj_frame(kf1)
    s2, k2 = proj_frame(kf2)
    p12, a12 = _fuse_points(pts12)
    p21, a21 = _fuse_points(pts21)
    m12 = np.zeros(max(p12.n, 1), np.int32)
    n = lib().oracle_search_by_sim3(C.byref(s1), C.byref(s2), C.byref(p12), C.byref(p21),
                                    C.c_float(th), _p(m12))
    return n, m12[:p12.n].copy()


# ---------------------------------------------------------------- AR marker path (cvorb_oracle.cc)
DMATCH_DTYPE = np.dtype([("query_idx", "<i4"), ("train_idx", "<i4"), ("img_idx", "<i4"),
                         ("distance", "<f4")])
HARRIS_SCORE, FAST_SCORE = 0, 1


class CvOrbParams(C.Structure):
    _fields_ = [("nfeatures", C.c_int32), ("scale_factor", C.c_float), ("nlevels", C.c_int32),
                ("edge_threshold", C.c_int32), ("first_level", C.c_int32), ("wta_k", C.c_int32),
                ("score_type", C.c_int32), ("patch_size", C.c_int32)]


def cvorb_params(nfeatures=500, scale_factor=1.2, nlevels=8, edge_threshold=31, first_level=0,
                 wta_k=2, score_type=HARRIS_SCORE, patch_size=31):
    """cv::ORB 2.4 constructor defaults (the ones Marker.cc:83, 107 uses)."""
    return CvOrbParams(nfeatures, scale_factor, nlevels, edge_threshold, first_level, wta_k,
                       score_type, patch_size)


def cvorb_levels(p, w, h):
    n = p.nlevels
    lw, lh, fe = (np.zeros(n, np.int32) for _ in range(3))
    sc = np.zeros(n, np.float32)
    rc = lib().oracle_cvorb_levels(C.byref(p), C.c_int(w), C.c_int(h), _p(lw), _p(lh), _p(sc),
                                   _p(fe))
    assert rc == 0, rc
    return dict(w=lw, h=lh, scale=sc, feats=fe)


def cvorb_detect(img, p=None, want_pyramid=False):
    """cv::ORB::operator()(img, noArray(), kps, desc) restated (OpenCV 2.4 orb.cpp)."""
    p = p or cvorb_params()
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    cap = max(1, w * h // 4)
    kps = np.zeros(cap, KEYPOINT_DTYPE)
    desc = np.zeros((cap, 32), np.uint8)
    n = C.c_int()
    lv = cvorb_levels(p, w, h)
    tot = int((lv["w"].astype(np.int64) * lv["h"]).sum())
    pyr = np.zeros(tot, np.uint8) if want_pyramid else None
    rc = lib().oracle_cvorb_detect(C.byref(p), _p(img), C.c_int(w), C.c_int(h), C.c_int64(w),
                                   _p(kps), _p(desc), C.c_int(cap), C.byref(n), _p(pyr),
                                   C.c_int64(tot))
    assert rc == 0, rc
    kps, desc = kps[:n.value].copy(), desc[:n.value].copy()
    if not want_pyramid:
        return kps, desc
    levels, off = [], 0
    for lw_, lh_ in zip(lv["w"], lv["h"]):
        levels.append(pyr[off:off + lw_ * lh_].reshape(lh_, lw_))
        off += lw_ * lh_
    return kps, desc, levels


def retain_best(resp, n_points):
    """KeyPointsFilter::retainBest with GCC 4.8 nth_element/partition; returns the retained
    (responses, original indices) in their final order."""
    resp = np.ascontiguousarray(resp, np.float32).copy()
    ids = np.arange(len(resp), dtype=np.int32)
    n = C.c_int()
    lib().oracle_retain_best(_p(resp), _p(ids), C.c_int(len(resp)), C.c_int(n_points), C.byref(n))
    return resp[:n.value].copy(), ids[:n.value].copy()


def harris(img, x, y):
    img = np.ascontiguousarray(img, np.uint8)
    f = lib().oracle_harris
    f.restype = C.c_float
    return f(_p(img), C.c_int64(img.shape[1]), C.c_int(x), C.c_int(y))


def cvorb_descriptor(blurred, x, y, angle):
    blurred = np.ascontiguousarray(blurred, np.uint8)
    d = np.zeros(32, np.uint8)
    lib().oracle_cvorb_descriptor(_p(blurred), C.c_int64(blurred.shape[1]), C.c_int(x),
                                  C.c_int(y), C.c_float(angle), _p(d))
    return d


def cos_sin_f64(deg):
    c, s = C.c_float(), C.c_float()
    lib().oracle_cos_sin_f64(C.c_float(deg), C.byref(c), C.byref(s))
    return c.value, s.value


def cos_sin_f64_range(bits0, n, threads=8):
    """(float)cos/sin((double)(deg * (float)(pi/180))) for the n float bit patterns from bits0."""
    c = np.zeros(n, np.float32)
    s = np.zeros(n, np.float32)
    lib().oracle_cos_sin_f64_range(C.c_uint32(bits0), C.c_int64(n), _p(c), _p(s),
                                   C.c_int(threads))
    return c, s


def bf_match(query, train):
    q = np.ascontiguousarray(query, np.uint8).reshape(-1, 32)
    t = np.ascontiguousarray(train, np.uint8).reshape(-1, 32)
    out = np.zeros(max(1, len(q)), DMATCH_DTYPE)
    n = C.c_int()
    lib().oracle_bf_match(_p(q), C.c_int(len(q)), _p(t), C.c_int(len(t)), _p(out), C.byref(n))
    return out[:n.value].copy()


def good_matches(matches):
    m = np.ascontiguousarray(matches, DMATCH_DTYPE)
    good = np.zeros(max(1, len(m)), DMATCH_DTYPE)
    n = C.c_int()
    mn, mx = C.c_double(), C.c_double()
    lib().oracle_good_matches(_p(m), C.c_int(len(m)), _p(good), C.byref(n), C.byref(mn),
                              C.byref(mx))
    return good[:n.value].copy(), mn.value, mx.value


def nn_match(query, train, ratio=0.8, max_dist=50):
    q = np.ascontiguousarray(query, np.uint8).reshape(-1, 32)
    t = np.ascontiguousarray(train, np.uint8).reshape(-1, 32)
    out = np.zeros(max(1, len(q)), DMATCH_DTYPE)
    n, mn, mx = C.c_int(), C.c_int(), C.c_int()
    lib().oracle_nn_match(_p(q), C.c_int(len(q)), _p(t), C.c_int(len(t)), C.c_double(ratio),
                          C.c_int(max_dist), _p(out), C.byref(n), C.byref(mn), C.byref(mx))
    return out[:n.value].copy(), mn.value, mx.value
