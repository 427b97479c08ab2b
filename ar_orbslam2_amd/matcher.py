"""ORBmatcher — host-side mirror of ORB_SLAM2::ORBmatcher's BoW / triangulation searches.

Mirrors ORB_SLAM2/include/ORBmatcher.h:37-80 (constructor, DescriptorDistance, both
SearchByBoW overloads, SearchForTriangulation, TH_LOW/TH_HIGH/HISTO_LENGTH).  Frames and
keyframes are passed as plain objects carrying the members the reference reads:

    KF side : mDescriptors (n,32) u8, mvKeysUn / mvKeys (KEYPOINT_DTYPE), mFeatVec
              (FeatureVector), map-point validity as `valid` (pMP && !pMP->isBad()) or
              `has_mp` (GetMapPoint(i) != NULL), mvuRight, mvScaleFactors, mvLevelSigma2
    Frame   : mDescriptors, mvKeys, mFeatVec

Outputs are indices instead of MapPoint pointers: SearchByBoW(KF, F) returns
(nmatches, match) with match[f] = KF feature index or -1 (the caller maps it to
vpMapPointsKF[match[f]]); SearchByBoW(KF1, KF2) returns match12[i1] = KF2 index or -1;
SearchForTriangulation returns (nmatches, pairs[n,2]).  All work runs on the GPU.
"""
from __future__ import annotations

import ctypes as C
from types import SimpleNamespace

import numpy as np

from . import _ffi
from ._ffi import KEYPOINT_DTYPE, check, lib, ptr


class _Keep(SimpleNamespace):
    pass


def _fv(fv):
    ids, offs, feats = fv.as_tuple() if hasattr(fv, "as_tuple") else fv
    k = _Keep(ids=np.ascontiguousarray(ids, np.uint32), offs=np.ascontiguousarray(offs, np.int32),
              feats=np.ascontiguousarray(feats, np.int32))
    return _ffi.FeatVec(len(k.ids), ptr(k.ids), ptr(k.offs), ptr(k.feats)), k


def _bow_side(desc, keys, valid, fv):
    desc = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
    angle = np.ascontiguousarray(np.asarray(keys)["angle"], np.float32)
    valid = None if valid is None else np.ascontiguousarray(valid, np.uint8)
    fvs, fk = _fv(fv)
    s = _ffi.BowSide(desc.shape[0], ptr(desc), ptr(angle), ptr(valid), fvs)
    return s, _Keep(desc=desc, angle=angle, valid=valid, fk=fk)


def _tri_side(kf):
    desc = np.ascontiguousarray(kf.mDescriptors, np.uint8).reshape(-1, 32)
    keys = np.ascontiguousarray(kf.mvKeysUn, KEYPOINT_DTYPE)
    ur = getattr(kf, "mvuRight", None)
    ur = None if ur is None else np.ascontiguousarray(ur, np.float32)
    hm = getattr(kf, "has_mp", None)
    hm = None if hm is None else np.ascontiguousarray(hm, np.uint8)
    sf = np.ascontiguousarray(kf.mvScaleFactors, np.float32)
    s2 = np.ascontiguousarray(kf.mvLevelSigma2, np.float32)
    fvs, fk = _fv(kf.mFeatVec)
    s = _ffi.TriSide(desc.shape[0], ptr(desc), ptr(keys), ptr(ur), ptr(hm), fvs, ptr(sf), ptr(s2),
                     len(sf))
    return s, _Keep(desc=desc, keys=keys, ur=ur, hm=hm, sf=sf, s2=s2, fk=fk)


class ORBmatcher:
    TH_HIGH = 100
    TH_LOW = 50
    HISTO_LENGTH = 30

    def __init__(self, nnratio=0.6, checkOri=True):
        self.mfNNratio = float(np.float32(nnratio))
        self.mbCheckOrientation = bool(checkOri)

    @staticmethod
    def DescriptorDistance(a, b):
        a = np.ascontiguousarray(a, np.uint8).reshape(-1, 32)
        b = np.ascontiguousarray(b, np.uint8).reshape(-1, 32)
        if a.shape != b.shape:
            raise ValueError("descriptor sets must have the same shape")
        out = np.zeros(a.shape[0], np.int32)
        check("orbx_descriptor_distance",
              lib().orbx_descriptor_distance(ptr(a), ptr(b), C.c_int32(a.shape[0]), ptr(out)))
        return int(out[0]) if out.shape[0] == 1 else out

    def SearchByBoW(self, kf, other):
        """SearchByBoW(KeyFrame*, Frame&) when `other` has no map-point masks, otherwise the
        KeyFrame/KeyFrame overload (`other.is_keyframe` forces the latter)."""
        if getattr(other, "is_keyframe", False):
            return self._bow_kf_kf(kf, other)
        return self._bow_kf_f(kf, other)

    def _bow_kf_f(self, kf, f):
        ks, kk = _bow_side(kf.mDescriptors, kf.mvKeysUn, getattr(kf, "valid", None), kf.mFeatVec)
        fs, fk = _bow_side(f.mDescriptors, f.mvKeys, None, f.mFeatVec)
        match = np.full(fs.n, -1, np.int32)
        n = C.c_int32()
        check("orbx_search_by_bow_kf_f",
              lib().orbx_search_by_bow_kf_f(C.byref(ks), C.byref(fs), C.c_float(self.mfNNratio),
                                            C.c_int32(int(self.mbCheckOrientation)), ptr(match),
                                            C.byref(n)))
        return n.value, match

    def _bow_kf_kf(self, kf1, kf2):
        s1, k1 = _bow_side(kf1.mDescriptors, kf1.mvKeysUn, getattr(kf1, "valid", None),
                           kf1.mFeatVec)
        s2, k2 = _bow_side(kf2.mDescriptors, kf2.mvKeysUn, getattr(kf2, "valid", None),
                           kf2.mFeatVec)
        match = np.full(s1.n, -1, np.int32)
        n = C.c_int32()
        check("orbx_search_by_bow_kf_kf",
              lib().orbx_search_by_bow_kf_kf(C.byref(s1), C.byref(s2), C.c_float(self.mfNNratio),
                                             C.c_int32(int(self.mbCheckOrientation)), ptr(match),
                                             C.byref(n)))
        return n.value, match

    def SearchForTriangulation(self, kf1, kf2, F12, bOnlyStereo=False, epipole=None):
        """`epipole` = (ex, ey) of KF1's centre in KF2 (ORBmatcher.cc:667-673); compute it with
        `epipole()` from the keyframe poses."""
        s1, k1 = _tri_side(kf1)
        s2, k2 = _tri_side(kf2)
        F = np.ascontiguousarray(F12, np.float32).reshape(9)
        ex, ey = epipole
        pairs = np.zeros((max(s1.n, 1), 2), np.int32)
        n = C.c_int32()
        check("orbx_search_for_triangulation",
              lib().orbx_search_for_triangulation(
                  C.byref(s1), C.byref(s2), ptr(F), C.c_float(ex), C.c_float(ey),
                  C.c_int32(int(bOnlyStereo)), C.c_float(self.mfNNratio),
                  C.c_int32(int(self.mbCheckOrientation)), ptr(pairs), C.byref(n)))
        return n.value, pairs[:n.value].copy()


    # -------------------------------------------------------------- tracking searches
    def SearchByProjection(self, F, points, th=3.0, bMono=None, forward=False, backward=False):
        """Both tracking overloads (ORBmatcher.cc:45-137 and 1331-1474), on the GPU.

        F: current frame — mvKeysUn, mDescriptors, mvuRight (None = mono), `has_mp_obs`
           (mvpMapPoints[i] && Observations() > 0), grid frame mnMinX, mnMinY, mnMaxX, mnMaxY,
           mfGridElementWidthInv, mfGridElementHeightInv, mvScaleFactors.
        points with `proj_x` — local-map points (SearchByProjection(F, vpMapPoints, th)):
           track, proj_x, proj_y, proj_xr, pred_level, view_cos, desc.
        points with `u` — the last frame (SearchByProjection(CurrentFrame, LastFrame, th,
           bMono)): valid, u, v, ur, octave, angle, desc and optionally blocks
           (pMP->Observations() > 0; absent = all); forward / backward are bForward /
           bBackward (both False when bMono).
        Returns (nmatches, match) with match[f] = point / last-frame index or -1."""
        fr, keep = _proj_frame(F)
        n = fr.n
        match = np.zeros(max(n, 1), np.int32)
        nm = C.c_int32()
        if hasattr(points, "proj_x") or (isinstance(points, dict) and "proj_x" in points):
            p, pk = _proj_struct(points, _ffi.ProjPoints, [
                ("track", np.uint8), ("proj_x", np.float32), ("proj_y", np.float32),
                ("proj_xr", np.float32), ("pred_level", np.int32), ("view_cos", np.float32),
                ("desc", np.uint8)])
            check("orbx_search_by_projection",
                  lib().orbx_search_by_projection(C.byref(fr), C.byref(p), C.c_float(th),
                                                  C.c_float(self.mfNNratio), ptr(match),
                                                  C.byref(nm)))
        else:
            if bMono:
                forward = backward = False
            p, pk = _proj_struct(points, _ffi.ProjLast, [
                ("valid", np.uint8), ("u", np.float32), ("v", np.float32), ("ur", np.float32),
                ("octave", np.int32), ("angle", np.float32), ("desc", np.uint8),
                ("blocks", np.uint8)])
            check("orbx_search_by_projection_last",
                  lib().orbx_search_by_projection_last(C.byref(fr), C.byref(p), C.c_float(th),
                                                       C.c_int32(int(forward)),
                                                       C.c_int32(int(backward)),
                                                       C.c_int32(int(self.mbCheckOrientation)),
                                                       ptr(match), C.byref(nm)))
        return nm.value, match[:n].copy()

    # -------------------------------------------------------------- monocular initialisation
    def SearchForInitialization(self, F1, F2, vbPrevMatched, windowSize=10):
        """ORBmatcher::SearchForInitialization (ORBmatcher.cc:405-523) on the GPU.

        F1, F2: frames as for SearchByProjection (F1 needs only mvKeysUn and mDescriptors, F2
        also its grid frame).  vbPrevMatched: float32 array (F1.N, 2), updated in place like the
        reference's vector<cv::Point2f>&.  Returns (nmatches, vnMatches12)."""
        f1, k1 = _proj_frame(F1, grid=False)
        f2, k2 = _proj_frame(F2)
        prev = vbPrevMatched
        if not (isinstance(prev, np.ndarray) and prev.dtype == np.float32 and prev.flags.c_contiguous
                and prev.shape == (f1.n, 2)):
            raise ValueError("vbPrevMatched must be a C-contiguous float32 array of shape (N1, 2)")
        m12 = np.zeros(max(f1.n, 1), np.int32)
        nm = C.c_int32()
        check("orbx_search_for_initialization",
              lib().orbx_search_for_initialization(C.byref(f1), C.byref(f2), ptr(prev),
                                                   C.c_int32(int(windowSize)),
                                                   C.c_float(self.mfNNratio),
                                                   C.c_int32(int(self.mbCheckOrientation)),
                                                   ptr(m12), C.byref(nm)))
        return nm.value, m12[:f1.n].copy()


    # -------------------------------------------------------------- local mapping / loop closing
    def Fuse(self, pKF, points, th=3.0, sim3=False):
        """ORBmatcher::Fuse's per-point search on the GPU: Fuse(KeyFrame*, vector<MapPoint*>, th)
        (ORBmatcher.cc:828-978) or, with sim3=True, Fuse(KeyFrame*, Scw, vpPoints, th,
        vpReplacePoint) (:980-1103).

        pKF: keyframe as for SearchByProjection's frame (mvKeysUn, mDescriptors, mvuRight, grid
        frame, mvScaleFactors) plus mvInvLevelSigma2.  points: use, u, v, ur (not for sim3),
        pred_level, desc — the caller's gates and projections (include/orbx.h).
        Returns (nfused, best_idx, best_dist); the caller applies the replace / add-observation
        step in point order as the reference does."""
        kf, keep = _proj_frame(pKF)
        spec = [("use", np.uint8), ("u", np.float32), ("v", np.float32), ("ur", np.float32),
                ("pred_level", np.int32), ("desc", np.uint8)]
        if sim3:
            spec[3] = ("__none__", np.float32)
        p, pk = _proj_struct(points, _ffi.FusePoints, spec)
        bi = np.zeros(max(p.n, 1), np.int32)
        bd = np.zeros(max(p.n, 1), np.int32)
        nf = C.c_int32()
        if sim3:
            check("orbx_fuse_sim3",
                  lib().orbx_fuse_sim3(C.byref(kf), C.byref(p), C.c_float(th), ptr(bi), ptr(bd),
                                       C.byref(nf)))
        else:
            isg = np.ascontiguousarray(_get(pKF, "mvInvLevelSigma2", "inv_level_sigma2"), np.float32)
            check("orbx_fuse",
                  lib().orbx_fuse(C.byref(kf), ptr(isg), C.byref(p), C.c_float(th), ptr(bi), ptr(bd),
                                  C.byref(nf)))
        return nf.value, bi[:p.n].copy(), bd[:p.n].copy()

    # -------------------------------------------------------------- relocalization / loop closing
    _SIM3_SPEC = [("use", np.uint8), ("u", np.float32), ("v", np.float32), ("__none__", np.float32),
                  ("pred_level", np.int32), ("desc", np.uint8)]

    def SearchByProjectionKF(self, CurrentFrame, kf_points, th, ORBdist):
        """SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF, sAlreadyFound, th, ORBdist)
        (ORBmatcher.cc:1475-1602, Tracking::Relocalization) on the GPU.

        CurrentFrame: as for SearchByProjection, with `has_mp_obs` = mvpMapPoints[i] != NULL.
        kf_points: valid, u, v (projection into the current frame), octave (the predicted
        level), angle (pKF->mvKeysUn[i].angle), desc — include/orbx.h.
        Returns (nmatches, match) with match[f] = keyframe index or -1."""
        fr, keep = _proj_frame(CurrentFrame)
        p, pk = _proj_struct(kf_points, _ffi.ProjLast, [
            ("valid", np.uint8), ("u", np.float32), ("v", np.float32), ("__none__", np.float32),
            ("octave", np.int32), ("angle", np.float32), ("desc", np.uint8)])
        match = np.zeros(max(fr.n, 1), np.int32)
        nm = C.c_int32()
        check("orbx_search_by_projection_kf",
              lib().orbx_search_by_projection_kf(C.byref(fr), C.byref(p), C.c_float(th),
                                                 C.c_int32(int(ORBdist)),
                                                 C.c_int32(int(self.mbCheckOrientation)),
                                                 ptr(match), C.byref(nm)))
        return nm.value, match[:fr.n].copy()

    def SearchByProjectionSim3(self, pKF, points, th):
        """SearchByProjection(KeyFrame* pKF, cv::Mat Scw, vpPoints, vpMatched, int th)
        (ORBmatcher.cc:290-403, loop closing) on the GPU.  pKF: keyframe with `has_mp_obs` =
        vpMatched[i] != NULL; points: use, u, v, pred_level, desc (the caller's Scw projection
        and gates).  Returns (nmatches, match) with match[f] = point index assigned to keyframe
        feature f in this call, else -1."""
        kf, keep = _proj_frame(pKF)
        p, pk = _proj_struct(points, _ffi.FusePoints, self._SIM3_SPEC)
        match = np.zeros(max(kf.n, 1), np.int32)
        nm = C.c_int32()
        check("orbx_search_by_projection_sim3",
              lib().orbx_search_by_projection_sim3(C.byref(kf), C.byref(p), C.c_float(th),
                                                   ptr(match), C.byref(nm)))
        return nm.value, match[:kf.n].copy()

    def SearchBySim3(self, pKF1, pKF2, points12, points21, th):
        """SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th) (ORBmatcher.cc:1105-1329)
        on the GPU.  points12: KF1's map points projected into KF2 (one per KF1 keypoint: use,
        u, v, pred_level, desc), points21: KF2's into KF1.  Returns (nFound, m12) with m12[i1]
        = idx2 where both directions agree, else -1."""
        k1, keep1 = _proj_frame(pKF1)
        k2, keep2 = _proj_frame(pKF2)
        p12, pk12 = _proj_struct(points12, _ffi.FusePoints, self._SIM3_SPEC)
        p21, pk21 = _proj_struct(points21, _ffi.FusePoints, self._SIM3_SPEC)
        m12 = np.zeros(max(p12.n, 1), np.int32)
        nf = C.c_int32()
        check("orbx_search_by_sim3",
              lib().orbx_search_by_sim3(C.byref(k1), C.byref(k2), C.byref(p12), C.byref(p21),
                                        C.c_float(th), ptr(m12), C.byref(nf)))
        return nf.value, m12[:p12.n].copy()


def epipole(R2w, t2w, Cw, fx, fy, cx, cy):
    ex, ey = C.c_float(), C.c_float()
    R = np.ascontiguousarray(R2w, np.float32).reshape(9)
    t = np.ascontiguousarray(t2w, np.float32).reshape(3)
    c = np.ascontiguousarray(Cw, np.float32).reshape(3)
    check("orbx_epipole", lib().orbx_epipole(ptr(R), ptr(t), ptr(c), C.c_float(fx), C.c_float(fy),
                                             C.c_float(cx), C.c_float(cy), C.byref(ex),
                                             C.byref(ey)))
    return ex.value, ey.value


def _get(obj, name, alt=None):
    if isinstance(obj, dict):
        return obj.get(name, obj.get(alt) if alt else None)
    v = getattr(obj, name, None)
    return getattr(obj, alt, None) if v is None and alt else v


def _proj_frame(F, grid=True):
    keys = np.ascontiguousarray(_get(F, "mvKeysUn", "keys_un"), KEYPOINT_DTYPE)
    desc = np.ascontiguousarray(_get(F, "mDescriptors", "desc"), np.uint8).reshape(-1, 32)
    if not grid:  # only the keypoints and descriptors are read
        s = _ffi.ProjFrame(len(keys), ptr(keys), ptr(desc), None, None, 0.0, 0.0, 0.0, 0.0, 0.0,
                           0.0, None, 0)
        return s, _Keep(keys=keys, desc=desc)
    ur = _get(F, "mvuRight", "u_right")
    ur = None if ur is None else np.ascontiguousarray(ur, np.float32)
    hm = _get(F, "has_mp_obs")
    hm = None if hm is None else np.ascontiguousarray(hm, np.uint8)
    sf = np.ascontiguousarray(_get(F, "mvScaleFactors", "scale_factors"), np.float32)
    vals = [float(_get(F, a, b)) for a, b in (("mnMinX", "min_x"), ("mnMinY", "min_y"),
                                              ("mnMaxX", "max_x"), ("mnMaxY", "max_y"),
                                              ("mfGridElementWidthInv", "grid_w_inv"),
                                              ("mfGridElementHeightInv", "grid_h_inv"))]
    s = _ffi.ProjFrame(len(keys), ptr(keys), ptr(desc), ptr(ur), ptr(hm), *vals, ptr(sf), len(sf))
    return s, _Keep(keys=keys, desc=desc, ur=ur, hm=hm, sf=sf)


def _proj_struct(points, cls, spec):
    arrs = []
    for name, t in spec:
        v = _get(points, name)
        arrs.append(None if v is None else np.ascontiguousarray(v, t))
    n = len(arrs[0])
    return cls(n, *[ptr(a) for a in arrs]), arrs
