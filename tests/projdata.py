"""Inputs for the tracking-search tests: a current frame extracted by the oracle and map
points derived from the previous synthetic frame's features (descriptors with a few bits
flipped, projections jittered around where the feature moved), seeded."""
import numpy as np

from ar_orbslam2_amd import synth
from oracle import oracle as O


def frame_dict(kps, desc, w, h, scale, u_right=None, has_mp_obs=None):
    return dict(keys_un=kps, desc=desc, u_right=u_right, has_mp_obs=has_mp_obs,
                min_x=0.0, min_y=0.0, max_x=float(w), max_y=float(h),
                grid_w_inv=float(np.float32(64) / np.float32(w)),
                grid_h_inv=float(np.float32(48) / np.float32(h)), scale_factors=scale)


def scene(w=640, h=480, nf=1000, t=5, seed=0, stereo=False, mp_frac=0.1):
    p = O.params(nf)
    tb = O.tables(p, w, h)
    base = synth.canvas(w, h, 2)
    prev = synth.frame(w, h, t - 1, 2, base)
    cur = synth.frame(w, h, t, 2, base)
    kp0, d0 = O.extract(prev, p)
    kp1, d1 = O.extract(cur, p)
    rng = np.random.default_rng(seed)
    n1 = len(kp1)
    u_right = None
    if stereo:
        u_right = np.where(rng.random(n1) < 0.6, kp1["x"] - rng.uniform(2, 30, n1),
                           -1.0).astype(np.float32)
    has = (rng.random(n1) < mp_frac).astype(np.uint8)
    F = frame_dict(kp1, d1, w, h, tb["scale"], u_right, has)
    # frame t is the canvas crop at (t mod 17, t mod 11): features move by (-1, -1)
    n0 = len(kp0)
    dx = np.float32(-1.0) + rng.normal(0, 1.0, n0).astype(np.float32)
    dy = np.float32(-1.0) + rng.normal(0, 1.0, n0).astype(np.float32)
    desc = d0.copy()
    flips = rng.integers(0, 256, (n0, 6))
    for k in range(6):
        desc[np.arange(n0), flips[:, k] // 8] ^= (1 << (flips[:, k] % 8)).astype(np.uint8)
    x = (kp0["x"] + dx).astype(np.float32)
    y = (kp0["y"] + dy).astype(np.float32)
    disp = rng.uniform(2, 30, n0).astype(np.float32)
    pts = dict(track=(rng.random(n0) < 0.9).astype(np.uint8), proj_x=x, proj_y=y,
               proj_xr=(x - disp).astype(np.float32),
               pred_level=np.clip(kp0["octave"] + rng.integers(-1, 2, n0), 0, 7).astype(np.int32),
               view_cos=rng.uniform(0.99, 1.0, n0).astype(np.float32), desc=desc)
    last = dict(valid=(rng.random(n0) < 0.85).astype(np.uint8), u=x, v=y,
                ur=(x - disp).astype(np.float32), octave=kp0["octave"].astype(np.int32),
                angle=kp0["angle"].astype(np.float32), desc=desc)
    return F, pts, last


def init_scene(w=640, h=480, nf=2000, t0=3, t1=6, jitter=0.0, seed=0):
    """Monocular initialisation (Tracking::MonocularInitialization, Tracking.cc:922-960): the
    initial frame and a later one from the 2*nFeatures initialisation extractor
    (Tracking.cc:463-464), mvbPrevMatched = the initial keypoints' positions (:931),
    optionally jittered as after earlier SearchForInitialization rounds."""
    p = O.params(nf)
    tb = O.tables(p, w, h)
    base = synth.canvas(w, h, 4)
    k1, d1 = O.extract(synth.frame(w, h, t0, 4, base), p)
    k2, d2 = O.extract(synth.frame(w, h, t1, 4, base), p)
    F1 = frame_dict(k1, d1, w, h, tb["scale"])
    F2 = frame_dict(k2, d2, w, h, tb["scale"])
    rng = np.random.default_rng(seed)
    prev = np.stack([k1["x"], k1["y"]], 1).astype(np.float32)
    if jitter:
        prev = (prev + rng.normal(0, jitter, prev.shape)).astype(np.float32)
    return F1, F2, prev


def fuse_scene(w=640, h=480, nf=1000, t=5, seed=0, stereo=False, jitter=1.5):
    """LocalMapping::SearchInNeighbors (LocalMapping.cc:469, 495) fusing map points into a
    keyframe: the keyframe is frame t (oracle extraction, optional mvuRight), the points are
    frame t-1's features carried to where they moved, with jittered projections (u, v, ur),
    descriptors with a few bits flipped and a predicted level near their octave."""
    F, _, _ = scene(w, h, nf, t, seed, stereo, mp_frac=0.0)
    p = O.params(nf)
    tb = O.tables(p, w, h)
    base = synth.canvas(w, h, 2)
    kp0, d0 = O.extract(synth.frame(w, h, t - 1, 2, base), p)
    rng = np.random.default_rng(100 + seed)
    n0 = len(kp0)
    u = (kp0["x"] - 1 + rng.normal(0, jitter, n0)).astype(np.float32)
    v = (kp0["y"] - 1 + rng.normal(0, jitter, n0)).astype(np.float32)
    desc = d0.copy()
    flips = rng.integers(0, 256, (n0, 8))
    for k in range(8):
        desc[np.arange(n0), flips[:, k] // 8] ^= (1 << (flips[:, k] % 8)).astype(np.uint8)
    pts = dict(use=(rng.random(n0) < 0.9).astype(np.uint8), u=u, v=v,
               ur=(u - rng.uniform(2, 30, n0)).astype(np.float32),
               pred_level=np.clip(kp0["octave"] + rng.integers(-1, 2, n0), 0, 7).astype(np.int32),
               desc=desc)
    F["inv_level_sigma2"] = tb["inv_sigma2"]
    return F, pts


def reloc_scene(w=640, h=480, nf=1000, t=5, seed=0):
    """Tracking::Relocalization (Tracking.cc:1441-1468): the current frame (with the map points
    SearchByBoW / an earlier pass already assigned: mvpMapPoints != NULL blocks a feature) and a
    candidate keyframe's map points projected into it; octave = the predicted level, angle = the
    keyframe keypoint's."""
    F, _, last = scene(w, h, nf, t, seed, stereo=False, mp_frac=0.15)
    F["u_right"] = None
    rng = np.random.default_rng(200 + seed)
    n0 = len(last["valid"])
    pts = dict(last, octave=np.clip(last["octave"] + rng.integers(-1, 2, n0), 0, 7).astype(np.int32))
    return F, pts


def loop_scene(w=640, h=480, nf=1000, t=5, seed=0):
    """LoopClosing::ComputeSim3 / CorrectLoop's SearchByProjection(pKF, Scw, vpPoints, vpMatched,
    th): the keyframe with vpMatched already set for some features, the loop's map points
    projected with Scw."""
    K, P = fuse_scene(w, h, nf, t, seed, stereo=False)
    rng = np.random.default_rng(300 + seed)
    K["has_mp_obs"] = (rng.random(len(K["keys_un"])) < 0.1).astype(np.uint8)
    K["u_right"] = None
    return K, P


def sim3_scene(w=640, h=480, nf=1000, t=5, seed=0):
    """LoopClosing::ComputeSim3's SearchBySim3 (LoopClosing.cc:305): KF1 = frame t-1, KF2 =
    frame t of the synthetic sequence (features move by (-1, -1)); KF1's map points projected
    into KF2 near where their features moved and KF2's projected back, one entry per keypoint,
    with descriptor bit flips, jitter and predicted levels near the octave."""
    p = O.params(nf)
    tb = O.tables(p, w, h)
    base = synth.canvas(w, h, 2)
    k1, d1 = O.extract(synth.frame(w, h, t - 1, 2, base), p)
    k2, d2 = O.extract(synth.frame(w, h, t, 2, base), p)
    K1 = frame_dict(k1, d1, w, h, tb["scale"])
    K2 = frame_dict(k2, d2, w, h, tb["scale"])
    rng = np.random.default_rng(400 + seed)

    def project(kp, desc, dxy):
        n = len(kp)
        d = desc.copy()
        flips = rng.integers(0, 256, (n, 6))
        for k in range(6):
            d[np.arange(n), flips[:, k] // 8] ^= (1 << (flips[:, k] % 8)).astype(np.uint8)
        return dict(use=(rng.random(n) < 0.85).astype(np.uint8),
                    u=(kp["x"] + dxy + rng.normal(0, 1.0, n)).astype(np.float32),
                    v=(kp["y"] + dxy + rng.normal(0, 1.0, n)).astype(np.float32),
                    ur=np.zeros(n, np.float32),
                    pred_level=np.clip(kp["octave"] + rng.integers(-1, 2, n), 0, 7).astype(np.int32),
                    desc=d)
    return K1, K2, project(k1, d1, -1.0), project(k2, d2, 1.0)
