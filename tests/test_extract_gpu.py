"""GPU parity: ORBextractor on gfx950 vs the CPU oracle, bit for bit.

Keypoints (every cv::KeyPoint field) and 32-byte descriptors must be identical to the oracle
with the canonical octree tie-break, on the committed real frames and on
seeded synthetic frames at every BASELINE.json configuration size.
"""
import os

import numpy as np
import pytest

from ar_orbslam2_amd import ORBextractor, synth
from oracle import oracle as O

pytestmark = pytest.mark.gpu

CONFIGS = {
    "C1": (640, 480, 1000),
    "C3": (752, 480, 1200),
    "C4": (1241, 376, 2000),
    "C5": (1920, 1080, 4000),
}


def _batch_extract(img, nfeatures, scale, nlevels, ini, mn, n=5):
    """The image through a batch plan (orbx_plan_*, the throughput path: batches above 4 images
    run the FAST cell pairs in k_fast_pairs, the drop-in extractor's batch of 1 does not),
    replicated n times; returns the keypoints and descriptors of images 0 and n - 1."""
    import ctypes as C
    import torch
    from ar_orbslam2_amd import KEYPOINT_DTYPE
    from ar_orbslam2_amd._ffi import Params, check, lib
    h, w = img.shape
    prm = Params(int(nfeatures), float(scale), int(nlevels), int(ini), int(mn))
    plan = C.c_void_p()
    check("orbx_plan_create", lib().orbx_plan_create(C.byref(prm), w, h, n, 0, C.byref(plan)))
    try:
        d = torch.from_numpy(np.ascontiguousarray(np.stack([img] * n))).cuda()
        check("orbx_plan_extract", lib().orbx_plan_extract(plan, C.c_void_p(d.data_ptr()), n))
        check("orbx_plan_sync", lib().orbx_plan_sync(plan))
        cap = C.c_int32()
        check("orbx_plan_capacity", lib().orbx_plan_capacity(plan, C.byref(cap)))
        kp, ds, ct = C.c_void_p(), C.c_void_p(), C.c_void_p()
        check("orbx_plan_outputs", lib().orbx_plan_outputs(plan, C.byref(kp), C.byref(ds),
                                                            C.byref(ct)))
        hip = C.CDLL("libamdhip64.so")

        def d2h(ptr, nbytes):
            out = np.zeros(nbytes, np.uint8)
            assert hip.hipMemcpy(C.c_void_p(out.ctypes.data), C.c_void_p(ptr), C.c_size_t(nbytes), 2) == 0
            return out
        k = cap.value
        counts = d2h(ct.value, 4 * n).view(np.int32)
        kps = d2h(kp.value, n * k * 28).view(KEYPOINT_DTYPE).reshape(n, k)
        desc = d2h(ds.value, n * k * 32).reshape(n, k, 32)
        return [(kps[i, :counts[i]], desc[i, :counts[i]]) for i in (0, n - 1)]
    finally:
        lib().orbx_plan_destroy(plan)


def _compare(img, nfeatures, scale=1.2, nlevels=8, ini=20, mn=7):
    ex = ORBextractor(nfeatures, scale, nlevels, ini, mn)
    kps, desc = ex(img)
    okps, odesc, olevels, _ = O.extract(img, O.params(nfeatures, scale, nlevels, ini, mn),
                                        want_pyramid=True)
    for bk, bd in _batch_extract(img, nfeatures, scale, nlevels, ini, mn):
        assert np.array_equal(bk, okps), (len(bk), len(okps))
        assert np.array_equal(bd, odesc)
    pyr = ex.mvImagePyramid
    for l, (a, b) in enumerate(zip(pyr, olevels)):
        assert a.shape == b.shape, l
        bad = np.argwhere(a != b)
        assert bad.size == 0, f"level {l}: {len(bad)} pyramid px differ, first {bad[:5]}"
    assert len(kps) == len(okps), (len(kps), len(okps), np.bincount(kps["octave"]),
                                   np.bincount(okps["octave"]))
    for f in ("x", "y", "size", "response", "octave", "class_id"):
        bad = np.nonzero(kps[f] != okps[f])[0]
        assert bad.size == 0, f"field {f}: {bad.size} differ, first idx {bad[:5]}"
    bad = np.nonzero(kps["angle"].view(np.uint32) != okps["angle"].view(np.uint32))[0]
    assert bad.size == 0, f"angle: {bad.size} differ, first {bad[:5]}"
    if len(kps):
        bad = np.nonzero((desc != odesc).any(1))[0]
        assert bad.size == 0, f"descriptors: {bad.size} rows differ, first {bad[:5]}"
    return kps


@pytest.mark.parametrize("name", ["tmp", "book1", "target"])
def test_real_frames(golden_dir, name):
    img = synth.read_pgm(os.path.join(golden_dir, name + ".pgm"))
    kps = _compare(img, 1000)
    assert len(kps) > 500


@pytest.mark.parametrize("cfg", list(CONFIGS))
@pytest.mark.parametrize("t", [0, 5])
def test_synthetic_configs(cfg, t):
    w, h, n = CONFIGS[cfg]
    img = synth.frame(w, h, t=t, stream=1)
    _compare(img, n)


def test_mono_init_extractor(golden_dir):
    # Tracking builds mpIniORBextractor with 2*nFeatures (Tracking.cc:462-464)
    img = synth.read_pgm(os.path.join(golden_dir, "tmp.pgm"))
    _compare(img, 2000)


def test_flat_and_tiny_images():
    _compare(np.full((480, 640), 128, np.uint8), 1000)
    rng = np.random.default_rng(3)
    _compare(rng.integers(0, 256, (240, 320), dtype=np.uint8), 500)


@pytest.mark.parametrize("name", ["tmp", "book1", "target"])
def test_committed_goldens(golden_dir, name):
    """GPU output equals the committed golden vectors (tests/golden/make_goldens.py)."""
    img = synth.read_pgm(os.path.join(golden_dir, name + ".pgm"))
    kps, desc = ORBextractor(1000, 1.2, 8, 20, 7)(img)
    assert np.array_equal(kps, np.load(os.path.join(golden_dir, f"{name}_kps.npy")))
    assert np.array_equal(desc, np.load(os.path.join(golden_dir, f"{name}_desc.npy")))


def test_descriptor_sincosf_device_exhaustive_angles():
    """Keypoint angles on many frames: every descriptor equals the oracle's, which calls the
    host libm sincosf (the device port is checked exhaustively on the host build too)."""
    ex = ORBextractor(1000)
    for t in range(6):
        img = synth.frame(640, 480, t=t, stream=5)
        kps, desc = ex(img)
        okps, odesc = O.extract(img, O.params(1000))
        assert np.array_equal(desc, odesc)


@pytest.mark.parametrize("nlevels,scale", [(1, 1.2), (2, 1.2), (4, 1.2), (5, 1.3), (8, 1.1),
                                           (6, 1.5)])
@pytest.mark.parametrize("w,h", [(640, 480), (321, 203)])
def test_level_counts_and_scales(nlevels, scale, w, h):
    """Pyramid stages and row bands for other level counts, scale factors and widths that are
    not multiples of 16 (byte-assembled level-0 rows)."""
    _compare(synth.frame(w, h, t=2, stream=4), 800, scale=scale, nlevels=nlevels)


@pytest.mark.parametrize("contrast", [3, 5, 8])
def test_min_threshold_fallback_cells(contrast):
    """Low-contrast texture (left half) next to full contrast: many cells find nothing at
    iniThFAST and retry at minThFAST (k_fast_cells' second pass), the others do not."""
    img = synth.frame(640, 480, t=1, stream=2).astype(np.int32)
    img[:, :320] = 128 + (img[:, :320] - 128) // contrast
    kps = _compare(img.astype(np.uint8), 1000)
    assert len(kps) > 300


@pytest.mark.parametrize("w,h,nf", [(1920, 1080, 4000), (1280, 960, 2000), (1024, 768, 1500)])
def test_noise_octree_chunked_levels(w, h, nf):
    """Uniform noise: tens of thousands of FAST candidates per level, so k_octree runs its
    chunked global-scratch path (levels above 16 keys per thread) next to the register path,
    with 1024-thread (level-0 octree frame above 1 Mpx) and 256-thread workgroups."""
    rng = np.random.default_rng(w + h)
    _compare(rng.integers(0, 256, (h, w), dtype=np.uint8), nf)


@pytest.mark.parametrize("kind", ["patch", "dots", "pairs"])
def test_octree_deep_divisions(kind):
    """Keypoints packed into a small region or spread as a few isolated pairs: the octree
    divides far below the first refine's bin depth (k_octree refines its bins several times per
    level, and levels with fewer keys than features divide down to single keys)."""
    rng = np.random.default_rng(11)
    img = np.full((480, 640), 90, np.uint8)
    if kind == "patch":    # one 56 x 56 noise patch: every level's keys in one corner of a node
        img[200:256, 300:356] = rng.integers(0, 256, (56, 56), dtype=np.uint8)
    elif kind == "dots":   # isolated 3 x 3 bright squares, some 5-8 px apart
        for _ in range(40):
            y, x = rng.integers(40, 440), rng.integers(40, 600)
            img[y:y + 3, x:x + 3] = 250
            img[y + 6:y + 9, x + 5:x + 8] = 250
    else:                  # a few tight pairs: keys 2-4 px apart, many levels deep
        for _ in range(12):
            y, x = rng.integers(40, 440), rng.integers(40, 600)
            img[y, x] = 255
            img[y + 2, x + 3] = 0
    _compare(img, 1000)


def _blurred_levels(ex):
    import ctypes as C
    from ar_orbslam2_amd._ffi import lib, check, ptr
    out = []
    for l, lv in enumerate(ex.mvImagePyramid):
        a = np.zeros_like(lv)
        check("orbx_debug_extractor_blur",
              lib().orbx_debug_extractor_blur(ex._h, C.c_int32(l), ptr(a), C.c_int64(a.shape[1])))
        out.append((lv, a))
    return out


@pytest.mark.parametrize("w,h,kind", [(640, 480, "synth"), (1241, 376, "synth"), (643, 361, "noise"),
                                      (517, 389, "flat255"), (401, 301, "steps")])
def test_blur_every_pixel_matches_oracle(w, h, kind):
    """k_blur (GaussianBlur 7x7 sigma 2, reflect-101, OpenCV 2.4 fixed point: SURVEY A.4)
    pixel for pixel on every pyramid level against the oracle, including widths that are not a
    multiple of 4 (the half-up scalar tail), saturating images and noise (rounding ties)."""
    rng = np.random.default_rng(w * h)
    if kind == "synth":
        img = synth.frame(w, h, 3, 1)
    elif kind == "noise":
        img = rng.integers(0, 256, (h, w), dtype=np.uint8)
    elif kind == "flat255":
        img = np.full((h, w), 255, np.uint8)
        img[::7, ::5] = 254
    else:
        img = np.repeat(np.repeat(rng.integers(0, 256, (h // 8 + 1, w // 8 + 1), dtype=np.uint8),
                                  8, 0), 8, 1)[:h, :w].copy()
    ex = ORBextractor(1000)
    ex(img)
    for l, (lv, got) in enumerate(_blurred_levels(ex)):
        ref = O.gaussian7(lv)
        bad = np.argwhere(got != ref)
        assert bad.size == 0, f"level {l} ({lv.shape}): {len(bad)} blurred px differ, first {bad[:5]}"


@pytest.mark.parametrize("w,h,kind", [(640, 480, "synth"), (752, 480, "noise"), (1241, 376, "synth"),
                                      (1920, 1080, "synth"), (643, 361, "noise"), (37, 29, "noise"),
                                      (4000, 70, "noise")])
def test_blur_every_pixel_batch_plans(w, h, kind):
    """Batch plans (the throughput path: 32-row pyramid bands) build the pyramid and its
    GaussianBlur in k_pyramid itself — each band blurs its own rows of every level from the rows
    it holds in LDS, halo rows and reflected pad columns included — except for frames whose bands
    do not fit LDS with the blur's halo (4000 x 70 here), which keep the separate k_blur launch.
    Every pixel of every level of three distinct images against the oracle (ORBextractor.cc:
    1024-1026, 1047-1072)."""
    import ctypes as C
    import torch
    from ar_orbslam2_amd._ffi import Params, check, lib, ptr
    rng = np.random.default_rng(w * 7 + h)
    imgs = [synth.frame(w, h, 2, i) if kind == "synth" else rng.integers(0, 256, (h, w), dtype=np.uint8)
            for i in range(3)]
    n = len(imgs)
    prm = Params(1000, 1.2, 8, 20, 7)
    plan = C.c_void_p()
    check("orbx_plan_create", lib().orbx_plan_create(C.byref(prm), w, h, 8, 0, C.byref(plan)))
    try:
        d = torch.from_numpy(np.ascontiguousarray(np.stack(imgs))).cuda()
        check("orbx_plan_extract", lib().orbx_plan_extract(plan, C.c_void_p(d.data_ptr()), n))
        check("orbx_plan_sync", lib().orbx_plan_sync(plan))
        for i, img in enumerate(imgs):
            _, _, olevels, _ = O.extract(img, O.params(1000, 1.2, 8, 20, 7), want_pyramid=True)
            for l, lv in enumerate(olevels):
                for blurred, ref in ((0, lv), (1, O.gaussian7(lv))):
                    got = np.zeros_like(lv)
                    check("orbx_debug_plan_level",
                          lib().orbx_debug_plan_level(plan, i, l, blurred, ptr(got), C.c_int64(lv.shape[1])))
                    bad = np.argwhere(got != ref)
                    assert bad.size == 0, (f"image {i} level {l} {'blurred' if blurred else 'pyramid'} "
                                           f"({lv.shape}): {len(bad)} px differ, first {bad[:5]}")
    finally:
        lib().orbx_plan_destroy(plan)


@pytest.mark.parametrize("w,h", [(640, 480), (1241, 376)])
def test_dense_corner_pattern_fills_pretest_queues(w, h):
    """Every level-0 pixel of the detection region is a pretest candidate, so k_fast_cells
    queues every detection pixel of a cell: the per-wave queue bound (the cell's detection
    pixels) must hold that."""
    img = synth.dense_corners(w, h)
    _compare(img, 1000)
    # the same texture on half the frame next to a flat region (fallback cells beside full ones)
    img[:, : w // 2] = 128
    _compare(img, 1000)


@pytest.mark.parametrize("w,h", [(4000, 70), (2600, 64)])
def test_wide_frames_many_initial_octree_nodes(w, h):
    """Panorama-like frames: DistributeOctTree starts from nIni = round(W / H) > 64 initial
    nodes (ORBextractor.cc:530-567; 104 and 80 here) — round 2 returned ORBX_EUNSUPPORTED above
    64, the reference has no limit."""
    rng = np.random.default_rng(w)
    img = synth.frame(w, h, 1, 3) if w <= 2600 else rng.integers(0, 256, (h, w), dtype=np.uint8)
    kps = _compare(img, 1500)
    assert len(kps) > 100


@pytest.mark.parametrize("w,h,nf", [(4400, 500, 2000), (4200, 4200, 4000)])
def test_levels_wider_than_4095_px(w, h, nf):
    """Octree frames of 4096 px and more (level 0 of a frame wider or taller than ~4134 px)
    switch the plan to 64-bit candidate keys (x:16 y:16 score:8); round 2 returned
    ORBX_EUNSUPPORTED there, the reference has no limit (ORBextractor.cc:1047-1072, 525-733)."""
    img = synth.frame(w, h, 1, 3)
    kps = _compare(img, nf)
    assert len(kps) > nf // 2
    assert (kps["x"] > 4096).any() if w > 4096 else True


@pytest.mark.parametrize("w,h,nlevels", [(640, 480, 6), (752, 480, 8)])
def test_scale_factor_exactly_two(w, h, nlevels):
    """scaleFactor 2: cv::resize takes its fast INTER_AREA path at the exact 2x2 decimations
    (OpenCV 2.4.9), which the linear taps reproduce (tests/test_oracle_kat.py); round 2 returned
    ORBX_EUNSUPPORTED here.  752 x 480 mixes exact levels with non-exact ones (47 -> 24)."""
    img = synth.frame(w, h, 1, 3)
    kps = _compare(img, 1000, scale=2.0, nlevels=nlevels)
    assert len(kps) > 300
