"""Seeded synthetic camera frames (SURVEY §8d "Synthetic generator").

A u8 gray canvas of random axis-aligned rectangles and disks (intensities U[0,255]),
box-blurred 3x3, plus Gaussian noise sigma=4, clipped.  Frame t of stream s is a crop at offset
(t mod 17, t mod 11) of the canvas seeded 0x5EED+s, with per-frame noise seeded (s, t), so
consecutive frames share structure (Hamming-close descriptors exist for the matchers).
"""
from __future__ import annotations

import numpy as np

PAD_X, PAD_Y = 17, 11


def canvas(w, h, stream=0, n_shapes=None):
    rng = np.random.default_rng(0x5EED + stream)
    W, H = w + PAD_X, h + PAD_Y
    img = np.full((H, W), rng.integers(0, 256), np.float32)
    n = int(n_shapes if n_shapes is not None else rng.integers(200, 2001))
    yy, xx = np.mgrid[0:H, 0:W]
    for _ in range(n):
        val = float(rng.integers(0, 256))
        if rng.random() < 0.5:
            x0, y0 = rng.integers(0, W), rng.integers(0, H)
            bw, bh = rng.integers(4, max(5, W // 6)), rng.integers(4, max(5, H // 6))
            img[y0:y0 + bh, x0:x0 + bw] = val
        else:
            cx, cy = rng.integers(0, W), rng.integers(0, H)
            r = int(rng.integers(3, max(4, min(W, H) // 10)))
            y0, y1, x0, x1 = max(0, cy - r), min(H, cy + r + 1), max(0, cx - r), min(W, cx + r + 1)
            m = (yy[y0:y1, x0:x1] - cy) ** 2 + (xx[y0:y1, x0:x1] - cx) ** 2 <= r * r
            img[y0:y1, x0:x1][m] = val
    # 3x3 box blur (edge replicate)
    p = np.pad(img, 1, mode="edge")
    img = sum(p[dy:dy + H, dx:dx + W] for dy in range(3) for dx in range(3)) / 9.0
    return img


def frame(w, h, t=0, stream=0, base=None):
    base = canvas(w, h, stream) if base is None else base
    ox, oy = t % PAD_X, t % PAD_Y
    crop = base[oy:oy + h, ox:ox + w]
    rng = np.random.default_rng([stream, t, 4])
    noisy = crop + rng.normal(0.0, 4.0, crop.shape)
    return np.clip(np.rint(noisy), 0, 255).astype(np.uint8)


def frames(w, h, n, stream=0, t0=0):
    base = canvas(w, h, stream)
    return np.stack([frame(w, h, t0 + i, stream, base) for i in range(n)])


def read_pgm(path):
    data = open(path, "rb").read()
    parts = data.split(b"\n", 3)
    w, h = map(int, parts[1].split())
    return np.frombuffer(parts[3], np.uint8, count=w * h).reshape(h, w).copy()


STEREO_PAD = 48  # extra canvas columns for the disparities


def stereo_pair(w, h, t=0, stream=0, disparity=(12, 20), base=None):
    """Rectified synthetic stereo frame t of stream s: the left image is a crop of the seeded
    canvas, the right one the same scene seen with disparity d (a left pixel (u, v) appears
    at (u - d, v) on the right): d = disparity[0] on the background and disparity[1] inside a
    central rectangle (a nearer plane).  Independent per-image noise, seeded (s, t, side)."""
    Wc = w + STEREO_PAD
    base = canvas(Wc, h, stream + 1000) if base is None else base
    ox, oy = t % PAD_X, t % PAD_Y
    d0, d1 = disparity
    left = base[oy:oy + h, ox:ox + w]
    right = base[oy:oy + h, ox + d0:ox + d0 + w].copy()
    # nearer plane: right columns [x0-d1, x1-d1) show left columns [x0, x1)
    x0, x1, y0, y1 = w // 3, 2 * w // 3, h // 3, 2 * h // 3
    right[y0:y1, x0 - d1:x1 - d1] = left[y0:y1, x0:x1]
    out = []
    for side, img in enumerate((left, right)):
        rng = np.random.default_rng([stream, t, 7, side])
        noisy = img + rng.normal(0.0, 4.0, img.shape)
        out.append(np.clip(np.rint(noisy), 0, 255).astype(np.uint8))
    return out[0], out[1]


# a 4 x 4 tile on which every pixel passes FAST's even-point pretest at threshold 20 (found by a
# search over three-level tiles): the worst case for the FAST kernels' candidate queues
DENSE_CORNER_TILE = np.array([[254, 0, 0, 254], [0, 254, 254, 127], [254, 0, 127, 254],
                              [0, 254, 254, 127]], np.uint8)


def dense_corners(w, h):
    """A w x h frame tiled with DENSE_CORNER_TILE (every pixel a FAST pretest candidate)."""
    return np.tile(DENSE_CORNER_TILE, (h // 4 + 1, w // 4 + 1))[:h, :w].copy()
