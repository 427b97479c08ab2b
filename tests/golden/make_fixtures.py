"""Regenerate the committed gray fixtures from the reference's real frames.

Inputs (reference tree, read here once; not present on the GPU box):
  AR-1.3/tmp.jpg, AR-1.3/bin/data/book1.jpg (640x480 webcam dumps written by
  AR-1.3/src/ofApp.cpp:364-385), AR-1.3/bin/data/target.jpg (512x512).
Decoded once with PIL and converted to gray with OpenCV 2.4's fixed-point BGR2GRAY
(4899 R + 9617 G + 1868 B + 8192) >> 14, then stored as binary PGM so the GPU box needs no JPEG
decoder.  The goldens (keypoints/descriptors) are produced from these by
tests/golden/make_goldens.py with the CPU oracle.
"""
import os
import numpy as np
from PIL import Image

REF = "/root/reference/AR-1.3"
HERE = os.path.dirname(os.path.abspath(__file__))
SRC = {"tmp": "tmp.jpg", "book1": "bin/data/book1.jpg", "target": "bin/data/target.jpg"}


def to_gray(rgb):
    r, g, b = (rgb[..., i].astype(np.int32) for i in range(3))
    return ((4899 * r + 9617 * g + 1868 * b + 8192) >> 14).astype(np.uint8)


def write_pgm(path, g):
    with open(path, "wb") as f:
        f.write(b"P5\n%d %d\n255\n" % (g.shape[1], g.shape[0]))
        f.write(g.tobytes())


if __name__ == "__main__":
    for name, rel in SRC.items():
        rgb = np.asarray(Image.open(os.path.join(REF, rel)).convert("RGB"))
        g = to_gray(rgb)
        write_pgm(os.path.join(HERE, name + ".pgm"), g)
        print(name, g.shape)
