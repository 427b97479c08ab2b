"""CPU checks of the AR marker path's host side (no GPU): Marker::Match's good-match filter in
liborbx (orbx_good_matches is host code, Marker.cc:115-133) against the oracle, and the
Python mirror's argument handling."""
import numpy as np
import pytest

from ar_orbslam2_amd import marker as M
from ar_orbslam2_amd._ffi import DMATCH_DTYPE
from oracle import oracle as O


def _matches(dist):
    m = np.zeros(len(dist), DMATCH_DTYPE)
    m["query_idx"] = np.arange(len(dist))
    m["train_idx"] = np.arange(len(dist))[::-1]
    m["distance"] = dist
    return m


@pytest.mark.parametrize("dist", [[], [0.0], [10.0, 20.0, 40.0, 39.0, 19.0, 20.0],
                                  [150.0, 3.0, 75.0, 74.0, 76.0], [120.0] * 7])
def test_good_matches_matches_oracle(dist):
    m = _matches(np.array(dist, np.float32))
    g, mn, mx = M.good_matches(m)
    og, omn, omx = O.good_matches(m)
    assert g.tobytes() == og.tobytes() and mn == omn and mx == omx


def test_good_matches_random():
    rng = np.random.default_rng(3)
    for _ in range(20):
        m = _matches(rng.integers(0, 257, rng.integers(1, 600)).astype(np.float32))
        g, mn, mx = M.good_matches(m)
        og, omn, omx = O.good_matches(m)
        assert g.tobytes() == og.tobytes() and (mn, mx) == (omn, omx)
        # distance < 0.5 * max_dist, order kept (Marker.cc:129-133)
        assert (g["distance"] < 0.5 * mx).all()
        assert np.all(np.diff(g["query_idx"]) > 0)


def test_descriptor_shape_checked():
    with pytest.raises(ValueError):
        M._desc(np.zeros((4, 31), np.uint8))
    assert M._desc(None).shape == (0, 32)


def test_dmatch_layout_is_cv_dmatch():
    # cv::DMatch (OpenCV 2.4): int queryIdx, trainIdx, imgIdx; float distance -> 16 B
    assert DMATCH_DTYPE.itemsize == 16
    assert [DMATCH_DTYPE.fields[f][1] for f in DMATCH_DTYPE.names] == [0, 4, 8, 12]
