"""GPU parity of the tracking searches (orbx_search_by_projection / _last: grid, k_proj_cand,
k_proj_resolve) against the CPU oracle: identical match arrays and counts."""
import numpy as np
import pytest

from ar_orbslam2_amd import ORBmatcher
from oracle import oracle as O

from projdata import scene

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("stereo,th,nn,seed", [(False, 1.0, 0.8, 0), (True, 1.0, 0.8, 1),
                                               (False, 3.0, 0.6, 2), (True, 5.0, 0.9, 3),
                                               (False, 1.0, 1.0, 4)])
def test_search_by_projection_local_map(stereo, th, nn, seed):
    F, P, _ = scene(stereo=stereo, seed=seed)
    n, m = ORBmatcher(nn, True).SearchByProjection(F, P, th)
    on, om = O.search_by_projection(F, P, th, nn)
    assert n == on and np.array_equal(m, om)
    assert n > 200


@pytest.mark.parametrize("stereo,th,fwd,bwd,ori", [(False, 7.0, 0, 0, True), (True, 15.0, 0, 0, True),
                                                  (True, 7.0, 1, 0, True), (True, 7.0, 0, 1, False),
                                                  (False, 14.0, 0, 0, False), (False, 30.0, 0, 0, True)])
def test_search_by_projection_last_frame(stereo, th, fwd, bwd, ori):
    F, _, L = scene(stereo=stereo, seed=int(th) + fwd)
    n, m = ORBmatcher(0.9, ori).SearchByProjection(F, L, th, forward=fwd, backward=bwd)
    on, om = O.search_by_projection_last(F, L, th, fwd, bwd, ori)
    assert n == on and np.array_equal(m, om)
    assert n > 200


def test_projection_edge_cases():
    F, P, L = scene(w=376, h=240, nf=400)
    # no points
    e = {k: v[:0] for k, v in P.items()}
    n, m = ORBmatcher(0.8).SearchByProjection(F, e, 1.0)
    assert n == 0 and (m == -1).all()
    # every feature already holds a MapPoint with observations
    Fall = dict(F, has_mp_obs=np.ones(len(F["keys_un"]), np.uint8))
    n, m = ORBmatcher(0.8).SearchByProjection(Fall, P, 1.0)
    assert n == 0
    # points projected outside the image are skipped (last-frame search)
    Lout = dict(L, u=L["u"] + 1000)
    n, _ = ORBmatcher(0.9).SearchByProjection(F, Lout, 7.0)
    assert n == 0
