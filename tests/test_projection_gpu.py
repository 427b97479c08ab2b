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


@pytest.mark.parametrize("stereo,th,fwd,bwd,ori", [(True, 7.0, 0, 0, True), (True, 15.0, 1, 0, True),
                                                  (False, 7.0, 0, 0, False), (True, 7.0, 0, 1, True),
                                                  (False, 30.0, 0, 0, True)])
def test_search_by_projection_last_frame_vo_points(stereo, th, fwd, bwd, ori):
    """Last-frame points without observations (Tracking::UpdateLastFrame's visual-odometry
    points, Tracking.cc:1181-1221) do not block their feature (ORBmatcher.cc:1406-1408): later
    points take it over, nmatches and the rotation histogram count every assignment."""
    from test_projection_oracle import last_with_vo_points
    F, _, L = scene(stereo=stereo, seed=int(th) + fwd)
    L2 = last_with_vo_points(L, int(th))
    n, m = ORBmatcher(0.9, ori).SearchByProjection(F, L2, th, forward=fwd, backward=bwd)
    on, om = O.search_by_projection_last(F, L2, th, fwd, bwd, ori)
    assert n == on and np.array_equal(m, om)
    assert (om >= len(L["valid"])).any()  # some copies took their feature over


@pytest.mark.parametrize("stereo,th,fwd", [(True, 7.0, 0), (False, 15.0, 1)])
def test_search_by_projection_last_frame_split_takeovers(stereo, th, fwd):
    """A feature taken over by a point whose rotation bin is on the other side of the top-3 cut
    (ORBmatcher.cc:1440-1468, advisor round 4): k_proj_resolve's log-based removal nulls it and
    counts each removed entry once, as the oracle and its Python restatement do."""
    from test_projection_oracle import last_with_split_takeovers, py_last, split_takeover_features
    F, _, L = scene(stereo=stereo, seed=int(th) + fwd)
    L2 = last_with_split_takeovers(L, int(th))
    n, m = ORBmatcher(0.9, True).SearchByProjection(F, L2, th, forward=fwd, backward=0)
    on, om = O.search_by_projection_last(F, L2, th, fwd, 0, True)
    assert n == on and np.array_equal(m, om)
    st = {}
    py_last(F, L2, th, fwd, 0, True, st)
    split, removed = split_takeover_features(st["hist"], st["kept"])
    assert len(split) >= 10 and (m[split] == -1).all()
    assert n == sum(len(b) for b in st["hist"]) - removed


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


@pytest.mark.parametrize("t1,jitter,nn,ori,window", [(6, 0.0, 0.9, True, 100), (4, 3.0, 0.9, True, 100),
                                                     (9, 0.0, 0.7, False, 50), (5, 8.0, 1.0, True, 10)])
def test_search_for_initialization(t1, jitter, nn, ori, window):
    """SearchForInitialization (ORBmatcher.cc:405-523), as Tracking::MonocularInitialization
    calls it (Tracking.cc:953: window 100, ORBmatcher(0.9, true)): vnMatches12, the count and the
    updated vbPrevMatched equal the oracle's."""
    from projdata import init_scene
    F1, F2, prev = init_scene(t1=t1, jitter=jitter, seed=t1)
    on, om, opv = O.search_for_initialization(F1, F2, prev, nn, ori, window)
    pv = prev.copy()
    n, m = ORBmatcher(nn, ori).SearchForInitialization(F1, F2, pv, window)
    assert n == on and np.array_equal(m, om)
    assert pv.tobytes() == opv.tobytes()
    assert n > 100


def test_search_for_initialization_edge_cases():
    from projdata import init_scene
    F1, F2, prev = init_scene()
    # a window covering the whole frame: every level-0 feature of F2 (~430) is a candidate of
    # each level-0 F1 feature, more than the candidate pool's first size (256 per point), so
    # the call reruns with the pool sized to the total
    assert (F2["keys_un"]["octave"] == 0).sum() > 300
    sel = np.nonzero(F1["keys_un"]["octave"] == 0)[0][:20]
    F1s = dict(F1, keys_un=F1["keys_un"][sel], desc=F1["desc"][sel])
    p1 = prev[sel].copy()
    on, om, opv = O.search_for_initialization(F1s, F2, p1, 0.9, True, 1000)
    n, m = ORBmatcher(0.9, True).SearchForInitialization(F1s, F2, p1, 1000)
    assert n == on and np.array_equal(m, om) and p1.tobytes() == opv.tobytes()
    # empty frames
    e1 = dict(F1, keys_un=F1["keys_un"][:0], desc=F1["desc"][:0])
    n, m = ORBmatcher(0.9, True).SearchForInitialization(e1, F2, np.zeros((0, 2), np.float32), 100)
    assert n == 0 and len(m) == 0
    e2 = dict(F2, keys_un=F2["keys_un"][:0], desc=F2["desc"][:0])
    pv = prev.copy()
    n, m = ORBmatcher(0.9, True).SearchForInitialization(F1, e2, pv, 100)
    assert n == 0 and (m == -1).all() and pv.tobytes() == prev.tobytes()


@pytest.mark.parametrize("stereo,th,sim3,seed", [(False, 3.0, False, 0), (True, 3.0, False, 1),
                                                 (True, 1.0, False, 2), (False, 10.0, True, 3),
                                                 (True, 3.0, True, 4)])
def test_fuse(stereo, th, sim3, seed):
    """ORBmatcher::Fuse's per-point search, both overloads (ORBmatcher.cc:828-978, 980-1103):
    best index and distance of every point equal the oracle's."""
    from projdata import fuse_scene
    K, P = fuse_scene(stereo=stereo, seed=seed)
    on, obi, obd = O.fuse(K, K["inv_level_sigma2"], P, th, not sim3)
    n, bi, bd = ORBmatcher(0.6, True).Fuse(K, P, th, sim3=sim3)
    assert n == on and np.array_equal(bi, obi) and np.array_equal(bd, obd)
    assert n > 100


def test_fuse_edge_cases():
    from projdata import fuse_scene
    K, P = fuse_scene(w=376, h=240, nf=400)
    e = {k: v[:0] for k, v in P.items()}
    n, bi, bd = ORBmatcher().Fuse(K, e, 3.0)
    assert n == 0 and len(bi) == 0
    # no point passes the caller's gates
    n, bi, bd = ORBmatcher().Fuse(K, dict(P, use=np.zeros_like(P["use"])), 3.0)
    assert n == 0 and (bi == -1).all() and (bd == 256).all()
    # projections outside the keyframe's grid
    n, bi, _ = ORBmatcher().Fuse(K, dict(P, u=P["u"] + 5000), 3.0, sim3=True)
    assert n == 0 and (bi == -1).all()


@pytest.mark.parametrize("th,orb_dist,ori", [(10.0, 100, True), (10.0, 50, False), (5.0, 64, True)])
def test_search_by_projection_relocalization(th, orb_dist, ori):
    """SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist) (ORBmatcher.cc:1475-1602),
    as Tracking::Relocalization calls it (th 10 / ORBdist 100, then th 3 / 64): match array and
    count equal the oracle's."""
    from projdata import reloc_scene
    F, L = reloc_scene(seed=int(th) + orb_dist)
    on, om = O.search_by_projection_kf(F, L, th, orb_dist, ori)
    n, m = ORBmatcher(0.75, ori).SearchByProjectionKF(F, L, th, orb_dist)
    assert n == on and np.array_equal(m, om)
    assert n > 100


@pytest.mark.parametrize("th,seed", [(10.0, 0), (5.0, 1)])
def test_search_by_projection_sim3(th, seed):
    """SearchByProjection(pKF, Scw, vpPoints, vpMatched, th) (ORBmatcher.cc:290-403)."""
    from projdata import loop_scene
    K, P = loop_scene(seed=seed)
    on, om = O.search_by_projection_sim3(K, P, th)
    n, m = ORBmatcher(0.75, True).SearchByProjectionSim3(K, P, th)
    assert n == on and np.array_equal(m, om)
    assert n > 100


@pytest.mark.parametrize("th,seed", [(7.5, 0), (3.0, 1)])
def test_search_by_sim3(th, seed):
    """SearchBySim3 (ORBmatcher.cc:1105-1329; LoopClosing::ComputeSim3, th 7.5): both directions'
    searches and the agreement equal the oracle's."""
    from projdata import sim3_scene
    K1, K2, P12, P21 = sim3_scene(seed=seed)
    on, om = O.search_by_sim3(K1, K2, P12, P21, th)
    n, m = ORBmatcher(0.75, True).SearchBySim3(K1, K2, P12, P21, th)
    assert n == on and np.array_equal(m, om)
    assert n > 100


def test_relocalization_and_loop_searches_edge_cases():
    from projdata import loop_scene, reloc_scene, sim3_scene
    F, L = reloc_scene()
    mt = ORBmatcher(0.75, True)
    # every current feature already holds a map point: nothing can be assigned
    n, m = mt.SearchByProjectionKF(dict(F, has_mp_obs=np.ones(len(F["keys_un"]), np.uint8)), L, 10, 100)
    assert n == 0 and (m == -1).all()
    # no valid keyframe point / ORBdist 0
    n, _ = mt.SearchByProjectionKF(F, dict(L, valid=np.zeros_like(L["valid"])), 10, 100)
    assert n == 0
    on, om = O.search_by_projection_kf(F, L, 10, 0, True)
    n, m = mt.SearchByProjectionKF(F, L, 10, 0)
    assert n == on and np.array_equal(m, om)
    K, P = loop_scene()
    e = {k: v[:0] for k, v in P.items()}
    n, m = mt.SearchByProjectionSim3(K, e, 10)
    assert n == 0 and (m == -1).all()
    K1, K2, P12, P21 = sim3_scene()
    # nothing usable in one direction: no agreement
    n, m = mt.SearchBySim3(K1, K2, P12, dict(P21, use=np.zeros_like(P21["use"])), 7.5)
    assert n == 0 and (m == -1).all()
