"""The tracking-search restatement (oracle/projection_oracle.cc) against a second restatement
written here in Python/float32, line by line from ORB_SLAM2/src/Frame.cc:235-398 and
ORB_SLAM2/src/ORBmatcher.cc:45-137, 405-523, 828-1103, 1331-1474, 1604-1645 and
KeyFrame.cc:518-558.  CPU only."""
import math

import numpy as np
import pytest

from oracle import oracle as O

from projdata import fuse_scene, init_scene, scene

F32 = np.float32


def grid(F):
    g = {}
    for i, k in enumerate(F["keys_un"]):
        px = int(np.round(F32(F32(k["x"]) - F32(F["min_x"])) * F32(F["grid_w_inv"])))
        py = int(np.round(F32(F32(k["y"]) - F32(F["min_y"])) * F32(F["grid_h_inv"])))
        # std::round is half away from zero; np.round is half-even: fix the .5 cases
        for axis, (v, c) in enumerate(((k["x"], F["min_x"]), (k["y"], F["min_y"]))):
            t = F32(F32(v) - F32(c)) * F32(F["grid_w_inv"] if axis == 0 else F["grid_h_inv"])
            r = math.floor(abs(float(t)) + 0.5) * (1 if t >= 0 else -1)
            if axis == 0:
                px = r
            else:
                py = r
        if 0 <= px < 64 and 0 <= py < 48:
            g.setdefault((px, py), []).append(i)
    return g


def in_area(F, g, x, y, r, minLevel=-1, maxLevel=-1):
    x, y, r = F32(x), F32(y), F32(r)
    gw, gh = F32(F["grid_w_inv"]), F32(F["grid_h_inv"])
    mx, my = F32(F["min_x"]), F32(F["min_y"])
    x0 = max(0, int(math.floor(F32(F32(x - mx) - r) * gw)))
    if x0 >= 64:
        return []
    x1 = min(63, int(math.ceil(F32(F32(x - mx) + r) * gw)))
    if x1 < 0:
        return []
    y0 = max(0, int(math.floor(F32(F32(y - my) - r) * gh)))
    if y0 >= 48:
        return []
    y1 = min(47, int(math.ceil(F32(F32(y - my) + r) * gh)))
    if y1 < 0:
        return []
    check = minLevel > 0 or maxLevel >= 0
    out = []
    for ix in range(x0, x1 + 1):
        for iy in range(y0, y1 + 1):
            for i in g.get((ix, iy), []):
                k = F["keys_un"][i]
                if check and (k["octave"] < minLevel or (maxLevel >= 0 and k["octave"] > maxLevel)):
                    continue
                if abs(F32(k["x"]) - x) < r and abs(F32(k["y"]) - y) < r:
                    out.append(i)
    return out


def ham(a, b):
    return int(np.unpackbits(np.bitwise_xor(a, b)).sum())


def py_local(F, P, th, nnratio):
    g = grid(F)
    n = len(F["keys_un"])
    claimed = [bool(F["has_mp_obs"][i]) for i in range(n)]
    match = [-1] * n
    nm = 0
    sc = F["scale_factors"]
    for i in range(len(P["track"])):
        if not P["track"][i]:
            continue
        lev = int(P["pred_level"][i])
        r = F32(2.5) if float(P["view_cos"][i]) > 0.998 else F32(4.0)
        if th != 1.0:
            r = F32(r * F32(th))
        rs = F32(r * F32(sc[lev]))
        idxs = in_area(F, g, P["proj_x"][i], P["proj_y"][i], rs, lev - 1, lev)
        bd, bl, bd2, bl2, bi = 256, -1, 256, -1, -1
        for idx in idxs:
            if claimed[idx]:
                continue
            if F["u_right"] is not None and F["u_right"][idx] > 0:
                if abs(F32(P["proj_xr"][i]) - F32(F["u_right"][idx])) > rs:
                    continue
            d = ham(P["desc"][i], F["desc"][idx])
            if d < bd:
                bd2, bd, bl2, bl, bi = bd, d, bl, int(F["keys_un"][idx]["octave"]), idx
            elif d < bd2:
                bl2, bd2 = int(F["keys_un"][idx]["octave"]), d
        if bd <= 100:
            if bl == bl2 and F32(bd) > F32(nnratio) * F32(bd2):
                continue
            match[bi] = i
            claimed[bi] = True
            nm += 1
    return nm, np.array(match, np.int32)


def py_last(F, L, th, fwd, bwd, ori, stats=None):
    g = grid(F)
    n = len(F["keys_un"])
    claimed = [bool(F["has_mp_obs"][i]) for i in range(n)]
    blocks = L.get("blocks")
    match = [-1] * n
    hist = [[] for _ in range(30)]
    nm = 0
    takeovers = 0
    for i in range(len(L["valid"])):
        if not L["valid"][i]:
            continue
        u, v = F32(L["u"][i]), F32(L["v"][i])
        if u < F["min_x"] or u > F["max_x"] or v < F["min_y"] or v > F["max_y"]:
            continue
        o = int(L["octave"][i])
        rad = F32(F32(th) * F32(F["scale_factors"][o]))
        if fwd:
            idxs = in_area(F, g, u, v, rad, o, -1)
        elif bwd:
            idxs = in_area(F, g, u, v, rad, 0, o)
        else:
            idxs = in_area(F, g, u, v, rad, o - 1, o + 1)
        bd, bi = 256, -1
        for idx in idxs:
            if claimed[idx]:
                continue
            if F["u_right"] is not None and F["u_right"][idx] > 0:
                if abs(F32(L["ur"][i]) - F32(F["u_right"][idx])) > rad:
                    continue
            d = ham(L["desc"][i], F["desc"][idx])
            if d < bd:
                bd, bi = d, idx
        if bd <= 100:
            takeovers += match[bi] >= 0
            match[bi] = i  # CurrentFrame.mvpMapPoints[bestIdx2] = pMP (:1431)
            # only a point with observations makes later points skip the feature (:1406-1408)
            claimed[bi] = blocks is None or bool(blocks[i])
            nm += 1
            if ori:
                rot = F32(F32(L["angle"][i]) - F32(F["keys_un"][bi]["angle"]))
                if rot < 0:
                    rot = F32(rot + F32(360))
                t = F32(rot * F32(F32(1) / F32(30)))
                b = int(math.floor(abs(float(t)) + 0.5))
                hist[0 if b == 30 else b].append(bi)
    if ori:
        m1 = m2 = m3 = 0
        i1 = i2 = i3 = -1
        for b in range(30):
            s = len(hist[b])
            if s > m1:
                m3, m2, m1, i3, i2, i1 = m2, m1, s, i2, i1, b
            elif s > m2:
                m3, m2, i3, i2 = m2, s, i2, b
            elif s > m3:
                m3, i3 = s, b
        if m2 < F32(0.1) * F32(m1):
            i2 = i3 = -1
        elif m3 < F32(0.1) * F32(m1):
            i3 = -1
        for b in range(30):
            if b not in (i1, i2, i3):
                for idx in hist[b]:
                    match[idx] = -1
                    nm -= 1
    if stats is not None:
        stats["takeovers"] = takeovers
        stats["hist"] = hist
        stats["kept"] = {i1, i2, i3} - {-1} if ori else set(range(30))
    return nm, np.array(match, np.int32)


@pytest.mark.parametrize("stereo", [False, True])
def test_features_in_area_order(stereo):
    F, P, _ = scene(stereo=stereo)
    g = grid(F)
    rng = np.random.default_rng(1)
    for _ in range(40):
        x, y = rng.uniform(-20, 660), rng.uniform(-20, 500)
        r = rng.uniform(1, 60)
        lo, hi = int(rng.integers(-1, 4)), int(rng.integers(-1, 8))
        assert O.features_in_area(F, x, y, r, lo, hi).tolist() == in_area(F, g, x, y, r, lo, hi)


@pytest.mark.parametrize("stereo,th", [(False, 1.0), (True, 1.0), (False, 3.0), (True, 5.0)])
def test_search_by_projection_local_map(stereo, th):
    F, P, _ = scene(stereo=stereo, seed=int(th))
    n, m = O.search_by_projection(F, P, th, 0.8)
    pn, pm = py_local(F, P, th, 0.8)
    assert n == pn and np.array_equal(m, pm)
    assert n > 200


@pytest.mark.parametrize("stereo,th,fwd,bwd,ori", [(False, 7.0, 0, 0, True), (True, 15.0, 0, 0, True),
                                                  (True, 7.0, 1, 0, True), (True, 7.0, 0, 1, False),
                                                  (False, 14.0, 0, 0, False)])
def test_search_by_projection_last_frame(stereo, th, fwd, bwd, ori):
    F, _, L = scene(stereo=stereo, seed=int(th) + fwd)
    n, m = O.search_by_projection_last(F, L, th, fwd, bwd, ori)
    pn, pm = py_last(F, L, th, fwd, bwd, ori)
    assert n == pn and np.array_equal(m, pm)
    assert n > 200


def last_with_vo_points(L, seed):
    """The last frame as Tracking::UpdateLastFrame leaves it for stereo / RGB-D
    (Tracking.cc:1181-1221): some of its points are visual-odometry points with no observations.
    Every point is listed twice so that a feature one of them wins stays open to its copy."""
    rng = np.random.default_rng(seed)
    L2 = {k: (None if v is None else np.concatenate([v, v])) for k, v in L.items()}
    L2["blocks"] = (rng.random(len(L2["valid"])) < 0.5).astype(np.uint8)
    return L2


@pytest.mark.parametrize("stereo,th,fwd,bwd,ori", [(True, 7.0, 0, 0, True), (True, 15.0, 1, 0, True),
                                                  (False, 7.0, 0, 0, False), (True, 7.0, 0, 1, True)])
def test_search_by_projection_last_frame_vo_points(stereo, th, fwd, bwd, ori):
    """ORBmatcher.cc:1406-1408: a feature assigned a point without observations is not skipped
    by later points; the later point takes it over and nmatches / rotHist count both."""
    F, _, L = scene(stereo=stereo, seed=int(th) + fwd)
    L2 = last_with_vo_points(L, int(th))
    n, m = O.search_by_projection_last(F, L2, th, fwd, bwd, ori)
    st = {}
    pn, pm = py_last(F, L2, th, fwd, bwd, ori, st)
    assert n == pn and np.array_equal(m, pm)
    assert st["takeovers"] > 50
    # every point blocking is the same search as blocks = NULL
    L2["blocks"][:] = 1
    n1, m1 = O.search_by_projection_last(F, L2, th, fwd, bwd, ori)
    n0, m0 = O.search_by_projection_last(F, dict(L2, blocks=None), th, fwd, bwd, ori)
    assert n1 == n0 and np.array_equal(m1, m0)


def last_with_split_takeovers(L, seed):
    """last_with_vo_points with the copies' angles turned by 150 degrees: a copy that takes a
    feature over lands in a rotation bin 5 away from the original's, so the feature has one
    histogram entry inside the three maxima and one outside (ORBmatcher.cc:1440-1468).  The
    reference nulls mvpMapPoints[feature] for the entry outside — whichever point holds it by
    then — and decrements nmatches once per such entry."""
    L2 = last_with_vo_points(L, seed)
    n0 = len(L["valid"])
    L2["angle"] = L2["angle"].copy()
    L2["angle"][n0:] = np.mod(L2["angle"][n0:] + np.float32(150), np.float32(360)).astype(np.float32)
    L2["blocks"][:n0] = 0  # every original is a visual-odometry point: its copy may take over
    return L2


def split_takeover_features(hist, kept):
    """Features with one rotation-histogram entry in a kept bin and one in a removed bin."""
    inside = {i for b in kept for i in hist[b]}
    outside = {i for b in range(30) if b not in kept for i in hist[b]}
    return sorted(inside & outside), sum(len(hist[b]) for b in range(30) if b not in kept)


@pytest.mark.parametrize("stereo,th,fwd", [(True, 7.0, 0), (False, 15.0, 1)])
def test_search_by_projection_last_frame_split_takeovers(stereo, th, fwd):
    """A feature taken over (advisor, round 4): its two rotHist entries straddle the top-3 cut.
    The oracle's log-based removal equals the Python restatement, every such feature ends
    unmatched, and nmatches = assignments - entries in the removed bins."""
    F, _, L = scene(stereo=stereo, seed=int(th) + fwd)
    L2 = last_with_split_takeovers(L, int(th))
    n, m = O.search_by_projection_last(F, L2, th, fwd, 0, True)
    st = {}
    pn, pm = py_last(F, L2, th, fwd, 0, True, st)
    assert n == pn and np.array_equal(m, pm)
    split, removed = split_takeover_features(st["hist"], st["kept"])
    assert len(split) >= 10
    assert (m[split] == -1).all()
    assigned = sum(len(b) for b in st["hist"])
    assert n == assigned - removed


def three_maxima(counts):
    m1 = m2 = m3 = 0
    i1 = i2 = i3 = -1
    for b in range(30):
        s = counts[b]
        if s > m1:
            m3, m2, m1, i3, i2, i1 = m2, m1, s, i2, i1, b
        elif s > m2:
            m3, m2, i3, i2 = m2, s, i2, b
        elif s > m3:
            m3, i3 = s, b
    if m2 < F32(0.1) * F32(m1):
        i2 = i3 = -1
    elif m3 < F32(0.1) * F32(m1):
        i3 = -1
    return i1, i2, i3


def py_init(F1, F2, prev, nnratio, ori, window):
    """SearchForInitialization, ORBmatcher.cc:405-523 line by line."""
    g = grid(F2)
    n1, n2 = len(F1["keys_un"]), len(F2["keys_un"])
    m12 = [-1] * n1
    hist = [[] for _ in range(30)]
    mdist = [2 ** 31 - 1] * n2
    m21 = [-1] * n2
    nm = 0
    for i1 in range(n1):
        lev = int(F1["keys_un"][i1]["octave"])
        if lev > 0:
            continue
        idxs = in_area(F2, g, prev[i1, 0], prev[i1, 1], F32(window), lev, lev)
        if not idxs:
            continue
        bd = bd2 = 2 ** 31 - 1
        bi = -1
        for i2 in idxs:
            d = ham(F1["desc"][i1], F2["desc"][i2])
            if mdist[i2] <= d:
                continue
            if d < bd:
                bd2, bd, bi = bd, d, i2
            elif d < bd2:
                bd2 = d
        if bd <= 50 and F32(bd) < F32(bd2) * F32(nnratio):
            if m21[bi] >= 0:
                m12[m21[bi]] = -1
                nm -= 1
            m12[i1] = bi
            m21[bi] = i1
            mdist[bi] = bd
            nm += 1
            if ori:
                rot = F32(F32(F1["keys_un"][i1]["angle"]) - F32(F2["keys_un"][bi]["angle"]))
                if rot < 0:
                    rot = F32(rot + F32(360))
                t = F32(rot * F32(F32(1) / F32(30)))
                b = int(math.floor(abs(float(t)) + 0.5))
                hist[0 if b == 30 else b].append(i1)
    if ori:
        keep = three_maxima([len(h) for h in hist])
        for b in range(30):
            if b not in keep:
                for i1 in hist[b]:
                    if m12[i1] >= 0:
                        m12[i1] = -1
                        nm -= 1
    out = prev.copy()
    for i1 in range(n1):
        if m12[i1] >= 0:
            out[i1] = (F2["keys_un"][m12[i1]]["x"], F2["keys_un"][m12[i1]]["y"])
    return nm, np.array(m12, np.int32), out


@pytest.mark.parametrize("t1,jitter,nn,ori,window", [(6, 0.0, 0.9, True, 100), (4, 3.0, 0.9, True, 100),
                                                     (9, 0.0, 0.7, False, 50), (5, 8.0, 1.0, True, 10)])
def test_search_for_initialization(t1, jitter, nn, ori, window):
    F1, F2, prev = init_scene(t1=t1, jitter=jitter, seed=t1)
    n, m, pv = O.search_for_initialization(F1, F2, prev, nn, ori, window)
    pn, pm, ppv = py_init(F1, F2, prev, nn, ori, window)
    assert n == pn and np.array_equal(m, pm)
    assert pv.tobytes() == ppv.tobytes()
    assert n > 100
    assert (m >= 0).sum() == n


def py_fuse(K, P, th, reproj):
    """Fuse's per-point search, ORBmatcher.cc:845-975 (reproj) / 1003-1099, with the reference
    binary's contraction of e2 emulated by exact float64 products rounded once."""
    g = grid(K)
    none = 256 if reproj else 2 ** 31 - 1
    out_i, out_d = [], []
    isg = K["inv_level_sigma2"]

    def fma(a, b, c):  # float32 fused multiply-add: the exact double result rounded once
        return F32(float(a) * float(b) + float(c))

    for i in range(len(P["use"])):
        bi, bd = -1, none
        if P["use"][i]:
            lev = int(P["pred_level"][i])
            u, v = F32(P["u"][i]), F32(P["v"][i])
            rad = F32(F32(th) * F32(K["scale_factors"][lev]))
            for idx in in_area(K, g, u, v, rad):
                k = K["keys_un"][idx]
                kl = int(k["octave"])
                if kl < lev - 1 or kl > lev:
                    continue
                if reproj:
                    ex, ey = F32(u - F32(k["x"])), F32(v - F32(k["y"]))
                    if K["u_right"] is not None and K["u_right"][idx] >= 0:
                        er = F32(F32(P["ur"][i]) - F32(K["u_right"][idx]))
                        e2 = fma(er, er, fma(ex, ex, F32(ey * ey)))
                        if float(F32(e2 * F32(isg[kl]))) > 7.8:
                            continue
                    else:
                        e2 = fma(ex, ex, F32(ey * ey))
                        if float(F32(e2 * F32(isg[kl]))) > 5.99:
                            continue
                d = ham(P["desc"][i], K["desc"][idx])
                if d < bd:
                    bd, bi = d, idx
        out_d.append(bd)
        out_i.append(bi if bd <= 50 else -1)
    return np.array(out_i, np.int32), np.array(out_d, np.int32)


@pytest.mark.parametrize("stereo,th,reproj", [(False, 3.0, True), (True, 3.0, True),
                                              (True, 1.0, True), (False, 10.0, False)])
def test_fuse(stereo, th, reproj):
    K, P = fuse_scene(stereo=stereo, seed=int(th))
    n, bi, bd = O.fuse(K, K["inv_level_sigma2"], P, th, reproj)
    pi, pd = py_fuse(K, P, th, reproj)
    assert np.array_equal(bi, pi) and np.array_equal(bd, pd)
    assert n == (pi >= 0).sum() and n > 100


def _rot_bin(a_point, a_feat):
    rot = F32(F32(a_point) - F32(a_feat))
    if rot < 0:
        rot = F32(rot + F32(360))
    t = F32(rot * F32(F32(1) / F32(30)))
    b = int(math.floor(abs(float(t)) + 0.5))
    return 0 if b == 30 else b


def _keep_three_maxima(hist, match, nm):
    """ComputeThreeMaxima (ORBmatcher.cc:1604-1645) and the removal of the other bins."""
    m1 = m2 = m3 = 0
    i1 = i2 = i3 = -1
    for b in range(30):
        s = len(hist[b])
        if s > m1:
            m3, m2, m1, i3, i2, i1 = m2, m1, s, i2, i1, b
        elif s > m2:
            m3, m2, i3, i2 = m2, s, i2, b
        elif s > m3:
            m3, i3 = s, b
    if m2 < F32(0.1) * F32(m1):
        i2 = i3 = -1
    elif m3 < F32(0.1) * F32(m1):
        i3 = -1
    for b in range(30):
        if b not in (i1, i2, i3):
            for idx in hist[b]:
                match[idx] = -1
                nm -= 1
    return nm


def py_reloc(F, L, th, orb_dist, ori):
    """SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist), ORBmatcher.cc:1475-1602."""
    g = grid(F)
    n = len(F["keys_un"])
    has = [bool(F["has_mp_obs"][i]) for i in range(n)]
    match = [-1] * n
    hist = [[] for _ in range(30)]
    nm = 0
    for i in range(len(L["valid"])):
        if not L["valid"][i]:
            continue
        u, v = F32(L["u"][i]), F32(L["v"][i])
        if u < F["min_x"] or u > F["max_x"] or v < F["min_y"] or v > F["max_y"]:
            continue
        lev = int(L["octave"][i])
        rad = F32(F32(th) * F32(F["scale_factors"][lev]))
        bd, bi = 256, -1
        for idx in in_area(F, g, u, v, rad, lev - 1, lev + 1):
            if has[idx]:
                continue
            d = ham(L["desc"][i], F["desc"][idx])
            if d < bd:
                bd, bi = d, idx
        if bd <= orb_dist:
            has[bi] = True
            match[bi] = i
            nm += 1
            if ori:
                hist[_rot_bin(L["angle"][i], F["keys_un"][bi]["angle"])].append(bi)
    if ori:
        nm = _keep_three_maxima(hist, match, nm)
    return nm, np.array(match, np.int32)


def py_proj_sim3(K, P, th):
    """SearchByProjection(pKF, Scw, vpPoints, vpMatched, th), ORBmatcher.cc:290-403."""
    g = grid(K)
    n = len(K["keys_un"])
    matched = [bool(K["has_mp_obs"][i]) for i in range(n)]
    match = [-1] * n
    nm = 0
    for i in range(len(P["use"])):
        if not P["use"][i]:
            continue
        lev = int(P["pred_level"][i])
        rad = F32(F32(th) * F32(K["scale_factors"][lev]))
        bd, bi = 256, -1
        for idx in in_area(K, g, F32(P["u"][i]), F32(P["v"][i]), rad):
            if matched[idx]:
                continue
            kl = int(K["keys_un"][idx]["octave"])
            if kl < lev - 1 or kl > lev:
                continue
            d = ham(P["desc"][i], K["desc"][idx])
            if d < bd:
                bd, bi = d, idx
        if bd <= 50:
            matched[bi] = True
            match[bi] = i
            nm += 1
    return nm, np.array(match, np.int32)


def py_search_by_sim3(K1, K2, P12, P21, th):
    """SearchBySim3, ORBmatcher.cc:1105-1329 (the two per-point searches and the agreement)."""
    def direction(K, P):
        g = grid(K)
        out = []
        for i in range(len(P["use"])):
            best = -1
            if P["use"][i]:
                lev = int(P["pred_level"][i])
                rad = F32(F32(th) * F32(K["scale_factors"][lev]))
                bd, bi = 2 ** 31 - 1, -1
                for idx in in_area(K, g, F32(P["u"][i]), F32(P["v"][i]), rad):
                    kl = int(K["keys_un"][idx]["octave"])
                    if kl < lev - 1 or kl > lev:
                        continue
                    d = ham(P["desc"][i], K["desc"][idx])
                    if d < bd:
                        bd, bi = d, idx
                if bd <= 100:
                    best = bi
            out.append(best)
        return out
    v1, v2 = direction(K2, P12), direction(K1, P21)
    m12 = [-1] * len(v1)
    for i1, idx2 in enumerate(v1):
        if idx2 >= 0 and v2[idx2] == i1:
            m12[i1] = idx2
    m12 = np.array(m12, np.int32)
    return int((m12 >= 0).sum()), m12


@pytest.mark.parametrize("th,orb_dist,ori", [(10.0, 100, True), (10.0, 50, False), (5.0, 64, True)])
def test_search_by_projection_relocalization(th, orb_dist, ori):
    from projdata import reloc_scene
    F, L = reloc_scene(seed=int(th) + orb_dist)
    n, m = O.search_by_projection_kf(F, L, th, orb_dist, ori)
    pn, pm = py_reloc(F, L, th, orb_dist, ori)
    assert n == pn and np.array_equal(m, pm)
    assert n > 100


@pytest.mark.parametrize("th,seed", [(10.0, 0), (5.0, 1)])
def test_search_by_projection_sim3(th, seed):
    from projdata import loop_scene
    K, P = loop_scene(seed=seed)
    n, m = O.search_by_projection_sim3(K, P, th)
    pn, pm = py_proj_sim3(K, P, th)
    assert n == pn and np.array_equal(m, pm)
    assert n > 100


@pytest.mark.parametrize("th,seed", [(7.5, 0), (3.0, 1)])
def test_search_by_sim3(th, seed):
    from projdata import sim3_scene
    K1, K2, P12, P21 = sim3_scene(seed=seed)
    n, m = O.search_by_sim3(K1, K2, P12, P21, th)
    pn, pm = py_search_by_sim3(K1, K2, P12, P21, th)
    assert n == pn and np.array_equal(m, pm)
    assert n > 100
