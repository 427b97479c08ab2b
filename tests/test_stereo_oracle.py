"""Frame::ComputeStereoMatches restatement (oracle/stereo_oracle.cc) against a second,
independent restatement written here in numpy float32 (ORB_SLAM2/src/Frame.cc:471-643), on
synthetic rectified stereo pairs with known disparities.  CPU only."""
import math

import numpy as np
import pytest

from ar_orbslam2_amd import synth
from ar_orbslam2_amd.stereo import stereo_params
from oracle import oracle as O

F32 = np.float32
EUROC = stereo_params(47.90639384423901, 435.2046959714599)  # Examples/Stereo/EuRoC.yaml


def py_stereo(kl, dl, kr, dr, pl, pr, scale, inv_scale, mb, mbf):
    """Frame.cc:471-643 line by line, float32 where the reference uses float."""
    N = len(kl)
    ur = np.full(N, -1, F32)
    dp = np.full(N, -1, F32)
    nrows = pl[0].shape[0]
    rows = [[] for _ in range(nrows)]
    for iR, k in enumerate(kr):
        r = F32(2.0) * F32(scale[k["octave"]])
        for yi in range(int(math.floor(F32(k["y"]) - r)), int(math.ceil(F32(k["y"]) + r)) + 1):
            rows[yi].append(iR)
    maxD = F32(mbf) / F32(mb)
    minD = F32(-3)
    pairs = []
    pop = np.unpackbits(np.bitwise_xor(dl[:, None, :], dr[None, :, :]), axis=2).sum(2)
    for iL, k in enumerate(kl):
        lev = int(k["octave"])
        vL, uL = F32(k["y"]), F32(k["x"])
        cand = rows[int(vL)]
        if not cand:
            continue
        minU, maxU = uL - maxD, uL - minD
        if maxU < 0:
            continue
        best, bi = 100, 0
        for iR in cand:
            if kr[iR]["octave"] < lev - 1 or kr[iR]["octave"] > lev + 1:
                continue
            uR = F32(kr[iR]["x"])
            if minU <= uR <= maxU and pop[iL, iR] < best:
                best, bi = int(pop[iL, iR]), iR
        if best >= 100:
            continue
        sf = F32(inv_scale[lev])
        rnd = lambda v: F32(math.floor(abs(float(v)) + 0.5) * (1 if v >= 0 else -1))  # noqa
        suL, svL, suR0 = rnd(F32(k["x"]) * sf), rnd(F32(k["y"]) * sf), rnd(F32(kr[bi]["x"]) * sf)
        w = L = 5
        if suR0 + L - w < 0 or suR0 + L + w + 1 >= pr[lev].shape[1]:
            continue
        y0, xl0 = int(svL) - w, int(suL) - w
        IL = pl[lev][y0:y0 + 11, xl0:xl0 + 11].astype(F32)
        IL = IL - IL[w, w]
        dists = []
        for inc in range(-L, L + 1):
            xr0 = int(suR0) + inc - w
            IR = pr[lev][y0:y0 + 11, xr0:xr0 + 11].astype(F32)
            IR = IR - IR[w, w]
            dists.append(F32(np.abs((IL - IR).astype(np.float64)).sum()))
        binc = int(np.argmin(dists)) - L  # first minimum
        if binc in (-L, L):
            continue
        d1, d2, d3 = dists[L + binc - 1], dists[L + binc], dists[L + binc + 1]
        with np.errstate(divide="ignore", invalid="ignore"):
            dR = F32(d1 - d3) / F32(F32(2) * (d1 + d3 - F32(2) * d2))
        if dR < -1 or dR > 1:
            continue
        buR = F32(scale[lev]) * (suR0 + F32(binc) + dR)
        disp = uL - buR
        if disp >= 0 and disp < maxD:
            if disp <= 0:
                disp, buR = F32(0.01), F32(float(uL) - 0.01)
            dp[iL], ur[iL] = F32(mbf) / disp, buR
            pairs.append((int(dists[L + binc]), iL))
    if pairs:
        pairs.sort()
        th = F32(F32(1.5) * F32(1.4)) * F32(pairs[len(pairs) // 2][0])
        for d, i in pairs[::-1]:
            if F32(d) < th:
                break
            ur[i] = dp[i] = -1
    return ur, dp


def _pair(w, h, nf, t, disparity=(12, 20)):
    l, r = synth.stereo_pair(w, h, t, 0, disparity)
    p = O.params(nf)
    kl, dl, pl, _ = O.extract(l, p, want_pyramid=True)
    kr, dr, pr, _ = O.extract(r, p, want_pyramid=True)
    return kl, dl, kr, dr, pl, pr, O.tables(p, w, h)


@pytest.mark.parametrize("t", [0, 5])
def test_oracle_equals_independent_restatement(t):
    kl, dl, kr, dr, pl, pr, tb = _pair(376, 240, 600, t)
    a = O.stereo_matches(kl, dl, kr, dr, pl, pr, tb["scale"], tb["inv_scale"], *EUROC)
    b = py_stereo(kl, dl, kr, dr, pl, pr, tb["scale"], tb["inv_scale"], *EUROC)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    assert (a[0] >= 0).sum() > 100


def test_known_disparities_recovered():
    kl, dl, kr, dr, pl, pr, tb = _pair(752, 480, 1200, 3)
    ur, dp, sad = O.stereo_matches(kl, dl, kr, dr, pl, pr, tb["scale"], tb["inv_scale"], *EUROC)
    m = ur >= 0
    assert m.sum() > 400
    disp = (kl["x"] - ur)[m]
    # background plane d=12, nearer plane d=20 (synth.stereo_pair)
    assert np.median(disp) == pytest.approx(12, abs=0.5)
    assert ((np.abs(disp - 12) < 1.5) | (np.abs(disp - 20) < 1.5)).mean() > 0.9
    # depth = mbf / disparity for every retained match, SAD kept for exactly those
    assert np.array_equal(dp[m], (np.float32(EUROC[1]) / (kl["x"] - ur)[m]).astype(np.float32)) \
        or np.allclose(dp[m], EUROC[1] / disp, rtol=1e-6)
    assert ((sad >= 0) == m).all()


def test_no_right_keypoints_and_out_of_range_disparity():
    kl, dl, kr, dr, pl, pr, tb = _pair(376, 240, 600, 1)
    ur, dp, _ = O.stereo_matches(kl, dl, kr[:0], dr[:0], pl, pr, tb["scale"], tb["inv_scale"],
                                 *EUROC)
    assert (ur == -1).all() and (dp == -1).all()
    # maxD = mbf / mb = fx: with fx tiny no disparity of 12 px is admissible
    mb, mbf = stereo_params(1.0, 0.001)  # maxD = mbf / mb = fx = 0.001 px
    ur, _, _ = O.stereo_matches(kl, dl, kr, dr, pl, pr, tb["scale"], tb["inv_scale"], mb, mbf)
    assert (ur == -1).all()
