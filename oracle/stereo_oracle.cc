// stereo_oracle.cc — CPU restatement of Frame::ComputeStereoMatches
// (ORB_SLAM2/src/Frame.cc:471-643).  TEST INFRASTRUCTURE ONLY (see orb_oracle.h): the checker
// for the product's stereo kernels, never linked into the product.
//
// Arithmetic follows the reference's types: float keypoint math, `round` (half away from
// zero) for the level coordinates, cv::norm(IL, IR, NORM_L1) of the centred 11x11 float
// windows — every term an integer, so the double sum is exact and equals the integer SAD —
// float parabola, `uL - 0.01` in double, the int-vs-float comparisons of the median filter.
// The one undefined case, an empty vDistIdx (`vDistIdx[0]` of an empty vector), is defined
// here as "no filtering".
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <utility>
#include <vector>

#include "orb_oracle.h"

namespace {

int hamming(const uint8_t* a, const uint8_t* b) {
  int d = 0;
  for (int i = 0; i < 32; i++) d += __builtin_popcount((unsigned)(a[i] ^ b[i]));
  return d;
}

}  // namespace

extern "C" {

// pyrL/pyrR: per level, pointer to the level image (w_l x h_l, row stride stride_l bytes).
void oracle_stereo_matches(const orbx_keypoint* kl, int nl, const uint8_t* dl,
                           const orbx_keypoint* kr, int nr, const uint8_t* dr,
                           const uint8_t* const* pyrL, const uint8_t* const* pyrR,
                           const int* lw, const int* lh, const int64_t* lstride,
                           const float* scale, const float* inv_scale, float mb, float mbf,
                           float* uright, float* depth, int* sad) {
  for (int i = 0; i < nl; i++) {
    uright[i] = -1.0f;
    depth[i] = -1.0f;
    if (sad) sad[i] = -1;
  }
  const int nRows = lh[0];
  std::vector<std::vector<size_t>> rows(nRows);
  for (int iR = 0; iR < nr; iR++) {  // Frame.cc:486-497
    const float kpY = kr[iR].y;
    const float r = 2.0f * scale[kr[iR].octave];
    const int maxr = (int)std::ceil(kpY + r);
    const int minr = (int)std::floor(kpY - r);
    for (int yi = minr; yi <= maxr; yi++)
      if (yi >= 0 && yi < nRows) rows[yi].push_back((size_t)iR);  // in range on real input
  }
  const float minZ = mb;
  const float minD = -3;
  const float maxD = mbf / minZ;
  std::vector<std::pair<int, int>> vDistIdx;
  for (int iL = 0; iL < nl; iL++) {
    const orbx_keypoint& kpL = kl[iL];
    const int levelL = kpL.octave;
    const float vL = kpL.y, uL = kpL.x;
    const size_t row = (size_t)vL;
    if (row >= (size_t)nRows) continue;
    const std::vector<size_t>& cand = rows[row];
    if (cand.empty()) continue;
    const float minU = uL - maxD;
    const float maxU = uL - minD;
    if (maxU < 0) continue;
    int bestDist = 100;  // ORBmatcher::TH_HIGH
    size_t bestIdxR = 0;
    for (size_t iC = 0; iC < cand.size(); iC++) {
      const size_t iR = cand[iC];
      const orbx_keypoint& kpR = kr[iR];
      if (kpR.octave < levelL - 1 || kpR.octave > levelL + 1) continue;
      const float uR = kpR.x;
      if (uR >= minU && uR <= maxU) {
        const int dist = hamming(dl + (size_t)iL * 32, dr + iR * 32);
        if (dist < bestDist) {
          bestDist = dist;
          bestIdxR = iR;
        }
      }
    }
    if (bestDist >= 100) continue;
    // subpixel match by correlation (Frame.cc:555-618)
    const float uR0 = kr[bestIdxR].x;
    const float scaleFactor = inv_scale[levelL];
    const float scaleduL = std::round(kpL.x * scaleFactor);
    const float scaledvL = std::round(kpL.y * scaleFactor);
    const float scaleduR0 = std::round(uR0 * scaleFactor);
    const int w = 5, L = 5;
    const uint8_t* PL = pyrL[levelL];
    const uint8_t* PR = pyrR[levelL];
    const int64_t sL = lstride[levelL];
    const int y0 = (int)scaledvL - w, xl0 = (int)scaleduL - w;
    const float iniu = scaleduR0 + L - w;
    const float endu = scaleduR0 + L + w + 1;
    if (iniu < 0 || endu >= lw[levelL]) continue;
    const int cL = PL[(int64_t)(y0 + w) * sL + xl0 + w];
    int bestSad = INT_MAX;
    int bestincR = 0;
    float vDists[2 * L + 1];
    for (int incR = -L; incR <= L; incR++) {
      const int xr0 = (int)scaleduR0 + incR - w;
      const int cR = PR[(int64_t)(y0 + w) * sL + xr0 + w];
      double dsum = 0;  // cv::norm NORM_L1 of float windows; every term an exact integer
      for (int yy = 0; yy < 2 * w + 1; yy++)
        for (int xx = 0; xx < 2 * w + 1; xx++) {
          const float a = (float)PL[(int64_t)(y0 + yy) * sL + xl0 + xx] - (float)cL;
          const float b = (float)PR[(int64_t)(y0 + yy) * sL + xr0 + xx] - (float)cR;
          dsum += std::fabs((double)(a - b));
        }
      const float dist = (float)dsum;
      if (dist < bestSad) {
        bestSad = (int)dist;
        bestincR = incR;
      }
      vDists[L + incR] = dist;
    }
    if (bestincR == -L || bestincR == L) continue;
    const float dist1 = vDists[L + bestincR - 1];
    const float dist2 = vDists[L + bestincR];
    const float dist3 = vDists[L + bestincR + 1];
    const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
    if (deltaR < -1 || deltaR > 1) continue;
    float bestuR = scale[levelL] * ((float)scaleduR0 + (float)bestincR + deltaR);
    float disparity = (uL - bestuR);
    if (disparity >= 0 && disparity < maxD) {
      if (disparity <= 0) {
        disparity = 0.01;
        bestuR = uL - 0.01;
      }
      depth[iL] = mbf / disparity;
      uright[iL] = bestuR;
      if (sad) sad[iL] = bestSad;
      vDistIdx.push_back(std::pair<int, int>(bestSad, iL));
    }
  }
  if (vDistIdx.empty()) return;  // the reference reads vDistIdx[0] of an empty vector
  std::sort(vDistIdx.begin(), vDistIdx.end());
  const float median = vDistIdx[vDistIdx.size() / 2].first;
  const float thDist = 1.5f * 1.4f * median;
  for (int i = (int)vDistIdx.size() - 1; i >= 0; i--) {
    if (vDistIdx[i].first < thDist) break;
    uright[vDistIdx[i].second] = -1;
    depth[vDistIdx[i].second] = -1;
    if (sad) sad[vDistIdx[i].second] = -1;
  }
}

}  // extern "C"
