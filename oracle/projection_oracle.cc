// projection_oracle.cc — CPU restatement of the tracking searches
//   Frame::AssignFeaturesToGrid / PosInGrid / GetFeaturesInArea (ORB_SLAM2/src/Frame.cc:235-250,
//     332-398)
//   ORBmatcher::SearchByProjection(Frame&, const vector<MapPoint*>&, th)   (ORBmatcher.cc:45-137)
//   ORBmatcher::SearchByProjection(Frame&, const Frame& LastFrame, th, bMono)
//                                                                          (ORBmatcher.cc:1331-1474)
//   ORBmatcher::SearchForInitialization(Frame&, Frame&, vbPrevMatched, vnMatches12, windowSize)
//                                                                          (ORBmatcher.cc:405-523)
//   ORBmatcher::Fuse(KeyFrame*, vector<MapPoint*>, th)                     (ORBmatcher.cc:828-978)
//   ORBmatcher::Fuse(KeyFrame*, Scw, vector<MapPoint*>, th, vpReplacePoint) (ORBmatcher.cc:980-1103)
//   (the per-point search; KeyFrame::GetFeaturesInArea, KeyFrame.cc:518-558)
//   ORBmatcher::SearchByProjection(Frame&, KeyFrame*, sAlreadyFound, th, ORBdist)
//                                                                          (ORBmatcher.cc:1475-1602)
//   ORBmatcher::SearchByProjection(KeyFrame*, Scw, vpPoints, vpMatched, th) (ORBmatcher.cc:290-403)
//   ORBmatcher::SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th)    (ORBmatcher.cc:1105-1329)
// TEST INFRASTRUCTURE ONLY (see orb_oracle.h).  MapPoint state enters as plain arrays: the
// caller evaluates mbTrackInView / isBad / the projections (Frame::isInFrustum, the pose
// products) exactly as the reference does and passes the results.  A frame feature matched
// earlier in the same call is skipped by the later points when its point has Observations() > 0
// (every point of the local-map and keyframe searches; per point `blocks` in the last-frame
// search, whose visual-odometry points have none, Tracking.cc:1181-1221).
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "orb_oracle.h"

namespace {

constexpr int kCols = 64, kRows = 48;  // FRAME_GRID_COLS / FRAME_GRID_ROWS (Frame.h:39-40)

int hamming(const uint8_t* a, const uint8_t* b) {
  int d = 0;
  for (int i = 0; i < 32; i++) d += __builtin_popcount((unsigned)(a[i] ^ b[i]));
  return d;
}

struct Grid {
  std::vector<int> cell[kCols][kRows];
};

void assign_grid(const orbx_proj_frame* F, Grid* G) {
  for (int i = 0; i < F->n; i++) {  // AssignFeaturesToGrid + PosInGrid
    const orbx_keypoint& kp = F->keys_un[i];
    const int posX = (int)std::round((kp.x - F->min_x) * F->grid_w_inv);
    const int posY = (int)std::round((kp.y - F->min_y) * F->grid_h_inv);
    if (posX < 0 || posX >= kCols || posY < 0 || posY >= kRows) continue;
    G->cell[posX][posY].push_back(i);
  }
}

std::vector<int> features_in_area(const orbx_proj_frame* F, const Grid& G, float x, float y,
                                  float r, int minLevel, int maxLevel) {
  std::vector<int> out;
  const int nMinCellX = std::max(0, (int)std::floor((x - F->min_x - r) * F->grid_w_inv));
  if (nMinCellX >= kCols) return out;
  const int nMaxCellX = std::min(kCols - 1, (int)std::ceil((x - F->min_x + r) * F->grid_w_inv));
  if (nMaxCellX < 0) return out;
  const int nMinCellY = std::max(0, (int)std::floor((y - F->min_y - r) * F->grid_h_inv));
  if (nMinCellY >= kRows) return out;
  const int nMaxCellY = std::min(kRows - 1, (int)std::ceil((y - F->min_y + r) * F->grid_h_inv));
  if (nMaxCellY < 0) return out;
  const bool bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
  for (int ix = nMinCellX; ix <= nMaxCellX; ix++)
    for (int iy = nMinCellY; iy <= nMaxCellY; iy++)
      for (int idx : G.cell[ix][iy]) {
        const orbx_keypoint& kpUn = F->keys_un[idx];
        if (bCheckLevels) {
          if (kpUn.octave < minLevel) continue;
          if (maxLevel >= 0 && kpUn.octave > maxLevel) continue;
        }
        const float distx = kpUn.x - x, disty = kpUn.y - y;
        if (std::fabs(distx) < r && std::fabs(disty) < r) out.push_back(idx);
      }
  return out;
}

void three_maxima(const int* histo, int L, int* i1, int* i2, int* i3) {  // :1604-1645
  int max1 = 0, max2 = 0, max3 = 0;
  *i1 = *i2 = *i3 = -1;
  for (int i = 0; i < L; i++) {
    const int s = histo[i];
    if (s > max1) {
      max3 = max2;
      max2 = max1;
      max1 = s;
      *i3 = *i2;
      *i2 = *i1;
      *i1 = i;
    } else if (s > max2) {
      max3 = max2;
      max2 = s;
      *i3 = *i2;
      *i2 = i;
    } else if (s > max3) {
      max3 = s;
      *i3 = i;
    }
  }
  if (max2 < 0.1f * (float)max1) {
    *i2 = -1;
    *i3 = -1;
  } else if (max3 < 0.1f * (float)max1) {
    *i3 = -1;
  }
}

}  // namespace

extern "C" {

// GetFeaturesInArea on the frame's grid: indices in the reference's order, count returned.
int oracle_features_in_area(const orbx_proj_frame* F, float x, float y, float r, int minLevel,
                            int maxLevel, int32_t* out, int cap) {
  Grid G;
  assign_grid(F, &G);
  std::vector<int> v = features_in_area(F, G, x, y, r, minLevel, maxLevel);
  for (size_t i = 0; i < v.size() && (int)i < cap; i++) out[i] = v[i];
  return (int)v.size();
}

// SearchByProjection(Frame&, vector<MapPoint*>, th): match[f] = map point index assigned to
// frame feature f in this call, else -1.  Returns nmatches.
int oracle_search_by_projection(const orbx_proj_frame* F, const orbx_proj_points* M, float th,
                                float nnratio, int32_t* match) {
  Grid G;
  assign_grid(F, &G);
  std::vector<uint8_t> claimed(F->n, 0);
  for (int i = 0; i < F->n; i++) {
    match[i] = -1;
    if (F->has_mp_obs && F->has_mp_obs[i]) claimed[i] = 1;
  }
  const bool bFactor = th != 1.0;
  int nmatches = 0;
  for (int iMP = 0; iMP < M->n; iMP++) {
    if (!M->track[iMP]) continue;  // !mbTrackInView || isBad()
    const int nPredictedLevel = M->pred_level[iMP];
    float r = M->view_cos[iMP] > 0.998 ? 2.5f : 4.0f;  // RadiusByViewingCos (:130-136)
    if (bFactor) r *= th;
    const float rs = r * F->scale_factors[nPredictedLevel];
    const std::vector<int> vIndices = features_in_area(F, G, M->proj_x[iMP], M->proj_y[iMP], rs,
                                                       nPredictedLevel - 1, nPredictedLevel);
    if (vIndices.empty()) continue;
    const uint8_t* MPdescriptor = M->desc + (size_t)iMP * 32;
    int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
    for (int idx : vIndices) {
      if (claimed[idx]) continue;
      if (F->u_right && F->u_right[idx] > 0) {
        const float er = std::fabs(M->proj_xr[iMP] - F->u_right[idx]);
        if (er > r * F->scale_factors[nPredictedLevel]) continue;
      }
      const int dist = hamming(MPdescriptor, F->desc + (size_t)idx * 32);
      if (dist < bestDist) {
        bestDist2 = bestDist;
        bestDist = dist;
        bestLevel2 = bestLevel;
        bestLevel = F->keys_un[idx].octave;
        bestIdx = idx;
      } else if (dist < bestDist2) {
        bestLevel2 = F->keys_un[idx].octave;
        bestDist2 = dist;
      }
    }
    if (bestDist <= 100) {  // TH_HIGH
      if (bestLevel == bestLevel2 && bestDist > nnratio * bestDist2) continue;
      match[bestIdx] = iMP;
      claimed[bestIdx] = 1;
      nmatches++;
    }
  }
  return nmatches;
}

// SearchByProjection(CurrentFrame, LastFrame, th, bMono): match[f] = last-frame index whose
// MapPoint was assigned to current feature f, else -1.  forward/backward are the reference's
// bForward/bBackward (tlc.z vs mb, already false when mono).
int oracle_search_by_projection_last(const orbx_proj_frame* F, const orbx_proj_last* P, float th,
                                     int forward, int backward, int check_ori, int32_t* match) {
  Grid G;
  assign_grid(F, &G);
  std::vector<uint8_t> claimed(F->n, 0);
  for (int i = 0; i < F->n; i++) {
    match[i] = -1;
    if (F->has_mp_obs && F->has_mp_obs[i]) claimed[i] = 1;
  }
  const int HISTO = 30;
  const float factor = 1.0f / HISTO;
  std::vector<int> rotHist[30];
  int nmatches = 0;
  for (int i = 0; i < P->n; i++) {
    if (!P->valid[i]) continue;  // pMP && !mvbOutlier[i] && invzc >= 0
    const float u = P->u[i], v = P->v[i];
    if (u < F->min_x || u > F->max_x) continue;
    if (v < F->min_y || v > F->max_y) continue;
    const int nLastOctave = P->octave[i];
    const float radius = th * F->scale_factors[nLastOctave];
    std::vector<int> vIndices2;
    if (forward) vIndices2 = features_in_area(F, G, u, v, radius, nLastOctave, -1);
    else if (backward) vIndices2 = features_in_area(F, G, u, v, radius, 0, nLastOctave);
    else vIndices2 = features_in_area(F, G, u, v, radius, nLastOctave - 1, nLastOctave + 1);
    if (vIndices2.empty()) continue;
    const uint8_t* dMP = P->desc + (size_t)i * 32;
    int bestDist = 256, bestIdx2 = -1;
    for (int i2 : vIndices2) {
      if (claimed[i2]) continue;
      if (F->u_right && F->u_right[i2] > 0) {
        const float er = std::fabs(P->ur[i] - F->u_right[i2]);
        if (er > radius) continue;
      }
      const int dist = hamming(dMP, F->desc + (size_t)i2 * 32);
      if (dist < bestDist) {
        bestDist = dist;
        bestIdx2 = i2;
      }
    }
    if (bestDist <= 100) {
      match[bestIdx2] = i;
      // the feature blocks later points only if its point has observations (:1406-1408)
      if (!P->blocks || P->blocks[i]) claimed[bestIdx2] = 1;
      nmatches++;
      if (check_ori) {
        float rot = P->angle[i] - F->keys_un[bestIdx2].angle;
        if (rot < 0.0) rot += 360.0f;
        int bin = (int)std::round(rot * factor);
        if (bin == HISTO) bin = 0;
        rotHist[bin].push_back(bestIdx2);
      }
    }
  }
  if (check_ori) {
    int hs[30];
    for (int b = 0; b < HISTO; b++) hs[b] = (int)rotHist[b].size();
    int ind1, ind2, ind3;
    three_maxima(hs, HISTO, &ind1, &ind2, &ind3);
    for (int b = 0; b < HISTO; b++) {
      if (b == ind1 || b == ind2 || b == ind3) continue;
      for (int idx : rotHist[b]) {
        match[idx] = -1;
        nmatches--;
      }
    }
  }
  return nmatches;
}

// SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize): prev[2 i1 .. 2 i1 + 1]
// = vbPrevMatched[i1] (x, y), updated in place; m12[i1] = vnMatches12[i1].  Returns nmatches.
// F1 uses n, keys_un, desc; F2 keys_un, desc and its grid frame.
int oracle_search_for_initialization(const orbx_proj_frame* F1, const orbx_proj_frame* F2,
                                     float* prev, float nnratio, int check_ori, int window,
                                     int32_t* m12) {
  Grid G;
  assign_grid(F2, &G);
  const int n1 = F1->n, n2 = F2->n;
  int nmatches = 0;
  for (int i = 0; i < n1; i++) m12[i] = -1;                     // :408
  const int HISTO = 30;
  std::vector<int> rotHist[30];                                  // :410-413
  const float factor = 1.0f / HISTO;
  std::vector<int> vMatchedDistance(n2, INT_MAX), vnMatches21(n2, -1);  // :415-416
  const float r = (float)window;  // GetFeaturesInArea(const float& r) of the int windowSize
  for (int i1 = 0; i1 < n1; i1++) {                              // :418-490
    const orbx_keypoint& kp1 = F1->keys_un[i1];
    const int level1 = kp1.octave;
    if (level1 > 0) continue;
    const std::vector<int> vIndices2 =
        features_in_area(F2, G, prev[2 * i1], prev[2 * i1 + 1], r, level1, level1);
    if (vIndices2.empty()) continue;
    const uint8_t* d1 = F1->desc + (size_t)i1 * 32;
    int bestDist = INT_MAX, bestDist2 = INT_MAX, bestIdx2 = -1;
    for (int i2 : vIndices2) {
      const int dist = hamming(d1, F2->desc + (size_t)i2 * 32);
      if (vMatchedDistance[i2] <= dist) continue;
      if (dist < bestDist) {
        bestDist2 = bestDist;
        bestDist = dist;
        bestIdx2 = i2;
      } else if (dist < bestDist2) {
        bestDist2 = dist;
      }
    }
    if (bestDist <= 50) {                                        // TH_LOW
      if (bestDist < (float)bestDist2 * nnratio) {
        if (vnMatches21[bestIdx2] >= 0) {
          m12[vnMatches21[bestIdx2]] = -1;
          nmatches--;
        }
        m12[i1] = bestIdx2;
        vnMatches21[bestIdx2] = i1;
        vMatchedDistance[bestIdx2] = bestDist;
        nmatches++;
        if (check_ori) {
          float rot = F1->keys_un[i1].angle - F2->keys_un[bestIdx2].angle;
          if (rot < 0.0) rot += 360.0f;
          int bin = (int)std::round(rot * factor);
          if (bin == HISTO) bin = 0;
          rotHist[bin].push_back(i1);
        }
      }
    }
  }
  if (check_ori) {                                               // :492-515
    int hs[30];
    for (int b = 0; b < HISTO; b++) hs[b] = (int)rotHist[b].size();
    int ind1, ind2, ind3;
    three_maxima(hs, HISTO, &ind1, &ind2, &ind3);
    for (int b = 0; b < HISTO; b++) {
      if (b == ind1 || b == ind2 || b == ind3) continue;
      for (int idx1 : rotHist[b])
        if (m12[idx1] >= 0) {
          m12[idx1] = -1;
          nmatches--;
        }
    }
  }
  for (int i1 = 0; i1 < n1; i1++)                                // :517-520
    if (m12[i1] >= 0) {
      prev[2 * i1] = F2->keys_un[m12[i1]].x;
      prev[2 * i1 + 1] = F2->keys_un[m12[i1]].y;
    }
  return nmatches;
}

// Fuse, both overloads: the per-point search (the caller evaluates the gates before it and
// applies the replace / add-observation step after it).  reproj = 1: Fuse(KeyFrame*,
// vector<MapPoint*>, th) with its reprojection gates, whose float expressions follow the
// reference binary's contraction (e2 = fmaf(ex, ex, ey*ey), stereo fmaf(er, er, e2): RB
// 0x7474c-0x74797, 0x7490b-0x74931); 0: the Sim3 overload.  best_idx[i] = bestIdx when
// bestDist <= TH_LOW else -1, best_dist[i] = bestDist.  Returns the count of best_idx >= 0.
int oracle_fuse(const orbx_proj_frame* KF, const float* inv_sigma2, const orbx_fuse_points* M,
                float th, int reproj, int32_t* best_idx, int32_t* best_dist) {
  Grid G;
  assign_grid(KF, &G);
  int nf = 0;
  for (int i = 0; i < M->n; i++) {
    const int none = reproj ? 256 : INT_MAX;  // :904, :1063
    best_idx[i] = -1;
    best_dist[i] = none;
    if (!M->use[i]) continue;
    const int nPredictedLevel = M->pred_level[i];
    const float u = M->u[i], v = M->v[i];
    const float radius = th * KF->scale_factors[nPredictedLevel];       // :893
    const std::vector<int> vIndices = features_in_area(KF, G, u, v, radius, -1, -1);
    if (vIndices.empty()) continue;
    const uint8_t* dMP = M->desc + (size_t)i * 32;
    int bestDist = none, bestIdx = -1;
    for (int idx : vIndices) {
      const orbx_keypoint& kp = KF->keys_un[idx];
      const int kpLevel = kp.octave;
      if (kpLevel < nPredictedLevel - 1 || kpLevel > nPredictedLevel) continue;
      if (reproj) {
        const float ex = u - kp.x, ey = v - kp.y;
        if (KF->u_right && KF->u_right[idx] >= 0) {                    // :917-930
          const float er = M->ur[i] - KF->u_right[idx];
          const float e2 = std::fmaf(er, er, std::fmaf(ex, ex, ey * ey));
          if (e2 * inv_sigma2[kpLevel] > 7.8) continue;
        } else {                                                       // :931-941
          const float e2 = std::fmaf(ex, ex, ey * ey);
          if (e2 * inv_sigma2[kpLevel] > 5.99) continue;
        }
      }
      const int dist = hamming(dMP, KF->desc + (size_t)idx * 32);
      if (dist < bestDist) {
        bestDist = dist;
        bestIdx = idx;
      }
    }
    best_dist[i] = bestDist;
    if (bestDist <= 50) {                                              // TH_LOW
      best_idx[i] = bestIdx;
      nf++;
    }
  }
  return nf;
}

// SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist) (relocalization): F's
// has_mp_obs = mvpMapPoints[i] != NULL on entry; P: valid (pMP, !isBad, not already found, the
// distance-invariance gate), u, v, octave = the predicted level, angle = pKF->mvKeysUn[i].angle,
// desc.  match[f] = the keyframe index whose map point was assigned to f, else -1.
int oracle_search_by_projection_kf(const orbx_proj_frame* F, const orbx_proj_last* P, float th,
                                   int ORBdist, int check_ori, int32_t* match) {
  Grid G;
  assign_grid(F, &G);
  std::vector<uint8_t> has(F->n, 0);  // CurrentFrame.mvpMapPoints[i2] != NULL
  for (int i = 0; i < F->n; i++) {
    match[i] = -1;
    if (F->has_mp_obs && F->has_mp_obs[i]) has[i] = 1;
  }
  const int HISTO = 30;
  const float factor = 1.0f / HISTO;
  std::vector<int> rotHist[30];
  int nmatches = 0;
  for (int i = 0; i < P->n; i++) {
    if (!P->valid[i]) continue;
    const float u = P->u[i], v = P->v[i];
    if (u < F->min_x || u > F->max_x) continue;  // :1512-1515
    if (v < F->min_y || v > F->max_y) continue;
    const int nPredictedLevel = P->octave[i];
    const float radius = th * F->scale_factors[nPredictedLevel];  // :1530
    const std::vector<int> vIndices2 =
        features_in_area(F, G, u, v, radius, nPredictedLevel - 1, nPredictedLevel + 1);
    if (vIndices2.empty()) continue;
    const uint8_t* dMP = P->desc + (size_t)i * 32;
    int bestDist = 256, bestIdx2 = -1;
    for (int i2 : vIndices2) {
      if (has[i2]) continue;  // :1546-1547
      const int dist = hamming(dMP, F->desc + (size_t)i2 * 32);
      if (dist < bestDist) {
        bestDist = dist;
        bestIdx2 = i2;
      }
    }
    if (bestDist <= ORBdist) {  // :1560-1576
      has[bestIdx2] = 1;
      match[bestIdx2] = i;
      nmatches++;
      if (check_ori) {
        float rot = P->angle[i] - F->keys_un[bestIdx2].angle;
        if (rot < 0.0) rot += 360.0f;
        int bin = (int)std::round(rot * factor);
        if (bin == HISTO) bin = 0;
        rotHist[bin].push_back(bestIdx2);
      }
    }
  }
  if (check_ori) {  // :1582-1598
    int hs[30];
    for (int b = 0; b < HISTO; b++) hs[b] = (int)rotHist[b].size();
    int ind1, ind2, ind3;
    three_maxima(hs, HISTO, &ind1, &ind2, &ind3);
    for (int b = 0; b < HISTO; b++) {
      if (b == ind1 || b == ind2 || b == ind3) continue;
      for (int idx : rotHist[b]) {
        match[idx] = -1;
        nmatches--;
      }
    }
  }
  return nmatches;
}

// SearchByProjection(pKF, Scw, vpPoints, vpMatched, th) (loop closing): KF's has_mp_obs =
// vpMatched[f] != NULL on entry; M: use (the gates of :318-352), u, v, pred_level, desc.
// match[f] = the point index assigned to keyframe feature f in this call, else -1.
int oracle_search_by_projection_sim3(const orbx_proj_frame* KF, const orbx_fuse_points* M,
                                     float th, int32_t* match) {
  Grid G;
  assign_grid(KF, &G);
  std::vector<uint8_t> matched(KF->n, 0);  // vpMatched[idx] != NULL
  for (int i = 0; i < KF->n; i++) {
    match[i] = -1;
    if (KF->has_mp_obs && KF->has_mp_obs[i]) matched[i] = 1;
  }
  int nmatches = 0;
  for (int iMP = 0; iMP < M->n; iMP++) {
    if (!M->use[iMP]) continue;
    const int nPredictedLevel = M->pred_level[iMP];
    const float radius = th * KF->scale_factors[nPredictedLevel];  // :354-356
    // KeyFrame::GetFeaturesInArea(u, v, radius): no level window (KeyFrame.cc:518-558)
    const std::vector<int> vIndices = features_in_area(KF, G, M->u[iMP], M->v[iMP], radius, -1, -1);
    if (vIndices.empty()) continue;
    const uint8_t* dMP = M->desc + (size_t)iMP * 32;
    int bestDist = 256, bestIdx = -1;
    for (int idx : vIndices) {
      if (matched[idx]) continue;  // :360-361
      const int kpLevel = KF->keys_un[idx].octave;
      if (kpLevel < nPredictedLevel - 1 || kpLevel > nPredictedLevel) continue;  // :364-367
      const int dist = hamming(dMP, KF->desc + (size_t)idx * 32);
      if (dist < bestDist) {
        bestDist = dist;
        bestIdx = idx;
      }
    }
    if (bestDist <= 50) {  // TH_LOW (:384-388)
      matched[bestIdx] = 1;
      match[bestIdx] = iMP;
      nmatches++;
    }
  }
  return nmatches;
}

// SearchBySim3 (:1105-1329): one direction's per-point search (KeyFrame::GetFeaturesInArea, the
// level window [pred - 1, pred], first minimum from INT_MAX, accepted when <= TH_HIGH).
static void sim3_direction(const orbx_proj_frame* KF, const orbx_fuse_points* M, float th,
                           std::vector<int>* vnMatch) {
  Grid G;
  assign_grid(KF, &G);
  vnMatch->assign(M->n, -1);
  for (int i = 0; i < M->n; i++) {
    if (!M->use[i]) continue;
    const int nPredictedLevel = M->pred_level[i];
    const float radius = th * KF->scale_factors[nPredictedLevel];  // :1183, :1258
    const std::vector<int> vIndices = features_in_area(KF, G, M->u[i], M->v[i], radius, -1, -1);
    if (vIndices.empty()) continue;
    const uint8_t* dMP = M->desc + (size_t)i * 32;
    int bestDist = INT_MAX, bestIdx = -1;
    for (int idx : vIndices) {
      const int kl = KF->keys_un[idx].octave;
      if (kl < nPredictedLevel - 1 || kl > nPredictedLevel) continue;
      const int dist = hamming(dMP, KF->desc + (size_t)idx * 32);
      if (dist < bestDist) {
        bestDist = dist;
        bestIdx = idx;
      }
    }
    if (bestDist <= 100) (*vnMatch)[i] = bestIdx;  // TH_HIGH
  }
}

// m12[i1] = idx2 where both directions agree (vpMatches12[i1] = vpMapPoints2[idx2]), else -1.
// Returns nFound.  M12: KF1's points projected into KF2 (n = KF1->n); M21: KF2's into KF1.
int oracle_search_by_sim3(const orbx_proj_frame* KF1, const orbx_proj_frame* KF2,
                          const orbx_fuse_points* M12, const orbx_fuse_points* M21, float th,
                          int32_t* m12) {
  std::vector<int> vnMatch1, vnMatch2;
  sim3_direction(KF2, M12, th, &vnMatch1);
  sim3_direction(KF1, M21, th, &vnMatch2);
  int nFound = 0;
  for (int i1 = 0; i1 < M12->n; i1++) {  // :1305-1326
    m12[i1] = -1;
    const int idx2 = vnMatch1[i1];
    if (idx2 >= 0 && idx2 < M21->n && vnMatch2[idx2] == i1) {
      m12[i1] = idx2;
      nFound++;
    }
  }
  return nFound;
}

}  // extern "C"
