// orbx_project.hip — the tracking searches on the GPU:
//   Frame::AssignFeaturesToGrid / GetFeaturesInArea        (ORB_SLAM2/src/Frame.cc:235-250, 332-398)
//   ORBmatcher::SearchByProjection(Frame&, vector<MapPoint*>, th)       (ORBmatcher.cc:45-137)
//   ORBmatcher::SearchByProjection(Frame&, const Frame&, th, bMono)     (ORBmatcher.cc:1331-1474)
//   ORBmatcher::SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize)
//                                                                        (ORBmatcher.cc:405-523)
// (GetFeaturesInArea runs fused inside the searches; it has no entry point of its own.)
//
//   k_grid_cells   cell of every feature (PosInGrid: round((x - mnMinX) * inv)); k_csr then
//                  buckets the features by cell, ascending index inside a cell (mGrid order)
//   k_grid_dense   per-cell [begin, end) table over all 64 x 48 cells
//   k_proj_cand    one wave per point: GetFeaturesInArea in the reference's order (cells
//                  column-major over the window, lanes over cells, wave prefix sum for the
//                  output position), the static filters (level range, |dx| < r && |dy| < r,
//                  features already holding a MapPoint with observations, the stereo uR test)
//                  and the Hamming distance; the ordered candidate list goes to a global pool
//                  (one atomic per point for its range; no per-point limit: a call whose lists
//                  outgrow the pool is rerun once with the pool sized to their total)
//   k_proj_resolve one wave per frame, points in order: the greedy part of the reference — a
//                  feature matched by an earlier point is skipped by the later ones — over the
//                  candidate lists with a claimed-feature bitmap in LDS.  Best / second of the
//                  reference's sequential update are recovered in parallel: best = first
//                  minimum; second = first minimum of {best-before-best} + {candidates after
//                  best}.  Motion-model variant: rotation histogram + ComputeThreeMaxima.
//   k_init_resolve one wave per frame pair, F1 features in order: SearchForInitialization's
//                  vMatchedDistance / vnMatches21 state (a feature of F2 taken by a closer match
//                  later) in LDS, best / second by a wave key minimum, the rotation histogram
//                  with every pushed entry (ComputeThreeMaxima counts them all), vbPrevMatched.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <vector>

#include "orbx_internal.h"
#include "orbx_match.h"

#pragma clang fp contract(off)

namespace orbx {

constexpr int kGridCols = 64, kGridRows = 48, kCells = kGridCols * kGridRows;
constexpr int kPoolPerPoint = 256;  // first-try pool size per point (any list length works)
constexpr int kTH_HIGH = 100;
constexpr int kTH_LOW = 50;
constexpr int kHisto = 30;

struct ProjFrameDev {
  int n;
  const orbx_keypoint* keys;
  const uint8_t* desc;
  const float* u_right;
  const uint8_t* has_mp_obs;
  float min_x, min_y, max_x, max_y, gw, gh;
  float scale[kMaxLevels];
  const int* cell_begin;  // [kCells + 1]
  const int* cell_feats;  // [n]
};

// mode 0: local-map points (SearchByProjection(F, vpMapPoints, th)); 1: last frame;
// 2: SearchForInitialization (x, y = vbPrevMatched, level = F1 octave, th = windowSize);
// 3: relocalization (SearchByProjection(F, pKF, sAlreadyFound, th, ORBdist): level = the
//    predicted level, window levels +-1, angle = the keyframe keypoint's);
// 4: loop closing (SearchByProjection(pKF, Scw, vpPoints, vpMatched, th): the keyframe's grid,
//    levels [predicted - 1, predicted])
struct ProjPointsDev {
  int mode;
  int max_dist;         // accepted best distance (modes 1, 3, 4): TH_HIGH, ORBdist, TH_LOW
  int n;
  const uint8_t* use;   // track (mode 0) / valid (mode 1)
  const float *x, *y, *xr;
  const int* level;     // predicted level (mode 0) / last octave (mode 1)
  const float* view_cos;
  const float* angle;
  const uint8_t* desc;
  float th, nnratio;
  int forward, backward, check_ori;
  const uint8_t* blocks;  // mode 1: the point has observations, its feature blocks later points
  int2* log;              // modes 1 / 3 with check_ori: (feature, bin) of every assignment
};

__global__ __launch_bounds__(256) void k_grid_cells(ProjFrameDev F, uint32_t* __restrict__ cell) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= F.n) return;
  const orbx_keypoint k = F.keys[i];
  const int px = (int)roundf((k.x - F.min_x) * F.gw);  // Frame::PosInGrid (:387-398)
  const int py = (int)roundf((k.y - F.min_y) * F.gh);
  cell[i] = (px < 0 || px >= kGridCols || py < 0 || py >= kGridRows)
                ? 0xFFFFFFFFu
                : (uint32_t)(px * kGridRows + py);  // column-major: mGrid[ix][iy]
}

__global__ __launch_bounds__(256) void k_grid_dense(const uint32_t* __restrict__ ids,
                                                    const int* __restrict__ off,
                                                    const int* __restrict__ nn,
                                                    int* __restrict__ begin) {
  // begin[c] = CSR start of the first non-empty cell >= c (so cell c is [begin[c], begin[c+1]))
  const int m = *nn;
  const int total = m > 0 ? off[m] : 0;
  for (int c = blockIdx.x * 256 + threadIdx.x; c <= kCells; c += gridDim.x * 256) {
    int lo = 0, hi = m;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if ((int)ids[mid] < c) lo = mid + 1;
      else hi = mid;
    }
    begin[c] = lo < m ? off[lo] : total;
  }
}

__device__ __forceinline__ int wave_excl_sum(int v, int* total) {
  const int lane = threadIdx.x & 63;
  int incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int x = __shfl_up(incl, o);
    if (lane >= o) incl += x;
  }
  *total = __shfl(incl, 63);
  return incl - v;
}

// candidates of point p: (feature index, distance, octave) in GetFeaturesInArea order, at
// lists[base[p] ..] of a pool of pool_cap entries (*pool_used: entries taken; a point whose range
// does not fit gets count 0 and the host reruns with a larger pool)
__global__ __launch_bounds__(256) void k_proj_cand(ProjFrameDev F, ProjPointsDev P,
                                                   int4* __restrict__ lists,
                                                   int* __restrict__ base_out,
                                                   int* __restrict__ counts,
                                                   int* __restrict__ pool_used, int pool_cap) {
  const int lane = threadIdx.x & 63;
  const int p = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (p >= P.n) return;
  bool go = P.use[p] != 0;
  const float x = P.x[p], y = P.y[p];
  float r = 0.f, rs = 0.f;
  int minLevel = 0, maxLevel = 0;
  if (go && P.mode == 0) {
    const int lev = P.level[p];
    r = P.view_cos[p] > 0.998 ? 2.5f : 4.0f;  // RadiusByViewingCos (ORBmatcher.cc:130-136)
    if (P.th != 1.0) r *= P.th;
    rs = r * F.scale[lev];
    minLevel = lev - 1;
    maxLevel = lev;
  } else if (go && P.mode == 1) {
    if (x < F.min_x || x > F.max_x || y < F.min_y || y > F.max_y) go = false;  // :1377-1380
    const int oct = P.level[p];
    rs = P.th * F.scale[oct];
    if (P.forward) minLevel = oct, maxLevel = -1;
    else if (P.backward) minLevel = 0, maxLevel = oct;
    else minLevel = oct - 1, maxLevel = oct + 1;
  } else if (go && P.mode == 2) {  // GetFeaturesInArea(prev.x, prev.y, windowSize, level1, level1) (:425)
    rs = P.th;
    minLevel = maxLevel = P.level[p];
  } else if (go && P.mode == 3) {
    if (x < F.min_x || x > F.max_x || y < F.min_y || y > F.max_y) go = false;  // :1512-1515
    const int lev = P.level[p];
    rs = P.th * F.scale[lev];  // :1530-1532
    minLevel = lev - 1;
    maxLevel = lev + 1;
  } else if (go) {  // mode 4: the level test sits in the reference's loop (:364-367), same set
    const int lev = P.level[p];
    rs = P.th * F.scale[lev];  // :354-356
    minLevel = lev - 1;
    maxLevel = lev;
  }
  int cx0 = 0, cx1 = -1, cy0 = 0, cy1 = -1;
  if (go) {  // GetFeaturesInArea window (Frame.cc:337-351)
    cx0 = max(0, (int)floorf((x - F.min_x - rs) * F.gw));
    cx1 = min(kGridCols - 1, (int)ceilf((x - F.min_x + rs) * F.gw));
    cy0 = max(0, (int)floorf((y - F.min_y - rs) * F.gh));
    cy1 = min(kGridRows - 1, (int)ceilf((y - F.min_y + rs) * F.gh));
    if (cx0 >= kGridCols || cx1 < 0 || cy0 >= kGridRows || cy1 < 0) go = false;
  }
  if (!go) {
    if (lane == 0) counts[p] = 0;
    return;
  }
  const bool bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
  const int ny = cy1 - cy0 + 1, ncell = (cx1 - cx0 + 1) * ny;
  auto pass = [&](int idx) -> bool {
    const orbx_keypoint k = F.keys[idx];
    if (bCheckLevels) {
      if (k.octave < minLevel) return false;
      if (maxLevel >= 0 && k.octave > maxLevel) return false;
    }
    const float dx = k.x - x, dy = k.y - y;
    return fabsf(dx) < rs && fabsf(dy) < rs;
  };
  auto cell_range = [&](int c, int& b, int& e) {
    b = e = 0;
    if (c < ncell) {
      const int cell = (cx0 + c / ny) * kGridRows + cy0 + c % ny;
      b = F.cell_begin[cell];
      e = F.cell_begin[cell + 1];
    }
  };
  // the list length first (one pool range per point), then the ordered writes
  int total = 0;
  for (int c0 = 0; c0 < ncell; c0 += 64) {
    int b, e, mine = 0;
    cell_range(c0 + lane, b, e);
    for (int j = b; j < e; j++) mine += pass(F.cell_feats[j]);
    int t;
    wave_excl_sum(mine, &t);
    total += t;
  }
  int base = 0;
  if (lane == 0 && total > 0) base = atomicAdd(pool_used, total);
  base = __shfl(base, 0);
  const bool fits = base + total <= pool_cap;
  if (lane == 0) {
    counts[p] = fits ? total : 0;
    base_out[p] = base;
  }
  if (!fits || total == 0) return;
  const uint64_t* q = (const uint64_t*)(P.desc + (int64_t)p * 32);
  const uint64_t d0 = q[0], d1 = q[1], d2 = q[2], d3 = q[3];
  const float xr = P.xr ? P.xr[p] : 0.f;
  int4* out = lists + base;
  int cnt_out = 0;
  for (int c0 = 0; c0 < ncell; c0 += 64) {
    int b, e, mine = 0;
    cell_range(c0 + lane, b, e);
    for (int j = b; j < e; j++) mine += pass(F.cell_feats[j]);
    int tot;
    int pos = cnt_out + wave_excl_sum(mine, &tot);
    for (int j = b; j < e; j++) {
      const int idx = F.cell_feats[j];
      if (!pass(idx)) continue;
      // static per-candidate filters of the searches; the order slot is kept either way
      int dist = 256;
      bool ok = P.mode == 2 || !(F.has_mp_obs && F.has_mp_obs[idx]);
      if (ok && P.mode <= 1 && F.u_right && F.u_right[idx] > 0) {
        const float er = fabsf((P.mode == 0 ? P.xr[p] : xr) - F.u_right[idx]);
        ok = !(er > (P.mode == 0 ? r * F.scale[P.level[p]] : rs));
      }
      if (ok) {
        const uint64_t* t = (const uint64_t*)(F.desc + (int64_t)idx * 32);
        dist = __popcll(d0 ^ t[0]) + __popcll(d1 ^ t[1]) + __popcll(d2 ^ t[2]) +
               __popcll(d3 ^ t[3]);
      }
      out[pos++] = make_int4(idx, dist, F.keys[idx].octave, 0);
    }
    cnt_out += tot;
  }
}

// one wave: points in order, greedy claims in an LDS bitmap
__global__ __launch_bounds__(64) void k_proj_resolve(ProjFrameDev F, ProjPointsDev P,
                                                     const int4* __restrict__ lists,
                                                     const int* __restrict__ bases,
                                                     const int* __restrict__ counts,
                                                     int* __restrict__ match,
                                                     int* __restrict__ nmatch) {
  extern __shared__ uint32_t s_claim[];  // [ceil(n / 32)]
  __shared__ int s_hist[kHisto];
  const int lane = threadIdx.x;
  const int nw = (F.n + 31) >> 5;
  for (int w = lane; w < nw; w += 64) s_claim[w] = 0;
  for (int i = lane; i < F.n; i += 64) match[i] = -1;
  if (lane < kHisto) s_hist[lane] = 0;
  __syncthreads();
  int nm = 0;
  const float factor = 1.0f / kHisto;
  for (int p = 0; p < P.n; p++) {
    const int L = counts[p];
    if (L == 0) continue;
    const int4* lst = lists + bases[p];
    // pass 1: best = first minimum over unclaimed candidates with dist < 256 (key: distance
    // in the top 9 bits, list position in the low 22)
    int key1 = INT_MAX;
    for (int j = lane; j < L; j += 64) {
      const int4 c = lst[j];
      const bool claimed = (s_claim[c.x >> 5] >> (c.x & 31)) & 1;
      if (!claimed && c.y < 256) key1 = min(key1, (c.y << 22) | j);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) key1 = min(key1, __shfl_xor(key1, o));
    if (key1 == INT_MAX) continue;
    const int bestDist = key1 >> 22, bestPos = key1 & 0x3FFFFF;
    if (bestDist > (P.mode == 0 ? kTH_HIGH : P.max_dist)) continue;
    const int4 best = lst[bestPos];
    if (P.mode == 0) {
      // second: first minimum of {the best among candidates before bestPos} followed by the
      // candidates after bestPos, in order
      int kpre = INT_MAX, ksuf = INT_MAX;
      for (int j = lane; j < L; j += 64) {
        const int4 c = lst[j];
        const bool claimed = (s_claim[c.x >> 5] >> (c.x & 31)) & 1;
        if (claimed || c.y >= 256 || j == bestPos) continue;
        if (j < bestPos) kpre = min(kpre, (c.y << 22) | j);
        else ksuf = min(ksuf, (c.y << 22) | j);
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        kpre = min(kpre, __shfl_xor(kpre, o));
        ksuf = min(ksuf, __shfl_xor(ksuf, o));
      }
      int bestDist2 = 256, bestLevel2 = -1;
      const int dpre = kpre == INT_MAX ? 256 : kpre >> 22;
      const int dsuf = ksuf == INT_MAX ? 256 : ksuf >> 22;
      if (kpre != INT_MAX && dpre <= dsuf) {
        bestDist2 = dpre;
        bestLevel2 = lst[kpre & 0x3FFFFF].z;
      } else if (ksuf != INT_MAX) {
        bestDist2 = dsuf;
        bestLevel2 = lst[ksuf & 0x3FFFFF].z;
      }
      const int bestLevel = best.z;
      if (bestLevel == bestLevel2 && (float)bestDist > P.nnratio * (float)bestDist2) continue;
    }
    if (lane == 0) {
      match[best.x] = p;
      // a point without observations leaves its feature open to later points, which may take
      // it over (ORBmatcher.cc:1406-1408)
      if (!P.blocks || P.blocks[p]) s_claim[best.x >> 5] |= 1u << (best.x & 31);
      if ((P.mode == 1 || P.mode == 3) && P.check_ori) {
        float rot = P.angle[p] - F.keys[best.x].angle;
        if (rot < 0.0) rot += 360.0f;
        int bin = (int)roundf(rot * factor);
        if (bin == kHisto) bin = 0;
        s_hist[bin]++;
        P.log[nm] = make_int2(best.x, bin);  // rotHist[bin].push_back(bestIdx2)
      }
    }
    nm++;
    __syncthreads();
  }
  if ((P.mode == 1 || P.mode == 3) && P.check_ori) {
    __syncthreads();
    int ind1 = -1, ind2 = -1, ind3 = -1;  // ComputeThreeMaxima (ORBmatcher.cc:1604-1645)
    int max1 = 0, max2 = 0, max3 = 0;
    for (int i = 0; i < kHisto; i++) {
      const int s = s_hist[i];
      if (s > max1) {
        max3 = max2; max2 = max1; max1 = s;
        ind3 = ind2; ind2 = ind1; ind1 = i;
      } else if (s > max2) {
        max3 = max2; max2 = s;
        ind3 = ind2; ind2 = i;
      } else if (s > max3) {
        max3 = s; ind3 = i;
      }
    }
    if (max2 < 0.1f * (float)max1) ind2 = ind3 = -1;
    else if (max3 < 0.1f * (float)max1) ind3 = -1;
    // every pushed entry of a bin outside the three maxima: its feature loses its point and
    // nmatches drops by one per entry (:1459-1468; a feature taken over twice has two entries)
    int removed = 0;
    for (int k = lane; k < nm; k += 64) {
      const int2 e = P.log[k];
      if (e.y != ind1 && e.y != ind2 && e.y != ind3) {
        match[e.x] = -1;
        removed++;
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) removed += __shfl_xor(removed, o);
    nm -= removed;
  }
  if (lane == 0) *nmatch = nm;
}

// SearchForInitialization's sequential pass (ORBmatcher.cc:418-523), one wave.  Per F2 feature
// the pair (vMatchedDistance, vnMatches21 + 1) packed in one dword (distance <= 256, 0x7FFF for
// INT_MAX; F1 index < 65535), vnMatches12 and the histogram bin pushed for each F1 feature
// (-1: none) in LDS when they fit (kLDS), else in global scratch read and written with
// device-scope atomics (coherent for the wave's own later reads).
template <bool kLDS>
__global__ __launch_bounds__(64) void k_init_resolve(ProjFrameDev F2, const orbx_keypoint* __restrict__ keys1,
                                                     int n1, const int4* __restrict__ lists,
                                                     const int* __restrict__ bases,
                                                     const int* __restrict__ counts, float nnratio,
                                                     int check_ori, float* __restrict__ prev,
                                                     int* __restrict__ m12_out,
                                                     int* __restrict__ scratch,
                                                     int* __restrict__ nmatch) {
  extern __shared__ int s_dyn[];
  __shared__ int s_hist[kHisto];
  const int lane = threadIdx.x;
  const int n2 = F2.n;
  int* st2 = kLDS ? s_dyn : scratch;            // [n2] (dist << 16) | (m21 + 1)
  int* m12 = (kLDS ? s_dyn : scratch) + n2;      // [n1]
  int* bin1 = m12 + n1;                          // [n1]
  auto ld = [&](const int* a, int i) -> int {
    if constexpr (kLDS) return a[i];
    else return __hip_atomic_load(a + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  auto stv = [&](int* a, int i, int v) {
    if constexpr (kLDS) a[i] = v;
    else __hip_atomic_store(a + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  constexpr int kNone = 0x7FFF;
  for (int i = lane; i < n2; i += 64) stv(st2, i, kNone << 16);
  for (int i = lane; i < n1; i += 64) {
    stv(m12, i, -1);
    stv(bin1, i, -1);
  }
  if (lane < kHisto) s_hist[lane] = 0;
  __syncthreads();
  int nm = 0;
  const float factor = 1.0f / kHisto;
  for (int i0 = 0; i0 < n1; i0 += 64) {
    const int cnt_l = i0 + lane < n1 ? counts[i0 + lane] : 0;
    const int base_l = i0 + lane < n1 ? bases[i0 + lane] : 0;
    uint64_t act = __ballot(cnt_l > 0);
    while (act) {
      const int j = __builtin_ctzll(act);
      act &= act - 1;
      const int i1 = i0 + j;
      const int L = __shfl(cnt_l, j), base = __shfl(base_l, j);
      // each lane: first minimum (dist << 22 | position) and the second distance over its
      // candidates not blocked by vMatchedDistance[i2] <= dist (:444-445)
      int k1 = INT_MAX, b2 = INT_MAX;
      for (int q = lane; q < L; q += 64) {
        const int4 c = lists[base + q];
        const int md = ld(st2, c.x) >> 16;
        const int dist = c.y;
        if ((md == kNone ? INT_MAX : md) <= dist) continue;
        const int key = (dist << 22) | q;
        if (key < k1) {
          b2 = k1 == INT_MAX ? INT_MAX : (k1 >> 22);
          k1 = key;
        } else if (dist < b2) {
          b2 = dist;
        }
      }
      // wave merge as the sequential scan: best = first minimum; second = the minimum over
      // the lanes of their best, except the winning lane, which offers its own second
      int K = k1;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) K = min(K, __shfl_xor(K, o));
      if (K == INT_MAX) continue;
      int B2 = k1 == K ? b2 : (k1 == INT_MAX ? INT_MAX : (k1 >> 22));
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) B2 = min(B2, __shfl_xor(B2, o));
      const int bestDist = K >> 22;
      if (bestDist > kTH_LOW) continue;                                       // :459
      if (!((float)bestDist < (float)B2 * nnratio)) continue;                // :461
      if (lane == 0) {
        const int bestIdx2 = lists[base + (K & 0x3FFFFF)].x;
        const int prev21 = (ld(st2, bestIdx2) & 0xFFFF) - 1;
        if (prev21 >= 0) {                                                   // :463-467
          stv(m12, prev21, -1);
          nm--;
        }
        stv(m12, i1, bestIdx2);
        stv(st2, bestIdx2, (bestDist << 16) | (i1 + 1));
        nm++;
        if (check_ori) {                                                     // :473-486
          float rot = keys1[i1].angle - F2.keys[bestIdx2].angle;
          if (rot < 0.0) rot += 360.0f;
          int bin = (int)roundf(rot * factor);
          if (bin == kHisto) bin = 0;
          stv(bin1, i1, bin);
          s_hist[bin]++;
        }
      }
      nm = __shfl(nm, 0);
      __syncthreads();
    }
  }
  int removed = 0;
  if (check_ori) {  // :492-515 (every pushed entry counts in the histogram)
    int ind1 = -1, ind2 = -1, ind3 = -1;
    int max1 = 0, max2 = 0, max3 = 0;
    for (int i = 0; i < kHisto; i++) {  // ComputeThreeMaxima (:1604-1645)
      const int sv = s_hist[i];
      if (sv > max1) {
        max3 = max2; max2 = max1; max1 = sv;
        ind3 = ind2; ind2 = ind1; ind1 = i;
      } else if (sv > max2) {
        max3 = max2; max2 = sv;
        ind3 = ind2; ind2 = i;
      } else if (sv > max3) {
        max3 = sv; ind3 = i;
      }
    }
    if (max2 < 0.1f * (float)max1) ind2 = ind3 = -1;
    else if (max3 < 0.1f * (float)max1) ind3 = -1;
    for (int i = lane; i < n1; i += 64) {
      const int b = ld(bin1, i);
      if (b < 0 || b == ind1 || b == ind2 || b == ind3) continue;
      if (ld(m12, i) >= 0) {
        stv(m12, i, -1);
        removed++;
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) removed += __shfl_xor(removed, o);
  }
  for (int i = lane; i < n1; i += 64) {  // vnMatches12 out, vbPrevMatched update (:517-520)
    const int m = ld(m12, i);
    m12_out[i] = m;
    if (m >= 0) {
      prev[2 * i] = F2.keys[m].x;
      prev[2 * i + 1] = F2.keys[m].y;
    }
  }
  if (lane == 0) *nmatch = nm - removed;
}

// ORBmatcher::Fuse, both overloads (ORBmatcher.cc:828-978, 980-1103): one wave per map point.
// KeyFrame::GetFeaturesInArea(u, v, th * mvScaleFactors[nPredictedLevel]) (KeyFrame.cc:518-558:
// the frame grid, no level test), then per candidate in that order the level window
// [nPredictedLevel - 1, nPredictedLevel] and, for the KeyFrame overload, the reprojection gate
// with the reference binary's contraction (e2 = fma(ex, ex, ey * ey), stereo
// fma(er, er, that); e2 * mvInvLevelSigma2 compared in double with 5.99 / 7.8), and the first
// strict minimum of the Hamming distance.  best[p] = (index or -1 when bestDist > TH_LOW or no
// candidate, bestDist (256 / INT_MAX when none)).
struct FusePointsDev {
  int n;
  const uint8_t* use;
  const float *u, *v, *ur;
  const int* level;
  const uint8_t* desc;
  float th;
  int reproj;  // 1: Fuse(KeyFrame*, vector<MapPoint*>, th); 0: Fuse(KeyFrame*, Scw, ...)
  int max_dist;  // accepted best distance: TH_LOW (Fuse), TH_HIGH (SearchBySim3)
  float inv_sigma2[kMaxLevels];
};

__global__ __launch_bounds__(256) void k_fuse(ProjFrameDev F, FusePointsDev P,
                                              int2* __restrict__ best) {
  const int lane = threadIdx.x & 63;
  const int p = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (p >= P.n) return;
  const int none_dist = P.reproj ? 256 : INT_MAX;  // bestDist's initial value (:904, :1063)
  bool go = P.use[p] != 0;
  const float u = P.u[p], v = P.v[p];
  const int lev = go ? P.level[p] : 0;
  const float rs = P.th * F.scale[lev];  // radius (:893, :1052)
  int cx0 = 0, cx1 = -1, cy0 = 0, cy1 = -1;
  if (go) {  // KeyFrame::GetFeaturesInArea window (KeyFrame.cc:523-541)
    cx0 = max(0, (int)floorf((u - F.min_x - rs) * F.gw));
    cx1 = min(kGridCols - 1, (int)ceilf((u - F.min_x + rs) * F.gw));
    cy0 = max(0, (int)floorf((v - F.min_y - rs) * F.gh));
    cy1 = min(kGridRows - 1, (int)ceilf((v - F.min_y + rs) * F.gh));
    if (cx0 >= kGridCols || cx1 < 0 || cy0 >= kGridRows || cy1 < 0) go = false;
  }
  if (!go) {
    if (lane == 0) best[p] = make_int2(-1, none_dist);
    return;
  }
  const int ny = cy1 - cy0 + 1, ncell = (cx1 - cx0 + 1) * ny;
  const uint64_t* q = (const uint64_t*)(P.desc + (int64_t)p * 32);
  const uint64_t d0 = q[0], d1 = q[1], d2 = q[2], d3 = q[3];
  const float ur = P.reproj && P.ur ? P.ur[p] : 0.f;
  // the minimum of (dist << 22 | candidate order) is the reference's first strict minimum
  int key = INT_MAX, kidx = -1, order0 = 0;
  for (int c0 = 0; c0 < ncell; c0 += 64) {
    const int c = c0 + lane;
    int b = 0, e = 0;
    if (c < ncell) {
      const int cell = (cx0 + c / ny) * kGridRows + cy0 + c % ny;
      b = F.cell_begin[cell];
      e = F.cell_begin[cell + 1];
    }
    auto in_area = [&](const orbx_keypoint& k) {
      const float dx = k.x - u, dy = k.y - v;
      return fabsf(dx) < rs && fabsf(dy) < rs;
    };
    int mine = 0;
    for (int j = b; j < e; j++) mine += in_area(F.keys[F.cell_feats[j]]);
    int tot;
    int pos = order0 + wave_excl_sum(mine, &tot);
    for (int j = b; j < e; j++) {
      const int idx = F.cell_feats[j];
      const orbx_keypoint k = F.keys[idx];
      if (!in_area(k)) continue;
      const int order = pos++;
      const int kl = k.octave;
      if (kl < lev - 1 || kl > lev) continue;  // (:914-915, :1070-1071)
      if (P.reproj) {
        const float ex = u - k.x, ey = v - k.y;
        const float e2xy = __builtin_fmaf(ex, ex, ey * ey);
        if (F.u_right && F.u_right[idx] >= 0) {  // (:917-930)
          const float er = ur - F.u_right[idx];
          const float e2 = __builtin_fmaf(er, er, e2xy);
          if ((double)(e2 * P.inv_sigma2[kl]) > 7.8) continue;
        } else {                                 // (:931-941)
          if ((double)(e2xy * P.inv_sigma2[kl]) > 5.99) continue;
        }
      }
      const uint64_t* t = (const uint64_t*)(F.desc + (int64_t)idx * 32);
      const int dist = __popcll(d0 ^ t[0]) + __popcll(d1 ^ t[1]) + __popcll(d2 ^ t[2]) +
                       __popcll(d3 ^ t[3]);
      const int kk = (dist << 22) | order;
      if (dist < none_dist && kk < key) {
        key = kk;
        kidx = idx;
      }
    }
    order0 += tot;
  }
  int K = key;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) K = min(K, __shfl_xor(K, o));
  const uint64_t win = __ballot(key == K);  // one lane: candidate orders are distinct
  const int idx = __shfl(kidx, __builtin_ctzll(win));
  if (lane == 0) {
    if (K == INT_MAX) best[p] = make_int2(-1, none_dist);
    else best[p] = make_int2((K >> 22) <= P.max_dist ? idx : -1, K >> 22);  // (:955, :1085, :1212)
  }
}

}  // namespace orbx

using namespace orbx;

namespace {

struct Staged {
  ProjFrameDev F;
  size_t cell, ids, off, feats, nn, begin, lists, cnts, err, match, nmatch;
};

// SearchBySim3's agreement (ORBmatcher.cc:1305-1326): KF1 point i1's best KF2 feature idx2 is
// kept when KF2 point idx2's best KF1 feature is i1.  best12 / best21: k_fuse results of the two
// directions (index or -1); m12[i1] = idx2 or -1; *nfound = the kept count.
__global__ __launch_bounds__(256) void k_sim3_agree(const int2* __restrict__ best12, int n1,
                                                    const int2* __restrict__ best21, int n2,
                                                    int* __restrict__ m12, int* __restrict__ nfound) {
  const int i1 = blockIdx.x * 256 + threadIdx.x;
  int keep = 0;
  if (i1 < n1) {
    const int idx2 = best12[i1].x;
    keep = idx2 >= 0 && idx2 < n2 && best21[idx2].x == i1;
    m12[i1] = keep ? idx2 : -1;
  }
  const int c = __popcll(__ballot(keep));
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(nfound, c);
}

// The frame's arrays and its grid (Frame::AssignFeaturesToGrid: k_grid_cells, k_csr,
// k_grid_dense) in one workspace: offsets of the uploaded arrays and of the grid scratch.
struct GridOffs {
  size_t keys, desc, ur, mp, cell, ids, off, feats, nn, beg;
};

void stage_frame(Stager& st, const orbx_proj_frame* f, GridOffs* g) {
  g->keys = st.add(f->keys_un, sizeof(orbx_keypoint) * f->n);
  g->desc = st.add(f->desc, (size_t)f->n * 32);
  g->ur = f->u_right ? st.add(f->u_right, 4 * (size_t)f->n) : 0;
  g->mp = f->has_mp_obs ? st.add(f->has_mp_obs, (size_t)f->n) : 0;
}

// after the uploads: the grid scratch (not uploaded)
void stage_grid(Stager& st, const orbx_proj_frame* f, GridOffs* g) {
  const size_t n = (size_t)std::max(f->n, 1);
  g->cell = st.add(nullptr, 4 * n);
  g->ids = st.add(nullptr, 4 * kCells);
  g->off = st.add(nullptr, 4 * (kCells + 1));
  g->feats = st.add(nullptr, 4 * n);
  g->nn = st.add(nullptr, 4);
  g->beg = st.add(nullptr, 4 * (kCells + 1));
}

// the device view of the frame (u_right / has_mp_obs only when `extras`) and its grid build
int launch_grid(const orbx_proj_frame* f, char* base, const GridOffs& g, bool extras,
                hipStream_t s, ProjFrameDev* out) {
  ProjFrameDev F{};
  F.n = f->n;
  F.keys = dptr<orbx_keypoint>(base, g.keys);
  F.desc = dptr<uint8_t>(base, g.desc);
  F.u_right = f->u_right && extras ? dptr<float>(base, g.ur) : nullptr;
  F.has_mp_obs = f->has_mp_obs && extras ? dptr<uint8_t>(base, g.mp) : nullptr;
  F.min_x = f->min_x;
  F.min_y = f->min_y;
  F.max_x = f->max_x;
  F.max_y = f->max_y;
  F.gw = f->grid_w_inv;
  F.gh = f->grid_h_inv;
  for (int l = 0; l < kMaxLevels; l++) F.scale[l] = l < f->nlevels ? f->scale_factors[l] : 1.f;
  F.cell_begin = dptr<int>(base, g.beg);
  F.cell_feats = dptr<int>(base, g.feats);
  if (f->n > 0) {
    hipLaunchKernelGGL(k_grid_cells, dim3((f->n + 255) / 256), dim3(256), 0, s, F,
                       dptr<uint32_t>(base, g.cell));
    const int rc = launch_csr(dptr<uint32_t>(base, g.cell), 0, nullptr, f->n, 0, kCells, nullptr,
                              dptr<uint32_t>(base, g.ids), dptr<int>(base, g.off),
                              dptr<int>(base, g.feats), 0, dptr<int>(base, g.nn), 1, s);
    if (rc) return rc;
    hipLaunchKernelGGL(k_grid_dense, dim3((kCells + 256) / 256), dim3(256), 0, s,
                       dptr<uint32_t>(base, g.ids), dptr<int>(base, g.off),
                       dptr<int>(base, g.nn), dptr<int>(base, g.beg));
  } else {
    ORBX_HIP(hipMemsetAsync(base + g.beg, 0, 4 * (kCells + 1), s));
  }
  *out = F;
  return ORBX_OK;
}

bool frame_ok(const orbx_proj_frame* f) {
  return f && f->n >= 0 && f->n <= 65535 && (f->n == 0 || (f->keys_un && f->desc)) &&
         f->scale_factors && f->nlevels >= 1 && f->nlevels <= kMaxLevels;
}

// SearchForInitialization's extra arguments (mode 2): src[8] = F1 keypoints, src[9] = the
// interleaved vbPrevMatched, copied back to prev_out after the call
struct InitCall {
  int n1;
  float nnratio;
  int check_ori;
  float* prev_out;
};

// Uploads the frame (and its grid) and the point arrays, finds every point's candidates, then
// resolves the search.  The candidate pool starts at kPoolPerPoint entries per point; a call
// whose lists need more is run again with the pool sized to their total (known after the
// first run), so no window size or feature density is unsupported.
int run_projection(const orbx_proj_frame* f, ProjPointsDev P, const std::vector<const void*>& src,
                   const std::vector<size_t>& bytes, int32_t* match, int32_t* nmatches,
                   const InitCall* ic = nullptr) {
  const int n = std::max(f->n, 1), np = std::max(P.n, 1);
  size_t pool_cap = std::max<size_t>((size_t)np * kPoolPerPoint, 4096);
  for (int attempt = 0; attempt < 2; attempt++) {
    Stager st;
    GridOffs go;
    stage_frame(st, f, &go);
    std::vector<size_t> offs;
    for (size_t i = 0; i < src.size(); i++) offs.push_back(src[i] ? st.add(src[i], bytes[i]) : 0);
    const size_t upload = st.host.size();
    stage_grid(st, f, &go);
    const size_t olists = st.add(nullptr, sizeof(int4) * pool_cap),
                 obases = st.add(nullptr, 4 * (size_t)np), ocnt = st.add(nullptr, 4 * (size_t)np),
                 oused = st.add(nullptr, 16), omatch = st.add(nullptr, 4 * (size_t)std::max(n, np)),
                 onm = st.add(nullptr, 4), olog = st.add(nullptr, 8 * (size_t)np);
    // SearchForInitialization state: in LDS when it fits one workgroup, else global scratch
    const size_t init_words = ic ? (size_t)f->n + 2 * (size_t)ic->n1 : 0;
    const bool init_lds = init_words * 4 <= 150 * 1024;
    const size_t oscratch = ic && !init_lds ? st.add(nullptr, 4 * init_words) : 0;
    int rc = tls_ws.reserve(st.host.size());
    if (rc) return rc;
    char* base = tls_ws.d;
    hipStream_t s = tls_ws.stream;
    ORBX_HIP(host_copy(base, st.host.data(), upload, st.host.pinned, hipMemcpyHostToDevice, s));
    ORBX_HIP(hipMemsetAsync(base + oused, 0, 16, s));
    ProjFrameDev F{};
    rc = launch_grid(f, base, go, !ic, s, &F);
    if (rc) return rc;
    // point arrays: fixed order of the `src` vector (use, x, y, xr, level, view_cos, angle, desc)
    ProjPointsDev Q = P;
    Q.use = dptr<uint8_t>(base, offs[0]);
    Q.x = dptr<float>(base, offs[1]);
    Q.y = dptr<float>(base, offs[2]);
    Q.xr = src[3] ? dptr<float>(base, offs[3]) : nullptr;
    Q.level = dptr<int>(base, offs[4]);
    Q.view_cos = src[5] ? dptr<float>(base, offs[5]) : nullptr;
    Q.angle = src[6] ? dptr<float>(base, offs[6]) : nullptr;
    Q.desc = dptr<uint8_t>(base, offs[7]);
    Q.blocks = src.size() > 10 && src[10] ? dptr<uint8_t>(base, offs[10]) : nullptr;
    Q.log = dptr<int2>(base, olog);
    if (P.n > 0)
      hipLaunchKernelGGL(k_proj_cand, dim3((P.n + 3) / 4), dim3(256), 0, s, F, Q,
                         dptr<int4>(base, olists), dptr<int>(base, obases), dptr<int>(base, ocnt),
                         dptr<int>(base, oused), (int)std::min<size_t>(pool_cap, INT32_MAX));
    if (ic) {
      const orbx_keypoint* k1 = dptr<const orbx_keypoint>(base, offs[8]);
      float* prev = dptr<float>(base, offs[9]);
      if (init_lds)
        hipLaunchKernelGGL(k_init_resolve<true>, dim3(1), dim3(64), 4 * init_words, s, F, k1,
                           ic->n1, dptr<int4>(base, olists), dptr<int>(base, obases),
                           dptr<int>(base, ocnt), ic->nnratio, ic->check_ori, prev,
                           dptr<int>(base, omatch), nullptr, dptr<int>(base, onm));
      else
        hipLaunchKernelGGL(k_init_resolve<false>, dim3(1), dim3(64), 0, s, F, k1, ic->n1,
                           dptr<int4>(base, olists), dptr<int>(base, obases), dptr<int>(base, ocnt),
                           ic->nnratio, ic->check_ori, prev, dptr<int>(base, omatch),
                           dptr<int>(base, oscratch), dptr<int>(base, onm));
    } else {
      hipLaunchKernelGGL(k_proj_resolve, dim3(1), dim3(64), 4 * (size_t)((n + 31) / 32), s, F, Q,
                         dptr<int4>(base, olists), dptr<int>(base, obases), dptr<int>(base, ocnt),
                         dptr<int>(base, omatch), dptr<int>(base, onm));
    }
    ORBX_HIP(hipGetLastError());
    int used = 0, nm = 0;
    ORBX_HIP(hipMemcpyAsync(&used, base + oused, 4, hipMemcpyDeviceToHost, s));
    ORBX_HIP(hipMemcpyAsync(&nm, base + onm, 4, hipMemcpyDeviceToHost, s));
    const int nout = ic ? ic->n1 : f->n;
    if (nout > 0)
      ORBX_HIP(hipMemcpyAsync(match, base + omatch, 4 * (size_t)nout, hipMemcpyDeviceToHost, s));
    ORBX_HIP(orbx::wait_stream(s));
    if ((size_t)(unsigned)used > pool_cap) {  // some list did not fit: rerun with the total
      pool_cap = (size_t)(unsigned)used;
      continue;
    }
    if (ic && ic->n1 > 0) {
      ORBX_HIP(hipMemcpyAsync(ic->prev_out, base + offs[9], 8 * (size_t)ic->n1,
                              hipMemcpyDeviceToHost, s));
      ORBX_HIP(orbx::wait_stream(s));
    }
    if (nmatches) *nmatches = nm;
    return ORBX_OK;
  }
  return report(ORBX_EDEVICE, "projection search: candidate pool still short after resizing");
}

// Fuse (both overloads): upload, grid, one k_fuse launch, download of (index, distance).
int run_fuse(const orbx_proj_frame* kf, const float* inv_sigma2, const orbx_fuse_points* m,
             float th, int reproj, int32_t* best_idx, int32_t* best_dist, int32_t* n_fused) {
  Stager st;
  GridOffs go;
  stage_frame(st, kf, &go);
  const size_t n = (size_t)m->n;
  const size_t ouse = st.add(m->use, n), ou = st.add(m->u, 4 * n), ov = st.add(m->v, 4 * n),
               our = reproj && m->ur ? st.add(m->ur, 4 * n) : 0,
               olev = st.add(m->pred_level, 4 * n), odesc = st.add(m->desc, 32 * n);
  const size_t upload = st.host.size();
  stage_grid(st, kf, &go);
  const size_t obest = st.add(nullptr, 8 * std::max<size_t>(n, 1));
  int rc = tls_ws.reserve(st.host.size());
  if (rc) return rc;
  char* base = tls_ws.d;
  hipStream_t s = tls_ws.stream;
  ORBX_HIP(host_copy(base, st.host.data(), upload, st.host.pinned, hipMemcpyHostToDevice, s));
  ProjFrameDev F{};
  rc = launch_grid(kf, base, go, reproj != 0, s, &F);
  if (rc) return rc;
  FusePointsDev P{};
  P.n = m->n;
  P.use = dptr<uint8_t>(base, ouse);
  P.u = dptr<float>(base, ou);
  P.v = dptr<float>(base, ov);
  P.ur = reproj && m->ur ? dptr<float>(base, our) : nullptr;
  P.level = dptr<int>(base, olev);
  P.desc = dptr<uint8_t>(base, odesc);
  P.th = th;
  P.reproj = reproj;
  P.max_dist = kTH_LOW;
  for (int l = 0; l < kMaxLevels; l++)
    P.inv_sigma2[l] = reproj && l < kf->nlevels ? inv_sigma2[l] : 1.f;
  if (m->n > 0)
    hipLaunchKernelGGL(k_fuse, dim3((m->n + 3) / 4), dim3(256), 0, s, F, P,
                       dptr<int2>(base, obest));
  ORBX_HIP(hipGetLastError());
  std::vector<int2> best(std::max<size_t>(n, 1));
  if (n) ORBX_HIP(hipMemcpyAsync(best.data(), base + obest, 8 * n, hipMemcpyDeviceToHost, s));
  ORBX_HIP(orbx::wait_stream(s));
  int nf = 0;
  for (size_t i = 0; i < n; i++) {
    best_idx[i] = best[i].x;
    if (best_dist) best_dist[i] = best[i].y;
    nf += best[i].x >= 0;
  }
  if (n_fused) *n_fused = nf;
  return ORBX_OK;
}

// SearchBySim3: both keyframes and both point sets in one upload, the two grids, the two
// per-point searches (k_fuse without reprojection gates, TH_HIGH) and the agreement.
int run_sim3(const orbx_proj_frame* kf1, const orbx_proj_frame* kf2, const orbx_fuse_points* m12,
             const orbx_fuse_points* m21, float th, int32_t* matches12, int32_t* n_found) {
  Stager st;
  GridOffs g1, g2;
  stage_frame(st, kf1, &g1);
  stage_frame(st, kf2, &g2);
  struct Offs { size_t use, u, v, lev, desc; } o[2];
  const orbx_fuse_points* ms[2] = {m12, m21};
  for (int k = 0; k < 2; k++) {
    const size_t n = (size_t)ms[k]->n;
    o[k].use = st.add(ms[k]->use, n);
    o[k].u = st.add(ms[k]->u, 4 * n);
    o[k].v = st.add(ms[k]->v, 4 * n);
    o[k].lev = st.add(ms[k]->pred_level, 4 * n);
    o[k].desc = st.add(ms[k]->desc, 32 * n);
  }
  const size_t upload = st.host.size();
  stage_grid(st, kf1, &g1);
  stage_grid(st, kf2, &g2);
  const size_t ob12 = st.add(nullptr, 8 * (size_t)std::max(m12->n, 1)),
               ob21 = st.add(nullptr, 8 * (size_t)std::max(m21->n, 1)),
               om12 = st.add(nullptr, 4 * (size_t)std::max(m12->n, 1)), ofound = st.add(nullptr, 4);
  int rc = tls_ws.reserve(st.host.size());
  if (rc) return rc;
  char* base = tls_ws.d;
  hipStream_t s = tls_ws.stream;
  ORBX_HIP(host_copy(base, st.host.data(), upload, st.host.pinned, hipMemcpyHostToDevice, s));
  ORBX_HIP(hipMemsetAsync(base + ofound, 0, 4, s));
  ProjFrameDev F1{}, F2{};
  rc = launch_grid(kf1, base, g1, false, s, &F1);
  if (rc) return rc;
  rc = launch_grid(kf2, base, g2, false, s, &F2);
  if (rc) return rc;
  // points of KF1 searched in KF2's grid, points of KF2 in KF1's
  for (int k = 0; k < 2; k++) {
    FusePointsDev P{};
    P.n = ms[k]->n;
    P.use = dptr<uint8_t>(base, o[k].use);
    P.u = dptr<float>(base, o[k].u);
    P.v = dptr<float>(base, o[k].v);
    P.ur = nullptr;
    P.level = dptr<int>(base, o[k].lev);
    P.desc = dptr<uint8_t>(base, o[k].desc);
    P.th = th;
    P.reproj = 0;
    P.max_dist = kTH_HIGH;
    for (int l = 0; l < kMaxLevels; l++) P.inv_sigma2[l] = 1.f;
    if (P.n > 0)
      hipLaunchKernelGGL(k_fuse, dim3((P.n + 3) / 4), dim3(256), 0, s, k == 0 ? F2 : F1, P,
                         dptr<int2>(base, k == 0 ? ob12 : ob21));
  }
  if (m12->n > 0)
    hipLaunchKernelGGL(k_sim3_agree, dim3((m12->n + 255) / 256), dim3(256), 0, s,
                       dptr<const int2>(base, ob12), m12->n, dptr<const int2>(base, ob21), m21->n,
                       dptr<int>(base, om12), dptr<int>(base, ofound));
  ORBX_HIP(hipGetLastError());
  ORBX_HIP(tls_ws.download(om12, ofound + 4 - om12));
  ORBX_HIP(orbx::wait_stream(s));
  if (m12->n > 0) memcpy(matches12, tls_ws.h + om12, 4 * (size_t)m12->n);
  *n_found = *(const int*)(tls_ws.h + ofound);
  return ORBX_OK;
}

bool fuse_args_ok(const orbx_proj_frame* kf, const orbx_fuse_points* m, int32_t* best_idx,
                  bool reproj) {
  if (!frame_ok(kf) || !m || m->n < 0 || (m->n > 0 && !best_idx)) return false;
  if (m->n > 0 && (!m->use || !m->u || !m->v || !m->pred_level || !m->desc ||
                   (reproj && kf->u_right && !m->ur)))
    return false;
  for (int i = 0; i < m->n; i++)
    if (m->use[i] && (m->pred_level[i] < 0 || m->pred_level[i] >= kf->nlevels)) return false;
  return true;
}

}  // namespace

extern "C" {

int orbx_search_by_projection(const orbx_proj_frame* f, const orbx_proj_points* m, float th,
                              float nnratio, int32_t* match, int32_t* nmatches) {
  if (!frame_ok(f) || !m || m->n < 0 || (f->n > 0 && !match)) return ORBX_EINVAL;
  if (m->n > 0 && (!m->track || !m->proj_x || !m->proj_y || !m->pred_level || !m->view_cos ||
                   !m->desc || (f->u_right && !m->proj_xr)))
    return ORBX_EINVAL;
  for (int i = 0; i < m->n; i++)
    if (m->track[i] && (m->pred_level[i] < 0 || m->pred_level[i] >= f->nlevels))
      return ORBX_EINVAL;
  ProjPointsDev P{};
  P.mode = 0;
  P.n = m->n;
  P.th = th;
  P.nnratio = nnratio;
  const size_t n = (size_t)m->n;
  return run_projection(f, P,
                        {m->track, m->proj_x, m->proj_y, m->proj_xr, m->pred_level, m->view_cos,
                         nullptr, m->desc},
                        {n, 4 * n, 4 * n, 4 * n, 4 * n, 4 * n, 0, 32 * n}, match, nmatches);
}

int orbx_search_by_projection_last(const orbx_proj_frame* f, const orbx_proj_last* l, float th,
                                   int32_t forward, int32_t backward, int32_t check_ori,
                                   int32_t* match, int32_t* nmatches) {
  if (!frame_ok(f) || !l || l->n < 0 || (f->n > 0 && !match)) return ORBX_EINVAL;
  if (l->n > 0 && (!l->valid || !l->u || !l->v || !l->octave || !l->angle || !l->desc ||
                   (f->u_right && !l->ur)))
    return ORBX_EINVAL;
  for (int i = 0; i < l->n; i++)
    if (l->valid[i] && (l->octave[i] < 0 || l->octave[i] >= f->nlevels)) return ORBX_EINVAL;
  ProjPointsDev P{};
  P.mode = 1;
  P.max_dist = kTH_HIGH;
  P.n = l->n;
  P.th = th;
  P.forward = forward;
  P.backward = backward;
  P.check_ori = check_ori;
  const size_t n = (size_t)l->n;
  return run_projection(f, P,
                        {l->valid, l->u, l->v, l->ur, l->octave, nullptr, l->angle, l->desc,
                         nullptr, nullptr, l->blocks},
                        {n, 4 * n, 4 * n, 4 * n, 4 * n, 0, 4 * n, 32 * n, 0, 0, n}, match,
                        nmatches);
}

int orbx_search_for_initialization(const orbx_proj_frame* f1, const orbx_proj_frame* f2,
                                   float* prev_matched, int32_t window_size, float nnratio,
                                   int32_t check_ori, int32_t* matches12, int32_t* nmatches) {
  if (!f1 || f1->n < 0 || f1->n > 65534 || (f1->n > 0 && (!f1->keys_un || !f1->desc)) ||
      !frame_ok(f2) || (f1->n > 0 && (!prev_matched || !matches12)))
    return ORBX_EINVAL;
  const int n1 = f1->n;
  // per F1 feature: use = (octave <= 0) (:421-423), window centre vbPrevMatched, level range
  // [octave, octave] (:425)
  std::vector<uint8_t> use(std::max(n1, 1));
  std::vector<float> px(std::max(n1, 1)), py(std::max(n1, 1));
  std::vector<int32_t> lev(std::max(n1, 1));
  for (int i = 0; i < n1; i++) {
    use[i] = f1->keys_un[i].octave <= 0;
    lev[i] = f1->keys_un[i].octave;
    px[i] = prev_matched[2 * i];
    py[i] = prev_matched[2 * i + 1];
  }
  ProjPointsDev P{};
  P.mode = 2;
  P.n = n1;
  P.th = (float)window_size;  // GetFeaturesInArea(..., const float& r = windowSize, ...)
  InitCall ic{n1, nnratio, check_ori, prev_matched};
  const size_t n = (size_t)n1;
  return run_projection(f2, P,
                        {use.data(), px.data(), py.data(), nullptr, lev.data(), nullptr, nullptr,
                         f1->desc, f1->keys_un, prev_matched},
                        {n, 4 * n, 4 * n, 0, 4 * n, 0, 0, 32 * n, sizeof(orbx_keypoint) * n, 8 * n},
                        matches12, nmatches, &ic);
}

int orbx_search_by_projection_kf(const orbx_proj_frame* f, const orbx_proj_last* k, float th,
                                 int32_t orb_dist, int32_t check_ori, int32_t* match,
                                 int32_t* nmatches) {
  if (!frame_ok(f) || !k || k->n < 0 || (f->n > 0 && !match)) return ORBX_EINVAL;
  if (k->n > 0 && (!k->valid || !k->u || !k->v || !k->octave || !k->angle || !k->desc))
    return ORBX_EINVAL;
  for (int i = 0; i < k->n; i++)
    if (k->valid[i] && (k->octave[i] < 0 || k->octave[i] >= f->nlevels)) return ORBX_EINVAL;
  ProjPointsDev P{};
  P.mode = 3;
  P.max_dist = orb_dist;
  P.n = k->n;
  P.th = th;
  P.check_ori = check_ori;
  const size_t n = (size_t)k->n;
  return run_projection(f, P, {k->valid, k->u, k->v, nullptr, k->octave, nullptr, k->angle, k->desc},
                        {n, 4 * n, 4 * n, 0, 4 * n, 0, 4 * n, 32 * n}, match, nmatches);
}

int orbx_search_by_projection_sim3(const orbx_proj_frame* kf, const orbx_fuse_points* m,
                                   float th, int32_t* match, int32_t* nmatches) {
  if (!fuse_args_ok(kf, m, match, false) || (kf->n > 0 && !match)) return ORBX_EINVAL;
  ProjPointsDev P{};
  P.mode = 4;
  P.max_dist = kTH_LOW;
  P.n = m->n;
  P.th = th;
  const size_t n = (size_t)m->n;
  return run_projection(kf, P, {m->use, m->u, m->v, nullptr, m->pred_level, nullptr, nullptr, m->desc},
                        {n, 4 * n, 4 * n, 0, 4 * n, 0, 0, 32 * n}, match, nmatches);
}

int orbx_search_by_sim3(const orbx_proj_frame* kf1, const orbx_proj_frame* kf2,
                        const orbx_fuse_points* points12, const orbx_fuse_points* points21,
                        float th, int32_t* matches12, int32_t* n_found) {
  if (!n_found || !fuse_args_ok(kf2, points12, matches12, false) ||
      !fuse_args_ok(kf1, points21, matches12, false))
    return ORBX_EINVAL;
  if (points12->n != kf1->n || points21->n != kf2->n) return ORBX_EINVAL;  // one point per keypoint
  return run_sim3(kf1, kf2, points12, points21, th, matches12, n_found);
}

int orbx_fuse(const orbx_proj_frame* kf, const float* inv_level_sigma2,
              const orbx_fuse_points* points, float th, int32_t* best_idx, int32_t* best_dist,
              int32_t* n_fused) {
  if (!fuse_args_ok(kf, points, best_idx, true) || !inv_level_sigma2) return ORBX_EINVAL;
  return run_fuse(kf, inv_level_sigma2, points, th, 1, best_idx, best_dist, n_fused);
}

int orbx_fuse_sim3(const orbx_proj_frame* kf, const orbx_fuse_points* points, float th,
                   int32_t* best_idx, int32_t* best_dist, int32_t* n_fused) {
  if (!fuse_args_ok(kf, points, best_idx, false)) return ORBX_EINVAL;
  return run_fuse(kf, nullptr, points, th, 0, best_idx, best_dist, n_fused);
}

}  // extern "C"
