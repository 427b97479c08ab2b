// orbx_project.hip — the tracking searches on the GPU:
//   Frame::AssignFeaturesToGrid / GetFeaturesInArea        (ORB_SLAM2/src/Frame.cc:235-250, 332-398)
//   ORBmatcher::SearchByProjection(Frame&, vector<MapPoint*>, th)       (ORBmatcher.cc:45-137)
//   ORBmatcher::SearchByProjection(Frame&, const Frame&, th, bMono)     (ORBmatcher.cc:1331-1474)
// (GetFeaturesInArea runs fused inside the searches; it has no entry point of its own.)
//
//   k_grid_cells   cell of every feature (PosInGrid: round((x - mnMinX) * inv)); k_csr then
//                  buckets the features by cell, ascending index inside a cell (mGrid order)
//   k_grid_dense   per-cell [begin, end) table over all 64 x 48 cells
//   k_proj_cand    one wave per point: GetFeaturesInArea in the reference's order (cells
//                  column-major over the window, lanes over cells, wave prefix sum for the
//                  output position), the static filters (level range, |dx| < r && |dy| < r,
//                  features already holding a MapPoint with observations, the stereo uR test)
//                  and the Hamming distance; the ordered candidate list goes to global memory
//   k_proj_resolve one wave per frame, points in order: the greedy part of the reference — a
//                  feature matched by an earlier point is skipped by the later ones — over the
//                  candidate lists with a claimed-feature bitmap in LDS.  Best / second of the
//                  reference's sequential update are recovered in parallel: best = first
//                  minimum; second = first minimum of {best-before-best} + {candidates after
//                  best}.  Motion-model variant: rotation histogram + ComputeThreeMaxima.
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
constexpr int kCandCap = 512;  // candidates one point may collect
constexpr int kTH_HIGH = 100;
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

// mode 0: local-map points (SearchByProjection(F, vpMapPoints, th)); 1: last frame
struct ProjPointsDev {
  int mode;
  int n;
  const uint8_t* use;   // track (mode 0) / valid (mode 1)
  const float *x, *y, *xr;
  const int* level;     // predicted level (mode 0) / last octave (mode 1)
  const float* view_cos;
  const float* angle;
  const uint8_t* desc;
  float th, nnratio;
  int forward, backward, check_ori;
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

// candidates of point p: (feature index, distance, octave) in GetFeaturesInArea order
__global__ __launch_bounds__(256) void k_proj_cand(ProjFrameDev F, ProjPointsDev P,
                                                   int4* __restrict__ lists,
                                                   int* __restrict__ counts,
                                                   int* __restrict__ error) {
  const int lane = threadIdx.x & 63;
  const int p = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (p >= P.n) return;
  int cnt_out = 0;
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
  } else if (go) {
    if (x < F.min_x || x > F.max_x || y < F.min_y || y > F.max_y) go = false;  // :1377-1380
    const int oct = P.level[p];
    rs = P.th * F.scale[oct];
    if (P.forward) minLevel = oct, maxLevel = -1;
    else if (P.backward) minLevel = 0, maxLevel = oct;
    else minLevel = oct - 1, maxLevel = oct + 1;
  }
  int cx0 = 0, cx1 = -1, cy0 = 0, cy1 = -1;
  if (go) {  // GetFeaturesInArea window (Frame.cc:337-351)
    cx0 = max(0, (int)floorf((x - F.min_x - rs) * F.gw));
    cx1 = min(kGridCols - 1, (int)ceilf((x - F.min_x + rs) * F.gw));
    cy0 = max(0, (int)floorf((y - F.min_y - rs) * F.gh));
    cy1 = min(kGridRows - 1, (int)ceilf((y - F.min_y + rs) * F.gh));
    if (cx0 >= kGridCols || cx1 < 0 || cy0 >= kGridRows || cy1 < 0) go = false;
  }
  if (go) {
    const bool bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
    const int ny = cy1 - cy0 + 1, ncell = (cx1 - cx0 + 1) * ny;
    const uint64_t* q = (const uint64_t*)(P.desc + (int64_t)p * 32);
    const uint64_t d0 = q[0], d1 = q[1], d2 = q[2], d3 = q[3];
    const float xr = P.xr ? P.xr[p] : 0.f;
    int4* out = lists + (int64_t)p * kCandCap;
    for (int c0 = 0; c0 < ncell; c0 += 64) {
      const int c = c0 + lane;
      int b = 0, e = 0;
      if (c < ncell) {
        const int cell = (cx0 + c / ny) * kGridRows + cy0 + c % ny;
        b = F.cell_begin[cell];
        e = F.cell_begin[cell + 1];
      }
      auto pass = [&](int idx) -> bool {
        const orbx_keypoint k = F.keys[idx];
        if (bCheckLevels) {
          if (k.octave < minLevel) return false;
          if (maxLevel >= 0 && k.octave > maxLevel) return false;
        }
        const float dx = k.x - x, dy = k.y - y;
        return fabsf(dx) < rs && fabsf(dy) < rs;
      };
      int mine = 0;
      for (int j = b; j < e; j++) mine += pass(F.cell_feats[j]);
      int tot;
      int pos = cnt_out + wave_excl_sum(mine, &tot);
      for (int j = b; j < e; j++) {
        const int idx = F.cell_feats[j];
        if (!pass(idx)) continue;
        // static per-candidate filters of the searches; the order slot is kept either way
        int dist = 256;
        bool ok = !(F.has_mp_obs && F.has_mp_obs[idx]);
        if (ok && F.u_right && F.u_right[idx] > 0) {
          const float er = fabsf((P.mode == 0 ? P.xr[p] : xr) - F.u_right[idx]);
          ok = !(er > (P.mode == 0 ? r * F.scale[P.level[p]] : rs));
        }
        if (ok) {
          const uint64_t* t = (const uint64_t*)(F.desc + (int64_t)idx * 32);
          dist = __popcll(d0 ^ t[0]) + __popcll(d1 ^ t[1]) + __popcll(d2 ^ t[2]) +
                 __popcll(d3 ^ t[3]);
        }
        if (pos < kCandCap) out[pos] = make_int4(idx, dist, F.keys[idx].octave, 0);
        pos++;
      }
      cnt_out += tot;
    }
  }
  if (lane == 0) {
    counts[p] = min(cnt_out, kCandCap);
    if (cnt_out > kCandCap) atomicOr(error, 1);
  }
}

// one wave: points in order, greedy claims in an LDS bitmap
__global__ __launch_bounds__(64) void k_proj_resolve(ProjFrameDev F, ProjPointsDev P,
                                                     const int4* __restrict__ lists,
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
    const int4* lst = lists + (int64_t)p * kCandCap;
    // pass 1: best = first minimum over unclaimed candidates with dist < 256
    int key1 = INT_MAX;
    for (int j = lane; j < L; j += 64) {
      const int4 c = lst[j];
      const bool claimed = (s_claim[c.x >> 5] >> (c.x & 31)) & 1;
      if (!claimed && c.y < 256) key1 = min(key1, (c.y << 10) | j);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) key1 = min(key1, __shfl_xor(key1, o));
    if (key1 == INT_MAX) continue;
    const int bestDist = key1 >> 10, bestPos = key1 & 1023;
    if (bestDist > kTH_HIGH) continue;
    const int4 best = lst[bestPos];
    if (P.mode == 0) {
      // second: first minimum of {the best among candidates before bestPos} followed by the
      // candidates after bestPos, in order
      int kpre = INT_MAX, ksuf = INT_MAX;
      for (int j = lane; j < L; j += 64) {
        const int4 c = lst[j];
        const bool claimed = (s_claim[c.x >> 5] >> (c.x & 31)) & 1;
        if (claimed || c.y >= 256 || j == bestPos) continue;
        if (j < bestPos) kpre = min(kpre, (c.y << 10) | j);
        else ksuf = min(ksuf, (c.y << 10) | j);
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        kpre = min(kpre, __shfl_xor(kpre, o));
        ksuf = min(ksuf, __shfl_xor(ksuf, o));
      }
      int bestDist2 = 256, bestLevel2 = -1;
      const int dpre = kpre == INT_MAX ? 256 : kpre >> 10;
      const int dsuf = ksuf == INT_MAX ? 256 : ksuf >> 10;
      if (kpre != INT_MAX && dpre <= dsuf) {
        bestDist2 = dpre;
        bestLevel2 = lst[kpre & 1023].z;
      } else if (ksuf != INT_MAX) {
        bestDist2 = dsuf;
        bestLevel2 = lst[ksuf & 1023].z;
      }
      const int bestLevel = best.z;
      if (bestLevel == bestLevel2 && (float)bestDist > P.nnratio * (float)bestDist2) continue;
    }
    if (lane == 0) {
      match[best.x] = p;
      s_claim[best.x >> 5] |= 1u << (best.x & 31);
      if (P.mode == 1 && P.check_ori) {
        float rot = P.angle[p] - F.keys[best.x].angle;
        if (rot < 0.0) rot += 360.0f;
        int bin = (int)roundf(rot * factor);
        if (bin == kHisto) bin = 0;
        s_hist[bin]++;
      }
    }
    nm++;
    __syncthreads();
  }
  if (P.mode == 1 && P.check_ori) {
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
    int removed = 0;
    for (int i = lane; i < F.n; i += 64) {
      const int p = match[i];
      if (p < 0) continue;
      float rot = P.angle[p] - F.keys[i].angle;
      if (rot < 0.0) rot += 360.0f;
      int bin = (int)roundf(rot * factor);
      if (bin == kHisto) bin = 0;
      if (bin != ind1 && bin != ind2 && bin != ind3) {
        match[i] = -1;
        removed++;
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) removed += __shfl_xor(removed, o);
    nm -= removed;
  }
  if (lane == 0) *nmatch = nm;
}

}  // namespace orbx

using namespace orbx;

namespace {

struct Staged {
  ProjFrameDev F;
  size_t cell, ids, off, feats, nn, begin, lists, cnts, err, match, nmatch;
};

// uploads the frame and the point arrays, builds the grid, returns device descriptors
int stage_frame(Stager& st, const orbx_proj_frame* f, size_t* off_keys, size_t* off_desc,
                size_t* off_ur, size_t* off_mp) {
  *off_keys = st.add(f->keys_un, sizeof(orbx_keypoint) * f->n);
  *off_desc = st.add(f->desc, (size_t)f->n * 32);
  *off_ur = f->u_right ? st.add(f->u_right, 4 * (size_t)f->n) : 0;
  *off_mp = f->has_mp_obs ? st.add(f->has_mp_obs, (size_t)f->n) : 0;
  return ORBX_OK;
}

bool frame_ok(const orbx_proj_frame* f) {
  return f && f->n >= 0 && f->n <= 65535 && (f->n == 0 || (f->keys_un && f->desc)) &&
         f->scale_factors && f->nlevels >= 1 && f->nlevels <= kMaxLevels;
}

int run_projection(const orbx_proj_frame* f, ProjPointsDev P, const std::vector<const void*>& src,
                   const std::vector<size_t>& bytes, int32_t* match, int32_t* nmatches) {
  Stager st;
  size_t ok_, od, our, omp;
  stage_frame(st, f, &ok_, &od, &our, &omp);
  std::vector<size_t> offs;
  for (size_t i = 0; i < src.size(); i++) offs.push_back(src[i] ? st.add(src[i], bytes[i]) : 0);
  const size_t upload = st.host.size();
  const int n = std::max(f->n, 1), np = std::max(P.n, 1);
  const size_t ocell = st.add(nullptr, 4 * (size_t)n), oids = st.add(nullptr, 4 * kCells),
               ooff = st.add(nullptr, 4 * (kCells + 1)), ofeats = st.add(nullptr, 4 * (size_t)n),
               onn = st.add(nullptr, 4), obeg = st.add(nullptr, 4 * (kCells + 1)),
               olists = st.add(nullptr, sizeof(int4) * kCandCap * (size_t)np),
               ocnt = st.add(nullptr, 4 * (size_t)np), oerr = st.add(nullptr, 4),
               omatch = st.add(nullptr, 4 * (size_t)n), onm = st.add(nullptr, 4);
  int rc = tls_ws.reserve(st.host.size());
  if (rc) return rc;
  char* base = tls_ws.d;
  hipStream_t s = tls_ws.stream;
  ORBX_HIP(hipMemcpyAsync(base, st.host.data(), upload, hipMemcpyHostToDevice, s));
  ORBX_HIP(hipMemsetAsync(base + oerr, 0, 4, s));
  ProjFrameDev F{};
  F.n = f->n;
  F.keys = dptr<orbx_keypoint>(base, ok_);
  F.desc = dptr<uint8_t>(base, od);
  F.u_right = f->u_right ? dptr<float>(base, our) : nullptr;
  F.has_mp_obs = f->has_mp_obs ? dptr<uint8_t>(base, omp) : nullptr;
  F.min_x = f->min_x;
  F.min_y = f->min_y;
  F.max_x = f->max_x;
  F.max_y = f->max_y;
  F.gw = f->grid_w_inv;
  F.gh = f->grid_h_inv;
  for (int l = 0; l < kMaxLevels; l++) F.scale[l] = l < f->nlevels ? f->scale_factors[l] : 1.f;
  F.cell_begin = dptr<int>(base, obeg);
  F.cell_feats = dptr<int>(base, ofeats);
  // point arrays: fixed order of the `src` vector (use, x, y, xr, level, view_cos, angle, desc)
  P.use = dptr<uint8_t>(base, offs[0]);
  P.x = dptr<float>(base, offs[1]);
  P.y = dptr<float>(base, offs[2]);
  P.xr = src[3] ? dptr<float>(base, offs[3]) : nullptr;
  P.level = dptr<int>(base, offs[4]);
  P.view_cos = src[5] ? dptr<float>(base, offs[5]) : nullptr;
  P.angle = src[6] ? dptr<float>(base, offs[6]) : nullptr;
  P.desc = dptr<uint8_t>(base, offs[7]);
  if (f->n > 0) {
    hipLaunchKernelGGL(k_grid_cells, dim3((f->n + 255) / 256), dim3(256), 0, s, F,
                       dptr<uint32_t>(base, ocell));
    rc = launch_csr(dptr<uint32_t>(base, ocell), 0, nullptr, f->n, 0, kCells, nullptr,
                    dptr<uint32_t>(base, oids), dptr<int>(base, ooff), dptr<int>(base, ofeats), 0,
                    dptr<int>(base, onn), 1, s);
    if (rc) return rc;
    hipLaunchKernelGGL(k_grid_dense, dim3((kCells + 256) / 256), dim3(256), 0, s,
                       dptr<uint32_t>(base, oids),
                       dptr<int>(base, ooff), dptr<int>(base, onn), dptr<int>(base, obeg));
  } else {
    ORBX_HIP(hipMemsetAsync(base + obeg, 0, 4 * (kCells + 1), s));
  }
  if (P.n > 0)
    hipLaunchKernelGGL(k_proj_cand, dim3((P.n + 3) / 4), dim3(256), 0, s, F, P,
                       dptr<int4>(base, olists), dptr<int>(base, ocnt), dptr<int>(base, oerr));
  hipLaunchKernelGGL(k_proj_resolve, dim3(1), dim3(64), 4 * (size_t)((n + 31) / 32), s, F, P,
                     dptr<int4>(base, olists), dptr<int>(base, ocnt), dptr<int>(base, omatch),
                     dptr<int>(base, onm));
  ORBX_HIP(hipGetLastError());
  int err = 0, nm = 0;
  ORBX_HIP(hipMemcpyAsync(&err, base + oerr, 4, hipMemcpyDeviceToHost, s));
  ORBX_HIP(hipMemcpyAsync(&nm, base + onm, 4, hipMemcpyDeviceToHost, s));
  if (f->n > 0)
    ORBX_HIP(hipMemcpyAsync(match, base + omatch, 4 * (size_t)f->n, hipMemcpyDeviceToHost, s));
  ORBX_HIP(hipStreamSynchronize(s));
  if (err) return ORBX_EUNSUPPORTED;  // a window held more than kCandCap features
  if (nmatches) *nmatches = nm;
  return ORBX_OK;
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
  P.n = l->n;
  P.th = th;
  P.forward = forward;
  P.backward = backward;
  P.check_ori = check_ori;
  const size_t n = (size_t)l->n;
  return run_projection(f, P, {l->valid, l->u, l->v, l->ur, l->octave, nullptr, l->angle, l->desc},
                        {n, 4 * n, 4 * n, 4 * n, 4 * n, 0, 4 * n, 32 * n}, match, nmatches);
}

}  // extern "C"
