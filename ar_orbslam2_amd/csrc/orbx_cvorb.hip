// orbx_cvorb.hip — the AR marker path on gfx950: cv::ORB::operator() of OpenCV 2.4 (orb.cpp)
// with HARRIS_SCORE or FAST_SCORE, as ORB_SLAM2/src/Marker.cc:76-84, 98-108 and
// AR-1.3/src/ORBMatcher.cpp:121-122 call it, plus the brute-force Hamming matchers of the same
// path (Marker.cc:110-133, AR-1.3/src/ORBMatcher.cpp:44-102).
//
// One plan = one image size + one cv::ORB parameter set + a maximum batch.  A batch runs as a
// fixed launch sequence on the plan's stream (captured once into a hipGraph):
//   k_pyramid      levels (cv::resize INTER_LINEAR from the previous level; shared with the
//                  ORBextractor plan, orbx_extract.hip)
//   k_cvfast       64x64 tiles of every level's border region [edge, w-edge) x [edge, h-edge):
//                  FAST-9/16 cornerScore at threshold 20 + whole-image 8-neighbour NMS
//                  (cv::FAST(..., nonmax=true) followed by runByImageBorder) -> keep bitmaps
//   k_cvselect     one wave per (image, level): raster-order compaction of the keep bitmaps,
//                  KeyPointsFilter::retainBest(2N), HarrisResponses(7, 0.04), retainBest(N)
//                  with the exact element order GCC 4.8's nth_element / partition leave
//   k_blur         GaussianBlur 7x7 sigma 2 of every level (shared with the ORBextractor plan)
//   k_cvdescribe   one half-wave per keypoint: IC_Angle, fastAtan2, rBRIEF (WTA_K 2) on the
//                  blurred level with double cos/sin, level-0 scaling, level-major output
// and for the marker: k_bfmatch (BruteForceMatcher<HammingLUT>::match, query = target) and
// k_good (Marker::Match's distance < 0.5 * max_dist filter).
//
// retainBest on the GPU.  KeyPointsFilter::retainBest is std::nth_element(begin, begin + N,
// end, response-greater) + std::partition(begin + N, end, response >= ambiguous), so which of
// the keypoints tied at the boundary survive, and the order of the survivors (the order of
// the output keypoints and descriptors), are those algorithms' outputs.  Both run here as the
// same sequence of partitioning steps, each done in parallel: a Hoare-style partition (two
// scans that stop at "left stoppers" and "right stoppers" and swap) swaps the k-th left stopper
// with the k-th right stopper from the right exactly while the first is left of the second, so
// with both stoppers' ranks from ballots and prefix counts every swap pair is known at once.
// The cut the sequential loop returns is min(first unswapped left stopper, last swapped
// right stopper).  The median-of-three pivot, the depth-limited heap_select fallback and the
// final insertion sort of <= 3 elements run on lane 0.  DESIGN.md §10 gives the derivation.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/orbx_pattern.h"
#include "orbx_describe.h"
#include "orbx_internal.h"
#include "orbx_match.h"
#include "orbx_math.h"

#pragma clang fp contract(off)

namespace orbx {
namespace cvorb {

__constant__ int8_t c_cv_pattern[1024];            // bit_pattern_31_ (512 points)
__constant__ IcMask c_cv_icmask;                   // IC_Angle row masks (umax, half 15)

constexpr float kHarrisK = 0.04f;  // HARRIS_K (orb.cpp)
constexpr int kFastTh = 20;        // computeKeyPoints: FastFeatureDetector fd(20, true)
constexpr int kTW = 64, kTH = 64;  // k_cvfast tile
constexpr int kSelCap = 2560;  // k_cvselect: keypoints kept in LDS (30 KB: 5 waves per CU; more: global)

struct CvLevel {
  int w, h, pitch, pyr_off;
  int rx0, rx1, ry0, ry1;  // border region [edge, w-edge) x [edge, h-edge) (empty: rx1 <= rx0)
  int bm_off, bm_wpr;      // keep bitmap words of this level inside one image's block
  int feats;               // nfeaturesPerLevel
  int cand_off, cand_cap;  // global candidate scratch (max strict-NMS survivors of the region)
  int kp_off, kp_cap;      // per-image keypoint slots of this level
  float scale, size;       // getScale(level, 0, scaleFactor), patchSize * scale
};

struct CvTile {
  int16_t level, tx, ty, pad;
};

struct __align__(8) CvKey {
  float r;     // response (FAST score, then Harris)
  uint32_t k;  // y << 16 | x in level coordinates
};

__device__ __forceinline__ void xcd_block(int& bx, int& by) {
  const int gx = gridDim.x, total = gx * gridDim.y;
  int lin = blockIdx.y * gx + blockIdx.x;
  const int q = total >> 3;
  if (lin < (q << 3)) lin = (lin & 7) * q + (lin >> 3);
  by = lin / gx;
  bx = lin - by * gx;
}

// ------------------------------------------------------------------ k_cvfast
// cv::FAST(level, keypoints, 20, true) keeps p when score(p) >= 20 and score(p) > V(q) for the
// 8 neighbours, V(q) = score(q) if q is a corner at 20, else 0 (fast.cpp); then
// runByImageBorder drops every keypoint outside [edge, w-edge) x [edge, h-edge) (edge >= 18,
// so every neighbour of a kept pixel is a detection pixel).  A 64 x 64 tile stages rows
// Y0-4..Y0+67 and columns X0-16..X0+79 (16-byte loads); the V window is the tile plus a 1-px
// ring, restricted to [edge-1, w-edge] x [edge-1, h-edge].  The even-circle-point pretest runs
// one pixel per lane with the compares as lane masks (fast_pretest), only its survivors are
// queued (per wave, mbcnt ranks) and scored; the strict NMS is evaluated at the queued pixels
// of the tile proper, survivors set their bit in the row's keep word (ds_or) and store their
// score for k_cvselect.
__global__ __launch_bounds__(256) void k_cvfast(const uint8_t* __restrict__ pyr, int64_t pyr_bytes,
                                                const CvLevel* __restrict__ lv,
                                                const CvTile* __restrict__ tiles,
                                                uint64_t* __restrict__ bitmaps, int64_t bm_words,
                                                uint8_t* __restrict__ smap) {
  constexpr int kInR = kTH + 8;           // staged rows Y0-4 .. Y0+kTH+3
  constexpr int kInD = (kTW + 32) / 4;    // staged dwords: columns X0-16 .. X0+79
  constexpr int kRowB = kInD * 4;         // staged row stride (bytes)
  constexpr int kWinR = kTH + 2;          // V rows Y0-1 .. Y0+kTH
  constexpr int kVS = kTW + 8;            // V row stride: columns X0-4 .. X0+67
  // per-wave queue bound: wave w pretests the row pairs starting at 2w mod 8, i.e. at most
  // ceil(kWinR / 8) pairs = 2 * ceil(kWinR / 8) full rows, and wave 0 also takes one ring
  // pass of 64 pixels (waves 1 and 2 take the rest of the ring, fewer rows)
  constexpr int kQ = 2 * ((kWinR + 7) / 8) * 64 + 64;
  __shared__ __align__(16) uint32_t s_in[kInR][kInD];
  __shared__ __align__(16) uint32_t s_v32[kWinR * kVS / 4];
  __shared__ uint16_t s_q[4][kQ + 64];
  __shared__ uint64_t s_keep[kTH];
  int bx, img;
  xcd_block(bx, img);
  const CvTile T = tiles[bx];
  const CvLevel L = lv[T.level];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int X0 = T.tx * kTW, Y0 = L.ry0 + T.ty * kTH;
  const uint8_t* src = pyr + (int64_t)img * pyr_bytes + L.pyr_off;
  for (int i = tid; i < kInR * (kInD / 4); i += 256) {
    const int r = i / (kInD / 4), c = i - r * (kInD / 4);
    const int y = min(max(Y0 + r - 4, 0), L.h - 1);
    const int x = X0 - 16 + 16 * c;
    *(uint4*)&s_in[r][4 * c] = (x >= 0 && x < L.pitch)
                                   ? *(const uint4*)(src + (uint32_t)(__mul24(y, L.pitch) + x))
                                   : make_uint4(0u, 0u, 0u, 0u);
  }
  for (int i = tid; i < kWinR * kVS / 4; i += 256) s_v32[i] = 0;
  if (tid < kTH) s_keep[tid] = 0;
  __syncthreads();
  const int t = kFastTh;
  // V window: x = X0 - 4 + vx, y = Y0 - 1 + vy; staged row vy + 3, byte vx + 12
  const int xlo = L.rx0 - 1, xhi = L.rx1, ylo = L.ry0 - 1, yhi = L.ry1;  // inclusive
  uint16_t* q = s_q[wid];
  int nq = 0;
  const uint8_t* sin8 = (const uint8_t*)s_in;
  auto enqueue = [&](uint64_t pass, int idx) {
    q[(pass >> lane) & 1 ? nq + lane_rank(pass) : kQ + lane] = (uint16_t)idx;
    nq += __popcll(pass);
  };
  const uint64_t col_ok = __ballot(X0 + lane >= xlo && X0 + lane <= xhi);
  if (col_ok != 0) {
    const int vy_lo = max(0, ylo - (Y0 - 1)), vy_hi = min(kWinR, yhi - (Y0 - 1) + 1);
    // row pairs (vy, vy + 1) on the dual-issue pretest (orbx_internal.h fast_pretest2), pair
    // index = wid mod 4; vy_lo is 0, so the last pair's second row is at most kWinR - 1
    // the lane's flag bits of interest: its column inside the detection region
    const uint32_t fm = (X0 + lane >= xlo && X0 + lane <= xhi) ? 0x80008000u : 0u;
    for (int vy = vy_lo + 2 * wid; vy < vy_hi; vy += 8) {
      const uint32_t f = fast_pretest2<kRowB>(sin8 + vy * kRowB + lane + 13, t) &
                         (vy + 1 < vy_hi ? fm : fm & 0x8000u);
      wave_enqueue(q, nq, kQ, (f & 0x8000u) != 0, vy * kVS + 4 + lane, lane);
      wave_enqueue(q, nq, kQ, (int32_t)f < 0, (vy + 1) * kVS + 4 + lane, lane);
    }
  }
  // ring columns X0-1 (vx 3) and X0+64 (vx 68)
  for (int k0 = wid * 64; k0 < 2 * kWinR; k0 += 256) {
    const int k = k0 + lane;
    const int vy = min(k >> 1, kWinR - 1), vx = k & 1 ? 4 + kTW : 3;
    const int x = X0 - 4 + vx, y = Y0 - 1 + vy;
    const uint64_t ok = __ballot(k < 2 * kWinR && x >= xlo && x <= xhi && y >= ylo && y <= yhi);
    if (ok != 0) enqueue(fast_pretest<kRowB>(sin8 + vy * kRowB + vx + 9, t, ok), vy * kVS + vx);
  }
  uint8_t* s_v = (uint8_t*)s_v32;
  for (int j0 = 0; j0 < nq; j0 += 64) {
    const int j = j0 + lane;
    if (j < nq) {
      const int i = q[j];
      const int vy = i / kVS, vx = i - vy * kVS;
      const int sc = fast_score(sin8, kRowB, vx + 12, vy + 3);
      s_v[i] = (uint8_t)(sc >= t ? sc : 0);
    }
  }
  __syncthreads();
  uint8_t* sm = smap + (int64_t)img * pyr_bytes + L.pyr_off;
  for (int j0 = 0; j0 < nq; j0 += 64) {
    const int j = j0 + lane;
    if (j >= nq) break;
    const int i = q[j];
    const int vy = i / kVS, vx = i - vy * kVS;
    const int tx = vx - 4, ty = vy - 1;
    const int x = X0 + tx, y = Y0 + ty;
    if (tx < 0 || tx >= kTW || ty < 0 || ty >= kTH || x < L.rx0 || x >= L.rx1 || y >= L.ry1)
      continue;
    const int v = s_v[i];
    if (v == 0) continue;
    const uint8_t* pu = s_v + i - kVS;
    const uint8_t* pd = s_v + i + kVS;
    const int nmax = max(max(max((int)pu[-1], (int)pu[0]), max((int)pu[1], (int)s_v[i - 1])),
                         max(max((int)s_v[i + 1], (int)pd[-1]), max((int)pd[0], (int)pd[1])));
    if (v > nmax) {
      atomicOr((unsigned long long*)&s_keep[ty], 1ull << tx);
      sm[(int64_t)y * L.pitch + x] = (uint8_t)v;
    }
  }
  __syncthreads();
  if (tid < kTH) {
    const int y = Y0 + tid;
    if (y < L.ry1)
      bitmaps[(int64_t)img * bm_words + L.bm_off + (int64_t)y * L.bm_wpr + T.tx] = s_keep[tid];
  }
}

// ------------------------------------------------------------------ retainBest (one wave)
__device__ __forceinline__ int wave_incl_scan(int v) {
  return wave_scan_incl(v);
}

__device__ __forceinline__ void kswap(CvKey* a, int i, int j) {
  const CvKey t = a[i];
  a[i] = a[j];
  a[j] = t;
}

struct Stoppers {
  int K;     // swap pairs
  int cutL;  // first left stopper that is not swapped (INT_MAX: none)
  int cutR;  // smallest swapped right-stopper position (hi: none)
  int rtot;  // right stoppers in [lo, hi)
};

// The swap sequence of a two-scan partition of [lo, hi): the left scan stops at elements with
// ls(e), the right scan at rs(e); pair k = (k-th left stopper from lo, k-th right stopper from
// hi - 1) swaps while the first is left of the second.  Lpos / Rpos hold up to (hi-lo)/2 ints.
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int lane) {
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, lane);
  const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), lane);
  return ((uint64_t)hi << 32) | lo;
}

// (For up to 64 chunks of 64 elements the first pass leaves each chunk's two stopper ballots
// in lane `chunk` and the second pass reads them back with v_readlane instead of reloading
// and re-testing the elements.)
template <class LS, class RS>
__device__ Stoppers wave_partition(CvKey* a, int lo, int hi, uint32_t* Lpos, uint32_t* Rpos,
                                   LS ls, RS rs) {
  const int lane = threadIdx.x & 63;
  const uint64_t lt = (1ull << lane) - 1, le = lt | (1ull << lane);
  const int nch = (hi - lo + 63) >> 6;
  const bool cached = nch <= 64;
  uint64_t myL = 0, myR = 0;
  int rtot = 0;
  for (int c = 0; c < nch; c++) {
    const int p = lo + 64 * c + lane;
    bool lf = false, rf = false;
    if (p < hi) {
      const CvKey e = a[p];
      lf = ls(e);
      rf = rs(e);
    }
    const uint64_t lb = __ballot(lf), rb = __ballot(rf);
    rtot += __popcll(rb);
    if (lane == c) myL = lb, myR = rb;
  }
  int lcnt = 0, rcnt = 0, K = 0, cutL = INT_MAX, cutR = hi;
  for (int c = 0; c < nch; c++) {
    const int p0 = lo + 64 * c, p = p0 + lane;
    uint64_t lb, rb;
    if (cached) {
      lb = readlane64(myL, c);
      rb = readlane64(myR, c);
    } else {
      bool lf = false, rf = false;
      if (p < hi) {
        const CvKey e = a[p];
        lf = ls(e);
        rf = rs(e);
      }
      lb = __ballot(lf);
      rb = __ballot(rf);
    }
    const bool lf = (lb >> lane) & 1, rf = (rb >> lane) & 1;
    const int lrank = lcnt + __popcll(lb & lt);
    const int rrank = rtot - (rcnt + __popcll(rb & le));
    const bool lsw = lf && rrank > lrank;
    const bool rsw = rf && lrank > rrank;
    if (lsw) Lpos[lrank] = p;
    if (rsw) Rpos[rrank] = p;
    K += __popcll(__ballot(lsw));
    const uint64_t un = __ballot(lf && !lsw);
    if (cutL == INT_MAX && un) cutL = p0 + __ffsll((unsigned long long)un) - 1;
    const uint64_t rm = __ballot(rsw);
    if (rm) cutR = min(cutR, p0 + __ffsll((unsigned long long)rm) - 1);
    lcnt += __popcll(lb);
    rcnt += __popcll(rb);
  }
  __syncthreads();
  for (int k = lane; k < K; k += 64) kswap(a, Lpos[k], Rpos[k]);
  __syncthreads();
  return {K, cutL, cutR, rtot};
}

__device__ __forceinline__ bool kgreater(const CvKey& x, const CvKey& y) { return x.r > y.r; }

// libstdc++ (GCC 4.8) __move_median_first, __adjust_heap / __heap_select, __insertion_sort with
// comp = KeypointResponseGreater: sequential, lane 0 only (3 elements; the depth-exhausted
// fallback; <= 3 elements).
__device__ void move_median_first(CvKey* a, int x, int y, int z) {
  if (kgreater(a[x], a[y])) {
    if (kgreater(a[y], a[z]))
      kswap(a, x, y);
    else if (kgreater(a[x], a[z]))
      kswap(a, x, z);
  } else if (kgreater(a[x], a[z])) {
    return;
  } else if (kgreater(a[y], a[z])) {
    kswap(a, x, z);
  } else {
    kswap(a, x, y);
  }
}

__device__ void adjust_heap(CvKey* first, long hole, long len, CvKey value) {
  const long top = hole;
  long second = hole;
  while (second < (len - 1) / 2) {
    second = 2 * (second + 1);
    if (kgreater(first[second], first[second - 1])) second--;
    first[hole] = first[second];
    hole = second;
  }
  if ((len & 1) == 0 && second == (len - 2) / 2) {
    second = 2 * (second + 1);
    first[hole] = first[second - 1];
    hole = second - 1;
  }
  long parent = (hole - 1) / 2;
  while (hole > top && kgreater(first[parent], value)) {
    first[hole] = first[parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  first[hole] = value;
}

__device__ void heap_select(CvKey* first, long middle, long last) {
  const long len = middle;
  if (len >= 2) {
    for (long parent = (len - 2) / 2;; parent--) {
      adjust_heap(first, parent, len, first[parent]);
      if (parent == 0) break;
    }
  }
  for (long i = middle; i < last; ++i)
    if (kgreater(first[i], first[0])) {
      const CvKey value = first[i];
      first[i] = first[0];
      adjust_heap(first, 0, len, value);
    }
}

__device__ void insertion_sort(CvKey* a, int first, int last) {
  if (first == last) return;
  for (int i = first + 1; i != last; ++i) {
    const CvKey val = a[i];
    if (kgreater(val, a[first])) {
      for (int k = i; k > first; k--) a[k] = a[k - 1];
      a[first] = val;
    } else {
      int l = i, next = i - 1;
      while (kgreater(val, a[next])) {
        a[l] = a[next];
        l = next;
        --next;
      }
      a[l] = val;
    }
  }
}

// std::nth_element(a + first, a + nth, a + last, greater) as GCC 4.8 implements it
// (__introselect with __unguarded_partition_pivot).
__device__ void wave_nth_element(CvKey* a, int first, int nth, int last, uint32_t* Lpos,
                                 uint32_t* Rpos) {
  const int lane = threadIdx.x & 63;
  if (first == last || nth == last) return;
  int depth = 2 * (31 - __clz(last - first));
  while (last - first > 3) {
    if (depth == 0) {
      if (lane == 0) {
        heap_select(a + first, nth + 1 - first, last - first);
        kswap(a, first, nth);
      }
      __syncthreads();
      return;
    }
    --depth;
    if (lane == 0) move_median_first(a, first, first + (last - first) / 2, last - 1);
    __syncthreads();
    const float piv = a[first].r;
    const Stoppers s = wave_partition(
        a, first + 1, last, Lpos, Rpos, [piv](const CvKey& e) { return !(e.r > piv); },
        [piv](const CvKey& e) { return !(piv > e.r); });
    const int cut = min(s.cutL, s.cutR);
    if (cut <= nth)
      first = cut;
    else
      last = cut;
  }
  if (lane == 0) insertion_sort(a, first, last);
  __syncthreads();
}

// KeyPointsFilter::retainBest (OpenCV 2.4 keypoint.cpp); returns the new size.
__device__ int wave_retain_best(CvKey* a, int n, int n_points, uint32_t* Lpos, uint32_t* Rpos) {
  if (n_points <= 0 || n <= n_points) return n;
  wave_nth_element(a, 0, n_points, n, Lpos, Rpos);
  const float amb = a[n_points - 1].r;
  const Stoppers s = wave_partition(
      a, n_points, n, Lpos, Rpos, [amb](const CvKey& e) { return !(e.r >= amb); },
      [amb](const CvKey& e) { return e.r >= amb; });
  return n_points + s.rtot;
}

// HarrisResponses(img, pts, 7, 0.04) for an integral keypoint (orb.cpp): the 9 x 9 window
// (x-4 .. x+4, y-4 .. y+4) is loaded as 9 rows of three aligned dwords (the pitched level rows
// are padded, so x+8 < pitch) and funnel-shifted to start at x-4; the sums are exact integers.
__device__ float harris_response(const uint8_t* img, int step, int x, int y) {
  float scale = (float)((1 << 2) * 7) * 255.0f;
  scale = 1.0f / scale;
  const float scale_sq_sq = scale * scale * scale * scale;
  const int x0 = x - 4, xa = x0 & ~3, sh = x0 - xa;
  int px[9][9];
#pragma unroll
  for (int r = 0; r < 9; r++) {
    const uint32_t* rp = (const uint32_t*)(img + (int64_t)(y - 4 + r) * step + xa);
    const uint32_t w0 = rp[0], w1 = rp[1], w2 = rp[2];
    const uint32_t d0 = __builtin_amdgcn_alignbyte(w1, w0, sh);
    const uint32_t d1 = __builtin_amdgcn_alignbyte(w2, w1, sh);
    const uint32_t d2 = w2 >> (8 * sh);
#pragma unroll
    for (int c = 0; c < 4; c++) {
      px[r][c] = (d0 >> (8 * c)) & 255;
      px[r][c + 4] = (d1 >> (8 * c)) & 255;
    }
    px[r][8] = d2 & 255;
  }
  int a = 0, b = 0, c = 0;
#pragma unroll
  for (int i = 1; i <= 7; i++)
#pragma unroll
    for (int j = 1; j <= 7; j++) {
      const int Ix = (px[i][j + 1] - px[i][j - 1]) * 2 + (px[i - 1][j + 1] - px[i - 1][j - 1]) +
                     (px[i + 1][j + 1] - px[i + 1][j - 1]);
      const int Iy = (px[i + 1][j] - px[i - 1][j]) * 2 + (px[i + 1][j - 1] - px[i - 1][j - 1]) +
                     (px[i + 1][j + 1] - px[i - 1][j + 1]);
      a += Ix * Ix;
      b += Iy * Iy;
      c += Ix * Iy;
    }
  const float fa = (float)a, fb = (float)b, fc = (float)c;
  const float t0 = fa * fb;
  const float t1 = fc * fc;
  const float s = fa + fb;
  const float t2 = kHarrisK * s * s;
  return (t0 - t1 - t2) * scale_sq_sq;
}

// ------------------------------------------------------------------ k_cvselect
// One wave per (image, level): computeKeyPoints after FAST (orb.cpp): the raster-order
// keypoint list, retainBest(2N) + HarrisResponses for HARRIS_SCORE, retainBest(N); the
// survivors (in their retained order) go to the level's keypoint slots, the count to ocount
// (a count above kp_cap is reported and the describe stage flags the image).
__global__ __launch_bounds__(64) void k_cvselect(
    const uint8_t* __restrict__ pyr, int64_t pyr_bytes, const CvLevel* __restrict__ lv,
    int nlevels, const uint64_t* __restrict__ bitmaps, int64_t bm_words,
    const uint8_t* __restrict__ smap, CvKey* __restrict__ gcand, uint32_t* __restrict__ gpos,
    int cand_total, int harris, CvKey* __restrict__ okey, int kp_total, int* __restrict__ ocount) {
  extern __shared__ __align__(16) char s_sel[];
  const int level = blockIdx.x, img = blockIdx.y;
  const int lane = threadIdx.x;
  const CvLevel L = lv[level];
  int* oc = ocount + img * nlevels + level;
  if (L.rx1 <= L.rx0 || L.ry1 <= L.ry0) {
    if (lane == 0) *oc = 0;
    return;
  }
  // lane = region row: its keep words (nw <= 64, in registers 8 at a time), survivor count
  const uint64_t* bm = bitmaps + (int64_t)img * bm_words + L.bm_off;
  const int w0 = L.rx0 >> 6, nw = ((L.rx1 - 1) >> 6) - w0 + 1, nr = L.ry1 - L.ry0;
  auto row_words = [&](int r, int k0, uint64_t (&wv)[8]) {
    const uint64_t* rp = bm + (int64_t)(L.ry0 + r) * L.bm_wpr + w0;
#pragma unroll
    for (int k = 0; k < 8; k++) wv[k] = (r < nr && k0 + k < nw) ? rp[k0 + k] : 0ull;
  };
  // raster order = row order (prefix over the rows' counts), then ascending x within a row;
  // keys go to LDS while they fit (the usual case), else the pass is repeated into the
  // level's global scratch
  auto emit = [&](CvKey* dst, int cap) {
    int base = 0;
    for (int r0 = 0; r0 < nr; r0 += 64) {
      const int r = r0 + lane;
      int c = 0;
      for (int k0 = 0; k0 < nw; k0 += 8) {
        uint64_t wv[8];
        row_words(r, k0, wv);
#pragma unroll
        for (int k = 0; k < 8; k++) c += __popcll(wv[k]);
      }
      const int incl = wave_incl_scan(c);
      int pos = base + incl - c;
      const uint32_t yk = (uint32_t)(L.ry0 + r) << 16;
      if (base + __shfl(incl, 63) <= cap) {  // wave-uniform
        for (int k0 = 0; k0 < nw; k0 += 8) {
          uint64_t wv[8];
          row_words(r, k0, wv);
#pragma unroll
          for (int k = 0; k < 8; k++) {
            uint64_t word = wv[k];
            const int xb = 64 * (w0 + k0 + k);
            while (word) {
              const int bit = __ffsll((unsigned long long)word) - 1;
              word &= word - 1;
              dst[pos++].k = yk | (uint32_t)(xb + bit);
            }
          }
        }
      }
      base += __shfl(incl, 63);
    }
    return base;
  };
  CvKey* a = (CvKey*)s_sel;
  uint32_t* Lpos = (uint32_t*)(s_sel + 8 * kSelCap);
  uint32_t* Rpos = Lpos + kSelCap / 2;
  int n = emit(a, kSelCap);
  if (n > kSelCap) {
    a = gcand + (int64_t)img * cand_total + L.cand_off;
    Lpos = gpos + (int64_t)img * cand_total + L.cand_off;
    Rpos = Lpos + (L.cand_cap + 1) / 2;
    emit(a, INT_MAX);
  }
  __syncthreads();
  const uint8_t* sm = smap + (int64_t)img * pyr_bytes + L.pyr_off;
  for (int i0 = 0; i0 < n; i0 += 256) {  // four loads in flight per lane
    uint32_t key[4];
    int sc[4];
#pragma unroll
    for (int u = 0; u < 4; u++) key[u] = i0 + 64 * u + lane < n ? a[i0 + 64 * u + lane].k : 0u;
#pragma unroll
    for (int u = 0; u < 4; u++)
      sc[u] = i0 + 64 * u + lane < n ? sm[(int64_t)(key[u] >> 16) * L.pitch + (key[u] & 0xFFFF)] : 0;
#pragma unroll
    for (int u = 0; u < 4; u++)
      if (i0 + 64 * u + lane < n) a[i0 + 64 * u + lane].r = (float)sc[u];
  }
  __syncthreads();
  const int feats = L.feats;
  if (harris) {
    n = wave_retain_best(a, n, 2 * feats, Lpos, Rpos);
    const uint8_t* img0 = pyr + (int64_t)img * pyr_bytes + L.pyr_off;
    for (int i = lane; i < n; i += 64) {
      const uint32_t key = a[i].k;
      a[i].r = harris_response(img0, L.pitch, (int)(key & 0xFFFF), (int)(key >> 16));
    }
    __syncthreads();
  }
  n = wave_retain_best(a, n, feats, Lpos, Rpos);
  CvKey* out = okey + (int64_t)img * kp_total + L.kp_off;
  const int m = min(n, L.kp_cap);
  for (int i = lane; i < m; i += 64) out[i] = a[i];
  if (lane == 0) *oc = n;
}

// computeOrbDescriptor's rotation: angle *= (float)(CV_PI/180.f); a = (float)cos(angle),
// b = (float)sin(angle) through the double ::cos / ::sin (OCML f64 here, glibc in the
// reference; tests/test_cvorb_gpu.py compares every float angle in [0, 360] with the host libm).
__device__ __forceinline__ void cv_cos_sin(float angle_deg, float* a, float* b) {
  float ang = angle_deg;
  ang *= (float)(3.14159265358979323846 / 180.f);
  *a = (float)cos((double)ang);
  *b = (float)sin((double)ang);
}

// ------------------------------------------------------------------ k_cvdescribe
// One half-wave per keypoint slot, 8 per workgroup: computeOrientation (IC_Angle on the
// unblurred level, cvRound(pt) centre = the integral keypoint), then computeOrbDescriptor on
// the blurred level: a = (float)cos(angle), b = (float)sin(angle) in double, sample
// (cvRound(x*b + y*a), cvRound(x*a - y*b)) without contraction, bit = I0 < I1; lane j makes
// byte j.  Then operator()'s `keypoint->pt *= scale` for levels != firstLevel.  Output is
// level-major (descriptors.rowRange(offset, offset + nkeypoints) per level).
struct KpOff {
  int off[kMaxLevels + 1];
};

__global__ __launch_bounds__(256) void k_cvdescribe(
    const uint8_t* __restrict__ pyr, int64_t pyr_bytes, const uint8_t* __restrict__ blur,
    const CvLevel* __restrict__ lv, int nlevels, KpOff ko, const CvKey* __restrict__ okey,
    const int* __restrict__ ocount, int kp_total, orbx_keypoint* __restrict__ kps,
    uint8_t* __restrict__ desc, int* __restrict__ counts) {
  constexpr int RW = 10, BW = 11;  // dwords per staged row (31+3 / 37+3 bytes, rounded up)
  constexpr int RN = 31 * RW, BN = 37 * BW;
  __shared__ uint32_t s_raw[8][RN];
  __shared__ uint32_t s_blr[8][BN];
  int bx, img;
  xcd_block(bx, img);
  const int lane = threadIdx.x & 63, hl = lane & 31;
  const int hw = threadIdx.x >> 5;
  const int slot = bx * 8 + hw;
  const int* oc = ocount + img * nlevels;
  if (bx == 0 && threadIdx.x == 0) {
    int t = 0;
    bool over = false;
    for (int l = 0; l < nlevels; l++) {
      t += oc[l];
      over |= oc[l] > lv[l].kp_cap;
    }
    counts[img] = over ? -t : t;
  }
  int level = 0;
#pragma unroll
  for (int l = 1; l < kMaxLevels; l++) level += (l < nlevels && slot >= ko.off[l]);
  const CvLevel& G = lv[level];
  const int idx = slot - ko.off[level];
  int noc = min(oc[level], G.kp_cap);
  const CvKey kk = okey[(int64_t)img * kp_total + min(slot, kp_total - 1)];
  uint32_t key = kk.k;
  float resp = kk.r;
  int pitch = G.pitch, pyr_off = G.pyr_off;
  float lscale = G.scale, lsize = G.size;
  asm volatile("" : "+v"(noc), "+v"(key), "+v"(pitch), "+v"(pyr_off), "+v"(lscale), "+v"(lsize));
  const bool active = slot < kp_total && idx < noc;  // uniform within the half-wave
  if (!active) key = 0;
  const int cx = active ? (int)(key & 0xFFFF) : 0;
  const int cy = active ? (int)(key >> 16) : 0;
  const uint8_t* Lb = pyr + (int64_t)img * pyr_bytes + pyr_off;
  const uint8_t* Bp = blur + (int64_t)img * pyr_bytes + pyr_off;
  const int fr = (cx - 15) >> 2, lr = (cx + 15) >> 2;
  const int fb = (cx - 18) >> 2, lb = (cx + 18) >> 2;
  if (active) {
    uint32_t vr[(RN + 31) / 32], vb[(BN + 31) / 32];
#pragma unroll
    for (int k = 0; k < (RN + 31) / 32; k++) {
      const int i = hl + 32 * k, r = i / RW, c = i - r * RW;
      vr[k] = (i < RN && fr + c <= lr)
                  ? *(const uint32_t*)(Lb + (uint32_t)((cy - 15 + r) * pitch + 4 * (fr + c)))
                  : 0u;
    }
#pragma unroll
    for (int k = 0; k < (BN + 31) / 32; k++) {
      const int i = hl + 32 * k, r = i / BW, c = i - r * BW;
      vb[k] = (i < BN && fb + c <= lb)
                  ? *(const uint32_t*)(Bp + (uint32_t)((cy - 18 + r) * pitch + 4 * (fb + c)))
                  : 0u;
    }
#pragma unroll
    for (int k = 0; k < (RN + 31) / 32; k++)
      if (hl + 32 * k < RN) s_raw[hw][hl + 32 * k] = vr[k];
#pragma unroll
    for (int k = 0; k < (BN + 31) / 32; k++)
      if (hl + 32 * k < BN) s_blr[hw][hl + 32 * k] = vb[k];
  }
  constexpr int BS = 4 * BW;
  const uint8_t* bc = (const uint8_t*)s_blr[hw] + 18 * BS + (cx - 4 * fb);
  int m10 = 0, m01 = 0;
  if (active && hl < 31)  // row v = hl - 15 of the circular patch
    ic_row_moments(s_raw[hw] + hl * RW, (cx - 15) - 4 * fr, c_cv_icmask.m[hl], hl - 15, m10, m01);
  // sums within the half-wave: 16-lane rows on DPP, then the two rows of the half
  m10 = row16_sum(m10);
  m01 = row16_sum(m01);
  m10 += __shfl_xor(m10, 16);
  m01 += __shfl_xor(m01, 16);
  if (!active) return;
  const float angle = orbx_fast_atan2((float)m01, (float)m10);
  float ca, sb;
  cv_cos_sin(angle, &ca, &sb);
  const uint8_t* bcb = bc - sample_bias(BS);
  const float nsb = -sb;
  uint32_t byte = 0;
#pragma unroll
  for (int m = 0; m < 8; m++) {
    const int8_t* p8 = c_cv_pattern + (hl * 8 + m) * 4;  // (x0, y0, x1, y1) of pair 8 hl + m
    const float4 pp = make_float4((float)p8[0], (float)p8[1], (float)p8[2], (float)p8[3]);
    const int t0 = bcb[sample_offset(rotate_plain(pp.x, pp.y, ca, sb, nsb), BS)];
    const int t1 = bcb[sample_offset(rotate_plain(pp.z, pp.w, ca, sb, nsb), BS)];
    byte |= (uint32_t)(t0 < t1) << m;
  }
  int outpos = idx;
  for (int l = 0; l < level; l++) outpos += oc[l];
  if (outpos >= kp_total) return;  // an overflowed image (count reported negative)
  const int64_t o = (int64_t)img * kp_total + outpos;
  desc[o * 32 + hl] = (uint8_t)byte;
  if (hl == 0) {
    orbx_keypoint k;
    k.x = level ? (float)cx * lscale : (float)cx;
    k.y = level ? (float)cy * lscale : (float)cy;
    k.size = lsize;
    k.angle = angle;
    k.response = resp;
    k.octave = level;
    k.class_id = -1;
    kps[o] = k;
  }
}

// ------------------------------------------------------------------ matchers
__device__ __forceinline__ int hamming8(const uint32_t* q, uint4 t0, uint4 t1) {
  int d = __popc(q[0] ^ t0.x);
  d += __popc(q[1] ^ t0.y);
  d += __popc(q[2] ^ t0.z);
  d += __popc(q[3] ^ t0.w);
  d += __popc(q[4] ^ t1.x);
  d += __popc(q[5] ^ t1.y);
  d += __popc(q[6] ^ t1.z);
  d += __popc(q[7] ^ t1.w);
  return d;
}

constexpr int kBfQ = 128;     // queries per workgroup (one per thread)
constexpr int kBfChunk = 256;  // train rows staged in LDS per step

// For every query row the nearest train row (strict `<`: the first minimum) and, for mode 1,
// the second-nearest distance with naive_nn_search2's update rule, plus the extremes over all
// pairs.  Train set t of problem p = train + p * train_stride rows, count from tcount[p] (a
// negative count is treated as empty).  Out: best index (-1 if empty), best and second
// distance per query.
__global__ __launch_bounds__(kBfQ) void k_bfmatch(const uint8_t* __restrict__ query, int nq,
                                                  const uint8_t* __restrict__ train,
                                                  int64_t train_stride, const int* __restrict__ tcount,
                                                  int2* __restrict__ best, int* __restrict__ second,
                                                  int* __restrict__ extremes) {
  __shared__ uint4 s_t[kBfChunk][2];
  const int p = blockIdx.y;
  const int qi = blockIdx.x * kBfQ + threadIdx.x;
  const int nt = max(tcount[p], 0);
  const uint8_t* T = train + (int64_t)p * train_stride * 32;
  uint32_t q[8];
  if (qi < nq) {
    const uint4* qp = (const uint4*)(query + (int64_t)qi * 32);
    const uint4 a = qp[0], b = qp[1];
    q[0] = a.x, q[1] = a.y, q[2] = a.z, q[3] = a.w, q[4] = b.x, q[5] = b.y, q[6] = b.z, q[7] = b.w;
  } else {
    for (int i = 0; i < 8; i++) q[i] = 0;
  }
  int bd = INT_MAX, sd = INT_MAX, bi = -1, mn = INT_MAX, mx = 0;
  for (int j0 = 0; j0 < nt; j0 += kBfChunk) {
    const int nc = min(kBfChunk, nt - j0);
    __syncthreads();
    for (int i = threadIdx.x; i < 2 * nc; i += kBfQ)
      s_t[i >> 1][i & 1] = ((const uint4*)(T + (int64_t)j0 * 32))[i];
    __syncthreads();
    if (qi < nq) {
      for (int j = 0; j < nc; j++) {
        const int d = hamming8(q, s_t[j][0], s_t[j][1]);
        if (d < bd) {
          sd = bd;
          bd = d;
          bi = j0 + j;
        } else if (d < sd) {
          sd = d;
        }
        mn = min(mn, d);
        mx = max(mx, d);
      }
    }
  }
  if (qi < nq) {
    best[(int64_t)p * nq + qi] = make_int2(bi, bd);
    if (second) second[(int64_t)p * nq + qi] = sd;
  }
  if (extremes) {
    for (int o = 32; o > 0; o >>= 1) {
      mn = min(mn, __shfl_xor(mn, o));
      mx = max(mx, __shfl_xor(mx, o));
    }
    if ((threadIdx.x & 63) == 0 && nt > 0) {
      atomicMin(extremes + 2 * p, mn);
      atomicMax(extremes + 2 * p + 1, mx);
    }
  }
}

// Marker::Match after matcher.match(target, frame): DMatch list (queryIdx = target row), then
// max_dist over the matches and the good flags `distance < 0.5 * max_dist` (Marker.cc:115-133).
// One wave per frame.  A frame without keypoints gets train -1 and no good match (Marker::Match
// returns false before matching).
__global__ __launch_bounds__(64) void k_good(const int2* __restrict__ best, int nq,
                                             const int* __restrict__ tcount,
                                             orbx_dmatch* __restrict__ matches,
                                             uint8_t* __restrict__ good, int* __restrict__ good_count) {
  const int p = blockIdx.x, lane = threadIdx.x;
  const bool empty = tcount[p] <= 0 || nq <= 0;
  int mx = 0;
  for (int i = lane; i < nq; i += 64) mx = max(mx, best[(int64_t)p * nq + i].y);
  for (int o = 32; o > 0; o >>= 1) mx = max(mx, __shfl_xor(mx, o));
  int cnt = 0;
  for (int i = lane; i < nq; i += 64) {
    const int2 b = best[(int64_t)p * nq + i];
    orbx_dmatch m;
    m.query_idx = i;
    m.train_idx = empty ? -1 : b.x;
    m.img_idx = 0;
    m.distance = empty ? 0.f : (float)b.y;
    matches[(int64_t)p * nq + i] = m;
    // (double)d < 0.5 * (double)max_dist with integral distances
    const bool g = !empty && 2 * b.y < mx;
    good[(int64_t)p * nq + i] = g;
    cnt += g;
  }
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
  if (lane == 0) good_count[p] = cnt;
}

// ------------------------------------------------------------------ test hooks
__global__ void k_debug_cossin(const float* __restrict__ deg, int64_t n, float* __restrict__ c,
                               float* __restrict__ sn) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    cv_cos_sin(deg[i], c + i, sn + i);
}

// KeyPointsFilter::retainBest on one array, through LDS (n <= kSelCap) or global memory.
__global__ __launch_bounds__(64) void k_debug_retain(CvKey* __restrict__ a, int n, int n_points,
                                                     uint32_t* __restrict__ gpos, int use_lds,
                                                     int* __restrict__ n_out) {
  extern __shared__ __align__(16) char s_sel[];
  CvKey* w = a;
  uint32_t *Lpos = gpos, *Rpos = gpos + (n + 1) / 2;
  if (use_lds) {
    w = (CvKey*)s_sel;
    Lpos = (uint32_t*)(s_sel + 8 * kSelCap);
    Rpos = Lpos + kSelCap / 2;
    for (int i = threadIdx.x; i < n; i += 64) w[i] = a[i];
    __syncthreads();
  }
  const int m = wave_retain_best(w, n, n_points, Lpos, Rpos);
  if (use_lds)
    for (int i = threadIdx.x; i < m; i += 64) a[i] = w[i];
  if (threadIdx.x == 0) *n_out = m;
}

// ------------------------------------------------------------------ plan
static inline int cv_round(double v) { return (int)nearbyint(v); }

bool params_supported(const orbx_cvorb_params& p) {
  return p.nlevels >= 1 && p.nlevels <= kMaxLevels && p.first_level == 0 && p.wta_k == 2 &&
         p.patch_size == 31 && p.edge_threshold >= 18 && p.scale_factor > 0 &&
         p.nfeatures >= 0 && (p.score_type == ORBX_HARRIS_SCORE || p.score_type == ORBX_FAST_SCORE);
}

struct Plan {
  orbx_cvorb_params p{};
  int w = 0, h = 0, max_batch = 0, device = 0;
  bool exact = false;  // keypoint capacity = every possible survivor (drop-in)
  hipStream_t stream = nullptr;
  Geometry g;
  PyrDev pd;
  CvLevel lv[kMaxLevels];
  CvLevel* d_lv = nullptr;
  CvTile* d_tiles = nullptr;
  int ntiles = 0;
  int64_t bm_words = 0;
  int cand_total = 0, kp_total = 0;
  uint8_t *d_pyr = nullptr, *d_blur = nullptr, *d_smap = nullptr;
  uint64_t* d_bm = nullptr;
  CvKey *d_cand = nullptr, *d_okey = nullptr;
  uint32_t* d_pos = nullptr;
  int *d_ocount = nullptr, *d_counts = nullptr;
  orbx_keypoint* d_kps = nullptr;
  uint8_t* d_desc = nullptr;
  GraphCache graphs;
  Profiler* prof = nullptr;  // owned by the caller
};

template <class T>
int dalloc(T** p, size_t count) {
  if (count == 0) count = 1;
  if (hipMalloc((void**)p, count * sizeof(T)) != hipSuccess) return ORBX_ENOMEM;
  return ORBX_OK;
}

void plan_destroy(Plan* P) {
  if (!P) return;
  P->graphs.clear(P->stream);
  pyr_dev_destroy(&P->pd);
  void* bufs[] = {P->d_lv, P->d_tiles, P->d_pyr, P->d_blur, P->d_smap, P->d_bm, P->d_cand,
                  P->d_okey, P->d_pos, P->d_ocount, P->d_counts, P->d_kps, P->d_desc};
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  if (P->stream) (void)hipStreamDestroy(P->stream);
  delete P;
}

// Level sizes, per-level feature counts and scales of cv::ORB::operator() (orb.cpp):
// getScale = (float)pow(scaleFactor, level) with the member `double scaleFactor`,
// sz = (cvRound(cols * (1/scale)), ...), nfeaturesPerLevel by the float geometric series.
void levels(const orbx_cvorb_params& p, int cols, int rows, int* lw, int* lh, float* sc,
            int* feats) {
  const double sf = (double)p.scale_factor;
  for (int l = 0; l < p.nlevels; l++) {
    const float s = (float)pow(sf, (double)(l - p.first_level));
    const float inv = 1 / s;
    sc[l] = s;
    lw[l] = cv_round(cols * inv);
    lh[l] = cv_round(rows * inv);
  }
  const float factor = (float)(1.0 / sf);
  float nd = p.nfeatures * (1 - factor) / (1 - (float)pow((double)factor, (double)p.nlevels));
  int sum = 0;
  for (int l = 0; l < p.nlevels - 1; l++) {
    feats[l] = cv_round(nd);
    sum += feats[l];
    nd *= factor;
  }
  feats[p.nlevels - 1] = std::max(p.nfeatures - sum, 0);
}

int plan_create(const orbx_cvorb_params& p, int w, int h, int max_batch, int device, bool exact,
                Plan** out) {
  *out = nullptr;
  if (w <= 0 || h <= 0 || max_batch <= 0) return ORBX_EINVAL;
  if (!params_supported(p)) return ORBX_EUNSUPPORTED;
  Plan* P = new (std::nothrow) Plan();
  if (!P) return ORBX_ENOMEM;
  P->p = p;
  P->w = w;
  P->h = h;
  P->max_batch = max_batch;
  P->device = device;
  P->exact = exact;
  auto fail = [&](int code) {
    plan_destroy(P);
    return code;
  };
  int lw[kMaxLevels], lh[kMaxLevels], feats[kMaxLevels];
  float sc[kMaxLevels];
  levels(p, w, h, lw, lh, sc, feats);
  Geometry& g = P->g;
  g.nlevels = p.nlevels;
  g.w = w;
  g.h = h;
  for (int l = 0; l < p.nlevels; l++) {
    g.lv[l] = LevelGeom{};
    g.lv[l].w = lw[l];
    g.lv[l].h = lh[l];
    if (lw[l] >= 4096 * 16 || lh[l] >= 65536) return fail(ORBX_EUNSUPPORTED);
  }
  std::string why;
  int rc = build_pyramid(&g, &why);
  if (rc != ORBX_OK) {
    fprintf(stderr, "[orbx] cv::ORB plan %dx%d unsupported: %s\n", w, h, why.c_str());
    return fail(rc);
  }
  const int b = p.edge_threshold;
  std::vector<CvTile> tiles;
  int64_t bm = 0;
  int cand = 0, kp = 0;
  for (int l = 0; l < p.nlevels; l++) {
    CvLevel& L = P->lv[l];
    const LevelGeom& G = g.lv[l];
    L = CvLevel{};
    L.w = G.w;
    L.h = G.h;
    L.pitch = G.pitch;
    L.pyr_off = (int)G.pyr_off;
    // runByImageBorder: an image no larger than 2 * edge keeps nothing
    const bool has = G.h > 2 * b && G.w > 2 * b;
    L.rx0 = b;
    L.ry0 = b;
    L.rx1 = has ? G.w - b : b;
    L.ry1 = has ? G.h - b : b;
    L.bm_wpr = L.pitch / 64;
    L.bm_off = (int)bm;
    bm += (int64_t)L.bm_wpr * L.h;
    L.feats = feats[l];
    const int rw = L.rx1 - L.rx0, rh = L.ry1 - L.ry0;
    const int maxsurv = has ? ((rw + 1) / 2) * ((rh + 1) / 2) : 0;
    L.cand_off = cand;
    L.cand_cap = maxsurv;
    cand += maxsurv;
    L.kp_off = kp;
    L.kp_cap = exact ? maxsurv : std::min(maxsurv, std::max(2 * feats[l], feats[l] + 64));
    kp += L.kp_cap;
    L.scale = sc[l];
    L.size = p.patch_size * sc[l];
    if (has)
      for (int ty = 0; ty * kTH < rh; ty++)
        for (int tx = L.rx0 / kTW; tx <= (L.rx1 - 1) / kTW; tx++)
          tiles.push_back({(int16_t)l, (int16_t)tx, (int16_t)ty, 0});
  }
  if (bm >= INT_MAX || g.pyr_bytes >= INT_MAX) return fail(ORBX_EUNSUPPORTED);
  P->bm_words = std::max<int64_t>(bm, 1);
  P->cand_total = std::max(cand, 1);
  P->kp_total = std::max(kp, 1);
  P->ntiles = (int)tiles.size();
  if (hipSetDevice(device) != hipSuccess) return fail(ORBX_EDEVICE);
  if (hipStreamCreateWithFlags(&P->stream, hipStreamNonBlocking) != hipSuccess)
    return fail(ORBX_EDEVICE);
  {
    orbx_params op{p.nfeatures, p.scale_factor, p.nlevels, 20, 7};
    Geometry t;
    build_tables(op, &t);  // umax for halfPatchSize 15 (orb.cpp computes it the same way)
    IcMask icm;
    build_ic_mask(t.umax, &icm);
    if (hipMemcpyToSymbol(HIP_SYMBOL(c_cv_icmask), &icm, sizeof(icm)) != hipSuccess ||
        hipMemcpyToSymbol(HIP_SYMBOL(c_cv_pattern), ORBX_PATTERN, sizeof(ORBX_PATTERN)) != hipSuccess)
      return fail(ORBX_EDEVICE);
  }
  rc = pyr_dev_create(g, &P->pd);
  if (rc != ORBX_OK) return fail(rc);
  const size_t B = (size_t)max_batch;
  if (dalloc(&P->d_lv, p.nlevels) || dalloc(&P->d_tiles, tiles.size()) ||
      dalloc(&P->d_pyr, B * g.pyr_bytes) || dalloc(&P->d_blur, B * g.pyr_bytes) ||
      dalloc(&P->d_smap, B * g.pyr_bytes) || dalloc(&P->d_bm, B * P->bm_words) ||
      dalloc(&P->d_cand, B * P->cand_total) || dalloc(&P->d_pos, B * P->cand_total + 2) ||
      dalloc(&P->d_okey, B * P->kp_total) || dalloc(&P->d_ocount, B * p.nlevels) ||
      dalloc(&P->d_counts, B) || dalloc(&P->d_kps, B * P->kp_total) ||
      dalloc(&P->d_desc, B * P->kp_total * 32))
    return fail(ORBX_ENOMEM);
  if (hipMemcpy(P->d_lv, P->lv, sizeof(CvLevel) * p.nlevels, hipMemcpyHostToDevice) ||
      (tiles.size() && hipMemcpy(P->d_tiles, tiles.data(), sizeof(CvTile) * tiles.size(),
                                 hipMemcpyHostToDevice)) ||
      hipMemset(P->d_counts, 0, 4 * B))
    return fail(ORBX_EDEVICE);
  const int smem = 8 * kSelCap + 4 * kSelCap;
  if (hipFuncSetAttribute((const void*)k_cvselect, hipFuncAttributeMaxDynamicSharedMemorySize,
                          smem) != hipSuccess)
    return fail(ORBX_EDEVICE);
  *out = P;
  return ORBX_OK;
}

int enqueue(Plan* P, const uint8_t* d_in, int n) {
  const Geometry& g = P->g;
  const int L = P->p.nlevels;
  Profiler dummy;
  Profiler& pr = P->prof ? *P->prof : dummy;
  const int st_pyr = pr.stage("k_pyramid"), st_fast = pr.stage("k_cvfast"),
            st_sel = pr.stage("k_cvselect"), st_blur = pr.stage("k_blur"),
            st_desc = pr.stage("k_cvdescribe");
  hipStream_t s = P->stream;
  ProfScope scope(pr);
  pr.mark(s, -1);
  int rc = launch_pyramid(g, P->pd, d_in, P->d_pyr, P->d_blur, n, s, &pr, st_pyr);
  if (rc) return rc;
  if (P->ntiles > 0) note_kernel("k_cvfast");
  if (P->ntiles > 0)
    hipLaunchKernelGGL(k_cvfast, dim3(P->ntiles, n), dim3(256), 0, s, P->d_pyr, g.pyr_bytes,
                       P->d_lv, P->d_tiles, P->d_bm, P->bm_words, P->d_smap);
  pr.mark(s, st_fast);
  note_kernel("k_cvselect");
  hipLaunchKernelGGL(k_cvselect, dim3(L, n), dim3(64), 12 * kSelCap, s, P->d_pyr, g.pyr_bytes,
                     P->d_lv, L, P->d_bm, P->bm_words, P->d_smap, P->d_cand, P->d_pos,
                     P->cand_total, (int)(P->p.score_type == ORBX_HARRIS_SCORE), P->d_okey,
                     P->kp_total, P->d_ocount);
  pr.mark(s, st_sel);
  rc = launch_blur(g, P->pd, P->d_pyr, P->d_blur, n, s);  // (no-op with the blur fused)
  if (rc) return rc;
  if (!g.blur_fused) pr.mark(s, st_blur);
  KpOff ko{};
  for (int l = 0; l < L; l++) ko.off[l] = P->lv[l].kp_off;
  ko.off[L] = P->kp_total;
  note_kernel("k_cvdescribe");
  hipLaunchKernelGGL(k_cvdescribe, dim3((P->kp_total + 7) / 8, n), dim3(256), 0, s, P->d_pyr,
                     g.pyr_bytes, P->d_blur, P->d_lv, L, ko, P->d_okey, P->d_ocount, P->kp_total,
                     P->d_kps, P->d_desc, P->d_counts);
  pr.mark(s, st_desc);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? ORBX_OK : report_hip(e, "cvorb launch");
}

// Runs a batch: captured into a hipGraph per (input pointer, batch) unless profiling.
int plan_run(Plan* P, const uint8_t* d_in, int n) {
  if (!P || !d_in || n <= 0 || n > P->max_batch) return ORBX_EINVAL;
  ORBX_HIP(hipSetDevice(P->device));
  if (P->prof && P->prof->on) return enqueue(P, d_in, n);
  return run_graph(P->graphs, P->stream, d_in, n, [&] {
    Profiler* keep = P->prof;
    P->prof = nullptr;
    const int rc = enqueue(P, d_in, n);
    P->prof = keep;
    return rc;
  });
}

int launch_bf(const uint8_t* d_query, int nq, const uint8_t* d_train, int64_t train_stride,
              const int* d_tcount, int nprob, int2* d_best, int* d_second, int* d_extremes,
              hipStream_t s) {
  if (nq <= 0 || nprob <= 0) return ORBX_OK;
  note_kernel("k_bfmatch");
  hipLaunchKernelGGL(k_bfmatch, dim3((nq + kBfQ - 1) / kBfQ, nprob), dim3(kBfQ), 0, s, d_query,
                     nq, d_train, train_stride, d_tcount, d_best, d_second, d_extremes);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? ORBX_OK : report_hip(e, "k_bfmatch");
}

int profile_read(Profiler& pr, int32_t cap, char (*names)[32], double* total_ms,
                 int64_t* launches, int32_t* n_stages) {
  if (pr.collect() != 0) return ORBX_EDEVICE;
  const int n = (int)pr.names.size();
  if (n_stages) *n_stages = n;
  for (int i = 0; i < n && i < cap; i++) {
    if (names) {
      strncpy(names[i], pr.names[i].c_str(), 31);
      names[i][31] = 0;
    }
    if (total_ms) total_ms[i] = pr.ms[i];
    if (launches) launches[i] = pr.launches[i];
  }
  return ORBX_OK;
}

}  // namespace cvorb
}  // namespace orbx

using namespace orbx;
using namespace orbx::cvorb;

struct orbx_cvorb {
  orbx_cvorb_params params{};
  int device = 0;
  Plan* tp = nullptr;  // throughput plan (w, h, max_batch)
  Plan* dp = nullptr;  // drop-in plan: batch 1, exact capacity, rebuilt on a size change
  uint8_t* d_img = nullptr;
  Profiler prof;
};

struct orbx_marker {
  Plan* plan = nullptr;
  int device = 0;
  uint8_t* d_target = nullptr;
  int n_target = 0;
  int2* d_best = nullptr;
  orbx_dmatch* d_matches = nullptr;
  uint8_t* d_good = nullptr;
  int* d_good_count = nullptr;
  int match_cap = 0;  // n_target capacity of the match buffers
  Profiler prof;
};

namespace {

int marker_enqueue(orbx_marker* M, int n) {
  Plan* P = M->plan;
  Profiler dummy;
  Profiler& pr = P->prof ? *P->prof : dummy;
  const int st_bf = pr.stage("k_bfmatch"), st_good = pr.stage("k_good");
  ProfScope scope(pr);
  hipStream_t s = P->stream;
  int rc = launch_bf(M->d_target, M->n_target, (const uint8_t*)P->d_desc, P->kp_total,
                     P->d_counts, n, M->d_best, nullptr, nullptr, s);
  if (rc) return rc;
  pr.mark(s, st_bf);
  note_kernel("k_good");
  hipLaunchKernelGGL(k_good, dim3(n), dim3(64), 0, s, M->d_best, M->n_target, P->d_counts,
                     M->d_matches, M->d_good, M->d_good_count);
  pr.mark(s, st_good);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? ORBX_OK : report_hip(e, "k_good");
}

}  // namespace

extern "C" {

int orbx_cvorb_create(const orbx_cvorb_params* params, int32_t w, int32_t h, int32_t max_batch,
                      int hip_device, orbx_cvorb** out) {
  ORBX_RESOURCE_LOCK;
  if (!params || !out || w <= 0 || h <= 0 || max_batch <= 0) return ORBX_EINVAL;
  *out = nullptr;
  if (!params_supported(*params)) return ORBX_EUNSUPPORTED;
  orbx_cvorb* o = new (std::nothrow) orbx_cvorb();
  if (!o) return ORBX_ENOMEM;
  o->params = *params;
  o->device = hip_device;
  int rc = plan_create(*params, w, h, max_batch, hip_device, false, &o->tp);
  if (rc != ORBX_OK) {
    delete o;
    return rc;
  }
  o->tp->prof = &o->prof;
  *out = o;
  return ORBX_OK;
}

int orbx_cvorb_destroy(orbx_cvorb* o) {
  ORBX_RESOURCE_LOCK;
  if (!o) return ORBX_OK;
  plan_destroy(o->tp);
  plan_destroy(o->dp);
  if (o->d_img) (void)hipFree(o->d_img);
  delete o;
  return ORBX_OK;
}

int orbx_cvorb_capacity(const orbx_cvorb* o, int32_t* kp_cap) {
  if (!o || !kp_cap) return ORBX_EINVAL;
  *kp_cap = o->tp->kp_total;
  return ORBX_OK;
}

int orbx_cvorb_detect(orbx_cvorb* o, const uint8_t* img, int32_t w, int32_t h, int64_t stride,
                      orbx_keypoint* kps, uint8_t* desc, int32_t cap, int32_t* n_out) {
  if (!o || !n_out) return ORBX_EINVAL;
  if (w <= 0 || h <= 0) {  // orb.cpp: `if (_image.empty()) return;`
    *n_out = -1;
    return ORBX_OK;
  }
  if (!img || stride < w || cap < 0 || (cap > 0 && (!kps || !desc))) return ORBX_EINVAL;
  ORBX_HIP(hipSetDevice(o->device));
  if (!o->dp || o->dp->w != w || o->dp->h != h) {
    plan_destroy(o->dp);
    o->dp = nullptr;
    if (o->d_img) (void)hipFree(o->d_img);
    o->d_img = nullptr;
    int rc = plan_create(o->params, w, h, 1, o->device, true, &o->dp);
    if (rc != ORBX_OK) return rc;
    ORBX_HIP(hipMalloc(&o->d_img, (size_t)w * h));
  }
  Plan* P = o->dp;
  hipStream_t s = P->stream;
  ORBX_HIP(hipMemcpy2DAsync(o->d_img, w, img, stride, w, h, hipMemcpyHostToDevice, s));
  int rc = plan_run(P, o->d_img, 1);
  if (rc != ORBX_OK) return rc;
  int32_t n = 0;
  ORBX_HIP(hipMemcpyAsync(&n, P->d_counts, 4, hipMemcpyDeviceToHost, s));
  ORBX_HIP(orbx::wait_stream(s));
  if (n < 0) return ORBX_ECAPACITY;  // cannot happen with exact capacity
  *n_out = n;
  if (n > cap) return ORBX_ECAPACITY;
  if (n > 0) {
    ORBX_HIP(hipMemcpyAsync(kps, P->d_kps, sizeof(orbx_keypoint) * n, hipMemcpyDeviceToHost, s));
    ORBX_HIP(hipMemcpyAsync(desc, P->d_desc, (size_t)32 * n, hipMemcpyDeviceToHost, s));
    ORBX_HIP(orbx::wait_stream(s));
  }
  return ORBX_OK;
}

int orbx_cvorb_run(orbx_cvorb* o, const uint8_t* d_imgs, int32_t n) {
  if (!o) return ORBX_EINVAL;
  return plan_run(o->tp, d_imgs, n);
}

int orbx_cvorb_outputs(orbx_cvorb* o, orbx_keypoint** d_kps, uint8_t** d_desc,
                       int32_t** d_counts) {
  if (!o) return ORBX_EINVAL;
  if (d_kps) *d_kps = o->tp->d_kps;
  if (d_desc) *d_desc = o->tp->d_desc;
  if (d_counts) *d_counts = o->tp->d_counts;
  return ORBX_OK;
}

int orbx_cvorb_sync(orbx_cvorb* o) {
  if (!o) return ORBX_EINVAL;
  ORBX_HIP(orbx::wait_stream(o->tp->stream));
  return ORBX_OK;
}

void* orbx_cvorb_stream(orbx_cvorb* o) { return o ? (void*)o->tp->stream : nullptr; }

int orbx_bf_match(const uint8_t* query, int32_t nq, const uint8_t* train, int32_t nt,
                  orbx_dmatch* out, int32_t* n_out) {
  if (!n_out || nq < 0 || nt < 0) return ORBX_EINVAL;
  *n_out = 0;
  if (nq == 0 || nt == 0) return ORBX_OK;  // knnMatch returns early on an empty side
  if (!query || !train || !out) return ORBX_EINVAL;
  Stager st;
  const size_t oq = st.add(query, (size_t)nq * 32), ot = st.add(train, (size_t)nt * 32);
  const size_t oc = st.add(&nt, 4), ob = st.add(nullptr, (size_t)nq * 8);
  int rc = tls_ws.reserve(st.host.size());
  if (rc) return rc;
  char* base = tls_ws.d;
  hipStream_t s = tls_ws.stream;
  ORBX_HIP(host_copy(base, st.host.data(), ob, st.host.pinned, hipMemcpyHostToDevice, s));
  rc = launch_bf(dptr<uint8_t>(base, oq), nq, dptr<uint8_t>(base, ot), 0, dptr<int>(base, oc), 1,
                 dptr<int2>(base, ob), nullptr, nullptr, s);
  if (rc) return rc;
  std::vector<int2> best(nq);
  ORBX_HIP(hipMemcpyAsync(best.data(), base + ob, (size_t)nq * 8, hipMemcpyDeviceToHost, s));
  ORBX_HIP(orbx::wait_stream(s));
  for (int i = 0; i < nq; i++) out[i] = {i, best[i].x, 0, (float)best[i].y};
  *n_out = nq;
  return ORBX_OK;
}

int orbx_good_matches(const orbx_dmatch* m, int32_t n, orbx_dmatch* good, int32_t* n_good,
                      double* min_dist, double* max_dist) {
  if (n < 0 || !n_good || (n > 0 && (!m || !good))) return ORBX_EINVAL;
  double mx = 0, mn = 100;  // Marker.cc:115-120
  for (int i = 0; i < n; i++) {
    const double d = m[i].distance;
    if (d < mn) mn = d;
    if (d > mx) mx = d;
  }
  int k = 0;
  for (int i = 0; i < n; i++)
    if (m[i].distance < 0.5 * mx) good[k++] = m[i];
  *n_good = k;
  if (min_dist) *min_dist = mn;
  if (max_dist) *max_dist = mx;
  return ORBX_OK;
}

int orbx_nn_match(const uint8_t* query, int32_t nq, const uint8_t* train, int32_t nt,
                  double ratio, int32_t max_dist, orbx_dmatch* out, int32_t* n_out,
                  int32_t* min_d, int32_t* max_d) {
  if (!n_out || nq < 0 || nt < 0) return ORBX_EINVAL;
  *n_out = 0;
  if (min_d) *min_d = 100;  // the reference's globals start at minD = 100, maxD = 0
  if (max_d) *max_d = 0;
  if (nq == 0) return ORBX_OK;
  if (!query || !out || (nt > 0 && !train)) return ORBX_EINVAL;
  std::vector<int2> best(nq);
  std::vector<int> second(nq);
  int ext[2] = {INT_MAX, 0};
  if (nt > 0) {
    Stager st;
    const size_t oq = st.add(query, (size_t)nq * 32), ot = st.add(train, (size_t)nt * 32);
    const size_t oc = st.add(&nt, 4), oe = st.add(ext, 8);
    const size_t ob = st.add(nullptr, (size_t)nq * 8), os = st.add(nullptr, (size_t)nq * 4);
    int rc = tls_ws.reserve(st.host.size());
    if (rc) return rc;
    char* base = tls_ws.d;
    hipStream_t s = tls_ws.stream;
    ORBX_HIP(host_copy(base, st.host.data(), ob, st.host.pinned, hipMemcpyHostToDevice, s));
    rc = launch_bf(dptr<uint8_t>(base, oq), nq, dptr<uint8_t>(base, ot), 0, dptr<int>(base, oc),
                   1, dptr<int2>(base, ob), dptr<int>(base, os), dptr<int>(base, oe), s);
    if (rc) return rc;
    ORBX_HIP(hipMemcpyAsync(best.data(), base + ob, (size_t)nq * 8, hipMemcpyDeviceToHost, s));
    ORBX_HIP(hipMemcpyAsync(second.data(), base + os, (size_t)nq * 4, hipMemcpyDeviceToHost, s));
    ORBX_HIP(hipMemcpyAsync(ext, base + oe, 8, hipMemcpyDeviceToHost, s));
    ORBX_HIP(orbx::wait_stream(s));
  } else {
    for (int i = 0; i < nq; i++) best[i] = make_int2(-1, INT_MAX), second[i] = INT_MAX;
  }
  // AR-1.3/src/ORBMatcher.cpp:96-101 (unsigned arithmetic as the reference)
  int k = 0;
  for (int i = 0; i < nq; i++) {
    const unsigned int mind = (unsigned)best[i].y, secd = (unsigned)second[i];
    const bool ratio_ok = ratio <= 0 || mind <= (unsigned int)(secd * ratio);
    if (ratio_ok && mind <= (unsigned)max_dist) out[k++] = {i, best[i].x, 0, (float)mind};
  }
  *n_out = k;
  if (nt > 0) {
    if (min_d) *min_d = std::min(100, ext[0]);
    if (max_d) *max_d = ext[1];
  }
  return ORBX_OK;
}

int orbx_debug_cvorb_cossin(const float* deg, int64_t n, float* c, float* s) {
  if (n < 0 || (n > 0 && (!deg || !c || !s))) return ORBX_EINVAL;
  if (n == 0) return ORBX_OK;
  float *d_in = nullptr, *d_c = nullptr, *d_s = nullptr;
  ORBX_HIP(hipMalloc(&d_in, 4 * (size_t)n));
  hipError_t e = hipMalloc(&d_c, 4 * (size_t)n);
  if (e == hipSuccess) e = hipMalloc(&d_s, 4 * (size_t)n);
  if (e == hipSuccess) e = hipMemcpy(d_in, deg, 4 * (size_t)n, hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_debug_cossin, dim3(2048), dim3(256), 0, 0, d_in, n, d_c, d_s);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpy(c, d_c, 4 * (size_t)n, hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(s, d_s, 4 * (size_t)n, hipMemcpyDeviceToHost);
  (void)hipFree(d_in);
  if (d_c) (void)hipFree(d_c);
  if (d_s) (void)hipFree(d_s);
  return e == hipSuccess ? ORBX_OK : report_hip(e, "orbx_debug_cvorb_cossin");
}

int orbx_debug_retain_best(float* resp, uint32_t* ids, int32_t n, int32_t n_points,
                           int32_t force_global, int32_t* n_out) {
  if (n < 0 || !n_out || (n > 0 && (!resp || !ids))) return ORBX_EINVAL;
  std::vector<CvKey> v(std::max(n, 1));
  for (int i = 0; i < n; i++) v[i] = {resp[i], ids[i]};
  CvKey* d_a = nullptr;
  uint32_t* d_pos = nullptr;
  int* d_n = nullptr;
  ORBX_HIP(hipMalloc(&d_a, sizeof(CvKey) * v.size()));
  hipError_t e = hipMalloc(&d_pos, 4 * (v.size() + 2));
  if (e == hipSuccess) e = hipMalloc(&d_n, 4);
  if (e == hipSuccess) e = hipMemcpy(d_a, v.data(), sizeof(CvKey) * v.size(), hipMemcpyHostToDevice);
  const int use_lds = !force_global && n <= kSelCap;
  if (e == hipSuccess)
    e = hipFuncSetAttribute((const void*)k_debug_retain,
                            hipFuncAttributeMaxDynamicSharedMemorySize, 12 * kSelCap);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_debug_retain, dim3(1), dim3(64), 12 * kSelCap, 0, d_a, n, n_points,
                       d_pos, use_lds, d_n);
    e = hipGetLastError();
  }
  int m = 0;
  if (e == hipSuccess) e = hipMemcpy(&m, d_n, 4, hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(v.data(), d_a, sizeof(CvKey) * v.size(), hipMemcpyDeviceToHost);
  (void)hipFree(d_a);
  if (d_pos) (void)hipFree(d_pos);
  if (d_n) (void)hipFree(d_n);
  if (e != hipSuccess) return report_hip(e, "orbx_debug_retain_best");
  for (int i = 0; i < m; i++) resp[i] = v[i].r, ids[i] = v[i].k;
  *n_out = m;
  return ORBX_OK;
}

int orbx_marker_create(const orbx_cvorb_params* params, int32_t w, int32_t h, int32_t max_batch,
                       int hip_device, orbx_marker** out) {
  ORBX_RESOURCE_LOCK;
  if (!params || !out || w <= 0 || h <= 0 || max_batch <= 0) return ORBX_EINVAL;
  *out = nullptr;
  orbx_marker* M = new (std::nothrow) orbx_marker();
  if (!M) return ORBX_ENOMEM;
  M->device = hip_device;
  int rc = plan_create(*params, w, h, max_batch, hip_device, false, &M->plan);
  if (rc != ORBX_OK) {
    delete M;
    return rc;
  }
  M->plan->prof = &M->prof;
  if (hipMalloc(&M->d_good_count, 4 * (size_t)max_batch) != hipSuccess) {
    orbx_marker_destroy(M);
    return ORBX_ENOMEM;
  }
  *out = M;
  return ORBX_OK;
}

int orbx_marker_destroy(orbx_marker* M) {
  ORBX_RESOURCE_LOCK;
  if (!M) return ORBX_OK;
  plan_destroy(M->plan);
  void* bufs[] = {M->d_target, M->d_best, M->d_matches, M->d_good, M->d_good_count};
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  delete M;
  return ORBX_OK;
}

// Marker::setTargetImage's descriptors (mDescriptors1), n x 32 host bytes.
int orbx_marker_set_target(orbx_marker* M, const uint8_t* desc, int32_t n) {
  if (!M || n < 0 || (n > 0 && !desc)) return ORBX_EINVAL;
  ORBX_HIP(hipSetDevice(M->device));
  ORBX_HIP(orbx::wait_stream(M->plan->stream));
  if (n > M->match_cap) {
    void* bufs[] = {M->d_target, M->d_best, M->d_matches, M->d_good};
    for (void* b : bufs)
      if (b) (void)hipFree(b);
    M->d_target = nullptr;
    M->d_best = nullptr;
    M->d_matches = nullptr;
    M->d_good = nullptr;
    M->match_cap = 0;
    const size_t B = (size_t)M->plan->max_batch;
    if (hipMalloc(&M->d_target, (size_t)n * 32) != hipSuccess ||
        hipMalloc(&M->d_best, B * n * sizeof(int2)) != hipSuccess ||
        hipMalloc(&M->d_matches, B * n * sizeof(orbx_dmatch)) != hipSuccess ||
        hipMalloc(&M->d_good, B * n) != hipSuccess)
      return ORBX_ENOMEM;
    M->match_cap = n;
  }
  if (n > 0) ORBX_HIP(hipMemcpy(M->d_target, desc, (size_t)n * 32, hipMemcpyHostToDevice));
  M->n_target = n;
  return ORBX_OK;
}

int orbx_marker_run(orbx_marker* M, const uint8_t* d_imgs, int32_t n) {
  if (!M) return ORBX_EINVAL;
  Plan* P = M->plan;
  if (!d_imgs || n <= 0 || n > P->max_batch) return ORBX_EINVAL;
  ORBX_HIP(hipSetDevice(M->device));
  // the extraction graph (one per input pointer and batch), then the two matcher launches
  int rc = plan_run(P, d_imgs, n);
  if (rc) return rc;
  return marker_enqueue(M, n);
}

int orbx_marker_sync(orbx_marker* M) {
  if (!M) return ORBX_EINVAL;
  ORBX_HIP(orbx::wait_stream(M->plan->stream));
  return ORBX_OK;
}

int orbx_marker_results(orbx_marker* M, int32_t n, int32_t* kp_counts, int32_t* good_counts) {
  if (!M || n < 0 || n > M->plan->max_batch) return ORBX_EINVAL;
  hipStream_t s = M->plan->stream;
  if (kp_counts)
    ORBX_HIP(hipMemcpyAsync(kp_counts, M->plan->d_counts, 4 * (size_t)n, hipMemcpyDeviceToHost, s));
  if (good_counts)
    ORBX_HIP(hipMemcpyAsync(good_counts, M->d_good_count, 4 * (size_t)n, hipMemcpyDeviceToHost, s));
  ORBX_HIP(orbx::wait_stream(s));
  return ORBX_OK;
}

int orbx_marker_outputs(orbx_marker* M, orbx_dmatch** d_matches, uint8_t** d_good,
                        orbx_keypoint** d_kps, uint8_t** d_desc) {
  if (!M) return ORBX_EINVAL;
  if (d_matches) *d_matches = M->d_matches;
  if (d_good) *d_good = M->d_good;
  if (d_kps) *d_kps = M->plan->d_kps;
  if (d_desc) *d_desc = M->plan->d_desc;
  return ORBX_OK;
}

void* orbx_marker_stream(orbx_marker* M) { return M ? (void*)M->plan->stream : nullptr; }

int orbx_marker_profile(orbx_marker* M, int32_t enable) {
  if (!M) return ORBX_EINVAL;
  M->prof.on = enable != 0;
  M->prof.reset();
  return ORBX_OK;
}

int orbx_marker_profile_read(orbx_marker* M, int32_t cap, char (*names)[32], double* total_ms,
                             int64_t* launches, int32_t* n_stages) {
  if (!M) return ORBX_EINVAL;
  return profile_read(M->prof, cap, names, total_ms, launches, n_stages);
}

int orbx_marker_profile_kernels(orbx_marker* M, int32_t stage, char* buf, int32_t cap) {
  if (!M) return ORBX_EINVAL;
  const int r = M->prof.kernels_of(stage, buf, cap);
  return r == 0 ? ORBX_OK : r > 0 ? ORBX_ECAPACITY : ORBX_EINVAL;
}

}  // extern "C"
