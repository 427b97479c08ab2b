// cvorb_oracle.cc — CPU restatement of the AR marker path (TEST INFRASTRUCTURE ONLY).
//
// Imported only by tests/ (and bench.py's cpu_baseline leg) as the checker; the product
// library never links or calls it.
//
// What it restates:
//   * cv::ORB::operator() of OpenCV 2.4 (modules/features2d/src/orb.cpp), the extractor the
//     AR marker code calls: Marker::setTargetImage / Marker::Match (ORB_SLAM2/src/Marker.cc:76-84,
//     98-108, default arguments: 500 features, 1.2, 8 levels, edgeThreshold 31, HARRIS_SCORE)
//     and AR-1.3/src/ORBMatcher.cpp:121-122 (300 features).  Steps: scale pyramid (resize
//     INTER_LINEAR from the previous level), FAST-9/16 threshold 20 with NMS on every level,
//     KeyPointsFilter::runByImageBorder(edgeThreshold), retainBest(2N), HarrisResponses
//     (block 7, k 0.04), retainBest(N), IC_Angle, GaussianBlur 7x7 sigma 2, computeOrbDescriptor
//     (WTA_K 2, 31x31 pattern), keypoints scaled to level 0.
//   * KeyPointsFilter::retainBest's std::nth_element + std::partition as libstdc++ of GCC 4.8
//     implements them (introselect with median-of-three Hoare partitions; the reference tree was
//     built with GCC 4.8.4): the order of the retained keypoints, and which of the
//     keypoints tied at the boundary survive, are those algorithms' outputs.
//   * BruteForceMatcher<HammingLUT>::match (OpenCV 2.4 BFMatcher NORM_HAMMING, k = 1), the
//     good-match filter of Marker::Match (Marker.cc:115-133), naive_nn_search /
//     naive_nn_search2 (AR-1.3/src/ORBMatcher.cpp:44-102) = Marker::searchMatches
//     (Marker.cc:314-349).
// OpenCV 2.4 and its cv::ORB are not in the reference tree nor in this image: parity against
// real OpenCV is UNPINNED.  Assumptions (first to verify if OpenCV 2.4 ever becomes available):
// computeOrbDescriptor evaluates `(float)cos(angle)` / `(float)sin(angle)` in double (the
// global ::cos overload; no -ffast-math narrowing) and its sample coordinates without FMA
// contraction (SSE2 build, no -mfma); HarrisResponses' float expression likewise.
// The FAST, resize, blur, fastAtan2 and IC_Angle primitives are the ones orb_oracle.cc
// restates for ORBextractor (same OpenCV 2.4 functions), called through its exports.
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstring>
#include <thread>
#include <vector>

#include "../include/orbx_pattern.h"
#include "orb_oracle.h"

namespace {

inline int cv_round(double v) { return (int)std::nearbyint(v); }  // cvRound, half-even

struct KPf {
  float x, y, size, angle, response;
  int octave, class_id;
};

// ---------------------------------------------------------------- libstdc++ (GCC 4.8) algorithms
// bits/stl_algo.h / bits/stl_heap.h of GCC 4.8, with `comp` = KeypointResponseGreater
// (a.response > b.response) for nth_element.
template <class T, class C>
void move_median_first(T* a, T* b, T* c, C comp) {
  if (comp(*a, *b)) {
    if (comp(*b, *c))
      std::swap(*a, *b);
    else if (comp(*a, *c))
      std::swap(*a, *c);
  } else if (comp(*a, *c)) {
    return;
  } else if (comp(*b, *c)) {
    std::swap(*a, *c);
  } else {
    std::swap(*a, *b);
  }
}

template <class T, class C>
T* unguarded_partition(T* first, T* last, const T& pivot, C comp) {
  while (true) {
    while (comp(*first, pivot)) ++first;
    --last;
    while (comp(pivot, *last)) --last;
    if (!(first < last)) return first;
    std::swap(*first, *last);
    ++first;
  }
}

template <class T, class C>
T* unguarded_partition_pivot(T* first, T* last, C comp) {
  T* mid = first + (last - first) / 2;
  move_median_first(first, mid, last - 1, comp);
  return unguarded_partition(first + 1, last, *first, comp);
}

template <class T, class C>
void push_heap_(T* first, long hole, long top, T value, C comp) {
  long parent = (hole - 1) / 2;
  while (hole > top && comp(first[parent], value)) {
    first[hole] = first[parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  first[hole] = value;
}

template <class T, class C>
void adjust_heap(T* first, long hole, long len, T value, C comp) {
  const long top = hole;
  long second = hole;
  while (second < (len - 1) / 2) {
    second = 2 * (second + 1);
    if (comp(first[second], first[second - 1])) second--;
    first[hole] = first[second];
    hole = second;
  }
  if ((len & 1) == 0 && second == (len - 2) / 2) {
    second = 2 * (second + 1);
    first[hole] = first[second - 1];
    hole = second - 1;
  }
  push_heap_(first, hole, top, value, comp);
}

template <class T, class C>
void make_heap_(T* first, T* last, C comp) {
  const long len = last - first;
  if (len < 2) return;
  long parent = (len - 2) / 2;
  while (true) {
    T value = first[parent];
    adjust_heap(first, parent, len, value, comp);
    if (parent == 0) return;
    parent--;
  }
}

template <class T, class C>
void heap_select(T* first, T* middle, T* last, C comp) {
  make_heap_(first, middle, comp);
  for (T* i = middle; i < last; ++i)
    if (comp(*i, *first)) {  // __pop_heap(first, middle, i)
      T value = *i;
      *i = *first;
      adjust_heap(first, 0L, (long)(middle - first), value, comp);
    }
}

template <class T, class C>
void insertion_sort(T* first, T* last, C comp) {
  if (first == last) return;
  for (T* i = first + 1; i != last; ++i) {
    if (comp(*i, *first)) {
      T val = *i;
      std::move_backward(first, i, i + 1);
      *first = val;
    } else {  // __unguarded_linear_insert
      T val = *i;
      T* l = i;
      T* next = i - 1;
      while (comp(val, *next)) {
        *l = *next;
        l = next;
        --next;
      }
      *l = val;
    }
  }
}

inline long lg(long n) { return (long)(sizeof(long) * 8 - 1) - __builtin_clzl((unsigned long)n); }

template <class T, class C>
void nth_element_48(T* first, T* nth, T* last, C comp) {
  if (first == last || nth == last) return;
  long depth = lg(last - first) * 2;
  while (last - first > 3) {
    if (depth == 0) {
      heap_select(first, nth + 1, last, comp);
      std::swap(*first, *nth);
      return;
    }
    --depth;
    T* cut = unguarded_partition_pivot(first, last, comp);
    if (cut <= nth)
      first = cut;
    else
      last = cut;
  }
  insertion_sort(first, last, comp);
}

// std::partition for bidirectional iterators (GCC 4.8 __partition, bidirectional_iterator_tag)
template <class T, class P>
T* partition_48(T* first, T* last, P pred) {
  while (true) {
    while (true)
      if (first == last)
        return first;
      else if (pred(*first))
        ++first;
      else
        break;
    --last;
    while (true)
      if (first == last)
        return first;
      else if (!pred(*last))
        --last;
      else
        break;
    std::swap(*first, *last);
    ++first;
  }
}

// KeyPointsFilter::retainBest (OpenCV 2.4 keypoint.cpp)
template <class T>
void retain_best(std::vector<T>& kps, int n_points) {
  if (n_points > 0 && kps.size() > (size_t)n_points) {
    auto greater = [](const T& a, const T& b) { return a.response > b.response; };
    nth_element_48(kps.data(), kps.data() + n_points, kps.data() + kps.size(), greater);
    const float amb = kps[n_points - 1].response;
    T* new_end = partition_48(kps.data() + n_points, kps.data() + kps.size(),
                              [amb](const T& k) { return k.response >= amb; });
    kps.resize(new_end - kps.data());
  }
}

// ---------------------------------------------------------------- orb.cpp (OpenCV 2.4)
const float HARRIS_K = 0.04f;

// HarrisResponses(img, pts, blockSize, harris_k)
float harris_response(const uint8_t* img, int64_t step, float px, float py, int block,
                      float k) {
  const int r = block / 2;
  float scale = (1 << 2) * block * 255.0f;
  scale = 1.0f / scale;
  const float scale_sq_sq = scale * scale * scale * scale;
  const int x0 = cv_round(px - r), y0 = cv_round(py - r);
  const uint8_t* ptr0 = img + (int64_t)y0 * step + x0;
  int a = 0, b = 0, c = 0;
  for (int i = 0; i < block; i++)
    for (int j = 0; j < block; j++) {
      const uint8_t* p = ptr0 + (int64_t)i * step + j;
      const int Ix = (p[1] - p[-1]) * 2 + (p[-step + 1] - p[-step - 1]) + (p[step + 1] - p[step - 1]);
      const int Iy = (p[step] - p[-step]) * 2 + (p[step - 1] - p[-step - 1]) + (p[step + 1] - p[-step + 1]);
      a += Ix * Ix;
      b += Iy * Iy;
      c += Ix * Iy;
    }
  return ((float)a * b - (float)c * c - k * ((float)a + b) * ((float)a + b)) * scale_sq_sq;
}

// computeOrbDescriptor (WTA_K == 2)
void cvorb_descriptor(const uint8_t* img, int64_t step, int cx, int cy, float kp_angle,
                      uint8_t* desc) {
  float angle = kp_angle;
  angle *= (float)(M_PI / 180.f);
  const float a = (float)cos((double)angle), b = (float)sin((double)angle);
  const uint8_t* center = img + (int64_t)cy * step + cx;
  auto value = [&](int idx) {
    const int px = ORBX_PATTERN[2 * idx], py = ORBX_PATTERN[2 * idx + 1];
    const float x = px * a - py * b;
    const float y = px * b + py * a;
    const int ix = cv_round(x), iy = cv_round(y);
    return (int)center[(int64_t)iy * step + ix];
  };
  for (int i = 0; i < 32; ++i) {
    int val = 0;
    for (int k = 0; k < 8; k++) val |= (value(16 * i + 2 * k) < value(16 * i + 2 * k + 1)) << k;
    desc[i] = (uint8_t)val;
  }
}

struct Levels {
  int n = 0;
  std::vector<int> w, h, feats;
  std::vector<float> scale;  // getScale(level, 0, scaleFactor)
};

// getScale / the pyramid sizes of operator() / nfeaturesPerLevel of computeKeyPoints
Levels cvorb_levels(const orbx_cvorb_params& p, int cols, int rows) {
  Levels L;
  L.n = p.nlevels;
  const double sf = (double)p.scale_factor;  // member `double scaleFactor`
  for (int l = 0; l < p.nlevels; l++) {
    const float s = (float)std::pow(sf, (double)(l - p.first_level));
    const float inv = 1 / s;
    L.scale.push_back(s);
    L.w.push_back(cv_round(cols * inv));
    L.h.push_back(cv_round(rows * inv));
  }
  const float factor = (float)(1.0 / sf);
  float nd = p.nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)p.nlevels));
  int sum = 0;
  L.feats.assign(p.nlevels, 0);
  for (int l = 0; l < p.nlevels - 1; l++) {
    L.feats[l] = cv_round(nd);
    sum += L.feats[l];
    nd *= factor;
  }
  L.feats[p.nlevels - 1] = std::max(p.nfeatures - sum, 0);
  return L;
}

bool supported(const orbx_cvorb_params& p) {
  return p.nlevels >= 1 && p.nlevels <= 16 && p.first_level == 0 && p.wta_k == 2 &&
         p.patch_size == 31 && p.edge_threshold >= 18 && p.scale_factor > 0 &&
         p.nfeatures >= 0 && (p.score_type == ORBX_HARRIS_SCORE || p.score_type == ORBX_FAST_SCORE);
}

}  // namespace

extern "C" {

int oracle_cvorb_levels(const orbx_cvorb_params* p, int w, int h, int* lw, int* lh, float* scale,
                        int* feats) {
  if (!p || !supported(*p)) return ORBX_EUNSUPPORTED;
  Levels L = cvorb_levels(*p, w, h);
  for (int l = 0; l < L.n; l++) {
    if (lw) lw[l] = L.w[l];
    if (lh) lh[l] = L.h[l];
    if (scale) scale[l] = L.scale[l];
    if (feats) feats[l] = L.feats[l];
  }
  return ORBX_OK;
}

// KeyPointsFilter::retainBest on (response, id) pairs; ids come back in the retained order.
void oracle_retain_best(float* resp, int32_t* ids, int n, int n_points, int* n_out) {
  struct E {
    float response;
    int32_t id;
  };
  std::vector<E> v(n);
  for (int i = 0; i < n; i++) v[i] = {resp[i], ids[i]};
  retain_best(v, n_points);
  for (size_t i = 0; i < v.size(); i++) resp[i] = v[i].response, ids[i] = v[i].id;
  *n_out = (int)v.size();
}

float oracle_harris(const uint8_t* img, int64_t stride, int x, int y) {
  return harris_response(img, stride, (float)x, (float)y, 7, HARRIS_K);
}

void oracle_cvorb_descriptor(const uint8_t* blurred, int64_t stride, int cx, int cy, float angle,
                             uint8_t* d) {
  cvorb_descriptor(blurred, stride, cx, cy, angle, d);
}

void oracle_cos_sin_f64(float deg, float* c, float* s) {
  float angle = deg * (float)(M_PI / 180.f);
  *c = (float)cos((double)angle);
  *s = (float)sin((double)angle);
}

// The same for the n consecutive float bit patterns from bits0 (host libm), on `threads` threads.
void oracle_cos_sin_f64_range(uint32_t bits0, int64_t n, float* c, float* s, int threads) {
  if (threads < 1) threads = 1;
  std::vector<std::thread> pool;
  for (int t = 0; t < threads; t++)
    pool.emplace_back([=]() {
      for (int64_t i = t; i < n; i += threads) {
        const uint32_t b = bits0 + (uint32_t)i;
        float deg;
        memcpy(&deg, &b, 4);
        oracle_cos_sin_f64(deg, c + i, s + i);
      }
    });
  for (auto& th : pool) th.join();
}

// cv::ORB::operator()(image, noArray(), keypoints, descriptors) (orb.cpp, OpenCV 2.4)
int oracle_cvorb_detect(const orbx_cvorb_params* p, const uint8_t* img, int w, int h,
                        int64_t stride, orbx_keypoint* kps_out, uint8_t* desc_out, int cap,
                        int* n_out, uint8_t* pyr_out, int64_t pyr_cap) {
  if (!p || !n_out) return ORBX_EINVAL;
  if (w <= 0 || h <= 0) {  // _image.empty(): return before touching the outputs
    *n_out = -1;
    return ORBX_OK;
  }
  if (!supported(*p)) return ORBX_EUNSUPPORTED;
  const Levels L = cvorb_levels(*p, w, h);
  const int half = p->patch_size / 2;
  // image pyramid: level 0 the input, level l resized from level l-1 (INTER_LINEAR)
  std::vector<std::vector<uint8_t>> pyr(L.n);
  for (int l = 0; l < L.n; l++) {
    pyr[l].assign((size_t)L.w[l] * L.h[l], 0);
    if (l == 0) {
      for (int y = 0; y < h; y++) memcpy(&pyr[0][(size_t)y * w], img + (int64_t)y * stride, w);
    } else if (L.w[l] > 0 && L.h[l] > 0) {
      oracle_resize_linear(pyr[l - 1].data(), L.w[l - 1], L.h[l - 1], L.w[l - 1], pyr[l].data(),
                           L.w[l], L.h[l], L.w[l]);
    }
  }
  if (pyr_out) {
    int64_t off = 0;
    for (int l = 0; l < L.n; l++) {
      const int64_t bytes = (int64_t)L.w[l] * L.h[l];
      if (off + bytes <= pyr_cap) memcpy(pyr_out + off, pyr[l].data(), bytes);
      off += bytes;
    }
  }
  // computeKeyPoints
  std::vector<std::vector<KPf>> all(L.n);
  std::vector<int> xs, ys, sc;
  for (int l = 0; l < L.n; l++) {
    const int lw = L.w[l], lh = L.h[l];
    std::vector<KPf>& k = all[l];
    if (lw >= 7 && lh >= 7) {
      const int cap_c = lw * lh;
      xs.resize(cap_c);
      ys.resize(cap_c);
      sc.resize(cap_c);
      const int nc = oracle_fast_roi(pyr[l].data(), lh, lw, lw, 20, xs.data(), ys.data(),
                                     sc.data(), cap_c);
      for (int i = 0; i < nc; i++)
        k.push_back({(float)xs[i], (float)ys[i], 7.f, -1.f, (float)sc[i], 0, -1});
    }
    // KeyPointsFilter::runByImageBorder(keypoints, size, edgeThreshold) (stable remove_if)
    const int b = p->edge_threshold;
    if (lh <= 2 * b || lw <= 2 * b) {
      k.clear();
    } else {
      std::vector<KPf> kept;
      for (const KPf& q : k)
        if (q.x >= b && q.x < lw - b && q.y >= b && q.y < lh - b) kept.push_back(q);
      k.swap(kept);
    }
    const int featuresNum = L.feats[l];
    if (p->score_type == ORBX_HARRIS_SCORE) {
      retain_best(k, 2 * featuresNum);
      for (KPf& q : k) q.response = harris_response(pyr[l].data(), lw, q.x, q.y, 7, HARRIS_K);
    }
    retain_best(k, featuresNum);
    const float sf = L.scale[l];
    for (KPf& q : k) {
      q.octave = l;
      q.size = p->patch_size * sf;
    }
    for (KPf& q : k)  // computeOrientation: IC_Angle at cvRound(pt)
      q.angle = oracle_ic_angle(pyr[l].data(), lw, cv_round(q.x), cv_round(q.y));
    (void)half;
  }
  int total = 0;
  for (int l = 0; l < L.n; l++) total += (int)all[l].size();
  *n_out = total;
  if (total > cap) return ORBX_ECAPACITY;
  int off = 0;
  std::vector<uint8_t> blurred;
  for (int l = 0; l < L.n; l++) {
    std::vector<KPf>& k = all[l];
    if (!k.empty()) {
      blurred.assign(pyr[l].size(), 0);
      oracle_gaussian7(pyr[l].data(), L.w[l], L.h[l], blurred.data());
      for (size_t i = 0; i < k.size(); i++)
        cvorb_descriptor(blurred.data(), L.w[l], cv_round(k[i].x), cv_round(k[i].y), k[i].angle,
                         desc_out + (size_t)(off + i) * 32);
    }
    if (l != p->first_level) {
      const float s = L.scale[l];
      for (KPf& q : k) q.x *= s, q.y *= s;
    }
    for (size_t i = 0; i < k.size(); i++) {
      orbx_keypoint& o = kps_out[off + i];
      o.x = k[i].x;
      o.y = k[i].y;
      o.size = k[i].size;
      o.angle = k[i].angle;
      o.response = k[i].response;
      o.octave = k[i].octave;
      o.class_id = k[i].class_id;
    }
    off += (int)k.size();
  }
  return ORBX_OK;
}

static inline int hamming32(const uint8_t* a, const uint8_t* b) {
  int d = 0;
  for (int i = 0; i < 32; i++) d += __builtin_popcount((unsigned)(a[i] ^ b[i]));
  return d;
}

// BFMatcher(NORM_HAMMING)::match via knnMatch(k = 1): batchDistance keeps the first minimum
int oracle_bf_match(const uint8_t* q, int nq, const uint8_t* t, int nt, orbx_dmatch* out,
                    int* n_out) {
  *n_out = 0;
  if (nq <= 0 || nt <= 0) return ORBX_OK;
  for (int i = 0; i < nq; i++) {
    int best = INT_MAX, bi = -1;
    for (int j = 0; j < nt; j++) {
      const int d = hamming32(q + (size_t)i * 32, t + (size_t)j * 32);
      if (d < best) best = d, bi = j;
    }
    out[i] = {i, bi, 0, (float)best};
  }
  *n_out = nq;
  return ORBX_OK;
}

// Marker::Match (Marker.cc:115-133)
int oracle_good_matches(const orbx_dmatch* m, int n, orbx_dmatch* good, int* n_good,
                        double* min_dist_out, double* max_dist_out) {
  double max_dist = 0, min_dist = 100;
  for (int i = 0; i < n; i++) {
    const double dist = m[i].distance;
    if (dist < min_dist) min_dist = dist;
    if (dist > max_dist) max_dist = dist;
  }
  int k = 0;
  for (int i = 0; i < n; i++)
    if (m[i].distance < 0.5 * max_dist) good[k++] = m[i];
  *n_good = k;
  if (min_dist_out) *min_dist_out = min_dist;
  if (max_dist_out) *max_dist_out = max_dist;
  return ORBX_OK;
}

// naive_nn_search2 (ratio > 0) / naive_nn_search (ratio <= 0), AR-1.3/src/ORBMatcher.cpp:44-102
int oracle_nn_match(const uint8_t* q, int nq, const uint8_t* t, int nt, double ratio,
                    int max_dist, orbx_dmatch* out, int* n_out, int* min_d, int* max_d) {
  unsigned int minD = 100, maxD = 0;
  int k = 0;
  for (int i = 0; i < nq; i++) {
    unsigned int min_dist = INT_MAX, sec_dist = INT_MAX;
    int min_idx = -1;
    for (int j = 0; j < nt; j++) {
      const unsigned int dist = (unsigned)hamming32(q + (size_t)i * 32, t + (size_t)j * 32);
      if (dist < min_dist) {
        sec_dist = min_dist;
        min_dist = dist;
        min_idx = j;
      } else if (dist < sec_dist) {
        sec_dist = dist;
      }
      if (dist <= minD) minD = dist;
      if (dist > maxD) maxD = dist;
    }
    const bool ratio_ok = ratio <= 0 || min_dist <= (unsigned int)(sec_dist * ratio);
    if (ratio_ok && min_dist <= (unsigned)max_dist) out[k++] = {i, min_idx, 0, (float)min_dist};
  }
  *n_out = k;
  if (min_d) *min_d = (int)minD;
  if (max_d) *max_d = (int)maxD;
  return ORBX_OK;
}

}  // extern "C"
