// orb_oracle.cc — CPU restatement of the reference ORB front end (TEST INFRASTRUCTURE ONLY).
//
// Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the
// checker.  The product library (ar_orbslam2_amd/csrc) never links or calls this file.
//
// What it restates, with the reference file:line each function follows:
//   * ORB-SLAM2 logic: ORB_SLAM2/src/ORBextractor.cc:69-1072, ORB_SLAM2/src/ORBmatcher.cc
//     :140-288, 525-826, 1604-1666, DBoW2 TemplatedVocabulary.h:1218-1259.
//   * OpenCV 2.4 primitives (a system dependency of the reference, not vendored, absent in
//     this image — SURVEY §8c): cv::FAST (FAST_t<16> + SSE2 cornerScore<16>), cv::resize
//     INTER_LINEAR 8U (HResizeLinear + VResizeLinearVec_32s8u SSE2 vertical pass + scalar tail),
//     cv::GaussianBlur 8U fixed-point (RowFilter + SymmColumnVec_32s8u f32 column pass),
//     cv::fastAtan2, cvRound.  SURVEY Appendix A gives the semantics.
//   * glibc 2.35 sincosf (sysdeps/ieee754/flt-32/s_sincosf.c; the reference binary imports
//     sincosf for computeOrbDescriptor) — the oracle calls the host libm directly.
// Parity against real OpenCV 2.4 is UNPINNED (no OpenCV in the image, no golden vectors in
// the reference); see DESIGN.md §Parity.
//
// Build: oracle/Makefile (g++ -O3 -ffp-contract=off; explicit std::fma only where the
// reference binary fuses).
#include "orb_oracle.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <list>
#include <thread>
#include <utility>
#include <vector>

#include "../include/orbx_pattern.h"

namespace {

const int PATCH_SIZE = 31;
const int HALF_PATCH_SIZE = 15;
const int EDGE_THRESHOLD = 19;

inline int cv_round(double v) { return (int)std::nearbyint(v); }  // cvtsd2si, half-even
inline int cv_floor(double v) { return (int)std::floor(v); }
inline int cv_ceil(double v) { return (int)std::ceil(v); }

struct Img {
  int w = 0, h = 0;
  std::vector<uint8_t> px;
  uint8_t* row(int y) { return px.data() + (size_t)y * w; }
  const uint8_t* row(int y) const { return px.data() + (size_t)y * w; }
};

// ---------------------------------------------------------------- cv::resize (A.3)
void resize_linear(const uint8_t* src, int sw, int sh, int64_t sstride, uint8_t* dst, int dw,
                   int dh, int64_t dstride) {
  const double inv_sx = (double)dw / sw, inv_sy = (double)dh / sh;
  const double sx = 1. / inv_sx, sy = 1. / inv_sy;
  const int ONE = 2048;
  std::vector<int> xofs(dw), yofs(dh);
  std::vector<short> ia(2 * dw), ib(2 * dh);
  int xmax = dw;
  for (int dx = 0; dx < dw; dx++) {
    float fx = (float)((dx + 0.5) * sx - 0.5);
    int x0 = cv_floor(fx);
    fx -= x0;
    if (x0 < 0) fx = 0, x0 = 0;
    if (x0 + 1 >= sw) {
      xmax = std::min(xmax, dx);
      if (x0 >= sw - 1) fx = 0, x0 = sw - 1;
    }
    xofs[dx] = x0;
    float c0 = 1.f - fx, c1 = fx;
    ia[2 * dx] = (short)std::min(32767, std::max(-32768, cv_round(c0 * ONE)));
    ia[2 * dx + 1] = (short)std::min(32767, std::max(-32768, cv_round(c1 * ONE)));
  }
  for (int dy = 0; dy < dh; dy++) {
    float fy = (float)((dy + 0.5) * sy - 0.5);
    int y0 = cv_floor(fy);
    fy -= y0;
    yofs[dy] = y0;
    float c0 = 1.f - fy, c1 = fy;
    ib[2 * dy] = (short)std::min(32767, std::max(-32768, cv_round(c0 * ONE)));
    ib[2 * dy + 1] = (short)std::min(32767, std::max(-32768, cv_round(c1 * ONE)));
  }
  auto clip = [](int v, int a, int b) { return v >= a ? (v < b ? v : b - 1) : a; };
  auto hrow = [&](int y, int* out) {
    const uint8_t* S = src + (int64_t)y * sstride;
    int dx = 0;
    for (; dx < xmax; dx++) out[dx] = S[xofs[dx]] * ia[2 * dx] + S[xofs[dx] + 1] * ia[2 * dx + 1];
    for (; dx < dw; dx++) out[dx] = S[xofs[dx]] * ONE;
  };
  // SSE2 region of VResizeLinearVec_32s8u: 16-wide loop while x <= W-16, then 4-wide while
  // x < W-4 (strict); the rest is the scalar FixedPtCast<int,uchar,22> tail.
  int xs = 0;
  while (xs <= dw - 16) xs += 16;
  while (xs < dw - 4) xs += 4;
  std::vector<int> H0(dw), H1(dw);
  for (int dy = 0; dy < dh; dy++) {
    int ya = clip(yofs[dy], 0, sh), yb = clip(yofs[dy] + 1, 0, sh);
    hrow(ya, H0.data());
    hrow(yb, H1.data());
    const int b0 = ib[2 * dy], b1 = ib[2 * dy + 1];
    uint8_t* D = dst + (int64_t)dy * dstride;
    for (int x = 0; x < dw; x++) {
      int v;
      if (x < xs) {
        int t0 = (int16_t)std::min(32767, std::max(-32768, H0[x] >> 4));
        int t1 = (int16_t)std::min(32767, std::max(-32768, H1[x] >> 4));
        int m = ((t0 * b0) >> 16) + ((t1 * b1) >> 16);
        m = std::min(32767, std::max(-32768, m));
        m = std::min(32767, std::max(-32768, m + 2));
        v = m >> 2;
      } else {
        v = (H0[x] * b0 + H1[x] * b1 + (1 << 21)) >> 22;
      }
      D[x] = (uint8_t)std::min(255, std::max(0, v));
    }
  }
}

// ---------------------------------------------------------------- GaussianBlur 7x7 s=2 (A.4)
int reflect101(int p, int len) {
  if (len == 1) return 0;
  while (p < 0 || p >= len) {
    if (p < 0) p = -p;
    if (p >= len) p = 2 * len - p - 2;
  }
  return p;
}

void gaussian_kernel_int(int k[7]) {
  // getGaussianKernel(7, 2, CV_32F): exp(-x^2/8) in double -> f32, normalised by the double
  // sum of the f32 values, then convertTo(CV_32S, 256) (cvRound).
  float cf[7];
  double sum = 0;
  const double scale2X = -0.5 / (2.0 * 2.0);
  for (int i = 0; i < 7; i++) {
    double x = i - 3.0;
    cf[i] = (float)std::exp(scale2X * x * x);
    sum += cf[i];
  }
  sum = 1. / sum;
  for (int i = 0; i < 7; i++) {
    cf[i] = (float)(cf[i] * sum);
    k[i] = cv_round((double)cf[i] * 256.0);
  }
}

void gaussian7(const uint8_t* src, int w, int h, uint8_t* dst) {
  int k[7];
  gaussian_kernel_int(k);
  std::vector<int> R((size_t)w * h);
  for (int y = 0; y < h; y++) {
    const uint8_t* S = src + (size_t)y * w;
    for (int x = 0; x < w; x++) {
      int s = 0;
      for (int j = 0; j < 7; j++) s += k[j] * S[reflect101(x + j - 3, w)];
      R[(size_t)y * w + x] = s;
    }
  }
  // column pass: f32 SSE region for x < 4*floor(w/4) (cvtps2dq: half-even), scalar tail
  // (m + 32768) >> 16; both saturate to u8.
  const int xs = (w / 4) * 4;
  float kf[7];
  for (int i = 0; i < 7; i++) kf[i] = (float)(k[i] * (1.0 / 65536.0));
  for (int y = 0; y < h; y++) {
    int rows[7];
    for (int i = 0; i < 7; i++) rows[i] = reflect101(y + i - 3, h);
    for (int x = 0; x < w; x++) {
      int v;
      if (x < xs) {
        float s = (float)R[(size_t)rows[3] * w + x] * kf[3];
        s = s + 0.f;
        for (int i = 1; i <= 3; i++) {
          int pair = R[(size_t)rows[3 + i] * w + x] + R[(size_t)rows[3 - i] * w + x];
          s = s + (float)pair * kf[3 + i];
        }
        v = (int)std::nearbyint(s);
      } else {
        int m = k[3] * R[(size_t)rows[3] * w + x];
        for (int i = 1; i <= 3; i++)
          m += k[3 + i] * (R[(size_t)rows[3 + i] * w + x] + R[(size_t)rows[3 - i] * w + x]);
        v = (m + 32768) >> 16;
      }
      dst[(size_t)y * w + x] = (uint8_t)std::min(255, std::max(0, v));
    }
  }
}

// ---------------------------------------------------------------- fastAtan2 (A.5)
float fast_atan2(float y, float x) {
  static const float k = (float)(180 / M_PI);
  static const float p1 = 0.9997878412794807f * k;
  static const float p3 = -0.3258083974640975f * k;
  static const float p5 = 0.1555786518463281f * k;
  static const float p7 = -0.04432655554792128f * k;
  float ax = std::fabs(x), ay = std::fabs(y);
  float a, c, c2;
  if (ax >= ay) {
    c = ay / (ax + (float)DBL_EPSILON);
    c2 = c * c;
    a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
  } else {
    c = ax / (ay + (float)DBL_EPSILON);
    c2 = c * c;
    a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
  }
  if (x < 0) a = 180.f - a;
  if (y < 0) a = 360.f - a;
  return a;
}

// ---------------------------------------------------------------- FAST-9/16 (A.2)
const int kCircle[16][2] = {{0, 3},  {1, 3},   {2, 2},   {3, 1},  {3, 0},   {3, -1},
                            {2, -2}, {1, -3},  {0, -3},  {-1, -3}, {-2, -2}, {-3, -1},
                            {-3, 0}, {-3, 1},  {-2, 2},  {-1, 3}};

int fast_score(const uint8_t* c, int64_t stride) {
  // cornerScore<16>, SSE2 form: q0 = max_k min(d_k..d_k+8), q1 = min_k max(..), indices mod 16.
  int d[25];
  const int v = c[0];
  for (int k = 0; k < 16; k++) d[k] = v - c[kCircle[k][0] + kCircle[k][1] * stride];
  for (int k = 16; k < 25; k++) d[k] = d[k - 16];
  int q0 = -1000, q1 = 1000;
  for (int k = 0; k < 16; k++) {
    int a = d[k], b = d[k];
    for (int j = 1; j <= 8; j++) a = std::min(a, d[k + j]), b = std::max(b, d[k + j]);
    q0 = std::max(q0, a);
    q1 = std::min(q1, b);
  }
  return std::max(q0, -q1) - 1;
}

bool fast_is_corner(const uint8_t* c, int64_t stride, int t) {
  // FAST_t<16> detection: 9 contiguous circle pixels (of 25 with wrap) all < v-t or all > v+t.
  const int v = c[0];
  int cd = 0, cb = 0;
  for (int k = 0; k < 25; k++) {
    const int kk = k & 15;
    const int x = c[kCircle[kk][0] + kCircle[kk][1] * stride];
    if (x < v - t) {
      if (++cd > 8) return true;
    } else {
      cd = 0;
    }
    if (x > v + t) {
      if (++cb > 8) return true;
    } else {
      cb = 0;
    }
  }
  return false;
}

struct Cand {
  int x, y, score;
};

// cv::FAST(roi, kps, t, nonmax=true) on a standalone ROI: detection rows/cols [3, n-3),
// strict 8-neighbour NMS with out-of-region / non-corner neighbours at 0, raster order.
void fast_roi(const uint8_t* roi, int rows, int cols, int64_t stride, int t,
              std::vector<Cand>& out) {
  out.clear();
  t = std::min(std::max(t, 0), 255);
  if (rows < 7 || cols < 7) return;
  std::vector<int> sc((size_t)rows * cols, 0);
  std::vector<uint8_t> corner((size_t)rows * cols, 0);
  for (int i = 3; i < rows - 3; i++)
    for (int j = 3; j < cols - 3; j++) {
      const uint8_t* c = roi + (int64_t)i * stride + j;
      if (fast_is_corner(c, stride, t)) {
        corner[(size_t)i * cols + j] = 1;
        sc[(size_t)i * cols + j] = (uint8_t)fast_score(c, stride);
      }
    }
  for (int i = 3; i < rows - 3; i++)
    for (int j = 3; j < cols - 3; j++) {
      if (!corner[(size_t)i * cols + j]) continue;
      const int s = sc[(size_t)i * cols + j];
      bool keep = true;
      for (int dy = -1; dy <= 1 && keep; dy++)
        for (int dx = -1; dx <= 1; dx++) {
          if (!dy && !dx) continue;
          if (!(s > sc[(size_t)(i + dy) * cols + j + dx])) {
            keep = false;
            break;
          }
        }
      if (keep) out.push_back({j, i, s});
    }
}

// ---------------------------------------------------------------- IC_Angle (ORBextractor.cc:73-98)
float ic_angle(const uint8_t* img, int64_t step, int cx, int cy, const int* umax) {
  int m_01 = 0, m_10 = 0;
  const uint8_t* center = img + (int64_t)cy * step + cx;
  for (int u = -HALF_PATCH_SIZE; u <= HALF_PATCH_SIZE; ++u) m_10 += u * center[u];
  for (int v = 1; v <= HALF_PATCH_SIZE; ++v) {
    int v_sum = 0;
    const int d = umax[v];
    for (int u = -d; u <= d; ++u) {
      const int vp = center[u + v * step], vm = center[u - v * step];
      v_sum += vp - vm;
      m_10 += u * (vp + vm);
    }
    m_01 += v * v_sum;
  }
  return fast_atan2((float)m_01, (float)m_10);
}

// ---------------------------------------------------------------- computeOrbDescriptor (:101-144)
void orb_descriptor(const uint8_t* img, int64_t step, int cx, int cy, float kp_angle,
                    uint8_t* desc) {
  const float factorPI = (float)(M_PI / 180.f);
  const float angle = kp_angle * factorPI;
  float b, a;  // sin, cos
  sincosf(angle, &b, &a);
  const uint8_t* center = img + (int64_t)cy * step + cx;
  for (int i = 0; i < 32; ++i) {
    int val = 0;
    for (int k = 0; k < 8; k++) {
      int t[2];
      for (int e = 0; e < 2; e++) {
        const int idx = (i * 16 + k * 2 + e) * 2;
        const float px = (float)ORBX_PATTERN[idx], py = (float)ORBX_PATTERN[idx + 1];
        // reference binary: row = cvRound(fmaf(x, sin, y*cos)), col = cvRound(fmaf(x, cos,
        // -(y*sin)))
        const int row = cv_round(std::fma(px, b, py * a));
        const int col = cv_round(std::fma(px, a, -(py * b)));
        t[e] = center[(int64_t)row * step + col];
      }
      val |= (t[0] < t[1]) << k;
    }
    desc[i] = (uint8_t)val;
  }
}

// ---------------------------------------------------------------- ExtractorNode / octree
struct KP {
  float x, y, size, angle, response;
  int octave, class_id;
};

struct Node {
  std::vector<KP> keys;
  int ULx, ULy, URx, URy, BLx, BLy, BRx, BRy;
  std::list<Node>::iterator lit;
  bool noMore = false;
  unsigned long long seq = 0;
};

// ExtractorNode::DivideNode (ORBextractor.cc:470-523)
void divide_node(const Node& p, Node& n1, Node& n2, Node& n3, Node& n4) {
  const int halfX = (int)std::ceil(static_cast<float>(p.URx - p.ULx) / 2);
  const int halfY = (int)std::ceil(static_cast<float>(p.BRy - p.ULy) / 2);
  n1.ULx = p.ULx; n1.ULy = p.ULy;
  n1.URx = p.ULx + halfX; n1.URy = p.ULy;
  n1.BLx = p.ULx; n1.BLy = p.ULy + halfY;
  n1.BRx = p.ULx + halfX; n1.BRy = p.ULy + halfY;
  n2.ULx = n1.URx; n2.ULy = n1.URy;
  n2.URx = p.URx; n2.URy = p.URy;
  n2.BLx = n1.BRx; n2.BLy = n1.BRy;
  n2.BRx = p.URx; n2.BRy = p.ULy + halfY;
  n3.ULx = n1.BLx; n3.ULy = n1.BLy;
  n3.URx = n1.BRx; n3.URy = n1.BRy;
  n3.BLx = p.BLx; n3.BLy = p.BLy;
  n3.BRx = n1.BRx; n3.BRy = p.BLy;
  n4.ULx = n3.URx; n4.ULy = n3.URy;
  n4.URx = n2.BRx; n4.URy = n2.BRy;
  n4.BLx = n3.BRx; n4.BLy = n3.BRy;
  n4.BRx = p.BRx; n4.BRy = p.BRy;
  for (const KP& kp : p.keys) {
    if (kp.x < n1.URx) {
      if (kp.y < n1.BRy) n1.keys.push_back(kp);
      else n3.keys.push_back(kp);
    } else if (kp.y < n1.BRy) {
      n2.keys.push_back(kp);
    } else {
      n4.keys.push_back(kp);
    }
  }
  if (n1.keys.size() == 1) n1.noMore = true;
  if (n2.keys.size() == 1) n2.noMore = true;
  if (n3.keys.size() == 1) n3.noMore = true;
  if (n4.keys.size() == 1) n4.noMore = true;
}

struct Rec {
  int size;
  Node* node;
};

// ORBextractor::DistributeOctTree (ORBextractor.cc:525-733), with the final-refinement sort
// key made explicit: tie_mode 0 = (size, creation sequence), 1 = (size, address).
std::vector<KP> distribute_octree(const std::vector<KP>& keys, int minX, int maxX, int minY,
                                  int maxY, int N, int tie_mode) {
  const int nIni = (int)std::round(static_cast<float>(maxX - minX) / (maxY - minY));
  const float hX = static_cast<float>(maxX - minX) / nIni;
  std::list<Node> lNodes;
  unsigned long long seq = 0;
  std::vector<Node*> ini(nIni);
  for (int i = 0; i < nIni; i++) {
    Node ni;
    ni.ULx = (int)(hX * static_cast<float>(i)); ni.ULy = 0;
    ni.URx = (int)(hX * static_cast<float>(i + 1)); ni.URy = 0;
    ni.BLx = ni.ULx; ni.BLy = maxY - minY;
    ni.BRx = ni.URx; ni.BRy = maxY - minY;
    ni.seq = seq++;
    lNodes.push_back(ni);
    ini[i] = &lNodes.back();
  }
  for (const KP& kp : keys) ini[(size_t)(kp.x / hX)]->keys.push_back(kp);
  for (auto lit = lNodes.begin(); lit != lNodes.end();) {
    if (lit->keys.size() == 1) {
      lit->noMore = true;
      ++lit;
    } else if (lit->keys.empty()) {
      lit = lNodes.erase(lit);
    } else {
      ++lit;
    }
  }
  auto less = [tie_mode](const Rec& a, const Rec& b) {
    if (a.size != b.size) return a.size < b.size;
    if (tie_mode == 0) return a.node->seq < b.node->seq;
    return a.node < b.node;
  };
  auto push_children = [&](Node& parent, std::vector<Rec>* rec, int* nToExpand) {
    Node c[4];
    divide_node(parent, c[0], c[1], c[2], c[3]);
    for (int q = 0; q < 4; q++) {
      if (c[q].keys.empty()) continue;
      c[q].seq = seq++;
      lNodes.push_front(c[q]);
      if (c[q].keys.size() > 1) {
        if (nToExpand) (*nToExpand)++;
        rec->push_back({(int)c[q].keys.size(), &lNodes.front()});
        lNodes.front().lit = lNodes.begin();
      }
    }
  };
  bool bFinish = false;
  std::vector<Rec> recs;
  while (!bFinish) {
    int prevSize = (int)lNodes.size();
    int nToExpand = 0;
    recs.clear();
    for (auto lit = lNodes.begin(); lit != lNodes.end();) {
      if (lit->noMore) {
        ++lit;
        continue;
      }
      push_children(*lit, &recs, &nToExpand);
      lit = lNodes.erase(lit);
    }
    if ((int)lNodes.size() >= N || (int)lNodes.size() == prevSize) {
      bFinish = true;
    } else if ((int)lNodes.size() + nToExpand * 3 > N) {
      while (!bFinish) {
        prevSize = (int)lNodes.size();
        std::vector<Rec> prev = recs;
        recs.clear();
        std::sort(prev.begin(), prev.end(), less);
        for (int j = (int)prev.size() - 1; j >= 0; j--) {
          push_children(*prev[j].node, &recs, nullptr);
          lNodes.erase(prev[j].node->lit);
          if ((int)lNodes.size() >= N) break;
        }
        if ((int)lNodes.size() >= N || (int)lNodes.size() == prevSize) bFinish = true;
      }
    }
  }
  std::vector<KP> out;
  out.reserve(lNodes.size());
  for (auto& n : lNodes) {
    const KP* best = &n.keys[0];
    float maxResponse = best->response;
    for (size_t k = 1; k < n.keys.size(); k++)
      if (n.keys[k].response > maxResponse) {
        best = &n.keys[k];
        maxResponse = n.keys[k].response;
      }
    out.push_back(*best);
  }
  return out;
}

// ---------------------------------------------------------------- ORBextractor
struct Extractor {
  int nfeatures, nlevels, iniThFAST, minThFAST;
  double scaleFactor;
  std::vector<float> scale, invScale, sigma2, invSigma2;
  std::vector<int> featsPerLevel;
  int umax[HALF_PATCH_SIZE + 1];
  std::vector<Img> pyr;
  bool unsupported = false;

  // ORBextractor::ORBextractor (ORBextractor.cc:404-460)
  explicit Extractor(const orbx_params& p)
      : nfeatures(p.nfeatures), nlevels(p.nlevels), iniThFAST(p.ini_th_fast),
        minThFAST(p.min_th_fast), scaleFactor(p.scale_factor) {
    scale.resize(nlevels);
    sigma2.resize(nlevels);
    scale[0] = 1.0f;
    sigma2[0] = 1.0f;
    for (int i = 1; i < nlevels; i++) {
      scale[i] = (float)(scale[i - 1] * scaleFactor);
      sigma2[i] = scale[i] * scale[i];
    }
    invScale.resize(nlevels);
    invSigma2.resize(nlevels);
    for (int i = 0; i < nlevels; i++) {
      invScale[i] = 1.0f / scale[i];
      invSigma2[i] = 1.0f / sigma2[i];
    }
    featsPerLevel.resize(nlevels);
    const float factor = (float)(1.0f / scaleFactor);
    float nDesired = nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)nlevels));
    int sum = 0;
    for (int l = 0; l < nlevels - 1; l++) {
      featsPerLevel[l] = cv_round(nDesired);
      sum += featsPerLevel[l];
      nDesired *= factor;
    }
    featsPerLevel[nlevels - 1] = std::max(nfeatures - sum, 0);
    const int vmax = cv_floor(HALF_PATCH_SIZE * std::sqrt(2.f) / 2 + 1);
    const int vmin = cv_ceil(HALF_PATCH_SIZE * std::sqrt(2.f) / 2);
    const double hp2 = HALF_PATCH_SIZE * HALF_PATCH_SIZE;
    int v, v0;
    for (v = 0; v <= vmax; ++v) umax[v] = cv_round(std::sqrt(hp2 - v * v));
    for (v = HALF_PATCH_SIZE, v0 = 0; v >= vmin; --v) {
      while (umax[v0] == umax[v0 + 1]) ++v0;
      umax[v] = v0;
      ++v0;
    }
  }

  void level_size(int w, int h, int l, int* lw, int* lh) const {
    *lw = cv_round((float)w * invScale[l]);
    *lh = cv_round((float)h * invScale[l]);
  }

  // ORBextractor::ComputePyramid (ORBextractor.cc:1047-1072).  The 19-px border written by
  // copyMakeBorder is never read on the hot path (SURVEY §8a A1 notes), so only ROIs are kept.
  void compute_pyramid(const uint8_t* img, int w, int h, int64_t stride) {
    pyr.assign(nlevels, Img());
    for (int l = 0; l < nlevels; l++) {
      Img& L = pyr[l];
      level_size(w, h, l, &L.w, &L.h);
      L.px.assign((size_t)L.w * L.h, 0);
      if (l == 0) {
        for (int y = 0; y < h; y++) std::memcpy(L.row(y), img + (int64_t)y * stride, w);
      } else {
        const Img& P = pyr[l - 1];
        resize_linear(P.px.data(), P.w, P.h, P.w, L.px.data(), L.w, L.h, L.w);
      }
    }
  }

  // ORBextractor::ComputeKeyPointsOctTree (ORBextractor.cc:735-819)
  void compute_keypoints(std::vector<std::vector<KP>>& all, int tie_mode, int* ncand) {
    all.assign(nlevels, {});
    const float W = 30;
    std::vector<Cand> cell;
    for (int level = 0; level < nlevels; ++level) {
      const Img& I = pyr[level];
      const int minBorderX = EDGE_THRESHOLD - 3, minBorderY = minBorderX;
      const int maxBorderX = I.w - EDGE_THRESHOLD + 3, maxBorderY = I.h - EDGE_THRESHOLD + 3;
      std::vector<KP> toDistribute;
      const float width = (float)(maxBorderX - minBorderX);
      const float height = (float)(maxBorderY - minBorderY);
      const int nCols = (int)(width / W), nRows = (int)(height / W);
      if (nCols > 0 && nRows > 0) {
        const int wCell = (int)std::ceil(width / nCols), hCell = (int)std::ceil(height / nRows);
        for (int i = 0; i < nRows; i++) {
          const float iniY = (float)(minBorderY + i * hCell);
          float maxY = iniY + hCell + 6;
          if (iniY >= maxBorderY - 3) continue;
          if (maxY > maxBorderY) maxY = (float)maxBorderY;
          for (int j = 0; j < nCols; j++) {
            const float iniX = (float)(minBorderX + j * wCell);
            float maxX = iniX + wCell + 6;
            if (iniX >= maxBorderX - 6) continue;
            if (maxX > maxBorderX) maxX = (float)maxBorderX;
            const int y0 = (int)iniY, y1 = (int)maxY, x0 = (int)iniX, x1 = (int)maxX;
            const uint8_t* roi = I.row(y0) + x0;
            fast_roi(roi, y1 - y0, x1 - x0, I.w, iniThFAST, cell);
            if (cell.empty()) fast_roi(roi, y1 - y0, x1 - x0, I.w, minThFAST, cell);
            for (const Cand& c : cell) {
              KP kp{(float)c.x, (float)c.y, 7.f, -1.f, (float)c.score, 0, -1};
              kp.x += j * wCell;
              kp.y += i * hCell;
              toDistribute.push_back(kp);
            }
          }
        }
      }
      if (ncand) ncand[level] = (int)toDistribute.size();
      std::vector<KP>& kps = all[level];
      // With no candidates DistributeOctTree returns nothing; it is skipped so degenerate
      // level geometry (nIni < 1) is only an error when there is something to distribute.
      if (!toDistribute.empty()) {
        const int nIni = (int)std::round(static_cast<float>(maxBorderX - minBorderX) /
                                         (maxBorderY - minBorderY));
        if (nIni < 1) {
          unsupported = true;
          continue;
        }
        kps = distribute_octree(toDistribute, minBorderX, maxBorderX, minBorderY, maxBorderY,
                                featsPerLevel[level], tie_mode);
      }
      const int scaledPatchSize = (int)(PATCH_SIZE * scale[level]);
      for (KP& kp : kps) {
        kp.x += minBorderX;
        kp.y += minBorderY;
        kp.octave = level;
        kp.size = (float)scaledPatchSize;
      }
    }
    for (int level = 0; level < nlevels; ++level) {
      const Img& I = pyr[level];
      for (KP& kp : all[level])
        kp.angle = ic_angle(I.px.data(), I.w, cv_round(kp.x), cv_round(kp.y), umax);
    }
  }

  // ORBextractor::operator() (ORBextractor.cc:985-1045)
  int run(const uint8_t* img, int w, int h, int64_t stride, int tie_mode, orbx_keypoint* out,
          uint8_t* desc, int cap, int* n_out, int* ncand) {
    if (w <= 0 || h <= 0) {
      *n_out = -1;
      return ORBX_OK;
    }
    compute_pyramid(img, w, h, stride);
    std::vector<std::vector<KP>> all;
    compute_keypoints(all, tie_mode, ncand);
    if (unsupported) return ORBX_EUNSUPPORTED;
    int n = 0;
    for (auto& v : all) n += (int)v.size();
    *n_out = n;
    if (n > cap) return ORBX_ECAPACITY;
    int off = 0;
    for (int level = 0; level < nlevels; ++level) {
      std::vector<KP>& kps = all[level];
      if (kps.empty()) continue;
      const Img& I = pyr[level];
      std::vector<uint8_t> blurred((size_t)I.w * I.h);
      gaussian7(I.px.data(), I.w, I.h, blurred.data());
      for (size_t i = 0; i < kps.size(); i++)
        orb_descriptor(blurred.data(), I.w, cv_round(kps[i].x), cv_round(kps[i].y),
                       kps[i].angle, desc + (size_t)(off + i) * 32);
      if (level != 0) {
        const float s = scale[level];
        for (KP& kp : kps) kp.x *= s, kp.y *= s;
      }
      for (size_t i = 0; i < kps.size(); i++) {
        const KP& k = kps[i];
        out[off + i] = {k.x, k.y, k.size, k.angle, k.response, k.octave, k.class_id};
      }
      off += (int)kps.size();
    }
    return ORBX_OK;
  }
};

// ---------------------------------------------------------------- ORBmatcher
const int TH_LOW = 50;
const int HISTO_LENGTH = 30;

int descriptor_distance(const uint8_t* a, const uint8_t* b) {
  // ORBmatcher::DescriptorDistance (ORBmatcher.cc:1650-1666): 8x 32-bit SWAR popcount.
  int dist = 0;
  for (int i = 0; i < 8; i++) {
    uint32_t pa, pb;
    std::memcpy(&pa, a + 4 * i, 4);
    std::memcpy(&pb, b + 4 * i, 4);
    uint32_t v = pa ^ pb;
    v = v - ((v >> 1) & 0x55555555);
    v = (v & 0x33333333) + ((v >> 2) & 0x33333333);
    dist += (((v + (v >> 4)) & 0xF0F0F0F) * 0x1010101) >> 24;
  }
  return dist;
}

// ORBmatcher::ComputeThreeMaxima (ORBmatcher.cc:1604-1645)
void three_maxima(const std::vector<int>* histo, int L, int& ind1, int& ind2, int& ind3) {
  int max1 = 0, max2 = 0, max3 = 0;
  for (int i = 0; i < L; i++) {
    const int s = (int)histo[i].size();
    if (s > max1) {
      max3 = max2; max2 = max1; max1 = s;
      ind3 = ind2; ind2 = ind1; ind1 = i;
    } else if (s > max2) {
      max3 = max2; max2 = s;
      ind3 = ind2; ind2 = i;
    } else if (s > max3) {
      max3 = s;
      ind3 = i;
    }
  }
  if (max2 < 0.1f * (float)max1) {
    ind2 = -1;
    ind3 = -1;
  } else if (max3 < 0.1f * (float)max1) {
    ind3 = -1;
  }
}

int rot_bin(float a1, float a2) {
  const float factor = 1.0f / HISTO_LENGTH;
  float rot = a1 - a2;
  if (rot < 0.0) rot += 360.0f;
  int bin = (int)std::round(rot * factor);
  if (bin == HISTO_LENGTH) bin = 0;
  return bin;
}

// Walk two FeatureVectors over equal node ids (the lower_bound merge of ORBmatcher.cc:175-264).
template <class F>
void for_common_nodes(const orbx_featvec& a, const orbx_featvec& b, F f) {
  int i = 0, j = 0;
  while (i < a.n_nodes && j < b.n_nodes) {
    if (a.node_ids[i] == b.node_ids[j]) {
      f(i, j);
      i++;
      j++;
    } else if (a.node_ids[i] < b.node_ids[j]) {
      i = (int)(std::lower_bound(a.node_ids + i, a.node_ids + a.n_nodes, b.node_ids[j]) - a.node_ids);
    } else {
      j = (int)(std::lower_bound(b.node_ids + j, b.node_ids + b.n_nodes, a.node_ids[i]) - b.node_ids);
    }
  }
}

}  // namespace

// ================================================================ C API
extern "C" {

int oracle_extract_ex(const orbx_params* p, const uint8_t* img, int w, int h, int64_t stride,
                      int tie_mode, orbx_keypoint* kps, uint8_t* desc, int cap, int* n_out,
                      uint8_t* pyr, int64_t pyr_cap, int* lw, int* lh, int* n_candidates) {
  if (!p || !n_out || p->nlevels < 1 || p->nlevels > 32) return ORBX_EINVAL;
  Extractor ex(*p);
  int rc = ex.run(img, w, h, stride, tie_mode, kps, desc, cap, n_out, n_candidates);
  if (w > 0 && h > 0) {
    int64_t off = 0;
    for (int l = 0; l < p->nlevels; l++) {
      if (lw) lw[l] = ex.pyr[l].w;
      if (lh) lh[l] = ex.pyr[l].h;
      const int64_t sz = (int64_t)ex.pyr[l].px.size();
      if (pyr && off + sz <= pyr_cap) std::memcpy(pyr + off, ex.pyr[l].px.data(), sz);
      off += sz;
    }
  }
  return rc;
}

int oracle_extract(const orbx_params* p, const uint8_t* img, int w, int h, int64_t stride,
                   int tie_mode, orbx_keypoint* kps, uint8_t* desc, int cap, int* n_out) {
  return oracle_extract_ex(p, img, w, h, stride, tie_mode, kps, desc, cap, n_out, nullptr, 0,
                           nullptr, nullptr, nullptr);
}

int oracle_tables(const orbx_params* p, float* scale, float* inv_scale, float* sigma2,
                  float* inv_sigma2, int* fpl, int* umax16, int* level_w, int* level_h, int w,
                  int h) {
  if (!p || p->nlevels < 1 || p->nlevels > 32) return ORBX_EINVAL;
  Extractor ex(*p);
  for (int l = 0; l < p->nlevels; l++) {
    if (scale) scale[l] = ex.scale[l];
    if (inv_scale) inv_scale[l] = ex.invScale[l];
    if (sigma2) sigma2[l] = ex.sigma2[l];
    if (inv_sigma2) inv_sigma2[l] = ex.invSigma2[l];
    if (fpl) fpl[l] = ex.featsPerLevel[l];
    if (level_w && level_h) ex.level_size(w, h, l, &level_w[l], &level_h[l]);
  }
  if (umax16)
    for (int v = 0; v <= HALF_PATCH_SIZE; v++) umax16[v] = ex.umax[v];
  return ORBX_OK;
}

void oracle_resize_linear(const uint8_t* src, int sw, int sh, int64_t sstride, uint8_t* dst,
                          int dw, int dh, int64_t dstride) {
  resize_linear(src, sw, sh, sstride, dst, dw, dh, dstride);
}
void oracle_gaussian7(const uint8_t* src, int w, int h, uint8_t* dst) { gaussian7(src, w, h, dst); }
float oracle_fast_atan2(float y, float x) { return fast_atan2(y, x); }
int oracle_fast_score(const uint8_t* c, int64_t stride) { return fast_score(c, stride); }
int oracle_fast_roi(const uint8_t* roi, int rows, int cols, int64_t stride, int t, int* xs,
                    int* ys, int* scores, int cap) {
  std::vector<Cand> v;
  fast_roi(roi, rows, cols, stride, t, v);
  int n = std::min((int)v.size(), cap);
  for (int i = 0; i < n; i++) xs[i] = v[i].x, ys[i] = v[i].y, scores[i] = v[i].score;
  return (int)v.size();
}
float oracle_ic_angle(const uint8_t* img, int64_t stride, int cx, int cy) {
  orbx_params p{1000, 1.2f, 8, 20, 7};
  Extractor ex(p);
  return ic_angle(img, stride, cx, cy, ex.umax);
}
void oracle_orb_descriptor(const uint8_t* blurred, int64_t stride, int cx, int cy, float angle,
                           uint8_t* d) {
  orb_descriptor(blurred, stride, cx, cy, angle, d);
}
void oracle_sincosf(float x, float* s, float* c) { sincosf(x, s, c); }
// host libm sincosf over the floats with bit patterns lo .. lo+n-1 (reference outputs of the
// device port's exhaustive test), on `threads` threads
void oracle_sincosf_bits(uint32_t lo, int64_t n, float* s, float* c, int threads) {
  if (threads < 1) threads = 1;
  std::vector<std::thread> th;
  const int64_t per = (n + threads - 1) / threads;
  for (int t = 0; t < threads; t++)
    th.emplace_back([=] {
      const int64_t b = t * per, e = std::min(n, b + per);
      for (int64_t i = b; i < e; i++) {
        const uint32_t u = lo + (uint32_t)i;
        float x;
        memcpy(&x, &u, 4);
        sincosf(x, s + i, c + i);
      }
    });
  for (auto& x : th) x.join();
}

int oracle_descriptor_distance(const uint8_t* a, const uint8_t* b) {
  return descriptor_distance(a, b);
}

// ORBmatcher::SearchByBoW(KeyFrame*, Frame&) (ORBmatcher.cc:159-288)
int oracle_search_by_bow_kf_f(const orbx_bow_side* kf, const orbx_bow_side* f, float nnratio,
                              int check_ori, int32_t* match) {
  for (int i = 0; i < f->n; i++) match[i] = -1;
  std::vector<int> rotHist[HISTO_LENGTH];
  int nmatches = 0;
  for_common_nodes(kf->fv, f->fv, [&](int a, int b) {
    for (int ia = kf->fv.node_offsets[a]; ia < kf->fv.node_offsets[a + 1]; ia++) {
      const int realIdxKF = kf->fv.node_feats[ia];
      if (kf->valid && !kf->valid[realIdxKF]) continue;
      const uint8_t* dKF = kf->desc + (size_t)realIdxKF * 32;
      int best1 = 256, bestIdxF = -1, best2 = 256;
      for (int ib = f->fv.node_offsets[b]; ib < f->fv.node_offsets[b + 1]; ib++) {
        const int realIdxF = f->fv.node_feats[ib];
        if (match[realIdxF] >= 0) continue;
        const int dist = descriptor_distance(dKF, f->desc + (size_t)realIdxF * 32);
        if (dist < best1) {
          best2 = best1;
          best1 = dist;
          bestIdxF = realIdxF;
        } else if (dist < best2) {
          best2 = dist;
        }
      }
      if (best1 <= TH_LOW && static_cast<float>(best1) < nnratio * static_cast<float>(best2)) {
        match[bestIdxF] = realIdxKF;
        if (check_ori) rotHist[rot_bin(kf->angle[realIdxKF], f->angle[bestIdxF])].push_back(bestIdxF);
        nmatches++;
      }
    }
  });
  if (check_ori) {
    int ind1 = -1, ind2 = -1, ind3 = -1;
    three_maxima(rotHist, HISTO_LENGTH, ind1, ind2, ind3);
    for (int i = 0; i < HISTO_LENGTH; i++) {
      if (i == ind1 || i == ind2 || i == ind3) continue;
      for (int j : rotHist[i]) {
        match[j] = -1;
        nmatches--;
      }
    }
  }
  return nmatches;
}

// ORBmatcher::SearchByBoW(KeyFrame*, KeyFrame*) (ORBmatcher.cc:525-658)
int oracle_search_by_bow_kf_kf(const orbx_bow_side* k1, const orbx_bow_side* k2, float nnratio,
                               int check_ori, int32_t* match12) {
  for (int i = 0; i < k1->n; i++) match12[i] = -1;
  std::vector<char> matched2(k2->n, 0);
  std::vector<int> rotHist[HISTO_LENGTH];
  int nmatches = 0;
  for_common_nodes(k1->fv, k2->fv, [&](int a, int b) {
    for (int ia = k1->fv.node_offsets[a]; ia < k1->fv.node_offsets[a + 1]; ia++) {
      const int idx1 = k1->fv.node_feats[ia];
      if (k1->valid && !k1->valid[idx1]) continue;
      const uint8_t* d1 = k1->desc + (size_t)idx1 * 32;
      int best1 = 256, bestIdx2 = -1, best2 = 256;
      for (int ib = k2->fv.node_offsets[b]; ib < k2->fv.node_offsets[b + 1]; ib++) {
        const int idx2 = k2->fv.node_feats[ib];
        if (matched2[idx2] || (k2->valid && !k2->valid[idx2])) continue;
        const int dist = descriptor_distance(d1, k2->desc + (size_t)idx2 * 32);
        if (dist < best1) {
          best2 = best1;
          best1 = dist;
          bestIdx2 = idx2;
        } else if (dist < best2) {
          best2 = dist;
        }
      }
      if (best1 < TH_LOW && static_cast<float>(best1) < nnratio * static_cast<float>(best2)) {
        match12[idx1] = bestIdx2;
        matched2[bestIdx2] = 1;
        if (check_ori) rotHist[rot_bin(k1->angle[idx1], k2->angle[bestIdx2])].push_back(idx1);
        nmatches++;
      }
    }
  });
  if (check_ori) {
    int ind1 = -1, ind2 = -1, ind3 = -1;
    three_maxima(rotHist, HISTO_LENGTH, ind1, ind2, ind3);
    for (int i = 0; i < HISTO_LENGTH; i++) {
      if (i == ind1 || i == ind2 || i == ind3) continue;
      for (int j : rotHist[i]) {
        match12[j] = -1;
        nmatches--;
      }
    }
  }
  return nmatches;
}

// ORBmatcher::CheckDistEpipolarLine (ORBmatcher.cc:140-157) with the reference binary's FMA
// pattern.
static bool check_dist_epipolar(const orbx_keypoint& kp1, const orbx_keypoint& kp2,
                                const float* F, const orbx_tri_side* kf2) {
  const float x1 = kp1.x, y1 = kp1.y;
  const float a = std::fma(x1, F[0], y1 * F[3]) + F[6];
  const float b = std::fma(x1, F[1], y1 * F[4]) + F[7];
  const float c = std::fma(y1, F[5], x1 * F[2]) + F[8];
  const float num = std::fma(b, kp2.y, kp2.x * a) + c;
  const float den = std::fma(a, a, b * b);
  if (den == 0) return false;
  const float dsqr = num * num / den;
  return (double)dsqr < 3.84 * (double)kf2->level_sigma2[kp2.octave];
}

// ORBmatcher::SearchForTriangulation (ORBmatcher.cc:660-826)
int oracle_search_for_triangulation(const orbx_tri_side* k1, const orbx_tri_side* k2,
                                    const float F12[9], float ex, float ey, int only_stereo,
                                    float /*nnratio: unused by the reference here*/,
                                    int check_ori, int32_t* pairs) {
  std::vector<int> m12(k1->n, -1);
  std::vector<int> rotHist[HISTO_LENGTH];
  int nmatches = 0;
  for_common_nodes(k1->fv, k2->fv, [&](int a, int b) {
    for (int ia = k1->fv.node_offsets[a]; ia < k1->fv.node_offsets[a + 1]; ia++) {
      const int idx1 = k1->fv.node_feats[ia];
      if (k1->has_mp && k1->has_mp[idx1]) continue;
      const bool st1 = k1->u_right ? k1->u_right[idx1] >= 0 : false;
      if (only_stereo && !st1) continue;
      const orbx_keypoint& kp1 = k1->keys_un[idx1];
      const uint8_t* d1 = k1->desc + (size_t)idx1 * 32;
      int bestDist = TH_LOW, bestIdx2 = -1;
      for (int ib = k2->fv.node_offsets[b]; ib < k2->fv.node_offsets[b + 1]; ib++) {
        const int idx2 = k2->fv.node_feats[ib];
        // `vbMatched2[idx2] || pMP2` (:728): vbMatched2 is never set in this function
        if (k2->has_mp && k2->has_mp[idx2]) continue;
        const bool st2 = k2->u_right ? k2->u_right[idx2] >= 0 : false;
        if (only_stereo && !st2) continue;
        const int dist = descriptor_distance(d1, k2->desc + (size_t)idx2 * 32);
        if (dist > TH_LOW || dist > bestDist) continue;
        const orbx_keypoint& kp2 = k2->keys_un[idx2];
        if (!st1 && !st2) {
          const float dex = ex - kp2.x, dey = ey - kp2.y;
          if (std::fma(dex, dex, dey * dey) < 100 * k2->scale_factors[kp2.octave]) continue;
        }
        if (check_dist_epipolar(kp1, kp2, F12, k2)) {
          bestIdx2 = idx2;
          bestDist = dist;
        }
      }
      if (bestIdx2 >= 0) {
        m12[idx1] = bestIdx2;
        nmatches++;
        if (check_ori) rotHist[rot_bin(kp1.angle, k2->keys_un[bestIdx2].angle)].push_back(idx1);
      }
    }
  });
  if (check_ori) {
    int ind1 = -1, ind2 = -1, ind3 = -1;
    three_maxima(rotHist, HISTO_LENGTH, ind1, ind2, ind3);
    for (int i = 0; i < HISTO_LENGTH; i++) {
      if (i == ind1 || i == ind2 || i == ind3) continue;
      for (int j : rotHist[i]) {
        m12[j] = -1;
        nmatches--;
      }
    }
  }
  int n = 0;
  for (int i = 0; i < k1->n; i++)
    if (m12[i] >= 0) {
      pairs[2 * n] = i;
      pairs[2 * n + 1] = m12[i];
      n++;
    }
  return nmatches;
}

// Epipole (ORBmatcher.cc:667-673): C2 = R2w*Cw + t2w (cv::Mat f32 gemm, then add);
// ex = fmaf(invz, fx*C2x, cx) per the reference binary.
void oracle_epipole(const float R[9], const float t[3], const float Cw[3], float fx, float fy,
                    float cx, float cy, float* ex, float* ey) {
  float C2[3];
  for (int r = 0; r < 3; r++) {
    // cv::gemm on 3x3 * 3x1 f32 accumulates in double and stores f32
    double s = 0;
    for (int c = 0; c < 3; c++) s += (double)R[3 * r + c] * (double)Cw[c];
    C2[r] = (float)s + t[r];
  }
  const float invz = 1.0f / C2[2];
  *ex = std::fma(invz, fx * C2[0], cx);
  *ey = std::fma(invz, fy * C2[1], cy);
}

// TemplatedVocabulary::transform node-id part (TemplatedVocabulary.h:1218-1259): greedy
// descent, first child wins ties (strict <), nid recorded at level L - levelsup.
void oracle_feature_vector(const uint8_t* voc, int k, int L, int levelsup, const uint8_t* desc,
                           int n, uint32_t* out) {
  const int nid_level = L - levelsup;
  for (int i = 0; i < n; i++) {
    if (nid_level <= 0) {
      out[i] = 0;
      continue;
    }
    uint64_t level_off = 1, level_size = 1;  // level 1 starts at id 1
    uint64_t j = 0;                          // index within current level
    uint32_t id = 0;
    for (int lvl = 1; lvl <= nid_level; lvl++) {
      level_size *= k;
      const uint64_t first = level_off + j * k;
      uint64_t best = first;
      int bestd = descriptor_distance(desc + (size_t)i * 32, voc + first * 32);
      for (int c = 1; c < k; c++) {
        const int d = descriptor_distance(desc + (size_t)i * 32, voc + (first + c) * 32);
        if (d < bestd) bestd = d, best = first + c;
      }
      id = (uint32_t)best;
      j = best - level_off;
      level_off += level_size;
    }
    out[i] = id;
  }
}

}  // extern "C"
