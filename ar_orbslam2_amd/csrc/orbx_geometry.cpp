// orbx_geometry.cpp — host-side tables of a plan.  Every float expression below is evaluated
// with the reference's types (ORB_SLAM2/src/ORBextractor.cc) and without contraction, so the
// GPU path sees exactly the level sizes, cell grid, resize coefficients and octree frame the
// reference computes.
#include <math.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstdio>

#include "orbx_internal.h"

#pragma clang fp contract(off)

namespace orbx {

static inline int cv_round(double v) { return (int)nearbyint(v); }  // cvRound: half-even

int report_hip(hipError_t e, const char* what) {
  fprintf(stderr, "[orbx] HIP error %d (%s) at %s\n", (int)e, hipGetErrorString(e), what);
  return ORBX_EDEVICE;
}

hipError_t wait_stream(hipStream_t s) {
  static const long spin_us = [] {
    const char* e = getenv("ORBX_SPIN_US");
    return e ? std::max(0L, atol(e)) : 2000L;
  }();
  if (spin_us > 0) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
      const hipError_t e = hipStreamQuery(s);
      if (e != hipErrorNotReady) return e;
      if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(spin_us)) break;
      for (int i = 0; i < 32; i++) __builtin_ia32_pause();  // (a yield can lose the core)
    }
  }
  return hipStreamSynchronize(s);
}

std::recursive_mutex& resource_mutex() {
  static std::recursive_mutex m;
  return m;
}

int report(int code, const char* what) {
  fprintf(stderr, "[orbx] error %d: %s\n", code, what);
  return code;
}

// ORBextractor::ORBextractor (ORBextractor.cc:404-460)
void build_tables(const orbx_params& p, Geometry* g) {
  const int L = p.nlevels;
  const double sf = (double)p.scale_factor;  // member `double scaleFactor` (ORBextractor.h:104)
  g->nlevels = L;
  g->scale[0] = 1.0f;
  g->sigma2[0] = 1.0f;
  for (int i = 1; i < L; i++) {
    g->scale[i] = (float)((double)g->scale[i - 1] * sf);
    g->sigma2[i] = g->scale[i] * g->scale[i];
  }
  for (int i = 0; i < L; i++) {
    g->inv_scale[i] = 1.0f / g->scale[i];
    g->inv_sigma2[i] = 1.0f / g->sigma2[i];
  }
  const float factor = (float)(1.0f / sf);
  float nDesired =
      (float)p.nfeatures * (1 - factor) / (1 - (float)pow((double)factor, (double)L));
  int sum = 0;
  for (int l = 0; l < L - 1; l++) {
    g->feats[l] = cv_round(nDesired);
    sum += g->feats[l];
    nDesired *= factor;
  }
  g->feats[L - 1] = std::max(p.nfeatures - sum, 0);
  // umax (ORBextractor.cc:445-459)
  const int vmax = (int)floor(kHalfPatch * sqrtf(2.f) / 2 + 1);
  const int vmin = (int)ceil(kHalfPatch * sqrtf(2.f) / 2);
  const double hp2 = kHalfPatch * kHalfPatch;
  int v, v0;
  for (v = 0; v <= vmax; ++v) g->umax[v] = cv_round(sqrt(hp2 - v * v));
  for (v = kHalfPatch, v0 = 0; v >= vmin; --v) {
    while (g->umax[v0] == g->umax[v0 + 1]) ++v0;
    g->umax[v] = v0;
    ++v0;
  }
}

// cv::resize INTER_LINEAR coefficient tables (OpenCV 2.4 imgwarp.cpp).
static bool resize_tables(int sw, int sh, int dw, int dh, Geometry* g, LevelGeom* L) {
  const double inv_sx = (double)dw / sw, inv_sy = (double)dh / sh;
  const double sx = 1. / inv_sx, sy = 1. / inv_sy;
  L->coef_x = (int)g->xtap.size() / 2;  // multiple of 4 (every run padded)
  L->coef_y = (int)g->ytap.size() / 2;
  int xmax = dw;
  for (int dx = 0; dx < dw; dx++) {
    float fx = (float)((dx + 0.5) * sx - 0.5);
    int x0 = (int)floorf(fx);
    fx -= x0;
    if (x0 < 0) fx = 0, x0 = 0;
    if (x0 + 1 >= sw) {
      xmax = std::min(xmax, dx);
      if (x0 >= sw - 1) fx = 0, x0 = sw - 1;
    }
    g->xofs.push_back(x0);
    const float c0 = 1.f - fx, c1 = fx;
    g->xa.push_back((int16_t)std::min(32767, std::max(-32768, cv_round(c0 * 2048))));
    g->xa.push_back((int16_t)std::min(32767, std::max(-32768, cv_round(c1 * 2048))));
  }
  for (int dy = 0; dy < dh; dy++) {
    float fy = (float)((dy + 0.5) * sy - 0.5);
    const int y0 = (int)floorf(fy);
    fy -= y0;
    g->yofs.push_back(y0);
    const float c0 = 1.f - fy, c1 = fy;
    g->yb.push_back((int16_t)std::min(32767, std::max(-32768, cv_round(c0 * 2048))));
    g->yb.push_back((int16_t)std::min(32767, std::max(-32768, cv_round(c1 * 2048))));
  }
  L->xmax = xmax;
  int xs = 0;  // VResizeLinearVec_32s8u: 16-wide while x <= W-16, 4-wide while x < W-4
  while (xs <= dw - 16) xs += 16;
  while (xs < dw - 4) xs += 4;
  L->vxs = xs;
  // k_pyramid taps: columns -4 .. 4*(gl+2)-1 (gl = (dw-1)/4, the last 4-column group holding a
  // pixel); coef_x indexes column 0.  A column outside [0, dw) carries the taps of its
  // BORDER_REFLECT_101 image, so the level rows k_pyramid keeps in LDS hold GaussianBlur's
  // 3-column halo on both sides (the fused blur reads it), and a column at or past vxs is marked
  // by bit 30 of its source offset (the scalar vertical form, per column).
  auto reflect = [](int p, int len) {
    if (len == 1) return 0;
    while (p < 0 || p >= len) p = p < 0 ? -p : 2 * len - p - 2;
    return p;
  };
  const int gl = (dw - 1) / 4;
  for (int dx = -4; dx < 4 * (gl + 2); dx++) {
    if (dx == 0) L->coef_x = (int)g->xtap.size() / 2;
    const int r = reflect(dx, dw);
    const int i = 2 * ((int)g->xofs.size() - dw + r);
    const int a0 = r >= xmax ? 2048 : g->xa[i];
    const int a1 = r >= xmax ? 0 : g->xa[i + 1];
    g->xtap.push_back(g->xofs[i / 2] | (r >= xs ? 1 << 30 : 0));
    g->xtap.push_back((int32_t)((uint32_t)(a0 << 4) | ((uint32_t)(a1 << 4) << 16)));  // Q15
  }
  for (int dy = 0; dy < dh; dy++) {
    const int i = (int)g->yofs.size() - dh + dy;
    g->ytap.push_back(g->yofs[i]);
    g->ytap.push_back((g->yb[2 * i] & 0xFFFF) | (g->yb[2 * i + 1] << 16));
  }
  bool ok = true;
  // k_pyramid drops OpenCV's saturations: they are no-ops while every coefficient is in
  // [0, 2048] and each pair sums to at most 2049 (rounding may give 2049).
  for (size_t i = 2 * (g->xofs.size() - dw); i < g->xa.size(); i += 2)
    if (g->xa[i] < 0 || g->xa[i + 1] < 0 || g->xa[i] + g->xa[i + 1] > 2049) ok = false;
  for (size_t i = 2 * (g->yofs.size() - dh); i < g->yb.size(); i += 2)
    if (g->yb[i] < 0 || g->yb[i + 1] < 0 || g->yb[i] + g->yb[i + 1] > 2049) ok = false;
  return ok;
}

// Stage `st` as nb row bands x ncol column tiles (PyrBand).  Every level's rows split into nb
// bands and its 4-column groups into ncol tiles on 16-column boundaries; a tile computes, going
// down from the stage's last level, the rows and groups its levels' cones need (rows and groups
// shared by two tiles are computed by both, identically; only the owner stores them), and with
// the blur fused its blurred levels carry GaussianBlur's 3-row / one-group halo (clipped rows:
// the reflected rows lie inside; the groups -1 and gl + 1 hold the reflected pad columns).
// Returns the LDS bytes of the stage (st.smem, st.buf_b set) and the pixels the resize passes
// compute and own (levels l0 .. l1).
static int stage_tiles(const Geometry& g, PyrStage& st, int nb, int ncol, bool fused,
                       std::vector<PyrBand>& tiles, double& comp, double& own) {
  tiles.assign((size_t)nb * ncol, PyrBand{});
  int need[2] = {0, 0};
  comp = own = 0;
  constexpr int kEmpty = 1 << 30;
  for (int b = 0; b < nb; b++)
    for (int t = 0; t < ncol; t++) {
      PyrBand& B = tiles[(size_t)b * ncol + t];
      for (int l = st.l0 - 1; l <= st.l1; l++) {
        const LevelGeom& L = g.lv[l];
        const int h = L.h, ng = ((L.w - 1) >> 2) + 1, n16 = (ng + 3) / 4;
        B.own_lo[l] = (int)((int64_t)b * h / nb);
        B.own_hi[l] = (int)((int64_t)(b + 1) * h / nb);
        B.own_glo[l] = std::min(ng, 4 * (int)((int64_t)t * n16 / ncol));
        B.own_ghi[l] = std::min(ng, 4 * (int)((int64_t)(t + 1) * n16 / ncol));
        const bool owns = B.own_hi[l] > B.own_lo[l] && B.own_ghi[l] > B.own_glo[l];
        const bool blurred = fused && (l >= st.l0 || st.l0 == 1);
        // the source level is computed only for the cone of the level above it
        if (!owns || (l == st.l0 - 1 && st.l0 > 1)) {
          B.lo[l] = B.glo[l] = kEmpty;
          B.hi[l] = B.ghi[l] = -kEmpty;
        } else if (blurred) {
          B.lo[l] = std::max(0, B.own_lo[l] - 3);
          B.hi[l] = std::min(h, B.own_hi[l] + 3);
          B.glo[l] = B.own_glo[l] - 1;
          B.ghi[l] = B.own_ghi[l] + 1;
        } else {
          B.lo[l] = B.own_lo[l];
          B.hi[l] = B.own_hi[l];
          B.glo[l] = B.own_glo[l];
          B.ghi[l] = B.own_ghi[l];
        }
      }
      for (int l = st.l1; l >= st.l0; l--) {  // the source rows and columns of level l's ranges
        const LevelGeom& D = g.lv[l];
        const LevelGeom& S = g.lv[l - 1];
        if (B.hi[l] <= B.lo[l] || B.ghi[l] <= B.glo[l]) continue;
        const int slo = std::min(std::max(g.yofs[D.coef_y + B.lo[l]], 0), S.h - 1);
        const int shi = std::min(std::max(g.yofs[D.coef_y + B.hi[l] - 1] + 1, 0), S.h - 1) + 1;
        int xmin = kEmpty, xmax = -1;
        for (int dx = 4 * B.glo[l]; dx < 4 * B.ghi[l]; dx++) {
          const int xs = g.xtap[2 * (D.coef_x + dx)] & 0xFFFFF;
          xmin = std::min(xmin, xs);
          xmax = std::max(xmax, xs + 1);  // py_horiz reads S0 and S1
        }
        B.lo[l - 1] = std::min(B.lo[l - 1], slo);
        B.hi[l - 1] = std::max(B.hi[l - 1], shi);
        B.glo[l - 1] = std::min(B.glo[l - 1], xmin >> 2);
        B.ghi[l - 1] = std::max(B.ghi[l - 1], (xmax >> 2) + 1);
      }
      for (int l = st.l0 - 1; l <= st.l1; l++) {
        if (B.hi[l] <= B.lo[l] || B.ghi[l] <= B.glo[l]) {
          B.lo[l] = B.hi[l] = B.own_lo[l];
          B.glo[l] = B.ghi[l] = std::max(0, B.own_glo[l]);
          B.cb[l] = 0;
          B.lp[l] = 16;
          continue;
        }
        // LDS row: columns cb .. cb + lp - 1, cb = 4 glo rounded down to 16 bytes
        B.cb[l] = (4 * B.glo[l]) & ~15;
        B.lp[l] = (4 * B.ghi[l] - B.cb[l] + 15) & ~15;
        need[l & 1] = std::max(need[l & 1], (B.hi[l] - B.lo[l]) * B.lp[l]);
        if (l >= st.l0) {
          comp += (double)(B.hi[l] - B.lo[l]) * 4 * (B.ghi[l] - B.glo[l]);
          own += (double)(B.own_hi[l] - B.own_lo[l]) * 4 * (B.own_ghi[l] - B.own_glo[l]);
        }
      }
    }
  st.buf_b = (need[0] + 15) & ~15;
  st.smem = std::max(16, st.buf_b + need[1]);
  return st.smem;
}

// k_pyramid's stages and tiles (the comment in build_pyramid); false when no tiling of a stage
// fits kPyMaxSmemLimit bytes of LDS.  Per stage, for every column split 1 .. kPyMaxCols, the
// tallest bands (at most kPyBandHMul x py_band_h source rows, at least py_min_tiles tiles per
// image) whose two LDS buffers fit the bound, then the split whose tiles compute the fewest
// pixels.
static bool build_stages(Geometry* g, bool fused, double* recompute) {
  const int nl = g->nlevels;
  g->pyr_stages.clear();
  g->bands.clear();
  const int py_max_smem = fused ? kPyMaxSmemFused : kPyMaxSmem;  // a tile's two level buffers
  const int stage0 = fused ? kPyStage0Fused : kPyStage0, stage_n = fused ? kPyStageNFused : kPyStageN;
  double comp_all = 0, own_all = 0;
  for (int l0 = 1; l0 <= std::max(nl - 1, 1); ) {
    PyrStage st{};
    st.l0 = l0;
    st.l1 = nl == 1 ? 0 : std::min(nl - 1, l0 + (l0 == 1 ? stage0 : stage_n) - 1);
    const int hs = g->lv[l0 - 1].h;
    std::vector<PyrBand> best, tiles;
    PyrStage best_st{};
    double best_comp = 0, best_own = 0;
    bool found = false;
    for (int cap : {py_max_smem, kPyMaxSmemLimit}) {
      // the few-image plans keep their short bands (more workgroups for one image's chain)
      const int ncmax = g->py_band_h < kPyBandH ? 1 : kPyMaxCols;
      for (int ncol = 1; ncol <= ncmax; ncol++) {
        const int band_h = g->py_band_h < kPyBandH ? g->py_band_h : g->py_band_h * kPyBandHMul;
        // enough tiles per image that a batch's launch fills the chip several times over
        const int nb_lo = std::max({1, hs / std::max(1, band_h), (g->py_min_tiles + ncol - 1) / ncol});
        const int nb_hi = std::max(nb_lo, hs);
        for (int nb = nb_lo; nb <= nb_hi; nb++) {
          PyrStage s2 = st;
          double comp, own;
          if (stage_tiles(*g, s2, nb, ncol, fused, tiles, comp, own) > cap) continue;
          if (!found || comp < best_comp) {
            found = true;
            best.swap(tiles);
            best_st = s2;
            best_comp = comp;
            best_own = own;
          }
          break;  // taller bands than the first that fits do not fit
        }
      }
      if (found) break;  // the larger carve only when nothing fits the bound
    }
    if (!found) return false;
    best_st.band0 = (int)g->bands.size();
    best_st.nbands = (int)best.size();
    g->bands.insert(g->bands.end(), best.begin(), best.end());
    g->pyr_stages.push_back(best_st);
    comp_all += best_comp;
    own_all += best_own;
    l0 = st.l1 + 1;
    if (nl == 1) break;
  }
  if (recompute) *recompute = own_all > 0 ? comp_all / own_all : 1.0;
  return true;
}

// The pyramid part of a plan for the level sizes already in g->lv[0 .. g->nlevels): cv::resize
// tables of every level >= 1, pitches and offsets in the pyramid block, k_pyramid stages.
int build_pyramid(Geometry* g, std::string* why) {
  g->xofs.clear();
  g->yofs.clear();
  g->xa.clear();
  g->yb.clear();
  g->xtap.clear();
  g->ytap.clear();
  const int nl = g->nlevels;
  int64_t pyr = 0;
  for (int l = 0; l < nl; l++) {
    LevelGeom& L = g->lv[l];
    if (L.w < 1 || L.h < 1) {
      if (why) *why = "empty pyramid level";
      return ORBX_EUNSUPPORTED;
    }
    if (l > 0) {
      const LevelGeom& P = g->lv[l - 1];
      // cv::resize (OpenCV 2.4.9, the version the reference links) switches INTER_LINEAR to
      // the fast INTER_AREA path at an exact 2x2 decimation: (a + b + c + d + 2) >> 2 per
      // output pixel.  The linear taps at that scale are 1024 / 1024 in both passes, and both
      // of OpenCV's vertical paths (SSE2 mulhi of the >>4 sums, scalar >>22) round that same
      // way, so the tables below produce it unchanged (tests/test_oracle_kat.py).
      if (!resize_tables(P.w, P.h, L.w, L.h, g, &L)) {
        if (why) *why = "resize coefficients outside [0, 2048]";
        return ORBX_EUNSUPPORTED;
      }
    }
    // every level (level 0 is copied in) lives in the pitched pyramid block
    L.pitch = (L.w + 4 + 63) & ~63;  // >= w + 4: a row's last dword never straddles the row end
    L.pyr_off = pyr;
    pyr += ((int64_t)L.pitch * L.h + 255) / 256 * 256;
    L.bxs = (L.w / 4) * 4;
  }
  g->pyr_bytes = std::max<int64_t>(pyr, 256);
  // k_pyramid stages: levels 1..kPyStage0, then kPyStageN at a time.  In a stage, band b
  // owns rows [b*h_l/nb, (b+1)*h_l/nb) of every level and computes, going down from the
  // stage's last level, the rows the next level's rows need as well (rows shared by two bands
  // are computed by both, identically; only the owner stores them).  Its level l rows stay in
  // LDS for level l+1: even levels in buffer A, odd ones in B.  The recomputed cone grows by
  // ~2 rows per level below the top, so stages stay short.
  // With the blur fused (kPyFused), a band blurs its own rows of every level it builds (and of
  // level 0 in the first stage) from the rows it holds in LDS: those levels' row ranges carry
  // GaussianBlur's 3-row halo, clipped to the level (the reflected rows lie inside the range).
  // The blur is fused where the bands fit (every configuration the benchmarks run); frames too
  // wide for its halo rows keep the separate k_blur launch.
  double rc = 0;
  g->blur_fused = kPyFused && build_stages(g, true, &rc) && rc <= kPyFuseMaxRecompute;
  if (!g->blur_fused && !build_stages(g, false, nullptr)) {
    if (why) *why = "image too wide for the pyramid bands";
    return ORBX_EUNSUPPORTED;
  }
  return ORBX_OK;
}

int build_geometry(const orbx_params& p, int w, int h, Geometry* g, std::string* why) {
  if (p.nlevels < 1 || p.nlevels > kMaxLevels || p.nfeatures < 0 || !(p.scale_factor > 0)) {
    if (why) *why = "bad params";
    return ORBX_EINVAL;
  }
  build_tables(p, g);
  g->w = w;
  g->h = h;
  g->ini_th = std::min(std::max(p.ini_th_fast, 0), 255);
  g->min_th = std::min(std::max(p.min_th_fast, 0), 255);
  g->cells.clear();
  g->octpath.clear();
  g->wide_keys = false;
  for (int l = 0; l < p.nlevels; l++) {
    LevelGeom& L = g->lv[l];
    L = LevelGeom{};
    // ComputePyramid (ORBextractor.cc:1049-1051)
    L.w = cv_round((float)w * g->inv_scale[l]);
    L.h = cv_round((float)h * g->inv_scale[l]);
  }
  int rc = build_pyramid(g, why);
  if (rc != ORBX_OK) return rc;
  int cand = 0, kp = 0, ncmax = 0;
  for (int l = 0; l < p.nlevels; l++) {
    LevelGeom& L = g->lv[l];
    L.scale = g->scale[l];
    L.inv_scale = g->inv_scale[l];
    L.size = (float)(int)(kPatch * g->scale[l]);
    L.nfeat = g->feats[l];
    // ComputeKeyPointsOctTree cell grid (ORBextractor.cc:742-796)
    const int minB = kEdge - 3;
    const int maxBX = L.w - kEdge + 3, maxBY = L.h - kEdge + 3;
    const float width = (float)(maxBX - minB), height = (float)(maxBY - minB);
    const int nCols = (int)(width / 30.f), nRows = (int)(height / 30.f);
    L.cell_begin = (int)g->cells.size();
    L.cand_off = cand;
    if (nCols > 0 && nRows > 0) {
      const int wCell = (int)ceilf(width / nCols), hCell = (int)ceilf(height / nRows);
      L.wcell = wCell;
      L.hcell = hCell;
      for (int i = 0; i < nRows; i++) {
        const float iniY = (float)(minB + i * hCell);
        float maxY = iniY + hCell + 6;
        if (iniY >= maxBY - 3) continue;
        if (maxY > maxBY) maxY = (float)maxBY;
        for (int j = 0; j < nCols; j++) {
          const float iniX = (float)(minB + j * wCell);
          float maxX = iniX + wCell + 6;
          if (iniX >= maxBX - 6) continue;
          if (maxX > maxBX) maxX = (float)maxBX;
          CellGeom c{};
          c.x0 = (int16_t)(int)iniX;
          c.y0 = (int16_t)(int)iniY;
          c.x1 = (int16_t)(int)maxX;
          c.y1 = (int16_t)(int)maxY;
          c.offx = (int16_t)(j * wCell);
          c.offy = (int16_t)(i * hCell);
          c.level = (int16_t)l;
          const int dc = c.x1 - c.x0 - 6, dr = c.y1 - c.y0 - 6;
          // strict 8-neighbour NMS survivors form an independent set of the king graph
          c.slot_cap = (dc > 0 && dr > 0) ? ((dc + 1) / 2) * ((dr + 1) / 2) : 0;
          c.slot_off = cand;
          cand += c.slot_cap;
          c.v_row0 = (int)(L.pyr_off + (int64_t)(c.y0 + 3) * L.pitch + c.x0 + 3);
          c.pitch = L.pitch;
          g->cells.push_back(c);
        }
      }
      // DistributeOctTree frame (ORBextractor.cc:530-532)
      L.W = maxBX - minB;
      L.H = maxBY - minB;
      L.nini = (int)roundf(static_cast<float>(L.W) / L.H);
      if (L.nini < 1) {  // aspect below 1:2: the reference indexes vpIniNodes out of bounds
        if (why) *why = "octree initial column count below 1 (portrait aspect under 1:2)";
        return ORBX_EUNSUPPORTED;
      }
      L.hx = static_cast<float>(L.W) / L.nini;
      // candidate keys: x:12 y:12 in a u32 up to 4095 px, x:16 y:16 in a u64 above (the
      // node and cell bounds are int16)
      if (L.W > 32767 || L.H > 32767) {
        if (why) *why = "level wider or taller than 32767 px";
        return ORBX_EUNSUPPORTED;
      }
      g->wide_keys |= L.W >= 4096 || L.H >= 4096;
      // quadrant paths (ORBextractor.cc:472-522: halfX = ceil((UR.x - UL.x) / 2), a key goes
      // right when x >= UL.x + halfX); below depth 16 every node is at most 1 px wide and high,
      // so every key of it stays in quadrant 0 and the path is all zeros there
      auto spread = [](uint32_t v) {
        v = (v | (v << 8)) & 0x00FF00FFu;
        v = (v | (v << 4)) & 0x0F0F0F0Fu;
        v = (v | (v << 2)) & 0x33333333u;
        return (v | (v << 1)) & 0x55555555u;
      };
      auto path = [&](int c, int lo, int hi) {
        uint32_t bits = 0;
        for (int t = 0; t < 16; t++) {
          const int m = lo + (hi - lo + 1) / 2;
          if (c >= m) {
            bits |= 1u << (15 - t);
            lo = m;
          } else {
            hi = m;
          }
        }
        return spread(bits);
      };
      L.path_x = (int)g->octpath.size();
      for (int x = 0; x < L.W; x++) {
        // the key's initial node as k_octree and DistributeOctTree take it ((int)(x / hX),
        // :555), the node's columns from the truncated products (:540-544)
        const int i = std::min((int)(static_cast<float>(x) / L.hx), L.nini - 1);
        g->octpath.push_back(path(x, (int)(L.hx * static_cast<float>(i)),
                                  (int)(L.hx * static_cast<float>(i + 1))));
      }
      L.path_y = (int)g->octpath.size();
      for (int y = 0; y < L.H; y++) g->octpath.push_back(path(y, 0, L.H) << 1);
    }
    L.ncells = (int)g->cells.size() - L.cell_begin;
    L.cand_cap = cand - L.cand_off;
    if (L.cand_cap >= (1 << 24)) {  // k_octree's retention packs a level's key index in 24 bits
      if (why) *why = "level candidate capacity exceeds 2^24";
      return ORBX_EUNSUPPORTED;
    }
    ncmax = std::max(ncmax, L.ncells);
    L.node_cap = L.ncells ? std::max(L.nfeat + 3, 4 * L.nini + 4) : 1;
    L.kp_off = kp;
    L.kp_cap = L.node_cap;
    kp += L.kp_cap;
    g->node_cap_max = std::max(g->node_cap_max, L.node_cap);
  }

  g->cand_total = cand;
  g->kp_total = kp;
  (void)ncmax;
  return ORBX_OK;
}

}  // namespace orbx
