// orbx_internal.h — plan geometry and helpers shared by the orbx HIP translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/orbx.h"

#pragma clang fp contract(off)

namespace orbx {

constexpr int kMaxLevels = 16;
constexpr int kEdge = 19;       // EDGE_THRESHOLD (ORBextractor.cc:71)
constexpr int kPatch = 31;      // PATCH_SIZE (:69)
constexpr int kHalfPatch = 15;  // HALF_PATCH_SIZE (:70)
constexpr int kMaxIni = 64;     // initial octree columns supported (nIni)

// Per pyramid level, computed on the host once per plan (ORBextractor.cc:404-460,
// 735-757, 1047-1072).
struct LevelGeom {
  int w, h;            // level size (cvRound((float)cols * invScale))
  int64_t pyr_off;     // offset of the level inside one image's pyramid block
  int coef_x, coef_y;  // offsets into the resize coefficient tables (levels >= 1)
  int xmax;            // HResizeLinear clamp start (dx >= xmax reads S[x0]*2048)
  int vxs;             // VResizeLinearVec_32s8u SSE2 region: x < vxs
  int bxs;             // SymmColumnVec_32s8u region: x < 4*floor(w/4)
  int cell_begin, ncells;  // range in the cell table
  int cand_off, cand_cap;  // candidate region (keys) inside one image's candidate block
  int nfeat;               // mnFeaturesPerLevel
  int nini;                // DistributeOctTree initial columns
  float hx;                // (float)(maxX-minX)/nIni
  int ini_x[kMaxIni + 1];  // (int)(hX * i)
  int W, H;                // maxX-minX, maxY-minY (octree frame, origin at minBorder=16)
  int node_cap;            // max alive octree nodes: max(N+3, 4*nIni+4)
  int kp_off, kp_cap;      // per-image final keypoint slots for this level
  float scale;             // mvScaleFactor
  float size;              // (float)(int)(PATCH_SIZE * scale)
};

struct CellGeom {
  int16_t x0, y0, x1, y1;  // cell image ROI in level coordinates [x0,x1) x [y0,y1)
  int16_t offx, offy;      // j*wCell, i*hCell (ORBextractor.cc:789-790)
  int16_t level, pad;
  int slot_off, slot_cap;  // candidate slot inside the image's candidate block
};

struct Geometry {
  int w = 0, h = 0, nlevels = 0;
  int ini_th = 20, min_th = 7;
  LevelGeom lv[kMaxLevels];
  std::vector<CellGeom> cells;
  std::vector<int> xofs, yofs;        // resize source offsets
  std::vector<int16_t> xa, yb;        // resize fixed-point coefficients (pairs)
  int64_t pyr_bytes = 0;              // per image
  int cand_total = 0;                 // per image candidate keys
  int kp_total = 0;                   // per image final keypoint slots
  int node_cap_max = 0;
  float scale[kMaxLevels], inv_scale[kMaxLevels], sigma2[kMaxLevels], inv_sigma2[kMaxLevels];
  int feats[kMaxLevels];
  int umax[kHalfPatch + 1];
};

// Builds every table of a plan; returns ORBX_OK / ORBX_EUNSUPPORTED / ORBX_EINVAL.
int build_geometry(const orbx_params& p, int w, int h, Geometry* g, std::string* why);
// Tables only (no image size): scale factors, sigma2, features per level, umax.
void build_tables(const orbx_params& p, Geometry* g);

#define ORBX_HIP(call)                                       \
  do {                                                       \
    hipError_t e_ = (call);                                  \
    if (e_ != hipSuccess) return orbx::report_hip(e_, #call); \
  } while (0)

int report_hip(hipError_t e, const char* what);

}  // namespace orbx
