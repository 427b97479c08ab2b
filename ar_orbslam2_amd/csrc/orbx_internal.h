// orbx_internal.h — plan geometry and helpers shared by the orbx HIP translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "../../include/orbx.h"

#pragma clang fp contract(off)

namespace orbx {

constexpr int kMaxLevels = 16;
constexpr int kEdge = 19;       // EDGE_THRESHOLD (ORBextractor.cc:71)
constexpr int kPatch = 31;      // PATCH_SIZE (:69)
constexpr int kHalfPatch = 15;  // HALF_PATCH_SIZE (:70)

// Per pyramid level, computed on the host once per plan (ORBextractor.cc:404-460,
// 735-757, 1047-1072).
// k_pyramid: the levels are built in a few stages (one launch each); a stage splits every
// image into row bands, one workgroup per (image, band) builds the stage's levels of its band
// with the band's previous level held in LDS (two ping-pong buffers)
constexpr int kPyBandH = 32;  // source-level rows per band (more if LDS is short)
// plans of at most kPyFewImages images (the drop-in extractor's batch of 1) use short bands:
// more workgroups for one image's latency-chained level builds
constexpr int kPyBandHSmall = 8;
constexpr int kPyFewImages = 4;
constexpr int kPyFewTiles = 128;  // k_pyramid tiles per image at least, few-image plans
constexpr int kPyNT = 512;     // k_pyramid threads per workgroup
// levels per stage (launch): the first from the input, the others from the last level stored;
// with the blur fused, shorter stages (each blurred level's 3-row halo widens the band cones)
constexpr int kPyStage0 = 3, kPyStageN = 4, kPyStage0Fused = 2, kPyStageNFused = 3;
// k_pyramid dynamic LDS bound (both buffers): bands are narrowed until they fit.  40 KB keeps
// four workgroups per CU; the 64 KB this was measured C4's pyramid at 0.76 vs 0.62 ms per 256
// frames (wide 1241-px rows: two workgroups per CU), C2 0.31 vs 0.30 ms (32 KB: C4 0.65,
// 24 KB: more recomputed band cones, C4 0.76).  With the blur fused: 53 KB, three per CU.
constexpr int kPyMaxSmem = 40 * 1024;
constexpr int kPyMaxSmemFused = 53 * 1024;
constexpr int kPyMaxSmemLimit = 64 * 1024;
constexpr int kPyStrip = 4;    // k_pyramid output rows per work item (2: 170, 8: 184 vs 166 us)
// GaussianBlur 7x7 fused into k_pyramid (each band blurs its own rows of the levels it holds in
// LDS) where the bands' recomputed rows stay below kPyFuseMaxRecompute x the level rows (C2, C3
// and the AR path's 640-px frames: 1.27-1.31); wider frames and the drop-in extractor's short
// bands (C4 1.69, C5 3.12, 8-row bands 2.1-2.4) keep the separate k_blur launch.
constexpr bool kPyFused = true;
constexpr double kPyFuseMaxRecompute = 1.4;
constexpr int kPyBlurStrip = 4;  // fused blur: output rows per lane
// column tiles: up to kPyMaxCols per row band, and batch plans' bands up to kPyBandHMul x
// kPyBandH source rows (the tallest that fit the LDS bound)
constexpr int kPyMaxCols = 8;
constexpr int kPyBandHMul = 4;
constexpr int kPyMinGrid = 3072;
// A band is a tile: a range of rows and of 4-column groups of every level of its stage.  Wide
// frames split their rows into several column tiles, so a tile's rows can be many without its
// LDS outgrowing the bound, and the rows and columns the tile recomputes for the next level's
// cone (and the blur's halo) stay a small share of what it owns.
struct PyrBand {
  int lo[kMaxLevels], hi[kMaxLevels];      // rows of each level this band computes (with halo)
  int own_lo[kMaxLevels], own_hi[kMaxLevels];  // rows it writes to the pyramid (a partition)
  int glo[kMaxLevels], ghi[kMaxLevels];    // column groups it computes (-1 / gl + 1: blur pads)
  int own_glo[kMaxLevels], own_ghi[kMaxLevels];  // groups it writes (a partition of 0 .. gl)
  int cb[kMaxLevels];                      // LDS row byte 0 = column cb (a multiple of 16)
  int lp[kMaxLevels];                      // LDS row pitch (a multiple of 16)
};
struct PyrStage {
  int l0, l1;          // builds levels l0..l1 from level l0 - 1 (the input when l0 == 1)
  int band0, nbands;   // its bands in Geometry::bands
  int smem, buf_b;     // LDS bytes, offset of the odd-level buffer
};

struct LevelGeom {
  int w, h;            // level size (cvRound((float)cols * invScale))
  int pitch;           // row pitch in the pyramid / blur blocks (w rounded up to 64 B)
  int64_t pyr_off;     // offset of the level inside one image's pyramid (and blur) block
  int coef_x, coef_y;  // offsets into the k_pyramid tap tables (xtap, ytap entries; levels >= 1)
  int xmax;            // HResizeLinear clamp start (dx >= xmax reads S[x0]*2048)
  int vxs;             // VResizeLinearVec_32s8u SSE2 region: x < vxs
  int bxs;             // SymmColumnVec_32s8u region: x < 4*floor(w/4)
  int cell_begin, ncells;  // range in the cell table
  int wcell, hcell;        // FAST cell size (ORBextractor.cc:755-756)
  int cand_off, cand_cap;  // candidate region (keys) inside one image's candidate block
  int nfeat;               // mnFeaturesPerLevel
  int nini;                // DistributeOctTree initial columns
  float hx;                // (float)(maxX-minX)/nIni; node i spans [(int)(hx*i), (int)(hx*(i+1)))
  int W, H;                // maxX-minX, maxY-minY (octree frame, origin at minBorder=16)
  int node_cap;            // max alive octree nodes: max(N+3, 4*nIni+4)
  int path_x, path_y;      // k_octree's quadrant paths of x in [0, W) and y in [0, H): offsets
                           // into Geometry::octpath
  int kp_off, kp_cap;      // per-image final keypoint slots for this level
  float scale;             // mvScaleFactor
  float size;              // (float)(int)(PATCH_SIZE * scale)
  float inv_scale;         // mvInvScaleFactor
};

struct CellGeom {
  int16_t x0, y0, x1, y1;  // cell image ROI in level coordinates [x0,x1) x [y0,y1)
  int16_t offx, offy;      // j*wCell, i*hCell (ORBextractor.cc:789-790)
  int16_t level, pad16;
  int slot_off, slot_cap;  // candidate slot inside the image's candidate block
  int v_row0;              // offset of the ROI's first detection pixel (x0 + 3, y0 + 3) in the
                           // image's pyramid block
  int pitch;  // a whole aligned dword: k_fast_cells reads the next cell's geometry with scalar
              // loads (an int16 field here became a vector load whose wait it exposed per cell)
};
static_assert(sizeof(CellGeom) == 32, "CellGeom layout");

struct Geometry {
  int w = 0, h = 0, nlevels = 0;
  int ini_th = 20, min_th = 7;
  LevelGeom lv[kMaxLevels];
  std::vector<CellGeom> cells;
  // per level, the DivideNode path of every octree-frame column and row below its initial node
  // (LevelGeom::path_x / path_y): bit 2 (15 - t) (x) or 2 (15 - t) + 1 (y) set when the
  // coordinate lies at or past the depth-t midpoint, so a key's path is path_x[x] | path_y[y]
  std::vector<uint32_t> octpath;
  std::vector<int> xofs, yofs;        // resize source offsets
  std::vector<int16_t> xa, yb;        // resize fixed-point coefficients (pairs)
  // k_pyramid taps, one int32 pair per output column / row: {x0, a0 << 4 | a1 << 20} (past
  // xmax already a0 = 2048, a1 = 0; coefficients in [0, 2049]), every level's column run
  // padded to a multiple of 4 entries; {y0, b0 | b1 << 16}
  std::vector<int32_t> xtap, ytap;
  int64_t pyr_bytes = 0;              // per image
  std::vector<PyrStage> pyr_stages;   // k_pyramid launches, in order
  std::vector<PyrBand> bands;         // every stage's row bands
  int cand_total = 0;                 // per image candidate keys
  int kp_total = 0;                   // per image final keypoint slots
  int node_cap_max = 0;
  bool wide_keys = false;             // an octree frame >= 4096 px: 64-bit candidate keys
  bool blur_fused = false;            // k_pyramid blurs the levels (else the k_blur launch)
  int py_band_h = kPyBandH;           // k_pyramid source rows per band (set before building)
  int py_min_tiles = 1;               // k_pyramid tiles per image and stage, at least (idem)
  float scale[kMaxLevels], inv_scale[kMaxLevels], sigma2[kMaxLevels], inv_sigma2[kMaxLevels];
  int feats[kMaxLevels];
  int umax[kHalfPatch + 1];
};

// Fills n 32-bit words with v on stream s.  Used instead of hipMemsetAsync inside captured
// hipGraphs: a captured memset node of more than 512 KiB left part of its range unwritten on
// the MI355X box (C5 batches of 32 frames: d_match kept stale indices, SearchByBoW's finish
// kernel then read angles out of bounds).
int launch_fill_u32(uint32_t* p, size_t n, uint32_t v, hipStream_t s);

// Builds every table of a plan; returns ORBX_OK / ORBX_EUNSUPPORTED / ORBX_EINVAL.
int build_geometry(const orbx_params& p, int w, int h, Geometry* g, std::string* why);
// Tables only (no image size): scale factors, sigma2, features per level, umax.
void build_tables(const orbx_params& p, Geometry* g);
// The pyramid part of a Geometry for the level sizes already in lv[0 .. nlevels).w / h:
// cv::resize tables, pitches, offsets and k_pyramid stages (shared with the cv::ORB plan).
int build_pyramid(Geometry* g, std::string* why);

// Device tables of k_pyramid / k_blur for one Geometry (orbx_extract.hip), and their launches:
// the pitched pyramid of n dense h x w input images, and its GaussianBlur 7x7 sigma 2 copy.
struct PyrDev {
  LevelGeom* d_lv = nullptr;
  int2 *d_xtap = nullptr, *d_ytap = nullptr;
  PyrBand* d_bands = nullptr;
  void* d_tiles = nullptr;  // BlurTile[ntiles]
  int ntiles = 0;
};
int pyr_kernel_init();
int pyr_dev_create(const Geometry& g, PyrDev* d);
void pyr_dev_destroy(PyrDev* d);
// the pyramid, and with kPyFused its blurred copy (launch_blur is then a no-op)
struct Profiler;
int launch_pyramid(const Geometry& g, const PyrDev& d, const uint8_t* d_in, uint8_t* d_pyr,
                   uint8_t* d_blur, int n, hipStream_t s, Profiler* pr = nullptr, int stage = -1);
int launch_blur(const Geometry& g, const PyrDev& d, const uint8_t* d_pyr, uint8_t* d_blur, int n,
                hipStream_t s);

// Even-point pretest for one pixel per lane (row stride RS of the staged bytes; c = top-left
// byte of the pixel's 7x7 neighbourhood): lane mask of the pixels in ok that may be corners at
// t.  Any 9-arc contains 4 cyclically consecutive even circle points, all darker or all
// brighter; each point's compare is a v_cmp into a lane mask and, with A_k = D_k & D_k+1,
// OR_k A_k & A_k+2 = (A0|A4)&(A2|A6) | (A1|A5)&(A3|A7) runs in the scalar unit.
template <int RS, int CS = 1>
__device__ __forceinline__ uint64_t fast_pretest(const uint8_t* c, int t, uint64_t ok) {
  const int v = c[3 * RS + 3 * CS];
  const int lo = v - t, hi = v + t;
  // even circle points in circle order: (0,3) (2,2) (3,0) (2,-2) (0,-3) (-2,-2) (-3,0) (-2,2)
  const int e[8] = {c[6 * RS + 3 * CS], c[5 * RS + 5 * CS], c[3 * RS + 6 * CS], c[RS + 5 * CS],
                    c[3 * CS],          c[RS + CS],         c[3 * RS],          c[5 * RS + CS]};
  uint64_t pd[8], pb[8], dk[8], bk[8];
#pragma unroll
  for (int k = 0; k < 8; k++) {
    dk[k] = __ballot(e[k] < lo);
    bk[k] = __ballot(e[k] > hi);
  }
#pragma unroll
  for (int k = 0; k < 8; k++) {
    pd[k] = dk[k] & dk[(k + 1) & 7];
    pb[k] = bk[k] & bk[(k + 1) & 7];
  }
  const uint64_t any = ((pd[0] | pd[4]) & (pd[2] | pd[6])) | ((pd[1] | pd[5]) & (pd[3] | pd[7])) |
                       ((pb[0] | pb[4]) & (pb[2] | pb[6])) | ((pb[1] | pb[5]) & (pb[3] | pb[7]));
  return any & ok;
}

// The nine pairs of fast_pretest2 (centre, then the even circle points) from LDS: row r by
// ds_read_u8, row r + 1 by ds_read_u8_d16_hi (the byte lands in bits 16..23; with SRAM ECC on,
// as on MI355X, a d16 load zeroes the other half rather than keeping it, so the two are merged
// by a full-rate v_or instead of loading into one register).  The compiler assembles such pairs
// with a quarter-rate v_perm each.  c must point into LDS.  The v_or needs the d16 load's low
// half to be zero, which holds only with SRAM ECC enabled: the library is built for
// gfx950:sramecc+ (csrc/Makefile), so the loader refuses a device without it instead of this
// reading stale register bits.
template <int RS>
__device__ __forceinline__ void fast_pairs9(const uint8_t* c, uint32_t P[9]) {
  const uint32_t a = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint8_t*)c;
  uint32_t H[9];
  asm volatile(
      "ds_read_u8 %0, %18 offset:%19\n\t"
      "ds_read_u8_d16_hi %9, %18 offset:%28\n\t"
      "ds_read_u8 %1, %18 offset:%20\n\t"
      "ds_read_u8_d16_hi %10, %18 offset:%29\n\t"
      "ds_read_u8 %2, %18 offset:%21\n\t"
      "ds_read_u8_d16_hi %11, %18 offset:%30\n\t"
      "ds_read_u8 %3, %18 offset:%22\n\t"
      "ds_read_u8_d16_hi %12, %18 offset:%31\n\t"
      "ds_read_u8 %4, %18 offset:%23\n\t"
      "ds_read_u8_d16_hi %13, %18 offset:%32\n\t"
      "ds_read_u8 %5, %18 offset:%24\n\t"
      "ds_read_u8_d16_hi %14, %18 offset:%33\n\t"
      "ds_read_u8 %6, %18 offset:%25\n\t"
      "ds_read_u8_d16_hi %15, %18 offset:%34\n\t"
      "ds_read_u8 %7, %18 offset:%26\n\t"
      "ds_read_u8_d16_hi %16, %18 offset:%35\n\t"
      "ds_read_u8 %8, %18 offset:%27\n\t"
      "ds_read_u8_d16_hi %17, %18 offset:%36\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(P[0]), "=&v"(P[1]), "=&v"(P[2]), "=&v"(P[3]), "=&v"(P[4]), "=&v"(P[5]),
        "=&v"(P[6]), "=&v"(P[7]), "=&v"(P[8]), "=&v"(H[0]), "=&v"(H[1]), "=&v"(H[2]),
        "=&v"(H[3]), "=&v"(H[4]), "=&v"(H[5]), "=&v"(H[6]), "=&v"(H[7]), "=&v"(H[8])
      : "v"(a), "i"(3 * RS + 3), "i"(6 * RS + 3), "i"(5 * RS + 5), "i"(3 * RS + 6), "i"(RS + 5),
        "i"(3), "i"(RS + 1), "i"(3 * RS), "i"(5 * RS + 1), "i"(4 * RS + 3), "i"(7 * RS + 3),
        "i"(6 * RS + 5), "i"(4 * RS + 6), "i"(2 * RS + 5), "i"(RS + 3), "i"(2 * RS + 1),
        "i"(4 * RS), "i"(6 * RS + 1)
      : "memory");
#pragma unroll
  for (int k = 0; k < 9; k++) P[k] |= H[k];
}

// The same pretest for two pixels per lane — rows r and r+1 of one column — in the 16-bit
// halves of each dword, on the VALU operations that issue at full rate on gfx950 (32-bit add /
// sub / and / or: 2 cycles per wave instruction where compares, min/max, shifts and packed
// ops take 4; profiles/valu_calibration.json).  With C the centre pair, a circle-point pair E
// and H = 0x80008000 (all values < 2^9, so no half borrows from the other):
//   darker  e < v - t   <=>  bit 15 of each half of  (C + (0x8000 - t - 1)) - E     is set
//   brighter e > v + t  <=>  bit 15 of each half of  (E | H) - (C + t + 1)          is set
// and the arc logic of fast_pretest runs on those flag words with and / or.  Returns the lane
// masks of rows r (low halves) and r+1 (high halves).
// c: the top-left byte (in LDS) of the row-r pixel's 7 x 7 neighbourhood with row stride RS;
// the pairs (row r, row r + 1) come from fast_pairs9.  (A staged row-pair dword layout that
// makes each pair one ds_read_b32 measured slower: 515 vs 392 us per 256 C2 frames, from the
// staging's extra VALU and the halved occupancy of its 23 KB window.)
// Returns the flag word: bit 15 = the row-r pixel may be a corner, bit 31 = the row-r+1 pixel.
template <int RS>
__device__ __forceinline__ uint32_t fast_pretest2(const uint8_t* c, int t) {
  uint32_t P[9];
  fast_pairs9<RS>(c, P);
  const uint32_t C = P[0];
  const uint32_t rep = 0x10001u;
  const uint32_t L = C + (uint32_t)(0x8000 - t - 1) * rep;
  // (E | H) - (C + t + 1) == E - (C + t + 1 - H) (E has no bits at 15 / 31), one dual-issue sub
  const uint32_t K = C + (uint32_t)(t + 1) * rep - 0x80008000u;
  const uint32_t* E = P + 1;
  uint32_t D[8], B[8];
#pragma unroll
  for (int k = 0; k < 8; k++) {
    D[k] = L - E[k];
    B[k] = E[k] - K;
  }
  uint32_t pd[8], pb[8];
#pragma unroll
  for (int k = 0; k < 8; k++) {
    pd[k] = D[k] & D[(k + 1) & 7];
    pb[k] = B[k] & B[(k + 1) & 7];
  }
  return ((pd[0] | pd[4]) & (pd[2] | pd[6])) | ((pd[1] | pd[5]) & (pd[3] | pd[7])) |
         ((pb[0] | pb[4]) & (pb[2] | pb[6])) | ((pb[1] | pb[5]) & (pb[3] | pb[7]));
}

// The five pairs of fast_cardinal2 (centre, then the circle points (0, 3), (3, 0), (0, -3),
// (-3, 0)) from LDS, loaded as fast_pairs9 loads its nine.  c must point into LDS.
template <int RS>
__device__ __forceinline__ void fast_pairs5(const uint8_t* c, uint32_t P[5]) {
  const uint32_t a = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint8_t*)c;
  uint32_t H[5];
  asm volatile(
      "ds_read_u8 %0, %10 offset:%11\n\t"
      "ds_read_u8_d16_hi %5, %10 offset:%16\n\t"
      "ds_read_u8 %1, %10 offset:%12\n\t"
      "ds_read_u8_d16_hi %6, %10 offset:%17\n\t"
      "ds_read_u8 %2, %10 offset:%13\n\t"
      "ds_read_u8_d16_hi %7, %10 offset:%18\n\t"
      "ds_read_u8 %3, %10 offset:%14\n\t"
      "ds_read_u8_d16_hi %8, %10 offset:%19\n\t"
      "ds_read_u8 %4, %10 offset:%15\n\t"
      "ds_read_u8_d16_hi %9, %10 offset:%20\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(P[0]), "=&v"(P[1]), "=&v"(P[2]), "=&v"(P[3]), "=&v"(P[4]), "=&v"(H[0]),
        "=&v"(H[1]), "=&v"(H[2]), "=&v"(H[3]), "=&v"(H[4])
      : "v"(a), "i"(3 * RS + 3), "i"(6 * RS + 3), "i"(3 * RS + 6), "i"(3), "i"(3 * RS),
        "i"(4 * RS + 3), "i"(7 * RS + 3), "i"(4 * RS + 6), "i"(RS + 3), "i"(4 * RS)
      : "memory");
#pragma unroll
  for (int k = 0; k < 5; k++) P[k] |= H[k];
}

// First stage of the per-cell FAST (k_fast_cells): the cardinal-point test on two pixels per
// lane (rows r and r + 1 of one column, 16-bit halves, as fast_pretest2).  Any arc of 9
// consecutive circle points holds two adjacent points of the four at circle indices 0, 4, 8,
// 12, so a FAST-9 corner at t has an adjacent cardinal pair all darker or all brighter:
//   (D0 | D8) & (D4 | D12)  |  (B0 | B8) & (B4 | B12)
// Half the loads and a third of the arithmetic of the even-point test (fast_pretest2) for
// ~1.5x its pass rate; the pixels it passes are scored directly (cornerScore decides).
// Returns bit 15 = the row-r pixel may be a corner at t, bit 31 = the row-r+1 pixel.
template <int RS>
__device__ __forceinline__ uint32_t fast_cardinal2(const uint8_t* c, int t) {
  uint32_t P[5];
  fast_pairs5<RS>(c, P);
  const uint32_t C = P[0];
  const uint32_t rep = 0x10001u;
  const uint32_t L = C + (uint32_t)(0x8000 - t - 1) * rep;
  const uint32_t K = C + (uint32_t)(t + 1) * rep - 0x80008000u;
  uint32_t D[4], B[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    D[k] = L - P[k + 1];
    B[k] = P[k + 1] - K;
  }
  // P[1..4] = circle points 0, 4, 8, 12
  return (((D[0] | D[2]) & (D[1] | D[3])) | ((B[0] | B[2]) & (B[1] | B[3]))) & 0x80008000u;
}

// fast_cardinal2 for two row pairs at once, the second D bytes below the first (D = the step
// between pairs times the row stride): the 20 LDS loads are issued together and waited for once,
// so a wave exposes one LDS latency per two steps.
template <int RS, int D>
__device__ __forceinline__ void fast_cardinal2x2(const uint8_t* c, int t, uint32_t& f0,
                                                 uint32_t& f1) {
  const uint32_t a = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint8_t*)c;
  uint32_t P[10], H[10];
  asm volatile(
      "ds_read_u8 %0, %20 offset:%21\n\t"
      "ds_read_u8_d16_hi %10, %20 offset:%26\n\t"
      "ds_read_u8 %1, %20 offset:%22\n\t"
      "ds_read_u8_d16_hi %11, %20 offset:%27\n\t"
      "ds_read_u8 %2, %20 offset:%23\n\t"
      "ds_read_u8_d16_hi %12, %20 offset:%28\n\t"
      "ds_read_u8 %3, %20 offset:%24\n\t"
      "ds_read_u8_d16_hi %13, %20 offset:%29\n\t"
      "ds_read_u8 %4, %20 offset:%25\n\t"
      "ds_read_u8_d16_hi %14, %20 offset:%30\n\t"
      "ds_read_u8 %5, %20 offset:%31\n\t"
      "ds_read_u8_d16_hi %15, %20 offset:%36\n\t"
      "ds_read_u8 %6, %20 offset:%32\n\t"
      "ds_read_u8_d16_hi %16, %20 offset:%37\n\t"
      "ds_read_u8 %7, %20 offset:%33\n\t"
      "ds_read_u8_d16_hi %17, %20 offset:%38\n\t"
      "ds_read_u8 %8, %20 offset:%34\n\t"
      "ds_read_u8_d16_hi %18, %20 offset:%39\n\t"
      "ds_read_u8 %9, %20 offset:%35\n\t"
      "ds_read_u8_d16_hi %19, %20 offset:%40\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(P[0]), "=&v"(P[1]), "=&v"(P[2]), "=&v"(P[3]), "=&v"(P[4]), "=&v"(P[5]),
        "=&v"(P[6]), "=&v"(P[7]), "=&v"(P[8]), "=&v"(P[9]), "=&v"(H[0]), "=&v"(H[1]),
        "=&v"(H[2]), "=&v"(H[3]), "=&v"(H[4]), "=&v"(H[5]), "=&v"(H[6]), "=&v"(H[7]),
        "=&v"(H[8]), "=&v"(H[9])
      : "v"(a), "i"(3 * RS + 3), "i"(6 * RS + 3), "i"(3 * RS + 6), "i"(3), "i"(3 * RS),
        "i"(4 * RS + 3), "i"(7 * RS + 3), "i"(4 * RS + 6), "i"(RS + 3), "i"(4 * RS),
        "i"(D + 3 * RS + 3), "i"(D + 6 * RS + 3), "i"(D + 3 * RS + 6), "i"(D + 3), "i"(D + 3 * RS),
        "i"(D + 4 * RS + 3), "i"(D + 7 * RS + 3), "i"(D + 4 * RS + 6), "i"(D + RS + 3),
        "i"(D + 4 * RS)
      : "memory");
  const uint32_t rep = 0x10001u;
  uint32_t f[2];
#pragma unroll
  for (int h = 0; h < 2; h++) {
    uint32_t Q[5];
#pragma unroll
    for (int k = 0; k < 5; k++) Q[k] = P[5 * h + k] | H[5 * h + k];
    const uint32_t C = Q[0];
    const uint32_t L = C + (uint32_t)(0x8000 - t - 1) * rep;
    const uint32_t K = C + (uint32_t)(t + 1) * rep - 0x80008000u;
    uint32_t Dk[4], Bk[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      Dk[k] = L - Q[k + 1];
      Bk[k] = Q[k + 1] - K;
    }
    f[h] = (((Dk[0] | Dk[2]) & (Dk[1] | Dk[3])) | ((Bk[0] | Bk[2]) & (Bk[1] | Bk[3]))) & 0x80008000u;
  }
  f0 = f[0];
  f1 = f[1];
}

// rank of this lane among the set lanes of m
__device__ __forceinline__ int lane_rank(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
}

// Cross-lane reductions on DPP moves (no LDS crossbar round trip, unlike __shfl_xor's
// ds_bpermute): quad, half-row and row pairings give every lane of a 16-lane row the row's
// result.  All lanes of the row must be active.
template <int CTRL>
__device__ __forceinline__ int dpp(int v) {
  return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, false);
}
__device__ __forceinline__ int row16_sum(int v) {
  v += dpp<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp<0x141>(v);  // row_half_mirror
  return v + dpp<0x140>(v);  // row_mirror
}
__device__ __forceinline__ uint32_t row16_min(uint32_t v) {
  v = min(v, (uint32_t)dpp<0xB1>((int)v));
  v = min(v, (uint32_t)dpp<0x4E>((int)v));
  v = min(v, (uint32_t)dpp<0x141>((int)v));
  return min(v, (uint32_t)dpp<0x140>((int)v));
}
// Inclusive prefix sum over the 64 lanes on DPP moves (Hillis-Steele within each 16-lane row
// with row_shr 1 / 2 / 4 / 8, then row_bcast 15 / 31 carry the row totals up), instead of six
// ds_bpermute round trips.  Every lane of the wave must be active.
template <int CTRL, int ROWS, bool BOUND>
__device__ __forceinline__ uint32_t dpp0(uint32_t v) {  // DPP move, 0 where there is no source
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWS, 0xF, BOUND);
}
__device__ __forceinline__ int wave_scan_incl(int v) {
  uint32_t u = (uint32_t)v;
  u += dpp0<0x111, 0xF, true>(u);   // row_shr:1
  u += dpp0<0x112, 0xF, true>(u);   // row_shr:2
  u += dpp0<0x114, 0xF, true>(u);   // row_shr:4
  u += dpp0<0x118, 0xF, true>(u);   // row_shr:8
  u += dpp0<0x142, 0xA, false>(u);  // row_bcast:15 into rows 1 and 3
  u += dpp0<0x143, 0xC, false>(u);  // row_bcast:31 into rows 2 and 3
  return (int)u;
}
__device__ __forceinline__ uint64_t wave_scan_incl64(uint64_t v) {
  auto step = [](uint64_t& x, auto mv) {
    x += (uint64_t)mv((uint32_t)x) | ((uint64_t)mv((uint32_t)(x >> 32)) << 32);
  };
  step(v, [](uint32_t w) { return dpp0<0x111, 0xF, true>(w); });
  step(v, [](uint32_t w) { return dpp0<0x112, 0xF, true>(w); });
  step(v, [](uint32_t w) { return dpp0<0x114, 0xF, true>(w); });
  step(v, [](uint32_t w) { return dpp0<0x118, 0xF, true>(w); });
  step(v, [](uint32_t w) { return dpp0<0x142, 0xA, false>(w); });
  step(v, [](uint32_t w) { return dpp0<0x143, 0xC, false>(w); });
  return v;
}

// minimum over the 64 lanes, wave-uniform (the four row minima through readlane)
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
  v = row16_min(v);
  const uint32_t a = __builtin_amdgcn_readlane(v, 0), b = __builtin_amdgcn_readlane(v, 16),
                 c = __builtin_amdgcn_readlane(v, 32), d = __builtin_amdgcn_readlane(v, 48);
  return min(min(a, b), min(c, d));
}

// Wave-local candidate queue: lanes with `pred` append `idx` in lane order (mbcnt rank); every
// lane stores — the others into the wave's 64 spare slots past `spare` (no exec juggling).
// Taking the lane's own predicate (not the lane's bit of the ballot) saves the 64-bit shift,
// and and compare per row.
__device__ __forceinline__ void wave_enqueue(uint16_t* q, int& nq, int spare, bool pred, int idx,
                                             int lane) {
  const uint64_t m = __ballot(pred);
  q[pred ? nq + lane_rank(m) : spare + lane] = (uint16_t)idx;
  nq += __popcll(m);
}

// OpenCV 2.4 cornerScore<16> at (x, y) of a u8 image with row stride `stride`:
// the pixel is a FAST-9/16 corner at threshold t iff the score is >= t.
// With d_k = v - c_k an arc's min d is v - max c and its max d is v - min c, so the score is
// max(v - min_k maxc_k, max_k minc_k - v) - 1 over the 16 arcs of 9 points.  The arc minima run
// on packed pairs (c, 255 - c) giving min c and 255 - max c together, held as the f16 bit
// patterns 0x6400 + c (the halves 1024 + c, exact and ordered like c) so that gfx950's
// three-input v_pk_minimum3_f16 / v_pk_maximum3_f16 apply: runs of 3, then arcs of 3 runs, then
// the maximum over the arcs, 40 packed operations (the u16 two-input form took 80).
typedef _Float16 fast_f16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ fast_f16x2 fast_min3(fast_f16x2 a, fast_f16x2 b, fast_f16x2 c) {
  return __builtin_elementwise_minimum(__builtin_elementwise_minimum(a, b), c);
}
__device__ __forceinline__ fast_f16x2 fast_max3(fast_f16x2 a, fast_f16x2 b, fast_f16x2 c) {
  return __builtin_elementwise_maximum(__builtin_elementwise_maximum(a, b), c);
}
template <int CS = 1>  // bytes per column
__device__ __forceinline__ int fast_score(const uint8_t* s, int stride, int x, int y) {
  const uint8_t* c = s + y * stride + x * CS;
  const int v = c[0];
  const int px[16] = {c[3 * stride],           c[3 * stride + CS],      c[2 * stride + 2 * CS],
                      c[stride + 3 * CS],      c[3 * CS],               c[-stride + 3 * CS],
                      c[-2 * stride + 2 * CS], c[-3 * stride + CS],     c[-3 * stride],
                      c[-3 * stride - CS],     c[-2 * stride - 2 * CS], c[-stride - 3 * CS],
                      c[-3 * CS],              c[stride - 3 * CS],      c[2 * stride - 2 * CS],
                      c[3 * stride - CS]};
  fast_f16x2 p[16], m3[16], a[16];
#pragma unroll
  for (int k = 0; k < 16; k++)  // (0x6400 + c) | (0x6400 + 255 - c) << 16: one v_mad_i32_i24
    p[k] = __builtin_bit_cast(fast_f16x2, (uint32_t)(__mul24(px[k], -65535) + 0x64FF6400));
#pragma unroll
  for (int k = 0; k < 16; k++) m3[k] = fast_min3(p[k], p[(k + 1) & 15], p[(k + 2) & 15]);
#pragma unroll
  for (int k = 0; k < 16; k++) a[k] = fast_min3(m3[k], m3[(k + 3) & 15], m3[(k + 6) & 15]);
  fast_f16x2 r = fast_max3(a[0], a[1], a[2]);
#pragma unroll
  for (int k = 3; k < 15; k += 2) r = fast_max3(r, a[k], a[k + 1]);
  r = __builtin_elementwise_maximum(r, a[15]);
  const uint32_t R = __builtin_bit_cast(uint32_t, r);
  // low half: 0x6400 + max_k (min c over arc k); high half: 0x6400 + 255 - min_k (max c over arc k)
  return max(v + (int)(R >> 16) - (0x6400 + 255), (int)(R & 0xFFFFu) - 0x6400 - v) - 1;
}

// Stage timing with HIP events recorded on the launching stream between kernels.  Marks are
// only read back in collect(), so profiling adds no host synchronisation to the timed loop.
// A stage also records the kernel instances launched for it, under the names rocprofv3 reports
// ("k_pyramid<true>", "k_fast_cells<44, 42, unsigned int>"): launch helpers call note_kernel(),
// which reaches the profiler active on the calling thread (ProfScope), and mark() files the
// names noted since the previous mark under its stage.  bench.py binds a stage's PMC counters to
// exactly these instances.
struct Profiler;
inline thread_local Profiler* t_prof = nullptr;

struct Profiler {
  bool on = false;
  std::vector<std::string> names;
  std::vector<double> ms;
  std::vector<long long> launches;
  std::vector<std::vector<std::string>> kernels;  // per stage: instances launched
  std::vector<std::string> pending;               // noted since the last mark
  std::vector<hipEvent_t> pool;
  size_t used = 0;
  std::vector<std::pair<int, hipEvent_t>> marks;  // stage -1 = segment start
  int stage(const char* name) {
    for (size_t i = 0; i < names.size(); i++)
      if (names[i] == name) return (int)i;
    names.push_back(name);
    ms.push_back(0);
    launches.push_back(0);
    kernels.emplace_back();
    return (int)names.size() - 1;
  }
  void note(const std::string& k) {
    for (const auto& p : pending)
      if (p == k) return;
    pending.push_back(k);
  }
  void mark(hipStream_t s, int st) {
    if (!on) return;
    if (st >= 0 && st < (int)kernels.size())
      for (const auto& k : pending) {
        bool have = false;
        for (const auto& e : kernels[st]) have = have || e == k;
        if (!have) kernels[st].push_back(k);
      }
    pending.clear();
    if (used == pool.size()) {
      hipEvent_t e;
      if (hipEventCreate(&e) != hipSuccess) return;
      pool.push_back(e);
    }
    hipEvent_t e = pool[used++];
    hipEventRecord(e, s);
    marks.push_back({st, e});
    static const bool sync_stages = getenv("ORBX_SYNC_STAGES") != nullptr;
    if (sync_stages) {  // debugging aid: locate the stage of an asynchronous device fault
      const hipError_t err = hipStreamSynchronize(s);
      if (err != hipSuccess)
        fprintf(stderr, "[orbx] stage %s: %s\n", st >= 0 ? names[st].c_str() : "(start)",
                hipGetErrorString(err));
    }
  }
  int collect() {
    if (marks.empty()) return 0;
    if (hipEventSynchronize(marks.back().second) != hipSuccess) return -3;
    for (size_t i = 1; i < marks.size(); i++) {
      if (marks[i].first < 0) continue;
      float t = 0;
      hipEventElapsedTime(&t, marks[i - 1].second, marks[i].second);
      ms[marks[i].first] += t;
      launches[marks[i].first] += 1;
    }
    marks.clear();
    used = 0;
    return 0;
  }
  void reset() {
    marks.clear();
    used = 0;
    pending.clear();
    for (auto& m : ms) m = 0;
    for (auto& l : launches) l = 0;
    for (auto& k : kernels) k.clear();
  }
  // the stage's instances, ';'-separated, into buf (cap bytes, NUL-terminated): 0, -1 on a
  // bad argument, 1 when the list does not fit (buf then holds the empty string, never a cut
  // name)
  int kernels_of(int st, char* buf, int cap) const {
    if (st < 0 || st >= (int)kernels.size() || !buf || cap <= 0) return -1;
    std::string j;
    for (const auto& k : kernels[st]) j += (j.empty() ? "" : ";") + k;
    if (j.size() + 1 > (size_t)cap) {
      buf[0] = 0;
      return 1;
    }
    memcpy(buf, j.data(), j.size());
    buf[j.size()] = 0;
    return 0;
  }
  ~Profiler() {
    for (auto e : pool) hipEventDestroy(e);
  }
};

// Makes `pr` the thread's active profiler for the enclosing enqueue (nested enqueues of the same
// or another profiler restore the outer one); inactive unless pr.on.
struct ProfScope {
  Profiler* prev;
  explicit ProfScope(Profiler& pr) : prev(t_prof) {
    if (pr.on) t_prof = &pr;
  }
  ~ProfScope() { t_prof = prev; }
};
inline void note_kernel(const char* k) {
  if (t_prof) t_prof->note(k);
}
template <class K>
inline void note_kernel(const char* base, const char* args_before = "") {
  if (!t_prof) return;
  // rocprofv3's demangled template arguments: uint32_t "unsigned int", uint64_t "unsigned long"
  const char* kt = sizeof(K) == 8 ? "unsigned long" : "unsigned int";
  t_prof->note(std::string(base) + "<" + args_before + kt + ">");
}

#define ORBX_HIP(call)                                       \
  do {                                                       \
    hipError_t e_ = (call);                                  \
    if (e_ != hipSuccess) return orbx::report_hip(e_, #call); \
  } while (0)

int report_hip(hipError_t e, const char* what);
// Waits for a stream's work on the one-call (drop-in) paths: polls hipStreamQuery for up to
// ORBX_SPIN_US microseconds (default 2000; 0 = block at once) before a blocking
// hipStreamSynchronize — a blocking wait adds the runtime's interrupt wake-up latency to every
// call, which for calls whose GPU work takes ~50-200 us is a large share.
hipError_t wait_stream(hipStream_t s);
// logs a library-detected error (stderr) and returns `code`
int report(int code, const char* what);

// Process-wide lock around device resource changes (allocation, free, stream / symbol setup)
// and stream capture.  ROCm may synchronise the device inside hipMalloc / hipFree, which
// invalidates a capture running in another thread (hipErrorStreamCaptureInvalidated, seen with
// several extractors on several host threads); captures and allocations therefore never
// overlap.  Recursive: create functions call other create functions.
std::recursive_mutex& resource_mutex();
#define ORBX_RESOURCE_LOCK std::lock_guard<std::recursive_mutex> orbx_res_lock_(orbx::resource_mutex())

// Executable graphs of one stream, keyed by (input pointer, batch): a caller that alternates
// input buffers replays one graph per buffer instead of re-capturing.  Graphs are destroyed
// only after the stream has drained (an exec may still be running).
struct GraphCache {
  struct Entry {
    const void* in;
    int n;
    hipGraphExec_t exec;
  };
  std::vector<Entry> e;
  static constexpr size_t kMax = 8;
  hipGraphExec_t find(const void* in, int n) const {
    for (const Entry& x : e)
      if (x.in == in && x.n == n) return x.exec;
    return nullptr;
  }
  void clear(hipStream_t s) {
    if (e.empty()) return;
    ORBX_RESOURCE_LOCK;
    if (s) (void)hipStreamSynchronize(s);
    for (Entry& x : e) (void)hipGraphExecDestroy(x.exec);
    e.clear();
  }
  void add(const void* in, int n, hipGraphExec_t exec, hipStream_t s) {
    if (e.size() >= kMax) clear(s);
    e.push_back({in, n, exec});
  }
};

// Captures what `enqueue()` puts on stream s into an executable graph; the partial graph of a
// failed enqueue is destroyed.
template <class Fn>
int capture_graph(hipStream_t s, Fn&& enqueue, hipGraphExec_t* out) {
  ORBX_RESOURCE_LOCK;
  hipGraph_t gr = nullptr;
  hipError_t e = hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
  if (e != hipSuccess) return report_hip(e, "hipStreamBeginCapture");
  const int rc = enqueue();
  e = hipStreamEndCapture(s, &gr);
  if (rc != ORBX_OK) {
    if (e == hipSuccess && gr) (void)hipGraphDestroy(gr);
    return rc;
  }
  if (e != hipSuccess) return report_hip(e, "hipStreamEndCapture");
  e = hipGraphInstantiate(out, gr, nullptr, nullptr, 0);
  (void)hipGraphDestroy(gr);
  return e == hipSuccess ? ORBX_OK : report_hip(e, "hipGraphInstantiate");
}

// Replays the cached graph of (in, n) on s, capturing it first if needed.
template <class Fn>
int run_graph(GraphCache& cache, hipStream_t s, const void* in, int n, Fn&& enqueue) {
  hipGraphExec_t exec = cache.find(in, n);
  if (!exec) {
    const int rc = capture_graph(s, enqueue, &exec);
    if (rc != ORBX_OK) return rc;
    cache.add(in, n, exec, s);
  }
  const hipError_t e = hipGraphLaunch(exec, s);
  return e == hipSuccess ? ORBX_OK : report_hip(e, "hipGraphLaunch");
}

// Internal plan access for the frame pipeline (orbx_frames.hip).
struct PlanView {
  const Geometry* g;
  hipStream_t stream;
  orbx_keypoint* d_kps;
  uint8_t* d_desc;
  int* d_counts;
  int kp_total;
  int max_batch;
  const uint8_t* d_pyr;   // [max_batch][pyr_bytes] pitched raw pyramid (mvImagePyramid)
  int64_t pyr_bytes;
  const LevelGeom* d_lv;  // [nlevels] device copy of g->lv
};
int plan_view(orbx_plan* P, PlanView* v);
int plan_enqueue(orbx_plan* P, const uint8_t* d_in, int n, Profiler* prof);
// one allocation holds counts [max_batch] at 0, keypoints at kps_off, descriptors at desc_off
int plan_output_block(const orbx_plan* P, size_t* kps_off, size_t* desc_off, size_t* bytes);

}  // namespace orbx
