// orbx_extract.hip — gfx950 kernels and batch plan for ORBextractor::operator()
// (ORB_SLAM2/src/ORBextractor.cc:985-1072).
//
// One plan = one image size + one parameter set + a maximum batch.  A batch of images runs
// as a fixed launch sequence on the plan's stream (captured once into a hipGraph):
//   k_resize      x (nlevels-1)  pyramid level l from level l-1     (cv::resize INTER_LINEAR)
//   k_blur        x 1            all levels, 64x16 LDS tiles         (GaussianBlur 7x7 s=2)
//   k_fast_score  x 1            64x16 tiles, all levels            (FAST score map)
//   k_fast_nms    x 1            one wave per FAST cell             (cv::FAST NMS + cell fallback)
//   k_octree      x 1            one workgroup per (image, level)    (DistributeOctTree)
//   k_describe    x 1            one wave per keypoint               (IC_Angle + rBRIEF)
// Level 0 is read in place from the caller's input buffer; levels >= 1 live in the pyramid
// block.  Everything is integer or bit-exact float (see orbx_math.h); compiled with
// -ffp-contract=off.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/orbx_pattern.h"
#include "orbx_internal.h"
#include "orbx_math.h"

#pragma clang fp contract(off)

namespace orbx {

__constant__ int8_t c_pattern[1024];
__constant__ int c_umax[kHalfPatch + 1];

// ------------------------------------------------------------------ helpers
// Every level (level 0 copied in by k_copy0) lives in the image's pitched pyramid block.
__device__ __forceinline__ const uint8_t* level_base(const uint8_t* pyr, int64_t pyr_bytes,
                                                     const LevelGeom& g, int img) {
  return pyr + (int64_t)img * pyr_bytes + g.pyr_off;
}

__device__ __forceinline__ int reflect101(int p, int len) {
  if (len == 1) return 0;
  while (p < 0 || p >= len) {
    if (p < 0) p = -p;
    if (p >= len) p = 2 * len - p - 2;
  }
  return p;
}

template <int NT>
__device__ int block_sum(int v, int* s_tmp) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) s_tmp[wid] = v;
  __syncthreads();
  int t = 0;
#pragma unroll
  for (int w = 0; w < NT / 64; w++) t += s_tmp[w];
  __syncthreads();
  return t;
}

// Exclusive scan of a[0..M) in place (LDS array), chunked per thread so the scan is stable.
template <int NT>
__device__ int block_scan_excl(int* a, int M, int* s_tmp) {
  const int per = (M + NT - 1) / NT;
  const int t = threadIdx.x;
  const int beg = min(t * per, M), end = min(beg + per, M);
  int sum = 0;
  for (int i = beg; i < end; i++) sum += a[i];
  const int lane = t & 63, wid = t >> 6;
  int v = sum;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int n = __shfl_up(v, off);
    if (lane >= off) v += n;
  }
  __syncthreads();
  if (lane == 63) s_tmp[wid] = v;
  __syncthreads();
  if (t == 0) {
    int acc = 0;
    for (int w = 0; w < NT / 64; w++) {
      const int x = s_tmp[w];
      s_tmp[w] = acc;
      acc += x;
    }
    s_tmp[NT / 64] = acc;
  }
  __syncthreads();
  int run = s_tmp[wid] + v - sum;
  for (int i = beg; i < end; i++) {
    const int x = a[i];
    a[i] = run;
    run += x;
  }
  const int total = s_tmp[NT / 64];
  __syncthreads();
  return total;
}

// ------------------------------------------------------------------ k_copy0
// Level 0 = the input image (ComputePyramid level 0, ORBextractor.cc:1066-1068) copied into the
// 64-B pitched pyramid block so every later kernel reads aligned dwords.
__global__ __launch_bounds__(256) void k_copy0(const uint8_t* __restrict__ in,
                                               uint8_t* __restrict__ pyr, int64_t pyr_bytes,
                                               const LevelGeom* __restrict__ lv) {
  const LevelGeom& G = lv[0];
  const int img = blockIdx.z, y = blockIdx.y;
  const int x4 = (blockIdx.x * 256 + threadIdx.x) * 4;
  if (x4 >= G.w) return;
  const uint8_t* src = in + ((int64_t)img * G.h + y) * G.w + x4;
  uint32_t v = src[0];
  if (x4 + 1 < G.w) v |= (uint32_t)src[1] << 8;
  if (x4 + 2 < G.w) v |= (uint32_t)src[2] << 16;
  if (x4 + 3 < G.w) v |= (uint32_t)src[3] << 24;
  *(uint32_t*)(pyr + (int64_t)img * pyr_bytes + G.pyr_off + (int64_t)y * G.pitch + x4) = v;
}

// ------------------------------------------------------------------ k_resize
// cv::resize(level l-1 ROI -> level l ROI, INTER_LINEAR), 8UC1 fixed point:
// horizontal taps Q11 ints, vertical pass = SSE2 mulhi form for x < vxs, scalar
// (H0*b0 + H1*b1 + 2^21) >> 22 tail.  One thread per 4 output pixels (one aligned dword
// store); the two source rows of level l-1 are L2 resident (written by the previous launch).
__device__ __forceinline__ int resize_px(const uint8_t* r0, const uint8_t* r1, int dx,
                                         const LevelGeom& D, const int* __restrict__ xofs,
                                         const int16_t* __restrict__ xa, int b0, int b1) {
  const int x0 = xofs[D.coef_x + dx];
  int h0, h1;
  if (dx < D.xmax) {
    const int a0 = xa[2 * (D.coef_x + dx)], a1 = xa[2 * (D.coef_x + dx) + 1];
    h0 = r0[x0] * a0 + r0[x0 + 1] * a1;
    h1 = r1[x0] * a0 + r1[x0 + 1] * a1;
  } else {
    h0 = r0[x0] * 2048;
    h1 = r1[x0] * 2048;
  }
  int v;
  if (dx < D.vxs) {
    const int t0 = max(-32768, min(32767, h0 >> 4));
    const int t1 = max(-32768, min(32767, h1 >> 4));
    int m = ((t0 * b0) >> 16) + ((t1 * b1) >> 16);
    m = max(-32768, min(32767, m));
    m = max(-32768, min(32767, m + 2));
    v = m >> 2;
  } else {
    v = (h0 * b0 + h1 * b1 + (1 << 21)) >> 22;
  }
  return max(0, min(255, v));
}

__global__ __launch_bounds__(256) void k_resize(uint8_t* __restrict__ pyr, int64_t pyr_bytes,
                                                const LevelGeom* __restrict__ lv, int level,
                                                const int* __restrict__ xofs,
                                                const int16_t* __restrict__ xa,
                                                const int* __restrict__ yofs,
                                                const int16_t* __restrict__ yb) {
  const LevelGeom& D = lv[level];
  const LevelGeom& S = lv[level - 1];
  const int img = blockIdx.z, dy = blockIdx.y;
  const int dx0 = (blockIdx.x * 256 + threadIdx.x) * 4;
  if (dx0 >= D.w) return;
  const uint8_t* src = level_base(pyr, pyr_bytes, S, img);
  uint8_t* dst = pyr + (int64_t)img * pyr_bytes + D.pyr_off;
  const int sy0 = yofs[D.coef_y + dy];
  const int ya = sy0 >= 0 ? (sy0 < S.h ? sy0 : S.h - 1) : 0;
  const int yb1 = sy0 + 1 >= 0 ? (sy0 + 1 < S.h ? sy0 + 1 : S.h - 1) : 0;
  const uint8_t* r0 = src + (int64_t)ya * S.pitch;
  const uint8_t* r1 = src + (int64_t)yb1 * S.pitch;
  const int b0 = yb[2 * (D.coef_y + dy)], b1 = yb[2 * (D.coef_y + dy) + 1];
  uint32_t out = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int dx = dx0 + k;
    if (dx < D.w) out |= (uint32_t)resize_px(r0, r1, dx, D, xofs, xa, b0, b1) << (8 * k);
  }
  // pitch is a multiple of 64, so the padding bytes of the last dword are in the row's pad
  *(uint32_t*)(dst + (int64_t)dy * D.pitch + dx0) = out;
}

// ------------------------------------------------------------------ k_blur
// GaussianBlur(level, 7x7, sigma 2, BORDER_REFLECT_101) in OpenCV 2.4's 8U fixed point
// (SURVEY A.4): integer row pass with taps [18,34,49,55,49,34,18], column pass rounded
// half-even (SSE2 f32 region x < 4*floor(w/4)) or half-up (scalar tail).  Values below 256
// are exact in f32, so half-even rounding of m/65536 is done on the integer m.
// Tile 64 x 32 outputs: interior tiles stage the (32+6) x 72 input window with aligned dword
// loads, border tiles byte-wise through reflect101; every thread then produces 4 adjacent
// row sums (ds_write_b128) and 4 adjacent outputs (7 x ds_read_b128, one dword store).
constexpr int kBlurTW = 64, kBlurTH = 32;
struct BlurTile {
  int16_t level, tx, ty, interior;
};

__global__ __launch_bounds__(256) void k_blur(const uint8_t* __restrict__ pyr, int64_t pyr_bytes,
                                              uint8_t* __restrict__ blur,
                                              const LevelGeom* __restrict__ lv,
                                              const BlurTile* __restrict__ tiles) {
  __shared__ __align__(16) uint32_t s_in[kBlurTH + 6][(kBlurTW + 8) / 4];
  __shared__ __align__(16) int s_row[kBlurTH + 6][kBlurTW];
  const BlurTile T = tiles[blockIdx.x];
  const int img = blockIdx.y;
  const LevelGeom& G = lv[T.level];
  const uint8_t* src = level_base(pyr, pyr_bytes, G, img);
  uint8_t* dst = blur + (int64_t)img * pyr_bytes + G.pyr_off;
  const int X0 = T.tx * kBlurTW, Y0 = T.ty * kBlurTH;
  const int tid = threadIdx.x;
  constexpr int kWords = (kBlurTW + 8) / 4;  // window columns X0-4 .. X0+67
  if (T.interior) {
    for (int i = tid; i < (kBlurTH + 6) * kWords; i += 256) {
      const int r = i / kWords, c = i - r * kWords;
      s_in[r][c] = *(const uint32_t*)(src + (int64_t)(Y0 + r - 3) * G.pitch + X0 - 4 + 4 * c);
    }
  } else {
    uint8_t* sb = (uint8_t*)s_in;
    for (int i = tid; i < (kBlurTH + 6) * (kBlurTW + 8); i += 256) {
      const int r = i / (kBlurTW + 8), c = i - r * (kBlurTW + 8);
      const int y = reflect101(min(Y0 + r - 3, G.h + 8), G.h);
      const int x = reflect101(min(X0 + c - 4, G.w + 8), G.w);
      sb[r * (kBlurTW + 8) + c] = src[(int64_t)y * G.pitch + x];
    }
  }
  __syncthreads();
  const int k0 = 18, k1 = 34, k2 = 49, k3 = 55;
  for (int i = tid; i < (kBlurTH + 6) * (kBlurTW / 4); i += 256) {
    const int r = i / (kBlurTW / 4), q = i - r * (kBlurTW / 4);
    // bytes X0+4q-4 .. X0+4q+7 of row r
    const uint32_t w0 = s_in[r][q], w1 = s_in[r][q + 1], w2 = s_in[r][q + 2];
    int b[12];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      b[k] = (w0 >> (8 * k)) & 0xFF;
      b[4 + k] = (w1 >> (8 * k)) & 0xFF;
      b[8 + k] = (w2 >> (8 * k)) & 0xFF;
    }
    int4 o;
    o.x = k0 * (b[1] + b[7]) + k1 * (b[2] + b[6]) + k2 * (b[3] + b[5]) + k3 * b[4];
    o.y = k0 * (b[2] + b[8]) + k1 * (b[3] + b[7]) + k2 * (b[4] + b[6]) + k3 * b[5];
    o.z = k0 * (b[3] + b[9]) + k1 * (b[4] + b[8]) + k2 * (b[5] + b[7]) + k3 * b[6];
    o.w = k0 * (b[4] + b[10]) + k1 * (b[5] + b[9]) + k2 * (b[6] + b[8]) + k3 * b[7];
    *(int4*)&s_row[r][4 * q] = o;
  }
  __syncthreads();
  for (int i = tid; i < kBlurTH * (kBlurTW / 4); i += 256) {
    const int r = i / (kBlurTW / 4), q = i - r * (kBlurTW / 4);
    const int x = X0 + 4 * q, y = Y0 + r;
    if (x >= G.w || y >= G.h) continue;
    int4 R[7];
#pragma unroll
    for (int k = 0; k < 7; k++) R[k] = *(const int4*)&s_row[r + k][4 * q];
    int m[4];
    m[0] = k0 * (R[0].x + R[6].x) + k1 * (R[1].x + R[5].x) + k2 * (R[2].x + R[4].x) + k3 * R[3].x;
    m[1] = k0 * (R[0].y + R[6].y) + k1 * (R[1].y + R[5].y) + k2 * (R[2].y + R[4].y) + k3 * R[3].y;
    m[2] = k0 * (R[0].z + R[6].z) + k1 * (R[1].z + R[5].z) + k2 * (R[2].z + R[4].z) + k3 * R[3].z;
    m[3] = k0 * (R[0].w + R[6].w) + k1 * (R[1].w + R[5].w) + k2 * (R[2].w + R[4].w) + k3 * R[3].w;
    uint32_t out = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      int v;
      if (x + k < G.bxs) {
        const int qv = m[k] >> 16, rem = m[k] & 0xFFFF;  // m >= 0
        v = qv + (rem > 0x8000 || (rem == 0x8000 && (qv & 1)));
      } else {
        v = (m[k] + 32768) >> 16;
      }
      out |= (uint32_t)min(255, v) << (8 * k);
    }
    *(uint32_t*)(dst + (int64_t)y * G.pitch + x) = out;  // bytes past w land in the row pad
  }
}

// ------------------------------------------------------------------ k_fast_cells
// One workgroup per FAST cell of ComputeKeyPointsOctTree (ORBextractor.cc:758-796): cv::FAST
// with NMS on the cell ROI at iniThFAST, again at minThFAST when no keypoint survives, then an
// order-preserving (raster) compaction into the cell's candidate slot.  Score = OpenCV 2.4
// cornerScore<16>; V = score+1 clamped to [0,255] so "corner at t" is V > t.
constexpr int kCellMax = 66;  // wCell, hCell < 60 (+6)

__device__ __forceinline__ int fast_score(const uint8_t* s, int stride, int x, int y) {
  const uint8_t* c = s + y * stride + x;
  const int v = c[0];
  int d[16];
  d[0] = v - c[3 * stride];
  d[1] = v - c[3 * stride + 1];
  d[2] = v - c[2 * stride + 2];
  d[3] = v - c[stride + 3];
  d[4] = v - c[3];
  d[5] = v - c[-stride + 3];
  d[6] = v - c[-2 * stride + 2];
  d[7] = v - c[-3 * stride + 1];
  d[8] = v - c[-3 * stride];
  d[9] = v - c[-3 * stride - 1];
  d[10] = v - c[-2 * stride - 2];
  d[11] = v - c[-stride - 3];
  d[12] = v - c[-3];
  d[13] = v - c[stride - 3];
  d[14] = v - c[2 * stride - 2];
  d[15] = v - c[3 * stride - 1];
  // sliding min/max over 9 consecutive circle points (wrap-around)
  int mn2[16], mx2[16];
#pragma unroll
  for (int k = 0; k < 16; k++) {
    mn2[k] = min(d[k], d[(k + 1) & 15]);
    mx2[k] = max(d[k], d[(k + 1) & 15]);
  }
  int mn4[16], mx4[16];
#pragma unroll
  for (int k = 0; k < 16; k++) {
    mn4[k] = min(mn2[k], mn2[(k + 2) & 15]);
    mx4[k] = max(mx2[k], mx2[(k + 2) & 15]);
  }
  int q0 = -1000, q1 = 1000;
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const int a = min(min(mn4[k], mn4[(k + 4) & 15]), d[(k + 8) & 15]);
    const int b = max(max(mx4[k], mx4[(k + 4) & 15]), d[(k + 8) & 15]);
    q0 = max(q0, a);
    q1 = min(q1, b);
  }
  return max(q0, -q1) - 1;
}

__device__ __forceinline__ bool nms_keep(const uint8_t* V, int vs, int p, int t) {
  const int v = V[p];
  if (v <= t) return false;
  const int s = v - 1;
  const int nb[8] = {p - vs - 1, p - vs, p - vs + 1, p - 1, p + 1, p + vs - 1, p + vs, p + vs + 1};
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const int q = V[nb[k]];
    const int nq = q > t ? q - 1 : 0;
    if (!(s > nq)) return false;
  }
  return true;
}

// Necessary condition for "corner at t" (9 contiguous darker/brighter): two consecutive
// quarter points of the circle (0,4,8,12) both darker or both brighter.
__device__ __forceinline__ bool fast_maybe(const uint8_t* s, int stride, int x, int y, int t) {
  const uint8_t* c = s + y * stride + x;
  const int v = c[0];
  const int p0 = c[3 * stride], p4 = c[3], p8 = c[-3 * stride], p12 = c[-3];
  const int lo = v - t, hi = v + t;
  const bool d0 = p0 < lo, d4 = p4 < lo, d8 = p8 < lo, d12 = p12 < lo;
  const bool b0 = p0 > hi, b4 = p4 > hi, b8 = p8 > hi, b12 = p12 > hi;
  return ((d0 & d4) | (d4 & d8) | (d8 & d12) | (d12 & d0)) |
         ((b0 & b4) | (b4 & b8) | (b8 & b12) | (b12 & b0));
}

// ---- k_fast_score: FAST score map V = clamp(cornerScore+1, 0, 255) of every pixel of the
// detection region [19, w-19) x [19, h-19) of every level (0 elsewhere).  A pixel that fails the
// quarter-point test at min(iniThFAST, minThFAST) cannot be a corner at either threshold, so
// its V (<= threshold) is equivalent to 0 in every NMS; only candidates get the full score.
// Tile 64 x 64: aligned-dword staging of the (64+6) x 72 window, then per wave 16 rows, a
// wave-local queue of candidates (ballot + mbcnt, no block barrier) scored 64 at a time.
constexpr int kFastTW = 64, kFastTH = 64;
struct FastTile {
  int16_t level, tx, ty, pad;
};

__global__ __launch_bounds__(256) void k_fast_score(const uint8_t* __restrict__ pyr,
                                                    int64_t pyr_bytes,
                                                    uint8_t* __restrict__ vmap,
                                                    const LevelGeom* __restrict__ lv,
                                                    const FastTile* __restrict__ tiles, int t_lo) {
  constexpr int kW = (kFastTW + 8) / 4;  // dwords per staged row: X0-4 .. X0+67
  __shared__ __align__(16) uint32_t s_in[kFastTH + 6][kW];
  __shared__ __align__(16) uint8_t s_v[kFastTH][kFastTW];
  __shared__ uint16_t s_q[4][(kFastTH / 4) * 64];
  const FastTile T = tiles[blockIdx.x];
  const int img = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const LevelGeom& G = lv[T.level];
  const uint8_t* src = level_base(pyr, pyr_bytes, G, img);
  const int X0 = T.tx * kFastTW, Y0 = T.ty * kFastTH;
  for (int i = tid; i < (kFastTH + 6) * kW; i += 256) {
    const int r = i / kW, c = i - r * kW;
    const int y = min(max(Y0 + r - 3, 0), G.h - 1);
    const int x = X0 - 4 + 4 * c;
    s_in[r][c] = (x >= 0 && x + 4 <= G.pitch) ? *(const uint32_t*)(src + (int64_t)y * G.pitch + x)
                                              : 0u;
  }
  __syncthreads();
  const uint8_t* sb = (const uint8_t*)s_in;
  constexpr int SB = kW * 4;  // staged row stride in bytes
  const int x = X0 + lane;
  const bool xin = x >= kEdge && x < G.w - kEdge;
  uint16_t* q = s_q[wid];
  int nq = 0;
#pragma unroll 4
  for (int rr = 0; rr < kFastTH / 4; rr++) {
    const int r = wid * (kFastTH / 4) + rr, y = Y0 + r;
    s_v[r][lane] = 0;
    const bool f = xin && y >= kEdge && y < G.h - kEdge &&
                   fast_maybe(sb, SB, lane + 4, r + 3, t_lo);
    const uint64_t m = __ballot(f);
    const int rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                               __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
    if (f) q[nq + rank] = (uint16_t)((r << 6) | lane);
    nq += __popcll(m);
  }
  for (int i0 = 0; i0 < nq; i0 += 64) {
    const int i = i0 + lane;
    if (i < nq) {
      const int e = q[i], r = e >> 6, c = e & 63;
      const int sc = fast_score(sb, SB, c + 4, r + 3);
      s_v[r][c] = (uint8_t)min(255, max(0, sc + 1));
    }
  }
  __syncthreads();
  for (int i = tid; i < kFastTH * (kFastTW / 4); i += 256) {
    const int r = i >> 4, c4 = (i & 15) * 4;  // kFastTH rows x 16 dwords
    const int y = Y0 + r;
    if (y < G.h && X0 + c4 < G.pitch)
      *(uint32_t*)(vmap + (int64_t)img * pyr_bytes + G.pyr_off + (int64_t)y * G.pitch + X0 + c4) =
          *(const uint32_t*)&s_v[r][c4];
  }
}

// ---- k_fast_nms: cv::FAST's strict 8-neighbour NMS restricted to each cell's detection
// region (neighbours outside it count as 0), survivors at iniThFAST, else at minThFAST
// (ORBextractor.cc:776-784), raster-ordered compaction into the cell's candidate slot.
// One wave per cell; the cell's V window (<= 62 x 62) is staged in LDS with the ring zeroed.
__global__ __launch_bounds__(256) void k_fast_nms(const uint8_t* __restrict__ vmap,
                                                  int64_t pyr_bytes,
                                                  const LevelGeom* __restrict__ lv,
                                                  const CellGeom* __restrict__ cells, int ncells,
                                                  int ini_th, int min_th,
                                                  uint32_t* __restrict__ cand, int cand_total,
                                                  int* __restrict__ cell_counts) {
  constexpr int VS = kCellMax - 2;  // 64 >= dc + 2
  __shared__ uint8_t s_w[4][(kCellMax - 4) * VS];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int ci = blockIdx.x * 4 + wid, img = blockIdx.y;
  if (ci >= ncells) return;
  const CellGeom C = cells[ci];
  const LevelGeom& G = lv[C.level];
  const int dr = C.y1 - C.y0 - 6, dc = C.x1 - C.x0 - 6;
  int* cnt_out = cell_counts + (int64_t)img * ncells + ci;
  if (dr <= 0 || dc <= 0) {
    if (lane == 0) *cnt_out = 0;
    return;
  }
  uint8_t* W = s_w[wid];
  const uint8_t* V = vmap + (int64_t)img * pyr_bytes + G.pyr_off +
                     (int64_t)(C.y0 + 3) * G.pitch + C.x0 + 3;
  // W[(r+1)*VS + c+1] = V at detection pixel (r, c); the ring is 0 (cell-local NMS)
  for (int i = lane; i < (dr + 2) * VS; i += 64) W[i] = 0;
  const int npix = dr * dc;
  const float rdc = 1.0f / (float)dc;  // (p + 0.5) / dc is never within 1/120 of an integer
  constexpr int U = 8;
  for (int b = 0; b < npix; b += 64 * U) {
    uint8_t v[U];
    int wi[U];
#pragma unroll
    for (int k = 0; k < U; k++) {  // issue every load of the batch before any LDS store
      const int p = b + k * 64 + lane;
      wi[k] = -1;
      v[k] = 0;
      if (p < npix) {
        const int r = (int)(((float)p + 0.5f) * rdc), c = p - r * dc;
        wi[k] = (r + 1) * VS + c + 1;
        v[k] = V[(int64_t)r * G.pitch + c];
      }
    }
#pragma unroll
    for (int k = 0; k < U; k++)
      if (wi[k] >= 0) W[wi[k]] = v[k];
  }
  // survivors at iniThFAST, in raster order = flattened order; keep bits per iteration
  const int iters = (npix + 63) >> 6;  // <= 57
  uint64_t kb = 0;
  int total = 0;
  for (int it = 0; it < iters; it++) {
    const int p = it * 64 + lane;
    bool k = false;
    if (p < npix) {
      const int r = (int)(((float)p + 0.5f) * rdc), c = p - r * dc;
      k = nms_keep(W, VS, (r + 1) * VS + c + 1, ini_th);
    }
    kb |= (uint64_t)k << it;
    total += __popcll(__ballot(k));
  }
  const int t = ini_th;
  uint32_t* out = cand + (int64_t)img * cand_total + C.slot_off;
  int nout = 0;
  const bool redo = total == 0 && min_th != ini_th;  // ORBextractor.cc:780-784
  for (int it = 0; it < iters; it++) {
    const int p = it * 64 + lane;
    int r = 0, c = 0;
    bool k = (kb >> it) & 1;
    if (p < npix) {
      r = (int)(((float)p + 0.5f) * rdc);
      c = p - r * dc;
      if (redo) k = nms_keep(W, VS, (r + 1) * VS + c + 1, min_th);
    }
    const uint64_t m = __ballot(k);
    if (k) {
      const int rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
      const uint32_t x = (uint32_t)(c + 3 + C.offx), y = (uint32_t)(r + 3 + C.offy);
      out[nout + rank] = x | (y << 12) | ((uint32_t)(W[(r + 1) * VS + c + 1] - 1) << 24);
    }
    nout += __popcll(m);
  }
  (void)t;
  if (lane == 0) *cnt_out = nout;
}

// ------------------------------------------------------------------ k_octree
// ORBextractor::DistributeOctTree (ORBextractor.cc:525-733) for one (image, level) per
// workgroup.  The std::list is represented by node arrays kept in list order in LDS:
// a division pass pushes children to the front, so after each step the order is
// [children, newest seq first] + [undivided nodes, previous order].  Keys keep
// candidate order inside every node (DivideNode is a stable partition), so a node's retained
// key is its max response with the lowest candidate index.  The final-refinement sort uses the
// canonical (size, creation sequence) tie-break.
constexpr int kOctNT = 256;

struct OctNodes {
  int16_t *x0, *x1, *y0, *y1;
  int *cnt, *seq;
};

__device__ __forceinline__ int quad_of(uint32_t key, int x0, int x1, int y0, int y1) {
  const int x = key & 0xFFF, y = (key >> 12) & 0xFFF;
  const int xm = x0 + (x1 - x0 + 1) / 2;  // ceil((float)(UR.x-UL.x)/2)
  const int ym = y0 + (y1 - y0 + 1) / 2;
  return x < xm ? (y < ym ? 0 : 2) : (y < ym ? 1 : 3);
}

__global__ __launch_bounds__(kOctNT) void k_octree(
    const LevelGeom* __restrict__ lv, const int* __restrict__ cell_counts, int ncells,
    const CellGeom* __restrict__ cells, const uint32_t* __restrict__ cand, int cand_total,
    uint32_t* __restrict__ lin, int* __restrict__ label, uint32_t* __restrict__ okey,
    int* __restrict__ ocount, int kp_total, int nlevels, int node_cap, int cell_cap) {
  extern __shared__ __align__(16) unsigned char smem[];
  __shared__ int s_tmp[kOctNT / 64 + 1];
  __shared__ int s_misc[8];
  const int level = blockIdx.x, img = blockIdx.y, tid = threadIdx.x;
  const LevelGeom& G = lv[level];
  int* oc = ocount + img * nlevels + level;
  if (G.ncells == 0) {
    if (tid == 0) *oc = 0;
    return;
  }
  const int NC = node_cap;
  // LDS carve
  unsigned char* p = smem;
  auto take = [&](size_t bytes) {
    unsigned char* r = p;
    p += (bytes + 15) & ~size_t(15);
    return r;
  };
  OctNodes A, B;
  A.x0 = (int16_t*)take(2 * NC); A.x1 = (int16_t*)take(2 * NC);
  A.y0 = (int16_t*)take(2 * NC); A.y1 = (int16_t*)take(2 * NC);
  A.cnt = (int*)take(4 * NC); A.seq = (int*)take(4 * NC);
  B.x0 = (int16_t*)take(2 * NC); B.x1 = (int16_t*)take(2 * NC);
  B.y0 = (int16_t*)take(2 * NC); B.y1 = (int16_t*)take(2 * NC);
  B.cnt = (int*)take(4 * NC); B.seq = (int*)take(4 * NC);
  int* cc = (int*)take(16 * NC);
  int* t1 = (int*)take(4 * NC);
  int* t2 = (int*)take(4 * NC);
  int* t3 = (int*)take(4 * NC);
  int* t4 = (int*)take(4 * NC);
  int* cpre = (int*)take(4 * (cell_cap + 1));

  // 1. gather candidates of this level in cell order (vToDistributeKeys)
  const int* cntv = cell_counts + (int64_t)img * ncells + G.cell_begin;
  for (int i = tid; i < G.ncells; i += kOctNT) cpre[i] = cntv[i];
  __syncthreads();
  const int n = block_scan_excl<kOctNT>(cpre, G.ncells, s_tmp);
  const uint32_t* cb = cand + (int64_t)img * cand_total;
  uint32_t* keys = lin + (int64_t)img * cand_total + G.cand_off;
  int* lab = label + (int64_t)img * cand_total + G.cand_off;
  {
    const int wid = tid >> 6, lane = tid & 63;
    for (int c = wid; c < G.ncells; c += kOctNT / 64) {
      const CellGeom C = cells[G.cell_begin + c];
      const int k = cntv[c], o = cpre[c];
      for (int i = lane; i < k; i += 64) keys[o + i] = cb[C.slot_off + i];
    }
  }
  __syncthreads();
  uint32_t* outk = okey + (int64_t)img * kp_total + G.kp_off;
  if (n == 0) {
    if (tid == 0) *oc = 0;
    return;
  }
  // 2. initial nodes (ORBextractor.cc:530-567)
  const int nini = G.nini;
  for (int i = tid; i < nini; i += kOctNT) {
    A.x0[i] = (int16_t)G.ini_x[i];
    A.x1[i] = (int16_t)G.ini_x[i + 1];
    A.y0[i] = 0;
    A.y1[i] = (int16_t)G.H;
    A.cnt[i] = 0;
    A.seq[i] = i;
  }
  __syncthreads();
  for (int k = tid; k < n; k += kOctNT) {
    const float x = (float)(keys[k] & 0xFFF);
    const int ni = min((int)(x / G.hx), nini - 1);
    lab[k] = ni;
    atomicAdd(&A.cnt[ni], 1);
  }
  __syncthreads();
  // drop empty initial nodes, keep order
  for (int i = tid; i < nini; i += kOctNT) t1[i] = A.cnt[i] > 0;
  __syncthreads();
  int size = block_scan_excl<kOctNT>(t1, nini, s_tmp);
  for (int i = tid; i < nini; i += kOctNT)
    if (A.cnt[i] > 0) {
      const int j = t1[i];
      B.x0[j] = A.x0[i]; B.x1[j] = A.x1[i]; B.y0[j] = A.y0[i]; B.y1[j] = A.y1[i];
      B.cnt[j] = A.cnt[i]; B.seq[j] = A.seq[i];
    }
  __syncthreads();
  for (int k = tid; k < n; k += kOctNT) lab[k] = t1[lab[k]];
  __syncthreads();
  OctNodes cur = B, nxt = A;
  int seqc = nini;
  bool final_mode = false;
  const int N = G.nfeat;
  for (int iter = 0; iter < 4096; iter++) {
    const int prevSize = size;
    for (int i = tid; i < 4 * size; i += kOctNT) cc[i] = 0;
    __syncthreads();
    for (int k = tid; k < n; k += kOctNT) {
      const int nd = lab[k];
      if (cur.cnt[nd] > 1) {
        const int q = quad_of(keys[k], cur.x0[nd], cur.x1[nd], cur.y0[nd], cur.y1[nd]);
        atomicAdd(&cc[4 * nd + q], 1);
      }
    }
    __syncthreads();
    // per-node stats: t1 = nonEmpty children (0 if not expandable), t2 = children with >1
    int nexp_local = 0;
    for (int i = tid; i < size; i += kOctNT) {
      const bool e = cur.cnt[i] > 1;
      int ne = 0, nx = 0;
      if (e) {
#pragma unroll
        for (int q = 0; q < 4; q++) {
          ne += cc[4 * i + q] > 0;
          nx += cc[4 * i + q] > 1;
        }
      }
      t1[i] = ne;
      t2[i] = e;  // divided flag (outer pass divides every expandable node)
      nexp_local += nx;
    }
    const int nToExpand = block_sum<kOctNT>(nexp_local, s_tmp);
    int T, newSize;
    if (!final_mode) {
      // outer pass: process order = list order; t1 -> childPre
      T = block_scan_excl<kOctNT>(t1, size, s_tmp);
      for (int i = tid; i < size; i += kOctNT) t3[i] = !t2[i];
      __syncthreads();
      const int nd_total = block_scan_excl<kOctNT>(t3, size, s_tmp);
      newSize = T + nd_total;
      // base: divided -> T-1-childPre (child j at base-j); else newpos
      for (int i = tid; i < size; i += kOctNT) t4[i] = t2[i] ? T - 1 - t1[i] : T + t3[i];
      __syncthreads();
    } else {
      // final refinement: visit expandable nodes by (size desc, seq desc)
      int E_local = 0;
      for (int i = tid; i < size; i += kOctNT) {
        if (cur.cnt[i] > 1) {
          const int ci = cur.cnt[i], si = cur.seq[i];
          int r = 0;
          for (int j = 0; j < size; j++) {
            const int cj = cur.cnt[j];
            r += cj > 1 && (cj > ci || (cj == ci && cur.seq[j] > si));
          }
          t3[r] = i;  // vis[r] = node
          t4[i] = r;  // rank
          E_local++;
        }
      }
      const int E = block_sum<kOctNT>(E_local, s_tmp);
      // per visiting rank: nonEmpty -> childPre (exclusive scan over visiting order); t2 reused
      for (int v = tid; v < E; v += kOctNT) t2[v] = t1[t3[v]];
      __syncthreads();
      if (tid == 0) s_misc[0] = E > 0 ? E - 1 : -1;
      __syncthreads();
      const int Tall = block_scan_excl<kOctNT>(t2, E, s_tmp);
      (void)Tall;
      // cut = first v with size + childPre_v + ne_v - (v+1) >= N
      for (int v = tid; v < E; v += kOctNT) {
        const int ne = t1[t3[v]];
        if (size + t2[v] + ne - (v + 1) >= N) atomicMin(&s_misc[0], v);
      }
      __syncthreads();
      const int cut = s_misc[0];
      if (cut >= 0) {
        T = t2[cut] + t1[t3[cut]];
        newSize = size + T - (cut + 1);
      } else {
        T = 0;
        newSize = size;
      }
      __syncthreads();
      // divided flag & childPre per node: reuse t1 (keep nonEmpty in cc) -> store childPre
      // in t1 for divided nodes; t2 becomes divided flag per node (indexed by node).
      // First move childPre (indexed by v) into a per-node array (t4 holds rank).
      for (int i = tid; i < size; i += kOctNT) {
        const bool e = cur.cnt[i] > 1;
        const int r = e ? t4[i] : -1;
        t4[i] = (e && r <= cut) ? r : -1;  // rank if divided, else -1
      }
      __syncthreads();
      for (int i = tid; i < size; i += kOctNT) {
        const int r = t4[i];
        t1[i] = r >= 0 ? t2[r] : 0;  // childPre
      }
      __syncthreads();
      for (int i = tid; i < size; i += kOctNT) {
        t2[i] = t4[i] >= 0;
        t3[i] = !(t4[i] >= 0);
      }
      __syncthreads();
      const int nd_total = block_scan_excl<kOctNT>(t3, size, s_tmp);
      (void)nd_total;
      for (int i = tid; i < size; i += kOctNT) t4[i] = t2[i] ? T - 1 - t1[i] : T + t3[i];
      __syncthreads();
    }
    // write next node arrays: t2 = divided, t1 = childPre, t4 = base
    for (int i = tid; i < size; i += kOctNT) {
      if (t2[i]) {
        const int x0 = cur.x0[i], x1 = cur.x1[i], y0 = cur.y0[i], y1 = cur.y1[i];
        const int xm = x0 + (x1 - x0 + 1) / 2, ym = y0 + (y1 - y0 + 1) / 2;
        int j = 0;
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const int c = cc[4 * i + q];
          if (c > 0) {
            const int pos = t4[i] - j;
            nxt.x0[pos] = (int16_t)((q & 1) ? xm : x0);
            nxt.x1[pos] = (int16_t)((q & 1) ? x1 : xm);
            nxt.y0[pos] = (int16_t)((q & 2) ? ym : y0);
            nxt.y1[pos] = (int16_t)((q & 2) ? y1 : ym);
            nxt.cnt[pos] = c;
            nxt.seq[pos] = seqc + t1[i] + j;
            j++;
          }
        }
      } else {
        const int pos = t4[i];
        nxt.x0[pos] = cur.x0[i]; nxt.x1[pos] = cur.x1[i];
        nxt.y0[pos] = cur.y0[i]; nxt.y1[pos] = cur.y1[i];
        nxt.cnt[pos] = cur.cnt[i]; nxt.seq[pos] = cur.seq[i];
      }
    }
    // relabel keys
    for (int k = tid; k < n; k += kOctNT) {
      const int nd = lab[k];
      if (t2[nd]) {
        const int q = quad_of(keys[k], cur.x0[nd], cur.x1[nd], cur.y0[nd], cur.y1[nd]);
        int j = 0;
        for (int qq = 0; qq < q; qq++) j += cc[4 * nd + qq] > 0;
        lab[k] = t4[nd] - j;
      } else {
        lab[k] = t4[nd];
      }
    }
    __syncthreads();
    {
      OctNodes tmp = cur;
      cur = nxt;
      nxt = tmp;
    }
    size = newSize;
    seqc += T;
    if (!final_mode) {
      if (size >= N || size == prevSize) break;
      if (size + nToExpand * 3 > N) final_mode = true;
    } else {
      if (size >= N || size == prevSize) break;
    }
  }
  // 3. retain the best key per node (max response, first in candidate order)
  unsigned* best = (unsigned*)t1;
  for (int i = tid; i < size; i += kOctNT) best[i] = 0;
  __syncthreads();
  for (int k = tid; k < n; k += kOctNT) {
    const uint32_t key = keys[k];
    atomicMax(&best[lab[k]], ((key >> 24) << 24) | (0xFFFFFFu - (unsigned)k));
  }
  __syncthreads();
  for (int i = tid; i < size; i += kOctNT) {
    const int k = (int)(0xFFFFFFu - (best[i] & 0xFFFFFFu));
    outk[i] = keys[k];
  }
  if (tid == 0) *oc = size;
}

// ------------------------------------------------------------------ k_describe
// One wave per retained keypoint: IC_Angle on the unblurred level (ORBextractor.cc:73-98),
// cv::fastAtan2, glibc sincosf, rBRIEF on the blurred level with the reference binary's
// fmaf + cvRound sampling (ORBextractor.cc:101-144), then the level-0 scaling of
// operator() (:1035-1041).  Output is level-major like `_keypoints`/`descriptors`.
__global__ __launch_bounds__(256) void k_describe(
    const uint8_t* __restrict__ pyr, int64_t pyr_bytes, const uint8_t* __restrict__ blur,
    const LevelGeom* __restrict__ lv, int nlevels, const uint32_t* __restrict__ okey,
    const int* __restrict__ ocount, int kp_total, orbx_keypoint* __restrict__ kps,
    uint8_t* __restrict__ desc, int* __restrict__ counts) {
  const int img = blockIdx.y;
  const int lane = threadIdx.x & 63;
  const int slot = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int* oc = ocount + img * nlevels;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    int t = 0;
    for (int l = 0; l < nlevels; l++) t += oc[l];
    counts[img] = t;
  }
  if (slot >= kp_total) return;
  int level = 0;
  while (level + 1 < nlevels && slot >= lv[level + 1].kp_off) level++;
  const LevelGeom& G = lv[level];
  const int idx = slot - G.kp_off;
  if (idx >= oc[level]) return;
  int outpos = idx;
  for (int l = 0; l < level; l++) outpos += oc[l];
  const uint32_t key = okey[(int64_t)img * kp_total + slot];
  const int cx = (int)(key & 0xFFF) + (kEdge - 3), cy = (int)((key >> 12) & 0xFFF) + (kEdge - 3);
  const float response = (float)(key >> 24);
  // IC_Angle: lanes 0..30 rows v = 0..7, lanes 32..62 rows v = 8..15; u = (lane & 31) - 15
  const uint8_t* L = level_base(pyr, pyr_bytes, G, img);
  const uint8_t* center = L + (int64_t)cy * G.pitch + cx;
  int m10 = 0, m01 = 0;
  const int u = (lane & 31) - 15;
  if ((lane & 31) < 31) {
    const int vb = lane < 32 ? 0 : 8, ve = lane < 32 ? 8 : 16;
    for (int v = vb; v < ve; v++) {
      const int d = c_umax[v];
      if (u < -d || u > d) continue;
      if (v == 0) {
        m10 += u * center[u];
      } else {
        const int vp = center[u + v * G.pitch], vm = center[u - v * G.pitch];
        m10 += u * (vp + vm);
        m01 += v * (vp - vm);
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    m10 += __shfl_xor(m10, o);
    m01 += __shfl_xor(m01, o);
  }
  const float angle = orbx_fast_atan2((float)m01, (float)m10);
  // descriptor on the blurred level
  const float factorPI = (float)(3.14159265358979323846 / 180.f);
  float sn, cs;
  orbx_sincosf(angle * factorPI, &sn, &cs);
  const uint8_t* B = blur + (int64_t)img * pyr_bytes + G.pyr_off;
  const uint8_t* bc = B + (int64_t)cy * G.pitch + cx;
  int nib = 0;
#pragma unroll
  for (int m = 0; m < 4; m++) {
    const int pair = lane * 4 + m;
    int t[2];
#pragma unroll
    for (int e = 0; e < 2; e++) {
      const float px = (float)c_pattern[pair * 4 + e * 2];
      const float py = (float)c_pattern[pair * 4 + e * 2 + 1];
      const int row = (int)__builtin_rintf(__builtin_fmaf(px, sn, py * cs));
      const int col = (int)__builtin_rintf(__builtin_fmaf(px, cs, -(py * sn)));
      t[e] = bc[(int64_t)row * G.pitch + col];
    }
    nib |= (t[0] < t[1]) << m;
  }
  const int other = __shfl_xor(nib, 1);
  const int64_t o = (int64_t)img * kp_total + outpos;
  if ((lane & 1) == 0) desc[o * 32 + (lane >> 1)] = (uint8_t)(nib | (other << 4));
  if (lane == 0) {
    orbx_keypoint k;
    k.x = level ? (float)(cx) * G.scale : (float)cx;
    k.y = level ? (float)(cy) * G.scale : (float)cy;
    k.size = G.size;
    k.angle = angle;
    k.response = response;
    k.octave = level;
    k.class_id = -1;
    kps[o] = k;
  }
}

}  // namespace orbx

// ==================================================================== plan
using namespace orbx;

struct orbx_plan {
  Geometry g;
  orbx_params params{};
  int max_batch = 0;
  int device = 0;
  hipStream_t stream = nullptr;
  LevelGeom* d_lv = nullptr;
  CellGeom* d_cells = nullptr;
  int *d_xofs = nullptr, *d_yofs = nullptr;
  int16_t *d_xa = nullptr, *d_yb = nullptr;
  BlurTile* d_tiles = nullptr;
  int ntiles = 0;
  FastTile* d_ftiles = nullptr;
  int nftiles = 0;
  uint8_t* d_vmap = nullptr;
  uint8_t *d_pyr = nullptr, *d_blur = nullptr;
  uint32_t *d_cand = nullptr, *d_lin = nullptr, *d_okey = nullptr;
  int *d_cell_counts = nullptr, *d_label = nullptr, *d_ocount = nullptr, *d_counts = nullptr;
  orbx_keypoint* d_kps = nullptr;
  uint8_t* d_desc = nullptr;
  size_t oct_smem = 0;
  int cell_cap = 0;
  const uint8_t* last_in = nullptr;
  int last_n = 0;
  // graph cache keyed by (input pointer, batch)
  hipGraphExec_t graph = nullptr;
  const uint8_t* graph_in = nullptr;
  int graph_n = -1;
  Profiler prof;
};

namespace {

template <class T>
int dalloc(T** p, size_t count) {
  if (count == 0) count = 1;
  if (hipMalloc((void**)p, count * sizeof(T)) != hipSuccess) return ORBX_ENOMEM;
  return ORBX_OK;
}

int enqueue(orbx_plan* P, const uint8_t* d_in, int n, Profiler* prof) {
  const Geometry& g = P->g;
  const int L = g.nlevels;
  Profiler dummy;
  Profiler& pr = prof ? *prof : dummy;
  const int st_copy = pr.stage("k_copy0"), st_resize = pr.stage("k_resize"),
            st_blur = pr.stage("k_blur"), st_fs = pr.stage("k_fast_score"),
            st_fast = pr.stage("k_fast_nms"),
            st_oct = pr.stage("k_octree"), st_desc = pr.stage("k_describe");
  pr.mark(P->stream, -1);
  {
    const LevelGeom& G = g.lv[0];
    dim3 grid((G.w / 4 + 256) / 256, G.h, n);
    hipLaunchKernelGGL(k_copy0, grid, dim3(256), 0, P->stream, d_in, P->d_pyr, g.pyr_bytes,
                       P->d_lv);
    pr.mark(P->stream, st_copy);
  }
  for (int l = 1; l < L; l++) {
    const LevelGeom& D = g.lv[l];
    dim3 grid((D.w / 4 + 256) / 256, D.h, n);
    hipLaunchKernelGGL(k_resize, grid, dim3(256), 0, P->stream, P->d_pyr, g.pyr_bytes, P->d_lv, l,
                       P->d_xofs, P->d_xa, P->d_yofs, P->d_yb);
    pr.mark(P->stream, st_resize);
  }
  if (P->ntiles > 0) {
    hipLaunchKernelGGL(k_blur, dim3(P->ntiles, n), dim3(256), 0, P->stream, P->d_pyr,
                       g.pyr_bytes, P->d_blur, P->d_lv, P->d_tiles);
    pr.mark(P->stream, st_blur);
  }
  const int ncells = (int)g.cells.size();
  if (ncells > 0) {
    hipLaunchKernelGGL(k_fast_score, dim3(P->nftiles, n), dim3(256), 0, P->stream, P->d_pyr,
                       g.pyr_bytes, P->d_vmap, P->d_lv, P->d_ftiles, min(g.ini_th, g.min_th));
    pr.mark(P->stream, st_fs);
    hipLaunchKernelGGL(k_fast_nms, dim3((ncells + 3) / 4, n), dim3(256), 0, P->stream,
                       P->d_vmap, g.pyr_bytes, P->d_lv, P->d_cells, ncells, g.ini_th, g.min_th,
                       P->d_cand, g.cand_total, P->d_cell_counts);
    pr.mark(P->stream, st_fast);
  }
  hipLaunchKernelGGL(k_octree, dim3(L, n), dim3(kOctNT), P->oct_smem, P->stream, P->d_lv,
                     P->d_cell_counts, ncells, P->d_cells, P->d_cand, g.cand_total, P->d_lin,
                     P->d_label, P->d_okey, P->d_ocount, g.kp_total, L, g.node_cap_max,
                     P->cell_cap);
  pr.mark(P->stream, st_oct);
  hipLaunchKernelGGL(k_describe, dim3((g.kp_total + 3) / 4, n), dim3(256), 0, P->stream,
                     P->d_pyr, g.pyr_bytes, P->d_blur, P->d_lv, L, P->d_okey, P->d_ocount,
                     g.kp_total, P->d_kps, P->d_desc, P->d_counts);
  pr.mark(P->stream, st_desc);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return report_hip(e, "extract launch");
  return ORBX_OK;
}

}  // namespace

extern "C" {

int orbx_plan_create(const orbx_params* params, int32_t w, int32_t h, int32_t max_batch,
                     int hip_device, orbx_plan** out) {
  if (!params || !out || w <= 0 || h <= 0 || max_batch <= 0) return ORBX_EINVAL;
  *out = nullptr;
  orbx_plan* P = new (std::nothrow) orbx_plan();
  if (!P) return ORBX_ENOMEM;
  std::string why;
  int rc = build_geometry(*params, w, h, &P->g, &why);
  if (rc != ORBX_OK) {
    fprintf(stderr, "[orbx] plan %dx%d unsupported: %s\n", w, h, why.c_str());
    delete P;
    return rc;
  }
  P->params = *params;
  P->max_batch = max_batch;
  P->device = hip_device;
  const Geometry& g = P->g;
  auto fail = [&](int code) {
    orbx_plan_destroy(P);
    return code;
  };
  if (hipSetDevice(hip_device) != hipSuccess) return fail(ORBX_EDEVICE);
  if (hipStreamCreateWithFlags(&P->stream, hipStreamNonBlocking) != hipSuccess)
    return fail(ORBX_EDEVICE);
  ORBX_HIP(hipMemcpyToSymbol(HIP_SYMBOL(c_pattern), ORBX_PATTERN, sizeof(ORBX_PATTERN)));
  ORBX_HIP(hipMemcpyToSymbol(HIP_SYMBOL(c_umax), g.umax, sizeof(g.umax)));
  // blur tiles over every level (the blurred pyramid has the pyramid's pitched layout)
  std::vector<BlurTile> tiles;
  for (int l = 0; l < g.nlevels; l++) {
    const LevelGeom& G = g.lv[l];
    for (int ty = 0; ty * kBlurTH < G.h; ty++)
      for (int tx = 0; tx * kBlurTW < G.w; tx++) {
        const int X0 = tx * kBlurTW, Y0 = ty * kBlurTH;
        const bool interior = X0 >= 4 && X0 + kBlurTW + 4 <= G.w && Y0 >= 3 &&
                              Y0 + kBlurTH + 3 <= G.h;
        tiles.push_back({(int16_t)l, (int16_t)tx, (int16_t)ty, (int16_t)interior});
      }
  }
  for (const CellGeom& c : g.cells)
    if (c.x1 - c.x0 > kCellMax || c.y1 - c.y0 > kCellMax) return fail(ORBX_EUNSUPPORTED);
  P->ntiles = (int)tiles.size();
  // FAST score tiles: those intersecting the detection region [19, w-19) x [19, h-19)
  std::vector<FastTile> ftiles;
  for (int l = 0; l < g.nlevels; l++) {
    const LevelGeom& G = g.lv[l];
    if (!G.ncells) continue;
    for (int ty = 0; ty * kFastTH < G.h; ty++)
      for (int tx = 0; tx * kFastTW < G.w; tx++) {
        const int X0 = tx * kFastTW, Y0 = ty * kFastTH;
        if (X0 + kFastTW <= kEdge || X0 >= G.w - kEdge || Y0 + kFastTH <= kEdge ||
            Y0 >= G.h - kEdge)
          continue;
        ftiles.push_back({(int16_t)l, (int16_t)tx, (int16_t)ty, 0});
      }
  }
  P->nftiles = (int)ftiles.size();
  for (int l = 0; l < g.nlevels; l++) P->cell_cap = std::max(P->cell_cap, g.lv[l].ncells);
  const size_t B = (size_t)max_batch;
  if (dalloc(&P->d_lv, g.nlevels) || dalloc(&P->d_cells, g.cells.size()) ||
      dalloc(&P->d_xofs, g.xofs.size()) || dalloc(&P->d_yofs, g.yofs.size()) ||
      dalloc(&P->d_xa, g.xa.size()) || dalloc(&P->d_yb, g.yb.size()) ||
      dalloc(&P->d_tiles, tiles.size()) || dalloc(&P->d_ftiles, ftiles.size()) ||
      dalloc(&P->d_vmap, B * g.pyr_bytes) ||
      dalloc(&P->d_pyr, B * g.pyr_bytes) || dalloc(&P->d_blur, B * g.pyr_bytes) ||
      dalloc(&P->d_cand, B * g.cand_total) || dalloc(&P->d_lin, B * g.cand_total) ||
      dalloc(&P->d_label, B * g.cand_total) || dalloc(&P->d_cell_counts, B * g.cells.size()) ||
      dalloc(&P->d_okey, B * g.kp_total) || dalloc(&P->d_ocount, B * g.nlevels) ||
      dalloc(&P->d_counts, B) || dalloc(&P->d_kps, B * g.kp_total) ||
      dalloc(&P->d_desc, B * g.kp_total * 32))
    return fail(ORBX_ENOMEM);
  auto up = [&](void* d, const void* h, size_t bytes) {
    return bytes ? hipMemcpy(d, h, bytes, hipMemcpyHostToDevice) : hipSuccess;
  };
  if (up(P->d_lv, g.lv, sizeof(LevelGeom) * g.nlevels) ||
      up(P->d_cells, g.cells.data(), sizeof(CellGeom) * g.cells.size()) ||
      up(P->d_xofs, g.xofs.data(), 4 * g.xofs.size()) ||
      up(P->d_yofs, g.yofs.data(), 4 * g.yofs.size()) ||
      up(P->d_xa, g.xa.data(), 2 * g.xa.size()) || up(P->d_yb, g.yb.data(), 2 * g.yb.size()) ||
      up(P->d_tiles, tiles.data(), sizeof(BlurTile) * tiles.size()) ||
      up(P->d_ftiles, ftiles.data(), sizeof(FastTile) * ftiles.size()))
    return fail(ORBX_EDEVICE);
  if (hipMemset(P->d_counts, 0, 4 * B) != hipSuccess) return fail(ORBX_EDEVICE);
  const size_t NC = (size_t)g.node_cap_max;
  auto r16 = [](size_t b) { return (b + 15) & ~size_t(15); };
  P->oct_smem = 2 * (4 * r16(2 * NC) + 2 * r16(4 * NC)) + r16(16 * NC) + 4 * r16(4 * NC) +
                r16(4 * (P->cell_cap + 1));
  if (P->oct_smem > 160 * 1024) return fail(ORBX_EUNSUPPORTED);
  if (hipFuncSetAttribute((const void*)k_octree, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)P->oct_smem) != hipSuccess)
    return fail(ORBX_EDEVICE);
  *out = P;
  return ORBX_OK;
}

int orbx_plan_destroy(orbx_plan* P) {
  if (!P) return ORBX_OK;
  if (P->graph) hipGraphExecDestroy(P->graph);
  void* ptrs[] = {P->d_lv,  P->d_cells, P->d_xofs,   P->d_yofs,  P->d_xa,
                  P->d_yb,  P->d_tiles, P->d_ftiles, P->d_vmap, P->d_pyr,  P->d_blur,
                  P->d_cand, P->d_lin,   P->d_okey,   P->d_cell_counts, P->d_label,
                  P->d_ocount, P->d_counts, P->d_kps, P->d_desc};
  for (void* p : ptrs)
    if (p) hipFree(p);
  if (P->stream) hipStreamDestroy(P->stream);
  delete P;
  return ORBX_OK;
}

int orbx_plan_capacity(const orbx_plan* P, int32_t* kp_cap) {
  if (!P || !kp_cap) return ORBX_EINVAL;
  *kp_cap = P->g.kp_total;
  return ORBX_OK;
}

int orbx_plan_extract(orbx_plan* P, const uint8_t* d_imgs, int32_t n) {
  if (!P || !d_imgs || n <= 0 || n > P->max_batch) return ORBX_EINVAL;
  ORBX_HIP(hipSetDevice(P->device));
  P->last_in = d_imgs;
  P->last_n = n;
  if (P->prof.on) return enqueue(P, d_imgs, n, &P->prof);
  if (!(P->graph && P->graph_in == d_imgs && P->graph_n == n)) {
    if (P->graph) {
      hipGraphExecDestroy(P->graph);
      P->graph = nullptr;
    }
    hipGraph_t gr;
    ORBX_HIP(hipStreamBeginCapture(P->stream, hipStreamCaptureModeThreadLocal));
    int rc = enqueue(P, d_imgs, n, nullptr);
    hipError_t e = hipStreamEndCapture(P->stream, &gr);
    if (rc != ORBX_OK) return rc;
    if (e != hipSuccess) return report_hip(e, "hipStreamEndCapture");
    e = hipGraphInstantiate(&P->graph, gr, nullptr, nullptr, 0);
    hipGraphDestroy(gr);
    if (e != hipSuccess) return report_hip(e, "hipGraphInstantiate");
    P->graph_in = d_imgs;
    P->graph_n = n;
  }
  ORBX_HIP(hipGraphLaunch(P->graph, P->stream));
  return ORBX_OK;
}

int orbx_plan_outputs(orbx_plan* P, orbx_keypoint** d_kps, uint8_t** d_desc, int32_t** d_counts) {
  if (!P) return ORBX_EINVAL;
  if (d_kps) *d_kps = P->d_kps;
  if (d_desc) *d_desc = P->d_desc;
  if (d_counts) *d_counts = P->d_counts;
  return ORBX_OK;
}

int orbx_plan_sync(orbx_plan* P) {
  if (!P) return ORBX_EINVAL;
  ORBX_HIP(hipStreamSynchronize(P->stream));
  return ORBX_OK;
}

void* orbx_plan_stream(orbx_plan* P) { return P ? (void*)P->stream : nullptr; }

int orbx_plan_profile(orbx_plan* P, int32_t enable) {
  if (!P) return ORBX_EINVAL;
  P->prof.on = enable != 0;
  P->prof.reset();
  return ORBX_OK;
}

int orbx_plan_profile_read(orbx_plan* P, int32_t cap, char (*names)[32], double* total_ms,
                           int64_t* launches, int32_t* n_stages) {
  if (!P) return ORBX_EINVAL;
  if (P->prof.collect() != 0) return ORBX_EDEVICE;
  const int n = (int)P->prof.names.size();
  if (n_stages) *n_stages = n;
  for (int i = 0; i < n && i < cap; i++) {
    if (names) {
      strncpy(names[i], P->prof.names[i].c_str(), 31);
      names[i][31] = 0;
    }
    if (total_ms) total_ms[i] = P->prof.ms[i];
    if (launches) launches[i] = P->prof.launches[i];
  }
  return ORBX_OK;
}

// Internal accessors used by the single-image extractor (orbx_api.hip).
int orbx_plan_level_dims(const orbx_plan* P, int level, int* w, int* h) {
  if (!P || level < 0 || level >= P->g.nlevels) return ORBX_EINVAL;
  *w = P->g.lv[level].w;
  *h = P->g.lv[level].h;
  return ORBX_OK;
}

int orbx_plan_level_download(orbx_plan* P, int img, int level, uint8_t* out, int64_t stride) {
  if (!P || !P->last_in || img < 0 || img >= P->last_n || level < 0 || level >= P->g.nlevels)
    return ORBX_EINVAL;
  const LevelGeom& G = P->g.lv[level];
  const uint8_t* src = P->d_pyr + (int64_t)img * P->g.pyr_bytes + G.pyr_off;
  ORBX_HIP(hipMemcpy2DAsync(out, stride, src, G.pitch, G.w, G.h, hipMemcpyDeviceToHost,
                            P->stream));
  ORBX_HIP(hipStreamSynchronize(P->stream));
  return ORBX_OK;
}

}  // extern "C"

namespace orbx {
int plan_view(orbx_plan* P, PlanView* v) {
  if (!P || !v) return ORBX_EINVAL;
  v->g = &P->g;
  v->stream = P->stream;
  v->d_kps = P->d_kps;
  v->d_desc = P->d_desc;
  v->d_counts = P->d_counts;
  v->kp_total = P->g.kp_total;
  v->max_batch = P->max_batch;
  return ORBX_OK;
}
int plan_enqueue(orbx_plan* P, const uint8_t* d_in, int n, Profiler* prof) {
  if (!P || !d_in || n <= 0 || n > P->max_batch) return ORBX_EINVAL;
  P->last_in = d_in;
  P->last_n = n;
  return enqueue(P, d_in, n, prof);
}
}  // namespace orbx
