// orbx_extract.hip — gfx950 kernels and batch plan for ORBextractor::operator()
// (ORB_SLAM2/src/ORBextractor.cc:985-1072).
//
// One plan = one image size + one parameter set + a maximum batch.  A batch of images runs
// as a fixed launch sequence on the plan's stream (captured once into a hipGraph):
//   k_pyramid       2-3 launches band x column tiles     (level 0 copy + cv::resize INTER_LINEAR;
//                                                         k_pyramid<true> also GaussianBlur 7x7
//                                                         s=2 of its rows, Geometry::blur_fused)
//   k_blur          x 0-1        64x64 tiles, all levels (GaussianBlur 7x7 s=2, unfused plans)
//   k_fast_pairs    x 0-1        two FAST cells, a wave  (FAST + cell-local NMS at iniThFAST, the
//   k_fast_cells    x 1-3        up to 4 cells, a wave    minThFAST retry, raster compaction)
//   k_octree        x 1-2        (image, level)          (DistributeOctTree on quadrant-path bins)
//   k_describe      x 1          half-wave per keypoint  (IC_Angle + rBRIEF)
// The first k_pyramid launch copies level 0 from the caller's input into the pitched pyramid
// block, where every level lives.  Everything is integer or bit-exact float (see orbx_math.h); compiled with
// -ffp-contract=off.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <new>
#include <type_traits>
#include <string>
#include <vector>

#include "../../include/orbx_pattern.h"
#include "orbx_describe.h"
#include "orbx_internal.h"
#include "orbx_math.h"

#pragma clang fp contract(off)

namespace orbx {

__constant__ int8_t c_pattern[1024];
__constant__ int c_umax[kHalfPatch + 1];
__constant__ IcMask c_icmask;                   // IC_Angle row masks from umax

// ------------------------------------------------------------------ helpers
// Every level (level 0 copied in by k_pyramid) lives in the image's pitched pyramid block.
__device__ __forceinline__ const uint8_t* level_base(const uint8_t* pyr, int64_t pyr_bytes,
                                                     const LevelGeom& g, int img) {
  return pyr + (int64_t)img * pyr_bytes + g.pyr_off;
}

// XCD-aware block order (MI355X_MICROARCH.md: workgroups go round-robin to the 8 XCDs by
// linear block id, each XCD with its own L2).  Remaps the linear id so each XCD runs one
// contiguous range of (image, tile) blocks: neighbouring tiles share their halo rows and
// columns in the same L2 instead of fetching them on different XCDs.
__device__ __forceinline__ void xcd_block(int& bx, int& by) {
  const int gx = gridDim.x, total = gx * gridDim.y;
  int lin = blockIdx.y * gx + blockIdx.x;
  const int q = total >> 3;
  if (lin < (q << 3)) lin = (lin & 7) * q + (lin >> 3);
  by = lin / gx;
  bx = lin - by * gx;
}

__device__ __forceinline__ int reflect101(int p, int len) {
  if (len == 1) return 0;
  while (p < 0 || p >= len) {
    if (p < 0) p = -p;
    if (p >= len) p = 2 * len - p - 2;
  }
  return p;
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
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

// exclusive prefix over the threads of one value each (and the total)
template <int NT>
__device__ __forceinline__ int grp_excl(int v, int* s_tmp, int& total) {
  const int inc = wave_scan_incl(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 63) s_tmp[wid] = inc;
  __syncthreads();
  int pre = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < NT / 64; w++) {
    const int x = s_tmp[w];
    pre += w < wid ? x : 0;
    tot += x;
  }
  __syncthreads();
  total = tot;
  return pre + inc - v;
}

// Exclusive scan of a[0..M) in place (LDS array), chunked per thread so the scan is stable.
template <int NT>
__device__ int block_scan_excl(int* a, int M, int* s_tmp) {
  const int per = (M + NT - 1) / NT;
  const int beg = min((int)threadIdx.x * per, M), end = min(beg + per, M);
  int sum = 0;
  for (int i = beg; i < end; i++) sum += a[i];
  int total;
  int run = grp_excl<NT>(sum, s_tmp, total);
  for (int i = beg; i < end; i++) {
    const int x = a[i];
    a[i] = run;
    run += x;
  }
  __syncthreads();
  return total;
}

// 64-bit exclusive scan in place (packed counters; one scan instead of several).
template <int NT>
__device__ uint64_t block_scan_excl64(uint64_t* a, int M, uint64_t* s_tmp) {
  const int per = (M + NT - 1) / NT;
  const int t = threadIdx.x;
  const int beg = min(t * per, M), end = min(beg + per, M);
  uint64_t sum = 0;
  for (int i = beg; i < end; i++) sum += a[i];
  const int lane = t & 63, wid = t >> 6;
  const uint64_t v = wave_scan_incl64(sum);
  __syncthreads();
  if (lane == 63) s_tmp[wid] = v;
  __syncthreads();
  if (t == 0) {
    uint64_t acc = 0;
    for (int w = 0; w < NT / 64; w++) {
      const uint64_t x = s_tmp[w];
      s_tmp[w] = acc;
      acc += x;
    }
    s_tmp[NT / 64] = acc;
  }
  __syncthreads();
  uint64_t run = s_tmp[wid] + v - sum;
  for (int i = beg; i < end; i++) {
    const uint64_t x = a[i];
    a[i] = run;
    run += x;
  }
  const uint64_t total = s_tmp[NT / 64];
  __syncthreads();
  return total;
}

// exclusive max-scan of one value >= -1 per thread (-1 below the first): DPP row shifts and
// row broadcasts as wave_scan_incl, on v + 1 so that a missing source (0) is neutral
template <int NT>
__device__ int block_max_excl(int v, int* s_tmp) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t u = (uint32_t)(v + 1);
  u = max(u, dpp0<0x111, 0xF, true>(u));
  u = max(u, dpp0<0x112, 0xF, true>(u));
  u = max(u, dpp0<0x114, 0xF, true>(u));
  u = max(u, dpp0<0x118, 0xF, true>(u));
  u = max(u, dpp0<0x142, 0xA, false>(u));
  u = max(u, dpp0<0x143, 0xC, false>(u));
  const int ex = (int)dpp0<0x138, 0xF, true>(u) - 1;  // wave_shr:1 (lane 0: none)
  __syncthreads();
  if (lane == 63) s_tmp[wid] = (int)u - 1;
  __syncthreads();
  int pre = -1;
  for (int w = 0; w < wid; w++) pre = max(pre, s_tmp[w]);
  __syncthreads();
  return max(pre, ex);
}

// ------------------------------------------------------------------ k_pyramid
// 16-B source chunks per thread in flight while a band is staged (8 or 2 measured slower:
// 0.426 / 0.303 vs 0.298 ms per 512 C2 frames)
constexpr int kPyLoads = 4;
// ComputePyramid (ORBextractor.cc:1047-1072) in a few launches (Geometry::pyr_stages): the first
// copies level 0 into the 64-B pitched pyramid block (every later kernel reads aligned dwords)
// and builds levels 1..3, the next ones build four levels each from the last level stored.
// One workgroup per (image, row band) builds its band of the stage's levels, each from the
// previous one, with cv::resize INTER_LINEAR 8UC1: horizontal Q11 taps, vertical
// SSE2 mulhi form for x < vxs, scalar (H0*b0 + H1*b1 + 2^21) >> 22 tail.  Bands overlap by
// the rows the next level needs (Geometry::bands), so no band waits for another; a band keeps
// its rows of the level just built in LDS (even levels in buffer A, odd ones at buf_b) and
// reads the next level's sources there, so each level costs one barrier and the pyramid block
// is only written, by the band that owns the row.  Work items are (strip of kPyStrip rows,
// 4-pixel column group) pairs dealt round-robin over the kPyNT threads; along its strip an
// item reuses the horizontal sums of the source row two consecutive output rows share.
// i = r * n + c for 0 <= i < 2^20, 1 <= n: (i + 0.5) / n is >= 0.5 / n from an integer, so
// the float quotient truncates to r; the two fix-ups are insurance.
__device__ __forceinline__ void py_divmod(int i, int n, float inv_n, int& r, int& c) {
  r = (int)(((float)i + 0.5f) * inv_n);
  c = i - __mul24(r, n);
  if (c < 0) r--, c += n;
  if (c >= n) r++, c -= n;
}

__device__ __forceinline__ uint32_t mulhi_u24(uint32_t a, uint32_t b) {  // a, b < 2^24
  return (uint32_t)(((uint64_t)(a & 0xFFFFFF) * (uint64_t)(b & 0xFFFFFF)) >> 32);
}

typedef unsigned short py_u16x2 __attribute__((ext_vector_type(2)));

// Horizontal pass of cv::resize INTER_LINEAR 8UC1 for the 4 output pixels of one
// column group on one source row: g = S0 * (a0 << 4) + S1 * (a1 << 4) (the taps carry << 4,
// packed as u16 pairs), the source pair (S0, S1) one unaligned ds_read_u16 spread into u16
// halves, the two products one v_dot2_u32_u16.  Coefficients are in [0, 2049] (checked in
// resize_tables), so every OpenCV saturation on the way is a no-op: H = g >> 4 < 2^19.
__device__ __forceinline__ void py_horiz(const uint8_t* row, const int (&xs)[4],
                                         const uint32_t (&as)[4], uint32_t (&g)[4]) {
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint32_t p = __builtin_amdgcn_perm((uint32_t)row[xs[k] + 1], (uint32_t)row[xs[k]],
                                             0x0c040c00u);  // (S0, S1)
    g[k] = __builtin_amdgcn_udot2(__builtin_bit_cast(py_u16x2, p),
                                  __builtin_bit_cast(py_u16x2, as[k]), 0u, false);
  }
}

// Vertical pass for the 4 pixels from the horizontal sums of their two source rows.  SSE2
// region: _mm_mulhi_epi16(H >> 4, b) = ((H >> 4) * b) >> 16 = mulhi_u24((H >> 4) << 8, b << 8)
// with (H >> 4) << 8 = g & ~0xFF, the mulhi sum <= 1020, result (m + 2) >> 2; past vxs (a
// column whose tap carries bit 30, `sc` holds those bits at 0..3) the scalar
// (H0*b0 + H1*b1 + 2^21) >> 22.  Results are in [0, 255].
__device__ __forceinline__ uint32_t py_vert(const uint32_t (&g0)[4], const uint32_t (&g1)[4],
                                           uint32_t yb, uint32_t sc) {
  const uint32_t b0 = yb & 0xFFFF, b1 = yb >> 16;
  uint32_t out = 0;
  if (sc == 0) {  // VResizeLinearVec_32s8u: the whole group in the SSE2 region
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t m = mulhi_u24(g0[k] & 0x7FFF00, b0 << 8) + mulhi_u24(g1[k] & 0x7FFF00, b1 << 8);
      out |= ((m + 2) >> 2) << (8 * k);
    }
  } else {  // the row end (or a reflected column): SSE2 up to vxs, then the scalar form
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t m = mulhi_u24(g0[k] & 0x7FFF00, b0 << 8) + mulhi_u24(g1[k] & 0x7FFF00, b1 << 8);
      const uint32_t vsc = (__umul24(g0[k] >> 4, b0) + __umul24(g1[k] >> 4, b1) + (1u << 21)) >> 22;
      out |= ((sc >> k) & 1 ? vsc : (m + 2) >> 2) << (8 * k);
    }
  }
  return out;
}

typedef unsigned short blur_u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ blur_u16x2 byte_pair(uint32_t hi, uint32_t lo, uint32_t sel) {
  return __builtin_bit_cast(blur_u16x2, __builtin_amdgcn_perm(hi, lo, sel));
}

// GaussianBlur 7x7 sigma 2 of 4 output pixels from the column sums of their
// 4-column dword (c, d: column pairs (x, x+1), (x+2, x+3)) and of the dwords left (a, b: x-4 ..
// x-1) and right (e, f: x+4 .. x+7): four v_dot2_u32_u16 per output with the taps laid over the
// pairs, m / 65536 rounded half-even for x < bxs (the SSE2 region) and half-up in the scalar
// tail, two results per dword by one v_perm of the high halves, clamped by v_pk_min_u16, the four
// low bytes gathered by one more v_perm.
__device__ __forceinline__ uint32_t blur_row4(uint32_t a, uint32_t b, uint32_t c, uint32_t d,
                                              uint32_t e, uint32_t f, uint32_t tail) {
  constexpr unsigned short k0 = 18, k1 = 34, k2 = 49, k3 = 55;
  const blur_u16x2 W0k0 = {0, k0}, Wk1k2 = {k1, k2}, Wk3k2 = {k3, k2}, Wk1k0 = {k1, k0},
                   Wk0k1 = {k0, k1}, Wk2k3 = {k2, k3}, Wk2k1 = {k2, k1}, Wk00 = {k0, 0};
  const blur_u16x2 P0 = __builtin_bit_cast(blur_u16x2, a), P1 = __builtin_bit_cast(blur_u16x2, b),
                   P2 = __builtin_bit_cast(blur_u16x2, c), P3 = __builtin_bit_cast(blur_u16x2, d),
                   P4 = __builtin_bit_cast(blur_u16x2, e), P5 = __builtin_bit_cast(blur_u16x2, f);
  auto d2 = [](blur_u16x2 p, blur_u16x2 k, uint32_t acc) { return __builtin_amdgcn_udot2(p, k, acc, false); };
  const uint32_t m[4] = {d2(P3, Wk1k0, d2(P2, Wk3k2, d2(P1, Wk1k2, d2(P0, W0k0, 0u)))),
                         d2(P4, Wk00, d2(P3, Wk2k1, d2(P2, Wk2k3, d2(P1, Wk0k1, 0u)))),
                         d2(P4, Wk1k0, d2(P3, Wk3k2, d2(P2, Wk1k2, d2(P1, W0k0, 0u)))),
                         d2(P5, Wk00, d2(P4, Wk2k1, d2(P3, Wk2k3, d2(P2, Wk0k1, 0u))))};
  uint32_t rq[4];
#pragma unroll
  for (int k = 0; k < 4; k++) rq[k] = m[k] + (0x7FFFu + tail) + __builtin_amdgcn_ubfe(m[k], 16, 1u - tail);
  const blur_u16x2 lim = {255, 255};
  const blur_u16x2 h01 = __builtin_elementwise_min(byte_pair(rq[1], rq[0], 0x07060302u), lim),
                   h23 = __builtin_elementwise_min(byte_pair(rq[3], rq[2], 0x07060302u), lim);
  return __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, h23), __builtin_bit_cast(uint32_t, h01),
                               0x06040200u);
}

// Column sums (taps [18, 34, 49, 55, 49, 34, 18], packed u16: at most 255 * 257) of one dword
// column's two byte pairs over 7 consecutive rows starting at j.
// The symmetric pair sums (at most 510 a half: no carry crosses into the high half) as plain
// 32-bit adds, which dual-issue (profiles/valu_calibration.json), where v_pk_add_u16 does not.
__device__ __forceinline__ blur_u16x2 blur_pair_add(blur_u16x2 a, blur_u16x2 b) {
  return __builtin_bit_cast(blur_u16x2, __builtin_bit_cast(uint32_t, a) + __builtin_bit_cast(uint32_t, b));
}
template <int N>
__device__ __forceinline__ blur_u16x2 blur_col(const blur_u16x2 (&U)[N], int j) {
  const blur_u16x2 K0 = {18, 18}, K1 = {34, 34}, K2 = {49, 49}, K3 = {55, 55};
  return blur_pair_add(U[j], U[j + 6]) * K0 + blur_pair_add(U[j + 1], U[j + 5]) * K1 +
         blur_pair_add(U[j + 2], U[j + 4]) * K2 + U[j + 3] * K3;
}

// The fused blur (k_pyramid<true>) of one level's own tile: rows [own_lo, own_hi), groups
// [own_glo, own_ghi), from the tile's rows [lo, hi) of the level in LDS (row stride lp, column c
// at byte c - cb; the tile holds the group left and right of its own ones, at the level's edges
// the reflected columns -4..-1 and w..: no lane handles a column border).
// A lane holds one dword column (own_glo - 1 .. own_ghi) over a strip of S output rows: it
// unpacks its S + 6 input dwords into byte pairs once, and per output row forms the column sums
// of its 4 columns and takes its neighbours' by DPP wave shifts (lanes are consecutive columns
// of a strip; each wave's first and last lane only lend their sums, so consecutive waves overlap
// by two columns).  Rows outside the level reflect (BORDER_REFLECT_101).
template <int S>
__device__ __forceinline__ void py_blur_band(const uint8_t* __restrict__ sb, int lp, int cb, int lo,
                                             int hi, const LevelGeom& G, int own_lo, int own_hi,
                                             int own_glo, int own_ghi, uint8_t* __restrict__ dst) {
  const int R = own_hi - own_lo;
  if (R <= 0 || own_ghi <= own_glo) return;
  const int h = G.h, pitch = G.pitch, bxs = G.bxs;
  const int ngp = own_ghi - own_glo + 2;
  const int nitems = ((R + S - 1) / S) * ngp;
  const int lane = threadIdx.x & 63;
  const float inv = 1.0f / (float)ngp;
  for (int base = (threadIdx.x >> 6) * 62; base < nitems; base += (kPyNT / 64) * 62) {
    const int iu = base + lane - 1;
    int st, c;
    py_divmod(min(max(iu, 0), nitems - 1), ngp, inv, st, c);
    const int cc = own_glo - 1 + c, y0 = own_lo + st * S;
    const uint8_t* col = sb + 4 * cc - cb;
    blur_u16x2 U[S + 6], V[S + 6];
    if (__all(y0 - 3 >= lo && y0 + S + 2 < hi)) {  // the strip's rows lie in the band
      const uint8_t* p = col + __mul24(y0 - 3 - lo, lp);
#pragma unroll
      for (int k = 0; k < S + 6; k++) {
        const uint32_t d = *(const uint32_t*)(p + __mul24(k, lp));
        U[k] = byte_pair(d, d, 0x0c010c00u);
        V[k] = byte_pair(d, d, 0x0c030c02u);
      }
    } else {  // the level's top / bottom rows (reflected), or a strip past the band's last row
#pragma unroll
      for (int k = 0; k < S + 6; k++) {
        const int y = min(max(reflect101(y0 + k - 3, h), lo), hi - 1);
        const uint32_t d = *(const uint32_t*)(col + __mul24(y - lo, lp));
        U[k] = byte_pair(d, d, 0x0c010c00u);
        V[k] = byte_pair(d, d, 0x0c030c02u);
      }
    }
    const bool out = lane >= 1 && lane <= 62 && iu < nitems && cc >= own_glo && cc < own_ghi;
    const uint32_t tail = 4 * cc < bxs ? 0u : 1u;
    uint8_t* drow = dst + __mul24(y0, pitch) + 4 * cc;
#pragma unroll
    for (int j = 0; j < S; j++) {
      const uint32_t su = __builtin_bit_cast(uint32_t, blur_col(U, j)),
                     sv = __builtin_bit_cast(uint32_t, blur_col(V, j));
      // wave_shr:1 (lane n reads lane n - 1) and wave_shl:1 (lane n + 1)
      const uint32_t lu = __builtin_amdgcn_mov_dpp(su, 0x138, 0xf, 0xf, true),
                     lv = __builtin_amdgcn_mov_dpp(sv, 0x138, 0xf, 0xf, true),
                     ru = __builtin_amdgcn_mov_dpp(su, 0x130, 0xf, 0xf, true),
                     rv = __builtin_amdgcn_mov_dpp(sv, 0x130, 0xf, 0xf, true);
      const uint32_t o = blur_row4(lu, lv, su, sv, ru, rv, tail);
      if (out && y0 + j < own_hi) *(uint32_t*)(drow + __mul24(j, pitch)) = o;  // bytes past w: row pad
    }
  }
}

// With BLUR (the fused GaussianBlur, kPyFused), the band also blurs its own rows of every level
// it builds, and of level 0 in the first stage, into `blur` (py_blur_band) from the rows it holds
// in LDS: the bands carry the blur's 3-row halo, every level is kept in LDS, and the resize also
// computes each row's reflected pad columns (-4..-1 and past w, the tap table's reflected
// entries) into LDS only.  A level's blur runs in the phase that builds the next level from it
// (both only read its buffer), so the blur adds no barrier but the stage's last.
template <bool BLUR>
__global__ __launch_bounds__(kPyNT) void k_pyramid(const uint8_t* __restrict__ in,
                                                  uint8_t* __restrict__ pyr, int64_t pyr_bytes,
                                                  const LevelGeom* __restrict__ lv, int l0, int l1,
                                                  const PyrBand* __restrict__ bands,
                                                  const int2* __restrict__ xtap,
                                                  const int2* __restrict__ ytap, int buf_b,
                                                  uint8_t* __restrict__ blur) {
  extern __shared__ __align__(16) uint8_t s_pyr[];
  int band, img;
  xcd_block(band, img);
  const PyrBand& B = bands[band];
  const int tid = threadIdx.x;
  uint8_t* base = pyr + (int64_t)img * pyr_bytes;
  uint8_t* bbase = BLUR ? blur + (int64_t)img * pyr_bytes : nullptr;
  {  // the source level's tile (rows lo..hi-1, columns cb .. cb + lp - 1) into LDS (buffer of
     // parity l0 - 1); level 0 is copied into the pyramid by the tile that owns it
    const LevelGeom& G = lv[l0 - 1];
    const int lo = B.lo[l0 - 1], nr = B.hi[l0 - 1] - lo, pitch = G.pitch;
    const int cb = B.cb[l0 - 1], lp = B.lp[l0 - 1];
    uint8_t* sdst = s_pyr + ((l0 - 1) & 1 ? buf_b : 0);
    const bool input = l0 == 1;  // level 0 comes from the input (ORBextractor.cc:1066-1068)
    const int w = input ? G.w : pitch;  // a pyramid row is copied pad and all
    const uint8_t* src = input ? in + (int64_t)img * G.h * G.w : base + G.pyr_off;
    const int own_lo = input ? B.own_lo[0] : 0, own_hi = input ? B.own_hi[0] : 0;
    const int own_x0 = 4 * B.own_glo[0], own_x1 = 4 * B.own_ghi[0];
    uint8_t* dst = base + G.pyr_off;
    const bool pads = BLUR && input;  // level 0 is blurred: its rows' reflected pad columns
    const int c0 = max(cb, 0) >> 4, c1 = min((cb + lp) >> 4, (w + 15) >> 4);  // 16-B chunks
    if ((w & 15) == 0) {  // 16-byte chunks, four per thread in flight
      const int nch = c1 - c0, items = nr * nch;
      const float inv = 1.0f / (float)max(nch, 1);
      for (int i0 = tid; i0 < items; i0 += kPyLoads * kPyNT) {
        // past the end a thread repeats the last chunk: identical bytes to identical places
        uint4 v[kPyLoads];
        int rr[kPyLoads], cc[kPyLoads];
#pragma unroll
        for (int u = 0; u < kPyLoads; u++) {
          py_divmod(min(i0 + kPyNT * u, items - 1), nch, inv, rr[u], cc[u]);
          cc[u] += c0;
          v[u] = *(const uint4*)(src + (int64_t)(lo + rr[u]) * w + 16 * cc[u]);
        }
#pragma unroll
        for (int u = 0; u < kPyLoads; u++)  // pin the loads here: all four in flight together
          asm volatile("" : "+v"(v[u].x), "+v"(v[u].y), "+v"(v[u].z), "+v"(v[u].w));
#pragma unroll
        for (int u = 0; u < kPyLoads; u++) {
          const int y = lo + rr[u], x = 16 * cc[u];
          uint8_t* srow = sdst + __mul24(rr[u], lp) - cb;  // column c at srow + c
          *(uint4*)(srow + x) = v[u];
          if (y >= own_lo && y < own_hi && x >= own_x0 && x < own_x1)
            *(uint4*)(dst + (uint32_t)__mul24(y, pitch) + x) = v[u];
          if (pads) {  // columns -4..-1 = 4, 3, 2, 1; w..w+3 = w-2 .. w-5 (w >= 16 here)
            if (x == 0 && cb < 0) *(uint32_t*)(srow - 4) = __builtin_amdgcn_perm(v[u].y, v[u].x, 0x01020304u);
            if (x == w - 16 && cb + lp > w) *(uint32_t*)(srow + w) = __builtin_amdgcn_perm(v[u].w, v[u].z, 0x03040506u);
          }
        }
      }
    } else {  // any input width: dwords assembled from bytes, the columns outside the level
              // reflected (only the blurred level 0 reads them)
      const int q0 = cb >> 2, q4 = lp >> 2, items = nr * q4;
      const float inv = 1.0f / (float)q4;
      for (int i = tid; i < items; i += kPyNT) {
        int r, c;
        py_divmod(i, q4, inv, r, c);
        const int x4 = 4 * (q0 + c), y = lo + r;
        const uint8_t* s = src + (int64_t)y * w;
        uint32_t v = 0;
        if (x4 >= 0 && x4 + 3 < w) {
          v = s[x4] | (uint32_t)s[x4 + 1] << 8 | (uint32_t)s[x4 + 2] << 16 | (uint32_t)s[x4 + 3] << 24;
        } else if (pads) {
#pragma unroll
          for (int k = 0; k < 4; k++) v |= (uint32_t)s[reflect101(x4 + k, w)] << (8 * k);
        } else {
#pragma unroll
          for (int k = 0; k < 4; k++)
            if (x4 + k >= 0 && x4 + k < w) v |= (uint32_t)s[x4 + k] << (8 * k);
        }
        *(uint32_t*)(sdst + __mul24(r, lp) + 4 * c) = v;
        if (y >= own_lo && y < own_hi && x4 >= own_x0 && x4 < own_x1)
          *(uint32_t*)(dst + (uint32_t)__mul24(y, pitch) + x4) = v;
      }
    }
  }
  for (int l = l0; l <= l1; l++) {
    __syncthreads();  // level l-1 of this tile is in LDS
    const LevelGeom& D = lv[l];
    const LevelGeom& S = lv[l - 1];
    const uint8_t* sb = s_pyr + ((l - 1) & 1 ? buf_b : 0);
    uint8_t* db = s_pyr + (l & 1 ? buf_b : 0) - B.cb[l];  // column c of a row at + c
    uint8_t* dp = base + D.pyr_off;
    const int slo = B.lo[l - 1], dlo = B.lo[l];
    const int scb = B.cb[l - 1];
    // column groups glo .. ghi - 1: with BLUR the pad groups -1 and gl + 1 at the level's edges
    // (LDS only)
    const int g0 = B.glo[l], ng = max(0, B.ghi[l] - g0);
    const int nr = max(0, B.hi[l] - dlo), nstrip = (nr + kPyStrip - 1) / kPyStrip;
    const int items = nstrip * ng;
    const float inv_ng = 1.0f / (float)max(ng, 1);
    const bool keep = BLUR || l < l1;  // without the blur the stage's last level is not read back
    const int dpitch = D.pitch, dlp = B.lp[l], slp = B.lp[l - 1], sh1 = S.h - 1;
    const int own_lo = B.own_lo[l], own_hi = B.own_hi[l], own_glo = B.own_glo[l], own_ghi = B.own_ghi[l];
    const int2* xt = xtap + D.coef_x;
    const int2* yt = ytap + D.coef_y + dlo;
    const uint8_t* sbx = sb - scb;  // column c of a source row at + c
    // work item = (strip of kPyStrip output rows, 4-pixel column group): the taps are loaded
    // once per item, and a source row's horizontal sums carry over to the next output row
    // that reads it (scale 1.2: 1.2 horizontal passes per output row instead of 2)
    for (int i = tid; i < items; i += kPyNT) {
      int st, gi;
      py_divmod(i, ng, inv_ng, st, gi);
      gi += g0;
      const int dx0 = 4 * gi;
      const int4 t01 = *(const int4*)(xt + dx0);  // every run starts 4 entries before column 0 and
      const int4 t23 = *(const int4*)(xt + dx0 + 2);  // is a multiple of 4: aligned, in range
      const uint32_t sc = ((uint32_t)t01.x >> 30) | ((uint32_t)t01.z >> 29) |
                          ((uint32_t)t23.x >> 28) | ((uint32_t)t23.z >> 27);  // bit 30: scalar form
      const int xs[4] = {t01.x & 0xFFFFF, t01.z & 0xFFFFF, t23.x & 0xFFFFF, t23.z & 0xFFFFF};
      const uint32_t as[4] = {(uint32_t)t01.y, (uint32_t)t01.w, (uint32_t)t23.y, (uint32_t)t23.w};
      const int r0 = st * kPyStrip, r1 = min(nr, r0 + kPyStrip);
      const bool gwrite = gi >= own_glo && gi < own_ghi;
      int prev = -1;
      uint32_t gp[4] = {0u, 0u, 0u, 0u};
      for (int r = r0; r < r1; r++) {
        const int2 ty = yt[r];
        const int ya = min(max(ty.x, 0), sh1), yb = min(max(ty.x + 1, 0), sh1);
        if (ya != prev) py_horiz(sbx + __mul24(ya - slo, slp), xs, as, gp);
        uint32_t g1[4];
        py_horiz(sbx + __mul24(yb - slo, slp), xs, as, g1);
        const uint32_t o = py_vert(gp, g1, (uint32_t)ty.y, sc);
        // pitch >= w + 4: bytes past w of the last group land in the row's pad
        if (keep) *(uint32_t*)(db + __mul24(r, dlp) + dx0) = o;
        if (gwrite && dlo + r >= own_lo && dlo + r < own_hi)
          *(uint32_t*)(dp + (uint32_t)__mul24(dlo + r, dpitch) + dx0) = o;
#pragma unroll
        for (int k = 0; k < 4; k++) gp[k] = g1[k];
        prev = yb;
      }
    }
    if (BLUR && (l > l0 || l0 == 1))  // level l-1 is blurred from the same buffer
      py_blur_band<kPyBlurStrip>(sb, slp, scb, slo, B.hi[l - 1], S, B.own_lo[l - 1], B.own_hi[l - 1],
                                 B.own_glo[l - 1], B.own_ghi[l - 1], bbase + S.pyr_off);
  }
  if (BLUR) {  // the stage's last level (level 0 alone for a one-level pyramid)
    __syncthreads();
    const LevelGeom& D = lv[l1];
    py_blur_band<kPyBlurStrip>(s_pyr + (l1 & 1 ? buf_b : 0), B.lp[l1], B.cb[l1], B.lo[l1], B.hi[l1], D,
                               B.own_lo[l1], B.own_hi[l1], B.own_glo[l1], B.own_ghi[l1],
                               bbase + D.pyr_off);
  }
}

// ------------------------------------------------------------------ k_blur
// GaussianBlur(level, 7x7, sigma 2, BORDER_REFLECT_101) in OpenCV 2.4's 8U fixed point
// (SURVEY A.4): integer row pass with taps [18,34,49,55,49,34,18], column pass rounded
// half-even (SSE2 f32 region x < 4*floor(w/4)) or half-up (scalar tail).  Values below 256
// are exact in f32, so half-even rounding of m/65536 is done on the integer m.
// Tile 64 x 64 outputs: tiles stage the (64+6) x 72 input window as aligned 16-B pieces, border
// tiles reflecting rows and, byte-wise, the pieces crossing the left / right edge (reflect101).  The separable sum is exact in integers, so
// the column pass runs first, in packed u16 (a column sum is at most 255 * 257 = 65535), a
// thread unpacking one dword column once for 4 output rows; the row pass then takes the 32-bit
// products with v_dot2_u32_u16 on the stored u16 pairs, 4 per output.  (Row pass first, with the
// column pass in 24-bit multiplies on extracted halves, issued 56 instead of 16 VALU per 4
// outputs: 292 us per 256 C2 frames.  Both passes in exact f32 on the dual-issue add / fma
// measured 303 us: the f32 buffer doubles the LDS traffic of the second pass.)
constexpr int kBlurTW = 64, kBlurTH = 64;
struct BlurTile {
  int16_t level, tx, ty, interior;
};

__global__ __launch_bounds__(256) void k_blur(const uint8_t* __restrict__ pyr, int64_t pyr_bytes,
                                              uint8_t* __restrict__ blur,
                                              const LevelGeom* __restrict__ lv,
                                              const BlurTile* __restrict__ tiles) {
  constexpr int kWords = (kBlurTW + 8) / 4;  // window columns X0-4 .. X0+67
  // staged row: 16-B pieces of columns X0-16 .. X0+79 (window dword c at c + 3), 28 dwords apart
  // (112 B: rows 4 apart in the column pass land 48 banks on, not 8)
  constexpr int kChunks = (kBlurTW + 32) / 16, kSt = 28;
  constexpr int kRows = kBlurTH + 6;         // window rows Y0-3 .. Y0+66
  __shared__ __align__(16) uint32_t s_in[kRows][kSt];
  __shared__ __align__(16) uint32_t s_col[kBlurTH][kWords * 2];  // column sums, u16 pairs
  int bx, img;
  xcd_block(bx, img);
  const BlurTile T = tiles[bx];
  const LevelGeom& G = lv[T.level];
  int pitch = G.pitch, w = G.w, h = G.h, bxs = G.bxs, pyr_off = (int)G.pyr_off;
  asm volatile("" : "+s"(pitch), "+s"(w), "+s"(h), "+s"(bxs), "+s"(pyr_off));
  const uint8_t* src = pyr + (int64_t)img * pyr_bytes + pyr_off;
  uint8_t* dst = blur + (int64_t)img * pyr_bytes + pyr_off;
  const int X0 = T.tx * kBlurTW, Y0 = T.ty * kBlurTH;
  const int tid = threadIdx.x;
  if (T.interior) {
    // interior: X0 >= 64 and the pitch (a multiple of 64 past X0 + 67) covers X0 + 79
    for (int i = tid; i < kRows * kChunks; i += 256) {
      const int r = i / kChunks, c = i - r * kChunks;
      *(uint4*)&s_in[r][4 * c] =
          *(const uint4*)(src + (uint32_t)((Y0 + r - 3) * pitch + X0 - 16 + 16 * c));
    }
  } else {
    // border tile: each window row reflected once (reflect-101), whole 16-B pieces where they
    // lie inside the level; in a piece crossing the left / right edge, whole dwords where they
    // lie inside and a byte-wise reflect only for the window dwords (3 .. 20) that cross;
    // dwords wholly past the last column any output reads (w + 2) stay unset
    for (int i = tid; i < kRows * kChunks; i += 256) {
      const int r = i / kChunks, c = i - r * kChunks;
      const int y = reflect101(min(Y0 + r - 3, h + 8), h);
      const uint8_t* row = src + (int64_t)y * pitch;
      const int x = X0 - 16 + 16 * c;
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (x >= 0 && x + 16 <= w) {
        v = *(const uint4*)(row + x);
      } else {  // per window dword: whole inside the level, reflected byte-wise, or unused
        uint32_t d[4] = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const int dw = 4 * c + j, xd = x + 4 * j;
          if (dw >= 3 && dw <= 20 && xd < w + 3) {
            if (xd >= 0 && xd + 4 <= w) {
              d[j] = *(const uint32_t*)(row + xd);
            } else {
#pragma unroll
              for (int k = 0; k < 4; k++)
                d[j] |= (uint32_t)row[reflect101(min(xd + k, w + 8), w)] << (8 * k);
            }
          }
        }
        v = make_uint4(d[0], d[1], d[2], d[3]);
      }
      *(uint4*)&s_in[r][4 * c] = v;
    }
  }
  __syncthreads();
  // column pass (the sum is separable and exact, so columns first gives the same m): a thread
  // takes one window dword column and 4 output rows; its 10 input dwords unpack once into byte
  // pairs (b0, b1) and (b2, b3), each output row is 7 packed u16 ops per pair (a column sum is
  // at most 255 * 257 = 65535)
  {
    for (int i = tid; i < kWords * (kBlurTH / 4); i += 256) {
      const int rb = i / kWords, c = i - rb * kWords, r0 = 4 * rb;
      blur_u16x2 U[10], V[10];
#pragma unroll
      for (int k = 0; k < 10; k++) {
        const uint32_t w = s_in[r0 + k][c + 3];
        U[k] = byte_pair(w, w, 0x0c010c00u);
        V[k] = byte_pair(w, w, 0x0c030c02u);
      }
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const blur_u16x2 su = blur_col(U, j), sv = blur_col(V, j);
        *(uint2*)&s_col[r0 + j][2 * c] =
            make_uint2(__builtin_bit_cast(uint32_t, su), __builtin_bit_cast(uint32_t, sv));
      }
    }
  }
  __syncthreads();
  // row pass: 4 adjacent outputs per thread from the 6 column-sum pairs P_j = (c[4q + 2j],
  // c[4q + 2j + 1]) around them (window column i = x - X0 + 4); m / 65536 rounded half-even in
  // the SSE2 region (m + 0x7FFF + lsb(m >> 16)), half-up in the scalar tail (m + 0x8000); x is a
  // multiple of 4, as is bxs: one test per group (blur_row4)
  for (int i = tid; i < kBlurTH * (kBlurTW / 4); i += 256) {
    const int r = i >> 4, q = i & 15;
    const int x = X0 + 4 * q, y = Y0 + r;
    if (x >= w || y >= h) continue;
    const uint2 A = *(const uint2*)&s_col[r][2 * q], B = *(const uint2*)&s_col[r][2 * q + 2],
                C = *(const uint2*)&s_col[r][2 * q + 4];
    const uint32_t out = blur_row4(A.x, A.y, B.x, B.y, C.x, C.y, x < bxs ? 0u : 1u);
    *(uint32_t*)(dst + (uint32_t)(y * pitch + x)) = out;  // bytes past w land in the row pad
  }
}

// ------------------------------------------------------------------ FAST
// cv::FAST with NMS on each cell ROI of ComputeKeyPointsOctTree (ORBextractor.cc:758-796) at
// iniThFAST, again at minThFAST when no keypoint survives, then an order-preserving (raster)
// compaction into the cell's candidate slot.  Score = OpenCV 2.4 cornerScore<16>;
// V = score+1 clamped to [0,255] so "corner at t" is V > t.
constexpr int kCellMax = 66;  // wCell, hCell < 60 (+6)

// fast_score, fast_cardinal2x2: orbx_internal.h

// Candidate keys: position in the octree frame (level coordinates - minBorder + 3) and FAST
// score - 1.  Plans whose octree frames fit 4095 px pack x:12 y:12 score:8 into a u32; wider
// ones (Geometry::wide_keys) use a u64 with x:16 y:16 and the score at bit 32.
template <class K>
struct KeyFmt;
template <>
struct KeyFmt<uint32_t> {
  static __device__ __forceinline__ uint32_t make(int x, int y, int v) {
    return (uint32_t)(x - (kEdge - 3)) | ((uint32_t)(y - (kEdge - 3)) << 12) | ((uint32_t)(v - 1) << 24);
  }
  static __device__ __forceinline__ int x(uint32_t k) { return (int)(k & 0xFFF); }
  static __device__ __forceinline__ int y(uint32_t k) { return (int)((k >> 12) & 0xFFF); }
  static __device__ __forceinline__ unsigned score(uint32_t k) { return k >> 24; }
};
template <>
struct KeyFmt<uint64_t> {
  static __device__ __forceinline__ uint64_t make(int x, int y, int v) {
    return (uint64_t)((uint32_t)(x - (kEdge - 3)) | ((uint32_t)(y - (kEdge - 3)) << 16)) |
           ((uint64_t)(uint32_t)(v - 1) << 32);
  }
  static __device__ __forceinline__ int x(uint64_t k) { return (int)(k & 0xFFFF); }
  static __device__ __forceinline__ int y(uint64_t k) { return (int)((k >> 16) & 0xFFFF); }
  static __device__ __forceinline__ unsigned score(uint64_t k) { return (unsigned)(k >> 32); }
};

// A cell's geometry by whole dwords from a wave-uniform index: two 16-B scalar loads (a field
// read as int16 became a vector load, and the wait for it exposed a memory latency per cell)
__device__ __forceinline__ CellGeom load_cell(const CellGeom* __restrict__ cells, int i) {
  const int4* p = (const int4*)(cells + i);
  const int4 a = p[0], b = p[1];
  CellGeom c;
  c.x0 = (int16_t)(a.x & 0xFFFF);
  c.y0 = (int16_t)(a.x >> 16);
  c.x1 = (int16_t)(a.y & 0xFFFF);
  c.y1 = (int16_t)(a.y >> 16);
  c.offx = (int16_t)(a.z & 0xFFFF);
  c.offy = (int16_t)(a.z >> 16);
  c.level = (int16_t)(a.w & 0xFFFF);
  c.pad16 = (int16_t)(a.w >> 16);
  c.slot_off = b.x;
  c.slot_cap = b.y;
  c.v_row0 = b.z;
  c.pitch = b.w;
  return c;
}

// raster-order compaction of a cell's keep rows (lane = detection row): out slot, count
template <class K, class VAt>
__device__ __forceinline__ void compact_rows(uint64_t bits, int lane, int y, int cx0,
                                             K* out, int* cnt_out, VAt v_at) {
  const int cnt = __popcll(bits);
  const int incl = wave_scan_incl(cnt);
  int pos = incl - cnt;
  const int nout = __shfl(incl, 63);
  while (bits) {
    const int k = __builtin_ctzll(bits);
    bits &= bits - 1;
    out[pos++] = KeyFmt<K>::make(cx0 + k, y, v_at(k));
  }
  if (lane == 0) *cnt_out = nout;
}

// ---- k_fast_cells: the whole per-cell FAST of ComputeKeyPointsOctTree (ORBextractor.cc:758-796)
// in one wave per cell: the cell ROI is staged in the wave's LDS once; cv::FAST with NMS at
// iniThFAST (:776-780) and, only if no keypoint survives, again at minThFAST on the same staged
// pixels (:782-784); the survivors go to the cell's candidate slot in raster order.  FAST on the
// cell ROI makes the NMS cell-local, so nothing outside the cell's detection pixels is scored,
// and no score map or keep bitmap leaves the wave.
//  (1) cardinal pretest (fast_cardinal2) on row pairs: lanes are columns (two half-waves of
//      two rows each when the cell is at most 32 wide); each lane shifts its flag pair into a
//      register, 8 steps at a time, and the wave compacts the flagged pixels into a queue
//      (lane prefix sum, then each lane writes its own);
//  (2) cornerScore<16> (fast_score) of the queued pixels into a zero-ringed V map (V = score + 1
//      clamped; every other pixel has V = 0, equivalent in the NMS to a score below t);
//  (3) the strict 8-neighbour NMS at the queued pixels with V > t, setting keep bits per row.
// Instantiated for RS x MAXR staged windows: <44, kFcSmallRows> (ROIs up to 41 wide with their
// alignment slack, kFcSmallRows high: the usual ~30-px grid), <48, kCellMax> (up to 45 wide and
// kCellMax high: levels with 2-3 cell rows, 46 KB of LDS per workgroup instead of 70) and
// <72, kCellMax> (any cell); `list` holds the instance's cells.
constexpr int kFcSmallRows = 42;  // ROI rows of the small k_fast_cells instance (44 measured slower)
constexpr int kFcTallRS = 48;     // staged row of the tall instance: ROIs up to 45 px wide
// Stage 1 of one detection chunk (up to 8 steps of STEP rows per lane, two steps per LDS round
// trip): the flags of step s end at bits 15 - 2 (nst - 1 - s) (row r) and 31 - 2 (...) (row
// r + 1) of the returned word; the caller masks rows and columns outside the cell.
template <int RS, int STEP>
__device__ __forceinline__ uint32_t cardinal_chunk(const uint8_t* c0, int nst, int t) {
  uint32_t acc = 0;
  const uint8_t* c = c0;
  int s = 0;
  for (; s + 2 <= nst; s += 2, c += 2 * STEP * RS) {
    uint32_t f0, f1;
    fast_cardinal2x2<RS, STEP * RS>(c, t, f0, f1);
    acc = (acc >> 4) | (f0 >> 2) | f1;
  }
  if (s < nst) acc = (acc >> 2) | fast_cardinal2<RS>(c, t);
  return acc;
}

// the odd bits of [lo, hi] (both odd, lo <= hi), 0 if hi < lo
__device__ __forceinline__ uint32_t odd_bits(int lo, int hi) {
  if (hi < lo) return 0u;
  const uint32_t upto = hi >= 31 ? 0xFFFFFFFFu : ((2u << hi) - 1u);
  return 0xAAAAAAAAu & upto & ~((1u << lo) - 1u);
}

// Each wave takes `cpw` consecutive cells of the list (neighbours: their ROIs share halo rows in
// L2; at most kCellsPerWave, fewer when the launch has few cells, e.g. one drop-in frame); the
// next cell's ROI loads are issued while the current one is processed, so their latency hides
// behind it.
constexpr int kCellsPerWave = 4;

template <int RS, int MAXR, class K>
__global__ __launch_bounds__(256) void k_fast_cells(const uint8_t* __restrict__ pyr,
                                                    int64_t pyr_bytes,
                                                    const CellGeom* __restrict__ cells,
                                                    const int* __restrict__ list, int nlist,
                                                    int ncells, int ini_th, int min_th,
                                                    K* __restrict__ cand, int cand_total,
                                                    int* __restrict__ cell_counts, int cpw) {
  // staged ROI (+ the rows the last pair steps of a half-wave may read past it, masked)
  __shared__ __align__(16) uint8_t s_src[4][(MAXR + 12) * RS];
  __shared__ __align__(16) uint8_t s_vv[4][(MAXR - 4) * RS];
  constexpr int QCAP = (MAXR - 6) * (RS - 9);  // detection pixels of the largest cell
  __shared__ uint16_t s_q[4][QCAP];
  // the keep bits per detection row live in the last 512 B of the wave's staging buffer: slack
  // rows past any ROI (the pretest reads them only masked; a cell is staged before its NMS and
  // its bits are in registers before the next cell is staged)
  static_assert((MAXR + 12) * RS - 512 >= MAXR * RS, "keep rows past every ROI row");
  static_assert(((MAXR + 12) * RS - 512) % 8 == 0, "keep rows 8-B aligned");
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint64_t* const krows = (uint64_t*)(s_src[wid] + (MAXR + 12) * RS - 512);
  int bx, img;
  xcd_block(bx, img);
  const int l0 = (bx * 4 + wid) * cpw;
  if (l0 >= nlist) return;  // wave-uniform; no workgroup barrier below
  const int l1 = min(l0 + cpw, nlist);
  uint8_t* S = s_src[wid];
  uint8_t* V = s_vv[wid];
  uint16_t* q = s_q[wid];
  const uint8_t* pimg = pyr + (int64_t)img * pyr_bytes;
  // ROI staging as aligned dwords: lane l takes word l % kW of rows l / kW + kG u
  constexpr int kW = RS / 4, kG = 64 / kW, kPf = (MAXR + kG - 1) / kG;
  static_assert(63 / kW + kG * (kPf - 1) < MAXR + 12, "staging rows stay inside s_src");
  const int lrow = lane / kW, lword = lane - lrow * kW;
  uint32_t pv[kPf];
  // every lane loads and stores every round, branch-free: rows past the ROI and words past its
  // last one read clamped (in-level) addresses, and those staged bytes are never used (stage 1
  // masks their flags, scores read only detection pixels' windows)
  auto issue = [&](const CellGeom& C) {
    const int rows = C.y1 - C.y0, words = ((C.x0 & 3) + (C.x1 - C.x0) + 3) >> 2;
    const uint8_t* srow = pimg + (C.v_row0 - 3 * C.pitch - 3) + (C.x0 & ~3) - C.x0 +
                          4 * min(lword, words - 1);
#pragma unroll
    for (int u = 0; u < kPf; u++)
      pv[u] = *(const uint32_t*)(srow + (uint32_t)__mul24(min(lrow + kG * u, rows - 1), C.pitch));
  };
  int ci = list[l0];
  CellGeom C = load_cell(cells, ci);
  issue(C);
  for (int li = l0; li < l1; li++) {
    const int rows = C.y1 - C.y0, cols = C.x1 - C.x0;  // <= MAXR, <= RS - 3
    const int dr = rows - 6, cw = cols - 6;            // detection rows / columns
    int* cnt_out = cell_counts + (int64_t)img * ncells + ci;
    // this cell's ROI into LDS (rows up to lrow + kG (kPf - 1) < MAXR + 12), then the next
    // cell's loads in flight
    wave_sync();  // the previous cell's reads of S are done
#pragma unroll
    for (int u = 0; u < kPf; u++) *(uint32_t*)(S + (lrow + kG * u) * RS + 4 * lword) = pv[u];
    const CellGeom Cc = C;
    const int cic = ci;
    if (li + 1 < l1) {
      ci = list[li + 1];
      C = load_cell(cells, ci);
      issue(C);
    }
    if (dr <= 0 || cw <= 0) {
      if (lane == 0) *cnt_out = 0;
      continue;
    }
    (void)cic;
    for (int i = lane; i < (dr + 2) * RS / 4; i += 64) ((uint32_t*)V)[i] = 0u;
    wave_sync();
    const uint8_t* Sx = S + (Cc.x0 & 3);  // pixel (r, c) of the ROI at Sx[r * RS + c]
    const bool half = cw <= 32;           // wave-uniform
    const int col = half ? lane & 31 : lane, sub = half ? 2 * (lane >> 5) : 0, step = half ? 4 : 2;
    const int lstep = half ? 2 : 1;       // log2(step)
    const bool col_ok = col < cw;
    int t = ini_th;
    uint64_t bits = 0;  // this lane's keep row (lane = detection row)
    for (int pass = 0; pass < 2; pass++) {
      // (1) cardinal pretest at t, compacted into q (row << 6 | column)
      int nq = 0;
      for (int rc = 0; rc < dr; rc += 8 * step) {
        const int nst = min(8, (dr - rc + step - 1) >> lstep);  // wave-uniform
        uint32_t acc = half ? cardinal_chunk<RS, 4>(Sx + (rc + sub) * RS + col, nst, t)
                            : cardinal_chunk<RS, 2>(Sx + rc * RS + col, nst, t);
        // rows of this lane in the chunk: rc + sub + step s (+1 in the high half), s < nst;
        // step s's bits sit at 15 - 2 (nst - 1 - s): keep rows < dr and columns < cw
        const int lo = 17 - 2 * nst;
        const int nlo = min(nst, max(0, dr - rc - sub + step - 1) >> lstep);
        const int nhi = min(nst, max(0, dr - rc - sub + step - 2) >> lstep);
        acc &= col_ok ? odd_bits(lo, lo + 2 * nlo - 2) | (odd_bits(lo, lo + 2 * nhi - 2) << 16) : 0u;
        const int cnt = __popc(acc);
        const int incl = wave_scan_incl(cnt);
        int pos = nq + incl - cnt;
        nq += __builtin_amdgcn_readlane(incl, 63);
        // bit b: step s = nst - 8 + (b & 15) / 2, row + 1 in the high half
        const int rbase = rc + sub + step * (nst - 8);
        while (acc) {
          const int b = __builtin_ctz(acc);
          acc &= acc - 1;
          const int r = rbase + step * ((b & 15) >> 1) + (b >> 4);
          q[pos++] = (uint16_t)((r << 6) | col);
        }
      }
      wave_sync();
      // (2) scores of the queued pixels (a fallback pass rescores the iniThFAST ones: same
      // value; two candidates per lane per round measured slower, 0.637 vs 0.595 ms per 512 C2
      // frames)
      for (int j = lane; j < nq; j += 64) {
        const int e = q[j], r = e >> 6, c = e & 63;
        const int sc = fast_score(Sx, RS, c + 3, r + 3);
        V[(r + 1) * RS + c + 1] = (uint8_t)min(255, max(0, sc + 1));
      }
      krows[lane] = 0;
      wave_sync();
      // (3) cv::FAST's strict 8-neighbour NMS at t: a neighbour counts with its score V-1 only
      // if it is a corner at t (V > t), and the count is monotone in V, so the largest
      // neighbour decides: keep <=> V > (nmax > t ? nmax : max(t,1))
      const int t1 = max(t, 1);
      for (int j = lane; j < nq; j += 64) {
        const int e = q[j], r = e >> 6, c = e & 63;
        const uint8_t* p = V + (r + 1) * RS + c + 1;
        const int v = p[0];
        if (v <= t1) continue;
        const int nmax = max(max(max((int)p[-RS - 1], (int)p[-RS]), max((int)p[-RS + 1], (int)p[-1])),
                             max(max((int)p[1], (int)p[RS - 1]), max((int)p[RS], (int)p[RS + 1])));
        if (v > (nmax > t ? nmax : t1)) atomicOr((unsigned long long*)&krows[r], 1ull << c);
      }
      wave_sync();
      bits = lane < dr ? krows[lane] : 0;
      if (__ballot(bits != 0) != 0 || t == min_th) break;  // cell has keypoints, or retried
      t = min_th;  // no keypoint at iniThFAST: FAST again at minThFAST (ORBextractor.cc:782-784)
    }
    const uint8_t* Vr = V + (lane + 1) * RS + 1;
    compact_rows(bits, lane, Cc.y0 + 3 + lane, Cc.x0 + 3,
                 cand + (int64_t)img * cand_total + Cc.slot_off, cnt_out,
                 [&](int kk) { return (int)Vr[kk]; });
  }
}

// ---- k_fast_pairs: two horizontally adjacent FAST cells of one cell row per wave.  Cell j's
// ROI ends 3 px past its detection columns, where cell j + 1's detection columns begin
// (ORBextractor.cc:766-773: iniX = minBorderX + j wCell, maxX = iniX + wCell + 6), so the two
// cells' detection columns are contiguous and one staged ROI of up to 70 x 42 px serves both:
// the cardinal pretest runs on all 64 lanes (one detection column each, cwA + cwB <= 64) instead
// of the 31-32 lanes of a single ~31-px cell, the candidates of both cells share the scoring and
// NMS rounds, and staging, the V map, the scans and the compaction are paid once per pair.  The
// NMS stays cell-local: the V map holds a zero column between the two cells' columns (and the
// zero ring around them), so a neighbour across the cell edge counts as 0, as on the reference's
// per-cell ROI.  A cell without a keypoint at iniThFAST runs FAST again at minThFAST on its own
// columns (:782-784); each cell's survivors go to its own slot in raster order.
// Queue entries: (detection row r) << 6 | column c.  A pass whose candidates outgrow the queue
// (dense texture) scores the rest in place, lane by lane, and then runs the NMS over the V map
// instead of the queue (same result: the NMS candidates are the pixels with V > t).
constexpr int kPairRS = 76;                          // staged ROI row: <= 70 px + 3 alignment
constexpr int kPairRows = kFcSmallRows;              // ROI rows (detection rows <= 36)
constexpr int kPairStage = 14;                       // staging rounds of three 19-dword rows
constexpr int kPairSrc = kPairRS * (kPairRows + 6);  // + the keep rows (krows)
constexpr int kPairKeepRows = 40;                    // >= detection rows
constexpr int kPairVS = 72;                          // V row: ring, cwA, gap, cwB, ring
constexpr int kPairVRows = kPairRows - 4;            // detection rows + 2 ring rows
constexpr int kPairQ = 768;                          // queue entries
constexpr int kPairsPerWave = 4;
#ifndef ORBX_EXP_NO_SINGLES
constexpr bool SINGLES_IN_PAIRS = true;   // unpaired cells through k_fast_pairs
#else
constexpr bool SINGLES_IN_PAIRS = false;
#endif
static_assert(kPairStage * 3 >= kPairRows, "staging covers the ROI");
static_assert(kPairStage * 3 * kPairRS <= kPairSrc - 8 * kPairKeepRows, "keep rows past the staged bytes");
static_assert(kPairKeepRows >= kPairRows - 6, "a keep row per detection row");
static_assert((kPairVS * kPairVRows) % 16 == 0, "V map in 16-B pieces");

// Stage 1 of one detection chunk on all 64 lanes: rows r0 + STEP s and r0 + STEP s + 1 for
// steps s < nst <= 16, two steps per LDS round trip; the flags of step s end at bit s (row
// r0 + STEP s) and bit 16 + s (row r0 + STEP s + 1).  STEP 2: a lane's column over 32 rows;
// STEP 4: the half-wave form (each half-wave takes two of every four rows of one cell at most
// 32 wide, so a single cell's retry pass keeps all 64 lanes busy).
template <int RS, int STEP>
__device__ __forceinline__ uint32_t cardinal_chunk16(const uint8_t* c0, int nst, int t) {
  uint32_t acc = 0;
  const uint8_t* c = c0;
  int s = 0;
  for (; s + 2 <= nst; s += 2, c += 2 * STEP * RS) {
    uint32_t f0, f1;
    fast_cardinal2x2<RS, STEP * RS>(c, t, f0, f1);
    acc = (acc >> 2) | (f0 >> 1) | f1;
  }
  if (s < nst) acc = (acc >> 1) | fast_cardinal2<RS>(c, t);
  return acc >> (16 - nst);
}

#ifdef ORBX_FAST_PROF  // experiment builds only: per-phase wave time of k_fast_pairs (s_memtime)
__device__ unsigned long long g_fast_prof[16];
#define FP_NOW() __builtin_amdgcn_s_memtime()
#define FP_ADD(i, x) (pf[i] += (x))
#else
#define FP_NOW() 0ull
#define FP_ADD(i, x) ((void)(x))
#endif

template <class K>
__global__ __launch_bounds__(256) void k_fast_pairs(const uint8_t* __restrict__ pyr,
                                                    int64_t pyr_bytes,
                                                    const CellGeom* __restrict__ cells,
                                                    const int2* __restrict__ pairs, int npairs,
                                                    int ncells, int ini_th, int min_th,
                                                    K* __restrict__ cand, int cand_total,
                                                    int* __restrict__ cell_counts, int ppw) {
  __shared__ __align__(16) uint8_t s_src[4][kPairSrc];
  __shared__ __align__(16) uint8_t s_vv[4][kPairVS * kPairVRows];
  __shared__ uint16_t s_q[4][kPairQ];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int bx, img;
  xcd_block(bx, img);
  const int p0 = (bx * 4 + wid) * ppw;
  if (p0 >= npairs) return;  // wave-uniform; no workgroup barrier below
  const int p1 = min(p0 + ppw, npairs);
  uint8_t* S = s_src[wid];
  uint8_t* V = s_vv[wid];
  uint16_t* q = s_q[wid];
  // keep bits per detection row: the end of the staging buffer, past every staged byte (the
  // pretest reads rows up to dr + 6 <= 42: inside the staged bytes)
  uint64_t* const krows = (uint64_t*)(S + kPairSrc - 8 * kPairKeepRows);
  // per-row output bases of the emit (2 ints a row): the start of the staging buffer, whose ROI
  // bytes are dead once both passes are done
  int* const rbase = (int*)S;
  static_assert(8 * kPairKeepRows <= kPairSrc - 8 * kPairKeepRows, "row bases below the keep rows");
  const uint8_t* pimg = pyr + (int64_t)img * pyr_bytes;
  // ROI staging: lane = (row lane / 19 of three, dword lane % 19 of the 76-B staged row; lanes
  // 57-63 idle), round u adds three rows: the per-round offsets are uniform.  A lane loads
  // exactly the ROI's dwords: rows past its last row and words past its last dword are not read
  // (their staged bytes are stale and never used: stage 1 masks their flags, scores read
  // detection pixels' windows only), and a round wholly past the ROI issues nothing.
  constexpr int kW = kPairRS / 4;
  const int lrow = lane / kW, lwof = 4 * (lane - kW * lrow);
  const bool sl = lane < 3 * kW;
  uint32_t pv[kPairStage];
#pragma unroll
  for (int u = 0; u < kPairStage; u++) pv[u] = 0u;
  auto issue = [&](const CellGeom& A, const CellGeom& B) {
    const int rows = A.y1 - A.y0;
    const int wb = (A.x0 & 3) + (B.x1 - A.x0);  // staged bytes per row (from the aligned start)
    const uint8_t* src = pimg + (A.v_row0 - 3 * A.pitch - 3) + (A.x0 & ~3) - A.x0 +
                         (uint32_t)(__mul24(lrow, A.pitch) + lwof);
    const bool ok = sl && lwof < wb;
#pragma unroll
    for (int u = 0; u < kPairStage; u++)
      if (ok && lrow + 3 * u < rows) pv[u] = *(const uint32_t*)(src + (uint32_t)(3 * u * A.pitch));
  };
  // a single cell runs as a pair with an empty cell B (pr.y >= ncells: a geometry entry past
  // the level cells with no detection columns, ending where cell A ends)
  int2 pr = pairs[p0];
  CellGeom A = load_cell(cells, pr.x), B = load_cell(cells, pr.y);
  issue(A, B);
#ifdef ORBX_FAST_PROF
  uint64_t pf[16] = {};
  const uint64_t tk0 = FP_NOW();
#endif
  for (int pi = p0; pi < p1; pi++) {
    uint64_t tp = FP_NOW();
    FP_ADD(8, 1);
    wave_sync();  // the previous pair's reads of S are done
    if (sl) {
#pragma unroll
      for (int u = 0; u < kPairStage; u++) *(uint32_t*)(S + (lrow + 3 * u) * kPairRS + lwof) = pv[u];
    }
    const CellGeom Ac = A, Bc = B;
    const int2 pc = pr;
    if (pi + 1 < p1) {  // the next pair's loads in flight while this one is processed
      pr = pairs[pi + 1];
      A = load_cell(cells, pr.x);
      B = load_cell(cells, pr.y);
      issue(A, B);
    }
    const int dr = Ac.y1 - Ac.y0 - 6;                      // detection rows, both cells
    const int cwA = Ac.x1 - Ac.x0 - 6, cw = cwA + (Bc.x1 - Bc.x0 - 6);  // detection columns
    for (int i = lane; i < ((dr + 2) * kPairVS + 15) / 16; i += 64) ((uint4*)V)[i] = make_uint4(0u, 0u, 0u, 0u);
    wave_sync();
    const uint8_t* Sx = S + (Ac.x0 & 3);  // pixel (r, c) of the ROI at Sx[r * RS + c]
    const uint64_t mA = (1ull << cwA) - 1;  // cwA <= 60
    const uint64_t mB = (cw >= 64 ? ~0ull : (1ull << cw) - 1) & ~mA;
    // V byte of detection pixel (r, c): one ring row and column, the gap column after cell A
    auto vofs = [&](int r, int c) { return __mul24(r + 1, kPairVS) + c + 1 + (c >= cwA ? 1 : 0); };
    auto score_at = [&](int r, int c) {
      const int sc = fast_score(Sx, kPairRS, c + 3, r + 3);
      const int v = min(255, max(0, sc + 1));
      V[vofs(r, c)] = (uint8_t)v;
      return v;
    };
    uint64_t allow = mA | mB;  // the columns this pass detects on
    uint64_t bits1 = 0, keep1 = 0;
    uint64_t bits = 0;  // this lane's keep row (lane = detection row)
    int t = ini_th;
    bool any_dense = false;
    // a pass over one cell at most 32 wide (a single cell, or a pair's retry pass) takes the
    // half-wave form
    bool half = cw == cwA && cwA <= 32;
    int c_off = 0, cw_r = cw; // the half-wave pass's cell: first detection column and width
    int qbase = 0;            // pass 2 queues past pass 1's corners (kept for the emit)
    int nc = 0;               // corners (decoded (r << 6) | c) at q[0, nc)
    { const uint64_t t2 = FP_NOW(); FP_ADD(0, t2 - tp); tp = t2; }
#if defined(ORBX_EXP_FAST_STAGE_ONLY)  // timing experiments only (wrong output: no keys)
    if (lane == 0) cell_counts[(int64_t)img * ncells + pc.x] = 0;
    if (lane == 0 && pc.y < ncells) cell_counts[(int64_t)img * ncells + pc.y] = 0;
    continue;
#endif
    for (int pass = 0; pass < 2; pass++) {
      // (1) cardinal pretest at t, the flagged pixels queued as raw flag bits (b << 6 | column,
      // bit 11 = the 32-row chunk, or the half-wave in the half form; decoded when scored), or
      // scored in place past kPairQ
      // full form: lane = column, rows rc + 2 (b & 15) + (b >> 4); half form: lane & 31 = the
      // cell's column, rows 2 (lane >> 5) + 4 (b & 15) + (b >> 4)
      const int hsub = lane >> 5;
      const int lcol = half ? c_off + min(lane & 31, cw_r - 1) : lane;
      const bool col_ok = half ? (lane & 31) < cw_r : ((allow >> lane) & 1) != 0;
      const int hsh = half ? 1 : 5, bsh = half ? 2 : 1;  // r = (hb << hsh) + ((b & 15) << bsh) + (b >> 4)
      int nq = qbase;
      bool dense = false;
      const int nchunks = half ? 1 : (dr + 31) >> 5;
      for (int ch = 0; ch < nchunks; ch++) {
        uint32_t acc;
        int hb;
        if (half) {
          const int sub = 2 * hsub;
          const int nst = (dr + 3) >> 2;  // wave-uniform
          acc = cardinal_chunk16<kPairRS, 4>(Sx + sub * kPairRS + lcol, nst, t);
          const int nlo = min(nst, max(0, dr - sub + 3) >> 2), nhi = min(nst, max(0, dr - sub + 2) >> 2);
          acc &= col_ok ? (((1u << nlo) - 1u) | (((1u << nhi) - 1u) << 16)) : 0u;
          hb = hsub;
        } else {
          const int rc = ch << 5;
          const int nst = min(16, (dr - rc + 1) >> 1);  // wave-uniform
          const int nodd = min(16, (dr - rc) >> 1);     // steps whose second row is a detection row
          acc = cardinal_chunk16<kPairRS, 2>(Sx + rc * kPairRS + lane, nst, t);
          acc &= col_ok ? (((1u << nst) - 1u) | (((1u << nodd) - 1u) << 16)) : 0u;
          hb = ch;
        }
        const int cnt = __popc(acc);
        const int incl = wave_scan_incl(cnt);
        const int tot = __builtin_amdgcn_readlane(incl, 63);
        if (nq + tot > kPairQ) {  // wave-uniform, rare: score this chunk's pixels in place
          dense = true;
          while (acc) {
            const int b = __builtin_ctz(acc);
            acc &= acc - 1;
            score_at((hb << hsh) + ((b & 15) << bsh) + (b >> 4), lcol);
          }
          continue;
        }
        const int ebase = (hb << 11) | lcol;
        int pos = nq + incl - cnt;
        nq += tot;
        while (acc) {
          const int b = __builtin_ctz(acc);
          acc &= acc - 1;
          q[pos++] = (uint16_t)((b << 6) | ebase);
        }
      }
      any_dense = any_dense || dense;
      wave_sync();
#if defined(ORBX_EXP_FAST_PRETEST_ONLY)
      break;
#endif
#if defined(ORBX_EXP_FAST_RETRY_PRETEST_ONLY)
      if (pass == 1) {
        bits = bits1 & keep1;
        break;
      }
#endif
      { const uint64_t t2 = FP_NOW(); FP_ADD(1 + 3 * pass, t2 - tp); tp = t2; FP_ADD(11, nq - qbase); FP_ADD(10, half ? 1 : 0); }
      // (2) cornerScore of the queued pixels (a fallback pass rescores its cell's iniThFAST
      // candidates: same value); the corners at t (V > max(t, 1): the NMS candidates, about a
      // quarter of the queue) are compacted in place, decoded to (r << 6) | c, after the corners
      // already kept (a round reads its entries before any lane writes, and writes only below
      // the next round's)
      const int t1 = max(t, 1);
      const int cbase = qbase;
      nc = qbase;
      for (int j0 = qbase; j0 < nq; j0 += 64) {
        const int j = j0 + lane;
        int rcode = 0;
        bool corner = false;
        if (j < nq) {
          const int e = q[j], hbb = e >> 6, c = e & 63;
          const int r = ((hbb >> 5) << hsh) + ((hbb & 15) << bsh) + ((hbb >> 4) & 1);
          rcode = (r << 6) | c;
          corner = score_at(r, c) > t1;
        }
        const uint64_t m = __ballot(corner);
        if (corner) q[nc + lane_rank(m)] = (uint16_t)rcode;
        nc += __popcll(m);
      }
      if (lane < kPairKeepRows) krows[lane] = 0;
      wave_sync();
      { const uint64_t t2 = FP_NOW(); FP_ADD(2 + 3 * pass, t2 - tp); tp = t2; FP_ADD(12, nc - cbase); }
      // (3) the strict 8-neighbour NMS at t over this pass's corners: keep <=> V > (nmax > t ?
      // nmax : max(t,1)), the largest neighbour deciding (k_fast_cells)
      auto keep_at = [&](int r, int c) -> bool {
        const uint8_t* p = V + vofs(r, c);
        const int v = p[0];
        if (v <= t1) return false;
        const int nmax =
            max(max(max((int)p[-kPairVS - 1], (int)p[-kPairVS]), max((int)p[-kPairVS + 1], (int)p[-1])),
                max(max((int)p[1], (int)p[kPairVS - 1]), max((int)p[kPairVS], (int)p[kPairVS + 1])));
        return v > (nmax > t ? nmax : t1);
      };
      if (!dense) {
        for (int j = cbase + lane; j < nc; j += 64) {
          const int e = q[j], r = e >> 6, c = e & 63;
          if (keep_at(r, c)) atomicOr((unsigned long long*)&krows[r], 1ull << c);
        }
        wave_sync();
        bits = lane < dr ? krows[lane] : 0;
      } else {  // some candidates were not queued: every pixel of this lane's row (rare)
        bits = 0;
        if (lane < dr)
          for (int c = 0; c < cw; c++)
            if (((allow >> c) & 1) && keep_at(lane, c)) bits |= 1ull << c;
      }
      bits &= allow;
      { const uint64_t t2 = FP_NOW(); FP_ADD(3 + 3 * pass, t2 - tp); tp = t2; FP_ADD(9, pass); }
      if (pass == 1) {
        bits |= bits1 & keep1;
        break;
      }
      // a cell without keypoints at iniThFAST (an empty cell B has nothing to retry)
      const bool needA = __ballot((bits & mA) != 0) == 0;
      const bool needB = mB != 0 && __ballot((bits & mB) != 0) == 0;
#if defined(ORBX_EXP_FAST_NO_RETRY)
      break;
#endif
      if ((!needA && !needB) || t == min_th) break;  // every cell has keypoints, or no retry left
      // FAST again at minThFAST on the columns of the cells without keypoints
      bits1 = bits;
      keep1 = (needA ? 0 : mA) | (needB ? 0 : mB);
      allow = (needA ? mA : 0) | (needB ? mB : 0);
      t = min_th;
      if (needA != needB) {  // one cell: the half-wave form when it is at most 32 wide
        c_off = needA ? 0 : cwA;
        cw_r = needA ? cwA : cw - cwA;
        half = cw_r <= 32;
      }
      qbase = nc;
    }
    // (4) each cell's survivors to its slot in raster order
#if defined(ORBX_EXP_FAST_PRETEST_ONLY) || defined(ORBX_EXP_FAST_NO_EMIT)
    if (lane == 0) cell_counts[(int64_t)img * ncells + pc.x] = __popcll(bits) & 0;
    if (lane == 0 && pc.y < ncells) cell_counts[(int64_t)img * ncells + pc.y] = 0;
    continue;
#endif
    uint64_t bA = bits & mA, bB = bits >> cwA;
    const int nA = __popcll(bA), nB = __popcll(bB);
    const int packed = nA | (nB << 16);
    const int incl = wave_scan_incl(packed);
    const int tot = __builtin_amdgcn_readlane(incl, 63);
    if (lane == 0) {
      cell_counts[(int64_t)img * ncells + pc.x] = tot & 0xFFFF;
      if (pc.y < ncells) cell_counts[(int64_t)img * ncells + pc.y] = tot >> 16;
    }
    K* const candA = cand + (int64_t)img * cand_total + Ac.slot_off;
    K* const candB = cand + (int64_t)img * cand_total + Bc.slot_off;
    const int x0 = Ac.x0 + 3;
    if (!any_dense) {
      // by rank, one lane per corner: a kept corner (r, c) goes to its cell's keys of the rows
      // above r plus the kept bits left of c in row r; every kept pixel is a corner of the pass
      // that kept it, queued in q[0, nc) (pass 1's corners stay in front of pass 2's; a pixel
      // queued by both passes writes the same key to the same place twice)
      if (lane < dr) {
        const int ex = incl - packed;
        rbase[2 * lane] = ex & 0xFFFF;
        rbase[2 * lane + 1] = (ex >> 16) - nA;  // cell B: its rank counts cell A's bits of the row
        krows[lane] = bits;
      }
      wave_sync();
      for (int j = lane; j < nc; j += 64) {
        const int e = q[j], r = e >> 6, c = e & 63;
        const uint64_t kr = krows[r];
        if ((kr >> c) & 1) {
          const bool isB = c >= cwA;
          const int pos = rbase[2 * r + (isB ? 1 : 0)] + __popcll(kr & ((1ull << c) - 1));
          (isB ? candB : candA)[pos] = KeyFmt<K>::make(x0 + c, Ac.y0 + 3 + r, (int)V[vofs(r, c)]);
        }
      }
    } else {
      // each lane (detection row) writes its row's keys, cell A's and cell B's in two loops
      K* outA = candA + ((incl - packed) & 0xFFFF);
      K* outB = candB + ((incl - packed) >> 16);
      const int y = Ac.y0 + 3 + lane;
      const uint8_t* Vr = V + __mul24(lane + 1, kPairVS) + 1;
      while (bA) {
        const int c = __builtin_ctzll(bA);
        bA &= bA - 1;
        *outA++ = KeyFmt<K>::make(x0 + c, y, (int)Vr[c]);
      }
      const uint8_t* VrB = Vr + cwA + 1;  // cell B's columns, past the gap column
      while (bB) {
        const int c = __builtin_ctzll(bB);
        bB &= bB - 1;
        *outB++ = KeyFmt<K>::make(x0 + cwA + c, y, (int)VrB[c]);
      }
    }
    { const uint64_t t2 = FP_NOW(); FP_ADD(7, t2 - tp); }
  }
#ifdef ORBX_FAST_PROF
  pf[13] = FP_NOW() - tk0;
  if (lane == 0)
    for (int i = 0; i < 16; i++) atomicAdd(&g_fast_prof[i], (unsigned long long)pf[i]);
#endif
}

// ------------------------------------------------------------------ k_octree
// ORBextractor::DistributeOctTree (ORBextractor.cc:525-733) for one (image, level) per
// workgroup.  The std::list is represented by node arrays kept in list order in LDS:
// a division pass pushes children to the front, so after each step the order is
// [children, newest seq first] + [undivided nodes, previous order].  A node's
// retained key is its max response with the lowest candidate index (DivideNode is a stable
// partition, so a node's keys stay in candidate order).  The final-refinement sort uses the
// canonical (size, creation sequence) tie-break.
//
// Counting by bins instead of key passes.  A node's division is fixed by its rectangle (the
// ceil midpoints of DivideNode, ORBextractor.cc:472-473), so every key's path down the tree —
// its quadrant digit at each depth below a node — is known in advance.  A refine sweep gives
// every node that may still divide (> 1 key) a block of 4^R bins, one per R-digit path below
// it, and every other node one bin; each key adds itself to the bin of its path, and the bins'
// prefix sums then give the key count of every descendant down to R levels as the difference
// of two sums (a node's bin range splits into four quarters, one per child).  Passes only touch
// node arrays; the keys are swept again only when a node that may divide has no digit left
// (at most a few times per level, usually once), and once at the end to retain the best key of
// each node (a key's node = the node whose bin range holds the key's bin).
// Threads per (image, level) workgroup: 256, or 1024 for levels whose octree frame exceeds
// kOctBigArea px (a workgroup holds ~130 KB of LDS there, one per CU, and its key sweeps run 16
// waves wide).
constexpr int kOctNT = 256, kOctNTBig = 1024;
constexpr int64_t kOctBigArea = 1 << 20;
constexpr int kOctRegKeys = 8;        // keys per thread per register chunk
constexpr int kOctBins = 1024;        // bins per (image, level) at least: batch plans,
constexpr int kOctBinsFew = 8192;     // few-image plans and the 1024-thread instance
constexpr size_t kOctMaxSmem = 150 * 1024;  // dynamic LDS of one octree workgroup

#ifdef ORBX_OCT_PROF  // experiment builds only: per-phase workgroup time of k_octree (s_memtime)
__device__ unsigned long long g_oct_prof[8 * 16];
#define OP_NOW() __builtin_amdgcn_s_memtime()
#define OP_ADD(i, x) (opf[i] += (x))
#else
#define OP_NOW() 0ull
#define OP_ADD(i, x) ((void)(x))
#endif

#ifdef ORBX_OCT_PROF
__device__ unsigned long long g_oct_sub[8];  // oct_refine's steps, level 0 only
#define OS_MARK(i) do { if (X.level0) { const uint64_t t_ = OP_NOW(); if (threadIdx.x == 0) atomicAdd(&g_oct_sub[i], (unsigned long long)(t_ - ts_)); ts_ = t_; } } while (0)
#else
#define OS_MARK(i) ((void)0)
#endif

// Where the octree keeps its keys (KeyFmt<K>) and their bins.  Thread t owns keys t, t + NT,
// t + 2 NT, ... (NT threads); they are processed in chunks of kOctRegKeys held in registers,
// slot r of chunk c being key t + NT (c kOctRegKeys + r).
//   RegKeys<NT>: one chunk (n <= kOctRegKeys NT): keys and bins stay in registers;
//   MemKeys<NT>: larger levels, keys and bins in global scratch (L2-resident): a sweep loads a
//                chunk with all its loads in flight, works on the registers and stores the bins
//                back (one load latency per chunk instead of one per key).
template <int NT, class K>
struct RegKeys {
  using Key = K;
  K key[kOctRegKeys];
  int lab[kOctRegKeys];
  int n;
  __device__ int nchunks() const { return 1; }
  __device__ void load(int, bool) {}
  __device__ void store_labs(int) {}
  __device__ K get_key(int r) const { return key[r]; }
  __device__ int get_lab(int r) const { return lab[r]; }
  __device__ void set_lab(int r, int v) { lab[r] = v; }
};

template <int NT, class K>
struct MemKeys {
  using Key = K;
  K* keys;
  int* labs;
  int n;
  K key[kOctRegKeys];
  int lab[kOctRegKeys];
  __device__ int nchunks() const { return (n + NT * kOctRegKeys - 1) / (NT * kOctRegKeys); }
  __device__ void load(int c, bool want_labs) {
#pragma unroll
    for (int r = 0; r < kOctRegKeys; r++) {
      const int k = threadIdx.x + NT * (c * kOctRegKeys + r);
      key[r] = k < n ? keys[k] : K(0);
      lab[r] = (want_labs && k < n) ? labs[k] : 0;
    }
  }
  __device__ void store_labs(int c) {
#pragma unroll
    for (int r = 0; r < kOctRegKeys; r++) {
      const int k = threadIdx.x + NT * (c * kOctRegKeys + r);
      if (k < n) labs[k] = lab[r];
    }
  }
  __device__ K get_key(int r) const { return key[r]; }
  __device__ int get_lab(int r) const { return lab[r]; }
  __device__ void set_lab(int r, int v) { lab[r] = v; }
};

// every key of this thread: f(r, k) for key k < n in register slot r, then g(r, k) for every
// such key of the chunk.  f only reads LDS (the loads of all slots overlap); g holds the LDS
// atomics, which would otherwise order every slot's loads behind the previous slot's atomic.
// `want_labs` loads a chunk's bins with its keys, `labs_out` stores them back after it
// (MemKeys only).
template <int NT, class KS, class F, class G>
__device__ __forceinline__ void each_key(KS& ks, bool want_labs, bool labs_out, F f, G g) {
  const int nc = ks.nchunks();
  for (int c = 0; c < nc; c++) {
    ks.load(c, want_labs);
#pragma unroll
    for (int r = 0; r < kOctRegKeys; r++) {
      const int k = threadIdx.x + NT * (c * kOctRegKeys + r);
      if (k < ks.n) f(r, k);
    }
#pragma unroll
    for (int r = 0; r < kOctRegKeys; r++) {
      const int k = threadIdx.x + NT * (c * kOctRegKeys + r);
      if (k < ks.n) g(r, k);
    }
    if (labs_out) ks.store_labs(c);
  }
}

// ---- node storage, shared steps
// A node is its bin range: its rectangle never needs storing, since a key's digits below the
// node come from the path tables and the node's depth, and its children's counts from the bins.
struct OctNodes {
  int *cnt, *seq;
  // first bin << 9 | depth << 4 | digits left: the node's bins are [first, first + 4^digits)
  int* bl;
};

struct OctCtx {
  OctNodes A, B;
  int *cc, *t1, *t2, *t3, *t4, *s_tmp, *s_misc;
  int* bins;   // [bin_cap + 8]: keys per bin, then their exclusive prefix sums
  int* table;  // [bin_cap + 8], in cc's LDS: bin -> node position (forward-filled per node)
  int bin_cap;
  uint64_t *pk, *s_tmp64;
  void* outk;  // K[] of the level's retained keys, in candidate order
  int* opos;   // their node-order (output) positions
  int tcap;    // ints in the table's LDS
  int* oc;
  const uint32_t *px, *py;  // the level's quadrant paths (Geometry::octpath)
  int level0;               // profiling builds: this workgroup runs level 0
};

// Per-thread chunks of whole int4s over [0, M) (bin arrays are 16-B aligned): [beg, end)
template <int NT>
__device__ __forceinline__ void int4_chunk(int M, int& beg, int& end) {
  const int per = ((M + NT - 1) / NT + 3) & ~3;
  beg = min((int)threadIdx.x * per, M);
  end = min(beg + per, M);
}

// exclusive scan of a bin array a[0..M) in place, four bins per LDS access (GUARD false: the
// caller knows s_tmp has no pending reader, so the scan skips grp_excl's leading barrier)
template <int NT, bool GUARD = true>
__device__ int bins_scan_excl(int* a, int M, int* s_tmp) {
  int beg, end;
  int4_chunk<NT>(M, beg, end);
  int sum = 0, i = beg;
  for (; i + 4 <= end; i += 4) {
    const int4 v = *(const int4*)(a + i);
    sum += v.x + v.y + v.z + v.w;
  }
  for (; i < end; i++) sum += a[i];
  int total;
  int run;
  if constexpr (GUARD) {
    run = grp_excl<NT>(sum, s_tmp, total);
  } else {
    const int inc = wave_scan_incl(sum);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 63) s_tmp[wid] = inc;
    __syncthreads();
    int pre = 0;
    total = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; w++) {
      const int x = s_tmp[w];
      pre += w < wid ? x : 0;
      total += x;
    }
    run = pre + inc - sum;
  }
  for (i = beg; i + 4 <= end; i += 4) {
    const int4 v = *(const int4*)(a + i);
    int4 o;
    o.x = run; run += v.x;
    o.y = run; run += v.y;
    o.z = run; run += v.z;
    o.w = run; run += v.w;
    *(int4*)(a + i) = o;
  }
  for (; i < end; i++) {
    const int x = a[i];
    a[i] = run;
    run += x;
  }
  __syncthreads();
  return total;
}

// table[b] = the node whose bin range holds bin b: each node's first bin marked, then every
// thread's chunk forward-filled from the last mark before it (bins of dropped empty children
// take their predecessor's node; no key lies in them)
template <int NT>
__device__ void oct_fill_table(int* table, const OctNodes& cur, int size, int gen_total,
                               int* s_tmp) {
  int beg, end;
  int4_chunk<NT>(gen_total, beg, end);
  int i = beg;
  for (; i + 4 <= end; i += 4) *(int4*)(table + i) = make_int4(-1, -1, -1, -1);
  for (; i < end; i++) table[i] = -1;
  __syncthreads();
  for (int k = threadIdx.x; k < size; k += NT) table[cur.bl[k] >> 9] = k;
  __syncthreads();
  int last = -1;
  for (i = beg; i + 4 <= end; i += 4) {
    const int4 v = *(const int4*)(table + i);
    last = v.w >= 0 ? i + 3 : v.z >= 0 ? i + 2 : v.y >= 0 ? i + 1 : v.x >= 0 ? i : last;
  }
  for (; i < end; i++)
    if (table[i] >= 0) last = i;
  const int carry = block_max_excl<NT>(last, s_tmp);
  int nd = carry >= 0 ? table[carry] : -1;
  for (i = beg; i + 4 <= end; i += 4) {
    int4 v = *(const int4*)(table + i);
    v.x = v.x >= 0 ? (nd = v.x) : nd;
    v.y = v.y >= 0 ? (nd = v.y) : nd;
    v.z = v.z >= 0 ? (nd = v.z) : nd;
    v.w = v.w >= 0 ? (nd = v.w) : nd;
    *(int4*)(table + i) = v;
  }
  for (; i < end; i++) {
    const int v = table[i];
    if (v >= 0) nd = v;
    else table[i] = nd;
  }
  __syncthreads();
}

// initial nodes (ORBextractor.cc:530-567): the keys' first bins are their initial node
// indices; the non-empty nodes go to X.B in order with one bin each.  Returns their count.
template <int NT, class KS>
__device__ int oct_initial(const LevelGeom& G, const OctCtx& X, KS& ks) {
  using K = typename KS::Key;
  const int tid = threadIdx.x, nini = G.nini;
  const OctNodes A = X.A, B = X.B;
  // (the initial nodes' columns, ni.UL / ni.UR = cv::Point2i(hX * (float)i, 0), :540-544, are
  // in the path tables)
  for (int i = tid; i < nini; i += NT) {
    A.cnt[i] = 0;
    A.seq[i] = i;
  }
  __syncthreads();
  each_key<NT>(
      ks, false, true,
      [&](int j, int) {
        const float x = (float)KeyFmt<K>::x(ks.get_key(j));
        ks.set_lab(j, min((int)(x / G.hx), nini - 1));
      },
      [&](int j, int) { atomicAdd(&A.cnt[ks.get_lab(j)], 1); });
  __syncthreads();
  // drop empty initial nodes, keep order
  for (int i = tid; i < nini; i += NT) X.t1[i] = A.cnt[i] > 0;
  __syncthreads();
  const int size = block_scan_excl<NT>(X.t1, nini, X.s_tmp);
  for (int i = tid; i < nini; i += NT)
    if (A.cnt[i] > 0) {
      const int j = X.t1[i];
      B.cnt[j] = A.cnt[i]; B.seq[j] = A.seq[i];
      B.bl[j] = i << 9;
    }
  __syncthreads();
  return size;
}

// A new generation of bins: R digits below every node with > 1 key, one bin for the others
// (R as large as the bin capacity allows, capped near the key count: the bins are scanned and
// filled per refine, so a refine costs O(bins + keys)).
template <int NT, class KS>
__device__ void oct_refine(const OctCtx& X, KS& ks, const OctNodes& cur, int size,
                           int& gen_total) {
  using K = typename KS::Key;
  const int tid = threadIdx.x;
  int *t2 = X.t2, *t3 = X.t3, *bins = X.bins, *table = X.table;
#ifdef ORBX_OCT_PROF
  uint64_t ts_ = OP_NOW();
#endif
  oct_fill_table<NT>(table, cur, size, gen_total, X.s_tmp);
  OS_MARK(0);
  // the nodes that may divide and the digits R, then each node's first new bin (t3): every
  // thread owns a contiguous chunk of nodes, so one wave scan and one barrier per total
  const int lane = tid & 63, wid = tid >> 6;
  const int per = (size + NT - 1) / NT;
  const int beg = min(tid * per, size), end = min(beg + per, size);
  int act = 0;
  for (int i = beg; i < end; i++) {
    const int a = cur.cnt[i] > 1;
    t2[i] = a;
    act += a;
  }
  {
    const int ai = wave_scan_incl(act);
    if (lane == 63) X.s_tmp[wid] = ai;
  }
  __syncthreads();
  int nact = 0;
#pragma unroll
  for (int w = 0; w < NT / 64; w++) nact += X.s_tmp[w];
  const int nin = size - nact;
  const int lim = min(X.bin_cap, max(4 * size, ks.n));
  int R = 1;
  while (R < 15 && nin + ((int64_t)nact << (2 * (R + 1))) <= lim) R++;
  int run = 0;
  for (int i = beg; i < end; i++) {
    t3[i] = run;
    run += t2[i] ? 1 << (2 * R) : 1;
  }
  const int ri = wave_scan_incl(run);
  if (lane == 63) X.s_tmp64[wid] = (uint64_t)ri;
  __syncthreads();
  int off = ri - run;
  gen_total = 0;
#pragma unroll
  for (int w = 0; w < NT / 64; w++) {
    const int x = (int)X.s_tmp64[w];
    off += w < wid ? x : 0;
    gen_total += x;
  }
  for (int i = beg; i < end; i++) t3[i] += off;  // t3: each node's first new bin
  OS_MARK(1);
  for (int i = 4 * tid; i <= gen_total; i += 4 * NT) *(int4*)(bins + i) = make_int4(0, 0, 0, 0);
  __syncthreads();
  OS_MARK(2);
  each_key<NT>(
      ks, true, true,
      [&](int j, int) {
        const int nd = table[ks.get_lab(j)];
        int b = t3[nd];
        if (t2[nd]) {  // the key's quadrant digits below its node (DivideNode, :487-522)
          const K key = ks.get_key(j);
          const uint64_t path =
              (uint64_t)(X.px[KeyFmt<K>::x(key)] | X.py[KeyFmt<K>::y(key)]) << 32;
          const int sh = 2 * (32 - ((cur.bl[nd] >> 4) & 31) - R);  // < 0: below depth 32, 0s
          b += sh >= 0 ? (int)((path >> sh) & ((1u << (2 * R)) - 1)) : 0;
        }
        ks.set_lab(j, b);
      },
      [&](int j, int) { atomicAdd(&bins[ks.get_lab(j)], 1); });
  __syncthreads();
  OS_MARK(3);
  bins_scan_excl<NT, false>(bins, gen_total + 1, X.s_tmp);
  OS_MARK(4);
  for (int i = tid; i < size; i += NT)
    cur.bl[i] = (t3[i] << 9) | (cur.bl[i] & (31 << 4)) | (t2[i] ? R : 0);
  __syncthreads();
  OS_MARK(5);
}

// 3. retain the best key per node (max response, first in candidate order)
template <int NT, class KS>
__device__ void oct_retain(const OctCtx& X, KS& ks, const OctNodes& cur, int size,
                           int gen_total, const typename KS::Key* keys_mem) {
  using K = typename KS::Key;
  const int tid = threadIdx.x;
  oct_fill_table<NT>(X.table, cur, size, gen_total, X.s_tmp);
  unsigned* best = (unsigned*)X.t1;
  for (int i = tid; i < size; i += NT) best[i] = 0;
  __syncthreads();
  each_key<NT>(
      ks, true, false, [&](int j, int) { ks.set_lab(j, X.table[ks.get_lab(j)]); },
      [&](int j, int k) {
        atomicMax(&best[ks.get_lab(j)],
                  (KeyFmt<K>::score(ks.get_key(j)) << 24) | (0xFFFFFFu - (unsigned)k));
      });
  __syncthreads();
  K* outk = (K*)X.outk;
  // every node holds a key; the clamp only keeps a broken invariant from reading past them
  auto winner = [&](int i) { return min((int)(0xFFFFFFu - (best[i] & 0xFFFFFFu)), ks.n - 1); };
  // The retained keys go out in candidate order (cells in raster order, raster order inside a
  // cell) with their node-order positions, where k_describe writes each keypoint: its
  // workgroups then take spatial neighbours, whose patches share cache lines.  A key's place is
  // the number of retained keys before it in candidate order: a bitmap over the candidates
  // (the bin table's LDS, free after the sweep) and its prefix popcounts.
  const int W = (ks.n + 31) >> 5;
  if (2 * W > X.tcap) {  // no room: node order
    for (int i = tid; i < size; i += NT) {
      outk[i] = keys_mem[winner(i)];
      X.opos[i] = i;
    }
  } else {
    unsigned* bm = (unsigned*)X.table;
    int* pre = X.table + W;
    for (int w = tid; w < W; w += NT) bm[w] = 0u;
    __syncthreads();
    for (int i = tid; i < size; i += NT) {
      const int k = winner(i);
      atomicOr(&bm[k >> 5], 1u << (k & 31));
    }
    __syncthreads();
    int beg, end;
    int4_chunk<NT>(W, beg, end);
    int sum = 0;
    for (int w = beg; w < end; w++) sum += __popc(bm[w]);
    int total;
    int run = grp_excl<NT>(sum, X.s_tmp, total);
    for (int w = beg; w < end; w++) {
      pre[w] = run;
      run += __popc(bm[w]);
    }
    __syncthreads();
    for (int i = tid; i < size; i += NT) {
      const int k = winner(i);
      const int r = pre[k >> 5] + __popc(bm[k >> 5] & ((1u << (k & 31)) - 1u));
      outk[r] = keys_mem[k];
      X.opos[r] = i;
    }
  }
  if (tid == 0) *X.oc = size;
}

// A divided node's children into the next list (nxt): the non-empty quadrants in order at
// base, base - 1, ..., sequence numbers seq0, seq0 + 1, ..., each with its quarter of the
// parent's bin range, one level deeper
__device__ __forceinline__ void oct_push_children(const OctNodes& nxt, int bl, const int (&c)[4],
                                                  int base, int seq0) {
  const int ls = (bl & 15) - 1, s4 = 1 << (2 * ls);
  const int depth = min((bl & (31 << 4)) + (1 << 4), 31 << 4);
  int j = 0;
#pragma unroll
  for (int q = 0; q < 4; q++) {
    if (c[q] > 0) {
      const int pos = base - j;
      nxt.cnt[pos] = c[q];
      nxt.seq[pos] = seq0 + j;
      nxt.bl[pos] = (((bl >> 9) + q * s4) << 9) | depth | ls;
      j++;
    }
  }
}

// ---- the passes, workgroup form (256 / 1024 threads): node arrays in LDS, one barrier per step
template <int NT, class KS>
__device__ __forceinline__ void octree_core(const LevelGeom& G, const OctCtx& X, KS& ks,
                                            const typename KS::Key* keys_mem, int level = 0) {
  const int tid = threadIdx.x;
#ifdef ORBX_OCT_PROF
  uint64_t opf[16] = {};
#endif
  uint64_t tq = OP_NOW();
  int *cc = X.cc, *t1 = X.t1, *t2 = X.t2, *t3 = X.t3, *t4 = X.t4, *s_tmp = X.s_tmp,
      *s_misc = X.s_misc, *bins = X.bins;
  int size = oct_initial<NT>(G, X, ks);
  { const uint64_t t2 = OP_NOW(); OP_ADD(0, t2 - tq); tq = t2; }
  OctNodes cur = X.B, nxt = X.A;
  int gen_total = G.nini;  // bins of the current generation
  int seqc = G.nini;
  bool final_mode = false;
  const int N = G.nfeat;
  // -1: the next pass checks its nodes for a refine itself; else the previous outer pass's
  // verdict (a child without digits left that may divide)
  int need_known = -1;
  const int lane = tid & 63, wid = tid >> 6;
  for (int iter = 0; iter < 4096; iter++) {
    const int prevSize = size;
    // a node that may divide with no digit left in its bin block: new bins first
    int need = need_known;
    if (need < 0) {
      need = 0;
      for (int i = tid; i < size; i += NT) need |= cur.cnt[i] > 1 && (cur.bl[i] & 15) == 0;
      need = block_sum<NT>(need, s_tmp);
    }
    if (need) oct_refine<NT>(X, ks, cur, size, gen_total);
    { const uint64_t t2 = OP_NOW(); OP_ADD(1, t2 - tq); tq = t2; OP_ADD(7, need ? 1 : 0); }
    int T, newSize, nToExpand = 0;
    if (!final_mode) {
      // Outer pass (list order) in two steps, one barrier each.  Every thread owns a contiguous
      // chunk of nodes for the whole pass (the scan's chunks), so a node's quadrant counts,
      // flags and chunk-local prefix never cross threads before the scan: (1) quadrant counts
      // (the four quarters of the node's bin range) and the packed per-node terms — childPre
      // (bits 0-19), rank among undivided nodes (20-39), children with > 1 key (40-) — summed
      // along the chunk, one wave scan, the wave totals in LDS; (2) every node to the next
      // list (children pushed to the front, newest first; the undivided after them in order),
      // and whether a child without digits left may divide (the next pass's refine check).
      const int par = iter & 1;
      if (tid == 0) s_misc[2 + (par ^ 1)] = 0;
      const int per = (size + NT - 1) / NT;
      const int beg = min(tid * per, size), end = min(beg + per, size);
      uint64_t* pk = X.pk;
      uint64_t run = 0;
      for (int i = beg; i < end; i++) {
        uint64_t v = (uint64_t)1 << 20;  // undivided
        if (cur.cnt[i] > 1) {
          const int bl = cur.bl[i], b = bl >> 9, s4 = 1 << (2 * ((bl & 15) - 1));
          const int e0 = bins[b], e1 = bins[b + s4], e2 = bins[b + 2 * s4], e3 = bins[b + 3 * s4],
                    e4 = bins[b + 4 * s4];
          const int c0 = e1 - e0, c1 = e2 - e1, c2 = e3 - e2, c3 = e4 - e3;
          cc[4 * i] = c0;
          cc[4 * i + 1] = c1;
          cc[4 * i + 2] = c2;
          cc[4 * i + 3] = c3;
          v = (uint64_t)((c0 > 0) + (c1 > 0) + (c2 > 0) + (c3 > 0)) |
              ((uint64_t)((c0 > 1) + (c1 > 1) + (c2 > 1) + (c3 > 1)) << 40);
        }
        pk[i] = run;
        run += v;
      }
      const uint64_t incl = wave_scan_incl64(run);
      if (lane == 63) X.s_tmp64[wid] = incl;
      __syncthreads();
      uint64_t off = incl - run, tot = 0;
#pragma unroll
      for (int w = 0; w < NT / 64; w++) {
        const uint64_t x = X.s_tmp64[w];
        off += w < wid ? x : 0;
        tot += x;
      }
      T = (int)(tot & 0xFFFFF);
      newSize = T + (int)((tot >> 20) & 0xFFFFF);
      nToExpand = (int)(tot >> 40);
      bool nd = false;
      for (int i = beg; i < end; i++) {
        const uint64_t pre = off + pk[i];
        const int childPre = (int)(pre & 0xFFFFF), ndr = (int)((pre >> 20) & 0xFFFFF);
        if (cur.cnt[i] > 1) {
          const int bl = cur.bl[i];
          const int c[4] = {cc[4 * i], cc[4 * i + 1], cc[4 * i + 2], cc[4 * i + 3]};
          oct_push_children(nxt, bl, c, T - 1 - childPre, seqc + childPre);
          nd |= (bl & 15) == 1 && (c[0] > 1 || c[1] > 1 || c[2] > 1 || c[3] > 1);
        } else {
          const int pos = T + ndr;
          nxt.cnt[pos] = cur.cnt[i]; nxt.seq[pos] = cur.seq[i];
          nxt.bl[pos] = cur.bl[i];
        }
      }
      if (nd) s_misc[2 + (par ^ 1)] = 1;
      __syncthreads();
      need_known = s_misc[2 + (par ^ 1)];
      { const uint64_t t2 = OP_NOW(); OP_ADD(2, t2 - tq); tq = t2; OP_ADD(5, 1); }
    } else {
      // Final refinement (ORBextractor.cc:687-727): the expandable nodes are visited by (size,
      // seq) descending, each adding its children until the list would reach N.  Six barrier
      // steps, every thread owning a contiguous chunk of nodes (and of visiting ranks):
      //  A  quadrant counts, children per node, the rank keys, the expandable count E;
      //  B  each expandable node's visiting rank (all-pairs count of larger keys), the visiting
      //     order;
      //  C  children per visiting rank, prefix-summed in visiting order (childPre);
      //  D  the cut: the first rank whose children reach N (a minimum over the ranks);
      //  E  the undivided nodes' ranks in list order;
      //  F  the next list: children of the ranks up to the cut at the front, the rest in order.
      need_known = -1;
      const int per = (size + NT - 1) / NT;
      const int beg = min(tid * per, size), end = min(beg + per, size);
      uint64_t* pk = X.pk;
      int e_local = 0;
      for (int i = beg; i < end; i++) {
        uint64_t key = 0;
        int ne = 0;
        if (cur.cnt[i] > 1) {
          const int bl = cur.bl[i], b = bl >> 9, s4 = 1 << (2 * ((bl & 15) - 1));
          const int e0 = bins[b], e1 = bins[b + s4], e2 = bins[b + 2 * s4], e3 = bins[b + 3 * s4],
                    e4 = bins[b + 4 * s4];
          const int c0 = e1 - e0, c1 = e2 - e1, c2 = e3 - e2, c3 = e4 - e3;
          cc[4 * i] = c0;
          cc[4 * i + 1] = c1;
          cc[4 * i + 2] = c2;
          cc[4 * i + 3] = c3;
          ne = (c0 > 0) + (c1 > 0) + (c2 > 0) + (c3 > 0);
          key = ((uint64_t)cur.cnt[i] << 32) | (uint32_t)cur.seq[i];
          e_local++;
        }
        t1[i] = ne;
        pk[i] = key;
      }
      {
        const int ew = wave_scan_incl(e_local);
        if (lane == 63) s_tmp[wid] = ew;
      }
      __syncthreads();  // A
      int E = 0;
#pragma unroll
      for (int w = 0; w < NT / 64; w++) E += s_tmp[w];
      for (int i = beg; i < end; i++) {
        const uint64_t ki = pk[i];
        int rank = -1;
        if (ki != 0) {
          int r = 0, j = 0;
          for (; j + 4 <= size; j += 4) {
            const uint64_t a = pk[j], b = pk[j + 1], c = pk[j + 2], d = pk[j + 3];
            r += (a > ki) + (b > ki) + (c > ki) + (d > ki);
          }
          for (; j < size; j++) r += pk[j] > ki;
          t3[r] = i;  // visiting order
          rank = r;
        }
        t4[i] = rank;
      }
      __syncthreads();  // B
      const int vper = (E + NT - 1) / NT;
      const int vb = min(tid * vper, E), ve = min(vb + vper, E);
      int run = 0;
      for (int v = vb; v < ve; v++) {
        t2[v] = run;  // chunk-local exclusive prefix of the children in visiting order
        run += t1[t3[v]];
      }
      const int vincl = wave_scan_incl(run);
      if (lane == 63) s_tmp[wid] = vincl;
      if (tid == 0) s_misc[0] = E > 0 ? E - 1 : -1;
      __syncthreads();  // C
      int voff = vincl - run;
#pragma unroll
      for (int w = 0; w < NT / 64; w++) voff += w < wid ? s_tmp[w] : 0;
      for (int v = vb; v < ve; v++) {
        const int childPre = voff + t2[v];
        t2[v] = childPre;
        // cut = the first v with size + childPre_v + ne_v - (v + 1) >= N
        if (size + childPre + t1[t3[v]] - (v + 1) >= N) atomicMin(&s_misc[0], v);
      }
      __syncthreads();  // D
      const int cut = s_misc[0];
      if (cut >= 0) {
        T = t2[cut] + t1[t3[cut]];
        newSize = size + T - (cut + 1);
      } else {
        T = 0;
        newSize = size;
      }
      int und = 0;
      for (int i = beg; i < end; i++) und += !(t4[i] >= 0 && t4[i] <= cut);
      const int uincl = wave_scan_incl(und);
      if (lane == 63) s_tmp[wid] = uincl;
      __syncthreads();  // E
      int upos = uincl - und;
#pragma unroll
      for (int w = 0; w < NT / 64; w++) upos += w < wid ? s_tmp[w] : 0;
      for (int i = beg; i < end; i++) {
        const int r = t4[i];
        if (r >= 0 && r <= cut) {
          const int childPre = t2[r];
          const int c[4] = {cc[4 * i], cc[4 * i + 1], cc[4 * i + 2], cc[4 * i + 3]};
          oct_push_children(nxt, cur.bl[i], c, T - 1 - childPre, seqc + childPre);
        } else {
          const int pos = T + upos++;
          nxt.cnt[pos] = cur.cnt[i]; nxt.seq[pos] = cur.seq[i];
          nxt.bl[pos] = cur.bl[i];
        }
      }
      __syncthreads();  // F
      { const uint64_t t2 = OP_NOW(); OP_ADD(3, t2 - tq); tq = t2; OP_ADD(6, 1); }
    }
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
  oct_retain<NT>(X, ks, cur, size, gen_total, keys_mem);
  { const uint64_t t2 = OP_NOW(); OP_ADD(4, t2 - tq); tq = t2; OP_ADD(8, size); OP_ADD(9, ks.n); }
#ifdef ORBX_OCT_PROF
  if (tid == 0)
    for (int i = 0; i < 16; i++) atomicAdd(&g_oct_prof[(level & 7) * 16 + i], (unsigned long long)opf[i]);
#endif
}

// 256-thread instances: 6 waves per SIMD (80 VGPRs; a few spill, but C2's octree took 0.120
// vs 0.128 ms per 512 frames against 4 waves without spills); the 1024-thread instance keeps
// its registers.
constexpr int kOctWaves = 6;
// PLDS: the level's quadrant paths staged in LDS (ds_read in the refine sweeps; a pointer that
// may be either kind would compile to flat loads, which measured as slow as global ones)
template <int NT, bool PLDS, class K>
__global__ __launch_bounds__(NT)
__attribute__((amdgpu_waves_per_eu(NT <= 256 ? kOctWaves : 1)))
void k_octree(
    const LevelGeom* __restrict__ lv, const int* __restrict__ cell_counts, int ncells,
    const CellGeom* __restrict__ cells, const K* __restrict__ cand, int cand_total,
    K* __restrict__ lin, int* __restrict__ label, K* __restrict__ okey, int* __restrict__ oidx,
    int* __restrict__ ocount, int kp_total, int nlevels, int node_cap, int cell_cap,
    int bin_cap, int level_base, int* __restrict__ cell_scr, const uint32_t* __restrict__ octpath,
    int path_cap) {
  extern __shared__ __align__(16) unsigned char smem[];
  __shared__ int s_tmp[NT / 64 + 1];
  __shared__ int s_misc[8];
  // grid (image, level): every image's largest level is dispatched first and the small levels
  // last, so the launch does not end on one late large-level workgroup's serial pass chain
  const int level = level_base + blockIdx.y, img = blockIdx.x, tid = threadIdx.x;
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
  for (OctNodes* L : {&A, &B}) {
    L->cnt = (int*)take(4 * NC); L->seq = (int*)take(4 * NC); L->bl = (int*)take(4 * NC);
  }
  // the quadrant counts (counts step to the next list) and the bin -> node table (refine and
  // retain sweeps) are never live together: one array
  int* cc = (int*)take(4 * max(4 * NC, bin_cap + 8));
  int* table = cc;
  int* t1 = (int*)take(4 * NC);
  int* t2 = (int*)take(4 * NC);
  int* t3 = (int*)take(4 * NC);
  int* t4 = (int*)take(4 * NC);
  uint64_t* pk = (uint64_t*)take(8 * (NC + 1));
  // the level's quadrant paths (x then y: one contiguous run of Geometry::octpath) in LDS: the
  // refine sweeps look them up per key (loaded here beside the gather's loads)
  // (path_cap 0: the plan keeps them in global memory, where the LDS would cost occupancy)
  const uint32_t* pxy = octpath + G.path_x;
  if constexpr (PLDS) {
    uint32_t* s_path = (uint32_t*)take(4 * (size_t)path_cap);
    for (int i = tid; i < G.W + G.H; i += NT) s_path[i] = pxy[i];
    pxy = s_path;
  }
  // one region for the gather's per-cell key starts and slots and, after it, the bins and
  // their node table.  Cells: in LDS, or (cell_cap == 0: levels with too many cells for it)
  // in this (image, level)'s part of cell_scr, [2 (ncells + nlevels)] ints per image
  unsigned char* region = p;
  int* bins = (int*)take(4 * (bin_cap + 8));
  p = region;
  int* cpre = cell_cap > 0 ? (int*)take(4 * (cell_cap + 1))
                           : cell_scr + (int64_t)img * 2 * (ncells + nlevels) + 2 * (G.cell_begin + level);
  int* s_slot = cell_cap > 0 ? (int*)take(4 * cell_cap) : cpre + G.ncells + 1;
  __shared__ uint64_t s_tmp64[NT / 64 + 1];

  // 1. gather candidates of this level in cell order (vToDistributeKeys): counts and slots of
  // every cell in one round of loads, each key's cell by a binary search of the cell starts
  // (all searches of a thread in lockstep), then every key load of a chunk in flight at once
  const int* cntv = cell_counts + (int64_t)img * ncells + G.cell_begin;
  for (int i = tid; i < G.ncells; i += NT) {
    cpre[i] = cntv[i];
    s_slot[i] = cells[G.cell_begin + i].slot_off;
  }
  __syncthreads();
  const int n = block_scan_excl<NT>(cpre, G.ncells, s_tmp);
  if (tid == 0) cpre[G.ncells] = n;  // cell c holds keys cpre[c] .. cpre[c + 1] - 1
  __syncthreads();
  K* outk = okey + (int64_t)img * kp_total + G.kp_off;
  if (n == 0) {
    if (tid == 0) *oc = 0;
    return;
  }
  const K* cb = cand + (int64_t)img * cand_total;
  K* keys = lin + (int64_t)img * cand_total + G.cand_off;
  int* lab = label + (int64_t)img * cand_total + G.cand_off;
  int top = 1;  // largest power of two <= ncells
  while (2 * top <= G.ncells) top *= 2;
  // keys k0 + tid + NT j (j < kOctRegKeys), 0 past n; a key's cell is the last one starting at
  // or before it (cells without keys share their successor's start)
  auto load_keys = [&](int k0, K(&v)[kOctRegKeys]) {
    int cs[kOctRegKeys];
#pragma unroll
    for (int j = 0; j < kOctRegKeys; j++) cs[j] = 0;
    for (int st = top; st > 0; st >>= 1) {
#pragma unroll
      for (int j = 0; j < kOctRegKeys; j++) {
        const int c = cs[j] + st;
        if (c <= G.ncells && cpre[c] <= k0 + tid + NT * j) cs[j] = c;
      }
    }
#pragma unroll
    for (int j = 0; j < kOctRegKeys; j++) {
      const int k = k0 + tid + NT * j, c = cs[j];
      v[j] = k < n ? cb[s_slot[c] + k - cpre[c]] : K(0);
    }
  };
  // (the bins are first written by octree_core's refine, several barriers after the gather)
  OctCtx X{A,    B,       cc,   t1, t2, t3, t4, s_tmp, s_misc, bins, table, bin_cap,
           pk,   s_tmp64, outk, oidx + (int64_t)img * kp_total + G.kp_off,
           max(4 * NC, bin_cap + 8), oc, pxy, pxy + G.W, level == 0};
  if (n <= kOctRegKeys * NT) {  // keys + bins in registers: every sweep stays on-chip
    RegKeys<NT, K> ks;
    ks.n = n;
    load_keys(0, ks.key);
#pragma unroll
    for (int j = 0; j < kOctRegKeys; j++) {  // the final lookup of retained keys reads lin
      const int k = tid + NT * j;
      ks.lab[j] = 0;
      if (k < n) keys[k] = ks.key[j];
    }
    octree_core<NT>(G, X, ks, keys, level);
  } else {  // keys + bins in global scratch, swept in register chunks
    for (int k0 = 0; k0 < n; k0 += NT * kOctRegKeys) {
      K v[kOctRegKeys];
      load_keys(k0, v);
#pragma unroll
      for (int j = 0; j < kOctRegKeys; j++) {
        const int k = k0 + tid + NT * j;
        if (k < n) keys[k] = v[j];
      }
    }
    MemKeys<NT, K> ks;
    ks.keys = keys;
    ks.labs = lab;
    ks.n = n;
    octree_core<NT>(G, X, ks, keys, level);
  }
}

// ------------------------------------------------------------------ k_describe
// One half-wave (32 lanes) per retained keypoint, 8 keypoints per workgroup: IC_Angle on the
// unblurred level (ORBextractor.cc:73-98), cv::fastAtan2, glibc sincosf, rBRIEF on the blurred
// level with the reference binary's fmaf + cvRound sampling (ORBextractor.cc:101-144, SURVEY
// A.6) — lane j produces descriptor byte j from pairs 8j..8j+7 — then the level-0 scaling of
// operator() (:1035-1041).  Output is level-major like `_keypoints`/`descriptors`.  Two
// keypoints per wave share the per-keypoint scalar work (angle, sincos, addressing).
struct KpOffsets {  // per-level first keypoint slot (LevelGeom::kp_off), by value
  int off[kMaxLevels + 1];
};

// keypoints (half-waves) per workgroup (16 / 32 measured 8 % / 45 % slower at C2)
constexpr int kDescKP = 8;

template <class K>
__global__ __launch_bounds__(32 * kDescKP) void k_describe(
    const uint8_t* __restrict__ pyr, int64_t pyr_bytes, const uint8_t* __restrict__ blur,
    const LevelGeom* __restrict__ lv, int nlevels, KpOffsets ko, const K* __restrict__ okey,
    const int* __restrict__ oidx, const int* __restrict__ ocount, int kp_total,
    orbx_keypoint* __restrict__ kps,
    uint8_t* __restrict__ desc, int* __restrict__ counts) {
  // dwords per staged row: raw 31+3 bytes rounded up; blurred 16-B pieces from a 16-B aligned
  // start (offset <= 15 plus 37 bytes: 13 dwords) — an odd stride, so the rBRIEF samples of
  // different rows spread over the LDS banks
  constexpr int RW = 10, BW = 13, BC = 4;  // BC: 16-B pieces per blurred row
  constexpr int RN = 31 * RW, BN = 37 * BW;
  __shared__ uint32_t s_raw[kDescKP][RN];
  __shared__ uint32_t s_blr[kDescKP][BN];
  int bx, img;
  xcd_block(bx, img);
  const int lane = threadIdx.x & 63, hl = lane & 31;
  const int hw = threadIdx.x >> 5;  // half-wave of the workgroup, 0..7
  const int slot = bx * kDescKP + hw;
  const int* oc = ocount + img * nlevels;
  if (bx == 0 && threadIdx.x == 0) {
    int t = 0;
    for (int l = 0; l < nlevels; l++) t += oc[l];
    counts[img] = t;
  }
  int level = 0;
#pragma unroll
  for (int l = 1; l < kMaxLevels; l++) level += (l < nlevels && slot >= ko.off[l]);
  const LevelGeom& G = lv[level];
  const int idx = slot - ko.off[level];
  // the count, the key and the level's fields in one round of loads, pinned in registers (a
  // rematerialised load of G per patch row would serialise the patch loads behind it)
  // the level's keys come in candidate order (spatial neighbours together, k_octree's retain),
  // each with the node-order position it is written to
  int noc = oc[level];
  K key = okey[(int64_t)img * kp_total + min(slot, kp_total - 1)];
  int opos = oidx[(int64_t)img * kp_total + min(slot, kp_total - 1)];
  int pitch = G.pitch, pyr_off = (int)G.pyr_off;
  float lscale = G.scale, lsize = G.size;
  asm volatile("" : "+v"(noc), "+v"(key), "+v"(opos), "+v"(pitch), "+v"(pyr_off), "+v"(lscale),
               "+v"(lsize));
  const bool active = slot < kp_total && idx < noc;  // uniform within the half-wave
  if (!active) key = 0;
  const int cx = active ? KeyFmt<K>::x(key) + (kEdge - 3) : 0;
  const int cy = active ? KeyFmt<K>::y(key) + (kEdge - 3) : 0;
  // stage both patches with aligned dword loads issued together: the raw 31 x 31 patch
  // (IC_Angle, radius 15) and the blurred 37 x 37 patch (rBRIEF samples, radius <= 18)
  const uint8_t* L = pyr + (int64_t)img * pyr_bytes + pyr_off;
  const uint8_t* Bp = blur + (int64_t)img * pyr_bytes + pyr_off;
  const int fr = (cx - 15) >> 2, lr = (cx + 15) >> 2;  // raw dword columns
  const int ab = (cx - 18) & ~15, lb = ((cx + 18) & ~15) - ab;  // blurred first piece, last offset
  if (active) {
    uint32_t vr[(RN + 31) / 32];
    uint4 vb[(37 * BC + 31) / 32];
#pragma unroll
    for (int k = 0; k < (RN + 31) / 32; k++) {
      const int i = hl + 32 * k, r = i / RW, c = i - r * RW;
      vr[k] = (i < RN && fr + c <= lr)
                  ? *(const uint32_t*)(L + (uint32_t)((cy - 15 + r) * pitch + 4 * (fr + c)))
                  : 0u;
    }
#pragma unroll
    for (int k = 0; k < (37 * BC + 31) / 32; k++) {  // 16-B pieces: 5 loads per lane, not 13
      const int i = hl + 32 * k, r = i >> 2, c = i & 3;
      vb[k] = (i < 37 * BC && 16 * c <= lb)
                  ? *(const uint4*)(Bp + (uint32_t)((cy - 18 + r) * pitch + ab + 16 * c))
                  : make_uint4(0u, 0u, 0u, 0u);
    }
#pragma unroll
    for (int k = 0; k < (RN + 31) / 32; k++)
      if (hl + 32 * k < RN) s_raw[hw][hl + 32 * k] = vr[k];
#pragma unroll
    for (int k = 0; k < (37 * BC + 31) / 32; k++) {
      const int i = hl + 32 * k, r = i >> 2, c = i & 3;
      if (i < 37 * BC) {
        uint32_t* d = s_blr[hw] + r * BW + 4 * c;
        d[0] = vb[k].x;
        if (4 * c + 1 < BW) d[1] = vb[k].y;
        if (4 * c + 2 < BW) d[2] = vb[k].z;
        if (4 * c + 3 < BW) d[3] = vb[k].w;
      }
    }
  }
  constexpr int BS = 4 * BW;
  const uint8_t* bc = (const uint8_t*)s_blr[hw] + 18 * BS + (cx - ab);
  // IC_Angle (ORBextractor.cc:73-98): lane hl < 31 sums row v = hl - 15 of the circular patch
  // (v_dot4_u32_u8 over the row's bytes masked to |u| <= umax[|v|])
  int m10 = 0, m01 = 0;
  if (active && hl < 31)
    ic_row_moments(s_raw[hw] + hl * RW, (cx - 15) - 4 * fr, c_icmask.m[hl], hl - 15, m10, m01);
  // sums within the half-wave: 16-lane rows on DPP, then the two rows of the half
  m10 = row16_sum(m10);
  m01 = row16_sum(m01);
  m10 += __shfl_xor(m10, 16);
  m01 += __shfl_xor(m01, 16);
  if (!active) return;
  const float angle = orbx_fast_atan2((float)m01, (float)m10);
  // descriptor on the blurred level: byte hl from pairs 8 hl .. 8 hl + 7, LSB first
  const float factorPI = (float)(3.14159265358979323846 / 180.f);
  float sn, cs;
  orbx_sincosf(angle * factorPI, &sn, &cs);
  // rotated samples in packed f32 with the reference's fmaf pattern, rounded by the magic
  // addend; the (row, col) -> byte offset bias is folded into the centre address
  const uint8_t* bcb = bc - sample_bias(BS);
  const float nsn = -sn;
  uint32_t byte = 0;
#pragma unroll
  for (int m = 0; m < 8; m++) {
    // (x0, y0, x1, y1) of pair 8 hl + m: int8 loads + cvt (a float table read per lane as
    // 8 x dwordx4 made the kernel 30 % slower)
    const int8_t* p8 = c_pattern + (hl * 8 + m) * 4;
    const float4 pp = make_float4((float)p8[0], (float)p8[1], (float)p8[2], (float)p8[3]);
    const int t0 = bcb[sample_offset(rotate_fma(pp.x, pp.y, cs, sn, nsn), BS)];
    const int t1 = bcb[sample_offset(rotate_fma(pp.z, pp.w, cs, sn, nsn), BS)];
    byte |= (uint32_t)(t0 < t1) << m;
  }
  int outpos = opos;
  for (int l = 0; l < level; l++) outpos += oc[l];
  const int64_t o = (int64_t)img * kp_total + outpos;
  desc[o * 32 + hl] = (uint8_t)byte;
  if (hl == 0) {
    orbx_keypoint k;
    k.x = level ? (float)(cx) * lscale : (float)cx;
    k.y = level ? (float)(cy) * lscale : (float)cy;
    k.size = lsize;
    k.angle = angle;
    k.response = (float)KeyFmt<K>::score(key);
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
  uint32_t* d_octpath = nullptr;  // Geometry::octpath
  CellGeom* d_cells = nullptr;
  int2 *d_xtap = nullptr, *d_ytap = nullptr;
  BlurTile* d_tiles = nullptr;
  int ntiles = 0;
  PyrBand* d_bands = nullptr;
  uint8_t *d_pyr = nullptr, *d_blur = nullptr;
  // candidate keys, the octree's gathered keys and the retained keys: u32 or u64 (wide_keys)
  void *d_cand = nullptr, *d_lin = nullptr, *d_okey = nullptr;
  int *d_cell_counts = nullptr, *d_label = nullptr, *d_ocount = nullptr, *d_counts = nullptr;
  int* d_oidx = nullptr;  // per retained key (candidate order): its node-order position
  orbx_keypoint* d_kps = nullptr;
  uint8_t* d_desc = nullptr;
  // counts, keypoints and descriptors share one allocation (d_counts is its base) so the
  // drop-in path brings a frame's results back with one copy
  size_t out_kps_off = 0, out_desc_off = 0, out_bytes = 0;
  // k_octree instances (kOctNTBig, kOctNT threads): levels [lo, hi) each, with LDS for nc
  // nodes, cc cells (0: the cell tables in d_cell_scr) and `bins` bins
  struct OctInst {
    int paths = 0;  // quadrant-path entries of the instance's largest level (W + H)
    int lo = 0, hi = 0, nc = 1, cc = 1, bins = 1;
    size_t smem = 0;
  } oct[2];
  int* d_cell_scr = nullptr;
  int cell_cap = 0;
  // k_fast_pairs: adjacent cell pairs; k_fast_cells: the other cells, in its <44,
  // kFcSmallRows> and <72, kCellMax> instances
  int2* d_pairs = nullptr;
  int n_pairs = 0;
  int *d_cells_small = nullptr, *d_cells_tall = nullptr, *d_cells_big = nullptr;
  int n_cells_small = 0, n_cells_tall = 0, n_cells_big = 0;
  const uint8_t* last_in = nullptr;
  int last_n = 0;
  // graph cache keyed by (input pointer, batch)
  GraphCache graphs;
  Profiler prof;
};

namespace {

template <class T>
int dalloc(T** p, size_t count) {
  if (count == 0) count = 1;
  if (hipMalloc((void**)p, count * sizeof(T)) != hipSuccess) return ORBX_ENOMEM;
  return ORBX_OK;
}

__global__ void k_fill_u32(uint32_t* __restrict__ p, size_t n, uint32_t v) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    p[i] = v;
}

}  // namespace

int orbx::launch_fill_u32(uint32_t* p, size_t n, uint32_t v, hipStream_t s) {
  if (n == 0) return ORBX_OK;
  const unsigned blocks = (unsigned)std::min<size_t>((n + 255) / 256, 2048);
  hipLaunchKernelGGL(k_fill_u32, dim3(blocks), dim3(256), 0, s, p, n, v);
  return ORBX_OK;
}

// Blur tiles over every level (the blurred pyramid has the pyramid's pitched layout).
static std::vector<BlurTile> blur_tiles(const Geometry& g) {
  std::vector<BlurTile> tiles;
  for (int l = 0; l < g.nlevels; l++) {
    const LevelGeom& G = g.lv[l];
    for (int ty = 0; ty * kBlurTH < G.h; ty++)
      for (int tx = 0; tx * kBlurTW < G.w; tx++) {
        const int X0 = tx * kBlurTW, Y0 = ty * kBlurTH;
        // (X0 >= 64 then, and the 64-B pitch covers k_blur's 16-B pieces up to X0 + 79)
        const bool interior = X0 >= 4 && X0 + kBlurTW + 4 <= G.w && Y0 >= 3 &&
                              Y0 + kBlurTH + 3 <= G.h;
        tiles.push_back({(int16_t)l, (int16_t)tx, (int16_t)ty, (int16_t)interior});
      }
  }
  return tiles;
}

// k_pyramid's dynamic LDS bound (bands of up to kPyMaxSmemLimit bytes); under the resource lock
int orbx::pyr_kernel_init() {
  static bool done = false;
  if (!done) {
    if (hipFuncSetAttribute((const void*)k_pyramid<true>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, kPyMaxSmemLimit) != hipSuccess ||
        hipFuncSetAttribute((const void*)k_pyramid<false>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, kPyMaxSmemLimit) != hipSuccess)
      return ORBX_EDEVICE;
    done = true;
  }
  return ORBX_OK;
}

int orbx::pyr_dev_create(const Geometry& g, PyrDev* d) {
  *d = PyrDev{};
  if (pyr_kernel_init() != ORBX_OK) return ORBX_EDEVICE;
  const std::vector<BlurTile> tiles = blur_tiles(g);
  d->ntiles = (int)tiles.size();
  BlurTile* dt = nullptr;
  if (dalloc(&d->d_lv, g.nlevels) || dalloc(&d->d_xtap, g.xtap.size() / 2 + 1) ||
      dalloc(&d->d_ytap, g.ytap.size() / 2 + 1) || dalloc(&d->d_bands, g.bands.size()) ||
      dalloc(&dt, tiles.size())) {
    d->d_tiles = dt;
    pyr_dev_destroy(d);
    return ORBX_ENOMEM;
  }
  d->d_tiles = dt;
  auto up = [&](void* p, const void* h, size_t bytes) {
    return bytes ? hipMemcpy(p, h, bytes, hipMemcpyHostToDevice) : hipSuccess;
  };
  if (up(d->d_lv, g.lv, sizeof(LevelGeom) * g.nlevels) ||
      up(d->d_xtap, g.xtap.data(), 4 * g.xtap.size()) ||
      up(d->d_ytap, g.ytap.data(), 4 * g.ytap.size()) ||
      up(d->d_bands, g.bands.data(), sizeof(PyrBand) * g.bands.size()) ||
      up(dt, tiles.data(), sizeof(BlurTile) * tiles.size())) {
    pyr_dev_destroy(d);
    return ORBX_EDEVICE;
  }
  return ORBX_OK;
}

void orbx::pyr_dev_destroy(PyrDev* d) {
  if (d->d_lv) (void)hipFree(d->d_lv);
  if (d->d_xtap) (void)hipFree(d->d_xtap);
  if (d->d_ytap) (void)hipFree(d->d_ytap);
  if (d->d_bands) (void)hipFree(d->d_bands);
  if (d->d_tiles) (void)hipFree(d->d_tiles);
  *d = PyrDev{};
}

// k_pyramid's stages, and with the blur fused (Geometry::blur_fused) the blurred pyramid too
// (a profiler marks every launch: the stage's launch count is its dispatches)
static void enqueue_pyramid(const Geometry& g, const LevelGeom* d_lv, const PyrBand* d_bands,
                            const int2* d_xtap, const int2* d_ytap, const uint8_t* d_in,
                            uint8_t* d_pyr, uint8_t* d_blur, int n, hipStream_t s,
                            Profiler* pr = nullptr, int stage = -1) {
  note_kernel(g.blur_fused ? "k_pyramid<true>" : "k_pyramid<false>");
  for (const PyrStage& st : g.pyr_stages) {
    if (g.blur_fused)
      hipLaunchKernelGGL(k_pyramid<true>, dim3(st.nbands, n), dim3(kPyNT), st.smem, s, d_in,
                         d_pyr, g.pyr_bytes, d_lv, st.l0, st.l1, d_bands + st.band0, d_xtap,
                         d_ytap, st.buf_b, d_blur);
    else
      hipLaunchKernelGGL(k_pyramid<false>, dim3(st.nbands, n), dim3(kPyNT), st.smem, s, d_in,
                         d_pyr, g.pyr_bytes, d_lv, st.l0, st.l1, d_bands + st.band0, d_xtap,
                         d_ytap, st.buf_b, nullptr);
    if (pr) pr->mark(s, stage);
  }
}

int orbx::launch_pyramid(const Geometry& g, const PyrDev& d, const uint8_t* d_in, uint8_t* d_pyr,
                         uint8_t* d_blur, int n, hipStream_t s, Profiler* pr, int stage) {
  enqueue_pyramid(g, d.d_lv, d.d_bands, d.d_xtap, d.d_ytap, d_in, d_pyr, d_blur, n, s, pr, stage);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? ORBX_OK : report_hip(e, "launch_pyramid");
}

int orbx::launch_blur(const Geometry& g, const PyrDev& d, const uint8_t* d_pyr, uint8_t* d_blur,
                      int n, hipStream_t s) {
  if (!g.blur_fused && d.ntiles > 0) note_kernel("k_blur");
  if (!g.blur_fused && d.ntiles > 0)
    hipLaunchKernelGGL(k_blur, dim3(d.ntiles, n), dim3(256), 0, s, d_pyr, g.pyr_bytes, d_blur,
                       d.d_lv, (const BlurTile*)d.d_tiles);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? ORBX_OK : report_hip(e, "launch_blur");
}

namespace {

// k_fast_cells, k_octree and k_describe on K-wide candidate keys (KeyFmt)
template <class K>
void enqueue_keyed(orbx_plan* P, int n, Profiler& pr, int st_fcell, int st_oct, int st_desc) {
  const Geometry& g = P->g;
  const int L = g.nlevels;
  const int ncells = (int)g.cells.size();
  K *cand = (K*)P->d_cand, *lin = (K*)P->d_lin, *okey = (K*)P->d_okey;
  if (ncells > 0) {
    // pairs (cells) per wave: up to kPairsPerWave (kCellsPerWave) while the launch keeps
    // >= 16 k waves in flight
    if (P->n_pairs > 0) {
      const int ppw = std::max(1, std::min(kPairsPerWave, P->n_pairs * n / 16384));
      note_kernel<K>("k_fast_pairs");
      hipLaunchKernelGGL((k_fast_pairs<K>), dim3((P->n_pairs + 4 * ppw - 1) / (4 * ppw), n),
                         dim3(256), 0, P->stream, P->d_pyr, g.pyr_bytes, P->d_cells, P->d_pairs,
                         P->n_pairs, ncells, g.ini_th, g.min_th, cand, g.cand_total,
                         P->d_cell_counts, ppw);
    }
    const int cpw = std::max(1, std::min(kCellsPerWave, P->n_cells_small * n / 16384));
    if (P->n_cells_small > 0) note_kernel<K>("k_fast_cells", "44, 42, ");
    static_assert(kFcSmallRows == 42 && kFcTallRS == 48 && kCellMax == 66, "instance names");
    if (P->n_cells_small > 0)
      hipLaunchKernelGGL((k_fast_cells<44, kFcSmallRows, K>),
                         dim3((P->n_cells_small + 4 * cpw - 1) / (4 * cpw), n), dim3(256), 0,
                         P->stream, P->d_pyr, g.pyr_bytes, P->d_cells, P->d_cells_small,
                         P->n_cells_small, ncells, g.ini_th, g.min_th, cand, g.cand_total,
                         P->d_cell_counts, cpw);
    // cells up to 45 px wide and kCellMax rows (levels with 2-3 cell rows, e.g. C4's levels 5
    // and 7, C2's level 7): several per wave on the narrow staging, not one per wave on <72,
    // kCellMax>'s
    const int cpt = std::max(1, std::min(kCellsPerWave, P->n_cells_tall * n / 16384));
    if (P->n_cells_tall > 0) note_kernel<K>("k_fast_cells", "48, 66, ");
    if (P->n_cells_tall > 0)
      hipLaunchKernelGGL((k_fast_cells<kFcTallRS, kCellMax, K>),
                         dim3((P->n_cells_tall + 4 * cpt - 1) / (4 * cpt), n), dim3(256), 0,
                         P->stream, P->d_pyr, g.pyr_bytes, P->d_cells, P->d_cells_tall,
                         P->n_cells_tall, ncells, g.ini_th, g.min_th, cand, g.cand_total,
                         P->d_cell_counts, cpt);
    if (P->n_cells_big > 0) note_kernel<K>("k_fast_cells", "72, 66, ");
    if (P->n_cells_big > 0)
      hipLaunchKernelGGL((k_fast_cells<72, kCellMax, K>), dim3((P->n_cells_big + 3) / 4, n), dim3(256),
                         0, P->stream, P->d_pyr, g.pyr_bytes, P->d_cells, P->d_cells_big,
                         P->n_cells_big, ncells, g.ini_th, g.min_th, cand, g.cand_total,
                         P->d_cell_counts, 1);
    pr.mark(P->stream, st_fcell);
  }
  // levels by octree frame area: 1024-thread and 256-thread workgroups
  static_assert(kOctNTBig == 1024 && kOctNT == 256, "instance names");
  auto launch_oct = [&](auto kern, int nt, const orbx_plan::OctInst& o, const char* name) {
    if (o.hi <= o.lo) return;
    note_kernel<K>("k_octree", name);
    hipLaunchKernelGGL(kern, dim3(n, o.hi - o.lo), dim3(nt), o.smem, P->stream, P->d_lv,
                       P->d_cell_counts, ncells, P->d_cells, cand, g.cand_total, lin, P->d_label,
                       okey, P->d_oidx, P->d_ocount, g.kp_total, L, o.nc, o.cc, o.bins, o.lo, P->d_cell_scr,
                       P->d_octpath, o.paths);
  };
  if (P->oct[0].paths > 0)
    launch_oct(k_octree<kOctNTBig, true, K>, kOctNTBig, P->oct[0], "1024, true, ");
  else
    launch_oct(k_octree<kOctNTBig, false, K>, kOctNTBig, P->oct[0], "1024, false, ");
  if (P->oct[1].paths > 0)
    launch_oct(k_octree<kOctNT, true, K>, kOctNT, P->oct[1], "256, true, ");
  else
    launch_oct(k_octree<kOctNT, false, K>, kOctNT, P->oct[1], "256, false, ");
  pr.mark(P->stream, st_oct);
  KpOffsets ko{};
  for (int l = 0; l < L; l++) ko.off[l] = g.lv[l].kp_off;
  note_kernel<K>("k_describe");
  hipLaunchKernelGGL(k_describe<K>, dim3((g.kp_total + kDescKP - 1) / kDescKP, n), dim3(32 * kDescKP), 0, P->stream,
                     P->d_pyr, g.pyr_bytes, P->d_blur, P->d_lv, L, ko, okey, P->d_oidx,
                     P->d_ocount, g.kp_total, P->d_kps, P->d_desc, P->d_counts);
  pr.mark(P->stream, st_desc);
}

int enqueue(orbx_plan* P, const uint8_t* d_in, int n, Profiler* prof) {
  const Geometry& g = P->g;
  Profiler dummy;
  Profiler& pr = prof ? *prof : dummy;
  const int st_pyr = pr.stage("k_pyramid"), st_blur = pr.stage("k_blur"),
            st_oct = pr.stage("k_octree"), st_desc = pr.stage("k_describe"),
            st_fcell = pr.stage("k_fast_cells");
  ProfScope scope(pr);
  pr.mark(P->stream, -1);
  enqueue_pyramid(g, P->d_lv, P->d_bands, P->d_xtap, P->d_ytap, d_in, P->d_pyr, P->d_blur, n,
                  P->stream, &pr, st_pyr);
  if (!g.blur_fused && P->ntiles > 0) {
    note_kernel("k_blur");
    hipLaunchKernelGGL(k_blur, dim3(P->ntiles, n), dim3(256), 0, P->stream, P->d_pyr,
                       g.pyr_bytes, P->d_blur, P->d_lv, P->d_tiles);
    pr.mark(P->stream, st_blur);
  }
  if (g.wide_keys)
    enqueue_keyed<uint64_t>(P, n, pr, st_fcell, st_oct, st_desc);
  else
    enqueue_keyed<uint32_t>(P, n, pr, st_fcell, st_oct, st_desc);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return report_hip(e, "extract launch");
  return ORBX_OK;
}

}  // namespace

extern "C" {

int orbx_plan_create(const orbx_params* params, int32_t w, int32_t h, int32_t max_batch,
                     int hip_device, orbx_plan** out) {
  ORBX_RESOURCE_LOCK;
  if (!params || !out || w <= 0 || h <= 0 || max_batch <= 0) return ORBX_EINVAL;
  *out = nullptr;
  orbx_plan* P = new (std::nothrow) orbx_plan();
  if (!P) return ORBX_ENOMEM;
  std::string why;
  P->g.py_band_h = max_batch <= kPyFewImages ? kPyBandHSmall : kPyBandH;
  // batch plans: a k_pyramid launch of at least kPyMinGrid workgroups (4 rounds of the chip's
  // ~768 resident tiles), however few tiles a stage's small levels need; few-image plans: at
  // least kPyFewTiles per image, so one frame's stage spreads over half the CUs (the drop-in's
  // launches 11.3 -> 9.9 us)
  P->g.py_min_tiles = max_batch <= kPyFewImages ? kPyFewTiles
                                                : std::max(1, (kPyMinGrid + max_batch - 1) / max_batch);
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
  if (pyr_kernel_init() != ORBX_OK) return fail(ORBX_EDEVICE);
  ORBX_HIP(hipMemcpyToSymbol(HIP_SYMBOL(c_pattern), ORBX_PATTERN, sizeof(ORBX_PATTERN)));
  ORBX_HIP(hipMemcpyToSymbol(HIP_SYMBOL(c_umax), g.umax, sizeof(g.umax)));
  {
    IcMask icm;
    build_ic_mask(g.umax, &icm);
    ORBX_HIP(hipMemcpyToSymbol(HIP_SYMBOL(c_icmask), &icm, sizeof(icm)));
  }
  const std::vector<BlurTile> tiles = blur_tiles(g);
  for (const CellGeom& c : g.cells)
    if (c.x1 - c.x0 > kCellMax || c.y1 - c.y0 > kCellMax) return fail(ORBX_EUNSUPPORTED);
  P->ntiles = (int)tiles.size();
  for (int l = 0; l < g.nlevels; l++) P->cell_cap = std::max(P->cell_cap, g.lv[l].ncells);
  std::vector<int> cells_small, cells_tall, cells_big;
  std::vector<int2> pairs, singles;
  std::vector<CellGeom> empties;  // k_fast_pairs' empty partners, past the level cells
  // a few-image plan runs every cell in the <72, kCellMax> instance: one launch instead of two
  // on the drop-in path's one-frame chain (either instance handles any cell)
  const bool one_fast_launch = max_batch <= kPyFewImages;
  // k_fast_pairs takes two consecutive cells of one cell row whose detection columns are
  // contiguous and fill at most 64 lanes, ROI at most kPairRows rows; the <44, kFcSmallRows>
  // instance takes ROIs up to 41 + its alignment slack wide and kFcSmallRows rows high
  auto det = [](const CellGeom& C, int* dc, int* dr) {
    *dc = C.x1 - C.x0 - 6;
    *dr = C.y1 - C.y0 - 6;
    return *dc > 0 && *dr > 0;
  };
  for (int c = 0; c < (int)g.cells.size(); c++) {
    const CellGeom& C = g.cells[c];
    if (!one_fast_launch && c + 1 < (int)g.cells.size()) {
      const CellGeom& D = g.cells[c + 1];
      int dca, dra, dcb, drb;
      if (det(C, &dca, &dra) && det(D, &dcb, &drb) && D.level == C.level && D.y0 == C.y0 &&
          D.y1 == C.y1 && D.x0 + 3 == C.x1 - 3 && dca + dcb <= 64 && C.y1 - C.y0 <= kPairRows &&
          D.x1 - C.x0 + 3 <= kPairRS) {
        pairs.push_back(make_int2(c, c + 1));
        c++;
        continue;
      }
    }
    // a single cell whose ROI fits the pair staging runs in k_fast_pairs with an empty partner
    // (half-wave form when it is at most 32 wide): one launch instead of a k_fast_cells one
    int dcs, drs;
    if (SINGLES_IN_PAIRS && !one_fast_launch && det(C, &dcs, &drs) && C.y1 - C.y0 <= kPairRows &&
        C.x1 - C.x0 + 3 <= kPairRS) {
      CellGeom e = C;  // the empty partner: no detection columns, ending where C ends
      e.x0 = (int16_t)(C.x1 - 6);
      singles.push_back(make_int2(c, (int)g.cells.size() + (int)empties.size()));
      empties.push_back(e);
      continue;
    }
    const bool small = C.x1 - C.x0 + 3 <= 44 && C.y1 - C.y0 <= kFcSmallRows;
    const bool tall = C.x1 - C.x0 + 3 <= kFcTallRS && C.y1 - C.y0 <= kCellMax;
    (one_fast_launch ? cells_big : small ? cells_small : tall ? cells_tall : cells_big).push_back(c);
  }
  pairs.insert(pairs.end(), singles.begin(), singles.end());  // singles after the pairs
  P->n_pairs = (int)pairs.size();
  P->n_cells_small = (int)cells_small.size();
  P->n_cells_tall = (int)cells_tall.size();
  P->n_cells_big = (int)cells_big.size();
  const size_t B = (size_t)max_batch;
  const size_t ksz = g.wide_keys ? 8 : 4;  // bytes per candidate key
  std::vector<CellGeom> cells_dev(g.cells);  // + the empty partners of single cells
  cells_dev.insert(cells_dev.end(), empties.begin(), empties.end());
  if (dalloc(&P->d_lv, g.nlevels) || dalloc(&P->d_cells, cells_dev.size()) ||
      dalloc(&P->d_xtap, g.xtap.size() / 2) || dalloc(&P->d_ytap, g.ytap.size() / 2) ||
      dalloc(&P->d_tiles, tiles.size()) || dalloc(&P->d_bands, g.bands.size()) ||
      dalloc(&P->d_pyr, B * g.pyr_bytes) || dalloc(&P->d_blur, B * g.pyr_bytes) ||
      dalloc((char**)&P->d_cand, B * g.cand_total * ksz) ||
      dalloc((char**)&P->d_lin, B * g.cand_total * ksz) ||
      dalloc(&P->d_label, B * g.cand_total) || dalloc(&P->d_cell_counts, B * g.cells.size()) ||
      dalloc((char**)&P->d_okey, B * g.kp_total * ksz) || dalloc(&P->d_oidx, B * g.kp_total) ||
      dalloc(&P->d_ocount, B * g.nlevels) ||
      dalloc(&P->d_cells_small, cells_small.size()) || dalloc(&P->d_cells_tall, cells_tall.size()) ||
      dalloc(&P->d_cells_big, cells_big.size()) ||
      dalloc(&P->d_pairs, pairs.size()) || dalloc(&P->d_octpath, g.octpath.size()))
    return fail(ORBX_ENOMEM);
  {
    auto r256 = [](size_t b) { return (b + 255) & ~size_t(255); };
    P->out_kps_off = r256(4 * B);
    P->out_desc_off = P->out_kps_off + r256(B * g.kp_total * sizeof(orbx_keypoint));
    P->out_bytes = P->out_desc_off + B * g.kp_total * 32;
    char* blk = nullptr;
    if (dalloc(&blk, P->out_bytes)) return fail(ORBX_ENOMEM);
    P->d_counts = (int*)blk;
    P->d_kps = (orbx_keypoint*)(blk + P->out_kps_off);
    P->d_desc = (uint8_t*)(blk + P->out_desc_off);
  }
  auto up = [&](void* d, const void* h, size_t bytes) {
    return bytes ? hipMemcpy(d, h, bytes, hipMemcpyHostToDevice) : hipSuccess;
  };
  if (up(P->d_lv, g.lv, sizeof(LevelGeom) * g.nlevels) ||
      up(P->d_octpath, g.octpath.data(), 4 * g.octpath.size()) ||
      up(P->d_cells, cells_dev.data(), sizeof(CellGeom) * cells_dev.size()) ||
      up(P->d_xtap, g.xtap.data(), 4 * g.xtap.size()) ||
      up(P->d_ytap, g.ytap.data(), 4 * g.ytap.size()) ||
      up(P->d_tiles, tiles.data(), sizeof(BlurTile) * tiles.size()) ||
      up(P->d_bands, g.bands.data(), sizeof(PyrBand) * g.bands.size()) ||
      up(P->d_cells_small, cells_small.data(), 4 * cells_small.size()) ||
      up(P->d_cells_tall, cells_tall.data(), 4 * cells_tall.size()) ||
      up(P->d_cells_big, cells_big.data(), 4 * cells_big.size()) ||
      up(P->d_pairs, pairs.data(), sizeof(int2) * pairs.size()))
    return fail(ORBX_EDEVICE);
  if (hipMemset(P->d_counts, 0, 4 * B) != hipSuccess) return fail(ORBX_EDEVICE);
  auto r16 = [](size_t b) { return (b + 15) & ~size_t(15); };
  // node arrays (two lists of cnt seq bl), quadrant counts, four scratch arrays and
  // the rank keys, then one region for the gather's cell tables or the bins + node table
  auto oct_bytes = [&](size_t NC, size_t CC, size_t BC, size_t PC) {
    return 2 * 3 * r16(4 * NC) + r16(4 * std::max(4 * NC, BC + 8)) + 4 * r16(4 * NC) +
           r16(8 * (NC + 1)) + r16(4 * PC) +
           std::max(CC ? r16(4 * (CC + 1)) + r16(4 * CC) : 0, r16(4 * (BC + 8)));
  };
  // levels are in decreasing area: each instance takes a contiguous range
  int inst_of[kMaxLevels];
  for (int l = 0; l < g.nlevels; l++)
    inst_of[l] = (int64_t)g.lv[l].W * g.lv[l].H > kOctBigArea ? 0 : 1;
  for (int i = 0, l = 0; i < 2; i++) {
    orbx_plan::OctInst& o = P->oct[i];
    o.lo = l;
    while (l < g.nlevels && inst_of[l] == i) {
      o.nc = std::max(o.nc, g.lv[l].node_cap);
      o.cc = std::max(o.cc, g.lv[l].ncells);
      o.paths = std::max(o.paths, g.lv[l].W + g.lv[l].H);
      if (g.lv[l].path_y != g.lv[l].path_x + g.lv[l].W) return fail(ORBX_EUNSUPPORTED);
      l++;
    }
    o.hi = l;
    // bins: every refine gives each node with > 1 key at least one digit (4 bins) and needs
    // the initial nodes' bins first, so at least 4 x the node capacity; more bins, fewer refine
    // sweeps (few-image plans and the 1024-thread instance are not bound by LDS occupancy)
    o.bins = std::max(4 * o.nc + 4, (i == 0 || max_batch <= kPyFewImages) ? kOctBinsFew : kOctBins);
    // a level with more cells than fit beside its nodes keeps its cell table in global scratch
    if (oct_bytes(o.nc, o.cc, o.bins, 0) > kOctMaxSmem) o.cc = 0;
    // the quadrant paths in LDS only where that keeps the workgroups per CU and the LDS bound
    // (C2: octree 0.115 -> 0.101 ms per 512 frames; C5's 256-thread levels lost a workgroup per
    // CU to them and took longer)
    const int nt = i == 0 ? kOctNTBig : kOctNT;
    const int wave_cap = i == 0 ? 1 : 4 * kOctWaves / (nt / 64);  // workgroups per CU by waves
    auto per_cu = [&](size_t b) { return std::min<int>(wave_cap, (int)((160 * 1024) / std::max<size_t>(b, 1))); };
#ifdef ORBX_EXP_OCT_DEBUG
    fprintf(stderr, "[oct] inst %d levels %d..%d nc %d cc %d bins %d paths %d bytes %zu / %zu per_cu %d / %d\n",
            i, o.lo, o.hi, o.nc, o.cc, o.bins, o.paths, oct_bytes(o.nc, o.cc, o.bins, 0),
            oct_bytes(o.nc, o.cc, o.bins, o.paths), per_cu(oct_bytes(o.nc, o.cc, o.bins, 0)),
            per_cu(oct_bytes(o.nc, o.cc, o.bins, o.paths)));
#endif
#ifndef ORBX_EXP_OCT_PATHS_ALWAYS
    if (oct_bytes(o.nc, o.cc, o.bins, o.paths) > kOctMaxSmem ||
        per_cu(oct_bytes(o.nc, o.cc, o.bins, o.paths)) < per_cu(oct_bytes(o.nc, o.cc, o.bins, 0)))
      o.paths = 0;
#endif
    o.smem = o.hi > o.lo ? oct_bytes(o.nc, o.cc, o.bins, o.paths) : 0;
    if (o.smem > kOctMaxSmem) return fail(ORBX_EUNSUPPORTED);
  }
  bool cell_scr = false;
  for (const orbx_plan::OctInst& o : P->oct) cell_scr |= o.hi > o.lo && o.cc == 0;
  if (cell_scr && dalloc(&P->d_cell_scr, B * 2 * (g.cells.size() + g.nlevels)))
    return fail(ORBX_ENOMEM);
  // keys and their bins live in registers (up to kOctRegKeys * threads per level) or in global
  // scratch.  The dynamic-LDS attribute is per function and shared by every plan of the
  // process: only ever raised.
  static size_t attr[2] = {0, 0};  // guarded by the resource lock
  const void* fns[2][4] = {
      {(const void*)k_octree<kOctNTBig, false, uint32_t>, (const void*)k_octree<kOctNTBig, false, uint64_t>,
       (const void*)k_octree<kOctNTBig, true, uint32_t>, (const void*)k_octree<kOctNTBig, true, uint64_t>},
      {(const void*)k_octree<kOctNT, false, uint32_t>, (const void*)k_octree<kOctNT, false, uint64_t>,
       (const void*)k_octree<kOctNT, true, uint32_t>, (const void*)k_octree<kOctNT, true, uint64_t>}};
  for (int i = 0; i < 2; i++) {
    if (P->oct[i].smem <= attr[i]) continue;
    for (const void* f : fns[i])
      if (hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)P->oct[i].smem) != hipSuccess)
        return fail(ORBX_EDEVICE);
    attr[i] = P->oct[i].smem;
  }
  *out = P;
  return ORBX_OK;
}

int orbx_plan_destroy(orbx_plan* P) {
  ORBX_RESOURCE_LOCK;
  if (!P) return ORBX_OK;
  P->graphs.clear(P->stream);
  void* ptrs[] = {P->d_lv,   P->d_cells, P->d_xtap, P->d_ytap,        P->d_tiles, P->d_bands,
                  P->d_pyr,  P->d_blur,  P->d_cand, P->d_lin,         P->d_okey,  P->d_cell_counts,
                  P->d_label, P->d_oidx,
                  P->d_ocount, P->d_cells_small, P->d_cells_tall, P->d_cells_big, P->d_pairs,
                  P->d_cell_scr, P->d_octpath,
                  P->d_counts /* base of kps and desc too */};
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
  return run_graph(P->graphs, P->stream, d_imgs, n,
                   [&] { return enqueue(P, d_imgs, n, nullptr); });
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

int orbx_plan_profile_kernels(orbx_plan* P, int32_t stage, char* buf, int32_t cap) {
  if (!P) return ORBX_EINVAL;
  const int r = P->prof.kernels_of(stage, buf, cap);
  return r == 0 ? ORBX_OK : r > 0 ? ORBX_ECAPACITY : ORBX_EINVAL;
}

// Internal accessors used by the single-image extractor (orbx_api.hip).
int orbx_plan_level_dims(const orbx_plan* P, int level, int* w, int* h) {
  if (!P || level < 0 || level >= P->g.nlevels) return ORBX_EINVAL;
  *w = P->g.lv[level].w;
  *h = P->g.lv[level].h;
  return ORBX_OK;
}

int orbx_plan_level_download_buf(orbx_plan* P, int img, int level, uint8_t* out, int64_t stride,
                                 int blurred) {
  if (!P || !P->last_in || img < 0 || img >= P->last_n || level < 0 || level >= P->g.nlevels)
    return ORBX_EINVAL;
  const LevelGeom& G = P->g.lv[level];
  const uint8_t* src = (blurred ? P->d_blur : P->d_pyr) + (int64_t)img * P->g.pyr_bytes + G.pyr_off;
  ORBX_HIP(hipMemcpy2DAsync(out, stride, src, G.pitch, G.w, G.h, hipMemcpyDeviceToHost,
                            P->stream));
  ORBX_HIP(hipStreamSynchronize(P->stream));
  return ORBX_OK;
}

int orbx_plan_level_download(orbx_plan* P, int img, int level, uint8_t* out, int64_t stride) {
  return orbx_plan_level_download_buf(P, img, level, out, stride, 0);
}

#ifdef ORBX_OCT_PROF
int orbx_debug_oct_prof(uint64_t* out, int32_t reset) {
  if (out && (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_oct_prof), sizeof(g_oct_prof)) != hipSuccess ||
              hipMemcpyFromSymbol(out + 8 * 16, HIP_SYMBOL(g_oct_sub), sizeof(g_oct_sub)) != hipSuccess))
    return ORBX_EDEVICE;
  if (reset) {
    static const unsigned long long z[8 * 16] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_oct_prof), z, sizeof(z)) != hipSuccess ||
        hipMemcpyToSymbol(HIP_SYMBOL(g_oct_sub), z, 8 * 8) != hipSuccess)
      return ORBX_EDEVICE;
  }
  return ORBX_OK;
}
#endif

#ifdef ORBX_FAST_PROF
int orbx_debug_fast_prof(uint64_t* out, int32_t reset) {
  if (out && hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fast_prof), sizeof(g_fast_prof)) != hipSuccess)
    return ORBX_EDEVICE;
  if (reset) {
    static const unsigned long long z[16] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_fast_prof), z, sizeof(z)) != hipSuccess) return ORBX_EDEVICE;
  }
  return ORBX_OK;
}
#endif

int orbx_debug_plan_level(orbx_plan* P, int32_t img, int32_t level, int32_t blurred, uint8_t* out,
                          int64_t stride) {
  if (!out) return ORBX_EINVAL;
  return orbx_plan_level_download_buf(P, img, level, out, stride, blurred != 0);
}

// Test hook: the device sincosf port over a range of float bit patterns (orbx.h).
__global__ void k_debug_sincosf(uint32_t lo, int64_t n, float* __restrict__ s, float* __restrict__ c) {
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    float sv, cv;
    orbx_sincosf(__uint_as_float(lo + (uint32_t)i), &sv, &cv);
    s[i] = sv;
    c[i] = cv;
  }
}

int orbx_debug_sincosf(uint32_t lo, int64_t n, float* s, float* c) {
  if (n < 0 || (n > 0 && (!s || !c)) || (uint64_t)lo + (uint64_t)n > 0x100000000ull)
    return ORBX_EINVAL;
  if (n == 0) return ORBX_OK;
  float* d = nullptr;
  {
    ORBX_RESOURCE_LOCK;
    ORBX_HIP(hipMalloc(&d, 8 * (size_t)n));
  }
  hipLaunchKernelGGL(k_debug_sincosf, dim3(4096), dim3(256), 0, 0, lo, n, d, d + n);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipMemcpy(s, d, 4 * (size_t)n, hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(c, d + n, 4 * (size_t)n, hipMemcpyDeviceToHost);
  {
    ORBX_RESOURCE_LOCK;
    (void)hipFree(d);
  }
  return e == hipSuccess ? ORBX_OK : report_hip(e, "orbx_debug_sincosf");
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
  v->d_pyr = P->d_pyr;
  v->pyr_bytes = P->g.pyr_bytes;
  v->d_lv = P->d_lv;
  return ORBX_OK;
}
int plan_output_block(const orbx_plan* P, size_t* kps_off, size_t* desc_off, size_t* bytes) {
  if (!P) return ORBX_EINVAL;
  *kps_off = P->out_kps_off;
  *desc_off = P->out_desc_off;
  *bytes = P->out_bytes;
  return ORBX_OK;
}
int plan_enqueue(orbx_plan* P, const uint8_t* d_in, int n, Profiler* prof) {
  if (!P || !d_in || n <= 0 || n > P->max_batch) return ORBX_EINVAL;
  P->last_in = d_in;
  P->last_n = n;
  return enqueue(P, d_in, n, prof);
}
}  // namespace orbx
