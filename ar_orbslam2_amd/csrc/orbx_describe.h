// orbx_describe.h — device helpers shared by the two descriptor kernels (k_describe for
// ORBextractor, k_cvdescribe for cv::ORB): the intensity-centroid moments of IC_Angle by rows
// with v_dot4_u32_u8, and the rotated-pattern sample offsets in packed f32 with the rounding
// done by the 1.5 * 2^23 magic addend.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#pragma clang fp contract(off)

namespace orbx {

typedef float orbx_f2 __attribute__((ext_vector_type(2)));

// (x, y) by element: a braced compound literal `(orbx_f2){x, y}` splats x in HIP C++.
__device__ __forceinline__ orbx_f2 f2(float x, float y) {
  orbx_f2 v;
  v.x = x;
  v.y = y;
  return v;
}

// IC_Angle's circular patch by rows: row r = v + 15 (v = -15..15) holds the bytes j = u + 15
// with |u| <= umax[|v|] (ORBextractor.cc:73-98, orb.cpp IC_Angle).  mask[r][k] selects bytes
// 4k .. 4k+3 of the row's 32-byte window.
struct IcMask {
  uint32_t m[31][8];
};

inline void build_ic_mask(const int* umax, IcMask* out) {
  for (int r = 0; r < 31; r++) {
    const int v = r - 15, d = umax[v < 0 ? -v : v];
    for (int k = 0; k < 8; k++) {
      uint32_t m = 0;
      for (int b = 0; b < 4; b++) {
        const int u = 4 * k + b - 15;
        if (u >= -d && u <= d) m |= 0xFFu << (8 * b);
      }
      out->m[r][k] = m;
    }
  }
}

// One row of the moments: `row` = the staged row's dwords, the pixel u = -15 at byte `sb`
// (0..3) of row[0]; adds sum_u u * I(u, v) to m10 and v * sum_u I(u, v) to m01.  Exact
// integers: the same sums in another order.
__device__ __forceinline__ void ic_row_moments(const uint32_t* row, int sb, const uint32_t* mask,
                                               int v, int& m10, int& m01) {
  uint32_t w[9];
#pragma unroll
  for (int k = 0; k < 9; k++) w[k] = row[k];
  uint32_t s0 = 0, s1 = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const uint32_t px = __builtin_amdgcn_alignbyte(w[k + 1], w[k], sb) & mask[k];
    const uint32_t wt = (4u * k) | ((4u * k + 1) << 8) | ((4u * k + 2) << 16) | ((4u * k + 3) << 24);
    s0 = __builtin_amdgcn_udot4(px, 0x01010101u, s0, false);
    s1 = __builtin_amdgcn_udot4(px, wt, s1, false);
  }
  m10 += (int)s1 - 15 * (int)s0;  // sum (j - 15) I_j with j = u + 15
  m01 += v * (int)s0;
}

constexpr float kRoundMagic = 12582912.0f;  // 1.5 * 2^23: fl(x + M) = M + rint(x), |x| < 2^22
constexpr uint32_t kRoundBits = 0x4B400000u;

// LDS byte offset (relative to the patch centre, row stride `stride`) of a pattern point from
// the two rounded coordinates held as magic-biased floats: (row bits, col bits) -> row * stride
// + col + bias(stride), bias = 0x400000 * stride + 0x4B400000 (mod 2^32), which the caller
// folds into the centre address (`centre - bias`).
__device__ __forceinline__ uint32_t sample_offset(orbx_f2 rc, uint32_t stride) {
  // (copied to scalars first: __builtin_bit_cast of an ext_vector element access reads
  // element 0 with this clang)
  const float row = rc.x, col = rc.y;
  const uint32_t rb = __float_as_uint(row), cb = __float_as_uint(col);
  return __umul24(rb, stride) + cb;  // low 24 bits of rb = 0x400000 + row
}
__host__ __device__ constexpr uint32_t sample_bias(uint32_t stride) {
  return 0x400000u * stride + kRoundBits;
}

// ORBextractor (the reference binary's FMA pattern):
//   row = rint(fmaf(px, b, py * a)), col = rint(fmaf(px, a, -(py * b))), (a, b) = (cos, sin);
// nb = -b, so py * nb == -(py * b) exactly.
__device__ __forceinline__ orbx_f2 rotate_fma(float px, float py, float a, float b, float nb) {
  const orbx_f2 t = f2(py, py) * f2(a, nb);
  const orbx_f2 r = __builtin_elementwise_fma(f2(px, px), f2(b, a), t);
  return r + f2(kRoundMagic, kRoundMagic);
}

// cv::ORB 2.4 (no contraction): row = cvRound(px*b + py*a), col = cvRound(px*a - py*b),
// the subtraction as px*a + py*nb (x - y == x + (-y) exactly).
__device__ __forceinline__ orbx_f2 rotate_plain(float px, float py, float a, float b, float nb) {
  const orbx_f2 p = f2(px, px) * f2(b, a);
  const orbx_f2 q = f2(py, py) * f2(a, nb);
  return (p + q) + f2(kRoundMagic, kRoundMagic);
}

}  // namespace orbx
