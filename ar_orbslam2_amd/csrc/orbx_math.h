// orbx_math.h — bit-exact scalar math shared by the gfx950 kernels (and compiled for the host
// by tests/test_math_port.py to check it exhaustively against the host libm).
//
//  * orbx_sincosf: port of glibc 2.35 sincosf (sysdeps/ieee754/flt-32/s_sincosf.c +
//    sincosf.h + sincosf_data.c), the function the reference binary imports for
//    computeOrbDescriptor (ORB_SLAM2/src/ORBextractor.cc:103-104).  Only the
//    |x| < 120 paths are needed: descriptor angles are in [0, 2*pi].  Double-precision
//    polynomial; results agree with libm for every float in [0, 2*pi] with or without
//    contraction of the polynomial (checked exhaustively).
//  * orbx_fast_atan2: cv::fastAtan2 of OpenCV 2.4 (degrees), evaluated in f32 with no
//    contraction; used by IC_Angle (ORBextractor.cc:97).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define ORBX_HD __host__ __device__ inline
#else
#define ORBX_HD inline
#include <math.h>
#include <string.h>
#endif

#pragma clang fp contract(off)

namespace orbx {

ORBX_HD uint32_t f32_bits(float f) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __float_as_uint(f);
#else
  uint32_t u;
  memcpy(&u, &f, 4);
  return u;
#endif
}

ORBX_HD uint32_t abstop12(float x) { return (f32_bits(x) >> 20) & 0x7ff; }

ORBX_HD double dfma(double a, double b, double c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_fma(a, b, c);
#else
  return fma(a, b, c);
#endif
}

// sincosf_poly (glibc sincosf.h): quadrant n odd swaps the sine/cosine outputs.
ORBX_HD void sincosf_poly(double x, double x2, bool neg_cos_table, int n, float* sinp,
                          float* cosp) {
  // __sincosf_table[0] / [1] (the second negates the cosine polynomial)
  const double c0 = neg_cos_table ? -0x1p0 : 0x1p0;
  const double c1 = neg_cos_table ? 0x1.ffffffd0c621cp-2 : -0x1.ffffffd0c621cp-2;
  const double c2 = neg_cos_table ? -0x1.55553e1068f19p-5 : 0x1.55553e1068f19p-5;
  const double c3 = neg_cos_table ? 0x1.6c087e89a359dp-10 : -0x1.6c087e89a359dp-10;
  const double c4 = neg_cos_table ? -0x1.99343027bf8c3p-16 : 0x1.99343027bf8c3p-16;
  const double s1c = -0x1.555545995a603p-3, s2c = 0x1.1107605230bc4p-7,
               s3c = -0x1.994eb3774cf24p-13;
  const double x4 = x2 * x2, x3 = x2 * x;
  const double cc2 = dfma(x2, c4, c3);
  const double ss1 = dfma(x2, s3c, s2c);
  const double cc1 = dfma(x2, c1, c0);
  const double x5 = x3 * x2, x6 = x4 * x2;
  const double s = dfma(x3, s1c, x);
  const double c = dfma(x4, c2, cc1);
  const float so = (float)dfma(x5, ss1, s);
  const float co = (float)dfma(x6, cc2, c);
  if (n & 1) {
    *sinp = co;
    *cosp = so;
  } else {
    *sinp = so;
    *cosp = co;
  }
}

// glibc sincosf for |y| < 120 (reduce_fast with the 2^24-prescaled 2/pi, !TOINT_INTRINSICS).
ORBX_HD void orbx_sincosf(float y, float* sinp, float* cosp) {
  double x = (double)y;
  if (abstop12(y) < abstop12(0x1.921fb6p-1f)) {  // |y| < pi/4
    if (abstop12(y) < abstop12(0x1p-12f)) {
      *sinp = y;
      *cosp = 1.0f;
      return;
    }
    sincosf_poly(x, x * x, false, 0, sinp, cosp);
    return;
  }
  const double hpi_inv = 0x1.45F306DC9C883p+23, hpi = 0x1.921FB54442D18p0;
  const double r = x * hpi_inv;
  const int n = ((int32_t)r + 0x800000) >> 24;
  x = dfma(-(double)n, hpi, x);
  const double s = (n & 3) == 1 || (n & 3) == 2 ? -1.0 : 1.0;  // sign[4] = {1,-1,-1,1}
  sincosf_poly(x * s, x * x, (n & 2) != 0, n, sinp, cosp);
}

// cv::fastAtan2 (OpenCV 2.4 core/src/mathfuncs.cpp) — degrees in [0, 360).
ORBX_HD float orbx_fast_atan2(float y, float x) {
  const float k = 57.295780181884765625f;  // (float)(180/CV_PI)
  const float p1 = 0.9997878412794807f * k;
  const float p3 = -0.3258083974640975f * k;
  const float p5 = 0.1555786518463281f * k;
  const float p7 = -0.04432655554792128f * k;
  const float eps = 2.220446049250313e-16f;  // (float)DBL_EPSILON
  const float ax = x < 0 ? -x : x, ay = y < 0 ? -y : y;
  float a, c, c2;
  if (ax >= ay) {
    c = ay / (ax + eps);
    c2 = c * c;
    a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
  } else {
    c = ax / (ay + eps);
    c2 = c * c;
    a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
  }
  if (x < 0) a = 180.f - a;
  if (y < 0) a = 360.f - a;
  return a;
}

}  // namespace orbx
