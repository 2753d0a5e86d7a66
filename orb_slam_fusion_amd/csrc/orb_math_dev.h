// Device-side scalar math with the exact float semantics of the reference
// build (compiled with -ffp-contract=off; every fused multiply-add is
// explicit).
//  * dev_sinf / dev_cosf: glibc 2.35 single-precision sin/cos (FMA variant),
//    which the reference reaches via `cos(angle)` / `sin(angle)` on a float
//    (orb_extractor.cc:105-106).  Double-precision polynomial on the
//    quadrant-reduced argument; valid for |x| < 120 (angles are in [0, 2pi]).
//  * dev_fast_atan2: OpenCV 4.5.4 fastAtan2 (degrees), called by IC_Angle
//    (orb_extractor.cc:99).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace orbgpu {

struct SinCosPoly {
  double sign[4];
  double hpi_inv, hpi;
  double c0, c1, c2, c3, c4;
  double s1, s2, s3;
};

__device__ __forceinline__ const SinCosPoly& sincos_poly(int which) {
  static constexpr SinCosPoly tab[2] = {
      {{1.0, -1.0, -1.0, 1.0}, 0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0, 0x1p0,
       -0x1.ffffffd0c621cp-2, 0x1.55553e1068f19p-5, -0x1.6c087e89a359dp-10,
       0x1.99343027bf8c3p-16, -0x1.555545995a603p-3, 0x1.1107605230bc4p-7,
       -0x1.994eb3774cf24p-13},
      {{1.0, -1.0, -1.0, 1.0}, 0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0, -0x1p0,
       0x1.ffffffd0c621cp-2, -0x1.55553e1068f19p-5, 0x1.6c087e89a359dp-10,
       -0x1.99343027bf8c3p-16, -0x1.555545995a603p-3, 0x1.1107605230bc4p-7,
       -0x1.994eb3774cf24p-13}};
  return tab[which];
}

__device__ __forceinline__ uint32_t abstop12(float x) {
  return (__float_as_uint(x) >> 20) & 0x7ff;
}

__device__ __forceinline__ float sc_poly(double x, double x2, const SinCosPoly& p, int n) {
  if ((n & 1) == 0) {
    const double x3 = x * x2;
    const double s1 = __builtin_fma(x2, p.s3, p.s2);
    const double x7 = x3 * x2;
    const double s = __builtin_fma(x3, p.s1, x);
    return (float)__builtin_fma(x7, s1, s);
  }
  const double x4 = x2 * x2;
  const double c2 = __builtin_fma(x2, p.c4, p.c3);
  const double c1 = __builtin_fma(x2, p.c1, p.c0);
  const double x6 = x4 * x2;
  const double c = __builtin_fma(x4, p.c2, c1);
  return (float)__builtin_fma(x6, c2, c);
}

// Evaluates sin (want_cos = 0) or cos (want_cos = 1) of y.
__device__ __forceinline__ float dev_sincosf(float y, int want_cos) {
  const float pio4 = 0x1.921FB6p-1f;
  double x = y;
  if (abstop12(y) < abstop12(pio4)) {
    if (abstop12(y) < abstop12(0x1p-12f)) return want_cos ? 1.0f : y;
    return sc_poly(x, x * x, sincos_poly(0), want_cos);
  }
  const SinCosPoly& p0 = sincos_poly(0);
  const double r = x * p0.hpi_inv;
  const int n = ((int32_t)r + 0x800000) >> 24;
  x = __builtin_fma(-(double)n, p0.hpi, x);
  const double s = p0.sign[n & 3];
  const SinCosPoly& p = sincos_poly((n & 2) ? 1 : 0);
  return sc_poly(x * s, x * x, p, want_cos ? (n ^ 1) : n);
}

__device__ __forceinline__ float dev_sinf(float y) { return dev_sincosf(y, 0); }
__device__ __forceinline__ float dev_cosf(float y) { return dev_sincosf(y, 1); }

__device__ __forceinline__ float dev_fast_atan2(float y, float x) {
  const float k = (float)(180 / 3.14159265358979323846);
  const float p1 = 0.9997878412794807f * k, p3 = -0.3258083974640975f * k;
  const float p5 = 0.1555786518463281f * k, p7 = -0.04432655554792128f * k;
  const float eps = (float)2.2204460492503131e-16;  // (float)DBL_EPSILON
  const float ax = __builtin_fabsf(x), ay = __builtin_fabsf(y);
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

__device__ __forceinline__ int dev_round(float v) { return (int)__builtin_rintf(v); }

}  // namespace orbgpu
