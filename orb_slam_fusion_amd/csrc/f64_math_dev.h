// IEEE-valued f64 division and square root without the range handling the
// compiler's generic lowering carries (shared by the pose, inertial and BA
// kernels).  Each helper is the compiler's own sequence minus the steps that
// only matter for denormal / huge / zero / infinite operands, so it returns
// the same value for the normal, finite operands of a projection or a robust
// kernel; a reciprocal is computed once per denominator and reused.
#pragma once

#include <hip/hip_runtime.h>

namespace orbgpu {

// f64 division as the compiler lowers it (v_rcp_f64, two Newton steps, one
// residual correction), minus its v_div_scale / v_div_fmas scaling and
// v_div_fixup special cases: the same value for the normal, finite operands
// of a projection, and the reciprocal is computed once for every division
// by the same denominator (an edge divides by z up to three times).
struct RecipF64 {
  double d, r;
};
__device__ __forceinline__ RecipF64 recip_f64(double d) {
  double r = __builtin_amdgcn_rcp(d);
  r = fma(r, fma(-d, r, 1.0), r);
  r = fma(r, fma(-d, r, 1.0), r);
  return RecipF64{d, r};
}
__device__ __forceinline__ double div_by(double n, const RecipF64& q) {
  const double m = n * q.r;
  return fma(fma(-q.d, m, n), q.r, m);
}

// f64 sqrt as the compiler lowers it (v_rsq_f64, then the Goldschmidt /
// Newton refinement), minus its v_ldexp range scaling for x < 2^-767 and the
// zero / infinity class check: the same value for the normal, finite x here.
__device__ __forceinline__ double sqrt_f64(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  double s = x * y, h = y * 0.5;
  const double r = fma(-h, s, 0.5);
  s = fma(s, r, s);
  const double d0 = fma(-s, s, x);
  h = fma(h, r, h);
  s = fma(d0, h, s);
  const double d1 = fma(-s, s, x);
  return fma(d1, h, s);
}

}  // namespace orbgpu
