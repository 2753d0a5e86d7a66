// Inertial device math shared by the tracking optimisations
// (inertial_kernels.hip) and LocalInertialBA (lba_kernels.hip): 3x3 algebra,
// the SO3 maps of g2o_types.cc:779-848 and the float side of
// IMU::Preintegrated (imu_types.cc:283-310).  The branches on the rotation
// angle are made wave-uniform (readfirstlane): every lane of a wave must
// evaluate the same rotation.  Include after `#pragma clang fp contract(fast)`
// (fp64 solver TUs, parity by tolerance).
#pragma once
#include "f64_math_dev.h"
#include "uniform_dev.h"
#include <hip/hip_runtime.h>

#include "../../include/orbgpu.h"

namespace orbgpu {

struct CalibD {
  double fx, fy, cx, cy, bf;
  double Rcb[9], tcb[3], Rbc[9], tbc[3];
};

struct StateD {
  double Rwb[9], twb[3], Rcw[9], tcw[3], v[3], bg[3], ba[3];
};

// ---- 3x3 helpers (row-major) ------------------------------------------------
__device__ __forceinline__ void m3_mul(const double* A, const double* B, double* C) {
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      C[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
}
__device__ __forceinline__ void m3_tr(const double* A, double* C) {
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) C[3 * i + j] = A[3 * j + i];
}
__device__ __forceinline__ void m3_mv(const double* A, const double* v, double* o) {
#pragma unroll
  for (int i = 0; i < 3; ++i) o[i] = A[3 * i] * v[0] + A[3 * i + 1] * v[1] + A[3 * i + 2] * v[2];
}
__device__ __forceinline__ void m3_hat(const double* w, double* W) {
  W[0] = 0;
  W[1] = -w[2];
  W[2] = w[1];
  W[3] = w[2];
  W[4] = 0;
  W[5] = -w[0];
  W[6] = -w[1];
  W[7] = w[0];
  W[8] = 0;
}

// NormalizeRotation: orthogonal polar factor by Newton steps X <- (X + X^-T)/2.
// The inputs here are rotations up to float (preintegration) or double
// (ExpSO3) rounding, where the iteration converges quadratically: two steps
// reach double precision (the oracle takes three; same result to rounding).
__device__ __forceinline__ void polar3(double* X) {
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    double C[9];
    C[0] = X[4] * X[8] - X[5] * X[7];
    C[1] = X[5] * X[6] - X[3] * X[8];
    C[2] = X[3] * X[7] - X[4] * X[6];
    C[3] = X[2] * X[7] - X[1] * X[8];
    C[4] = X[0] * X[8] - X[2] * X[6];
    C[5] = X[1] * X[6] - X[0] * X[7];
    C[6] = X[1] * X[5] - X[2] * X[4];
    C[7] = X[2] * X[3] - X[0] * X[5];
    C[8] = X[0] * X[4] - X[1] * X[3];
    // det ~ 1: the IEEE quotient by f64_math_dev.h (no range steps)
    const double rdet = div_by(1.0, recip_f64(X[0] * C[0] + X[1] * C[1] + X[2] * C[2]));
#pragma unroll
    for (int i = 0; i < 9; ++i) X[i] = 0.5 * (X[i] + C[i] * rdet);
  }
}

// below this squared angle the SO(3) coefficients come from series, not sincos
constexpr double kSeriesD2 = 0.0025;

// profiling hook of the inertial kernel's stamps build (phase marks inside
// the IMU edge); empty elsewhere
#ifndef IMU_EDGE_MARK
#define IMU_EDGE_MARK(i) (void)0
#define IMU_EDGE_MARK_INIT (void)0
#endif

// ExpSO3 (g2o_types.cc:783-796)
// kUniform: every lane of the wave evaluates the same rotation (the branches
// are taken by readfirstlane); false: each lane its own (divergent branches)
template <bool kUniform = true>
__device__ __forceinline__ void exp_so3(const double* w, double* R) {
  const double d2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
  const double d = sqrt(d2);
  double W[9], WW[9];
  m3_hat(w, W);
  m3_mul(W, W, WW);
  double s, c;
  auto uni = [](bool b) { return kUniform ? uniform_branch(b ? 1 : 0) != 0 : b; };
  if (uni(d < 1e-5)) {
    s = 1.0;
    c = 0.5;
  } else if (uni(d2 < kSeriesD2)) {
    // sin(d)/d and (1 - cos d)/d^2 by their Taylor series (truncation
    // < 1e-20 below d = 0.05; the updates near convergence all land here)
    s = 1.0 + d2 * (-1.0 / 6 + d2 * (1.0 / 120 + d2 * (-1.0 / 5040 + d2 * (1.0 / 362880))));
    c = 0.5 + d2 * (-1.0 / 24 + d2 * (1.0 / 720 + d2 * (-1.0 / 40320 + d2 * (1.0 / 3628800))));
  } else {
    double sn, cs;
    sincos(d, &sn, &cs);
    s = sn / d;
    c = (1.0 - cs) / d2;
  }
#pragma unroll
  for (int i = 0; i < 9; ++i) R[i] = (i % 4 == 0 ? 1.0 : 0.0) + W[i] * s + WW[i] * c;
  polar3(R);
}

// LogSO3 (g2o_types.cc:798-811)
__device__ __forceinline__ void log_so3(const double* R, double* w) {
  const double t = R[0] + R[4] + R[8];
  w[0] = (R[7] - R[5]) / 2;
  w[1] = (R[2] - R[6]) / 2;
  w[2] = (R[3] - R[1]) / 2;
  const double ct = (t - 1.0) * 0.5;
  if (uniform_branch(ct > 1 || ct < -1 ? 1 : 0)) return;
  const double th = acos(ct);
  const double s = sin(th);
  if (uniform_branch(fabs(s) < 1e-5 ? 1 : 0)) return;
  const double f = div_by(th, recip_f64(s));  // |s| >= 1e-5 here
  w[0] *= f;
  w[1] *= f;
  w[2] *= f;
}

// InverseRightJacobianSO3 (kInv) / RightJacobianSO3 (g2o_types.cc:817-848)
template <bool kInv>
__device__ __forceinline__ void right_j(const double* v, double* J) {
  const double d2 = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
  const double d = sqrt(d2);
#pragma unroll
  for (int i = 0; i < 9; ++i) J[i] = i % 4 == 0 ? 1.0 : 0.0;
  if (uniform_branch(d < 1e-5 ? 1 : 0)) return;
  double W[9], WW[9];
  m3_hat(v, W);
  m3_mul(W, W, WW);
  double a, b;
  if (uniform_branch(d2 < kSeriesD2 ? 1 : 0)) {
    // the coefficients' Taylor series in d^2 (truncation < 1e-20 below 0.05)
    if (kInv) {  // 1/d^2 - (1 + cos d) / (2 d sin d)
      a = 0.5;
      b = 1.0 / 12 + d2 * (1.0 / 720 + d2 * (1.0 / 30240 + d2 * (1.0 / 1209600 + d2 * (1.0 / 47900160))));
    } else {  // -(1 - cos d) / d^2, (d - sin d) / d^3
      a = -(0.5 + d2 * (-1.0 / 24 + d2 * (1.0 / 720 + d2 * (-1.0 / 40320 + d2 * (1.0 / 3628800)))));
      b = 1.0 / 6 + d2 * (-1.0 / 120 + d2 * (1.0 / 5040 + d2 * (-1.0 / 362880 + d2 * (1.0 / 39916800))));
    }
  } else {
    double sn, cs;
    sincos(d, &sn, &cs);
    if (kInv) {
      a = 0.5;
      b = 1.0 / d2 - (1.0 + cs) / (2.0 * d * sn);
    } else {
      a = -(1.0 - cs) / d2;
      b = (d - sn) / (d2 * d);
    }
  }
#pragma unroll
  for (int i = 0; i < 9; ++i) J[i] += W[i] * a + WW[i] * b;
}

// ---- float side of IMU::Preintegrated ---------------------------------------
// Preintegrated::GetDeltaRotation(b) (imu_types.cc:289-294): Sophus SO3f::exp
// of JRg * dbg (so3.hpp:584-618, unnormalised quaternion -> matrix), dR * it,
// NormalizeRotation (polar factor), cast to double.
__device__ __forceinline__ void delta_rotation(const orbgpu_imu_preint& p, const float* dbg,
                                               double* out) {
  float w[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) w[i] = p.JRg[3 * i] * dbg[0] + p.JRg[3 * i + 1] * dbg[1] + p.JRg[3 * i + 2] * dbg[2];
  const float th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
  float imag, real;
  if (uniform_branch(th2 < 1e-5f * 1e-5f ? 1 : 0)) {
    const float po4 = th2 * th2;
    imag = 0.5f - (float)(1.0 / 48.0) * th2 + (float)(1.0 / 3840.0) * po4;
    real = 1.f - (float)(1.0 / 8.0) * th2 + (float)(1.0 / 384.0) * po4;
  } else {
    const float th = sqrtf(th2);
    const float half = 0.5f * th;
    imag = sinf(half) / th;
    real = cosf(half);
  }
  const float qx = imag * w[0], qy = imag * w[1], qz = imag * w[2], qw = real;
  const float tx = 2 * qx, ty = 2 * qy, tz = 2 * qz;
  const float twx = tx * qw, twy = ty * qw, twz = tz * qw;
  const float txx = tx * qx, txy = ty * qx, txz = tz * qx;
  const float tyy = ty * qy, tyz = tz * qy, tzz = tz * qz;
  const float E[9] = {1.f - (tyy + tzz), txy - twz, txz + twy, txy + twz, 1.f - (txx + tzz),
                      tyz - twx, txz - twy, tyz + twx, 1.f - (txx + tyy)};
  double M[9];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      M[3 * i + j] = (double)(p.dR[3 * i] * E[j] + p.dR[3 * i + 1] * E[3 + j] + p.dR[3 * i + 2] * E[6 + j]);
  polar3(M);
#pragma unroll
  for (int i = 0; i < 9; ++i) out[i] = (double)(float)M[i];
}

__device__ __forceinline__ void delta_lin(const float* d0, const float* Jg, const float* Ja,
                                          const float* dbg, const float* dba, double* out) {
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const float g = Jg[3 * i] * dbg[0] + Jg[3 * i + 1] * dbg[1] + Jg[3 * i + 2] * dbg[2];
    const float a = Ja[3 * i] * dba[0] + Ja[3 * i + 1] * dba[1] + Ja[3 * i + 2] * dba[2];
    out[i] = (double)(d0[i] + g + a);
  }
}

// ImuCamPose::Update (g2o_types.cc:192-214); the NormalizeRotation there
// discards its result.
template <bool kUniform = true>
__device__ __forceinline__ void pose_update(StateD& s, const double* u, const CalibD& c, bool store) {
  double R[9], E[9], Rn[9], d[3], ut[3] = {u[3], u[4], u[5]};
#pragma unroll
  for (int i = 0; i < 9; ++i) R[i] = s.Rwb[i];
  m3_mv(R, ut, d);
  exp_so3<kUniform>(u, E);
  m3_mul(R, E, Rn);
  double t[3] = {s.twb[0] + d[0], s.twb[1] + d[1], s.twb[2] + d[2]};
  double Rbw[9], tbw[3], Rcw[9], tcw[3];
  m3_tr(Rn, Rbw);
  m3_mv(Rbw, t, tbw);
  tbw[0] = -tbw[0];
  tbw[1] = -tbw[1];
  tbw[2] = -tbw[2];
  m3_mul(c.Rcb, Rbw, Rcw);
  m3_mv(c.Rcb, tbw, tcw);
  if (store) {
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      s.Rwb[i] = Rn[i];
      s.Rcw[i] = Rcw[i];
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      s.twb[i] = t[i];
      s.tcw[i] = tcw[i] + c.tcb[i];
    }
  }
}

// ---- EdgeInertial::computeError / linearizeOplus (g2o_types.cc:494-578)
// between vertex set 1 (s1: VP1 VV1 VG1 VA1) and 2 (s2: VP2 VV2), one wave,
// every lane the same values; lane 0 stores the error to ei[9] and the
// estimate-dependent Jacobian blocks to J[9][24] (columns VP1 VV1 VG1 VA1 VP2
// VV2).  The constant blocks (-I, -JVg, -JPg, -JVa, -JPa) and the zeros are
// the caller's (written once).
// The Jacobian blocks of EdgeInertial that depend on the two states only
// (not on the preintegration): -Rbw1 (VV1 rows 3-5 and, x dt, 6-8), Rbw1
// (VV2), [Rbw1 dv]x and [Rbw1 dp]x (VP1 rotation), Rbw1 Rwb2 (VP2
// translation).  inertial_edge_core<false> leaves them to this function, so
// another wave can form them at the same time.
__device__ __forceinline__ void inertial_edge_lin(const StateD& s1, const StateD& s2, double dt, int lane,
                                                  double* J) {
  const double g2 = -(double)9.81f;
  double Rbw1[9];
  m3_tr(s1.Rwb, Rbw1);
  auto put = [&](int r0, int c0, const double* m, double sc) {
    if (lane == 0)
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) J[(r0 + i) * 24 + c0 + j] = sc * m[3 * i + j];
  };
  put(3, 6, Rbw1, -1.0);
  put(6, 6, Rbw1, -dt);
  put(3, 21, Rbw1, 1.0);
  {
    double dv[3], rv[3], hv[9];
#pragma unroll
    for (int i = 0; i < 3; ++i) dv[i] = s2.v[i] - s1.v[i] - (i == 2 ? g2 * dt : 0.0);
    m3_mv(Rbw1, dv, rv);
    m3_hat(rv, hv);
    put(3, 0, hv, 1.0);
  }
  {
    double dp2[3], rp2[3], hp[9];
#pragma unroll
    for (int i = 0; i < 3; ++i) dp2[i] = s2.twb[i] - s1.twb[i] - s1.v[i] * dt - (i == 2 ? 0.5 * g2 * dt * dt : 0.0);
    m3_mv(Rbw1, dp2, rp2);
    m3_hat(rp2, hp);
    put(6, 0, hp, 1.0);
  }
  {
    double R12[9];
    m3_mul(Rbw1, s2.Rwb, R12);
    put(6, 18, R12, 1.0);
  }
}

template <bool kLin = true>
__device__ __forceinline__ void inertial_edge_core(const StateD& s1, const StateD& s2,
                                                   const orbgpu_imu_preint& pi, double dt, int lane,
                                                   double* J, double* ei) {
  IMU_EDGE_MARK_INIT;
  float bg[3], ba[3], dbg[3], dba[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    bg[i] = (float)s1.bg[i];
    ba[i] = (float)s1.ba[i];
    dbg[i] = bg[i] - pi.bg[i];
    dba[i] = ba[i] - pi.ba[i];
  }
  double dR[9], dV[3], dP[3];
  delta_rotation(pi, dbg, dR);
  delta_lin(pi.dV, pi.JVg, pi.JVa, dbg, dba, dV);
  delta_lin(pi.dP, pi.JPg, pi.JPa, dbg, dba, dP);
  IMU_EDGE_MARK(7);
  const double g2 = -(double)9.81f;  // g = (0, 0, -GRAVITY_VALUE)
  double Rbw1[9], dRt[9], T[9], eR[9];
  m3_tr(s1.Rwb, Rbw1);
  m3_tr(dR, dRt);
  m3_mul(dRt, Rbw1, T);
  m3_mul(T, s2.Rwb, eR);
  double er[3];
  log_so3(eR, er);
  IMU_EDGE_MARK(9);
  double dv[3], dp[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    dv[i] = s2.v[i] - s1.v[i] - (i == 2 ? g2 * dt : 0.0);
    dp[i] = s2.twb[i] - s1.twb[i] - s1.v[i] * dt - (i == 2 ? g2 * dt * dt / 2 : 0.0);
  }
  double rv[3], rp[3];
  m3_mv(Rbw1, dv, rv);
  m3_mv(Rbw1, dp, rp);
  double e[9];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    e[i] = er[i];
    e[3 + i] = rv[i] - dV[i];
    e[6 + i] = rp[i] - dP[i];
  }
  // Jacobian blocks (g2o_types.cc:523-578); the constant ones (-I, -JVg,
  // -JPg, -JVa, -JPa) and the zeros are in place from inertial_edge_const.
  // Each block is stored as soon as it is formed (short live ranges).
  auto put = [&](int r0, int c0, const double* m, double sc) {
    if (lane == 0)
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) J[(r0 + i) * 24 + c0 + j] = sc * m[3 * i + j];
  };
  if (lane == 0)
#pragma unroll
    for (int i = 0; i < 9; ++i) ei[i] = e[i];
  if constexpr (kLin) inertial_edge_lin(s1, s2, dt, lane, J);
  IMU_EDGE_MARK(15);
  double invJr[9];
  right_j<true>(er, invJr);
  put(0, 15, invJr, 1.0);
  {
    double Rt2[9], A[9], J0r[9];
    m3_tr(s2.Rwb, Rt2);
    m3_mul(invJr, Rt2, A);
    m3_mul(A, s1.Rwb, J0r);
    put(0, 0, J0r, -1.0);  // -invJr * Rwb2^T * Rwb1
  }
  {
    double JRg[9], jd[3], RJ[9], eRt[9], A[9], B[9], Gb[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) JRg[i] = pi.JRg[i];
    const double dbgd[3] = {dbg[0], dbg[1], dbg[2]};
    m3_mv(JRg, dbgd, jd);
    right_j<false>(jd, RJ);
    m3_tr(eR, eRt);
    m3_mul(invJr, eRt, A);
    m3_mul(A, RJ, B);
    m3_mul(B, JRg, Gb);
    put(0, 9, Gb, -1.0);  // -invJr * eR^T * Jr(JRg dbg) * JRg
  }
}

}  // namespace orbgpu
