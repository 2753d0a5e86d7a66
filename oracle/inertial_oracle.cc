// ORACLE (test infrastructure only): restatement of
// Optimizer::PoseInertialOptimizationLastFrame (src/solver/g2o_solver/
// optimizer.cc:4762-5160) and PoseInertialOptimizationLastKeyFrame
// (:4394-4760) for the pinhole, non-fisheye case (Frame::Nleft == -1):
//   vertices   VertexPose / ImuCamPose::Update (g2o_types.cc:74-118,192-214),
//              VertexVelocity / GyroBias / AccBias (g2o_types.h:181-237)
//   edges      EdgeMonoOnlyPose / EdgeStereoOnlyPose (g2o_types.h:354-456,
//              g2o_types.cc:361-446), EdgeInertial (g2o_types.cc:472-578),
//              EdgeGyroRW / EdgeAccRW (g2o_types.h:592-662), EdgePriorPoseImu
//              (g2o_types.cc:729-764)
//   SO3        ExpSO3 / LogSO3 / (Inverse)RightJacobianSO3 (g2o_types.cc:
//              779-848), Preintegrated::GetDelta* (imu_types.cc:283-310),
//              Sophus SO3f::exp (so3.hpp:584-618)
//   solver     g2o Gauss-Newton (optimization_algorithm_gauss_newton.cpp),
//              BlockSolverX without Schur, LinearSolverDense (Eigen LDLT,
//              linear_solver_dense.h:56-104), multi-edge quadratic form
//              (base_multi_edge.hpp:34-45), Huber (robust_kernel_impl.cpp)
//   Marginalize (optimizer.cc:2904-2984)
//
// Restated semantics worth naming:
// * ImuCamPose::Update calls NormalizeRotation(Rwb) every third update but
//   discards the result (g2o_types.cc:204): a no-op, kept as one.
// * NormalizeRotation (Eigen JacobiSVD U V^T) is the orthogonal polar factor;
//   it is computed here by Newton iterations X <- (X + X^-T) / 2 (three, in
//   double; the float version rounds the double result).  Equal to the SVD
//   form up to rounding -- the reference's float SVD is not bit-reproducible
//   without Eigen, so parity for this path is by tolerance.
// * Marginalize's JacobiSVD pseudo-inverse with the 1e-6 singular value cut is
//   restated for the symmetric block it is applied to: eigen-decomposition by
//   cyclic Jacobi, pinv = sum over |lambda| > 1e-6 of v v^T / lambda.
// * When the LDLT is not positive g2o leaves the solver's x untouched, still
//   applies it and stops the round: x persists across iterations here, zero
//   at the start (the reference's buffer starts uninitialised).
// * The classification reads each inlier edge's error from the last
//   computeActiveErrors, i.e. at the state before the round's last update.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "g2o_math.h"
#include "inertial_math.h"
#include "../include/orbgpu.h"

namespace oracle {
namespace inertial {

M3 eye() {
  M3 m{};
  m(0, 0) = m(1, 1) = m(2, 2) = 1;
  return m;
}
M3 mul(const M3& A, const M3& B) {
  M3 C{};
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) C(i, j) = A(i, 0) * B(0, j) + A(i, 1) * B(1, j) + A(i, 2) * B(2, j);
  return C;
}
M3 tr(const M3& A) {
  M3 C;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) C(i, j) = A(j, i);
  return C;
}
V3 mv(const M3& A, const V3& v) {
  V3 o;
  for (int i = 0; i < 3; ++i) o[i] = A(i, 0) * v[0] + A(i, 1) * v[1] + A(i, 2) * v[2];
  return o;
}
V3 add(const V3& a, const V3& b) { return V3{{a[0] + b[0], a[1] + b[1], a[2] + b[2]}}; }
V3 sub(const V3& a, const V3& b) { return V3{{a[0] - b[0], a[1] - b[1], a[2] - b[2]}}; }
V3 scl(const V3& a, double s) { return V3{{a[0] * s, a[1] * s, a[2] * s}}; }
M3 hat(const V3& w) {
  M3 W{};
  W(0, 1) = -w[2];
  W(0, 2) = w[1];
  W(1, 0) = w[2];
  W(1, 2) = -w[0];
  W(2, 0) = -w[1];
  W(2, 1) = w[0];
  return W;
}
M3 from_f(const float* f) {
  M3 m;
  for (int i = 0; i < 9; ++i) m.a[i] = f[i];
  return m;
}
V3 from_f3(const float* f) { return V3{{f[0], f[1], f[2]}}; }
M3 from_d(const double* f) {
  M3 m;
  for (int i = 0; i < 9; ++i) m.a[i] = f[i];
  return m;
}
V3 from_d3(const double* f) { return V3{{f[0], f[1], f[2]}}; }

// Orthogonal polar factor by Newton iterations (NormalizeRotation).
M3 polar(const M3& R) {
  M3 X = R;
  for (int it = 0; it < 3; ++it) {
    // X^-T = cofactor(X) / det(X)
    M3 C;
    C(0, 0) = X(1, 1) * X(2, 2) - X(1, 2) * X(2, 1);
    C(0, 1) = X(1, 2) * X(2, 0) - X(1, 0) * X(2, 2);
    C(0, 2) = X(1, 0) * X(2, 1) - X(1, 1) * X(2, 0);
    C(1, 0) = X(0, 2) * X(2, 1) - X(0, 1) * X(2, 2);
    C(1, 1) = X(0, 0) * X(2, 2) - X(0, 2) * X(2, 0);
    C(1, 2) = X(0, 1) * X(2, 0) - X(0, 0) * X(2, 1);
    C(2, 0) = X(0, 1) * X(1, 2) - X(0, 2) * X(1, 1);
    C(2, 1) = X(0, 2) * X(1, 0) - X(0, 0) * X(1, 2);
    C(2, 2) = X(0, 0) * X(1, 1) - X(0, 1) * X(1, 0);
    const double det = X(0, 0) * C(0, 0) + X(0, 1) * C(0, 1) + X(0, 2) * C(0, 2);
    for (int i = 0; i < 9; ++i) X.a[i] = 0.5 * (X.a[i] + C.a[i] / det);
  }
  return X;
}

// g2o_types.cc:783-796
M3 ExpSO3(double x, double y, double z) {
  const double d2 = x * x + y * y + z * z;
  const double d = std::sqrt(d2);
  const M3 W = hat(V3{{x, y, z}});
  const M3 WW = mul(W, W);
  M3 res = eye();
  if (d < 1e-5) {
    for (int i = 0; i < 9; ++i) res.a[i] += W.a[i] + 0.5 * WW.a[i];
  } else {
    const double s = std::sin(d) / d, c = (1.0 - std::cos(d)) / d2;
    for (int i = 0; i < 9; ++i) res.a[i] += W.a[i] * s + WW.a[i] * c;
  }
  return polar(res);
}

// g2o_types.cc:798-811
V3 LogSO3(const M3& R) {
  const double t = R(0, 0) + R(1, 1) + R(2, 2);
  V3 w{{(R(2, 1) - R(1, 2)) / 2, (R(0, 2) - R(2, 0)) / 2, (R(1, 0) - R(0, 1)) / 2}};
  const double costheta = (t - 1.0) * 0.5;
  if (costheta > 1 || costheta < -1) return w;
  const double theta = std::acos(costheta);
  const double s = std::sin(theta);
  if (std::fabs(s) < 1e-5) return w;
  return scl(w, theta / s);
}

// g2o_types.cc:817-829
M3 InvRightJ(const V3& v) {
  const double d2 = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
  const double d = std::sqrt(d2);
  M3 r = eye();
  if (d < 1e-5) return r;
  const M3 W = hat(v), WW = mul(W, W);
  const double c = 1.0 / d2 - (1.0 + std::cos(d)) / (2.0 * d * std::sin(d));
  for (int i = 0; i < 9; ++i) r.a[i] += W.a[i] / 2 + WW.a[i] * c;
  return r;
}

// g2o_types.cc:835-848
M3 RightJ(const V3& v) {
  const double d2 = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
  const double d = std::sqrt(d2);
  M3 r = eye();
  if (d < 1e-5) return r;
  const M3 W = hat(v), WW = mul(W, W);
  const double a = (1.0 - std::cos(d)) / d2, b = (d - std::sin(d)) / (d2 * d);
  for (int i = 0; i < 9; ++i) r.a[i] += -W.a[i] * a + WW.a[i] * b;
  return r;
}

// ---- float side of IMU::Preintegrated -------------------------------------
struct F3x3 {
  float a[9];
};

// Sophus::SO3f::exp(w).matrix(): the (unnormalised) quaternion of so3.hpp:
// 584-618 through Eigen's toRotationMatrix.
F3x3 so3f_exp(const float w[3]) {
  const float theta_sq = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
  float imag, real;
  if (theta_sq < 1e-5f * 1e-5f) {
    const float po4 = theta_sq * theta_sq;
    imag = 0.5f - (float)(1.0 / 48.0) * theta_sq + (float)(1.0 / 3840.0) * po4;
    real = 1.f - (float)(1.0 / 8.0) * theta_sq + (float)(1.0 / 384.0) * po4;
  } else {
    const float theta = std::sqrt(theta_sq);
    const float half = 0.5f * theta;
    imag = std::sin(half) / theta;
    real = std::cos(half);
  }
  const float qx = imag * w[0], qy = imag * w[1], qz = imag * w[2], qw = real;
  const float tx = 2 * qx, ty = 2 * qy, tz = 2 * qz;
  const float twx = tx * qw, twy = ty * qw, twz = tz * qw;
  const float txx = tx * qx, txy = ty * qx, txz = tz * qx;
  const float tyy = ty * qy, tyz = tz * qy, tzz = tz * qz;
  F3x3 m;
  m.a[0] = 1.f - (tyy + tzz);
  m.a[1] = txy - twz;
  m.a[2] = txz + twy;
  m.a[3] = txy + twz;
  m.a[4] = 1.f - (txx + tzz);
  m.a[5] = tyz - twx;
  m.a[6] = txz - twy;
  m.a[7] = tyz + twx;
  m.a[8] = 1.f - (txx + tyy);
  return m;
}

Preint preint_view(const orbgpu_imu_preint& p) {
  return Preint{p.dR, p.dV, p.dP, p.JRg, p.JVg, p.JVa, p.JPg, p.JPa, p.bg, p.ba};
}

void fmv(const float* A, const float* v, float* o) {
  for (int i = 0; i < 3; ++i) o[i] = A[3 * i] * v[0] + A[3 * i + 1] * v[1] + A[3 * i + 2] * v[2];
}

// Preintegrated::GetDeltaRotation(b_) (imu_types.cc:289-294)
M3 delta_rotation(const Preint& p, const float bg[3]) {
  const float dbg[3] = {bg[0] - p.bg[0], bg[1] - p.bg[1], bg[2] - p.bg[2]};
  float w[3];
  fmv(p.JRg, dbg, w);
  const F3x3 E = so3f_exp(w);
  float prod[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      prod[3 * i + j] = p.dR[3 * i] * E.a[j] + p.dR[3 * i + 1] * E.a[3 + j] + p.dR[3 * i + 2] * E.a[6 + j];
  M3 m;
  for (int i = 0; i < 9; ++i) m.a[i] = prod[i];
  const M3 q = polar(m);
  for (int i = 0; i < 9; ++i) m.a[i] = (double)(float)q.a[i];
  return m;
}

// GetDeltaVelocity / GetDeltaPosition (imu_types.cc:296-310)
V3 delta_lin(const float* d0, const float* Jg, const float* Ja, const Preint& p, const float bg[3],
             const float ba[3]) {
  const float dbg[3] = {bg[0] - p.bg[0], bg[1] - p.bg[1], bg[2] - p.bg[2]};
  const float dba[3] = {ba[0] - p.ba[0], ba[1] - p.ba[1], ba[2] - p.ba[2]};
  float g[3], a[3];
  fmv(Jg, dbg, g);
  fmv(Ja, dba, a);
  return V3{{(double)(d0[0] + g[0] + a[0]), (double)(d0[1] + g[1] + a[1]),
             (double)(d0[2] + g[2] + a[2])}};
}

// ---- problem ---------------------------------------------------------------
void pose_update(State& s, const double* u, const Calib& c) {  // ImuCamPose::Update
  const V3 ut{{u[3], u[4], u[5]}};
  s.twb = add(s.twb, mv(s.Rwb, ut));
  s.Rwb = mul(s.Rwb, ExpSO3(u[0], u[1], u[2]));
  // its++ / NormalizeRotation(Rwb) with the result discarded: no-op
  const M3 Rbw = tr(s.Rwb);
  const V3 tbw = scl(mv(Rbw, s.twb), -1.0);
  s.Rcw = mul(c.Rcb, Rbw);
  s.tcw = add(mv(c.Rcb, tbw), c.tcb);
}

struct VisEdge {
  double Xw[3], obs[3];
  bool stereo, close;
  double info, delta;
  bool robust = true;
  int level = 0;
  double err[3] = {0, 0, 0};
};

void vis_error(const VisEdge& e, const State& s, const Calib& c, double err[3]) {
  const V3 Xc = add(mv(s.Rcw, V3{{e.Xw[0], e.Xw[1], e.Xw[2]}}), s.tcw);
  const double u = c.fx * Xc[0] / Xc[2] + c.cx;
  const double v = c.fy * Xc[1] / Xc[2] + c.cy;
  err[0] = e.obs[0] - u;
  err[1] = e.obs[1] - v;
  err[2] = 0;
  if (e.stereo) {
    const double invz = 1 / Xc[2];
    err[2] = e.obs[2] - (u - c.bf * invz);
  }
}

double vis_chi2(const VisEdge& e) {
  double s = e.err[0] * e.info * e.err[0] + e.err[1] * e.info * e.err[1];
  if (e.stereo) s += e.err[2] * e.info * e.err[2];
  return s;
}

bool vis_depth_positive(const VisEdge& e, const State& s) {
  return s.Rcw(2, 0) * e.Xw[0] + s.Rcw(2, 1) * e.Xw[1] + s.Rcw(2, 2) * e.Xw[2] + s.tcw[2] > 0.0;
}

// EdgeMono/StereoOnlyPose::linearizeOplus: proj_jac * Rcb * SE3deriv(Xb)
void vis_jacobian(const VisEdge& e, const State& s, const Calib& c, double J[3][6]) {
  const V3 Xc = add(mv(s.Rcw, V3{{e.Xw[0], e.Xw[1], e.Xw[2]}}), s.tcw);
  const V3 Xb = add(mv(c.Rbc, Xc), c.tbc);
  double pj[3][3] = {{c.fx / Xc[2], 0, -c.fx * Xc[0] / (Xc[2] * Xc[2])},
                     {0, c.fy / Xc[2], -c.fy * Xc[1] / (Xc[2] * Xc[2])},
                     {0, 0, 0}};
  if (e.stereo) {
    for (int k = 0; k < 3; ++k) pj[2][k] = pj[0][k];
    pj[2][2] += c.bf * (1.0 / (Xc[2] * Xc[2]));
  }
  const double x = Xb[0], y = Xb[1], z = Xb[2];
  const double S[3][6] = {{0, z, -y, 1, 0, 0}, {-z, 0, x, 0, 1, 0}, {y, -x, 0, 0, 0, 1}};
  double PR[3][3];
  for (int r = 0; r < 3; ++r)
    for (int k = 0; k < 3; ++k) PR[r][k] = pj[r][0] * c.Rcb(0, k) + pj[r][1] * c.Rcb(1, k) + pj[r][2] * c.Rcb(2, k);
  for (int r = 0; r < 3; ++r)
    for (int k = 0; k < 6; ++k) J[r][k] = PR[r][0] * S[0][k] + PR[r][1] * S[1][k] + PR[r][2] * S[2][k];
}

struct Problem {
  int mode;  // 0 LastFrame, 1 LastKeyFrame
  Calib c;
  State cur, prev;
  Preint pi;
  double dt;
  V3 g;
  double info[81], info_g[9], info_a[9];
  // prior
  M3 pRwb;
  V3 ptwb, pvwb, pbg, pba;
  double pH[225];
  std::vector<VisEdge> E;
};

// Edge blocks in solver order: VP 0, VV 6, VG 9, VA 12 and, LastFrame only,
// VPk 15, VVk 21, VGk 24, VAk 27.
enum { kVP = 0, kVV = 6, kVG = 9, kVA = 12, kVPk = 15, kVVk = 21, kVGk = 24, kVAk = 27 };

int dim(const Problem& P) { return P.mode == 0 ? 30 : 15; }

void bias_f(const State& s, float bg[3], float ba[3]) {  // IMU::Bias from double estimates
  for (int i = 0; i < 3; ++i) {
    bg[i] = (float)s.bg[i];
    ba[i] = (float)s.ba[i];
  }
}

// EdgeInertial::computeError (g2o_types.cc:494-521)
void inertial_edge_error(const State& s1, const State& s2, const Preint& pi, double dt, const V3& g,
                         double e[9]) {
  float bg[3], ba[3];
  bias_f(s1, bg, ba);
  const M3 dR = delta_rotation(pi, bg);
  const V3 dV = delta_lin(pi.dV, pi.JVg, pi.JVa, pi, bg, ba);
  const V3 dP = delta_lin(pi.dP, pi.JPg, pi.JPa, pi, bg, ba);
  const M3 R1t = tr(s1.Rwb);
  const V3 er = LogSO3(mul(mul(tr(dR), R1t), s2.Rwb));
  const V3 ev = sub(mv(R1t, sub(sub(s2.v, s1.v), scl(g, dt))), dV);
  const V3 ep = sub(mv(R1t, sub(sub(sub(s2.twb, s1.twb), scl(s1.v, dt)), scl(g, dt * dt / 2))), dP);
  for (int i = 0; i < 3; ++i) {
    e[i] = er[i];
    e[3 + i] = ev[i];
    e[6 + i] = ep[i];
  }
}

// EdgeInertial::linearizeOplus (g2o_types.cc:523-578): J[9][24], columns in
// edge-vertex order VP1(6) VV1(3) VG1(3) VA1(3) VP2(6) VV2(3)
void inertial_edge_jacobian(const State& s1, const State& s2, const Preint& pi, double dt,
                            const V3& g, double J[9][24]) {
  float bg[3], ba[3];
  bias_f(s1, bg, ba);
  const V3 dbg{{(double)(bg[0] - pi.bg[0]), (double)(bg[1] - pi.bg[1]), (double)(bg[2] - pi.bg[2])}};
  const M3 Rwb1 = s1.Rwb, Rbw1 = tr(Rwb1), Rwb2 = s2.Rwb;
  const M3 dR = delta_rotation(pi, bg);
  const M3 eR = mul(mul(tr(dR), Rbw1), Rwb2);
  const V3 er = LogSO3(eR);
  const M3 invJr = InvRightJ(er);
  const M3 JRg = from_f(pi.JRg);
  std::memset(J, 0, sizeof(double) * 9 * 24);
  auto put = [&](int r0, int c0, const M3& m, double s) {
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) J[r0 + i][c0 + j] = s * m(i, j);
  };
  put(0, 0, mul(mul(invJr, tr(Rwb2)), Rwb1), -1.0);
  put(3, 0, hat(mv(Rbw1, sub(sub(s2.v, s1.v), scl(g, dt)))), 1.0);
  put(6, 0, hat(mv(Rbw1, sub(sub(sub(s2.twb, s1.twb), scl(s1.v, dt)), scl(g, 0.5 * dt * dt)))), 1.0);
  put(6, 3, eye(), -1.0);
  put(3, 6, Rbw1, -1.0);
  put(6, 6, Rbw1, -dt);
  put(0, 9, mul(mul(mul(invJr, tr(eR)), RightJ(mv(JRg, dbg))), JRg), -1.0);
  put(3, 9, from_f(pi.JVg), -1.0);
  put(6, 9, from_f(pi.JPg), -1.0);
  put(3, 12, from_f(pi.JVa), -1.0);
  put(6, 12, from_f(pi.JPa), -1.0);
  put(0, 15, invJr, 1.0);
  put(6, 18, mul(Rbw1, Rwb2), 1.0);
  put(3, 21, Rbw1, 1.0);
}

// the tracking problem's EdgeInertial: vertex set 1 = prev, 2 = cur
void inertial_error(const Problem& P, double e[9]) {
  inertial_edge_error(P.prev, P.cur, P.pi, P.dt, P.g, e);
}

void inertial_jacobian(const Problem& P, double J[9][24]) {
  inertial_edge_jacobian(P.prev, P.cur, P.pi, P.dt, P.g, J);
}

// EdgePriorPoseImu::computeError / linearizeOplus (g2o_types.cc:739-764) on
// the previous frame's vertices; J[15][15] columns VP(6) VV(3) VG(3) VA(3)
void prior_error(const Problem& P, double e[15]) {
  const State& s = P.prev;
  const V3 er = LogSO3(mul(tr(P.pRwb), s.Rwb));
  const V3 et = mv(tr(P.pRwb), sub(s.twb, P.ptwb));
  const V3 ev = sub(s.v, P.pvwb), ebg = sub(s.bg, P.pbg), eba = sub(s.ba, P.pba);
  for (int i = 0; i < 3; ++i) {
    e[i] = er[i];
    e[3 + i] = et[i];
    e[6 + i] = ev[i];
    e[9 + i] = ebg[i];
    e[12 + i] = eba[i];
  }
}

void prior_jacobian(const Problem& P, double J[15][15]) {
  const State& s = P.prev;
  const V3 er = LogSO3(mul(tr(P.pRwb), s.Rwb));
  const M3 A = InvRightJ(er), B = mul(tr(P.pRwb), s.Rwb);
  std::memset(J, 0, sizeof(double) * 15 * 15);
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      J[i][j] = A(i, j);
      J[3 + i][3 + j] = B(i, j);
    }
  for (int i = 0; i < 9; ++i) J[6 + i][6 + i] = 1.0;
}

// One edge's quadratic form into the n x n system (BaseMultiEdge::
// constructQuadraticForm with weight w = rho'(chi2), 1 without kernel).
// blocks: (solver offset or -1 for a fixed vertex, dim) in column order.
void add_quadratic(double* H, double* b, int n, int D, const double* J, int ldj, const double* Om,
                   const double* e, double w, const int (*blocks)[2], int nblk) {
  double Oe[15], OJ[15 * 24];
  for (int r = 0; r < D; ++r) {
    double s = 0;
    for (int q = 0; q < D; ++q) s += Om[r * D + q] * e[q];
    Oe[r] = -s * w;
  }
  for (int r = 0; r < D; ++r)
    for (int c = 0; c < ldj; ++c) {
      double s = 0;
      for (int q = 0; q < D; ++q) s += (w * Om[r * D + q]) * J[q * ldj + c];
      OJ[r * ldj + c] = s;
    }
  int col_i = 0;
  for (int i = 0; i < nblk; ++i) {
    const int oi = blocks[i][0], di = blocks[i][1];
    if (oi >= 0) {
      for (int a = 0; a < di; ++a) {
        double s = 0;
        for (int r = 0; r < D; ++r) s += J[r * ldj + col_i + a] * Oe[r];
        b[oi + a] += s;
      }
      int col_j = 0;
      for (int j = 0; j < nblk; ++j) {
        const int oj = blocks[j][0], dj = blocks[j][1];
        if (oj >= 0)
          for (int a = 0; a < di; ++a)
            for (int c = 0; c < dj; ++c) {
              double s = 0;
              for (int r = 0; r < D; ++r) s += J[r * ldj + col_i + a] * OJ[r * ldj + col_j + c];
              H[(oi + a) * n + oj + c] += s;
            }
        col_j += dj;
      }
    }
    col_i += di;
  }
}

double quad(const double* Om, const double* e, int D) {
  double s = 0;
  for (int r = 0; r < D; ++r) {
    double t = 0;
    for (int q = 0; q < D; ++q) t += Om[r * D + q] * e[q];
    s += e[r] * t;
  }
  return s;
}

// buildSystem over the active edges at the current state (errors computed
// first, as computeActiveErrors).  Returns nothing; H, b are n x n / n.
void build_system(Problem& P, double* H, double* b, bool include_kernels = true) {
  const int n = dim(P);
  const bool lf = P.mode == 0;
  std::fill(H, H + n * n, 0.0);
  std::fill(b, b + n, 0.0);
  const int vis_blk[1][2] = {{kVP, 6}};
  for (VisEdge& e : P.E) {
    if (e.level != 0) continue;
    vis_error(e, P.cur, P.c, e.err);
    double J[3][6];
    vis_jacobian(e, P.cur, P.c, J);
    const int D = e.stereo ? 3 : 2;
    double w = 1.0;
    if (e.robust && include_kernels) {
      double r0;
      huber(vis_chi2(e), e.delta, r0, w);
    }
    const double Om[9] = {e.info, 0, 0, 0, e.info, 0, 0, 0, e.info};
    double Om2[9], Jf[18];
    for (int r = 0; r < D; ++r)
      for (int q = 0; q < D; ++q) Om2[r * D + q] = Om[r * 3 + q];
    for (int r = 0; r < D; ++r)
      for (int k = 0; k < 6; ++k) Jf[r * 6 + k] = J[r][k];
    add_quadratic(H, b, n, D, Jf, 6, Om2, e.err, w, vis_blk, 1);
  }
  {  // EdgeInertial (no kernel)
    double e[9], J[9][24];
    inertial_error(P, e);
    inertial_jacobian(P, J);
    const int blk[6][2] = {{lf ? kVPk : -1, 6}, {lf ? kVVk : -1, 3}, {lf ? kVGk : -1, 3},
                           {lf ? kVAk : -1, 3}, {kVP, 6},           {kVV, 3}};
    add_quadratic(H, b, n, 9, &J[0][0], 24, P.info, e, 1.0, blk, 6);
  }
  for (int k = 0; k < 2; ++k) {  // EdgeGyroRW, EdgeAccRW
    const V3& x1 = k == 0 ? P.prev.bg : P.prev.ba;
    const V3& x2 = k == 0 ? P.cur.bg : P.cur.ba;
    const double e[3] = {x2[0] - x1[0], x2[1] - x1[1], x2[2] - x1[2]};
    double J[3 * 6] = {0};
    for (int i = 0; i < 3; ++i) {
      J[i * 6 + i] = -1.0;
      J[i * 6 + 3 + i] = 1.0;
    }
    const int blk[2][2] = {{lf ? (k == 0 ? kVGk : kVAk) : -1, 3}, {k == 0 ? kVG : kVA, 3}};
    add_quadratic(H, b, n, 3, J, 6, k == 0 ? P.info_g : P.info_a, e, 1.0, blk, 2);
  }
  if (lf) {  // EdgePriorPoseImu, Huber delta 5
    double e[15], J[15][15];
    prior_error(P, e);
    prior_jacobian(P, J);
    double w = 1.0;
    if (include_kernels) {
      double r0;
      huber(quad(P.pH, e, 15), 5.0, r0, w);
    }
    const int blk[4][2] = {{kVPk, 6}, {kVVk, 3}, {kVGk, 3}, {kVAk, 3}};
    add_quadratic(H, b, n, 15, &J[0][0], 15, P.pH, e, w, blk, 4);
  }
}

void apply_update(Problem& P, const double* x) {
  pose_update(P.cur, x + kVP, P.c);
  for (int i = 0; i < 3; ++i) {
    P.cur.v[i] += x[kVV + i];
    P.cur.bg[i] += x[kVG + i];
    P.cur.ba[i] += x[kVA + i];
  }
  if (P.mode == 0) {
    pose_update(P.prev, x + kVPk, P.c);
    for (int i = 0; i < 3; ++i) {
      P.prev.v[i] += x[kVVk + i];
      P.prev.bg[i] += x[kVGk + i];
      P.prev.ba[i] += x[kVAk + i];
    }
  }
}

// OptimizationAlgorithmGaussNewton::solve: errors, system, LDLT, update.
bool gn_iteration(Problem& P, std::vector<double>& x) {
  const int n = dim(P);
  std::vector<double> H(n * n), b(n), xs(n);
  build_system(P, H.data(), b.data());
  const bool ok = ldlt_solve(H.data(), n, b.data(), xs.data());
  if (ok) x = xs;
  apply_update(P, x.data());
  return ok;
}

// Symmetric pseudo-inverse with the 1e-6 cut (Marginalize's JacobiSVD).
void sym_pinv(const double* A_in, int m, double* out) {
  std::vector<double> A(A_in, A_in + m * m), V(m * m, 0.0);
  for (int i = 0; i < m; ++i) V[i * m + i] = 1.0;
  for (int sweep = 0; sweep < 60; ++sweep) {
    double off = 0, diag = 0;
    for (int i = 0; i < m; ++i) {
      diag += A[i * m + i] * A[i * m + i];
      for (int j = i + 1; j < m; ++j) off += A[i * m + j] * A[i * m + j];
    }
    if (off <= 1e-32 * diag) break;
    for (int p = 0; p < m; ++p)
      for (int q = p + 1; q < m; ++q) {
        const double apq = A[p * m + q];
        if (apq == 0.0) continue;
        const double theta = (A[q * m + q] - A[p * m + p]) / (2 * apq);
        const double t = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1));
        const double c = 1 / std::sqrt(t * t + 1), s = t * c;
        for (int k = 0; k < m; ++k) {  // A <- A G (columns p, q)
          const double akp = A[k * m + p], akq = A[k * m + q];
          A[k * m + p] = c * akp - s * akq;
          A[k * m + q] = s * akp + c * akq;
        }
        for (int k = 0; k < m; ++k) {  // A <- G^T A (rows p, q)
          const double apk = A[p * m + k], aqk = A[q * m + k];
          A[p * m + k] = c * apk - s * aqk;
          A[q * m + k] = s * apk + c * aqk;
        }
        for (int k = 0; k < m; ++k) {
          const double vkp = V[k * m + p], vkq = V[k * m + q];
          V[k * m + p] = c * vkp - s * vkq;
          V[k * m + q] = s * vkp + c * vkq;
        }
      }
  }
  std::fill(out, out + m * m, 0.0);
  for (int k = 0; k < m; ++k) {
    const double l = A[k * m + k];
    if (!(std::fabs(l) > 1e-6)) continue;
    for (int i = 0; i < m; ++i)
      for (int j = 0; j < m; ++j) out[i * m + j] += V[i * m + k] * V[j * m + k] / l;
  }
}

State load_state(const orbgpu_imu_state& s) {
  State o;
  o.Rwb = from_f(s.Rwb);
  o.twb = from_f3(s.twb);
  o.Rcw = from_f(s.Rcw);
  o.tcw = from_f3(s.tcw);
  o.v = from_f3(s.v);
  o.bg = from_f3(s.bg);
  o.ba = from_f3(s.ba);
  return o;
}

Calib load_calib(const orbgpu_imu_calib& cb) {
  Calib c;
  c.fx = cb.fx;
  c.fy = cb.fy;
  c.cx = cb.cx;
  c.cy = cb.cy;
  c.bf = cb.bf;
  c.Rcb = from_f(cb.Rcb);
  c.tcb = from_f3(cb.tcb);
  c.Rbc = from_f(cb.Rbc);
  c.tbc = from_f3(cb.tbc);
  return c;
}

void load_problem(Problem& P, int mode, const orbgpu_imu_calib& cb, const orbgpu_imu_state& cur,
                  const orbgpu_imu_state& prev, const orbgpu_imu_preint& pi,
                  const orbgpu_imu_prior* prior, const orbgpu_inertial_obs* obs, int n) {
  P.mode = mode;
  P.c = load_calib(cb);
  P.cur = load_state(cur);
  P.prev = load_state(prev);
  P.pi = preint_view(pi);
  P.dt = pi.dT;
  P.g = gravity();  // IMU::GRAVITY_VALUE (float)
  std::memcpy(P.info, pi.info, sizeof(P.info));
  std::memcpy(P.info_g, pi.info_g, sizeof(P.info_g));
  std::memcpy(P.info_a, pi.info_a, sizeof(P.info_a));
  if (mode == 0) {
    P.pRwb = from_d(prior->Rwb);
    P.ptwb = from_d3(prior->twb);
    P.pvwb = from_d3(prior->vwb);
    P.pbg = from_d3(prior->bg);
    P.pba = from_d3(prior->ba);
    std::memcpy(P.pH, prior->H, sizeof(P.pH));
  }
  const float dmono = std::sqrt(5.991), dstereo = std::sqrt(7.815);
  P.E.resize(n);
  for (int i = 0; i < n; ++i) {
    VisEdge& e = P.E[i];
    for (int k = 0; k < 3; ++k) e.Xw[k] = obs[i].Xw[k];
    e.stereo = obs[i].ur >= 0.f;
    e.obs[0] = obs[i].u;
    e.obs[1] = obs[i].v;
    e.obs[2] = e.stereo ? obs[i].ur : 0.0;
    e.close = obs[i].close != 0;
    e.info = obs[i].inv_sigma2;
    e.delta = e.stereo ? dstereo : dmono;
  }
}

int optimize(int mode, const orbgpu_imu_calib& cb, const orbgpu_imu_state& cur,
             const orbgpu_imu_state& prev, const orbgpu_imu_preint& pi,
             const orbgpu_imu_prior* prior, const orbgpu_inertial_obs* obs, int n, bool rec_init,
             orbgpu_inertial_result& res, uint8_t* outlier, double* prev_out = nullptr) {
  Problem P;
  load_problem(P, mode, cb, cur, prev, pi, prior, obs, n);
  const int dn = dim(P);
  const float chi2MonoLF[4] = {5.991f, 5.991f, 5.991f, 5.991f};
  const float chi2MonoKF[4] = {12.f, 7.5f, 5.991f, 5.991f};
  const float* chi2Mono = mode == 0 ? chi2MonoLF : chi2MonoKF;
  const float chi2Stereo[4] = {15.6f, 9.8f, 7.815f, 7.815f};
  std::vector<double> x(dn, 0.0);
  std::vector<uint8_t> out(n, 0);
  int nBad = 0, nInliers = 0;
  const int n_edges = n + (mode == 0 ? 4 : 3);
  for (int it = 0; it < 4; ++it) {
    for (int k = 0; k < 10; ++k)
      if (!gn_iteration(P, x)) break;
    nBad = 0;
    nInliers = 0;
    const float chi2close = 1.5 * chi2Mono[it];
    for (int i = 0; i < n; ++i) {
      VisEdge& e = P.E[i];
      if (out[i]) vis_error(e, P.cur, P.c, e.err);
      const float chi2 = (float)vis_chi2(e);
      bool bad;
      if (!e.stereo)
        bad = (chi2 > chi2Mono[it] && !e.close) || (e.close && chi2 > chi2close) ||
              !vis_depth_positive(e, P.cur);
      else
        bad = chi2 > chi2Stereo[it];
      out[i] = bad;
      e.level = bad ? 1 : 0;
      if (bad)
        ++nBad;
      else
        ++nInliers;
      if (it == 2) e.robust = false;
    }
    if (n_edges < 10) break;
  }
  if (nInliers < 30 && !rec_init) {
    nBad = 0;
    for (int i = 0; i < n; ++i) {
      VisEdge& e = P.E[i];
      vis_error(e, P.cur, P.c, e.err);
      if ((float)vis_chi2(e) < (e.stereo ? 24.f : 18.f))
        out[i] = 0;
      else
        ++nBad;
    }
  }
  int nInitial = n;
  res.n_good = nInitial - nBad;
  res.n_inliers = nInliers;
  for (int i = 0; i < 9; ++i) {
    res.Rwb[i] = (float)P.cur.Rwb.a[i];
    res.Rwb_d[i] = P.cur.Rwb.a[i];
  }
  for (int i = 0; i < 3; ++i) {
    res.twb[i] = (float)P.cur.twb[i];
    res.v[i] = (float)P.cur.v[i];
    res.bg[i] = (float)P.cur.bg[i];
    res.ba[i] = (float)P.cur.ba[i];
    res.twb_d[i] = P.cur.twb[i];
    res.v_d[i] = P.cur.v[i];
    res.bg_d[i] = P.cur.bg[i];
    res.ba_d[i] = P.cur.ba[i];
  }
  for (int i = 0; i < n; ++i) outlier[i] = out[i];
  if (prev_out) {
    for (int i = 0; i < 9; ++i) prev_out[i] = P.prev.Rwb.a[i];
    for (int i = 0; i < 3; ++i) {
      prev_out[9 + i] = P.prev.twb[i];
      prev_out[12 + i] = P.prev.v[i];
      prev_out[15 + i] = P.prev.bg[i];
      prev_out[18 + i] = P.prev.ba[i];
    }
  }

  // the Hessian handed to the new ConstraintPoseImu
  double Hv[36] = {0};
  for (int i = 0; i < n; ++i) {
    if (out[i]) continue;
    const VisEdge& e = P.E[i];
    double J[3][6];
    vis_jacobian(e, P.cur, P.c, J);
    const int D = e.stereo ? 3 : 2;
    for (int a = 0; a < 6; ++a)
      for (int c = 0; c < 6; ++c) {
        double s = 0;
        for (int r = 0; r < D; ++r) s += J[r][a] * (e.info * J[r][c]);
        Hv[a * 6 + c] += s;
      }
  }
  double J[9][24];
  inertial_jacobian(P, J);
  double Hi[24 * 24];
  for (int a = 0; a < 24; ++a)
    for (int c = 0; c < 24; ++c) {
      double s = 0;
      for (int r = 0; r < 9; ++r) {
        double t = 0;
        for (int q = 0; q < 9; ++q) t += P.info[r * 9 + q] * J[q][c];
        s += J[r][a] * t;
      }
      Hi[a * 24 + c] = s;
    }
  if (mode == 0) {
    double H[30 * 30] = {0};
    for (int a = 0; a < 24; ++a)
      for (int c = 0; c < 24; ++c) H[a * 30 + c] += Hi[a * 24 + c];
    const int og[2] = {9, 24}, oa[2] = {12, 27};
    for (int k = 0; k < 2; ++k) {
      const double* Om = k == 0 ? P.info_g : P.info_a;
      const int* o = k == 0 ? og : oa;
      for (int p = 0; p < 2; ++p)
        for (int q = 0; q < 2; ++q) {
          const double sg = p == q ? 1.0 : -1.0;  // J = [-I, I]
          for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) H[(o[p] + i) * 30 + o[q] + j] += sg * Om[i * 3 + j];
        }
    }
    double Jp[15][15];
    prior_jacobian(P, Jp);
    for (int a = 0; a < 15; ++a)
      for (int c = 0; c < 15; ++c) {
        double s = 0;
        for (int r = 0; r < 15; ++r) {
          double t = 0;
          for (int q = 0; q < 15; ++q) t += P.pH[r * 15 + q] * Jp[q][c];
          s += Jp[r][a] * t;
        }
        H[a * 30 + c] += s;
      }
    for (int a = 0; a < 6; ++a)
      for (int c = 0; c < 6; ++c) H[(15 + a) * 30 + 15 + c] += Hv[a * 6 + c];
    // Marginalize(H, 0, 14): Hcc - Hcb pinv(Hbb) Hbc, b = 0..14, c = 15..29
    double Hbb[225], Pb[225], T[225];
    for (int i = 0; i < 15; ++i)
      for (int j = 0; j < 15; ++j) Hbb[i * 15 + j] = H[i * 30 + j];
    sym_pinv(Hbb, 15, Pb);
    for (int i = 0; i < 15; ++i)  // T = Hcb pinv
      for (int j = 0; j < 15; ++j) {
        double s = 0;
        for (int k = 0; k < 15; ++k) s += H[(15 + i) * 30 + k] * Pb[k * 15 + j];
        T[i * 15 + j] = s;
      }
    for (int i = 0; i < 15; ++i)
      for (int j = 0; j < 15; ++j) {
        double s = 0;
        for (int k = 0; k < 15; ++k) s += T[i * 15 + k] * H[k * 30 + 15 + j];
        res.H[i * 15 + j] = H[(15 + i) * 30 + 15 + j] - s;
      }
  } else {
    double* H = res.H;
    std::fill(H, H + 225, 0.0);
    for (int a = 0; a < 9; ++a)  // GetHessian2: the (VP2, VV2) block
      for (int c = 0; c < 9; ++c) H[a * 15 + c] += Hi[(15 + a) * 24 + 15 + c];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        H[(9 + i) * 15 + 9 + j] += P.info_g[i * 3 + j];
        H[(12 + i) * 15 + 12 + j] += P.info_a[i * 3 + j];
      }
    for (int a = 0; a < 6; ++a)
      for (int c = 0; c < 6; ++c) H[a * 15 + c] += Hv[a * 6 + c];
  }
  return res.n_good;
}

}  // namespace inertial
}  // namespace oracle

using namespace oracle::inertial;

extern "C" int orc_pose_inertial(int mode, const orbgpu_imu_calib* calib, const orbgpu_imu_state* cur,
                                 const orbgpu_imu_state* prev, const orbgpu_imu_preint* preint,
                                 const orbgpu_imu_prior* prior, const orbgpu_inertial_obs* obs, int n,
                                 int rec_init, orbgpu_inertial_result* res, uint8_t* outlier) {
  return optimize(mode, *calib, *cur, *prev, *preint, prior, obs, n, rec_init != 0, *res, outlier);
}

// Test hook: as orc_pose_inertial, plus the previous frame's final double
// state [Rwb(9) twb v bg ba] (LastFrame optimises it too).
extern "C" int orc_pose_inertial_ex(int mode, const orbgpu_imu_calib* calib,
                                    const orbgpu_imu_state* cur, const orbgpu_imu_state* prev,
                                    const orbgpu_imu_preint* preint, const orbgpu_imu_prior* prior,
                                    const orbgpu_inertial_obs* obs, int n, int rec_init,
                                    orbgpu_inertial_result* res, uint8_t* outlier, double* prev_out) {
  return optimize(mode, *calib, *cur, *prev, *preint, prior, obs, n, rec_init != 0, *res, outlier,
                  prev_out);
}

// Test hook: the Gauss-Newton system (H n x n, b n) at given double states
// (Rwb[9] twb[3] v[3] bg[3] ba[3] per frame; the camera pose follows from
// Rwb/twb as after an Update), all visual edges active, kernels on or off.
extern "C" void orc_inertial_system(int mode, const orbgpu_imu_calib* calib, const double* cur,
                                    const double* prev, const orbgpu_imu_preint* preint,
                                    const orbgpu_imu_prior* prior, const orbgpu_inertial_obs* obs,
                                    int n, int kernels, double* H, double* b) {
  orbgpu_imu_state dummy{};
  Problem P;
  load_problem(P, mode, *calib, dummy, dummy, *preint, prior, obs, n);
  auto set = [&](State& s, const double* d) {
    s.Rwb = from_d(d);
    s.twb = from_d3(d + 9);
    s.v = from_d3(d + 12);
    s.bg = from_d3(d + 15);
    s.ba = from_d3(d + 18);
    const M3 Rbw = tr(s.Rwb);
    const V3 tbw = scl(mv(Rbw, s.twb), -1.0);
    s.Rcw = mul(P.c.Rcb, Rbw);
    s.tcw = add(mv(P.c.Rcb, tbw), P.c.tcb);
  };
  set(P.cur, cur);
  set(P.prev, prev);
  build_system(P, H, b, kernels != 0);
}

// Test hook: the pseudo-inverse Marginalize applies.
extern "C" void orc_sym_pinv(const double* A, int m, double* out) { sym_pinv(A, m, out); }
