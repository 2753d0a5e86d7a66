// ORACLE (test infrastructure only): the small dense pieces of g2o / Eigen that
// PoseOptimization and LocalBundleAdjustment run through, restated in plain
// C++ (Eigen is absent here).  Double precision throughout, as g2o.
//   SE3Quat map / exp / compose      3rdparty/g2o/g2o/types/se3quat.h:99-105,201-255
//   Quaternion from rotation matrix  Eigen QuaternionBase::operator=(Matrix3)
//   Eigen::LDLT (diagonal pivoting)  used by LinearSolverDense (linear_solver_dense.h:56-104)
//   RobustKernelHuber                core/robust_kernel_impl.cpp:61-85
#pragma once
#include <cmath>
#include <cstring>

namespace oracle {

struct Quat {
  double w = 1, x = 0, y = 0, z = 0;
};

// Eigen's q * v (QuaternionBase::_transformVector).
static inline void quat_rotate(const Quat& q, const double v[3], double out[3]) {
  double uv[3] = {q.y * v[2] - q.z * v[1], q.z * v[0] - q.x * v[2], q.x * v[1] - q.y * v[0]};
  uv[0] += uv[0];
  uv[1] += uv[1];
  uv[2] += uv[2];
  const double c[3] = {q.y * uv[2] - q.z * uv[1], q.z * uv[0] - q.x * uv[2],
                       q.x * uv[1] - q.y * uv[0]};
  for (int i = 0; i < 3; ++i) out[i] = v[i] + q.w * uv[i] + c[i];
}

static inline Quat quat_mul(const Quat& a, const Quat& b) {
  Quat r;
  r.w = a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z;
  r.x = a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y;
  r.y = a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z;
  r.z = a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x;
  return r;
}

static inline Quat quat_from_matrix(const double m[3][3]) {
  Quat q;
  double t = m[0][0] + m[1][1] + m[2][2];
  if (t > 0) {
    t = std::sqrt(t + 1.0);
    q.w = 0.5 * t;
    t = 0.5 / t;
    q.x = (m[2][1] - m[1][2]) * t;
    q.y = (m[0][2] - m[2][0]) * t;
    q.z = (m[1][0] - m[0][1]) * t;
  } else {
    int i = 0;
    if (m[1][1] > m[0][0]) i = 1;
    if (m[2][2] > m[i][i]) i = 2;
    const int j = (i + 1) % 3, k = (j + 1) % 3;
    double c[3];
    t = std::sqrt(m[i][i] - m[j][j] - m[k][k] + 1.0);
    c[i] = 0.5 * t;
    t = 0.5 / t;
    q.w = (m[k][j] - m[j][k]) * t;
    c[j] = (m[j][i] + m[i][j]) * t;
    c[k] = (m[k][i] + m[i][k]) * t;
    q.x = c[0];
    q.y = c[1];
    q.z = c[2];
  }
  return q;
}

struct SE3 {
  Quat r;
  double t[3] = {0, 0, 0};

  void map(const double p[3], double out[3]) const {
    quat_rotate(r, p, out);
    out[0] += t[0];
    out[1] += t[1];
    out[2] += t[2];
  }
  // SE3Quat::normalizeRotation: w >= 0, unit norm.
  void normalize() {
    if (r.w < 0) {
      r.w = -r.w;
      r.x = -r.x;
      r.y = -r.y;
      r.z = -r.z;
    }
    const double n = std::sqrt(r.x * r.x + r.y * r.y + r.z * r.z + r.w * r.w);
    r.w /= n;
    r.x /= n;
    r.y /= n;
    r.z /= n;
  }
  // this * o  (se3quat.h:99-105).
  SE3 compose(const SE3& o) const {
    SE3 res = *this;
    double rt[3];
    quat_rotate(r, o.t, rt);
    res.t[0] += rt[0];
    res.t[1] += rt[1];
    res.t[2] += rt[2];
    res.r = quat_mul(r, o.r);
    res.normalize();
    return res;
  }
};

// SE3Quat::exp of [omega; upsilon] (se3quat.h:203-229), including the
// small-angle branch R = I + Omega + Omega^2.
static inline SE3 se3_exp(const double u[6]) {
  const double w0 = u[0], w1 = u[1], w2 = u[2];
  const double theta = std::sqrt(w0 * w0 + w1 * w1 + w2 * w2);
  const double O[3][3] = {{0, -w2, w1}, {w2, 0, -w0}, {-w1, w0, 0}};
  double O2[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) O2[i][j] = O[i][0] * O[0][j] + O[i][1] * O[1][j] + O[i][2] * O[2][j];
  double R[3][3], V[3][3];
  if (theta < 0.00001) {
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) R[i][j] = V[i][j] = (i == j ? 1.0 : 0.0) + O[i][j] + O2[i][j];
  } else {
    const double s = std::sin(theta), c = std::cos(theta);
    const double a = s / theta, b = (1 - c) / (theta * theta);
    const double d = (theta - s) / std::pow(theta, 3);
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        const double I = i == j ? 1.0 : 0.0;
        R[i][j] = I + a * O[i][j] + b * O2[i][j];
        V[i][j] = I + b * O[i][j] + d * O2[i][j];
      }
  }
  SE3 e;
  e.r = quat_from_matrix(R);
  for (int i = 0; i < 3; ++i) e.t[i] = V[i][0] * u[3] + V[i][1] * u[4] + V[i][2] * u[5];
  e.normalize();
  return e;
}

// Eigen::LDLT<MatrixXd> (lower, diagonal pivoting on the not-yet-updated
// diagonal) of the n x n row-major matrix A, then solve A x = b.  Returns
// Eigen's isPositive(): no negative pivot.
static inline bool ldlt_solve(double* A, int n, const double* b, double* x) {
  int perm[64];
  bool neg = false;
  double temp[64];
  for (int k = 0; k < n; ++k) {
    int p = k;
    double big = std::fabs(A[k * n + k]);
    for (int i = k + 1; i < n; ++i)
      if (std::fabs(A[i * n + i]) > big) big = std::fabs(A[i * n + i]), p = i;
    perm[k] = p;
    if (p != k) {  // symmetric transposition touching the lower triangle only
      for (int j = 0; j < k; ++j) std::swap(A[k * n + j], A[p * n + j]);
      for (int i = p + 1; i < n; ++i) std::swap(A[i * n + k], A[i * n + p]);
      std::swap(A[k * n + k], A[p * n + p]);
      for (int i = k + 1; i < p; ++i) std::swap(A[i * n + k], A[p * n + i]);
    }
    if (k > 0) {
      double acc = 0;
      for (int j = 0; j < k; ++j) {
        temp[j] = A[j * n + j] * A[k * n + j];
        acc += A[k * n + j] * temp[j];
      }
      A[k * n + k] -= acc;
      for (int i = k + 1; i < n; ++i) {
        double s = 0;
        for (int j = 0; j < k; ++j) s += A[i * n + j] * temp[j];
        A[i * n + k] -= s;
      }
    }
    const double akk = A[k * n + k];
    if (std::fabs(akk) > 0)
      for (int i = k + 1; i < n; ++i) A[i * n + k] /= akk;
    if (akk < 0) neg = true;
  }
  for (int i = 0; i < n; ++i) x[i] = b[i];
  for (int k = 0; k < n; ++k) std::swap(x[k], x[perm[k]]);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < i; ++j) x[i] -= A[i * n + j] * x[j];
  for (int i = 0; i < n; ++i) {
    const double d = A[i * n + i];
    x[i] = std::fabs(d) > 1.0 / 1.79769313486231570815e+308 ? x[i] / d : 0.0;
  }
  for (int i = n - 1; i >= 0; --i)
    for (int j = i + 1; j < n; ++j) x[i] -= A[j * n + i] * x[j];
  for (int k = n - 1; k >= 0; --k) std::swap(x[k], x[perm[k]]);
  return !neg;
}

// RobustKernelHuber::robustify -> (rho0, rho1).
static inline void huber(double e2, double delta, double& rho0, double& rho1) {
  const double dsqr = delta * delta;
  if (e2 <= dsqr) {
    rho0 = e2;
    rho1 = 1.0;
  } else {
    const double s = std::sqrt(e2);
    rho0 = 2 * s * delta - dsqr;
    rho1 = delta / s;
  }
}

}  // namespace oracle
