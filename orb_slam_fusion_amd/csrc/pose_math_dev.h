// Device restatement of the g2o / Eigen dense pieces PoseOptimization runs
// through (double precision, as g2o):
//   SE3Quat map / exp / operator*   3rdparty/g2o/g2o/types/se3quat.h:99-105,201-255
//   Quaterniond(Matrix3d)           Eigen quaternionbase_assign_impl
//   Eigen::LDLT (pivot on the not-yet-updated diagonal, lower triangle only),
//                                   used by LinearSolverDense (linear_solver_dense.h:56-104)
//   RobustKernelHuber::robustify    core/robust_kernel_impl.cpp:72-85
#pragma once
#include <hip/hip_runtime.h>

namespace orbgpu {

struct Se3 {  // POD (lives in LDS); unit quaternion (x, y, z, w) + translation
  double qx, qy, qz, qw;
  double t[3];
};

__device__ __forceinline__ void quat_rot(double qx, double qy, double qz, double qw,
                                         const double v[3], double o[3]) {
  double u0 = qy * v[2] - qz * v[1], u1 = qz * v[0] - qx * v[2], u2 = qx * v[1] - qy * v[0];
  u0 += u0;
  u1 += u1;
  u2 += u2;
  const double c0 = qy * u2 - qz * u1, c1 = qz * u0 - qx * u2, c2 = qx * u1 - qy * u0;
  o[0] = v[0] + qw * u0 + c0;
  o[1] = v[1] + qw * u1 + c1;
  o[2] = v[2] + qw * u2 + c2;
}

__device__ __forceinline__ void se3_map(const Se3& T, const double p[3], double o[3]) {
  quat_rot(T.qx, T.qy, T.qz, T.qw, p, o);
  o[0] += T.t[0];
  o[1] += T.t[1];
  o[2] += T.t[2];
}

__device__ __forceinline__ void se3_normalize(Se3& T) {
  if (T.qw < 0) {
    T.qw = -T.qw;
    T.qx = -T.qx;
    T.qy = -T.qy;
    T.qz = -T.qz;
  }
  const double n = sqrt(T.qx * T.qx + T.qy * T.qy + T.qz * T.qz + T.qw * T.qw);
  T.qw /= n;
  T.qx /= n;
  T.qy /= n;
  T.qz /= n;
}

// a * b
__device__ __forceinline__ Se3 se3_compose(const Se3& a, const Se3& b) {
  Se3 r = a;
  double rt[3];
  quat_rot(a.qx, a.qy, a.qz, a.qw, b.t, rt);
  r.t[0] += rt[0];
  r.t[1] += rt[1];
  r.t[2] += rt[2];
  r.qw = a.qw * b.qw - a.qx * b.qx - a.qy * b.qy - a.qz * b.qz;
  r.qx = a.qw * b.qx + a.qx * b.qw + a.qy * b.qz - a.qz * b.qy;
  r.qy = a.qw * b.qy + a.qy * b.qw + a.qz * b.qx - a.qx * b.qz;
  r.qz = a.qw * b.qz + a.qz * b.qw + a.qx * b.qy - a.qy * b.qx;
  se3_normalize(r);
  return r;
}

__device__ __forceinline__ Se3 se3_exp(const double u[6]) {
  const double w0 = u[0], w1 = u[1], w2 = u[2];
  const double theta = sqrt(w0 * w0 + w1 * w1 + w2 * w2);
  const double O[3][3] = {{0, -w2, w1}, {w2, 0, -w0}, {-w1, w0, 0}};
  double O2[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) O2[i][j] = O[i][0] * O[0][j] + O[i][1] * O[1][j] + O[i][2] * O[2][j];
  double R[3][3], V[3][3];
  if (theta < 0.00001) {
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) R[i][j] = V[i][j] = (i == j ? 1.0 : 0.0) + O[i][j] + O2[i][j];
  } else {
    const double s = sin(theta), c = cos(theta);
    const double a = s / theta, b = (1 - c) / (theta * theta), d = (theta - s) / pow(theta, 3);
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        const double I = i == j ? 1.0 : 0.0;
        R[i][j] = I + a * O[i][j] + b * O2[i][j];
        V[i][j] = I + b * O[i][j] + d * O2[i][j];
      }
  }
  Se3 e{0, 0, 0, 1, {0, 0, 0}};
  double t = R[0][0] + R[1][1] + R[2][2];
  if (t > 0) {
    t = sqrt(t + 1.0);
    e.qw = 0.5 * t;
    t = 0.5 / t;
    e.qx = (R[2][1] - R[1][2]) * t;
    e.qy = (R[0][2] - R[2][0]) * t;
    e.qz = (R[1][0] - R[0][1]) * t;
  } else {
    int i = 0;
    if (R[1][1] > R[0][0]) i = 1;
    if (R[2][2] > R[i][i]) i = 2;
    const int j = (i + 1) % 3, k = (j + 1) % 3;
    double c[3];
    t = sqrt(R[i][i] - R[j][j] - R[k][k] + 1.0);
    c[i] = 0.5 * t;
    t = 0.5 / t;
    e.qw = (R[k][j] - R[j][k]) * t;
    c[j] = (R[j][i] + R[i][j]) * t;
    c[k] = (R[k][i] + R[i][k]) * t;
    e.qx = c[0];
    e.qy = c[1];
    e.qz = c[2];
  }
  for (int i = 0; i < 3; ++i) e.t[i] = V[i][0] * u[3] + V[i][1] * u[4] + V[i][2] * u[5];
  se3_normalize(e);
  return e;
}

// Eigen::LDLT of the 6x6 row-major A (lower triangle read), solve A x = b.
// Returns isPositive() (no negative pivot).
__device__ __forceinline__ bool ldlt6_solve(double* A, const double* b, double* x) {
  constexpr int n = 6;
  int perm[n];
  double temp[n];
  bool neg = false;
  for (int k = 0; k < n; ++k) {
    int p = k;
    double big = fabs(A[k * n + k]);
    for (int i = k + 1; i < n; ++i)
      if (fabs(A[i * n + i]) > big) big = fabs(A[i * n + i]), p = i;
    perm[k] = p;
    if (p != k) {
      for (int j = 0; j < k; ++j) {
        const double s = A[k * n + j];
        A[k * n + j] = A[p * n + j];
        A[p * n + j] = s;
      }
      for (int i = p + 1; i < n; ++i) {
        const double s = A[i * n + k];
        A[i * n + k] = A[i * n + p];
        A[i * n + p] = s;
      }
      const double s = A[k * n + k];
      A[k * n + k] = A[p * n + p];
      A[p * n + p] = s;
      for (int i = k + 1; i < p; ++i) {
        const double s2 = A[i * n + k];
        A[i * n + k] = A[p * n + i];
        A[p * n + i] = s2;
      }
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
    if (fabs(akk) > 0)
      for (int i = k + 1; i < n; ++i) A[i * n + k] /= akk;
    if (akk < 0) neg = true;
  }
  for (int i = 0; i < n; ++i) x[i] = b[i];
  for (int k = 0; k < n; ++k) {
    const double s = x[k];
    x[k] = x[perm[k]];
    x[perm[k]] = s;
  }
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < i; ++j) x[i] -= A[i * n + j] * x[j];
  for (int i = 0; i < n; ++i) {
    const double d = A[i * n + i];
    x[i] = fabs(d) > 1.0 / 1.79769313486231570815e+308 ? x[i] / d : 0.0;
  }
  for (int i = n - 1; i >= 0; --i)
    for (int j = i + 1; j < n; ++j) x[i] -= A[j * n + i] * x[j];
  for (int k = n - 1; k >= 0; --k) {
    const double s = x[k];
    x[k] = x[perm[k]];
    x[perm[k]] = s;
  }
  return !neg;
}

__device__ __forceinline__ void huber_rho(double e2, double delta, double& rho0, double& rho1) {
  const double dsqr = delta * delta;
  if (e2 <= dsqr) {
    rho0 = e2;
    rho1 = 1.0;
  } else {
    const double s = sqrt(e2);
    rho0 = 2 * s * delta - dsqr;
    rho1 = delta / s;
  }
}

}  // namespace orbgpu
