// Device restatement of the g2o / Eigen dense pieces PoseOptimization runs
// through (double precision, as g2o):
//   SE3Quat map / exp / operator*   3rdparty/g2o/g2o/types/se3quat.h:99-105,201-255
//   Quaterniond(Matrix3d)           Eigen quaternionbase_assign_impl
//   Eigen::LDLT (pivot on the not-yet-updated diagonal, lower triangle only),
//                                   used by LinearSolverDense (linear_solver_dense.h:56-104)
//   RobustKernelHuber::robustify    core/robust_kernel_impl.cpp:72-85
#pragma once
#include "f64_math_dev.h"
#include "uniform_dev.h"
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
  // |q| ~ 1: the IEEE sqrt and quotients by f64_math_dev.h (one reciprocal)
  const RecipF64 n = recip_f64(sqrt_f64(T.qx * T.qx + T.qy * T.qy + T.qz * T.qz + T.qw * T.qw));
  T.qw = div_by(T.qw, n);
  T.qx = div_by(T.qx, n);
  T.qy = div_by(T.qy, n);
  T.qz = div_by(T.qz, n);
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

// x^3 as std::pow(x, 3) returns it (correctly rounded but for double-double
// ties): the compensated product x*x*x, five instructions instead of the
// ocml pow routine.
__device__ __forceinline__ double cube(double x) {
  const double p = x * x, ep = fma(x, x, -p);
  const double c = p * x, ec = fma(p, x, -c);
  return c + fma(ep, x, ec);
}

// kUniform: every lane of the wave evaluates the same exp (PoseOptimization),
// so the branches are made wave-uniform with readfirstlane; otherwise each
// lane takes its own branch (LocalBundleAdjustment, one pose per lane).
template <bool kUniform = true>
__device__ __forceinline__ Se3 se3_exp(const double u[6]) {
  const double w0 = u[0], w1 = u[1], w2 = u[2];
  const double theta = sqrt(w0 * w0 + w1 * w1 + w2 * w2);
  const double O[3][3] = {{0, -w2, w1}, {w2, 0, -w0}, {-w1, w0, 0}};
  double O2[3][3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) O2[i][j] = O[i][0] * O[0][j] + O[i][1] * O[1][j] + O[i][2] * O[2][j];
  double R[3][3], V[3][3];
  // all lanes evaluate the same exp: wave-uniform branches (scalar, no exec masking)
  const int small = theta < 0.00001 ? 1 : 0;
  if (kUniform ? uniform_branch(small) : small) {
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) R[i][j] = V[i][j] = (i == j ? 1.0 : 0.0) + O[i][j] + O2[i][j];
  } else {
    // a = sin t / t, b = (1 - cos t) / t^2, d = (t - sin t) / t^3 (se3quat.h:210-217).
    // Below t = 0.25 (every LM step but the first few) as their Taylor series
    // in t^2 to the last term above 1e-19 (Horner, no sin / cos / divisions;
    // the series are at least as accurate as the closed forms, which lose
    // digits to cancellation there), else the closed forms.
    const double t2 = w0 * w0 + w1 * w1 + w2 * w2;
    const int series = t2 < 0.0625 ? 1 : 0;
    double a, b, d;
    if (kUniform ? uniform_branch(series) : series) {
      // 1/(2k+1)!, 1/(2k+2)!, 1/(2k+3)! with alternating signs, k = 0..7
      a = fma(t2, fma(t2, fma(t2, fma(t2, fma(t2, fma(t2, fma(t2, -7.6471637318198164759e-13,
          1.6059043836821614599e-10), -2.5052108385441718775e-08), 2.7557319223985890653e-06),
          -1.9841269841269841270e-04), 8.3333333333333333333e-03), -1.6666666666666666667e-01), 1.0);
      b = fma(t2, fma(t2, fma(t2, fma(t2, fma(t2, fma(t2, fma(t2, -4.7794773323873852974e-14,
          1.1470745597729724714e-11), -2.0876756987868098979e-09), 2.7557319223985890653e-07),
          -2.4801587301587301587e-05), 1.3888888888888888889e-03), -4.1666666666666666667e-02), 0.5);
      d = fma(t2, fma(t2, fma(t2, fma(t2, fma(t2, fma(t2, fma(t2, -2.8114572543455207632e-15,
          7.6471637318198164759e-13), -1.6059043836821614599e-10), 2.5052108385441718775e-08),
          -2.7557319223985890653e-06), 1.9841269841269841270e-04), -8.3333333333333333333e-03),
          1.6666666666666666667e-01);
    } else {
      const double s = sin(theta), c = cos(theta);
      a = s / theta;
      b = (1 - c) / (theta * theta);
      d = (theta - s) / cube(theta);
    }
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const double I = i == j ? 1.0 : 0.0;
        R[i][j] = I + a * O[i][j] + b * O2[i][j];
        V[i][j] = I + b * O[i][j] + d * O2[i][j];
      }
  }
  Se3 e{0, 0, 0, 1, {0, 0, 0}};
  // Eigen quaternionbase_assign_impl, the three pivot cases written out
  double t = R[0][0] + R[1][1] + R[2][2];
  const int qc = t > 0 ? 0 : R[2][2] > (R[1][1] > R[0][0] ? R[1][1] : R[0][0]) ? 1 : R[1][1] > R[0][0] ? 2 : 3;
  const int qcase = kUniform ? uniform_branch(qc) : qc;
  if (qcase == 0) {
    t = sqrt_f64(t + 1.0);  // the chosen pivot's argument is >= 1
    e.qw = 0.5 * t;
    t = div_by(0.5, recip_f64(t));
    e.qx = (R[2][1] - R[1][2]) * t;
    e.qy = (R[0][2] - R[2][0]) * t;
    e.qz = (R[1][0] - R[0][1]) * t;
  } else if (qcase == 1) {  // i = 2, j = 0, k = 1
    t = sqrt_f64(R[2][2] - R[0][0] - R[1][1] + 1.0);
    e.qz = 0.5 * t;
    t = div_by(0.5, recip_f64(t));
    e.qw = (R[1][0] - R[0][1]) * t;
    e.qx = (R[0][2] + R[2][0]) * t;
    e.qy = (R[1][2] + R[2][1]) * t;
  } else if (qcase == 2) {  // i = 1, j = 2, k = 0
    t = sqrt_f64(R[1][1] - R[2][2] - R[0][0] + 1.0);
    e.qy = 0.5 * t;
    t = div_by(0.5, recip_f64(t));
    e.qw = (R[0][2] - R[2][0]) * t;
    e.qz = (R[2][1] + R[1][2]) * t;
    e.qx = (R[0][1] + R[1][0]) * t;
  } else {  // i = 0, j = 1, k = 2
    t = sqrt_f64(R[0][0] - R[1][1] - R[2][2] + 1.0);
    e.qx = 0.5 * t;
    t = div_by(0.5, recip_f64(t));
    e.qw = (R[2][1] - R[1][2]) * t;
    e.qy = (R[1][0] + R[0][1]) * t;
    e.qz = (R[2][0] + R[0][2]) * t;
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) e.t[i] = V[i][0] * u[3] + V[i][1] * u[4] + V[i][2] * u[5];
  se3_normalize(e);
  return e;
}

// Symmetric transposition k <-> p (p > k) touching the lower triangle only,
// as Eigen's LDLT does.  K and Pp are compile-time after unrolling.
__device__ __forceinline__ void ldlt_swap(double (&A)[6][6], int k, int pp) {
#pragma unroll
  for (int j = 0; j < 6; ++j)
    if (j < k) {
      const double s = A[k][j];
      A[k][j] = A[pp][j];
      A[pp][j] = s;
    }
#pragma unroll
  for (int i = 0; i < 6; ++i)
    if (i > pp) {
      const double s = A[i][k];
      A[i][k] = A[i][pp];
      A[i][pp] = s;
    }
  {
    const double s = A[k][k];
    A[k][k] = A[pp][pp];
    A[pp][pp] = s;
  }
#pragma unroll
  for (int i = 0; i < 6; ++i)
    if (i > k && i < pp) {
      const double s = A[i][k];
      A[i][k] = A[pp][i];
      A[pp][i] = s;
    }
}

// Eigen::LDLT of A (lower triangle read; pivot on the not-yet-updated
// diagonal), then solve A x = b.  Every index is static after unrolling, so A
// stays in registers.  Returns isPositive() (no negative pivot).
__device__ __forceinline__ bool ldlt6_solve(double (&A)[6][6], const double (&b)[6],
                                            double (&x)[6]) {
  int perm[6];
  bool neg = false;
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    int p = k;
    double big = fabs(A[k][k]);
#pragma unroll
    for (int i = 0; i < 6; ++i)
      if (i > k && fabs(A[i][i]) > big) {
        big = fabs(A[i][i]);
        p = i;
      }
    // every lane holds the same matrix: make the pivot wave-uniform so the
    // swap below is a scalar branch, not exec-masked divergent code
    p = uniform_branch(p);
    perm[k] = p;
#pragma unroll
    for (int pp = 0; pp < 6; ++pp)
      if (pp > k && p == pp) {
        asm volatile("" ::: "memory");  // keep a real (scalar) branch: no if-conversion
        ldlt_swap(A, k, pp);
      }
    if (k > 0) {
      double temp[6];
      double acc = 0;
#pragma unroll
      for (int j = 0; j < 6; ++j)
        if (j < k) {
          temp[j] = A[j][j] * A[k][j];
          acc += A[k][j] * temp[j];
        }
      A[k][k] -= acc;
#pragma unroll
      for (int i = 0; i < 6; ++i)
        if (i > k) {
          double sacc = 0;
#pragma unroll
          for (int j = 0; j < 6; ++j)
            if (j < k) sacc += A[i][j] * temp[j];
          A[i][k] -= sacc;
        }
    }
    const double akk = A[k][k];
    if (fabs(akk) > 0) {
#pragma unroll
      for (int i = 0; i < 6; ++i)
        if (i > k) A[i][k] /= akk;
    }
    if (akk < 0) neg = true;
  }
#pragma unroll
  for (int i = 0; i < 6; ++i) x[i] = b[i];
#pragma unroll
  for (int k = 0; k < 6; ++k)
#pragma unroll
    for (int pp = 0; pp < 6; ++pp)
      if (pp > k && perm[k] == pp) {
        const double s = x[k];
        x[k] = x[pp];
        x[pp] = s;
      }
#pragma unroll
  for (int i = 0; i < 6; ++i)
#pragma unroll
    for (int j = 0; j < 6; ++j)
      if (j < i) x[i] -= A[i][j] * x[j];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const double d = A[i][i];
    x[i] = fabs(d) > 1.0 / 1.79769313486231570815e+308 ? x[i] / d : 0.0;
  }
#pragma unroll
  for (int i = 5; i >= 0; --i)
#pragma unroll
    for (int j = 0; j < 6; ++j)
      if (j > i) x[i] -= A[j][i] * x[j];
#pragma unroll
  for (int k = 5; k >= 0; --k)
#pragma unroll
    for (int pp = 0; pp < 6; ++pp)
      if (pp > k && perm[k] == pp) {
        const double s = x[k];
        x[k] = x[pp];
        x[pp] = s;
      }
  return !neg;
}

__device__ __forceinline__ double readlane_f64(double v, int lane) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), lane),
                          __builtin_amdgcn_readlane(__double2loint(v), lane));
}

// The same LDLT solve of (H + lambda I) x = b for H = hb[1..21] (lower
// triangle, row-major) and b = hb[22..27] (LDS), lane-parallel inside each
// wave: lanes 0..5 own the rows of the pivot-permuted matrix.  Eigen pivots
// on the not-yet-updated diagonal, i.e. the original one, so the order is
// fixed up front (ties in index order; Eigen breaks them by position, which
// only changes rounding) and the factorisation runs right-looking with D_k
// and the column broadcast by v_readlane.  Every lane returns the full x and
// isPositive(); the solve is carried out even when a pivot is negative, as
// ldlt6_solve.
__device__ __forceinline__ bool ldlt6_wave(const double* hb, double lambda, double (&x)[6]) {
  const int lane = threadIdx.x & 63;
  const int li = lane < 6 ? lane : 0;
  const double dl = lane < 6 ? fabs(hb[1 + li * (li + 1) / 2 + li] + lambda) : -1.0;
  int rank = 0;
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    const double dj = readlane_f64(dl, j);
    rank += (dj > dl || (dj == dl && j < lane)) ? 1 : 0;
  }
  // perm[q] = original index at position q: lane q finds the index ranked q
  int pi = 0;
#pragma unroll
  for (int j = 0; j < 6; ++j) pi = __builtin_amdgcn_readlane(rank, j) == lane ? j : pi;
  double a[6];
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    const int pj = __builtin_amdgcn_readlane(pi, j);
    const int r = max(pi, pj), c = min(pi, pj);
    a[j] = hb[1 + r * (r + 1) / 2 + c] + (r == c ? lambda : 0.0);
  }
  bool neg = false;
  double dd = 1.0;
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    const double dk = readlane_f64(a[k], k);
    if (dk < 0) neg = true;
    if (lane == k) dd = dk;
    const bool nz = fabs(dk) > 0;
    const double c = a[k];
    const double lu = nz ? c / dk : 0.0;
#pragma unroll
    for (int j = k + 1; j < 6; ++j) a[j] = fma(-c, readlane_f64(lu, j), a[j]);
    if (lane > k && nz) a[k] = lu;
  }
  double y = hb[22 + pi];
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    const double yj = readlane_f64(y, j);
    y = lane > j ? fma(-a[j], yj, y) : y;
  }
  double z = fabs(dd) > 1.0 / 1.79769313486231570815e+308 ? y / dd : 0.0;
  // L^T solve: lane i needs L_ji, lane j's a[i]
#pragma unroll
  for (int j = 5; j > 0; --j) {
    const double zj = readlane_f64(z, j);
#pragma unroll
    for (int i = 0; i < 5; ++i)
      if (i < j) {
        const double lji = readlane_f64(a[i], j);
        z = lane == i ? fma(-lji, zj, z) : z;
      }
  }
#pragma unroll
  for (int k = 0; k < 6; ++k) x[k] = readlane_f64(z, __builtin_amdgcn_readlane(rank, k));
  return !neg;
}

// The same system by Gauss-Jordan elimination with DPP64 row broadcasts: lane
// li of every 16-lane row owns row li (li < 6; the others zero) in the
// natural order, with b appended; pivot K's row is read from lane K of the
// lane's own row by v_fmac_f64_dpp row_newbcast, one instruction per entry (a
// fixed window of 6 entries after the pivot column: the row's rest, b, zero
// padding), every row but the pivot's subtracting l_i times it.  For a
// symmetric positive definite system the pivot signs do not depend on the
// order, so isPositive() is ldlt6_wave's; x_i = b'_i / D_i with Eigen's
// tolerance, solved even when a pivot is negative (as ldlt6_wave).  A zero or
// near-zero pivot (|d| <= kGj6NearZero x the largest diagonal entry, where
// rounding in another order could flip a sign) takes ldlt6_wave: Eigen's
// pivot order and semantics.  ldlt6_wave / ldlt_wave run only in that case.
constexpr double kGj6NearZero = 1e-12;

template <int N>
__device__ __forceinline__ double row16_bcast_f64(double v) {
  double o;
  asm volatile("s_nop 1\n\tv_mov_b64_dpp %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf"
               : "=v"(o)
               : "v"(v), "i"(N));
  return o;
}
#define POSE_FMC(k) "v_fmac_f64_dpp %" #k ", %" #k ", -%6 row_newbcast:%7 row_mask:0xf bank_mask:0xf\n\t"
template <int K>
__device__ __forceinline__ void gj6_pivot(double (&w)[12], double l) {
  asm volatile("s_nop 1\n\t" POSE_FMC(0) POSE_FMC(1) POSE_FMC(2) POSE_FMC(3) POSE_FMC(4) POSE_FMC(5)
               : "+v"(w[K + 1]), "+v"(w[K + 2]), "+v"(w[K + 3]), "+v"(w[K + 4]), "+v"(w[K + 5]),
                 "+v"(w[K + 6])
               : "v"(l), "i"(K));
}
#undef POSE_FMC
template <int K>
__device__ __forceinline__ void gj6_pivots(double (&w)[12], int li, double& dmine, int& flags, double tiny) {
  if constexpr (K < 6) {
    const double d = row16_bcast_f64<K>(w[K]);
    flags |= (d < 0.0 ? 1 : 0) | (fabs(d) <= tiny ? 2 : 0);
    double r = __builtin_amdgcn_rcp(d);
    r = fma(r, fma(-d, r, 1.0), r);
    dmine = li == K ? d : dmine;
    gj6_pivot<K>(w, li != K ? w[K] * r : 0.0);
    gj6_pivots<K + 1>(w, li, dmine, flags, tiny);
  }
}

// The Gauss-Jordan solve with a lambda per 16-lane row: the four rows of a wave solve four
// systems H + lambda_r I at once (the row broadcasts never leave a row).  A
// row with a zero pivot is redone alone by ldlt6_wave (Eigen's pivoting).
// Every lane of row r returns row r's x and isPositive().
__device__ __forceinline__ bool ldlt6_gj_rows(const double* hb, const double* hf, double lambda,
                                              double (&x)[6]) {
  const int lane = threadIdx.x & 63, li = lane & 15;
  const double* row = hf + 6 * (li < 6 ? li : 0);
  double w[12];
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    const double h = row[j];
    w[j] = li < 6 ? (li == j ? h + lambda : h) : 0.0;
  }
  w[6] = li < 6 ? hb[22 + li] : 0.0;
#pragma unroll
  for (int j = 7; j < 12; ++j) w[j] = 0.0;
  double dmine = 1.0;
  int flags = 0;
  double dmax = 0;  // the largest |diagonal entry| of this row's system
#pragma unroll
  for (int j = 0; j < 6; ++j) dmax = fmax(dmax, fabs(hf[7 * j] + lambda));
  gj6_pivots<0>(w, li, dmine, flags, kGj6NearZero * dmax);
  const double z = li < 6 && fabs(dmine) > 1.0 / 1.79769313486231570815e+308 ? w[6] / dmine : 0.0;
  x[0] = row16_bcast_f64<0>(z);
  x[1] = row16_bcast_f64<1>(z);
  x[2] = row16_bcast_f64<2>(z);
  x[3] = row16_bcast_f64<3>(z);
  x[4] = row16_bcast_f64<4>(z);
  x[5] = row16_bcast_f64<5>(z);
  bool ok = !(flags & 1);
  const uint64_t zero = __builtin_amdgcn_ballot_w64((flags & 2) != 0);
  if (zero) {
#pragma unroll 1
    for (int r = 0; r < 4; ++r)
      if ((zero >> (16 * r)) & 0xffffu) {
        double xr[6];
        const bool okr = ldlt6_wave(hb, readlane_f64(lambda, 16 * r), xr);
        if ((lane >> 4) == r) {
#pragma unroll
          for (int k = 0; k < 6; ++k) x[k] = xr[k];
          ok = okr;
        }
      }
  }
  return ok;
}

// g2o RobustKernelHuber::robustify; e2 > delta^2 >= 1 in the sqrt branch
__device__ __forceinline__ void huber_rho(double e2, double delta, double& rho0, double& rho1) {
  const double dsqr = delta * delta;
  if (e2 <= dsqr) {
    rho0 = e2;
    rho1 = 1.0;
  } else {
    const double s = sqrt_f64(e2);
    rho0 = 2 * s * delta - dsqr;
    rho1 = div_by(delta, recip_f64(s));
  }
}

}  // namespace orbgpu
