// ORACLE (test infrastructure only): restatement of
// Optimizer::LocalBundleAdjustment's solve (src/solver/g2o_solver/optimizer.cc
// :1127-1441) for the pinhole, non-fisheye case: pose vertices
// VertexSE3Expmap (fixed ones excluded from the system), point vertices
// VertexSBAPointXYZ marginalized (Schur complement, core/block_solver.hpp
// :364-514), binary edges ORB_SLAM_FUSION::EdgeSE3ProjectXYZ (mono,
// optimizable_types.h:105-125, optimizable_types.cc:134-155) and
// g2o::EdgeStereoSE3ProjectXYZ (types_six_dof_expmap.cpp:174-257), Huber
// kernels (core/robust_kernel_impl.cpp:72-85) with the quadratic form of
// core/base_binary_edge.hpp:56-119, g2o Levenberg-Marquardt
// (core/optimization_algorithm_levenberg.cpp:59-191) for optimize(10), then
// the outlier classification of optimizer.cc:1362-1400.
//
// The reduced camera system is solved with a dense LDLT in the natural order
// (the reference uses Eigen's SimplicialLDLT with an AMD fill-reducing
// ordering: same factorisation up to rounding), so parity with the GPU path
// is by tolerance (poses/points), exact on outlier flags away from the
// thresholds.
//
// Sharding: the caller may restrict the points to [pt_begin,
// pt_end); everything a point contributes (its Hll, its edges' Hpp/Hpl/b and
// robust chi2) is then partial, and `reduce` (sum / max over ranks) completes
// the reduced system, the chi2 and the LM scale -- the same structure as the
// GPU path's RCCL all-reduce.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "g2o_math.h"

namespace oracle {

struct LbaEdge {  // == orbgpu_lba_edge
  int32_t point, kf;
  float u, v, ur;  // ur < 0 -> monocular observation
  float inv_sigma2;
};

using LbaReduceFn = int (*)(void* user, double* buf, int n, int op);  // op: 0 sum, 1 max

namespace {

struct Cam {
  double fx, fy, cx, cy, bf;
};

// Edge error at (pose T, point X); returns false when the depth is not positive
// (isDepthPositive on the same state).
bool edge_error(const LbaEdge& e, const SE3& T, const double X[3], const Cam& c, double err[3]) {
  double p[3];
  T.map(X, p);
  if (e.ur < 0) {  // Pinhole::project
    err[0] = (double)e.u - (c.fx * p[0] / p[2] + c.cx);
    err[1] = (double)e.v - (c.fy * p[1] / p[2] + c.cy);
    err[2] = 0;
  } else {  // EdgeStereoSE3ProjectXYZ::cam_project (float invz)
    const float invz = 1.0f / (float)p[2];
    const double u = p[0] * invz * c.fx + c.cx;
    const double v = p[1] * invz * c.fy + c.cy;
    err[0] = (double)e.u - u;
    err[1] = (double)e.v - v;
    err[2] = (double)e.ur - (u - c.bf * invz);
  }
  return p[2] > 0.0;
}

double edge_chi2(const LbaEdge& e, const double err[3]) {
  const double info = (double)e.inv_sigma2;
  double s = err[0] * (info * err[0]) + err[1] * (info * err[1]);
  if (e.ur >= 0) s += err[2] * (info * err[2]);
  return s;
}

double edge_delta(const LbaEdge& e) {
  return e.ur < 0 ? (double)(float)std::sqrt(5.991) : (double)(float)std::sqrt(7.815);
}

// Jacobians of the error w.r.t. the point (Jl, D x 3) and the pose (Jp, D x 6).
void edge_jacobians(const LbaEdge& e, const SE3& T, const double X[3], const Cam& c,
                    double Jl[3][3], double Jp[3][6]) {
  double p[3];
  T.map(X, p);
  const double x = p[0], y = p[1], z = p[2];
  // rotation matrix of T
  const double e0[3] = {1, 0, 0}, e1[3] = {0, 1, 0}, e2[3] = {0, 0, 1};
  double c0[3], c1[3], c2[3];
  quat_rotate(T.r, e0, c0);
  quat_rotate(T.r, e1, c1);
  quat_rotate(T.r, e2, c2);
  const double R[3][3] = {{c0[0], c1[0], c2[0]}, {c0[1], c1[1], c2[1]}, {c0[2], c1[2], c2[2]}};
  if (e.ur < 0) {
    // projectJac = -ProjectJac(xyz_trans) (pinhole_model.cc); Jl = projectJac * R,
    // Jp = projectJac * [[0 z -y 1 0 0], [-z 0 x 0 1 0], [y -x 0 0 0 1]]
    const double pj[2][3] = {{-(c.fx / z), 0.0, -(-c.fx * x / (z * z))},
                             {0.0, -(c.fy / z), -(-c.fy * y / (z * z))}};
    const double S[3][6] = {{0, z, -y, 1, 0, 0}, {-z, 0, x, 0, 1, 0}, {y, -x, 0, 0, 0, 1}};
    for (int r = 0; r < 2; ++r) {
      for (int k = 0; k < 3; ++k) Jl[r][k] = pj[r][0] * R[0][k] + pj[r][1] * R[1][k] + pj[r][2] * R[2][k];
      for (int k = 0; k < 6; ++k) Jp[r][k] = pj[r][0] * S[0][k] + pj[r][1] * S[1][k] + pj[r][2] * S[2][k];
    }
    for (int k = 0; k < 3; ++k) Jl[2][k] = 0;
    for (int k = 0; k < 6; ++k) Jp[2][k] = 0;
  } else {  // types_six_dof_expmap.cpp:211-257
    const double z_2 = z * z, fx = c.fx, fy = c.fy, bf = c.bf;
    for (int k = 0; k < 3; ++k) {
      Jl[0][k] = -fx * R[0][k] / z + fx * x * R[2][k] / z_2;
      Jl[1][k] = -fy * R[1][k] / z + fy * y * R[2][k] / z_2;
      Jl[2][k] = Jl[0][k] - bf * R[2][k] / z_2;
    }
    Jp[0][0] = x * y / z_2 * fx;
    Jp[0][1] = -(1 + (x * x / z_2)) * fx;
    Jp[0][2] = y / z * fx;
    Jp[0][3] = -1. / z * fx;
    Jp[0][4] = 0;
    Jp[0][5] = x / z_2 * fx;
    Jp[1][0] = (1 + y * y / z_2) * fy;
    Jp[1][1] = -x * y / z_2 * fy;
    Jp[1][2] = -x / z * fy;
    Jp[1][3] = 0;
    Jp[1][4] = -1. / z * fy;
    Jp[1][5] = y / z_2 * fy;
    Jp[2][0] = Jp[0][0] - bf * y / z_2;
    Jp[2][1] = Jp[0][1] + bf * x / z_2;
    Jp[2][2] = Jp[0][2];
    Jp[2][3] = Jp[0][3];
    Jp[2][4] = 0;
    Jp[2][5] = Jp[0][5] - bf / z_2;
  }
}

// Inverse of a symmetric 3x3 by cofactors (Eigen compute_inverse_size3).
bool inv3(const double A[3][3], double Ai[3][3]) {
  const double c00 = A[1][1] * A[2][2] - A[1][2] * A[2][1];
  const double c10 = A[1][2] * A[2][0] - A[1][0] * A[2][2];
  const double c20 = A[1][0] * A[2][1] - A[1][1] * A[2][0];
  const double det = A[0][0] * c00 + A[0][1] * c10 + A[0][2] * c20;
  if (det == 0) return false;
  const double id = 1.0 / det;
  Ai[0][0] = c00 * id;
  Ai[1][0] = c10 * id;
  Ai[2][0] = c20 * id;
  Ai[0][1] = (A[0][2] * A[2][1] - A[0][1] * A[2][2]) * id;
  Ai[1][1] = (A[0][0] * A[2][2] - A[0][2] * A[2][0]) * id;
  Ai[2][1] = (A[0][1] * A[2][0] - A[0][0] * A[2][1]) * id;
  Ai[0][2] = (A[0][1] * A[1][2] - A[0][2] * A[1][1]) * id;
  Ai[1][2] = (A[0][2] * A[1][0] - A[0][0] * A[1][2]) * id;
  Ai[2][2] = (A[0][0] * A[1][1] - A[0][1] * A[1][0]) * id;
  return true;
}

// Dense LDLT (natural order, lower triangle) of the n x n row-major S, then
// solve S x = b in place of x.  Returns false on a zero pivot: Eigen's
// SimplicialLDLT (linear_solver_eigen.h:101-104) reports NumericalIssue only
// for D(k,k) == 0 (SimplicialCholesky_impl.h, the DoLDLT branch); a negative
// pivot factorises and the LM step is judged by rho.
// Row i's entries left of its first structural non-zero (fst[i]) stay zero
// through the factorisation, so every sum runs from max(fst[i], fst[k]): the
// terms left out are exact zeros, and the result is the full loop's (a large
// banded window factorises in O(n b^2)).
bool ldlt_dense(std::vector<double>& S, int n, const double* b, double* x) {
  std::vector<double> d(n);
  std::vector<int> fst(n);
  for (int i = 0; i < n; ++i) {
    int j = 0;
    while (j < i && S[(size_t)i * n + j] == 0.0) ++j;
    fst[i] = j;
  }
  bool ok = true;
  for (int k = 0; k < n; ++k) {
    double dk = S[(size_t)k * n + k];
    for (int j = fst[k]; j < k; ++j) dk -= S[(size_t)k * n + j] * S[(size_t)k * n + j] * d[j];
    d[k] = dk;
    if (dk == 0) ok = false;
    for (int i = k + 1; i < n; ++i) {
      if (fst[i] > k) continue;  // S(i, k) = 0 and stays 0
      double s = S[(size_t)i * n + k];
      for (int j = std::max(fst[i], fst[k]); j < k; ++j) s -= S[(size_t)i * n + j] * S[(size_t)k * n + j] * d[j];
      S[(size_t)i * n + k] = dk != 0 ? s / dk : 0.0;
    }
  }
  for (int i = 0; i < n; ++i) {
    double s = b[i];
    for (int j = fst[i]; j < i; ++j) s -= S[(size_t)i * n + j] * x[j];
    x[i] = s;
  }
  for (int i = 0; i < n; ++i) x[i] = d[i] != 0 ? x[i] / d[i] : 0.0;
  for (int i = n - 1; i >= 0; --i) {
    double s = x[i];
    for (int j = i + 1; j < n; ++j)
      if (fst[j] <= i) s -= S[(size_t)j * n + i] * x[j];
    x[i] = s;
  }
  return ok;
}

SE3 pose_from_float(const float* p) {
  SE3 T;
  T.r.x = p[0];
  T.r.y = p[1];
  T.r.z = p[2];
  T.r.w = p[3];
  for (int k = 0; k < 3; ++k) T.t[k] = p[4 + k];
  return T;
}

}  // namespace

// Returns 0, or -1 on invalid input / a failed reduce.  stats (6 doubles):
// initial robust chi2, final robust chi2, LM iterations, trials, final lambda,
// edges flagged as outliers (all over this shard's edges except the chi2,
// which are global).  lambda_init > 0: setUserLambdaInit (optimizer.cc:1137,
// 100 for an inertial map).  stop_after_trials >= 0: SparseOptimizer::
// terminate() (the pbStopFlag) reads true once that many LM trials have run;
// it is polled where g2o polls it: before every iteration
// (sparse_optimizer.cpp:406) and after every trial
// (optimization_algorithm_levenberg.cpp:153-154).
int lba_optimize(const float cam5[5], int n_kf, const float* poses, const uint8_t* fixed,
                 int n_pts, const float* pts, int n_edges, const LbaEdge* edges, int pt_begin,
                 int pt_end, int iters, double lambda_init, int stop_after_trials,
                 LbaReduceFn reduce, void* user, double* poses_out, double* pts_out,
                 uint8_t* outlier, double* stats, double* chi2_out = nullptr) {
  const Cam c{cam5[0], cam5[1], cam5[2], cam5[3], cam5[4]};
  if (n_kf <= 0 || n_pts < 0 || pt_begin < 0 || pt_end > n_pts || pt_begin > pt_end) return -1;
  auto red = [&](double* buf, int n, int op) { return reduce ? reduce(user, buf, n, op) : 0; };

  // vertices: free poses get Hessian indices in keyframe (vertex id) order
  std::vector<int> hidx(n_kf, -1);
  int nf = 0;
  for (int k = 0; k < n_kf; ++k)
    if (!fixed[k]) hidx[k] = nf++;
  const int n = 6 * nf;
  std::vector<SE3> T(n_kf);
  for (int k = 0; k < n_kf; ++k) T[k] = pose_from_float(poses + 7 * k);
  std::vector<double> X((size_t)3 * n_pts);
  for (size_t i = 0; i < X.size(); ++i) X[i] = pts[i];

  // this shard's edges, grouped by point in insertion order
  std::vector<std::vector<int>> pe(n_pts);
  for (int i = 0; i < n_edges; ++i) {
    const LbaEdge& e = edges[i];
    if (e.point < 0 || e.point >= n_pts || e.kf < 0 || e.kf >= n_kf) return -1;
    if (e.point >= pt_begin && e.point < pt_end) pe[e.point].push_back(i);
  }
  std::vector<double> err((size_t)3 * n_edges, 0.0);  // errors of the last computeActiveErrors

  auto active_chi2 = [&](const std::vector<SE3>& Ts, const std::vector<double>& Xs) {
    double chi = 0;
    for (int p = pt_begin; p < pt_end; ++p)
      for (int i : pe[p]) {
        const LbaEdge& e = edges[i];
        edge_error(e, Ts[e.kf], &Xs[(size_t)3 * p], c, &err[(size_t)3 * i]);
        double r0, r1;
        huber(edge_chi2(e, &err[(size_t)3 * i]), edge_delta(e), r0, r1);
        chi += r0;
      }
    return chi;
  };

  // per-iteration linear system pieces (this shard)
  std::vector<double> Hll((size_t)9 * n_pts), bl((size_t)3 * n_pts), Hpl((size_t)18 * n_edges);
  std::vector<double> Hpp_own((size_t)n * n), bp_own(n);

  auto build = [&]() {
    std::fill(Hll.begin(), Hll.end(), 0.0);
    std::fill(bl.begin(), bl.end(), 0.0);
    std::fill(Hpp_own.begin(), Hpp_own.end(), 0.0);
    std::fill(bp_own.begin(), bp_own.end(), 0.0);
    for (int p = pt_begin; p < pt_end; ++p)
      for (int i : pe[p]) {
        const LbaEdge& e = edges[i];
        const double* ev = &err[(size_t)3 * i];
        const int D = e.ur < 0 ? 2 : 3;
        double Jl[3][3], Jp[3][6];
        edge_jacobians(e, T[e.kf], &X[(size_t)3 * p], c, Jl, Jp);
        double r0, w;
        huber(edge_chi2(e, ev), edge_delta(e), r0, w);
        const double info = (double)e.inv_sigma2, wi = w * info;
        double om_r[3];  // omega_r = -omega * e * rho'
        for (int r = 0; r < 3; ++r) om_r[r] = (-info * ev[r]) * w;
        double* H = &Hll[(size_t)9 * p];
        double* b = &bl[(size_t)3 * p];
        for (int a = 0; a < 3; ++a) {
          for (int r = 0; r < D; ++r) b[a] += Jl[r][a] * om_r[r];
          for (int q = 0; q < 3; ++q) {
            double h = 0;
            for (int r = 0; r < D; ++r) h += Jl[r][a] * wi * Jl[r][q];
            H[3 * a + q] += h;
          }
        }
        const int hk = hidx[e.kf];
        if (hk < 0) continue;
        double* Hp = &Hpp_own[(size_t)(6 * hk) * n + 6 * hk];
        for (int a = 0; a < 6; ++a) {
          for (int r = 0; r < D; ++r) bp_own[6 * hk + a] += Jp[r][a] * om_r[r];
          for (int q = 0; q < 6; ++q) {
            double h = 0;
            for (int r = 0; r < D; ++r) h += Jp[r][a] * wi * Jp[r][q];
            Hp[(size_t)a * n + q] += h;
          }
          for (int q = 0; q < 3; ++q) {  // Hpl = Jp^T W Jl (6 x 3)
            double h = 0;
            for (int r = 0; r < D; ++r) h += Jp[r][a] * wi * Jl[r][q];
            Hpl[(size_t)18 * i + 3 * a + q] = h;
          }
        }
      }
  };

  const double tau = 1e-5;
  double lambda = 0, ni = 2;
  int nbad = 0, iters_done = 0, trials = 0;
  double cur = active_chi2(T, X);
  if (red(&cur, 1, 0)) return -1;
  const double chi_init = cur;
  // reduce buffer: S (n*n), b_s (n), b_p (n)
  std::vector<double> rbuf((size_t)n * n + 2 * n);
  std::vector<double> xp(n), xl((size_t)3 * n_pts), Dinv((size_t)9 * n_pts);
  std::vector<SE3> Tn(n_kf);
  std::vector<double> Xn(X);

  auto terminate = [&]() { return stop_after_trials >= 0 && trials >= stop_after_trials; };
  for (int it = 0; it < iters && !terminate(); ++it) {
    if (it > 0) {  // computeActiveErrors at the accepted state (same values as its trial)
      cur = active_chi2(T, X);
      if (red(&cur, 1, 0)) return -1;
    }
    const double ini = cur;
    build();
    if (it == 0) {  // computeLambdaInit: tau * max |diag| over pose and point blocks
      std::vector<double> dg(n + 1, 0.0);
      for (int k = 0; k < n; ++k) dg[k] = Hpp_own[(size_t)k * n + k];
      if (red(dg.data(), n, 0)) return -1;
      double mx = 0;
      for (int k = 0; k < n; ++k) mx = std::max(std::fabs(dg[k]), mx);
      double ml = 0;
      for (int p = pt_begin; p < pt_end; ++p)
        for (int a = 0; a < 3; ++a) ml = std::max(std::fabs(Hll[(size_t)9 * p + 4 * a]), ml);
      if (red(&ml, 1, 1)) return -1;
      lambda = lambda_init > 0 ? lambda_init : tau * std::max(mx, ml);
      ni = 2;
      nbad = 0;
    }
    double rho = 0;
    int q = 0;
    do {
      ++trials;
      // Schur complement of this shard's points at the current lambda
      double* S = rbuf.data();
      double* bs = S + (size_t)n * n;
      double* bp = bs + n;
      std::copy(Hpp_own.begin(), Hpp_own.end(), S);
      std::copy(bp_own.begin(), bp_own.end(), bs);
      std::copy(bp_own.begin(), bp_own.end(), bp);
      bool ok = true;
      for (int p = pt_begin; p < pt_end; ++p) {
        double Dm[3][3], Di[3][3];
        for (int a = 0; a < 3; ++a)
          for (int b2 = 0; b2 < 3; ++b2) Dm[a][b2] = Hll[(size_t)9 * p + 3 * a + b2] + (a == b2 ? lambda : 0.0);
        if (!inv3(Dm, Di)) ok = false;
        for (int a = 0; a < 3; ++a)
          for (int b2 = 0; b2 < 3; ++b2) Dinv[(size_t)9 * p + 3 * a + b2] = Di[a][b2];
        const double* blp = &bl[(size_t)3 * p];
        for (int i : pe[p]) {
          const int hi = hidx[edges[i].kf];
          if (hi < 0) continue;
          double W[6][3];  // Hpl_i * Dinv
          const double* Bi = &Hpl[(size_t)18 * i];
          for (int a = 0; a < 6; ++a)
            for (int b2 = 0; b2 < 3; ++b2)
              W[a][b2] = Bi[3 * a] * Di[0][b2] + Bi[3 * a + 1] * Di[1][b2] + Bi[3 * a + 2] * Di[2][b2];
          for (int a = 0; a < 6; ++a)
            bs[6 * hi + a] -= W[a][0] * blp[0] + W[a][1] * blp[1] + W[a][2] * blp[2];
          for (int j : pe[p]) {
            const int hj = hidx[edges[j].kf];
            if (hj < 0) continue;
            const double* Bj = &Hpl[(size_t)18 * j];
            for (int a = 0; a < 6; ++a)
              for (int b2 = 0; b2 < 6; ++b2)
                S[(size_t)(6 * hi + a) * n + 6 * hj + b2] -=
                    W[a][0] * Bj[3 * b2] + W[a][1] * Bj[3 * b2 + 1] + W[a][2] * Bj[3 * b2 + 2];
          }
        }
      }
      if (red(rbuf.data(), (int)rbuf.size(), 0)) return -1;
      for (int k = 0; k < n; ++k) S[(size_t)k * n + k] += lambda;
      std::vector<double> Sm(S, S + (size_t)n * n);
      if (!ldlt_dense(Sm, n, bs, xp.data())) ok = false;
      // back-substitution and trial state
      double sl = 0;  // this shard's landmark part of computeScale
      for (int p = pt_begin; p < pt_end; ++p) {
        double cp[3] = {bl[(size_t)3 * p], bl[(size_t)3 * p + 1], bl[(size_t)3 * p + 2]};
        for (int i : pe[p]) {
          const int hi = hidx[edges[i].kf];
          if (hi < 0) continue;
          const double* Bi = &Hpl[(size_t)18 * i];
          for (int b2 = 0; b2 < 3; ++b2)
            for (int a = 0; a < 6; ++a) cp[b2] -= Bi[3 * a + b2] * xp[6 * hi + a];
        }
        const double* Di = &Dinv[(size_t)9 * p];
        for (int a = 0; a < 3; ++a) {
          const double v = Di[3 * a] * cp[0] + Di[3 * a + 1] * cp[1] + Di[3 * a + 2] * cp[2];
          xl[(size_t)3 * p + a] = v;
          Xn[(size_t)3 * p + a] = X[(size_t)3 * p + a] + v;
          sl += v * (lambda * v + bl[(size_t)3 * p + a]);
        }
      }
      for (int k = 0; k < n_kf; ++k) Tn[k] = hidx[k] < 0 ? T[k] : se3_exp(&xp[6 * hidx[k]]).compose(T[k]);
      double tr[2] = {active_chi2(Tn, Xn), sl};
      if (red(tr, 2, 0)) return -1;
      double tmp = tr[0];
      if (!ok) tmp = DBL_MAX;
      rho = cur - tmp;
      double scale = tr[1];
      for (int k = 0; k < n; ++k) scale += xp[k] * (lambda * xp[k] + bp[k]);
      scale += 1e-3;
      rho /= scale;
      if (rho > 0 && std::isfinite(tmp)) {
        double alpha = 1. - std::pow(2 * rho - 1, 3);
        alpha = std::min(alpha, 2. / 3.);
        lambda *= std::max(1. / 3., alpha);
        ni = 2;
        cur = tmp;
        T = Tn;
        for (int p = pt_begin; p < pt_end; ++p)
          for (int a = 0; a < 3; ++a) X[(size_t)3 * p + a] = Xn[(size_t)3 * p + a];
      } else {
        lambda *= ni;
        ni *= 2;
      }
      ++q;
    } while (rho < 0 && q < 10 && !terminate());
    ++iters_done;
    if (q == 10 || rho == 0) break;
    if ((ini - cur) * 1e3 < ini)
      nbad++;
    else
      nbad = 0;
    if (nbad >= 3) break;
  }

  // outliers (optimizer.cc:1362-1400): chi2 of the last computeActiveErrors,
  // depth at the final estimates
  int n_out = 0;
  for (int p = pt_begin; p < pt_end; ++p)
    for (int i : pe[p]) {
      const LbaEdge& e = edges[i];
      double tmp[3];
      const bool depth_ok = edge_error(e, T[e.kf], &X[(size_t)3 * p], c, tmp);
      const double chi = edge_chi2(e, &err[(size_t)3 * i]);
      const bool out = chi > (e.ur < 0 ? 5.991 : 7.815) || !depth_ok;
      outlier[i] = out ? 1 : 0;
      if (chi2_out) chi2_out[i] = chi;
      n_out += out;
    }
  for (int k = 0; k < n_kf; ++k) {
    const double o[7] = {T[k].r.x, T[k].r.y, T[k].r.z, T[k].r.w, T[k].t[0], T[k].t[1], T[k].t[2]};
    for (int a = 0; a < 7; ++a) poses_out[7 * k + a] = o[a];
  }
  for (int p = pt_begin; p < pt_end; ++p)
    for (int a = 0; a < 3; ++a) pts_out[(size_t)3 * p + a] = X[(size_t)3 * p + a];
  if (stats) {
    stats[0] = chi_init;
    stats[1] = cur;
    stats[2] = iters_done;
    stats[3] = trials;
    stats[4] = lambda;
    stats[5] = n_out;
  }
  return 0;
}

}  // namespace oracle

extern "C" int orc_lba(const float* cam5, int n_kf, const float* poses, const uint8_t* fixed,
                       int n_pts, const float* pts, int n_edges, const void* edges, int pt_begin,
                       int pt_end, int iters, double lambda_init, int stop_after_trials,
                       oracle::LbaReduceFn reduce, void* user, double* poses_out, double* pts_out,
                       uint8_t* outlier, double* stats, double* chi2_out) {
  return oracle::lba_optimize(cam5, n_kf, poses, fixed, n_pts, pts, n_edges,
                              static_cast<const oracle::LbaEdge*>(edges), pt_begin, pt_end, iters,
                              lambda_init, stop_after_trials, reduce, user, poses_out, pts_out,
                              outlier, stats, chi2_out);
}

// Edge linearisation probe for the finite-difference tests: error (3),
// point Jacobian Jl (3x3 row-major) and pose Jacobian Jp (3x6) at pose7
// (double qx, qy, qz, qw, tx, ty, tz) and point X.
extern "C" int orc_lba_edge_linearize(const float* cam5, const double* pose7, const double* X,
                                      const void* edge, double* err, double* Jl, double* Jp) {
  using namespace oracle;
  const Cam c{cam5[0], cam5[1], cam5[2], cam5[3], cam5[4]};
  SE3 T;
  T.r.x = pose7[0];
  T.r.y = pose7[1];
  T.r.z = pose7[2];
  T.r.w = pose7[3];
  for (int k = 0; k < 3; ++k) T.t[k] = pose7[4 + k];
  const LbaEdge& e = *static_cast<const LbaEdge*>(edge);
  double l[3][3], p[3][6];
  const bool depth = edge_error(e, T, X, c, err);
  edge_jacobians(e, T, X, c, l, p);
  for (int r = 0; r < 3; ++r) {
    for (int k = 0; k < 3; ++k) Jl[3 * r + k] = l[r][k];
    for (int k = 0; k < 6; ++k) Jp[6 * r + k] = p[r][k];
  }
  return depth ? 1 : 0;
}

// se3 exp composed on the left of pose7 (for the finite-difference tests).
extern "C" void orc_se3_exp_compose(const double* u6, const double* pose7, double* out7) {
  using namespace oracle;
  SE3 T;
  T.r.x = pose7[0];
  T.r.y = pose7[1];
  T.r.z = pose7[2];
  T.r.w = pose7[3];
  for (int k = 0; k < 3; ++k) T.t[k] = pose7[4 + k];
  const SE3 R = se3_exp(u6).compose(T);
  const double o[7] = {R.r.x, R.r.y, R.r.z, R.r.w, R.t[0], R.t[1], R.t[2]};
  for (int k = 0; k < 7; ++k) out7[k] = o[k];
}
