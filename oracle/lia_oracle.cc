// ORACLE (test infrastructure only): restatement of Optimizer::LocalInertialBA's
// solve (src/solver/g2o_solver/optimizer.cc:2440-2826) for the pinhole,
// non-fisheye case (cam2_ == NULL):
//   vertices  VertexPose (ImuCamPose(KeyFrame*), g2o_types.cc:28-72; update
//             ImuCamPose::Update, :192-216), VertexVelocity / GyroBias /
//             AccBias (additive), VertexSBAPointXYZ marginalised
//   edges     EdgeMono / EdgeStereo (g2o_types.h:306-427, g2o_types.cc:334-415:
//             error obs - Project(Rcw X + tcw), Jacobians -proj_jac Rcw and
//             proj_jac Rcb SE3deriv(Xb)), Huber sqrt(5.991) / sqrt(7.815) as
//             floats (:2630-2633); EdgeInertial (g2o_types.cc:472-578) with
//             the optional Huber sqrt(16.92) and x1e-2 information
//             (:2571-2581); EdgeGyroRW / EdgeAccRW (g2o_types.h:592-662)
//   solver    g2o Levenberg-Marquardt (optimization_algorithm_levenberg.cpp:
//             59-168) with setUserLambdaInit (:2448-2459), BlockSolverX: the
//             Schur complement on the points (core/block_solver.hpp:364-514),
//             the reduced system by a dense LDLT in the natural order (the
//             reference: SimplicialLDLT + AMD, linear_solver_eigen.h:93-126 --
//             the same factorisation up to rounding)
//   then      the outlier test of :2796-2826 (float thresholds chi2Mono2 =
//             5.991f, 1.5f * 5.991f for close points, chi2Stereo2 = 7.815f;
//             mono edges also on !isDepthPositive) on the errors of the last
//             computeActiveErrors, and err / err_end of :2790-2793.
//
// Layout of the reduced system: the free key frames in window order, each
// owning its vertices' rows -- VP(6) VV(3) VG(3) VA(3) for a key frame with
// IMU data, VP(6) alone for one without (`!pKFi->bImu`: optimizer.cc:
// 2466-2484 adds only the VertexPose; no inertial edge reaches it, :2503).
// The factorisation is the dense natural-order LDLT restricted to the
// envelope of S (ldlt_dense): the same operations on the same values, the
// products with structural zeros left out.  Parity with the GPU path is by tolerance
// (states) and exact on outlier flags away from the thresholds.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "g2o_math.h"
#include "inertial_math.h"
#include "../include/orbgpu.h"

namespace oracle {
namespace lia {

using namespace oracle::inertial;

namespace {

constexpr int kDimImu = 15;  // VP VV VG VA
constexpr int kDimPose = 6;  // VP

struct VisEdge {  // == orbgpu_lba_edge
  int32_t point, kf;
  float u, v, ur, inv_sigma2;
};

// Xc = Rcw X + tcw, and the EdgeMono / EdgeStereo error (ImuCamPose::Project /
// ProjectStereo, g2o_types.cc:171-186, Pinhole::Project in double)
void vis_error(const VisEdge& e, const State& s, const Calib& c, const double X[3], double err[3],
               double Xc[3]) {
  const V3 p = add(mv(s.Rcw, V3{{X[0], X[1], X[2]}}), s.tcw);
  for (int k = 0; k < 3; ++k) Xc[k] = p[k];
  const double u = c.fx * p[0] / p[2] + c.cx;
  const double v = c.fy * p[1] / p[2] + c.cy;
  err[0] = (double)e.u - u;
  err[1] = (double)e.v - v;
  err[2] = 0;
  if (e.ur >= 0.f) {
    const double invz = 1 / p[2];
    err[2] = (double)e.ur - (u - c.bf * invz);
  }
}

double vis_chi2(const VisEdge& e, const double err[3]) {
  const double info = (double)e.inv_sigma2;
  double s = err[0] * info * err[0] + err[1] * info * err[1];
  if (e.ur >= 0.f) s += err[2] * info * err[2];
  return s;
}

double vis_delta(const VisEdge& e) {
  // const float thHuberMono = sqrt(5.991), thHuberStereo = sqrt(7.815) (:2630-2633)
  return e.ur >= 0.f ? (double)(float)std::sqrt(7.815) : (double)(float)std::sqrt(5.991);
}

// EdgeMono / EdgeStereo::linearizeOplus (g2o_types.cc:334-415): Jl = -proj_jac Rcw
// (point), Jp = proj_jac Rcb SE3deriv(Xb) (body-frame pose)
void vis_jacobians(const VisEdge& e, const State& s, const Calib& c, const double Xc[3],
                   double Jl[3][3], double Jp[3][6]) {
  const V3 xc{{Xc[0], Xc[1], Xc[2]}};
  const V3 Xb = add(mv(c.Rbc, xc), c.tbc);
  double pj[3][3] = {{c.fx / Xc[2], 0, -c.fx * Xc[0] / (Xc[2] * Xc[2])},
                     {0, c.fy / Xc[2], -c.fy * Xc[1] / (Xc[2] * Xc[2])},
                     {0, 0, 0}};
  const bool st = e.ur >= 0.f;
  if (st) {
    const double inv_z2 = 1.0 / (Xc[2] * Xc[2]);
    for (int k = 0; k < 3; ++k) pj[2][k] = pj[0][k];
    pj[2][2] += c.bf * inv_z2;
  }
  for (int r = 0; r < 3; ++r)
    for (int k = 0; k < 3; ++k)
      Jl[r][k] = -(pj[r][0] * s.Rcw(0, k) + pj[r][1] * s.Rcw(1, k) + pj[r][2] * s.Rcw(2, k));
  const double x = Xb[0], y = Xb[1], z = Xb[2];
  const double S[3][6] = {{0, z, -y, 1, 0, 0}, {-z, 0, x, 0, 1, 0}, {y, -x, 0, 0, 0, 1}};
  for (int r = 0; r < 3; ++r) {
    double PR[3];
    for (int k = 0; k < 3; ++k) PR[k] = pj[r][0] * c.Rcb(0, k) + pj[r][1] * c.Rcb(1, k) + pj[r][2] * c.Rcb(2, k);
    for (int k = 0; k < 6; ++k) Jp[r][k] = PR[0] * S[0][k] + PR[1] * S[1][k] + PR[2] * S[2][k];
  }
  if (!st) {
    for (int k = 0; k < 3; ++k) Jl[2][k] = 0;
    for (int k = 0; k < 6; ++k) Jp[2][k] = 0;
  }
}

bool inv3(const double A[3][3], double Ai[3][3]) {  // Eigen compute_inverse_size3
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

// Dense LDLT (natural order) of S, solve S x = b; false on a zero pivot
// (SimplicialLDLT's only NumericalIssue, linear_solver_eigen.h:101-104).
// Row i's entries left of its first structural non-zero (fst[i]) stay zero
// through the factorisation, so every sum runs from max(fst[i], fst[k]):
// the terms left out are exact zeros, and the result is the full loop's.
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

struct ImuEdge {
  int kf1, kf2, flags;
  Preint pi;
  double dt;
  double info[81], info_g[9], info_a[9];
  double delta;  // Huber delta (flags & ROBUST)
};

// EdgeInertial + EdgeGyroRW + EdgeAccRW of one temporal link: robust chi2
// contributions (activeRobustChi2) at the states.
double imu_chi2(const ImuEdge& E, const State& s1, const State& s2, const V3& g) {
  double e[9];
  inertial_edge_error(s1, s2, E.pi, E.dt, g, e);
  double chi = quad(E.info, e, 9);
  if (E.flags & ORBGPU_LIA_ROBUST) {
    double r0, r1;
    huber(chi, E.delta, r0, r1);
    chi = r0;
  }
  const V3 eg = sub(s2.bg, s1.bg), ea = sub(s2.ba, s1.ba);
  chi += quad(E.info_g, eg.a, 3);
  chi += quad(E.info_a, ea.a, 3);
  return chi;
}

void add_update(State& s, const double* u, const Calib& c, bool imu) {
  pose_update(s, u, c);
  if (!imu) return;  // VertexPose only
  for (int i = 0; i < 3; ++i) {
    s.v[i] += u[6 + i];
    s.bg[i] += u[9 + i];
    s.ba[i] += u[12 + i];
  }
}

}  // namespace

// Returns 0, or -1 on invalid input.  kfs_out: 21 doubles per key frame
// (Rwb, twb, v, bg, ba); pts_out: 3 doubles per point.  stats (7): err,
// err_end, LM iterations, trials, final lambda, outliers, accepted chi2.
int lia_optimize(const orbgpu_imu_calib& cb, int n_kf, const orbgpu_imu_state* kfs,
                 const uint8_t* fixed, const uint8_t* imu, int n_pts, const float* pts,
                 const uint8_t* close, int n_edges, const VisEdge* edges, int n_imu,
                 const orbgpu_lia_imu_edge* imu_edges, int iters, double lambda_init,
                 double* kfs_out, double* pts_out, uint8_t* outlier, double* stats,
                 double* sys_H = nullptr, double* sys_b = nullptr, double* chi2_out = nullptr) {
  if (n_kf <= 0 || n_pts < 0 || n_edges < 0 || n_imu < 0 || !(lambda_init > 0)) return -1;
  const Calib c = load_calib(cb);
  const V3 g = gravity();
  std::vector<int> hidx(n_kf, -1);  // first reduced-system row of a free key frame
  int n = 0;
  for (int k = 0; k < n_kf; ++k)
    if (!fixed[k]) {
      hidx[k] = n;
      n += imu[k] ? kDimImu : kDimPose;
    }
  std::vector<State> S(n_kf);
  for (int k = 0; k < n_kf; ++k) S[k] = load_state(kfs[k]);
  std::vector<double> X((size_t)3 * n_pts);
  for (size_t i = 0; i < X.size(); ++i) X[i] = pts[i];
  std::vector<std::vector<int>> pe(n_pts);
  for (int i = 0; i < n_edges; ++i) {
    const VisEdge& e = edges[i];
    if (e.point < 0 || e.point >= n_pts || e.kf < 0 || e.kf >= n_kf) return -1;
    pe[e.point].push_back(i);
  }
  std::vector<ImuEdge> IE(n_imu);
  for (int i = 0; i < n_imu; ++i) {
    const orbgpu_lia_imu_edge& s = imu_edges[i];
    if (s.kf1 < 0 || s.kf1 >= n_kf || s.kf2 < 0 || s.kf2 >= n_kf || !imu[s.kf1] || !imu[s.kf2])
      return -1;
    ImuEdge& E = IE[i];
    E.kf1 = s.kf1;
    E.kf2 = s.kf2;
    E.flags = s.flags;
    E.pi = preint_view(s.preint);
    E.dt = s.preint.dT;
    const double sc = (s.flags & ORBGPU_LIA_DOWNWEIGHT) ? 1e-2 : 1.0;  // information() * 1e-2
    for (int k = 0; k < 81; ++k) E.info[k] = s.preint.info[k] * sc;
    std::memcpy(E.info_g, s.preint.info_g, sizeof(E.info_g));
    std::memcpy(E.info_a, s.preint.info_a, sizeof(E.info_a));
    E.delta = std::sqrt(16.92);
  }
  std::vector<double> err((size_t)3 * n_edges, 0.0);  // visual errors of the last computeActiveErrors

  auto active_chi2 = [&](const std::vector<State>& Ss, const std::vector<double>& Xs) {
    double chi = 0;
    for (int p = 0; p < n_pts; ++p)
      for (int i : pe[p]) {
        const VisEdge& e = edges[i];
        double Xc[3];
        vis_error(e, Ss[e.kf], c, &Xs[(size_t)3 * p], &err[(size_t)3 * i], Xc);
        double r0, r1;
        huber(vis_chi2(e, &err[(size_t)3 * i]), vis_delta(e), r0, r1);
        chi += r0;
      }
    for (const ImuEdge& E : IE) chi += imu_chi2(E, Ss[E.kf1], Ss[E.kf2], g);
    return chi;
  };

  std::vector<double> Hll((size_t)9 * n_pts), bl((size_t)3 * n_pts), Hpl((size_t)18 * n_edges);
  std::vector<double> Hpp((size_t)n * n), bp(n);
  auto build = [&]() {
    std::fill(Hll.begin(), Hll.end(), 0.0);
    std::fill(bl.begin(), bl.end(), 0.0);
    std::fill(Hpp.begin(), Hpp.end(), 0.0);
    std::fill(bp.begin(), bp.end(), 0.0);
    for (int p = 0; p < n_pts; ++p)
      for (int i : pe[p]) {
        const VisEdge& e = edges[i];
        const double* ev = &err[(size_t)3 * i];
        const int D = e.ur < 0.f ? 2 : 3;
        double tmp[3], Xc[3];
        vis_error(e, S[e.kf], c, &X[(size_t)3 * p], tmp, Xc);
        double Jl[3][3], Jp[3][6];
        vis_jacobians(e, S[e.kf], c, Xc, Jl, Jp);
        double r0, w;
        huber(vis_chi2(e, ev), vis_delta(e), r0, w);
        const double info = (double)e.inv_sigma2, wi = w * info;
        double om_r[3];
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
        const int o = hk;
        for (int a = 0; a < 6; ++a) {
          for (int r = 0; r < D; ++r) bp[o + a] += Jp[r][a] * om_r[r];
          for (int q = 0; q < 6; ++q) {
            double h = 0;
            for (int r = 0; r < D; ++r) h += Jp[r][a] * wi * Jp[r][q];
            Hpp[(size_t)(o + a) * n + o + q] += h;
          }
          for (int q = 0; q < 3; ++q) {
            double h = 0;
            for (int r = 0; r < D; ++r) h += Jp[r][a] * wi * Jl[r][q];
            Hpl[(size_t)18 * i + 3 * a + q] = h;
          }
        }
      }
    // the inertial edges (no points: straight into the camera-side system)
    for (const ImuEdge& E : IE) {
      const State &s1 = S[E.kf1], &s2 = S[E.kf2];
      const int o1 = hidx[E.kf1], o2 = hidx[E.kf2];
      auto at = [](int o, int d) { return o >= 0 ? o + d : -1; };
      double e[9], J[9][24];
      inertial_edge_error(s1, s2, E.pi, E.dt, g, e);
      inertial_edge_jacobian(s1, s2, E.pi, E.dt, g, J);
      double w = 1.0;
      if (E.flags & ORBGPU_LIA_ROBUST) {
        double r0;
        huber(quad(E.info, e, 9), E.delta, r0, w);
      }
      const int bi[6][2] = {{at(o1, 0), 6}, {at(o1, 6), 3}, {at(o1, 9), 3},
                            {at(o1, 12), 3}, {at(o2, 0), 6}, {at(o2, 6), 3}};
      add_quadratic(Hpp.data(), bp.data(), n, 9, &J[0][0], 24, E.info, e, w, bi, 6);
      const double Jrw[3][6] = {{-1, 0, 0, 1, 0, 0}, {0, -1, 0, 0, 1, 0}, {0, 0, -1, 0, 0, 1}};
      const V3 eg = sub(s2.bg, s1.bg), ea = sub(s2.ba, s1.ba);
      const int bg_[2][2] = {{at(o1, 9), 3}, {at(o2, 9), 3}};
      const int ba_[2][2] = {{at(o1, 12), 3}, {at(o2, 12), 3}};
      add_quadratic(Hpp.data(), bp.data(), n, 3, &Jrw[0][0], 6, E.info_g, eg.a, 1.0, bg_, 2);
      add_quadratic(Hpp.data(), bp.data(), n, 3, &Jrw[0][0], 6, E.info_a, ea.a, 1.0, ba_, 2);
    }
  };

  double lambda = 0, ni = 2;
  int nbad = 0, iters_done = 0, trials = 0;
  double cur = active_chi2(S, X);
  if (sys_H) {  // the full system at the initial state (test probe)
    build();
    const int m = n + 3 * n_pts;
    std::fill(sys_H, sys_H + (size_t)m * m, 0.0);
    for (int r = 0; r < n; ++r) {
      sys_b[r] = bp[r];
      for (int q = 0; q < n; ++q) sys_H[(size_t)r * m + q] = Hpp[(size_t)r * n + q];
    }
    for (int p = 0; p < n_pts; ++p) {
      const int o = n + 3 * p;
      for (int a = 0; a < 3; ++a) {
        sys_b[o + a] = bl[(size_t)3 * p + a];
        for (int q = 0; q < 3; ++q) sys_H[(size_t)(o + a) * m + o + q] = Hll[(size_t)9 * p + 3 * a + q];
      }
      for (int i : pe[p]) {
        const int hi = hidx[edges[i].kf];
        if (hi < 0) continue;
        for (int a = 0; a < 6; ++a)
          for (int q = 0; q < 3; ++q) {
            const double h = Hpl[(size_t)18 * i + 3 * a + q];
            sys_H[(size_t)(hi + a) * m + o + q] += h;
            sys_H[(size_t)(o + q) * m + hi + a] += h;
          }
      }
    }
    return 0;
  }
  const double chi_init = cur;
  double last = cur;  // robust chi2 of the last computeActiveErrors
  std::vector<double> xp(n), Dinv((size_t)9 * n_pts);
  std::vector<State> Sn(n_kf);
  std::vector<double> Xn(X);

  for (int it = 0; it < iters; ++it) {
    if (it > 0) cur = last = active_chi2(S, X);
    const double ini = cur;
    build();
    if (it == 0) {
      lambda = lambda_init;  // setUserLambdaInit
      ni = 2;
      nbad = 0;
    }
    double rho = 0;
    int q = 0;
    do {
      ++trials;
      std::vector<double> Sm(Hpp), bs(bp);
      bool ok = true;
      for (int p = 0; p < n_pts; ++p) {
        double Dm[3][3], Di[3][3] = {};  // a singular block leaves 0 (and fails the trial)
        for (int a = 0; a < 3; ++a)
          for (int b2 = 0; b2 < 3; ++b2) Dm[a][b2] = Hll[(size_t)9 * p + 3 * a + b2] + (a == b2 ? lambda : 0.0);
        if (!inv3(Dm, Di)) ok = false;
        for (int a = 0; a < 3; ++a)
          for (int b2 = 0; b2 < 3; ++b2) Dinv[(size_t)9 * p + 3 * a + b2] = Di[a][b2];
        const double* blp = &bl[(size_t)3 * p];
        for (int i : pe[p]) {
          const int hi = hidx[edges[i].kf];
          if (hi < 0) continue;
          double W[6][3];
          const double* Bi = &Hpl[(size_t)18 * i];
          for (int a = 0; a < 6; ++a)
            for (int b2 = 0; b2 < 3; ++b2)
              W[a][b2] = Bi[3 * a] * Di[0][b2] + Bi[3 * a + 1] * Di[1][b2] + Bi[3 * a + 2] * Di[2][b2];
          for (int a = 0; a < 6; ++a)
            bs[hi + a] -= W[a][0] * blp[0] + W[a][1] * blp[1] + W[a][2] * blp[2];
          for (int j : pe[p]) {
            const int hj = hidx[edges[j].kf];
            if (hj < 0) continue;
            const double* Bj = &Hpl[(size_t)18 * j];
            for (int a = 0; a < 6; ++a)
              for (int b2 = 0; b2 < 6; ++b2)
                Sm[(size_t)(hi + a) * n + hj + b2] -=
                    W[a][0] * Bj[3 * b2] + W[a][1] * Bj[3 * b2 + 1] + W[a][2] * Bj[3 * b2 + 2];
          }
        }
      }
      for (int k = 0; k < n; ++k) Sm[(size_t)k * n + k] += lambda;
      if (!ldlt_dense(Sm, n, bs.data(), xp.data())) ok = false;
      double sl = 0;  // landmark part of computeScale
      for (int p = 0; p < n_pts; ++p) {
        double cp[3] = {bl[(size_t)3 * p], bl[(size_t)3 * p + 1], bl[(size_t)3 * p + 2]};
        for (int i : pe[p]) {
          const int hi = hidx[edges[i].kf];
          if (hi < 0) continue;
          const double* Bi = &Hpl[(size_t)18 * i];
          for (int b2 = 0; b2 < 3; ++b2)
            for (int a = 0; a < 6; ++a) cp[b2] -= Bi[3 * a + b2] * xp[hi + a];
        }
        const double* Di = &Dinv[(size_t)9 * p];
        for (int a = 0; a < 3; ++a) {
          const double v = Di[3 * a] * cp[0] + Di[3 * a + 1] * cp[1] + Di[3 * a + 2] * cp[2];
          Xn[(size_t)3 * p + a] = X[(size_t)3 * p + a] + v;
          sl += v * (lambda * v + bl[(size_t)3 * p + a]);
        }
      }
      for (int k = 0; k < n_kf; ++k) {
        Sn[k] = S[k];
        if (hidx[k] >= 0) add_update(Sn[k], &xp[hidx[k]], c, imu[k] != 0);
      }
      double tmp = active_chi2(Sn, Xn);
      last = tmp;
      if (!ok) tmp = DBL_MAX;
      rho = cur - tmp;
      double scale = sl;
      for (int k = 0; k < n; ++k) scale += xp[k] * (lambda * xp[k] + bp[k]);
      scale += 1e-3;
      rho /= scale;
      if (rho > 0 && std::isfinite(tmp)) {
        double alpha = 1. - std::pow(2 * rho - 1, 3);
        alpha = std::min(alpha, 2. / 3.);
        lambda *= std::max(1. / 3., alpha);
        ni = 2;
        cur = tmp;
        S = Sn;
        X = Xn;
      } else {
        lambda *= ni;
        ni *= 2;
      }
      ++q;
    } while (rho < 0 && q < 10);
    ++iters_done;
    if (q == 10 || rho == 0) break;
    if ((ini - cur) * 1e3 < ini)
      nbad++;
    else
      nbad = 0;
    if (nbad >= 3) break;
  }

  // outliers (optimizer.cc:2799-2826)
  const double th_mono = 5.991f, th_mono_close = 1.5f * 5.991f, th_stereo = 7.815f;
  int n_out = 0;
  for (int p = 0; p < n_pts; ++p)
    for (int i : pe[p]) {
      const VisEdge& e = edges[i];
      const double chi = vis_chi2(e, &err[(size_t)3 * i]);
      bool out;
      if (e.ur < 0.f) {
        const State& s = S[e.kf];
        const double* x = &X[(size_t)3 * p];
        const bool depth = s.Rcw(2, 0) * x[0] + s.Rcw(2, 1) * x[1] + s.Rcw(2, 2) * x[2] + s.tcw[2] > 0.0;
        const bool cl = close && close[p];
        out = (chi > th_mono && !cl) || (chi > th_mono_close && cl) || !depth;
      } else {
        out = chi > th_stereo;
      }
      outlier[i] = out ? 1 : 0;
      if (chi2_out) chi2_out[i] = chi;
      n_out += out;
    }
  for (int k = 0; k < n_kf; ++k) {
    double* o = kfs_out + 21 * (size_t)k;
    std::memcpy(o, S[k].Rwb.a, 9 * sizeof(double));
    std::memcpy(o + 9, S[k].twb.a, 3 * sizeof(double));
    std::memcpy(o + 12, S[k].v.a, 3 * sizeof(double));
    std::memcpy(o + 15, S[k].bg.a, 3 * sizeof(double));
    std::memcpy(o + 18, S[k].ba.a, 3 * sizeof(double));
  }
  std::copy(X.begin(), X.end(), pts_out);
  if (stats) {
    stats[0] = chi_init;
    stats[1] = last;
    stats[2] = iters_done;
    stats[3] = trials;
    stats[4] = lambda;
    stats[5] = n_out;
    stats[6] = cur;
  }
  return 0;
}

}  // namespace lia
}  // namespace oracle

extern "C" int orc_lia(const orbgpu_imu_calib* cb, int n_kf, const orbgpu_imu_state* kfs,
                       const uint8_t* fixed, const uint8_t* imu, int n_pts, const float* pts,
                       const uint8_t* close, int n_edges, const void* edges, int n_imu,
                       const orbgpu_lia_imu_edge* imu_edges, int iters, double lambda_init,
                       double* kfs_out, double* pts_out, uint8_t* outlier, double* stats,
                       double* chi2_out) {
  return oracle::lia::lia_optimize(*cb, n_kf, kfs, fixed, imu, n_pts, pts, close, n_edges,
                                   static_cast<const oracle::lia::VisEdge*>(edges), n_imu,
                                   imu_edges, iters, lambda_init, kfs_out, pts_out, outlier,
                                   stats, nullptr, nullptr, chi2_out);
}

extern "C" int orc_lia_system(const orbgpu_imu_calib* cb, int n_kf, const orbgpu_imu_state* kfs,
                              const uint8_t* fixed, const uint8_t* imu, int n_pts, const float* pts,
                              int n_edges, const void* edges, int n_imu,
                              const orbgpu_lia_imu_edge* imu_edges, double* H, double* b) {
  std::vector<double> ko((size_t)21 * n_kf), po((size_t)3 * n_pts + 3);
  std::vector<uint8_t> out(n_edges + 1);
  return oracle::lia::lia_optimize(*cb, n_kf, kfs, fixed, imu, n_pts, pts, nullptr, n_edges,
                                   static_cast<const oracle::lia::VisEdge*>(edges), n_imu,
                                   imu_edges, 0, 1.0, ko.data(), po.data(), out.data(), nullptr, H,
                                   b);
}

// Linearisation probe for the finite-difference tests: one visual edge's
// error (3), Jl (3x3) and Jp (3x6) at a key frame state and point.
extern "C" void orc_lia_vis_linearize(const orbgpu_imu_calib* cb, const orbgpu_imu_state* kf,
                                      const double* X, const void* edge, double* err, double* Jl,
                                      double* Jp) {
  using namespace oracle::lia;
  using namespace oracle::inertial;
  const Calib c = load_calib(*cb);
  const State s = load_state(*kf);
  const auto& e = *static_cast<const oracle::lia::VisEdge*>(edge);
  double Xc[3], l[3][3], p[3][6];
  vis_error(e, s, c, X, err, Xc);
  vis_jacobians(e, s, c, Xc, l, p);
  for (int r = 0; r < 3; ++r) {
    for (int k = 0; k < 3; ++k) Jl[3 * r + k] = l[r][k];
    for (int k = 0; k < 6; ++k) Jp[6 * r + k] = p[r][k];
  }
}
