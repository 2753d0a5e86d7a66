// ORACLE (test infrastructure only): restatement of Optimizer::PoseOptimization
// (src/solver/g2o_solver/optimizer.cc:762-1051) for the pinhole, non-fisheye
// case, with g2o's Levenberg-Marquardt (core/optimization_algorithm_levenberg.cpp
// :59-191), BlockSolver_6_3 without Schur (core/block_solver.hpp:530-638),
// LinearSolverDense (solvers/linear_solver_dense.h:56-104), unary edges
// (core/base_unary_edge.hpp:42-70), Huber (core/robust_kernel_impl.cpp:61-85),
// mono edge ORB_SLAM_FUSION::EdgeSE3ProjectXYZOnlyPose
// (optimizable_types.h:45-50, optimizable_types.cc:49-62, pinhole_model.cc:38-43,
// 71-80) and g2o::EdgeStereoSE3ProjectXYZOnlyPose (types_six_dof_expmap.h:
// 229-234, types_six_dof_expmap.cpp:318-381).  Sequential accumulation in edge
// insertion order, as g2o with OpenMP off.
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <limits>
#include <vector>

#include "g2o_math.h"

namespace oracle {

struct PoseObs {  // == orbgpu_pose_obs
  float Xw[3];
  float u, v, ur;  // ur < 0 -> monocular observation
  float inv_sigma2;
};

namespace {

struct Edge {
  bool stereo;
  double Xw[3];
  double obs[3];
  double info;   // information = I * inv_sigma2
  double delta;  // Huber delta (float sqrt(5.991) / sqrt(7.815))
  bool robust = true;
  int level = 0;
  double err[3] = {0, 0, 0};
};

struct Cam {
  double fx, fy, cx, cy, bf;
};

void compute_error(const Edge& e, const SE3& T, const Cam& c, double err[3]) {
  double p[3];
  T.map(e.Xw, p);
  if (!e.stereo) {
    err[0] = e.obs[0] - (c.fx * p[0] / p[2] + c.cx);
    err[1] = e.obs[1] - (c.fy * p[1] / p[2] + c.cy);
    err[2] = 0;
  } else {
    const float invz = (float)(1.0 / p[2]);  // `const float invz = 1.0f / z` (:320)
    const double u = p[0] * invz * c.fx + c.cx;
    const double v = p[1] * invz * c.fy + c.cy;
    err[0] = e.obs[0] - u;
    err[1] = e.obs[1] - v;
    err[2] = e.obs[2] - (u - c.bf * invz);
  }
}

double chi2_of(const Edge& e) {
  const int d = e.stereo ? 3 : 2;
  double s = 0;
  for (int i = 0; i < d; ++i) s += e.err[i] * (e.info * e.err[i]);
  return s;
}

// 2x6 / 3x6 Jacobian of the error w.r.t. the left-multiplied se3 increment.
void jacobian(const Edge& e, const SE3& T, const Cam& c, double J[3][6]) {
  double p[3];
  T.map(e.Xw, p);
  const double x = p[0], y = p[1], z = p[2];
  if (!e.stereo) {
    const double pj[2][3] = {{-(c.fx / z), -0.0, -(-c.fx * x / (z * z))},
                             {-0.0, -(c.fy / z), -(-c.fy * y / (z * z))}};
    const double S[3][6] = {{0, z, -y, 1, 0, 0}, {-z, 0, x, 0, 1, 0}, {y, -x, 0, 0, 0, 1}};
    for (int r = 0; r < 2; ++r)
      for (int k = 0; k < 6; ++k) J[r][k] = pj[r][0] * S[0][k] + pj[r][1] * S[1][k] + pj[r][2] * S[2][k];
    for (int k = 0; k < 6; ++k) J[2][k] = 0;
  } else {
    const double invz = 1.0 / z, invz2 = invz * invz;
    J[0][0] = x * y * invz2 * c.fx;
    J[0][1] = -(1 + (x * x * invz2)) * c.fx;
    J[0][2] = y * invz * c.fx;
    J[0][3] = -invz * c.fx;
    J[0][4] = 0;
    J[0][5] = x * invz2 * c.fx;
    J[1][0] = (1 + y * y * invz2) * c.fy;
    J[1][1] = -x * y * invz2 * c.fy;
    J[1][2] = -x * invz * c.fy;
    J[1][3] = 0;
    J[1][4] = -invz * c.fy;
    J[1][5] = y * invz2 * c.fy;
    J[2][0] = J[0][0] - c.bf * y * invz2;
    J[2][1] = J[0][1] + c.bf * x * invz2;
    J[2][2] = J[0][2];
    J[2][3] = J[0][3];
    J[2][4] = 0;
    J[2][5] = J[0][5] - c.bf * invz2;
  }
}

struct Lm {
  double lambda = -1, ni = 2;
  int nbad = 0;
};

// computeActiveErrors + activeRobustChi2.
double active_errors(std::vector<Edge>& E, const SE3& T, const Cam& c) {
  double chi = 0;
  for (Edge& e : E) {
    if (e.level != 0) continue;
    compute_error(e, T, c, e.err);
    const double c2 = chi2_of(e);
    if (e.robust) {
      double r0, r1;
      huber(c2, e.delta, r0, r1);
      chi += r0;
    } else {
      chi += c2;
    }
  }
  return chi;
}

enum { kOk, kTerminate };

// OptimizationAlgorithmLevenberg::solve (levenberg.cpp:59-168).
int lm_iteration(int it, std::vector<Edge>& E, SE3& T, const Cam& c, Lm& lm) {
  double cur = active_errors(E, T, c);
  const double ini = cur;

  double H[36] = {0}, b[6] = {0};
  for (Edge& e : E) {
    if (e.level != 0) continue;
    double J[3][6];
    jacobian(e, T, c, J);
    const int d = e.stereo ? 3 : 2;
    double w = 1.0;
    if (e.robust) {
      double r0;
      huber(chi2_of(e), e.delta, r0, w);
    }
    const double wi = w * e.info;
    for (int i = 0; i < 6; ++i) {
      double g = 0;
      for (int k = 0; k < d; ++k) g += J[k][i] * (e.info * e.err[k]);
      b[i] -= w * g;
      for (int j = 0; j < 6; ++j) {
        double h = 0;
        for (int k = 0; k < d; ++k) h += (J[k][i] * wi) * J[k][j];
        H[i * 6 + j] += h;
      }
    }
  }
  if (it == 0) {
    double mx = 0;
    for (int j = 0; j < 6; ++j) mx = std::max(std::fabs(H[j * 6 + j]), mx);
    lm.lambda = 1e-5 * mx;
    lm.ni = 2;
    lm.nbad = 0;
  }

  double rho = 0;
  int q = 0;
  do {
    const SE3 saved = T;
    double A[36], x[6];
    for (int i = 0; i < 36; ++i) A[i] = H[i];
    for (int j = 0; j < 6; ++j) A[j * 6 + j] += lm.lambda;
    const bool ok = ldlt_solve(A, 6, b, x);
    T = se3_exp(x).compose(T);
    double tmp = active_errors(E, T, c);
    if (!ok) tmp = std::numeric_limits<double>::max();
    rho = cur - tmp;
    double scale = 0;
    for (int j = 0; j < 6; ++j) scale += x[j] * (lm.lambda * x[j] + b[j]);
    scale += 1e-3;
    rho /= scale;
    if (rho > 0 && std::isfinite(tmp)) {
      double alpha = 1. - std::pow(2 * rho - 1, 3);
      alpha = std::min(alpha, 2. / 3.);
      lm.lambda *= std::max(1. / 3., alpha);
      lm.ni = 2;
      cur = tmp;
    } else {
      lm.lambda *= lm.ni;
      lm.ni *= 2;
      T = saved;
    }
    ++q;
  } while (rho < 0 && q < 10);

  if (q == 10 || rho == 0) return kTerminate;
  if ((ini - cur) * 1e3 < ini)
    lm.nbad++;
  else
    lm.nbad = 0;
  if (lm.nbad >= 3) return kTerminate;
  return kOk;
}

}  // namespace

// Returns the inlier count (0 when fewer than 3 correspondences, pose
// untouched).  pose = (qx, qy, qz, qw, tx, ty, tz), float like Sophus::SE3f.
int pose_optimization(const float cam[5], const float pose_in[7], const PoseObs* obs, int n,
                      float pose_out[7], uint8_t* outlier, double pose_out_d[7]) {
  for (int i = 0; i < 7; ++i) pose_out[i] = pose_in[i];
  if (n < 3) return 0;
  const Cam c{cam[0], cam[1], cam[2], cam[3], cam[4]};
  const float delta_mono = std::sqrt(5.991), delta_stereo = std::sqrt(7.815);

  std::vector<Edge> E(n);
  for (int i = 0; i < n; ++i) {
    Edge& e = E[i];
    e.stereo = obs[i].ur >= 0;
    for (int k = 0; k < 3; ++k) e.Xw[k] = obs[i].Xw[k];
    e.obs[0] = obs[i].u;
    e.obs[1] = obs[i].v;
    e.obs[2] = e.stereo ? obs[i].ur : 0.0;
    e.info = obs[i].inv_sigma2;
    e.delta = e.stereo ? delta_stereo : delta_mono;
    outlier[i] = 0;
  }

  SE3 init;
  init.r.x = pose_in[0];
  init.r.y = pose_in[1];
  init.r.z = pose_in[2];
  init.r.w = pose_in[3];
  init.t[0] = pose_in[4];
  init.t[1] = pose_in[5];
  init.t[2] = pose_in[6];

  const float chi2_mono = 5.991f, chi2_stereo = 7.815f;
  SE3 T = init;
  int nbad = 0;
  for (int it = 0; it < 4; ++it) {
    T = init;
    Lm lm;
    for (int i = 0; i < 10; ++i)
      if (lm_iteration(i, E, T, c, lm) != kOk) break;

    nbad = 0;
    for (int i = 0; i < n; ++i) {
      Edge& e = E[i];
      if (outlier[i]) compute_error(e, T, c, e.err);
      const float chi2 = (float)chi2_of(e);
      if (chi2 > (e.stereo ? chi2_stereo : chi2_mono)) {
        outlier[i] = 1;
        e.level = 1;
        nbad++;
      } else {
        outlier[i] = 0;
        e.level = 0;
      }
      if (it == 2) e.robust = false;
    }
    if (n < 10) break;
  }

  const double out[7] = {T.r.x, T.r.y, T.r.z, T.r.w, T.t[0], T.t[1], T.t[2]};
  for (int i = 0; i < 7; ++i) {
    pose_out[i] = (float)out[i];
    if (pose_out_d) pose_out_d[i] = out[i];
  }
  // Sophus::SE3f(Quaternionf, Vector3f) re-normalises the cast quaternion.
  const float qn = std::sqrt(pose_out[0] * pose_out[0] + pose_out[1] * pose_out[1] +
                             pose_out[2] * pose_out[2] + pose_out[3] * pose_out[3]);
  for (int i = 0; i < 4; ++i) pose_out[i] /= qn;
  return n - nbad;
}

}  // namespace oracle

extern "C" int orc_pose_opt(const float cam[5], const float pose_in[7], const float* obs, int n,
                            float pose_out[7], uint8_t* outlier, double* pose_out_d) {
  return oracle::pose_optimization(cam, pose_in, reinterpret_cast<const oracle::PoseObs*>(obs), n,
                                   pose_out, outlier, pose_out_d);
}
