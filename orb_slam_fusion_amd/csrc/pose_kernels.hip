// gfx950 PoseOptimization: one 256-thread workgroup runs a whole problem --
// Optimizer::PoseOptimization (optimizer.cc:762-1051): 4 outlier-rejection
// rounds x g2o Levenberg-Marquardt (optimization_algorithm_levenberg.cpp:59-168)
// over unary SE3 edges, dense 6x6 LDLT.  The working set (< 40 KB) stays on
// chip; edges are swept by all lanes, per-sweep sums use a fixed reduction
// tree (deterministic), the 6x6 solve and the se3 exp run on lane 0.  The
// pass is latency-bound (40+ dependent sweeps), so problems are batched one
// workgroup each.
//
// Per-edge errors are not stored: g2o's classification reads the error of the
// last computeActiveErrors() (possibly at a rejected trial pose), so the
// kernel remembers that pose and recomputes -- bit-identical values.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pose_math_dev.h"

namespace orbgpu {

struct PoseObsDev {
  float Xw[3];
  float u, v, ur;
  float inv_sigma2;
};

struct CamDev {
  double fx, fy, cx, cy, bf;
};

constexpr int kPoseThreads = 256;

__device__ __forceinline__ void edge_error(const PoseObsDev& o, const Se3& T, const CamDev& c,
                                           double e[3], bool& stereo) {
  const double X[3] = {o.Xw[0], o.Xw[1], o.Xw[2]};
  double p[3];
  se3_map(T, X, p);
  stereo = o.ur >= 0.f;
  if (!stereo) {  // EdgeSE3ProjectXYZOnlyPose + Pinhole::Project
    e[0] = (double)o.u - (c.fx * p[0] / p[2] + c.cx);
    e[1] = (double)o.v - (c.fy * p[1] / p[2] + c.cy);
    e[2] = 0;
  } else {  // EdgeStereoSE3ProjectXYZOnlyPose::cam_project (float invz)
    const float invz = (float)(1.0 / p[2]);
    const double u = p[0] * (double)invz * c.fx + c.cx;
    const double v = p[1] * (double)invz * c.fy + c.cy;
    e[0] = (double)o.u - u;
    e[1] = (double)o.v - v;
    e[2] = (double)o.ur - (u - c.bf * (double)invz);
  }
}

__device__ __forceinline__ double edge_chi2(const double e[3], double info, bool stereo) {
  double s = e[0] * (info * e[0]) + e[1] * (info * e[1]);
  if (stereo) s += e[2] * (info * e[2]);
  return s;
}

__device__ __forceinline__ void edge_jacobian(const PoseObsDev& o, const Se3& T, const CamDev& c,
                                              bool stereo, double J[3][6]) {
  const double X[3] = {o.Xw[0], o.Xw[1], o.Xw[2]};
  double p[3];
  se3_map(T, X, p);
  const double x = p[0], y = p[1], z = p[2];
  if (!stereo) {
    const double pj00 = -(c.fx / z), pj02 = -(-c.fx * x / (z * z));
    const double pj11 = -(c.fy / z), pj12 = -(-c.fy * y / (z * z));
    const double S[3][6] = {{0, z, -y, 1, 0, 0}, {-z, 0, x, 0, 1, 0}, {y, -x, 0, 0, 0, 1}};
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      J[0][k] = pj00 * S[0][k] + -0.0 * S[1][k] + pj02 * S[2][k];
      J[1][k] = -0.0 * S[0][k] + pj11 * S[1][k] + pj12 * S[2][k];
      J[2][k] = 0;
    }
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

// Block-wide sum of NV doubles per thread (fixed tree: wave butterfly, then
// the 4 wave partials in order).  Result broadcast to every thread.
template <int NV>
__device__ __forceinline__ void block_sum_d(double (&v)[NV], double* red) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    double x = v[k];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    v[k] = x;
  }
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < NV; ++k) red[wave * NV + k] = v[k];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = ((red[k] + red[NV + k]) + red[2 * NV + k]) + red[3 * NV + k];
  __syncthreads();
}

__device__ __forceinline__ int block_sum_i(int v, int* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  const int r = red[0] + red[1] + red[2] + red[3];
  __syncthreads();
  return r;
}

struct PoseShared {
  double red[4 * 27];
  int ired[4];
};

// Robust chi2 of the active (level-0) edges at pose T.
__device__ double active_chi(const PoseObsDev* __restrict__ obs, const uint8_t* level, int n,
                             const Se3& T, const CamDev& c, bool robust, double dmono,
                             double dstereo, PoseShared& sh) {
  double acc[1] = {0.0};
  for (int i = threadIdx.x; i < n; i += kPoseThreads) {
    if (level[i]) continue;
    const PoseObsDev o = obs[i];
    double e[3];
    bool st;
    edge_error(o, T, c, e, st);
    const double c2 = edge_chi2(e, (double)o.inv_sigma2, st);
    if (robust) {
      double r0, r1;
      huber_rho(c2, st ? dstereo : dmono, r0, r1);
      acc[0] += r0;
    } else {
      acc[0] += c2;
    }
  }
  block_sum_d<1>(acc, sh.red);
  return acc[0];
}

__global__ __launch_bounds__(kPoseThreads) void k_pose_opt(
    CamDev cam, const float* __restrict__ pose_in, const PoseObsDev* __restrict__ obs_all,
    const int* __restrict__ nobs, int obs_stride, float* __restrict__ pose_out,
    uint8_t* __restrict__ outlier_all, int* __restrict__ inliers, double* __restrict__ pose_out_d) {
  __shared__ PoseShared sh;
  const int p = blockIdx.x, t = threadIdx.x;
  const int n = nobs[p];
  const PoseObsDev* obs = obs_all + (size_t)p * obs_stride;
  uint8_t* level = outlier_all + (size_t)p * obs_stride;
  const float* pin = pose_in + 7 * p;
  if (n < 3) {  // optimizer.cc:951
    if (t < 7) pose_out[7 * p + t] = pin[t];
    if (t == 0) inliers[p] = 0;
    return;
  }
  for (int i = t; i < n; i += kPoseThreads) level[i] = 0;
  Se3 init{0, 0, 0, 1, {0, 0, 0}};
  init.qx = pin[0];
  init.qy = pin[1];
  init.qz = pin[2];
  init.qw = pin[3];
  init.t[0] = pin[4];
  init.t[1] = pin[5];
  init.t[2] = pin[6];
  const double dmono = (double)(float)sqrt(5.991);  // `const float deltaMono = sqrt(5.991)`
  const double dstereo = (double)(float)sqrt(7.815);
  bool robust = true;
  int nbad_round = 0;
  Se3 T = init;
  __syncthreads();

  for (int it = 0; it < 4; ++it) {
    T = init;
    Se3 Teval = init;
    double lambda = 0, ni = 2;
    int nbad = 0;
    for (int iter = 0; iter < 10; ++iter) {
      // computeActiveErrors + activeRobustChi2 at T
      double cur = active_chi(obs, level, n, T, cam, robust, dmono, dstereo, sh);
      Teval = T;
      const double ini = cur;
      // BlockSolver::buildSystem: H (lower triangle, 21) and b (6)
      double hb[27];
#pragma unroll
      for (int k = 0; k < 27; ++k) hb[k] = 0;
      for (int i = t; i < n; i += kPoseThreads) {
        if (level[i]) continue;
        const PoseObsDev o = obs[i];
        double e[3];
        bool st;
        edge_error(o, T, cam, e, st);
        const double info = (double)o.inv_sigma2;
        double w = 1.0;
        if (robust) {
          double r0;
          huber_rho(edge_chi2(e, info, st), st ? dstereo : dmono, r0, w);
        }
        double J[3][6];
        edge_jacobian(o, T, cam, st, J);
        const double wi = w * info;
        const int d = st ? 3 : 2;
        int hk = 0;
#pragma unroll
        for (int r = 0; r < 6; ++r) {
          double g = J[0][r] * (info * e[0]) + J[1][r] * (info * e[1]);
          if (d == 3) g += J[2][r] * (info * e[2]);
          hb[21 + r] -= w * g;
#pragma unroll
          for (int q = 0; q <= r; ++q) {
            double h = (J[0][r] * wi) * J[0][q] + (J[1][r] * wi) * J[1][q];
            if (d == 3) h += (J[2][r] * wi) * J[2][q];
            hb[hk++] += h;
          }
        }
      }
      block_sum_d<27>(hb, sh.red);
      if (iter == 0) {  // computeLambdaInit: tau * max diag
        double mx = 0;
        int dk = 0;
#pragma unroll
        for (int r = 0; r < 6; ++r) {
          dk += r;
          mx = fmax(fabs(hb[dk + r]), mx);
        }
        lambda = 1e-5 * mx;
        ni = 2;
        nbad = 0;
      }
      double rho = 0;
      int q = 0;
      do {
        // every lane solves the (identical) 6x6 system: no broadcast barrier
        double A[6][6], bb[6], x[6];
        {
          int hk = 0;
#pragma unroll
          for (int r = 0; r < 6; ++r) {
#pragma unroll
            for (int c2 = 0; c2 <= r; ++c2) A[r][c2] = A[c2][r] = hb[hk++];
            bb[r] = hb[21 + r];
          }
        }
#pragma unroll
        for (int j = 0; j < 6; ++j) A[j][j] += lambda;
        const bool ok = ldlt6_solve(A, bb, x);
        const Se3 Tn = se3_compose(se3_exp(x), T);
        double tmp = active_chi(obs, level, n, Tn, cam, robust, dmono, dstereo, sh);
        Teval = Tn;
        if (!ok) tmp = 1.79769313486231570815e+308;
        rho = cur - tmp;
        double scale = 0;
#pragma unroll
        for (int j = 0; j < 6; ++j) scale += x[j] * (lambda * x[j] + hb[21 + j]);
        scale += 1e-3;
        rho /= scale;
        if (rho > 0 && isfinite(tmp)) {
          double alpha = 1. - pow(2 * rho - 1, 3);
          alpha = fmin(alpha, 2. / 3.);
          lambda *= fmax(1. / 3., alpha);
          ni = 2;
          cur = tmp;
          T = Tn;
        } else {
          lambda *= ni;
          ni *= 2;
        }
        ++q;
      } while (rho < 0 && q < 10);
      if (q == 10 || rho == 0) break;
      if ((ini - cur) * 1e3 < ini)
        nbad++;
      else
        nbad = 0;
      if (nbad >= 3) break;
    }

    // classify (optimizer.cc:966-1037): level-1 edges recompute at T, level-0
    // edges keep the error of the last sweep (at Teval)
    int bad = 0;
    for (int i = t; i < n; i += kPoseThreads) {
      const PoseObsDev o = obs[i];
      double e[3];
      bool st;
      edge_error(o, level[i] ? T : Teval, cam, e, st);
      const float chi2 = (float)edge_chi2(e, (double)o.inv_sigma2, st);
      const bool out = chi2 > (st ? 7.815f : 5.991f);
      level[i] = out ? 1 : 0;
      bad += out;
    }
    nbad_round = block_sum_i(bad, sh.ired);
    if (it == 2) robust = false;
    if (n < 10) break;
  }

  if (t == 0) {
    const double o[7] = {T.qx, T.qy, T.qz, T.qw, T.t[0], T.t[1], T.t[2]};
    float f[7];
    for (int i = 0; i < 7; ++i) {
      f[i] = (float)o[i];
      if (pose_out_d) pose_out_d[7 * p + i] = o[i];
    }
    const float qn = sqrtf(f[0] * f[0] + f[1] * f[1] + f[2] * f[2] + f[3] * f[3]);
    for (int i = 0; i < 4; ++i) f[i] /= qn;
    for (int i = 0; i < 7; ++i) pose_out[7 * p + i] = f[i];
    inliers[p] = n - nbad_round;
  }
}

hipError_t launch_pose_opt(const double cam[5], const float* d_pose_in, const void* d_obs,
                           const int* d_nobs, int obs_stride, int n_problems, float* d_pose_out,
                           uint8_t* d_outlier, int* d_inliers, double* d_pose_out_d,
                           hipStream_t st) {
  CamDev c{cam[0], cam[1], cam[2], cam[3], cam[4]};
  hipLaunchKernelGGL(k_pose_opt, dim3(n_problems), dim3(kPoseThreads), 0, st, c, d_pose_in,
                     reinterpret_cast<const PoseObsDev*>(d_obs), d_nobs, obs_stride, d_pose_out,
                     d_outlier, d_inliers, d_pose_out_d);
  return hipGetLastError();
}

}  // namespace orbgpu
