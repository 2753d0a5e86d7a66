// gfx950 LocalBundleAdjustment (Optimizer::LocalBundleAdjustment,
// src/solver/g2o_solver/optimizer.cc:1127-1441): g2o Levenberg-Marquardt over
// SE3 keyframe poses and marginalized XYZ points (BlockSolver_6_3 Schur
// complement, core/block_solver.hpp:364-514), fp64 throughout.
//
// The LM loop itself runs on the device (lba_launch.h): every kernel reads
// the LbaCtrl state at entry and returns when its stage is not due, and the
// single thread that closes a stage (the last block to finish it) takes the
// LM decision of optimization_algorithm_levenberg.cpp:59-168 in place.  One
// LM trial is five launches:
//
//   k_lba_linearize  thread / edge      Jacobians + per-edge Hessian terms  } once per
//   k_lba_sums       block / pose,      Hpp / bp and Hll / bl sums,          } iteration
//                    thread / point     lambda init (computeLambdaInit)      }
//   k_lba_schur      block / pose pair  S_ij = [i=j]Hpp_i - sum Hpl_i Dinv Hpl_j^T, b_s
//   k_lba_solve      one block          (S + lambda I) = L D L^T by 16 x 16 tiles:
//                                       diagonal tile in registers, panel and
//                                       trailing update as v_mfma_f64_16x16x4
//   k_lba_trial      thread / edge      back-substitution, trial state, errors,
//                                       robust chi2 and computeScale -> decision
//
// LocalInertialBA (optimizer.cc:2440-2826) runs on the same kernels with the
// kModelImu key frame (lba_launch.h): ImuCamPose state, body-frame visual
// Jacobians (EdgeMono / EdgeStereo, g2o_types.cc:334-415), 15 reduced-system
// rows per free key frame, and the IMU links (EdgeInertial + EdgeGyroRW +
// EdgeAccRW, no points) evaluated a block per link (lia_link) by extra blocks
// of the begin / linearize / trial launches, and added to the camera-side
// system (lia_assemble_entry, in k_lba_sums) before the solve.
//
// Sums inside a launch have a fixed order (per-thread loops in edge order,
// fixed trees, block partials summed by the last block in block order), so
// results are reproducible run to run.  The reduction orders differ from
// g2o's sequential ones: parity is by tolerance (tests/test_gpu_lba.py).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "lba_launch.h"
#include "lds_optin.h"
#include "pose_math_dev.h"

// fp64 solver TU (tolerance parity, not bit parity): products may fuse.
#pragma clang fp contract(fast)

#include "imu_math_dev.h"

namespace orbgpu {

namespace {

constexpr int kThreads = 256;
constexpr int kMaxKfLds = 1024;  // trial poses staged in LDS up to this many keyframes
constexpr int kMaxKfImuLds = 128;  // kModelImu trial states (33 doubles) likewise
constexpr double kTau = 1e-5;    // OptimizationAlgorithmLevenberg _tau

typedef double d4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ Se3 load_pose(const double* p) {
  Se3 T;
  T.qx = p[0];
  T.qy = p[1];
  T.qz = p[2];
  T.qw = p[3];
  T.t[0] = p[4];
  T.t[1] = p[5];
  T.t[2] = p[6];
  return T;
}

__device__ __forceinline__ void store_pose(const Se3& T, double* p) {
  p[0] = T.qx;
  p[1] = T.qy;
  p[2] = T.qz;
  p[3] = T.qw;
  p[4] = T.t[0];
  p[5] = T.t[1];
  p[6] = T.t[2];
}

// error of one edge (EdgeSE3ProjectXYZ, optimizable_types.h:105-125 /
// EdgeStereoSE3ProjectXYZ, types_six_dof_expmap.cpp:174-257); returns
// isDepthPositive on the same state
__device__ __forceinline__ bool lba_error(const LbaEdgeDev& e, const Se3& T, const double X[3],
                                          const LbaCamDev& c, double err[3]) {
  double p[3];
  se3_map(T, X, p);
  if (e.ur < 0.f) {
    const RecipF64 rz = recip_f64(p[2]);  // (f64_math_dev.h: the IEEE quotients)
    err[0] = (double)e.u - (div_by(c.fx * p[0], rz) + c.cx);
    err[1] = (double)e.v - (div_by(c.fy * p[1], rz) + c.cy);
    err[2] = 0;
  } else {
    const float invz = 1.0f / (float)p[2];
    const double u = p[0] * (double)invz * c.fx + c.cx;
    const double v = p[1] * (double)invz * c.fy + c.cy;
    err[0] = (double)e.u - u;
    err[1] = (double)e.v - v;
    err[2] = (double)e.ur - (u - c.bf * (double)invz);
  }
  return p[2] > 0.0;
}

__device__ __forceinline__ double lba_chi2(const LbaEdgeDev& e, const double err[3]) {
  const double info = (double)e.inv_sigma2;
  double s = err[0] * (info * err[0]) + err[1] * (info * err[1]);
  if (e.ur >= 0.f) s += err[2] * (info * err[2]);
  return s;
}

__device__ __forceinline__ double lba_delta(const LbaEdgeDev& e) {
  return e.ur < 0.f ? (double)(float)sqrt(5.991) : (double)(float)sqrt(7.815);
}

__device__ __forceinline__ void lba_jacobians(const LbaEdgeDev& e, const Se3& T, const double X[3],
                                              const LbaCamDev& c, double Jl[3][3], double Jp[3][6]) {
  double p[3];
  se3_map(T, X, p);
  const double x = p[0], y = p[1], z = p[2];
  double R[3][3];
  {
    const double e0[3] = {1, 0, 0}, e1[3] = {0, 1, 0}, e2[3] = {0, 0, 1};
    double c0[3], c1[3], c2[3];
    quat_rot(T.qx, T.qy, T.qz, T.qw, e0, c0);
    quat_rot(T.qx, T.qy, T.qz, T.qw, e1, c1);
    quat_rot(T.qx, T.qy, T.qz, T.qw, e2, c2);
    for (int r = 0; r < 3; ++r) {
      R[r][0] = c0[r];
      R[r][1] = c1[r];
      R[r][2] = c2[r];
    }
  }
  // one reciprocal per denominator (z, z^2) for the IEEE quotients below
  const RecipF64 rz = recip_f64(z), rzz = recip_f64(z * z);
  if (e.ur < 0.f) {  // optimizable_types.cc:134-155
    const double pj[2][3] = {{-div_by(c.fx, rz), 0.0, -div_by(-c.fx * x, rzz)},
                             {0.0, -div_by(c.fy, rz), -div_by(-c.fy * y, rzz)}};
    const double S[3][6] = {{0, z, -y, 1, 0, 0}, {-z, 0, x, 0, 1, 0}, {y, -x, 0, 0, 0, 1}};
#pragma unroll
    for (int r = 0; r < 2; ++r) {
#pragma unroll
      for (int k = 0; k < 3; ++k) Jl[r][k] = pj[r][0] * R[0][k] + pj[r][1] * R[1][k] + pj[r][2] * R[2][k];
#pragma unroll
      for (int k = 0; k < 6; ++k) Jp[r][k] = pj[r][0] * S[0][k] + pj[r][1] * S[1][k] + pj[r][2] * S[2][k];
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) Jl[2][k] = 0;
#pragma unroll
    for (int k = 0; k < 6; ++k) Jp[2][k] = 0;
  } else {  // types_six_dof_expmap.cpp:211-257
    const double fx = c.fx, fy = c.fy, bf = c.bf;  // q / z and q / z_2 by div_by
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      Jl[0][k] = div_by(-fx * R[0][k], rz) + div_by(fx * x * R[2][k], rzz);
      Jl[1][k] = div_by(-fy * R[1][k], rz) + div_by(fy * y * R[2][k], rzz);
      Jl[2][k] = Jl[0][k] - div_by(bf * R[2][k], rzz);
    }
    Jp[0][0] = div_by(x * y, rzz) * fx;
    Jp[0][1] = -(1 + div_by(x * x, rzz)) * fx;
    Jp[0][2] = div_by(y, rz) * fx;
    Jp[0][3] = div_by(-1., rz) * fx;
    Jp[0][4] = 0;
    Jp[0][5] = div_by(x, rzz) * fx;
    Jp[1][0] = (1 + div_by(y * y, rzz)) * fy;
    Jp[1][1] = div_by(-x * y, rzz) * fy;
    Jp[1][2] = div_by(-x, rz) * fy;
    Jp[1][3] = 0;
    Jp[1][4] = div_by(-1., rz) * fy;
    Jp[1][5] = div_by(y, rzz) * fy;
    Jp[2][0] = Jp[0][0] - div_by(bf * y, rzz);
    Jp[2][1] = Jp[0][1] + div_by(bf * x, rzz);
    Jp[2][2] = Jp[0][2];
    Jp[2][3] = Jp[0][3];
    Jp[2][4] = 0;
    Jp[2][5] = Jp[0][5] - div_by(bf, rzz);
  }
}

// ---- key-frame models --------------------------------------------------------
static_assert(sizeof(LiaCalibDev) == sizeof(CalibD), "LiaCalibDev == CalibD");

__device__ __forceinline__ CalibD calib_of(const LbaArgs& a) {
  CalibD c;
  c.fx = a.icb.fx;
  c.fy = a.icb.fy;
  c.cx = a.icb.cx;
  c.cy = a.icb.cy;
  c.bf = a.icb.bf;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    c.Rcb[i] = a.icb.Rcb[i];
    c.Rbc[i] = a.icb.Rbc[i];
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    c.tcb[i] = a.icb.tcb[i];
    c.tbc[i] = a.icb.tbc[i];
  }
  return c;
}

// camera point Xc = Rcw X + tcw of an ImuCamPose state (Rcw at +12, tcw at +21)
__device__ __forceinline__ void imu_cam_point(const double* ks, const double X[3], double Xc[3]) {
  const double* R = ks + 12;
  const double* t = ks + 21;
#pragma unroll
  for (int r = 0; r < 3; ++r) Xc[r] = R[3 * r] * X[0] + R[3 * r + 1] * X[1] + R[3 * r + 2] * X[2] + t[r];
}

// Visual edge error at key-frame state ks (7 or 33 doubles); returns
// isDepthPositive on the same state.  kModelImu: EdgeMono / EdgeStereo
// (ImuCamPose::Project / ProjectStereo, g2o_types.cc:171-190; the stereo
// invZ in double).
template <int M>
__device__ __forceinline__ bool vis_error(const LbaArgs& a, const LbaEdgeDev& e, const double* ks,
                                          const double X[3], double err[3]) {
  if constexpr (M == kModelSe3) {
    return lba_error(e, load_pose(ks), X, a.cam, err);
  } else {
    double Xc[3];
    imu_cam_point(ks, X, Xc);
    const RecipF64 rz = recip_f64(Xc[2]);
    const double u = div_by(a.cam.fx * Xc[0], rz) + a.cam.cx;
    const double v = div_by(a.cam.fy * Xc[1], rz) + a.cam.cy;
    err[0] = (double)e.u - u;
    err[1] = (double)e.v - v;
    err[2] = e.ur >= 0.f ? (double)e.ur - (u - a.cam.bf * div_by(1.0, rz)) : 0.0;
    return Xc[2] > 0.0;
  }
}

// Visual edge Jacobians (point Jl, pose Jp).  kModelImu: Jl = -proj_jac Rcw,
// Jp = proj_jac Rcb SE3deriv(Xb) (g2o_types.cc:334-415); mono rows 2 = 0.
template <int M>
__device__ __forceinline__ void vis_jacobians(const LbaArgs& a, const LbaEdgeDev& e, const double* ks,
                                              const double X[3], double Jl[3][3], double Jp[3][6]) {
  if constexpr (M == kModelSe3) {
    lba_jacobians(e, load_pose(ks), X, a.cam, Jl, Jp);
  } else {
    const LiaCalibDev& c = a.icb;
    double Xc[3];
    imu_cam_point(ks, X, Xc);
    const double* R = ks + 12;
    const bool st = e.ur >= 0.f;
    const RecipF64 rz = recip_f64(Xc[2]), rzz = recip_f64(Xc[2] * Xc[2]);
    double pj[3][3] = {{div_by(c.fx, rz), 0, div_by(-c.fx * Xc[0], rzz)},
                       {0, div_by(c.fy, rz), div_by(-c.fy * Xc[1], rzz)},
                       {0, 0, 0}};
    if (st) {
      pj[2][0] = pj[0][0];
      pj[2][1] = pj[0][1];
      pj[2][2] = pj[0][2] + c.bf * div_by(1.0, rzz);
    }
    double Xb[3];
#pragma unroll
    for (int r = 0; r < 3; ++r)
      Xb[r] = c.Rbc[3 * r] * Xc[0] + c.Rbc[3 * r + 1] * Xc[1] + c.Rbc[3 * r + 2] * Xc[2] + c.tbc[r];
    const double x = Xb[0], y = Xb[1], z = Xb[2];
    const double S[3][6] = {{0, z, -y, 1, 0, 0}, {-z, 0, x, 0, 1, 0}, {y, -x, 0, 0, 0, 1}};
#pragma unroll
    for (int r = 0; r < 3; ++r) {
#pragma unroll
      for (int k = 0; k < 3; ++k) Jl[r][k] = -(pj[r][0] * R[k] + pj[r][1] * R[3 + k] + pj[r][2] * R[6 + k]);
      double PR[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) PR[k] = pj[r][0] * c.Rcb[k] + pj[r][1] * c.Rcb[3 + k] + pj[r][2] * c.Rcb[6 + k];
#pragma unroll
      for (int k = 0; k < 6; ++k) Jp[r][k] = PR[0] * S[0][k] + PR[1] * S[1][k] + PR[2] * S[2][k];
    }
  }
}

// (Hll + lambda I)^-1 by cofactors (Eigen compute_inverse_size3); returns the
// determinant (0 = singular landmark block: the trial fails).
__device__ __forceinline__ double inv3_lambda(const double* __restrict__ h, double lambda, double Di[9]) {
  double A[3][3];
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c) A[r][c] = h[3 * r + c] + (r == c ? lambda : 0.0);
  const double c00 = A[1][1] * A[2][2] - A[1][2] * A[2][1];
  const double c10 = A[1][2] * A[2][0] - A[1][0] * A[2][2];
  const double c20 = A[1][0] * A[2][1] - A[1][1] * A[2][0];
  const double det = A[0][0] * c00 + A[0][1] * c10 + A[0][2] * c20;
  const double id = det != 0 ? 1.0 / det : 0.0;
  Di[0] = c00 * id;
  Di[3] = c10 * id;
  Di[6] = c20 * id;
  Di[1] = (A[0][2] * A[2][1] - A[0][1] * A[2][2]) * id;
  Di[4] = (A[0][0] * A[2][2] - A[0][2] * A[2][0]) * id;
  Di[7] = (A[0][1] * A[2][0] - A[0][0] * A[2][1]) * id;
  Di[2] = (A[0][1] * A[1][2] - A[0][2] * A[1][1]) * id;
  Di[5] = (A[0][2] * A[1][0] - A[0][0] * A[1][2]) * id;
  Di[8] = (A[0][0] * A[1][1] - A[0][1] * A[1][0]) * id;
  return det;
}

// DPP lane move of a double (two 32-bit halves); lanes whose source is out of
// range or whose row is masked off read 0.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ double dpp_f64(double v) {
  // full row mask: bound_ctrl reads 0 for out-of-range sources, so the
  // destination needs no zeroed old value (one v_mov_b32_dpp per half)
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, ROW_MASK, 0xf, ROW_MASK == 0xf);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, ROW_MASK, 0xf, ROW_MASK == 0xf);
  return __hiloint2double(hi, lo);
}

// The wave's own LDS writes visible to its other lanes.
__device__ __forceinline__ void wave_lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// Fixed-tree sum of K doubles over a 256-thread block; valid in every thread.
template <int K>
__device__ __forceinline__ void block_sum(double (&v)[K], double* red /* 4 * K */) {
#pragma unroll
  for (int k = 0; k < K; ++k) {
    double x = v[k];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    v[k] = x;
  }
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int k = 0; k < K; ++k) red[K * (threadIdx.x >> 6) + k] = v[k];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] = ((red[k] + red[K + k]) + red[2 * K + k]) + red[3 * K + k];
  __syncthreads();
}

// Last-block-done ticket (cdna_hip_programming.md §6 Guideline 16, counter
// form): every storing wave drains, the block joins, lane 0 releases at agent
// scope and takes a ticket; the last block acquires before reading the other
// blocks' stores.  The counter resets itself for the next launch.
__device__ __forceinline__ bool last_block(unsigned* counter) {
  __shared__ int last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned t = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = t == gridDim.x - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  return last != 0;
}

// The same ticket for launches whose cross-block payload (what the last
// block reads: the partials, pose quarters, link chi2s) is stored
// write-through (st_wt: agent-scope relaxed atomic stores, sc1, straight to
// L2) and drained before the barrier -- no release fence per block (its L2
// write-back cost each block several microseconds at the kernel's tail).
// The last block still acquires (an L1 / L2 invalidate) before reading.
__device__ __forceinline__ void st_wt(double* p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), (unsigned long long)__double_as_longlong(v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
#ifndef ORB_LBA_WT_TICKET
#define ORB_LBA_WT_TICKET 1  // 0: the release-fence ticket everywhere (A/B)
#endif
__device__ __forceinline__ bool last_block_wt(unsigned* counter) {
#if !ORB_LBA_WT_TICKET
  return last_block(counter);
#else
  __shared__ int last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = t == gridDim.x - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  return last != 0;
#endif
}

// Sum of K per-block partials (partials[K * b + k]) in a fixed tree, by the
// last block; valid in every thread.
template <int K>
__device__ __forceinline__ void sum_partials(const double* partials, int nb, double (&out)[K], double* red) {
  double v[K];
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] = 0;
  for (int b = threadIdx.x; b < nb; b += kThreads)
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] += partials[K * b + k];
  block_sum<K>(v, red);
#pragma unroll
  for (int k = 0; k < K; ++k) out[k] = v[k];
}

__device__ __forceinline__ void publish(const LbaArgs& a, const LbaCtrl& c) {
  const unsigned long long w = ((unsigned long long)(c.done ? 1u : 0u) << 32) | (unsigned)c.trials;
  __hip_atomic_store(&a.host->progress, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ int host_stop(const LbaArgs& a) {
  return __hip_atomic_load(&a.host->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
}

// ---- the LM decisions (one thread) --------------------------------------
// start of optimize(): computeActiveErrors at the initial state
__device__ void ctl_init(const LbaArgs& a, double chi, int stop) {
  LbaCtrl& c = *a.ctrl;
  c.cur = chi;
  c.chi_init = chi;
  c.ini = chi;
  c.last = chi;
  c.it = 0;
  c.q = 0;
  c.nbad = 0;
  c.state = 0;
  c.iters_done = 0;
  c.trials = 0;
  c.need_build = 1;
  c.lin_state = 0;  // k_lba_begin wrote state 0's per-edge terms
  c.stopped = stop;
  // SparseOptimizer::optimize: for (i < iterations && !terminate() ...)
  c.done = (c.max_iters <= 0 || stop) ? 1 : 0;
  publish(a, c);
}

// computeLambdaInit (optimization_algorithm_levenberg.cpp:180-191)
__device__ void ctl_lambda(const LbaArgs& a, double maxdiag) {
  LbaCtrl& c = *a.ctrl;
  c.lambda = c.user_lambda > 0 ? c.user_lambda : kTau * maxdiag;
  c.ni = 2;
  c.nbad = 0;
}

// one trial's verdict (optimization_algorithm_levenberg.cpp:118-167)
__device__ void ctl_decide(const LbaArgs& a, double chi_trial, double scale_l, int bad, int stop) {
  LbaCtrl& c = *a.ctrl;
  c.last = chi_trial;
  double tmp = chi_trial;
  if (bad) tmp = 1.7976931348623157e308;  // !ok2 -> tempChi = max
  double rho = c.cur - tmp;
  const double scale = a.scal[0] + scale_l + 1e-3;
  rho /= scale;
  if (rho > 0 && isfinite(tmp)) {
    double alpha = 1. - cube(2 * rho - 1);
    alpha = fmin(alpha, 2. / 3.);
    c.lambda *= fmax(1. / 3., alpha);
    c.ni = 2;
    c.cur = tmp;
    c.state ^= 1;  // discardTop: the trial state becomes current
    c.lin_state = c.state;  // its per-edge terms were written by the trial
  } else {
    c.lambda *= c.ni;  // pop: the current state stays
    c.ni *= 2;
  }
  ++c.q;
  ++c.trials;
  c.stopped = stop;
  if (!(rho < 0 && c.q < 10 && !stop)) {  // the do-while ends: the iteration is over
    ++c.iters_done;
    int done = 0;
    if (c.q == 10 || rho == 0) {
      done = 1;  // Terminate
    } else {
      if ((c.ini - c.cur) * 1e3 < c.ini)
        c.nbad++;
      else
        c.nbad = 0;
      if (c.nbad >= 3) done = 1;
    }
    ++c.it;
    if (c.it >= c.max_iters || stop) done = 1;  // the for loop's bound and terminate()
    c.done = done;
    c.need_build = done ? 0 : 1;
  }
  publish(a, c);
}

// ---- computeActiveErrors at the initial state ----------------------------
__device__ __forceinline__ void load_state(StateD& s, const double* p) {
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    s.Rwb[i] = p[i];
    s.Rcw[i] = p[12 + i];
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    s.twb[i] = p[9 + i];
    s.tcw[i] = p[21 + i];
    s.v[i] = p[24 + i];
    s.bg[i] = p[27 + i];
    s.ba[i] = p[30 + i];
  }
}

// ---- LocalInertialBA's IMU links: the EdgeInertial error (and, building,
// its Jacobian), every lane of the link's wave computing the same values
// (inertial_edge_core); the link's robust chi2 (Huber sqrt(16.92) on flagged
// links, the information x1e-2 on the window's last link) plus EdgeGyroRW /
// EdgeAccRW.  Building, the link's quadratic form over its 30 dims (kf1 VP
// VV VG VA | kf2 VP VV VG VA; EdgeInertial's 24 columns are the first 24) and
// the gradient -J^T W e.  The links ride as extra blocks (a block per link) in
// k_lba_begin (chi2 at the initial state), k_lba_linearize (the first build's
// forms) and k_lba_trial (chi2 and, speculatively, forms at the trial state);
// each link's chi2 goes to imu_tot[2 + l] and the launch's last block sums
// them in link order.  (Round 2 ran the links on the four waves of one
// workgroup, three in a row: 36 us per build; round 3 a workgroup per link
// in a launch of its own.)
//
// One link by one 256-thread block (tid; every thread must call): its data
// and the two key-frame states staged in LDS (states from the table ts --
// k_lba_trial's trial states -- when given, else from the state array st);
// every wave runs the error chain (the same values), so the chi2 needs no
// exchange, and the form's 216 + 900 entries are spread over the block.
// kBuild: the form and gradient into copy qcopy of imu_q.  Returns the link's
// chi2 (every thread).
struct LinkLds {
  double J[9 * 24];
  double OJ[9 * 24];
  double E[9];      // the link's error (inertial_edge_core, lane 0)
  double Info[81];  // the link's information (x1e-2 when downweighted)
  LiaImuDev L;      // the link (preintegration)
  double S[2 * kImuStateStride];
};

template <bool kBuild>
__device__ __forceinline__ double lia_link(const LbaArgs& a, int l, int tid, const double* st, const double* ts,
                                           int qcopy, LinkLds& sh) {
  constexpr int NT = kThreads;  // the link's block
  const int lane = tid & 63;
  {
    // every load in flight before the first store: the edge chain below
    // then reads LDS, not one HBM round trip per field it reaches
    constexpr int kW = (int)(sizeof(LiaImuDev) / 4), kU = (kW + NT - 1) / NT;
    static_assert(sizeof(LiaImuDev) % 8 == 0, "LiaImuDev staging");
    const uint32_t* src = reinterpret_cast<const uint32_t*>(a.imu + l);
    const int k1 = a.imu[l].kf1, k2 = a.imu[l].kf2;
    const double* sb = ts ? ts : st;
    uint32_t w[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) w[u] = tid + NT * u < kW ? src[tid + NT * u] : 0u;
    const int k = tid, which = k >= kImuStateStride ? 1 : 0;
    const double sv =
        k < 2 * kImuStateStride ? sb[kImuStateStride * (which ? k2 : k1) + k - which * kImuStateStride] : 0.0;
    static_assert(2 * kImuStateStride <= NT, "one state double a thread");
    uint32_t* dst = reinterpret_cast<uint32_t*>(&sh.L);
#pragma unroll
    for (int u = 0; u < kU; ++u)
      if (tid + NT * u < kW) dst[tid + NT * u] = w[u];
    if (k < 2 * kImuStateStride) sh.S[k] = sv;
    __syncthreads();
  }
  const LiaImuDev& E = sh.L;
  const double isc = (E.flags & ORBGPU_LIA_DOWNWEIGHT) ? 1e-2 : 1.0;  // information() * 1e-2
  for (int k = tid; k < 81; k += NT) sh.Info[k] = E.pi.info[k] * isc;
  StateD s1, s2;
  load_state(s1, sh.S);
  load_state(s2, sh.S + kImuStateStride);
  double* J = sh.J;
  if (kBuild) {  // the constant blocks and the zeros (inertial_edge_core writes the rest)
    for (int k = tid; k < 9 * 24; k += NT) J[k] = 0;
    __syncthreads();
    if (tid < 9) {
      const int i = tid / 3, j = tid % 3;
      J[(6 + i) * 24 + 3 + j] = i == j ? -1.0 : 0.0;
      J[(3 + i) * 24 + 9 + j] = -(double)E.pi.JVg[3 * i + j];
      J[(6 + i) * 24 + 9 + j] = -(double)E.pi.JPg[3 * i + j];
      J[(3 + i) * 24 + 12 + j] = -(double)E.pi.JVa[3 * i + j];
      J[(6 + i) * 24 + 12 + j] = -(double)E.pi.JPa[3 * i + j];
    }
  }
  // every wave runs the chain (the same values); thread 0 stores J's blocks and e
  inertial_edge_core(s1, s2, E.pi, (double)E.pi.dT, tid, J, sh.E);
  __syncthreads();
  double e[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) e[k] = sh.E[k];
  // chi2 = e^T Omega e, one row per lane, then a fixed-order sum
  double part = 0;
  if (lane < 9) {
    double t = 0;
#pragma unroll
    for (int q = 0; q < 9; ++q) t += sh.Info[lane * 9 + q] * e[q];
    double el = 0;
#pragma unroll
    for (int q = 0; q < 9; ++q) el = lane == q ? e[q] : el;
    part = el * t;
  }
  double chi = 0;
#pragma unroll
  for (int q = 0; q < 9; ++q) chi += readlane_f64(part, q);
  double rho0 = chi, w = 1.0;
  if (E.flags & ORBGPU_LIA_ROBUST) huber_rho(chi, sqrt(16.92), rho0, w);
  double eg[3], ea[3], Og[3], Oa[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    eg[i] = s2.bg[i] - s1.bg[i];
    ea[i] = s2.ba[i] - s1.ba[i];
  }
  double cg = 0, ca = 0;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    Og[i] = E.pi.info_g[3 * i] * eg[0] + E.pi.info_g[3 * i + 1] * eg[1] + E.pi.info_g[3 * i + 2] * eg[2];
    Oa[i] = E.pi.info_a[3 * i] * ea[0] + E.pi.info_a[3 * i + 1] * ea[1] + E.pi.info_a[3 * i + 2] * ea[2];
    cg += eg[i] * Og[i];
    ca += ea[i] * Oa[i];
  }
  if (kBuild) {
    // W = w Omega; OJ = W J (9 x 24) into LDS, We = W e in registers
    for (int k = tid; k < 9 * 24; k += NT) {
      const int r = k / 24, col = k - 24 * r;
      double v = 0;
#pragma unroll
      for (int q = 0; q < 9; ++q) v += (w * sh.Info[r * 9 + q]) * J[q * 24 + col];
      sh.OJ[k] = v;
    }
    double We[9];
#pragma unroll
    for (int r = 0; r < 9; ++r) {
      double v = 0;
#pragma unroll
      for (int q = 0; q < 9; ++q) v += (w * sh.Info[r * 9 + q]) * e[q];
      We[r] = v;
    }
    __syncthreads();
    double* Q = a.imu_q + (size_t)kImuPairQ * (l + (size_t)a.n_imu * qcopy);
    for (int k = tid; k < 900; k += NT) {
      const int p = k / 30, q = k - 30 * p;
      double v = 0;
      if (p < 24 && q < 24) {
#pragma unroll
        for (int r = 0; r < 9; ++r) v += J[r * 24 + p] * sh.OJ[r * 24 + q];
      }
      // EdgeGyroRW (VG1 = -I at 9, VG2 = +I at 24), EdgeAccRW (12 / 27)
      const int pg = p < 15 ? p - 9 : p - 24, qg = q < 15 ? q - 9 : q - 24;
      if ((p >= 9 && p < 12) || (p >= 24 && p < 27))
        if ((q >= 9 && q < 12) || (q >= 24 && q < 27)) v += ((p < 15) == (q < 15) ? 1.0 : -1.0) * E.pi.info_g[3 * pg + qg];
      const int pa = p < 15 ? p - 12 : p - 27, qa = q < 15 ? q - 12 : q - 27;
      if ((p >= 12 && p < 15) || (p >= 27))
        if ((q >= 12 && q < 15) || (q >= 27)) v += ((p < 15) == (q < 15) ? 1.0 : -1.0) * E.pi.info_a[3 * pa + qa];
      Q[k] = v;
    }
    if (tid < 30) {
      const int p = tid;
      double g = 0;
      if (p < 24) {
#pragma unroll
        for (int r = 0; r < 9; ++r) g -= J[r * 24 + p] * We[r];
      }
      double og = 0, oa = 0;
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        og = p - 9 == i || p - 24 == i ? Og[i] : og;
        oa = p - 12 == i || p - 27 == i ? Oa[i] : oa;
      }
      if (p >= 9 && p < 12) g += og;  // -J^T Omega e with J = -I / +I
      if (p >= 24 && p < 27) g -= og;
      if (p >= 12 && p < 15) g += oa;
      if (p >= 27) g -= oa;
      Q[900 + p] = g;
    }
  }
  return (rho0 + cg) + ca;
}

// ---- buildSystem, edge side: Jacobians at the current state and each
// edge's terms of Hll / bl (point), Hpl and Hpp / bp (free pose)
// (base_binary_edge.hpp:56-119 with the robust weight of base_edge.h:91-97).
// The row loops run over 3 rows for mono edges too: their third Jacobian
// row and error are zero, and adding an exact 0 changes no sum (constant
// trip counts keep the Jacobians in registers, not in scratch).
// The per-edge terms live in two copies, one per LM state (lin_of(a, s)):
// the build at state s reads / writes copy s, and every trial writes the
// terms of its trial state into the other copy as it evaluates the edges
// (k_lba_trial), so an accepted trial leaves the next build nothing to
// linearise (LbaCtrl::lin_state; the values are those k_lba_linearize would
// compute from the same state and errors).
struct LinPtr {
  double* hpl;    // [18 E]
  double* hpp_e;  // [27][n_slots]
  double* hll_e;  // [12][E]
};
__device__ __forceinline__ LinPtr lin_of(const LbaArgs& a, int s) {
  return LinPtr{a.hpl + (size_t)s * 18 * a.n_edges, a.hpp_e + (size_t)s * 27 * a.n_slots,
                a.hll_e + (size_t)s * 12 * a.n_edges};
}

template <int M>
__device__ __forceinline__ void lin_edge(const LbaArgs& a, const LbaEdgeDev& e, int i, const double* ks,
                                         const double X[3], const double ev[3], const LinPtr& L) {
  double Jl[3][3], Jp[3][6];
  vis_jacobians<M>(a, e, ks, X, Jl, Jp);
  double r0, w;
  huber_rho(lba_chi2(e, ev), lba_delta(e), r0, w);
  const double info = (double)e.inv_sigma2, wi = w * info;
  double om[3];
#pragma unroll
  for (int r = 0; r < 3; ++r) om[r] = (-info * ev[r]) * w;
  double hl[12];  // 9 Hll terms (row-major), 3 bl terms
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    double g = 0;
#pragma unroll
    for (int r = 0; r < 3; ++r) g += Jl[r][s] * om[r];
    hl[9 + s] = g;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      double h = 0;
#pragma unroll
      for (int r = 0; r < 3; ++r) h += Jl[r][s] * wi * Jl[r][q];
      hl[3 * s + q] = h;
    }
  }
  double* hlo = L.hll_e + i;  // component-major: a wave's stores are contiguous
#pragma unroll
  for (int k = 0; k < 12; ++k) hlo[(size_t)k * a.n_edges] = hl[k];
  if (e.f < 0) return;
  double hp[27], hpl[18];  // 21 lower-triangle Hpp terms, 6 bp terms; Hpl 6 x 3
  int hk = 0;
#pragma unroll
  for (int s = 0; s < 6; ++s) {
    double g = 0;
#pragma unroll
    for (int r = 0; r < 3; ++r) g += Jp[r][s] * om[r];
    hp[21 + s] = g;
#pragma unroll
    for (int q = 0; q <= s; ++q) {
      double h = 0;
#pragma unroll
      for (int r = 0; r < 3; ++r) h += Jp[r][s] * wi * Jp[r][q];
      hp[hk++] = h;
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      double h = 0;
#pragma unroll
      for (int r = 0; r < 3; ++r) h += Jp[r][s] * wi * Jl[r][q];
      hpl[3 * s + q] = h;
    }
  }
  double* hpo = L.hpp_e + a.eslot[i];  // the edge's pose slot, component-major
#pragma unroll
  for (int k = 0; k < 27; ++k) hpo[(size_t)k * a.n_slots] = hp[k];
  double* hplo = L.hpl + 18 * (size_t)i;
#pragma unroll
  for (int k = 0; k < 18; ++k) hplo[k] = hpl[k];
}

// computeActiveErrors at the initial state, the robust chi2 and the LM's
// start (ctl_init), the first build's per-edge terms, the system cleared;
// kModelImu: the links' chi2 and forms
template <int M>
__global__ __launch_bounds__(kThreads) void k_lba_begin(LbaArgs a) {
  __shared__ double red[4];
  const int i = blockIdx.x * kThreads + threadIdx.x;
  if constexpr (M == kModelImu) {
    // blocks past the edges' take the IMU links at the initial state, a wave
    // per link: its chi2 to imu_tot[2 + l] and its form into copy 0 of imu_q
    // -- the first build's (state 0), so that build has no link work left
    // (k_lba_linearize takes the links only when every build relinearises)
    __shared__ LinkLds lsh;
    const int neb = (max(a.n_edges, 1) + kThreads - 1) / kThreads;
    const int l = (int)blockIdx.x - neb;
    if (l >= 0 && l < a.n_imu) {  // (block-uniform)
      const double chi = lia_link<true>(a, l, threadIdx.x, a.poses[0], nullptr, 0, lsh);
      if (threadIdx.x == 0) st_wt(a.imu_tot + 2 + l, chi);
    }
  }
  // the system's blocks no pose pair writes (and, kModelImu, the IMU rows,
  // which get no Schur terms) stay zero: clear it once per call
  for (size_t k = i, nz = (size_t)a.n_sys * a.n_sys + 2 * (size_t)a.n_sys; k < nz;
       k += (size_t)gridDim.x * kThreads)
    a.sys[k] = 0.0;
  double r0 = 0;
  if (i < a.n_edges) {
    const LbaEdgeDev e = a.edges[i];
    // the pose-slot record of a free-pose edge (read by the Schur kernels,
    // which run after this launch): built here, not uploaded
    const int ks = a.eslot[i];
    if (ks >= 0)
      const_cast<int4*>(a.pslot)[ks] = make_int4(i, e.point, a.pt_begin[e.point], a.pt_begin[e.point + 1]);
    const double* x = a.pts[0] + 3 * e.point;
    const double X[3] = {x[0], x[1], x[2]};
    double err[3];
    vis_error<M>(a, e, a.poses[0] + a.pstride * e.kf, X, err);
    a.err[3 * i] = err[0];
    a.err[3 * i + 1] = err[1];
    a.err[3 * i + 2] = err[2];
    double w;
    huber_rho(lba_chi2(e, err), lba_delta(e), r0, w);
    // the first build's per-edge terms (state 0, these errors: what
    // k_lba_linearize would compute), so no step needs a linearize launch
    lin_edge<M>(a, e, i, a.poses[0] + a.pstride * e.kf, X, err, lin_of(a, 0));
  }
  double v[1] = {r0};
  block_sum<1>(v, red);
  if (threadIdx.x == 0) st_wt(a.partials + blockIdx.x, v[0]);
  if (!last_block_wt(a.counter + 0)) return;
  double s[1];
  sum_partials<1>(a.partials, gridDim.x, s, red);
  if (threadIdx.x == 0) {
    if (M == kModelImu) {  // the IMU links at the initial state (this launch's link waves), in link order
      double tot = 0;
      for (int k = 0; k < a.n_imu; ++k) tot += a.imu_tot[2 + k];
      s[0] += tot;
    }
    const int stop = host_stop(a);
    if (a.sharded) {
      a.red[0] = s[0];
      a.red[1] = stop;
    } else {
      ctl_init(a, s[0], stop);
    }
  }
}

template <int M>
__global__ __launch_bounds__(kThreads) void k_lba_linearize(LbaArgs a) {
  const LbaCtrl& c = *a.ctrl;
  // nothing due, or the accepted trial already left this state's terms
  if (c.done || !c.need_build || (c.lin_state == c.state && !a.force_lin)) return;
  if constexpr (M == kModelImu) {
    // blocks past the edges' build the IMU links' forms, a block per link (launched
    // only when every build relinearises; else k_lba_begin / k_lba_trial wrote them)
    __shared__ LinkLds lsh;
    const int neb = (a.n_edges + kThreads - 1) / kThreads;
    if ((int)blockIdx.x >= neb) {
      const int l = (int)blockIdx.x - neb;
      if (l < a.n_imu) lia_link<true>(a, l, threadIdx.x, a.poses[c.state], nullptr, c.state, lsh);
      return;
    }
  }
  const int i = blockIdx.x * kThreads + threadIdx.x;
  if (i >= a.n_edges) return;
  const LbaEdgeDev e = a.edges[i];
  const double* x = a.pts[c.state] + 3 * e.point;
  const double X[3] = {x[0], x[1], x[2]};
  const double ev[3] = {a.err[3 * i], a.err[3 * i + 1], a.err[3 * i + 2]};
  lin_edge<M>(a, e, i, a.poses[c.state] + a.pstride * e.kf, X, ev, lin_of(a, c.state));
}

// The links' part of the camera-side system: entry (r, c) of free key frames
// (fr, fc) sums, over the links incident to fr in link order, the form
// entries whose dims land on (r, c); the last n entries are the gradient.
// Run by extra blocks of k_lba_sums (one launch for the build's sums).
__device__ __forceinline__ void lia_assemble_entry(const LbaArgs& a, int state, long idx) {
  const int n = a.n_sys;
  if (idx >= (long)n * n + n) return;
  const bool grad = idx >= (long)n * n;
  const int r = grad ? (int)(idx - (long)n * n) : (int)(idx / n);
  const int cc = grad ? 0 : (int)(idx - (long)r * n);
  const int fr = r / kImuDim, dr = r - kImuDim * fr;
  const int fc = cc / kImuDim, dc = cc - kImuDim * fc;
  double v = 0;
  for (int j = a.imu_inc[fr]; j < a.imu_inc[fr + 1]; ++j) {
    const int4 rec = a.imu_inc_rec[j];  // {link, fr's side, the other's free index, its side}
    const double* Q = a.imu_q + (size_t)kImuPairQ * (rec.x + (size_t)a.n_imu * state);
    if (grad) {
      v += Q[900 + kImuDim * rec.y + dr];
    } else {
      const int sc = fc == fr ? rec.y : (rec.z == fc ? rec.w : -1);
      if (sc >= 0) v += Q[(kImuDim * rec.y + dr) * 30 + kImuDim * sc + dc];
    }
  }
  a.himu[idx] = v;
  // the system takes the links' part directly (the solves stage one array):
  // every entry here, and the Schur writes add it to the pose pairs' blocks
  // and the pose rows of b_s / b_p they overwrite per trial
  if (grad) {
    a.sys[(size_t)n * n + r] = v;
    a.sys[(size_t)n * n + n + r] = v;
  } else {
    a.sys[idx] = v;
  }
}

template <int M>
__device__ __forceinline__ void classify_elem(const LbaArgs& a, int s, int i, uint8_t* __restrict__ outlier,
                                              double* __restrict__ out, uint32_t* __restrict__ ctrl_out) {
  // the final LM state for the host's one copy back
  if (i < (int)(sizeof(LbaCtrl) / 4)) ctrl_out[i] = reinterpret_cast<const uint32_t*>(a.ctrl)[i];
  if (i < a.pstride * a.n_kf) out[i] = a.poses[s][i];
  if (i < 3 * a.n_pts) out[(size_t)a.pstride * a.n_kf + i] = a.pts[s][i];
  if (i >= a.n_edges) return;
  const LbaEdgeDev e = a.edges[i];
  const double* x = a.pts[s] + 3 * e.point;
  const double X[3] = {x[0], x[1], x[2]};
  double tmp[3];
  const bool depth = vis_error<M>(a, e, a.poses[s] + a.pstride * e.kf, X, tmp);
  const double ev[3] = {a.err[3 * i], a.err[3 * i + 1], a.err[3 * i + 2]};
  const double chi = lba_chi2(e, ev);
  if constexpr (M == kModelSe3) {
    outlier[i] = (chi > (e.ur < 0.f ? 5.991 : 7.815) || !depth) ? 1 : 0;
  } else {
    constexpr float chi2Mono2 = 5.991f, chi2Stereo2 = 7.815f;
    bool bad;
    if (e.ur < 0.f) {
      const bool close = a.close[e.point] != 0;
      bad = (chi > chi2Mono2 && !close) || (chi > 1.5f * chi2Mono2 && close) || !depth;
    } else {
      bad = chi > chi2Stereo2;
    }
    outlier[i] = bad ? 1 : 0;
  }
}

__device__ __forceinline__ int classify_items(const LbaArgs& a) {
  return max(max(a.n_edges, a.pstride * a.n_kf), max(3 * a.n_pts, (int)(sizeof(LbaCtrl) / 4)));
}

// The results straight into host-mapped memory (a.res_*), grid-stride over
// any grid; every block releases its stores at system scope before its
// ticket, and the last block publishes the call's number
// (LbaHostWords::results) and marks the call classified.  Run by every
// block of k_lba_sums once the LM is done (the step queued behind the one
// that ended it), or by k_lba_classify_host when no step follows.
template <int M>
__device__ void classify_to_host(const LbaArgs& a) {
  const LbaCtrl& c = *a.ctrl;
  const int n = classify_items(a);
  for (int i = blockIdx.x * kThreads + threadIdx.x; i < n; i += gridDim.x * kThreads)
    classify_elem<M>(a, c.state, i, a.res_outlier, a.res_out, a.res_ctrl);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope
  if (!last_block(a.counter + 3)) return;
  if (threadIdx.x == 0) {
    a.ctrl->classified = 1;  // later no-op steps' sums skip it (stream-ordered)
    __hip_atomic_store(&a.host->results, (uint32_t)c.call, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// ---- buildSystem, vertex side.  Blocks [0, kSumsQ n_free): a quarter of
// one free pose's slots each (slot j of the pose to block j / 256 mod kSumsQ),
// a fixed tree per term (DPP row sums, then the 16 rows in order) -> a
// partial of Hpp (lower 21) and bp per (pose, quarter) in a.pose_part.
// Blocks [kSumsQ n_free, +points): one point per thread summing its edges'
// Hll / bl in insertion order.  kModelImu: then the link-assembly blocks.
// The last block adds each pose's quarters in order (Hpp 6 x 6 full, bp,
// the pose diagonal) and opens the iteration: iniChi, and at iteration 0
// computeLambdaInit (tau * max |diag| over pose and point blocks).
template <int M>
__global__ __launch_bounds__(kThreads) void k_lba_sums(LbaArgs a) {
  __shared__ double red[16 * 27];
  const LbaCtrl& c = *a.ctrl;
  if (c.done) {  // the first kernel of a step queued behind the LM's end: the results
    if (a.early_out && !c.classified) classify_to_host<M>(a);
    return;
  }
  if (!c.need_build) return;
  const LinPtr L = lin_of(a, c.state);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n_pose_blocks = kSumsQ * a.n_free;
  const int n_pt_blocks = (max(a.n_pts, 1) + kThreads - 1) / kThreads;
  double hmax = 0;
  if ((int)blockIdx.x < n_pose_blocks) {
    const int f = blockIdx.x / kSumsQ, q = blockIdx.x - kSumsQ * f;
    double acc[27];
#pragma unroll
    for (int k = 0; k < 27; ++k) acc[k] = 0;
    const int j1 = a.pose_begin[f + 1];
    // the pose's slots are contiguous in hpp_e's component rows: every load
    // of a wave reads 512 consecutive bytes (two slots' terms in flight)
    constexpr int kStep = kSumsQ * kThreads;
    for (int jb = a.pose_begin[f] + q * kThreads + threadIdx.x; jb < j1; jb += 2 * kStep) {
      double hv[2][27];
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int k = 0; k < 27; ++k)
          hv[u][k] = jb + u * kStep < j1 ? L.hpp_e[(size_t)k * a.n_slots + jb + u * kStep] : 0.0;
#pragma unroll
      for (int u = 0; u < 2; ++u)
        if (jb + u * kStep < j1)
#pragma unroll
          for (int k = 0; k < 27; ++k) acc[k] += hv[u][k];
    }
#pragma unroll
    for (int k = 0; k < 27; ++k) {
      double v = acc[k];
      v += dpp_f64<0x111, 0xf>(v);
      v += dpp_f64<0x112, 0xf>(v);
      v += dpp_f64<0x114, 0xf>(v);
      v += dpp_f64<0x118, 0xf>(v);
      if ((lane & 15) == 15) red[(wave * 4 + (lane >> 4)) * 27 + k] = v;
    }
    __syncthreads();
    if (threadIdx.x < 27) {
      const int k = threadIdx.x;
      double v = 0;
#pragma unroll
      for (int r = 0; r < 16; ++r) v += red[r * 27 + k];
      st_wt(a.pose_part + 27 * (size_t)blockIdx.x + k, v);
    }
  } else if ((int)blockIdx.x >= n_pose_blocks + n_pt_blocks) {
    // kModelImu: the links' part of the system (lia_assemble_entry)
    const long b = (long)blockIdx.x - n_pose_blocks - n_pt_blocks;
    lia_assemble_entry(a, c.state, b * kThreads + threadIdx.x);
  } else {
    const int p = (blockIdx.x - n_pose_blocks) * kThreads + threadIdx.x;
    if (p < a.n_pts) {
      double H[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
      const int i0 = a.pt_begin[p], i1 = a.pt_begin[p + 1];
      for (int ib = i0; ib < i1; ib += 4) {  // four edges' loads in flight
        double hl[4][12];
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int k = 0; k < 12; ++k) hl[u][k] = ib + u < i1 ? L.hll_e[(size_t)k * a.n_edges + ib + u] : 0.0;
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (ib + u < i1)
#pragma unroll
            for (int k = 0; k < 12; ++k) H[k] += hl[u][k];
      }
#pragma unroll
      for (int k = 0; k < 9; ++k) a.hll[9 * (size_t)p + k] = H[k];
#pragma unroll
      for (int k = 0; k < 3; ++k) a.bl[3 * (size_t)p + k] = H[9 + k];
      hmax = fmax(fabs(H[0]), fmax(fabs(H[4]), fabs(H[8])));
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) hmax = fmax(hmax, __shfl_xor(hmax, o, 64));
    if (lane == 0) red[wave] = hmax;
    __syncthreads();
    hmax = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
  }
  if (threadIdx.x == 0) st_wt(a.partials + blockIdx.x, hmax);
  if (!last_block_wt(a.counter + 1)) return;
  // each pose's quarters in order -> Hpp (6 x 6 full), bp, the pose diagonal
  for (int idx = threadIdx.x; idx < 27 * a.n_free; idx += kThreads) {
    const int f = idx / 27, k = idx - 27 * f;
    const double* pp = a.pose_part + 27 * (size_t)kSumsQ * f + k;
    double v = 0;
#pragma unroll
    for (int q = 0; q < kSumsQ; ++q) v += pp[27 * q];
    if (k < 21) {
      int s2 = 0, q2 = k;  // lower-triangle index k -> (s2, q2)
      while (q2 > s2) {
        q2 -= s2 + 1;
        ++s2;
      }
      a.hpp[36 * (size_t)f + 6 * s2 + q2] = v;
      a.hpp[36 * (size_t)f + 6 * q2 + s2] = v;
      if (s2 == q2) a.diag[a.pdim * f + s2] = v;
    } else {
      a.bp[6 * (size_t)f + (k - 21)] = v;
    }
  }
  __syncthreads();
  // the maxima only feed computeLambdaInit (the first build): later builds
  // skip their loads.  max is order-independent: every reduction order gives
  // the same value
  const bool first = c.it == 0;
  double m = 0;
  if (first) {
    for (int b = threadIdx.x; b < (int)gridDim.x; b += kThreads) m = fmax(m, a.partials[b]);
    // pose rows only: the inertial model (pdim 15) writes a.diag for rows
    // 0..5 of a key frame (its lambda is the caller's, lambda_init > 0)
    for (int k = threadIdx.x; k < a.n_sys; k += kThreads)
      if (k % a.pdim < 6) m = fmax(m, fabs(a.diag[k]));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o, 64));
  __syncthreads();
  if (lane == 0) red[wave] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    LbaCtrl& cw = *a.ctrl;
    const double mx = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
    if (a.sharded) {
      // this shard's point maximum; the host max-reduces it and sum-reduces
      // the pose diagonal, then k_lba_ctl(kCtlLambda) finishes lambda init
      double hm = 0;
      if (first)
        for (int b = a.n_free; b < (int)gridDim.x; ++b) hm = fmax(hm, a.partials[b]);
      a.diag[a.n_sys] = hm;  // (reduced, and read, only at the first build)
      cw.lambda_due = cw.it == 0 ? 1 : 0;
    } else if (cw.it == 0) {
      ctl_lambda(a, mx);
    }
    cw.ini = cw.cur;
    cw.q = 0;
    cw.need_build = 0;
  }
}

// one Schur entry of pose pair (fi, fj): t < 36 the block entry (s, q) = (t /
// 6, t % 6) (a diagonal pair: its lower entries, mirrored -- exactly
// symmetric), else b_s / b_p of row t - 36; sum = the points' part
__device__ __forceinline__ void schur_write(const LbaArgs& a, int fi, int fj, int t, double sum) {
  const bool diag = fi == fj;
  const int n = a.n_sys, P = a.pdim;  // P: the pose block's rows (VP first in a kModelImu key frame)
  if (t < 36) {
    const int s = t / 6, q = t - 6 * s;
    if (diag && q > s) return;  // diagonal block: lower triangle, mirrored (exactly symmetric)
    const size_t o = (size_t)(P * fi + s) * n + P * fj + q;
    // kModelImu: + the links' part (symmetric: the link forms are)
    const double v = (diag ? a.hpp[36 * (size_t)fi + 6 * s + q] : 0.0) - sum + (a.himu ? a.himu[o] : 0.0);
    a.sys[o] = v;
    a.sys[(size_t)(P * fj + q) * n + P * fi + s] = v;
  } else {
    const int s = t - 36;
    const double hb = a.himu ? a.himu[(size_t)n * n + P * fi + s] : 0.0;
    a.sys[(size_t)n * n + P * fi + s] = a.bp[6 * (size_t)fi + s] - sum + hb;  // b_s
    a.sys[(size_t)n * n + n + P * fi + s] = a.bp[6 * (size_t)fi + s] + hb;   // b_p (computeScale)
  }
}

// ---- Schur complement of the points at the trial's lambda: one 512-thread
// block per free-pose pair (fi <= fj).  Threads stride over pose fi's edges
// (point order); each finds its point's edges to pose fj and adds
// W_i Hpl_j^T with W_i = Hpl_i (Hll + lambda I)^-1; the diagonal pair also
// takes b_s = bp - sum W_i bl.  (block_solver.hpp:392-460)  Loads are issued
// in batches (slot record -> point data + the point's free indices -> the
// matching Hpl) so each thread waits on three memory round trips.
constexpr int kSchurThreads = 512;
constexpr int kSchurWaves = kSchurThreads / 64;

__global__ __launch_bounds__(kSchurThreads) void k_lba_schur(LbaArgs a) {
  __shared__ double red[kSchurWaves * 4 * 42];
  const LbaCtrl& c = *a.ctrl;
  if (c.done) return;
  const double lambda = c.lambda;
  const double* const hpl = lin_of(a, c.state).hpl;
  const int pr = blockIdx.x;
  const int fi = a.pair_i[pr], fj = a.pair_j[pr];
  const bool diag = fi == fj;
  double acc[42];
#pragma unroll
  for (int k = 0; k < 42; ++k) acc[k] = 0;
  for (int k = a.pose_begin[fi] + threadIdx.x; k < a.pose_begin[fi + 1]; k += kSchurThreads) {
    const int4 sl = a.pslot[k];  // {edge, point, first edge of the point, end}
    const int ei = sl.x, p = sl.y;
    double hll[9], B[18];
#pragma unroll
    for (int q = 0; q < 9; ++q) hll[q] = a.hll[9 * (size_t)p + q];
#pragma unroll
    for (int q = 0; q < 18; ++q) B[q] = hpl[18 * (size_t)ei + q];
    double blp[3] = {0, 0, 0};
    if (diag)
#pragma unroll
      for (int q = 0; q < 3; ++q) blp[q] = a.bl[3 * (size_t)p + q];
    int fs[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) fs[u] = sl.z + u < sl.w ? a.ef[sl.z + u] : -2;
    // a point not seen by pose fj adds nothing off the diagonal: skip its
    // inverse and W (points seen by more than 8 key frames take the full path)
    if (!diag && sl.w - sl.z <= 8) {
      bool hit = false;
#pragma unroll
      for (int u = 0; u < 8; ++u) hit |= fs[u] == fj;
      if (!hit) continue;
    }
    double Di[9];
    inv3_lambda(hll, lambda, Di);
    double W[6][3];
#pragma unroll
    for (int s = 0; s < 6; ++s)
#pragma unroll
      for (int q = 0; q < 3; ++q) W[s][q] = B[3 * s] * Di[q] + B[3 * s + 1] * Di[3 + q] + B[3 * s + 2] * Di[6 + q];
    for (int base = sl.z;;) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (fs[u] != fj) continue;
        const double* Bj = hpl + 18 * (size_t)(base + u);
#pragma unroll
        for (int s = 0; s < 6; ++s)
#pragma unroll
          for (int q = 0; q < 6; ++q)
            acc[6 * s + q] += W[s][0] * Bj[3 * q] + W[s][1] * Bj[3 * q + 1] + W[s][2] * Bj[3 * q + 2];
      }
      base += 8;
      if (base >= sl.w) break;  // points seen by more than 8 keyframes: next chunk
#pragma unroll
      for (int u = 0; u < 8; ++u) fs[u] = base + u < sl.w ? a.ef[base + u] : -2;
    }
    if (diag)
#pragma unroll
      for (int s = 0; s < 6; ++s) acc[36 + s] += W[s][0] * blp[0] + W[s][1] * blp[1] + W[s][2] * blp[2];
  }
  // fixed tree: DPP row sums (lane 15 of each 16-lane row), then the block's
  // row partials in row order
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nk = diag ? 42 : 36;
#pragma unroll
  for (int k = 0; k < 42; ++k) {
    double x = acc[k];
    x += dpp_f64<0x111, 0xf>(x);
    x += dpp_f64<0x112, 0xf>(x);
    x += dpp_f64<0x114, 0xf>(x);
    x += dpp_f64<0x118, 0xf>(x);
    if ((lane & 15) == 15) red[(wave * 4 + (lane >> 4)) * 42 + k] = x;
  }
  __syncthreads();
  const int t = threadIdx.x;
  if (t < nk) {
    double sum = 0;
#pragma unroll 8
    for (int r = 0; r < kSchurWaves * 4; ++r) sum += red[r * 42 + t];
    schur_write(a, fi, fj, t, sum);
  }
}

// ---- Schur complement by point range (k_lba_schur_split + k_lba_schur_fold):
// the shard's points cut into a.sc_split contiguous ranges of about equal edge
// counts (lba_api.cpp), one 128-thread block per (pose pair, range) -- blocks
// pair * S + x, so with S = 8 the blocks of range x share blockIdx % 8 and
// (under the round-robin dispatch, for speed only) one XCD: every byte of a
// range's points is then fetched into one XCD's L2, not all eight.  Each
// thread takes one of pose fi's edges in the range (a.pose_split bounds them
// in the point-ordered pslot list), looks up the point's edge to pose fj
// FIRST and loads Hll / Hpl_i / Hpl_j only for a hit (about one edge in four
// at C4), so the HBM bytes are those of the hits.  The block's partial of S_ij
// (and, diagonal pairs, of W bl) goes to a.sc_part in a fixed DPP / LDS tree;
// k_lba_schur_fold adds the S partials of each pair in range order (S = 1:
// the block writes the system itself).  Deterministic run to run.
constexpr int kSplitThreads = 128;
constexpr int kSplitWaves = kSplitThreads / 64;


__global__ __launch_bounds__(kSplitThreads) void k_lba_schur_split(LbaArgs a) {
  __shared__ double red[kSplitWaves * 4 * 42];
  const LbaCtrl& c = *a.ctrl;
  if (c.done) return;
  const double lambda = c.lambda;
  const double* const hpl = lin_of(a, c.state).hpl;
  const int S = a.sc_split;
  const int pr = blockIdx.x / S, x = blockIdx.x - pr * S;
  const int fi = a.pair_i[pr], fj = a.pair_j[pr];
  const bool diag = fi == fj;
  const int* ps = a.pose_split + (size_t)fi * (S + 1);
  const int k1 = ps[x + 1];
  double acc[42];
#pragma unroll
  for (int k = 0; k < 42; ++k) acc[k] = 0;
  for (int k = ps[x] + threadIdx.x; k < k1; k += kSplitThreads) {
    const int4 sl = a.pslot[k];  // {edge, point, first edge of the point, end}
    const int ei = sl.x, p = sl.y;
    int fs[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) fs[u] = sl.z + u < sl.w ? a.ef[sl.z + u] : -2;
    int uj = -1;  // the point's first edge to pose fj among its first 8
#pragma unroll
    for (int u = 7; u >= 0; --u)
      if (fs[u] == fj) uj = u;
    if (uj < 0 && sl.w - sl.z <= 8) continue;  // not seen by pose fj: adds nothing
    // a hit (or a point seen by more than 8 key frames): its data, the first
    // matching Hpl_j in the same batch of loads
    double hll[9], B[18], Bj[18], blp[3] = {0, 0, 0};
#pragma unroll
    for (int q = 0; q < 9; ++q) hll[q] = a.hll[9 * (size_t)p + q];
#pragma unroll
    for (int q = 0; q < 18; ++q) B[q] = hpl[18 * (size_t)ei + q];
    const size_t ej = 18 * (size_t)(sl.z + (uj < 0 ? 0 : uj));
#pragma unroll
    for (int q = 0; q < 18; ++q) Bj[q] = hpl[ej + q];
    if (diag)
#pragma unroll
      for (int q = 0; q < 3; ++q) blp[q] = a.bl[3 * (size_t)p + q];
    double Di[9];
    inv3_lambda(hll, lambda, Di);
    double W[6][3];
#pragma unroll
    for (int s = 0; s < 6; ++s)
#pragma unroll
      for (int q = 0; q < 3; ++q) W[s][q] = B[3 * s] * Di[q] + B[3 * s + 1] * Di[3 + q] + B[3 * s + 2] * Di[6 + q];
    auto add = [&](const double* Bq) {
#pragma unroll
      for (int s = 0; s < 6; ++s)
#pragma unroll
        for (int q = 0; q < 6; ++q)
          acc[6 * s + q] += W[s][0] * Bq[3 * q] + W[s][1] * Bq[3 * q + 1] + W[s][2] * Bq[3 * q + 2];
    };
    // the point's edges to pose fj in edge order (normally exactly one)
    for (int base = sl.z;;) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (fs[u] != fj) continue;
        if (base == sl.z && u == uj)
          add(Bj);
        else
          add(hpl + 18 * (size_t)(base + u));
      }
      base += 8;
      if (base >= sl.w) break;  // points seen by more than 8 keyframes: next chunk
#pragma unroll
      for (int u = 0; u < 8; ++u) fs[u] = base + u < sl.w ? a.ef[base + u] : -2;
    }
    if (diag)
#pragma unroll
      for (int s = 0; s < 6; ++s) acc[36 + s] += W[s][0] * blp[0] + W[s][1] * blp[1] + W[s][2] * blp[2];
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < 42; ++k) {
    double v = acc[k];
    v += dpp_f64<0x111, 0xf>(v);
    v += dpp_f64<0x112, 0xf>(v);
    v += dpp_f64<0x114, 0xf>(v);
    v += dpp_f64<0x118, 0xf>(v);
    if ((lane & 15) == 15) red[(wave * 4 + (lane >> 4)) * 42 + k] = v;
  }
  __syncthreads();
  const int t = threadIdx.x, nk = diag ? 42 : 36;
  double sum = 0;
  if (t < nk) {
#pragma unroll
    for (int r = 0; r < kSplitWaves * 4; ++r) sum += red[r * 42 + t];
  }
  if (S == 1) {
    if (t < nk) schur_write(a, fi, fj, t, sum);
    return;
  }
  if (!a.sc_fold_inline) {  // k_lba_schur_fold adds the ranges
    if (t < nk) a.sc_part[42 * (size_t)blockIdx.x + t] = sum;
    return;
  }
  // the pair's last block to finish (a ticket per pair, self-resetting) adds
  // its S range partials in range order -- k_lba_schur_fold's sum, without
  // the launch.  The partials are stored write-through (agent-scope relaxed
  // atomic stores: sc1, straight to L2) and drained (vmcnt 0) before the
  // barrier and the ticket -- no release fence (its L2 write-back made the
  // first form of this, 17.9 us, slower than the extra launch)
  if (t < nk)
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(a.sc_part) + 42 * (size_t)blockIdx.x + t,
                       (unsigned long long)__double_as_longlong(sum), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __shared__ int last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) {
    const unsigned tk = __hip_atomic_fetch_add(a.pair_cnt + pr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = tk == (unsigned)(S - 1);
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // (an L1 invalidate: the partials come from L2)
      __hip_atomic_store(a.pair_cnt + pr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  if (!last || t >= nk) return;
  const double* part = a.sc_part + 42 * (size_t)pr * S + t;
  double v[kSchurSplitMax];
#pragma unroll
  for (int y = 0; y < kSchurSplitMax; ++y) v[y] = y < S ? part[42 * y] : 0.0;
  double tot = 0;
#pragma unroll
  for (int y = 0; y < kSchurSplitMax; ++y)
    if (y < S) tot += v[y];
  schur_write(a, fi, fj, t, tot);
}

// each pair's S range partials added in range order, then written as above
__global__ __launch_bounds__(64) void k_lba_schur_fold(LbaArgs a) {
  const LbaCtrl& c = *a.ctrl;
  if (c.done) return;
  const int pr = blockIdx.x, t = threadIdx.x, S = a.sc_split;
  const int fi = a.pair_i[pr], fj = a.pair_j[pr];
  if (t >= (fi == fj ? 42 : 36)) return;
  const double* part = a.sc_part + 42 * (size_t)pr * S + t;
  double v[8];
#pragma unroll
  for (int x = 0; x < 8; ++x) v[x] = x < S ? part[42 * x] : 0.0;
  double sum = 0;
#pragma unroll
  for (int x = 0; x < 8; ++x)
    if (x < S) sum += v[x];
  schur_write(a, fi, fj, t, sum);
}

// ---- Schur complement, point-major (block_solver.hpp:392-460 visits each
// landmark once): one block per chunk of points (lba_api.cpp orders the points
// by their lowest free pose and cuts chunks spanning <= kSchurBandMax poses).
// The chunk's part of S_ij = sum_p W_pi Hpl_pj^T (W = Hpl (Hll + lambda I)^-1)
// and of b_s = sum_p W_pi bl_p is one matrix product over the chunk:
//   W_all (band rows x 4 per point) . H_all^T,
// row 6 (f - b0) + s of point p's slice holding W_pe[s] (H: Hpl_pe[s]) for
// its edge e to free pose f, zeros for the band's other poses, and one more H
// row holding bl_p (so the product's last column is W bl).
//   1. a thread per point: (Hll + lambda I)^-1 once, W for each of its free
//      edges, both slices into LDS (component-major: conflict-free MFMA reads);
//   2. a wave per upper 16 x 16 tile of the product: one
//      v_mfma_f64_16x16x4f64 per point (k-step = the point's 3 components +
//      a zero), two accumulators for the even / odd points (ILP), added at
//      the end -- a fixed order, reproducible run to run;
//   3. the upper tiles to HBM; k_lba_schur_sum adds each pose pair's entries
//      over the chunks covering it, in chunk order.
// Each edge's Hll / Hpl / bl are read once per trial (the pair kernel below
// re-reads a pose's edges for every pair it is in).
constexpr int kBandThreads = 256;
constexpr int kBandWaves = kBandThreads / 64;

__global__ __launch_bounds__(kBandThreads) void k_lba_schur_band(LbaArgs a) {
  extern __shared__ double sb[];
  const LbaCtrl& c = *a.ctrl;
  if (c.done) return;
  const double lambda = c.lambda;
  const double* const hpl = lin_of(a, c.state).hpl;
  const int4 ch = a.sc_chunk[blockIdx.x];  // {first in sc_order, points, b0, w}
  const int P = ch.y, b0 = ch.z, w = ch.w;
  const int NB = schur_band_rows(w), T = NB >> 4;
  double* const sW = sb;                        // [P][4][NB]
  double* const sH = sb + (size_t)P * 4 * NB;   // [P][4][NB]
  const int t = threadIdx.x;
  {
    double2* z = reinterpret_cast<double2*>(sb);
    const int n2 = P * 4 * NB;  // (2 * P * 4 * NB doubles)
    for (int k = t; k < n2; k += kBandThreads) z[k] = make_double2(0.0, 0.0);
  }
  __syncthreads();
  for (int k = t; k < P; k += kBandThreads) {
    const int p = a.sc_order[ch.x + k];
    double hll[9], bl[3];
#pragma unroll
    for (int q = 0; q < 9; ++q) hll[q] = a.hll[9 * (size_t)p + q];
#pragma unroll
    for (int q = 0; q < 3; ++q) bl[q] = a.bl[3 * (size_t)p + q];
    double Di[9];
    inv3_lambda(hll, lambda, Di);
    double* const wk = sW + (size_t)k * 4 * NB;
    double* const hk = sH + (size_t)k * 4 * NB;
#pragma unroll
    for (int q = 0; q < 3; ++q) hk[q * NB + 6 * w] = bl[q];
    const int u0 = a.pt_begin[p], u1 = a.pt_begin[p + 1];
    for (int ub = u0; ub < u1; ub += 4) {  // four edges' loads in flight
      int fs[4];
      double B[4][18];
#pragma unroll
      for (int v = 0; v < 4; ++v) fs[v] = ub + v < u1 ? a.ef[ub + v] : -1;
#pragma unroll
      for (int v = 0; v < 4; ++v)
#pragma unroll
        for (int q = 0; q < 18; ++q) B[v][q] = fs[v] >= 0 ? hpl[18 * (size_t)(ub + v) + q] : 0.0;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        if (fs[v] < 0) continue;
        const int r0 = 6 * (fs[v] - b0);
#pragma unroll
        for (int s6 = 0; s6 < 6; ++s6)
#pragma unroll
          for (int q = 0; q < 3; ++q) {
            hk[q * NB + r0 + s6] = B[v][3 * s6 + q];
            wk[q * NB + r0 + s6] =
                B[v][3 * s6] * Di[q] + B[v][3 * s6 + 1] * Di[3 + q] + B[v][3 * s6 + 2] * Di[6 + q];
          }
      }
    }
  }
  __syncthreads();
  const int lane = t & 63, li = lane & 15, lk = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  double* const part = a.sc_part + 256 * (size_t)a.sc_tile0[blockIdx.x];
  for (int q = wave, I = 0, J = wave; q < T * (T + 1) / 2; q += kBandWaves) {
    while (J >= T) {  // tile q -> (I, J), J >= I, row-major over the upper triangle
      J -= T - I;
      ++I;
      J += 1;
    }
    d4 acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
    int k = 0;
    for (; k + 1 < P; k += 2) {
      const double a0 = sW[((size_t)k * 4 + lk) * NB + 16 * I + li];
      const double c0 = sH[((size_t)k * 4 + lk) * NB + 16 * J + li];
      const double a1 = sW[((size_t)(k + 1) * 4 + lk) * NB + 16 * I + li];
      const double c1 = sH[((size_t)(k + 1) * 4 + lk) * NB + 16 * J + li];
      acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, c0, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, c1, acc1, 0, 0, 0);
    }
    if (k < P) {
      const double a0 = sW[((size_t)k * 4 + lk) * NB + 16 * I + li];
      const double c0 = sH[((size_t)k * 4 + lk) * NB + 16 * J + li];
      acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, c0, acc0, 0, 0, 0);
    }
    // C[lk + 4 rr][li] of tile q
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) part[256 * (size_t)q + (lk + 4 * rr) * 16 + li] = acc0[rr] + acc1[rr];
    J += kBandWaves;
  }
}

// one wave per pose pair (fi <= fj): the entries of its block (and, for a
// diagonal pair, of b_s) summed over the chunks whose band covers both poses,
// in chunk order, then written as k_lba_schur writes them (a diagonal block
// from its upper entries, mirrored: exactly symmetric)
constexpr int kSumChunksLds = 1024;

__global__ __launch_bounds__(64) void k_lba_schur_sum(LbaArgs a) {
  __shared__ int4 sch[kSumChunksLds];
  __shared__ int st0[kSumChunksLds];
  const LbaCtrl& c = *a.ctrl;
  if (c.done) return;
  const int pr = blockIdx.x, t = threadIdx.x;
  const int fi = a.pair_i[pr], fj = a.pair_j[pr];
  const bool diag = fi == fj;
  const int s = t < 36 ? t / 6 : t - 36, q = t < 36 ? t - 6 * (t / 6) : 0;
  const bool live = t < 36 ? (!diag || s <= q) : (diag && t < 42);
  // covering chunks have b0 in [fj - kSchurBandMax + 1, fi] (chunks sorted by b0)
  int lo = 0, hi = a.n_chunks;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a.sc_chunk[mid].z < fj - kSchurBandMax + 1)
      lo = mid + 1;
    else
      hi = mid;
  }
  double sum = 0;
  for (int c0 = lo; c0 < a.n_chunks; c0 += kSumChunksLds) {
    const int nc = min(kSumChunksLds, a.n_chunks - c0);
    __syncthreads();
    for (int k = t; k < nc; k += 64) {
      sch[k] = a.sc_chunk[c0 + k];
      st0[k] = a.sc_tile0[c0 + k];
    }
    __syncthreads();
    bool past = false;
    for (int k = 0; k < nc; k += 4) {  // four chunks' loads in flight, summed in order
      double v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        v[u] = 0.0;
        if (k + u >= nc) continue;
        const int4 ck = sch[k + u];
        if (ck.z > fi) {
          past = true;
          continue;
        }
        if (!live || fj >= ck.z + ck.w) continue;
        const int T = schur_band_rows(ck.w) >> 4;
        const int row = 6 * (fi - ck.z) + s, col = t < 36 ? 6 * (fj - ck.z) + q : 6 * ck.w;
        const int I = row >> 4, J = col >> 4;  // I <= J: fi < fj, s <= q on the diagonal, or the bl column
        const int tile = I * T - I * (I - 1) / 2 + (J - I);
        v[u] = a.sc_part[256 * ((size_t)st0[k + u] + tile) + (row & 15) * 16 + (col & 15)];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) sum += v[u];
      if (uniform_branch(past ? 1 : 0)) break;
    }
    if (past) break;
  }
  if (!live) return;
  // (a diagonal pair's live entries are its upper ones, s <= q: the transposed
  // lower entry, which schur_write takes, has the same sum)
  schur_write(a, fi, fj, t < 36 ? (diag ? 6 * q + s : t) : t, sum);
}

// ---- reduced camera system (S + lambda I) x = b_s: L D L^T by 16 x 16 tiles
// (linear_solver_eigen.h:93-126 factorises the same matrix with
// SimplicialLDLT; the factorisation order here is natural, tiled).
// Per tile step K:
//   1. wave 0 factors the diagonal tile in registers (lane i owns row i, the
//      pivot row broadcast by v_readlane) and inverts its unit-lower L_KK;
//   2. the panel L_IK = A_IK L_KK^-T D_K^-1 -- v_mfma_f64_16x16x4 (A_IK
//      times L_KK^-T, 4 k-steps), waves over tiles I;
//   3. the trailing update A_IJ -= L_IK D_K L_JK^T for K < J <= I -- MFMA,
//      waves over tiles.
// Then forward / diagonal / backward substitution by tiles with the saved
// L_KK^-1 (16 x 16 mat-vecs, no serial chains), the pose part of
// computeScale, and the failure flag (a zero pivot: Eigen's SimplicialLDLT
// reports NumericalIssue only for D(k,k) == 0).
// kLds: the lower-triangle tiles of S packed in LDS (tile (I, J), J <= I, at
// (I (I + 1) / 2 + J) x 272 doubles, rows 17 apart: odd stride, conflict-free
// tile columns -- only the lower triangle is ever read) and the L_KK^-1
// tiles; up to n_pad = 160 (10 inertial or 26 SE3 key frames).  Else S row-
// major in a.work (stride n_pad + 1) and the L_KK^-1 tiles after it.
// Phase clocks of the solve (tools/lba_solve_bench.hip builds with
// LBA_SOLVE_STAMPS): thread 0 adds the s_memtime delta since its previous
// stamp to bucket k.
constexpr int kSolveThreads = 512;
constexpr int kSolveWaves = kSolveThreads / 64;
constexpr int kTileLd = 17;             // row stride inside a packed LDS tile
constexpr int kTileSz = 16 * kTileLd;   // doubles per packed tile

// 1 / d: v_rcp_f64 and one Newton step (the pivot chain's latency; not the
// IEEE division sequence)
__device__ __forceinline__ double rcp_f64(double d) {
  const double x = __builtin_amdgcn_rcp(d);
  return fma(x, fma(-d, x, 1.0), x);
}

constexpr int kSolveStageTiles = 8;  // LDS path: n_pad <= 160 -> <= 55 tiles: tile 0 + <= 8 per wave of 1-7
static_assert(1 + (kSolveWaves - 1) * kSolveStageTiles >= 55, "LDS solve staging covers T = 10 (the LDS budget's largest)");

// ---- DPP64 row broadcasts for the diagonal tile (lane li of every 16-lane
// row owns row li): v_mov_b64_dpp / v_fmac_f64_dpp with row_newbcast:N read
// lane N of the lane's row, so an updated entry costs one instruction instead
// of a v_readlane pair + an FMA.  Inline asm: the compiler forms neither DPP64
// form itself.  Each block starts with s_nop 1: a VALU write of a VGPR
// followed by a DPP read of it needs 2 wait states, and a block's inputs may
// come straight from compiler-scheduled VALU code.
template <int N>
__device__ __forceinline__ double row_bcast_f64(double v) {
  double o;
  asm volatile("s_nop 1\n\tv_mov_b64_dpp %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf"
               : "=v"(o)
               : "v"(v), "i"(N));
  return o;
}

#define LBA_FMAC_BC(k) "v_fmac_f64_dpp %" #k ", %" #k ", %17 row_newbcast:%18 row_mask:0xf bank_mask:0xf\n\t"
// Pivot N of the augmented elimination: the 16 entries after the pivot column
// (aug[N+1 .. N+16] = the rest of the A_KK row, then the first N+1 entries of
// the inverse row, the only non-zero entries of pivot row N's inverse part)
// and y take nl = -l_i times lane N's value; aug[N+1] first (the next pivot).
template <int N>
__device__ __forceinline__ void pivot_update(double (&aug)[32], double& y, double nl) {
  asm volatile("s_nop 1\n\t" LBA_FMAC_BC(0) LBA_FMAC_BC(1) LBA_FMAC_BC(2) LBA_FMAC_BC(3) LBA_FMAC_BC(4)
                   LBA_FMAC_BC(5) LBA_FMAC_BC(6) LBA_FMAC_BC(7) LBA_FMAC_BC(8) LBA_FMAC_BC(9) LBA_FMAC_BC(10)
                       LBA_FMAC_BC(11) LBA_FMAC_BC(12) LBA_FMAC_BC(13) LBA_FMAC_BC(14) LBA_FMAC_BC(15)
                           LBA_FMAC_BC(16)
               : "+v"(aug[N + 1]), "+v"(aug[N + 2]), "+v"(aug[N + 3]), "+v"(aug[N + 4]), "+v"(aug[N + 5]),
                 "+v"(aug[N + 6]), "+v"(aug[N + 7]), "+v"(aug[N + 8]), "+v"(aug[N + 9]), "+v"(aug[N + 10]),
                 "+v"(aug[N + 11]), "+v"(aug[N + 12]), "+v"(aug[N + 13]), "+v"(aug[N + 14]),
                 "+v"(aug[N + 15]), "+v"(aug[N + 16]), "+v"(y)
               : "v"(nl), "i"(N));
}
#undef LBA_FMAC_BC

// Pivots N..15 of the diagonal tile: d_N broadcast from lane N (zero pivot =
// Eigen's NumericalIssue: flagged, the pivot's multipliers 0), l_i = a_iN / d_N
// below the pivot, 0 at and above it (those rows are unchanged).
template <int N>
__device__ __forceinline__ void diag_pivots(double (&aug)[32], double& y, double& dmine, int& zero, int li) {
  if constexpr (N < 16) {
    const double dc = row_bcast_f64<N>(aug[N]);
    dmine = li == N ? dc : dmine;
    zero |= dc == 0.0;
    const double inv = dc != 0.0 ? rcp_f64(dc) : 0.0;
    const double l = li > N ? aug[N] * inv : 0.0;
    pivot_update<N>(aug, y, -l);
    diag_pivots<N + 1>(aug, y, dmine, zero, li);
  }
}

// The same elimination with each pivot's reciprocal chain interleaved into
// the previous pivot's FMAs: block N applies pivot N (l = l_N, subtracted)
// and, between its 17 row-broadcast FMAs, forms pivot N+1 -- the broadcast
// d_{N+1} (read two FMAs after its column entry is final), v_rcp_f64 + one
// Newton step, and l_{N+1} = [i > N+1] a_{i,N+1} / d_{N+1}.  No zero-pivot
// guard: a zero pivot gives infinities, and the caller then redoes the tile
// with diag_pivots (which keeps Eigen's NumericalIssue semantics).
#define LBA_FMC(k) "v_fmac_f64_dpp %" #k ", %" #k ", -%[l] row_newbcast:%[n] row_mask:0xf bank_mask:0xf\n\t"
template <int N>  // N <= 14
__device__ __forceinline__ void pivot_step(double (&aug)[32], double& y, double l, double m01, double& d,
                                           double& lnext) {
  double inv, e, tt;
  asm volatile("s_nop 1\n\t" LBA_FMC(0)                        // a_{i,N+1}: the next pivot column
               "v_mul_f64 %[t], %0, %[m]\n\t" LBA_FMC(1) LBA_FMC(2)  //
               "v_mov_b64_dpp %[d], %0 row_newbcast:%[n1] row_mask:0xf bank_mask:0xf\n\t" LBA_FMC(3)
               "v_rcp_f64 %[inv], %[d]\n\t" LBA_FMC(4) LBA_FMC(5)  //
               "v_fma_f64 %[e], -%[d], %[inv], 1.0\n\t" LBA_FMC(6)   //
               "v_fma_f64 %[inv], %[inv], %[e], %[inv]\n\t" LBA_FMC(7)
               "v_mul_f64 %[ln], %[t], %[inv]\n\t" LBA_FMC(8) LBA_FMC(9) LBA_FMC(10) LBA_FMC(11) LBA_FMC(12)
                   LBA_FMC(13) LBA_FMC(14) LBA_FMC(15) LBA_FMC(16)
               : "+v"(aug[N + 1]), "+v"(aug[N + 2]), "+v"(aug[N + 3]), "+v"(aug[N + 4]), "+v"(aug[N + 5]),
                 "+v"(aug[N + 6]), "+v"(aug[N + 7]), "+v"(aug[N + 8]), "+v"(aug[N + 9]), "+v"(aug[N + 10]),
                 "+v"(aug[N + 11]), "+v"(aug[N + 12]), "+v"(aug[N + 13]), "+v"(aug[N + 14]),
                 "+v"(aug[N + 15]), "+v"(aug[N + 16]), "+v"(y), [d] "=&v"(d), [inv] "=&v"(inv), [e] "=&v"(e),
                 [t] "=&v"(tt), [ln] "=&v"(lnext)
               : [l] "v"(l), [m] "v"(m01), [n] "i"(N), [n1] "i"(N + 1));
}
#undef LBA_FMC

template <int N>
__device__ __forceinline__ void diag_chain(double (&aug)[32], double& y, double l, double& dmine, int li) {
  if constexpr (N < 15) {
    double d, ln;
    pivot_step<N>(aug, y, l, li > N + 1 ? 1.0 : 0.0, d, ln);
    dmine = li == N + 1 ? d : dmine;
    diag_chain<N + 1>(aug, y, ln, dmine, li);
  } else {
    pivot_update<15>(aug, y, -l);
  }
}

// The diagonal tile K by elimination of the augmented rows [A_KK | I | y_K]
// (one wave; lane li of every 16-lane row owns row li): pivot c subtracts
// l_i = a_ic / d_c times row c from the rows below it, which leaves D_K on
// the diagonal, L_KK^-1 in the identity's place and L_KK^-1 y_K in y -- the
// factorisation, the inverse and the tile's forward substitution in one pass
// of 16 row-broadcast FMAs per pivot.  SKK: the tile (row stride ts), yk: y_K
// (read), then L_KK^-1 -> li_out (16 x kTileLd), D_K -> d_out, the
// substituted y_K -> y_out; a zero pivot sets *bad.
__device__ __forceinline__ void diag_tile_factor(const double* SKK, int ts, const double* yk, double* li_out,
                                                 double* d_out, double* y_out, int* bad, int lane) {
  const int li = lane & 15;
  double aug[32];
#pragma unroll
  for (int j = 0; j < 16; ++j) aug[j] = SKK[li * ts + j];
#pragma unroll
  for (int j = 0; j < 16; ++j) aug[16 + j] = j == li ? 1.0 : 0.0;
  double yv = yk[li];
  double dmine = 0;
  int zero = 0;
  {
    const double d0 = row_bcast_f64<0>(aug[0]);
    dmine = li == 0 ? d0 : 0.0;
    diag_chain<0>(aug, yv, (li > 0 ? aug[0] : 0.0) * rcp_f64(d0), dmine, li);
  }
  if (__builtin_amdgcn_ballot_w64(lane < 16 && dmine == 0.0) != 0) {
    // a zero pivot (Eigen: NumericalIssue): the guarded elimination of the
    // tile from its original rows (SKK and y_K are not written above)
#pragma unroll
    for (int j = 0; j < 16; ++j) aug[j] = SKK[li * ts + j];
#pragma unroll
    for (int j = 0; j < 16; ++j) aug[16 + j] = j == li ? 1.0 : 0.0;
    yv = yk[li];
    diag_pivots<0>(aug, yv, dmine, zero, li);
  }
  if (lane < 16) {
#pragma unroll
    for (int j = 0; j < 16; ++j) li_out[li * kTileLd + j] = aug[16 + j];
    d_out[li] = dmine;
    y_out[li] = yv;
  }
  if (lane == 0 && zero) *bad = 1;
}

#ifdef LBA_SOLVE_STAMPS
__device__ unsigned long long g_lba_stamps[16];
#define LBA_STAMP(k)                                                  \
  do {                                                                \
    if (t == 0) {                                                     \
      const unsigned long long now_ = __builtin_amdgcn_s_memtime();   \
      stamp_acc[k] += now_ - stamp_last;                              \
      stamp_last = now_;                                              \
    }                                                                 \
  } while (0)
#else
#define LBA_STAMP(k) \
  do {               \
  } while (0)
#endif

template <bool kLds>
__global__ __launch_bounds__(kSolveThreads) void k_lba_solve(LbaArgs a) {
  extern __shared__ double smem[];
  const LbaCtrl& c = *a.ctrl;
  if (c.done) return;
  const double lambda = c.lambda;
  const int n = a.n_sys, N = a.n_pad, LD = N + 1, T = N >> 4;
  const int TS = kLds ? kTileLd : LD;  // row stride inside a tile
  const int t = threadIdx.x, lane = t & 63, li = lane & 15, lk = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);  // wave-uniform: scalar loops
#ifdef LBA_SOLVE_STAMPS
  unsigned long long stamp_last = __builtin_amdgcn_s_memtime();
  unsigned long long stamp_acc[16] = {};  // registers (constant indices): no memory round trip per stamp
#endif
  double* S;
  double* Li;
  double* Dg;
  double* y;
  double* Wscr = nullptr;  // kLds: a transposition tile per wave
  __shared__ double red[kSolveWaves];
  __shared__ int bad;
  if constexpr (kLds) {
    S = smem;
    Li = smem + (size_t)(T * (T + 1) / 2) * kTileSz;
    Dg = Li + (size_t)T * kTileSz;
    y = Dg + N;
    Wscr = y + N;
  } else {
    S = a.work;
    Li = a.work + (size_t)N * LD;
    Dg = smem;
    y = smem + N;
  }
  // tile (I, J) of S, J <= I
  auto tile = [&](int I, int J) -> double* {
    if constexpr (kLds)
      return S + (size_t)(I * (I + 1) / 2 + J) * kTileSz;
    else
      return S + (size_t)(16 * I) * LD + 16 * J;
  };
  const double* src = a.sys;
  const double* hm = nullptr;  // (the links' part is in a.sys already: lia_assemble_entry, schur_write)
  if constexpr (kLds) {
    // S + lambda I (lower tiles) with identity padding (D = 1, L = 0): wave 0
    // stages tile 0 alone and factors it while waves 1-7 stage tiles w, w +
    // 7, ... (tile (I, J) of the row-major enumeration), a lane 4 consecutive
    // entries of one tile row; every load of the wave in flight before the
    // LDS writes, no index divisions
    const int ntile = T * (T + 1) / 2;
    auto tile_q = [&](int u) { return wave == 0 ? (u == 0 ? 0 : ntile) : wave + (kSolveWaves - 1) * u; };
    const int lr = lane >> 2, lc = 4 * (lane & 3);
    double v[kSolveStageTiles][4];
    auto tile_of = [&](int q, int& I, int& J) {
      I = 0;
      while ((I + 1) * (I + 2) / 2 <= q) ++I;
      J = q - I * (I + 1) / 2;
    };
    auto stage = [&](auto with_imu) {
#pragma unroll
      for (int u = 0; u < kSolveStageTiles; ++u) {
        const int q = tile_q(u);
        if (q < ntile) {
          int I, J;
          tile_of(q, I, J);
          const int r = 16 * I + lr, c0 = 16 * J + lc;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const size_t o = (size_t)r * n + c0 + e;
            const bool in = r < n && c0 + e < n;
            double x = in ? src[o] : 0.0;
            if constexpr (decltype(with_imu)::value) x += in ? hm[o] : 0.0;
            v[u][e] = x;
          }
        }
      }
    };
    if (hm)
      stage(std::true_type{});
    else
      stage(std::false_type{});
#pragma unroll
    for (int u = 0; u < kSolveStageTiles; ++u) {
      const int q = tile_q(u);
      if (q < ntile) {
        int I, J;
        tile_of(q, I, J);
        const int r = 16 * I + lr, c0 = 16 * J + lc;
        double* dst = tile(I, J) + lr * TS + lc;
#pragma unroll
        for (int e = 0; e < 4; ++e) dst[e] = v[u][e] + (r == c0 + e ? (r < n ? lambda : 1.0) : 0.0);
      }
    }
  } else {
    // S row-major in a.work (n_pad beyond the LDS budget): 16 loads in flight
    // per thread before the writes
    for (int e0 = t; e0 < N * N; e0 += 16 * kSolveThreads) {
      double v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int e = e0 + u * kSolveThreads, r = e / N, cc = e - r * N;
        v[u] = e < N * N && r < n && cc < n && (cc >> 4) <= (r >> 4)
                   ? src[(size_t)r * n + cc] + (hm ? hm[(size_t)r * n + cc] : 0.0)
                   : 0.0;
      }
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int e = e0 + u * kSolveThreads, r = e / N, cc = e - r * N;
        if (e < N * N && (cc >> 4) <= (r >> 4))
          tile(r >> 4, cc >> 4)[(r & 15) * TS + (cc & 15)] = v[u] + (r == cc ? (r < n ? lambda : 1.0) : 0.0);
      }
    }
  }
  for (int r = t; r < N; r += kSolveThreads)
    y[r] = r < n ? src[(size_t)n * n + r] + (hm ? hm[(size_t)n * n + r] : 0.0) : 0.0;
  if (t == 0) bad = 0;
  if constexpr (kLds) {
    // diagonal tile 0 from wave 0's own writes (tile 0, y_0) while the other
    // waves still stage
    if (wave == 0 && T > 0) {
      wave_lds_sync();
      diag_tile_factor(tile(0, 0), TS, y, Li, Dg, y, &bad, lane);
    }
  }
  __syncthreads();
  LBA_STAMP(0);

  // 1-3. the diagonal tile K (diag_tile_factor): one wave
  auto diag_tile = [&](int K) {
    const int k0 = 16 * K;
    diag_tile_factor(tile(K, K), TS, y + k0, Li + (size_t)K * kTileSz, Dg + k0, y + k0, &bad, lane);
  };

  if constexpr (kLds) {
    // 4. one phase per step K, a wave per block row I > K:
    //   L_IK = (A_IK L_KK^-T) D_K^-1 and y_I -= L_IK y_K (DPP row sums);
    //   R_I = L_IK L_KK^-1, formed transposed (R_I^T = L_KK^-T L_IK^T) so
    //   that its MFMA result already sits in the A-operand layout;
    //   A_IJ -= R_I A_JK^T for K < J <= I (= L_IK D_K L_JK^T).
    // Look-ahead: wave 0 takes row K+1 (one tile) and then factors diagonal
    // tile K+1 in the same phase, while waves 1-7 take rows K+2.. (heaviest
    // first, on SIMDs 1, 2, 3 before sharing one): one barrier per step.
    // Every wave reads the raw A_JK of column K, so L_IK is written back into
    // tile (I, K) only after the step's barrier (held in registers).
    d4 L_held[2];
    int I_held[2] = {0, 0}, n_held = 0;
    double* const scr = Wscr + wave * kTileSz;
    auto row = [&](int K, int I) {
      const int k0 = 16 * K, i0 = 16 * I;
      const double* const SIK = tile(I, K);
      d4 acc = {0, 0, 0, 0};
#pragma unroll
      for (int kc = 0; kc < 4; ++kc) {
        const int kk = 4 * kc + lk;
        const double av = SIK[li * TS + kk];
        const double bv = Li[(size_t)K * kTileSz + li * kTileLd + kk];  // (L^-1)^T[kk][li]
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
      }
      const double dinv = rcp_f64(Dg[k0 + li]);
      const double ykl = y[k0 + li];
      double p[4];
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const double l = acc[rr] * dinv;
        acc[rr] = l;
        scr[(lk + 4 * rr) * kTileLd + li] = l;
        p[rr] = l * ykl;
      }
      // the four row sums' DPP steps interleaved (same order per sum)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) p[rr] += dpp_f64<0x111, 0xf>(p[rr]);
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) p[rr] += dpp_f64<0x112, 0xf>(p[rr]);
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) p[rr] += dpp_f64<0x114, 0xf>(p[rr]);
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) p[rr] += dpp_f64<0x118, 0xf>(p[rr]);
      if (li == 15) {
        double yo[4];
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) yo[rr] = y[i0 + lk + 4 * rr];
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) y[i0 + lk + 4 * rr] = yo[rr] - p[rr];
      }
      LBA_STAMP(8);
      wave_lds_sync();  // the scratch tile back in the transposed order
      d4 rt = {0, 0, 0, 0};
#pragma unroll
      for (int kc = 0; kc < 4; ++kc) {
        const int kk = 4 * kc + lk;
        const double av = Li[(size_t)K * kTileSz + kk * kTileLd + li];  // (L^-T)[li][kk]
        const double bv = scr[li * kTileLd + kk];                       // (L_IK^T)[kk][li]
        rt = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, rt, 0, 0, 0);
      }
      // rt[kc] = R_I[li][lk + 4 kc]: the A operand of k-step kc
      LBA_STAMP(9);
      // the row's tiles, the next tile's operands loaded before this one's
      // MFMAs (neg:[1,0,0] on A: A_IJ - R_I A_JK^T)
      auto ld = [&](int J, d4& c, d4& b) {
        const double* const SIJ = tile(I, J);
        const double* const SJK = tile(J, K);
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) c[rr] = SIJ[(lk + 4 * rr) * TS + li];
#pragma unroll
        for (int kc = 0; kc < 4; ++kc) b[kc] = SJK[li * TS + 4 * kc + lk];
      };
      d4 cn, bn;
      ld(K + 1, cn, bn);
      for (int J = K + 1; J <= I; ++J) {
        d4 c = cn;
        const d4 b = bn;
        if (J < I) ld(J + 1, cn, bn);
#pragma unroll
        for (int kc = 0; kc < 4; ++kc) c = __builtin_amdgcn_mfma_f64_16x16x4f64(rt[kc], b[kc], c, 0, 0, 1);
        double* const SIJ = tile(I, J);
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) SIJ[(lk + 4 * rr) * TS + li] = c[rr];
      }
      LBA_STAMP(10);
      // T <= 10: at most 8 rows for waves 1-7, so a wave holds two at most
      if (n_held == 0) {
        L_held[0] = acc;
        I_held[0] = I;
      } else {
        L_held[1] = acc;
        I_held[1] = I;
      }
      ++n_held;
      wave_lds_sync();  // the scratch tile is rewritten by the wave's next row
    };
    auto write_back = [&](int K) {  // the L tiles this wave computed in step K
#pragma unroll
      for (int h = 0; h < 2; ++h)
        if (h < n_held) {
          double* const SH = tile(I_held[h], K);
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) SH[(lk + 4 * rr) * TS + li] = L_held[h][rr];
        }
      n_held = 0;
    };
    // rows K+2.. to waves 1..7: the heaviest on SIMDs 1, 2, 3, then 5, 6, 7, 4
    constexpr int kRowWave[7] = {1, 2, 3, 5, 6, 7, 4};
    int slot = -1;
#pragma unroll
    for (int q = 0; q < 7; ++q)
      if (kRowWave[q] == wave) slot = q;
    // (diagonal tile 0 was factored during the staging; T == 0: every key
    // frame fixed, nothing to factor)
    LBA_STAMP(1);
    for (int K = 0; K < T - 1; ++K) {
      if (K > 0) write_back(K - 1);
      if (wave == 0) {
        row(K, K + 1);
        diag_tile(K + 1);
        LBA_STAMP(2);
      } else {
        for (int q = slot; q < T - K - 2; q += 7) row(K, T - 1 - q);
      }
      __syncthreads();
      LBA_STAMP(3);
    }
    write_back(T - 2);
    __syncthreads();
  } else {
    for (int K = 0; K < T; ++K) {
      const int k0 = 16 * K;
      if (wave == 0) diag_tile(K);
      __syncthreads();
      LBA_STAMP(1);
      // 4. panel: L_IK = (A_IK L_KK^-T) D_K^-1 (MFMA), and the rows' forward
      // substitution y_I -= L_IK y_K (DPP row sums over the tile's columns)
      for (int I = K + 1 + wave; I < T; I += kSolveWaves) {
        const int i0 = 16 * I;
        double* const SIK = tile(I, K);
        d4 acc = {0, 0, 0, 0};
#pragma unroll
        for (int kc = 0; kc < 4; ++kc) {
          const int kk = 4 * kc + lk;
          const double av = SIK[li * TS + kk];
          const double bv = Li[(size_t)K * kTileSz + li * kTileLd + kk];  // (L^-1)^T[kk][li]
          acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
        }
        const double dinv = rcp_f64(Dg[k0 + li]);
        const double ykl = y[k0 + li];
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const double l = acc[rr] * dinv;
          SIK[(lk + 4 * rr) * TS + li] = l;
          double p = l * ykl;
          p += dpp_f64<0x111, 0xf>(p);
          p += dpp_f64<0x112, 0xf>(p);
          p += dpp_f64<0x114, 0xf>(p);
          p += dpp_f64<0x118, 0xf>(p);
          if (li == 15) y[i0 + lk + 4 * rr] -= p;
        }
      }
      __syncthreads();
      LBA_STAMP(3);
      // 5. trailing: A_IJ -= L_IK (D_K L_JK^T), tiles K < J <= I enumerated
      // row-major, v_mfma_f64_16x16x4 over the tile's 16 columns
      const int m = T - K - 1;
      const int ntile = m * (m + 1) / 2;
      for (int q = wave; q < ntile; q += kSolveWaves) {
        int I = 0;
        while ((I + 1) * (I + 2) / 2 <= q) ++I;
        const int J = q - I * (I + 1) / 2;
        double* const SIJ = tile(K + 1 + I, K + 1 + J);
        const double* const SIK = tile(K + 1 + I, K);
        const double* const SJK = tile(K + 1 + J, K);
        d4 acc;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) acc[rr] = SIJ[(lk + 4 * rr) * TS + li];
#pragma unroll
        for (int kc = 0; kc < 4; ++kc) {
          const int kk = 4 * kc + lk;
          const double av = -SIK[li * TS + kk];
          const double bv = SJK[li * TS + kk] * Dg[k0 + kk];
          acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
        }
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) SIJ[(lk + 4 * rr) * TS + li] = acc[rr];
      }
      __syncthreads();
      LBA_STAMP(4);
    }
  }
  for (int r = t; r < N; r += kSolveThreads) y[r] = y[r] * rcp_f64(Dg[r]);
  __syncthreads();
  LBA_STAMP(5);
  // backward: L^T x = y by tiles from the last (L_KK^-T mat-vec, then the
  // rows above take the tile's contribution) -- by wave 0 alone: a step is
  // two 16-FMA chains and LDS round trips, and wave-level syncs instead of
  // two workgroup barriers a step (the same operations in the same order)
  if (wave == 0) {
    for (int K = T - 1; K >= 0; --K) {
      const int k0 = 16 * K;
      double s = 0;
      if (lane < 16) {
#pragma unroll
        for (int k = 0; k < 16; ++k) s = fma(Li[(size_t)K * kTileSz + k * kTileLd + lane], y[k0 + k], s);
      }
      wave_lds_sync();  // every read of y_K before the writes
      if (lane < 16) y[k0 + lane] = s;
      wave_lds_sync();
      for (int r = lane; r < k0; r += 64) {
        double u = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k) u = fma(tile(K, r >> 4)[k * TS + (r & 15)], y[k0 + k], u);
        y[r] -= u;
      }
      wave_lds_sync();
    }
  }
  __syncthreads();
  LBA_STAMP(6);
  // x_p and the pose part of computeScale: x . (lambda x + b_p)
  double sc = 0;
  for (int r = t; r < n; r += kSolveThreads) {
    const double xv = y[r];
    a.xp[r] = xv;
    sc += xv * (lambda * xv + src[(size_t)n * n + n + r] + (hm ? hm[(size_t)n * n + r] : 0.0));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) sc += __shfl_xor(sc, o, 64);
  if (lane == 0) red[wave] = sc;
  __syncthreads();
  if (t == 0) {
    double v = 0;
#pragma unroll
    for (int w = 0; w < kSolveWaves; ++w) v += red[w];
    a.scal[0] = v;
    a.scal[1] = bad;
  }
  LBA_STAMP(7);
#ifdef LBA_SOLVE_STAMPS
  if (t == 0)
    for (int k = 0; k < 16; ++k) g_lba_stamps[k] += stamp_acc[k];
#endif
}

// ---- the reduced camera system of a large window (kSolveGrid): the same
// tiled L D L^T and substitutions as k_lba_solve<false>, spread over the
// whole device.  Everything lives in a.work (hbm_solve): S row-major (stride
// n_pad + 1, lower tiles only), the L_KK^-1 tiles, D, y and the zero-pivot
// flag -- no LDS bound on the window.  Per tile step K two launches:
//   k_lba_ldl_panel   every block factors diagonal tile K into LDS
//                     (diag_tile_factor, block 0 also stores it), then a wave
//                     per block row I > K: L_IK = A_IK L_KK^-T D_K^-1 (MFMA)
//                     and y_I -= L_IK y_K
//   k_lba_ldl_update  a wave per trailing tile (I, J), K < J <= I:
//                     A_IJ -= L_IK D_K L_JK^T (MFMA)
// after k_lba_ldl_stage (S + lambda I, y = b_s) and before k_lba_ldl_back
// (D^-1, backward substitution, x_p and computeScale on one block).  The
// arithmetic per entry is k_lba_solve<false>'s (same tile operations in the
// same order), so both paths give the same x_p.
struct HbmSolve {
  double* S;
  double* Li;
  double* Dg;
  double* y;   // the right-hand side, rows below the current step updated in place
  double* ys;  // L^-1 y after the forward substitution (written per diagonal tile)
  int* bad;
};

__device__ __forceinline__ HbmSolve hbm_solve(const LbaArgs& a) {
  const size_t N = a.n_pad, T = N >> 4;
  HbmSolve h;
  h.S = a.work;
  h.Li = h.S + N * (N + 1);
  h.Dg = h.Li + T * kTileSz;
  h.y = h.Dg + N;
  h.ys = h.y + N;
  h.bad = reinterpret_cast<int*>(h.ys + N);
  return h;
}

// one block per padded row r: its lower-tile entries of S + lambda I (identity
// padding past n_sys), y_r = b_s (+ the IMU links' gradient), the flag cleared
__global__ __launch_bounds__(kThreads) void k_lba_ldl_stage(LbaArgs a) {
  const LbaCtrl& c = *a.ctrl;
  if (c.done) return;
  const HbmSolve h = hbm_solve(a);
  const double lambda = c.lambda;
  const int n = a.n_sys, N = a.n_pad, r = blockIdx.x;
  const size_t LD = (size_t)N + 1;
  const double* src = a.sys;
  const double* hm = nullptr;  // (in a.sys already)
  const int cend = 16 * ((r >> 4) + 1);
  for (int cc = threadIdx.x; cc < cend; cc += kThreads) {
    const bool in = r < n && cc < n;
    const size_t o = (size_t)r * n + cc;
    double x = in ? src[o] : 0.0;
    if (hm && in) x += hm[o];
    h.S[(size_t)r * LD + cc] = x + (r == cc ? (r < n ? lambda : 1.0) : 0.0);
  }
  if (threadIdx.x == 0) {
    h.y[r] = r < n ? src[(size_t)n * n + r] + (hm ? hm[(size_t)n * n + r] : 0.0) : 0.0;
    if (r == 0) *h.bad = 0;
  }
}

__global__ __launch_bounds__(kSolveThreads) void k_lba_ldl_panel(LbaArgs a, int K) {
  __shared__ double sLi[kTileSz];
  __shared__ double sD[16], sY[16];
  __shared__ int sbad;
  const LbaCtrl& c = *a.ctrl;
  if (c.done) return;
  const HbmSolve h = hbm_solve(a);
  const int T = a.n_pad >> 4, k0 = 16 * K;
  const size_t LD = (size_t)a.n_pad + 1;
  const int t = threadIdx.x, lane = t & 63, li = lane & 15, lk = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  if (t == 0) sbad = 0;
  __syncthreads();
  if (wave == 0) diag_tile_factor(h.S + (size_t)k0 * LD + k0, (int)LD, h.y + k0, sLi, sD, sY, &sbad, lane);
  __syncthreads();
  if (blockIdx.x == 0) {
    for (int q = t; q < kTileSz; q += kSolveThreads) h.Li[(size_t)K * kTileSz + q] = sLi[q];
    if (t < 16) {  // (every block reads y_K: the substituted values go to ys)
      h.Dg[k0 + t] = sD[t];
      h.ys[k0 + t] = sY[t];
    }
    if (t == 0 && sbad) *h.bad = 1;
  }
  const int I = K + 1 + (int)blockIdx.x * kSolveWaves + wave;
  if (I >= T) return;
  const int i0 = 16 * I;
  double* const SIK = h.S + (size_t)i0 * LD + k0;
  d4 acc = {0, 0, 0, 0};
#pragma unroll
  for (int kc = 0; kc < 4; ++kc) {
    const int kk = 4 * kc + lk;
    const double av = SIK[li * LD + kk];
    const double bv = sLi[li * kTileLd + kk];  // (L^-1)^T[kk][li]
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
  }
  const double dinv = rcp_f64(sD[li]);
  const double ykl = sY[li];
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const double l = acc[rr] * dinv;
    SIK[(lk + 4 * rr) * LD + li] = l;
    double p = l * ykl;
    p += dpp_f64<0x111, 0xf>(p);
    p += dpp_f64<0x112, 0xf>(p);
    p += dpp_f64<0x114, 0xf>(p);
    p += dpp_f64<0x118, 0xf>(p);
    if (li == 15) h.y[i0 + lk + 4 * rr] -= p;
  }
}

__global__ __launch_bounds__(kSolveThreads) void k_lba_ldl_update(LbaArgs a, int K) {
  const LbaCtrl& c = *a.ctrl;
  if (c.done) return;
  const HbmSolve h = hbm_solve(a);
  const int T = a.n_pad >> 4, k0 = 16 * K, m = T - K - 1;
  const size_t LD = (size_t)a.n_pad + 1;
  const int lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4;
  const int q = (int)blockIdx.x * kSolveWaves + __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  if (q >= m * (m + 1) / 2) return;
  // q -> (I, J), J <= I, row-major over the trailing triangle
  int I = (int)((sqrt(8.0 * q + 1.0) - 1.0) * 0.5);
  while ((I + 1) * (I + 2) / 2 <= q) ++I;
  while (I * (I + 1) / 2 > q) --I;
  const int J = q - I * (I + 1) / 2;
  const size_t r0 = (size_t)16 * (K + 1 + I), c0 = (size_t)16 * (K + 1 + J);
  double* const SIJ = h.S + r0 * LD + c0;
  const double* const SIK = h.S + r0 * LD + k0;
  const double* const SJK = h.S + c0 * LD + k0;
  d4 acc;
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) acc[rr] = SIJ[(lk + 4 * rr) * LD + li];
#pragma unroll
  for (int kc = 0; kc < 4; ++kc) {
    const int kk = 4 * kc + lk;
    const double av = -SIK[li * LD + kk];
    const double bv = SJK[li * LD + kk] * h.Dg[k0 + kk];
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
  }
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) SIJ[(lk + 4 * rr) * LD + li] = acc[rr];
}

__global__ __launch_bounds__(kSolveThreads) void k_lba_ldl_back(LbaArgs a) {
  __shared__ double red[kSolveWaves];
  const LbaCtrl& c = *a.ctrl;
  if (c.done) return;
  const HbmSolve h = hbm_solve(a);
  const double lambda = c.lambda;
  const int n = a.n_sys, N = a.n_pad, T = N >> 4;
  const size_t LD = (size_t)N + 1;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  double* const y = h.ys;
  for (int r = t; r < N; r += kSolveThreads) y[r] = y[r] * rcp_f64(h.Dg[r]);
  __syncthreads();
  for (int K = T - 1; K >= 0; --K) {
    const int k0 = 16 * K;
    if (t < 16) {
      double s = 0;
#pragma unroll
      for (int k = 0; k < 16; ++k) s = fma(h.Li[(size_t)K * kTileSz + k * kTileLd + t], y[k0 + k], s);
      __builtin_amdgcn_wave_barrier();
      y[k0 + t] = s;
    }
    __syncthreads();
    const double* const rowK = h.S + (size_t)k0 * LD;
    for (int r = t; r < k0; r += kSolveThreads) {
      double s = 0;
#pragma unroll
      for (int k = 0; k < 16; ++k) s = fma(rowK[k * LD + r], y[k0 + k], s);
      y[r] -= s;
    }
    __syncthreads();
  }
  const double* src = a.sys;
  const double* hm = nullptr;  // (in a.sys already)
  double sc = 0;
  for (int r = t; r < n; r += kSolveThreads) {
    const double xv = y[r];
    a.xp[r] = xv;
    sc += xv * (lambda * xv + src[(size_t)n * n + n + r] + (hm ? hm[(size_t)n * n + r] : 0.0));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) sc += __shfl_xor(sc, o, 64);
  if (lane == 0) red[wave] = sc;
  __syncthreads();
  if (t == 0) {
    double v = 0;
#pragma unroll
    for (int w = 0; w < kSolveWaves; ++w) v += red[w];
    a.scal[0] = v;
    a.scal[1] = *h.bad;
  }
}


// Trial key-frame states: ImuCamPose::Update of VP (g2o_types.cc:192-216) and
// the additive VV / VG / VA updates from the reduced solve (fixed key frames
// copied); src: key frame k's current state (33 doubles), dst may be src.
// Per-lane branches (each lane may hold another key frame): the link
// kernel's trial states and k_lba_trial's are the same bits.
__device__ __forceinline__ void lia_trial_state(const LbaArgs& a, int k, const double* src, double* dst) {
  const int h = a.hidx[k];
  if (h < 0) {
    if (dst != src)
      for (int i = 0; i < kImuStateStride; ++i) dst[i] = src[i];
    return;
  }
  StateD s;
  load_state(s, src);
  const double* u = a.xp + kImuDim * h;
  double up[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) up[i] = u[i];
  pose_update<false>(s, up, calib_of(a), true);
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    s.v[i] += u[6 + i];
    s.bg[i] += u[9 + i];
    s.ba[i] += u[12 + i];
  }
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    dst[i] = s.Rwb[i];
    dst[12 + i] = s.Rcw[i];
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    dst[9 + i] = s.twb[i];
    dst[21 + i] = s.tcw[i];
    dst[24 + i] = s.v[i];
    dst[27 + i] = s.bg[i];
    dst[30 + i] = s.ba[i];
  }
}

// ---- the trial poses T' = exp(x_p) T (free keyframes; fixed ones copied)
__device__ __forceinline__ void trial_pose(const LbaArgs& a, int s0, int k, double* out) {
  Se3 T = load_pose(a.poses[s0] + 7 * k);
  const int h = a.hidx[k];
  if (h >= 0) {
    double u[6];
#pragma unroll
    for (int s = 0; s < 6; ++s) u[s] = a.xp[6 * h + s];
    T = se3_compose(se3_exp<false>(u), T);
  }
  store_pose(T, out);
}

// windows with more keyframes than the LDS table holds: the trial poses go
// to the state buffer first
__global__ __launch_bounds__(kThreads) void k_lba_trial_poses(LbaArgs a) {
  const LbaCtrl& c = *a.ctrl;
  if (c.done) return;
  const int k = blockIdx.x * kThreads + threadIdx.x;
  if (k < a.n_kf) trial_pose(a, c.state, k, a.poses[c.state ^ 1] + 7 * k);
}

// ---- one LM trial, edge side: back-substitution x_l = Dinv (b_l - sum
// Hpl^T x_p) of the block's points (a thread per point; the block holding a
// point's first edge writes it), each edge's error and robust chi2 at the trial state
// (computeActiveErrors), the landmark part of computeScale; the last block
// sums the partials in block order and takes the LM decision.
// kModelImu: the trial key-frame states come from k_lia_trial_states.
template <int M>
__global__ __launch_bounds__(kThreads) void k_lba_trial(LbaArgs a) {
  __shared__ double red[4 * 3];
  const LbaCtrl& c = *a.ctrl;
  if (c.done) return;
  const double lambda = c.lambda;
  const int s0 = c.state, s1 = s0 ^ 1;
  const double* tposes = a.poses[s1];
  const double* const hpl0 = lin_of(a, s0).hpl;
  if constexpr (M == kModelSe3) {
    __shared__ double tp[kMaxKfLds * 7];
    if (a.n_kf <= kMaxKfLds) {
      for (int k = threadIdx.x; k < a.n_kf; k += kThreads) {
        trial_pose(a, s0, k, tp + 7 * k);
        if (blockIdx.x == 0)
#pragma unroll
          for (int q = 0; q < 7; ++q) a.poses[s1][7 * k + q] = tp[7 * k + q];
      }
      tposes = tp;  // (read after the back-substitution's barrier below)
    }
  } else {
    // the trial key-frame states, every block its own copy in LDS (block 0
    // also writes the state buffer); larger windows: k_lia_trial_states
    __shared__ double ts[kMaxKfImuLds * kImuStateStride];
    if (a.n_kf <= kMaxKfImuLds) {
      for (int k = threadIdx.x; k < a.n_kf; k += kThreads) {
        double* const d = ts + kImuStateStride * k;
        lia_trial_state(a, k, a.poses[s0] + kImuStateStride * k, d);
        if (blockIdx.x == 0)
          for (int q = 0; q < kImuStateStride; ++q) a.poses[s1][kImuStateStride * k + q] = d[q];
      }
      tposes = ts;  // (read after the barrier below / the back-substitution's)
    }
  }
  const int i = blockIdx.x * kThreads + threadIdx.x;
  double part[3] = {0, 0, 0};  // robust chi2, landmark scale, singular landmark blocks
  // kModelImu: blocks past the edges' take the IMU links, a block per link,
  // at the trial states of the LDS table (the same bits the edges use): each
  // link's chi2 to imu_tot[2 + l] and, speculatively, its form into the
  // other copy of imu_q -- in the same launch as the edges, not after them
  bool link_block = false;
  if constexpr (M == kModelImu) {
    __shared__ LinkLds lsh;
    const int neb = (max(a.n_edges, 1) + kThreads - 1) / kThreads;
    if ((int)blockIdx.x >= neb) {
      const int l = (int)blockIdx.x - neb;
      __syncthreads();  // the trial states' table
      if (l < a.n_imu) {  // (block-uniform)
        const double chi = lia_link<true>(a, l, threadIdx.x, tposes, nullptr, s1, lsh);
        if (threadIdx.x == 0) st_wt(a.imu_tot + 2 + l, chi);
      }
      link_block = true;
    }
  }
  if (!link_block) {  // (block-uniform)
  // the points of this block's edges (a contiguous range: edges are point-
  // major), each back-substituted once by one thread into LDS -- not once per
  // edge; the block holding a point's first edge writes it and adds its
  // landmark scale and failure
  // (points past the first kThreads of the range -- only edgeless points
  // between can make it longer -- are read back from pts[s1]: every point
  // but the first has its first edge here, so this block wrote it)
  __shared__ double sX[kThreads * 3];
  const int i_first = blockIdx.x * kThreads;
  int pA = 0, n_bp = 0;
  if (i_first < a.n_edges) {
    pA = a.edges[i_first].point;
    n_bp = a.edges[min(i_first + kThreads, a.n_edges) - 1].point - pA + 1;
  }
  // (the points are dealt starting from the second wave: threads k < n_kf
  // stage the trial poses / states above -- only wave 0 when n_kf <= 64, as
  // in the C4 / LIA windows the overlap was measured on -- and this rotation
  // puts wave 0 last in the back-substitution, so the two run side by side
  // up to the one barrier below, which makes any n_kf correct)
  for (int k = (threadIdx.x + kThreads - 64) % kThreads; k < n_bp; k += kThreads) {
    const int p = pA + k;
    const int e0 = a.pt_begin[p], e1 = a.pt_begin[p + 1];
    const double* blp = a.bl + 3 * (size_t)p;
    double cp[3] = {blp[0], blp[1], blp[2]};
    for (int base = e0; base < e1; base += 4) {  // four edges' loads in flight
      int fs[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) fs[u] = base + u < e1 ? a.ef[base + u] : -1;
      double B[4][18], xv[4][6];
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int q = 0; q < 18; ++q) B[u][q] = fs[u] >= 0 ? hpl0[18 * (size_t)(base + u) + q] : 0.0;
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int q = 0; q < 6; ++q) xv[u][q] = fs[u] >= 0 ? a.xp[a.pdim * fs[u] + q] : 0.0;
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (fs[u] >= 0)
#pragma unroll
          for (int b2 = 0; b2 < 3; ++b2)
#pragma unroll
            for (int s = 0; s < 6; ++s) cp[b2] -= B[u][3 * s + b2] * xv[u][s];
    }
    double Di[9];
    const double det = inv3_lambda(a.hll + 9 * (size_t)p, lambda, Di);
    const double* X0 = a.pts[s0] + 3 * (size_t)p;
    double X[3], v[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      v[r] = Di[3 * r] * cp[0] + Di[3 * r + 1] * cp[1] + Di[3 * r + 2] * cp[2];
      X[r] = X0[r] + v[r];
      if (k < kThreads) sX[3 * k + r] = X[r];
    }
    if (e0 >= i_first) {
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        a.pts[s1][3 * (size_t)p + r] = X[r];
        part[1] += v[r] * (lambda * v[r] + blp[r]);
      }
      part[2] = det == 0 ? 1.0 : 0.0;
    }
  }
  __syncthreads();
  if (i < a.n_edges) {
    const LbaEdgeDev e = a.edges[i];
    const int k = e.point - pA;
    const double* xs = k < kThreads ? sX + 3 * k : a.pts[s1] + 3 * (size_t)e.point;
    const double X[3] = {xs[0], xs[1], xs[2]};
    double err[3];
    vis_error<M>(a, e, tposes + a.pstride * e.kf, X, err);
    a.err[3 * i] = err[0];
    a.err[3 * i + 1] = err[1];
    a.err[3 * i + 2] = err[2];
    double w;
    huber_rho(lba_chi2(e, err), lba_delta(e), part[0], w);
    // the trial state's per-edge terms, for the build that follows if the
    // trial is accepted (LinPtr above)
    lin_edge<M>(a, e, i, tposes + a.pstride * e.kf, X, err, lin_of(a, s1));
  }
  }  // !link_block
  block_sum<3>(part, red);
  if (threadIdx.x == 0)
#pragma unroll
    for (int k = 0; k < 3; ++k) st_wt(a.partials + 3 * blockIdx.x + k, part[k]);
  if (!last_block_wt(a.counter + 2)) return;
  double s[3];
  sum_partials<3>(a.partials, gridDim.x, s, red);
  if (threadIdx.x == 0) {
    if (M == kModelImu) {  // the IMU links at the trial state (this launch's link waves), in link order
      double tot = 0;
      for (int k = 0; k < a.n_imu; ++k) tot += a.imu_tot[2 + k];
      s[0] += tot;
    }
    if (a.n_edgeless > 0) {  // points without edges: (0 + lambda I)^-1
      const double h0[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
      double Di[9];
      if (inv3_lambda(h0, lambda, Di) == 0) s[2] += 1;
    }
    const int stop = host_stop(a);
    if (a.sharded) {
      a.red[0] = s[0];
      a.red[1] = s[1];
      a.red[2] = s[2];
      a.red[3] = stop;
    } else {
      ctl_decide(a, s[0], s[1], s[2] > 0 || a.scal[1] != 0, stop);
    }
  }
}

// ---- LM decisions of a point-sharded run, after the host's all-reduce
__global__ void k_lba_ctl(LbaArgs a, int mode) {
  if (threadIdx.x != 0) return;
  LbaCtrl& c = *a.ctrl;
  if (mode == kCtlInit) {
    ctl_init(a, a.red[0], a.red[1] > 0);
    return;
  }
  if (c.done) return;
  if (mode == kCtlLambda) {
    // due once, after the first build (k_lba_sums sets the flag when it == 0);
    // a stream-ordered run enqueues this every step
    if (!c.lambda_due) return;
    c.lambda_due = 0;
    double m = a.diag[a.n_sys];
    for (int k = 0; k < a.n_sys; ++k)
      if (k % a.pdim < 6) m = fmax(m, fabs(a.diag[k]));  // pose rows (see k_lba_sums)
    ctl_lambda(a, m);
    return;
  }
  ctl_decide(a, a.red[0], a.red[1], a.red[2] > 0 || a.scal[1] != 0, a.red[3] > 0);
}

// ---- optimizer.cc:1362-1400: chi2 of the last computeActiveErrors, depth at
// the final estimates; the final state copied out in one buffer.
// kModelImu: optimizer.cc:2799-2826 -- the float thresholds chi2Mono2 =
// 5.991f (1.5f * 5.991f for a close point) and chi2Stereo2 = 7.815f, depth
// only for mono edges.
template <int M>
__global__ __launch_bounds__(kThreads) void k_lba_classify(LbaArgs a, uint8_t* __restrict__ outlier,
                                                           double* __restrict__ out,
                                                           uint32_t* __restrict__ ctrl_out) {
  const int i = blockIdx.x * kThreads + threadIdx.x;
  if (i < classify_items(a)) classify_elem<M>(a, a.ctrl->state, i, outlier, out, ctrl_out);
}

template <int M>
__global__ __launch_bounds__(kThreads) void k_lba_classify_host(LbaArgs a) {
  if (a.ctrl->classified) return;
  classify_to_host<M>(a);
}

// windows with more key frames than k_lba_trial<kModelImu> stages in LDS
// (kMaxKfImuLds): the trial states to the state buffer first, a thread per
// key frame
__global__ __launch_bounds__(kThreads) void k_lia_trial_states(LbaArgs a) {
  const LbaCtrl& c = *a.ctrl;
  if (c.done) return;
  const int k = blockIdx.x * kThreads + threadIdx.x;
  if (k < a.n_kf)
    lia_trial_state(a, k, a.poses[c.state] + kImuStateStride * k, a.poses[c.state ^ 1] + kImuStateStride * k);
}

inline unsigned blocks(long n, int t) { return (unsigned)((n + t - 1) / t); }

}  // namespace

size_t lba_solve_lds_bytes(int n_pad) {
  const size_t T = (size_t)n_pad / 16;
  return 8 * (T * (T + 1) / 2 * kTileSz + T * kTileSz + 2 * (size_t)n_pad + (size_t)kSolveWaves * kTileSz);
}

// LDS a workgroup may hold, less a margin for the solve kernels' static
// __shared__ arrays (red[kSolveWaves] and a flag: < 100 B) next to the
// dynamic block
constexpr size_t kLdsBudget = 160 * 1024;
constexpr size_t kStaticLdsMargin = 1024;
static_assert(sizeof(double) * kSolveWaves + sizeof(int) <= kStaticLdsMargin, "static LDS margin");

// One block factorises up to this many padded rows from HBM (kSolveBlock);
// larger systems take the device-wide path (orbgpu_lba_ctx_set_solver forces
// either for A/B timing).
constexpr int kGridMinPad = 224;  // tools/lba_solver_ab.py: block wins at 176 rows, grid at 272

bool lba_solve_mode_fits(int mode, int n_pad) {
  switch (mode) {
    case kSolveLds:
      return lba_solve_lds_bytes(n_pad) + kStaticLdsMargin <= kLdsBudget;
    case kSolveBlock:
      return 16 * (size_t)n_pad + kStaticLdsMargin <= kLdsBudget;
    default:
      return true;
  }
}

int lba_solve_mode(int n_pad) {
  if (lba_solve_mode_fits(kSolveLds, n_pad)) return kSolveLds;
  if (n_pad < kGridMinPad && lba_solve_mode_fits(kSolveBlock, n_pad)) return kSolveBlock;
  return kSolveGrid;
}

size_t lba_solve_work_doubles(int mode, int n_pad) {
  const size_t N = n_pad, T = N / 16;
  switch (mode) {
    case kSolveLds:
      return 2;
    case kSolveBlock:
      return N * (N + 1) + T * kTileSz;  // S + the L_KK^-1 tiles
    default:
      return N * (N + 1) + T * kTileSz + 3 * N + 2;  // S, L_KK^-1 tiles, D, y, ys, flag (hbm_solve)
  }
}

hipError_t lba_begin(const LbaArgs& a, hipStream_t st) {
  const dim3 g(blocks(a.n_edges > 0 ? a.n_edges : 1, kThreads));
  if (a.model == kModelImu) {
    // the links ride in the launch: n_imu more blocks, a block per link
    hipLaunchKernelGGL(k_lba_begin<kModelImu>, dim3(g.x + a.n_imu), dim3(kThreads), 0, st, a);
  } else {
    hipLaunchKernelGGL(k_lba_begin<kModelSe3>, g, dim3(kThreads), 0, st, a);
  }
  return hipGetLastError();
}

hipError_t lba_build(const LbaArgs& a, hipStream_t st, bool linearize) {
  const bool imu = a.model == kModelImu;
  // (before k_lba_sums, which closes the build: need_build = 0) kModelImu:
  // the first build's link forms come from k_lba_begin and every later
  // build's from the accepted trial; only when every build relinearises
  // (force_lin) do the links ride in this launch, n_imu more blocks
  const unsigned lin_blocks =
      blocks(a.n_edges, kThreads) + (imu && a.force_lin && a.n_sys > 0 ? a.n_imu : 0);
  if (linearize && lin_blocks > 0) {
    if (imu)
      hipLaunchKernelGGL(k_lba_linearize<kModelImu>, dim3(lin_blocks), dim3(kThreads), 0, st, a);
    else
      hipLaunchKernelGGL(k_lba_linearize<kModelSe3>, dim3(lin_blocks), dim3(kThreads), 0, st, a);
  }
  // kModelImu: extra blocks assemble the links' part of the system
  const unsigned asm_blocks = imu && a.n_sys > 0 ? blocks((long)a.n_sys * a.n_sys + a.n_sys, kThreads) : 0;
  const dim3 sg(kSumsQ * a.n_free + blocks(a.n_pts > 0 ? a.n_pts : 1, kThreads) + asm_blocks);
  if (imu)
    hipLaunchKernelGGL(k_lba_sums<kModelImu>, sg, dim3(kThreads), 0, st, a);
  else
    hipLaunchKernelGGL(k_lba_sums<kModelSe3>, sg, dim3(kThreads), 0, st, a);
  return hipGetLastError();
}

hipError_t lba_schur(const LbaArgs& a, hipStream_t st) {
  if (a.n_pairs <= 0) return hipSuccess;
  if (a.sc_split > 0) {
    hipLaunchKernelGGL(k_lba_schur_split, dim3(a.n_pairs * a.sc_split), dim3(kSplitThreads), 0, st, a);
    if (a.sc_split > 1 && !a.sc_fold_inline)
      hipLaunchKernelGGL(k_lba_schur_fold, dim3(a.n_pairs), dim3(64), 0, st, a);
  } else if (a.n_chunks > 0) {
    if (lds_optin(reinterpret_cast<const void*>(&k_lba_schur_band), kSchurChunkLds) != hipSuccess)
      return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_lba_schur_band, dim3(a.n_chunks), dim3(kBandThreads), kSchurChunkLds, st, a);
    hipLaunchKernelGGL(k_lba_schur_sum, dim3(a.n_pairs), dim3(64), 0, st, a);
  } else {
    hipLaunchKernelGGL(k_lba_schur, dim3(a.n_pairs), dim3(kSchurThreads), 0, st, a);
  }
  return hipGetLastError();
}

hipError_t lba_solve_trial(const LbaArgs& a, hipStream_t st) {
  if (a.solve_mode == kSolveLds) {
    const size_t lds = lba_solve_lds_bytes(a.n_pad);
    if (lds > 64 * 1024 &&
        lds_optin(reinterpret_cast<const void*>(&k_lba_solve<true>), (int)lds) != hipSuccess)
      return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_lba_solve<true>, dim3(1), dim3(kSolveThreads), lds, st, a);
  } else if (a.solve_mode == kSolveBlock) {
    const size_t lds = 16 * (size_t)a.n_pad;  // D and y (lba_solve_mode bounds it)
    if (lds > 64 * 1024 &&
        lds_optin(reinterpret_cast<const void*>(&k_lba_solve<false>), (int)lds) != hipSuccess)
      return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_lba_solve<false>, dim3(1), dim3(kSolveThreads), lds, st, a);
  } else {
    const int T = a.n_pad >> 4;
    hipLaunchKernelGGL(k_lba_ldl_stage, dim3(a.n_pad), dim3(kThreads), 0, st, a);
    for (int K = 0; K < T; ++K) {
      const int m = T - K - 1;
      hipLaunchKernelGGL(k_lba_ldl_panel, dim3(m > 0 ? blocks(m, kSolveWaves) : 1), dim3(kSolveThreads), 0, st,
                         a, K);
      if (m > 0)
        hipLaunchKernelGGL(k_lba_ldl_update, dim3(blocks((long)m * (m + 1) / 2, kSolveWaves)),
                           dim3(kSolveThreads), 0, st, a, K);
    }
    hipLaunchKernelGGL(k_lba_ldl_back, dim3(1), dim3(kSolveThreads), 0, st, a);
  }
  const dim3 g(blocks(a.n_edges > 0 ? a.n_edges : 1, kThreads));
  if (a.model == kModelImu) {
    if (a.n_kf > kMaxKfImuLds)
      hipLaunchKernelGGL(k_lia_trial_states, dim3(blocks(a.n_kf, kThreads)), dim3(kThreads), 0, st, a);
    // the links ride in the trial launch: n_imu more blocks, a block per link
    hipLaunchKernelGGL(k_lba_trial<kModelImu>, dim3(g.x + a.n_imu), dim3(kThreads), 0, st, a);
  } else {
    if (a.n_kf > kMaxKfLds)
      hipLaunchKernelGGL(k_lba_trial_poses, dim3(blocks(a.n_kf, kThreads)), dim3(kThreads), 0, st, a);
    hipLaunchKernelGGL(k_lba_trial<kModelSe3>, g, dim3(kThreads), 0, st, a);
  }
  return hipGetLastError();
}

hipError_t lba_step(const LbaArgs& a, hipStream_t st, bool linearize) {
  hipError_t e = lba_build(a, st, linearize);
  if (e == hipSuccess) e = lba_schur(a, st);
  if (e == hipSuccess) e = lba_solve_trial(a, st);
  return e;
}

hipError_t lba_ctl(const LbaArgs& a, int mode, hipStream_t st) {
  hipLaunchKernelGGL(k_lba_ctl, dim3(1), dim3(64), 0, st, a, mode);
  return hipGetLastError();
}

hipError_t lba_classify_to_host(const LbaArgs& a, hipStream_t st) {
  long n = a.n_edges;
  if ((long)a.pstride * a.n_kf > n) n = (long)a.pstride * a.n_kf;
  if (3L * a.n_pts > n) n = 3L * a.n_pts;
  if (a.model == kModelImu)
    hipLaunchKernelGGL(k_lba_classify_host<kModelImu>, dim3(blocks(n > 0 ? n : 1, kThreads)), dim3(kThreads), 0, st, a);
  else
    hipLaunchKernelGGL(k_lba_classify_host<kModelSe3>, dim3(blocks(n > 0 ? n : 1, kThreads)), dim3(kThreads), 0, st, a);
  return hipGetLastError();
}

hipError_t lba_classify(const LbaArgs& a, uint8_t* outlier, double* out, void* ctrl_out, hipStream_t st) {
  long n = a.n_edges;
  if ((long)a.pstride * a.n_kf > n) n = (long)a.pstride * a.n_kf;
  if (3L * a.n_pts > n) n = 3L * a.n_pts;
  if (a.model == kModelImu)
    hipLaunchKernelGGL(k_lba_classify<kModelImu>, dim3(blocks(n > 0 ? n : 1, kThreads)), dim3(kThreads), 0,
                       st, a, outlier, out, static_cast<uint32_t*>(ctrl_out));
  else
    hipLaunchKernelGGL(k_lba_classify<kModelSe3>, dim3(blocks(n > 0 ? n : 1, kThreads)), dim3(kThreads), 0,
                       st, a, outlier, out, static_cast<uint32_t*>(ctrl_out));
  return hipGetLastError();
}

}  // namespace orbgpu

ORBGPU_UNIFORM_READER(lba)
