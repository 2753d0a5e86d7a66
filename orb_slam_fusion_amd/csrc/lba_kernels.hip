// gfx950 LocalBundleAdjustment (Optimizer::LocalBundleAdjustment,
// src/solver/g2o_solver/optimizer.cc:1127-1441): g2o Levenberg-Marquardt over
// SE3 keyframe poses and marginalized XYZ points (BlockSolver_6_3 Schur
// complement, core/block_solver.hpp:364-514), fp64 throughout.
//
// One kernel per stage of an LM trial; the host drives the LM loop
// (lba_api.cpp) exactly as oracle/lba_oracle.cc does.  Every sum has a fixed
// order (per-point loops over the point's edges in insertion order, per-pose
// block reductions with a fixed tree, last-block-done partial sums in block
// order), so results are reproducible run to run.
//
// Layout (per call, this rank's point shard):
//   edges in point-major order (CSR pt_begin), pose-major index lists (CSR per
//   free pose) and, per free-pose pair (i <= j) sharing points, the list of
//   (edge of i, edge of j) pairs that the Schur complement sums over.
#include <hip/hip_runtime.h>

#include "lds_optin.h"
#include <stdint.h>

#include "lba_launch.h"
#include "pose_math_dev.h"

namespace orbgpu {

namespace {

constexpr int kLbaThreads = 256;

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

// error of one edge (EdgeSE3ProjectXYZ / EdgeStereoSE3ProjectXYZ); returns
// isDepthPositive on the same state
__device__ __forceinline__ bool lba_error(const LbaEdgeDev& e, const Se3& T, const double X[3],
                                          const LbaCamDev& c, double err[3]) {
  double p[3];
  se3_map(T, X, p);
  if (e.ur < 0.f) {
    err[0] = (double)e.u - (c.fx * p[0] / p[2] + c.cx);
    err[1] = (double)e.v - (c.fy * p[1] / p[2] + c.cy);
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
  if (e.ur < 0.f) {
    const double pj[2][3] = {{-(c.fx / z), 0.0, -(-c.fx * x / (z * z))},
                             {0.0, -(c.fy / z), -(-c.fy * y / (z * z))}};
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
  } else {
    const double z_2 = z * z, fx = c.fx, fy = c.fy, bf = c.bf;
#pragma unroll
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

// Fixed-tree block sum of one double (256 threads); valid in thread 0.
__device__ __forceinline__ double lba_block_sum(double v, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  const double r = ((red[0] + red[1]) + red[2]) + red[3];
  __syncthreads();
  return r;
}

// Last-block-done finish: block partials summed in block order into *out.
__device__ __forceinline__ void lba_finish_sum(double partial, volatile double* partials,
                                               unsigned* counter, double* out) {
  __shared__ bool last;
  if (threadIdx.x == 0) {
    partials[blockIdx.x] = partial;
    __threadfence();
    last = atomicAdd(counter, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (last && threadIdx.x == 0) {
    __threadfence();
    double s = 0;
    for (unsigned b = 0; b < gridDim.x; ++b) s += partials[b];
    *out = s;
    *counter = 0;
  }
}

__device__ __forceinline__ void atomic_max_pos(double* p, double v) {  // v >= 0
  atomicMax(reinterpret_cast<unsigned long long*>(p), (unsigned long long)__double_as_longlong(v));
}

// ---- computeActiveErrors + robust chi2 over this shard's edges at a state
__global__ __launch_bounds__(kLbaThreads) void k_lba_errors(LbaArgs a, const double* __restrict__ poses,
                                                            const double* __restrict__ pts, double* out) {
  __shared__ double red[4];
  const int i = blockIdx.x * kLbaThreads + threadIdx.x;
  double r0 = 0;
  if (i < a.n_edges) {
    const LbaEdgeDev e = a.edges[i];
    const Se3 T = load_pose(poses + 7 * e.kf);
    const double X[3] = {pts[3 * e.point], pts[3 * e.point + 1], pts[3 * e.point + 2]};
    double err[3];
    lba_error(e, T, X, a.cam, err);
    a.err[3 * i] = err[0];
    a.err[3 * i + 1] = err[1];
    a.err[3 * i + 2] = err[2];
    double w;
    huber_rho(lba_chi2(e, err), lba_delta(e), r0, w);
  }
  const double s = lba_block_sum(r0, red);
  lba_finish_sum(s, a.partials, a.counter, out);
}

// ---- buildSystem, edge side: one thread per edge of the shard.  Its
// Jacobians at the current state and its terms of Hll / bl (point), Hpl and
// Hpp / bp (free pose) -- summed per point and per pose in fixed order below.
__global__ __launch_bounds__(kLbaThreads) void k_lba_linearize(LbaArgs a, const double* __restrict__ poses,
                                                               const double* __restrict__ pts) {
  const int i = blockIdx.x * kLbaThreads + threadIdx.x;
  if (i >= a.n_edges) return;
  const LbaEdgeDev e = a.edges[i];
  const double X[3] = {pts[3 * e.point], pts[3 * e.point + 1], pts[3 * e.point + 2]};
  const Se3 T = load_pose(poses + 7 * e.kf);
  const double ev[3] = {a.err[3 * i], a.err[3 * i + 1], a.err[3 * i + 2]};
  const int D = e.ur < 0.f ? 2 : 3;
  double Jl[3][3], Jp[3][6];
  lba_jacobians(e, T, X, a.cam, Jl, Jp);
  double r0, w;
  huber_rho(lba_chi2(e, ev), lba_delta(e), r0, w);
  const double info = (double)e.inv_sigma2, wi = w * info;
  double om[3];
#pragma unroll
  for (int r = 0; r < 3; ++r) om[r] = (-info * ev[r]) * w;
  double* hl = a.hll_e + 12 * (size_t)i;  // 9 Hll terms (row-major), 3 bl terms
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    double g = 0;
    for (int r = 0; r < D; ++r) g += Jl[r][s] * om[r];
    hl[9 + s] = g;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      double h = 0;
      for (int r = 0; r < D; ++r) h += Jl[r][s] * wi * Jl[r][q];
      hl[3 * s + q] = h;
    }
  }
  if (a.hidx[e.kf] < 0) return;
  double* hpl = a.hpl + 18 * (size_t)i;
  double* hp = a.hpp_e + 27 * (size_t)i;  // 21 lower-triangle Hpp terms, then 6 bp terms
  int hk = 0;
#pragma unroll
  for (int s = 0; s < 6; ++s) {
    double g = 0;
    for (int r = 0; r < D; ++r) g += Jp[r][s] * om[r];
    hp[21 + s] = g;
#pragma unroll
    for (int q = 0; q <= s; ++q) {
      double h = 0;
      for (int r = 0; r < D; ++r) h += Jp[r][s] * wi * Jp[r][q];
      hp[hk++] = h;
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      double h = 0;
      for (int r = 0; r < D; ++r) h += Jp[r][s] * wi * Jl[r][q];
      hpl[3 * s + q] = h;
    }
  }
}

// ---- buildSystem, point side: one thread per point sums its edges' Hll / bl
// terms in insertion order (as g2o adds them edge by edge).
__global__ __launch_bounds__(kLbaThreads) void k_lba_point_sum(LbaArgs a) {
  const int p = blockIdx.x * kLbaThreads + threadIdx.x;
  if (p >= a.n_pts) return;
  double H[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = a.pt_begin[p]; i < a.pt_begin[p + 1]; ++i) {
    const double* hl = a.hll_e + 12 * (size_t)i;
#pragma unroll
    for (int k = 0; k < 12; ++k) H[k] += hl[k];
  }
#pragma unroll
  for (int k = 0; k < 9; ++k) a.hll[9 * (size_t)p + k] = H[k];
#pragma unroll
  for (int k = 0; k < 3; ++k) a.bl[3 * (size_t)p + k] = H[9 + k];
  atomic_max_pos(a.diag + a.n_sys, fmax(fabs(H[0]), fmax(fabs(H[4]), fabs(H[8]))));  // Hll max
}

// ---- buildSystem, pose side: one block per free pose, its edges strided over
// the threads, a fixed tree per term.  -> Hpp (6x6 full) and bp.
__global__ __launch_bounds__(kLbaThreads) void k_lba_pose_sum(LbaArgs a) {
  __shared__ double red[4 * 27];
  const int f = blockIdx.x;
  double acc[27];
#pragma unroll
  for (int k = 0; k < 27; ++k) acc[k] = 0;
  for (int j = a.pose_begin[f] + threadIdx.x; j < a.pose_begin[f + 1]; j += kLbaThreads) {
    const double* hp = a.hpp_e + 27 * (size_t)a.pose_edges[j];
#pragma unroll
    for (int k = 0; k < 27; ++k) acc[k] += hp[k];
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < 27; ++k) {
    double v = acc[k];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) red[27 * wave + k] = v;
  }
  __syncthreads();
  if (threadIdx.x < 27) {
    const int k = threadIdx.x;
    const double v = ((red[k] + red[27 + k]) + red[54 + k]) + red[81 + k];
    if (k < 21) {
      // lower-triangle index k -> (s, q)
      int s = 0, q = k;
      while (q > s) {
        q -= s + 1;
        ++s;
      }
      a.hpp[36 * (size_t)f + 6 * s + q] = v;
      a.hpp[36 * (size_t)f + 6 * q + s] = v;
      if (s == q) a.diag[6 * f + s] = v;  // this shard's Hpp diagonal (lambda init, summed over ranks)
    } else {
      a.bp[6 * (size_t)f + (k - 21)] = v;
    }
  }
}

// ---- Schur, point side (per trial lambda): Dinv = (Hll + lambda I)^-1 by
// cofactors (Eigen compute_inverse_size3).
__global__ __launch_bounds__(kLbaThreads) void k_lba_schur_points(LbaArgs a, double lambda) {
  const int p = blockIdx.x * kLbaThreads + threadIdx.x;
  if (p >= a.n_pts) return;
  double A[3][3];
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c) A[r][c] = a.hll[9 * (size_t)p + 3 * r + c] + (r == c ? lambda : 0.0);
  const double c00 = A[1][1] * A[2][2] - A[1][2] * A[2][1];
  const double c10 = A[1][2] * A[2][0] - A[1][0] * A[2][2];
  const double c20 = A[1][0] * A[2][1] - A[1][1] * A[2][0];
  const double det = A[0][0] * c00 + A[0][1] * c10 + A[0][2] * c20;
  if (det == 0) a.flags[0] = 1;  // singular landmark block: the trial fails (tmp = DBL_MAX)
  const double id = det != 0 ? 1.0 / det : 0.0;
  double* Di = a.dinv + 9 * (size_t)p;
  Di[0] = c00 * id;
  Di[3] = c10 * id;
  Di[6] = c20 * id;
  Di[1] = (A[0][2] * A[2][1] - A[0][1] * A[2][2]) * id;
  Di[4] = (A[0][0] * A[2][2] - A[0][2] * A[2][0]) * id;
  Di[7] = (A[0][1] * A[2][0] - A[0][0] * A[2][1]) * id;
  Di[2] = (A[0][1] * A[1][2] - A[0][2] * A[1][1]) * id;
  Di[5] = (A[0][2] * A[1][0] - A[0][0] * A[1][2]) * id;
  Di[8] = (A[0][0] * A[1][1] - A[0][1] * A[1][0]) * id;
}

// W = Hpl_e Dinv_point (6 x 3)
__device__ __forceinline__ void lba_w(const double* __restrict__ B, const double* __restrict__ Di,
                                      double W[6][3]) {
#pragma unroll
  for (int s = 0; s < 6; ++s)
#pragma unroll
    for (int c = 0; c < 3; ++c) W[s][c] = B[3 * s] * Di[c] + B[3 * s + 1] * Di[3 + c] + B[3 * s + 2] * Di[6 + c];
}

// ---- Schur, pose side: one 256-thread block per free-pose pair (i <= j)
// sharing points.  The pair's (edge of i, edge of j) entries are strided
// over the threads (each computes W_i Hpl_j^T, W from the point's Dinv),
// then a fixed tree per entry of the 6 x 6 block:
//   S_ij = [i == j] Hpp_i - sum W_i Hpl_j^T;
// diagonal pairs also produce b_s = bp - sum over the pose's edges W bl.
__global__ __launch_bounds__(kLbaThreads) void k_lba_schur_pairs(LbaArgs a) {
  __shared__ double red[4 * 42];
  const int pr = blockIdx.x;
  const int fi = a.pair_i[pr], fj = a.pair_j[pr];
  const int n = a.n_sys;
  double acc[42];
#pragma unroll
  for (int k = 0; k < 42; ++k) acc[k] = 0;
  for (int k = a.pair_begin[pr] + threadIdx.x; k < a.pair_begin[pr + 1]; k += kLbaThreads) {
    const int ei = a.pair_ei[k], ej = a.pair_ej[k];
    double W[6][3];
    lba_w(a.hpl + 18 * (size_t)ei, a.dinv + 9 * (size_t)a.edges[ei].point, W);
    const double* B = a.hpl + 18 * (size_t)ej;
#pragma unroll
    for (int s = 0; s < 6; ++s)
#pragma unroll
      for (int q = 0; q < 6; ++q) acc[6 * s + q] += W[s][0] * B[3 * q] + W[s][1] * B[3 * q + 1] + W[s][2] * B[3 * q + 2];
  }
  if (fi == fj) {
    for (int j = a.pose_begin[fi] + threadIdx.x; j < a.pose_begin[fi + 1]; j += kLbaThreads) {
      const int e = a.pose_edges[j];
      const int p = a.edges[e].point;
      double W[6][3];
      lba_w(a.hpl + 18 * (size_t)e, a.dinv + 9 * (size_t)p, W);
      const double* bl = a.bl + 3 * (size_t)p;
#pragma unroll
      for (int s = 0; s < 6; ++s) acc[36 + s] += W[s][0] * bl[0] + W[s][1] * bl[1] + W[s][2] * bl[2];
    }
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < 42; ++k) {
    double v = acc[k];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) red[42 * wave + k] = v;
  }
  __syncthreads();
  const int t = threadIdx.x;
  if (t < 36) {
    const int s = t / 6, q = t - 6 * s;
    const double sum = ((red[t] + red[42 + t]) + red[84 + t]) + red[126 + t];
    const double v = (fi == fj ? a.hpp[36 * (size_t)fi + 6 * s + q] : 0.0) - sum;
    a.sys[(size_t)(6 * fi + s) * n + 6 * fj + q] = v;
    a.sys[(size_t)(6 * fj + q) * n + 6 * fi + s] = v;
  } else if (fi == fj && t < 42) {
    const int s = t - 36;
    const double sum = ((red[t] + red[42 + t]) + red[84 + t]) + red[126 + t];
    a.sys[(size_t)n * n + 6 * fi + s] = a.bp[6 * (size_t)fi + s] - sum;  // b_s
    a.sys[(size_t)n * n + n + 6 * fi + s] = a.bp[6 * (size_t)fi + s];   // b_p (LM scale)
  }
}

// ---- reduced camera system: S + lambda I = L D L^T by 6 x 6 pose blocks
// (no pivoting: the same factorisation as the oracle's scalar LDLT up to
// rounding).  Per block step K: thread 0 factors the diagonal block; every
// row below solves its panel row (l = v / d, v = a L_KK^-T), v kept in the
// mirrored upper position; the trailing lower triangle takes the rank-6
// update.  Then block-column forward / diagonal / backward substitution.
// One block of 1024 threads, S in LDS when it fits.  Also the pose part of
// computeScale and the positivity of the pivots.
__global__ __launch_bounds__(1024) void k_lba_solve(LbaArgs a, double lambda, int in_lds) {
  extern __shared__ double Sl[];
  const int n = a.n_sys, t = threadIdx.x, nt = blockDim.x;
  double* S = in_lds ? Sl : a.work;
  const double* src = a.sys;
  for (int r = t >> 5; r < n; r += nt >> 5)
    for (int c = t & 31; c < n; c += 32) S[(size_t)r * n + c] = src[(size_t)r * n + c] + (r == c ? lambda : 0.0);
  double* y = a.xp;
  for (int i = t; i < n; i += nt) y[i] = src[(size_t)n * n + i];  // b_s
  __shared__ int bad;
  if (t == 0) bad = 0;
  __syncthreads();
  const int nb = n / 6;
  for (int K = 0; K < nb; ++K) {
    const int k0 = 6 * K;
    if (t == 0) {  // scalar LDLT of the (updated) diagonal block, in registers
      double B[6][6];
#pragma unroll
      for (int r = 0; r < 6; ++r)
#pragma unroll
        for (int c = 0; c <= r; ++c) B[r][c] = S[(size_t)(k0 + r) * n + k0 + c];
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        double d = B[c][c];
#pragma unroll
        for (int c2 = 0; c2 < c; ++c2) d -= B[c][c2] * B[c][c2] * B[c2][c2];
        B[c][c] = d;
        if (!(d > 0)) bad = 1;
#pragma unroll
        for (int r = c + 1; r < 6; ++r) {
          double v = B[r][c];
#pragma unroll
          for (int c2 = 0; c2 < c; ++c2) v -= B[r][c2] * B[c][c2] * B[c2][c2];
          B[r][c] = d != 0 ? v / d : 0.0;
        }
      }
#pragma unroll
      for (int r = 0; r < 6; ++r)
#pragma unroll
        for (int c = 0; c <= r; ++c) S[(size_t)(k0 + r) * n + k0 + c] = B[r][c];
    }
    __syncthreads();
    for (int i = k0 + 6 + t; i < n; i += nt) {  // panel rows
      double v[6];
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        double x = S[(size_t)i * n + k0 + c];
        for (int c2 = 0; c2 < c; ++c2) x -= v[c2] * S[(size_t)(k0 + c) * n + k0 + c2];
        v[c] = x;
      }
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        const double d = S[(size_t)(k0 + c) * n + k0 + c];
        S[(size_t)(k0 + c) * n + i] = v[c];
        S[(size_t)i * n + k0 + c] = d != 0 ? v[c] / d : 0.0;
      }
    }
    __syncthreads();
    // trailing lower triangle: thread (row group t >> 5, column lane t & 31)
    for (int ii = k0 + 6 + (t >> 5); ii < n; ii += nt >> 5) {
      double l[6];
#pragma unroll
      for (int c = 0; c < 6; ++c) l[c] = S[(size_t)ii * n + k0 + c];
      for (int jj = k0 + 6 + (t & 31); jj <= ii; jj += 32) {
        double acc = 0;
#pragma unroll
        for (int c = 0; c < 6; ++c) acc += l[c] * S[(size_t)(k0 + c) * n + jj];
        S[(size_t)ii * n + jj] -= acc;
      }
    }
    __syncthreads();
  }
  // forward: unit lower L, block columns
  for (int K = 0; K < nb; ++K) {
    const int k0 = 6 * K;
    if (t == 0) {
      double yy[6];
#pragma unroll
      for (int c = 0; c < 6; ++c) yy[c] = y[k0 + c];
#pragma unroll
      for (int c = 1; c < 6; ++c)
#pragma unroll
        for (int c2 = 0; c2 < c; ++c2) yy[c] -= S[(size_t)(k0 + c) * n + k0 + c2] * yy[c2];
#pragma unroll
      for (int c = 0; c < 6; ++c) y[k0 + c] = yy[c];
    }
    __syncthreads();
    for (int i = k0 + 6 + t; i < n; i += nt) {
      double acc = 0;
#pragma unroll
      for (int c = 0; c < 6; ++c) acc += S[(size_t)i * n + k0 + c] * y[k0 + c];
      y[i] -= acc;
    }
    __syncthreads();
  }
  for (int i = t; i < n; i += nt) {
    const double d = S[(size_t)i * n + i];
    y[i] = d != 0 ? y[i] / d : 0.0;
  }
  __syncthreads();
  // backward: L^T, block columns from the last
  for (int K = nb - 1; K >= 0; --K) {
    const int k0 = 6 * K;
    if (t == 0) {
      double yy[6];
#pragma unroll
      for (int c = 0; c < 6; ++c) yy[c] = y[k0 + c];
#pragma unroll
      for (int c = 4; c >= 0; --c)
#pragma unroll
        for (int c2 = c + 1; c2 < 6; ++c2) yy[c] -= S[(size_t)(k0 + c2) * n + k0 + c] * yy[c2];
#pragma unroll
      for (int c = 0; c < 6; ++c) y[k0 + c] = yy[c];
    }
    __syncthreads();
    for (int r = t; r < k0; r += nt) {
      double acc = 0;
#pragma unroll
      for (int c = 0; c < 6; ++c) acc += S[(size_t)(k0 + c) * n + r] * y[k0 + c];
      y[r] -= acc;
    }
    __syncthreads();
  }
  if (t == 0) {
    double sc = 0;  // x_p . (lambda x_p + b_p)
    for (int i = 0; i < n; ++i) sc += y[i] * (lambda * y[i] + src[(size_t)n * n + n + i]);
    a.scal[0] = sc;
    if (bad) a.flags[0] = 1;
  }
}

// ---- back-substitution and trial state: one thread per point (x_l, trial
// point, landmark part of computeScale) ...
__global__ __launch_bounds__(kLbaThreads) void k_lba_backsub(LbaArgs a, double lambda,
                                                             const double* __restrict__ pts,
                                                             double* __restrict__ pts_trial) {
  __shared__ double red[4];
  const int p = blockIdx.x * kLbaThreads + threadIdx.x;
  double sl = 0;
  if (p < a.n_pts) {
    double cp[3] = {a.bl[3 * (size_t)p], a.bl[3 * (size_t)p + 1], a.bl[3 * (size_t)p + 2]};
    for (int i = a.pt_begin[p]; i < a.pt_begin[p + 1]; ++i) {
      const int h = a.hidx[a.edges[i].kf];
      if (h < 0) continue;
      const double* B = a.hpl + 18 * (size_t)i;
#pragma unroll
      for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int s = 0; s < 6; ++s) cp[c] -= B[3 * s + c] * a.xp[6 * h + s];
    }
    const double* Di = a.dinv + 9 * (size_t)p;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const double v = Di[3 * r] * cp[0] + Di[3 * r + 1] * cp[1] + Di[3 * r + 2] * cp[2];
      pts_trial[3 * (size_t)p + r] = pts[3 * (size_t)p + r] + v;
      sl += v * (lambda * v + a.bl[3 * (size_t)p + r]);
    }
  }
  const double s = lba_block_sum(sl, red);
  lba_finish_sum(s, a.partials, a.counter, a.scal + 1);
}

// ... and one thread per keyframe: T' = exp(x_p) T for free poses.
__global__ __launch_bounds__(64) void k_lba_pose_update(LbaArgs a, const double* __restrict__ poses,
                                                        double* __restrict__ poses_trial) {
  const int k = blockIdx.x * 64 + threadIdx.x;
  if (k >= a.n_kf) return;
  const int h = a.hidx[k];
  Se3 T = load_pose(poses + 7 * k);
  if (h >= 0) {
    double u[6];
#pragma unroll
    for (int s = 0; s < 6; ++s) u[s] = a.xp[6 * h + s];
    T = se3_compose(se3_exp<false>(u), T);
  }
  store_pose(T, poses_trial + 7 * k);
}

// ---- optimizer.cc:1362-1400: chi2 of the last computeActiveErrors, depth at
// the final estimates.
__global__ __launch_bounds__(kLbaThreads) void k_lba_classify(LbaArgs a, const double* __restrict__ poses,
                                                              const double* __restrict__ pts,
                                                              uint8_t* __restrict__ outlier) {
  const int i = blockIdx.x * kLbaThreads + threadIdx.x;
  if (i >= a.n_edges) return;
  const LbaEdgeDev e = a.edges[i];
  const Se3 T = load_pose(poses + 7 * e.kf);
  const double X[3] = {pts[3 * e.point], pts[3 * e.point + 1], pts[3 * e.point + 2]};
  double tmp[3];
  const bool depth = lba_error(e, T, X, a.cam, tmp);
  const double ev[3] = {a.err[3 * i], a.err[3 * i + 1], a.err[3 * i + 2]};
  const double chi = lba_chi2(e, ev);
  outlier[i] = (chi > (e.ur < 0.f ? 5.991 : 7.815) || !depth) ? 1 : 0;
}

inline unsigned blocks(long n, int t) { return (unsigned)((n + t - 1) / t); }

}  // namespace

hipError_t lba_errors(const LbaArgs& a, const double* poses, const double* pts, double* out,
                      hipStream_t st) {
  hipLaunchKernelGGL(k_lba_errors, dim3(blocks(a.n_edges > 0 ? a.n_edges : 1, kLbaThreads)),
                     dim3(kLbaThreads), 0, st, a, poses, pts, out);
  return hipGetLastError();
}

hipError_t lba_build(const LbaArgs& a, const double* poses, const double* pts, hipStream_t st) {
  if (a.n_edges > 0)
    hipLaunchKernelGGL(k_lba_linearize, dim3(blocks(a.n_edges, kLbaThreads)), dim3(kLbaThreads), 0, st,
                       a, poses, pts);
  if (a.n_pts > 0)
    hipLaunchKernelGGL(k_lba_point_sum, dim3(blocks(a.n_pts, kLbaThreads)), dim3(kLbaThreads), 0, st, a);
  if (a.n_free > 0)
    hipLaunchKernelGGL(k_lba_pose_sum, dim3(a.n_free), dim3(kLbaThreads), 0, st, a);
  return hipGetLastError();
}

hipError_t lba_schur(const LbaArgs& a, double lambda, hipStream_t st) {
  if (a.n_pts > 0)
    hipLaunchKernelGGL(k_lba_schur_points, dim3(blocks(a.n_pts, kLbaThreads)), dim3(kLbaThreads), 0,
                       st, a, lambda);
  if (a.n_pairs > 0)
    hipLaunchKernelGGL(k_lba_schur_pairs, dim3(a.n_pairs), dim3(kLbaThreads), 0, st, a);
  return hipGetLastError();
}

hipError_t lba_solve(const LbaArgs& a, double lambda, hipStream_t st) {
  const size_t lds = (size_t)a.n_sys * a.n_sys * sizeof(double);
  const int in_lds = lds <= 150 * 1024 ? 1 : 0;
  if (in_lds && lds > 64 * 1024) {
    if (lds_optin(reinterpret_cast<const void*>(&k_lba_solve), 150 * 1024) != hipSuccess)
      return hipErrorInvalidValue;
  }
  hipLaunchKernelGGL(k_lba_solve, dim3(1), dim3(1024), in_lds ? lds : 0, st, a, lambda, in_lds);
  return hipGetLastError();
}

hipError_t lba_trial(const LbaArgs& a, double lambda, const double* poses, const double* pts,
                     double* poses_trial, double* pts_trial, hipStream_t st) {
  hipLaunchKernelGGL(k_lba_backsub, dim3(blocks(a.n_pts > 0 ? a.n_pts : 1, kLbaThreads)),
                     dim3(kLbaThreads), 0, st, a, lambda, pts, pts_trial);
  hipLaunchKernelGGL(k_lba_pose_update, dim3(blocks(a.n_kf, 64)), dim3(64), 0, st, a, poses,
                     poses_trial);
  return hipGetLastError();
}

hipError_t lba_classify(const LbaArgs& a, const double* poses, const double* pts, uint8_t* outlier,
                        hipStream_t st) {
  if (a.n_edges > 0)
    hipLaunchKernelGGL(k_lba_classify, dim3(blocks(a.n_edges, kLbaThreads)), dim3(kLbaThreads), 0, st,
                       a, poses, pts, outlier);
  return hipGetLastError();
}

}  // namespace orbgpu
