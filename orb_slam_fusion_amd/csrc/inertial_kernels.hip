// gfx950 PoseInertialOptimizationLastFrame / LastKeyFrame: one workgroup per
// problem runs the whole call -- 4 outlier-rejection rounds x 10 g2o
// Gauss-Newton iterations over the current frame's pose / velocity / bias
// vertices (and, LastFrame, the previous frame's, tied by the prior), the
// inlier classification, and the Hessian (marginalised, LastFrame) for the
// next ConstraintPoseImu.  Reference: optimizer.cc:4394-5160, g2o_types.cc,
// imu_types.cc:283-310 (see oracle/inertial_oracle.cc for the restatement).
//
// Roles inside the workgroup (8 waves):
//   wave 0     EdgeInertial (LogSO3, right Jacobians, the bias-corrected
//              preintegration in float): error and Jacobian into LDS; then
//              the dense LDLT of the n x n system (n = 30 / 15) and the
//              current frame's vertex updates;
//   wave 1     EdgePriorPoseImu (LastFrame) and the previous frame's updates;
//   waves 2-7  the visual edges (EdgeMono/StereoOnlyPose): errors, Huber
//              weights, body-frame Jacobians, the 6x6 block + gradient,
//              reduced by a fixed tree.
// Between them every thread assembles the system, each owning whole entries
// (all edge contributions to an entry summed by one thread: no atomics).
// Everything stays in LDS; observations are read once from HBM.
#include <hip/hip_runtime.h>

#include "lds_optin.h"
#include <stdint.h>

#include "../../include/orbgpu.h"

// fp64 solver arithmetic, parity by tolerance (not bit-exact like the
// extractor, whose TUs keep -ffp-contract=off): let products fuse into FMAs.
#pragma clang fp contract(fast)

#ifdef ORB_STAMPS
namespace orbgpu {
extern __device__ unsigned long long g_in_stamps[64 * 32];
}
// IMU-edge sub-phases (thread 0): slot i += time since the previous mark
#define IMU_EDGE_MARK(i)                                                                   \
  do {                                                                                     \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime();                          \
    if (threadIdx.x == 0 && blockIdx.x < 64) {                                             \
      atomicAdd(&orbgpu::g_in_stamps[blockIdx.x * 32 + (i)], now_ - ie_prev_); \
    }                                                                                      \
    ie_prev_ = now_;                                                                       \
  } while (0)
#define IMU_EDGE_MARK_INIT unsigned long long ie_prev_ = __builtin_amdgcn_s_memtime()
#endif
#include "f64_math_dev.h"
#include "imu_math_dev.h"
#include "row_halving_dev.h"

namespace orbgpu {

// Profiling build only (make stamps): per-phase s_memtime totals of thread 0
// (wave 0 runs the serial IMU / solve work), flushed once per workgroup.
#ifdef ORB_STAMPS
__device__ unsigned long long g_in_stamps[64 * 32];
#define ISTAMP_INIT                      \
  unsigned long long ist_acc_[16] = {};  \
  unsigned long long ist_prev_ = __builtin_amdgcn_s_memtime()
#define ISTAMP(i)                                                 \
  do {                                                            \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
    ist_acc_[i] += now_ - ist_prev_;                              \
    ist_prev_ = now_;                                             \
  } while (0)
#define ISTAMP_END                                                                          \
  do {                                                                                      \
    if (threadIdx.x == 0)                                                                   \
      for (int i_ = 0; i_ < 16; ++i_)                                                       \
        if (ist_acc_[i_]) atomicAdd(&g_in_stamps[(blockIdx.x & 63) * 32 + i_], ist_acc_[i_]); \
  } while (0)
#define ISTAMP_ADD_ITER (ist_acc_[8] += 1)
// a sub-phase of thread 0 (wave 0) straight into slot i
#define ISTAMP_T(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define ISTAMP_SUB(i, a, b) \
  do {                      \
    if (threadIdx.x == 0) atomicAdd(&g_in_stamps[(blockIdx.x & 63) * 32 + (i)], (b) - (a)); \
  } while (0)
#else
#define ISTAMP_T(v) (void)0
#define ISTAMP_SUB(i, a, b) (void)0
#define ISTAMP_ADD_ITER (void)0
#define ISTAMP_INIT (void)0
#define ISTAMP(i) (void)0
#define ISTAMP_END (void)0
#endif

constexpr int kInWaves = 8;
constexpr int kInThreads = 64 * kInWaves;
constexpr int kVisWave0 = 2;  // waves 0, 1: IMU edges / solve; 2..: visual edges
// visual sweep's row totals by recursive halving (1) or a row_shr chain (0)
#ifndef ORB_IN_VIS_HALVE
#define ORB_IN_VIS_HALVE 1
#endif
constexpr int kVisThreads = kInThreads - 64 * kVisWave0;
constexpr int kInLdsObs = 2048;  // observations staged in LDS (the rest re-read)
constexpr int kLd = 31;          // padded row stride of the n x n system

// ---- LDS ----------------------------------------------------------------------
struct PriorState {  // == the head of orbgpu_imu_prior
  double Rwb[9], twb[3], vwb[3], bg[3], ba[3];
};
static_assert(offsetof(orbgpu_imu_preint, info) == 68 * sizeof(float), "preint float part");
static_assert(offsetof(orbgpu_imu_prior, H) == sizeof(PriorState), "prior head");

struct InShared {
  StateD cur, prev;
  double ev_Rcw[9], ev_tcw[3];  // current camera pose at the last computeActiveErrors
  CalibD cal;
  double H[31 * kLd];           // the system (full, row-major, padded) + a zero row
  double b[30];
  double x[30];                 // solver x, persists over the call
  double Ji[9 * 24], ei[9];     // EdgeInertial Jacobian / error
  double OJ[9 * 24], Oe[9];     // info * Ji, -info * ei
  double Jp[15 * 15], epr[15];  // EdgePriorPoseImu
  double OJp[15 * 15], Oep[15];
  double wp;                    // prior Huber weight
  double info[81], info_g[9], info_a[9], pH[225];  // edge informations (LDS copies)
  // the preintegration's float part and the prior's state (LDS copies: read
  // from global memory they were hoisted into SGPRs over the whole loop and
  // spilled)
  orbgpu_imu_preint pre;  // dT .. ba valid (the doubles are the fields above)
  PriorState prs;
  double vis[27];               // visual 6x6 (lower, 21) + gradient (6)
  double red[kInWaves * 4 * 27];
  double temp[32];
  double pinv[15 * 16];
  double V[256];                // Jacobi eigenvectors (16 x 16)
  double HM[30 * kLd];          // final Hessian (LastFrame: 30 x 30 in EdgeInertial order)
  int perm[30];
  int ired[kInWaves * 2];
  int ok;
};

// LDS exchange between the lanes of one wave: a wave's LDS instructions
// execute in order, so it suffices that the compiler keeps program order
// (memory clobber) and the writes have left the queue (lgkmcnt(0)).
__device__ __forceinline__ void wave_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

template <int CTRL, int ROW_MASK>
__device__ __forceinline__ double dpp_d(double v) {
  // full row mask: bound_ctrl reads 0 for out-of-range sources, so the
  // destination needs no zeroed old value (one v_mov_b32_dpp per half)
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, ROW_MASK, 0xf, ROW_MASK == 0xf);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, ROW_MASK, 0xf, ROW_MASK == 0xf);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double wave_sum63(double v) {  // lane 63 holds the sum
  v += dpp_d<0x111, 0xf>(v);
  v += dpp_d<0x112, 0xf>(v);
  v += dpp_d<0x114, 0xf>(v);
  v += dpp_d<0x118, 0xf>(v);
  v += dpp_d<0x142, 0xa>(v);
  v += dpp_d<0x143, 0xc>(v);
  return v;
}
__device__ __forceinline__ double bcast(double v, int lane) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), lane),
                          __builtin_amdgcn_readlane(__double2loint(v), lane));
}

// ---- visual edges -------------------------------------------------------------
struct VisObs {  // == orbgpu_inertial_obs
  float Xw[3];
  float u, v, ur;
  float inv_sigma2;
  int32_t close;
};

__device__ __forceinline__ void vis_error(const VisObs& o, const double* Rcw, const double* tcw,
                                          const CalibD& c, double e[3], double Xc[3]) {
  const double X[3] = {o.Xw[0], o.Xw[1], o.Xw[2]};
  m3_mv(Rcw, X, Xc);
  Xc[0] += tcw[0];
  Xc[1] += tcw[1];
  Xc[2] += tcw[2];
  const RecipF64 rz = recip_f64(Xc[2]);  // (f64_math_dev.h: the IEEE quotients)
  const double u = div_by(c.fx * Xc[0], rz) + c.cx;
  const double v = div_by(c.fy * Xc[1], rz) + c.cy;
  e[0] = (double)o.u - u;
  e[1] = (double)o.v - v;
  e[2] = o.ur >= 0.f ? (double)o.ur - (u - c.bf * div_by(1.0, rz)) : 0.0;
}

__device__ __forceinline__ double vis_chi2(const double e[3], double info, bool stereo) {
  double s = e[0] * info * e[0] + e[1] * info * e[1];
  if (stereo) s += e[2] * info * e[2];
  return s;
}

// proj_jac * Rcb * SE3deriv(Xb) (g2o_types.cc:361-446)
__device__ __forceinline__ void vis_jacobian(const double Xc[3], const CalibD& c, bool stereo,
                                             double J[3][6]) {
  double Xb[3];
  m3_mv(c.Rbc, Xc, Xb);
  Xb[0] += c.tbc[0];
  Xb[1] += c.tbc[1];
  Xb[2] += c.tbc[2];
  const RecipF64 rz = recip_f64(Xc[2]), rzz = recip_f64(Xc[2] * Xc[2]);
  const double iz = div_by(1.0, rz);
  double pj[3][3] = {{c.fx * iz, 0, div_by(-c.fx * Xc[0], rzz)},
                     {0, c.fy * iz, div_by(-c.fy * Xc[1], rzz)},
                     {0, 0, 0}};
  if (stereo) {
    pj[2][0] = pj[0][0];
    pj[2][1] = pj[0][1];
    pj[2][2] = pj[0][2] + c.bf * div_by(1.0, rzz);
  }
  const double x = Xb[0], y = Xb[1], z = Xb[2];
  const double S[3][6] = {{0, z, -y, 1, 0, 0}, {-z, 0, x, 0, 1, 0}, {y, -x, 0, 0, 0, 1}};
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    double PR[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) PR[k] = pj[r][0] * c.Rcb[k] + pj[r][1] * c.Rcb[3 + k] + pj[r][2] * c.Rcb[6 + k];
#pragma unroll
    for (int k = 0; k < 6; ++k) J[r][k] = PR[0] * S[0][k] + PR[1] * S[1][k] + PR[2] * S[2][k];
  }
}

// Huber (robust_kernel_impl.cpp): rho'(e2)
__device__ __forceinline__ double huber_w(double e2, double delta) {
  // delta >= 1: the sqrt / division branch sees e2 > 1 only
  return e2 <= delta * delta ? 1.0 : div_by(delta, recip_f64(sqrt_f64(e2)));
}

// One visual edge's weighted 6x6 (lower, 21) + gradient (6) into acc[0..26].
__device__ __forceinline__ void vis_accumulate(const VisObs& o, const double* Rcw, const double* tcw,
                                               const CalibD& c, bool robust, double w_fixed,
                                               double (&acc)[27]) {
  double e[3], Xc[3];
  vis_error(o, Rcw, tcw, c, e, Xc);
  const bool st = o.ur >= 0.f;
  const double info = (double)o.inv_sigma2;
  double w = w_fixed;
  if (robust) w = huber_w(vis_chi2(e, info, st), st ? (double)(float)sqrt(7.815) : (double)(float)sqrt(5.991));
  double J[3][6];
  vis_jacobian(Xc, c, st, J);
  const double wi = w * info;
  int k = 0;
#pragma unroll
  for (int r = 0; r < 6; ++r) {
#pragma unroll
    for (int q = 0; q <= r; ++q) {
      double h = J[0][r] * wi * J[0][q] + J[1][r] * wi * J[1][q];
      if (st) h += J[2][r] * wi * J[2][q];
      acc[k++] += h;
    }
  }
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    double g = J[0][r] * (wi * e[0]) + J[1][r] * (wi * e[1]);
    if (st) g += J[2][r] * (wi * e[2]);
    acc[21 + r] -= g;
  }
}

// ---- the IMU edges (one wave each, every lane the same values; lane 0 stores)
__device__ void inertial_edge(InShared& sh, const orbgpu_imu_preint& pi, double dt, int lane) {
  inertial_edge_core<false>(sh.prev, sh.cur, pi, dt, lane, sh.Ji, sh.ei);
}
// the state-only Jacobian blocks, on another wave meanwhile
__device__ void inertial_edge_states(InShared& sh, double dt, int lane) {
  inertial_edge_lin(sh.prev, sh.cur, dt, lane, sh.Ji);
}

// The parts of EdgeInertial's Jacobian that do not depend on the estimates
// (and the zeros), written once per call.
__device__ void inertial_edge_const(InShared& sh, const orbgpu_imu_preint& pi, int t) {
  double* J = sh.Ji;
  for (int k = t; k < 9 * 24; k += kInThreads) J[k] = 0;
  __syncthreads();
  if (t < 9) {
    const int i = t / 3, j = t % 3;
    J[(6 + i) * 24 + 3 + j] = i == j ? -1.0 : 0.0;
    J[(3 + i) * 24 + 9 + j] = -(double)pi.JVg[3 * i + j];
    J[(6 + i) * 24 + 9 + j] = -(double)pi.JPg[3 * i + j];
    J[(3 + i) * 24 + 12 + j] = -(double)pi.JVa[3 * i + j];
    J[(6 + i) * 24 + 12 + j] = -(double)pi.JPa[3 * i + j];
  }
}

// EdgePriorPoseImu::computeError / linearizeOplus (g2o_types.cc:739-764) on
// the previous frame's vertices, and its Huber weight (delta 5)
__device__ void prior_edge(InShared& sh, const PriorState* pr, bool prior_kernel, int lane) {
  const StateD& s1 = sh.prev;
  {
    double PRt[9], Q[9], epr[15], dt3[3], et[3];
    m3_tr(pr->Rwb, PRt);
    m3_mul(PRt, s1.Rwb, Q);
    log_so3(Q, epr);
#pragma unroll
    for (int i = 0; i < 3; ++i) dt3[i] = s1.twb[i] - pr->twb[i];
    m3_mv(PRt, dt3, et);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      epr[3 + i] = et[i];
      epr[6 + i] = s1.v[i] - pr->vwb[i];
      epr[9 + i] = s1.bg[i] - pr->bg[i];
      epr[12 + i] = s1.ba[i] - pr->ba[i];
    }
    double ijr[9];
    right_j<true>(epr, ijr);
    // chi2 = e^T H e, lane-parallel over rows
    double part = 0;
    if (lane < 15) {
      double t = 0;
#pragma unroll
      for (int q = 0; q < 15; ++q) t += sh.pH[lane * 15 + q] * epr[q];
      double el = 0;
#pragma unroll
      for (int q = 0; q < 15; ++q) el = lane == q ? epr[q] : el;
      part = el * t;
    }
    const double chi2 = bcast(wave_sum63(part), 63);
    if (lane == 0) {
      double* J = sh.Jp;
#pragma unroll
      for (int i = 0; i < 225; ++i) J[i] = 0;
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          J[i * 15 + j] = ijr[3 * i + j];
          J[(3 + i) * 15 + 3 + j] = Q[3 * i + j];
        }
#pragma unroll
      for (int i = 6; i < 15; ++i) J[i * 15 + i] = 1.0;
#pragma unroll
      for (int i = 0; i < 15; ++i) sh.epr[i] = epr[i];
      sh.wp = prior_kernel ? huber_w(chi2, 5.0) : 1.0;
    }
  }
}

// Solver index -> EdgeInertial column (-1: not on the edge) and prior column.
template <int MODE>
__device__ __forceinline__ int ei_col(int s) {
  if (s < 6) return 15 + s;      // VP
  if (s < 9) return 21 + s - 6;  // VV
  if (s < 15) return -1;         // VG, VA
  return MODE == ORBGPU_INERTIAL_LAST_FRAME ? s - 15 : -1;  // VPk VVk VGk VAk
}

// sh.vis[k] from the visual waves' row partials (k < 27)
__device__ __forceinline__ void vis_sum(InShared& sh, int k) {
  double s = 0;
#pragma unroll
  for (int r = kVisWave0 * 4; r < kInWaves * 4; ++r) s += sh.red[r * 27 + k];
  sh.vis[k] = s;
}

// Row blocks (bit b: rows 3b..3b+2) of EdgeInertial's Jacobian column c that
// are not structural zeros (inertial_edge_core / inertial_edge_const).  The
// dot products below skip only exact zeros, keep the order of the others and
// so leave every sum unchanged; a block is issued when any lane of the wave
// needs it (unrolled, its loads batched).
__device__ __forceinline__ int ji_blocks(int c) {
  constexpr unsigned kMask = 07 | 04 << 3 | 06 << 6 | 07 << 9 | 06 << 12 | 01 << 15 | 04 << 18 | 02 << 21;
  return (kMask >> (3 * (c / 3))) & 7;
}
// sum_r A[r * lda] * B[r * ldb] over the rows of blocks m (ascending)
__device__ __forceinline__ double dot_blocks(int m, const double* A, int lda, const double* B, int ldb) {
  double h = 0;
#pragma unroll
  for (int b = 0; b < 3; ++b)
    if (m & (1 << b))
#pragma unroll
      for (int r = 3 * b; r < 3 * b + 3; ++r) h += A[r * lda] * B[r * ldb];
  return h;
}
// the same over EdgePriorPoseImu's Jacobian diag(InvJr, Q, I9) (prior_edge):
// column c < 6 has rows 3(c/3)..+2, column c >= 6 only row c
__device__ __forceinline__ double dot_prior(int c, const double* A, int lda, const double* B, int ldb) {
  double h = 0;
  if (c < 6) {
    const int r0 = c < 3 ? 0 : 3;
#pragma unroll
    for (int r = 0; r < 3; ++r) h += A[(r0 + r) * lda] * B[(r0 + r) * ldb];
  } else {
    h += A[c * lda] * B[c * ldb];
  }
  return h;
}

// The n x n system from the edge pieces: thread-owned entries.  Pass 1 runs
// its three jobs on disjoint threads (Omega J, the prior's Omega J, the visual
// block's final sums); pass 2 writes both triangles, so the solve reads rows.
template <int MODE>
__device__ void assemble(InShared& sh, const orbgpu_imu_preint& pi, const orbgpu_imu_prior* pr,
                         int t) {
  constexpr int n = MODE == ORBGPU_INERTIAL_LAST_FRAME ? 30 : 15;
  // pass 1: Omega * J and -Omega * e
  ISTAMP_T(at0);
  if (t < 9 * 24 + 9) {
    if (t < 9 * 24) {
      const int r = t / 24, c = t % 24;
      sh.OJ[t] = dot_blocks(ji_blocks(c), sh.info + r * 9, 1, sh.Ji + c, 24);
    } else {
      const int r = t - 9 * 24;
      double s = 0;
#pragma unroll
      for (int q = 0; q < 9; ++q) s += sh.info[r * 9 + q] * sh.ei[q];
      sh.Oe[r] = -s;
    }
  } else if (t < 9 * 24 + 9 + 27) {
    vis_sum(sh, t - (9 * 24 + 9));
  } else if (MODE == ORBGPU_INERTIAL_LAST_FRAME && t >= 256 && t < 256 + 225 + 15) {
    const int k = t - 256;
    const double w = sh.wp;
    if (k < 225) {
      const int r = k / 15, c = k % 15;
      double s = 0;  // sum_q (w pH_rq) Jp_qc over Jp's non-zero rows
      if (c < 6) {
        const int q0 = c < 3 ? 0 : 3;
#pragma unroll
        for (int q = 0; q < 3; ++q) s += (w * sh.pH[r * 15 + q0 + q]) * sh.Jp[(q0 + q) * 15 + c];
      } else {
        s += (w * sh.pH[r * 15 + c]) * sh.Jp[c * 15 + c];
      }
      sh.OJp[k] = s;
    } else {
      const int r = k - 225;
      double s = 0;
#pragma unroll
      for (int q = 0; q < 15; ++q) s += sh.pH[r * 15 + q] * sh.epr[q];
      sh.Oep[r] = -s * w;
    }
  }
  __syncthreads();
  ISTAMP_T(at1);
  ISTAMP_SUB(14, at0, at1);
  // pass 2: entry (i, j) = visual + EdgeInertial + random walks + prior,
  // the lower triangle mirrored into the upper, and b
  constexpr int nl = n * (n + 1) / 2;
  for (int k = t; k < nl + n; k += kInThreads) {
    const bool isb = k >= nl;
    int i = isb ? k - nl : (int)((sqrtf(8.f * k + 1.f) - 1.f) * 0.5f);
    if (!isb) {  // exact integer triangular root
      while (i * (i + 1) / 2 > k) --i;
      while ((i + 1) * (i + 2) / 2 <= k) ++i;
    }
    const int j = isb ? 0 : k - i * (i + 1) / 2;
    double s = 0;
    if (!isb) {
      if (i < 6 && j < 6) s += sh.vis[i >= j ? i * (i + 1) / 2 + j : j * (j + 1) / 2 + i];
      const int ci = ei_col<MODE>(i), cj = ei_col<MODE>(j);
      if (ci >= 0 && cj >= 0) s += dot_blocks(ji_blocks(ci), sh.Ji + ci, 24, sh.OJ + cj, 24);
      // random walks: VG (9..11) <-> VGk (24..26), VA (12..14) <-> VAk (27..29)
      const int ri = (i >= 9 && i < 15) ? i - 9 : (i >= 24 ? i - 24 : -1);
      const int rj = (j >= 9 && j < 15) ? j - 9 : (j >= 24 ? j - 24 : -1);
      if (ri >= 0 && rj >= 0 && ri / 3 == rj / 3) {
        const double* Om = ri < 3 ? sh.info_g : sh.info_a;
        const double sg = ((i < 15) == (j < 15)) ? 1.0 : -1.0;
        s += sg * Om[(ri % 3) * 3 + rj % 3];
      }
      if (MODE == ORBGPU_INERTIAL_LAST_FRAME && i >= 15 && j >= 15)
        s += dot_prior(i - 15, sh.Jp + i - 15, 15, sh.OJp + j - 15, 15);
      sh.H[i * kLd + j] = s;
      sh.H[j * kLd + i] = s;
    } else {
      if (i < 6) s += sh.vis[21 + i];
      const int ci = ei_col<MODE>(i);
      if (ci >= 0) s += dot_blocks(ji_blocks(ci), sh.Ji + ci, 24, sh.Oe, 1);
      const int ri = (i >= 9 && i < 15) ? i - 9 : (i >= 24 ? i - 24 : -1);
      if (ri >= 0) {  // b = -J^T Omega e with J = -I (previous) / +I (current), e = x2 - x1
        const double* Om = ri < 3 ? sh.info_g : sh.info_a;
        const double* x2 = ri < 3 ? sh.cur.bg : sh.cur.ba;
        const double* x1 = ri < 3 ? sh.prev.bg : sh.prev.ba;
        const int rr = ri % 3;
        double oe = 0;
#pragma unroll
        for (int q = 0; q < 3; ++q) oe += Om[rr * 3 + q] * (x2[q] - x1[q]);
        s += i < 15 ? -oe : oe;
      }
      if (MODE == ORBGPU_INERTIAL_LAST_FRAME && i >= 15) s += dot_prior(i - 15, sh.Jp + i - 15, 15, sh.Oep, 1);
      sh.b[i] = s;
    }
  }
}

// Eigen LDLT of sh.H (lower triangle, diagonal pivoting) and the solve into
// sh.x when it is positive: wave 0, lane i owns row i in registers.  Eigen
// pivots on the not-yet-updated diagonal (ldlt_inplace::unblocked: the
// diagonal past k is untouched until its own step), i.e. on the original
// diagonal: the pivot order is fixed up front (largest |H_ii| first, ties in
// index order -- Eigen breaks ties by the current position, which only
// changes rounding) and the permuted matrix is factorised right-looking:
// step k broadcasts D_k and the column L_jk (v_readlane) and every lane
// updates its row.  Returns isPositive().
template <int n>
__device__ bool ldlt_wave(InShared& sh, int lane) {
  const double dl = lane < n ? fabs(sh.H[lane * kLd + lane]) : -1.0;
  if (lane < n) sh.temp[lane] = dl;
  wave_sync();
  int rank = 0;
#pragma unroll
  for (int j = 0; j < n; ++j) {
    const double dj = sh.temp[j];
    rank += (dj > dl || (dj == dl && j < lane)) ? 1 : 0;
  }
  if (lane < n) sh.perm[rank] = lane;
  wave_sync();
  const int pi = lane < n ? sh.perm[lane] : 0;
  double a[n];
#pragma unroll
  for (int j = 0; j < n; ++j) {
    const int pj = __builtin_amdgcn_readlane(pi, j);
    a[j] = sh.H[max(pi, pj) * kLd + min(pi, pj)];
  }
  bool neg = false;
  double dd = 1.0;
#pragma unroll
  for (int k = 0; k < n; ++k) {
    const double dk = bcast(a[k], k);
    if (dk < 0) neg = true;
    if (lane == k) dd = dk;
    // 1/D_k: v_rcp_f64 + one Newton step (a rounding away from c / D_k); a
    // zero pivot leaves the column undivided and adds nothing to the rest,
    // as Eigen's left-looking update (temp = D_j A_kj) does
    double r = __builtin_amdgcn_rcp(dk);
    r = fma(r, fma(-dk, r, 1.0), r);
    const bool nz = fabs(dk) > 0;
    const double c = a[k];
    const double lu = nz ? c * r : 0.0;
#pragma unroll
    for (int j = k + 1; j < n; ++j) a[j] = fma(-c, bcast(lu, j), a[j]);
    if (lane > k && nz) a[k] = lu;
  }
  if (neg) return false;
  // solve P^T L D L^T P x = b
  double y = lane < n ? sh.b[pi] : 0.0;
#pragma unroll
  for (int j = 0; j < n; ++j) {
    const double yj = bcast(y, j);
    y = lane > j ? fma(-a[j], yj, y) : y;
  }
  double z = fabs(dd) > 1.0 / 1.79769313486231570815e+308 ? y / dd : 0.0;
  // L rows to LDS for the transposed solve (column i of L across lanes)
#pragma unroll
  for (int j = 0; j < n; ++j)
    if (lane < n && j < lane) sh.H[lane * kLd + j] = a[j];
  wave_sync();
#pragma unroll
  for (int j = n - 1; j > 0; --j) {
    const double zj = bcast(z, j);
    const double lji = lane < j ? sh.H[j * kLd + lane] : 0.0;
    z = fma(-lji, zj, z);
  }
  if (lane < n) sh.x[pi] = z;
  return true;
}

// relative size of a pivot treated as (near) zero by the natural-order solves
constexpr double kGjNearZero = 1e-12;

#include "inertial_gj.inc"

// The same system by Gauss-Jordan elimination (tools/gen_inertial_gj.py):
// wave 0, lane li of each 16-lane row owns rows li and li + 16 with b
// appended, pivot k's row read by DPP64 row broadcast (one v_fmac_f64_dpp
// per entry, no v_readlane chains, no substitution passes), every row but the
// pivot's eliminated (the rows above cost nothing extra in this layout), x_i
// = b'_i / D_i with Eigen's tolerance.  Pivots in natural order: the system
// is symmetric positive definite whenever the step succeeds, where
// elimination needs no pivoting and Eigen's diagonal pivot order changes
// only the rounding, and the signs of the pivots (isPositive) do not depend
// on the order -- in exact arithmetic.  A pivot within kGjNearZero of the
// largest diagonal entry (a zero or nearly singular system, where rounding
// in another order could flip a pivot's sign) takes ldlt_wave, Eigen's own
// pivot order and semantics, before any sign is judged; otherwise a negative
// pivot: not positive.  Rows load with compile-time column offsets (the
// permuted gather cost a tenth of the kernel).
template <int n>
__device__ bool gj_wave(InShared& sh, int lane) {
  ISTAMP_T(gt0);
  const int li = lane & 15, ia = li, ib = li + 16;
  // rows past n read the zero row 30
  const double* hA = sh.H + (ia < n ? ia : 30) * kLd;
  const double* hB = sh.H + (ib < n ? ib : 30) * kLd;
  double rA[n + 1], rB[n + 1];
#pragma unroll
  for (int j = 0; j < n; ++j) {
    rA[j] = hA[j];
    rB[j] = hB[j];
  }
  rA[n] = ia < n ? sh.b[ia] : 0.0;
  rB[n] = ib < n ? sh.b[ib] : 0.0;
  double dA = 1.0, dB = 1.0;
  double dmax = 0;  // the largest |diagonal entry| (uniform LDS reads)
#pragma unroll
  for (int j = 0; j < n; ++j) dmax = fmax(dmax, fabs(sh.H[j * kLd + j]));
  ISTAMP_T(gt1);
  const int f = gj_pivots<n>(rA, rB, li, dA, dB, kGjNearZero * dmax);
  ISTAMP_T(gt2);
  ISTAMP_SUB(12, gt0, gt1);
  ISTAMP_SUB(13, gt1, gt2);
  if (f & 2) return ldlt_wave<n>(sh, lane);
  if (f & 1) return false;
  constexpr double kTiny = 1.0 / 1.79769313486231570815e+308;
  if (lane < 16) {
    if (ia < n) sh.x[ia] = fabs(dA) > kTiny ? rA[n] / dA : 0.0;
    if (ib < n) sh.x[ib] = fabs(dB) > kTiny ? rB[n] / dB : 0.0;
  }
  return true;
}

__device__ __forceinline__ void load_state(StateD& s, const orbgpu_imu_state& g) {
  for (int i = 0; i < 9; ++i) {
    s.Rwb[i] = g.Rwb[i];
    s.Rcw[i] = g.Rcw[i];
  }
  for (int i = 0; i < 3; ++i) {
    s.twb[i] = g.twb[i];
    s.tcw[i] = g.tcw[i];
    s.v[i] = g.v[i];
    s.bg[i] = g.bg[i];
    s.ba[i] = g.ba[i];
  }
}

// Visual sweep over the active edges (waves 1..), reduced into sh.vis; wave 0
// meanwhile runs `imu` (its own work).  kind 0: Gauss-Newton system (Huber
// weights where robust); kind 1: unweighted J^T Omega J of the inlier edges
// (GetHessian) at the current pose.
// Waves 2..7 take the visual edges; wave kLinWave first forms the IMU
// edge's state-only Jacobian blocks (`w3`), off wave 0's critical path.
// (Handing the edges past kVisThreads to wave 1 after the prior edge instead
// of a second pass of wave 2 measured slower: wave 1 became the last.)
constexpr int kLinWave = 3;
template <typename W0, typename W1, typename W3>
__device__ void vis_sweep(InShared& sh, const VisObs* ob, const uint8_t* lv, const VisObs* gobs,
                          const uint8_t* glv, int cap, int n, bool robust, int kind, int t,
                          bool sum_here, W0&& w0, W1&& w1, W3&& w3) {
  const int wave = t >> 6, lane = t & 63;
#ifdef ORB_STAMPS
  const unsigned long long vt0 = __builtin_amdgcn_s_memtime();
  unsigned long long vt1 = vt0;
#endif
  if (wave == 0) {
    w0();
  } else {
    if (wave == 1) w1();
    if (wave == kLinWave) w3();
    if (wave >= kVisWave0) {
      // the accumulators live in this branch only, so they add nothing to the
      // register pressure of the IMU-edge wave's code
      double acc[27];
#pragma unroll
      for (int k = 0; k < 27; ++k) acc[k] = 0;
      const int tv = t - 64 * kVisWave0;
      for (int i = tv; i < n; i += kVisThreads) {
        const bool in_lds = i < cap;
        const uint8_t l = in_lds ? lv[i] : glv[i];
        if (l) continue;
        const VisObs o = in_lds ? ob[i] : gobs[i];
        vis_accumulate(o, sh.cur.Rcw, sh.cur.tcw, sh.cal, kind == 0 && robust, 1.0, acc);
      }
#ifdef ORB_STAMPS
      vt1 = __builtin_amdgcn_s_memtime();
#endif
#if ORB_IN_VIS_HALVE
      // row totals by recursive halving (row_halving_dev.h)
      row_totals_halving<27>(acc, lane, sh.red + (wave * 4 + (lane >> 4)) * 27);
#else
      // DPP row sums; lane 15 of each row writes its partial
#pragma unroll
      for (int k = 0; k < 27; ++k) {
        double x = acc[k];
        x += dpp_d<0x111, 0xf>(x);
        x += dpp_d<0x112, 0xf>(x);
        x += dpp_d<0x114, 0xf>(x);
        x += dpp_d<0x118, 0xf>(x);
        acc[k] = x;
      }
      if ((lane & 15) == 15)
#pragma unroll
        for (int k = 0; k < 27; ++k) sh.red[(wave * 4 + (lane >> 4)) * 27 + k] = acc[k];
#endif
    }
  }
#ifdef ORB_STAMPS
  if (t == 64 * kVisWave0) {
    const unsigned long long vt2 = __builtin_amdgcn_s_memtime();
    atomicAdd(&g_in_stamps[(blockIdx.x & 63) * 32 + 10], vt1 - vt0);
    atomicAdd(&g_in_stamps[(blockIdx.x & 63) * 32 + 11], vt2 - vt1);
  }
  if (lane == 0)  // each wave's time in the sweep (slots 16 + wave)
    atomicAdd(&g_in_stamps[(blockIdx.x & 63) * 32 + 16 + wave], __builtin_amdgcn_s_memtime() - vt0);
#endif
  __syncthreads();
  if (sum_here && t < 27) vis_sum(sh, t);
}

// In-place LDL^T of the 15 x 15 symmetric A (lower triangle, stride kLd) on
// one wave, natural pivot order: D on the diagonal, L below it.  Lane-owned
// entries (k = lane + 64 u); one wave_sync per half step.  Returns whether
// every pivot was > 0 (A positive definite).
__device__ __forceinline__ bool ldlt15(double* A, int lane) {
  bool pd = true;
#pragma unroll 1
  for (int j = 0; j < 15; ++j) {
    const double d = A[j * kLd + j];
    pd = pd && d > 0.0;
    const double inv = d != 0.0 ? 1.0 / d : 0.0;
    double nv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int k = lane + 64 * u, i = k / 15, c = k - 15 * (k / 15);
      nv[u] = k < 225 && i > j && c > j && c <= i ? A[i * kLd + c] - A[i * kLd + j] * A[c * kLd + j] * inv : 0.0;
    }
    wave_sync();
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int k = lane + 64 * u, i = k / 15, c = k - 15 * (k / 15);
      if (k < 225 && i > j && c > j && c <= i) A[i * kLd + c] = nv[u];
    }
    if (lane > j && lane < 15) A[lane * kLd + j] *= inv;
    wave_sync();
  }
  return pd;
}

// X = A^-1 (15 x 15, row stride 16) from the LDL^T factors in A: column c of
// L^-1 by forward substitution (lane c, in registers), D^-1, then L^-T; the
// L entries are uniform LDS reads that do not wait on the chain (a rolled
// loop through X in LDS paid a store-to-load round trip per FMA).
__device__ __forceinline__ void ldlt15_inverse(const double* A, double* X, int lane) {
  if (lane < 15) {
    const int c = lane;
    double v[15];
#pragma unroll
    for (int i = 0; i < 15; ++i) {
      double s = i == c ? 1.0 : 0.0;
#pragma unroll
      for (int k = 0; k < i; ++k) s -= A[i * kLd + k] * v[k];
      v[i] = s;
    }
#pragma unroll
    for (int i = 14; i >= 0; --i) {
      double s = v[i] / A[i * kLd + i];
#pragma unroll
      for (int k = i + 1; k < 15; ++k) s -= A[k * kLd + i] * v[k];
      v[i] = s;
    }
#pragma unroll
    for (int i = 0; i < 15; ++i) X[i * 16 + c] = v[i];
  }
  wave_sync();
}

template <int MODE>
__global__ __launch_bounds__(kInThreads) void k_pose_inertial(
    CalibD cal, const orbgpu_imu_state* __restrict__ g_cur, const orbgpu_imu_state* __restrict__ g_prev,
    const orbgpu_imu_preint* __restrict__ g_preint, const orbgpu_imu_prior* __restrict__ g_prior,
    const VisObs* __restrict__ g_obs, const int* __restrict__ g_nobs, int obs_stride, int rec_init,
    orbgpu_inertial_result* __restrict__ g_res, uint8_t* __restrict__ g_out, int lds_obs,
    int* __restrict__ done_host, const int* __restrict__ seq_src) {
  constexpr int n = MODE == ORBGPU_INERTIAL_LAST_FRAME ? 30 : 15;
  __shared__ InShared sh;
  extern __shared__ __attribute__((aligned(16))) uint8_t in_lds[];
  const int p = blockIdx.x;
  int t = threadIdx.x, lane = t & 63, wave = t >> 6;  // laundered per iteration (below)
  const int nobs = max(0, min(g_nobs[p], obs_stride));
  const VisObs* gobs = g_obs + (size_t)p * obs_stride;
  uint8_t* glv = g_out + (size_t)p * obs_stride;
  const orbgpu_imu_preint& pi = g_preint[p];
  const orbgpu_imu_prior* pr = MODE == ORBGPU_INERTIAL_LAST_FRAME ? g_prior + p : nullptr;
  const double dt = (double)pi.dT;
  const int cap = min(nobs, lds_obs);
  VisObs* ob = reinterpret_cast<VisObs*>(in_lds);
  uint8_t* lv = in_lds + (size_t)lds_obs * sizeof(VisObs);
  for (int i = t; i < cap; i += kInThreads) {
    ob[i] = gobs[i];
    lv[i] = 0;
  }
  for (int i = cap + t; i < nobs; i += kInThreads) glv[i] = 0;
  if (t == 0) {
    sh.cal = cal;
    load_state(sh.cur, g_cur[p]);
    load_state(sh.prev, g_prev[p]);
  }
  if (t < 30) sh.x[t] = 0;
  if (t < kLd) sh.H[30 * kLd + t] = 0;  // gj_wave's zero row
  if (t < 68) reinterpret_cast<float*>(&sh.pre)[t] = reinterpret_cast<const float*>(&pi)[t];
  if (MODE == ORBGPU_INERTIAL_LAST_FRAME && t >= 128 && t < 128 + 21)
    reinterpret_cast<double*>(&sh.prs)[t - 128] = reinterpret_cast<const double*>(pr)[t - 128];
  for (int k = t; k < 81 + 18 + 225; k += kInThreads) {
    if (k < 81)
      sh.info[k] = pi.info[k];
    else if (k < 90)
      sh.info_g[k - 81] = pi.info_g[k - 81];
    else if (k < 99)
      sh.info_a[k - 90] = pi.info_a[k - 90];
    else if (MODE == ORBGPU_INERTIAL_LAST_FRAME)
      sh.pH[k - 99] = pr->H[k - 99];
  }
  __syncthreads();
  inertial_edge_const(sh, pi, t);
  __syncthreads();
  ISTAMP_INIT;

  const float chi2MonoLF[4] = {5.991f, 5.991f, 5.991f, 5.991f};
  const float chi2MonoKF[4] = {12.f, 7.5f, 5.991f, 5.991f};
  const float chi2Stereo[4] = {15.6f, 9.8f, 7.815f, 7.815f};
  const int n_edges = nobs + (MODE == ORBGPU_INERTIAL_LAST_FRAME ? 4 : 3);
  bool robust = true;
  int nBad = 0, nInl = 0;
  // (not unrolled: four copies of the round only multiplied the live uniform
  // values, spilled to VGPR lanes)
#pragma unroll 1
  for (int it = 0; it < 4; ++it) {
#pragma unroll 1
    for (int iter = 0; iter < 10; ++iter) {
      // the thread index is opaque to the optimiser from here: otherwise every
      // thread-predicate compare of the loop body is hoisted out of it and its
      // lane mask lives in (spilled) SGPRs for the whole loop
      asm volatile("" : "+v"(t), "+v"(lane), "+v"(wave));
      // computeActiveErrors + buildSystem
      // (the visual block's final sums happen in assemble's first pass)
      vis_sweep(
          sh, ob, lv, gobs, glv, cap, nobs, robust, 0, t, false,
          [&] {
            inertial_edge(sh, sh.pre, dt, lane);
            ISTAMP(6);
          },
          [&] {
            if (MODE == ORBGPU_INERTIAL_LAST_FRAME) prior_edge(sh, &sh.prs, true, lane);
          },
          [&] { inertial_edge_states(sh, dt, lane); });
      ISTAMP(0);
      assemble<MODE>(sh, pi, pr, t);
      __syncthreads();
      ISTAMP(1);
      if (wave == 0) {
        const bool ok = gj_wave<n>(sh, lane);
        if (lane == 0) {
#pragma unroll
          for (int i = 0; i < 9; ++i) sh.ev_Rcw[i] = sh.cur.Rcw[i];
#pragma unroll
          for (int i = 0; i < 3; ++i) sh.ev_tcw[i] = sh.cur.tcw[i];
          sh.ok = ok;
        }
      }
      __syncthreads();
      ISTAMP(2);
      // g2o applies x even when the solve failed (x then keeps its last
      // value); the current frame's vertices on wave 0, the previous on wave 1
      if (wave == 0 || (MODE == ORBGPU_INERTIAL_LAST_FRAME && wave == 1)) {
        StateD& st = wave == 0 ? sh.cur : sh.prev;
        const int o = wave == 0 ? 0 : 15;
        double xv[15];
#pragma unroll
        for (int i = 0; i < 15; ++i) xv[i] = sh.x[o + i];
        pose_update(st, xv, sh.cal, lane == 0);
        if (lane < 3) {
          st.v[lane] += xv[6 + lane];
          st.bg[lane] += xv[9 + lane];
          st.ba[lane] += xv[12 + lane];
        }
      }
      __syncthreads();
      ISTAMP(3);
      ISTAMP_ADD_ITER;
      if (!sh.ok) break;
    }
    // classification (optimizer.cc:5002-5057 / 4620-4673)
    const float cm = MODE == ORBGPU_INERTIAL_LAST_FRAME ? chi2MonoLF[it] : chi2MonoKF[it];
    const float cclose = 1.5 * cm;
    int bad = 0, good = 0;
    for (int i = t; i < nobs; i += kInThreads) {
      const bool in_lds = i < cap;
      const VisObs o = in_lds ? ob[i] : gobs[i];
      const uint8_t l = in_lds ? lv[i] : glv[i];
      double e[3], Xc[3], Xn[3];
      vis_error(o, l ? sh.cur.Rcw : sh.ev_Rcw, l ? sh.cur.tcw : sh.ev_tcw, sh.cal, e, Xc);
      const bool st = o.ur >= 0.f;
      const float chi2 = (float)vis_chi2(e, (double)o.inv_sigma2, st);
      bool out;
      if (!st) {
        const double X[3] = {o.Xw[0], o.Xw[1], o.Xw[2]};
        m3_mv(sh.cur.Rcw, X, Xn);
        const bool pos = Xn[2] + sh.cur.tcw[2] > 0.0;
        out = (chi2 > cm && !o.close) || (o.close && chi2 > cclose) || !pos;
      } else {
        out = chi2 > chi2Stereo[it];
      }
      if (in_lds)
        lv[i] = out;
      else
        glv[i] = out;
      bad += out;
      good += !out;
    }
    for (int o = 32; o > 0; o >>= 1) {
      bad += __shfl_xor(bad, o, 64);
      good += __shfl_xor(good, o, 64);
    }
    if (lane == 0) {
      sh.ired[wave * 2] = bad;
      sh.ired[wave * 2 + 1] = good;
    }
    __syncthreads();
    nBad = nInl = 0;
#pragma unroll
    for (int w = 0; w < kInWaves; ++w) {
      nBad += sh.ired[w * 2];
      nInl += sh.ired[w * 2 + 1];
    }
    __syncthreads();
    if (it == 2) robust = false;
    ISTAMP(4);
    if (n_edges < 10) break;
  }
  if (nInl < 30 && !rec_init) {  // recover not too bad points
    int bad = 0;
    for (int i = t; i < nobs; i += kInThreads) {
      const bool in_lds = i < cap;
      const VisObs o = in_lds ? ob[i] : gobs[i];
      double e[3], Xc[3];
      vis_error(o, sh.cur.Rcw, sh.cur.tcw, sh.cal, e, Xc);
      const bool st = o.ur >= 0.f;
      const float chi2 = (float)vis_chi2(e, (double)o.inv_sigma2, st);
      if (chi2 < (st ? 24.f : 18.f)) {
        if (in_lds)
          lv[i] = 0;
        else
          glv[i] = 0;
      } else {
        ++bad;
      }
    }
    for (int o = 32; o > 0; o >>= 1) bad += __shfl_xor(bad, o, 64);
    if (lane == 0) sh.ired[wave * 2] = bad;
    __syncthreads();
    nBad = 0;
#pragma unroll
    for (int w = 0; w < kInWaves; ++w) nBad += sh.ired[w * 2];
    __syncthreads();
  }

  // ---- the Hessian for the new ConstraintPoseImu ------------------------------
  // visual inliers' J^T Omega J (waves 2..) while waves 0, 1 linearise the IMU edges
  vis_sweep(
      sh, ob, lv, gobs, glv, cap, nobs, false, 1, t, true, [&] { inertial_edge(sh, sh.pre, dt, lane); },
      [&] {
        if (MODE == ORBGPU_INERTIAL_LAST_FRAME) prior_edge(sh, &sh.prs, false, lane);
      },
      [&] { inertial_edge_states(sh, dt, lane); });
  __syncthreads();
  orbgpu_inertial_result* res = g_res + p;
  if (MODE == ORBGPU_INERTIAL_LAST_FRAME) {
    // H (30 x 30, EdgeInertial order: previous 0..14, current 15..29)
    for (int k = t; k < 9 * 24; k += kInThreads) {
      const int r = k / 24, c = k % 24;
      double s = 0;
#pragma unroll
      for (int q = 0; q < 9; ++q) s += sh.info[r * 9 + q] * sh.Ji[q * 24 + c];
      sh.OJ[k] = s;
    }
    for (int k = t; k < 225; k += kInThreads) {
      const int r = k / 15, c = k % 15;
      double s = 0;
#pragma unroll
      for (int q = 0; q < 15; ++q) s += sh.pH[r * 15 + q] * sh.Jp[q * 15 + c];
      sh.OJp[k] = s;
    }
    __syncthreads();
    for (int k = t; k < 900; k += kInThreads) {
      const int i = k / 30, j = k % 30;
      double s = 0;
      if (i < 24 && j < 24) {
#pragma unroll
        for (int r = 0; r < 9; ++r) s += sh.Ji[r * 24 + i] * sh.OJ[r * 24 + j];
      }
      // gyro RW on 9..11 / 24..26, acc RW on 12..14 / 27..29
      const int gi = (i >= 9 && i < 12) ? i - 9 : (i >= 24 && i < 27 ? i - 24 : -1);
      const int gj = (j >= 9 && j < 12) ? j - 9 : (j >= 24 && j < 27 ? j - 24 : -1);
      if (gi >= 0 && gj >= 0) s += ((i < 15) == (j < 15) ? 1.0 : -1.0) * sh.info_g[gi * 3 + gj];
      const int ai = (i >= 12 && i < 15) ? i - 12 : (i >= 27 ? i - 27 : -1);
      const int aj = (j >= 12 && j < 15) ? j - 12 : (j >= 27 ? j - 27 : -1);
      if (ai >= 0 && aj >= 0) s += ((i < 15) == (j < 15) ? 1.0 : -1.0) * sh.info_a[ai * 3 + aj];
      if (i < 15 && j < 15) {
#pragma unroll
        for (int r = 0; r < 15; ++r) s += sh.Jp[r * 15 + i] * sh.OJp[r * 15 + j];
      }
      if (i >= 15 && i < 21 && j >= 15 && j < 21) {
        const int a = i - 15, c = j - 15;
        s += sh.vis[a >= c ? a * (a + 1) / 2 + c : c * (c + 1) / 2 + a];
      }
      sh.HM[i * kLd + j] = s;
    }
    __syncthreads();
    // Marginalize(H, 0, 14): pinv of the previous-frame block, then the Schur
    // complement.  The pseudo-inverse drops eigenvalues at or below 1e-6; when
    // H_pp - tau I is positive definite (an LDL^T with every pivot > 0, tau =
    // max(2e-6, 1e-12 max|diag|): larger than the cut plus the factorisation's
    // rounding) none is dropped and pinv = H_pp^-1, taken from the LDL^T of
    // H_pp (fast path, a few thousand cycles).  Otherwise the parallel cyclic
    // Jacobi below (wave 0, on a 16 x 16 padding) with the cut.
    // The shifted test (wave 0, rows 0..14 of sh.H) and the factorisation of
    // H_pp itself with its inverse (wave 1, rows 15..29) run side by side; a
    // failed test discards wave 1's pinv for the Jacobi path's.
    if (wave == 1) {
      double* A1 = sh.H + 15 * kLd;
      for (int k = lane; k < 225; k += 64) {
        const int i = k / 15, j = k - 15 * (k / 15);
        A1[i * kLd + j] = sh.HM[i * kLd + j];
      }
      wave_sync();
      (void)ldlt15(A1, lane);
      ldlt15_inverse(A1, sh.pinv, lane);
    }
    if (wave == 0) {
      double* A = sh.H;   // 16 x 16 working copy (stride kLd)
      double dmax = 0;
      for (int i = 0; i < 15; ++i) dmax = fmax(dmax, fabs(sh.HM[i * kLd + i]));
      const double tau = fmax(2e-6, 1e-12 * dmax);
      for (int k = lane; k < 225; k += 64) {
        const int i = k / 15, j = k - 15 * (k / 15);
        A[i * kLd + j] = sh.HM[i * kLd + j] - (i == j ? tau : 0.0);
      }
      wave_sync();
      const bool pd = ldlt15(A, lane);  // the whole wave; pd is uniform
      if (lane == 0) sh.ok = pd;
    }
    __syncthreads();
    if (wave == 0 && !sh.ok) {
      double* A = sh.H;   // 16 x 16 working copy (stride kLd)
      double* V = sh.V;   // 16 x 16 eigenvectors (stride 16)
      {
      for (int k = lane; k < 256; k += 64) {
        const int i = k >> 4, j = k & 15;
        A[i * kLd + j] = (i < 15 && j < 15) ? sh.HM[i * kLd + j] : 0.0;
        V[k] = i == j ? 1.0 : 0.0;
      }
      wave_sync();
      // cyclic Jacobi converges quadratically: stop at an off-diagonal norm
      // of 1e-13 of the diagonal (the pseudo-inverse is then exact to
      // rounding), at most 12 sweeps
      for (int sweep = 0; sweep < 12; ++sweep) {
        double off = 0, dg = 0;
        for (int k = lane; k < 256; k += 64) {
          const int i = k >> 4, j = k & 15;
          const double a = A[i * kLd + j];
          if (i == j) dg += a * a;
          if (i < j) off += a * a;
        }
        off = bcast(wave_sum63(off), 63);
        dg = bcast(wave_sum63(dg), 63);
        if (off <= 1e-26 * dg) break;
        for (int r = 0; r < 15; ++r) {
          // round-robin pairing of 16 indices: (15, r) and ((r+k)%15, (r-k+15)%15)
          double* cs = sh.temp;  // c[8], s[8]
          if (lane < 8) {
            int pp = lane == 0 ? r : (r + lane) % 15;
            int qq = lane == 0 ? 15 : (r - lane + 15) % 15;
            const double apq = A[pp * kLd + qq];
            double c = 1.0, s = 0.0;
            if (apq != 0.0) {
              const double th = (A[qq * kLd + qq] - A[pp * kLd + pp]) / (2 * apq);
              const double tt = (th >= 0 ? 1.0 : -1.0) / (fabs(th) + sqrt(th * th + 1));
              c = 1 / sqrt(tt * tt + 1);
              s = tt * c;
            }
            cs[lane] = c;
            cs[8 + lane] = s;
          }
          wave_sync();
          // partner / role of every index this round
          auto pair_of = [&](int i, int& pidx, int& role, int& mate) {
            if (i == 15 || i == r) {
              pidx = 0;
              role = i == r ? 0 : 1;
              mate = i == r ? 15 : r;
            } else {
              const int k1 = (i - r + 15) % 15;  // i = (r + k1) % 15 -> role p of pair k1
              if (k1 <= 7) {
                pidx = k1;
                role = 0;
                mate = (r - k1 + 15) % 15;
              } else {
                pidx = 15 - k1;
                role = 1;
                mate = (r + 15 - k1) % 15;
              }
            }
          };
          // A' = G^T A G with G[p][p] = c, G[q][p] = -s, G[p][q] = s, G[q][q] = c
          double nv[4], vv[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int k = lane + 64 * u, i = k >> 4, j = k & 15;
            int pi_, ri, mi, pj_, rj, mj;
            pair_of(i, pi_, ri, mi);
            pair_of(j, pj_, rj, mj);
            const double ci = cs[pi_], si = cs[8 + pi_], cj = cs[pj_], sj = cs[8 + pj_];
            // column i of G: G[i][i] = c, G[mate][i] = role p ? -s : s
            const double gii = ci, gmi = ri == 0 ? -si : si;
            const double gjj = cj, gmj = rj == 0 ? -sj : sj;
            const double a_ij = A[i * kLd + j], a_im = A[i * kLd + mj];
            const double a_mj = A[mi * kLd + j], a_mm = A[mi * kLd + mj];
            nv[u] = gii * (a_ij * gjj + a_im * gmj) + gmi * (a_mj * gjj + a_mm * gmj);
            vv[u] = V[i * 16 + j] * gjj + V[i * 16 + mj] * gmj;
          }
          wave_sync();
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int k = lane + 64 * u, i = k >> 4, j = k & 15;
            A[i * kLd + j] = nv[u];
            V[i * 16 + j] = vv[u];
          }
          wave_sync();
        }
      }
      // pinv = sum over |lambda| > 1e-6 of v v^T / lambda
      for (int k = lane; k < 225; k += 64) {
        const int i = k / 15, j = k % 15;
        double s = 0;
        for (int m = 0; m < 15; ++m) {
          const double l = A[m * kLd + m];
          if (fabs(l) > 1e-6) s += V[i * 16 + m] * V[j * 16 + m] / l;
        }
        sh.pinv[i * 16 + j] = s;
      }
      }  // Jacobi
    }
    __syncthreads();
    // T = Hcb pinv (into sh.H rows), then H15 = Hcc - T Hbc
    for (int k = t; k < 225; k += kInThreads) {
      const int i = k / 15, j = k % 15;
      double s = 0;
#pragma unroll
      for (int m = 0; m < 15; ++m) s += sh.HM[(15 + i) * kLd + m] * sh.pinv[m * 16 + j];
      sh.Jp[k] = s;
    }
    __syncthreads();
    for (int k = t; k < 225; k += kInThreads) {
      const int i = k / 15, j = k % 15;
      double s = 0;
#pragma unroll
      for (int m = 0; m < 15; ++m) s += sh.Jp[i * 15 + m] * sh.HM[m * kLd + 15 + j];
      res->H[k] = sh.HM[(15 + i) * kLd + 15 + j] - s;
    }
  } else {
    // H (15 x 15): EdgeInertial::GetHessian2 (VP2, VV2), the random walks'
    // GetHessian2, the visual inliers
    for (int k = t; k < 9 * 24; k += kInThreads) {
      const int r = k / 24, c = k % 24;
      double s = 0;
#pragma unroll
      for (int q = 0; q < 9; ++q) s += sh.info[r * 9 + q] * sh.Ji[q * 24 + c];
      sh.OJ[k] = s;
    }
    __syncthreads();
    for (int k = t; k < 225; k += kInThreads) {
      const int i = k / 15, j = k % 15;
      double s = 0;
      if (i < 9 && j < 9) {
#pragma unroll
        for (int r = 0; r < 9; ++r) s += sh.Ji[r * 24 + 15 + i] * sh.OJ[r * 24 + 15 + j];
      }
      if (i >= 9 && i < 12 && j >= 9 && j < 12) s += sh.info_g[(i - 9) * 3 + j - 9];
      if (i >= 12 && j >= 12) s += sh.info_a[(i - 12) * 3 + j - 12];
      if (i < 6 && j < 6) s += sh.vis[i >= j ? i * (i + 1) / 2 + j : j * (j + 1) / 2 + i];
      res->H[k] = s;
    }
  }
  for (int i = t; i < cap; i += kInThreads) glv[i] = lv[i];
  if (t == 0) {
    for (int i = 0; i < 9; ++i) {
      res->Rwb[i] = (float)sh.cur.Rwb[i];
      res->Rwb_d[i] = sh.cur.Rwb[i];
    }
    for (int i = 0; i < 3; ++i) {
      res->twb[i] = (float)sh.cur.twb[i];
      res->v[i] = (float)sh.cur.v[i];
      res->bg[i] = (float)sh.cur.bg[i];
      res->ba[i] = (float)sh.cur.ba[i];
      res->twb_d[i] = sh.cur.twb[i];
      res->v_d[i] = sh.cur.v[i];
      res->bg_d[i] = sh.cur.bg[i];
      res->ba_d[i] = sh.cur.ba[i];
    }
    res->n_good = nobs - nBad;
    res->n_inliers = nInl;
  }
  if (done_host) {
    // single-problem host call (outputs in host-mapped memory): the call's
    // number, from its input block, stored at system scope after every
    // output word of the workgroup -- the host polls it
    __syncthreads();
    if (t == 0) {
      __threadfence_system();
      __hip_atomic_store(done_host, *seq_src, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  ISTAMP(5);
  ISTAMP_END;
}

hipError_t launch_pose_inertial(int mode, const orbgpu_imu_calib& c, int n_problems,
                                const orbgpu_imu_state* d_cur, const orbgpu_imu_state* d_prev,
                                const orbgpu_imu_preint* d_preint, const orbgpu_imu_prior* d_prior,
                                const orbgpu_inertial_obs* d_obs, const int* d_nobs, int obs_stride,
                                int rec_init, orbgpu_inertial_result* d_res, uint8_t* d_outlier,
                                hipStream_t st, int* done_host, const int* seq_src) {
  CalibD cd;
  cd.fx = c.fx;
  cd.fy = c.fy;
  cd.cx = c.cx;
  cd.cy = c.cy;
  cd.bf = c.bf;
  for (int i = 0; i < 9; ++i) {
    cd.Rcb[i] = c.Rcb[i];
    cd.Rbc[i] = c.Rbc[i];
  }
  for (int i = 0; i < 3; ++i) {
    cd.tcb[i] = c.tcb[i];
    cd.tbc[i] = c.tbc[i];
  }
  const int lds_obs = obs_stride < kInLdsObs ? obs_stride : kInLdsObs;
  const size_t lds = ((size_t)lds_obs * (sizeof(VisObs) + 1) + 15) & ~(size_t)15;
  const auto* obs = reinterpret_cast<const VisObs*>(d_obs);
  {  // > 64 KB of LDS needs the opt-in (per kernel and device)
    const void* fn = mode == ORBGPU_INERTIAL_LAST_FRAME
                         ? reinterpret_cast<const void*>(&k_pose_inertial<ORBGPU_INERTIAL_LAST_FRAME>)
                         : reinterpret_cast<const void*>(&k_pose_inertial<ORBGPU_INERTIAL_LAST_KEYFRAME>);
    if (lds_optin(fn, 96 * 1024) != hipSuccess) return hipErrorInvalidValue;
  }
  if (mode == ORBGPU_INERTIAL_LAST_FRAME)
    hipLaunchKernelGGL(k_pose_inertial<ORBGPU_INERTIAL_LAST_FRAME>, dim3(n_problems),
                       dim3(kInThreads), lds, st, cd, d_cur, d_prev, d_preint, d_prior, obs, d_nobs,
                       obs_stride, rec_init, d_res, d_outlier, lds_obs, done_host, seq_src);
  else
    hipLaunchKernelGGL(k_pose_inertial<ORBGPU_INERTIAL_LAST_KEYFRAME>, dim3(n_problems),
                       dim3(kInThreads), lds, st, cd, d_cur, d_prev, d_preint, d_prior, obs, d_nobs,
                       obs_stride, rec_init, d_res, d_outlier, lds_obs, done_host, seq_src);
  return hipGetLastError();
}

}  // namespace orbgpu

#ifdef ORB_STAMPS
extern "C" int orbgpu_debug_inertial_stamps(unsigned long long* out, int n) {
  if (n > 32) n = 32;
  static unsigned long long buf[64 * 32];
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(buf, HIP_SYMBOL(orbgpu::g_in_stamps), sizeof(buf)) != hipSuccess) return -1;
  for (int i = 0; i < n; ++i) {
    out[i] = 0;
    for (int c = 0; c < 64; ++c) out[i] += buf[c * 32 + i];
  }
  static const unsigned long long z[64 * 32] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(orbgpu::g_in_stamps), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif

ORBGPU_UNIFORM_READER(inertial)
