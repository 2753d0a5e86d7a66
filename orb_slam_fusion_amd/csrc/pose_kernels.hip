// gfx950 PoseOptimization: one workgroup (G x 256 threads) runs a whole
// problem -- Optimizer::PoseOptimization (optimizer.cc:762-1051): 4
// outlier-rejection rounds x g2o Levenberg-Marquardt
// (optimization_algorithm_levenberg.cpp:59-168) over unary SE3 edges, dense
// 6x6 LDLT.  The working set (< 40 KB) stays on chip; edges are swept by all
// lanes (stereo observations first, so waves take one projection branch),
// per-sweep sums use a fixed reduction tree (deterministic), the 6x6 solve is
// lane-parallel per wave.  The pass is a chain of 60+ dependent sweeps that
// keep one CU's SIMDs issuing (4 waves), so problems are batched one
// workgroup each; G = 2 evaluates consecutive LM trials side by side.
//
// Per-edge errors are not stored: g2o's classification reads the error of the
// last computeActiveErrors() (possibly at a rejected trial pose), so the
// kernel remembers that pose and recomputes -- bit-identical values.
#include <hip/hip_runtime.h>

#include "lds_optin.h"
#include <stdint.h>

#include <algorithm>
#include <type_traits>

#include "pose_math_dev.h"

// fp64 solver arithmetic, parity by tolerance (not bit-exact like the
// extractor, whose TUs keep -ffp-contract=off): let products fuse into FMAs.
#pragma clang fp contract(fast)

namespace orbgpu {

// Profiling build only (make stamps): per-phase s_memtime totals, one flush
// per wave at exit into 64 spread copies (see orb_kernels.hip).
#ifdef ORB_STAMPS
__device__ unsigned long long g_pose_stamps[64 * 16];
#define PSTAMP_INIT                                            \
  unsigned long long pst_acc_[16] = {};                        \
  unsigned long long pst_prev_ = __builtin_amdgcn_s_memtime()
#define PSTAMP(i)                                                     \
  do {                                                                \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime();     \
    pst_acc_[i] += now_ - pst_prev_;                                  \
    pst_prev_ = now_;                                                 \
  } while (0)
#define PSTAMP_ADD(i, v) (pst_acc_[i] += (unsigned long long)(v))
#define PSTAMP_END                                                                  \
  do {                                                                              \
    if (threadIdx.x == 0) {                                                         \
      _Pragma("unroll") for (int i_ = 0; i_ < 16; ++i_)                             \
        if (pst_acc_[i_]) atomicAdd(&g_pose_stamps[(blockIdx.x & 63) * 16 + i_], pst_acc_[i_]); \
    }                                                                               \
  } while (0)
#else
#define PSTAMP_INIT (void)0
#define PSTAMP(i) (void)0
#define PSTAMP_ADD(i, v) (void)0
#define PSTAMP_END (void)0
#endif

struct PoseObsDev {
  float Xw[3];
  float u, v, ur;
  float inv_sigma2;
};

struct CamDev {
  double fx, fy, cx, cy, bf;
};

constexpr int kPoseThreads = 256;  // threads per trial group
constexpr int kPoseWaves = kPoseThreads / 64;

// A sweep's pose as a rotation matrix (Eigen's toRotationMatrix of the unit
// quaternion) + translation: the per-edge map is then 9 FMAs instead of the
// quaternion form's cross products (same value to rounding).
struct Se3R {
  double R[9], t[3];
};
__device__ __forceinline__ Se3R se3r(const Se3& T) {
  const double tx = 2 * T.qx, ty = 2 * T.qy, tz = 2 * T.qz;
  const double twx = tx * T.qw, twy = ty * T.qw, twz = tz * T.qw;
  const double txx = tx * T.qx, txy = ty * T.qx, txz = tz * T.qx;
  const double tyy = ty * T.qy, tyz = tz * T.qy, tzz = tz * T.qz;
  return Se3R{{1 - (tyy + tzz), txy - twz, txz + twy, txy + twz, 1 - (txx + tzz), tyz - twx,
               txz - twy, tyz + twx, 1 - (txx + tyy)},
              {T.t[0], T.t[1], T.t[2]}};
}
__device__ __forceinline__ void pose_map(const Se3R& T, const double X[3], double p[3]) {
#pragma unroll
  for (int i = 0; i < 3; ++i) p[i] = T.R[3 * i] * X[0] + T.R[3 * i + 1] * X[1] + T.R[3 * i + 2] * X[2] + T.t[i];
}

__device__ __forceinline__ void edge_error_p(const PoseObsDev& o, const double p[3], const RecipF64& rz,
                                             const CamDev& c, double e[3], bool stereo) {
  if (!stereo) {  // EdgeSE3ProjectXYZOnlyPose + Pinhole::Project
    e[0] = (double)o.u - (div_by(c.fx * p[0], rz) + c.cx);
    e[1] = (double)o.v - (div_by(c.fy * p[1], rz) + c.cy);
    e[2] = 0;
  } else {  // EdgeStereoSE3ProjectXYZOnlyPose::cam_project (float invz)
    const float invz = (float)div_by(1.0, rz);
    const double u = p[0] * (double)invz * c.fx + c.cx;
    const double v = p[1] * (double)invz * c.fy + c.cy;
    e[0] = (double)o.u - u;
    e[1] = (double)o.v - v;
    e[2] = (double)o.ur - (u - c.bf * (double)invz);
  }
}
__device__ __forceinline__ void edge_error(const PoseObsDev& o, const Se3R& T, const CamDev& c,
                                           double e[3], bool& stereo) {
  const double X[3] = {o.Xw[0], o.Xw[1], o.Xw[2]};
  double p[3];
  pose_map(T, X, p);
  stereo = o.ur >= 0.f;
  edge_error_p(o, p, recip_f64(p[2]), c, e, stereo);
}

__device__ __forceinline__ double edge_chi2(const double e[3], double info, bool stereo) {
  double s = e[0] * (info * e[0]) + e[1] * (info * e[1]);
  if (stereo) s += e[2] * (info * e[2]);
  return s;
}

__device__ __forceinline__ void edge_jacobian_p(const double p[3], const RecipF64& rz, const CamDev& c,
                                                bool stereo, double J[3][6]) {
  const double x = p[0], y = p[1], z = p[2];
  if (!stereo) {
    const RecipF64 rzz = recip_f64(z * z);
    const double pj00 = -div_by(c.fx, rz), pj02 = -div_by(-c.fx * x, rzz);
    const double pj11 = -div_by(c.fy, rz), pj12 = -div_by(-c.fy * y, rzz);
    const double S[3][6] = {{0, z, -y, 1, 0, 0}, {-z, 0, x, 0, 1, 0}, {y, -x, 0, 0, 0, 1}};
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      J[0][k] = pj00 * S[0][k] + -0.0 * S[1][k] + pj02 * S[2][k];
      J[1][k] = -0.0 * S[0][k] + pj11 * S[1][k] + pj12 * S[2][k];
      J[2][k] = 0;
    }
  } else {
    const double invz = div_by(1.0, rz), invz2 = invz * invz;
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

// DPP lane move of a double (two 32-bit halves); lanes whose source is out of
// range or whose row is masked off read 0.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ double dpp_f64(double v) {
  // full row mask: bound_ctrl reads 0 for out-of-range sources, so the
  // destination needs no zeroed old value (one v_mov_b32_dpp per half; the
  // build sweep's 28-value reduction was 224 of its VALU instructions)
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, ROW_MASK, 0xf, ROW_MASK == 0xf);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, ROW_MASK, 0xf, ROW_MASK == 0xf);
  return __hiloint2double(hi, lo);
}

// Wave sum with a fixed tree: in-row prefix by row_shr 1,2,4,8, then
// row_bcast15 / row_bcast31 carry the row totals up; lane 63 holds the sum.
__device__ __forceinline__ double wave_sum_to_lane63(double v) {
  v += dpp_f64<0x111, 0xf>(v);
  v += dpp_f64<0x112, 0xf>(v);
  v += dpp_f64<0x114, 0xf>(v);
  v += dpp_f64<0x118, 0xf>(v);
  v += dpp_f64<0x142, 0xa>(v);
  v += dpp_f64<0x143, 0xc>(v);
  return v;
}

__device__ __forceinline__ double uniform_f64(double v) {  // wave-uniform value -> SGPRs
  return __hiloint2double(__builtin_amdgcn_readfirstlane(__double2hiint(v)),
                          __builtin_amdgcn_readfirstlane(__double2loint(v)));
}

// Block-wide sums of NV doubles per thread into LDS (out[0..NV)), fixed tree:
// DPP row sums (lane 15 of each 16-lane row), the 4 NW row partials of the
// block in LDS, then (NW == 4) thread k adds value k's 16 partials in row
// order, or (NW > 4) 16-row slices first, the slices next.  Only LDS
// consumers need the result (the build sweep's system): no broadcast.
// (hf != nullptr, NV == 28: the H entries out[1..21] also land in hf as the
// full row-major 6x6, for the solves' row gathers)
__device__ __forceinline__ void mirror_h(int k, double a, double* hf) {
  if (k >= 1 && k < 22) {
    int r = 0;
#pragma unroll
    for (int q = 1; q < 6; ++q) r += (k - 1 >= q * (q + 1) / 2) ? 1 : 0;
    const int c = k - 1 - r * (r + 1) / 2;
    hf[r * 6 + c] = a;
    hf[c * 6 + r] = a;
  }
}
// The build's 28 sums over one 256-thread group mostly through LDS instead of
// DPP trees: one DPP step adds lane pairs (2i, 2i + 1), the odd lanes store
// the 28 pair sums (thread-major, 14 b128 writes), thread (k, c) = (t & 31,
// t >> 5) adds value k of pairs 16c .. 16c + 15 in order (k < 28), and thread
// k adds the 8 chunk sums in order.  Fixed order (reproducible); 84 VALU + 30
// LDS instructions a thread instead of 336 VALU.  T: 128 x 28 doubles of
// dynamic LDS (kPoseRedT), P: 224 doubles.
constexpr size_t kPoseRedT = 128 * 28 * sizeof(double);
__device__ __forceinline__ void block_sum28_lds_t(const double (&v)[28], double* T, double* P,
                                                  double* out, double* hf) {
  const int t = threadIdx.x;
  double w[28];
#pragma unroll
  for (int k = 0; k < 28; ++k) w[k] = v[k] + dpp_f64<0x111, 0xf>(v[k]);  // lane i: v_i + v_(i-1)
  if (t & 1)
#pragma unroll
    for (int k = 0; k < 28; k += 2)
      *reinterpret_cast<double2*>(T + (t >> 1) * 28 + k) = make_double2(w[k], w[k + 1]);
  __syncthreads();
  const int k = t & 31, c = t >> 5;
  if (k < 28) {
    const double* col = T + (16 * c) * 28 + k;
    double a = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) a += col[j * 28];
    P[k * 8 + c] = a;
  }
  __syncthreads();
  if (t < 28) {
    double a = P[t * 8];
#pragma unroll
    for (int q = 1; q < 8; ++q) a += P[t * 8 + q];
    out[t] = a;
    mirror_h(t, a, hf);
  }
  __syncthreads();
}

template <int NV, int NW>
__device__ __forceinline__ void block_sum_to_lds(double (&v)[NV], double* red, double* red2,
                                                 double* out, double* hf = nullptr) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    double x = v[k];
    x += dpp_f64<0x111, 0xf>(x);
    x += dpp_f64<0x112, 0xf>(x);
    x += dpp_f64<0x114, 0xf>(x);
    x += dpp_f64<0x118, 0xf>(x);
    v[k] = x;
  }
  if ((lane & 15) == 15)
#pragma unroll
    for (int k = 0; k < NV; ++k) red[(wave * 4 + (lane >> 4)) * NV + k] = v[k];
  __syncthreads();
  if constexpr (NW == 4) {
    if (threadIdx.x < NV) {
      double a = 0;
#pragma unroll
      for (int r = 0; r < 16; ++r) a += red[r * NV + threadIdx.x];
      out[threadIdx.x] = a;
      if (hf) mirror_h(threadIdx.x, a, hf);
    }
  } else {
    constexpr int S = NW / 4;  // 16-row slices
    if (threadIdx.x < NV * S) {
      const int k = threadIdx.x % NV, sl = threadIdx.x / NV;
      double a = 0;
#pragma unroll
      for (int r = 0; r < 16; ++r) a += red[(16 * sl + r) * NV + k];
      red2[sl * NV + k] = a;
    }
    __syncthreads();
    if (threadIdx.x < NV) {
      double a = red2[threadIdx.x];
#pragma unroll
      for (int sl = 1; sl < S; ++sl) a += red2[sl * NV + threadIdx.x];
      out[threadIdx.x] = a;
      if (hf) mirror_h(threadIdx.x, a, hf);
    }
  }
  __syncthreads();
}

__device__ __forceinline__ unsigned mbcnt64(uint64_t m) {  // set bits of m below this lane
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

template <int NW>
__device__ __forceinline__ int block_sum_i(int v, int* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  int r = 0;
#pragma unroll
  for (int w = 0; w < NW; ++w) r += red[w];
  __syncthreads();
  return r;
}

// G trial groups of kPoseThreads threads each.  The build sweep and the
// classification use the whole block; the LM trials of an iteration are
// evaluated G at a time (see k_pose_opt).
template <int G>
struct PoseShared {
  double red[G * kPoseWaves * 4 * 28];
  double red2[G * 28];
  double hb[28];                        // chi2, H (lower, 21), b (6) at the current pose
  double hf[36];                        // H as the full row-major 6x6 (the solves' gathers)
  double chi[2][G][kPoseWaves];         // trial chi2 wave partials, double-buffered by round
  double trial[16][14];                 // an iteration's trials q < 10: x (6), Tn (qx qy qz qw t0 t1 t2), ok
  double init[7];                       // the input pose (qx qy qz qw t0 t1 t2)
  int ired[G * kPoseWaves];
  int pcnt[2][G * kPoseWaves];          // observation partition: stereo / mono per wave
};

constexpr int kPoseLdsObs = 4096;  // observations staged in LDS (the rest re-read from HBM)

// One edge's contribution to a sweep at pose T: robust chi2 into acc[0] and
// BlockSolver::buildSystem's H (lower triangle, 21) and b (6) into
// acc[1..27].  Every sweep visits a thread's edges in the same order, so the
// sums are reproducible.  ST: the edge type when the caller knows it for the
// whole wave (1 EdgeStereo, 0 EdgeMono: only that projection is compiled),
// -1 to take it from the observation (both, selected per lane).
template <int ST = -1>
__device__ __forceinline__ void edge_accumulate(const PoseObsDev& o, const Se3R& T, const CamDev& cam,
                                                bool robust, double dmono, double dstereo,
                                                bool build, double (&acc)[28]) {
  const double X[3] = {o.Xw[0], o.Xw[1], o.Xw[2]};
  double p[3];
  pose_map(T, X, p);
  const RecipF64 rz = recip_f64(p[2]);
  double e[3];
  const bool st = ST < 0 ? o.ur >= 0.f : ST == 1;
  edge_error_p(o, p, rz, cam, e, st);
  const double info = (double)o.inv_sigma2;
  const double c2 = edge_chi2(e, info, st);
  double w = 1.0;
  if (robust) {
    double r0;
    huber_rho(c2, st ? dstereo : dmono, r0, w);
    acc[0] += r0;
  } else {
    acc[0] += c2;
  }
  if (!build) return;
  double J[3][6];
  edge_jacobian_p(p, rz, cam, st, J);
  const double wi = w * info;
  int hk = 1;
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    double g = J[0][r] * (info * e[0]) + J[1][r] * (info * e[1]);
    if (st) g += J[2][r] * (info * e[2]);
    acc[22 + r] -= w * g;
#pragma unroll
    for (int q = 0; q <= r; ++q) {
      double h = (J[0][r] * wi) * J[0][q] + (J[1][r] * wi) * J[1][q];
      if (st) h += (J[2][r] * wi) * J[2][q];
      acc[hk++] += h;
    }
  }
}

// One workgroup of G x 256 threads per problem.  g2o's inner LM loop
// (optimization_algorithm_levenberg.cpp:83-150) retries a rejected step with
// lambda *= ni, ni *= 2 and the same system, so the trial sequence of an
// iteration is known up front: group g evaluates trial q + g (its own LDLT,
// exp and chi2 sweep -- the same thread-to-edge map and reduction tree as a
// single group, so every trial's chi2 is the value the sequential loop would
// compute), then every thread scans the G outcomes in trial order and stops
// where the sequential loop would have.  Same path, G-fold fewer serial
// trial sweeps on rejection runs.  The build sweep spreads over all G x 256
// threads.
template <int G>
__global__ __launch_bounds__(kPoseThreads * G) void k_pose_opt(
    CamDev cam, const float* __restrict__ pose_in, const PoseObsDev* __restrict__ obs_all,
    const int* __restrict__ nobs, int obs_stride, float* __restrict__ pose_out,
    uint8_t* __restrict__ outlier_all, int* __restrict__ inliers, double* __restrict__ pose_out_d,
    int lds_obs, int* __restrict__ done_host, int seq) {
  // done_host (single-problem host call, outputs in host-mapped memory): the
  // call's number, stored at system scope after every output word of the
  // workgroup -- the host polls it instead of synchronising the stream
  auto signal_done = [&]() {
    if (!done_host) return;
    __syncthreads();  // every lane's output stores drained (vmcnt 0) before the barrier
    if (threadIdx.x == 0) {
      __threadfence_system();
      __hip_atomic_store(done_host, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  };
  constexpr int NT = kPoseThreads * G, NW = NT / 64;
  __shared__ PoseShared<G> sh;
  const int p = blockIdx.x;
  int t = threadIdx.x;  // t, tg, lane, gw: laundered per LM trial round (below)
  const int grp = __builtin_amdgcn_readfirstlane(t >> 8);
  int tg = t & (kPoseThreads - 1);
  int lane = t & 63, gw = (t >> 6) & (kPoseWaves - 1);
  const PoseObsDev* obs = obs_all + (size_t)p * obs_stride;
  // the observations up to the stride (in bounds whatever n is) are loaded
  // with n in one round trip when they fit kHold per thread -- the single-
  // problem path reads them straight from host memory (pose_api.cpp)
  constexpr int kHold = 3;
  const bool held = obs_stride <= NT * kHold;
  float oh[kHold][7];
  if (held) {
#pragma unroll
    for (int u = 0; u < kHold; ++u) {
      const int i = t + NT * u;
#pragma unroll
      for (int k = 0; k < 7; ++k) oh[u][k] = i < obs_stride ? reinterpret_cast<const float*>(obs + i)[k] : 0.f;
    }
  }
  const int n = nobs[p];
  uint8_t* level = outlier_all + (size_t)p * obs_stride;
  const float* pin = pose_in + 7 * p;
  if (n < 3) {  // optimizer.cc:951
    if (t < 7) pose_out[7 * p + t] = pin[t];
    if (t == 0) inliers[p] = 0;
    signal_done();
    return;
  }
  // observations (and their levels) live in LDS for the whole call: one
  // HBM read; only n > cap falls back to re-reading per sweep.  They are
  // stored as a stable partition, stereo first (pm[slot] = observation
  // index): a wave's 64 consecutive slots then take one projection branch
  // (EdgeStereo / EdgeMono) instead of both.  Only the order of the
  // per-thread partial sums changes.
  extern __shared__ __attribute__((aligned(16))) uint8_t pose_lds[];
  const int cap = min(n, lds_obs);
  PoseObsDev* ob = reinterpret_cast<PoseObsDev*>(pose_lds);
  uint8_t* lv = pose_lds + (size_t)lds_obs * sizeof(PoseObsDev);
  uint16_t* pm = reinterpret_cast<uint16_t*>(lv + ((lds_obs + 1) & ~1));
  // (G == 1) the build reduction's transpose buffer, 16-byte aligned after pm
  double* tred = reinterpret_cast<double*>(
      pose_lds + ((((size_t)lds_obs * sizeof(PoseObsDev) + ((lds_obs + 1) & ~1) + 2 * (size_t)lds_obs) + 15) &
                  ~(size_t)15));
  int n_st;
  {
    int c = 0;
    if (held) {
#pragma unroll
      for (int u = 0; u < kHold; ++u) c += t + NT * u < cap && oh[u][5] >= 0.f ? 1 : 0;
    } else {
      for (int i = t; i < cap; i += NT) c += obs[i].ur >= 0.f ? 1 : 0;
    }
    n_st = block_sum_i<NW>(c, sh.ired);
    const int w = t >> 6;
    int base_s = 0, base_m = n_st;
    // one NT-slot step of the stable partition (o: observation i0 + t)
    auto part_step = [&](int i0, const float (&o)[7]) {
      const int i = i0 + t;
      const bool in = i < cap;
      const bool st = in && o[5] >= 0.f;  // ur
      const uint64_t bs = __ballot(st), bm = __ballot(in && !st);
      if (lane == 0) {
        sh.pcnt[0][w] = __popcll(bs);
        sh.pcnt[1][w] = __popcll(bm);
      }
      __syncthreads();
      int ps = 0, pmn = 0, ts = 0, tm = 0;
#pragma unroll
      for (int v = 0; v < NW; ++v) {
        const int a = sh.pcnt[0][v], b = sh.pcnt[1][v];
        ps += v < w ? a : 0;
        pmn += v < w ? b : 0;
        ts += a;
        tm += b;
      }
      if (in) {
        const int pos = st ? base_s + ps + (int)mbcnt64(bs) : base_m + pmn + (int)mbcnt64(bm);
#pragma unroll
        for (int k = 0; k < 7; ++k) reinterpret_cast<float*>(ob + pos)[k] = o[k];
        lv[pos] = 0;
        pm[pos] = (uint16_t)i;
      }
      base_s += ts;
      base_m += tm;
      __syncthreads();
    };
    if (held) {
#pragma unroll
      for (int u = 0; u < kHold; ++u)
        if (NT * u < cap) part_step(NT * u, oh[u]);
    } else {
      for (int i0 = 0; i0 < cap; i0 += NT) {
        float o[7];  // PoseObsDev as 7 floats (no aggregate copy through scratch)
#pragma unroll
        for (int k = 0; k < 7; ++k) o[k] = reinterpret_cast<const float*>(obs + min(i0 + t, cap - 1))[k];
        part_step(i0, o);
      }
    }
  }
  for (int i = cap + t; i < n; i += NT) level[i] = 0;
  if (t < 7) sh.init[t] = pin[t];
  // poses kept in LDS and re-read where needed (register pressure)
  auto pose_at = [&](const double* a) { return Se3{a[0], a[1], a[2], a[3], {a[4], a[5], a[6]}}; };
  const double dmono = (double)(float)sqrt(5.991);  // `const float deltaMono = sqrt(5.991)`
  const double dstereo = (double)(float)sqrt(7.815);
  bool robust = true;
  int nbad_round = 0;
  Se3 T;
  __syncthreads();
  PSTAMP_INIT;

  // computeActiveErrors at pose X (robust chi2) by this thread's group: a
  // thread's edges i = tg + 256 j are taken three at a time (independent
  // chains, ILP), the accumulation stays in edge order; the wave sums land in
  // dst[wave of the group] (added in wave order by the readers).
  constexpr int kU = 3;  // (ILP only: the sums are the same for any kU)
  // Typed waves: when the stereo block [0, n_st) and the mono block
  // [n_st, cap) fit in the group's 4 waves at kU x 64 edges a wave, wave gw
  // takes one contiguous run of a single edge type (edges wbeg + lane + 64 u)
  // and runs only that projection; otherwise (wtype < 0) every wave takes
  // edges tg + 256 j and selects the projection per lane.  Wave-uniform.
  int wtype = -1, wbeg = 0, wend = 0;
  {
    constexpr int per = kU * 64;
    const int ws = (n_st + per - 1) / per, wm = (cap - n_st + per - 1) / per;
    if (ws + wm <= kPoseWaves) {
      const int gwu = __builtin_amdgcn_readfirstlane(gw);
      if (gwu < ws) {
        wtype = 1;
        wbeg = gwu * per;
        wend = min(wbeg + per, n_st);
      } else if (gwu - ws < wm) {
        wtype = 0;
        wbeg = n_st + (gwu - ws) * per;
        wend = min(wbeg + per, cap);
      } else {
        wtype = 2;  // no edges
      }
    }
  }
  auto chi_typed = [&](auto stc, const Se3R& X, double& acc0) {
    constexpr int ST = decltype(stc)::value;
    PoseObsDev o[kU];
    bool live[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int i = wbeg + lane + 64 * u;
      live[u] = i < wend && !lv[min(i, wend - 1)];
      o[u] = ob[min(i, wend - 1)];
    }
    double part[kU][28];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      part[u][0] = 0;
      edge_accumulate<ST>(o[u], X, cam, robust, dmono, dstereo, false, part[u]);
    }
#pragma unroll
    for (int u = 0; u < kU; ++u)
      if (live[u]) acc0 += part[u][0];
  };
  auto chi_sweep = [&](const Se3& Xq, double* dst) {
    const Se3R X = se3r(Xq);
    double acc[28];
    acc[0] = 0;
    if (wtype == 1)
      chi_typed(std::integral_constant<int, 1>{}, X, acc[0]);
    else if (wtype == 0)
      chi_typed(std::integral_constant<int, 0>{}, X, acc[0]);
    else if (wtype < 0)
    for (int i0 = tg; i0 < cap; i0 += kU * kPoseThreads) {
      PoseObsDev o[kU];
      bool live[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int i = i0 + u * kPoseThreads;
        live[u] = i < cap && !lv[min(i, cap - 1)];
        o[u] = ob[min(i, cap - 1)];
      }
      double part[kU][28];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        part[u][0] = 0;
        edge_accumulate(o[u], X, cam, robust, dmono, dstereo, false, part[u]);
      }
#pragma unroll
      for (int u = 0; u < kU; ++u)
        if (live[u]) acc[0] += part[u][0];
    }
    for (int i = cap + tg; i < n; i += kPoseThreads)
      if (!level[i]) edge_accumulate(obs[i], X, cam, robust, dmono, dstereo, false, acc);
    const double s = wave_sum_to_lane63(acc[0]);
    if (lane == 63) dst[gw] = s;
  };
  // computeActiveErrors + buildSystem at pose X -> sh.hb (chi2, H, b); one
  // edge at a time straight into the accumulators (three in flight held 84
  // partials: 306 VGPRs and 0.312 ms per 64 problems; one: 185 VGPRs, 0.296)
  auto build_sweep = [&](const Se3& Xq) {
    const Se3R X = se3r(Xq);
    double acc[28];
#pragma unroll
    for (int k = 0; k < 28; ++k) acc[k] = 0;
    // g2o adds each edge's block into H/b in edge order, the chi2 term first
    // as in computeActiveErrors
    if (G == 1 && wtype == 1) {
      for (int i = wbeg + lane; i < wend; i += 64)
        if (!lv[i]) edge_accumulate<1>(ob[i], X, cam, robust, dmono, dstereo, true, acc);
    } else if (G == 1 && wtype == 0) {
      for (int i = wbeg + lane; i < wend; i += 64)
        if (!lv[i]) edge_accumulate<0>(ob[i], X, cam, robust, dmono, dstereo, true, acc);
    } else if (G > 1 || wtype < 0) {
      for (int i = t; i < cap; i += NT)
        if (!lv[i]) edge_accumulate(ob[i], X, cam, robust, dmono, dstereo, true, acc);
    }
    for (int i = cap + t; i < n; i += NT)
      if (!level[i]) edge_accumulate(obs[i], X, cam, robust, dmono, dstereo, true, acc);
    if constexpr (G == 1)
      block_sum28_lds_t(acc, tred, sh.red, sh.hb, sh.hf);
    else
      block_sum_to_lds<28, NW>(acc, sh.red, sh.red2, sh.hb, sh.hf);
  };

  const double* hb = sh.hb;
  int buf = 0;
  for (int it = 0; it < 4; ++it) {
    T = pose_at(sh.init);
    PSTAMP(0);
    build_sweep(T);  // computeActiveErrors + buildSystem at the round's start
    PSTAMP(1);
    PSTAMP_ADD(8, 1);
    double cur = hb[0];
    const double* teval = sh.init;  // the pose of the last computeActiveErrors (a trial's)
    double lambda = 0, ni = 2;
    int nbad = 0;
    for (int iter = 0; iter < 10; ++iter) {
      asm volatile("" : "+s"(wtype), "+s"(wbeg), "+s"(wend));
      const double ini = cur;
      if (iter == 0) {  // computeLambdaInit: tau * max diag
        double mx = 0;
        int dk = 0;
#pragma unroll
        for (int r = 0; r < 6; ++r) {
          dk += r;
          mx = fmax(fabs(hb[1 + dk + r]), mx);
        }
        lambda = 1e-5 * mx;
        ni = 2;
        nbad = 0;
      }
      double rho = 0;
      int q = 0;
      bool accepted = false, done = false;
      // Every trial of this iteration up front: g2o retries a rejected step on
      // the same system with lambda *= ni, ni *= 2, so trial q solves
      // H + lambda_q I with the lambda the sequential loop holds after q
      // rejections (the same products in the same order).  The 16-lane rows of
      // the block's waves take trials q = 4 wave + row at once (ldlt6_gj_rows,
      // then the exp per row), so an iteration pays one solve + exp instead of
      // one per trial; the sweeps below read trial[q].
      PSTAMP(0);
      __syncthreads();  // the previous iteration's readers of sh.trial are done
      {
        const int qq = (t >> 4) & (4 * NW - 1);
        double lq = lambda, nq = ni;
        for (int k = 0; k < min(qq, 10); ++k) {
          lq *= nq;
          nq *= 2;
        }
        double x[6];
        const bool ok = ldlt6_gj_rows(hb, sh.hf, lq, x);
        PSTAMP(2);
        const Se3 Tn = se3_compose(se3_exp<false>(x), T);
        PSTAMP(3);
        if ((t & 15) == 0 && qq < 10) {
          double* tr = sh.trial[qq];
#pragma unroll
          for (int j = 0; j < 6; ++j) tr[j] = x[j];
          tr[6] = Tn.qx;
          tr[7] = Tn.qy;
          tr[8] = Tn.qz;
          tr[9] = Tn.qw;
          tr[10] = Tn.t[0];
          tr[11] = Tn.t[1];
          tr[12] = Tn.t[2];
          tr[13] = ok ? 1.0 : 0.0;
        }
      }
      __syncthreads();
      do {
        // the thread indices are opaque to the optimiser here, so the loop
        // body's thread-predicate compares are not hoisted into long-lived
        // SGPR lane masks
        asm volatile("" : "+v"(t), "+v"(tg), "+v"(lane), "+v"(gw));
        asm volatile("" : "+s"(wtype), "+s"(wbeg), "+s"(wend));
        // this group's trial q + grp (precomputed above; past trial 9 the
        // group idles: the sequential loop stops at 10)
        PSTAMP(0);
        if (q + grp < 10) chi_sweep(pose_at(sh.trial[q + grp] + 6), sh.chi[buf][grp]);
        __syncthreads();
        PSTAMP(4);
        PSTAMP_ADD(10, 1);
        // the outcomes in trial order, exactly as the sequential do-while
        const int gn = min(G, 10 - q);
        for (int g = 0; g < gn; ++g) {
          const double* tr = sh.trial[q];
          const double* cg = sh.chi[buf][g];
          double tmp = cg[0];
#pragma unroll
          for (int w = 1; w < kPoseWaves; ++w) tmp += cg[w];
          PSTAMP_ADD(9, 1);
          teval = tr + 6;
          if (tr[13] == 0.0) tmp = 1.79769313486231570815e+308;
          rho = cur - tmp;
          double scale = 0;
#pragma unroll
          for (int j = 0; j < 6; ++j) scale += tr[j] * (lambda * tr[j] + hb[22 + j]);
          scale += 1e-3;
          rho /= scale;
          ++q;
          if (rho > 0 && isfinite(tmp)) {
            double alpha = 1. - cube(2 * rho - 1);
            alpha = fmin(alpha, 2. / 3.);
            lambda *= fmax(1. / 3., alpha);
            ni = 2;
            cur = tmp;
            T = pose_at(teval);
            accepted = true;
            done = true;
            break;
          }
          lambda *= ni;
          ni *= 2;
          if (!(rho < 0) || q == 10) {
            done = true;
            break;
          }
        }
        buf ^= 1;
      } while (!done);
      if (q == 10 || rho == 0) break;
      if ((ini - cur) * 1e3 < ini)
        nbad++;
      else
        nbad = 0;
      if (nbad >= 3) break;
      // next iteration: its computeActiveErrors at T reproduces `cur` (the
      // accepted trial's sweep at the same pose), so only buildSystem runs;
      // after a rejected-but-terminal-free exit T is unchanged and so is the
      // system already in sh.hb
      PSTAMP(0);
      if (accepted) {
        build_sweep(T);
        PSTAMP(1);
        PSTAMP_ADD(8, 1);
      }
    }

    // classify (optimizer.cc:966-1037): level-1 edges recompute at T, level-0
    // edges keep the error of the last sweep (at Teval)
    int bad = 0;
    const Se3R TR = se3r(T), TevalR = se3r(pose_at(teval));
    auto classify = [&](const PoseObsDev& o, uint8_t& l) {
      double e[3];
      bool st;
      edge_error(o, l ? TR : TevalR, cam, e, st);
      const float chi2 = (float)edge_chi2(e, (double)o.inv_sigma2, st);
      const bool out = chi2 > (st ? 7.815f : 5.991f);
      l = out ? 1 : 0;
      bad += out;
    };
    for (int i = t; i < cap; i += NT) classify(ob[i], lv[i]);
    for (int i = cap + t; i < n; i += NT) {
      uint8_t l = level[i];
      classify(obs[i], l);
      level[i] = l;
    }
    nbad_round = block_sum_i<NW>(bad, sh.ired);
    PSTAMP(5);
    if (it == 2) robust = false;
    if (n < 10) break;
  }

  for (int i = t; i < cap; i += NT) level[pm[i]] = lv[i];
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
  signal_done();
  PSTAMP(0);
  PSTAMP_END;
}

template <int G>
static hipError_t launch_pose_opt_g(const CamDev& c, const float* d_pose_in, const void* d_obs,
                                    const int* d_nobs, int obs_stride, int n_problems,
                                    float* d_pose_out, uint8_t* d_outlier, int* d_inliers,
                                    double* d_pose_out_d, hipStream_t st, int* done_host, int seq) {
  // observations staged in LDS: up to kPoseLdsObs, and what fits beside the
  // static part and (G == 1) the reduction buffer in 160 KB
  const size_t fixed = sizeof(PoseShared<G>) + (G == 1 ? kPoseRedT : 0) + 64;
  const int fit = (int)((160 * 1024 - fixed) / (sizeof(PoseObsDev) + 3));
  const int lds_obs = std::min(std::min(obs_stride, kPoseLdsObs), fit);
  // observations, levels, slot -> observation index (k_pose_opt)
  const size_t lds = (((size_t)lds_obs * sizeof(PoseObsDev) + (((size_t)lds_obs + 1) & ~(size_t)1) +
                       2 * (size_t)lds_obs + 15) & ~(size_t)15) +
                     (G == 1 ? kPoseRedT : 0);  // + the build reduction's transpose buffer
  if (lds + sizeof(PoseShared<G>) > 64 * 1024) {
    if (lds_optin(reinterpret_cast<const void*>(&k_pose_opt<G>), (int)lds) != hipSuccess)
      return hipErrorInvalidValue;
  }
  hipLaunchKernelGGL(k_pose_opt<G>, dim3(n_problems), dim3(kPoseThreads * G), lds, st, c,
                     d_pose_in, reinterpret_cast<const PoseObsDev*>(d_obs), d_nobs, obs_stride,
                     d_pose_out, d_outlier, d_inliers, d_pose_out_d, lds_obs, done_host, seq);
  return hipGetLastError();
}

// groups: trial groups per problem (1 or 2); see k_pose_opt.  Four groups
// (1024 threads) cap a thread at 128 VGPRs and spill the build sweep
// (measured 0.61 ms per 64 problems vs 0.32 for two).
hipError_t launch_pose_opt(const double cam[5], const float* d_pose_in, const void* d_obs,
                           const int* d_nobs, int obs_stride, int n_problems, float* d_pose_out,
                           uint8_t* d_outlier, int* d_inliers, double* d_pose_out_d,
                           hipStream_t st, int groups, int* done_host, int seq) {
  CamDev c{cam[0], cam[1], cam[2], cam[3], cam[4]};
  switch (groups) {
    case 1:
      return launch_pose_opt_g<1>(c, d_pose_in, d_obs, d_nobs, obs_stride, n_problems, d_pose_out,
                                  d_outlier, d_inliers, d_pose_out_d, st, done_host, seq);
    case 2:
      return launch_pose_opt_g<2>(c, d_pose_in, d_obs, d_nobs, obs_stride, n_problems, d_pose_out,
                                  d_outlier, d_inliers, d_pose_out_d, st, done_host, seq);
    default:
      return hipErrorInvalidValue;
  }
}

}  // namespace orbgpu

#ifdef ORB_STAMPS
extern "C" int orbgpu_debug_pose_stamps(unsigned long long* out, int n) {
  if (n > 16) n = 16;
  static unsigned long long buf[64 * 16];
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(buf, HIP_SYMBOL(orbgpu::g_pose_stamps), sizeof(buf)) != hipSuccess) return -1;
  for (int i = 0; i < n; ++i) {
    out[i] = 0;
    for (int c = 0; c < 64; ++c) out[i] += buf[c * 16 + i];
  }
  static const unsigned long long z[64 * 16] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(orbgpu::g_pose_stamps), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif

ORBGPU_UNIFORM_READER(pose)
#if ORBGPU_CHECK_UNIFORM
extern "C" unsigned orbgpu_uniform_violations_inertial(void);
extern "C" unsigned orbgpu_uniform_violations_lba(void);
// Debug builds only (make checkuniform): wave-uniform branch violations
// since the last call, summed over the kernel translation units (uniform_dev.h).
extern "C" unsigned orbgpu_debug_uniform_violations(void) {
  return orbgpu_uniform_violations_pose() + orbgpu_uniform_violations_inertial() +
         orbgpu_uniform_violations_lba();
}

// Positive control of the checker: se3_exp<true> on a wave whose lanes do NOT
// agree (lane 0 takes the theta < 1e-5 branch, the rest the series) must be
// counted.  Returns the violations it raised (cleared), or ~0u on an error.
namespace orbgpu {
__global__ void k_uniform_selftest(double* out) {
  const int lane = threadIdx.x & 63;
  const double u[6] = {2e-3 * lane, 0, 0, 0, 0, 0};
  out[threadIdx.x] = se3_exp<true>(u).qw;
}
}  // namespace orbgpu
extern "C" unsigned orbgpu_debug_uniform_selftest(void) {
  double* d = nullptr;
  if (orbgpu_debug_uniform_violations() != 0 || hipMalloc(&d, 64 * sizeof(double)) != hipSuccess) return ~0u;
  hipLaunchKernelGGL(orbgpu::k_uniform_selftest, dim3(1), dim3(64), 0, nullptr, d);
  const unsigned v = hipDeviceSynchronize() == hipSuccess ? orbgpu_uniform_violations_pose() : ~0u;
  (void)hipFree(d);
  return v;
}
#endif
