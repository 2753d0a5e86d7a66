// Device-side layout of one LocalBundleAdjustment call (lba_kernels.hip) and
// the host launchers lba_api.cpp drives.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace orbgpu {

struct LbaEdgeDev {  // == orbgpu_lba_edge, point index local to the shard
  int32_t point, kf;
  float u, v, ur, inv_sigma2;
};

struct LbaCamDev {
  double fx, fy, cx, cy, bf;
};

struct LbaArgs {
  LbaCamDev cam;
  int n_kf, n_pts, n_edges, n_free, n_sys, n_pairs;
  const LbaEdgeDev* edges;   // this shard's edges, point-major (insertion order in a point)
  const int* pt_begin;       // [n_pts + 1] CSR of edges per point
  const int* hidx;           // [n_kf] free-pose index, -1 = fixed
  const int* pose_begin;     // [n_free + 1] CSR of edges per free pose
  const int* pose_edges;     //   edge indices (ascending)
  const int* pair_i;         // [n_pairs] free-pose pairs (i <= j) sharing points
  const int* pair_j;
  const int* pair_begin;     // [n_pairs + 1] CSR of (edge of i, edge of j) entries
  const int* pair_ei;
  const int* pair_ej;
  double* err;       // [3 E] errors of the last computeActiveErrors
  double* hpl;       // [18 E] Hpl = Jp^T W Jl (6 x 3)
  double* hpp_e;     // [27 E] per-edge Hpp (lower, 21) + bp (6) terms
  double* hll_e;     // [12 E] per-edge Hll (9) + bl (3) terms
  double* hll;       // [9 P]
  double* bl;        // [3 P]
  double* dinv;      // [9 P]
  double* hpp;       // [36 F] full 6 x 6 per free pose
  double* bp;        // [6 F]
  double* diag;      // [n_sys + 1]: Hpp diagonal (sum-reduced), Hll max (max-reduced)
  double* sys;       // [n_sys^2 + 2 n_sys]: S, b_s, b_p  (the reduced buffer)
  double* work;      // [n_sys^2] factorisation when S does not fit LDS
  double* xp;        // [n_sys]
  double* scal;      // [4]: pose scale part, landmark scale part, chi2 out, spare
  double* partials;  // block partial sums
  unsigned* counter; // last-block-done counter (self-resetting)
  int* flags;        // [1]: solve / landmark-inverse failure of the current trial
};

hipError_t lba_errors(const LbaArgs& a, const double* poses, const double* pts, double* out,
                      hipStream_t st);
hipError_t lba_build(const LbaArgs& a, const double* poses, const double* pts, hipStream_t st);
hipError_t lba_schur(const LbaArgs& a, double lambda, hipStream_t st);
hipError_t lba_solve(const LbaArgs& a, double lambda, hipStream_t st);
hipError_t lba_trial(const LbaArgs& a, double lambda, const double* poses, const double* pts,
                     double* poses_trial, double* pts_trial, hipStream_t st);
hipError_t lba_classify(const LbaArgs& a, const double* poses, const double* pts, uint8_t* outlier,
                        hipStream_t st);

}  // namespace orbgpu
