// Device-side layout of one LocalBundleAdjustment call (lba_kernels.hip) and
// the host launchers lba_api.cpp drives.
//
// The g2o Levenberg-Marquardt loop (optimization_algorithm_levenberg.cpp:59-168)
// runs on the device: its state (lambda, ni, current chi2, trial / iteration
// counters, the stop decision) lives in LbaCtrl and every kernel reads it at
// entry; a kernel whose stage is not due (the optimisation is done, or the
// system is already built this iteration) returns at once.  The host only
// queues "steps" (build + one LM trial) a few ahead of the device and stops
// when the device reports done through a host-mapped word.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/orbgpu.h"

namespace orbgpu {

// Key-frame models: LocalBundleAdjustment's VertexSE3Expmap (7 doubles: unit
// quaternion + t; 6 reduced-system rows) and LocalInertialBA's ImuCamPose +
// IMU vertices (StateD, 33 doubles: Rwb twb Rcw tcw v bg ba; 15 rows VP VV
// VG VA).
enum LbaModel { kModelSe3 = 0, kModelImu = 1 };
constexpr int kImuStateStride = 33;
constexpr int kImuDim = 15;
constexpr int kImuPairQ = 30 * 30 + 30;  // per IMU link: 30 x 30 form + gradient

struct LiaCalibDev {  // == CalibD (imu_math_dev.h)
  double fx, fy, cx, cy, bf;
  double Rcb[9], tcb[3], Rbc[9], tbc[3];
};

struct LiaImuDev {  // == orbgpu_lia_imu_edge
  int32_t kf1, kf2, flags, pad;
  orbgpu_imu_preint pi;
};
static_assert(sizeof(LiaImuDev) == sizeof(orbgpu_lia_imu_edge), "LiaImuDev layout");

struct LbaEdgeDev {  // one observation of the shard, point-major (insertion order in a point)
  int32_t point;     // shard-local point index
  int32_t kf;        // keyframe index
  int32_t f;         // free-pose (Hessian) index, -1 = fixed keyframe
  int32_t pad;
  float u, v, ur, inv_sigma2;
};

struct LbaCamDev {
  double fx, fy, cx, cy, bf;
};

// LM state (one per call, device memory).  Written only by the single thread
// that takes an LM decision (last block of a stage, or k_lba_ctl when sharded).
struct LbaCtrl {
  double lambda, ni, cur, ini, chi_init, user_lambda;
  double last;  // robust chi2 of the last computeActiveErrors (LocalInertialBA's err_end)
  int it, q, nbad, need_build, done, state, iters_done, trials, max_iters, stopped;
  int lin_state;   // the state whose per-edge terms (lin_of) are current; -1: none
  int lambda_due;  // sharded: the first build's lambda init waits for the all-reduce (k_lba_ctl)
  int call;        // the call's sequence number (LbaHostWords::results)
  int classified;  // the outliers and the final state are in the host-mapped results
};

// The reduced-camera-system factorisation (lba_kernels.hip): the packed
// lower-triangle tiles in LDS (one block), S in HBM with D and y in LDS (one
// block), or every piece in HBM over the whole device (any window size).
enum LbaSolveMode { kSolveLds = 0, kSolveBlock = 1, kSolveGrid = 2 };

// LM decision points whose inputs a point-sharded run all-reduces first
enum LbaCtlMode { kCtlInit = 0, kCtlLambda = 1, kCtlDecide = 2 };

static_assert(sizeof(LbaCtrl) % 4 == 0 && sizeof(LbaCtrl) <= 128, "LbaCtrl: copied by dwords into 128 B");

// host-mapped progress word: (done << 32) | trials completed
struct LbaHostWords {
  unsigned long long progress;
  uint32_t stop;     // mirror of the caller's *pbStopFlag, read by the device
  uint32_t results;  // LbaCtrl::call once that call's results are complete in host memory
};

struct LbaArgs {
  LbaCamDev cam;
  int n_kf, n_pts, n_edges, n_free, n_sys, n_pairs;
  int sharded;               // 1: LM decisions wait for the host's all-reduce (k_lba_ctl)
  int solve_mode;            // LbaSolveMode: where the reduced system is factorised
  int n_pad;                 // n_sys rounded up to the 16-wide MFMA tile
  int n_edgeless;            // points of the shard with no edge (their Hll is 0)
  const LbaEdgeDev* edges;   // [n_edges]
  const int* hidx;           // [n_kf] free-pose index, -1 = fixed
  const int* pt_begin;       // [n_pts + 1] CSR of edges per point
  const int* pose_begin;     // [n_free + 1] CSR of edges per free pose
  const int4* pslot;         //   {edge, point, point's first edge, end} (edge ascending; k_lba_begin writes it)
  const int* ef;             // [n_edges] free-pose index of each edge (edges[i].f, packed)
  const int* pair_i;         // [n_pairs] free-pose pairs (i <= j), row-major upper triangle
  const int* pair_j;
  // point-major Schur complement (k_lba_schur_band + k_lba_schur_sum): the
  // shard's points with a free edge, ordered by their lowest free pose (a
  // counting sort), cut into chunks whose free poses span a band of at most
  // kSchurBandMax poses [b0, b0 + w).  A chunk's part of the Schur complement
  // is the MFMA product W_all H_all^T over its points (W_all / H_all: the
  // band's 6 w rows x 4 columns per point, each point's W = Hpl (Hll +
  // lambda I)^-1 / Hpl in its poses' rows, zeros elsewhere; one more H row
  // holds bl, so the product also carries W bl).  n_chunks == 0: one block
  // per pose pair (k_lba_schur) -- a point whose free poses span more than
  // kSchurBandMax.
  // Schur complement by point range (k_lba_schur_split): sc_split ranges of
  // the shard's points (1..kSchurSplitMax; 0 = the band / pair kernels), and
  // per free pose the pslot offsets where each range starts
  int force_lin;             // 1: every build re-linearises (ORBGPU_LBA_RELINEARIZE; tests compare)
  int sc_split;
  const int* pose_split;  // [n_free * (sc_split + 1)]
  int sc_fold_inline;     // 1: each pair's last range block folds the ranges (else k_lba_schur_fold)
  unsigned* pair_cnt;     // [n_pairs] per-pair tickets (self-resetting; zero in every upload)
  int n_chunks;
  const int* sc_order;  // [points with a free edge] shard point index, chunk order
  const int4* sc_chunk;  // [n_chunks] {first in sc_order, points, b0, w}
  const int* sc_tile0;   // [n_chunks + 1] first partial tile of each chunk (256 doubles a tile)
  double* sc_part;       // the chunks' upper product tiles | split: [n_pairs * sc_split * 42]
  double* poses[2];          // [7 n_kf] current / trial state (ctrl.state selects)
  double* pts[2];            // [3 n_pts]
  double* err;               // [3 E] errors of the last computeActiveErrors
  // per-edge terms, two copies (one per LM state, lin_of in lba_kernels.hip):
  double* hpl;               // 2 x [18 E] Hpl = Jp^T W Jl (6 x 3), free-pose edges only
  double* hpp_e;             // 2 x [27][n_slots] per-edge Hpp (lower, 21) + bp (6) terms, component-
                             //   major in pslot order (k_lba_sums reads a pose's run coalesced)
  double* hll_e;             // 2 x [12][n_edges] per-edge Hll (9) + bl (3) terms, component-major
  const int* eslot;          // [n_edges] pslot index of each free-pose edge (-1: fixed pose)
  int n_slots;               // pslot entries (free-pose edges)
  double* hll;               // [9 P]
  double* bl;                // [3 P]
  double* hpp;               // [36 F] full 6 x 6 per free pose
  double* bp;                // [6 F]
  double* diag;              // [n_sys + 1]: Hpp diagonal | Hll max  (lambda init, reduced)
  double* sys;               // [n_sys^2 + 2 n_sys]: S | b_s | b_p  (reduced per trial)
  double* work;              // [n_pad (n_pad + 1)] factorisation when S does not fit LDS
  double* xp;                // [n_sys] pose step
  double* red;               // [4]: init / trial reduce buffer (chi2, landmark scale, bad, stop)
  double* scal;              // [2]: pose part of computeScale, solve failure
  double* partials;          // block partials (2 per block)
  double* pose_part;         // [kSumsQ n_free][27] k_lba_sums' per-(pose, quarter) Hpp / bp partials
  unsigned* counter;         // last-block-done tickets (self-resetting), one per stage
  LbaCtrl* ctrl;
  LbaHostWords* host;        // host-mapped
  // one-rank calls: the outliers, the final state and the LbaCtrl go straight
  // to host-mapped memory, written by the first kernel of the step queued
  // after the one that ends the LM (k_lba_sums) or by k_lba_classify
  int early_out;
  uint8_t* res_outlier;      // [n_edges]
  double* res_out;           // [pstride n_kf | 3 n_pts]
  uint32_t* res_ctrl;        // LbaCtrl copy
  // ---- key-frame model (LocalInertialBA: kModelImu)
  int model;                 // LbaModel
  int pdim;                  // reduced-system rows per free key frame (6 / 15)
  int pstride;               // doubles per key-frame state (7 / 33)
  LiaCalibDev icb;           // kModelImu: camera + mTcb / mTbc
  const uint8_t* close;      // [n_pts] MapPoint::mTrackDepth < 10 (kModelImu outlier rule)
  int n_imu;                 // IMU links (EdgeInertial + EdgeGyroRW + EdgeAccRW each)
  const LiaImuDev* imu;      // [n_imu]
  const int* free_kf;        // [n_free] key frame of each free index
  const int* imu_inc;        // [n_free + 1] CSR of the links incident to a free key frame,
  const int4* imu_inc_rec;   //   link order: {link, its side, the other's free index (-1 fixed), side}
  double* imu_q;             // 2 x [n_imu * kImuPairQ] (one copy per LM state) per link: form over
                             //   (kf1 dims, kf2 dims) + gradient
  double* himu;              // [n_sys^2 + n_sys] the links' part of the camera system | gradient
  double* imu_tot;           // [2 + n_imu]: per link (from 2) robust chi2 at the last evaluation
};

// Every launcher dispatches on a.model.  kModelImu adds, per stage: the IMU
// links' chi2 at the initial / trial state (lba_begin, lba_solve_trial), their
// quadratic forms and the camera-side system they add (lba_build), and the
// trial key-frame states (ImuCamPose::Update + additive IMU vertices) before
// the edge stage of a trial.
hipError_t lba_begin(const LbaArgs& a, hipStream_t st);   // initial errors + LM state
// linearize = false leaves out the edge / link linearisation launches: every
// build after the first finds its state's terms already written by the
// accepted trial (LbaCtrl::lin_state; an iteration that ends without
// accepting a trial either ends the optimisation or rebuilds at a state whose
// terms are current), so only the first step needs them.
hipError_t lba_step(const LbaArgs& a, hipStream_t st, bool linearize);  // build (if due) + one trial
// sharded pieces (the host all-reduces between them)
hipError_t lba_build(const LbaArgs& a, hipStream_t st, bool linearize = true);
hipError_t lba_schur(const LbaArgs& a, hipStream_t st);
hipError_t lba_solve_trial(const LbaArgs& a, hipStream_t st);
hipError_t lba_ctl(const LbaArgs& a, int mode, hipStream_t st);
// outliers + the final state: out = [poses 7 n_kf | pts 3 n_pts] (doubles),
// and a copy of the LbaCtrl at ctrl_out; to_host: into a.res_* (host-mapped)
// unless already there, then LbaHostWords::results = the call
hipError_t lba_classify(const LbaArgs& a, uint8_t* outlier, double* out, void* ctrl_out, hipStream_t st);
hipError_t lba_classify_to_host(const LbaArgs& a, hipStream_t st);
size_t lba_solve_lds_bytes(int n_pad);
constexpr int kSumsQ = 4;                // k_lba_sums blocks per free pose
constexpr int kSchurSplitMax = 8;        // point ranges of k_lba_schur_split (one per XCD)
constexpr int kSchurSplitEdges = 128;    // target pose edges per (pair, range) block
constexpr int kSchurBandMax = 15;       // free poses a Schur chunk spans (6 w + 1 <= 96 rows)
constexpr int kSchurChunkLds = 120 * 1024;  // W_all + H_all of a chunk: 64 x points x padded rows bytes

// padded product rows of a band of w poses (6 w rows + the bl row, to the 16-row MFMA tile)
__host__ __device__ inline int schur_band_rows(int w) { return (6 * w + 1 + 15) / 16 * 16; }

// the solver path for an n_pad-row system, and the doubles of a.work it needs
int lba_solve_mode(int n_pad);
bool lba_solve_mode_fits(int mode, int n_pad);
size_t lba_solve_work_doubles(int mode, int n_pad);

}  // namespace orbgpu
