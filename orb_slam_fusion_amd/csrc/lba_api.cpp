// C-ABI implementation of the LocalBundleAdjustment half of include/orbgpu.h.
//
// The host lays the shard's graph out once per call in O(edges) (the
// reference builds its g2o graph on the host too, optimizer.cc:1127-1354) and
// uploads it with the initial state in ONE copy; the whole g2o
// Levenberg-Marquardt loop (optimization_algorithm_levenberg.cpp:59-168) then
// runs on the device (lba_kernels.hip, LbaCtrl).  The host keeps a couple of
// LM steps queued ahead of the device, mirrors *pbStopFlag into a host-mapped
// word the device polls where g2o calls terminate(), and stops queueing when
// the device reports done; one copy brings the result back.
//
// A point-sharded multi-GPU call (reduce != NULL) runs the same
// kernels with the host in the loop: each rank's partial reduced camera
// system, chi2, landmark part of computeScale and lambda-init diagonal are
// all-reduced through the caller's callback, after which k_lba_ctl takes the
// (identical) LM decision on every rank.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <new>
#include <thread>
#include <vector>

#include "../../include/orbgpu.h"
#include "lba_launch.h"

using namespace orbgpu;

namespace {

constexpr int kAhead = 2;            // LM steps queued ahead of the device
constexpr size_t kLdsBudget = 160 * 1024;

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

}  // namespace

struct orbgpu_lba_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  char* arena = nullptr;  // device
  size_t arena_cap = 0;
  char* staging = nullptr;  // pinned host
  size_t staging_cap = 0;
  LbaHostWords* host = nullptr;  // pinned, mapped, coherent
  LbaHostWords* host_dev = nullptr;
  ~orbgpu_lba_ctx() {
    if (arena) (void)hipFree(arena);
    if (staging) (void)hipHostFree(staging);
    if (host) (void)hipHostFree(host);
  }
  bool reserve(size_t dev_bytes, size_t host_bytes) {
    if (dev_bytes > arena_cap) {
      if (arena) (void)hipFree(arena);
      arena = nullptr;
      arena_cap = 0;
      if (hipMalloc(&arena, dev_bytes) != hipSuccess) return false;
      arena_cap = dev_bytes;
    }
    if (host_bytes > staging_cap) {
      if (staging) (void)hipHostFree(staging);
      staging = nullptr;
      staging_cap = 0;
      if (hipHostMalloc(&staging, host_bytes) != hipSuccess) return false;
      staging_cap = host_bytes;
    }
    return true;
  }
};

extern "C" {

orbgpu_status orbgpu_lba_ctx_create(int device, orbgpu_lba_ctx** out) {
  if (!out) return ORBGPU_ERR_INVALID;
  *out = nullptr;
  if (hipSetDevice(device) != hipSuccess) return ORBGPU_ERR_DEVICE;
  auto* c = new (std::nothrow) orbgpu_lba_ctx();
  if (!c) return ORBGPU_ERR_NOMEM;
  c->device = device;
  void* hw = nullptr;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipHostMalloc(&hw, sizeof(LbaHostWords), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
    orbgpu_lba_ctx_destroy(c);
    return ORBGPU_ERR_DEVICE;
  }
  c->host = static_cast<LbaHostWords*>(hw);
  std::memset(c->host, 0, sizeof(LbaHostWords));
  void* dp = nullptr;
  if (hipHostGetDevicePointer(&dp, hw, 0) != hipSuccess) {
    orbgpu_lba_ctx_destroy(c);
    return ORBGPU_ERR_DEVICE;
  }
  c->host_dev = static_cast<LbaHostWords*>(dp);
  *out = c;
  return ORBGPU_OK;
}

void orbgpu_lba_ctx_destroy(orbgpu_lba_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

orbgpu_status orbgpu_lba_optimize(orbgpu_lba_ctx* h, const orbgpu_camera* cam, int n_kf,
                                  const orbgpu_pose* poses_in, const uint8_t* fixed, int n_pts,
                                  const float* pts_in, int n_edges, const orbgpu_lba_edge* edges,
                                  int pt_begin, int pt_end, int iterations, double lambda_init,
                                  const volatile uint8_t* stop_flag, orbgpu_lba_reduce_fn reduce,
                                  void* user, orbgpu_pose* poses_out, double* poses_out_d,
                                  float* pts_out, uint8_t* outlier, double* stats) {
  if (!h || !cam || n_kf <= 0 || !poses_in || !fixed || n_pts < 0 || n_edges < 0 ||
      (n_edges > 0 && !edges) || (n_pts > 0 && !pts_in) || pt_begin < 0 || pt_end > n_pts ||
      pt_begin > pt_end || iterations < 0 || !poses_out || (pt_end > pt_begin && !pts_out) ||
      (n_edges > 0 && !outlier) || (!reduce && (pt_begin != 0 || pt_end != n_pts)))
    return ORBGPU_ERR_INVALID;
  if (hipSetDevice(h->device) != hipSuccess) return ORBGPU_ERR_DEVICE;
  hipStream_t st = h->stream;

  // ---- graph layout of this shard, O(edges): free-pose indices, point-major
  // edges (insertion order kept inside a point), per-pose edge lists, pairs
  std::vector<int> hidx(n_kf, -1);
  int nf = 0;
  for (int k = 0; k < n_kf; ++k)
    if (!fixed[k]) hidx[k] = nf++;
  const int n = 6 * nf;
  const int npad = (n + 15) / 16 * 16;
  if (npad > 2048) return ORBGPU_ERR_INVALID;  // reduced system beyond the solver's LDS vectors
  const int np = pt_end - pt_begin;
  std::vector<int> cnt(np + 1, 0);
  for (int i = 0; i < n_edges; ++i) {
    const orbgpu_lba_edge& e = edges[i];
    if (e.point < 0 || e.point >= n_pts || e.kf < 0 || e.kf >= n_kf) return ORBGPU_ERR_INVALID;
    if (e.point >= pt_begin && e.point < pt_end) ++cnt[e.point - pt_begin + 1];
  }
  int n_edgeless = 0;
  for (int p = 0; p < np; ++p) {
    n_edgeless += cnt[p + 1] == 0;
    cnt[p + 1] += cnt[p];
  }
  const int ne = cnt[np];
  const int n_pairs = nf * (nf + 1) / 2;
  std::vector<int> gidx(ne);  // shard edge -> caller's edge index
  std::vector<int> pose_cnt(nf + 1, 0);

  // ---- sizes: upload | download | compute
  const size_t K7 = 7 * (size_t)n_kf, P3 = 3 * (size_t)std::max(np, 1);
  const size_t E = std::max(ne, 1), P = std::max(np, 1), F = std::max(nf, 1);
  const int nblk = (int)((std::max(std::max(ne, np), 1) + 255) / 256) + nf + 1;
  const size_t n_ints = 4 * E + (size_t)n_kf + (np + 1) + (nf + 1) + E + 2 * (size_t)std::max(n_pairs, 1);
  size_t up = 0;
  const size_t u_ctrl = up;
  up += 128;
  const size_t u_cnt = up;
  up += 128;
  const size_t u_edges = up;
  up = align_up(up + sizeof(LbaEdgeDev) * E, 256);
  const size_t u_ints = up;
  up = align_up(up + sizeof(int) * n_ints, 256);
  const size_t u_state = up;
  up = align_up(up + sizeof(double) * (2 * K7 + 2 * P3), 256);
  const size_t d_begin = up;  // download: ctrl copy | poses | pts | outlier
  size_t dn = 128;
  const size_t d_out = dn;
  dn += sizeof(double) * (K7 + P3);
  const size_t d_outlier = dn;
  dn = align_up(dn + E, 256);
  size_t cz = align_up(d_begin + dn, 256);
  auto take = [&](size_t doubles) {
    const size_t o = cz;
    cz = align_up(cz + sizeof(double) * doubles, 256);
    return o;
  };
  const bool solve_lds = lba_solve_lds_bytes(npad) <= kLdsBudget;
  const size_t c_err = take(3 * E), c_hpl = take(18 * E), c_hppe = take(27 * E), c_hlle = take(12 * E),
               c_hll = take(9 * P), c_bl = take(3 * P), c_hpp = take(36 * F), c_bp = take(6 * F),
               c_diag = take(n + 2), c_sys = take((size_t)n * n + 2 * n + 2),
               c_work = take(solve_lds ? 2 : (size_t)npad * (npad + 1) + (size_t)(npad / 16) * 256),
               c_xp = take(n + 2), c_red = take(4), c_scal = take(2), c_part = take(3 * (size_t)nblk);
  if (!h->reserve(cz, std::max(up, dn))) return ORBGPU_ERR_NOMEM;

  // ---- fill the upload image in pinned memory
  char* U = h->staging;
  LbaCtrl ctrl0{};
  ctrl0.ni = 2;
  ctrl0.user_lambda = lambda_init;
  ctrl0.max_iters = iterations;
  ctrl0.need_build = 1;
  std::memcpy(U + u_ctrl, &ctrl0, sizeof(ctrl0));
  std::memset(U + u_cnt, 0, 128);
  auto* le = reinterpret_cast<LbaEdgeDev*>(U + u_edges);
  {
    std::vector<int> fill(cnt.begin(), cnt.end() - 1);
    for (int i = 0; i < n_edges; ++i) {
      const orbgpu_lba_edge& e = edges[i];
      if (e.point < pt_begin || e.point >= pt_end) continue;
      const int j = fill[e.point - pt_begin]++;
      le[j] = LbaEdgeDev{e.point - pt_begin, e.kf, hidx[e.kf], 0, e.u, e.v, e.ur, e.inv_sigma2};
      gidx[j] = i;
      if (hidx[e.kf] >= 0) ++pose_cnt[hidx[e.kf] + 1];
    }
  }
  int* I = reinterpret_cast<int*>(U + u_ints);
  int* I_slot = I;  // int4 records first (16-B aligned)
  int* I_hidx = I_slot + 4 * E;
  int* I_pt = I_hidx + n_kf;
  int* I_pb = I_pt + (np + 1);
  int* I_ef = I_pb + (nf + 1);
  int* I_pi = I_ef + E;
  int* I_pj = I_pi + std::max(n_pairs, 1);
  std::copy(hidx.begin(), hidx.end(), I_hidx);
  std::copy(cnt.begin(), cnt.end(), I_pt);
  for (int f = 0; f < nf; ++f) pose_cnt[f + 1] += pose_cnt[f];
  std::copy(pose_cnt.begin(), pose_cnt.end(), I_pb);
  {
    std::vector<int> fill(pose_cnt.begin(), pose_cnt.end() - 1);
    for (int j = 0; j < ne; ++j) {
      I_ef[j] = le[j].f;
      if (le[j].f < 0) continue;
      int* r = I_slot + 4 * (size_t)fill[le[j].f]++;
      const int p = le[j].point;
      r[0] = j;
      r[1] = p;
      r[2] = cnt[p];
      r[3] = cnt[p + 1];
    }
  }
  for (int i = 0, k = 0; i < nf; ++i)
    for (int j = i; j < nf; ++j, ++k) {
      I_pi[k] = i;
      I_pj[k] = j;
    }
  auto* S0 = reinterpret_cast<double*>(U + u_state);
  for (int k = 0; k < n_kf; ++k) {
    const orbgpu_pose& q = poses_in[k];
    const double v[7] = {q.qx, q.qy, q.qz, q.qw, q.tx, q.ty, q.tz};
    for (int c = 0; c < 7; ++c) S0[7 * (size_t)k + c] = S0[K7 + 7 * (size_t)k + c] = v[c];
  }
  double* X0 = S0 + 2 * K7;
  for (int p = 0; p < np; ++p)
    for (int c = 0; c < 3; ++c)
      X0[3 * (size_t)p + c] = X0[P3 + 3 * (size_t)p + c] = pts_in[3 * (size_t)(pt_begin + p) + c];
  if (hipMemcpyAsync(h->arena, U, up, hipMemcpyHostToDevice, st) != hipSuccess)
    return ORBGPU_ERR_DEVICE;

  // ---- device argument block
  char* A = h->arena;
  auto dp = [&](size_t off) { return reinterpret_cast<double*>(A + off); };
  LbaArgs a{};
  a.cam = LbaCamDev{cam->fx, cam->fy, cam->cx, cam->cy, cam->bf};
  a.n_kf = n_kf;
  a.n_pts = np;
  a.n_edges = ne;
  a.n_free = nf;
  a.n_sys = n;
  a.n_pairs = n_pairs;
  a.sharded = reduce ? 1 : 0;
  a.solve_lds = solve_lds ? 1 : 0;
  a.n_pad = npad;
  a.n_edgeless = n_edgeless;
  a.edges = reinterpret_cast<const LbaEdgeDev*>(A + u_edges);
  const int* dI = reinterpret_cast<const int*>(A + u_ints);
  a.hidx = dI + (I_hidx - I);
  a.pt_begin = dI + (I_pt - I);
  a.pose_begin = dI + (I_pb - I);
  a.pslot = reinterpret_cast<const int4*>(dI + (I_slot - I));
  a.ef = dI + (I_ef - I);
  a.pair_i = dI + (I_pi - I);
  a.pair_j = dI + (I_pj - I);
  a.poses[0] = dp(u_state);
  a.poses[1] = dp(u_state) + K7;
  a.pts[0] = dp(u_state) + 2 * K7;
  a.pts[1] = dp(u_state) + 2 * K7 + P3;
  a.err = dp(c_err);
  a.hpl = dp(c_hpl);
  a.hpp_e = dp(c_hppe);
  a.hll_e = dp(c_hlle);
  a.hll = dp(c_hll);
  a.bl = dp(c_bl);
  a.hpp = dp(c_hpp);
  a.bp = dp(c_bp);
  a.diag = dp(c_diag);
  a.sys = dp(c_sys);
  a.work = dp(c_work);
  a.xp = dp(c_xp);
  a.red = dp(c_red);
  a.scal = dp(c_scal);
  a.partials = dp(c_part);
  a.counter = reinterpret_cast<unsigned*>(A + u_cnt);
  a.ctrl = reinterpret_cast<LbaCtrl*>(A + u_ctrl);
  a.host = h->host_dev;

  volatile LbaHostWords* hw = h->host;
  hw->progress = 0;
  hw->stop = (stop_flag && *stop_flag) ? 1u : 0u;
  if (lba_begin(a, st) != hipSuccess) return ORBGPU_ERR_DEVICE;

  if (!reduce) {
    // ---- the device runs the LM loop; keep kAhead steps queued
    const int max_steps = iterations * 10;  // every iteration ends within 10 trials
    int issued = 0;
    while (issued < max_steps) {
      const unsigned long long p = hw->progress;
      if (p >> 32) break;
      if (stop_flag) hw->stop = *stop_flag ? 1u : 0u;
      if (issued - (int)(p & 0xffffffffu) < kAhead) {
        if (lba_step(a, st) != hipSuccess) return ORBGPU_ERR_DEVICE;
        ++issued;
      } else {
        std::this_thread::yield();
      }
    }
  } else {
    // ---- point-sharded: the host completes every reduction
    auto red = [&](double* buf, int cnt_, int op) -> bool {
      if (hipStreamSynchronize(st) != hipSuccess) return false;
      return reduce(user, buf, cnt_, op, reinterpret_cast<void*>(st)) == 0;
    };
    auto read_ctrl = [&](LbaCtrl& c) {
      return hipMemcpyAsync(&c, a.ctrl, sizeof(LbaCtrl), hipMemcpyDeviceToHost, st) == hipSuccess &&
             hipStreamSynchronize(st) == hipSuccess;
    };
    if (!red(a.red, 2, 0) || lba_ctl(a, kCtlInit, st) != hipSuccess) return ORBGPU_ERR_DEVICE;
    for (int guard = 0; guard < iterations * 10 + 1; ++guard) {
      LbaCtrl c;
      if (!read_ctrl(c)) return ORBGPU_ERR_DEVICE;
      if (c.done) break;
      if (c.need_build) {
        if (lba_build(a, st) != hipSuccess) return ORBGPU_ERR_DEVICE;
        if (c.it == 0 && (!red(a.diag, n, 0) || !red(a.diag + n, 1, 1) ||
                          lba_ctl(a, kCtlLambda, st) != hipSuccess))
          return ORBGPU_ERR_DEVICE;
      }
      if (stop_flag) hw->stop = *stop_flag ? 1u : 0u;
      if (lba_schur(a, st) != hipSuccess || !red(a.sys, n * n + 2 * n, 0) ||
          lba_solve_trial(a, st) != hipSuccess || !red(a.red, 4, 0) ||
          lba_ctl(a, kCtlDecide, st) != hipSuccess)
        return ORBGPU_ERR_DEVICE;
    }
  }

  // ---- outliers, final state, one copy back
  char* D = A + d_begin;
  if (hipMemcpyAsync(D, a.ctrl, sizeof(LbaCtrl), hipMemcpyDeviceToDevice, st) != hipSuccess ||
      lba_classify(a, reinterpret_cast<uint8_t*>(D + d_outlier), reinterpret_cast<double*>(D + d_out), st) !=
          hipSuccess ||
      hipMemcpyAsync(h->staging, D, dn, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return ORBGPU_ERR_DEVICE;
  LbaCtrl c;
  std::memcpy(&c, h->staging, sizeof(c));
  const auto* out = reinterpret_cast<const double*>(h->staging + d_out);
  const auto* lo = reinterpret_cast<const uint8_t*>(h->staging + d_outlier);
  int n_out = 0;
  for (int j = 0; j < ne; ++j) {
    outlier[gidx[j]] = lo[j];
    n_out += lo[j];
  }
  for (int k = 0; k < n_kf; ++k) {
    const double* v = out + 7 * (size_t)k;
    if (poses_out_d)
      for (int q = 0; q < 7; ++q) poses_out_d[7 * k + q] = v[q];
    // Sophus::SE3f(rotation().cast<float>(), translation().cast<float>())
    float f[7];
    for (int q = 0; q < 7; ++q) f[q] = (float)v[q];
    const float qn = std::sqrt(f[0] * f[0] + f[1] * f[1] + f[2] * f[2] + f[3] * f[3]);
    for (int q = 0; q < 4; ++q) f[q] /= qn;
    poses_out[k] = orbgpu_pose{f[0], f[1], f[2], f[3], f[4], f[5], f[6]};
  }
  const double* xo = out + K7;
  for (int p = 0; p < np; ++p)
    for (int q = 0; q < 3; ++q) pts_out[3 * (size_t)(pt_begin + p) + q] = (float)xo[3 * (size_t)p + q];
  if (stats) {
    stats[0] = c.chi_init;
    stats[1] = c.cur;
    stats[2] = c.iters_done;
    stats[3] = c.trials;
    stats[4] = c.lambda;
    stats[5] = n_out;
  }
  return ORBGPU_OK;
}

}  // extern "C"
