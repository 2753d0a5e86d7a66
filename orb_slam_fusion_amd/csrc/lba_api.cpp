// C-ABI implementation of the LocalBundleAdjustment half of include/orbgpu.h:
// graph layout on the host (the reference builds its g2o graph on the host
// too, optimizer.cc:1127-1354), the g2o Levenberg-Marquardt loop
// (core/optimization_algorithm_levenberg.cpp:59-168) on the host, every
// linearisation / Schur / solve / update on the GPU (lba_kernels.hip).
// The loop is step for step the one in oracle/lba_oracle.cc, including the
// two reduce points a point-sharded multi-GPU run completes with RCCL.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <new>
#include <utility>
#include <vector>

#include "../../include/orbgpu.h"
#include "lba_launch.h"

using namespace orbgpu;

static_assert(sizeof(orbgpu_lba_edge) == sizeof(LbaEdgeDev), "orbgpu_lba_edge layout");

namespace {

template <typename T>
struct DevVec {
  T* p = nullptr;
  size_t cap = 0;
  bool reserve(size_t n) {
    if (n <= cap) return true;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    if (hipMalloc(&p, sizeof(T) * std::max<size_t>(n, 1)) != hipSuccess) return false;
    cap = std::max<size_t>(n, 1);
    return true;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

}  // namespace

struct orbgpu_lba_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  DevVec<LbaEdgeDev> edges;
  DevVec<int> ints;  // pt_begin | hidx | pose_begin | pose_edges | pair_i | pair_j | pair_begin | pair_ei | pair_ej
  DevVec<double> dbl;
  DevVec<double> state;  // poses[2], points[2]
  DevVec<unsigned> counter;
  DevVec<int> flags;
  DevVec<uint8_t> outlier;
  ~orbgpu_lba_ctx() {
    edges.release();
    ints.release();
    dbl.release();
    state.release();
    counter.release();
    flags.release();
    outlier.release();
  }
};

namespace {

bool check(hipError_t e) { return e == hipSuccess; }

}  // namespace

extern "C" {

orbgpu_status orbgpu_lba_ctx_create(int device, orbgpu_lba_ctx** out) {
  if (!out) return ORBGPU_ERR_INVALID;
  *out = nullptr;
  if (hipSetDevice(device) != hipSuccess) return ORBGPU_ERR_DEVICE;
  auto* c = new (std::nothrow) orbgpu_lba_ctx();
  if (!c) return ORBGPU_ERR_NOMEM;
  c->device = device;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      !c->counter.reserve(1) || !c->flags.reserve(1) ||
      hipMemset(c->counter.p, 0, sizeof(unsigned)) != hipSuccess) {
    orbgpu_lba_ctx_destroy(c);
    return ORBGPU_ERR_DEVICE;
  }
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
                                  int pt_begin, int pt_end, int iterations,
                                  const volatile uint8_t* stop_flag, orbgpu_lba_reduce_fn reduce,
                                  void* user, orbgpu_pose* poses_out, double* poses_out_d,
                                  float* pts_out, uint8_t* outlier, double* stats) {
  if (!h || !cam || n_kf <= 0 || !poses_in || !fixed || n_pts < 0 || n_edges < 0 ||
      (n_edges > 0 && !edges) || (n_pts > 0 && !pts_in) || pt_begin < 0 || pt_end > n_pts ||
      pt_begin > pt_end || iterations < 0 || !poses_out || (pt_end > pt_begin && !pts_out) ||
      (n_edges > 0 && !outlier))
    return ORBGPU_ERR_INVALID;
  if (hipSetDevice(h->device) != hipSuccess) return ORBGPU_ERR_DEVICE;
  hipStream_t st = h->stream;

  // ---- graph layout (this shard): free-pose indices, point-major edges,
  // pose lists and Schur pair lists
  std::vector<int> hidx(n_kf, -1);
  int nf = 0;
  for (int k = 0; k < n_kf; ++k)
    if (!fixed[k]) hidx[k] = nf++;
  const int n = 6 * nf;
  const int np = pt_end - pt_begin;
  std::vector<int> cnt(np + 1, 0);
  for (int i = 0; i < n_edges; ++i) {
    const orbgpu_lba_edge& e = edges[i];
    if (e.point < 0 || e.point >= n_pts || e.kf < 0 || e.kf >= n_kf) return ORBGPU_ERR_INVALID;
    if (e.point >= pt_begin && e.point < pt_end) ++cnt[e.point - pt_begin + 1];
  }
  for (int p = 0; p < np; ++p) cnt[p + 1] += cnt[p];
  const int ne = cnt[np];
  std::vector<LbaEdgeDev> le(ne);
  std::vector<int> gidx(ne);  // local edge -> caller's edge index
  {
    std::vector<int> fill(cnt.begin(), cnt.end() - 1);
    for (int i = 0; i < n_edges; ++i) {
      const orbgpu_lba_edge& e = edges[i];
      if (e.point < pt_begin || e.point >= pt_end) continue;
      const int j = fill[e.point - pt_begin]++;
      le[j] = LbaEdgeDev{e.point - pt_begin, e.kf, e.u, e.v, e.ur, e.inv_sigma2};
      gidx[j] = i;
    }
  }
  std::vector<int> pose_begin(nf + 1, 0), pose_edges;
  for (int j = 0; j < ne; ++j)
    if (hidx[le[j].kf] >= 0) ++pose_begin[hidx[le[j].kf] + 1];
  for (int f = 0; f < nf; ++f) pose_begin[f + 1] += pose_begin[f];
  pose_edges.resize(pose_begin[nf]);
  {
    std::vector<int> fill(pose_begin.begin(), pose_begin.end() - 1);
    for (int j = 0; j < ne; ++j)
      if (hidx[le[j].kf] >= 0) pose_edges[fill[hidx[le[j].kf]]++] = j;
  }
  // (fi <= fj) pair entries of every point, grouped by pair, point order kept
  std::vector<std::pair<long, std::pair<int, int>>> ent;
  for (int p = 0; p < np; ++p)
    for (int a = cnt[p]; a < cnt[p + 1]; ++a)
      for (int b = cnt[p]; b < cnt[p + 1]; ++b) {
        const int fa = hidx[le[a].kf], fb = hidx[le[b].kf];
        if (fa < 0 || fb < 0 || fa > fb) continue;
        if (fa == fb && a != b) continue;
        ent.push_back({(long)fa * nf + fb, {a, b}});
      }
  std::stable_sort(ent.begin(), ent.end(),
                   [](const auto& x, const auto& y) { return x.first < y.first; });
  std::vector<int> pair_i, pair_j, pair_begin, pair_ei(ent.size()), pair_ej(ent.size());
  for (size_t k = 0; k < ent.size(); ++k) {
    if (k == 0 || ent[k].first != ent[k - 1].first) {
      pair_i.push_back((int)(ent[k].first / nf));
      pair_j.push_back((int)(ent[k].first % nf));
      pair_begin.push_back((int)k);
    }
    pair_ei[k] = ent[k].second.first;
    pair_ej[k] = ent[k].second.second;
  }
  pair_begin.push_back((int)ent.size());
  const int n_pairs = (int)pair_i.size();

  // ---- device buffers
  std::vector<int> ints;
  auto put = [&](const std::vector<int>& v) {
    const size_t off = ints.size();
    ints.insert(ints.end(), v.begin(), v.end());
    return off;
  };
  const size_t o_pt = put(cnt), o_h = put(hidx), o_pb = put(pose_begin), o_pe = put(pose_edges),
               o_pi = put(pair_i), o_pj = put(pair_j), o_prb = put(pair_begin), o_ei = put(pair_ei),
               o_ej = put(pair_ej);
  const size_t E = std::max(ne, 1), P = std::max(np, 1), F = std::max(nf, 1);
  const size_t nblk = (std::max(ne, np) + 255) / 256 + 1;
  size_t dsz = 0;
  auto take = [&](size_t k) {
    const size_t o = dsz;
    dsz += (k + 1) & ~(size_t)1;
    return o;
  };
  const size_t d_err = take(3 * E), d_hpl = take(18 * E), d_hppe = take(27 * E),
               d_hlle = take(12 * E), d_hll = take(9 * P), d_bl = take(3 * P), d_dinv = take(9 * P),
               d_hpp = take(36 * F), d_bp = take(6 * F), d_diag = take(n + 2),
               d_sys = take((size_t)n * n + 2 * n + 2), d_work = take((size_t)n * n + 2),
               d_xp = take(n + 2), d_scal = take(4), d_part = take(nblk), d_out = take(2);
  if (!h->edges.reserve(E) || !h->ints.reserve(std::max<size_t>(ints.size(), 1)) ||
      !h->dbl.reserve(dsz) || !h->state.reserve(2 * 7 * (size_t)n_kf + 2 * 3 * P) ||
      !h->outlier.reserve(E))
    return ORBGPU_ERR_NOMEM;
  if (ne > 0 && !check(hipMemcpyAsync(h->edges.p, le.data(), sizeof(LbaEdgeDev) * ne,
                                      hipMemcpyHostToDevice, st)))
    return ORBGPU_ERR_DEVICE;
  if (!ints.empty() && !check(hipMemcpyAsync(h->ints.p, ints.data(), sizeof(int) * ints.size(),
                                             hipMemcpyHostToDevice, st)))
    return ORBGPU_ERR_DEVICE;
  double* D = h->dbl.p;
  double* poses[2] = {h->state.p, h->state.p + 7 * (size_t)n_kf};
  double* pts[2] = {h->state.p + 14 * (size_t)n_kf, h->state.p + 14 * (size_t)n_kf + 3 * P};
  {
    std::vector<double> hp(7 * (size_t)n_kf), hx(3 * P, 0.0);
    for (int k = 0; k < n_kf; ++k) {
      const orbgpu_pose& q = poses_in[k];
      const double v[7] = {q.qx, q.qy, q.qz, q.qw, q.tx, q.ty, q.tz};
      for (int a = 0; a < 7; ++a) hp[7 * (size_t)k + a] = v[a];
    }
    for (int p = 0; p < np; ++p)
      for (int a = 0; a < 3; ++a) hx[3 * (size_t)p + a] = pts_in[3 * (size_t)(pt_begin + p) + a];
    if (!check(hipMemcpyAsync(poses[0], hp.data(), sizeof(double) * hp.size(), hipMemcpyHostToDevice, st)) ||
        !check(hipMemcpyAsync(pts[0], hx.data(), sizeof(double) * hx.size(), hipMemcpyHostToDevice, st)))
      return ORBGPU_ERR_DEVICE;
  }

  LbaArgs a{};
  a.cam = LbaCamDev{cam->fx, cam->fy, cam->cx, cam->cy, cam->bf};
  a.n_kf = n_kf;
  a.n_pts = np;
  a.n_edges = ne;
  a.n_free = nf;
  a.n_sys = n;
  a.n_pairs = n_pairs;
  a.edges = h->edges.p;
  const int* I = h->ints.p;
  a.pt_begin = I + o_pt;
  a.hidx = I + o_h;
  a.pose_begin = I + o_pb;
  a.pose_edges = I + o_pe;
  a.pair_i = I + o_pi;
  a.pair_j = I + o_pj;
  a.pair_begin = I + o_prb;
  a.pair_ei = I + o_ei;
  a.pair_ej = I + o_ej;
  a.err = D + d_err;
  a.hpl = D + d_hpl;
  a.hpp_e = D + d_hppe;
  a.hll_e = D + d_hlle;
  a.hll = D + d_hll;
  a.bl = D + d_bl;
  a.dinv = D + d_dinv;
  a.hpp = D + d_hpp;
  a.bp = D + d_bp;
  a.diag = D + d_diag;
  a.sys = D + d_sys;
  a.work = D + d_work;
  a.xp = D + d_xp;
  a.scal = D + d_scal;
  a.partials = D + d_part;
  a.counter = h->counter.p;
  a.flags = h->flags.p;
  double* d_chi = D + d_out;

  // ---- g2o LM, as oracle/lba_oracle.cc
  auto red = [&](double* buf, int cnt_, int op) -> bool {
    if (!reduce) return true;
    if (hipStreamSynchronize(st) != hipSuccess) return false;
    return reduce(user, buf, cnt_, op, reinterpret_cast<void*>(st)) == 0;
  };
  auto fetch = [&](const double* src, double* dst, int k) {
    return check(hipMemcpyAsync(dst, src, sizeof(double) * k, hipMemcpyDeviceToHost, st)) &&
           check(hipStreamSynchronize(st));
  };
  int cur_state = 0;
  double cur = 0;
  if (!check(lba_errors(a, poses[0], pts[0], d_chi, st)) || !red(d_chi, 1, 0) || !fetch(d_chi, &cur, 1))
    return ORBGPU_ERR_DEVICE;
  const double chi_init = cur;
  const double tau = 1e-5;
  double lambda = 0, ni = 2;
  int nbad = 0, iters_done = 0, trials = 0;
  for (int it = 0; it < iterations; ++it) {
    if (stop_flag && *stop_flag) break;  // SparseOptimizer::terminate()
    const int s0 = cur_state;
    if (it > 0) {
      if (!check(lba_errors(a, poses[s0], pts[s0], d_chi, st)) || !red(d_chi, 1, 0) ||
          !fetch(d_chi, &cur, 1))
        return ORBGPU_ERR_DEVICE;
    }
    const double ini = cur;
    if (!check(hipMemsetAsync(a.diag, 0, sizeof(double) * (n + 1), st)) ||
        !check(lba_build(a, poses[s0], pts[s0], st)))
      return ORBGPU_ERR_DEVICE;
    if (it == 0) {  // computeLambdaInit
      std::vector<double> dg(n + 1);
      if (!red(a.diag, n, 0) || !red(a.diag + n, 1, 1) || !fetch(a.diag, dg.data(), n + 1))
        return ORBGPU_ERR_DEVICE;
      double mx = 0;
      for (int k = 0; k <= n; ++k) mx = std::max(std::fabs(dg[k]), mx);
      lambda = tau * mx;
      ni = 2;
      nbad = 0;
    }
    double rho = 0;
    int q = 0;
    do {
      ++trials;
      const int s1 = 1 - cur_state;
      if (!check(hipMemsetAsync(a.sys, 0, sizeof(double) * ((size_t)n * n + 2 * n), st)) ||
          !check(hipMemsetAsync(a.flags, 0, sizeof(int), st)) || !check(lba_schur(a, lambda, st)) ||
          !red(a.sys, n * n + 2 * n, 0) || !check(lba_solve(a, lambda, st)) ||
          !check(lba_trial(a, lambda, poses[s0], pts[s0], poses[s1], pts[s1], st)) ||
          !check(lba_errors(a, poses[s1], pts[s1], a.scal + 2, st)) || !red(a.scal + 1, 2, 0))
        return ORBGPU_ERR_DEVICE;
      double sc[3];
      int bad = 0;
      if (!check(hipMemcpyAsync(sc, a.scal, sizeof(sc), hipMemcpyDeviceToHost, st)) ||
          !check(hipMemcpyAsync(&bad, a.flags, sizeof(int), hipMemcpyDeviceToHost, st)) ||
          !check(hipStreamSynchronize(st)))
        return ORBGPU_ERR_DEVICE;
      double tmp = sc[2];
      if (bad) tmp = DBL_MAX;
      rho = cur - tmp;
      const double scale = sc[0] + sc[1] + 1e-3;
      rho /= scale;
      if (rho > 0 && std::isfinite(tmp)) {
        double alpha = 1. - std::pow(2 * rho - 1, 3);
        alpha = std::min(alpha, 2. / 3.);
        lambda *= std::max(1. / 3., alpha);
        ni = 2;
        cur = tmp;
        cur_state = s1;
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

  // ---- outliers and write-back
  std::vector<uint8_t> lo(ne);
  std::vector<double> hp(7 * (size_t)n_kf), hx(3 * P);
  if (!check(lba_classify(a, poses[cur_state], pts[cur_state], h->outlier.p, st)) ||
      (ne > 0 && !check(hipMemcpyAsync(lo.data(), h->outlier.p, ne, hipMemcpyDeviceToHost, st))) ||
      !check(hipMemcpyAsync(hp.data(), poses[cur_state], sizeof(double) * hp.size(), hipMemcpyDeviceToHost, st)) ||
      !check(hipMemcpyAsync(hx.data(), pts[cur_state], sizeof(double) * hx.size(), hipMemcpyDeviceToHost, st)) ||
      !check(hipStreamSynchronize(st)))
    return ORBGPU_ERR_DEVICE;
  int n_out = 0;
  for (int j = 0; j < ne; ++j) {
    outlier[gidx[j]] = lo[j];
    n_out += lo[j];
  }
  for (int k = 0; k < n_kf; ++k) {
    const double* v = &hp[7 * (size_t)k];
    if (poses_out_d)
      for (int c = 0; c < 7; ++c) poses_out_d[7 * k + c] = v[c];
    // Sophus::SE3f(rotation().cast<float>(), translation().cast<float>())
    float f[7];
    for (int c = 0; c < 7; ++c) f[c] = (float)v[c];
    const float qn = std::sqrt(f[0] * f[0] + f[1] * f[1] + f[2] * f[2] + f[3] * f[3]);
    for (int c = 0; c < 4; ++c) f[c] /= qn;
    poses_out[k] = orbgpu_pose{f[0], f[1], f[2], f[3], f[4], f[5], f[6]};
  }
  for (int p = 0; p < np; ++p)
    for (int c = 0; c < 3; ++c) pts_out[3 * (size_t)(pt_begin + p) + c] = (float)hx[3 * (size_t)p + c];
  if (stats) {
    stats[0] = chi_init;
    stats[1] = cur;
    stats[2] = iters_done;
    stats[3] = trials;
    stats[4] = lambda;
    stats[5] = n_out;
  }
  return ORBGPU_OK;
}

}  // extern "C"
