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
#include <numeric>
#include <chrono>
#include <climits>
#include <cstdio>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <new>
#include <thread>
#include <vector>

#include "../../include/orbgpu.h"
#include "lba_launch.h"

static_assert(ORBGPU_LBA_SOLVER_LDS == orbgpu::kSolveLds && ORBGPU_LBA_SOLVER_BLOCK == orbgpu::kSolveBlock &&
                  ORBGPU_LBA_SOLVER_GRID == orbgpu::kSolveGrid,
              "solver path ids");

using namespace orbgpu;

namespace {

// host phase clocks of run_window (tools/lba_host_bench.cpp builds with
// LBA_HOST_PHASES); nothing otherwise
#ifdef LBA_HOST_PHASES
double g_host_phase_us[16];
std::chrono::steady_clock::time_point g_host_phase_t;
#define LBA_HOST_PHASE(k)                                                                    \
  do {                                                                                       \
    const auto now_ = std::chrono::steady_clock::now();                                      \
    if ((k) > 0)                                                                             \
      g_host_phase_us[k] += std::chrono::duration<double, std::micro>(now_ - g_host_phase_t).count(); \
    g_host_phase_t = now_;                                                                   \
  } while (0)
#else
#define LBA_HOST_PHASE(k) \
  do {                    \
  } while (0)
#endif

constexpr int kAhead = 2;  // LM steps queued ahead of the device

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

}  // namespace

struct orbgpu_lba_ctx {
  int device = 0;
  int reduce_ordered = 0;  // orbgpu_lba_ctx_set_reduce_ordered
  int solver = ORBGPU_LBA_SOLVER_AUTO;  // orbgpu_lba_ctx_set_solver
  int schur = ORBGPU_LBA_SCHUR_SPLIT;   // orbgpu_lba_ctx_set_schur (default: ORBGPU_SCHUR at creation)
  int relinearize = 0;                  // orbgpu_lba_ctx_set_relinearize (default: ORBGPU_LBA_RELINEARIZE)
  size_t mem_limit = 0;                 // orbgpu_lba_ctx_set_memory_limit (0: none)
  hipStream_t stream = nullptr;
  char* arena = nullptr;  // device
  size_t arena_cap = 0;
  char* staging = nullptr;  // pinned host
  size_t staging_cap = 0;
  LbaHostWords* host = nullptr;  // pinned, mapped, coherent
  LbaHostWords* host_dev = nullptr;
  char* res = nullptr;  // pinned, mapped, coherent: a one-rank call's results (LbaArgs::res_*)
  char* res_dev = nullptr;
  size_t res_cap = 0;
  uint32_t calls = 0;
  ~orbgpu_lba_ctx() {
    if (arena) (void)hipFree(arena);
    if (staging) (void)hipHostFree(staging);
    if (host) (void)hipHostFree(host);
    if (res) (void)hipHostFree(res);
  }
  // The previous call may have left no-op LM steps queued on `stream` that
  // still read the arena and write the results block: they drain before either
  // buffer is replaced (explicitly -- not by relying on hipFree's implicit
  // synchronisation).
  bool reserve_results(size_t bytes) {
    if (bytes <= res_cap) return true;
    if (hipStreamSynchronize(stream) != hipSuccess) return false;
    if (res) (void)hipHostFree(res);
    res = res_dev = nullptr;
    res_cap = 0;
    void* dp = nullptr;
    if (hipHostMalloc(reinterpret_cast<void**>(&res), bytes, hipHostMallocMapped | hipHostMallocCoherent) !=
            hipSuccess ||
        hipHostGetDevicePointer(&dp, res, 0) != hipSuccess)
      return false;
    res_dev = static_cast<char*>(dp);
    res_cap = bytes;
    return true;
  }
  bool reserve(size_t dev_bytes, size_t host_bytes) {
    if (mem_limit && dev_bytes > mem_limit) return false;  // ORBGPU_ERR_NOMEM, nothing touched
    if ((dev_bytes > arena_cap || host_bytes > staging_cap) && hipStreamSynchronize(stream) != hipSuccess)
      return false;
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
  // A/B defaults for tools (read once here, never per call): ORBGPU_SCHUR =
  // split | pair | band, ORBGPU_LBA_RELINEARIZE set -> re-linearise every build
  if (const char* e = std::getenv("ORBGPU_SCHUR"))
    c->schur = std::strcmp(e, "pair") == 0 ? ORBGPU_LBA_SCHUR_PAIR
               : std::strcmp(e, "band") == 0 ? ORBGPU_LBA_SCHUR_BAND
                                             : ORBGPU_LBA_SCHUR_SPLIT;
  c->relinearize = std::getenv("ORBGPU_LBA_RELINEARIZE") != nullptr ? 1 : 0;
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

orbgpu_status orbgpu_lba_ctx_set_reduce_ordered(orbgpu_lba_ctx* c, int ordered) {
  if (!c) return ORBGPU_ERR_INVALID;
  c->reduce_ordered = ordered ? 1 : 0;
  return ORBGPU_OK;
}

orbgpu_status orbgpu_lba_ctx_set_schur(orbgpu_lba_ctx* c, int mode) {
  if (!c || mode < ORBGPU_LBA_SCHUR_SPLIT || mode > ORBGPU_LBA_SCHUR_BAND) return ORBGPU_ERR_INVALID;
  c->schur = mode;
  return ORBGPU_OK;
}

orbgpu_status orbgpu_lba_ctx_set_memory_limit(orbgpu_lba_ctx* c, size_t bytes) {
  if (!c) return ORBGPU_ERR_INVALID;
  c->mem_limit = bytes;
  return ORBGPU_OK;
}

orbgpu_status orbgpu_lba_ctx_set_relinearize(orbgpu_lba_ctx* c, int on) {
  if (!c) return ORBGPU_ERR_INVALID;
  c->relinearize = on ? 1 : 0;
  return ORBGPU_OK;
}

orbgpu_status orbgpu_lba_ctx_set_solver(orbgpu_lba_ctx* c, int solver) {
  if (!c || solver < ORBGPU_LBA_SOLVER_AUTO || solver > ORBGPU_LBA_SOLVER_GRID) return ORBGPU_ERR_INVALID;
  c->solver = solver;
  return ORBGPU_OK;
}

void orbgpu_lba_ctx_destroy(orbgpu_lba_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

}  // extern "C"

namespace {

// What distinguishes the two windows the context solves: the key-frame model
// and, for LocalInertialBA, the IMU links and the close flags.
struct ModelIn {
  int model = kModelSe3;
  int pdim = 6;
  int pstride = 7;
  const double* state0 = nullptr;  // [pstride * n_kf] initial key-frame states
  LiaCalibDev icb{};
  const uint8_t* close = nullptr;  // [n_pts]
  int n_imu = 0;
  const orbgpu_lia_imu_edge* imu = nullptr;
};

struct WindowOut {
  LbaCtrl ctrl;
  std::vector<double> state;  // [pstride * n_kf]
  int n_out = 0;
};

// The point-major Schur layout (LbaArgs::sc_*, k_lba_schur_band): the
// shard's points with a free edge ordered by their lowest free pose (a stable
// counting sort), cut greedily into chunks whose free poses span at most
// kSchurBandMax poses and whose W_all + H_all (64 bytes x points x padded band
// rows) fit kSchurChunkLds.  O(points + edges); ok = false (the pair kernel)
// when one point alone spans a wider band.
struct SchurChunks {
  std::vector<int> order, tile0{0};
  std::vector<int4> chunk;
  bool ok = false;
};

void build_schur_chunks(int np, int nf, const std::vector<int>& cnt, const std::vector<int>& pf,
                        SchurChunks& sc) {
  if (nf == 0) return;
  std::vector<int> lo(np, -1), hi(np, -1), start(nf + 1, 0);
  for (int p = 0; p < np; ++p) {
    for (int u = cnt[p]; u < cnt[p + 1]; ++u)
      if (pf[u] >= 0) {
        lo[p] = lo[p] < 0 ? pf[u] : std::min(lo[p], pf[u]);
        hi[p] = std::max(hi[p], pf[u]);
      }
    if (lo[p] >= 0) {
      if (hi[p] - lo[p] + 1 > kSchurBandMax) return;
      ++start[lo[p] + 1];
    }
  }
  for (int f = 0; f < nf; ++f) start[f + 1] += start[f];
  sc.order.resize(start[nf]);
  for (int p = 0; p < np; ++p)
    if (lo[p] >= 0) sc.order[start[lo[p]]++] = p;
  for (size_t i = 0; i < sc.order.size();) {
    const int b0 = lo[sc.order[i]];
    int top = hi[sc.order[i]];
    size_t j = i + 1;
    for (; j < sc.order.size(); ++j) {
      const int t = std::max(top, hi[sc.order[j]]);
      if (t - b0 + 1 > kSchurBandMax || 64 * (int)(j - i + 1) * schur_band_rows(t - b0 + 1) > kSchurChunkLds)
        break;
      top = t;
    }
    const int w = top - b0 + 1, T = schur_band_rows(w) / 16;
    sc.chunk.push_back(make_int4((int)i, (int)(j - i), b0, w));
    sc.tile0.push_back(sc.tile0.back() + T * (T + 1) / 2);
    i = j;
  }
  sc.ok = true;
}

// The shared body of orbgpu_lba_optimize / orbgpu_lia_optimize: layout,
// one upload, the device LM loop (or the host-in-the-loop sharded form), the
// outlier classification and one download.
orbgpu_status run_window(orbgpu_lba_ctx* h, const orbgpu_camera* cam, int n_kf, const uint8_t* fixed,
                         int n_pts, const float* pts_in, int n_edges, const orbgpu_lba_edge* edges,
                         int pt_begin, int pt_end, int iterations, double lambda_init,
                         const volatile uint8_t* stop_flag, orbgpu_lba_reduce_fn reduce, void* user,
                         const ModelIn& m, float* pts_out, uint8_t* outlier, WindowOut& wo) {
  if (hipSetDevice(h->device) != hipSuccess) return ORBGPU_ERR_DEVICE;
  hipStream_t st = h->stream;
  const bool imu = m.model == kModelImu;
  // ORBGPU_LBA_TRACE=1: host phase times of the call to stderr (tools/)
  static const bool trace = std::getenv("ORBGPU_LBA_TRACE") != nullptr;
  using clk = std::chrono::steady_clock;
  const auto t_enter = clk::now();
  auto us = [](clk::time_point a, clk::time_point b) {
    return std::chrono::duration<double, std::micro>(b - a).count();
  };
  int trace_steps = 0;

  LBA_HOST_PHASE(0);
  // ---- graph layout of this shard, O(edges): free-pose indices, point-major
  // edges (insertion order kept inside a point), per-pose edge lists, pairs
  std::vector<int> hidx(n_kf, -1), free_kf;
  int nf = 0;
  for (int k = 0; k < n_kf; ++k)
    if (!fixed[k]) {
      hidx[k] = nf++;
      free_kf.push_back(k);
    }
  if ((long long)m.pdim * nf > INT_MAX / 2) return ORBGPU_ERR_CAPACITY;  // row indices are int
  const int n = m.pdim * nf;
  const int npad = (n + 15) / 16 * 16;
  // a sharded rank all-reduces [S | b_s | b_p] through an int-counted callback
  if (reduce && (size_t)n * n + 2 * (size_t)n > (size_t)INT_MAX) return ORBGPU_ERR_CAPACITY;
  const int np = pt_end - pt_begin;
  std::vector<int> cnt(np + 1, 0);
  // point-major input (the reference adds a point's edges together, points in
  // turn: optimizer.cc:1187-1262) needs no scatter below: the shard's edges
  // are then the contiguous run after the i_lo edges of lower points
  bool sorted = true;
  int prev_pt = 0, i_lo = 0;
  for (int i = 0; i < n_edges; ++i) {
    const orbgpu_lba_edge& e = edges[i];
    if (e.point < 0 || e.point >= n_pts || e.kf < 0 || e.kf >= n_kf) return ORBGPU_ERR_INVALID;
    sorted &= e.point >= prev_pt;
    prev_pt = e.point;
    i_lo += e.point < pt_begin;
    if (e.point >= pt_begin && e.point < pt_end) ++cnt[e.point - pt_begin + 1];
  }
  int n_edgeless = 0;
  for (int p = 0; p < np; ++p) {
    n_edgeless += cnt[p + 1] == 0;
    cnt[p + 1] += cnt[p];
  }
  const int ne = cnt[np];
  // the structurally non-zero pose pairs of S: every diagonal block, and (i, j)
  // when some point of the shard is seen by both (the other blocks stay the
  // zeros the per-call clear leaves; a sharded rank's zeros add nothing)
  LBA_HOST_PHASE(1);
  std::vector<int> pair_list;
  std::vector<int> pose_cnt(nf + 1, 0);  // free-pose edges per pose (then its CSR)
  // point-major order: perm[j] = the caller's index of shard edge j (one
  // scatter of indices, then sequential gathers), pf[j] its free-pose index
  std::vector<int> perm(std::max(ne, 1)), pf(std::max(ne, 1));  // pf: -1 = fixed pose
  {
    if (sorted) {
      std::iota(perm.begin(), perm.begin() + ne, i_lo);
    } else {
      std::vector<int> fill(cnt.begin(), cnt.end() - 1);
      for (int i = 0; i < n_edges; ++i) {
        const int p = edges[i].point;
        if (p >= pt_begin && p < pt_end) perm[fill[p - pt_begin]++] = i;
      }
    }
  LBA_HOST_PHASE(2);
    auto add_pair = [&](int i, int j) {
      pair_list.push_back(i);
      pair_list.push_back(j);
    };
    // one walk in point order: each edge's free-pose index, the per-pose edge
    // counts and (nf <= 64) a point's free poses as one bit mask, OR-ed into
    // each of its poses' rows
    const bool masks = nf <= 64;
    std::vector<uint64_t> rows(masks ? nf : 0);
    for (int f = 0; f < (int)rows.size(); ++f) rows[f] = 1ull << f;
    for (int p = 0; p < np; ++p) {
      uint64_t msk = 0;
      for (int u = cnt[p]; u < cnt[p + 1]; ++u) {
        const int f = hidx[edges[perm[u]].kf];
        pf[u] = f;
        if (f >= 0) {
          ++pose_cnt[f + 1];
          msk |= 1ull << (f & 63);
        }
      }
      if (masks)
        for (int u = cnt[p]; u < cnt[p + 1]; ++u)
          if (pf[u] >= 0) rows[pf[u]] |= msk;
    }
    if (masks) {
      for (int i = 0; i < nf; ++i)
        for (int j = i; j < nf; ++j)
          if ((rows[i] >> j) & 1) add_pair(i, j);
    } else {
      std::vector<uint8_t> nz((size_t)nf * nf, 0);
      for (int f = 0; f < nf; ++f) nz[(size_t)f * nf + f] = 1;
      for (int p = 0; p < np; ++p)
        for (int u = cnt[p]; u < cnt[p + 1]; ++u)
          for (int v = u + 1; v < cnt[p + 1]; ++v) {
            const int fa = pf[u], fb = pf[v];
            if (fa >= 0 && fb >= 0) nz[(size_t)std::min(fa, fb) * nf + std::max(fa, fb)] = 1;
          }
      for (int i = 0; i < nf; ++i)
        for (int j = i; j < nf; ++j)
          if (nz[(size_t)i * nf + j]) add_pair(i, j);
    }
  }
  LBA_HOST_PHASE(3);
  const int n_pairs = (int)pair_list.size() / 2;
  // Schur path: point ranges (k_lba_schur_split), S of them so that a
  // (pair, range) block gets about kSchurSplitEdges of its pose's edges.
  // orbgpu_lba_ctx_set_schur picks a path for A/B runs and tests.
  const int n_free_edges = std::accumulate(pose_cnt.begin(), pose_cnt.end(), 0);
  int sc_split = nf > 0 ? (n_free_edges + nf * kSchurSplitEdges - 1) / (nf * kSchurSplitEdges) : 0;
  sc_split = std::min(std::max(sc_split, 1), kSchurSplitMax);
  SchurChunks sc;
  if (h->schur != ORBGPU_LBA_SCHUR_SPLIT) sc_split = 0;
  if (h->schur == ORBGPU_LBA_SCHUR_BAND) build_schur_chunks(np, nf, cnt, pf, sc);
  if (nf == 0 || n_pairs == 0) sc_split = 0;
  // range x = points [pbx[x], pbx[x + 1]), cut at about x ne / S edges
  std::vector<int> pbx(sc_split + 1, np);
  for (int x = 0; x < sc_split; ++x)
    pbx[x] = (int)(std::lower_bound(cnt.begin(), cnt.end() - 1, (int)((long long)x * ne / sc_split)) - cnt.begin());
  LBA_HOST_PHASE(4);
  const std::vector<int>& gidx = perm;  // shard edge -> caller's edge index
  // IMU links incident to each free key frame (link order), one record each:
  // {link, the key frame's side (0: kf1), the other key frame's free index
  // (-1: fixed), its side}
  std::vector<int> inc(nf + 1, 0), inc_list;
  if (imu) {
    std::vector<std::vector<int>> lists(nf);
    for (int l = 0; l < m.n_imu; ++l)
      for (int k : {m.imu[l].kf1, m.imu[l].kf2})
        if (hidx[k] >= 0) lists[hidx[k]].push_back(l);
    for (int f = 0; f < nf; ++f) {
      inc[f + 1] = inc[f] + (int)lists[f].size();
      for (int l : lists[f]) {
        const int sr = hidx[m.imu[l].kf1] == f ? 0 : 1;
        inc_list.insert(inc_list.end(), {l, sr, hidx[sr ? m.imu[l].kf1 : m.imu[l].kf2], 1 - sr});
      }
    }
  }

  LBA_HOST_PHASE(5);
  // ---- sizes: upload | download | compute
  const size_t KS = (size_t)m.pstride * n_kf, P3 = 3 * (size_t)std::max(np, 1);
  const size_t E = std::max(ne, 1), P = std::max(np, 1), F = std::max(nf, 1);
  const size_t NI = std::max(m.n_imu, 1);
  // blocks of the widest grid that writes a.partials (k_lba_sums with, for
  // kModelImu, its link-assembly blocks)
  const long nblk = (std::max(std::max(ne, np), 1) + 255) / 256 + kSumsQ * (long)nf + 1 +
                    (imu ? ((long)n * n + n + 255) / 256 + m.n_imu : 0);  // (+ the trial's link blocks)
  const size_t n_ints = (size_t)n_kf + (np + 1) + (nf + 1) + E + 2 * (size_t)std::max(n_pairs, 1) +
                        F + (nf + 1) + std::max(inc_list.size(), (size_t)4) + E;
  // the Schur chunk layout (ints): chunk table (int4 first), tile offsets, point order
  const size_t n_sc = (sc.ok ? 4 * sc.chunk.size() + sc.tile0.size() + sc.order.size() : 1) +
                      (size_t)nf * (sc_split + 1);
  size_t up = 0;
  const size_t u_ctrl = up;
  up += 128;
  const size_t u_cnt = up;
  up += 128;
  const size_t u_edges = up;
  up = align_up(up + sizeof(LbaEdgeDev) * E, 256);
  const size_t u_ints = up;
  up = align_up(up + sizeof(int) * n_ints, 256);
  const size_t u_sc = up;
  up = align_up(up + sizeof(int) * n_sc, 256);
  const size_t u_pcnt = up;  // per-pair tickets of k_lba_schur_split (zero)
  up = align_up(up + sizeof(unsigned) * (size_t)std::max(n_pairs, 1), 256);
  const size_t u_state = up;
  up = align_up(up + sizeof(double) * (2 * KS + 2 * P3), 256);
  const size_t u_imu = up;
  if (imu) up = align_up(up + sizeof(LiaImuDev) * NI, 256);
  const size_t u_close = up;
  if (imu) up = align_up(up + P, 256);
  const size_t d_begin = up;  // download: ctrl copy | states | pts | outlier
  size_t dn = 128;
  const size_t d_out = dn;
  dn += sizeof(double) * (KS + P3);
  const size_t d_outlier = dn;
  dn = align_up(dn + E, 256);
  size_t cz = align_up(d_begin + dn, 256);
  auto take = [&](size_t doubles) {
    const size_t o = cz;
    cz = align_up(cz + sizeof(double) * doubles, 256);
    return o;
  };
  int solve_mode = lba_solve_mode(npad);
  if (h->solver != ORBGPU_LBA_SOLVER_AUTO) {  // a forced path must hold the window
    if (!lba_solve_mode_fits(h->solver, npad)) return ORBGPU_ERR_CAPACITY;
    solve_mode = h->solver;
  }
  const size_t c_err = take(3 * E), c_hpl = take(2 * 18 * E), c_hppe = take(2 * 27 * E), c_hlle = take(2 * 12 * E),
               c_hll = take(9 * P), c_bl = take(3 * P), c_hpp = take(36 * F), c_bp = take(6 * F),
               c_diag = take(n + 2), c_sys = take((size_t)n * n + 2 * n + 2),
               c_work = take(lba_solve_work_doubles(solve_mode, npad)),
               c_xp = take(n + 2), c_red = take(4), c_scal = take(2), c_part = take(3 * (size_t)nblk),
               c_imuq = take(imu ? 2 * kImuPairQ * NI : 1), c_himu = take(imu ? (size_t)n * n + n : 1),
               c_itot = take(2 + NI),  // [2 + l] per link
               c_ppart = take(27 * (size_t)kSumsQ * F),
               c_pslot = take(2 * E),  // int4 slot records, device-built (k_lba_begin)
               c_scp = take(std::max(sc.ok ? 256 * (size_t)sc.tile0.back() : 1,
                                     sc_split > 1 ? 42 * (size_t)n_pairs * sc_split : 1));
  LBA_HOST_PHASE(6);
  if (!h->reserve(cz, std::max(up, dn)) || (!reduce && !h->reserve_results(dn))) return ORBGPU_ERR_NOMEM;

  // ---- fill the upload image in pinned memory
  char* U = h->staging;
  LbaCtrl ctrl0{};
  ctrl0.ni = 2;
  ctrl0.user_lambda = lambda_init;
  ctrl0.max_iters = iterations;
  ctrl0.need_build = 1;
  ctrl0.lin_state = -1;
  ctrl0.call = (int)(++h->calls & 0x7fffffffu);
  std::memcpy(U + u_ctrl, &ctrl0, sizeof(ctrl0));
  std::memset(U + u_cnt, 0, 128);
  std::memset(U + u_pcnt, 0, sizeof(unsigned) * (size_t)std::max(n_pairs, 1));
  auto* le = reinterpret_cast<LbaEdgeDev*>(U + u_edges);
  for (int j = 0; j < ne; ++j) {  // one sequential store stream into the pinned image
    const orbgpu_lba_edge& e = edges[perm[j]];
    le[j] = LbaEdgeDev{e.point - pt_begin, e.kf, pf[j], 0, e.u, e.v, e.ur, e.inv_sigma2};
  }
  LBA_HOST_PHASE(7);
  // the image's head (control words, the edge records) goes up now, its DMA
  // under the host's remaining layout work; the rest after it
  if (hipMemcpyAsync(h->arena, U, u_ints, hipMemcpyHostToDevice, st) != hipSuccess) return ORBGPU_ERR_DEVICE;
  int* I = reinterpret_cast<int*>(U + u_ints);
  int* I_incl = I;  // int4 link records first (16-B aligned)
  int* I_hidx = I_incl + std::max(inc_list.size(), (size_t)4);
  int* I_pt = I_hidx + n_kf;
  int* I_pb = I_pt + (np + 1);
  int* I_ef = I_pb + (nf + 1);
  int* I_pi = I_ef + E;
  int* I_pj = I_pi + std::max(n_pairs, 1);
  int* I_fk = I_pj + std::max(n_pairs, 1);
  int* I_inc = I_fk + F;
  int* I_es = I_inc + (nf + 1);
  std::copy(hidx.begin(), hidx.end(), I_hidx);
  std::copy(cnt.begin(), cnt.end(), I_pt);
  for (int f = 0; f < nf; ++f) pose_cnt[f + 1] += pose_cnt[f];
  std::copy(pose_cnt.begin(), pose_cnt.end(), I_pb);
  // one walk in point order (host-side arrays only: nothing is read back from
  // pinned memory): each edge's pose slot (k_lba_begin builds the slot
  // records from it) and (k_lba_schur_split) per free pose the slot where
  // each point range starts
  // (slots are in point order within a pose).  The edge image and the free-
  // pose indices go in sequential passes of their own: interleaving them here
  // measured slower (layout 87 -> 113 µs), the pinned image taking several
  // store streams at once
  std::copy(pf.begin(), pf.begin() + ne, I_ef);
  int* const SC = reinterpret_cast<int*>(U + u_sc);
  int* const SP = SC + (sc.ok ? 4 * sc.chunk.size() + sc.tile0.size() + sc.order.size() : 1);
  {
    std::vector<int> fill(pose_cnt.begin(), pose_cnt.end() - 1);
    int x = 0;
    const int S1 = sc_split + 1;
    auto range_starts = [&](int p) {  // range x starts at point pbx[x]
      while (x <= sc_split && pbx[x] <= p) {
        for (int f = 0; f < nf; ++f) SP[(size_t)f * S1 + x] = fill[f];
        ++x;
      }
    };
    for (int p = 0; p < np; ++p) {
      if (sc_split > 0) range_starts(p);
      for (int j = cnt[p]; j < cnt[p + 1]; ++j) {
        const int f = pf[j];
        if (f < 0) {
          I_es[j] = -1;
          continue;
        }
        I_es[j] = fill[f]++;  // (k_lba_begin writes slot I_es[j]'s record)
      }
    }
    if (sc_split > 0) range_starts(np);
  }
  for (int k = 0; k < n_pairs; ++k) {
    I_pi[k] = pair_list[2 * k];
    I_pj[k] = pair_list[2 * k + 1];
  }
  std::copy(free_kf.begin(), free_kf.end(), I_fk);
  std::copy(inc.begin(), inc.end(), I_inc);
  std::copy(inc_list.begin(), inc_list.end(), I_incl);
  LBA_HOST_PHASE(8);
  if (sc.ok) {
    std::memcpy(SC, sc.chunk.data(), sizeof(int4) * sc.chunk.size());
    std::memcpy(SC + 4 * sc.chunk.size(), sc.tile0.data(), sizeof(int) * sc.tile0.size());
    std::memcpy(SC + 4 * sc.chunk.size() + sc.tile0.size(), sc.order.data(), sizeof(int) * sc.order.size());
  }
  LBA_HOST_PHASE(9);
  auto* S0 = reinterpret_cast<double*>(U + u_state);
  std::copy(m.state0, m.state0 + KS, S0);
  std::copy(m.state0, m.state0 + KS, S0 + KS);
  double* X0 = S0 + 2 * KS;
  for (int p = 0; p < np; ++p)
    for (int c = 0; c < 3; ++c)
      X0[3 * (size_t)p + c] = X0[P3 + 3 * (size_t)p + c] = pts_in[3 * (size_t)(pt_begin + p) + c];
  if (imu) {
    std::memcpy(U + u_imu, m.imu, sizeof(LiaImuDev) * m.n_imu);
    std::memcpy(U + u_close, m.close + pt_begin, np);
  }
  LBA_HOST_PHASE(10);
  const auto t_layout = clk::now();
  if (hipMemcpyAsync(h->arena + u_ints, U + u_ints, up - u_ints, hipMemcpyHostToDevice, st) != hipSuccess)
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
  a.sc_split = sc_split;
  // the build re-linearises every iteration instead of taking the accepted
  // trial's terms (same values; tests/test_gpu_lba.py compares the two)
  a.force_lin = h->relinearize;
  a.pose_split = reinterpret_cast<const int*>(A + u_sc) + (SP - SC);
  a.pair_cnt = reinterpret_cast<unsigned*>(A + u_pcnt);
  // each pair's ranges folded by the pair's last range block (a per-pair
  // ticket over write-through partials: one launch fewer a step; with an
  // agent-scope release per block this measured slower, 17.9 µs against 8.7
  // + 4.8 at C4); ORBGPU_SCHUR_FOLD=launch: by k_lba_schur_fold (A/B)
  static const bool fold_inline = [] {
    const char* e = std::getenv("ORBGPU_SCHUR_FOLD");
    return !(e && std::strcmp(e, "launch") == 0);
  }();
  a.sc_fold_inline = fold_inline ? 1 : 0;
  if (sc_split > 1) a.sc_part = dp(c_scp);
  if (sc.ok) {
    const int* dS = reinterpret_cast<const int*>(A + u_sc);
    a.n_chunks = (int)sc.chunk.size();
    a.sc_chunk = reinterpret_cast<const int4*>(dS);
    a.sc_tile0 = dS + 4 * sc.chunk.size();
    a.sc_order = dS + 4 * sc.chunk.size() + sc.tile0.size();
    a.sc_part = dp(c_scp);
  }
  a.sharded = reduce ? 1 : 0;
  a.solve_mode = solve_mode;
  a.n_pad = npad;
  a.n_edgeless = n_edgeless;
  a.edges = reinterpret_cast<const LbaEdgeDev*>(A + u_edges);
  const int* dI = reinterpret_cast<const int*>(A + u_ints);
  a.hidx = dI + (I_hidx - I);
  a.pt_begin = dI + (I_pt - I);
  a.pose_begin = dI + (I_pb - I);
  a.pslot = reinterpret_cast<const int4*>(A + c_pslot);
  a.ef = dI + (I_ef - I);
  a.pair_i = dI + (I_pi - I);
  a.pair_j = dI + (I_pj - I);
  a.eslot = dI + (I_es - I);
  a.n_slots = nf > 0 ? pose_cnt[nf] : 0;
  a.poses[0] = dp(u_state);
  a.poses[1] = dp(u_state) + KS;
  a.pts[0] = dp(u_state) + 2 * KS;
  a.pts[1] = dp(u_state) + 2 * KS + P3;
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
  a.pose_part = dp(c_ppart);
  a.counter = reinterpret_cast<unsigned*>(A + u_cnt);
  a.ctrl = reinterpret_cast<LbaCtrl*>(A + u_ctrl);
  a.host = h->host_dev;
  a.early_out = reduce ? 0 : 1;
  if (!reduce) {  // the results' layout is the download block's (d_*)
    a.res_ctrl = reinterpret_cast<uint32_t*>(h->res_dev);
    a.res_out = reinterpret_cast<double*>(h->res_dev + d_out);
    a.res_outlier = reinterpret_cast<uint8_t*>(h->res_dev + d_outlier);
  }
  a.model = m.model;
  a.pdim = m.pdim;
  a.pstride = m.pstride;
  if (imu) {
    a.icb = m.icb;
    a.close = reinterpret_cast<const uint8_t*>(A + u_close);
    a.n_imu = m.n_imu;
    a.imu = reinterpret_cast<const LiaImuDev*>(A + u_imu);
    a.free_kf = dI + (I_fk - I);
    a.imu_inc = dI + (I_inc - I);
    a.imu_inc_rec = reinterpret_cast<const int4*>(dI + (I_incl - I));
    a.imu_q = dp(c_imuq);
    a.himu = dp(c_himu);
    a.imu_tot = dp(c_itot);
  }

  volatile LbaHostWords* hw = h->host;
  hw->progress = 0;
  hw->stop = (stop_flag && *stop_flag) ? 1u : 0u;
  if (lba_begin(a, st) != hipSuccess) return ORBGPU_ERR_DEVICE;

  // one-rank: whether a step was queued behind the one that ended the LM
  // (its k_lba_sums then writes the results to host memory)
  bool step_after_end = false;
  if (!reduce) {
    // ---- the device runs the LM loop; keep kAhead steps queued
    const int max_steps = iterations * 10;  // every iteration ends within 10 trials
    int issued = 0;
    while (issued < max_steps) {
      const unsigned long long p = hw->progress;
      if (p >> 32) {
        step_after_end = issued > (int)(p & 0xffffffffu);
        break;
      }
      if (stop_flag) hw->stop = *stop_flag ? 1u : 0u;
      if (issued - (int)(p & 0xffffffffu) < kAhead) {
        if (lba_step(a, st, a.force_lin) != hipSuccess) return ORBGPU_ERR_DEVICE;  // (state 0: k_lba_begin)
        ++issued;
        trace_steps = issued;
      } else {
        std::this_thread::yield();
      }
    }
  } else if (h->reduce_ordered) {
    // ---- point-sharded, LM on the device: every reduction is enqueued on
    // the stream between the stage kernels (no host synchronisation); the
    // kernels and k_lba_ctl skip what is not due (need_build, lambda_due,
    // done), so a step is the same kernel + collective sequence on every
    // rank.  The host keeps kAhead steps queued like the one-rank path and,
    // once the device reports done at trial j, tops the queue up to exactly
    // j + kAhead - 1 steps: it can have issued at most that many (it issues
    // step s only after seeing s - kAhead complete), and every rank issuing
    // the same number keeps the collectives matched.
    auto red = [&](double* buf, int cnt_, int op) {
      return reduce(user, buf, cnt_, op, reinterpret_cast<void*>(st)) == 0;
    };
    auto issue = [&]() {
      return lba_build(a, st) == hipSuccess && red(a.diag, n, 0) && red(a.diag + n, 1, 1) &&
             lba_ctl(a, kCtlLambda, st) == hipSuccess && lba_schur(a, st) == hipSuccess &&
             red(a.sys, n * n + 2 * n, 0) && lba_solve_trial(a, st) == hipSuccess && red(a.red, 4, 0) &&
             lba_ctl(a, kCtlDecide, st) == hipSuccess;
    };
    if (!red(a.red, 2, 0) || lba_ctl(a, kCtlInit, st) != hipSuccess) return ORBGPU_ERR_DEVICE;
    const int max_steps = iterations * 10;
    int issued = 0;
    while (issued < max_steps) {
      const unsigned long long p = hw->progress;
      if (p >> 32) {
        const int target = std::min(max_steps, (int)(p & 0xffffffffu) + kAhead - 1);
        while (issued < target) {
          if (!issue()) return ORBGPU_ERR_DEVICE;
          ++issued;
        }
        break;
      }
      if (stop_flag) hw->stop = *stop_flag ? 1u : 0u;
      if (issued - (int)(p & 0xffffffffu) < kAhead) {
        if (!issue()) return ORBGPU_ERR_DEVICE;
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

  // ---- outliers, final state
  const auto t_loop = clk::now();
  const char* R = nullptr;
  if (!reduce) {
    // one rank: the results arrive in host memory, written by the step queued
    // behind the LM's end or else by one launch now; the host returns as soon
    // as they are complete (the queued no-op kernels drain on the stream)
    if (!step_after_end && lba_classify_to_host(a, st) != hipSuccess) return ORBGPU_ERR_DEVICE;
    const uint32_t want = (uint32_t)ctrl0.call;
    for (unsigned spin = 0; __atomic_load_n(&hw->results, __ATOMIC_ACQUIRE) != want; ++spin) {
      if ((spin & 63u) == 63u) {  // a failed or drained stream without the results
        const hipError_t q = hipStreamQuery(st);
        if (q != hipSuccess && q != hipErrorNotReady) return ORBGPU_ERR_DEVICE;
        if (q == hipSuccess && __atomic_load_n(&hw->results, __ATOMIC_ACQUIRE) != want) return ORBGPU_ERR_DEVICE;
      }
      std::this_thread::yield();
    }
    R = h->res;
  } else {
    char* D = A + d_begin;
    if (lba_classify(a, reinterpret_cast<uint8_t*>(D + d_outlier), reinterpret_cast<double*>(D + d_out), D, st) !=
            hipSuccess ||
        hipMemcpyAsync(h->staging, D, dn, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
      return ORBGPU_ERR_DEVICE;
    R = h->staging;
  }
  std::memcpy(&wo.ctrl, R, sizeof(LbaCtrl));
  const auto* out = reinterpret_cast<const double*>(R + d_out);
  const auto* lo = reinterpret_cast<const uint8_t*>(R + d_outlier);
  wo.n_out = 0;
  for (int j = 0; j < ne; ++j) {
    outlier[gidx[j]] = lo[j];
    wo.n_out += lo[j];
  }
  wo.state.assign(out, out + KS);
  const double* xo = out + KS;
  for (int p = 0; p < np; ++p)
    for (int q = 0; q < 3; ++q) pts_out[3 * (size_t)(pt_begin + p) + q] = (float)xo[3 * (size_t)p + q];
  if (trace) {
    const auto t_end = clk::now();
    std::fprintf(stderr, "{\"lba_trace\": 1, \"layout_us\": %.1f, \"loop_us\": %.1f, \"tail_us\": %.1f, "
                 "\"steps_issued\": %d, \"trials\": %d, \"edges\": %d, \"pairs\": %d, \"sc_split\": %d}\n",
                 us(t_enter, t_layout), us(t_layout, t_loop), us(t_loop, t_end), trace_steps, wo.ctrl.trials, ne,
                 n_pairs, sc_split);
  }
  return ORBGPU_OK;
}

}  // namespace

extern "C" {

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
  std::vector<double> s0(7 * (size_t)n_kf);
  for (int k = 0; k < n_kf; ++k) {
    const orbgpu_pose& q = poses_in[k];
    const double v[7] = {q.qx, q.qy, q.qz, q.qw, q.tx, q.ty, q.tz};
    std::copy(v, v + 7, s0.begin() + 7 * (size_t)k);
  }
  ModelIn m;
  m.state0 = s0.data();
  WindowOut wo;
  const orbgpu_status r = run_window(h, cam, n_kf, fixed, n_pts, pts_in, n_edges, edges, pt_begin, pt_end,
                                     iterations, lambda_init, stop_flag, reduce, user, m, pts_out, outlier, wo);
  if (r != ORBGPU_OK) return r;
  for (int k = 0; k < n_kf; ++k) {
    const double* v = wo.state.data() + 7 * (size_t)k;
    if (poses_out_d)
      for (int q = 0; q < 7; ++q) poses_out_d[7 * k + q] = v[q];
    // Sophus::SE3f(rotation().cast<float>(), translation().cast<float>())
    float f[7];
    for (int q = 0; q < 7; ++q) f[q] = (float)v[q];
    const float qn = std::sqrt(f[0] * f[0] + f[1] * f[1] + f[2] * f[2] + f[3] * f[3]);
    for (int q = 0; q < 4; ++q) f[q] /= qn;
    poses_out[k] = orbgpu_pose{f[0], f[1], f[2], f[3], f[4], f[5], f[6]};
  }
  if (stats) {
    stats[0] = wo.ctrl.chi_init;
    stats[1] = wo.ctrl.cur;
    stats[2] = wo.ctrl.iters_done;
    stats[3] = wo.ctrl.trials;
    stats[4] = wo.ctrl.lambda;
    stats[5] = wo.n_out;
  }
  return ORBGPU_OK;
}

orbgpu_status orbgpu_lia_optimize(orbgpu_lba_ctx* h, const orbgpu_imu_calib* calib, int n_kf,
                                  const orbgpu_imu_state* kfs, const uint8_t* fixed,
                                  const uint8_t* imu, int n_pts, const float* pts_in,
                                  const uint8_t* close, int n_edges, const orbgpu_lba_edge* edges,
                                  int n_imu, const orbgpu_lia_imu_edge* imu_edges, int iterations,
                                  double lambda_init, orbgpu_imu_state* kfs_out, double* kfs_out_d,
                                  float* pts_out, uint8_t* outlier, double* stats) {
  if (!h || !calib || n_kf <= 0 || !kfs || !fixed || !imu || n_pts < 0 || n_edges < 0 ||
      (n_edges > 0 && !edges) || (n_pts > 0 && (!pts_in || !pts_out || !close)) || n_imu < 0 ||
      (n_imu > 0 && !imu_edges) || iterations < 0 || !(lambda_init > 0) || !kfs_out ||
      (n_edges > 0 && !outlier))
    return ORBGPU_ERR_INVALID;
  for (int l = 0; l < n_imu; ++l) {
    const orbgpu_lia_imu_edge& e = imu_edges[l];
    if (e.kf1 < 0 || e.kf1 >= n_kf || e.kf2 < 0 || e.kf2 >= n_kf || e.kf1 == e.kf2 || !imu[e.kf1] ||
        !imu[e.kf2])
      return ORBGPU_ERR_INVALID;
  }
  // ImuCamPose(pKF): Rwb, twb, Rcw, tcw (the float pose), and the vertex estimates
  std::vector<double> s0(kImuStateStride * (size_t)n_kf);
  for (int k = 0; k < n_kf; ++k) {
    const orbgpu_imu_state& g = kfs[k];
    double* d = s0.data() + kImuStateStride * (size_t)k;
    for (int i = 0; i < 9; ++i) {
      d[i] = g.Rwb[i];
      d[12 + i] = g.Rcw[i];
    }
    for (int i = 0; i < 3; ++i) {
      d[9 + i] = g.twb[i];
      d[21 + i] = g.tcw[i];
      d[24 + i] = g.v[i];
      d[27 + i] = g.bg[i];
      d[30 + i] = g.ba[i];
    }
  }
  ModelIn m;
  m.model = kModelImu;
  m.pdim = kImuDim;
  m.pstride = kImuStateStride;
  m.state0 = s0.data();
  m.icb = LiaCalibDev{calib->fx, calib->fy, calib->cx, calib->cy, calib->bf, {}, {}, {}, {}};
  for (int i = 0; i < 9; ++i) {
    m.icb.Rcb[i] = calib->Rcb[i];
    m.icb.Rbc[i] = calib->Rbc[i];
  }
  for (int i = 0; i < 3; ++i) {
    m.icb.tcb[i] = calib->tcb[i];
    m.icb.tbc[i] = calib->tbc[i];
  }
  m.close = close;
  m.n_imu = n_imu;
  m.imu = imu_edges;
  const orbgpu_camera cam{calib->fx, calib->fy, calib->cx, calib->cy, calib->bf};
  WindowOut wo;
  // *pbStopFlag is attached after optimize() (optimizer.cc:2794): no stop flag
  const orbgpu_status r = run_window(h, &cam, n_kf, fixed, n_pts, pts_in, n_edges, edges, 0, n_pts, iterations,
                                     lambda_init, nullptr, nullptr, nullptr, m, pts_out, outlier, wo);
  if (r != ORBGPU_OK) return r;
  for (int k = 0; k < n_kf; ++k) {
    const double* d = wo.state.data() + kImuStateStride * (size_t)k;
    orbgpu_imu_state& o = kfs_out[k];
    for (int i = 0; i < 9; ++i) {
      o.Rwb[i] = (float)d[i];
      o.Rcw[i] = (float)d[12 + i];
    }
    for (int i = 0; i < 3; ++i) {
      o.twb[i] = (float)d[9 + i];
      o.tcw[i] = (float)d[21 + i];
      o.v[i] = (float)d[24 + i];
      o.bg[i] = (float)d[27 + i];
      o.ba[i] = (float)d[30 + i];
    }
    if (kfs_out_d) {
      double* q = kfs_out_d + 21 * (size_t)k;
      std::copy(d, d + 12, q);            // Rwb, twb
      std::copy(d + 24, d + 33, q + 12);  // v, bg, ba
    }
  }
  if (stats) {
    stats[0] = wo.ctrl.chi_init;
    stats[1] = wo.ctrl.last;
    stats[2] = wo.ctrl.iters_done;
    stats[3] = wo.ctrl.trials;
    stats[4] = wo.ctrl.lambda;
    stats[5] = wo.n_out;
    stats[6] = wo.ctrl.cur;
  }
  return ORBGPU_OK;
}

}  // extern "C"
