// C-ABI implementation of the ORBmatcher projection searches of
// include/orbgpu.h (kernels: match_kernels.hip).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstring>
#include <new>

#include "../../include/orbgpu.h"
#include "match_launch.h"

static_assert(sizeof(orbgpu_keypoint) == 28, "orbgpu_keypoint layout");
static_assert(sizeof(orbgpu_proj_point) == 56, "orbgpu_proj_point layout");
static_assert(sizeof(orbgpu_map_point) == 68, "orbgpu_map_point layout");
static_assert(sizeof(orbgpu_track_view) == 28, "orbgpu_track_view layout");
static_assert(sizeof(orbgpu_frame_geom) == 24 + 4 * ORBGPU_MAX_LEVELS, "orbgpu_frame_geom layout");

using orbgpu::kGridCells;
using orbgpu::MatchLaunch;

namespace {

// Device arena of one context: inputs of a host call (one upload), scratch
// and outputs (one download).
struct Arena {
  size_t bytes = 0;
  uint8_t* d = nullptr;
  uint8_t* h = nullptr;   // pinned staging, same size (the output arena: host-mapped)
  uint8_t* hd = nullptr;  // the device's address of h (mapped arenas)
  bool mapped = false;
};

size_t align_up(size_t v) { return (v + 255) & ~(size_t)255; }

}  // namespace

struct orbgpu_matcher {
  int device = 0;
  hipStream_t stream = nullptr;
  int max_kp = 0, max_pts = 0;
  Arena in, out;
  // device scratch for batches (grown on demand)
  int* d_cell_start = nullptr;
  uint16_t* d_cell_idx = nullptr;
  uint32_t* d_res = nullptr;
  int32_t* d_acc = nullptr;
  int* d_err = nullptr;
  size_t cap_cells = 0, cap_idx = 0, cap_res = 0, cap_acc = 0;
  // PredictScale threshold cache
  float thr_lsf = 0.0f;
  int thr_levels = -1;
  float thr[ORBGPU_MAX_LEVELS] = {};
  // one-frame calls: the completion word k_mt_resolve stores (host-mapped)
  int* h_done = nullptr;
  int* h_done_dev = nullptr;
  int seq = 0;
};

namespace {

template <class T>
int grow(T** p, size_t& cap, size_t n) {
  if (n <= cap) return 0;
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  cap = 0;
  if (hipMalloc(p, sizeof(T) * n) != hipSuccess) return -1;
  cap = n;
  return 0;
}

// MapPoint::PredictScale (mappoint.cc:550-563) as the reference computes it:
// nScale = ceil(::log((double)ratio) / (double)mfLogScaleFactor), clamped to
// [0, n_levels - 1].  The function is nondecreasing in the float ratio, so the
// level is the number of thresholds T_j = min{r : ceil(...) >= j}, j >= 1,
// that the ratio reaches; each T_j is found by bisection over positive float
// bit patterns with the host libm (the reference's).  +inf is level 0 (the
// reference converts a non-finite ceil through cvttsd2si = INT_MIN).
void level_thresholds(float lsf, int n_levels, float* thr) {
  auto reaches = [&](uint32_t bits, int j) {
    float r;
    std::memcpy(&r, &bits, 4);
    const double c = std::ceil(std::log((double)r) / (double)lsf);
    return c >= (double)j;
  };
  for (int j = 1; j < ORBGPU_MAX_LEVELS; ++j) {
    if (j >= n_levels) {
      thr[j - 1] = INFINITY;
      continue;
    }
    uint32_t lo = 1, hi = 0x7f800000u;  // reaches(hi) treated as true (+inf)
    if (!reaches(0x7f7fffffu, j)) {
      thr[j - 1] = INFINITY;
      continue;
    }
    while (lo < hi) {
      const uint32_t mid = lo + (hi - lo) / 2;
      if (reaches(mid, j)) hi = mid;
      else lo = mid + 1;
    }
    std::memcpy(&thr[j - 1], &lo, 4);
  }
}

orbgpu_status fill_params(orbgpu_matcher* m, const orbgpu_frame_geom* g, const orbgpu_camera* cam,
                          float mb, orbgpu::MatchParams& p) {
  if (!g || g->n_levels <= 0 || g->n_levels > ORBGPU_MAX_LEVELS || !(g->log_scale_factor > 0) ||
      !(g->max_x > g->min_x) || !(g->max_y > g->min_y))
    return ORBGPU_ERR_INVALID;
  std::memset(&p, 0, sizeof(p));
  p.min_x = g->min_x, p.max_x = g->max_x, p.min_y = g->min_y, p.max_y = g->max_y;
  p.inv_w = (float)orbgpu::kGridCols / (g->max_x - g->min_x);  // frame.cc:201-204
  p.inv_h = (float)orbgpu::kGridRows / (g->max_y - g->min_y);
  p.n_levels = g->n_levels;
  for (int l = 0; l < ORBGPU_MAX_LEVELS; ++l) p.scale[l] = g->scale_factors[l];
  if (m->thr_levels != g->n_levels || m->thr_lsf != g->log_scale_factor) {
    level_thresholds(g->log_scale_factor, g->n_levels, m->thr);
    m->thr_levels = g->n_levels;
    m->thr_lsf = g->log_scale_factor;
  }
  for (int l = 0; l < ORBGPU_MAX_LEVELS; ++l) p.level_thr[l] = m->thr[l];
  if (cam) p.fx = cam->fx, p.fy = cam->fy, p.cx = cam->cx, p.cy = cam->cy, p.bf = cam->bf;
  p.mb = mb;
  return ORBGPU_OK;
}

orbgpu_status ensure_scratch(orbgpu_matcher* m, int n_frames, int kp_stride, int pt_stride) {
  if (grow(&m->d_cell_start, m->cap_cells, (size_t)n_frames * (kGridCells + 1)) ||
      grow(&m->d_cell_idx, m->cap_idx, (size_t)n_frames * kp_stride) ||
      grow(&m->d_res, m->cap_res, (size_t)n_frames * pt_stride * orbgpu::kMatchResWords) ||
      grow(&m->d_acc, m->cap_acc, (size_t)n_frames * pt_stride))
    return ORBGPU_ERR_NOMEM;
  return ORBGPU_OK;
}

orbgpu_status arena_reserve(Arena& a, size_t bytes) {
  if (bytes <= a.bytes) return ORBGPU_OK;
  if (a.d) (void)hipFree(a.d);
  if (a.h) (void)hipHostFree(a.h);
  a.d = a.h = nullptr;
  a.bytes = 0;
  if (hipMalloc(&a.d, bytes) != hipSuccess ||
      hipHostMalloc(&a.h, bytes, a.mapped ? hipHostMallocMapped | hipHostMallocCoherent : 0) != hipSuccess ||
      (a.mapped && hipHostGetDevicePointer(reinterpret_cast<void**>(&a.hd), a.h, 0) != hipSuccess))
    return ORBGPU_ERR_NOMEM;
  a.bytes = bytes;
  return ORBGPU_OK;
}

// Bump allocator over an arena: same offsets on the host staging and device side.
struct Bump {
  Arena& a;
  size_t off = 0;
  template <class T>
  T* take(size_t n, T** host = nullptr) {
    const size_t o = off;
    off = align_up(off + sizeof(T) * n);
    if (host) *host = reinterpret_cast<T*>(a.h + o);
    return reinterpret_cast<T*>(a.d + o);
  }
};

size_t in_bytes(int n, int n_pts, size_t pt_size) {
  return align_up(sizeof(orbgpu_keypoint) * n) + align_up(32 * (size_t)n) + align_up(4 * (size_t)n) +
         align_up(n) + align_up(pt_size * n_pts) + align_up(sizeof(orbgpu_track_view) * n_pts) +
         align_up(4 * (size_t)n_pts) +
         align_up(2 * sizeof(orbgpu_pose)) + align_up(16 * sizeof(float)) + align_up(2 * sizeof(int)) +
         8 * 256;
}

size_t out_bytes(int n, int n_pts) {
  return align_up(sizeof(int)) + align_up(4 * (size_t)n) + align_up(sizeof(int)) +
         align_up(sizeof(orbgpu_track_view) * n_pts) + align_up(4 * (size_t)n_pts) + 4 * 256;
}

// One host-buffer call: stage inputs, launch, download outputs.
struct HostCall {
  orbgpu_matcher* m;
  MatchLaunch L{};
  Bump bi, bo;
  int* h_counts = nullptr;  // n, npts (staged)
  int32_t* d_match = nullptr;
  int* d_nm = nullptr;
  int* d_call_err = nullptr;  // this call's error word: offset 0 of `out`, read back with the outputs
  orbgpu_track_view* d_views_out = nullptr;
  explicit HostCall(orbgpu_matcher* m_) : m(m_), bi{m_->in}, bo{m_->out} {}
};

orbgpu_status stage_frame(HostCall& c, const orbgpu_keypoint* kps, const uint8_t* descs,
                          const float* uright, const uint8_t* claimed, int n, int n_pts) {
  orbgpu_matcher* m = c.m;
  orbgpu_keypoint* hk;
  uint8_t *hd, *hc;
  float* hu;
  c.L.kps = reinterpret_cast<const float*>(c.bi.take<orbgpu_keypoint>(n, &hk));
  c.L.desc = c.bi.take<uint8_t>(32 * (size_t)n, &hd);
  float* du = c.bi.take<float>(n, &hu);
  uint8_t* dc = c.bi.take<uint8_t>(n, &hc);
  if (n > 0) {
    std::memcpy(hk, kps, sizeof(orbgpu_keypoint) * n);
    std::memcpy(hd, descs, 32 * (size_t)n);
  }
  c.L.uright = uright ? du : nullptr;
  if (uright && n > 0) std::memcpy(hu, uright, 4 * (size_t)n);
  c.L.claimed = claimed ? dc : nullptr;
  if (claimed && n > 0) std::memcpy(hc, claimed, n);
  int* dcounts = c.bi.take<int>(2, &c.h_counts);
  c.h_counts[0] = n, c.h_counts[1] = n_pts;
  c.L.n = dcounts;
  c.L.npts = dcounts + 1;
  c.L.kp_stride = n > 0 ? n : 1;
  c.L.pt_stride = n_pts > 0 ? n_pts : 1;
  c.L.max_pts = n_pts;
  c.L.n_frames = 1;
  c.d_call_err = c.bo.take<int>(1);
  c.L.err = c.d_call_err;
  if (ensure_scratch(m, 1, c.L.kp_stride, c.L.pt_stride) != ORBGPU_OK) return ORBGPU_ERR_NOMEM;
  c.L.cell_start = m->d_cell_start;
  c.L.cell_idx = m->d_cell_idx;
  c.L.res = m->d_res;
  c.L.acc = m->d_acc;
  c.d_match = c.bo.take<int32_t>(n);
  c.d_nm = c.bo.take<int>(1);
  c.L.match = c.d_match;
  c.L.nmatches = c.d_nm;
  return ORBGPU_OK;
}

orbgpu_status run_host(HostCall& c, int n, int32_t* match, int* nmatches,
                       orbgpu_track_view* views_out, int n_pts) {
  orbgpu_matcher* m = c.m;
  hipStream_t s = m->stream;
  c.L.zero_err = 1;  // k_mt_grid writes the call's error word first (no memset)
  // outputs: the error word, match, nmatches (+ views) are contiguous at the
  // front of `out`; k_mt_resolve mirrors them into the host-mapped arena and
  // then stores the call's number into h_done
  const size_t dl = views_out ? (size_t)((uint8_t*)c.d_views_out - m->out.d) +
                                    sizeof(orbgpu_track_view) * n_pts
                              : (size_t)((uint8_t*)c.d_nm - m->out.d) + sizeof(int);
  const int seq = m->seq = m->seq == 0x7fffffff ? 1 : m->seq + 1;
  c.L.mirror_src = m->out.d;
  c.L.mirror_dst = m->out.hd;
  c.L.mirror_bytes = (int)dl;
  c.L.done_host = m->h_done_dev;
  c.L.seq = seq;
  if (hipMemcpyAsync(m->in.d, m->in.h, c.bi.off, hipMemcpyHostToDevice, s) ||
      orbgpu::launch_match(c.L, s) != hipSuccess)
    return ORBGPU_ERR_DEVICE;
  volatile int* done = m->h_done;
  bool seen = false;
  for (long spin = 0; spin < (1L << 24); ++spin) {
    if (*done == seq) {
      seen = true;
      break;
    }
    if ((spin & 4095) == 4095 && hipStreamQuery(s) != hipErrorNotReady) {
      seen = *done == seq;
      break;
    }
    __builtin_ia32_pause();
  }
  __atomic_thread_fence(__ATOMIC_ACQUIRE);
  if (!seen && (hipStreamSynchronize(s) != hipSuccess || *done != seq)) return ORBGPU_ERR_DEVICE;
  int err = 0;
  std::memcpy(&err, m->out.h + ((uint8_t*)c.d_call_err - m->out.d), sizeof(int));
  if (err) return ORBGPU_ERR_CAPACITY;
  if (n > 0) std::memcpy(match, m->out.h + ((uint8_t*)c.d_match - m->out.d), 4 * (size_t)n);
  std::memcpy(nmatches, m->out.h + ((uint8_t*)c.d_nm - m->out.d), sizeof(int));
  if (views_out && n_pts > 0)
    std::memcpy(views_out, m->out.h + ((uint8_t*)c.d_views_out - m->out.d),
                sizeof(orbgpu_track_view) * n_pts);
  return ORBGPU_OK;
}

bool bad_frame(const orbgpu_keypoint* kps, const uint8_t* descs, int n, const int32_t* match,
               const int* nmatches) {
  return n < 0 || n > orbgpu::kMatchMaxKeypoints || (n > 0 && (!kps || !descs || !match)) ||
         !nmatches;
}

}  // namespace

extern "C" {

orbgpu_status orbgpu_matcher_create(int device, int max_keypoints, int max_points,
                                    orbgpu_matcher** out) {
  if (!out || max_keypoints <= 0 || max_keypoints > orbgpu::kMatchMaxKeypoints || max_points <= 0 ||
      max_points > orbgpu::kMatchMaxPoints)
    return ORBGPU_ERR_INVALID;
  *out = nullptr;
  if (hipSetDevice(device) != hipSuccess) return ORBGPU_ERR_DEVICE;
  auto* m = new (std::nothrow) orbgpu_matcher();
  if (!m) return ORBGPU_ERR_NOMEM;
  m->device = device;
  m->max_kp = max_keypoints;
  m->max_pts = max_points;
  const size_t pt = sizeof(orbgpu_map_point);
  m->out.mapped = true;  // k_mt_resolve writes a one-frame call's outputs into it
  const unsigned hflags = hipHostMallocMapped | hipHostMallocCoherent;
  if (hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void**>(&m->h_done), 64, hflags) != hipSuccess ||
      hipHostGetDevicePointer(reinterpret_cast<void**>(&m->h_done_dev), m->h_done, 0) != hipSuccess ||
      hipMalloc(&m->d_err, sizeof(int)) != hipSuccess ||
      hipMemset(m->d_err, 0, sizeof(int)) != hipSuccess ||
      arena_reserve(m->in, in_bytes(max_keypoints, max_points, pt)) != ORBGPU_OK ||
      arena_reserve(m->out, out_bytes(max_keypoints, max_points)) != ORBGPU_OK ||
      ensure_scratch(m, 1, max_keypoints, max_points) != ORBGPU_OK) {
    orbgpu_matcher_destroy(m);
    return ORBGPU_ERR_NOMEM;
  }
  *m->h_done = 0;
  *out = m;
  return ORBGPU_OK;
}

void orbgpu_matcher_destroy(orbgpu_matcher* m) {
  if (!m) return;
  (void)hipSetDevice(m->device);
  if (m->stream) (void)hipStreamSynchronize(m->stream);
  for (Arena* a : {&m->in, &m->out}) {
    if (a->d) (void)hipFree(a->d);
    if (a->h) (void)hipHostFree(a->h);
  }
  if (m->d_cell_start) (void)hipFree(m->d_cell_start);
  if (m->d_cell_idx) (void)hipFree(m->d_cell_idx);
  if (m->d_res) (void)hipFree(m->d_res);
  if (m->d_acc) (void)hipFree(m->d_acc);
  if (m->d_err) (void)hipFree(m->d_err);
  if (m->h_done) (void)hipHostFree(m->h_done);
  if (m->stream) (void)hipStreamDestroy(m->stream);
  delete m;
}

orbgpu_status orbgpu_matcher_status(orbgpu_matcher* m, void* hip_stream, int reset, int* err) {
  if (!m || !err) return ORBGPU_ERR_INVALID;
  *err = 0;
  if (hipSetDevice(m->device) != hipSuccess) return ORBGPU_ERR_DEVICE;
  if (hip_stream && hipStreamSynchronize((hipStream_t)hip_stream) != hipSuccess)
    return ORBGPU_ERR_DEVICE;
  int v = 0;
  if (hipMemcpyAsync(&v, m->d_err, sizeof(int), hipMemcpyDeviceToHost, m->stream) != hipSuccess ||
      (reset && hipMemsetAsync(m->d_err, 0, sizeof(int), m->stream) != hipSuccess) ||
      hipStreamSynchronize(m->stream) != hipSuccess)
    return ORBGPU_ERR_DEVICE;
  *err = v;
  return ORBGPU_OK;
}

orbgpu_status orbgpu_search_by_projection_last(
    orbgpu_matcher* m, const orbgpu_frame_geom* geom, const orbgpu_camera* cam, float mb,
    const orbgpu_pose* Tcw, const orbgpu_pose* Tlw, const orbgpu_keypoint* kps,
    const uint8_t* descs, const float* uright, const uint8_t* claimed, int n,
    const orbgpu_proj_point* pts, int n_pts, float th, int mono, int check_orientation,
    int32_t* match, int* nmatches) {
  if (!m || !cam || !Tcw || !Tlw || bad_frame(kps, descs, n, match, nmatches) || n_pts < 0 ||
      (n_pts > 0 && !pts))
    return ORBGPU_ERR_INVALID;
  if (n > m->max_kp || n_pts > m->max_pts) return ORBGPU_ERR_CAPACITY;
  if (hipSetDevice(m->device) != hipSuccess) return ORBGPU_ERR_DEVICE;
  HostCall c(m);
  orbgpu_status st = fill_params(m, geom, cam, mb, c.L.p);
  if (st != ORBGPU_OK) return st;
  c.L.p.th = th;
  c.L.p.mono = mono != 0;
  c.L.p.check_ori = check_orientation != 0;
  c.L.mode = orbgpu::kModeLast;
  if ((st = stage_frame(c, kps, descs, uright, claimed, n, n_pts)) != ORBGPU_OK) return st;
  orbgpu_proj_point* hp;
  orbgpu_pose* hpose;
  c.L.ppts = c.bi.take<orbgpu_proj_point>(n_pts, &hp);
  if (n_pts > 0) std::memcpy(hp, pts, sizeof(orbgpu_proj_point) * n_pts);
  orbgpu_pose* dpose = c.bi.take<orbgpu_pose>(2, &hpose);
  hpose[0] = *Tcw, hpose[1] = *Tlw;
  c.L.Tcw = dpose;
  c.L.Tlw = dpose + 1;
  return run_host(c, n, match, nmatches, nullptr, n_pts);
}

orbgpu_status orbgpu_search_by_projection_last_batch(
    orbgpu_matcher* m, int n_frames, const orbgpu_frame_geom* geom, const orbgpu_camera* cam,
    float mb, const orbgpu_pose* d_Tcw, const orbgpu_pose* d_Tlw, const orbgpu_keypoint* d_kps,
    const uint8_t* d_descs, const float* d_uright, const uint8_t* d_claimed, const int* d_n,
    int kp_stride, const orbgpu_proj_point* d_pts, const int* d_npts, int pt_stride, float th,
    int mono, int check_orientation, int32_t* d_match, int* d_nmatches, void* hip_stream) {
  if (!m || !cam || n_frames <= 0 || !d_Tcw || !d_Tlw || !d_kps || !d_descs || !d_n ||
      kp_stride <= 0 || kp_stride > orbgpu::kMatchMaxKeypoints || !d_pts || !d_npts ||
      pt_stride <= 0 || pt_stride > orbgpu::kMatchMaxPoints || !d_match || !d_nmatches)
    return ORBGPU_ERR_INVALID;
  if (hipSetDevice(m->device) != hipSuccess) return ORBGPU_ERR_DEVICE;
  MatchLaunch L{};
  orbgpu_status st = fill_params(m, geom, cam, mb, L.p);
  if (st != ORBGPU_OK) return st;
  L.p.th = th;
  L.p.mono = mono != 0;
  L.p.check_ori = check_orientation != 0;
  L.mode = orbgpu::kModeLast;
  L.n_frames = n_frames;
  L.kps = reinterpret_cast<const float*>(d_kps);
  L.desc = d_descs;
  L.uright = d_uright;
  L.claimed = d_claimed;
  L.n = d_n;
  L.kp_stride = kp_stride;
  L.ppts = d_pts;
  L.npts = d_npts;
  L.pt_stride = pt_stride;
  L.max_pts = pt_stride;
  L.Tcw = d_Tcw;
  L.Tlw = d_Tlw;
  if (ensure_scratch(m, n_frames, kp_stride, pt_stride) != ORBGPU_OK) return ORBGPU_ERR_NOMEM;
  L.cell_start = m->d_cell_start;
  L.cell_idx = m->d_cell_idx;
  L.res = m->d_res;
  L.acc = m->d_acc;
  L.match = d_match;
  L.nmatches = d_nmatches;
  L.err = m->d_err;
  hipStream_t s = hip_stream ? (hipStream_t)hip_stream : m->stream;
  return orbgpu::launch_match(L, s) == hipSuccess ? ORBGPU_OK : ORBGPU_ERR_DEVICE;
}

orbgpu_status orbgpu_matches_to_pose_obs_batch(
    orbgpu_matcher* m, int n_frames, const orbgpu_keypoint* d_kps, const float* d_uright,
    const int32_t* d_match, const int* d_n, int kp_stride, const orbgpu_proj_point* d_pts,
    int pt_stride, const float* inv_level_sigma2, int n_levels, orbgpu_pose_obs* d_obs,
    int obs_stride, int* d_nobs, int32_t* d_obs_index, void* hip_stream) {
  if (!m || n_frames <= 0 || !d_kps || !d_match || !d_n || kp_stride <= 0 || !d_pts ||
      pt_stride <= 0 || !inv_level_sigma2 || n_levels <= 0 || n_levels > ORBGPU_MAX_LEVELS ||
      !d_obs || obs_stride <= 0 || !d_nobs)
    return ORBGPU_ERR_INVALID;
  if (hipSetDevice(m->device) != hipSuccess) return ORBGPU_ERR_DEVICE;
  orbgpu::ObsLaunch L{};
  L.n_frames = n_frames;
  L.kps = reinterpret_cast<const float*>(d_kps);
  L.uright = d_uright;
  L.match = d_match;
  L.n = d_n;
  L.kp_stride = kp_stride;
  L.pts = d_pts;
  L.pt_stride = pt_stride;
  for (int l = 0; l < ORBGPU_MAX_LEVELS; ++l) L.inv_sigma2[l] = l < n_levels ? inv_level_sigma2[l] : 0.0f;
  L.obs = d_obs;
  L.obs_stride = obs_stride;
  L.nobs = d_nobs;
  L.obs_index = d_obs_index;
  L.err = m->d_err;
  hipStream_t s = hip_stream ? (hipStream_t)hip_stream : m->stream;
  return orbgpu::launch_pose_obs(L, s) == hipSuccess ? ORBGPU_OK : ORBGPU_ERR_DEVICE;
}

orbgpu_status orbgpu_unproject_stereo_batch(orbgpu_matcher* m, int n_frames,
                                           const orbgpu_camera* cam, const orbgpu_pose* d_Tcw,
                                           const orbgpu_keypoint* d_kps, const uint8_t* d_descs,
                                           const float* d_depth, const int* d_n, int kp_stride,
                                           orbgpu_proj_point* d_pts, int pt_stride, int* d_npts,
                                           void* hip_stream) {
  if (!m || n_frames <= 0 || !cam || !d_Tcw || !d_kps || !d_descs || !d_depth || !d_n ||
      kp_stride <= 0 || !d_pts || pt_stride <= 0 || !d_npts)
    return ORBGPU_ERR_INVALID;
  if (hipSetDevice(m->device) != hipSuccess) return ORBGPU_ERR_DEVICE;
  orbgpu::UnprojLaunch L{};
  L.n_frames = n_frames;
  L.fx = cam->fx;
  L.fy = cam->fy;
  L.cx = cam->cx;
  L.cy = cam->cy;
  L.Tcw = d_Tcw;
  L.kps = reinterpret_cast<const float*>(d_kps);
  L.desc = d_descs;
  L.depth = d_depth;
  L.n = d_n;
  L.kp_stride = kp_stride;
  L.pts = d_pts;
  L.pt_stride = pt_stride;
  L.npts = d_npts;
  L.err = m->d_err;
  hipStream_t s = hip_stream ? (hipStream_t)hip_stream : m->stream;
  return orbgpu::launch_unproject(L, s) == hipSuccess ? ORBGPU_OK : ORBGPU_ERR_DEVICE;
}

orbgpu_status orbgpu_matches_to_inertial_obs_batch(
    orbgpu_matcher* m, int n_frames, const orbgpu_keypoint* d_kps, const float* d_uright,
    const int32_t* d_match, const int* d_n, int kp_stride, const orbgpu_proj_point* d_pts,
    const uint8_t* d_close, int pt_stride, const float* inv_level_sigma2, int n_levels,
    orbgpu_inertial_obs* d_obs, int obs_stride, int* d_nobs, int32_t* d_obs_index,
    void* hip_stream) {
  if (!m || n_frames <= 0 || !d_kps || !d_match || !d_n || kp_stride <= 0 || !d_pts ||
      pt_stride <= 0 || !inv_level_sigma2 || n_levels <= 0 || n_levels > ORBGPU_MAX_LEVELS ||
      !d_obs || obs_stride <= 0 || !d_nobs)
    return ORBGPU_ERR_INVALID;
  if (hipSetDevice(m->device) != hipSuccess) return ORBGPU_ERR_DEVICE;
  orbgpu::ObsLaunch L{};
  L.n_frames = n_frames;
  L.kps = reinterpret_cast<const float*>(d_kps);
  L.uright = d_uright;
  L.match = d_match;
  L.n = d_n;
  L.kp_stride = kp_stride;
  L.pts = d_pts;
  L.pt_stride = pt_stride;
  for (int l = 0; l < ORBGPU_MAX_LEVELS; ++l) L.inv_sigma2[l] = l < n_levels ? inv_level_sigma2[l] : 0.0f;
  L.obs = nullptr;
  L.iobs = d_obs;
  L.close = d_close;
  L.obs_stride = obs_stride;
  L.nobs = d_nobs;
  L.obs_index = d_obs_index;
  L.err = m->d_err;
  hipStream_t s = hip_stream ? (hipStream_t)hip_stream : m->stream;
  return orbgpu::launch_pose_obs(L, s) == hipSuccess ? ORBGPU_OK : ORBGPU_ERR_DEVICE;
}

orbgpu_status orbgpu_frustum(orbgpu_matcher* m, const orbgpu_frame_geom* geom,
                             const orbgpu_camera* cam, const float Rcw[9], const float tcw[3],
                             const float Ow[3], const orbgpu_map_point* pts, int n_pts,
                             float view_cos_limit, orbgpu_track_view* views) {
  // the projection half of orbgpu_search_local_points on an empty frame
  int nm = 0;
  return orbgpu_search_local_points(m, geom, cam, Rcw, tcw, Ow, nullptr, nullptr, nullptr,
                                    nullptr, 0, pts, n_pts, view_cos_limit, 1.0f, 1.0f, 0, 0.0f,
                                    views, nullptr, &nm);
}

static orbgpu_status local_common(orbgpu_matcher* m, const orbgpu_frame_geom* geom,
                                  const orbgpu_camera* cam, const float* pose15,
                                  const orbgpu_keypoint* kps, const uint8_t* descs,
                                  const float* uright, const uint8_t* claimed, int n,
                                  const orbgpu_map_point* pts, const orbgpu_track_view* views_in,
                                  int n_pts, float view_cos_limit, float th, float nn_ratio,
                                  int far_points, float th_far_points,
                                  orbgpu_track_view* views_out, int32_t* match, int* nmatches) {
  if (!m || bad_frame(kps, descs, n, match, nmatches) || n_pts < 0 || (n_pts > 0 && !pts))
    return ORBGPU_ERR_INVALID;
  if (n > m->max_kp || n_pts > m->max_pts) return ORBGPU_ERR_CAPACITY;
  if (hipSetDevice(m->device) != hipSuccess) return ORBGPU_ERR_DEVICE;
  HostCall c(m);
  orbgpu_status st = fill_params(m, geom, cam, 0.0f, c.L.p);
  if (st != ORBGPU_OK) return st;
  c.L.p.th = th;
  c.L.p.nn_ratio = nn_ratio;
  c.L.p.far_points = far_points != 0;
  c.L.p.th_far = th_far_points;
  c.L.p.cos_limit = view_cos_limit;
  c.L.mode = pose15 ? orbgpu::kModeLocalFrustum : orbgpu::kModeLocal;
  if ((st = stage_frame(c, kps, descs, uright, claimed, n, n_pts)) != ORBGPU_OK) return st;
  orbgpu_map_point* hp;
  c.L.mpts = c.bi.take<orbgpu_map_point>(n_pts, &hp);
  if (n_pts > 0) std::memcpy(hp, pts, sizeof(orbgpu_map_point) * n_pts);
  if (pose15) {
    float* hpose;
    c.L.frustum_pose = c.bi.take<float>(15, &hpose);
    std::memcpy(hpose, pose15, 15 * sizeof(float));
    // views: the caller's values go up (isInFrustum leaves fields it does not
    // reach untouched) and come back down
    orbgpu_track_view* hv;
    c.d_views_out = c.bo.take<orbgpu_track_view>(n_pts);
    orbgpu_track_view* dv_in = c.bi.take<orbgpu_track_view>(n_pts, &hv);
    if (n_pts > 0) std::memcpy(hv, views_out, sizeof(orbgpu_track_view) * n_pts);
    c.L.views = c.d_views_out;
    c.L.views_init = dv_in;
  } else {
    orbgpu_track_view* hv;
    c.L.views = c.bi.take<orbgpu_track_view>(n_pts, &hv);
    if (n_pts > 0) std::memcpy(hv, views_in, sizeof(orbgpu_track_view) * n_pts);
  }
  int32_t* match_buf = match;
  int32_t dummy = 0;
  if (n == 0) match_buf = &dummy;
  return run_host(c, n, match_buf, nmatches, pose15 ? views_out : nullptr, n_pts);
}

orbgpu_status orbgpu_search_by_projection_local(
    orbgpu_matcher* m, const orbgpu_frame_geom* geom, const orbgpu_keypoint* kps,
    const uint8_t* descs, const float* uright, const uint8_t* claimed, int n,
    const orbgpu_map_point* pts, const orbgpu_track_view* views, int n_pts, float th,
    float nn_ratio, int far_points, float th_far_points, int32_t* match, int* nmatches) {
  if (n_pts > 0 && !views) return ORBGPU_ERR_INVALID;
  return local_common(m, geom, nullptr, nullptr, kps, descs, uright, claimed, n, pts, views, n_pts,
                      0.0f, th, nn_ratio, far_points, th_far_points, nullptr, match, nmatches);
}

orbgpu_status orbgpu_search_local_points(
    orbgpu_matcher* m, const orbgpu_frame_geom* geom, const orbgpu_camera* cam,
    const float Rcw[9], const float tcw[3], const float Ow[3], const orbgpu_keypoint* kps,
    const uint8_t* descs, const float* uright, const uint8_t* claimed, int n,
    const orbgpu_map_point* pts, int n_pts, float view_cos_limit, float th, float nn_ratio,
    int far_points, float th_far_points, orbgpu_track_view* views, int32_t* match,
    int* nmatches) {
  if (!cam || !Rcw || !tcw || !Ow || (n_pts > 0 && !views)) return ORBGPU_ERR_INVALID;
  float pose15[15];
  std::memcpy(pose15, Rcw, 9 * sizeof(float));
  std::memcpy(pose15 + 9, tcw, 3 * sizeof(float));
  std::memcpy(pose15 + 12, Ow, 3 * sizeof(float));
  return local_common(m, geom, cam, pose15, kps, descs, uright, claimed, n, pts, nullptr, n_pts,
                      view_cos_limit, th, nn_ratio, far_points, th_far_points, views, match,
                      nmatches);
}

orbgpu_status orbgpu_search_by_projection_kf(
    orbgpu_matcher* m, const orbgpu_frame_geom* geom, const orbgpu_camera* cam,
    const orbgpu_pose* Tcw, const orbgpu_keypoint* kps, const uint8_t* descs,
    const uint8_t* claimed, int n, const orbgpu_map_point* pts, const float* angles, int n_pts,
    float th, int orb_dist, int check_orientation, int32_t* match, int* nmatches) {
  if (!m || !cam || !Tcw || bad_frame(kps, descs, n, match, nmatches) || n_pts < 0 ||
      (n_pts > 0 && (!pts || (check_orientation && !angles))))
    return ORBGPU_ERR_INVALID;
  if (n > m->max_kp || n_pts > m->max_pts) return ORBGPU_ERR_CAPACITY;
  if (hipSetDevice(m->device) != hipSuccess) return ORBGPU_ERR_DEVICE;
  HostCall c(m);
  orbgpu_status st = fill_params(m, geom, cam, 0.0f, c.L.p);
  if (st != ORBGPU_OK) return st;
  c.L.p.th = th;
  c.L.p.orb_dist = orb_dist;
  c.L.p.check_ori = check_orientation != 0;
  c.L.mode = orbgpu::kModeKeyFrame;
  if ((st = stage_frame(c, kps, descs, nullptr, claimed, n, n_pts)) != ORBGPU_OK) return st;
  orbgpu_map_point* hp;
  float* ha;
  orbgpu_pose* hpose;
  c.L.mpts = c.bi.take<orbgpu_map_point>(n_pts, &hp);
  if (n_pts > 0) std::memcpy(hp, pts, sizeof(orbgpu_map_point) * n_pts);
  c.L.q_angle = c.bi.take<float>(n_pts, &ha);
  if (n_pts > 0 && angles) std::memcpy(ha, angles, sizeof(float) * n_pts);
  c.L.Tcw = c.bi.take<orbgpu_pose>(1, &hpose);
  hpose[0] = *Tcw;
  int32_t dummy = 0;
  return run_host(c, n, n > 0 ? match : &dummy, nmatches, nullptr, n_pts);
}

orbgpu_status orbgpu_search_by_projection_kf_batch(
    orbgpu_matcher* m, int n_frames, const orbgpu_frame_geom* geom, const orbgpu_camera* cam,
    const orbgpu_pose* d_Tcw, const orbgpu_keypoint* d_kps, const uint8_t* d_descs,
    const uint8_t* d_claimed, const int* d_n, int kp_stride, const orbgpu_map_point* d_pts,
    const float* d_angles, const int* d_npts, int pt_stride, float th, int orb_dist,
    int check_orientation, int32_t* d_match, int* d_nmatches, void* hip_stream) {
  if (!m || !cam || n_frames <= 0 || !d_Tcw || !d_kps || !d_descs || !d_n || kp_stride <= 0 ||
      kp_stride > orbgpu::kMatchMaxKeypoints || !d_pts || (check_orientation && !d_angles) ||
      !d_npts || pt_stride <= 0 || pt_stride > orbgpu::kMatchMaxPoints || !d_match || !d_nmatches)
    return ORBGPU_ERR_INVALID;
  if (hipSetDevice(m->device) != hipSuccess) return ORBGPU_ERR_DEVICE;
  MatchLaunch L{};
  orbgpu_status st = fill_params(m, geom, cam, 0.0f, L.p);
  if (st != ORBGPU_OK) return st;
  L.p.th = th;
  L.p.orb_dist = orb_dist;
  L.p.check_ori = check_orientation != 0;
  L.mode = orbgpu::kModeKeyFrame;
  L.n_frames = n_frames;
  L.kps = reinterpret_cast<const float*>(d_kps);
  L.desc = d_descs;
  L.claimed = d_claimed;
  L.n = d_n;
  L.kp_stride = kp_stride;
  L.mpts = d_pts;
  L.q_angle = d_angles;
  L.npts = d_npts;
  L.pt_stride = pt_stride;
  L.max_pts = pt_stride;
  L.Tcw = d_Tcw;
  if (ensure_scratch(m, n_frames, kp_stride, pt_stride) != ORBGPU_OK) return ORBGPU_ERR_NOMEM;
  L.cell_start = m->d_cell_start;
  L.cell_idx = m->d_cell_idx;
  L.res = m->d_res;
  L.acc = m->d_acc;
  L.match = d_match;
  L.nmatches = d_nmatches;
  L.err = m->d_err;
  hipStream_t s = hip_stream ? (hipStream_t)hip_stream : m->stream;
  return orbgpu::launch_match(L, s) == hipSuccess ? ORBGPU_OK : ORBGPU_ERR_DEVICE;
}

orbgpu_status orbgpu_search_by_bow_batch(
    orbgpu_matcher* m, int n_frames, const uint32_t* d_kf_nodes, const int32_t* d_kf_offsets,
    const uint32_t* d_kf_features, const int* d_kf_n_nodes, const uint8_t* d_kf_descs,
    const float* d_kf_angles, const uint8_t* d_kf_valid, int kf_stride, const uint32_t* d_f_nodes,
    const int32_t* d_f_offsets, const uint32_t* d_f_features, const int* d_f_n_nodes,
    const uint8_t* d_f_descs, const float* d_f_angles, int f_angle_step, const int* d_f_n,
    int f_stride, float nn_ratio, int check_orientation, int32_t* d_match, int* d_nmatches,
    void* hip_stream) {
  if (!m || n_frames <= 0 || !d_kf_nodes || !d_kf_offsets || !d_kf_features || !d_kf_n_nodes ||
      !d_kf_descs || (check_orientation && !d_kf_angles) || !d_kf_valid || kf_stride <= 0 ||
      !d_f_nodes || !d_f_offsets || !d_f_features || !d_f_n_nodes || !d_f_descs ||
      (check_orientation && !d_f_angles) || f_angle_step <= 0 || !d_f_n || f_stride <= 0 ||
      f_stride > orbgpu::kMatchMaxKeypoints || kf_stride > 32767 || !d_match || !d_nmatches)
    return ORBGPU_ERR_INVALID;
  if (hipSetDevice(m->device) != hipSuccess) return ORBGPU_ERR_DEVICE;
  orbgpu::BowSearchLaunch L{};
  L.n_frames = n_frames;
  L.nn_ratio = nn_ratio;
  L.check_ori = check_orientation != 0;
  L.kf_nodes = d_kf_nodes, L.kf_off = d_kf_offsets, L.kf_feat = d_kf_features;
  L.kf_n_nodes = d_kf_n_nodes, L.kf_desc = d_kf_descs, L.kf_angle = d_kf_angles;
  L.kf_valid = d_kf_valid, L.kf_stride = kf_stride;
  L.f_nodes = d_f_nodes, L.f_off = d_f_offsets, L.f_feat = d_f_features;
  L.f_n_nodes = d_f_n_nodes, L.f_desc = d_f_descs, L.f_angle = d_f_angles;
  L.angle_step = f_angle_step, L.f_n = d_f_n, L.f_stride = f_stride;
  L.match = d_match, L.nmatches = d_nmatches, L.err = m->d_err;
  hipStream_t s = hip_stream ? (hipStream_t)hip_stream : m->stream;
  return orbgpu::launch_bow_search(L, s) == hipSuccess ? ORBGPU_OK : ORBGPU_ERR_DEVICE;
}

orbgpu_status orbgpu_search_by_bow(orbgpu_matcher* m, const uint32_t* kf_nodes,
                                   const int32_t* kf_offsets, const uint32_t* kf_features,
                                   int kf_n_nodes, const uint8_t* kf_descs, const float* kf_angles,
                                   const uint8_t* kf_valid, int kf_n, const uint32_t* f_nodes,
                                   const int32_t* f_offsets, const uint32_t* f_features,
                                   int f_n_nodes, const uint8_t* f_descs, const float* f_angles,
                                   int f_n, float nn_ratio, int check_orientation, int32_t* match,
                                   int* nmatches) {
  if (!m || kf_n < 0 || f_n < 0 || kf_n_nodes < 0 || f_n_nodes < 0 || !nmatches ||
      (kf_n_nodes > 0 && (!kf_nodes || !kf_offsets || !kf_features)) ||
      (f_n_nodes > 0 && (!f_nodes || !f_offsets || !f_features)) ||
      (kf_n > 0 && (!kf_descs || !kf_valid || (check_orientation && !kf_angles))) ||
      (f_n > 0 && (!f_descs || !match || (check_orientation && !f_angles))) ||
      kf_n_nodes > kf_n || f_n_nodes > f_n)
    return ORBGPU_ERR_INVALID;
  if (f_n > m->max_kp || kf_n > 32767) return ORBGPU_ERR_CAPACITY;
  for (int j = 0; j < kf_n_nodes; ++j)
    if (kf_offsets[j + 1] < kf_offsets[j] || kf_offsets[j + 1] > kf_n) return ORBGPU_ERR_INVALID;
  for (int j = 0; j < f_n_nodes; ++j)
    if (f_offsets[j + 1] < f_offsets[j] || f_offsets[j + 1] > f_n) return ORBGPU_ERR_INVALID;
  if (hipSetDevice(m->device) != hipSuccess) return ORBGPU_ERR_DEVICE;
  const int KS = std::max(kf_n, 1), FS = std::max(f_n, 1);
  // one upload: both FeatureVectors, descriptors, angles, valid flags, counts
  const size_t need = 3 * align_up(4 * (size_t)KS) + align_up(4 * (size_t)(KS + 1)) +
                      align_up(32 * (size_t)KS) + align_up(KS) + 3 * align_up(4 * (size_t)FS) +
                      align_up(4 * (size_t)(FS + 1)) + align_up(32 * (size_t)FS) + align_up(12);
  if (arena_reserve(m->in, need) != ORBGPU_OK) return ORBGPU_ERR_NOMEM;
  Bump b2{m->in};
  uint32_t *hkn, *hkf, *hfn, *hff;
  int32_t *hko, *hfo;
  uint8_t *hkd, *hkv, *hfd;
  float *hka, *hfa;
  int* hcnt;
  const uint32_t* dkn = b2.take<uint32_t>(KS, &hkn);
  const int32_t* dko = b2.take<int32_t>(KS + 1, &hko);
  const uint32_t* dkf = b2.take<uint32_t>(KS, &hkf);
  const uint8_t* dkd = b2.take<uint8_t>(32 * (size_t)KS, &hkd);
  const float* dka = b2.take<float>(KS, &hka);
  const uint8_t* dkv = b2.take<uint8_t>(KS, &hkv);
  const uint32_t* dfn = b2.take<uint32_t>(FS, &hfn);
  const int32_t* dfo = b2.take<int32_t>(FS + 1, &hfo);
  const uint32_t* dff = b2.take<uint32_t>(FS, &hff);
  const uint8_t* dfd = b2.take<uint8_t>(32 * (size_t)FS, &hfd);
  const float* dfa = b2.take<float>(FS, &hfa);
  int* dcnt = b2.take<int>(3, &hcnt);
  hko[0] = 0;
  if (kf_n_nodes > 0) {
    std::memcpy(hkn, kf_nodes, 4 * (size_t)kf_n_nodes);
    std::memcpy(hko, kf_offsets, 4 * (size_t)(kf_n_nodes + 1));
    std::memcpy(hkf, kf_features, 4 * (size_t)kf_offsets[kf_n_nodes]);
  }
  hfo[0] = 0;
  if (f_n_nodes > 0) {
    std::memcpy(hfn, f_nodes, 4 * (size_t)f_n_nodes);
    std::memcpy(hfo, f_offsets, 4 * (size_t)(f_n_nodes + 1));
    std::memcpy(hff, f_features, 4 * (size_t)f_offsets[f_n_nodes]);
  }
  if (kf_n > 0) {
    std::memcpy(hkd, kf_descs, 32 * (size_t)kf_n);
    std::memcpy(hkv, kf_valid, kf_n);
    if (kf_angles) std::memcpy(hka, kf_angles, 4 * (size_t)kf_n);
  }
  if (f_n > 0) {
    std::memcpy(hfd, f_descs, 32 * (size_t)f_n);
    if (f_angles) std::memcpy(hfa, f_angles, 4 * (size_t)f_n);
  }
  hcnt[0] = kf_n_nodes, hcnt[1] = f_n_nodes, hcnt[2] = f_n;
  Bump bo{m->out};
  int32_t* dmatch = bo.take<int32_t>(FS);
  int* dnm = bo.take<int>(1);
  hipStream_t s = m->stream;
  if (hipMemsetAsync(m->d_err, 0, sizeof(int), s) ||
      hipMemcpyAsync(m->in.d, m->in.h, b2.off, hipMemcpyHostToDevice, s))
    return ORBGPU_ERR_DEVICE;
  const orbgpu_status st = orbgpu_search_by_bow_batch(
      m, 1, dkn, dko, dkf, dcnt, dkd, dka, dkv, KS, dfn, dfo, dff, dcnt + 1, dfd, dfa, 1, dcnt + 2, FS,
      nn_ratio, check_orientation, dmatch, dnm, s);
  if (st != ORBGPU_OK) return st;
  int err = 0;
  const size_t dl = (size_t)((uint8_t*)dnm - m->out.d) + sizeof(int);
  if (hipMemcpyAsync(m->out.h, m->out.d, dl, hipMemcpyDeviceToHost, s) ||
      hipMemcpyAsync(&err, m->d_err, sizeof(int), hipMemcpyDeviceToHost, s) || hipStreamSynchronize(s))
    return ORBGPU_ERR_DEVICE;
  if (err) return ORBGPU_ERR_CAPACITY;
  if (f_n > 0) std::memcpy(match, m->out.h + ((uint8_t*)dmatch - m->out.d), 4 * (size_t)f_n);
  std::memcpy(nmatches, m->out.h + ((uint8_t*)dnm - m->out.d), sizeof(int));
  return ORBGPU_OK;
}

int orbgpu_level_thresholds(float log_scale_factor, int n_levels, float* thr) {
  if (!thr || n_levels <= 0 || n_levels > ORBGPU_MAX_LEVELS || !(log_scale_factor > 0)) return -1;
  level_thresholds(log_scale_factor, n_levels, thr);
  return n_levels - 1;
}

}  // extern "C"
