// C-ABI implementation of the inertial tracking optimisation
// (orbgpu_pose_inertial*, include/orbgpu.h).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/orbgpu.h"

namespace orbgpu {
hipError_t launch_pose_inertial(int mode, const orbgpu_imu_calib& c, int n_problems,
                                const orbgpu_imu_state* d_cur, const orbgpu_imu_state* d_prev,
                                const orbgpu_imu_preint* d_preint, const orbgpu_imu_prior* d_prior,
                                const orbgpu_inertial_obs* d_obs, const int* d_nobs, int obs_stride,
                                int rec_init, orbgpu_inertial_result* d_res, uint8_t* d_outlier,
                                hipStream_t st, int* done_host = nullptr, const int* seq_src = nullptr);
}

static_assert(sizeof(orbgpu_imu_state) == 132, "orbgpu_imu_state layout");
static_assert(sizeof(orbgpu_imu_preint) == 1064, "orbgpu_imu_preint layout");
static_assert(sizeof(orbgpu_imu_prior) == 1968, "orbgpu_imu_prior layout");
static_assert(sizeof(orbgpu_inertial_obs) == 32, "orbgpu_inertial_obs layout");
static_assert(sizeof(orbgpu_inertial_result) == 2064, "orbgpu_inertial_result layout");

struct orbgpu_inertial_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  int max_problems = 0, max_obs = 0;
  // single-problem path: the input as one pinned block mirrored on the device
  // -- [cur | prev | preint | prior | n_obs | call number | obs] -- and the
  // output block [result | outlier flags] in host-mapped memory, written by
  // the kernel itself, which then stores the call number into h_done (the
  // host polls it): a call is one H2D copy and the kernel, sized by the
  // observation count's bucket, replayed as a hipGraph per (mode, bucket,
  // rec_init, calibration) from the second call of that key on
  uint8_t* h_in = nullptr;
  uint8_t* h_out = nullptr;
  uint8_t* h_out_dev = nullptr;
  uint8_t* d_in = nullptr;
  int* h_done = nullptr;
  int* h_done_dev = nullptr;
  int seq = 0;
  struct Graph {
    int mode = 0, bucket = 0, rec_init = 0;
    orbgpu_imu_calib calib{};
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
  };
  std::vector<Graph> graphs;  // a few keys, oldest replaced first
};

namespace {
constexpr size_t kOffPrev = 136, kOffPreint = 272, kOffPrior = 1336, kOffN = 3304, kOffSeq = 3308, kInBytes = 3312;
static_assert(kOffPrev >= sizeof(orbgpu_imu_state) && kOffPreint - kOffPrev >= sizeof(orbgpu_imu_state) &&
                  kOffPrior - kOffPreint >= sizeof(orbgpu_imu_preint) &&
                  kOffN - kOffPrior >= sizeof(orbgpu_imu_prior) && kOffPreint % 8 == 0 &&
                  kOffPrior % 8 == 0 && kInBytes % 16 == 0,
              "staging layout");
constexpr size_t kOutFlags = 2064;  // the result record, then the flags
static_assert(sizeof(orbgpu_inertial_result) <= kOutFlags && kOutFlags % 16 == 0, "output layout");
constexpr int kObsBucket = 128;
constexpr size_t kMaxGraphs = 6;

bool valid_calib(const orbgpu_imu_calib* c) {
  return c && c->fx > 0 && c->fy > 0;
}

hipError_t enqueue_single(orbgpu_inertial_ctx* c, int mode, const orbgpu_imu_calib& calib, int bucket,
                          int rec_init) {
  hipStream_t st = c->stream;
  hipError_t e = hipMemcpyAsync(c->d_in, c->h_in, kInBytes + sizeof(orbgpu_inertial_obs) * bucket,
                                hipMemcpyHostToDevice, st);
  if (e == hipSuccess)
    e = orbgpu::launch_pose_inertial(
        mode, calib, 1, reinterpret_cast<const orbgpu_imu_state*>(c->d_in),
        reinterpret_cast<const orbgpu_imu_state*>(c->d_in + kOffPrev),
        reinterpret_cast<const orbgpu_imu_preint*>(c->d_in + kOffPreint),
        reinterpret_cast<const orbgpu_imu_prior*>(c->d_in + kOffPrior),
        reinterpret_cast<const orbgpu_inertial_obs*>(c->d_in + kInBytes),
        reinterpret_cast<const int*>(c->d_in + kOffN), bucket, rec_init,
        reinterpret_cast<orbgpu_inertial_result*>(c->h_out_dev), c->h_out_dev + kOutFlags, st, c->h_done_dev,
        reinterpret_cast<const int*>(c->d_in + kOffSeq));
  return e;
}

void destroy_graph(orbgpu_inertial_ctx::Graph& g) {
  if (g.exec) (void)hipGraphExecDestroy(g.exec);
  if (g.graph) (void)hipGraphDestroy(g.graph);
  g.exec = nullptr;
  g.graph = nullptr;
}
}  // namespace

extern "C" {

orbgpu_status orbgpu_inertial_ctx_create(int device, int max_problems, int max_obs,
                                         orbgpu_inertial_ctx** out) {
  if (!out || max_obs <= 0 || max_problems <= 0) return ORBGPU_ERR_INVALID;
  *out = nullptr;
  if (hipSetDevice(device) != hipSuccess) return ORBGPU_ERR_DEVICE;
  auto* c = new (std::nothrow) orbgpu_inertial_ctx();
  if (!c) return ORBGPU_ERR_NOMEM;
  c->device = device;
  c->max_problems = max_problems;
  c->max_obs = max_obs;
  const size_t nb = (size_t)(max_obs + kObsBucket - 1) / kObsBucket * kObsBucket;
  const size_t in_bytes = kInBytes + sizeof(orbgpu_inertial_obs) * nb, out_bytes = kOutFlags + nb;
  const unsigned hflags = hipHostMallocMapped | hipHostMallocCoherent;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc(&c->d_in, in_bytes) != hipSuccess || hipHostMalloc(&c->h_in, in_bytes) != hipSuccess ||
      hipHostMalloc(&c->h_out, out_bytes, hflags) != hipSuccess ||
      hipHostGetDevicePointer(reinterpret_cast<void**>(&c->h_out_dev), c->h_out, 0) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void**>(&c->h_done), 64, hflags) != hipSuccess ||
      hipHostGetDevicePointer(reinterpret_cast<void**>(&c->h_done_dev), c->h_done, 0) != hipSuccess) {
    orbgpu_inertial_ctx_destroy(c);
    return ORBGPU_ERR_DEVICE;
  }
  *c->h_done = 0;
  *out = c;
  return ORBGPU_OK;
}

void orbgpu_inertial_ctx_destroy(orbgpu_inertial_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  for (auto& g : c->graphs) destroy_graph(g);
  if (c->d_in) (void)hipFree(c->d_in);

  if (c->h_in) (void)hipHostFree(c->h_in);
  if (c->h_out) (void)hipHostFree(c->h_out);
  if (c->h_done) (void)hipHostFree(c->h_done);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

orbgpu_status orbgpu_pose_inertial(orbgpu_inertial_ctx* c, int mode, const orbgpu_imu_calib* calib,
                                   const orbgpu_imu_state* cur, const orbgpu_imu_state* prev,
                                   const orbgpu_imu_preint* preint, const orbgpu_imu_prior* prior,
                                   const orbgpu_inertial_obs* obs, int n_obs, int rec_init,
                                   orbgpu_inertial_result* res, uint8_t* outlier) {
  if (!c || !valid_calib(calib) || !cur || !prev || !preint || !res || n_obs < 0 ||
      (n_obs > 0 && (!obs || !outlier)) ||
      (mode != ORBGPU_INERTIAL_LAST_FRAME && mode != ORBGPU_INERTIAL_LAST_KEYFRAME) ||
      (mode == ORBGPU_INERTIAL_LAST_FRAME && !prior))
    return ORBGPU_ERR_INVALID;
  if (n_obs > c->max_obs) return ORBGPU_ERR_CAPACITY;
  if (hipSetDevice(c->device) != hipSuccess) return ORBGPU_ERR_DEVICE;
  uint8_t* host = c->h_in;
  std::memcpy(host, cur, sizeof(*cur));
  std::memcpy(host + kOffPrev, prev, sizeof(*prev));
  std::memcpy(host + kOffPreint, preint, sizeof(*preint));
  if (prior)
    std::memcpy(host + kOffPrior, prior, sizeof(*prior));
  else
    std::memset(host + kOffPrior, 0, sizeof(orbgpu_imu_prior));
  std::memcpy(host + kOffN, &n_obs, sizeof(int));
  const int seq = c->seq = c->seq == 0x7fffffff ? 1 : c->seq + 1;
  std::memcpy(host + kOffSeq, &seq, sizeof(int));
  if (n_obs > 0) std::memcpy(host + kInBytes, obs, sizeof(*obs) * n_obs);
  const int bucket = std::min(c->max_obs, std::max(1, (n_obs + kObsBucket - 1) / kObsBucket) * kObsBucket);
  const int ri = rec_init ? 1 : 0;
  orbgpu_inertial_ctx::Graph* g = nullptr;
  for (auto& x : c->graphs)
    if (x.mode == mode && x.bucket == bucket && x.rec_init == ri && memcmp(&x.calib, calib, sizeof(*calib)) == 0)
      g = &x;
  hipError_t e = hipSuccess;
  if (g && g->exec) {
    e = hipGraphLaunch(g->exec, c->stream);
  } else if (g) {  // second call of this key: capture (the LDS opt-in is done)
    e = hipStreamBeginCapture(c->stream, hipStreamCaptureModeRelaxed);
    if (e == hipSuccess) {
      const hipError_t le = enqueue_single(c, mode, *calib, bucket, ri);
      e = hipStreamEndCapture(c->stream, &g->graph);
      if (e == hipSuccess) e = le;
    }
    if (e == hipSuccess) e = hipGraphInstantiate(&g->exec, g->graph, nullptr, nullptr, 0);
    if (e == hipSuccess) {
      e = hipGraphLaunch(g->exec, c->stream);
    } else {
      (void)hipGetLastError();
      destroy_graph(*g);
      e = enqueue_single(c, mode, *calib, bucket, ri);
    }
  } else {
    e = enqueue_single(c, mode, *calib, bucket, ri);
    if (c->graphs.size() >= kMaxGraphs) {
      destroy_graph(c->graphs.front());
      c->graphs.erase(c->graphs.begin());
    }
    orbgpu_inertial_ctx::Graph ng;
    ng.mode = mode;
    ng.bucket = bucket;
    ng.rec_init = ri;
    ng.calib = *calib;
    c->graphs.push_back(ng);
  }
  if (e != hipSuccess) return ORBGPU_ERR_DEVICE;
  // poll the completion word (the stream's own synchronisation decides past
  // ~0.5 s or on a stream error)
  volatile int* done = c->h_done;
  bool seen = false;
  for (long spin = 0; spin < (1L << 24); ++spin) {
    if (*done == seq) {
      seen = true;
      break;
    }
    if ((spin & 4095) == 4095 && hipStreamQuery(c->stream) != hipErrorNotReady) {
      seen = *done == seq;
      break;
    }
    __builtin_ia32_pause();
  }
  __atomic_thread_fence(__ATOMIC_ACQUIRE);
  if (!seen && (hipStreamSynchronize(c->stream) != hipSuccess || *done != seq)) return ORBGPU_ERR_DEVICE;
  std::memcpy(res, c->h_out, sizeof(*res));
  if (n_obs > 0) std::memcpy(outlier, c->h_out + kOutFlags, n_obs);
  return ORBGPU_OK;
}

orbgpu_status orbgpu_pose_inertial_batch(orbgpu_inertial_ctx* c, int mode,
                                         const orbgpu_imu_calib* calib, int n_problems,
                                         const orbgpu_imu_state* d_cur,
                                         const orbgpu_imu_state* d_prev,
                                         const orbgpu_imu_preint* d_preint,
                                         const orbgpu_imu_prior* d_prior,
                                         const orbgpu_inertial_obs* d_obs, const int* d_nobs,
                                         int obs_stride, int rec_init,
                                         orbgpu_inertial_result* d_res, uint8_t* d_outlier,
                                         void* hip_stream) {
  if (!c || !valid_calib(calib) || n_problems < 0 || obs_stride <= 0 ||
      (mode != ORBGPU_INERTIAL_LAST_FRAME && mode != ORBGPU_INERTIAL_LAST_KEYFRAME))
    return ORBGPU_ERR_INVALID;
  if (n_problems == 0) return ORBGPU_OK;
  if (!d_cur || !d_prev || !d_preint || !d_obs || !d_nobs || !d_res || !d_outlier ||
      (mode == ORBGPU_INERTIAL_LAST_FRAME && !d_prior))
    return ORBGPU_ERR_INVALID;
  if (n_problems > c->max_problems || obs_stride > c->max_obs) return ORBGPU_ERR_CAPACITY;
  if (hipSetDevice(c->device) != hipSuccess) return ORBGPU_ERR_DEVICE;
  hipStream_t st = hip_stream ? static_cast<hipStream_t>(hip_stream) : c->stream;
  if (orbgpu::launch_pose_inertial(mode, *calib, n_problems, d_cur, d_prev, d_preint, d_prior,
                                   d_obs, d_nobs, obs_stride, rec_init, d_res, d_outlier,
                                   st) != hipSuccess)
    return ORBGPU_ERR_DEVICE;
  return ORBGPU_OK;
}

}  // extern "C"
