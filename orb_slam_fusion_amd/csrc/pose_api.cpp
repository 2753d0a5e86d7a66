// C-ABI implementation of the pose-only optimisation half of include/orbgpu.h.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include <cstdlib>
#include <cstring>
#include <new>

#include "../../include/orbgpu.h"

namespace orbgpu {
hipError_t launch_pose_opt(const double cam[5], const float* d_pose_in, const void* d_obs,
                           const int* d_nobs, int obs_stride, int n_problems, float* d_pose_out,
                           uint8_t* d_outlier, int* d_inliers, double* d_pose_out_d,
                           hipStream_t st, int groups, int* done_host = nullptr, int seq = 0);
}

static_assert(sizeof(orbgpu_pose) == 7 * sizeof(float), "orbgpu_pose layout");
static_assert(sizeof(orbgpu_pose_obs) == 7 * sizeof(float), "orbgpu_pose_obs layout");

struct orbgpu_pose_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  int max_obs = 0;
  // speculative LM trial groups per problem (k_pose_opt), see
  // orbgpu_pose_ctx_set_trial_groups
  int groups_single = 1;
  int groups_batch = 1;
  // single-problem path: the input and output as one block each, pinned on
  // the host and mirrored on the device -- in: pose (28 B), n (4 B), obs;
  // out: pose (28 B), inliers (4 B), outlier flags -- so a call is one H2D
  // copy, the kernel and one D2H copy, sized by the observation count's
  // bucket (kObsBucket), replayed as a hipGraph per (bucket, groups, camera)
  // from the second call of that key on
  uint8_t* h_in = nullptr;
  uint8_t* h_out = nullptr;
  uint8_t* d_in = nullptr;
  uint8_t* d_out = nullptr;
  // zero-copy single path (the default): the kernel reads h_in and writes
  // h_out through their device mappings (fine-grained, uncached host memory),
  // so a call is one kernel launch -- no copy commands, no graph replay.
  // ORBGPU_POSE_IO=graph keeps the copy + graph path (A/B runs).
  bool zero_copy = true;
  uint8_t* h_in_dev = nullptr;
  uint8_t* h_out_dev = nullptr;
  // the zero-copy call's completion word (host-mapped): the kernel stores the
  // call's number after its outputs; the host polls it
  int* h_done = nullptr;
  int* h_done_dev = nullptr;
  int seq = 0;
  struct Graph {
    int bucket = 0, groups = 0;
    double cam[5] = {};
    bool warm = false;  // seen once: captured on the next call
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
  };
  std::vector<Graph> graphs;  // a few keys, oldest replaced first
};

namespace {
constexpr size_t kInPose = 0;  // h_in / d_in layout: pose (28 B), n (4 B), obs
constexpr size_t kInN = 28;
constexpr size_t kInObs = 32;
constexpr size_t kOutPose = 0;  // h_out / d_out layout: pose (28 B), inliers (4 B), outlier flags
constexpr size_t kOutInl = 28;
constexpr size_t kOutFlags = 32;
constexpr int kObsBucket = 128;  // copy sizes rounded up to this many observations
constexpr size_t kMaxGraphs = 6;

hipError_t enqueue_single(orbgpu_pose_ctx* c, const double cd[5], int bucket, int groups) {
  hipError_t e = hipMemcpyAsync(c->d_in, c->h_in, kInObs + sizeof(orbgpu_pose_obs) * bucket,
                                hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess)
    e = orbgpu::launch_pose_opt(cd, reinterpret_cast<const float*>(c->d_in + kInPose), c->d_in + kInObs,
                                reinterpret_cast<const int*>(c->d_in + kInN), bucket, 1,
                                reinterpret_cast<float*>(c->d_out + kOutPose), c->d_out + kOutFlags,
                                reinterpret_cast<int*>(c->d_out + kOutInl), nullptr, c->stream, groups);
  if (e == hipSuccess)
    e = hipMemcpyAsync(c->h_out, c->d_out, kOutFlags + bucket, hipMemcpyDeviceToHost, c->stream);
  return e;
}

void destroy_graph(orbgpu_pose_ctx::Graph& g) {
  if (g.exec) (void)hipGraphExecDestroy(g.exec);
  if (g.graph) (void)hipGraphDestroy(g.graph);
  g.exec = nullptr;
  g.graph = nullptr;
}
}  // namespace

extern "C" {

orbgpu_status orbgpu_pose_ctx_create(int device, int max_problems, int max_obs,
                                     orbgpu_pose_ctx** out) {
  if (!out || max_obs <= 0 || max_problems <= 0) return ORBGPU_ERR_INVALID;
  *out = nullptr;
  if (hipSetDevice(device) != hipSuccess) return ORBGPU_ERR_DEVICE;
  auto* c = new (std::nothrow) orbgpu_pose_ctx();
  if (!c) return ORBGPU_ERR_NOMEM;
  c->device = device;
  c->max_obs = max_obs;
  if (const char* e = getenv("ORBGPU_POSE_GROUPS")) {  // A/B runs (tools/pose_ab.sh)
    const int g = atoi(e);
    if (g == 1 || g == 2) c->groups_single = c->groups_batch = g;
  }
  const size_t in_bytes = kInObs + sizeof(orbgpu_pose_obs) * ((max_obs + kObsBucket - 1) / kObsBucket * kObsBucket);
  const size_t out_bytes = kOutFlags + (max_obs + kObsBucket - 1) / kObsBucket * kObsBucket;
  if (const char* e = getenv("ORBGPU_POSE_IO")) c->zero_copy = strcmp(e, "graph") != 0;
  const unsigned hflags = hipHostMallocMapped | hipHostMallocCoherent;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc(&c->d_in, in_bytes) != hipSuccess || hipMalloc(&c->d_out, out_bytes) != hipSuccess ||
      hipHostMalloc(&c->h_in, in_bytes, hflags) != hipSuccess ||
      hipHostMalloc(&c->h_out, out_bytes, hflags) != hipSuccess ||
      hipHostGetDevicePointer(reinterpret_cast<void**>(&c->h_in_dev), c->h_in, 0) != hipSuccess ||
      hipHostGetDevicePointer(reinterpret_cast<void**>(&c->h_out_dev), c->h_out, 0) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void**>(&c->h_done), 64, hflags) != hipSuccess ||
      hipHostGetDevicePointer(reinterpret_cast<void**>(&c->h_done_dev), c->h_done, 0) != hipSuccess) {
    orbgpu_pose_ctx_destroy(c);
    return ORBGPU_ERR_DEVICE;
  }
  *c->h_done = 0;
  *out = c;
  return ORBGPU_OK;
}

orbgpu_status orbgpu_pose_ctx_set_trial_groups(orbgpu_pose_ctx* c, int groups_single,
                                               int groups_batch) {
  auto valid = [](int g) { return g == 1 || g == 2; };
  if (!c || !valid(groups_single) || !valid(groups_batch)) return ORBGPU_ERR_INVALID;
  c->groups_single = groups_single;
  c->groups_batch = groups_batch;
  return ORBGPU_OK;
}

void orbgpu_pose_ctx_destroy(orbgpu_pose_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->d_in) (void)hipFree(c->d_in);
  if (c->d_out) (void)hipFree(c->d_out);
  for (auto& g : c->graphs) destroy_graph(g);
  if (c->h_in) (void)hipHostFree(c->h_in);
  if (c->h_out) (void)hipHostFree(c->h_out);
  if (c->h_done) (void)hipHostFree(c->h_done);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

orbgpu_status orbgpu_pose_opt(orbgpu_pose_ctx* c, const orbgpu_camera* cam,
                              const orbgpu_pose* Tcw_in, const orbgpu_pose_obs* obs, int n_obs,
                              orbgpu_pose* Tcw_out, uint8_t* outlier, int* n_inliers) {
  if (!c || !cam || !Tcw_in || !Tcw_out || !n_inliers || n_obs < 0 || (n_obs > 0 && !obs))
    return ORBGPU_ERR_INVALID;
  if (n_obs > c->max_obs) return ORBGPU_ERR_CAPACITY;
  if (n_obs > 0 && !outlier) return ORBGPU_ERR_INVALID;
  if (hipSetDevice(c->device) != hipSuccess) return ORBGPU_ERR_DEVICE;
  const double cd[5] = {cam->fx, cam->fy, cam->cx, cam->cy, cam->bf};
  // the camera is a kernel argument: a graph is kept for one camera
  static_assert(sizeof(orbgpu_pose) == 28, "pose staging layout");
  memcpy(c->h_in + kInPose, Tcw_in, sizeof(orbgpu_pose));
  memcpy(c->h_in + kInN, &n_obs, sizeof(int));
  if (n_obs > 0) memcpy(c->h_in + kInObs, obs, sizeof(orbgpu_pose_obs) * n_obs);
  const int bucket = std::min(c->max_obs, std::max(1, (n_obs + kObsBucket - 1) / kObsBucket) * kObsBucket);
  const int groups = c->groups_single;
  if (c->zero_copy) {
    const int seq = c->seq = c->seq == 0x7fffffff ? 1 : c->seq + 1;
    const hipError_t ze = orbgpu::launch_pose_opt(
        cd, reinterpret_cast<const float*>(c->h_in_dev + kInPose), c->h_in_dev + kInObs,
        reinterpret_cast<const int*>(c->h_in_dev + kInN), bucket, 1,
        reinterpret_cast<float*>(c->h_out_dev + kOutPose), c->h_out_dev + kOutFlags,
        reinterpret_cast<int*>(c->h_out_dev + kOutInl), nullptr, c->stream, groups, c->h_done_dev, seq);
    if (ze != hipSuccess) return ORBGPU_ERR_DEVICE;
    // poll the completion word (the stream's own synchronisation decides past
    // ~0.5 s or on a stream error), as the extractor's single-image path
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
    memcpy(Tcw_out, c->h_out + kOutPose, sizeof(orbgpu_pose));
    memcpy(n_inliers, c->h_out + kOutInl, sizeof(int));
    if (n_obs > 0) memcpy(outlier, c->h_out + kOutFlags, n_obs);
    return ORBGPU_OK;
  }
  orbgpu_pose_ctx::Graph* g = nullptr;
  for (auto& x : c->graphs)
    if (x.bucket == bucket && x.groups == groups && memcmp(x.cam, cd, sizeof(cd)) == 0) g = &x;
  hipError_t e = hipSuccess;
  if (g && g->exec) {
    e = hipGraphLaunch(g->exec, c->stream);
  } else if (g) {  // second call of this key: capture the chain (LDS opt-ins already done)
    e = hipStreamBeginCapture(c->stream, hipStreamCaptureModeRelaxed);
    if (e == hipSuccess) {
      const hipError_t le = enqueue_single(c, cd, bucket, groups);
      e = hipStreamEndCapture(c->stream, &g->graph);
      if (e == hipSuccess) e = le;
    }
    if (e == hipSuccess) e = hipGraphInstantiate(&g->exec, g->graph, nullptr, nullptr, 0);
    if (e == hipSuccess) {
      e = hipGraphLaunch(g->exec, c->stream);
    } else {
      (void)hipGetLastError();
      destroy_graph(*g);
      e = enqueue_single(c, cd, bucket, groups);
    }
  } else {
    e = enqueue_single(c, cd, bucket, groups);
    if (c->graphs.size() >= kMaxGraphs) {
      destroy_graph(c->graphs.front());
      c->graphs.erase(c->graphs.begin());
    }
    orbgpu_pose_ctx::Graph ng;
    ng.bucket = bucket;
    ng.groups = groups;
    memcpy(ng.cam, cd, sizeof(cd));
    c->graphs.push_back(ng);
  }
  if (e != hipSuccess || hipStreamSynchronize(c->stream)) return ORBGPU_ERR_DEVICE;
  memcpy(Tcw_out, c->h_out + kOutPose, sizeof(orbgpu_pose));
  int ints[2] = {0, 0};
  memcpy(&ints[1], c->h_out + kOutInl, sizeof(int));
  if (n_obs > 0) memcpy(outlier, c->h_out + kOutFlags, n_obs);
  *n_inliers = ints[1];
  return ORBGPU_OK;
}

orbgpu_status orbgpu_pose_opt_batch(orbgpu_pose_ctx* c, const orbgpu_camera* cam,
                                    const orbgpu_pose* d_Tcw_in, const orbgpu_pose_obs* d_obs,
                                    const int* d_nobs, int obs_stride, int n_problems,
                                    orbgpu_pose* d_Tcw_out, uint8_t* d_outlier, int* d_inliers,
                                    double* d_pose_out_d, void* hip_stream) {
  if (!c || !cam || !d_Tcw_in || !d_obs || !d_nobs || !d_Tcw_out || !d_outlier || !d_inliers ||
      n_problems <= 0 || obs_stride <= 0)
    return ORBGPU_ERR_INVALID;
  if (hipSetDevice(c->device) != hipSuccess) return ORBGPU_ERR_DEVICE;
  const double cd[5] = {cam->fx, cam->fy, cam->cx, cam->cy, cam->bf};
  hipStream_t s = hip_stream ? (hipStream_t)hip_stream : c->stream;
  if (orbgpu::launch_pose_opt(cd, reinterpret_cast<const float*>(d_Tcw_in), d_obs, d_nobs,
                              obs_stride, n_problems, reinterpret_cast<float*>(d_Tcw_out),
                              d_outlier, d_inliers, d_pose_out_d, s, c->groups_batch) != hipSuccess)
    return ORBGPU_ERR_DEVICE;
  return ORBGPU_OK;
}

}  // extern "C"
