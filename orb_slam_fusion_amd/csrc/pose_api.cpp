// C-ABI implementation of the pose-only optimisation half of include/orbgpu.h.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <new>

#include "../../include/orbgpu.h"

namespace orbgpu {
hipError_t launch_pose_opt(const double cam[5], const float* d_pose_in, const void* d_obs,
                           const int* d_nobs, int obs_stride, int n_problems, float* d_pose_out,
                           uint8_t* d_outlier, int* d_inliers, double* d_pose_out_d,
                           hipStream_t st, int groups);
}

static_assert(sizeof(orbgpu_pose) == 7 * sizeof(float), "orbgpu_pose layout");
static_assert(sizeof(orbgpu_pose_obs) == 7 * sizeof(float), "orbgpu_pose_obs layout");

struct orbgpu_pose_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  int max_obs = 0;
  orbgpu_pose_obs* d_obs = nullptr;
  float* d_pose = nullptr;  // in[7], out[7]
  uint8_t* d_outlier = nullptr;
  int* d_ints = nullptr;  // n, inliers
  // speculative LM trial groups per problem (k_pose_opt), see
  // orbgpu_pose_ctx_set_trial_groups
  int groups_single = 1;
  int groups_batch = 1;
  // single-problem path: pinned staging (obs[max_obs], pose in, n | pose out,
  // inliers, outlier[max_obs]) and the fixed-size copy + kernel + copy chain,
  // replayed as a hipGraph from the second call on
  uint8_t* h_in = nullptr;
  uint8_t* h_out = nullptr;
  hipGraph_t graph = nullptr;
  hipGraphExec_t graph_exec = nullptr;
  int graph_groups = 0;
  double graph_cam[5] = {};
  bool warm = false;
};

namespace {
constexpr size_t kInPose = 0;  // h_in layout: pose (28 B), n (4 B), pad, obs
constexpr size_t kInN = 28;
constexpr size_t kInObs = 32;
constexpr size_t kOutPose = 0;  // h_out layout: pose (28 B), inliers (4 B), outlier flags
constexpr size_t kOutInl = 28;
constexpr size_t kOutFlags = 32;

hipError_t enqueue_single(orbgpu_pose_ctx* c, const double cd[5]) {
  const size_t obs_bytes = sizeof(orbgpu_pose_obs) * c->max_obs;
  hipError_t e = hipMemcpyAsync(c->d_obs, c->h_in + kInObs, obs_bytes, hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess)
    e = hipMemcpyAsync(c->d_pose, c->h_in + kInPose, sizeof(orbgpu_pose), hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess)
    e = hipMemcpyAsync(c->d_ints, c->h_in + kInN, sizeof(int), hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess)
    e = orbgpu::launch_pose_opt(cd, c->d_pose, c->d_obs, c->d_ints, c->max_obs, 1, c->d_pose + 7,
                                c->d_outlier, c->d_ints + 1, nullptr, c->stream, c->groups_single);
  if (e == hipSuccess)
    e = hipMemcpyAsync(c->h_out + kOutPose, c->d_pose + 7, sizeof(orbgpu_pose), hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess)
    e = hipMemcpyAsync(c->h_out + kOutInl, c->d_ints + 1, sizeof(int), hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess)
    e = hipMemcpyAsync(c->h_out + kOutFlags, c->d_outlier, c->max_obs, hipMemcpyDeviceToHost, c->stream);
  return e;
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
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc(&c->d_obs, sizeof(orbgpu_pose_obs) * max_obs) != hipSuccess ||
      hipMalloc(&c->d_pose, sizeof(float) * 14) != hipSuccess ||
      hipMalloc(&c->d_outlier, max_obs) != hipSuccess ||
      hipMalloc(&c->d_ints, sizeof(int) * 2) != hipSuccess ||
      hipHostMalloc(&c->h_in, kInObs + sizeof(orbgpu_pose_obs) * max_obs) != hipSuccess ||
      hipHostMalloc(&c->h_out, kOutFlags + max_obs) != hipSuccess) {
    orbgpu_pose_ctx_destroy(c);
    return ORBGPU_ERR_DEVICE;
  }
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
  if (c->d_obs) (void)hipFree(c->d_obs);
  if (c->d_pose) (void)hipFree(c->d_pose);
  if (c->d_outlier) (void)hipFree(c->d_outlier);
  if (c->d_ints) (void)hipFree(c->d_ints);
  if (c->graph_exec) (void)hipGraphExecDestroy(c->graph_exec);
  if (c->graph) (void)hipGraphDestroy(c->graph);
  if (c->h_in) (void)hipHostFree(c->h_in);
  if (c->h_out) (void)hipHostFree(c->h_out);
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
  const bool same_graph = c->graph_exec && c->graph_groups == c->groups_single &&
                          memcmp(c->graph_cam, cd, sizeof(cd)) == 0;
  hipError_t e = hipSuccess;
  if (same_graph) {
    e = hipGraphLaunch(c->graph_exec, c->stream);
  } else if (c->warm) {  // second call: capture the chain (LDS opt-ins already done)
    if (c->graph_exec) (void)hipGraphExecDestroy(c->graph_exec);
    if (c->graph) (void)hipGraphDestroy(c->graph);
    c->graph_exec = nullptr;
    c->graph = nullptr;
    e = hipStreamBeginCapture(c->stream, hipStreamCaptureModeRelaxed);
    if (e == hipSuccess) {
      const hipError_t le = enqueue_single(c, cd);
      e = hipStreamEndCapture(c->stream, &c->graph);
      if (e == hipSuccess) e = le;
    }
    if (e == hipSuccess) e = hipGraphInstantiate(&c->graph_exec, c->graph, nullptr, nullptr, 0);
    if (e == hipSuccess) {
      c->graph_groups = c->groups_single;
      memcpy(c->graph_cam, cd, sizeof(cd));
      e = hipGraphLaunch(c->graph_exec, c->stream);
    } else {
      (void)hipGetLastError();
      e = enqueue_single(c, cd);
    }
  } else {
    e = enqueue_single(c, cd);
    c->warm = true;
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
