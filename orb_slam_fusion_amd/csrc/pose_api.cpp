// C-ABI implementation of the pose-only optimisation half of include/orbgpu.h.
#include <hip/hip_runtime.h>

#include <cstdlib>
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
};

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
      hipMalloc(&c->d_ints, sizeof(int) * 2) != hipSuccess) {
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
  int ints[2] = {n_obs, 0};
  if ((n_obs > 0 && hipMemcpyAsync(c->d_obs, obs, sizeof(orbgpu_pose_obs) * n_obs,
                                   hipMemcpyHostToDevice, c->stream)) ||
      hipMemcpyAsync(c->d_pose, Tcw_in, sizeof(orbgpu_pose), hipMemcpyHostToDevice, c->stream) ||
      hipMemcpyAsync(c->d_ints, ints, sizeof(int), hipMemcpyHostToDevice, c->stream))
    return ORBGPU_ERR_DEVICE;
  if (orbgpu::launch_pose_opt(cd, c->d_pose, c->d_obs, c->d_ints, c->max_obs, 1, c->d_pose + 7,
                              c->d_outlier, c->d_ints + 1, nullptr, c->stream,
                              c->groups_single) != hipSuccess)
    return ORBGPU_ERR_DEVICE;
  if (hipMemcpyAsync(Tcw_out, c->d_pose + 7, sizeof(orbgpu_pose), hipMemcpyDeviceToHost,
                     c->stream) ||
      hipMemcpyAsync(ints, c->d_ints, sizeof(ints), hipMemcpyDeviceToHost, c->stream) ||
      (n_obs > 0 &&
       hipMemcpyAsync(outlier, c->d_outlier, n_obs, hipMemcpyDeviceToHost, c->stream)) ||
      hipStreamSynchronize(c->stream))
    return ORBGPU_ERR_DEVICE;
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
