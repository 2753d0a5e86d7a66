// C-ABI implementation of the inertial tracking optimisation
// (orbgpu_pose_inertial*, include/orbgpu.h).
#include <hip/hip_runtime.h>

#include <cstring>
#include <new>

#include "../../include/orbgpu.h"

namespace orbgpu {
hipError_t launch_pose_inertial(int mode, const orbgpu_imu_calib& c, int n_problems,
                                const orbgpu_imu_state* d_cur, const orbgpu_imu_state* d_prev,
                                const orbgpu_imu_preint* d_preint, const orbgpu_imu_prior* d_prior,
                                const orbgpu_inertial_obs* d_obs, const int* d_nobs, int obs_stride,
                                int rec_init, orbgpu_inertial_result* d_res, uint8_t* d_outlier,
                                hipStream_t st);
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
  // single-problem staging: [cur | prev | preint | prior | nobs] then obs, result, outliers
  uint8_t* d_in = nullptr;
  orbgpu_inertial_obs* d_obs = nullptr;
  orbgpu_inertial_result* d_res = nullptr;
  uint8_t* d_out = nullptr;
};

namespace {
constexpr size_t kOffPrev = 136, kOffPreint = 272, kOffPrior = 1336, kOffN = 3304, kInBytes = 3312;
static_assert(kOffPrev >= sizeof(orbgpu_imu_state) && kOffPreint - kOffPrev >= sizeof(orbgpu_imu_state) &&
                  kOffPrior - kOffPreint >= sizeof(orbgpu_imu_preint) &&
                  kOffN - kOffPrior >= sizeof(orbgpu_imu_prior) && kOffPreint % 8 == 0 &&
                  kOffPrior % 8 == 0,
              "staging layout");

bool valid_calib(const orbgpu_imu_calib* c) {
  return c && c->fx > 0 && c->fy > 0;
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
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc(&c->d_in, kInBytes) != hipSuccess ||
      hipMalloc(&c->d_obs, sizeof(orbgpu_inertial_obs) * max_obs) != hipSuccess ||
      hipMalloc(&c->d_res, sizeof(orbgpu_inertial_result)) != hipSuccess ||
      hipMalloc(&c->d_out, max_obs) != hipSuccess) {
    orbgpu_inertial_ctx_destroy(c);
    return ORBGPU_ERR_DEVICE;
  }
  *out = c;
  return ORBGPU_OK;
}

void orbgpu_inertial_ctx_destroy(orbgpu_inertial_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->d_in) (void)hipFree(c->d_in);
  if (c->d_obs) (void)hipFree(c->d_obs);
  if (c->d_res) (void)hipFree(c->d_res);
  if (c->d_out) (void)hipFree(c->d_out);
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
  uint8_t host[kInBytes];
  std::memset(host, 0, sizeof(host));
  std::memcpy(host, cur, sizeof(*cur));
  std::memcpy(host + kOffPrev, prev, sizeof(*prev));
  std::memcpy(host + kOffPreint, preint, sizeof(*preint));
  if (prior) std::memcpy(host + kOffPrior, prior, sizeof(*prior));
  std::memcpy(host + kOffN, &n_obs, sizeof(int));
  hipStream_t st = c->stream;
  if (hipMemcpyAsync(c->d_in, host, kInBytes, hipMemcpyHostToDevice, st) != hipSuccess ||
      (n_obs > 0 && hipMemcpyAsync(c->d_obs, obs, sizeof(*obs) * n_obs, hipMemcpyHostToDevice,
                                   st) != hipSuccess))
    return ORBGPU_ERR_DEVICE;
  const auto* d_cur = reinterpret_cast<const orbgpu_imu_state*>(c->d_in);
  const auto* d_prev = reinterpret_cast<const orbgpu_imu_state*>(c->d_in + kOffPrev);
  const auto* d_pre = reinterpret_cast<const orbgpu_imu_preint*>(c->d_in + kOffPreint);
  const auto* d_pri = reinterpret_cast<const orbgpu_imu_prior*>(c->d_in + kOffPrior);
  const auto* d_n = reinterpret_cast<const int*>(c->d_in + kOffN);
  if (orbgpu::launch_pose_inertial(mode, *calib, 1, d_cur, d_prev, d_pre, d_pri, c->d_obs, d_n,
                                   c->max_obs, rec_init, c->d_res, c->d_out, st) != hipSuccess)
    return ORBGPU_ERR_DEVICE;
  if (hipMemcpyAsync(res, c->d_res, sizeof(*res), hipMemcpyDeviceToHost, st) != hipSuccess ||
      (n_obs > 0 &&
       hipMemcpyAsync(outlier, c->d_out, n_obs, hipMemcpyDeviceToHost, st) != hipSuccess) ||
      hipStreamSynchronize(st) != hipSuccess)
    return ORBGPU_ERR_DEVICE;
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
