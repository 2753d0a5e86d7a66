// Launch descriptor of the stereo matcher (Frame::ComputeStereoMatches,
// frame.cc:828-986) over extractor outputs that stay resident on the device.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "orb_plan.h"

namespace orbgpu {

// One side (left or right image) of n_frames stereo frames: frame f's level-0
// plane, pyramid block, keypoints (orbgpu_keypoint), descriptors and count
// sit at base + f * (frame stride).
struct StereoSide {
  const uint8_t* img0;
  size_t img_fstride;  // bytes between frames' level-0 planes
  int img_stride;      // bytes between level-0 rows
  const uint8_t* pyr;  // levels >= 1 (PlanHeader offsets / pitches)
  size_t pyr_fstride;
  const float* kps;    // orbgpu_keypoint rows (7 x 4 bytes)
  size_t kp_fstride;   // keypoints between frames
  const uint8_t* desc;  // 32 bytes per keypoint, same frame stride as kps
  const int* n;
  int n_fstride;
};

struct StereoLaunch {
  const PlanHeader* plan;  // device copy
  int n_frames, cap;       // frames; keypoint capacity per image
  int rows;                // level-0 height (row table size)
  int list_cap;            // row-list entries per frame
  StereoSide L, R;
  float bf, mb;
  float* uright;  // [n_frames][cap]
  float* depth;
  size_t out_fstride;
  uint16_t* lists;  // [n_frames][list_cap] right keypoint indices by row
  int* row_end;     // [n_frames][rows] end offset of each row's list
  int* sad;         // [n_frames][cap] window distance of kept matches, else -1
  int* err;
  // one-frame host call (orbgpu_stereo_match): k_stereo_rows stores the
  // call's error word (no memset before it); k_stereo_median copies the
  // output range [mirror_src, + mirror_bytes) into host-mapped memory and then
  // stores seq into done_host (the host polls it: no copy, no stream sync)
  int zero_err;
  const uint8_t* mirror_src;
  uint8_t* mirror_dst;
  int mirror_bytes;
  int* done_host;
  int seq;
};

hipError_t launch_stereo(const StereoLaunch& a, hipStream_t st);

}  // namespace orbgpu
