// Launch descriptor for one batched extraction (device pointers).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "orb_plan.h"

namespace orbgpu {

struct ExtractLaunch {
  const PlanHeader* host_plan;  // host copy (grid sizes)
  const PlanHeader* plan;       // device copy
  const Cell* cells;
  const int* rs_tab;
  const uint8_t* imgs;
  size_t image_pitch;
  int stride;
  int n_images;
  uint8_t* pyr;
  uint8_t* blur;
  uint32_t* slots;
  int* cell_count;
  uint32_t* dense;
  int* knode;
  uint32_t* oct_out;
  int* oct_count;
  float* angle;
  uint64_t* desc;
  size_t octree_lds;
  uint8_t* oct_nodes;  // HBM node arrays (plans with oct_hbm_nodes), else null
  int lap0, lap1;
  void* kps_out;   // orbgpu_keypoint[n_images][cap]
  void* desc_out;  // uint8_t[n_images][cap][32]
  int cap;
  int* n_out;
  int* mono_out;
  int* err;
  int n_cu;            // compute units of the device (persistent grids)
  int pyramid_groups;  // > 0: the resize chain as one k_pyramid launch, this many tile groups a workgroup
  hipEvent_t* events;  // optional: kStages + 1 events recorded around the stages
  hipEvent_t stage_event;  // optional: recorded right after stage stage_event_at (orbgpu_extractor_set_stage_event)
  int stage_event_at;
};

// Stage boundaries recorded when ExtractLaunch::events is set.
enum Stage : int { kStResize, kStBlur, kStFast, kStOctree, kStDescribe, kStAssemble, kStages };

hipError_t launch_extract(const ExtractLaunch& a, hipStream_t st);
hipError_t set_lds_limits(size_t octree_bytes, size_t resize_bytes);
// tile groups of a k_pyramid workgroup for the plan's resize tile LDS (0: none fits)
int pyramid_groups_for(size_t resize_bytes);

}  // namespace orbgpu
