// Launch descriptor for one batched extraction (device pointers).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <vector>

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

// ---- the single-image host path as ONE dataflow launch (k_extract_df) ----
// Work items (one 32-bit word each: type | level << 4 | index << 8), in the
// ticket order the workers take them; an item depends only on items of
// smaller tickets, so a worker that holds a ticket always finds its
// producers running or done (no residency assumption).
enum DfType : int { kDfCopy, kDfResize, kDfFast, kDfBlur, kDfOctree, kDfDescribe, kDfMirror };
// Counters in the handle's control block, one 128-B line each; zero at the
// start of every launch (the last workgroup to leave resets them).
enum DfCounter : int {
  kDfTicket = 0, kDfExit = 1, kDfImg = 2,
  kDfLvl = 3,                       // + level: resize units done (levels >= 1)
  kDfFastDone = kDfLvl + kMaxLevels,  // + level: FAST items done
  kDfBlurDone = kDfFastDone + kMaxLevels,
  kDfOctDone = kDfBlurDone + kMaxLevels,
  kDfDescDone = kDfOctDone + kMaxLevels,
  kDfDescLvl,                        // + level: describe items of level l done
  kDfMirrorDone = kDfDescLvl + kMaxLevels,
  kDfCounters
};
constexpr int kDfCtrStride = 32;  // ints between counters (128 B)
constexpr int kDfBandBytes = 12288;  // image bytes per copy item (a multiple of 16)

struct DfPlan {  // per (plan, image size): the item list's shape
  int n_items, n_bands, img_bytes;
  int units[kMaxLevels];       // resize tiles + tail blocks of level l (l >= 1)
  int fast_items[kMaxLevels];  // 4 cells an item
  int blur_items[kMaxLevels];  // blur tiles of level l
  int desc_items;              // 4 keypoint slots an item, all levels
  int lds_bytes;               // dynamic LDS of a worker
};

struct DfLaunch {
  const PlanHeader* plan;
  const Cell* cells;
  const int* rs_tab;
  const uint32_t* items;
  int* ctrl;                 // kDfCounters * kDfCtrStride ints
  const uint8_t* img_host;   // the image in pinned host memory (device view), rows at lev[0].pitch
  uint8_t* img;              // its device copy (level 0 of the pyramid)
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
  int lap0, lap1;             // (plans with oct_hbm_nodes take the per-stage launches)
  void* kps_out;             // device output block (as ExtractLaunch)
  void* desc_out;
  int* nm;                   // n, mono, err (device)
  void* kps_host;            // host-mapped mirrors of the same three
  void* desc_host;
  int* nm_host;
  int* done_host;            // host-mapped word: the call's sequence number once every output is written
  int cap;
  int grid;                  // workers
  DfPlan df;
  unsigned long long* trace;  // optional (ORBGPU_DF_TRACE): per ticket {grab, ready, done, item | hw ids}
};

// host planner (orb_plan.cpp): the item list of a plan
void make_df_items(const PlanHeader& P, int img_bytes, DfPlan& df, std::vector<uint32_t>& items);
size_t df_lds_bytes(const PlanHeader& P, size_t octree_lds);
// a: the host copy (grid, LDS); a_dev: the same record in device memory (read by
// the workers); band_flags: one int per copy band in host-mapped memory, which
// the host sets to `seq` once the band's bytes are in a.img_host
hipError_t launch_extract_df(const DfLaunch& a, const DfLaunch* a_dev, const int* band_flags, int seq,
                             hipStream_t st);
hipError_t set_df_lds_limit(size_t bytes);

// Stage boundaries recorded when ExtractLaunch::events is set.
enum Stage : int { kStResize, kStBlur, kStFast, kStOctree, kStDescribe, kStAssemble, kStages };

hipError_t launch_extract(const ExtractLaunch& a, hipStream_t st);
hipError_t set_lds_limits(size_t octree_bytes, size_t resize_bytes);
// tile groups of a k_pyramid workgroup for the plan's resize tile LDS (0: none fits)
int pyramid_groups_for(size_t resize_bytes);

}  // namespace orbgpu
