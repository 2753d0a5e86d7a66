// Launch descriptor of the ORBmatcher projection searches
// (orb_matcher.cc:42-206, 1518-1728, 1730-1839) over a batch of frames.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/orbgpu.h"

namespace orbgpu {

constexpr int kGridCols = ORBGPU_FRAME_GRID_COLS, kGridRows = ORBGPU_FRAME_GRID_ROWS;
constexpr int kGridCells = kGridCols * kGridRows;
constexpr int kMatchMaxKeypoints = 8192;  // per frame (LDS-resident claim state)
constexpr int kMatchMaxPoints = 1 << 20;  // per frame
// Per query the search keeps its kMatchTopK best candidates (in the
// reference's order) plus the candidate count: claims by earlier queries are
// then resolved from the list, a full re-search only when it runs out.
constexpr int kMatchTopK = 6;
constexpr int kMatchResWords = kMatchTopK + 1;

// kModeLast: SearchByProjection(CurrentFrame, LastFrame); kModeLocal /
// kModeLocalFrustum: SearchByProjection(F, vpMapPoints) (with isInFrustum);
// kModeKeyFrame: SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th,
// ORBdist) of Relocalization.
enum MatchMode : int { kModeLast = 0, kModeLocal = 1, kModeLocalFrustum = 2, kModeKeyFrame = 3 };

// Everything scalar the searches read (passed by value).
struct MatchParams {
  float min_x, max_x, min_y, max_y;
  float inv_w, inv_h;  // FRAME_GRID_COLS / (mnMaxX - mnMinX), ROWS / (mnMaxY - mnMinY)
  int n_levels;
  float scale[ORBGPU_MAX_LEVELS];
  // MapPoint::PredictScale as thresholds: level = #{j >= 1 : ratio >= thr[j-1]}
  // (host-computed from the reference's ::log(double), see match_api.cpp)
  float level_thr[ORBGPU_MAX_LEVELS];
  float fx, fy, cx, cy, bf, mb;
  float th, nn_ratio, th_far, cos_limit;
  int mono, check_ori, far_points;
  int orb_dist;  // kModeKeyFrame: accept bestDist <= ORBdist
};

struct MatchLaunch {
  MatchParams p;
  int mode;
  int n_frames;
  // current frames: frame f's arrays start at f * kp_stride (keypoints)
  const float* kps;  // orbgpu_keypoint rows (7 x 4 bytes)
  const uint8_t* desc;
  const float* uright;     // may be null
  const uint8_t* claimed;  // may be null
  const int* n;            // keypoints per frame (device)
  int kp_stride;
  // queries: frame f's points start at f * pt_stride
  const orbgpu_proj_point* ppts;  // kModeLast
  const orbgpu_map_point* mpts;   // kModeLocal*, kModeKeyFrame (the key frame's points)
  const float* q_angle;           // kModeKeyFrame: pKF->mvKeysUn[i].angle per point
  orbgpu_track_view* views;       // kModeLocal*: read (kModeLocal) / written (kModeLocalFrustum)
  // kModeLocalFrustum: prior field values for the ones isInFrustum does not
  // write (null: views itself, updated in place)
  const orbgpu_track_view* views_init;
  const int* npts;                // points per frame (device)
  int pt_stride;
  int max_pts;                    // max over frames of npts (grid sizing)
  const orbgpu_pose* Tcw;         // kModeLast, kModeKeyFrame: [n_frames]
  const orbgpu_pose* Tlw;
  // Rcw (row-major), tcw, Ow per frame, 15 floats: kModeLocalFrustum
  const float* frustum_pose;
  // scratch
  int* cell_start;      // [n_frames][kGridCells + 1]
  uint16_t* cell_idx;   // [n_frames][kp_stride]
  uint32_t* res;        // [n_frames][pt_stride][kMatchResWords]: top-K (dist << 16 | idx), count
  int32_t* acc;         // [n_frames][pt_stride]: accepted idx | bin << 16, or -1
  // outputs
  int32_t* match;       // [n_frames][kp_stride]
  int* nmatches;        // [n_frames]
  int* err;
  int zero_err;         // k_mt_grid stores err (a one-frame call's own word) instead of OR-ing into it
  // one-frame host call: k_mt_resolve copies the output range [mirror_src,
  // + mirror_bytes) of the device arena (error word, match row, count, views)
  // into the host-mapped arena, then stores seq into done_host (the host
  // polls it: no copy command, no stream synchronisation)
  const uint8_t* mirror_src;
  uint8_t* mirror_dst;
  int mirror_bytes;
  int* done_host;
  int seq;
};

hipError_t launch_match(const MatchLaunch& a, hipStream_t st);

// matches -> PoseOptimization observations (optimizer.cc:806-877)
struct ObsLaunch {
  int n_frames;
  const float* kps;       // orbgpu_keypoint rows, frame f at f * kp_stride
  const float* uright;    // may be null (every edge monocular)
  const int32_t* match;   // [n_frames][kp_stride]
  const int* n;
  int kp_stride;
  const orbgpu_proj_point* pts;
  int pt_stride;
  float inv_sigma2[ORBGPU_MAX_LEVELS];  // Frame::mvInvLevelSigma2
  orbgpu_pose_obs* obs;   // [n_frames][obs_stride] (or, iobs set, unused)
  orbgpu_inertial_obs* iobs;  // PoseInertialOptimization rows instead of obs
  const uint8_t* close;       // per point (pt_stride rows), mTrackDepth < 10; may be null
  int obs_stride;
  int* nobs;
  int32_t* obs_index;     // may be null
  int* err;
};

hipError_t launch_pose_obs(const ObsLaunch& a, hipStream_t st);

// ORBmatcher::SearchByBoW(KeyFrame*, Frame&, vector<MapPoint*>&) over a batch
// of (key frame, frame) pairs; FeatureVectors as orbgpu_bow_transform_batch
// writes them (ascending node ids, CSR feature lists).
struct BowSearchLaunch {
  int n_frames;
  float nn_ratio;
  int check_ori;
  const uint32_t* kf_nodes;    // [n_frames][kf_stride]
  const int32_t* kf_off;       // [n_frames][kf_stride + 1]
  const uint32_t* kf_feat;     // [n_frames][kf_stride]
  const int* kf_n_nodes;       // [n_frames]
  const uint8_t* kf_desc;      // [n_frames][kf_stride][32]
  const float* kf_angle;       // [n_frames][kf_stride]
  const uint8_t* kf_valid;     // [n_frames][kf_stride]
  int kf_stride;
  const uint32_t* f_nodes;     // [n_frames][f_stride]
  const int32_t* f_off;
  const uint32_t* f_feat;
  const int* f_n_nodes;
  const uint8_t* f_desc;       // [n_frames][f_stride][32]
  const float* f_angle;        // frame f keypoint k at f_angle[(f * f_stride + k) * angle_step]
  int angle_step;              // 1 (float array) or 7 (orbgpu_keypoint rows, &kps->angle)
  const int* f_n;              // keypoints per frame
  int f_stride;
  int32_t* match;              // [n_frames][f_stride]
  int* nmatches;
  int* err;
};

hipError_t launch_bow_search(const BowSearchLaunch& a, hipStream_t st);

// Frame::UnprojectStereo over the frames' stereo keypoints -> LastFrame points
struct UnprojLaunch {
  int n_frames;
  float fx, fy, cx, cy;
  const orbgpu_pose* Tcw;  // [n_frames]
  const float* kps;        // orbgpu_keypoint rows, frame f at f * kp_stride
  const uint8_t* desc;
  const float* depth;      // mvDepth
  const int* n;
  int kp_stride;
  orbgpu_proj_point* pts;  // [n_frames][pt_stride]
  int pt_stride;
  int* npts;
  int* err;
};

hipError_t launch_unproject(const UnprojLaunch& a, hipStream_t st);

}  // namespace orbgpu
