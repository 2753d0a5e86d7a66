/*
 * orbgpu -- MI355X (gfx950) ORB front-end and pose/bundle-adjustment back-end.
 *
 * C ABI: plain pointers, sizes and POD structs; integer status codes; one
 * handle per calling thread (each owns its HIP stream and workspace); no global
 * mutable state.  Every entry point below names the reference interface it
 * replaces (paths under J094/orb_slam_fusion).
 */
#ifndef ORBGPU_H
#define ORBGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int orbgpu_status;
#define ORBGPU_OK 0
#define ORBGPU_ERR_INVALID (-1)  /* bad argument / unsupported geometry        */
#define ORBGPU_ERR_EMPTY (-2)    /* empty image: reference operator() returns -1 */
#define ORBGPU_ERR_CAPACITY (-3) /* caller buffer or internal bound too small  */
#define ORBGPU_ERR_DEVICE (-4)   /* HIP runtime error                          */
#define ORBGPU_ERR_NOMEM (-5)     /* device or pinned host memory exhausted   */

/* OrbExtractor(int num_feats, float scale_factor, int num_levs,
 *              int ini_th_fast, int min_th_fast)
 *   include/cam/orb_feature/orb_extractor.h:48-49, orb_extractor.cc:407-465 */
typedef struct orbgpu_orb_params {
  int num_features;
  float scale_factor;
  int num_levels;
  int ini_th_fast;
  int min_th_fast;
} orbgpu_orb_params;

/* Field order and size (28 B) of cv::KeyPoint {pt.x, pt.y, size, angle,
 * response, octave, class_id}: the shim copies these straight into the
 * caller's std::vector<cv::KeyPoint>. */
typedef struct orbgpu_keypoint {
  float x, y, size, angle, response;
  int32_t octave, class_id;
} orbgpu_keypoint;

typedef struct orbgpu_extractor orbgpu_extractor;

/* Creates an extractor bound to `device` with workspace for batches of up to
 * `max_images` images of at most max_width x max_height.
 * Replaces: OrbExtractor::OrbExtractor (orb_extractor.cc:407). */
orbgpu_status orbgpu_extractor_create(const orbgpu_orb_params* params, int device, int max_width,
                                      int max_height, int max_images, orbgpu_extractor** out);
void orbgpu_extractor_destroy(orbgpu_extractor* h);

/* Scale tables, `num_levels` floats each (any pointer may be NULL).
 * Replaces: GetScaleFactors / GetInverseScaleFactors / GetScaleSigmaSquares /
 * GetInverseScaleSigmaSquares (orb_extractor.h:60-74). */
orbgpu_status orbgpu_extractor_scales(const orbgpu_extractor* h, float* scale, float* inv_scale,
                                      float* sigma2, float* inv_sigma2);
int orbgpu_extractor_levels(const orbgpu_extractor* h);
/* The resize vertical pass's rounding (the least certain OpenCV
 * rule: which columns take VResizeLinearVec_32s8u's SIMD rounding depends on
 * the OpenCV build).  ORBGPU_RESIZE_SSE (default): OpenCV 4.5.4 with 128-bit
 * universal intrinsics -- 16-lane blocks while x <= w-16, 8-lane blocks while
 * x < w-8, FixedPtCast<int, uchar, 22> after; ORBGPU_RESIZE_SCALAR: every
 * column FixedPtCast (a build without the vectorised pass).  Re-plans the
 * handle; pinning parity against a real OpenCV is this one switch. */
#define ORBGPU_RESIZE_SSE 0
#define ORBGPU_RESIZE_SCALAR 1
orbgpu_status orbgpu_extractor_set_resize_rounding(orbgpu_extractor* h, int mode);

/* Stage signal for pipelining batch extractions across streams: every later
 * orbgpu_extract_batch on this handle records `hip_event` (a hipEvent_t the
 * caller owns) on its stream right after `stage` -- 0 pyramid, 1 blur,
 * 2 FAST, 3 octree, 4 describe, 5 assembly -- so another stream can start
 * its own batch when this one is part-way (NULL: no signal).  bench.py
 * offsets its two extractor pipelines this way: one's VALU-bound stages
 * (pyramid, blur, FAST) then run beside the other's latency-bound ones. */
orbgpu_status orbgpu_extractor_set_stage_event(orbgpu_extractor* h, int stage, void* hip_event);

/* How the pyramid's resize chain is launched (same bytes either way):
 * ORBGPU_PYRAMID_PER_LEVEL (default) one launch per level over the whole
 * device; ORBGPU_PYRAMID_FUSED one launch, a workgroup per image walking the
 * levels (k_pyramid; slower at every measured batch, kept for A/B).  The
 * environment variable ORBGPU_RESIZE=fused sets the default at creation. */
#define ORBGPU_PYRAMID_PER_LEVEL 0
#define ORBGPU_PYRAMID_FUSED 1
orbgpu_status orbgpu_extractor_set_pyramid_launch(orbgpu_extractor* h, int mode);

/* How orbgpu_extract (one image from host buffers: the reference's
 * per-frame call) runs on the device (same bytes either way):
 * ORBGPU_SINGLE_DATAFLOW (default) ONE launch whose persistent workers take
 * the stages' work items by ticket, each item waiting only for the items it
 * reads (level 0's FAST and octree start while the resize chain runs), the
 * image read from pinned host memory and the outputs written back to it by
 * the launch itself; ORBGPU_SINGLE_GRAPH the batch path's per-stage launches
 * with two copies, replayed as a hipGraph.  Plans whose octree nodes live in
 * HBM always take the per-stage launches.  The environment variable
 * ORBGPU_SINGLE=graph sets the default at creation. */
#define ORBGPU_SINGLE_DATAFLOW 0
#define ORBGPU_SINGLE_GRAPH 1
orbgpu_status orbgpu_extractor_set_single_launch(orbgpu_extractor* h, int mode);

/* Where DistributeOctTree's node list lives (orb_extractor.cc:542-742; the
 * reference's std::list has no bound, and neither does its per-level budget,
 * :432-444).  ORBGPU_OCTREE_NODES_AUTO (default): in LDS whenever the plan's
 * node capacity fits a workgroup's 160 KB, else in HBM -- every num_features
 * the reference accepts, e.g. OrbExtractor(5 * nFeatures, ...) at
 * tracking.cc:202-204,811-813.  ORBGPU_OCTREE_NODES_HBM: always in HBM (same
 * results; the test switch for the large-plan path).  Re-plans the handle. */
#define ORBGPU_OCTREE_NODES_AUTO 0
#define ORBGPU_OCTREE_NODES_HBM 1
orbgpu_status orbgpu_extractor_set_octree_nodes(orbgpu_extractor* h, int mode);

/* Host-only plan probe (no device call): whether (params, width x height) is
 * a geometry the extractor accepts (ORBGPU_OK) -- every one whose pyramid
 * levels hold the FAST grid (orb_extractor.cc:748-760: a level narrower than
 * 2 * 16 + 35 px divides by a zero cell count in the reference) -- with the
 * per-image keypoint slots and whether the octree nodes go to HBM. */
orbgpu_status orbgpu_extractor_plan(const orbgpu_orb_params* params, int width, int height,
                                    int* kp_slots, int* octree_hbm);

/* Upper bound on keypoints one image can produce at the given geometry. */
int orbgpu_extractor_max_keypoints(orbgpu_extractor* h, int width, int height);

/* Host-buffer extraction of one grayscale 8-bit image.
 * Replaces: int OrbExtractor::operator()(InputArray img, InputArray msk,
 *   vector<KeyPoint>& kps, OutputArray descs, vector<int>& lapping_areas)
 *   (orb_extractor.h:56-58, orb_extractor.cc:1011-1091).
 * Writes n keypoints and n x 32 descriptor bytes (row i = keypoint i) when
 * n <= cap; *n_out always receives n.  *mono_out receives operator()'s return
 * value (keypoints with lapping[0] <= x <= lapping[1] fill the tail in reverse
 * order, the rest the head).  Empty image -> ORBGPU_ERR_EMPTY (reference: -1).
 * The mask argument of the reference is ignored there too (orb_extractor.h:54). */
orbgpu_status orbgpu_extract(orbgpu_extractor* h, const uint8_t* img, int width, int height,
                             int stride, const int lapping[2], orbgpu_keypoint* kps,
                             uint8_t* descs, int cap, int* n_out, int* mono_out);

/* Both images of a stereo frame from ONE host thread: the two handles'
 * extractions (each exactly orbgpu_extract on its image, outputs and errors
 * included) are in flight together on the handles' own streams.  Replaces the
 * two std::thread ExtractORB calls of the stereo Frame constructor
 * (frame.cc:179-182, ExtractORB :467-476): on the GPU the host threads buy no
 * parallelism and each costs a thread start per frame.  `left` and `right`
 * must be different handles; returns the left status if it is not OK, else
 * the right one. */
orbgpu_status orbgpu_extract_stereo(orbgpu_extractor* left, orbgpu_extractor* right, const uint8_t* img_left,
                                    const uint8_t* img_right, int width, int height, int stride,
                                    const int lapping_left[2], const int lapping_right[2],
                                    orbgpu_keypoint* kps_left, uint8_t* descs_left, int cap_left,
                                    int* n_left, int* mono_left, orbgpu_keypoint* kps_right,
                                    uint8_t* descs_right, int cap_right, int* n_right, int* mono_right);

/* Host copy of pyramid level `level` from the last orbgpu_extract call
 * (rows *stride bytes apart, *stride >= *width).  Replaces the public member
 * std::vector<cv::Mat> img_pyramid_ (orb_extractor.h:76) read by
 * Frame::ComputeStereoMatches (frame.cc:834,913-933).  The pointer stays valid
 * until the next extract/destroy on this handle. */
orbgpu_status orbgpu_extractor_pyramid_level(orbgpu_extractor* h, int level, const uint8_t** data,
                                             int* width, int* height, int* stride);

/* Device-resident batched extraction: n_images images at d_imgs + i*image_pitch
 * (row stride `stride`), all in device memory; outputs go to device buffers
 * d_kps[n_images][cap_per_image], d_descs[n_images][cap_per_image][32],
 * d_n[n_images], d_mono[n_images].  Asynchronous on `hip_stream` (NULL = the
 * handle's own stream).  This is the throughput path: N stereo frames ->
 * 2N images per call, one HIP-graph-friendly launch sequence. */
orbgpu_status orbgpu_extract_batch(orbgpu_extractor* h, const uint8_t* d_imgs, int n_images,
                                   int width, int height, int stride, size_t image_pitch,
                                   const int lapping[2], orbgpu_keypoint* d_kps, uint8_t* d_descs,
                                   int cap_per_image, int* d_n, int* d_mono, void* hip_stream);

/* ------------------------------------------------------------------------ */
/* Stereo matching (rectified pinhole stereo).
 * Replaces: void Frame::ComputeStereoMatches() (include/map/frame.h,
 *   src/map/frame.cc:828-986), called by the stereo Frame constructor after
 *   both ExtractORB calls (frame.cc:179-189).  Per left keypoint i: uright[i] =
 *   Frame::mvuRight[i], depth[i] = Frame::mvDepth[i] (-1 when unmatched).
 *   bf = Frame::bf_ (mbf), mb = Frame::mb (bf / fx); TH_HIGH / TH_LOW =
 *   100 / 50 (orb_matcher.cc:35-36).  Window reads beyond a level follow the
 *   reference's reflect-101 padded pyramid storage (orb_extractor.cc:1105-1114).
 *   A frame whose match list ends up empty is left as matched (the reference
 *   reads the median of an empty vector there, frame.cc:966).
 *
 * Batch: the handle's last orbgpu_extract_batch call took 2 * n_frames images
 *   ordered [left 0, right 0, left 1, right 1, ...]; d_imgs / stride /
 *   image_pitch are that call's level-0 planes and d_kps / d_descs /
 *   cap_per_image / d_n its outputs, all still on the device.  Writes
 *   d_uright / d_depth as [n_frames][cap_per_image] floats, stream-ordered on
 *   hip_stream (NULL: the handle's stream).  cap_per_image <= 65535 (the row
 *   lists and match keys hold 16-bit keypoint indices; larger: INVALID). */
orbgpu_status orbgpu_stereo_match_batch(orbgpu_extractor* h, int n_frames, const uint8_t* d_imgs,
                                        int stride, size_t image_pitch, const orbgpu_keypoint* d_kps,
                                        const uint8_t* d_descs, int cap_per_image, const int* d_n,
                                        float bf, float mb, float* d_uright, float* d_depth,
                                        void* hip_stream);

/* Host path: `left` / `right` are the Frame's two extractors
 *   (mpORBextractorLeft / Right) right after their orbgpu_extract calls on the
 *   frame's images (same parameters and size); their keypoints, descriptors
 *   and pyramids are used where they lie on the device.  Writes N = the left
 *   call's keypoint count floats to uright / depth (host), N <= cap.  Plans
 *   with more than 65535 keypoint slots are refused (INVALID), as the batch. */
orbgpu_status orbgpu_stereo_match(orbgpu_extractor* left, orbgpu_extractor* right, float bf,
                                  float mb, float* uright, float* depth, int cap);

/* Synchronises the handle's last batch and returns the first device-side
 * error (ORBGPU_ERR_CAPACITY when an internal bound was hit), else ORBGPU_OK. */
orbgpu_status orbgpu_extractor_check(orbgpu_extractor* h);

/* Per-stage timing of the next `max_calls` orbgpu_extract_batch calls with
 * HIP events recorded on the launch stream between the kernel stages
 * (0 resize, 1 blur, 2 FAST cells, 3 octree, 4 describe, 5 assemble).
 * orbgpu_extractor_profile_read waits for them, writes the summed
 * milliseconds per stage (6 doubles) and returns the number of calls timed. */
orbgpu_status orbgpu_extractor_profile(orbgpu_extractor* h, int max_calls);
int orbgpu_extractor_profile_read(orbgpu_extractor* h, double* ms_per_stage);

/* Diagnostics: internal stage buffers of image 0 of the last call (used by
 * the parity tests to localise a mismatch).  which = 0: blurred level plane
 * (w*h bytes); 1: FAST candidates of the level in the reference's to_dist
 * order; 2: octree output in node-list order.  Candidates are uint32
 * x | y << 12 | response << 24 (coordinates relative to the 16-px FAST
 * border).  Returns the element count, or -1. */
int orbgpu_extractor_stage(orbgpu_extractor* h, int which, int level, void* out, int cap);

/* ------------------------------------------------------------------------ */
/* Pose-only optimisation.
 * Replaces: static int Optimizer::PoseOptimization(Frame* pFrame)
 *   (include/solver/g2o_solver/optimizer.h:64, optimizer.cc:762-1051),
 *   pinhole rig (pFrame->cam2_ == NULL).  The shim flattens the Frame: one
 *   observation per i with pFrame->mvpMapPoints[i] != NULL, in index order. */
typedef struct orbgpu_camera {
  float fx, fy, cx, cy, bf; /* Frame::fx, fy, cx, cy, bf_ */
} orbgpu_camera;

typedef struct orbgpu_pose {
  float qx, qy, qz, qw; /* Tcw.unit_quaternion()  */
  float tx, ty, tz;     /* Tcw.translation()      */
} orbgpu_pose;

typedef struct orbgpu_pose_obs {
  float Xw[3];      /* MapPoint::GetWorldPos()                           */
  float u, v;       /* mvKeysUn[i].pt                                    */
  float ur;         /* mvuRight[i]; < 0 -> monocular edge                */
  float inv_sigma2; /* mvInvLevelSigma2[mvKeysUn[i].octave]              */
} orbgpu_pose_obs;

typedef struct orbgpu_pose_ctx orbgpu_pose_ctx;

orbgpu_status orbgpu_pose_ctx_create(int device, int max_problems, int max_obs,
                                     orbgpu_pose_ctx** out);
void orbgpu_pose_ctx_destroy(orbgpu_pose_ctx* c);

/* One problem from host buffers.  Writes the optimised pose (SetPose), the
 * per-observation outlier flags (mvbOutlier) and returns the inlier count in
 * *n_inliers (PoseOptimization's return value; 0 and pose unchanged when
 * n_obs < 3). */
orbgpu_status orbgpu_pose_opt(orbgpu_pose_ctx* c, const orbgpu_camera* cam,
                              const orbgpu_pose* Tcw_in, const orbgpu_pose_obs* obs, int n_obs,
                              orbgpu_pose* Tcw_out, uint8_t* outlier, int* n_inliers);

/* Device-resident batch: problem p uses d_obs[p*obs_stride .. +d_nobs[p]),
 * one shared camera.  Asynchronous on `hip_stream` (NULL = the context's
 * stream).  d_pose_out_d (optional) receives the 7 double-precision pose
 * components before the float cast. */
orbgpu_status orbgpu_pose_opt_batch(orbgpu_pose_ctx* c, const orbgpu_camera* cam,
                                    const orbgpu_pose* d_Tcw_in, const orbgpu_pose_obs* d_obs,
                                    const int* d_nobs, int obs_stride, int n_problems,
                                    orbgpu_pose* d_Tcw_out, uint8_t* d_outlier, int* d_inliers,
                                    double* d_pose_out_d, void* hip_stream);

/* Speculative LM trials: g2o retries a rejected step with lambda *= ni,
 * ni *= 2 on the same system, so `groups` (1 or 2) trial sweeps of an
 * iteration can run side by side, the outcomes scanned in trial order (same
 * path).  Defaults 1 / 1; the sweeps are issue-bound inside one CU, so two
 * groups cut the serial trial rounds (42.6 -> 28.9 per problem) but not the
 * time -- kept as an option. */
orbgpu_status orbgpu_pose_ctx_set_trial_groups(orbgpu_pose_ctx* c, int groups_single,
                                               int groups_batch);

/* ------------------------------------------------------------------------
 * LocalBundleAdjustment -- replaces the solve of
 * Optimizer::LocalBundleAdjustment(KeyFrame*, bool* pbStopFlag, Map*, int&,
 * int&, int&, int&) (optimizer.h:66-68, optimizer.cc:1053-1441): the caller
 * gathers the window as the reference does (:1057-1124: local keyframes,
 * their map points, fixed keyframes) and hands over the graph; the library
 * runs optimize(iterations) (g2o LM, BlockSolver_6_3 Schur complement on the
 * points, :1359-1360) and the outlier test (:1362-1400); the caller erases
 * the flagged observations under Map::mMutexMapUpdate and writes poses and
 * points back (:1402-1441).
 * ------------------------------------------------------------------------ */
typedef struct orbgpu_lba_edge {
  int32_t point;    /* map point index (vertex id MP.id_ + maxKFid + 1 -> 0..n_pts-1)     */
  int32_t kf;       /* keyframe index (vertex id KF.id_ -> 0..n_kf-1)                      */
  float u, v;       /* mvKeysUn[leftIndex].pt                                              */
  float ur;         /* mvuRight[leftIndex]; < 0 -> EdgeSE3ProjectXYZ (mono, :1248-1274),
                       else g2o::EdgeStereoSE3ProjectXYZ (:1275-1310)                      */
  float inv_sigma2; /* mvInvLevelSigma2[kpUn.octave]                                       */
} orbgpu_lba_edge;

typedef struct orbgpu_lba_ctx orbgpu_lba_ctx;

/* Completes a point-sharded reduction across ranks: called on
 * the host thread with a device buffer of n doubles (stream-synchronized),
 * op 0 = sum, 1 = max; must leave the reduced values in the buffer before
 * returning (e.g. an RCCL all-reduce + stream sync).  Returns 0 on success. */
typedef int (*orbgpu_lba_reduce_fn)(void* user, double* d_buf, int n, int op, void* hip_stream);

orbgpu_status orbgpu_lba_ctx_create(int device, orbgpu_lba_ctx** out);
void orbgpu_lba_ctx_destroy(orbgpu_lba_ctx* c);

/* Stream-ordered reductions for the point-sharded call (ordered != 0): the
 * reduce callback then only ENQUEUES its all-reduce on the hip_stream it is
 * given (e.g. ncclAllReduce / an RCCL all-reduce on that stream) and returns
 * without waiting, and the whole LM loop stays on the device as in the
 * one-rank call: no host synchronisation inside orbgpu_lba_optimize but the
 * final copy.  Every rank enqueues the same kernel + collective sequence
 * (4 all-reduces per LM trial: the pose diagonal (sum) and the point maximum
 * (max) for lambda init, [S | b_s | b_p] (sum), [chi2, scale, failures, stop]
 * (sum)), and the same number of trials, so the collectives stay matched. */
orbgpu_status orbgpu_lba_ctx_set_reduce_ordered(orbgpu_lba_ctx* c, int ordered);

/* The reduced-camera-system path (default AUTO: by size, see below).  LDS:
 * packed tiles in one workgroup's LDS; BLOCK: one workgroup, the matrix in
 * HBM; GRID: tile steps over the whole device.  A forced path a window does
 * not fit returns ORBGPU_ERR_CAPACITY from the optimise call.  BLOCK and GRID
 * perform the same tile operations in the same order (identical results). */
#define ORBGPU_LBA_SOLVER_AUTO (-1)
#define ORBGPU_LBA_SOLVER_LDS 0
#define ORBGPU_LBA_SOLVER_BLOCK 1
#define ORBGPU_LBA_SOLVER_GRID 2
orbgpu_status orbgpu_lba_ctx_set_solver(orbgpu_lba_ctx* c, int solver);

/* The Schur complement's path (identical results within rounding; for A/B
 * runs and tests): SPLIT (default) by point range, PAIR by pose pair, BAND by
 * point band (falls back to PAIR when a point spans more than 15 free key
 * frames).  The environment variable ORBGPU_SCHUR=split|pair|band sets the
 * default once, when the context is created. */
#define ORBGPU_LBA_SCHUR_SPLIT 0
#define ORBGPU_LBA_SCHUR_PAIR 1
#define ORBGPU_LBA_SCHUR_BAND 2
orbgpu_status orbgpu_lba_ctx_set_schur(orbgpu_lba_ctx* c, int mode);

/* on != 0: every LM build re-linearises at the accepted state instead of
 * taking the accepted trial's per-edge terms (bit-identical; a test switch).
 * Default: whether ORBGPU_LBA_RELINEARIZE is set when the context is created. */
orbgpu_status orbgpu_lba_ctx_set_relinearize(orbgpu_lba_ctx* c, int on);

/* Device-memory budget of the context (bytes; 0 = none, the default).  A
 * window whose device arena would exceed it returns ORBGPU_ERR_NOMEM before
 * any device work, the context stays usable -- the caller's hook for a
 * per-window memory bound (the drop-ins throw on NOMEM).
 * Only the device arena is counted: the pinned host staging and result
 * buffers, which also grow with the window (about the size of the uploaded
 * edges and of the returned state), are outside the budget. */
orbgpu_status orbgpu_lba_ctx_set_memory_limit(orbgpu_lba_ctx* c, size_t bytes);

/* Window size: the reduced camera system (6 rows per free key frame) is
 * factorised packed in LDS by one workgroup up to 160 rows, from HBM by one
 * workgroup below 224 rows, and by tile steps spread over the whole device
 * beyond (every factor in HBM): any
 * window the reference accepts runs on the device; only exhausted device
 * memory (ORBGPU_ERR_NOMEM, about 16 n^2 bytes for n reduced rows) or more
 * than INT_MAX / 2 rows (ORBGPU_ERR_CAPACITY) is refused. */

/* One window from host buffers.  Keyframe k is fixed iff fixed[k] (the map's
 * initial keyframe, :1161, and every fixed camera, :1169-1183).  Points
 * [pt_begin, pt_end) and their edges are this call's shard (the whole window:
 * 0, n_pts); with reduce == NULL the shard must be the whole window.
 * lambda_init > 0 sets g2o's user lambda (setUserLambdaInit: 100.0 when the
 * map is inertial, :1137); <= 0 = tau * max diag (computeLambdaInit).
 * *stop_flag (optional; the reference's bool, 1 byte, nonzero = stop) is read
 * where g2o polls SparseOptimizer::terminate(): before every LM iteration
 * (sparse_optimizer.cpp:406) and after every trial
 * (optimization_algorithm_levenberg.cpp:153-154).  The caller returns before
 * the call when it is already set (optimizer.cc:1356-1357).
 * The LM loop runs on the device; with reduce == NULL the call synchronises
 * once, at its end.
 * Edges may come in any order; a point's edges keep their order among
 * themselves.  Edges sorted by point (the reference's insertion order,
 * optimizer.cc:1187-1262) skip one host layout pass.
 * Outputs: optimised poses (float, unit quaternion; poses_out_d optional
 * doubles), pts_out rows of the shard's points, outlier[i] for the shard's
 * edges (chi2 > 5.991 / 7.815 or depth <= 0), stats (optional, 6 doubles):
 * initial / final robust chi2, LM iterations, trials, final lambda, outliers. */
orbgpu_status orbgpu_lba_optimize(orbgpu_lba_ctx* c, const orbgpu_camera* cam, int n_kf,
                                  const orbgpu_pose* poses_in, const uint8_t* fixed, int n_pts,
                                  const float* pts_in, int n_edges, const orbgpu_lba_edge* edges,
                                  int pt_begin, int pt_end, int iterations, double lambda_init,
                                  const volatile uint8_t* stop_flag, orbgpu_lba_reduce_fn reduce,
                                  void* user, orbgpu_pose* poses_out, double* poses_out_d,
                                  float* pts_out, uint8_t* outlier, double* stats);

/* ------------------------------------------------------------------------
 * ORBmatcher projection search (pinhole rig, Frame::Nleft == -1), the
 * matching that feeds PoseOptimization in Tracking::TrackWithMotionModel
 * (tracking.cc:2163-2216) and Tracking::SearchLocalPoints (:2626-2690).
 *
 * The current frame is given as the reference's Frame fields: keypoints
 * (mvKeysUn, cv::KeyPoint layout), descriptors (mDescriptors, 32 B rows),
 * uright (mvuRight; NULL = every keypoint monocular) and claimed (optional,
 * 1 byte per keypoint: mvpMapPoints[i] != NULL && ->Observations() > 0 before
 * the call).  The frame grid (FRAME_GRID_COLS x ROWS = 64 x 48,
 * Frame::AssignFeaturesToGrid, frame.cc:438-465) is built on the device.
 * Output match[i] per keypoint: >= 0 -> mvpMapPoints[i] = that query point;
 * -1 -> mvpMapPoints[i] untouched; -2 -> set to NULL (rotation-consistency
 * removal of a match made by this call).  *nmatches = the function's return.
 * ------------------------------------------------------------------------ */
#define ORBGPU_MAX_LEVELS 16
#define ORBGPU_FRAME_GRID_COLS 64 /* frame.h:41 */
#define ORBGPU_FRAME_GRID_ROWS 48 /* frame.h:40 */

typedef struct orbgpu_frame_geom {
  float min_x, max_x, min_y, max_y; /* Frame::mnMinX, mnMaxX, mnMinY, mnMaxY (ComputeImageBounds) */
  int32_t n_levels;                 /* Frame::mnScaleLevels                                       */
  float log_scale_factor;           /* Frame::mfLogScaleFactor                                   */
  float scale_factors[ORBGPU_MAX_LEVELS]; /* Frame::mvScaleFactors                              */
} orbgpu_frame_geom;

/* One LastFrame observation that SearchByProjection(CurrentFrame, LastFrame)
 * projects: LastFrame.mvpMapPoints[i] != NULL && !LastFrame.mvbOutlier[i], in
 * increasing i (orb_matcher.cc:1538-1541). */
typedef struct orbgpu_proj_point {
  float Xw[3];      /* pMP->GetWorldPos()                                    */
  int32_t octave;   /* LastFrame.mvKeys[i].octave                            */
  float angle;      /* LastFrame.mvKeysUn[i].angle (rotation histogram)      */
  int32_t has_obs;  /* pMP->Observations() > 0: its matches block later ones */
  uint8_t desc[32]; /* pMP->GetDescriptor()                                  */
} orbgpu_proj_point;

/* A local map point (Tracking::mvpLocalMapPoints[j]) as Frame::isInFrustum and
 * SearchByProjection(Frame&, vector<MapPoint*>, ...) read it. */
#define ORBGPU_MP_SKIP 1    /* isBad() or mnLastFrameSeen == frame id: not projected */
#define ORBGPU_MP_HAS_OBS 2 /* Observations() > 0                                      */
typedef struct orbgpu_map_point {
  float Xw[3];              /* GetWorldPos()                   */
  float normal[3];          /* GetNormal()                     */
  float min_dist, max_dist; /* mfMinDistance, mfMaxDistance    */
  int32_t flags;            /* ORBGPU_MP_*                     */
  uint8_t desc[32];         /* GetDescriptor()                 */
} orbgpu_map_point;

/* MapPoint tracking fields written by Frame::isInFrustum (frame.cc:548-603):
 * in_view = mbTrackInView; proj_x / proj_y = mTrackProjX / Y (-1 when the
 * projection fails the depth or image-bounds test); level, proj_xr, depth,
 * view_cos = mnTrackScaleLevel, mTrackProjXR, mTrackDepth, mTrackViewCos, only
 * meaningful (and only written by the reference) when in_view. */
typedef struct orbgpu_track_view {
  int32_t in_view, level;
  float proj_x, proj_y, proj_xr, depth, view_cos;
} orbgpu_track_view;

typedef struct orbgpu_matcher orbgpu_matcher;

/* One context per calling thread (own HIP stream and scratch), sized for
 * frames of up to max_keypoints keypoints and max_points query points. */
orbgpu_status orbgpu_matcher_create(int device, int max_keypoints, int max_points,
                                    orbgpu_matcher** out);
void orbgpu_matcher_destroy(orbgpu_matcher* m);

/* Sticky device error word of the context's *_batch calls (the host calls
 * report it themselves): bit 0 = a frame with more keypoints than kp_stride or
 * the kernels' bound (the frame was skipped), bit 1 = an observation list
 * truncated at obs_stride, bit 2 = more query points than pt_stride (only the
 * first pt_stride searched).  Synchronises the context's stream (and
 * hip_stream when not NULL); reset != 0 clears the word.  *err = 0 when clean. */
orbgpu_status orbgpu_matcher_status(orbgpu_matcher* m, void* hip_stream, int reset, int* err);

/* Replaces: int ORBmatcher::SearchByProjection(Frame& CurrentFrame,
 *   const Frame& LastFrame, const float th, const bool bMono)
 *   (orb_matcher.h, orb_matcher.cc:1518-1728) with mbCheckOrientation =
 *   check_orientation (TrackWithMotionModel: ORBmatcher(0.9, true), th = 7
 *   stereo / 15 otherwise, 2 th on the retry).  Tcw = CurrentFrame.GetPose(),
 *   Tlw = LastFrame.GetPose(), mb = CurrentFrame.mb; pts as orbgpu_proj_point. */
orbgpu_status orbgpu_search_by_projection_last(
    orbgpu_matcher* m, const orbgpu_frame_geom* geom, const orbgpu_camera* cam, float mb,
    const orbgpu_pose* Tcw, const orbgpu_pose* Tlw, const orbgpu_keypoint* kps,
    const uint8_t* descs, const float* uright, const uint8_t* claimed, int n,
    const orbgpu_proj_point* pts, int n_pts, float th, int mono, int check_orientation,
    int32_t* match, int* nmatches);

/* Device-resident batch of the above: frame f reads d_Tcw[f], d_Tlw[f],
 * keypoints / descriptors / uright / claimed at f * kp_stride (keypoints),
 * d_n[f] keypoints, d_pts + f * pt_stride with d_npts[f] points, and writes
 * d_match + f * kp_stride (d_n[f] entries) and d_nmatches[f].  d_uright /
 * d_claimed may be NULL.  Asynchronous on hip_stream (NULL: the context's). */
orbgpu_status orbgpu_search_by_projection_last_batch(
    orbgpu_matcher* m, int n_frames, const orbgpu_frame_geom* geom, const orbgpu_camera* cam,
    float mb, const orbgpu_pose* d_Tcw, const orbgpu_pose* d_Tlw, const orbgpu_keypoint* d_kps,
    const uint8_t* d_descs, const float* d_uright, const uint8_t* d_claimed, const int* d_n,
    int kp_stride, const orbgpu_proj_point* d_pts, const int* d_npts, int pt_stride, float th,
    int mono, int check_orientation, int32_t* d_match, int* d_nmatches, void* hip_stream);

/* The observation list Optimizer::PoseOptimization builds (optimizer.cc:
 *   806-877) for frames after orbgpu_search_by_projection_last_batch, whose
 *   mvpMapPoints held no point before the search (TrackWithMotionModel resets
 *   them, tracking.cc:2187-2188): for every keypoint i with d_match[i] >= 0,
 *   in increasing i, one orbgpu_pose_obs {Xw of point d_match[i], mvKeysUn[i].pt,
 *   mvuRight[i] (-1 when d_uright is NULL), mvInvLevelSigma2[octave]};
 *   d_obs_index (optional) receives i.  Frame f writes d_obs + f * obs_stride
 *   and d_nobs[f]: the input of orbgpu_pose_opt_batch, all on the device. */
orbgpu_status orbgpu_matches_to_pose_obs_batch(
    orbgpu_matcher* m, int n_frames, const orbgpu_keypoint* d_kps, const float* d_uright,
    const int32_t* d_match, const int* d_n, int kp_stride, const orbgpu_proj_point* d_pts,
    int pt_stride, const float* inv_level_sigma2, int n_levels, orbgpu_pose_obs* d_obs,
    int obs_stride, int* d_nobs, int32_t* d_obs_index, void* hip_stream);

/* Replaces: bool Frame::UnprojectStereo(const int& i, Eigen::Vector3f& x3D)
 *   (frame.cc:1008-1020) over Tracking::UpdateLastFrame's loop (tracking.cc:
 *   2099-2160) on the device: frame f's keypoints with mvDepth > 0, in index
 *   order, become LastFrame points at the frame's pose d_Tcw[f] (Xw = mRwc Xc
 *   + mOw; octave, angle and descriptor of the keypoint; has_obs = 1), ready
 *   for orbgpu_search_by_projection_last_batch.  d_npts[f] = the count (at
 *   most pt_stride; more sets bit 2 of orbgpu_matcher_status).  The
 *   reference keeps the tracked map points and adds temporal points for the
 *   closest stereo keypoints; a caller without a map (the synthetic sequence
 *   runner) takes every stereo keypoint. */
orbgpu_status orbgpu_unproject_stereo_batch(orbgpu_matcher* m, int n_frames,
                                           const orbgpu_camera* cam, const orbgpu_pose* d_Tcw,
                                           const orbgpu_keypoint* d_kps, const uint8_t* d_descs,
                                           const float* d_depth, const int* d_n, int kp_stride,
                                           orbgpu_proj_point* d_pts, int pt_stride, int* d_npts,
                                           void* hip_stream);

/* The same gather for PoseInertialOptimizationLastFrame / LastKeyFrame
 *   (optimizer.cc:4816-4900, 4466-4540): orbgpu_inertial_obs rows, with
 *   close = d_close[point] (MapPoint::mTrackDepth < 10; NULL: 0) and the
 *   pinhole Uncertainty2 = 1.  Declared with the inertial types below.
 *   In the reference these optimisations run in TrackLocalMap
 *   (tracking.cc:2262-2285) over mvpMapPoints as SearchLocalPoints left them
 *   (after IMU initialisation TrackWithMotionModel returns after
 *   PredictStateIMU without searching, :2170-2176): d_match is then
 *   orbgpu_search_local_points' match array over the local map points, and
 *   mTrackDepth is the depth its isInFrustum wrote (orbgpu_track_view). */

/* Replaces: bool Frame::isInFrustum(MapPoint* pMP, float viewingCosLimit)
 *   (frame.cc:548-603, Nleft == -1) over Tracking::SearchLocalPoints' loop
 *   (tracking.cc:2644-2661): points flagged ORBGPU_MP_SKIP are not projected
 *   (in_view = 0).  Rcw / tcw / Ow = the frame's mRcw (row-major), mtcw, mOw. */
orbgpu_status orbgpu_frustum(orbgpu_matcher* m, const orbgpu_frame_geom* geom,
                             const orbgpu_camera* cam, const float Rcw[9], const float tcw[3],
                             const float Ow[3], const orbgpu_map_point* pts, int n_pts,
                             float view_cos_limit, orbgpu_track_view* views);

/* Replaces: int ORBmatcher::SearchByProjection(Frame& F,
 *   const vector<MapPoint*>& vpMapPoints, const float th, const bool bFarPoints,
 *   const float thFarPoints) (orb_matcher.cc:42-206, Nleft == -1) with
 *   mfNNratio = nn_ratio; views[j] = point j's tracking fields (from
 *   orbgpu_frustum or the caller). */
orbgpu_status orbgpu_search_by_projection_local(
    orbgpu_matcher* m, const orbgpu_frame_geom* geom, const orbgpu_keypoint* kps,
    const uint8_t* descs, const float* uright, const uint8_t* claimed, int n,
    const orbgpu_map_point* pts, const orbgpu_track_view* views, int n_pts, float th,
    float nn_ratio, int far_points, float th_far_points, int32_t* match, int* nmatches);

/* Tracking::SearchLocalPoints' projection + search in one call: isInFrustum
 * over pts (views written back for the caller's IncreaseVisible /
 * mmProjectPoints bookkeeping), then the search above. */
orbgpu_status orbgpu_search_local_points(
    orbgpu_matcher* m, const orbgpu_frame_geom* geom, const orbgpu_camera* cam,
    const float Rcw[9], const float tcw[3], const float Ow[3], const orbgpu_keypoint* kps,
    const uint8_t* descs, const float* uright, const uint8_t* claimed, int n,
    const orbgpu_map_point* pts, int n_pts, float view_cos_limit, float th, float nn_ratio,
    int far_points, float th_far_points, orbgpu_track_view* views, int32_t* match,
    int* nmatches);

/* Replaces: int ORBmatcher::SearchByProjection(Frame& CurrentFrame,
 *   KeyFrame* pKF, const set<MapPoint*>& sAlreadyFound, const float th,
 *   const int ORBdist) (orb_matcher.cc:1730-1839, Nleft == -1), the search
 *   Tracking::Relocalization runs before its PoseOptimization calls
 *   (tracking.cc:2967-2997: ORBmatcher(0.9, true), th 10 / 3, ORBdist 100 /
 *   64).  pts[i] = pKF->GetMapPointMatches()[i] (ORBGPU_MP_SKIP: NULL,
 *   isBad() or in sAlreadyFound; normal unused), angles[i] =
 *   pKF->mvKeysUn[i].angle (may be NULL without the orientation check);
 *   claimed[k] = CurrentFrame.mvpMapPoints[k] != NULL (every claimed keypoint
 *   is skipped, and so is every keypoint this call matches).  Tcw =
 *   CurrentFrame.GetPose().  match[k] >= 0: mvpMapPoints[k] = the point of
 *   key-frame index match[k]; -1 untouched; -2 set to NULL by the rotation
 *   check. */
orbgpu_status orbgpu_search_by_projection_kf(
    orbgpu_matcher* m, const orbgpu_frame_geom* geom, const orbgpu_camera* cam,
    const orbgpu_pose* Tcw, const orbgpu_keypoint* kps, const uint8_t* descs,
    const uint8_t* claimed, int n, const orbgpu_map_point* pts, const float* angles, int n_pts,
    float th, int orb_dist, int check_orientation, int32_t* match, int* nmatches);

/* Device-resident batch of the above: frame f against its key frame's points
 * d_pts + f * pt_stride (d_npts[f] of them; angles likewise), pose d_Tcw[f];
 * layout and outputs as orbgpu_search_by_projection_last_batch. */
orbgpu_status orbgpu_search_by_projection_kf_batch(
    orbgpu_matcher* m, int n_frames, const orbgpu_frame_geom* geom, const orbgpu_camera* cam,
    const orbgpu_pose* d_Tcw, const orbgpu_keypoint* d_kps, const uint8_t* d_descs,
    const uint8_t* d_claimed, const int* d_n, int kp_stride, const orbgpu_map_point* d_pts,
    const float* d_angles, const int* d_npts, int pt_stride, float th, int orb_dist,
    int check_orientation, int32_t* d_match, int* d_nmatches, void* hip_stream);

/* Replaces: int ORBmatcher::SearchByBoW(KeyFrame* pKF, Frame& F,
 *   vector<MapPoint*>& vpMapPointMatches) (orb_matcher.cc:215-389, Nleft ==
 *   -1), the search of Tracking::TrackReferenceKeyFrame (tracking.cc:
 *   2043-2067, ORBmatcher(0.7, true)) and Relocalization (:2904-2926,
 *   ORBmatcher(0.75, true)).  The FeatureVectors pKF->mFeatVec / F.mFeatVec
 *   as orbgpu_bow_transform writes them (ascending node ids; node j's
 *   feature indices at features[offsets[j] .. offsets[j + 1])); kf_valid[i] =
 *   vpMapPointsKF[i] && !isBad(); kf_angles[i] = pKF->mvKeysUn[i].angle,
 *   f_angles[k] = F.mvKeys[k].angle (both may be NULL without the
 *   orientation check).  match[k] = i: vpMapPointMatches[k] = the point of
 *   key-frame feature i; -1: NULL.  *nmatches = the return value. */
orbgpu_status orbgpu_search_by_bow(orbgpu_matcher* m, const uint32_t* kf_nodes,
                                   const int32_t* kf_offsets, const uint32_t* kf_features,
                                   int kf_n_nodes, const uint8_t* kf_descs, const float* kf_angles,
                                   const uint8_t* kf_valid, int kf_n, const uint32_t* f_nodes,
                                   const int32_t* f_offsets, const uint32_t* f_features,
                                   int f_n_nodes, const uint8_t* f_descs, const float* f_angles,
                                   int f_n, float nn_ratio, int check_orientation, int32_t* match,
                                   int* nmatches);

/* Device-resident batch: pair f reads the key frame's FeatureVector at
 * d_kf_* + f * kf_stride (offsets at f * (kf_stride + 1), d_kf_n_nodes[f]
 * nodes), its descriptors / angles / valid flags at f * kf_stride, and the
 * frame's at f * f_stride the same way -- orbgpu_bow_transform_batch's output
 * layout; the frame's angle of keypoint k at d_f_angles[(f * f_stride + k) *
 * f_angle_step] (1 for a float array, 7 for orbgpu_keypoint rows starting at
 * the first row's angle), d_f_n[f] keypoints.  Writes d_match + f * f_stride
 * and d_nmatches[f]; asynchronous on hip_stream (NULL: the context's). */
orbgpu_status orbgpu_search_by_bow_batch(
    orbgpu_matcher* m, int n_frames, const uint32_t* d_kf_nodes, const int32_t* d_kf_offsets,
    const uint32_t* d_kf_features, const int* d_kf_n_nodes, const uint8_t* d_kf_descs,
    const float* d_kf_angles, const uint8_t* d_kf_valid, int kf_stride, const uint32_t* d_f_nodes,
    const int32_t* d_f_offsets, const uint32_t* d_f_features, const int* d_f_n_nodes,
    const uint8_t* d_f_descs, const float* d_f_angles, int f_angle_step, const int* d_f_n,
    int f_stride, float nn_ratio, int check_orientation, int32_t* d_match, int* d_nmatches,
    void* hip_stream);

/* ------------------------------------------------------------------------
 * DBoW2 bag-of-words conversion (3rdparty/DBoW2, ORBVocabulary =
 * TemplatedVocabulary<FORB::TDescriptor, FORB>): Frame::ComputeBoW
 * (frame.cc:761-766) and KeyFrame::ComputeBoW (keyframe.cc:202-208) call
 * transform(descriptors, mBowVec, mFeatVec, 4).
 * ------------------------------------------------------------------------ */
typedef struct orbgpu_vocab orbgpu_vocab;

/* Replaces: bool TemplatedVocabulary::loadFromTextFile(const std::string&)
 *   (TemplatedVocabulary.h:1248-1327), text format "k L scoring weighting" then
 *   one "parent isLeaf d0 .. d31 weight" line per node; the tree goes to
 *   `device`.  ORBGPU_ERR_INVALID for a header outside the reference's bounds
 *   (k in [0, 20], L in [1, 10], scoring in [0, 5], weighting in [0, 3]). */
orbgpu_status orbgpu_vocab_load_text(int device, const char* path, orbgpu_vocab** out);
void orbgpu_vocab_destroy(orbgpu_vocab* v);
/* info[0..5] = k, L, scoring (DBoW2::ScoringType), weighting (WeightingType),
 * nodes (root included), words. */
orbgpu_status orbgpu_vocab_info(const orbgpu_vocab* v, int info[6]);

/* Replaces: void TemplatedVocabulary::transform(const vector<TDescriptor>&
 *   features, BowVector& v, FeatureVector& fv, int levelsup) const
 *   (TemplatedVocabulary.h:1057-1118, per feature :1140-1179).  descs: n x 32
 *   bytes (mDescriptors rows).  BowVector (std::map<WordId, WordValue>) comes
 *   back as *n_words ascending word ids + weights; FeatureVector
 *   (std::map<NodeId, vector<unsigned>>) as *n_nodes ascending node ids, the
 *   feature indices of node j in fv_features[fv_offsets[j] .. fv_offsets[j+1]).
 *   Capacities: bow_* and fv_nodes / fv_features n entries, fv_offsets n + 1. */
orbgpu_status orbgpu_bow_transform(orbgpu_vocab* v, const uint8_t* descs, int n, int levelsup,
                                   uint32_t* bow_words, double* bow_weights, int* n_words,
                                   uint32_t* fv_nodes, int32_t* fv_offsets, uint32_t* fv_features,
                                   int* n_nodes);

/* Device-resident batch: frame f's descriptors at d_descs + f * stride * 32,
 * d_n[f] of them; outputs at f * stride (fv_offsets at f * (stride + 1)),
 * counts in d_n_words[f] / d_n_nodes[f].  Asynchronous on hip_stream (NULL:
 * the vocabulary's own stream). */
orbgpu_status orbgpu_bow_transform_batch(orbgpu_vocab* v, int n_frames, const uint8_t* d_descs,
                                         const int* d_n, int stride, int levelsup,
                                         uint32_t* d_bow_words, double* d_bow_weights,
                                         int* d_n_words, uint32_t* d_fv_nodes,
                                         int32_t* d_fv_offsets, uint32_t* d_fv_features,
                                         int* d_n_nodes, void* hip_stream);

/* MapPoint::PredictScale (mappoint.cc:550-563) as used by the kernels: the
 * level of a ratio mfMaxDistance / dist is the number of thresholds thr[j-1]
 * (j = 1 .. n_levels - 1) it reaches, thr[j-1] = the smallest float ratio with
 * ceil(log(ratio) / log_scale_factor) >= j under the host libm.  Writes
 * ORBGPU_MAX_LEVELS - 1 floats (+inf past n_levels - 1); returns n_levels - 1
 * or -1 on bad arguments.  Host-only (no device work). */
int orbgpu_level_thresholds(float log_scale_factor, int n_levels, float* thr);

/* ---- Inertial tracking optimisation -----------------
 * Optimizer::PoseInertialOptimizationLastFrame (optimizer.cc:4762-5160) and
 * Optimizer::PoseInertialOptimizationLastKeyFrame (:4394-4760): g2o
 * Gauss-Newton (optimization_algorithm_gauss_newton.cpp), dense LDLT over the
 * free vertices, 4 rounds x 10 iterations with outlier classification.
 * Pinhole left camera only (Frame::Nleft == -1; the fisheye right-camera
 * edges are out of scope).  Matrices are row-major. */

/* A frame's (or key frame's) IMU state: the estimates of VertexPose
 * (ImuCamPose(Frame*), g2o_types.cc:74-118), VertexVelocity, VertexGyroBias,
 * VertexAccBias (g2o_types.cc:448-470). */
typedef struct orbgpu_imu_state {
  float Rwb[9], twb[3]; /* GetImuRotation / GetImuPosition */
  float Rcw[9], tcw[3]; /* GetPose() (current frame only; ignored for the previous one) */
  float v[3];           /* GetVelocity */
  float bg[3], ba[3];   /* mImuBias (bwx..bwz), (bax..baz) */
} orbgpu_imu_state;

/* IMU::Preintegrated between the previous and the current frame
 * (imu_types.h) plus the information matrices the edges derive from it:
 * info = EdgeInertial's (C.block<9,9>(0,0) inverse, symmetrised, eigenvalues
 * below 1e-12 zeroed, g2o_types.cc:472-492), info_g / info_a =
 * C.block<3,3>(9,9) / (12,12) inverses (optimizer.cc:4933-4944). */
typedef struct orbgpu_imu_preint {
  float dT;
  float dR[9], dV[3], dP[3];
  float JRg[9], JVg[9], JVa[9], JPg[9], JPa[9];
  float bg[3], ba[3]; /* the linearisation bias b */
  float pad_;
  double info[81];
  double info_g[9], info_a[9];
} orbgpu_imu_preint;

/* ConstraintPoseImu of the previous frame (mpcpi), as its constructor left
 * it (H symmetrised and eigen-cleaned, imu_types / g2o_types.h:664-685).
 * LastFrame mode only. */
typedef struct orbgpu_imu_prior {
  double Rwb[9], twb[3], vwb[3], bg[3], ba[3];
  double H[225];
} orbgpu_imu_prior;

/* Camera intrinsics (Pinhole params_) + bf + mImuCalib mTcb / mTbc. */
typedef struct orbgpu_imu_calib {
  float fx, fy, cx, cy, bf;
  float Rcb[9], tcb[3];
  float Rbc[9], tbc[3];
} orbgpu_imu_calib;

/* One EdgeMonoOnlyPose / EdgeStereoOnlyPose, in frame keypoint order:
 * mvKeysUn[i].pt, mvuRight[i] (< 0: monocular), mvInvLevelSigma2[octave] /
 * Uncertainty2, close = (mTrackDepth < 10). */
typedef struct orbgpu_inertial_obs {
  float Xw[3];
  float u, v, ur;
  float inv_sigma2;
  int32_t close;
} orbgpu_inertial_obs;

/* Results: SetImuPoseVelocity(Rwb, twb, v) and mImuBias (float casts), the
 * double estimates and the 15x15 H (VP, VV, VG, VA order) the reference passes
 * to `new ConstraintPoseImu(...)` (LastFrame: after Marginalize(H, 0, 14);
 * LastKeyFrame: the current-frame Hessian), and the return value
 * nInitialCorrespondences - nBad. */
typedef struct orbgpu_inertial_result {
  float Rwb[9], twb[3], v[3], bg[3], ba[3];
  int32_t n_good;
  int32_t n_inliers;
  double Rwb_d[9], twb_d[3], v_d[3], bg_d[3], ba_d[3];
  double H[225];
} orbgpu_inertial_result;

#define ORBGPU_INERTIAL_LAST_FRAME 0
#define ORBGPU_INERTIAL_LAST_KEYFRAME 1

typedef struct orbgpu_inertial_ctx orbgpu_inertial_ctx;

orbgpu_status orbgpu_inertial_ctx_create(int device, int max_problems, int max_obs,
                                         orbgpu_inertial_ctx** out);
void orbgpu_inertial_ctx_destroy(orbgpu_inertial_ctx* c);

/* Replaces: int Optimizer::PoseInertialOptimizationLastFrame(Frame*, bool
 *   bRecInit) (mode ORBGPU_INERTIAL_LAST_FRAME: previous frame free, prior
 *   edge, marginalisation) and PoseInertialOptimizationLastKeyFrame (mode
 *   ORBGPU_INERTIAL_LAST_KEYFRAME: last key frame fixed, `prior` unused).  One
 *   problem from host buffers; outlier[i] = mvbOutlier of observation i. */
orbgpu_status orbgpu_pose_inertial(orbgpu_inertial_ctx* c, int mode, const orbgpu_imu_calib* calib,
                                   const orbgpu_imu_state* cur, const orbgpu_imu_state* prev,
                                   const orbgpu_imu_preint* preint, const orbgpu_imu_prior* prior,
                                   const orbgpu_inertial_obs* obs, int n_obs, int rec_init,
                                   orbgpu_inertial_result* res, uint8_t* outlier);

/* Device-resident batch: problem p reads d_cur[p], d_prev[p], d_preint[p],
 * d_prior[p] (LastFrame), d_obs[p * obs_stride .. + d_nobs[p]); one shared
 * calibration.  Asynchronous on hip_stream (NULL: the context's stream). */
orbgpu_status orbgpu_pose_inertial_batch(orbgpu_inertial_ctx* c, int mode,
                                         const orbgpu_imu_calib* calib, int n_problems,
                                         const orbgpu_imu_state* d_cur,
                                         const orbgpu_imu_state* d_prev,
                                         const orbgpu_imu_preint* d_preint,
                                         const orbgpu_imu_prior* d_prior,
                                         const orbgpu_inertial_obs* d_obs, const int* d_nobs,
                                         int obs_stride, int rec_init,
                                         orbgpu_inertial_result* d_res, uint8_t* d_outlier,
                                         void* hip_stream);

/* ------------------------------------------------------------------------
 * LocalInertialBA -- replaces the solve of Optimizer::LocalInertialBA(
 * KeyFrame* pKF, bool* pbStopFlag, Map* pMap, int& num_fixedKF, int&
 * num_OptKF, int& num_MPs, int& num_edges, bool bLarge, bool bRecInit)
 * (optimizer.h, optimizer.cc:2329-2902; LocalMapping dispatches it once the
 * IMU is initialised, localmapping.cc:108-145).  The caller gathers the
 * temporal window as the reference does (:2340-2436: the last Nd key frames
 * through mPrevKF, their map points, the key frame before the window and the
 * other observers as fixed key frames) and hands over the graph
 * (:2461-2781); the library runs optimize(opt_it) -- g2o LM with the
 * user lambda (:2448-2459), BlockSolverX with the points marginalised
 * (Schur complement), fp64 -- and the outlier test (:2796-2826).  The caller
 * applies the FAIL test (:2832-2836: 2 err < err_end or NaN, unless bLarge),
 * erases the flagged observations and writes the key frames and points back
 * (:2838-2901).  *pbStopFlag is attached only after optimize() (:2794), so it
 * never stops this optimisation: the call takes no stop flag.
 *
 * Key frame k: kfs[k] = ImuCamPose(pKF) (Rwb, twb, Rcw, tcw) + the vertex
 * estimates (v, bg, ba); fixed[k] = VertexPose (and its IMU vertices) fixed;
 * imu[k] = pKF->bImu (VertexVelocity / GyroBias / AccBias exist).  Every free
 * key frame must carry IMU vertices.  In the reduced system a free key frame
 * owns 15 consecutive rows, VP(6) VV(3) VG(3) VA(3) (g2o orders VP ids before
 * the IMU vertex ids; SimplicialLDLT's AMD ordering makes the order a
 * rounding matter only).  Visual edges are orbgpu_lba_edge rows read as
 * EdgeMono / EdgeStereo (cam_idx 0; inv_sigma2 = mvInvLevelSigma2[octave] /
 * Uncertainty2, 1 for the pinhole camera); close[p] = pMP->mTrackDepth < 10.
 * ------------------------------------------------------------------------ */
#define ORBGPU_LIA_ROBUST 1     /* EdgeInertial under RobustKernelHuber(sqrt(16.92)) (:2571-2581) */
#define ORBGPU_LIA_DOWNWEIGHT 2 /* EdgeInertial information x 1e-2 (i == N - 1, :2579)            */

typedef struct orbgpu_lia_imu_edge {
  int32_t kf1;   /* pKFi->mPrevKF: VP1 VV1 VG1 VA1                                  */
  int32_t kf2;   /* pKFi: VP2 VV2 (and EdgeGyroRW / EdgeAccRW's second vertices)   */
  int32_t flags; /* ORBGPU_LIA_*                                                    */
  int32_t pad_;
  orbgpu_imu_preint preint; /* pKFi->mpImuPreintegrated: deltas, Jacobians, EdgeInertial's
                               information and the random-walk informations (:2587-2599) */
} orbgpu_lia_imu_edge;

/* Runs on the LocalBundleAdjustment context (its stream and arena).
 * iterations = opt_it (10, bLarge 4); lambda_init = the user lambda (1e0,
 * bLarge 1e-2; must be > 0).  Outputs: kfs_out (float casts: SetPose(Tcw)
 * from Rcw / tcw, SetVelocity, SetNewBias), kfs_out_d (optional, 21 doubles
 * per key frame: Rwb(9) twb v bg ba), pts_out, outlier[i] per visual edge,
 * stats (optional, 7 doubles): err = the robust chi2 before optimize()
 * (:2790-2791), err_end = the robust chi2 of the last computed errors
 * (:2793), LM iterations, trials, final lambda, outliers, accepted chi2. */
/* A free key frame owns 15 reduced rows (VP VV VG VA); one without IMU data
 * (imu[k] == 0: the reference's VertexPose-only key frame,
 * optimizer.cc:2466-2484) has only its pose vertex, and no link may touch it
 * (:2503: an EdgeInertial needs bImu on both key frames; such a link is
 * ORBGPU_ERR_INVALID).  Its 9 inertial rows stay structurally zero with a
 * zero right-hand side, so the step leaves v / bg / ba as given.  Window size
 * and link count are bounded only by device memory (the solver paths above). */
orbgpu_status orbgpu_lia_optimize(orbgpu_lba_ctx* c, const orbgpu_imu_calib* calib, int n_kf,
                                  const orbgpu_imu_state* kfs, const uint8_t* fixed,
                                  const uint8_t* imu, int n_pts, const float* pts_in,
                                  const uint8_t* close, int n_edges, const orbgpu_lba_edge* edges,
                                  int n_imu, const orbgpu_lia_imu_edge* imu_edges, int iterations,
                                  double lambda_init, orbgpu_imu_state* kfs_out, double* kfs_out_d,
                                  float* pts_out, uint8_t* outlier, double* stats);

/* orbgpu_matches_to_pose_obs_batch's inertial form (see the comment there). */
orbgpu_status orbgpu_matches_to_inertial_obs_batch(
    orbgpu_matcher* m, int n_frames, const orbgpu_keypoint* d_kps, const float* d_uright,
    const int32_t* d_match, const int* d_n, int kp_stride, const orbgpu_proj_point* d_pts,
    const uint8_t* d_close, int pt_stride, const float* inv_level_sigma2, int n_levels,
    orbgpu_inertial_obs* d_obs, int obs_stride, int* d_nobs, int32_t* d_obs_index,
    void* hip_stream);

#ifdef __cplusplus
}
#endif
#endif /* ORBGPU_H */
