// gfx950 kernels of the ORBmatcher projection searches that feed
// PoseOptimization in tracking (pinhole rig, Frame::Nleft == -1):
//
//   k_mt_grid     block / frame: Frame::AssignFeaturesToGrid (frame.cc:438-465)
//                 -> per-cell index lists (64 x 48 cells, ascending keypoint
//                 index inside a cell), counting sort in LDS
//   k_mt_search   wave / query point: projection (SearchByProjection(Frame&,
//                 const Frame&) orb_matcher.cc:1538-1577, or Frame::isInFrustum
//                 frame.cc:548-603 + orb_matcher.cc:50-69, or the key frame
//                 form of Relocalization :1747-1779), then
//                 GetFeaturesInArea (frame.cc:679-746): lanes own grid cells
//                 of the window, filter, Hamming distance from 8 v_bcnt, and
//                 the wave keeps the best and second candidate by the packed
//                 key (dist, position in the reference's candidate order) --
//                 first strict minimum = smallest key; the reference's running
//                 second best = smallest key of the rest
//   k_mt_resolve  wave / frame: the reference's matches are sequential
//                 (a match by a point with observations hides that keypoint
//                 from every later point, orb_matcher.cc:86-87, 1591-1592).
//                 Each query carries its top-4 candidates: under the claims
//                 so far its result is the first (and second) unclaimed entry.
//                 64 queries at a time, in rounds: the queries before the first
//                 one whose pick an earlier pending query claims commit
//                 together (LDS claim bitmap + owner table); a query whose list
//                 runs out is searched again with the claims masked.  Then the
//                 rotation histogram
//                 (orb_matcher.cc:1614-1632, 1708-1725; ComputeThreeMaxima
//                 :1841-1873) and the mvpMapPoints writes.
//
// Float expressions follow the oracle (oracle/match_oracle.cc): every fused
// multiply-add the reference build performs is an explicit __builtin_fmaf;
// the file is compiled with -ffp-contract=off.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "match_launch.h"

namespace orbgpu {

#ifdef ORB_STAMPS
// profiling build only: k_mt_resolve chunks, rounds, list re-searches, queries
__device__ unsigned long long g_mt_stats[8];
#endif

namespace {

constexpr int kThHigh = 100;      // ORBmatcher::TH_HIGH (orb_matcher.cc:35)
constexpr int kHistoLength = 30;  // ORBmatcher::HISTO_LENGTH (:37)
constexpr int kKpFloats = 7;      // orbgpu_keypoint
constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr uint64_t kNoKey = ~0ull;

struct V3 {
  float x, y, z;
};

__device__ __forceinline__ float mul_sub(float a, float b, float c, float d) {
  return __builtin_fmaf(a, b, -(c * d));
}
__device__ __forceinline__ V3 cross(V3 a, V3 b) {
  return {mul_sub(a.y, b.z, a.z, b.y), mul_sub(a.z, b.x, a.x, b.z), mul_sub(a.x, b.y, a.y, b.x)};
}
// Sophus::SO3 * p (so3.hpp:359-367)
__device__ __forceinline__ V3 quat_rotate(float qx, float qy, float qz, float qw, V3 p) {
  const V3 qv{qx, qy, qz};
  V3 uv = cross(qv, p);
  uv = {uv.x + uv.x, uv.y + uv.y, uv.z + uv.z};
  const V3 c = cross(qv, uv);
  return {__builtin_fmaf(qw, uv.x, p.x) + c.x, __builtin_fmaf(qw, uv.y, p.y) + c.y,
          __builtin_fmaf(qw, uv.z, p.z) + c.z};
}
__device__ __forceinline__ V3 se3_apply(const orbgpu_pose& T, V3 p) {
  const V3 r = quat_rotate(T.qx, T.qy, T.qz, T.qw, p);
  return {r.x + T.tx, r.y + T.ty, r.z + T.tz};
}
// Tcw.inverse().translation() with SO3's renormalised conjugate (se3.hpp:208-211)
__device__ __forceinline__ V3 se3_inverse_translation(const orbgpu_pose& T) {
  float q0 = -T.qx, q1 = -T.qy, q2 = -T.qz, q3 = T.qw;
  const float s = (q0 * q0 + q2 * q2) + (q1 * q1 + q3 * q3);
  const float len = sqrtf(s);
  q0 /= len, q1 /= len, q2 /= len, q3 /= len;
  return quat_rotate(q0, q1, q2, q3, V3{-T.tx, -T.ty, -T.tz});
}
__device__ __forceinline__ float dot3(V3 a, V3 b) {
  return __builtin_fmaf(a.z, b.z, __builtin_fmaf(a.x, b.x, a.y * b.y));
}

__device__ __forceinline__ int kp_octave(const float* k) { return __float_as_int(k[5]); }

// A barrier for LDS hand-offs only: each wave waits for its own LDS operations,
// not for its global loads and stores, which __syncthreads' release fence also
// drains (a ~1 us store acknowledgement per round in k_mt_resolve, and the
// prefetch of the next queries).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const uint64_t o = __shfl_xor(v, off, 64);
    v = o < v ? o : v;
  }
  return v;
}

// A query as GetFeaturesInArea + the candidate loop see it (wave-uniform).
struct Query {
  bool valid;
  float x, y, r;  // window centre / half-size (factorX = factorY = r)
  int min_level, max_level;
  float ur_ref;   // predicted right coordinate (motion: u - bf * invzc; local: mTrackProjXR)
  uint32_t d[8];  // query descriptor
};

__device__ __forceinline__ void load_desc(const uint8_t* p, uint32_t d[8]) {
  // orbgpu_proj_point / orbgpu_map_point descriptors are 4-byte aligned
  const uint32_t* w = (const uint32_t*)p;
#pragma unroll
  for (int i = 0; i < 8; ++i) d[i] = w[i];
}

// SearchByProjection(CurrentFrame, LastFrame) query setup (orb_matcher.cc:1529-1577)
__device__ Query query_last(const MatchLaunch& a, int f, int q) {
  const MatchParams& p = a.p;
  Query Q;
  Q.valid = false;
  const orbgpu_pose Tcw = a.Tcw[f];
  const orbgpu_pose Tlw = a.Tlw[f];
  const V3 twc = se3_inverse_translation(Tcw);
  const V3 tlc = se3_apply(Tlw, twc);
  const bool forward = tlc.z > p.mb && !p.mono;
  const bool backward = -tlc.z > p.mb && !p.mono;
  const orbgpu_proj_point* P = a.ppts + (size_t)f * a.pt_stride + q;
  const V3 x3Dc = se3_apply(Tcw, V3{P->Xw[0], P->Xw[1], P->Xw[2]});
  const float invzc = (float)(1.0 / (double)x3Dc.z);
  if (invzc < 0) return Q;
  const float u = p.fx * x3Dc.x / x3Dc.z + p.cx;
  const float v = p.fy * x3Dc.y / x3Dc.z + p.cy;
  if (u < p.min_x || u > p.max_x) return Q;
  if (v < p.min_y || v > p.max_y) return Q;
  const int oct = P->octave;
  Q.r = p.th * p.scale[oct];
  if (forward) Q.min_level = oct, Q.max_level = -1;
  else if (backward) Q.min_level = 0, Q.max_level = oct;
  else Q.min_level = oct - 1, Q.max_level = oct + 1;
  Q.x = u, Q.y = v;
  Q.ur_ref = __builtin_fmaf(-p.bf, invzc, u);
  load_desc(P->desc, Q.d);
  Q.valid = true;
  return Q;
}

// Frame::isInFrustum (frame.cc:548-603); fills V only where the reference writes.
__device__ bool frustum(const MatchParams& p, const float* pose15, const orbgpu_map_point* M,
                        orbgpu_track_view& V) {
  V.in_view = 0;
  if (M->flags & ORBGPU_MP_SKIP) return false;
  V.proj_x = -1.0f, V.proj_y = -1.0f;
  const float* R = pose15;
  const float* t = pose15 + 9;
  const float* Ow = pose15 + 12;
  const V3 P{M->Xw[0], M->Xw[1], M->Xw[2]};
  V3 Pc;
  Pc.x = __builtin_fmaf(R[2], P.z, __builtin_fmaf(R[0], P.x, R[1] * P.y)) + t[0];
  Pc.y = __builtin_fmaf(R[5], P.z, __builtin_fmaf(R[3], P.x, R[4] * P.y)) + t[1];
  Pc.z = __builtin_fmaf(R[8], P.z, __builtin_fmaf(R[6], P.x, R[7] * P.y)) + t[2];
  const float pc_dist = sqrtf(dot3(Pc, Pc));
  const float invz = 1.0f / Pc.z;
  if (Pc.z < 0.0f) return false;
  const float u = p.fx * Pc.x / Pc.z + p.cx;
  const float v = p.fy * Pc.y / Pc.z + p.cy;
  if (u < p.min_x || u > p.max_x) return false;
  if (v < p.min_y || v > p.max_y) return false;
  V.proj_x = u, V.proj_y = v;
  const float maxD = 1.2f * M->max_dist, minD = 0.8f * M->min_dist;
  const V3 PO{P.x - Ow[0], P.y - Ow[1], P.z - Ow[2]};
  const float dist = sqrtf(dot3(PO, PO));
  if (dist < minD || dist > maxD) return false;
  const float view_cos = dot3(PO, V3{M->normal[0], M->normal[1], M->normal[2]}) / dist;
  if (view_cos < p.cos_limit) return false;
  // MapPoint::PredictScale via the host's thresholds of ceil(log(ratio) / lsf)
  const float ratio = M->max_dist / dist;
  int level = 0;
  if (ratio != __builtin_inff())
    for (int j = 1; j < p.n_levels; ++j) level += ratio >= p.level_thr[j - 1];
  V.level = level;
  V.in_view = 1;
  V.proj_xr = __builtin_fmaf(-p.bf, invz, u);
  V.depth = pc_dist;
  V.view_cos = view_cos;
  return true;
}

// SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist) query
// setup (orb_matcher.cc:1747-1779): the key frame's point q (ORBGPU_MP_SKIP:
// NULL, bad or already found) projected by Tcw without a depth test, the
// image bounds, the scale-invariance distances, PredictScale's level, the
// window th * scale[level] over levels [level - 1, level + 1].
__device__ Query query_keyframe(const MatchLaunch& a, int f, int q) {
  const MatchParams& p = a.p;
  Query Q;
  Q.valid = false;
  const orbgpu_map_point* M = a.mpts + (size_t)f * a.pt_stride + q;
  if (M->flags & ORBGPU_MP_SKIP) return Q;
  const orbgpu_pose Tcw = a.Tcw[f];
  const V3 X{M->Xw[0], M->Xw[1], M->Xw[2]};
  const V3 x3Dc = se3_apply(Tcw, X);
  const float u = p.fx * x3Dc.x / x3Dc.z + p.cx;
  const float v = p.fy * x3Dc.y / x3Dc.z + p.cy;
  if (u < p.min_x || u > p.max_x) return Q;
  if (v < p.min_y || v > p.max_y) return Q;
  const V3 Ow = se3_inverse_translation(Tcw);
  const V3 PO{X.x - Ow.x, X.y - Ow.y, X.z - Ow.z};
  const float dist = sqrtf(dot3(PO, PO));
  const float maxD = 1.2f * M->max_dist, minD = 0.8f * M->min_dist;
  if (dist < minD || dist > maxD) return Q;
  const float ratio = M->max_dist / dist;  // MapPoint::PredictScale by the host's thresholds
  int level = 0;
  if (ratio != __builtin_inff())
    for (int j = 1; j < p.n_levels; ++j) level += ratio >= p.level_thr[j - 1];
  Q.r = p.th * p.scale[level];
  Q.min_level = level - 1, Q.max_level = level + 1;
  Q.x = u, Q.y = v;
  Q.ur_ref = 0.0f;  // no right-coordinate test in this search
  load_desc(M->desc, Q.d);
  Q.valid = true;
  return Q;
}

// SearchByProjection(Frame&, vector<MapPoint*>) query setup (orb_matcher.cc:50-69)
__device__ Query query_local(const MatchParams& p, const orbgpu_map_point* M,
                             const orbgpu_track_view& V) {
  Query Q;
  Q.valid = false;
  if (!V.in_view) return Q;
  if (p.far_points && V.depth > p.th_far) return Q;
  const int level = V.level;
  float r = (double)V.view_cos > 0.998 ? 2.5f : 4.0f;  // RadiusByViewingCos (:208-213)
  if (p.th != 1.0f) r *= p.th;
  Q.r = r * p.scale[level];
  Q.min_level = level - 1, Q.max_level = level;
  Q.x = V.proj_x, Q.y = V.proj_y;
  Q.ur_ref = V.proj_xr;
  load_desc(M->desc, Q.d);
  Q.valid = true;
  return Q;
}

struct FrameRef {
  const float* kps;
  const uint4* desc;
  const float* uright;
  const uint8_t* claimed;
  const int* cell_start;
  const uint16_t* cell_idx;
};

__device__ __forceinline__ FrameRef frame_ref(const MatchLaunch& a, int f) {
  const size_t ko = (size_t)f * a.kp_stride;
  FrameRef F;
  F.kps = a.kps + ko * kKpFloats;
  F.desc = (const uint4*)(a.desc + ko * 32);
  F.uright = a.uright ? a.uright + ko : nullptr;
  F.claimed = a.claimed ? a.claimed + ko : nullptr;
  F.cell_start = a.cell_start + (size_t)f * (kGridCells + 1);
  F.cell_idx = a.cell_idx + ko;
  return F;
}

// GetFeaturesInArea (frame.cc:679-746) + the candidate loop: the kMatchTopK
// smallest keys (dist, position in the reference's candidate order) as packed
// (dist << 16 | idx), kNone-padded, and the number of candidates.  The
// reference's running best = top[0]; its running second best = top[1] (the
// smallest key of the rest).  claims (LDS bitmap, may be null) masks
// keypoints matched earlier in the call.
__device__ void wave_topk(const MatchParams& p, const FrameRef& F, const Query& Q,
                          const uint32_t* claims, uint32_t top[kMatchTopK], int& count) {
#pragma unroll
  for (int i = 0; i < kMatchTopK; ++i) top[i] = kNone;
  count = 0;
  if (!Q.valid) return;
  const float r = Q.r;
  const int minCx = max(0, (int)floorf((Q.x - p.min_x - r) * p.inv_w));
  if (minCx >= kGridCols) return;
  const int maxCx = min(kGridCols - 1, (int)ceilf((Q.x - p.min_x + r) * p.inv_w));
  if (maxCx < 0) return;
  const int minCy = max(0, (int)floorf((Q.y - p.min_y - r) * p.inv_h));
  if (minCy >= kGridRows) return;
  const int maxCy = min(kGridRows - 1, (int)ceilf((Q.y - p.min_y + r) * p.inv_h));
  if (maxCy < 0) return;
  const int ncy = maxCy - minCy + 1;
  const int ncells = (maxCx - minCx + 1) * ncy;
  if (ncells <= 0) return;
  const bool check_levels = Q.min_level >= 0 || Q.max_level >= 0;
  const int lane = threadIdx.x & 63;
  uint64_t b[kMatchTopK];  // this lane's smallest keys, ascending
#pragma unroll
  for (int i = 0; i < kMatchTopK; ++i) b[i] = kNoKey;
  int local = 0;
  for (int k = lane; k < ncells; k += 64) {
    const int cx = k / ncy;
    const int cell = (minCx + cx) * kGridRows + minCy + (k - cx * ncy);
    const int s = F.cell_start[cell], e = F.cell_start[cell + 1];
    for (int j = s; j < e; ++j) {
      const int idx = F.cell_idx[j];
      const float* kp = F.kps + (size_t)idx * kKpFloats;
      const int oct = kp_octave(kp);
      if (check_levels) {
        if (oct < Q.min_level) continue;
        if (Q.max_level >= 0 && oct > Q.max_level) continue;
      }
      const float dx = kp[0] - Q.x, dy = kp[1] - Q.y;
      if (!(fabsf(dx) < r && fabsf(dy) < r)) continue;
      if (F.claimed && F.claimed[idx]) continue;
      if (claims && ((claims[idx >> 5] >> (idx & 31)) & 1u)) continue;
      if (F.uright) {
        const float uR = F.uright[idx];
        if (uR > 0 && fabsf(Q.ur_ref - uR) > r) continue;
      }
      const uint4 d0 = F.desc[2 * idx], d1 = F.desc[2 * idx + 1];
      const int dist = __popc(d0.x ^ Q.d[0]) + __popc(d0.y ^ Q.d[1]) + __popc(d0.z ^ Q.d[2]) +
                       __popc(d0.w ^ Q.d[3]) + __popc(d1.x ^ Q.d[4]) + __popc(d1.y ^ Q.d[5]) +
                       __popc(d1.z ^ Q.d[6]) + __popc(d1.w ^ Q.d[7]);
      uint64_t key = ((uint64_t)dist << 40) | ((uint64_t)k << 16) | (uint64_t)idx;
      ++local;
#pragma unroll
      for (int i = 0; i < kMatchTopK; ++i) {  // insertion into the sorted registers
        const uint64_t lo = key < b[i] ? key : b[i];
        key = key < b[i] ? b[i] : key;
        b[i] = lo;
      }
    }
  }
  int total = local;
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) total += __shfl_xor(total, off, 64);
  count = total;
#pragma unroll
  for (int i = 0; i < kMatchTopK; ++i) {
    const uint64_t m = wave_min_u64(b[0]);
    top[i] = m == kNoKey ? kNone : (uint32_t)((m >> 40) << 16 | (m & 0xFFFF));
    if (b[0] == m && m != kNoKey) {  // the owning lane pops its head
#pragma unroll
      for (int j = 0; j + 1 < kMatchTopK; ++j) b[j] = b[j + 1];
      b[kMatchTopK - 1] = kNoKey;
    }
  }
}

__device__ __forceinline__ Query make_query(const MatchLaunch& a, int f, int q, bool write_view) {
  if (a.mode == kModeLast) return query_last(a, f, q);
  if (a.mode == kModeKeyFrame) return query_keyframe(a, f, q);
  const size_t o = (size_t)f * a.pt_stride + q;
  const orbgpu_map_point* M = a.mpts + o;
  orbgpu_track_view V;
  if (a.mode == kModeLocalFrustum && write_view) {
    frustum(a.p, a.frustum_pose + 15 * f, M, V);
    if ((threadIdx.x & 63) == 0) {
      // only the fields isInFrustum writes change
      orbgpu_track_view O = a.views_init ? a.views_init[o] : a.views[o];
      O.in_view = V.in_view;
      if (!(M->flags & ORBGPU_MP_SKIP)) O.proj_x = V.proj_x, O.proj_y = V.proj_y;
      if (V.in_view) O.level = V.level, O.proj_xr = V.proj_xr, O.depth = V.depth, O.view_cos = V.view_cos;
      a.views[o] = O;
    }
  } else {
    V = a.views[o];
  }
  return query_local(a.p, M, V);
}

// ---------------------------------------------------------------------------
// 1024 threads: a thread's keypoints' cells are computed once and kept in
// registers (n <= kMatchMaxKeypoints = 8 x 1024), the cell counts scanned by
// wave prefix sums (3 cells a thread) and one pass over the 16 wave totals.
constexpr int kGridThreads = 1024;
constexpr int kGridPerThread = kMatchMaxKeypoints / kGridThreads;
static_assert(kGridCells % kGridThreads == 0, "cells per thread");
__global__ __launch_bounds__(kGridThreads) void k_mt_grid(MatchLaunch a) {
  __shared__ int cnt[kGridCells];
  __shared__ int start[kGridCells];
  __shared__ uint16_t lidx[kMatchMaxKeypoints];
  __shared__ int wtot[kGridThreads / 64];
  const int f = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int n = a.n[f];
  if (t == 0) {
    const int e = (a.npts[f] > a.pt_stride ? 4 : 0) |  // searched up to pt_stride only
                  (n > kMatchMaxKeypoints || n > a.kp_stride ? 1 : 0);
    if (a.zero_err)
      *a.err = e;  // single-frame call: this call's own word, no memset before it
    else if (e)
      atomicOr(a.err, e);
  }
  if (n > kMatchMaxKeypoints || n > a.kp_stride) return;
  const float* kps = a.kps + (size_t)f * a.kp_stride * kKpFloats;
  for (int c = t; c < kGridCells; c += kGridThreads) cnt[c] = 0;
  // Frame::PosInGrid (frame.cc:748-759), keypoints t + 1024 j
  int cell[kGridPerThread];
#pragma unroll
  for (int j = 0; j < kGridPerThread; ++j) {
    const int i = t + kGridThreads * j;
    cell[j] = -1;
    if (i < n) {
      const float* k = kps + (size_t)i * kKpFloats;
      const int px = (int)roundf((k[0] - a.p.min_x) * a.p.inv_w);
      const int py = (int)roundf((k[1] - a.p.min_y) * a.p.inv_h);
      if (px >= 0 && px < kGridCols && py >= 0 && py < kGridRows) cell[j] = px * kGridRows + py;
    }
  }
  lds_barrier();
#pragma unroll
  for (int j = 0; j < kGridPerThread; ++j)
    if (cell[j] >= 0) atomicAdd(&cnt[cell[j]], 1);
  lds_barrier();
  constexpr int kPer = kGridCells / kGridThreads;  // 3 cells per thread
  int v[kPer], sum = 0;
#pragma unroll
  for (int j = 0; j < kPer; ++j) v[j] = cnt[t * kPer + j], sum += v[j];
  int incl = sum;  // inclusive wave scan
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int o = __shfl_up(incl, off, 64);
    if (lane >= off) incl += o;
  }
  if (lane == 63) wtot[w] = incl;
  lds_barrier();
  int run = incl - sum, total = 0;
#pragma unroll
  for (int q = 0; q < kGridThreads / 64; ++q) {
    const int x = wtot[q];
    run += q < w ? x : 0;
    total += x;
  }
  int* cs = a.cell_start + (size_t)f * (kGridCells + 1);
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int c = t * kPer + j;
    start[c] = run;
    cs[c] = run;
    cnt[c] = run;  // cursor
    run += v[j];
  }
  if (t == 0) cs[kGridCells] = total;
  lds_barrier();
#pragma unroll
  for (int j = 0; j < kGridPerThread; ++j)
    if (cell[j] >= 0) lidx[atomicAdd(&cnt[cell[j]], 1)] = (uint16_t)(t + kGridThreads * j);
  lds_barrier();
  // ascending keypoint index inside each cell (push_back order, frame.cc:452-464)
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int c = t * kPer + j;
    const int s0 = start[c], e = cnt[c];
    for (int i = s0 + 1; i < e; ++i) {
      const uint16_t x = lidx[i];
      int q = i - 1;
      while (q >= s0 && lidx[q] > x) lidx[q + 1] = lidx[q], --q;
      lidx[q + 1] = x;
    }
  }
  lds_barrier();
  uint16_t* out = a.cell_idx + (size_t)f * a.kp_stride;
  for (int i = t; i < total; i += kGridThreads) out[i] = lidx[i];
}

__global__ __launch_bounds__(256) void k_mt_search(MatchLaunch a) {
  const int f = blockIdx.y;
  const int q = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  if (q >= min(a.npts[f], a.pt_stride)) return;  // the scratch rows hold pt_stride points
  const FrameRef F = frame_ref(a, f);
  const Query Q = make_query(a, f, q, true);
  uint32_t top[kMatchTopK];
  int count;
  wave_topk(a.p, F, Q, nullptr, top, count);
  if ((threadIdx.x & 63) == 0) {
    uint32_t* r = a.res + (size_t)kMatchResWords * ((size_t)f * a.pt_stride + q);
#pragma unroll
    for (int i = 0; i < kMatchTopK; ++i) r[i] = top[i];
    r[kMatchTopK] = (uint32_t)count;
  }
}

// the distance a best candidate must not exceed (TH_HIGH, or ORBdist)
__device__ __forceinline__ int accept_dist(const MatchLaunch& a) {
  return a.mode == kModeKeyFrame ? a.p.orb_dist : kThHigh;
}

// does a match by query q hide its keypoint from later queries?  (the key
// frame search skips every keypoint holding a point, orb_matcher.cc:1791)
__device__ __forceinline__ bool has_obs(const MatchLaunch& a, int f, int q) {
  const size_t o = (size_t)f * a.pt_stride + q;
  if (a.mode == kModeKeyFrame) return true;
  return a.mode == kModeLast ? a.ppts[o].has_obs != 0 : (a.mpts[o].flags & ORBGPU_MP_HAS_OBS) != 0;
}

// rotation bin of a match (orb_matcher.cc:1626-1630, 1808-1812)
__device__ __forceinline__ int rot_bin(const MatchLaunch& a, const float* kps, int f, int q,
                                       int idx) {
  const float factor = kHistoLength / 360.0f;
  const size_t o = (size_t)f * a.pt_stride + q;
  const float ang = a.mode == kModeKeyFrame ? a.q_angle[o] : a.ppts[o].angle;
  float rot = ang - kps[(size_t)idx * kKpFloats + 3];
  if ((double)rot < 0.0) rot += 360.0f;
  int bin = (int)roundf(rot * factor);
  if (bin == kHistoLength) bin = 0;
  return bin;
}

// One wave per frame.  The call's mvpMapPoints row and the keypoint octaves
// live in LDS (the rounds below touch no global memory on the local-map and
// last-frame paths but the output stores), and the next 64 queries' top-K
// lists are loaded while the current ones resolve.
__global__ __launch_bounds__(64) void k_mt_resolve(MatchLaunch a) {
  __shared__ uint32_t owner[kMatchMaxKeypoints];    // in-round first claiming lane, 64 = none
  __shared__ uint32_t blocked[kMatchMaxKeypoints];  // in-round first stopped lane listing it, 64 = none
  __shared__ int32_t lmatch[kMatchMaxKeypoints];
  __shared__ uint8_t loct[kMatchMaxKeypoints];
  __shared__ uint32_t claims[kMatchMaxKeypoints / 32];
  __shared__ uint32_t removed[kMatchMaxKeypoints / 32];
  __shared__ int hist[kHistoLength];
  const int f = blockIdx.x, lane = threadIdx.x;
  const int n = a.n[f], nq = min(a.npts[f], a.pt_stride);
  if (n > kMatchMaxKeypoints || n > a.kp_stride) return;  // reported by k_mt_grid
  const FrameRef F = frame_ref(a, f);
  const bool rot_check = (a.mode == kModeLast || a.mode == kModeKeyFrame) && a.p.check_ori;
  const bool local = a.mode == kModeLocal || a.mode == kModeLocalFrustum;
  // mvpMapPoints of this call: the last matching query (later matches
  // overwrite, orb_matcher.cc:122, 1611), kept with atomicMax
  for (int i = lane; i < n; i += 64)
    lmatch[i] = -1, owner[i] = 64, blocked[i] = 64, loct[i] = (uint8_t)kp_octave(F.kps + (size_t)i * kKpFloats);
  for (int i = lane; i < kMatchMaxKeypoints / 32; i += 64) claims[i] = 0, removed[i] = 0;
  if (lane < kHistoLength) hist[lane] = 0;
  lds_barrier();
  const uint32_t* res = a.res + (size_t)kMatchResWords * f * a.pt_stride;
  int32_t* acc = a.acc + (size_t)f * a.pt_stride;
  int nmatch = 0;
  auto is_claimed = [&](uint32_t key) -> bool {
    const int idx = key & 0xFFFF;
    return (claims[idx >> 5] >> (idx & 31)) & 1u;
  };
  // (best, second) acceptance with the octaves from LDS (accept_of)
  auto accept = [&](uint32_t best, uint32_t second) -> bool {
    if (best == kNone) return false;
    const int d1 = (int)(best >> 16);
    if (d1 > accept_dist(a)) return false;
    if (a.mode == kModeLast || a.mode == kModeKeyFrame) return true;
    const int l1 = loct[best & 0xFFFF];
    const int l2 = second == kNone ? -1 : loct[second & 0xFFFF];
    const int d2 = second == kNone ? 256 : (int)(second >> 16);
    return !(l1 == l2 && (float)d1 > a.p.nn_ratio * (float)d2);
  };
  uint32_t ntop[kMatchTopK];  // the next chunk's lists, in flight
  int ncount = 0;
  bool nobs = false;
  auto fetch = [&](int base) {
    const int q = base + lane;
    const bool valid = q < nq;
#pragma unroll
    for (int i = 0; i < kMatchTopK; ++i) ntop[i] = valid ? res[(size_t)kMatchResWords * q + i] : kNone;
    ncount = valid ? (int)res[(size_t)kMatchResWords * q + kMatchTopK] : 0;
    nobs = valid && has_obs(a, f, q);
  };
  fetch(0);
#ifdef ORB_STAMPS
  const unsigned long long t_setup = __builtin_amdgcn_s_memtime();
#endif
  for (int base = 0; base < nq; base += 64) {
    const int q = base + lane;
    const bool valid = q < nq;
    uint32_t top[kMatchTopK];
#pragma unroll
    for (int i = 0; i < kMatchTopK; ++i) top[i] = ntop[i];
    int count = ncount;
    const bool obs = nobs;
    if (base + 64 < nq) fetch(base + 64);
    bool done = !valid;
    // Rounds: every pending query takes its best / second unclaimed entries;
    // the queries before the first one that an earlier pending claimer hits
    // (or whose list ran out) are final and commit together.
    while (true) {
      uint32_t b = kNone, s2 = kNone;
      int found = 0;
#pragma unroll
      for (int i = 0; i < kMatchTopK; ++i) {
        if (top[i] != kNone && !is_claimed(top[i])) {
          if (found == 0) b = top[i];
          else if (found == 1) s2 = top[i];
          ++found;
        }
      }
      // a best beyond TH_HIGH can only get worse as claims accumulate
      const bool hopeless = b != kNone && (int)(b >> 16) > accept_dist(a);
      const int need = local ? 2 : 1;
      const bool exhausted = !done && !hopeless && found < need && count > kMatchTopK;
      const bool ok = !done && !exhausted && accept(b, s2);
      const bool claimer = ok && obs;
      if (claimer) atomicMin(&owner[b & 0xFFFF], (uint32_t)lane);
      lds_barrier();
      bool hit = false;
      if (!done && !exhausted && b != kNone && !hopeless) {
        hit = owner[b & 0xFFFF] < (uint32_t)lane;
        if (local && s2 != kNone) hit = hit || owner[s2 & 0xFFFF] < (uint32_t)lane;
      }
      lds_barrier();
      if (claimer) owner[b & 0xFFFF] = 64;
      // Stopped: hit or exhausted, and every later query a stopped one could
      // still affect.  A stopped query whose top-K list is its complete
      // candidate set (count <= K) can only ever take an entry of that list,
      // so a later query whose best (and, local, second) is in no such list
      // is final now and commits past it -- its own claim cannot reach the
      // stopped one.  A stopped query whose list may run out (a full search
      // later, against every claim then made) blocks all later ones.  Hopeless
      // queries and queries with no candidate are final anyway.
      uint64_t stop_mask = __ballot(hit || exhausted);
      if (stop_mask) {
        const uint64_t inc = __ballot(!done && count > kMatchTopK);
        const bool live = !done && !hopeless && b != kNone;
        for (;;) {
          const uint64_t si = stop_mask & inc;
          const int first_inc = si ? __builtin_ctzll(si) : 64;
          if ((stop_mask >> lane) & 1)
#pragma unroll
            for (int i = 0; i < kMatchTopK; ++i)
              if (top[i] != kNone) atomicMin(&blocked[top[i] & 0xFFFF], (uint32_t)lane);
          lds_barrier();
          bool blk = false;
          if (live) {
            blk = lane > first_inc || blocked[b & 0xFFFF] < (uint32_t)lane;
            if (local && s2 != kNone) blk = blk || blocked[s2 & 0xFFFF] < (uint32_t)lane;
          }
          const uint64_t grown = stop_mask | __ballot(blk);
          lds_barrier();
          if (grown == stop_mask) break;
          stop_mask = grown;
        }
        if ((stop_mask >> lane) & 1)
#pragma unroll
          for (int i = 0; i < kMatchTopK; ++i)
            if (top[i] != kNone) blocked[top[i] & 0xFFFF] = 64;
      }
      const int stop = stop_mask ? __builtin_ctzll(stop_mask) : 64;
      const bool commit = !done && !((stop_mask >> lane) & 1);
      if (commit) {
        if (ok) {
          const int idx = b & 0xFFFF;
          atomicMax(&lmatch[idx], q);
          if (claimer) atomicOr(&claims[idx >> 5], 1u << (idx & 31));
          int bin = 0;
          if (rot_check) {
            bin = rot_bin(a, F.kps, f, q, idx);
            atomicAdd(&hist[bin], 1);
          }
          acc[q] = idx | (bin << 16);
        } else {
          acc[q] = -1;
        }
        done = true;
      }
      nmatch += __popcll(__ballot(commit && ok));
      lds_barrier();
#ifdef ORB_STAMPS
      if (lane == 0) atomicAdd(&g_mt_stats[1], 1ull);
#endif
      if (stop == 64) break;
      // the first stopped query: hit by a claim now committed (its next round
      // sees it), or its list ran out -> full search with the claims masked
      const bool ex_stop = (stop_mask >> stop) & 1 && __builtin_amdgcn_readlane((int)exhausted, stop);
      if (ex_stop) {
#ifdef ORB_STAMPS
        if (lane == 0) atomicAdd(&g_mt_stats[2], 1ull);
        const unsigned long long rs0 = __builtin_amdgcn_s_memtime();
#endif
        const Query Q = make_query(a, f, base + stop, false);
        uint32_t t2[kMatchTopK];
        int c2;
        wave_topk(a.p, F, Q, claims, t2, c2);
        if (lane == stop) {
#pragma unroll
          for (int i = 0; i < kMatchTopK; ++i) top[i] = t2[i];
          count = c2;
        }
#ifdef ORB_STAMPS
        if (lane == 0) atomicAdd(&g_mt_stats[5], __builtin_amdgcn_s_memtime() - rs0);
#endif
      }
    }
  }
  lds_barrier();
  if (rot_check) {
    // ComputeThreeMaxima (orb_matcher.cc:1841-1873), every lane
    int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
    for (int i = 0; i < kHistoLength; ++i) {
      const int s = hist[i];
      if (s > max1) {
        max3 = max2, max2 = max1, max1 = s;
        ind3 = ind2, ind2 = ind1, ind1 = i;
      } else if (s > max2) {
        max3 = max2, max2 = s;
        ind3 = ind2, ind2 = i;
      } else if (s > max3) {
        max3 = s, ind3 = i;
      }
    }
    if ((float)max2 < 0.1f * (float)max1) ind2 = ind3 = -1;
    else if ((float)max3 < 0.1f * (float)max1) ind3 = -1;
    // every match in another bin is set to NULL (:1716-1724)
    int dropped = 0;
    for (int q = lane; q < nq; q += 64) {
      const int v = acc[q];
      if (v < 0) continue;
      const int bin = v >> 16;
      if (bin != ind1 && bin != ind2 && bin != ind3) {
        const int idx = v & 0xFFFF;
        atomicOr(&removed[idx >> 5], 1u << (idx & 31));
        ++dropped;
      }
    }
    for (int off = 32; off >= 1; off >>= 1) dropped += __shfl_xor(dropped, off, 64);
    nmatch -= dropped;
    lds_barrier();
    for (int i = lane; i < n; i += 64)
      if ((removed[i >> 5] >> (i & 31)) & 1u) lmatch[i] = -2;
    lds_barrier();
  }
  int32_t* match = a.match + (size_t)f * a.kp_stride;
  for (int i = lane; i < n; i += 64) match[i] = lmatch[i];
#ifdef ORB_STAMPS
  if (lane == 0) {
    atomicAdd(&g_mt_stats[0], (unsigned long long)((nq + 63) / 64));
    atomicAdd(&g_mt_stats[3], (unsigned long long)nq);
    atomicAdd(&g_mt_stats[4], __builtin_amdgcn_s_memtime() - t_setup);  // chunks .. end
  }
#endif
  if (a.mirror_dst) {  // one-frame host call: the outputs into host memory by this one workgroup
    if (lane == 0) a.nmatches[f] = nmatch;
    __syncthreads();                                  // this wave's stores drained
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // fresh lines of the other kernels' outputs
    const uint4* s4 = reinterpret_cast<const uint4*>(a.mirror_src);
    uint4* d4 = reinterpret_cast<uint4*>(a.mirror_dst);
    for (int i = lane; i < (a.mirror_bytes + 15) >> 4; i += 64) d4[i] = s4[i];
    __syncthreads();
    if (lane == 0) {
      __threadfence_system();
      __hip_atomic_store(a.done_host, a.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    return;
  }
  if (lane == 0) a.nmatches[f] = nmatch;
}

// Optimizer::PoseOptimization's observation list (optimizer.cc:806-877) of a
// frame whose mvpMapPoints hold exactly this call's matches: keypoints with
// match[i] >= 0 in increasing i.  Block / frame, 256 keypoints per step.
__global__ __launch_bounds__(256) void k_mt_pose_obs(ObsLaunch a) {
  __shared__ int wsum[4];
  const int f = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
  if (t == 0 && a.n[f] > a.kp_stride) atomicOr(a.err, 1);
  const int n = min(a.n[f], a.kp_stride);  // the match row holds kp_stride entries
  const size_t ko = (size_t)f * a.kp_stride;
  const float* kps = a.kps + ko * kKpFloats;
  orbgpu_pose_obs* obs = a.obs ? a.obs + (size_t)f * a.obs_stride : nullptr;
  int32_t* index = a.obs_index ? a.obs_index + (size_t)f * a.obs_stride : nullptr;
  int base = 0;
  for (int i0 = 0; i0 < n; i0 += 256) {
    const int i = i0 + t;
    const int q = i < n ? a.match[ko + i] : -1;
    const bool take = q >= 0 && q < a.pt_stride;
    const uint64_t bal = __ballot(take);
    if (lane == 0) wsum[w] = __popcll(bal);
    __syncthreads();
    int off = base;
    for (int k = 0; k < w; ++k) off += wsum[k];
    const int total = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    if (take) {
      const int pos = off + __popcll(bal & ((1ull << lane) - 1ull));
      if (pos < a.obs_stride) {
        const orbgpu_proj_point& P = a.pts[(size_t)f * a.pt_stride + q];
        const float* k = kps + (size_t)i * kKpFloats;
        if (a.iobs) {  // EdgeMono/StereoOnlyPose rows (optimizer.cc:4816-4900, Uncertainty2 = 1)
          orbgpu_inertial_obs o;
          o.Xw[0] = P.Xw[0], o.Xw[1] = P.Xw[1], o.Xw[2] = P.Xw[2];
          o.u = k[0], o.v = k[1];
          o.ur = a.uright ? a.uright[ko + i] : -1.0f;
          o.inv_sigma2 = a.inv_sigma2[kp_octave(k)];
          o.close = a.close ? (int32_t)a.close[(size_t)f * a.pt_stride + q] : 0;
          a.iobs[(size_t)f * a.obs_stride + pos] = o;
        } else {
          orbgpu_pose_obs o;
          o.Xw[0] = P.Xw[0], o.Xw[1] = P.Xw[1], o.Xw[2] = P.Xw[2];
          o.u = k[0], o.v = k[1];
          o.ur = a.uright ? a.uright[ko + i] : -1.0f;
          o.inv_sigma2 = a.inv_sigma2[kp_octave(k)];
          obs[pos] = o;
        }
        if (index) index[pos] = i;
      }
    }
    base += total;
    __syncthreads();
  }
  if (t == 0) {
    a.nobs[f] = min(base, a.obs_stride);
    if (base > a.obs_stride) atomicOr(a.err, 2);
  }
}

// Frame::UnprojectStereo (frame.cc:1008-1020) of every keypoint with
// mvDepth > 0, in index order (one block per frame, ballot compaction):
// Xc = ((u - cx) z invfx, (v - cy) z invfy, z), Xw = mRwc Xc + mOw with
// mRwc = Tcw.rotationMatrix()^T (Eigen's quaternion-to-matrix) and mOw =
// Tcw.inverse().translation(); the point takes the keypoint's octave, angle
// and descriptor and counts as observed (Tracking::UpdateLastFrame's points).
__global__ __launch_bounds__(256) void k_mt_unproject(UnprojLaunch a) {
  __shared__ int wsum[4];
  const int f = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
  if (t == 0 && a.n[f] > a.kp_stride) atomicOr(a.err, 1);
  const int n = min(a.n[f], a.kp_stride);
  const size_t ko = (size_t)f * a.kp_stride;
  const orbgpu_pose T = a.Tcw[f];
  // Eigen QuaternionBase::toRotationMatrix (rows of Rcw)
  const float tx = 2 * T.qx, ty = 2 * T.qy, tz = 2 * T.qz;
  const float twx = tx * T.qw, twy = ty * T.qw, twz = tz * T.qw;
  const float txx = tx * T.qx, txy = ty * T.qx, txz = tz * T.qx;
  const float tyy = ty * T.qy, tyz = tz * T.qy, tzz = tz * T.qz;
  const float R[3][3] = {{1 - (tyy + tzz), txy - twz, txz + twy},
                         {txy + twz, 1 - (txx + tzz), tyz - twx},
                         {txz - twy, tyz + twx, 1 - (txx + tyy)}};
  const V3 Ow = se3_inverse_translation(T);
  const float invfx = 1.0f / a.fx, invfy = 1.0f / a.fy;
  int base = 0;
  for (int i0 = 0; i0 < n; i0 += 256) {
    const int i = i0 + t;
    const float z = i < n ? a.depth[ko + i] : 0.0f;
    const bool take = z > 0;
    const uint64_t bal = __ballot(take);
    if (lane == 0) wsum[w] = __popcll(bal);
    __syncthreads();
    int off = base;
    for (int k = 0; k < w; ++k) off += wsum[k];
    const int total = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    if (take) {
      const int pos = off + __popcll(bal & ((1ull << lane) - 1ull));
      if (pos < a.pt_stride) {
        const float* k = a.kps + (ko + i) * kKpFloats;
        const float x = (k[0] - a.cx) * z * invfx, y = (k[1] - a.cy) * z * invfy;
        orbgpu_proj_point P;
        // mRwc * x3Dc + mOw: (Rwc)_rc = R[c][r]
        P.Xw[0] = __builtin_fmaf(R[2][0], z, __builtin_fmaf(R[1][0], y, R[0][0] * x)) + Ow.x;
        P.Xw[1] = __builtin_fmaf(R[2][1], z, __builtin_fmaf(R[1][1], y, R[0][1] * x)) + Ow.y;
        P.Xw[2] = __builtin_fmaf(R[2][2], z, __builtin_fmaf(R[1][2], y, R[0][2] * x)) + Ow.z;
        P.octave = kp_octave(k);
        P.angle = k[3];
        P.has_obs = 1;
        const uint4* src = reinterpret_cast<const uint4*>(a.desc + (ko + i) * 32);
        uint4* dst = reinterpret_cast<uint4*>(P.desc);
        dst[0] = src[0];
        dst[1] = src[1];
        a.pts[(size_t)f * a.pt_stride + pos] = P;
      }
    }
    base += total;
    __syncthreads();
  }
  if (t == 0) {
    a.npts[f] = min(base, a.pt_stride);
    if (base > a.pt_stride) atomicOr(a.err, 4);
  }
}

}  // namespace

hipError_t launch_unproject(const UnprojLaunch& a, hipStream_t st) {
  if (a.n_frames <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_mt_unproject, dim3(a.n_frames), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_pose_obs(const ObsLaunch& a, hipStream_t st) {
  if (a.n_frames <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_mt_pose_obs, dim3(a.n_frames), dim3(256), 0, st, a);
  return hipGetLastError();
}

// ---- SearchByBoW(KeyFrame* pKF, Frame& F) (orb_matcher.cc:215-389) ------
// Block / (key frame, frame) pair, a wave per key-frame node (strided): the
// node's partner in the frame by binary search (the reference's merge join
// with lower_bound visits exactly the common nodes, in ascending order), then
// the node's key-frame features in order, each against the frame features of
// the node not yet matched: lanes over the features (64 per pass), the key
// (dist << 32 | position) -- the first strict minimum is the smallest key,
// the running second best the smallest of the rest.  A feature belongs to one
// node in each FeatureVector, so nodes are independent and only the claims
// inside a node are sequential.  Then the rotation histogram over every
// match (ComputeThreeMaxima) and the output.
constexpr int kBowSearchThreads = 256;
constexpr int kThLow = 50;  // ORBmatcher::TH_LOW (orb_matcher.cc:36)

__global__ __launch_bounds__(kBowSearchThreads) void k_bow_search(BowSearchLaunch a) {
  __shared__ int16_t mk[kMatchMaxKeypoints];  // matched key-frame feature per frame keypoint, -1
  __shared__ uint8_t bins[kMatchMaxKeypoints];
  __shared__ uint32_t claims[kMatchMaxKeypoints / 32];
  __shared__ int hist[kHistoLength];
  __shared__ int red[kBowSearchThreads / 64];
  const int f = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int nf = a.f_n[f];
  if (nf > kMatchMaxKeypoints || nf > a.f_stride || a.kf_n_nodes[f] > a.kf_stride ||
      a.f_n_nodes[f] > a.f_stride) {
    if (t == 0) atomicOr(a.err, 1);
    return;
  }
  for (int k = t; k < kMatchMaxKeypoints; k += kBowSearchThreads) mk[k] = -1;
  for (int k = t; k < kMatchMaxKeypoints / 32; k += kBowSearchThreads) claims[k] = 0;
  if (t < kHistoLength) hist[t] = 0;
  __syncthreads();
  const size_t ko = (size_t)f * a.kf_stride, fo = (size_t)f * a.f_stride;
  const uint32_t* kn = a.kf_nodes + ko;
  const int32_t* koff = a.kf_off + (size_t)f * (a.kf_stride + 1);
  const uint32_t* kfe = a.kf_feat + ko;
  const uint32_t* fn = a.f_nodes + fo;
  const int32_t* foff = a.f_off + (size_t)f * (a.f_stride + 1);
  const uint32_t* ffe = a.f_feat + fo;
  const int nkn = a.kf_n_nodes[f], nfn = a.f_n_nodes[f];
  const float factor = kHistoLength / 360.0f;
  for (int na = wave; na < nkn; na += kBowSearchThreads / 64) {
    const uint32_t node = kn[na];
    int lo = 0, hi = nfn;  // lower_bound over the frame's nodes (wave-uniform)
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (fn[mid] < node) lo = mid + 1;
      else hi = mid;
    }
    if (lo >= nfn || fn[lo] != node) continue;
    const int fb = foff[lo], fe = min(foff[lo + 1], a.f_stride);
    const int kb = koff[na], ke = min(koff[na + 1], a.kf_stride);
    for (int ia = kb; ia < ke; ++ia) {
      const int ik = (int)kfe[ia];
      if (ik >= a.kf_stride || !a.kf_valid[ko + ik]) continue;
      const uint32_t* qd = (const uint32_t*)(a.kf_desc + (ko + ik) * 32);
      uint32_t d[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) d[i] = qd[i];
      uint64_t k1 = kNoKey, k2 = kNoKey;  // this lane's two smallest keys
      for (int base = fb; base < fe; base += 64) {
        const int j = base + lane;
        if (j >= fe) continue;
        const int idx = (int)ffe[j];
        if (idx >= nf || ((claims[idx >> 5] >> (idx & 31)) & 1u)) continue;
        const uint4* fd = (const uint4*)(a.f_desc + (fo + idx) * 32);
        const uint4 d0 = fd[0], d1 = fd[1];
        const int dist = __popc(d0.x ^ d[0]) + __popc(d0.y ^ d[1]) + __popc(d0.z ^ d[2]) +
                         __popc(d0.w ^ d[3]) + __popc(d1.x ^ d[4]) + __popc(d1.y ^ d[5]) +
                         __popc(d1.z ^ d[6]) + __popc(d1.w ^ d[7]);
        const uint64_t key = ((uint64_t)dist << 32) | (uint64_t)(j - fb);
        if (key < k1) k2 = k1, k1 = key;
        else if (key < k2) k2 = key;
      }
      const uint64_t m1 = wave_min_u64(k1);
      const uint64_t m2 = wave_min_u64(k1 == m1 ? k2 : k1);
      const int best1 = m1 == kNoKey ? 256 : (int)(m1 >> 32);
      const int best2 = m2 == kNoKey ? 256 : (int)(m2 >> 32);
      if (best1 <= kThLow && (float)best1 < a.nn_ratio * (float)best2) {
        const int idx = (int)ffe[fb + (int)(m1 & 0xFFFFFFFFu)];
        if (lane == 0) {
          mk[idx] = (int16_t)ik;
          atomicOr(&claims[idx >> 5], 1u << (idx & 31));
          int bin = 0;
          if (a.check_ori) {
            float rot = a.kf_angle[ko + ik] - a.f_angle[(fo + idx) * a.angle_step];
            if ((double)rot < 0.0) rot += 360.0f;
            bin = (int)roundf(rot * factor);
            if (bin == kHistoLength) bin = 0;
            atomicAdd(&hist[bin], 1);
          }
          bins[idx] = (uint8_t)bin;
        }
        // the claim is read by this wave's next feature: drain the LDS write
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
      }
    }
  }
  __syncthreads();
  int ind1 = -1, ind2 = -1, ind3 = -1;
  if (a.check_ori) {  // ComputeThreeMaxima (orb_matcher.cc:1841-1873), every thread
    int max1 = 0, max2 = 0, max3 = 0;
    for (int i = 0; i < kHistoLength; ++i) {
      const int sz = hist[i];
      if (sz > max1) {
        max3 = max2, max2 = max1, max1 = sz;
        ind3 = ind2, ind2 = ind1, ind1 = i;
      } else if (sz > max2) {
        max3 = max2, max2 = sz;
        ind3 = ind2, ind2 = i;
      } else if (sz > max3) {
        max3 = sz, ind3 = i;
      }
    }
    if ((float)max2 < 0.1f * (float)max1) ind2 = ind3 = -1;
    else if ((float)max3 < 0.1f * (float)max1) ind3 = -1;
  }
  int kept = 0;
  int32_t* out = a.match + fo;
  for (int k = t; k < nf; k += kBowSearchThreads) {
    int v = mk[k];
    if (v >= 0 && a.check_ori) {
      const int b = bins[k];
      if (b != ind1 && b != ind2 && b != ind3) v = -1;
    }
    kept += v >= 0;
    out[k] = v;
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) kept += __shfl_xor(kept, off, 64);
  __syncthreads();
  if (lane == 0) red[wave] = kept;
  __syncthreads();
  if (t == 0) {
    int tot = 0;
    for (int w = 0; w < kBowSearchThreads / 64; ++w) tot += red[w];
    a.nmatches[f] = tot;
  }
}

hipError_t launch_bow_search(const BowSearchLaunch& a, hipStream_t st) {
  if (a.n_frames <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_bow_search, dim3(a.n_frames), dim3(kBowSearchThreads), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_match(const MatchLaunch& a, hipStream_t st) {
  if (a.n_frames <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_mt_grid, dim3(a.n_frames), dim3(kGridThreads), 0, st, a);
  if (a.max_pts > 0) {
    hipLaunchKernelGGL(k_mt_search, dim3((unsigned)((a.max_pts + 3) / 4), a.n_frames), dim3(256),
                       0, st, a);
  }
  hipLaunchKernelGGL(k_mt_resolve, dim3(a.n_frames), dim3(64), 0, st, a);
  return hipGetLastError();
}

}  // namespace orbgpu

#ifdef ORB_STAMPS
// profiling build only: the k_mt_resolve counters since the last call (chunks,
// rounds, re-searches, queries), then cleared
extern "C" int orbgpu_debug_mt_stats(unsigned long long* out) {
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(orbgpu::g_mt_stats), 6 * sizeof(unsigned long long)) != hipSuccess) return -1;
  static const unsigned long long z[8] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(orbgpu::g_mt_stats), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif
