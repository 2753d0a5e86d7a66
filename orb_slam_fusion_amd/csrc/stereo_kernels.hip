// gfx950 kernels of the stereo matcher: Frame::ComputeStereoMatches
// (src/map/frame.cc:828-986) for rectified pinhole stereo, over extractor
// outputs that never leave HBM (pyramids, keypoints, descriptors).
//
//   k_stereo_rows    per frame: right keypoints listed on every row of
//                    [floor(y - 2 s), ceil(y + 2 s)]  (:840-849)
//   k_stereo_match   per left keypoint (one wave): row candidates -> Hamming
//                    best (:859-893), 11-shift 11x11 L1 window sweep with
//                    v_sad_u8, parabola, disparity (:896-963)
//   k_stereo_median  per frame: median of the kept window distances, drop
//                    matches >= 1.5 * 1.4 * median (:965-980)
//
// Float expressions follow the reference's evaluation order; the file is
// compiled with -ffp-contract=off (no product in them is inexact anyway).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "orb_plan.h"
#include "stereo_launch.h"

namespace orbgpu {

namespace {

constexpr int kThHigh = 100, kThLow = 50;       // ORBmatcher::TH_HIGH / TH_LOW (orb_matcher.cc:35-36)
constexpr int kThOrbDist = (kThHigh + kThLow) / 2;  // :832
constexpr int kWin = 5, kSweep = 5;             // w, L (:902, :909)
constexpr int kKpFloats = 7;                    // orbgpu_keypoint

__device__ __forceinline__ int kp_octave(const float* k) { return __float_as_int(k[5]); }

__device__ __forceinline__ const uint8_t* side_plane(const PlanHeader* P, const StereoSide& s, int f,
                                                     int l, int& pitch) {
  if (l == 0) {
    pitch = s.img_stride;
    return s.img0 + (size_t)f * s.img_fstride;
  }
  pitch = P->lev[l].pitch;
  return s.pyr + (size_t)f * s.pyr_fstride + P->lev[l].pyr_off;
}

__device__ __forceinline__ int reflect101(int i, int n) {
  i = i < 0 ? -i : i;
  return i >= n ? 2 * n - 2 - i : i;
}

// wave minimum, result in every lane (DPP row shifts + row broadcasts, then
// lane 63 read back)
__device__ __forceinline__ uint32_t wave_umin(uint32_t v) {
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)0xffffffff, (int)v, 0x111, 0xf, 0xf, false));
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)0xffffffff, (int)v, 0x112, 0xf, 0xf, false));
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)0xffffffff, (int)v, 0x114, 0xf, 0xf, false));
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)0xffffffff, (int)v, 0x118, 0xf, 0xf, false));
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)0xffffffff, (int)v, 0x142, 0xa, 0xf, false));
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)0xffffffff, (int)v, 0x143, 0xc, 0xf, false));
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// rows [floor(y - 2 s), ceil(y + 2 s)] of right keypoint k, clipped to the table
__device__ __forceinline__ void kp_rows(const PlanHeader* P, const float* k, int rows, int& y0, int& y1) {
  const float y = k[1];
  const float r = 2.0f * P->lev[kp_octave(k)].scale;
  y1 = min((int)ceilf(y + r), rows - 1);
  y0 = max((int)floorf(y - r), 0);
}

// Block-wide inclusive scan of one int per thread (256 threads): wave scans
// by lane shuffles, the four wave totals through LDS -- two barriers (the
// LDS ladder it replaces took seventeen).  tmp[t] holds thread t's inclusive
// value on return (tmp[255]: the total).
__device__ __forceinline__ int block_scan256(int v, int* tmp) {
  __shared__ int wtot[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int incl = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int o = __shfl_up(incl, off, 64);
    if (lane >= off) incl += o;
  }
  if (lane == 63) wtot[w] = incl;
  __syncthreads();
  incl += (w > 0 ? wtot[0] : 0) + (w > 1 ? wtot[1] : 0) + (w > 2 ? wtot[2] : 0);
  tmp[threadIdx.x] = incl;
  __syncthreads();
  return incl;
}

}  // namespace

// Row table of frame blockIdx.x: counts, exclusive scan, scatter.  List order
// within a row is arbitrary: k_stereo_match takes the (distance, index)
// minimum, which is the reference's first strict minimum over its ascending
// candidate list.
__global__ __launch_bounds__(256) void k_stereo_rows(StereoLaunch a) {
  extern __shared__ int cnt[];  // a.rows
  __shared__ int tmp[256];
  const PlanHeader* P = a.plan;
  const int f = blockIdx.x, R = a.rows;
  const int nr = min(a.R.n[(size_t)f * a.R.n_fstride], a.cap);
  const float* kr = a.R.kps + (size_t)f * a.R.kp_fstride * kKpFloats;
  for (int y = threadIdx.x; y < R; y += 256) cnt[y] = 0;
  __syncthreads();
  for (int i = threadIdx.x; i < nr; i += 256) {
    int y0, y1;
    kp_rows(P, kr + kKpFloats * i, R, y0, y1);
    for (int y = y0; y <= y1; ++y) atomicAdd(&cnt[y], 1);
  }
  __syncthreads();
  const int per = (R + 255) / 256, lo = min((int)threadIdx.x * per, R), hi = min(lo + per, R);
  int s = 0;
  for (int y = lo; y < hi; ++y) s += cnt[y];
  const int incl = block_scan256(s, tmp);
  int base = incl - s;
  for (int y = lo; y < hi; ++y) {
    const int c = cnt[y];
    cnt[y] = base;
    base += c;
  }
  if (threadIdx.x == 255) {
    if (a.zero_err)
      *a.err = incl > a.list_cap ? 16 : 0;  // the one-frame call's own word (one block)
    else if (incl > a.list_cap)
      atomicOr(a.err, 16);
  }
  __syncthreads();
  uint16_t* list = a.lists + (size_t)f * a.list_cap;
  for (int i = threadIdx.x; i < nr; i += 256) {
    int y0, y1;
    kp_rows(P, kr + kKpFloats * i, R, y0, y1);
    for (int y = y0; y <= y1; ++y) {
      const int pos = atomicAdd(&cnt[y], 1);
      if (pos < a.list_cap) list[pos] = (uint16_t)i;
    }
  }
  __syncthreads();
  for (int y = threadIdx.x; y < R; y += 256) a.row_end[(size_t)f * R + y] = min(cnt[y], a.list_cap);
}

// One wave per left keypoint slot.
__global__ __launch_bounds__(256) void k_stereo_match(StereoLaunch a) {
  const PlanHeader* P = a.plan;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const long gid = (long)blockIdx.x * 4 + wave;
  const int f = (int)(gid / a.cap), iL = (int)(gid - (long)f * a.cap);
  if (f >= a.n_frames) return;
  const int nl = min(a.L.n[(size_t)f * a.L.n_fstride], a.cap);
  if (iL >= nl) return;
  const size_t o = (size_t)f * a.out_fstride + iL;
  float out_u = -1.0f, out_d = -1.0f;
  int out_s = -1;

  const float* kl = a.L.kps + ((size_t)f * a.L.kp_fstride + iL) * kKpFloats;
  const float uL = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__float_as_int(kl[0])));
  const float vL = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__float_as_int(kl[1])));
  const int octL = __builtin_amdgcn_readfirstlane(kp_octave(kl));
  const float maxD = a.bf / a.mb;  // minZ = mb, minD = 0 (:851-854)
  const float minU = uL - maxD, maxU = uL - 0.0f;
  const int row = (int)vL;  // vRowIndices[vL] (:864); vL >= 0
  do {
    if (vL < 0.0f || row >= a.rows || maxU < 0) break;
    const int* re = a.row_end + (size_t)f * a.rows;
    const int beg = row ? re[row - 1] : 0, end = re[row];
    if (beg >= end) break;

    // ---- Hamming search over the row's candidates (:872-893)
    const uint32_t* dl = reinterpret_cast<const uint32_t*>(a.L.desc + ((size_t)f * a.L.kp_fstride + iL) * 32);
    uint32_t dls[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) dls[k] = __builtin_amdgcn_readfirstlane(dl[k]);
    const uint16_t* list = a.lists + (size_t)f * a.list_cap;
    const float* krf = a.R.kps + (size_t)f * a.R.kp_fstride * kKpFloats;
    const uint8_t* drf = a.R.desc + (size_t)f * a.R.kp_fstride * 32;
    uint32_t key = 0xffffffffu;
    for (int j = beg + lane; j < end; j += 64) {
      const int iR = list[j];
      const float* kr = krf + kKpFloats * iR;
      const int oct = kp_octave(kr);
      const float uR = kr[0];
      if (oct < octL - 1 || oct > octL + 1) continue;
      if (uR >= minU && uR <= maxU) {
        const uint4* dr = reinterpret_cast<const uint4*>(drf + 32 * (size_t)iR);
        const uint4 x0 = dr[0], x1 = dr[1];
        const int dist = __popc(dls[0] ^ x0.x) + __popc(dls[1] ^ x0.y) + __popc(dls[2] ^ x0.z) +
                         __popc(dls[3] ^ x0.w) + __popc(dls[4] ^ x1.x) + __popc(dls[5] ^ x1.y) +
                         __popc(dls[6] ^ x1.z) + __popc(dls[7] ^ x1.w);
        // iR < 65536 (u16 row lists; the entry points refuse larger caps),
        // dist < kThHigh = 100: (dist << 16) | iR orders by (dist, iR)
        if (dist < kThHigh) key = min(key, ((uint32_t)dist << 16) | (uint32_t)iR);
      }
    }
    key = wave_umin(key);
    if (key == 0xffffffffu || (int)(key >> 16) >= kThOrbDist) break;
    const int best = (int)(key & 0xffff);

    // ---- window sweep at the keypoint's octave (:898-935)
    const float uR0 = krf[kKpFloats * best];
    const LevelGeom& g = P->lev[octL];
    const float scaleFactor = g.inv_scale;
    const float scaleduL = roundf(uL * scaleFactor);
    const float scaledvL = roundf(vL * scaleFactor);
    const float scaleduR0 = roundf(uR0 * scaleFactor);
    const float iniu = scaleduR0 + kSweep - kWin;
    const float endu = scaleduR0 + kSweep + kWin + 1;
    if (iniu < 0 || endu >= g.w) break;
    int lp, rp;
    const uint8_t* Lp = side_plane(P, a.L, f, octL, lp);
    const uint8_t* Rp = side_plane(P, a.R, f, octL, rp);
    const int xl = (int)scaleduL, yl = (int)scaledvL, xr = (int)scaleduR0;
    const int incR = lane - kSweep;
    uint32_t s = 0;
    if (lane <= 2 * kSweep) {
      // windows inside the level (and the 12th byte of each dword triple
      // inside the row): unaligned dword loads + v_sad_u8; otherwise bytes
      // with the reflect-101 border of the reference's padded pyramid storage
      const bool inside = yl - kWin >= 0 && yl + kWin < g.h && xl - kWin >= 0 && xl + kWin + 1 < g.w &&
                          xr - kWin - kSweep >= 0 && xr + kWin + kSweep + 1 < g.w;
      if (inside) {
#pragma unroll
        for (int dy = -kWin; dy <= kWin; ++dy) {
          const uint8_t* lr = Lp + (size_t)(yl + dy) * lp + (xl - kWin);
          const uint8_t* rr = Rp + (size_t)(yl + dy) * rp + (xr + incR - kWin);
          uint32_t l0, l1, l2, r0, r1, r2;
          __builtin_memcpy(&l0, lr, 4);
          __builtin_memcpy(&l1, lr + 4, 4);
          __builtin_memcpy(&l2, lr + 8, 4);
          __builtin_memcpy(&r0, rr, 4);
          __builtin_memcpy(&r1, rr + 4, 4);
          __builtin_memcpy(&r2, rr + 8, 4);
          s = __builtin_amdgcn_sad_u8(l0, r0, s);
          s = __builtin_amdgcn_sad_u8(l1, r1, s);
          s = __builtin_amdgcn_sad_u8(l2 & 0x00ffffffu, r2 & 0x00ffffffu, s);
        }
      } else {
        for (int dy = -kWin; dy <= kWin; ++dy) {
          const uint8_t* lr = Lp + (size_t)reflect101(yl + dy, g.h) * lp;
          const uint8_t* rr = Rp + (size_t)reflect101(yl + dy, g.h) * rp;
          for (int dx = -kWin; dx <= kWin; ++dx) {
            const int d = (int)lr[reflect101(xl + dx, g.w)] - (int)rr[reflect101(xr + incR + dx, g.w)];
            s += (uint32_t)(d < 0 ? -d : d);
          }
        }
      }
    }
    // first strict minimum in incR order (:926-931): min of (dist, lane)
    const uint32_t k2 = wave_umin(lane <= 2 * kSweep ? (s << 4) | (uint32_t)lane : 0xffffffffu);
    const int bi = (int)(k2 & 15), sadBest = (int)(k2 >> 4);
    if (bi == 0 || bi == 2 * kSweep) break;  // bestincR == -L or +L (:937)

    // ---- parabola, disparity (:939-962)
    const float dist1 = (float)__builtin_amdgcn_readlane((int)s, bi - 1);
    const float dist2 = (float)sadBest;
    const float dist3 = (float)__builtin_amdgcn_readlane((int)s, bi + 1);
    const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
    if (deltaR < -1 || deltaR > 1) break;
    float bestuR = g.scale * ((float)scaleduR0 + (float)(bi - kSweep) + deltaR);
    float disparity = uL - bestuR;
    if (disparity >= 0.0f && disparity < maxD) {
      if (disparity <= 0) {
        disparity = (float)0.01;
        bestuR = (float)((double)uL - 0.01);
      }
      out_d = a.bf / disparity;
      out_u = bestuR;
      out_s = sadBest;
    }
  } while (false);
  if (lane == 0) {
    a.uright[o] = out_u;
    a.depth[o] = out_d;
    a.sad[o] = out_s;
  }
}

// Median filter of frame blockIdx.x (:965-980): the (m/2)-th smallest kept
// window distance by a two-pass radix select (distances < 2^15).  m: kept
// matches (> 0), h / incl: this thread's first-pass bucket count and
// inclusive scan.
__device__ __forceinline__ void median_filter(const StereoLaunch& a, int f, int nl, const int* sad, int* hist,
                                              int* tmp, int* sel, int h, int incl, int m) {
  const int k = m / 2;
  if (incl > k && incl - h <= k) sel[0] = threadIdx.x, sel[1] = k - (incl - h);
  __syncthreads();
  const int hi = sel[0], k2 = sel[1];
  hist[threadIdx.x] = 0;
  __syncthreads();
  for (int i = threadIdx.x; i < nl; i += 256)
    if (sad[i] >= 0 && (sad[i] >> 7) == hi) atomicAdd(&hist[sad[i] & 127], 1);
  __syncthreads();
  h = threadIdx.x < 128 ? hist[threadIdx.x] : 0;
  incl = block_scan256(h, tmp);
  if (threadIdx.x < 128 && incl > k2 && incl - h <= k2) sel[0] = (hi << 7) | (int)threadIdx.x;
  __syncthreads();
  const float median = (float)sel[0];
  const float thDist = 1.5f * 1.4f * median;
  for (int i = threadIdx.x; i < nl; i += 256)
    if (sad[i] >= 0 && !((float)sad[i] < thDist)) {
      const size_t o = (size_t)f * a.out_fstride + i;
      a.uright[o] = -1;
      a.depth[o] = -1;
    }
}

__global__ __launch_bounds__(256) void k_stereo_median(StereoLaunch a) {
  __shared__ int hist[256];
  __shared__ int tmp[256];
  __shared__ int sel[2];
  const int f = blockIdx.x;
  const int nl = min(a.L.n[(size_t)f * a.L.n_fstride], a.cap);
  const int* sad = a.sad + (size_t)f * a.out_fstride;
  hist[threadIdx.x] = 0;
  __syncthreads();
  for (int i = threadIdx.x; i < nl; i += 256)
    if (sad[i] >= 0) atomicAdd(&hist[sad[i] >> 7], 1);
  __syncthreads();
  const int h = hist[threadIdx.x];
  const int incl = block_scan256(h, tmp);
  const int m = tmp[255];
  // m == 0 (uniform): the reference would read vDistIdx[0] of an empty list; nothing to filter
  if (m > 0) median_filter(a, f, nl, sad, hist, tmp, sel, h, incl, m);
  if (a.mirror_dst) {  // one-frame host call: the outputs into host memory by this one workgroup
    __syncthreads();                                   // this block's stores drained
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // fresh lines of k_stereo_match's outputs
    const uint4* s4 = reinterpret_cast<const uint4*>(a.mirror_src);
    uint4* d4 = reinterpret_cast<uint4*>(a.mirror_dst);
    for (int i = threadIdx.x; i < (a.mirror_bytes + 15) >> 4; i += 256) d4[i] = s4[i];
    __syncthreads();
    if (threadIdx.x == 0) {
      __threadfence_system();
      __hip_atomic_store(a.done_host, a.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

hipError_t launch_stereo(const StereoLaunch& a, hipStream_t st) {
  if (a.n_frames <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_stereo_rows, dim3(a.n_frames), dim3(256), (size_t)a.rows * sizeof(int), st, a);
  const long waves = (long)a.n_frames * a.cap;
  hipLaunchKernelGGL(k_stereo_match, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st, a);
  hipLaunchKernelGGL(k_stereo_median, dim3(a.n_frames), dim3(256), 0, st, a);
  return hipGetLastError();
}

}  // namespace orbgpu
