// gfx950 kernels of the ORB front-end.  One launch sequence per batch of
// images (stereo frames = 2 images each):
//
//   k_resize x (L-1)  pyramid level l from level l-1        orb_extractor.cc:1093-1117
//   k_blur            7x7 sigma-2 Gaussian of every level    :1054-1055
//   k_fast_cells      per-cell FAST-9/16 + NMS + fallback    :744-825
//   k_octree          DistributeOctTree per (image, level)   :542-742, 829-843
//   k_describe        IC_Angle + steered BRIEF per keypoint  :76-146, 847-848, 1060
//   k_assemble        level-0 scaling + mono/stereo layout   :1033-1090
//
// Integer stages are bit-exact restatements of the reference semantics
// (oracle/cv_semantics.h); the float stages (fastAtan2, cosf/sinf, sample
// coordinates) are compiled with -ffp-contract=off with every FMA explicit.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "orb_launch.h"
#include "orb_math_dev.h"
#include "orb_plan.h"

namespace orbgpu {

constexpr int8_t kPattern[1024] = {
#include "pattern31.inc"
};
// bit_pattern_31_ as floats (x0, x1, y0, y1) per test: one dwordx4 per lane,
// the x pair and the y pair each a packed-FP32 operand
struct PatternF {
  float4 p[256];
};
constexpr PatternF make_pattern_f() {
  PatternF t{};
  for (int i = 0; i < 256; ++i)
    t.p[i] = float4{(float)kPattern[4 * i], (float)kPattern[4 * i + 2], (float)kPattern[4 * i + 1],
                    (float)kPattern[4 * i + 3]};
  return t;
}
__constant__ PatternF c_pattern_f_tab = make_pattern_f();
#define c_pattern_f (c_pattern_f_tab.p)

// Profiling build only (make stamps): per-phase s_memtime totals.
#ifdef ORB_STAMPS
__device__ unsigned long long g_stamps[64 * 16];  // 64 spread copies of 16 counters
#define STAMP_ON_INIT                                        \
  unsigned long long st_acc_[16] = {};                       \
  unsigned long long st_prev_ = __builtin_amdgcn_s_memtime()
#define STAMP_ON(i)                                                  \
  do {                                                               \
    const unsigned long long st_now_ = __builtin_amdgcn_s_memtime(); \
    st_acc_[i] += st_now_ - st_prev_;                                \
    st_prev_ = st_now_;                                              \
  } while (0)
#define STAMP_ON_ADD(i, v) (st_acc_[i] += (unsigned long long)(v))
#define STAMP_ON_END                                                           \
  do {                                                                         \
    if ((threadIdx.x & 63) == 0) {                                             \
      _Pragma("unroll") for (int i_ = 0; i_ < 16; ++i_)                        \
        if (st_acc_[i_]) atomicAdd(&g_stamps[(blockIdx.x & 63) * 16 + i_], st_acc_[i_]); \
    }                                                                          \
  } while (0)
#endif
// ORB_STAMPS=1 instruments k_fast_cells, =2 k_octree (one kernel per build).
#if defined(ORB_STAMPS) && ORB_STAMPS == 1
#define STAMP_INIT STAMP_ON_INIT
#define STAMP(i) STAMP_ON(i)
#define STAMP_ADD(i, v) STAMP_ON_ADD(i, v)
#define STAMP_END STAMP_ON_END
#else
#define STAMP_INIT (void)0
#define STAMP(i) (void)0
#define STAMP_ADD(i, v) (void)0
#define STAMP_END (void)0
#endif
#if defined(ORB_STAMPS) && ORB_STAMPS == 2
#define OSTAMP_INIT STAMP_ON_INIT
#define OSTAMP(i) STAMP_ON(i)
#define OSTAMP_ADD(i, v) STAMP_ON_ADD(i, v)
#ifdef ORB_OCT_STAMP_L0  // level-0 blocks only (the single-image critical path)
#define OSTAMP_END \
  if (l == 0) STAMP_ON_END
#else
#define OSTAMP_END STAMP_ON_END
#endif
#else
#define OSTAMP_INIT (void)0
#define OSTAMP(i) (void)0
#define OSTAMP_ADD(i, v) (void)0
#define OSTAMP_END (void)0
#endif

// Row extents of the 31-px circular patch (orb_extractor.cc:452-464; fixed
// because kHalfPatchSize is fixed at 15).
__constant__ int kUmax[16] = {15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3};

enum : int { kErrNodeCap = 1, kErrOutCap = 2, kErrSlotCap = 4, kErrKpCap = 8 };

// Workgroups are dealt round-robin over the 8 XCDs (blockIdx % 8 labels the
// XCD group, MI355X_MICROARCH.md).  Consecutive work items share image rows
// (cell halos, keypoint patches), so give every XCD a contiguous range of
// them: its private L2 then serves the overlaps.  Bijective for any count.
__device__ __forceinline__ int xcd_remap(int bid, int nblocks) {
  const int q = nblocks >> 3, r = nblocks & 7;
  const int xcd = bid & 7, idx = bid >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

// kWT (the single-image dataflow launch, k_extract_df): a payload word that
// other workgroups of the same launch read is stored write-through (sc1: a
// relaxed agent-scope atomic store), so its producer needs no release fence
// before the counter that publishes it (MI355X_MICROARCH.md, inter-workgroup
// visibility, R1); the batch kernels store plainly.
template <bool kWT, class T>
__device__ __forceinline__ void st_pub(T* p, T v) {
  if constexpr (kWT)
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else
    *p = v;
}
// kWT: a wave-uniform read of another workgroup's output goes to a vector sc1
// load -- the consumer's acquire does not refresh the scalar cache, where a
// plain uniform load may be served from
template <bool kWT, class T>
__device__ __forceinline__ T ld_pub(const T* p) {
  if constexpr (kWT)
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else
    return *p;
}
constexpr int kAuxSc1 = 16;  // raw buffer store cache bits: sc1 (write-through)

struct ImgSrc {
  const uint8_t* base;  // image 0, level 0
  size_t pitch;         // bytes between images
  int stride;           // bytes between rows
};

__device__ __forceinline__ const uint8_t* level_plane(const PlanHeader* P, const ImgSrc& s,
                                                      const uint8_t* pyr, int img, int l,
                                                      int& pitch) {
  if (l == 0) {
    pitch = s.stride;
    return s.base + (size_t)img * s.pitch;
  }
  pitch = P->lev[l].pitch;
  return pyr + (size_t)img * P->pyr_bytes + P->lev[l].pyr_off;
}

// --------------------------------------------------------------------------
// k_resize: cv::resize INTER_LINEAR, 8UC1.  Horizontal
// taps are (sx, a0, a1) per column, vertical (r0, r1, b0, b1) per row, both
// precomputed by the planner.  Columns below vec8_end use the 128-bit SIMD
// rounding ((H>>4)*b >> 16 summed, +2 >> 2), the tail the scalar
// (H0*b0 + H1*b1 + 2^21) >> 22 -- exactly where OpenCV switches.
// A 256-thread block makes a kResizeTileW x kResizeTileH output tile from its
// source window staged in LDS (dwordx4 loads).  Each wave owns kResizeTileH/4
// consecutive output rows of it, each lane 4 adjacent columns; the wave
// streams the source rows once: the horizontal pass of a row (3 LDS dwords,
// two v_alignbyte_b32, then per column a v_perm_b32 with a per-lane selector
// and one v_dot2_u32_u16: h = s0*a0 + s1*a1) is kept in registers for the
// output rows that share it, with the next row's dwords already in flight.
// Tap weights lie in [0, 2048] and sum to <= 2049, so h < 2^19 and
// ((h>>4)*b) >> 16 is one full-rate v_mul_hi_u32_u24 of (h & ~15, b << 12);
// every result is <= 255.
// --------------------------------------------------------------------------
typedef unsigned short ushort2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ ushort2_t as_us2(uint32_t v) {
  return __builtin_bit_cast(ushort2_t, v);
}

struct RsRow {  // one source row of a lane's 4 columns: raw bytes
  uint32_t d[3];
};
__device__ __forceinline__ RsRow rs_load(const uint8_t* __restrict__ row, int base4,
                                         const int (&bi)[4], bool bytewise) {
  RsRow r;
  if (!bytewise) {
    r.d[0] = *reinterpret_cast<const uint32_t*>(row + base4);
    r.d[1] = *reinterpret_cast<const uint32_t*>(row + base4 + 4);
    r.d[2] = *reinterpret_cast<const uint32_t*>(row + base4 + 8);
  } else {  // tap span > 8 bytes (scale factors above 2): the 8 tap bytes
#pragma unroll
    for (int j = 0; j < 2; ++j)
      r.d[j] = (uint32_t)row[bi[2 * j] & 0xffff] | ((uint32_t)row[bi[2 * j] >> 16] << 8) |
               ((uint32_t)row[bi[2 * j + 1] & 0xffff] << 16) | ((uint32_t)row[bi[2 * j + 1] >> 16] << 24);
    r.d[2] = 0;
  }
  return r;
}
// (a * b) >> 32 of 24-bit operands: one full-rate v_mul_hi_u32_u24
__device__ __forceinline__ uint32_t mulhi24(uint32_t a, uint32_t b) {
  return (uint32_t)(((uint64_t)(a & 0xffffffu) * (uint64_t)(b & 0xffffffu)) >> 32);
}
// h[k] = s0*a0 + s1*a1 of column k; hq[k] = (h[k] >> 4) << 4 (the SIMD path's
// input, kept 16x scaled so the vertical step's ((h >> 4) * b) >> 16 is one
// mulhi24(hq, b << 12): h < 2^19, b << 12 <= 2^23)
__device__ __forceinline__ void rs_horiz(const RsRow& r, int off, const uint32_t (&sel)[4],
                                         const uint32_t (&aw)[4], bool bytewise, uint32_t (&h)[4],
                                         uint32_t (&hq)[4]) {
  if (!bytewise) {
    const uint32_t w0 = __builtin_amdgcn_alignbyte(r.d[1], r.d[0], off);
    const uint32_t w1 = __builtin_amdgcn_alignbyte(r.d[2], r.d[1], off);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      h[k] = __builtin_amdgcn_udot2(as_us2(__builtin_amdgcn_perm(w1, w0, sel[k])), as_us2(aw[k]), 0u, false);
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k)
      h[k] = __builtin_amdgcn_udot2(as_us2(__builtin_amdgcn_perm(0u, r.d[k >> 1], (k & 1) ? 0x0c030c02u : 0x0c010c00u)),
                                    as_us2(aw[k]), 0u, false);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) hq[k] = h[k] & ~15u;
}

// buffer resource word 3 for raw (stride 0, untyped dword) accesses on gfx9
constexpr int kBufRsrcWord3 = 0x00020000;

// Stages source rows [rr0, rr0 + nrow) x columns [c0, c1] (ncol = c1 - c0 + 1,
// a multiple of 16) of a level plane into LDS (row pitch ncol), 256 threads.
__device__ __forceinline__ void rs_stage(const uint8_t* S, int sp, int sw, int c0, int c1, int rr0, int nrow,
                                         uint8_t* __restrict__ lds, int tid) {
  const int ncol = c1 - c0 + 1;
  // 16-byte chunks when rows are 16-aligned and no chunk straddles the end of a
  // source row: chunks wholly past it are skipped (their LDS bytes only meet
  // the zero weight of the single-tap columns, sx + 1 = sw)
  if (((((uintptr_t)S) | (uintptr_t)sp) & 15) == 0 && (c1 < sp || (sw & 15) == 0)) {
    const int nq = (c1 < sp ? ncol : min(ncol, sw - c0)) >> 4, total = nrow * nq;
    const uint32_t mg = ((1u << 19) + nq - 1) / nq;
    // raw buffer loads on the window's first column: one 32-bit VGPR offset
    // per chunk, no 64-bit address arithmetic
    const __amdgpu_buffer_rsrc_t srs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t*>(S + c0), (short)0, (int)0xffffffff, kBufRsrcWord3);
    for (int i0 = 0; i0 < total; i0 += 1024) {
      uint4 v[4];
      int at[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = min(i0 + 256 * u + tid, total - 1);
        // i mg < rows 2^19 < 2^32: the 24-bit multiply's low word is the
        // product, and the shift gives i / nq exactly (rows nq^2 < 2^19, planner)
        const int r = (int)(__umul24((uint32_t)i, mg) >> 19), q = i - __mul24(r, nq);
        const auto w = __builtin_amdgcn_raw_buffer_load_b128(
            srs, (int)(__umul24((uint32_t)(rr0 + r), (uint32_t)sp) + 16u * (uint32_t)q), 0, 0);
        v[u] = make_uint4(w[0], w[1], w[2], w[3]);
        at[u] = __mul24(r, ncol) + 16 * q;  // LDS rows keep the window pitch ncol
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) *reinterpret_cast<uint4*>(lds + at[u]) = v[u];
    }
  } else {
    for (int i = tid; i < nrow * ncol; i += 256) {
      const int r = i / ncol, c = i - r * ncol;
      lds[i] = S[(size_t)(rr0 + r) * sp + min(c0 + c, sw - 1)];
    }
  }

}

// One output tile (tyx) of level l of image img by 256 threads (tid) with an
// LDS slice of PlanHeader::rs_lds bytes; every thread of the workgroup passes
// its one barrier.  live = false: the group takes part in the barrier and
// writes nothing (k_pyramid's spare groups).
// (the dataflow launch passes `wait`: its dependency wait, called by every
// thread once the plan-constant taps are in flight and before the source level
// is read; the batch kernels pass nothing)
struct NoWait {
  __device__ void operator()() const {}
};
template <bool kWT = false, class Wait = NoWait>
__device__ __forceinline__ void resize_tile(const PlanHeader* __restrict__ P, const int* __restrict__ rs_tab,
                                            const ImgSrc& src, uint8_t* __restrict__ pyr, int l, int img,
                                            int tyx, uint8_t* __restrict__ lds, int tid, bool live,
                                            const Wait& wait = Wait()) {
  constexpr int RW = kResizeTileH / 4;  // output rows per wave
  const LevelGeom& g = P->lev[l];
  const int sw = P->lev[l - 1].w;
  const int x0 = (tyx % g.rs_tiles_x) * kResizeTileW, y0 = (tyx / g.rs_tiles_x) * kResizeTileH;
  const int xl = min(x0 + kResizeTileW, g.w) - 1, yl = min(y0 + kResizeTileH, g.h) - 1;
  const int2* xt = reinterpret_cast<const int2*>(rs_tab + g.rs_x);
  const int2* yt = reinterpret_cast<const int2*>(rs_tab + g.rs_y);
  const int c0 = xt[x0].x & ~15;
  const int c1 = min(xt[xl].x + 1, sw - 1) | 15;
  const int rr0 = yt[y0].x & 0xffff, rr1 = yt[yl].x >> 16;
  const int ncol = c1 - c0 + 1, nrow = rr1 - rr0 + 1;  // ncol: multiple of 16
  int sp;
  const uint8_t* S = level_plane(P, src, pyr, img, l - 1, sp);

  // taps, fetched up front (before any store, so no wait ever queues behind one)
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int x = x0 + 4 * lane;
  const int ys = y0 + RW * wave;  // wave-uniform first output row
  int2 xa[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) xa[k] = xt[min(x + k, g.w - 1)];
  const int2 tl = yt[min(ys + (lane & (RW - 1)), yl)];

  wait();
  rs_stage(S, sp, sw, c0, c1, rr0, nrow, lds, tid);

  // per-lane column taps -> byte selectors relative to the lane's LDS window
  int sx[4], sx1[4];
  uint32_t aw[4], tail_k = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    sx[k] = xa[k].x - c0;
    sx1[k] = min(xa[k].x + 1, c1) - c0;
    aw[k] = (uint32_t)xa[k].y;
    if (min(x + k, g.w - 1) >= g.vec8_end) tail_k |= 1u << k;
  }
  const int lo = min(min(sx[0], sx[1]), min(sx[2], sx[3]));
  const int hi = max(max(sx1[0], sx1[1]), max(sx1[2], sx1[3]));
  const int base4 = lo & ~3, off = lo & 3;
  uint32_t sel[4];
  int bi[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    sel[k] = (uint32_t)(sx[k] - lo) | 0x0c00u | ((uint32_t)(sx1[k] - lo) << 16) | 0x0c000000u;
    bi[k] = sx[k] | (sx1[k] << 16);
  }
  const bool active = x < g.w;
  const bool bytewise = __builtin_amdgcn_ballot_w64(active && hi - lo > 7) != 0;
  const bool any_tail = __builtin_amdgcn_ballot_w64(active && tail_k != 0) != 0;
  __syncthreads();
  if (!live || ys > yl) return;  // after the barrier: every wave staged its share

  // stream the source rows: two register slots hold rows p and p+1 (slot sa
  // = row p; a wave-uniform flag, so advancing one row recomputes into the
  // freed slot and flips sa -- no register moves), row p+2 in flight
  const int last = nrow - 1;
  auto rowp = [&](int r) { return lds + min(r, last) * ncol; };
  uint32_t h0[4], h1[4], q0[4], q1[4];
  int sa = 0;
  RsRow nd;
  int p = -1000;
  uint8_t* D = pyr + (size_t)img * P->pyr_bytes + g.pyr_off + x;
  const int ye = min(ys + RW - 1, yl);
  // one output row from source rows A (= r0) and B (= r1; the call sites pass
  // A twice when r1 == r0, the clamped first / last source row)
  auto out_row = [&](int y, const uint32_t (&hA)[4], const uint32_t (&qA)[4], const uint32_t (&hB)[4],
                     const uint32_t (&qB)[4], uint32_t b0, uint32_t b1) {
    uint32_t v[4];  // 4x the output byte (< 2^12); the >> 2 is done packed below
    // (tail columns: h < 255 * 2^11 and b < 2^11, so 24-bit multiplies are exact)
    const uint32_t s0 = b0 << 12, s1 = b1 << 12;
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = mulhi24(qA[k], s0) + mulhi24(qB[k], s1) + 2;
    if (any_tail) {
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (tail_k & (1u << k)) v[k] = ((__umul24(hA[k], b0) + __umul24(hB[k], b1) + (1u << 21)) >> 22) << 2;
    }
    // two columns per 16-bit half: one packed shift per pair, one byte perm
    const ushort2_t p01 = as_us2(v[0] | (v[1] << 16)) >> (ushort2_t){2, 2};
    const ushort2_t p23 = as_us2(v[2] | (v[3] << 16)) >> (ushort2_t){2, 2};
    // columns past w land in the pitch padding (pitch is a multiple of 16)
    if (active)
      st_pub<kWT>(reinterpret_cast<uint32_t*>(D + __umul24((uint32_t)y, (uint32_t)g.pitch)),
                  __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, p23), __builtin_bit_cast(uint32_t, p01),
                                        0x06040200u));
  };
  for (int y = ys; y <= ye; ++y) {
    const int tx = __builtin_amdgcn_readlane(tl.x, y - ys), ty = __builtin_amdgcn_readlane(tl.y, y - ys);
    const int r0 = (tx & 0xffff) - rr0, r1 = (int)((uint32_t)tx >> 16) - rr0;
    if (r0 < p || r0 > p + 2) {
      p = r0;
      sa = 0;
      rs_horiz(rs_load(rowp(p), base4, bi, bytewise), off, sel, aw, bytewise, h0, q0);
      rs_horiz(rs_load(rowp(p + 1), base4, bi, bytewise), off, sel, aw, bytewise, h1, q1);
      nd = rs_load(rowp(p + 2), base4, bi, bytewise);
    } else {
      while (p < r0) {  // row p + 2 into the slot of row p, which becomes row p + 1's partner
        if (sa == 0)
          rs_horiz(nd, off, sel, aw, bytewise, h0, q0);
        else
          rs_horiz(nd, off, sel, aw, bytewise, h1, q1);
        sa ^= 1;
        ++p;
        nd = rs_load(rowp(p + 2), base4, bi, bytewise);
      }
    }
    const uint32_t b0 = (uint32_t)ty & 0xffffu, b1 = (uint32_t)ty >> 16;
    if (r1 == r0) {  // wave-uniform (SGPR) branch, rare
      if (sa == 0)
        out_row(y, h0, q0, h0, q0, b0, b1);
      else
        out_row(y, h1, q1, h1, q1, b0, b1);
    } else if (sa == 0) {
      out_row(y, h0, q0, h1, q1, b0, b1);
    } else {
      out_row(y, h1, q1, h0, q0, b0, b1);
    }
  }
}

// The narrow right-hand tail of level l (columns [rs_tail_x0, w): at most
// kRsTailGroups groups of 4) for output rows [64 tb, 64 tb + 64): in the tile
// layout those columns would leave most lanes of their waves idle.  Here lane
// = output row, the 4 waves share the 64 rows and take the column groups
// round robin; a group's taps are wave-uniform (scalar), every lane runs the
// horizontal pass on its own two source rows (no reuse across output rows)
// and the same vertical rounding as resize_tile: the same bytes.  One barrier
// (after staging), as resize_tile.
template <bool kWT = false, class Wait = NoWait>
__device__ __forceinline__ void resize_tail(const PlanHeader* __restrict__ P, const int* __restrict__ rs_tab,
                                            const ImgSrc& src, uint8_t* __restrict__ pyr, int l, int img,
                                            int tb, uint8_t* __restrict__ lds, int tid, const Wait& wait = Wait()) {
  const LevelGeom& g = P->lev[l];
  const int sw = P->lev[l - 1].w;
  const int2* xt = reinterpret_cast<const int2*>(rs_tab + g.rs_x);
  const int2* yt = reinterpret_cast<const int2*>(rs_tab + g.rs_y);
  const int x0 = g.rs_tail_x0, y0 = 64 * tb, yl = min(y0 + 63, g.h - 1);
  const int c0 = xt[x0].x & ~15;
  const int c1 = min(xt[g.w - 1].x + 1, sw - 1) | 15;
  const int rr0 = yt[y0].x & 0xffff, rr1 = yt[yl].x >> 16;
  const int ncol = c1 - c0 + 1, nrow = rr1 - rr0 + 1;
  int sp;
  const uint8_t* S = level_plane(P, src, pyr, img, l - 1, sp);
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int y = y0 + lane;
  const int2 ty = yt[min(y, yl)];
  wait();
  rs_stage(S, sp, sw, c0, c1, rr0, nrow, lds, tid);
  __syncthreads();
  const uint8_t* rowA = lds + ((ty.x & 0xffff) - rr0) * ncol;
  const uint8_t* rowB = lds + ((int)((uint32_t)ty.x >> 16) - rr0) * ncol;
  const uint32_t b0 = (uint32_t)ty.y & 0xffffu, b1 = (uint32_t)ty.y >> 16;
  const uint32_t s0 = b0 << 12, s1 = b1 << 12;
  uint8_t* D = pyr + (size_t)img * P->pyr_bytes + g.pyr_off + (size_t)min(y, yl) * g.pitch;
  const int ng = (g.w - x0 + 3) >> 2;
  for (int q = wave; q < ng; q += 4) {  // wave-uniform
    const int x = x0 + 4 * q;
    int sx[4], sx1[4], bi[4];
    uint32_t aw[4], tail_k = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int2 xa = xt[min(x + k, g.w - 1)];
      sx[k] = xa.x - c0;
      sx1[k] = min(xa.x + 1, c1) - c0;
      aw[k] = (uint32_t)xa.y;
      bi[k] = sx[k] | (sx1[k] << 16);
      if (min(x + k, g.w - 1) >= g.vec8_end) tail_k |= 1u << k;
    }
    const int lo = min(min(sx[0], sx[1]), min(sx[2], sx[3]));
    const int hi = max(max(sx1[0], sx1[1]), max(sx1[2], sx1[3]));
    const int base4 = lo & ~3, off = lo & 3;
    uint32_t sel[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      sel[k] = (uint32_t)(sx[k] - lo) | 0x0c00u | ((uint32_t)(sx1[k] - lo) << 16) | 0x0c000000u;
    const bool bytewise = hi - lo > 7;
    uint32_t hA[4], qA[4], hB[4], qB[4];
    rs_horiz(rs_load(rowA, base4, bi, bytewise), off, sel, aw, bytewise, hA, qA);
    rs_horiz(rs_load(rowB, base4, bi, bytewise), off, sel, aw, bytewise, hB, qB);
    uint32_t v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = mulhi24(qA[k], s0) + mulhi24(qB[k], s1) + 2;
    if (tail_k) {
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (tail_k & (1u << k)) v[k] = ((__umul24(hA[k], b0) + __umul24(hB[k], b1) + (1u << 21)) >> 22) << 2;
    }
    const ushort2_t p01 = as_us2(v[0] | (v[1] << 16)) >> (ushort2_t){2, 2};
    const ushort2_t p23 = as_us2(v[2] | (v[3] << 16)) >> (ushort2_t){2, 2};
    if (y <= yl)
      st_pub<kWT>(reinterpret_cast<uint32_t*>(D + x),
                  __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, p23), __builtin_bit_cast(uint32_t, p01),
                                        0x06040200u));
  }
}

// k_resize: one tile per workgroup, one launch per level (tiles of all the
// batch's images).
__global__ __launch_bounds__(256) void k_resize(const PlanHeader* __restrict__ P,
                                                const int* __restrict__ rs_tab, ImgSrc src,
                                                uint8_t* __restrict__ pyr, int l) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const LevelGeom& g = P->lev[l];
  const int nt = g.rs_tiles_x * g.rs_tiles_y, per = nt + g.rs_tail_blocks;
  const int wid = xcd_remap(blockIdx.x, gridDim.x);
  const int img = wid / per;
  const int t = wid - img * per;
  if (t < nt)
    resize_tile(P, rs_tab, src, pyr, l, img, t, lds, threadIdx.x, true);
  else
    resize_tail(P, rs_tab, src, pyr, l, img, t - nt, lds, threadIdx.x);
}

// k_pyramid: the whole chain (levels 1 .. L-1) of one image per workgroup of
// G x 256 threads in ONE launch: the G groups take a level's tiles G at a
// time (each its own LDS slice, the same tile code as k_resize, so the same
// bytes), and the workgroup barrier after a level's last round orders its
// stores before the next level's loads -- no cross-workgroup dependency, so
// no grid-wide flag or fence.  Opt-in (ORBGPU_RESIZE=fused): at 256 images
// a launch it took 0.28 ms against 0.22 ms for the seven per-level launches
// (each of which spreads one level over the whole device at full occupancy),
// DESIGN §4.
__global__ __launch_bounds__(1024) void k_pyramid(const PlanHeader* __restrict__ P,
                                                  const int* __restrict__ rs_tab, ImgSrc src,
                                                  uint8_t* __restrict__ pyr, int rs_lds) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int G = blockDim.x >> 8;
  const int grp = __builtin_amdgcn_readfirstlane(threadIdx.x >> 8), tid = threadIdx.x & 255;
  const int img = xcd_remap(blockIdx.x, gridDim.x);
  uint8_t* const my = lds + grp * rs_lds;
  for (int l = 1; l < P->levels; ++l) {
    const LevelGeom& g = P->lev[l];
    const int nm = g.rs_tiles_x * g.rs_tiles_y, nt = nm + g.rs_tail_blocks;
    for (int t0 = 0; t0 < nt; t0 += G) {
      const int tile = t0 + grp;
      if (tile >= nm && tile < nt)  // group-uniform; one barrier either way
        resize_tail(P, rs_tab, src, pyr, l, img, tile - nm, my, tid);
      else
        resize_tile(P, rs_tab, src, pyr, l, img, tile < nt ? tile : 0, my, tid, tile < nt);
      __syncthreads();  // the slice is restaged by the group's next tile; the level is complete
    }
  }
}

// --------------------------------------------------------------------------
// k_blur: GaussianBlur 7x7, sigma 2, BORDER_REFLECT_101, bit-exact fixed point
// (SURVEY Appendix A.3): Q8 taps [18 34 48 56 48 34 18], horizontal sums kept
// exact, (sum + 2^15) >> 16 once.  Interior: each thread owns 4 adjacent
// columns x 8 rows (3 dword loads per source row, dot4/dot2 taps); a 256-thread
// block covers 256 x 32 outputs and one launch covers every level of every
// image.  Edge lanes rebuild their reflected window with
// v_perm_b32 (see k_blur), so no wave runs a separate border path.
// --------------------------------------------------------------------------
__device__ __forceinline__ int reflect101(int i, int n) {
  i = i < 0 ? -i : i;
  return i >= n ? 2 * n - 2 - i : i;
}


// Every lane owns output columns x..x+3 (x = 4k) of R rows.  It loads the 12
// source bytes x-4..x+7 of each row as 3 dwords from an in-row offset clamped
// to [0, w-12]; lanes at the left/right edge (x = 0, x > w-8) rebuild the
// reflect-101 window from those bytes with v_perm_b32 and per-lane selectors.
// Only waves holding an edge lane take that (wave-uniform) branch, and the
// arithmetic after it is the same for every lane: no divergent border path.
__device__ __forceinline__ void blur_window_sel(int x, int w, int base, uint32_t (&lo)[3],
                                                uint32_t (&hi)[3]) {
#pragma unroll
  for (int v = 0; v < 3; ++v) {
    lo[v] = 0;
    hi[v] = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int idx = reflect101(x - 4 + 4 * v + b, w) - base;  // 0..11
      lo[v] |= (uint32_t)(idx < 8 ? idx : 0x0c) << (8 * b);      // 0x0c selects 0x00
      hi[v] |= (uint32_t)(idx < 8 ? 0x0c : idx - 8) << (8 * b);
    }
  }
}

// A/B switch: k_blur and k_octree held to 64 VGPRs (8 waves a SIMD), for
// the co-residency of the concurrent pipelines' kernels
#ifndef ORB_OCC8
#define ORB_OCC8 0
#endif
#if ORB_OCC8
#define ORB_WPE8 __attribute__((amdgpu_waves_per_eu(8, 8)))
#else
#define ORB_WPE8
#endif
// the tail-strip path must not raise k_blur's register count above the
// strip path's 68 (7 waves a SIMD)
#if ORB_OCC8
#define ORB_BLUR_WPE
#else
#define ORB_BLUR_WPE __attribute__((amdgpu_waves_per_eu(7, 8)))
#endif
#ifndef ORB_BLUR_PF
#define ORB_BLUR_PF 6  // (call L: 6 / 4 / 8 rows -> 68 / 62 / 73 VGPRs, 131.4k / 131.3k / 131.0k frames/s)
#endif
// One wave's blur strip: every lane owns columns x..x+3 of R output rows from
// ys (kTail: ys per lane -- the strips of a tail wave -- else wave-uniform).
template <bool kTail, int kAux = 0>
__device__ __forceinline__ void blur_strip(const PlanHeader* __restrict__ P, const LevelGeom& g,
                                           const uint8_t* S, int sp, uint8_t* __restrict__ dst,
                                           int x, int ys) {
  constexpr int R = kBlurTileH / 4;  // output rows per thread
  const uint32_t base = (uint32_t)min(max(x - 4, 0), g.w - 12);
  // Streamed down the strip: the 3 dword loads of source row r + kPf are
  // issued while row r is filtered horizontally, and output row r - 6 leaves
  // as soon as its 7 rows exist, so only a 7-row window of sums is live.
  constexpr int kPf = ORB_BLUR_PF;  // rows of loads in flight
  // edge: some lane's window is clamped at the right border (or the level is
  // narrower than a wave's span) -- every lane rebuilds its window by
  // per-lane selectors; edgeL: the only clamped lane is x = 0, whose window
  // -4..7 reflects to bytes (4 3 2 1)(0 1 2 3)(4 5 6 7) of its load: one
  // perm and two selects per row instead of three perms and three ors
  const bool edge = __builtin_amdgcn_ballot_w64((int)base != x - 4 && x != 0) != 0;
  const bool edgeL = !edge && __builtin_amdgcn_ballot_w64(x == 0) != 0;
  const bool isL = x == 0;
  uint32_t lo_sel[3] = {0, 0, 0}, hi_sel[3] = {0, 0, 0};
  if (edge) blur_window_sel(x, g.w, (int)base, lo_sel, hi_sel);
  uint32_t d[R + 6][3];
  // the level's height and pitch held in registers: the buffer stores are
  // opaque to alias analysis and would make them reloaded every row
  const int gh = g.h, pitch = g.pitch;
  // raw buffer accesses: the lane's column is the VGPR offset, the row the
  // SGPR offset (kTail: the row is per lane, in the VGPR offset), so no
  // per-row 64-bit address arithmetic on the VALU
  const __amdgpu_buffer_rsrc_t srs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t*>(S), (short)0, (int)0xffffffff, kBufRsrcWord3);
  auto load_row = [&](int r) {
    // (kTail: the row is per lane -- a 24-bit multiply, full rate; else
    // wave-uniform, on the scalar unit)
    const int ro = kTail ? (int)__umul24((uint32_t)reflect101(ys - 3 + r, gh), (uint32_t)sp)
                         : reflect101(ys - 3 + r, gh) * sp;
    const auto w = kTail ? __builtin_amdgcn_raw_buffer_load_b96(srs, (int)base + ro, 0, 0)
                         : __builtin_amdgcn_raw_buffer_load_b96(srs, (int)base, ro, 0);
#pragma unroll
    for (int k = 0; k < 3; ++k) d[r][k] = w[k];
  };
#pragma unroll
  for (int r = 0; r < kPf && r < R + 6; ++r) load_row(r);
  // horizontal taps: two v_dot4_u32_u8 per output on windows cut by alignbyte;
  // sums are <= 65280, so row pairs pack into one dword for the vertical dot2s
  const uint32_t K0 = 18u | (34u << 8) | (48u << 16) | (56u << 24);
  const uint32_t K1 = 48u | (34u << 8) | (18u << 16);
  // vertical taps (18,34)(48,56)(48,34)(18,0) as four v_dot2_u32_u16, the
  // +2^15 rounding in the first accumulator; results < 2^24, so each output
  // byte is byte 2 of its sum and two v_perm_b32 pack four of them.
  const ushort2_t k01 = as_us2(18u | (34u << 16)), k23 = as_us2(48u | (56u << 16));
  const ushort2_t k45 = as_us2(48u | (34u << 16)), k6 = as_us2(18u);
  // columns past w land in the row's pitch padding (pitch is a multiple of 16)
  const __amdgpu_buffer_rsrc_t drs = __builtin_amdgcn_make_buffer_rsrc(dst, (short)0, (int)0xffffffff,
                                                                       kBufRsrcWord3);
  uint32_t hw[R + 6][4];
  uint32_t pr[R + 5][4];  // pr[r] = hw[r] | hw[r+1] << 16
#pragma unroll
  for (int r = 0; r < R + 6; ++r) {
    if (r + kPf < R + 6) load_row(r + kPf);
    if (edge) {  // edge lanes rebuild their reflect-101 window (wave-uniform branch)
      uint32_t v[3];
#pragma unroll
      for (int k = 0; k < 3; ++k)
        v[k] = __builtin_amdgcn_perm(d[r][1], d[r][0], lo_sel[k]) | __builtin_amdgcn_perm(d[r][2], d[r][2], hi_sel[k]);
#pragma unroll
      for (int k = 0; k < 3; ++k) d[r][k] = v[k];
    } else if (edgeL) {
      const uint32_t d0 = d[r][0], d1 = d[r][1];
      d[r][0] = __builtin_amdgcn_perm(d1, d0, isL ? 0x01020304u : 0x03020100u);
      d[r][1] = isL ? d0 : d1;
      d[r][2] = isL ? d1 : d[r][2];
    }
    const uint32_t lo[4] = {__builtin_amdgcn_alignbyte(d[r][1], d[r][0], 1),
                            __builtin_amdgcn_alignbyte(d[r][1], d[r][0], 2),
                            __builtin_amdgcn_alignbyte(d[r][1], d[r][0], 3), d[r][1]};
    const uint32_t hi[4] = {__builtin_amdgcn_alignbyte(d[r][2], d[r][1], 1),
                            __builtin_amdgcn_alignbyte(d[r][2], d[r][1], 2),
                            __builtin_amdgcn_alignbyte(d[r][2], d[r][1], 3), d[r][2]};
#pragma unroll
    for (int j = 0; j < 4; ++j)
      hw[r][j] = __builtin_amdgcn_udot4(lo[j], K0, __builtin_amdgcn_udot4(hi[j], K1, 0u, false), false);
    if (r >= 1)
#pragma unroll
      for (int j = 0; j < 4; ++j) pr[r - 1][j] = hw[r - 1][j] | (hw[r][j] << 16);
    if (r >= 6) {
      const int o = r - 6;
      if (ys + o < gh) {
        uint32_t v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          uint32_t a = __builtin_amdgcn_udot2(as_us2(pr[o][j]), k01, 1u << 15, false);
          a = __builtin_amdgcn_udot2(as_us2(pr[o + 2][j]), k23, a, false);
          a = __builtin_amdgcn_udot2(as_us2(pr[o + 4][j]), k45, a, false);
          v[j] = __builtin_amdgcn_udot2(as_us2(hw[o + 6][j]), k6, a, false);
        }
        const uint32_t packed =
            __builtin_amdgcn_perm(v[1], v[0], 0x0c0c0602u) | __builtin_amdgcn_perm(v[3], v[2], 0x06020c0cu);
        if (kTail)
          __builtin_amdgcn_raw_buffer_store_b32(packed, drs, x + (int)__umul24((uint32_t)(ys + o), (uint32_t)pitch), 0, kAux);
        else
          __builtin_amdgcn_raw_buffer_store_b32(packed, drs, x, (ys + o) * pitch, kAux);
      }
    }
  }
}

// waves per k_blur workgroup (A/B: 1 = every strip its own workgroup; the
// strips never synchronise)
#ifndef ORB_BLUR_WAVES
#define ORB_BLUR_WAVES 4
#endif
// One wave of blur tile t (over all levels of an image, PlanHeader::blur_tiles)
// of image img: a full tile's R-row strip `wave` (threadIdx.x >> 6), or the
// tail strips of tail wave 4 (t - nfull) + wave.  No synchronisation.
// (ORB_BLUR_WAVES == 1: the wave is bid & 3 of the one-wave workgroups)
template <bool kWT>
__device__ __forceinline__ void blur_wave(const PlanHeader* __restrict__ P, ImgSrc src,
                                          const uint8_t* __restrict__ pyr, uint8_t* __restrict__ blur,
                                          int img, int t, int bid) {
  constexpr int R = kBlurTileH / 4;  // output rows per thread; one wave = one R-row strip
  int l = 0;
  while (l + 1 < P->levels && t >= P->lev[l + 1].blur_tile_begin) ++l;
  const LevelGeom& g = P->lev[l];
  t -= g.blur_tile_begin;
  const int lane = threadIdx.x & 63;
  const int wave = ORB_BLUR_WAVES == 4 ? __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) : (bid & 3);
  int sp;
  const uint8_t* S = level_plane(P, src, pyr, img, l, sp);
  uint8_t* dst = blur + (size_t)img * P->blur_bytes + g.blur_off;
  const int nfull = g.tiles_x * g.tiles_y;
  if (t < nfull) {
    const int ty = t / g.tiles_x, tx = t - ty * g.tiles_x;
    const int x = tx * kBlurTileW + 4 * lane;
    // wave-uniform row origin: row addressing and row bounds stay scalar
    const int ys = ty * kBlurTileH + R * wave;
    if (x >= g.w || ys >= g.h) return;
    blur_strip<false, kWT ? kAuxSc1 : 0>(P, g, S, sp, dst, x, ys);
  } else {
    // tail wave: tail_s strips of tail_nl lanes, strip s at rows ys0 + 32 s
    const int tw = 4 * (t - nfull) + wave;
    const int s = lane / g.tail_nl, c = lane - s * g.tail_nl;
    const int x = g.tiles_x * kBlurTileW + 4 * c, ys = (tw * g.tail_s + s) * R;
    if (s >= g.tail_s || x >= g.w || ys >= g.h) return;
    blur_strip<true, kWT ? kAuxSc1 : 0>(P, g, S, sp, dst, x, ys);
  }
}

// (the same body as blur_wave, kept verbatim: as a call of blur_wave the
// register allocation of the edge path came out one v_mov per row longer)
__global__ __launch_bounds__(64 * ORB_BLUR_WAVES) ORB_WPE8 ORB_BLUR_WPE void k_blur(const PlanHeader* __restrict__ P, ImgSrc src,
                                              const uint8_t* __restrict__ pyr,
                                              uint8_t* __restrict__ blur) {
  constexpr int R = kBlurTileH / 4;  // output rows per thread; one wave = one R-row strip
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int wid = ORB_BLUR_WAVES == 4 ? bid : bid >> 2;  // the 4-wave tile
  const int img = wid / P->blur_tiles;
  int t = wid - img * P->blur_tiles;
  int l = 0;
  while (l + 1 < P->levels && t >= P->lev[l + 1].blur_tile_begin) ++l;
  const LevelGeom& g = P->lev[l];
  t -= g.blur_tile_begin;
  const int lane = threadIdx.x & 63;
  const int wave = ORB_BLUR_WAVES == 4 ? __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) : (bid & 3);
  int sp;
  const uint8_t* S = level_plane(P, src, pyr, img, l, sp);
  uint8_t* dst = blur + (size_t)img * P->blur_bytes + g.blur_off;
  const int nfull = g.tiles_x * g.tiles_y;
  if (t < nfull) {
    const int ty = t / g.tiles_x, tx = t - ty * g.tiles_x;
    const int x = tx * kBlurTileW + 4 * lane;
    // wave-uniform row origin: row addressing and row bounds stay scalar
    const int ys = ty * kBlurTileH + R * wave;
    if (x >= g.w || ys >= g.h) return;
    blur_strip<false>(P, g, S, sp, dst, x, ys);
  } else {
    // tail wave: tail_s strips of tail_nl lanes, strip s at rows ys0 + 32 s
    const int tw = 4 * (t - nfull) + wave;
    const int s = lane / g.tail_nl, c = lane - s * g.tail_nl;
    const int x = g.tiles_x * kBlurTileW + 4 * c, ys = (tw * g.tail_s + s) * R;
    if (s >= g.tail_s || x >= g.w || ys >= g.h) return;
    blur_strip<true>(P, g, S, sp, dst, x, ys);
  }
}

// --------------------------------------------------------------------------
// k_fast_cells: one 64-lane wave per FAST cell.
// The reference runs cv::FAST(cell ROI, th, nonmax=true) and, when that
// returns nothing, again with minThFAST.  Restated without the ring buffers:
//   S(p) = max over the 16 nine-pixel arcs of min(v - p_k) (dark) or
//          min(p_k - v) (bright), minus 1  (== cornerScore<16>);
//   p is a corner at th  <=>  S(p) >= th  (the score is threshold-free then);
//   NMS keeps p iff S(p) > S'(q) for its 8 neighbours, where S'(q) = S(q) if q
//   is a corner at th inside the same cell's detection area, else 0.
// Work per pass: a 5-read compass test (every 9-arc holds one pixel of each
// opposite pair {0,8}, {4,12}, so it never rejects a corner) compacts the
// survivors in raster order; only survivors get the full score and the NMS.
// Output order = raster order = the reference's per-cell keypoint order.
// --------------------------------------------------------------------------
__device__ __forceinline__ ushort2_t sub_sat2(ushort2_t a, ushort2_t b) {
  return __builtin_elementwise_sub_sat(a, b);
}
__device__ __forceinline__ ushort2_t min2(ushort2_t a, ushort2_t b) {
  return __builtin_elementwise_min(a, b);
}
__device__ __forceinline__ ushort2_t max2(ushort2_t a, ushort2_t b) {
  return __builtin_elementwise_max(a, b);
}

// The FAST score of the pixel at p (ROI bytes, row stride ls) as the larger
// of the dark / bright arc maxima m = S + 1 (cornerScore<16>'s b0 negated).
// Dark and bright arcs run together as a packed f16 pair: a byte b loaded
// zero-extended is the f16 denormal b * 2^-24, so x_k = (p_k - v, v - p_k)
// is ONE v_pk_add_f16 of the two loaded registers (op_sel picks both low
// halves for both results, neg the other source per half) and exact, and the
// 9-arc minima and their maximum are v_pk_minimum3_f16 / v_pk_maximum3_f16 on
// exact multiples of 2^-24 (the kernel keeps f16 denormals: the default
// denorm mode 16/64 = 3): m3_k = min(x_k..x_k+2), arc_k = min(m3_k, m3_k+3,
// m3_k+6), 40 packed ops.  The bit pattern of a non-negative m is m * 2^24.
typedef _Float16 half2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ half2_t hmin3(half2_t a, half2_t b, half2_t c) {
  return __builtin_elementwise_minimum(__builtin_elementwise_minimum(a, b), c);
}
__device__ __forceinline__ half2_t hmax3(half2_t a, half2_t b, half2_t c) {
  return __builtin_elementwise_maximum(__builtin_elementwise_maximum(a, b), c);
}
__device__ __forceinline__ half2_t ring_diff(uint32_t pk, uint32_t v) {
  half2_t x;
  asm("v_pk_add_f16 %0, %1, %2 op_sel_hi:[0,0] neg_lo:[0,1] neg_hi:[1,0]" : "=v"(x) : "v"(pk), "v"(v));
  return x;
}
__device__ __forceinline__ _Float16 fast_arc_max(const uint8_t* p, int ls) {
  constexpr int cx[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
  constexpr int cy[16] = {3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3};
  const uint32_t vb = (uint32_t)p[0];
  half2_t x[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) x[k] = ring_diff((uint32_t)p[cx[k] + cy[k] * ls], vb);
  // The arcs starting at 2i and 2i + 1 share the core x[2i+1 .. 2i+8]:
  // max(min(core, x[2i]), min(core, x[2i+9])) = min(core, max(x[2i], x[2i+9])),
  // and core_i = min(pm_i .. pm_i+3) over the pair minima pm_j = min(x[2j+1],
  // x[2j+2]): 8 + 8 + 8 + 8 ops for the 8 core terms (min / max select their
  // inputs, so the result is the 16-arc form's, bit for bit), then their max
  half2_t pm[8], q[8], r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j)
    pm[j] = __builtin_elementwise_minimum(x[2 * j + 1], x[(2 * j + 2) & 15]);
#pragma unroll
  for (int i = 0; i < 8; ++i) q[i] = hmin3(pm[i], pm[(i + 1) & 7], pm[(i + 2) & 7]);
#pragma unroll
  for (int i = 0; i < 8; ++i)
    r[i] = hmin3(q[i], pm[(i + 3) & 7], __builtin_elementwise_maximum(x[2 * i], x[(2 * i + 9) & 15]));
  half2_t b = hmax3(hmax3(r[0], r[1], r[2]), hmax3(r[3], r[4], r[5]), __builtin_elementwise_maximum(r[6], r[7]));
  return __builtin_fmaxf16(b.x, b.y);
}

// compass value of 4 pixels (two u16 pairs): corner at th => value > th
__device__ __forceinline__ ushort2_t compass2(ushort2_t v, ushort2_t u, ushort2_t d, ushort2_t l,
                                              ushort2_t r) {
  const ushort2_t lo = max2(min2(u, d), min2(l, r));
  const ushort2_t hi = min2(max2(u, d), max2(l, r));
  return max2(sub_sat2(v, lo), sub_sat2(hi, v));
}
// Measurement-only build switch (wrong keypoints): ORB_FAST_SKIP bit 0 skips
// the NMS, bit 1 the scores, bit 2 the survivor expansion and scores, bit 3
// the compass loop, and the
// minTh pass never runs -- the VALU of a phase is the difference
// (tools/valu_ab.sh over `make var` builds)
#ifndef ORB_FAST_SKIP
#define ORB_FAST_SKIP 0
#endif
// A/B build switch (make varB): the survivor list expanded once and held
// whole (LDS 2 bytes a detection pixel) instead of per 64 group entries
#ifndef ORB_FAST_SV_FULL
#define ORB_FAST_SV_FULL 0
#endif
__device__ __forceinline__ uint32_t mbcnt64(uint64_t m, uint32_t acc) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, acc));
}

// In-wave inclusive integer scan by DPP (row_shr 1,2,4,8 within each 16-lane
// row, then row_bcast 15/31 carry the row totals): lane 63 holds the total.
// Full-mask steps read 0 out of range (bound_ctrl), so they need no zeroed
// destination.  The whole wave must be active.
__device__ __forceinline__ int wave_iscan(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true);
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true);
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true);
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);
  return v;
}

constexpr int kFastPf = 12;  // ROI dwords in flight per lane (one round trip up to 768)
constexpr int kFastSvChunk = 512;  // survivors of 64 group entries (the list is expanded per 64 entries)
constexpr int kFastSvCarry = 64;   // + the survivors carried from the previous chunk (< 64)

// LS > 0: the plan's LDS row pitch for every cell (PlanHeader::fast_pitch:
// the smallest of 48..64 that holds each cell's ROI row and score-map row;
// 48 at 752 x 480).  The ROI and the score map then share that compile-time
// pitch and a survivor is its own pixel offset r * LS + q -- every ring / NMS
// neighbour address is base + immediate, the score-map index i + LS + 1 (no
// per-survivor row multiplies or offset adds).  LS = 0: pitches per cell,
// survivors r << 7 | q.
// One wave's LDS hand-off (its LDS operations execute in order; the fences
// keep the compiler's order and drain lgkmcnt)
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// ORB_FAST_WAVES cells (one wave each, never synchronised with each other:
// every barrier below is the wave's own) per workgroup, each its own
// max_roi_lds slice of the workgroup's LDS.  A/B build switch (DESIGN §11:
// 2 and 4 measured no better than 1 and 4 less stable; a build with W > 1
// also needs W * max_roi_lds within the LDS limit)
#ifndef ORB_FAST_WAVES
#define ORB_FAST_WAVES 1
#endif
// FAST cell ci of image img by one wave (lane 0..63) with its own LDS slice
// of PlanHeader::max_roi_lds bytes; only wave-level synchronisation.
// (pre: the cell record, loaded by the dataflow launch before its dependency wait)
template <int LS, bool kWT = false>
__device__ __forceinline__ void fast_cell(const PlanHeader* __restrict__ P, const Cell* __restrict__ cells,
                                          const ImgSrc& src, const uint8_t* __restrict__ pyr,
                                          uint32_t* __restrict__ slots, int* __restrict__ cell_count,
                                          int img, int ci, uint8_t* __restrict__ lds, int lane,
                                          const Cell* pre = nullptr) {
  STAMP_INIT;
  const Cell c = pre ? *pre : cells[ci];
  const int dw = c.cols - 6, dh = c.rows - 6;
  const int nd = (dw > 0 && dh > 0) ? dw * dh : 0;
  uint32_t* out = slots + (size_t)img * P->slots + c.slot_off;
  if (nd == 0) {
    if (lane == 0) st_pub<kWT>(cell_count + (size_t)img * P->n_cells + ci, 0);
    return;
  }
  // LDS (fast_cell_lds_bytes[_pitch]): ROI rows of ls bytes (ROI column x at
  // row byte lead + x), score map of the detection area with a zero border
  // (row pitch sp2), the u16 survivors of 64 group entries (kFastSvChunk; the
  // list is expanded per 64 entries, twice: scores, then NMS -- never held
  // whole, which keeps a cell wave's LDS and so the occupancy down), u32 list
  // of the 8-pixel groups holding a survivor.  A survivor is r * LS + q (LS >
  // 0) or r << 7 | q (detection row, column; dw < 128, dh < 256 by the
  // planner).
  constexpr int QB = 7, QM = (1 << QB) - 1;  // (LS == 0) survivor index r << QB | q
  const int ls = LS ? LS : (c.cols + 6) & ~3;
  const int sp2 = LS ? LS : dw + 2, nsc = sp2 * (dh + 2);
  uint8_t* roi = lds;
  uint8_t* sc = lds + ((ls * c.rows + 15) & ~15);
  uint16_t* sv = reinterpret_cast<uint16_t*>(sc + ((nsc + 15) & ~15));
  uint32_t* ge = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(sv) +
                                             (ORB_FAST_SV_FULL ? ((2 * nd + 15) & ~15) : 2 * (kFastSvChunk + kFastSvCarry)));
  auto sci = [&](int i) {
    if constexpr (LS != 0) return i + LS + 1;
    return ((i >> QB) + 1) * sp2 + (i & QM) + 1;
  };
  // a survivor's pixel in the ROI, relative to detection pixel (0, 0)
  auto px = [&](int i) -> int {
    if constexpr (LS != 0) return i;
    return (int)__umul24((uint32_t)i >> QB, (uint32_t)ls) + (i & QM);
  };

  // ---- ROI -> LDS: raw dwords, all loads in flight before the first store
  int sp;
  const uint8_t* S = level_plane(P, src, pyr, img, c.level, sp) + (size_t)c.y0 * sp + c.x0;
  const int lead = (int)((uintptr_t)S & 3);
  {
    const uint8_t* Sa = S - lead;  // rows stay dword-aligned iff sp is; else unaligned loads
    const int ndw = (lead + c.cols + 3) >> 2;
    const uint32_t q4 = 4u * (uint32_t)min(lane & 15, ndw - 1), r0 = (uint32_t)lane >> 4;
    if (LS != 0 && ndw <= 16 && c.rows <= 4 * kFastPf && c.y0 + 4 * kFastPf <= P->lev[c.level].h) {
      // The whole ROI in one step of 4 * kFastPf rows from its top row, none
      // clamped: rows past the ROI (at most 4 kFastPf - rows) are still inside
      // the level plane (the condition) and land in this wave's LDS past the
      // ROI -- the score map, cleared below, and the survivor lists, written
      // later; 4 kFastPf * LS bytes is well inside fast_cell_lds_bytes.  The
      // row steps are scalar buffer offsets and LDS immediates: two VALU for
      // the 12 loads and stores instead of four each.
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(Sa), (short)0,
                                                                          (int)0xffffffff, kBufRsrcWord3);
      const int voff = (int)(__umul24(r0, (uint32_t)sp) + q4);
      uint32_t v[kFastPf];
#pragma unroll
      for (int u = 0; u < kFastPf; ++u) v[u] = __builtin_amdgcn_raw_buffer_load_b32(rs, voff, 4 * u * sp, 0);
      uint8_t* d = roi + (__umul24(r0, (uint32_t)(LS ? LS : 1)) + q4);
#pragma unroll
      for (int u = 0; u < kFastPf; ++u) *reinterpret_cast<uint32_t*>(d + 4 * u * LS) = v[u];
    } else if (ndw <= 16) {
      // 16 lanes per ROI row, 4 rows per step: lane (q, r0) copies dword q of
      // rows r0, r0 + 4, ... -- a uniform stride, kFastPf loads in flight.
      // Lanes past the ROI width or height are clamped onto its last dword /
      // row: they copy the same dword to the same LDS address as the lane
      // that owns it, so the stores need no predicate; 32-bit offsets from
      // the wave-uniform row base keep the loads on the scalar base.
      const uint32_t rlast = (uint32_t)c.rows - 1u;
      for (int k0 = 0; 4 * k0 < c.rows; k0 += kFastPf) {
        uint32_t v[kFastPf], rr[kFastPf];
#pragma unroll
        for (int u = 0; u < kFastPf; ++u) rr[u] = min(r0 + 4u * (uint32_t)(k0 + u), rlast);
#pragma unroll
        for (int u = 0; u < kFastPf; ++u)
          v[u] = *reinterpret_cast<const uint32_t*>(Sa + (__umul24(rr[u], (uint32_t)sp) + q4));
#pragma unroll
        for (int u = 0; u < kFastPf; ++u)
          *reinterpret_cast<uint32_t*>(roi + (__umul24(rr[u], (uint32_t)(LS ? LS : ls)) + q4)) = v[u];
      }
    } else {
      for (int i = lane; i < c.rows * ndw; i += 64) {
        const int r = i / ndw, q = i - r * ndw;
        *reinterpret_cast<uint32_t*>(roi + r * ls + 4 * q) =
            *reinterpret_cast<const uint32_t*>(Sa + (size_t)r * sp + 4 * q);
      }
    }
  }
  // (16-byte stores: the score map's region is rounded up to 16 bytes)
  for (int i = lane; i < ((nsc + 15) >> 4); i += 64) reinterpret_cast<uint4*>(sc)[i] = make_uint4(0u, 0u, 0u, 0u);
  wave_lds_sync();
  STAMP(6);
  STAMP_ADD(13, 1);

  const uint8_t* base = roi + 3 * ls + lead + 3;  // detection pixel (0, 0)
  const uint64_t lt = (1ull << lane) - 1ull;
  const int gpr = (dw + 7) >> 3;  // 8-pixel groups per detection row
  // lane / gpr as a 24-bit multiply by the scalar ceil(2^16 / gpr): exact for
  // lane < 64, gpr <= 16 (dw < 128), no VALU division sequence
  const uint32_t g_m = (65535u + (uint32_t)gpr) / (uint32_t)gpr;
  const int g_r0 = (int)(__umul24((uint32_t)lane, g_m) >> 16), g_q0 = lane - __mul24(g_r0, gpr);
  const int g_dr = 64 / gpr, g_dq = 64 - g_dr * gpr;
  const int tail = dw - 8 * (gpr - 1);  // valid pixels of a row's last group (1..8)

  // One threshold pass; returns the number of keypoints, leaves the survivor
  // list (raster order, kp flag in bit 15) in sv[0..*n_sv).
  // v_perm selectors of the compass windows (row bytes lead + 3: centre, up,
  // down; lead: left; lead + 6: right): pair (2j, 2j + 1) of a window at byte
  // offset s within its first dword is bytes s + 2j, s + 2j + 1 zero-extended
  auto psel = [](int b) {
    return (uint32_t)b | 0x0c00u | ((uint32_t)(b + 1) << 16) | 0x0c000000u;
  };
  const int s_v = (lead + 3) & 3, s_l = lead & 3, s_r = (lead + 6) & 3;
  const uint2 sel_v = make_uint2(psel(s_v), psel(s_v + 2));
  const uint2 sel_l = make_uint2(psel(s_l), psel(s_l + 2));
  const uint2 sel_r = make_uint2(psel(s_r), psel(s_r + 2));

  const uint32_t tail_mask = (1u << tail) - 1u;  // valid pixels of a row's tail group

  const int xrel0 = c.x0 + 3 - kFastBorder, yrel0 = c.y0 + 3 - kFastBorder;
  // One threshold pass: the compass, the scores, NMS; the keypoints go to the
  // cell's slots (raster order); returns how many were found (*n_sv: survivors).
  auto pass = [&](int th, int* n_sv) -> int {
    // compass pre-test on 8 pixels per lane in packed u16 pairs; the window
    // of centres q..q+7 starts at row byte lead + q + 3 (wave-uniform shifts)
    int ng = 0;
    const ushort2_t thv = {(unsigned short)(0x7fff - th), (unsigned short)(0x7fff - th)};
    const _Float16 thp1 = __builtin_bit_cast(_Float16, (uint16_t)(th + 1));  // (th + 1) * 2^-24, exact
    auto bal = [](bool b) { return __builtin_amdgcn_ballot_w64(b); };
    for (int r = g_r0, g = g_q0; !(ORB_FAST_SKIP & 8);) {
      const uint64_t mrv = bal(r < dh);  // lanes whose group row is valid
      if (mrv == 0) break;
      const uint32_t cr = (uint32_t)(min(r, dh - 1) + 3);
      const uint8_t* C = roi + __umul24(cr, (uint32_t)(LS ? LS : ls)) + 8 * g;  // (24-bit: full-rate)
      // window of 8 centre-relative pixels at row byte o as four u16 pairs
      // (pixels 2j, 2j + 1): one two-source v_perm each straight from the
      // three dwords covering the window (wave-uniform selectors, no align)
      auto win = [&](const uint8_t* row, int o, uint32_t sa, uint32_t sb, uint32_t (&q)[4]) {
        const uint32_t* w = reinterpret_cast<const uint32_t*>(row + (o & ~3));
        const uint32_t a = w[0], b = w[1], c = w[2];
        q[0] = __builtin_amdgcn_perm(b, a, sa);
        q[1] = __builtin_amdgcn_perm(b, a, sb);
        q[2] = __builtin_amdgcn_perm(c, b, sa);
        q[3] = __builtin_amdgcn_perm(c, b, sb);
      };
      uint32_t qv[4], ql[4], qr[4], qu[4], qd[4];
      win(C, lead + 3, sel_v.x, sel_v.y, qv);
      win(C, lead, sel_l.x, sel_l.y, ql);
      win(C, lead + 6, sel_r.x, sel_r.y, qr);
      win(C - 3 * ls, lead + 3, sel_v.x, sel_v.y, qu);
      win(C + 3 * ls, lead + 3, sel_v.x, sel_v.y, qd);
      // compass value per pixel pair; corner at th => value > th
      uint32_t tv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        tv[j] = __builtin_bit_cast(uint32_t, compass2(as_us2(qv[j]), as_us2(qu[j]), as_us2(qd[j]),
                                                      as_us2(ql[j]), as_us2(qr[j])));
      // value > th  <=>  bit 15 of the u16 value + (0x7fff - th) (value, th
      // <= 255: no carry out); one packed add per pixel pair, then the flag
      // bits 15 / 31 of the four pairs gathered by two v_perm into bits
      // 7, 15, 23, 31 of A (pixels 0-3) and B (pixels 4-7)
      uint32_t fb[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = __builtin_bit_cast(uint32_t, as_us2(tv[j]) + thv);
      const uint32_t A = __builtin_amdgcn_perm(fb[1], fb[0], 0x07050301u) & 0x80808080u;
      const uint32_t B = __builtin_amdgcn_perm(fb[3], fb[2], 0x07050301u) & 0x80808080u;
      // group mask (pixel k at bit 7 + k) by two v_dot4 with per-pixel weights
      // 2^k.  Pixels past the detection width in a row's tail group are
      // dropped at the expansion (once per entry, not once per group here).
      const uint32_t m7 = __builtin_amdgcn_udot4(A, 0x08040201u, __builtin_amdgcn_udot4(B, 0x80402010u, 0u, false),
                                                 false);
      // groups with a survivor append (r << 7 | 8 g) | mask << 16 in raster
      // order; the per-pixel list is expanded below, once per 64 entries
      const bool has = r < dh && m7 != 0;
      const uint64_t mg = bal(has);
      if (has) {
        // LS > 0: the row's tail group keeps its first `tail` pixels here (the
        // entry then holds only valid pixels); LS == 0 drops them at the expansion
        const uint32_t mv = LS ? (g == gpr - 1 ? m7 & (tail_mask << 7) : m7) : m7;
        const uint32_t i0 = LS ? __umul24((uint32_t)r, (uint32_t)LS) + 8 * g : (uint32_t)((r << QB) | (8 * g));
        ge[mbcnt64(mg, (uint32_t)ng)] = i0 | (mv << 9);
      }
      ng += __popcll(mg);
      g += g_dq;
      r += g_dr;
      if (g >= gpr) g -= gpr, ++r;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    STAMP(0);
    // NMS by group entries (LS > 0), the per-pixel list not needed: lane j
    // takes entry b0 + j (8 pixels, r * LS + 8 g) and its score-map window --
    // rows above / at / below, bytes q-1 .. q+8, 3 dwords each (entries are
    // dword-aligned: LS and 8 g are multiples of 4) -- as u16 pixel pairs
    // (one v_perm each, as the compass), the 8-neighbour maxima by packed
    // max, the test s > n by a saturating packed subtract whose bit 15 / 31
    // (after + 0x7fff) is the flag; keypoints go to the slots in raster order
    // (entries in order, pixels LSB-first) from a wave scan of the counts.
    auto nms_entries = [&](int& written) {
      // only entries holding a corner (a non-zero score among their 8 centre
      // bytes) can keep a keypoint: compact them first, in place (a write
      // index never passes its read index), so the NMS runs on about half
      // the waves (≈ 0.36 corners a survivor, profiles/r05/fast_survivors.json)
      int nce = 0;
      for (int b0 = 0; b0 < ng; b0 += 64) {
        const int j = b0 + lane;
        const uint32_t e = j < ng ? ge[j] : 0u;
        const uint32_t* B = reinterpret_cast<const uint32_t*>(sc + (e & 0xffffu) + sp2);
        const bool has = j < ng && ((B[0] >> 8) | B[1] | (B[2] & 0xffu)) != 0u;
        const uint64_t mg = __builtin_amdgcn_ballot_w64(has);
        if (has) ge[mbcnt64(mg, (uint32_t)nce)] = e;
        nce += __popcll(mg);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      for (int b0 = 0; b0 < nce; b0 += 64) {
        const int j = b0 + lane;
        const uint32_t e = j < nce ? ge[j] : 0u;
        const int i0 = (int)(e & 0xffffu);
        const uint32_t m = (e >> 16) & 0xffu;
        const uint32_t* A = reinterpret_cast<const uint32_t*>(sc + i0);
        const uint32_t* B = reinterpret_cast<const uint32_t*>(sc + i0 + sp2);
        const uint32_t* Cr = reinterpret_cast<const uint32_t*>(sc + i0 + 2 * sp2);
        const uint32_t a0 = A[0], a1 = A[1], a2 = A[2], c0 = Cr[0], c1 = Cr[1], c2 = Cr[2];
        const uint32_t m0 = B[0], m1 = B[1], m2 = B[2];
        // pair j (pixels 2j, 2j + 1) at window offset d: row bytes b = 2j + d,
        // b + 1, from (w1:w0) for b < 4, else (w2:w1) at b - 4 -- one form per
        // byte offset, so the 12 uses of a row are 9 distinct perms (CSE)
        auto pr = [&](uint32_t w0, uint32_t w1, uint32_t w2, int jj, int d) {
          const int b = 2 * jj + d;
          return b < 4 ? __builtin_amdgcn_perm(w1, w0, psel(b)) : __builtin_amdgcn_perm(w2, w1, psel(b - 4));
        };
        // the u16 scores (0..255) read as f16 are the denormals s * 2^-24, so
        // packed f16 maximum3 and subtract are exact on them: the 8-neighbour
        // maximum n is three v_pk_maximum3_f16 and a maximum, and n - s has
        // its sign bit (15 / 31) set iff s > n (s == n gives +0)
        auto h2 = [](uint32_t v) { return __builtin_bit_cast(half2_t, v); };
        uint32_t fb[4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const half2_t na = hmax3(h2(pr(a0, a1, a2, jj, 0)), h2(pr(a0, a1, a2, jj, 1)), h2(pr(a0, a1, a2, jj, 2)));
          const half2_t nc = hmax3(h2(pr(c0, c1, c2, jj, 0)), h2(pr(c0, c1, c2, jj, 1)), h2(pr(c0, c1, c2, jj, 2)));
          const half2_t n = hmax3(na, nc, __builtin_elementwise_maximum(h2(pr(m0, m1, m2, jj, 0)),
                                                                          h2(pr(m0, m1, m2, jj, 2))));
          fb[jj] = __builtin_bit_cast(uint32_t, n - h2(pr(m0, m1, m2, jj, 1)));
        }
        const uint32_t FA = __builtin_amdgcn_perm(fb[1], fb[0], 0x07050301u) & 0x80808080u;
        const uint32_t FB = __builtin_amdgcn_perm(fb[3], fb[2], 0x07050301u) & 0x80808080u;
        uint32_t km = (__builtin_amdgcn_udot4(FA, 0x08040201u, __builtin_amdgcn_udot4(FB, 0x80402010u, 0u, false),
                                              false) >> 7) & m;
        const int cnt = __popc(km);
        const int incl = wave_iscan(cnt);
        int pos = written + incl - cnt;
        if (km) {
          constexpr int LSD = LS ? LS : 1;
          const int r = i0 / LSD, q0 = i0 - r * LSD;
          const uint64_t mid = ((uint64_t)m1 << 32) | m0;  // centre bytes 1..8 (byte 8: m2)
          do {
            const int k = __builtin_ctz(km);
            const uint32_t sk = k < 7 ? (uint32_t)(mid >> (8 * (k + 1))) & 0xffu : m2 & 0xffu;
            if (pos < c.slot_cap)
              st_pub<kWT>(out + pos, (uint32_t)(xrel0 + q0 + k) | ((uint32_t)(yrel0 + r) << 12) | (sk << 24));
            ++pos;
            km &= km - 1;
          } while (km);
        }
        written += __builtin_amdgcn_readlane(incl, 63);
      }
    };
#if ORB_FAST_SV_FULL
    // the whole survivor list, expanded once (raster order: entries in order,
    // pixels LSB-first), then scores and NMS over it
    int ns = 0;
    for (int b0 = 0; b0 < ng; b0 += 64) {
      const int j = b0 + lane;
      const uint32_t e = j < ng ? ge[j] : 0u;
      const int i0 = (int)(e & 0xffffu);
      uint32_t m = LS ? (e >> 16) & 0xffu : (e >> 16) & (((i0 >> 3) & ((1 << (QB - 3)) - 1)) == gpr - 1 ? tail_mask : 0xffu);
      const int cnt = __popc(m);
      const int incl = wave_iscan(cnt);
      int pos = ns + incl - cnt;
      while (m) {
        sv[pos++] = (uint16_t)(i0 + __builtin_ctz(m));
        m &= m - 1;
      }
      ns += __builtin_amdgcn_readlane(incl, 63);
    }
    wave_lds_sync();
    *n_sv += ns;
    for (int j = lane; j < ns; j += 64) {
      const int i = sv[j];
      const _Float16 m = fast_arc_max(base + px(i), ls);
      const uint16_t bits = __builtin_bit_cast(uint16_t, m);
      sc[sci(i)] = m >= thp1 ? (uint8_t)(bits - 1) : (uint8_t)0;
    }
    wave_lds_sync();
    STAMP(1);
    int written = 0;
    if constexpr (LS != 0) {
      nms_entries(written);
    } else {
    for (int jb = 0; jb < ns; jb += 64) {
      const int j = jb + lane;
      bool kp = false;
      int i = 0, s = 0;
      if (j < ns) {
        i = sv[j];
        const uint8_t* mp = sc + sci(i);
        s = mp[0];
        const int n = max(max(max(mp[-sp2 - 1], mp[-sp2]), max(mp[-sp2 + 1], mp[-1])),
                          max(max(mp[1], mp[sp2 - 1]), max(mp[sp2], mp[sp2 + 1])));
        kp = s > n;
      }
      const uint64_t km = __ballot(kp);
      if (kp) {
        constexpr int LSD = LS ? LS : 1;
        const int r = LS ? i / LSD : i >> QB, q = LS ? i - r * LS : i & QM;
        const int pos = written + __popcll(km & lt);
        if (pos < c.slot_cap)
          st_pub<kWT>(out + pos, (uint32_t)(xrel0 + q) | ((uint32_t)(yrel0 + r) << 12) | ((uint32_t)s << 24));
      }
      written += __popcll(km);
    }
    }
    wave_lds_sync();
#else
    // survivors, 64 group entries at a time: lane j expands entry b0 + j into
    // sv[] from the wave's inclusive scan of the entries' popcounts (raster
    // order: entries in order, pixels LSB-first), at most kFastSvChunk
    auto expand = [&](int b0, int at) -> int {  // appends at sv[at]
      const int j = b0 + lane;
      const uint32_t e = j < ng ? ge[j] : 0u;
      const int i0 = (int)(e & 0xffffu);
      // (LS == 0) the row's tail group keeps its first `tail` pixels
      uint32_t m = LS ? (e >> 16) & 0xffu : (e >> 16) & (((i0 >> 3) & ((1 << (QB - 3)) - 1)) == gpr - 1 ? tail_mask : 0xffu);
      const int cnt = __popc(m);
      const int incl = wave_iscan(cnt);
      int pos = at + incl - cnt;
      while (m) {
        sv[pos++] = (uint16_t)(i0 + __builtin_ctz(m));
        m &= m - 1;
      }
      wave_lds_sync();
      return __builtin_amdgcn_readlane(incl, 63);
    };
    // scores of every survivor into the map: a chunk's survivors are scored
    // 64 at a time and the last partial wave's (< 64) carried to the front
    // of sv for the next chunk -- full waves except once per cell, not once
    // per chunk (the scores are independent of their order)
    auto score = [&](int i) {
      // S = max(m - 1, 0) is a corner's score iff m >= th + 1 (then m > 0
      // and its bit pattern is the integer m)
      const _Float16 m = fast_arc_max(base + px(i), ls);
      const uint16_t bits = __builtin_bit_cast(uint16_t, m);
      sc[sci(i)] = m >= thp1 ? (uint8_t)(bits - 1) : (uint8_t)0;
    };
    int pend = 0;  // survivors carried at sv[0, pend)
    for (int b0 = 0; b0 < ng && !(ORB_FAST_SKIP & 4); b0 += 64) {
      const int ns = expand(b0, pend);
      *n_sv += ns;
      const int tot = pend + ns, full = tot & ~63;
      for (int j = lane; j < full && !(ORB_FAST_SKIP & 2); j += 64) score(sv[j]);
      pend = tot - full;
      if (full > 0 && lane < pend) sv[lane] = sv[full + lane];  // (disjoint: full >= 64 > pend)
      wave_lds_sync();  // sv is rewritten by the next chunk
    }
    if (lane < pend && !(ORB_FAST_SKIP & 2)) score(sv[lane]);
    wave_lds_sync();
    STAMP(1);
    // NMS over the survivors again (re-expanded: the list is never held
    // whole), keypoints straight to the cell's slots in raster order: a corner
    // is kept iff its score beats all 8 neighbours' (0 for non-corners and
    // for the zero border outside the detection area)
    int written = 0;
    if constexpr (LS != 0) {
      if (!(ORB_FAST_SKIP & 1)) nms_entries(written);
    } else for (int b0 = 0; b0 < ng; b0 += 64) {
      const int ns = expand(b0, 0);
      for (int jb = 0; jb < ns; jb += 64) {
        const int j = jb + lane;
        bool kp = false;
        int i = 0, s = 0;
        if (j < ns) {
          i = sv[j];
          const uint8_t* mp = sc + sci(i);
          s = mp[0];
          const int n = max(max(max(mp[-sp2 - 1], mp[-sp2]), max(mp[-sp2 + 1], mp[-1])),
                            max(max(mp[1], mp[sp2 - 1]), max(mp[sp2], mp[sp2 + 1])));
          kp = s > n;
        }
        const uint64_t km = __ballot(kp);
        if (kp) {
          constexpr int LSD = LS ? LS : 1;  // (no division by zero in the LS == 0 instance)
          const int r = LS ? i / LSD : i >> QB, q = LS ? i - r * LS : i & QM;
          const int pos = written + __popcll(km & lt);
          if (pos < c.slot_cap)
            st_pub<kWT>(out + pos, (uint32_t)(xrel0 + q) | ((uint32_t)(yrel0 + r) << 12) | ((uint32_t)s << 24));
        }
        written += __popcll(km);
      }
      wave_lds_sync();
    }
#endif
    STAMP(2);
    return written;
  };

  int ns = 0;
  int written = pass(P->ini_th, &ns);
  STAMP_ADD(12, ns);
  if (written == 0 && !ORB_FAST_SKIP) {
    STAMP_ADD(10, 1);
    for (int i = lane; i < ((nsc + 3) >> 2); i += 64) reinterpret_cast<uint32_t*>(sc)[i] = 0u;
    wave_lds_sync();
    STAMP(3);
    ns = 0;
    written = pass(P->min_th, &ns);
    STAMP(4);
    STAMP_ADD(11, ns);
  }
  if (lane == 0) st_pub<kWT>(cell_count + (size_t)img * P->n_cells + ci, min(written, c.slot_cap));
  STAMP(5);
  STAMP_END;
}

template <int LS>
__global__ __launch_bounds__(64 * ORB_FAST_WAVES) void k_fast_cells(const PlanHeader* __restrict__ P,
                                                   const Cell* __restrict__ cells, ImgSrc src,
                                                   const uint8_t* __restrict__ pyr,
                                                   uint32_t* __restrict__ slots,
                                                   int* __restrict__ cell_count, int n_img) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds_all[];
  const int lane = threadIdx.x & 63;
  const int fw = ORB_FAST_WAVES > 1 ? __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) : 0;
  uint8_t* lds = lds_all + (ORB_FAST_WAVES > 1 ? fw * P->max_roi_lds : 0);
  const int wid = xcd_remap(blockIdx.x, gridDim.x) * ORB_FAST_WAVES + fw;
  const int img = wid / P->n_cells;
  if (img >= n_img) return;  // (wave-uniform: the last workgroup's spare waves)
  fast_cell<LS>(P, cells, src, pyr, slots, cell_count, img, wid - img * P->n_cells, lds, lane);
}

// --------------------------------------------------------------------------
// Block-wide helpers for the octree (256 threads).
// --------------------------------------------------------------------------
constexpr int kOctThreads = 256;

// In-place exclusive scan of a[0..n) in LDS; returns the total.  `tmp` holds
// kOctThreads + 1 ints of LDS.  Must be called by the whole block.
// kSmall: n <= 256 as one element a thread in two barriers -- the
// single-image dataflow launch's octree (its latency chain); the batch
// kernels keep the three-barrier form (the small path's registers cost the
// batch octree its co-residency in the bench mix: 146.7k vs 149.7k frames/s
// over three interleaved rounds, though 12 % faster alone)
template <bool kSmall = false>
__device__ int block_scan(int* a, int n, int* tmp) {
  const int t = threadIdx.x;
  if (kSmall && n <= kOctThreads) {
    // one element a thread: DPP scans within the waves, the four wave totals
    // through LDS -- two barriers instead of three (the octree's node-list
    // scans, most of them at a few hundred nodes or fewer)
    const int v = t < n ? a[t] : 0;
    const int incl = wave_iscan(v);
    const int w = t >> 6;
    if ((t & 63) == 63) tmp[w] = incl;
    __syncthreads();
    const int t0 = tmp[0], t1 = tmp[1], t2 = tmp[2], t3 = tmp[3];
    const int off = (w > 0 ? t0 : 0) + (w > 1 ? t1 : 0) + (w > 2 ? t2 : 0);
    if (t < n) a[t] = off + incl - v;
    __syncthreads();
    return t0 + t1 + t2 + t3;
  }
  const int per = (n + kOctThreads - 1) / kOctThreads;
  const int b = min(t * per, n), e = min(b + per, n);
  int s = 0;
  for (int i = b; i < e; ++i) s += a[i];
  tmp[t] = s;
  __syncthreads();
  if (t < 64) {
    int v0 = tmp[4 * t], v1 = tmp[4 * t + 1], v2 = tmp[4 * t + 2], v3 = tmp[4 * t + 3];
    int own = v0 + v1 + v2 + v3;
    int inc = own;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(inc, o, 64);
      if (t >= o) inc += y;
    }
    int ex = inc - own;
    tmp[4 * t] = ex;
    tmp[4 * t + 1] = ex + v0;
    tmp[4 * t + 2] = ex + v0 + v1;
    tmp[4 * t + 3] = ex + v0 + v1 + v2;
    if (t == 63) tmp[kOctThreads] = inc;
  }
  __syncthreads();
  int run = tmp[t];
  for (int i = b; i < e; ++i) {
    const int v = a[i];
    a[i] = run;
    run += v;
  }
  const int total = tmp[kOctThreads];
  __syncthreads();
  return total;
}

__device__ __forceinline__ int block_sum(int v, int* tmp) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((threadIdx.x & 63) == 0) tmp[threadIdx.x >> 6] = v;
  __syncthreads();
  const int r = tmp[0] + tmp[1] + tmp[2] + tmp[3];
  __syncthreads();
  return r;
}

// --------------------------------------------------------------------------
// k_octree: DistributeOctTree for one (image, level) per 256-thread block.
// The reference walks a std::list; here the list is an LDS array rebuilt per
// division round.  A round divides a set D of nodes in a processing order
// (phase 1: every node with > 1 point, list order; phase 2: the expandable
// nodes of the previous round, stable-sorted by (count, UL.x) and taken from
// the largest, stopping once the node count reaches the budget).  std::list
// push_front makes the new list
//     reverse(children of D in processing order, n1..n4 each) ++ (list \ D)
// which is computed with two block scans.  The node kept per leaf is the
// highest response, first in to_dist order on ties (64-bit LDS atomic max).
// --------------------------------------------------------------------------
// cnt[key] += 1 for every lane with key >= 0, one LDS atomic per run of equal
// keys over consecutive lanes: the candidates of a wave are consecutive in
// to_dist order (cell-major raster), so most of them fall into the same node
// and quadrant, and per-candidate atomics on a few counters serialise.  The
// whole wave must be active.
__device__ __forceinline__ void run_add(int* cnt, int key) {
  const int lane = threadIdx.x & 63;
  const int prev = __shfl_up(key, 1, 64);
  const bool head = lane == 0 || key != prev;
  const uint64_t heads = __ballot(head);
  if (head && key >= 0) {
    const uint64_t after = lane == 63 ? 0ull : (heads >> (lane + 1));
    const int len = after ? __builtin_ctzll(after) + 1 : 64 - lane;
    __hip_atomic_fetch_add(&cnt[key], len, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
}

struct OctLds {
  int *x0, *y0, *x1, *y1, *cnt;      // current list, position-indexed
  int *nx0, *ny0, *nx1, *ny1, *ncnt; // next list
  int *mx, *my;                      // division midlines
  int *ccnt;                         // 4 per node: child point counts
  int *cpos;                         // 4 per node: child position in the next list
  int *rank;                         // processing rank, -1 = not divided
  int *stay;                         // scan of "not divided" -> position offset
  int *pc;                           // per processing rank: children pushed
  int *exp_list;                     // expandable nodes (positions), push order
  int *tmp2;                         // scratch per node
  unsigned long long* best;
  int* scan_tmp;                     // kOctThreads + 1
  int* scal;                         // block scalars
  uint32_t* kdl;                     // candidates [0, kcap): packed keypoint
  int* knl;                          //                        node position
};

// kHbm: the node arrays (oct_node_bytes(NC) per block) live in a per-block
// HBM range instead of LDS -- plans whose node capacity does not fit the
// 160 KB (num_features of several thousand: the reference's
// OrbExtractor(5 * nFeatures, ...), tracking.cc:202-204).  Same code, same
// order; the counters' atomics are workgroup-scoped (the block's waves share
// one CU and its L1, so the barriers order them like LDS).  Only the scan
// scratch, the block scalars and the first kcap candidates stay in LDS.
// DistributeOctTree of level l of image img by the whole 256-thread workgroup
// (lds_raw: octree_lds_bytes of the plan; node_ws: this (image, level)'s HBM
// node range when kHbm).  Every exit is workgroup-uniform.
template <bool kHbm, bool kWT = false>
__device__ __forceinline__ void octree_level(
    const PlanHeader* __restrict__ P, const Cell* __restrict__ cells,
    const uint32_t* __restrict__ slots, const int* __restrict__ cell_count,
    uint32_t* __restrict__ dense, int* __restrict__ knode, uint32_t* __restrict__ oct_out,
    int* __restrict__ oct_count, int* __restrict__ err, int img, int l, int kcap,
    uint8_t* __restrict__ node_ws, uint8_t* __restrict__ lds_raw) {
  const int L = P->levels;
  const LevelGeom& g = P->lev[l];
  const int NC = P->node_cap;
  const int t = threadIdx.x;
  OSTAMP_INIT;

  OctLds s;
  {
    uint8_t* nodes = kHbm ? node_ws : lds_raw;
    unsigned long long* p64 = reinterpret_cast<unsigned long long*>(nodes);
    s.best = p64;
    int* p = reinterpret_cast<int*>(p64 + NC);
    int** fields[] = {&s.x0, &s.y0, &s.x1, &s.y1, &s.cnt, &s.nx0, &s.ny0, &s.nx1, &s.ny1,
                      &s.ncnt, &s.mx, &s.my, &s.rank, &s.stay, &s.pc, &s.exp_list, &s.tmp2};
    for (int** f : fields) {
      *f = p;
      p += NC;
    }
    s.ccnt = p;
    p += 4 * NC;
    s.cpos = p;
    p += 4 * NC;
    if (kHbm) p = reinterpret_cast<int*>(lds_raw);
    s.scan_tmp = p;
    p += kOctThreads + 1;
    s.scal = p;
    p += 16;
    s.kdl = reinterpret_cast<uint32_t*>(p);  // candidates [0, kcap) live in LDS
    s.knl = p + kcap;
  }

  // ---- gather this level's candidates in to_dist order (cell-major, raster):
  // counts and slot offsets of all cells in one round of loads, a scan, then
  // every candidate load in flight at once (its cell found by binary search).
  const int nc = g.cell_end - g.cell_begin;
  int* cell_off = s.tmp2;  // nc <= NC guaranteed by the planner
  int* cell_src = s.stay;
  for (int i = t; i < nc; i += kOctThreads) {
    cell_off[i] = cell_count[(size_t)img * P->n_cells + g.cell_begin + i];
    cell_src[i] = cells[g.cell_begin + i].slot_off;
  }
  __syncthreads();
  const int K = block_scan<kWT>(cell_off, nc, s.scan_tmp);
  uint32_t* kd = dense + (size_t)img * P->slots + g.slot_begin;  // overflow beyond kcap
  int* kn = knode + (size_t)img * P->slots + g.slot_begin;
  // candidate k: packed x|y<<12|score<<24 and its node; LDS below kcap, HBM above
  auto KD = [&](int k) -> uint32_t { return k < kcap ? s.kdl[k] : kd[k]; };
  auto KN = [&](int k) -> int { return k < kcap ? s.knl[k] : kn[k]; };
  auto set_kd = [&](int k, uint32_t v) {
    if (k < kcap)
      s.kdl[k] = v;
    else
      kd[k] = v;
  };
  auto set_kn = [&](int k, int v) {
    if (k < kcap)
      s.knl[k] = v;
    else
      kn[k] = v;
  };
  {
    const uint32_t* sl = slots + (size_t)img * P->slots;
    for (int k0 = 0; k0 < K; k0 += 4 * kOctThreads) {
      uint32_t v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int k = min(k0 + u * kOctThreads + t, K - 1);
        int lo = 0, hi = nc - 1;  // last cell with cell_off <= k
        while (lo < hi) {
          const int mid = (lo + hi + 1) >> 1;
          if (cell_off[mid] <= k)
            lo = mid;
          else
            hi = mid - 1;
        }
        v[u] = sl[cell_src[lo] + (k - cell_off[lo])];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (k0 + u * kOctThreads + t < K) set_kd(k0 + u * kOctThreads + t, v[u]);
    }
  }
  uint32_t* out = oct_out + (size_t)img * P->kp_slots + g.out_off;
  if (K == 0) {
    if (t == 0) st_pub<kWT>(oct_count + img * L + l, 0);
    return;
  }
  __syncthreads();

  OSTAMP(0);
  OSTAMP_ADD(10 + (l == 0), 1);
  // ---- roots: round(W/H) equal-width columns; empty roots are erased.
  const int R = g.n_roots;
  const float hx = g.root_w;
  for (int i = t; i < R; i += kOctThreads) s.ccnt[i] = 0;
  __syncthreads();
  for (int k0 = 0; k0 < K; k0 += kOctThreads) {  // whole waves active (run_add)
    const int k = k0 + t;
    int r = -1;
    if (k < K) {
      const float x = (float)(KD(k) & 0xfff);
      r = (int)(x / hx);
      set_kn(k, r);
    }
    run_add(s.ccnt, r);
  }
  __syncthreads();
  for (int i = t; i < R; i += kOctThreads) s.tmp2[i] = s.ccnt[i] > 0 ? 1 : 0;
  __syncthreads();
  int S = block_scan<kWT>(s.tmp2, R, s.scan_tmp);
  for (int i = t; i < R; i += kOctThreads) {
    if (s.ccnt[i] > 0) {
      const int p = s.tmp2[i];
      s.x0[p] = (int)(hx * (float)i);
      s.x1[p] = (int)(hx * (float)(i + 1));
      s.y0[p] = 0;
      s.y1[p] = g.rel_h;
      s.cnt[p] = s.ccnt[i];
    }
  }
  __syncthreads();
  for (int k = t; k < K; k += kOctThreads) set_kn(k, s.tmp2[KN(k)]);
  // per-node round state, prepared where the node list is (re)written so a
  // round starts without its own barriers for it: not yet chosen (rank -1),
  // the phase-1 flag cnt >= 2 (in ncnt, the scan input), the division
  // midlines, zeroed child counts
  auto prep = [&](int i) {
    s.rank[i] = -1;
    s.ncnt[i] = s.cnt[i] >= 2 ? 1 : 0;
    s.mx[i] = s.x0[i] + (int)ceilf((float)(s.x1[i] - s.x0[i]) / 2);
    s.my[i] = s.y0[i] + (int)ceilf((float)(s.y1[i] - s.y0[i]) / 2);
    s.ccnt[4 * i] = s.ccnt[4 * i + 1] = s.ccnt[4 * i + 2] = s.ccnt[4 * i + 3] = 0;
  };
  for (int i = t; i < S; i += kOctThreads) prep(i);
  __syncthreads();

  OSTAMP(1);
  const int N = g.budget;
  int phase = 1, n_exp = 0;
  bool finished = false;
  while (!finished) {
    // ---- choose D and its processing order (rank), uniform across the block
    int m;  // |D|
    OSTAMP_ADD(12 + (phase == 2), 1);
    if (phase == 1) {
      m = block_scan<kWT>(s.ncnt, S, s.scan_tmp);  // ranks of the nodes with cnt >= 2
      for (int i = t; i < S; i += kOctThreads)
        if (s.cnt[i] >= 2) s.rank[i] = s.ncnt[i];
    } else {
      // stable sort of exp_list[0..n_exp) by (cnt, x0); processed from the back.
      // Keys (cnt, x0, list index) are unique, so a node's rank is the number
      // of smaller keys: one LDS read + compare per other node.
      unsigned long long* key = s.best;  // free until the final selection
      for (int j = t; j < n_exp; j += kOctThreads) {
        const int pj = s.exp_list[j];
        key[j] = ((unsigned long long)(uint32_t)s.cnt[pj] << 32) |
                 ((unsigned long long)(uint32_t)s.x0[pj] << 16) | (unsigned long long)j;
      }
      __syncthreads();
      for (int j = t; j < n_exp; j += kOctThreads) {
        const unsigned long long kj = key[j];
        int r = 0;
#pragma unroll 8
        for (int i = 0; i < n_exp; ++i) r += key[i] < kj;
        s.rank[s.exp_list[j]] = n_exp - 1 - r;
      }
      m = n_exp;
    }
    __syncthreads();

    OSTAMP(4);
    // ---- child point counts of D (midlines prepared with the list)
    for (int k0 = 0; k0 < K; k0 += kOctThreads) {  // whole waves active (run_add)
      const int k = k0 + t;
      int key = -1;
      if (k < K) {
        const int n = KN(k);
        if (s.rank[n] >= 0) {
          const uint32_t e = KD(k);
          const int x = e & 0xfff, y = (e >> 12) & 0xfff;
          key = 4 * n + (x < s.mx[n] ? 0 : 1) + (y < s.my[n] ? 0 : 2);
        }
      }
      run_add(s.ccnt, key);
    }
    __syncthreads();
    for (int i = t; i < S; i += kOctThreads) {
      const int r = s.rank[i];
      if (r >= 0)
        s.pc[r] = (s.ccnt[4 * i] > 0) + (s.ccnt[4 * i + 1] > 0) + (s.ccnt[4 * i + 2] > 0) +
                  (s.ccnt[4 * i + 3] > 0);
    }
    __syncthreads();

    OSTAMP(5);
    // ---- phase 2 stops once the node count reaches the budget
    if (phase == 2) {
      for (int r = t; r < m; r += kOctThreads) s.tmp2[r] = s.pc[r] - 1;
      __syncthreads();
      const int tot = block_scan<kWT>(s.tmp2, m, s.scan_tmp);
      // size after processing rank r = S + (exclusive[r] + pc[r] - 1)
      if (t == 0) s.scal[0] = m;
      __syncthreads();
      for (int r = t; r < m; r += kOctThreads)
        if (S + s.tmp2[r] + s.pc[r] - 1 >= N) atomicMin(&s.scal[0], r + 1);
      __syncthreads();
      const int mm = s.scal[0];
      (void)tot;
      __syncthreads();
      if (mm < m) {
        for (int i = t; i < S; i += kOctThreads)
          if (s.rank[i] >= mm) s.rank[i] = -1;
        m = mm;
        __syncthreads();
      }
    }

    OSTAMP(6);
    // ---- push offsets (processing order) and stay offsets (list order)
    const int T = block_scan<kWT>(s.pc, m, s.scan_tmp);  // s.pc[r] = push offset of rank r
    for (int i = t; i < S; i += kOctThreads) s.stay[i] = s.rank[i] < 0 ? 1 : 0;
    __syncthreads();
    const int n_stay = block_scan<kWT>(s.stay, S, s.scan_tmp);
    const int S_new = T + n_stay;
    if (S_new > NC) {
      if (t == 0) atomicOr(err, kErrNodeCap);
      if (t == 0) st_pub<kWT>(oct_count + img * L + l, 0);
      return;  // uniform
    }

    OSTAMP(7);
    // ---- build the next list
    for (int i = t; i < S; i += kOctThreads) {
      const int r = s.rank[i];
      if (r < 0) {
        const int p = T + s.stay[i];
        s.nx0[p] = s.x0[i];
        s.ny0[p] = s.y0[i];
        s.nx1[p] = s.x1[i];
        s.ny1[p] = s.y1[i];
        s.ncnt[p] = s.cnt[i];
        s.tmp2[p] = 0;  // not pushed this round
      } else {
        int push = s.pc[r];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int n = s.ccnt[4 * i + q];
          if (n == 0) {
            s.cpos[4 * i + q] = -1;
            continue;
          }
          const int p = T - 1 - push;
          ++push;
          const int xa = (q & 1) ? s.mx[i] : s.x0[i];
          const int xb = (q & 1) ? s.x1[i] : s.mx[i];
          const int ya = (q & 2) ? s.my[i] : s.y0[i];
          const int yb = (q & 2) ? s.y1[i] : s.my[i];
          s.nx0[p] = xa;
          s.nx1[p] = xb;
          s.ny0[p] = ya;
          s.ny1[p] = yb;
          s.ncnt[p] = n;
          s.tmp2[p] = n > 1 ? 1 : 0;  // expandable child
          s.cpos[4 * i + q] = p;
        }
      }
    }
    __syncthreads();
    for (int k = t; k < K; k += kOctThreads) {
      const int n = KN(k);
      const int r = s.rank[n];
      if (r < 0) {
        set_kn(k, T + s.stay[n]);
      } else {
        const uint32_t e = KD(k);
        const int x = e & 0xfff, y = (e >> 12) & 0xfff;
        const int q = (x < s.mx[n] ? 0 : 1) + (y < s.my[n] ? 0 : 2);
        set_kn(k, s.cpos[4 * n + q]);
      }
    }
    OSTAMP(8);
    // expandable children in push order = positions T-1, T-2, ..., 0
    for (int i = t; i < T; i += kOctThreads) s.pc[i] = s.tmp2[T - 1 - i];
    __syncthreads();
    const int e = block_scan<kWT>(s.pc, T, s.scan_tmp);
    for (int i = t; i < T; i += kOctThreads)
      if (s.tmp2[T - 1 - i]) s.exp_list[s.pc[i]] = T - 1 - i;
    for (int i = t; i < S_new; i += kOctThreads) {
      s.x0[i] = s.nx0[i];
      s.y0[i] = s.ny0[i];
      s.x1[i] = s.nx1[i];
      s.y1[i] = s.ny1[i];
      s.cnt[i] = s.ncnt[i];
      prep(i);  // reads the entries this thread just wrote
    }
    __syncthreads();

    OSTAMP(9);
    const int S_prev = S;
    S = S_new;
    n_exp = e;
    if (S >= N || S == S_prev) {
      finished = true;
    } else if (phase == 1 && S + 3 * e > N) {
      phase = 2;
    }
  }

  OSTAMP(2);
  // ---- best response per node, first in to_dist order on ties
  for (int i = t; i < S; i += kOctThreads) s.best[i] = 0ull;
  __syncthreads();
  for (int k = t; k < K; k += kOctThreads) {
    const unsigned long long v =
        ((unsigned long long)(KD(k) >> 24) << 32) | (unsigned long long)(0xffffffffu - (uint32_t)k);
    __hip_atomic_fetch_max(&s.best[KN(k)], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  __syncthreads();
  const int n_out = min(S, g.out_cap);
  for (int i = t; i < n_out; i += kOctThreads) {
    const uint32_t k = 0xffffffffu - (uint32_t)(s.best[i] & 0xffffffffull);
    st_pub<kWT>(out + i, KD((int)k));
  }
  if (t == 0) {
    st_pub<kWT>(oct_count + img * L + l, n_out);
    if (S > g.out_cap) atomicOr(err, kErrOutCap);
  }
  OSTAMP(3);
  if (l == 0) OSTAMP_ADD(14, st_acc_[0] + st_acc_[1] + st_acc_[2] + st_acc_[3] + st_acc_[4] +
                               st_acc_[5] + st_acc_[6] + st_acc_[7] + st_acc_[8] + st_acc_[9]);
  OSTAMP_END;
}

template <bool kHbm>
__global__ __launch_bounds__(kOctThreads) ORB_WPE8 void k_octree(
    const PlanHeader* __restrict__ P, const Cell* __restrict__ cells,
    const uint32_t* __restrict__ slots, const int* __restrict__ cell_count,
    uint32_t* __restrict__ dense, int* __restrict__ knode, uint32_t* __restrict__ oct_out,
    int* __restrict__ oct_count, int* __restrict__ err, int n_img, int kcap,
    uint8_t* __restrict__ node_ws) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds_raw[];
  // level-major block order: the (largest) level-0 blocks are dispatched first
  const int l = blockIdx.x / n_img, img = blockIdx.x - l * n_img;
  octree_level<kHbm>(P, cells, slots, cell_count, dense, knode, oct_out, oct_count, err, img, l, kcap,
                     kHbm ? node_ws + (size_t)blockIdx.x * oct_node_bytes(P->node_cap) : nullptr, lds_raw);
}

// --------------------------------------------------------------------------
// k_describe: one wave per octree output slot.  IC_Angle on the raw level
// (integer moments over the 31-px circular patch, fastAtan2), then 256
// steered-BRIEF tests on the blurred level; test i is lane i%64 of ballot
// i/64, so the 4 ballots are the 32 descriptor bytes, LSB-first as
// ComputeOrbDescriptor packs them.
// --------------------------------------------------------------------------
typedef float f32x2 __attribute__((ext_vector_type(2)));
constexpr int kRawW = 36, kRawH = 31;   // 31x31 patch + dword alignment slack
constexpr int kBlurW = 40, kBlurH = 37;  // 37x37 (|sample offset| <= 18) + slack
constexpr int kDescLds = kRawW * kRawH + kBlurW * kBlurH;  // per wave (the round-4 kernel)
[[maybe_unused]] constexpr int kDescLdsUsed = kDescLds;


// IC_Angle by v_dot4_u32_u8 over the staged 31-row patch: item t = (row
// t / 9, dword t % 9) of the patch rows; for the patch's alignment offset o =
// (cx - 15) & 3 the table gives, per item, the byte weights (u + 15) and
// (v + 15) and a 0/1 mask, each zero outside the circle (|u| <= umax[|v|]),
// and the item's LDS offset.  Then m10 = A - 15 S, m01 = B - 15 S with
// A = sum (u+15) val, B = sum (v+15) val, S = sum val.  Items 279..319 are
// all-zero padding so every lane runs 5 items.
constexpr int kIcItems = 31 * 9, kIcSlots = 320;
struct IcTab {
  uint32_t e[4][kIcSlots][4];  // [o][item] = {W_u, W_v, W_1, lds offset}
};
constexpr int kUmaxC[16] = {15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3};
constexpr IcTab make_ic_tab() {
  IcTab T{};
  for (int o = 0; o < 4; ++o)
    for (int t = 0; t < kIcItems; ++t) {
      const int rv = t / 9, j = t % 9, v = rv - 15, av = v < 0 ? -v : v;
      uint32_t wu = 0, wv = 0, w1 = 0;
      for (int b = 0; b < 4; ++b) {
        const int u = 4 * j + b - o - 15, au = u < 0 ? -u : u;
        if (au <= 15 && au <= kUmaxC[av]) {
          wu |= (uint32_t)(u + 15) << (8 * b);
          wv |= (uint32_t)(v + 15) << (8 * b);
          w1 |= 1u << (8 * b);
        }
      }
      T.e[o][t][0] = wu;
      T.e[o][t][1] = wv;
      T.e[o][t][2] = w1;
      T.e[o][t][3] = (uint32_t)(rv * kRawW + 4 * j);
    }
  return T;
}
__constant__ IcTab c_ic = make_ic_tab();

#ifndef ORB_DESC_KPW
#define ORB_DESC_KPW 1  // keypoints per k_describe wave: 1 (default) or 4 (A/B: 16 lanes each)
#endif
#if ORB_DESC_KPW == 4
// Four keypoints per wave, 16 lanes each (lane 16 g + j: keypoint g).  The
// per-keypoint scalar work -- the moment reductions, fastAtan2, the glibc
// sinf / cosf port (≈100 VALU a keypoint, every lane computing the same
// value in a one-keypoint wave) -- now serves four keypoints per
// instruction.  A wave takes 4 consecutive output slots of ONE (image,
// level) (PlanHeader::kp_quads, LevelGeom::quad_off), so the level planes are
// wave-uniform: both patches are staged by raw buffer loads whose row step is
// the SGPR offset (2 rows x 8 dwords per step, the 9th / 9th-10th dword
// columns in their own steps) -- no per-load address VALU -- 42 dword loads a
// lane in flight.  The IC_Angle weights (W_u, W_1 per item; W_v = row x W_1,
// the item's LDS offset 4 i) and the BRIEF pattern live in the workgroup's
// LDS (filled once per 4-wave block): the constant-table round trips to the
// L1/L2 that made the first version of this kernel wait were most of its time.
// IC_Angle: item i = j + 16 k (row i / 9, dword i % 9), a 16-lane rotate-add
// reduction (row_ror 8, 4, 2, 1).  BRIEF: lane j computes tests 16 j .. 16 j +
// 15 of its keypoint -- the reference's fmaf offsets and cvRound as the
// one-keypoint kernel -- and shifts each t0 < t1 (the sign of t0 - t1) into
// its u16 by one v_alignbit, then stores descriptor bytes 2 j, 2 j + 1.
// Dead slots of a live wave replay the level's last live keypoint and store
// nothing.
constexpr int kRawRows = 32, kBlurRows = 38;  // one spare row each: 2-row load steps
#ifndef ORB_DESC_WG
#define ORB_DESC_WG 4  // waves per k_describe workgroup (they share the tables)
#endif
constexpr int kDescSlice = (kBlurW * kBlurRows + 15) & ~15;  // the blurred patch reuses the raw one's bytes
constexpr int kDescWaveLds = 4 * kDescSlice;
constexpr int kIcItems4 = 288;                  // 18 x 16 items (279 live)
constexpr int kDescPatLds = 256 * 16;           // BRIEF pattern, float4 per test
constexpr int kDescIcLds = 4 * kIcItems4 * 8;   // IC weights (W_u, W_1) per alignment o
constexpr int kDescTabLds = kDescPatLds + kDescIcLds;

__device__ __forceinline__ uint32_t row_sum16(uint32_t v) {  // sum over the lane's 16-lane row
  v += __builtin_amdgcn_update_dpp(0u, v, 0x128, 0xf, 0xf, false);  // row_ror:8
  v += __builtin_amdgcn_update_dpp(0u, v, 0x124, 0xf, 0xf, false);  // row_ror:4
  v += __builtin_amdgcn_update_dpp(0u, v, 0x122, 0xf, 0xf, false);  // row_ror:2
  v += __builtin_amdgcn_update_dpp(0u, v, 0x121, 0xf, 0xf, false);  // row_ror:1
  return v;
}

__global__ __launch_bounds__(64 * ORB_DESC_WG) void k_describe(const PlanHeader* __restrict__ P, ImgSrc src,
                                                 const uint8_t* __restrict__ pyr,
                                                 const uint8_t* __restrict__ blur,
                                                 const uint32_t* __restrict__ oct_out,
                                                 const int* __restrict__ oct_count,
                                                 float* __restrict__ angle_out,
                                                 uint64_t* __restrict__ desc_out, int n_img) {
  __shared__ __attribute__((aligned(16))) uint8_t lds_wg[kDescTabLds + ORB_DESC_WG * kDescWaveLds];
  // ---- the block's tables (every wave takes part: the barrier comes first)
  {
    const int t = threadIdx.x;
    for (int i = t; i < 256; i += 64 * ORB_DESC_WG)
      reinterpret_cast<float4*>(lds_wg)[i] = c_pattern_f[i];
    for (int i = t; i < 4 * kIcItems4; i += 64 * ORB_DESC_WG) {
      const int o = i / kIcItems4, it = i - o * kIcItems4;
      reinterpret_cast<uint2*>(lds_wg + kDescPatLds)[i] = make_uint2(c_ic.e[o][it][0], c_ic.e[o][it][2]);
    }
  }
  __syncthreads();
  const float4* pat = reinterpret_cast<const float4*>(lds_wg);
  const int lane = threadIdx.x & 63, g = lane >> 4, j = lane & 15;
  const int wave = ORB_DESC_WG > 1 ? __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) : 0;
  uint8_t* lds_all = lds_wg + kDescTabLds + wave * kDescWaveLds;
  const int nq = P->kp_quads;
  const int gidx = xcd_remap(blockIdx.x, gridDim.x) * ORB_DESC_WG + wave;
  if (gidx >= n_img * nq) return;  // wave-uniform
  const int img = gidx / nq, q = gidx - img * nq;
  int l = 0;
  while (l + 1 < P->levels && q >= P->lev[l + 1].quad_off) ++l;
  const LevelGeom& gl = P->lev[l];
  const int cnt = __builtin_amdgcn_readfirstlane(oct_count[img * P->levels + l]);
  const int s0 = 4 * (q - gl.quad_off);
  if (s0 >= cnt) return;  // wave-uniform: no live slot
  const bool live = s0 + g < cnt;
  const int slot = gl.out_off + min(s0 + g, cnt - 1);
  const uint32_t kp = oct_out[(size_t)img * P->kp_slots + slot];
  const int cx = (int)(kp & 0xfff) + kFastBorder, cy = (int)((kp >> 12) & 0xfff) + kFastBorder;
  uint8_t* raw = lds_all + g * kDescSlice;
  uint8_t* blp = raw;

  // ---- both patches: rows 2k + (j >> 3), dword j & 7 (SGPR row step), then
  // the raw 9th dword (rows j, j + 16) and the blurred 9th / 10th (rows
  // (j >> 1) + 8 m, dword 8 + (j & 1))
  int sp;
  const uint8_t* rbase = level_plane(P, src, pyr, img, l, sp);
  const uint8_t* bbase = blur + (size_t)img * P->blur_bytes + gl.blur_off;
  const int bp = gl.pitch;
  const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(rbase), (short)0,
                                                                      (int)0xffffffff, kBufRsrcWord3);
  const __amdgpu_buffer_rsrc_t br = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(bbase), (short)0,
                                                                      (int)0xffffffff, kBufRsrcWord3);
  const int rx0 = (cx - 15) & ~3, bx0 = (cx - 18) & ~3;
  const int rq = j & 7, rh = j >> 3;
  const int vr = (cy - 15 + rh) * sp + rx0 + 4 * rq;
  const int vb = (cy - 18 + rh) * bp + bx0 + 4 * rq;
  const int vr8 = (cy - 15 + j) * sp + rx0 + 32;
  const int vb8 = (cy - 18 + (j >> 1)) * bp + bx0 + 32 + 4 * (j & 1);
  uint32_t r_main[16], r_c8[2], b_main[19], b_c8[5];
#pragma unroll
  for (int k = 0; k < 16; ++k) r_main[k] = __builtin_amdgcn_raw_buffer_load_b32(rr, vr, 2 * k * sp, 0);
#pragma unroll
  for (int m = 0; m < 2; ++m) r_c8[m] = __builtin_amdgcn_raw_buffer_load_b32(rr, vr8, 16 * m * sp, 0);
#pragma unroll
  for (int k = 0; k < 19; ++k) b_main[k] = __builtin_amdgcn_raw_buffer_load_b32(br, vb, 2 * k * bp, 0);
  const bool b8_last = (j >> 1) + 32 < kBlurRows;  // rows 38, 39 do not exist
#pragma unroll
  for (int m = 0; m < 5; ++m)
    b_c8[m] = (m < 4 || b8_last) ? __builtin_amdgcn_raw_buffer_load_b32(br, vb8, 8 * m * bp, 0) : 0u;
  {
    uint32_t* d = reinterpret_cast<uint32_t*>(raw + rh * kRawW + 4 * rq);
#pragma unroll
    for (int k = 0; k < 16; ++k) d[k * 2 * kRawW / 4] = r_main[k];
    uint32_t* d8 = reinterpret_cast<uint32_t*>(raw + j * kRawW + 32);
#pragma unroll
    for (int m = 0; m < 2; ++m) d8[m * 16 * kRawW / 4] = r_c8[m];
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

  // ---- IC_Angle: items j + 16 k, k < 18 (288 >= 279; the rest zero).  Raw
  // rows are 9 dwords, so item i sits at byte 4 i
  int m10, m01;
  {
    const uint2* tab = reinterpret_cast<const uint2*>(lds_wg + kDescPatLds) + ((cx - 15) & 3) * kIcItems4;
    uint32_t A = 0, B = 0, S = 0;
#pragma unroll
    for (int k = 0; k < 18; ++k) {
      const int i = 16 * k + j;
      const uint2 w = tab[i];
      const uint32_t val = *reinterpret_cast<const uint32_t*>(raw + 4 * i);
      // the item's row sum s (<= 1020) weighted by its row i / 9 (exact
      // below 4369) is its part of B: every in-circle byte of a row has v + 15 = row
      const uint32_t si = __builtin_amdgcn_udot4(val, w.y, 0u, false);
      A = __builtin_amdgcn_udot4(val, w.x, A, false);
      B = __umul24((uint32_t)i * 7282u >> 16, si) + B;
      S += si;
    }
    const int s = (int)row_sum16(S);
    m10 = (int)row_sum16(A) - 15 * s;
    m01 = (int)row_sum16(B) - 15 * s;
  }
  {  // the raw patch's reads are done (in order within the wave): the blurred one takes its bytes
    uint32_t* e = reinterpret_cast<uint32_t*>(blp + rh * kBlurW + 4 * rq);
#pragma unroll
    for (int k = 0; k < 19; ++k) e[k * 2 * kBlurW / 4] = b_main[k];
    uint32_t* e8 = reinterpret_cast<uint32_t*>(blp + (j >> 1) * kBlurW + 32 + 4 * (j & 1));
#pragma unroll
    for (int m = 0; m < 5; ++m)
      if (m < 4 || b8_last) e8[m * 8 * kBlurW / 4] = b_c8[m];
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const float angle = dev_fast_atan2((float)m01, (float)m10);
  const float ang = angle * (float)(3.14159265358979323846 / 180.0);
  const float a = dev_cosf(ang), b = dev_sinf(ang);

  // ---- steered BRIEF: tests 16 j + 15 .. 16 j, each t0 < t1 shifted in
  const uint8_t* ctr = blp + 18 * kBlurW + (cx - bx0);
  const uint8_t* ctr_m = ctr - (uint32_t)(0x400000u * kBlurW + 0x4B400000u);
  uint32_t acc = 0;
#pragma unroll
  for (int i = 15; i >= 0; --i) {
    const float4 pt = pat[16 * j + i];
    const f32x2 X = {pt.x, pt.y}, Y = {pt.z, pt.w};
    constexpr float kMagic = 12582912.0f;  // cvRound as in the one-keypoint kernel (below)
    const f32x2 R = __builtin_elementwise_fma(X, (f32x2){b, b}, Y * (f32x2){a, a}) + (f32x2){kMagic, kMagic};
    const f32x2 Q = __builtin_elementwise_fma(X, (f32x2){a, a}, Y * (f32x2){-b, -b}) + (f32x2){kMagic, kMagic};
    const int t0 = ctr_m[__umul24(__float_as_uint(R.x), (uint32_t)kBlurW) + __float_as_uint(Q.x)];
    const int t1 = ctr_m[__umul24(__float_as_uint(R.y), (uint32_t)kBlurW) + __float_as_uint(Q.y)];
    acc = __builtin_amdgcn_alignbit(acc, (uint32_t)(t0 - t1), 31);  // (acc << 1) | (t0 < t1)
  }
  if (live) {
    const size_t o = (size_t)img * P->kp_slots + slot;
    reinterpret_cast<uint16_t*>(desc_out + o * 4)[j] = (uint16_t)acc;
    if (j == 0) angle_out[o] = angle;
  }
}
#else
// One wave per octree output slot (measured against a persistent, software-
// pipelined variant: the extra registers halved residency and lost, 201 vs
// 167 us).  The slot's count and keypoint are loaded together; dead slots
// leave before any patch load (their oct_out entries are stale).  Slot, level
// and keypoint are wave-uniform (scalar unit); the patches are staged as
// fixed row x dword grids so LDS stores take immediate offsets.
#ifndef ORB_DESC_WAVES
#define ORB_DESC_WAVES 4  // waves (one keypoint each) per k_describe workgroup
#endif
constexpr int kDescSlice = (kDescLds + 15) & ~15;  // LDS of one describe wave

struct KeyPointOut {  // orbgpu_keypoint (cv::KeyPoint field order)
  float x, y, size, angle, response;
  int octave, class_id;
};
// The dataflow launch's direct output (no lapping band: keypoint i of level l
// is output i + base, base = the keypoints of the lower levels): the wave
// writes its keypoint record and descriptor into the device output block
// itself (write-through: the launch's last item copies the block to the host
// mirror), and the slot arrays are not written.
struct DescFinal {
  KeyPointOut* kps;
  uint64_t* descs;
  int base;
};
// Octree output slot `slot` of image img by one wave (lane 0..63) with its own
// kDescSlice bytes of LDS (raw); only wave-level synchronisation.
template <bool kWT = false>
__device__ __forceinline__ void describe_slot(const PlanHeader* __restrict__ P, const ImgSrc& src,
                                              const uint8_t* __restrict__ pyr,
                                              const uint8_t* __restrict__ blur,
                                              const uint32_t* __restrict__ oct_out,
                                              const int* __restrict__ oct_count,
                                              float* __restrict__ angle_out,
                                              uint64_t* __restrict__ desc_out, int img, int slot,
                                              uint8_t* __restrict__ raw, int lane,
                                              const DescFinal* fin = nullptr) {
  uint8_t* blp = raw + kRawW * kRawH;
  const int kps = P->kp_slots;
  int l = 0;
  while (l + 1 < P->levels && slot >= P->lev[l + 1].out_off) ++l;
  const LevelGeom& g = P->lev[l];
  const int cnt = __builtin_amdgcn_readfirstlane(ld_pub<kWT>(oct_count + img * P->levels + l));
  const uint32_t kp = __builtin_amdgcn_readfirstlane(ld_pub<kWT>(oct_out + (size_t)img * kps + slot));
  if (slot - g.out_off >= cnt) return;  // wave-uniform
  const int cx = (int)(kp & 0xfff) + kFastBorder, cy = (int)((kp >> 12) & 0xfff) + kFastBorder;

  // Stage both patches with independent dword loads (one memory round trip;
  // unaligned only when the level-0 stride is not a multiple of 4):
  // raw 31 rows x 9 dwords as 7-row steps of 63 lanes, blurred 37 x 10 as
  // 6-row steps of 60 lanes.
  int sp;
  const uint8_t* img0 = level_plane(P, src, pyr, img, l, sp);
  const int rx0 = (cx - 15) & ~3, bx0 = (cx - 18) & ~3;
  const uint8_t* rsrc = img0 + (size_t)(cy - 15) * sp + rx0;
  const uint8_t* bsrc = blur + (size_t)img * P->blur_bytes + g.blur_off + (size_t)(cy - 18) * g.pitch + bx0;
  {
    constexpr int kRs = 5, kBs = 7;  // steps
    const int rr = min(lane / 9, 6), rq = lane - (lane / 9) * 9;      // lanes 63: duplicate of 62
    const int br = min(lane / 10, 5), bq = min(lane - (lane / 10) * 10, 9);
    uint32_t vr[kRs], vb[kBs];
#pragma unroll
    for (int k = 0; k < kRs; ++k)
      vr[k] = *reinterpret_cast<const uint32_t*>(rsrc + (uint32_t)(min(rr + 7 * k, kRawH - 1) * sp + 4 * rq));
#pragma unroll
    for (int k = 0; k < kBs; ++k)
      vb[k] = *reinterpret_cast<const uint32_t*>(bsrc + (uint32_t)(min(br + 6 * k, kBlurH - 1) * g.pitch + 4 * bq));
    uint32_t* rd = reinterpret_cast<uint32_t*>(raw + rr * kRawW + 4 * rq);
    uint32_t* bd = reinterpret_cast<uint32_t*>(blp + br * kBlurW + 4 * bq);
#pragma unroll
    for (int k = 0; k < kRs; ++k)
      if (rr + 7 * k < kRawH) rd[k * 7 * kRawW / 4] = vr[k];
#pragma unroll
    for (int k = 0; k < kBs; ++k)
      if (br + 6 * k < kBlurH) bd[k * 6 * kBlurW / 4] = vb[k];
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

  // IC_Angle (see c_ic)
  int m10, m01;
  {
    const uint32_t(*tab)[4] = c_ic.e[(cx - 15) & 3];
    uint32_t A = 0, B = 0, S = 0;
#pragma unroll
    for (int k = 0; k < kIcSlots / 64; ++k) {
      const uint4 w = *reinterpret_cast<const uint4*>(tab[64 * k + lane]);
      const uint32_t val = *reinterpret_cast<const uint32_t*>(raw + w.w);
      A = __builtin_amdgcn_udot4(val, w.x, A, false);
      B = __builtin_amdgcn_udot4(val, w.y, B, false);
      S = __builtin_amdgcn_udot4(val, w.z, S, false);
    }
    const int a = __builtin_amdgcn_readlane(wave_iscan((int)A), 63);
    const int b = __builtin_amdgcn_readlane(wave_iscan((int)B), 63);
    const int s = __builtin_amdgcn_readlane(wave_iscan((int)S), 63);
    m10 = a - 15 * s;
    m01 = b - 15 * s;
  }
  const float angle = dev_fast_atan2((float)m01, (float)m10);

  const float ang = angle * (float)(3.14159265358979323846 / 180.0);
  const float a = dev_cosf(ang), b = dev_sinf(ang);
  const uint8_t* ctr = blp + 18 * kBlurW + (cx - bx0);
  const uint8_t* ctr_m = ctr - (uint32_t)(0x400000u * kBlurW + 0x4B400000u);
  uint64_t words[4];
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const float4 pt = c_pattern_f[64 * w + lane];
    const f32x2 X = {pt.x, pt.y}, Y = {pt.z, pt.w};
    // the reference's fma(x, b, y * a) and fma(x, a, -(y * b)) for both points
    // as packed FP32 (v_pk_mul_f32 / v_pk_fma_f32, each lane IEEE-exact);
    // cvRound of |v| <= 18 by the 1.5 * 2^23 magic add (round-half-even, the
    // same as rintf): bits = 0x4B400000 + round(v).  The row bits' low 24 go
    // through one v_mad_u32_u24, so the offset carries the constant
    // 0x400000 * kBlurW + 0x4B400000, taken off the uniform base (mod 2^32).
    constexpr float kMagic = 12582912.0f;
    const f32x2 R = __builtin_elementwise_fma(X, (f32x2){b, b}, Y * (f32x2){a, a}) + (f32x2){kMagic, kMagic};
    const f32x2 Q = __builtin_elementwise_fma(X, (f32x2){a, a}, Y * (f32x2){-b, -b}) + (f32x2){kMagic, kMagic};
    const uint32_t r0 = __float_as_uint(R.x), r1 = __float_as_uint(R.y);
    const uint32_t q0 = __float_as_uint(Q.x), q1 = __float_as_uint(Q.y);
    const int t0 = ctr_m[__umul24(r0, (uint32_t)kBlurW) + q0];
    const int t1 = ctr_m[__umul24(r1, (uint32_t)kBlurW) + q1];
    words[w] = __ballot(t0 < t1);
  }
  if (fin) {
    const size_t dst = (size_t)fin->base + (slot - g.out_off);
    if (lane < 4) st_pub<true>(fin->descs + dst * 4 + lane, words[lane]);
    if (lane < 7) {  // the record's 7 words, one a lane
      float x = (float)cx, y = (float)cy;
      if (l != 0) {
        x *= g.scale;
        y *= g.scale;
      }
      const float fv[5] = {x, y, g.patch_size, angle, (float)(kp >> 24)};
      const uint32_t w = lane < 5 ? __float_as_uint(fv[lane]) : lane == 5 ? (uint32_t)l : 0xffffffffu;
      st_pub<true>(reinterpret_cast<uint32_t*>(fin->kps + dst) + lane, w);
    }
    return;
  }
  const size_t o = (size_t)img * P->kp_slots + slot;
  if (lane < 4) st_pub<kWT>(desc_out + o * 4 + lane, words[lane]);
  if (lane == 0) st_pub<kWT>(angle_out + o, angle);
}

__global__ __launch_bounds__(64 * ORB_DESC_WAVES) void k_describe(const PlanHeader* __restrict__ P, ImgSrc src,
                                                  const uint8_t* __restrict__ pyr,
                                                  const uint8_t* __restrict__ blur,
                                                  const uint32_t* __restrict__ oct_out,
                                                  const int* __restrict__ oct_count,
                                                  float* __restrict__ angle_out,
                                                  uint64_t* __restrict__ desc_out, int n_img) {
  __shared__ __attribute__((aligned(16))) uint8_t lds_all[ORB_DESC_WAVES * kDescSlice];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int kps = P->kp_slots;
  const int gidx = xcd_remap(blockIdx.x, gridDim.x) * ORB_DESC_WAVES + wave;
  if (gidx >= n_img * kps) return;  // wave-uniform
  const int img = gidx / kps;
  describe_slot(P, src, pyr, blur, oct_out, oct_count, angle_out, desc_out, img, gidx - img * kps,
                lds_all + wave * kDescSlice, lane);
}

#endif  // ORB_DESC_KPW

// --------------------------------------------------------------------------
// k_assemble: operator() tail (orb_extractor.cc:1033-1090) for one image:
// level order, node order inside a level; pt scaled to level 0 (one float
// multiply, level 0 untouched); points with lapping[0] <= x <= lapping[1] go
// to the back in reverse order (stereo), the rest to the front (mono).
// --------------------------------------------------------------------------
// kMirror: every output word also goes to the host-mapped copies (kps_h,
// descs_h, nm_h = {n, mono, err}) of the single-image launch.  LDS: lvl_base
// (kMaxLevels + 1 ints), flags (kAsmChunk ints), scan_tmp (kOctThreads + 1).
constexpr int kAsmChunk = 4096;  // keypoints partitioned per block scan (any n: chunks carry the count)
constexpr int kAsmLds = 4 * (kMaxLevels + 1 + kAsmChunk + kOctThreads + 1);
template <bool kMirror>
__device__ __forceinline__ void assemble_image(const PlanHeader* __restrict__ P,
                                               const uint32_t* __restrict__ oct_out,
                                               const int* __restrict__ oct_count,
                                               const float* __restrict__ angle_in,
                                               const uint64_t* __restrict__ desc_in, int lap0, int lap1,
                                               KeyPointOut* __restrict__ kps, uint64_t* __restrict__ descs,
                                               int cap, int* __restrict__ n_out, int* __restrict__ mono_out,
                                               int* __restrict__ err, int img, int* lvl_base, int* flags,
                                               int* scan_tmp, KeyPointOut* __restrict__ kps_h,
                                               uint64_t* __restrict__ descs_h, int* __restrict__ nm_h) {
  constexpr int kChunk = kAsmChunk;
  const int t = threadIdx.x, L = P->levels;
  if (kMirror) {  // the level counts in one round trip (sc1 loads), then the prefix from LDS
    if (t < L) lvl_base[t + 1] = ld_pub<kMirror>(oct_count + img * L + t);
    __syncthreads();
    if (t == 0) {
      lvl_base[0] = 0;
      for (int l = 0; l < L; ++l) lvl_base[l + 1] += lvl_base[l];
    }
  } else if (t == 0) {
    int acc = 0;
    for (int l = 0; l < L; ++l) {
      lvl_base[l] = acc;
      acc += oct_count[img * L + l];
    }
    lvl_base[L] = acc;
  }
  __syncthreads();
  const int n = lvl_base[L];
  if (n > cap) {
    if (t == 0) {
      n_out[img] = n;
      mono_out[img] = -1;
      atomicOr(err, kErrKpCap);
      if (kMirror) {
        nm_h[0] = n;
        nm_h[1] = -1;
        nm_h[2] = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    return;
  }
  auto locate = [&](int gi, int& l, int& idx) {
    l = 0;
    while (l + 1 < L && gi >= lvl_base[l + 1]) ++l;
    idx = gi - lvl_base[l];
  };
  auto xy_of = [&](int gi, float& x, float& y, int& l, int& slot) {
    int idx;
    locate(gi, l, idx);
    slot = P->lev[l].out_off + idx;
    const uint32_t kp = oct_out[(size_t)img * P->kp_slots + slot];
    x = (float)((int)(kp & 0xfff) + kFastBorder);
    y = (float)((int)((kp >> 12) & 0xfff) + kFastBorder);
    if (l != 0) {
      x *= P->lev[l].scale;
      y *= P->lev[l].scale;
    }
  };
  if (kMirror && (lap1 < kFastBorder || lap0 > lap1)) {
    // no keypoint can be stereo (every x >= kFastBorder): keypoint gi goes to
    // slot gi.  The single-image path's usual case, with every load of a
    // thread's keypoints in flight before its stores (the launch's tail)
    constexpr int U = 4;
    for (int b = t; b < n; b += 256 * U) {
      uint32_t kpv[U];
      float ang[U];
      uint4 dv[U][2];
      int lv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int gi = min(b + 256 * u, n - 1);
        int l, idx;
        locate(gi, l, idx);
        const size_t so = (size_t)img * P->kp_slots + P->lev[l].out_off + idx;
        lv[u] = l;
        kpv[u] = oct_out[so];
        ang[u] = angle_in[so];
        const uint4* d = reinterpret_cast<const uint4*>(desc_in + so * 4);
        dv[u][0] = d[0];
        dv[u][1] = d[1];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int gi = b + 256 * u;
        if (gi >= n) break;
        const int l = lv[u];
        const uint32_t kp = kpv[u];
        KeyPointOut o;
        o.x = (float)((int)(kp & 0xfff) + kFastBorder);
        o.y = (float)((int)((kp >> 12) & 0xfff) + kFastBorder);
        if (l != 0) {
          o.x *= P->lev[l].scale;
          o.y *= P->lev[l].scale;
        }
        o.size = P->lev[l].patch_size;
        o.angle = ang[u];
        o.response = (float)(kp >> 24);
        o.octave = l;
        o.class_id = -1;
        const size_t dst = (size_t)img * cap + gi;
        kps[dst] = o;
        kps_h[dst] = o;
        uint4* od = reinterpret_cast<uint4*>(descs + dst * 4);
        uint4* oh = reinterpret_cast<uint4*>(descs_h + dst * 4);
        od[0] = dv[u][0];
        od[1] = dv[u][1];
        oh[0] = dv[u][0];
        oh[1] = dv[u][1];
      }
    }
    if (t == 0) {
      n_out[img] = n;
      mono_out[img] = n;
      nm_h[0] = n;
      nm_h[1] = n;
      nm_h[2] = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  int n_stereo = 0;  // stereo keypoints before the current chunk
  for (int c0 = 0; c0 < n; c0 += kChunk) {
    const int cn = min(kChunk, n - c0);
    for (int i = t; i < cn; i += 256) {
      float x, y;
      int l, slot;
      xy_of(c0 + i, x, y, l, slot);
      flags[i] = (x >= (float)lap0 && x <= (float)lap1) ? 1 : 0;  // stereo
    }
    __syncthreads();
    const int chunk_stereo = block_scan(flags, cn, scan_tmp);
    for (int i = t; i < cn; i += 256) {
      const int gi = c0 + i;
      float x, y;
      int l, slot;
      xy_of(gi, x, y, l, slot);
      const bool st = (x >= (float)lap0 && x <= (float)lap1);
      const int before_st = n_stereo + flags[i];
      const int dst = st ? n - 1 - before_st : gi - before_st;
      const size_t so = (size_t)img * P->kp_slots + slot;
      const uint32_t kp = oct_out[so];
      KeyPointOut o;
      o.x = x;
      o.y = y;
      o.size = P->lev[l].patch_size;
      o.angle = angle_in[so];
      o.response = (float)(kp >> 24);
      o.octave = l;
      o.class_id = -1;
      kps[(size_t)img * cap + dst] = o;
      const uint64_t* d = desc_in + so * 4;
      uint64_t* od = descs + ((size_t)img * cap + dst) * 4;
      const uint64_t d0 = d[0], d1 = d[1], d2 = d[2], d3 = d[3];
      od[0] = d0;
      od[1] = d1;
      od[2] = d2;
      od[3] = d3;
      if (kMirror) {
        kps_h[(size_t)img * cap + dst] = o;
        uint64_t* oh = descs_h + ((size_t)img * cap + dst) * 4;
        oh[0] = d0;
        oh[1] = d1;
        oh[2] = d2;
        oh[3] = d3;
      }
    }
    n_stereo += chunk_stereo;
    __syncthreads();  // flags are the next chunk's
  }
  if (t == 0) {
    n_out[img] = n;
    mono_out[img] = n - n_stereo;
    if (kMirror) {
      nm_h[0] = n;
      nm_h[1] = n - n_stereo;
      nm_h[2] = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

__global__ __launch_bounds__(256) void k_assemble(const PlanHeader* __restrict__ P,
                                                  const uint32_t* __restrict__ oct_out,
                                                  const int* __restrict__ oct_count,
                                                  const float* __restrict__ angle_in,
                                                  const uint64_t* __restrict__ desc_in, int lap0,
                                                  int lap1, KeyPointOut* __restrict__ kps,
                                                  uint64_t* __restrict__ descs, int cap,
                                                  int* __restrict__ n_out, int* __restrict__ mono_out,
                                                  int* __restrict__ err) {
  __shared__ int lvl_base[kMaxLevels + 1];
  __shared__ int flags[kAsmChunk];
  __shared__ int scan_tmp[kOctThreads + 1];
  assemble_image<false>(P, oct_out, oct_count, angle_in, desc_in, lap0, lap1, kps, descs, cap, n_out, mono_out,
                        err, blockIdx.x, lvl_base, flags, scan_tmp, nullptr, nullptr, nullptr);
}



// --------------------------------------------------------------------------
// k_extract_df: the single-image host path (OrbExtractor::operator() from host
// buffers, orbgpu_extract) as ONE launch.  One frame at a time is a chain of
// small dependent stages (7 resize levels, blur, FAST, octree, describe,
// assemble): as separate launches each stage pays a kernel boundary and a
// launch that covers a fraction of the chip, and the whole chain waits for
// its slowest level.  Here persistent 256-thread workers take work items by
// ticket (orb_launch.h, make_df_items) and each item waits only for what it
// reads: level 0's FAST and octree start as soon as the image is copied,
// while the resize chain and the other levels run beside them.  Stage bodies
// are the batch kernels' own (resize_tile / resize_tail, blur_wave,
// fast_cell, octree_level, describe_slot, assemble_image): the same bytes.
//
// Hand-offs (MI355X_MICROARCH.md, inter-workgroup visibility, R1): every
// payload word a producer item writes for other workgroups is stored
// write-through (sc1: st_pub / the kAuxSc1 buffer stores), its waves drain
// them (vmcnt 0), the workgroup barrier, then one lane adds to the stage's
// counter -- no release fence (a buffer_wbl2 per item cost 2-6 µs on every
// hop of the resize chain); a consumer's lane polls the counter (agent-scope
// relaxed loads, s_sleep between), acquires at agent scope and releases the
// workgroup by a barrier; uniform reads of handed-off words are vector sc1
// loads (ld_pub: the acquire does not refresh the scalar cache).  Polls are bounded:
// a wait that never completes sets kErrDfTimeout and the item runs anyway,
// so every worker reaches the exit.  The last describe item to finish runs
// the assembly, mirroring the output block into host-mapped memory.
// --------------------------------------------------------------------------
enum : int { kErrDfTimeout = 64 };
#ifndef ORB_DF_SLEEP
#define ORB_DF_SLEEP 1  // s_sleep between a waiting worker's polls (x 64 clocks)
#endif

__device__ __forceinline__ void df_wait(int* ctrl, int id, int target, int* err) {
  int* c = ctrl + id * kDfCtrStride;
  for (int spin = 0; __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target; ++spin) {
    if (spin > (1 << 22)) {
      atomicOr(err, kErrDfTimeout);
      break;
    }
    __builtin_amdgcn_s_sleep(ORB_DF_SLEEP);
  }
}

__device__ __forceinline__ void df_acquire() {
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

__global__ __launch_bounds__(256) void k_extract_df(const DfLaunch* __restrict__ a_dev, int* __restrict__ ctrl,
                                                    const int* __restrict__ band_flags, int seq) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  __shared__ int s_item, s_last, s_base;
  for (;;) {
    // the launch record and the thread index laundered per item: values
    // derived from them cannot be hoisted out of the loop (every stage's
    // would stay live across all items); the record's fields are scalar
    // loads from the scalar cache
    const DfLaunch* ap = a_dev;
    asm volatile("" : "+s"(ap));
    const DfLaunch& a = *ap;
    const PlanHeader* __restrict__ P = a.plan;
    const DfPlan& df = a.df;
    int* err = a.nm + 2;
    const ImgSrc src{a.img, 0, P->lev[0].pitch};
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    unsigned long long tr_grab = 0, tr_ready = 0;
    int ticket = 0;
    if (tid == 0) {
      ticket = __hip_atomic_fetch_add(ctrl + kDfTicket * kDfCtrStride, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_item = ticket < df.n_items ? (int)a.items[ticket] : -1;
      if (a.trace) tr_grab = __builtin_amdgcn_s_memrealtime();
    }
    __syncthreads();
    const int it = s_item;
    if (it < 0) break;
    const int type = it & 15, l = (it >> 4) & 15, idx = (int)((uint32_t)it >> 8);
    // ---- wait for the producers of what this item reads (resize items wait
    // inside the tile code, once their plan-constant taps are loaded; FAST
    // items load their cell record first)
    Cell cell{};
    if (type == kDfFast) {
      const int ci = min(P->lev[l].cell_begin + 4 * idx + wave, P->lev[l].cell_end - 1);
      cell = a.cells[ci];
    }
    auto wait = [&]() {
      if (tid == 0) {
        if (type == kDfDescribe) {
          df_wait(ctrl, kDfBlurDone + l, df.blur_items[l], err);
        } else if (type == kDfOctree) {
          df_wait(ctrl, kDfFastDone + l, df.fast_items[l], err);
        } else {
          const int src_l = type == kDfResize ? l - 1 : l;  // the level plane it reads
          if (src_l == 0)
            df_wait(ctrl, kDfImg, df.n_bands, err);
          else
            df_wait(ctrl, kDfLvl + src_l, df.units[src_l], err);
        }
        df_acquire();
      }
      __syncthreads();
    };
    // no lapping band: every keypoint is mono and goes straight to its output
    // slot (DescFinal), so a describe item also waits for the lower levels'
    // octrees (the slot's base); wave 0 polls those counters lane-parallel
    const bool direct = a.lap1 < kFastBorder || a.lap0 > a.lap1;
    if (type == kDfDescribe && wave == 0) {
      const int* oc = ctrl + (kDfOctDone + min(lane, kMaxLevels - 1)) * kDfCtrStride;
      const bool need = direct ? lane <= l : lane == l;
      for (int spin = 0;; ++spin) {
        const bool ok = !need || __hip_atomic_load(oc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= 1;
        if (__builtin_amdgcn_ballot_w64(!ok) == 0) break;
        if (spin > (1 << 22)) {
          if (lane == 0) atomicOr(err, kErrDfTimeout);
          break;
        }
        __builtin_amdgcn_s_sleep(ORB_DF_SLEEP);
      }
    }
    if (type != kDfCopy && type != kDfResize) wait();
    if (type == kDfDescribe && direct) {  // the keypoints of the lower levels (sc1 loads)
      if (wave == 0) {
        int c = lane < l ? ld_pub<true>(a.oct_count + lane) : 0;
        c = wave_iscan(c);
        if (lane == 63) s_base = c;
      }
      __syncthreads();
    }
    if (a.trace && tid == 0) tr_ready = __builtin_amdgcn_s_memrealtime();
    // ---- the item
    int pub;
    if (type == kDfCopy) {
      // the host fills the pinned staging band by band after the launch and
      // stamps each band's flag with the call's sequence number (fine-grained
      // host memory: uncached on the device, so the flag read orders the data)
      if (tid == 0)
        for (int spin = 0; __hip_atomic_load(band_flags + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != seq;
             ++spin) {
          if (spin > (1 << 22)) {
            atomicOr(err, kErrDfTimeout);
            break;
          }
          __builtin_amdgcn_s_sleep(ORB_DF_SLEEP);
        }
      __syncthreads();
      const int b0 = idx * kDfBandBytes, nb = min(kDfBandBytes, df.img_bytes - b0) >> 4;
      const uint4* s4 = reinterpret_cast<const uint4*>(a.img_host + b0);
      // write-through (sc1) 16-B stores: published without a release fence
      const __amdgpu_buffer_rsrc_t drs =
          __builtin_amdgcn_make_buffer_rsrc(a.img + b0, (short)0, (int)0xffffffff, kBufRsrcWord3);
      uint4 v[kDfBandBytes / 16 / 256];
#pragma unroll
      for (int u = 0; u < kDfBandBytes / 16 / 256; ++u)
        if (tid + 256 * u < nb) v[u] = s4[tid + 256 * u];
#pragma unroll
      for (int u = 0; u < kDfBandBytes / 16 / 256; ++u)
        if (tid + 256 * u < nb)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v[u]),
                                                 drs, 16 * (tid + 256 * u), 0, kAuxSc1);
      pub = kDfImg;
    } else if (type == kDfResize) {
      const LevelGeom& g = P->lev[l];
      const int nt = g.rs_tiles_x * g.rs_tiles_y;
      if (idx < nt)
        resize_tile<true>(P, a.rs_tab, src, a.pyr, l, 0, idx, lds, tid, true, wait);
      else
        resize_tail<true>(P, a.rs_tab, src, a.pyr, l, 0, idx - nt, lds, tid, wait);
      pub = kDfLvl + l;
    } else if (type == kDfFast) {
      const int ci = P->lev[l].cell_begin + 4 * idx + wave;
      if (ci < P->lev[l].cell_end) {
        uint8_t* fl = lds + wave * P->max_roi_lds;
        switch (P->fast_pitch) {
          case 48: fast_cell<48, true>(P, a.cells, src, a.pyr, a.slots, a.cell_count, 0, ci, fl, lane, &cell); break;
          case 52: fast_cell<52, true>(P, a.cells, src, a.pyr, a.slots, a.cell_count, 0, ci, fl, lane, &cell); break;
          case 56: fast_cell<56, true>(P, a.cells, src, a.pyr, a.slots, a.cell_count, 0, ci, fl, lane, &cell); break;
          case 60: fast_cell<60, true>(P, a.cells, src, a.pyr, a.slots, a.cell_count, 0, ci, fl, lane, &cell); break;
          case 64: fast_cell<64, true>(P, a.cells, src, a.pyr, a.slots, a.cell_count, 0, ci, fl, lane, &cell); break;
          default: fast_cell<0, true>(P, a.cells, src, a.pyr, a.slots, a.cell_count, 0, ci, fl, lane, &cell); break;
        }
      }
      pub = kDfFastDone + l;
    } else if (type == kDfBlur) {
      static_assert(ORB_BLUR_WAVES == 4, "k_extract_df runs a blur tile per 4-wave worker");
      blur_wave<true>(P, src, a.pyr, a.blur, 0, P->lev[l].blur_tile_begin + idx, 0);
      pub = kDfBlurDone + l;
    } else if (type == kDfOctree) {
      // (plans whose node arrays live in HBM take the per-stage launches: one
      // octree instance keeps the worker's registers down)
      octree_level<false, true>(P, a.cells, a.slots, a.cell_count, a.dense, a.knode, a.oct_out, a.oct_count, err, 0, l,
                          P->oct_kcap, nullptr, lds);
      pub = kDfOctDone + l;
    } else if (type == kDfMirror) {
      // the output block's host mirror by this one workgroup (host-memory
      // writes of different CUs reach the host in no promised order), level
      // by level in output order as each level's describe items finish, so
      // only the last levels' few records are left when the final one lands;
      // then the counts and the call's number.  With a lapping band the last
      // describe item assembles and mirrors instead.
      if (direct) {
        if (a.trace && tid == 0) a.trace[4 * (size_t)df.n_items] = __builtin_amdgcn_s_memrealtime();
        auto copy = [&](const void* src, void* dst, int bytes) {
          const uint4* s4 = reinterpret_cast<const uint4*>(src);
          uint4* d4 = reinterpret_cast<uint4*>(dst);
          const int n16 = (bytes + 15) >> 4;
          for (int i0 = tid; i0 < n16; i0 += 256 * 4) {
            uint4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u)
              if (i0 + 256 * u < n16) v[u] = s4[i0 + 256 * u];
#pragma unroll
            for (int u = 0; u < 4; ++u)
              if (i0 + 256 * u < n16) d4[i0 + 256 * u] = v[u];
          }
        };
        int base = 0;
        for (int lv = 0; lv < P->levels; ++lv) {
          if (tid == 0) {
            df_wait(ctrl, kDfDescLvl + lv, (P->lev[lv].out_cap + 3) / 4, err);
            df_acquire();
            s_base = ld_pub<true>(a.oct_count + lv);
          }
          __syncthreads();
          const int nl = s_base;
          __syncthreads();
          {  // 28-B records: dwords (a level's range need not be 16-B aligned)
            const uint32_t* s1 = reinterpret_cast<const uint32_t*>(a.kps_out) + 7 * (size_t)base;
            uint32_t* d1 = reinterpret_cast<uint32_t*>(a.kps_host) + 7 * (size_t)base;
            for (int i = tid; i < 7 * nl; i += 256) d1[i] = s1[i];
          }
          copy(reinterpret_cast<const uint64_t*>(a.desc_out) + 4 * (size_t)base,
               reinterpret_cast<uint64_t*>(a.desc_host) + 4 * (size_t)base, nl * 32);
          base += nl;
        }
        if (tid == 0) {
          a.nm[0] = base;  // device counts (read by the stereo matcher)
          a.nm[1] = base;
          a.nm_host[0] = base;
          a.nm_host[1] = base;
          a.nm_host[2] = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {  // every mirror store of this workgroup drained: the host's word
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
          __hip_atomic_store(a.done_host, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        if (a.trace && tid == 0) a.trace[4 * (size_t)df.n_items + 1] = __builtin_amdgcn_s_memrealtime();
      }
      pub = kDfMirrorDone;
    } else {  // kDfDescribe: slots out_off + 4 idx + wave of level l
      const int k = 4 * idx + wave;
      const DescFinal fin{reinterpret_cast<KeyPointOut*>(a.kps_out), reinterpret_cast<uint64_t*>(a.desc_out), s_base};
      if (k < P->lev[l].out_cap)
        describe_slot<true>(P, src, a.pyr, a.blur, a.oct_out, a.oct_count, a.angle, a.desc, 0, P->lev[l].out_off + k,
                            lds + wave * kDescSlice, lane, direct ? &fin : nullptr);
      pub = kDfDescDone;
    }
    // ---- publish: every payload store was write-through (sc1); every wave
    // drains them, then one lane adds to the counter (no release fence)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      if (pub == kDfDescDone)  // the level's own count too (the host mirror's item waits on it)
        (void)__hip_atomic_fetch_add(ctrl + (kDfDescLvl + l) * kDfCtrStride, 1, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
      const int old = __hip_atomic_fetch_add(ctrl + pub * kDfCtrStride, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const bool last = pub == kDfDescDone && old == df.desc_items - 1;
      if (last) df_acquire();  // every describe (and so every octree) item's results
      s_last = last;
      if (a.trace) {
        unsigned long long* r = a.trace + 4 * (size_t)ticket;
        r[0] = tr_grab;
        r[1] = tr_ready;
        r[2] = __builtin_amdgcn_s_memrealtime();
        // HW_ID (CU / SIMD / SE ids) and XCC_ID (gfx950 hwreg 20) of this worker
        const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);
        const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);
        r[3] = (unsigned long long)(unsigned)it | ((unsigned long long)hw << 32) | ((unsigned long long)xcc << 60);
      }
    }
    __syncthreads();
    if (s_last && !direct) {
      if (a.trace && tid == 0) a.trace[4 * (size_t)df.n_items] = __builtin_amdgcn_s_memrealtime();
      int* ab = reinterpret_cast<int*>(lds);
      assemble_image<true>(P, a.oct_out, a.oct_count, a.angle, a.desc, a.lap0, a.lap1,
                           reinterpret_cast<KeyPointOut*>(a.kps_out), reinterpret_cast<uint64_t*>(a.desc_out), a.cap,
                           a.nm, a.nm + 1, err, 0, ab, ab + kMaxLevels + 1, ab + kMaxLevels + 1 + kAsmChunk,
                           reinterpret_cast<KeyPointOut*>(a.kps_host), reinterpret_cast<uint64_t*>(a.desc_host),
                           a.nm_host);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {  // (as above: every store of the assembly drained first)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        __hip_atomic_store(a.done_host, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      if (a.trace && tid == 0) a.trace[4 * (size_t)df.n_items + 1] = __builtin_amdgcn_s_memrealtime();
    }
  }
  // ---- the last worker out clears the control block for the next launch
  if (threadIdx.x == 0) {
    const int old = __hip_atomic_fetch_add(ctrl + kDfExit * kDfCtrStride, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == (int)gridDim.x - 1)
      for (int i = 0; i < kDfCounters; ++i)
        __hip_atomic_store(ctrl + i * kDfCtrStride, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

}  // namespace orbgpu

// ==========================================================================
// Host launchers (same translation unit as the kernels).
// ==========================================================================
#include "lds_optin.h"
#include "orb_launch.h"

namespace orbgpu {

hipError_t launch_extract(const ExtractLaunch& a, hipStream_t st) {
  const PlanHeader& H = *a.host_plan;
  ImgSrc src{a.imgs, a.image_pitch, a.stride};
  const int n = a.n_images;
  auto mark = [&](int i) {
    if (a.events) (void)hipEventRecord(a.events[i], st);
    if (a.stage_event && i == a.stage_event_at + 1) (void)hipEventRecord(a.stage_event, st);
  };
  mark(0);
  if (a.pyramid_groups > 0) {  // one launch: a workgroup per image (k_pyramid)
    hipLaunchKernelGGL(k_pyramid, dim3(n), dim3(256 * a.pyramid_groups), (size_t)a.pyramid_groups * H.rs_lds, st,
                       a.plan, a.rs_tab, src, a.pyr, H.rs_lds);
  } else {
    for (int l = 1; l < H.levels; ++l) {
      const LevelGeom& g = H.lev[l];
      const unsigned blocks = (unsigned)(g.rs_tiles_x * g.rs_tiles_y + g.rs_tail_blocks) * (unsigned)n;
      hipLaunchKernelGGL(k_resize, dim3(blocks), dim3(256), H.rs_lds, st, a.plan, a.rs_tab, src, a.pyr, l);
    }
  }
  mark(1);
  hipLaunchKernelGGL(k_blur, dim3(n * H.blur_tiles * (4 / ORB_BLUR_WAVES)), dim3(64 * ORB_BLUR_WAVES), 0, st, a.plan, src,
                     (const uint8_t*)a.pyr, a.blur);
  mark(2);
  auto fast = H.fast_pitch == 48   ? k_fast_cells<48>
              : H.fast_pitch == 52 ? k_fast_cells<52>
              : H.fast_pitch == 56 ? k_fast_cells<56>
              : H.fast_pitch == 60 ? k_fast_cells<60>
              : H.fast_pitch == 64 ? k_fast_cells<64>
                                   : k_fast_cells<0>;
  hipLaunchKernelGGL(fast, dim3((unsigned)(((long)n * H.n_cells + ORB_FAST_WAVES - 1) / ORB_FAST_WAVES)),
                     dim3(64 * ORB_FAST_WAVES), H.max_roi_lds * ORB_FAST_WAVES, st, a.plan,
                     a.cells, src, (const uint8_t*)a.pyr, a.slots, a.cell_count, n);
  mark(3);
  hipLaunchKernelGGL(H.oct_hbm_nodes ? k_octree<true> : k_octree<false>, dim3(n * H.levels),
                     dim3(kOctThreads), a.octree_lds, st, a.plan, a.cells, (const uint32_t*)a.slots,
                     (const int*)a.cell_count, a.dense, a.knode, a.oct_out, a.oct_count, a.err, n,
                     H.oct_kcap, a.oct_nodes);
  mark(4);
#if ORB_DESC_KPW == 4
  hipLaunchKernelGGL(k_describe, dim3((unsigned)(((long)n * H.kp_quads + ORB_DESC_WG - 1) / ORB_DESC_WG)),
                     dim3(64 * ORB_DESC_WG), 0, st, a.plan, src,
#else
  const long waves = (long)n * H.kp_slots;
  hipLaunchKernelGGL(k_describe, dim3((unsigned)((waves + ORB_DESC_WAVES - 1) / ORB_DESC_WAVES)),
                     dim3(64 * ORB_DESC_WAVES), 0, st, a.plan, src,
#endif
                     (const uint8_t*)a.pyr, (const uint8_t*)a.blur, (const uint32_t*)a.oct_out,
                     (const int*)a.oct_count, a.angle, a.desc, n);
  mark(5);
  hipLaunchKernelGGL(k_assemble, dim3(n), dim3(256), 0, st, a.plan, (const uint32_t*)a.oct_out,
                     (const int*)a.oct_count, (const float*)a.angle, (const uint64_t*)a.desc,
                     a.lap0, a.lap1, reinterpret_cast<KeyPointOut*>(a.kps_out),
                     reinterpret_cast<uint64_t*>(a.desc_out), a.cap, a.n_out, a.mono_out, a.err);
  mark(6);
  return hipGetLastError();
}

hipError_t launch_extract_df(const DfLaunch& a, const DfLaunch* a_dev, const int* band_flags, int seq,
                             hipStream_t st) {
  hipLaunchKernelGGL(k_extract_df, dim3(a.grid), dim3(256), a.df.lds_bytes, st, a_dev, a.ctrl, band_flags, seq);
  return hipGetLastError();
}

size_t df_lds_bytes(const PlanHeader& P, size_t octree_lds) {
  return std::max({(size_t)P.rs_lds, (size_t)4 * P.max_roi_lds, octree_lds, (size_t)4 * kDescSlice, (size_t)kAsmLds});
}

hipError_t set_df_lds_limit(size_t bytes) {
  return bytes > 64 * 1024 ? lds_optin((const void*)k_extract_df, (int)bytes) : hipSuccess;
}

// The plan's own LDS needs, raised per (kernel, device) only as far as a plan
// asks (lds_optin never lowers a grant, so handles with different plans never
// shrink each other's limit); sizes up to 64 KB need no opt-in.
hipError_t set_lds_limits(size_t octree_bytes, size_t resize_bytes) {
  if (octree_bytes > 64 * 1024) {
    for (const void* k : {(const void*)k_octree<false>, (const void*)k_octree<true>}) {
      const hipError_t e = lds_optin(k, (int)octree_bytes);
      if (e != hipSuccess) return e;
    }
  }
  if (resize_bytes > 64 * 1024) {
    const hipError_t e = lds_optin((const void*)k_resize, (int)resize_bytes);
    if (e != hipSuccess) return e;
  }
  const int G = pyramid_groups_for(resize_bytes);
  if (G > 0 && (size_t)G * resize_bytes > 64 * 1024) return lds_optin((const void*)k_pyramid, (int)(G * resize_bytes));
  return hipSuccess;
}

int pyramid_groups_for(size_t resize_bytes) {
  if (resize_bytes == 0) return 4;
  return (int)std::min<size_t>(4, (160 * 1024) / resize_bytes);
}

}  // namespace orbgpu

#ifdef ORB_STAMPS
extern "C" int orbgpu_debug_stamps(unsigned long long* out, int n) {
  if (n > 16) n = 16;
  static unsigned long long buf[64 * 16];
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(buf, HIP_SYMBOL(orbgpu::g_stamps), sizeof(buf)) != hipSuccess) return -1;
  for (int i = 0; i < n; ++i) {
    out[i] = 0;
    for (int c = 0; c < 64; ++c) out[i] += buf[c * 16 + i];
  }
  static const unsigned long long z[64 * 16] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(orbgpu::g_stamps), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif
