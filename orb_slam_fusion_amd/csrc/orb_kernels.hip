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

#include "orb_math_dev.h"
#include "orb_plan.h"

namespace orbgpu {

__constant__ int8_t c_pattern[1024] = {
#include "pattern31.inc"
};

enum : int { kErrNodeCap = 1, kErrOutCap = 2, kErrSlotCap = 4, kErrKpCap = 8 };

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
  pitch = P->lev[l].w;
  return pyr + (size_t)img * P->pyr_bytes + P->lev[l].pyr_off;
}

// --------------------------------------------------------------------------
// k_resize: cv::resize INTER_LINEAR, 8UC1.  Horizontal
// taps are (sx, a0, a1) per column, vertical (r0, r1, b0, b1) per row, both
// precomputed by the planner.  Columns below vec_end use the 128-bit SIMD
// rounding ((H>>4)*b >> 16 summed, +2 >> 2), the tail the scalar
// (H0*b0 + H1*b1 + 2^21) >> 22 -- exactly where OpenCV switches.
// Each thread produces 4 consecutive output pixels.
// --------------------------------------------------------------------------
__device__ __forceinline__ int h_tap(const uint8_t* S, int x, int xmax, int2 xa) {
  const int sx = xa.x;
  const int a0 = (int)(short)(xa.y & 0xffff), a1 = (int)(short)(xa.y >> 16);
  return x < xmax ? S[sx] * a0 + S[sx + 1] * a1 : S[sx] * 2048;
}

__global__ __launch_bounds__(256) void k_resize(const PlanHeader* __restrict__ P,
                                                const int* __restrict__ rs_tab, ImgSrc src,
                                                uint8_t* __restrict__ pyr, int l) {
  const LevelGeom& g = P->lev[l];
  const int x0 = (blockIdx.x * 64 + threadIdx.x) * 4;
  const int y = blockIdx.y * 4 + threadIdx.y;
  const int img = blockIdx.z;
  if (x0 >= g.w || y >= g.h) return;
  int sp;
  const uint8_t* S = level_plane(P, src, pyr, img, l - 1, sp);
  uint8_t* D = pyr + (size_t)img * P->pyr_bytes + g.pyr_off + (size_t)y * g.w;
  const int2 yt = reinterpret_cast<const int2*>(rs_tab + g.rs_y)[y];
  const int r0 = yt.x & 0xffff, r1 = yt.x >> 16;
  const int b0 = (int)(short)(yt.y & 0xffff), b1 = (int)(short)(yt.y >> 16);
  const uint8_t* S0 = S + (size_t)r0 * sp;
  const uint8_t* S1 = S + (size_t)r1 * sp;
  const int2* xt = reinterpret_cast<const int2*>(rs_tab + g.rs_x);
  uint32_t packed = 0;
  const int n = min(4, g.w - x0);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (k < n) {
      const int x = x0 + k;
      const int2 xa = xt[x];
      const int h0 = h_tap(S0, x, g.xmax, xa), h1 = h_tap(S1, x, g.xmax, xa);
      int v;
      if (x < g.vec8_end) {
        const int m0 = (max(min(h0 >> 4, 32767), -32768) * b0) >> 16;
        const int m1 = (max(min(h1 >> 4, 32767), -32768) * b1) >> 16;
        const int s = max(min(m0 + m1, 32767), -32768);
        v = (s + 2) >> 2;
      } else {
        v = (h0 * b0 + h1 * b1 + (1 << 21)) >> 22;
      }
      packed |= (uint32_t)min(max(v, 0), 255) << (8 * k);
    }
  }
  if (n == 4 && (((uintptr_t)(D + x0)) & 3) == 0) {
    *reinterpret_cast<uint32_t*>(D + x0) = packed;
  } else {
    for (int k = 0; k < n; ++k) D[x0 + k] = (uint8_t)(packed >> (8 * k));
  }
}

// --------------------------------------------------------------------------
// k_blur: GaussianBlur 7x7, sigma 2, BORDER_REFLECT_101, bit-exact fixed point
// (SURVEY Appendix A.3): Q8 taps [18 34 48 56 48 34 18], horizontal sums kept
// exact, (sum + 2^15) >> 16 once.  64x16 output tiles through LDS; one launch
// covers every level of every image.
// --------------------------------------------------------------------------
__device__ __forceinline__ int reflect101(int i, int n) {
  i = i < 0 ? -i : i;
  return i >= n ? 2 * n - 2 - i : i;
}

__global__ __launch_bounds__(256) void k_blur(const PlanHeader* __restrict__ P, ImgSrc src,
                                              const uint8_t* __restrict__ pyr,
                                              uint8_t* __restrict__ blur) {
  constexpr int TW = kBlurTileW, TH = kBlurTileH;
  constexpr int IW = TW + 6, IH = TH + 6;
  __shared__ uint8_t tin[IH][IW + 2];
  __shared__ int thor[IH][TW + 1];
  const int img = blockIdx.x / P->blur_tiles;
  int t = blockIdx.x - img * P->blur_tiles;
  int l = 0;
  while (l + 1 < P->levels && t >= P->lev[l + 1].blur_tile_begin) ++l;
  const LevelGeom& g = P->lev[l];
  t -= g.blur_tile_begin;
  const int ty = t / g.tiles_x, tx = t - ty * g.tiles_x;
  const int ox = tx * TW, oy = ty * TH;
  int sp;
  const uint8_t* S = level_plane(P, src, pyr, img, l, sp);
  for (int i = threadIdx.x; i < IH * IW; i += 256) {
    const int r = i / IW, c = i - r * IW;
    const int yy = reflect101(oy + r - 3, g.h), xx = reflect101(min(ox + c - 3, g.w + 2), g.w);
    tin[r][c] = S[(size_t)yy * sp + xx];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < IH * TW; i += 256) {
    const int r = i / TW, c = i - r * TW;
    const uint8_t* q = &tin[r][c];
    thor[r][c] = 18 * (q[0] + q[6]) + 34 * (q[1] + q[5]) + 48 * (q[2] + q[4]) + 56 * q[3];
  }
  __syncthreads();
  uint8_t* D = blur + (size_t)img * P->blur_bytes + g.blur_off;
  for (int i = threadIdx.x; i < TH * TW; i += 256) {
    const int r = i / TW, c = i - r * TW;
    const int y = oy + r, x = ox + c;
    if (y < g.h && x < g.w) {
      const uint32_t s = 18u * (thor[r][c] + thor[r + 6][c]) + 34u * (thor[r + 1][c] + thor[r + 5][c]) +
                         48u * (thor[r + 2][c] + thor[r + 4][c]) + 56u * thor[r + 3][c];
      D[(size_t)y * g.w + x] = (uint8_t)min((s + (1u << 15)) >> 16, 255u);
    }
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
// Candidates are compacted in raster order with ballot/mbcnt, giving exactly
// the reference's per-cell keypoint order.
// --------------------------------------------------------------------------
__device__ __forceinline__ int fast_score(const uint8_t* p, const int* off) {
  const int v = p[0];
  int d[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) d[k] = v - (int)p[off[k]];
  int mn[16], mx[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    mn[k] = min(d[k], d[(k + 1) & 15]);
    mx[k] = max(d[k], d[(k + 1) & 15]);
  }
  int mn4[16], mx4[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    mn4[k] = min(mn[k], mn[(k + 2) & 15]);
    mx4[k] = max(mx[k], mx[(k + 2) & 15]);
  }
  int a = -1024, b = 1024;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int m9 = min(min(mn4[k], mn4[(k + 4) & 15]), d[(k + 8) & 15]);
    const int M9 = max(max(mx4[k], mx4[(k + 4) & 15]), d[(k + 8) & 15]);
    a = max(a, m9);
    b = min(b, M9);
  }
  return max(a, -b) - 1;
}

__global__ __launch_bounds__(64) void k_fast_cells(const PlanHeader* __restrict__ P,
                                                   const Cell* __restrict__ cells, ImgSrc src,
                                                   const uint8_t* __restrict__ pyr,
                                                   uint32_t* __restrict__ slots,
                                                   int* __restrict__ cell_count) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int lane = threadIdx.x;
  const int img = blockIdx.x / P->n_cells;
  const int ci = blockIdx.x - img * P->n_cells;
  const Cell c = cells[ci];
  uint8_t* roi = lds;
  uint8_t* score = lds + P->max_roi;
  int sp;
  const uint8_t* S = level_plane(P, src, pyr, img, c.level, sp) + (size_t)c.y0 * sp + c.x0;
  const int npx = c.rows * c.cols;
  for (int i = lane; i < npx; i += 64) {
    const int r = i / c.cols, q = i - r * c.cols;
    roi[i] = S[(size_t)r * sp + q];
  }
  __syncthreads();

  const int dw = c.cols - 6, dh = c.rows - 6;
  const int nd = (dw > 0 && dh > 0) ? dw * dh : 0;
  const int th_ini = P->ini_th, th_min = P->min_th;
  const int th_lo = min(th_ini, th_min);
  int off[16];
  {
    const int cx[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
    const int cy[16] = {3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3};
#pragma unroll
    for (int k = 0; k < 16; ++k) off[k] = cx[k] + cy[k] * c.cols;
  }
  for (int i = lane; i < nd; i += 64) {
    const int r = i / dw, q = i - r * dw;
    const int s = fast_score(roi + (r + 3) * c.cols + q + 3, off);
    score[i] = (uint8_t)(s >= th_lo ? s : 0);
  }
  __syncthreads();

  auto is_kp = [&](int i, int th) -> bool {
    if (i >= nd) return false;
    const int s = score[i];
    if (s < th) return false;
    const int r = i / dw, q = i - r * dw;
#pragma unroll
    for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
      for (int dx = -1; dx <= 1; ++dx) {
        if (dx == 0 && dy == 0) continue;
        const int rr = r + dy, qq = q + dx;
        if (rr < 0 || rr >= dh || qq < 0 || qq >= dw) continue;
        const int t = score[rr * dw + qq];
        if (s <= (t >= th ? t : 0)) return false;
      }
    return true;
  };

  int n_ini = 0;
  for (int base = 0; base < nd; base += 64) n_ini += __popcll(__ballot(is_kp(base + lane, th_ini)));
  const int th = n_ini > 0 ? th_ini : th_min;

  uint32_t* out = slots + (size_t)img * P->slots + c.slot_off;
  const int xrel0 = c.x0 + 3 - kFastBorder, yrel0 = c.y0 + 3 - kFastBorder;
  int written = 0;
  const uint64_t lt = (1ull << lane) - 1ull;
  for (int base = 0; base < nd; base += 64) {
    const int i = base + lane;
    const bool k = is_kp(i, th);
    const uint64_t m = __ballot(k);
    if (k) {
      const int r = i / dw, q = i - r * dw;
      const int pos = written + __popcll(m & lt);
      if (pos < c.slot_cap)
        out[pos] = (uint32_t)(xrel0 + q) | ((uint32_t)(yrel0 + r) << 12) | ((uint32_t)score[i] << 24);
    }
    written += __popcll(m);
  }
  if (lane == 0) cell_count[(size_t)img * P->n_cells + ci] = min(written, c.slot_cap);
}

// --------------------------------------------------------------------------
// Block-wide helpers for the octree (256 threads).
// --------------------------------------------------------------------------
constexpr int kOctThreads = 256;

// In-place exclusive scan of a[0..n) in LDS; returns the total.  `tmp` holds
// kOctThreads + 1 ints of LDS.  Must be called by the whole block.
__device__ int block_scan(int* a, int n, int* tmp) {
  const int t = threadIdx.x;
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
};

__global__ __launch_bounds__(kOctThreads) void k_octree(
    const PlanHeader* __restrict__ P, const Cell* __restrict__ cells,
    const uint32_t* __restrict__ slots, const int* __restrict__ cell_count,
    uint32_t* __restrict__ dense, int* __restrict__ knode, uint32_t* __restrict__ oct_out,
    int* __restrict__ oct_count, int* __restrict__ err) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds_raw[];
  const int L = P->levels;
  const int img = blockIdx.x / L, l = blockIdx.x - img * L;
  const LevelGeom& g = P->lev[l];
  const int NC = P->node_cap;
  const int t = threadIdx.x;

  OctLds s;
  {
    unsigned long long* p64 = reinterpret_cast<unsigned long long*>(lds_raw);
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
    s.scan_tmp = p;
    p += kOctThreads + 1;
    s.scal = p;
  }

  // ---- gather this level's candidates in to_dist order (cell-major, raster).
  const int nc = g.cell_end - g.cell_begin;
  int* cell_off = s.tmp2;  // nc <= NC guaranteed by the planner
  for (int i = t; i < nc; i += kOctThreads)
    cell_off[i] = cell_count[(size_t)img * P->n_cells + g.cell_begin + i];
  __syncthreads();
  const int K = block_scan(cell_off, nc, s.scan_tmp);
  uint32_t* kd = dense + (size_t)img * P->slots + g.slot_begin;
  int* kn = knode + (size_t)img * P->slots + g.slot_begin;
  {
    const int wave = t >> 6, lane = t & 63;
    for (int i = wave; i < nc; i += kOctThreads / 64) {
      const Cell c = cells[g.cell_begin + i];
      const int n = cell_count[(size_t)img * P->n_cells + g.cell_begin + i];
      const uint32_t* src = slots + (size_t)img * P->slots + c.slot_off;
      for (int k = lane; k < n; k += 64) kd[cell_off[i] + k] = src[k];
    }
  }
  uint32_t* out = oct_out + (size_t)img * P->kp_slots + g.out_off;
  if (K == 0) {
    if (t == 0) oct_count[img * L + l] = 0;
    return;
  }
  __syncthreads();

  // ---- roots: round(W/H) equal-width columns; empty roots are erased.
  const int R = g.n_roots;
  const float hx = g.root_w;
  for (int i = t; i < R; i += kOctThreads) s.ccnt[i] = 0;
  __syncthreads();
  for (int k = t; k < K; k += kOctThreads) {
    const float x = (float)(kd[k] & 0xfff);
    const int r = (int)(x / hx);
    kn[k] = r;
    atomicAdd(&s.ccnt[r], 1);
  }
  __syncthreads();
  for (int i = t; i < R; i += kOctThreads) s.tmp2[i] = s.ccnt[i] > 0 ? 1 : 0;
  __syncthreads();
  int S = block_scan(s.tmp2, R, s.scan_tmp);
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
  for (int k = t; k < K; k += kOctThreads) kn[k] = s.tmp2[kn[k]];
  __syncthreads();

  const int N = g.budget;
  int phase = 1, n_exp = 0;
  bool finished = false;
  while (!finished) {
    // ---- choose D and its processing order (rank), uniform across the block
    int m;  // |D|
    for (int i = t; i < S; i += kOctThreads) s.rank[i] = -1;
    __syncthreads();
    if (phase == 1) {
      for (int i = t; i < S; i += kOctThreads) s.tmp2[i] = s.cnt[i] >= 2 ? 1 : 0;
      __syncthreads();
      m = block_scan(s.tmp2, S, s.scan_tmp);
      for (int i = t; i < S; i += kOctThreads)
        if (s.cnt[i] >= 2) s.rank[i] = s.tmp2[i];
    } else {
      // stable sort of exp_list[0..n_exp) by (cnt, x0); processed from the back
      for (int j = t; j < n_exp; j += kOctThreads) {
        const int pj = s.exp_list[j];
        const int cj = s.cnt[pj], xj = s.x0[pj];
        int r = 0;
        for (int i = 0; i < n_exp; ++i) {
          const int pi = s.exp_list[i];
          const int ci = s.cnt[pi], xi = s.x0[pi];
          r += (ci < cj) || (ci == cj && (xi < xj || (xi == xj && i < j)));
        }
        s.rank[pj] = n_exp - 1 - r;
      }
      m = n_exp;
    }
    __syncthreads();

    // ---- midlines of D and child point counts
    for (int i = t; i < S; i += kOctThreads) {
      if (s.rank[i] >= 0) {
        s.mx[i] = s.x0[i] + (int)ceilf((float)(s.x1[i] - s.x0[i]) / 2);
        s.my[i] = s.y0[i] + (int)ceilf((float)(s.y1[i] - s.y0[i]) / 2);
      }
      s.ccnt[4 * i] = s.ccnt[4 * i + 1] = s.ccnt[4 * i + 2] = s.ccnt[4 * i + 3] = 0;
    }
    __syncthreads();
    for (int k = t; k < K; k += kOctThreads) {
      const int n = kn[k];
      if (s.rank[n] >= 0) {
        const int x = kd[k] & 0xfff, y = (kd[k] >> 12) & 0xfff;
        const int q = (x < s.mx[n] ? 0 : 1) + (y < s.my[n] ? 0 : 2);
        atomicAdd(&s.ccnt[4 * n + q], 1);
      }
    }
    __syncthreads();
    for (int i = t; i < S; i += kOctThreads) {
      const int r = s.rank[i];
      if (r >= 0)
        s.pc[r] = (s.ccnt[4 * i] > 0) + (s.ccnt[4 * i + 1] > 0) + (s.ccnt[4 * i + 2] > 0) +
                  (s.ccnt[4 * i + 3] > 0);
    }
    __syncthreads();

    // ---- phase 2 stops once the node count reaches the budget
    if (phase == 2) {
      for (int r = t; r < m; r += kOctThreads) s.tmp2[r] = s.pc[r] - 1;
      __syncthreads();
      const int tot = block_scan(s.tmp2, m, s.scan_tmp);
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

    // ---- push offsets (processing order) and stay offsets (list order)
    const int T = block_scan(s.pc, m, s.scan_tmp);  // s.pc[r] = push offset of rank r
    for (int i = t; i < S; i += kOctThreads) s.stay[i] = s.rank[i] < 0 ? 1 : 0;
    __syncthreads();
    const int n_stay = block_scan(s.stay, S, s.scan_tmp);
    const int S_new = T + n_stay;
    if (S_new > NC) {
      if (t == 0) atomicOr(err, kErrNodeCap);
      if (t == 0) oct_count[img * L + l] = 0;
      return;  // uniform
    }

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
      const int n = kn[k];
      const int r = s.rank[n];
      if (r < 0) {
        kn[k] = T + s.stay[n];
      } else {
        const int x = kd[k] & 0xfff, y = (kd[k] >> 12) & 0xfff;
        const int q = (x < s.mx[n] ? 0 : 1) + (y < s.my[n] ? 0 : 2);
        kn[k] = s.cpos[4 * n + q];
      }
    }
    // expandable children in push order = positions T-1, T-2, ..., 0
    for (int i = t; i < T; i += kOctThreads) s.pc[i] = s.tmp2[T - 1 - i];
    __syncthreads();
    const int e = block_scan(s.pc, T, s.scan_tmp);
    for (int i = t; i < T; i += kOctThreads)
      if (s.tmp2[T - 1 - i]) s.exp_list[s.pc[i]] = T - 1 - i;
    for (int i = t; i < S_new; i += kOctThreads) {
      s.x0[i] = s.nx0[i];
      s.y0[i] = s.ny0[i];
      s.x1[i] = s.nx1[i];
      s.y1[i] = s.ny1[i];
      s.cnt[i] = s.ncnt[i];
    }
    __syncthreads();

    const int S_prev = S;
    S = S_new;
    n_exp = e;
    if (S >= N || S == S_prev) {
      finished = true;
    } else if (phase == 1 && S + 3 * e > N) {
      phase = 2;
    }
  }

  // ---- best response per node, first in to_dist order on ties
  for (int i = t; i < S; i += kOctThreads) s.best[i] = 0ull;
  __syncthreads();
  for (int k = t; k < K; k += kOctThreads) {
    const unsigned long long v =
        ((unsigned long long)(kd[k] >> 24) << 32) | (unsigned long long)(0xffffffffu - (uint32_t)k);
    atomicMax(&s.best[kn[k]], v);
  }
  __syncthreads();
  const int n_out = min(S, g.out_cap);
  for (int i = t; i < n_out; i += kOctThreads) {
    const uint32_t k = 0xffffffffu - (uint32_t)(s.best[i] & 0xffffffffull);
    out[i] = kd[k];
  }
  if (t == 0) {
    oct_count[img * L + l] = n_out;
    if (S > g.out_cap) atomicOr(err, kErrOutCap);
  }
}

// --------------------------------------------------------------------------
// k_describe: one wave per octree output slot.  IC_Angle on the raw level
// (integer moments over the 31-px circular patch, fastAtan2), then 256
// steered-BRIEF tests on the blurred level; test i is lane i%64 of ballot
// i/64, so the 4 ballots are the 32 descriptor bytes, LSB-first as
// ComputeOrbDescriptor packs them.
// --------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_describe(const PlanHeader* __restrict__ P, ImgSrc src,
                                                  const uint8_t* __restrict__ pyr,
                                                  const uint8_t* __restrict__ blur,
                                                  const uint32_t* __restrict__ oct_out,
                                                  const int* __restrict__ oct_count,
                                                  float* __restrict__ angle_out,
                                                  uint64_t* __restrict__ desc_out, int n_img) {
  const int lane = threadIdx.x & 63;
  const long gidx = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (gidx >= (long)n_img * P->kp_slots) return;  // wave-uniform
  const int img = (int)(gidx / P->kp_slots);
  const int slot = (int)(gidx - (long)img * P->kp_slots);
  int l = 0;
  while (l + 1 < P->levels && slot >= P->lev[l + 1].out_off) ++l;
  const LevelGeom& g = P->lev[l];
  const int idx = slot - g.out_off;
  if (idx >= oct_count[img * P->levels + l]) return;  // wave-uniform
  const uint32_t kp = oct_out[(size_t)img * P->kp_slots + slot];
  const int cx = (int)(kp & 0xfff) + kFastBorder, cy = (int)((kp >> 12) & 0xfff) + kFastBorder;

  // IC_Angle: lanes 0..61 -> (column u, half), rows -15..0 / 1..15.
  int sp;
  const uint8_t* img0 = level_plane(P, src, pyr, img, l, sp);
  int m10 = 0, m01 = 0;
  if (lane < 62) {
    const int u = lane % 31 - 15, half = lane / 31;
    const int au = u < 0 ? -u : u;
    const int vb = half ? 1 : -15, ve = half ? 15 : 0;
    for (int v = vb; v <= ve; ++v) {
      const int av = v < 0 ? -v : v;
      if (au <= P->umax[av]) {
        const int val = img0[(size_t)(cy + v) * sp + cx + u];
        m10 += u * val;
        m01 += v * val;
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    m10 += __shfl_xor(m10, o, 64);
    m01 += __shfl_xor(m01, o, 64);
  }
  const float angle = dev_fast_atan2((float)m01, (float)m10);

  const float ang = angle * (float)(3.14159265358979323846 / 180.0);
  const float a = dev_cosf(ang), b = dev_sinf(ang);
  const uint8_t* B = blur + (size_t)img * P->blur_bytes + g.blur_off;
  const uint8_t* ctr = B + (size_t)cy * g.w + cx;
  const int step = g.w;
  uint64_t words[4];
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const int8_t* pt = c_pattern + 4 * (64 * w + lane);
    const float x0 = pt[0], y0 = pt[1], x1 = pt[2], y1 = pt[3];
    const int r0 = dev_round(__builtin_fmaf(x0, b, y0 * a));
    const int q0 = dev_round(__builtin_fmaf(x0, a, -(y0 * b)));
    const int r1 = dev_round(__builtin_fmaf(x1, b, y1 * a));
    const int q1 = dev_round(__builtin_fmaf(x1, a, -(y1 * b)));
    const int t0 = ctr[r0 * step + q0], t1 = ctr[r1 * step + q1];
    words[w] = __ballot(t0 < t1);
  }
  const size_t o = (size_t)img * P->kp_slots + slot;
  if (lane < 4) desc_out[o * 4 + lane] = words[lane];
  if (lane == 0) angle_out[o] = angle;
}

// --------------------------------------------------------------------------
// k_assemble: operator() tail (orb_extractor.cc:1033-1090) for one image:
// level order, node order inside a level; pt scaled to level 0 (one float
// multiply, level 0 untouched); points with lapping[0] <= x <= lapping[1] go
// to the back in reverse order (stereo), the rest to the front (mono).
// --------------------------------------------------------------------------
struct KeyPointOut {
  float x, y, size, angle, response;
  int octave, class_id;
};

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
  __shared__ int flags[4096];
  __shared__ int scan_tmp[kOctThreads + 1];
  const int img = blockIdx.x, t = threadIdx.x, L = P->levels;
  if (t == 0) {
    int acc = 0;
    for (int l = 0; l < L; ++l) {
      lvl_base[l] = acc;
      acc += oct_count[img * L + l];
    }
    lvl_base[L] = acc;
  }
  __syncthreads();
  const int n = lvl_base[L];
  if (n > 4096 || n > cap) {
    if (t == 0) {
      n_out[img] = n;
      mono_out[img] = -1;
      atomicOr(err, kErrKpCap);
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
  for (int gi = t; gi < n; gi += 256) {
    float x, y;
    int l, slot;
    xy_of(gi, x, y, l, slot);
    flags[gi] = (x >= (float)lap0 && x <= (float)lap1) ? 1 : 0;  // stereo
  }
  __syncthreads();
  const int n_stereo = block_scan(flags, n, scan_tmp);
  for (int gi = t; gi < n; gi += 256) {
    float x, y;
    int l, slot;
    xy_of(gi, x, y, l, slot);
    const bool st = (x >= (float)lap0 && x <= (float)lap1);
    const int before_st = flags[gi];
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
    od[0] = d[0];
    od[1] = d[1];
    od[2] = d[2];
    od[3] = d[3];
  }
  if (t == 0) {
    n_out[img] = n;
    mono_out[img] = n - n_stereo;
  }
}

}  // namespace orbgpu

// ==========================================================================
// Host launchers (same translation unit as the kernels).
// ==========================================================================
#include "orb_launch.h"

namespace orbgpu {

hipError_t launch_extract(const ExtractLaunch& a, hipStream_t st) {
  const PlanHeader& H = *a.host_plan;
  ImgSrc src{a.imgs, a.image_pitch, a.stride};
  const int n = a.n_images;
  auto mark = [&](int i) {
    if (a.events) (void)hipEventRecord(a.events[i], st);
  };
  mark(0);
  for (int l = 1; l < H.levels; ++l) {
    const LevelGeom& g = H.lev[l];
    dim3 grid((g.w + 255) / 256, (g.h + 3) / 4, n), block(64, 4);
    hipLaunchKernelGGL(k_resize, grid, block, 0, st, a.plan, a.rs_tab, src, a.pyr, l);
  }
  mark(1);
  hipLaunchKernelGGL(k_blur, dim3(n * H.blur_tiles), dim3(256), 0, st, a.plan, src,
                     (const uint8_t*)a.pyr, a.blur);
  mark(2);
  hipLaunchKernelGGL(k_fast_cells, dim3(n * H.n_cells), dim3(64), 2 * H.max_roi, st, a.plan,
                     a.cells, src, (const uint8_t*)a.pyr, a.slots, a.cell_count);
  mark(3);
  hipLaunchKernelGGL(k_octree, dim3(n * H.levels), dim3(kOctThreads), a.octree_lds, st, a.plan,
                     a.cells, (const uint32_t*)a.slots, (const int*)a.cell_count, a.dense, a.knode,
                     a.oct_out, a.oct_count, a.err);
  mark(4);
  const long waves = (long)n * H.kp_slots;
  hipLaunchKernelGGL(k_describe, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st, a.plan, src,
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

hipError_t set_octree_lds_limit(size_t bytes) {
  return hipFuncSetAttribute((const void*)k_octree, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)bytes);
}

}  // namespace orbgpu
