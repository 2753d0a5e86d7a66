// Host planner: everything the reference derives from (params, image size)
// -- scale tables, level sizes, resize taps, the FAST cell grid, octree roots,
// buffer layout -- computed once per geometry with the reference's float
// arithmetic (compiled -ffp-contract=off).
#include "orb_plan_host.h"
#include "orb_launch.h"

#include <algorithm>
#include <cmath>

namespace orbgpu {

namespace {
inline int cv_round(float v) { return (int)std::lrintf(v); }
inline short sat_short(float v) {
  return (short)std::min(std::max(cv_round(v), -32768), 32767);
}
}  // namespace

void scale_tables(const orbgpu_orb_params& p, std::vector<float>& scale, std::vector<float>& inv,
                  std::vector<float>& s2, std::vector<float>& inv_s2,
                  std::vector<int>& feats_per_level) {
  const int L = p.num_levels;
  const double sf = p.scale_factor;  // float member widened, orb_extractor.h:91
  scale.assign(L, 1.0f);
  s2.assign(L, 1.0f);
  for (int i = 1; i < L; ++i) {  // orb_extractor.cc:418-421
    scale[i] = (float)(scale[i - 1] * sf);
    s2[i] = scale[i] * scale[i];
  }
  inv.resize(L);
  inv_s2.resize(L);
  for (int i = 0; i < L; ++i) {  // :423-428
    inv[i] = 1.0f / scale[i];
    inv_s2[i] = 1.0f / s2[i];
  }
  feats_per_level.assign(L, 0);  // :432-444
  const float factor = (float)(1.0f / sf);
  float per = (float)p.num_features * (1 - factor) /
              (1 - (float)std::pow((double)factor, (double)L));
  int sum = 0;
  for (int l = 0; l < L - 1; ++l) {
    feats_per_level[l] = cv_round(per);
    sum += feats_per_level[l];
    per *= factor;
  }
  feats_per_level[L - 1] = std::max(p.num_features - sum, 0);
}

bool make_plan(const orbgpu_orb_params& p, int W, int H, HostPlan& out, std::string& why,
               int resize_rounding, int octree_nodes) {
  const int L = p.num_levels;
  if (L < 1 || L > kMaxLevels) return why = "num_levels out of range", false;
  if (!(p.scale_factor > 1.0f)) return why = "scale_factor must be > 1", false;
  if (W <= 0 || H <= 0 || W > 4096 || H > 4096) return why = "image size out of range", false;
  PlanHeader& P = out.hdr;
  P = PlanHeader{};
  P.width = W;
  P.height = H;
  P.levels = L;
  P.ini_th = std::min(std::max(p.ini_th_fast, 0), 255);
  P.min_th = std::min(std::max(p.min_th_fast, 0), 255);
  scale_tables(p, out.scale, out.inv_scale, out.sigma2, out.inv_sigma2, out.feats_per_level);

  // umax (:452-464)
  {
    int umax[16] = {0};
    const float r2 = 15.0f * std::sqrt(2.f) / 2;
    const int vmax = (int)std::floor(r2 + 1), vmin = (int)std::ceil(r2);
    for (int v = 0; v <= vmax; ++v) umax[v] = (int)std::lrint(std::sqrt(225.0 - v * v));
    for (int v = 15, v0 = 0; v >= vmin; --v) {
      while (umax[v0] == umax[v0 + 1]) ++v0;
      umax[v] = v0;
      ++v0;
    }
    std::copy(umax, umax + 16, P.umax);
  }

  out.cells.clear();
  out.rs_tab.clear();
  int pyr = 0, blur = 0, slots = 0, kps = 0, quads = 0, tiles = 0, max_roi = 0, node_cap = 64, rs_lds = 0;
  int max_roi_lds = 0, need_pitch = 0;
  for (int l = 0; l < L; ++l) {
    LevelGeom& g = P.lev[l];
    g.w = cv_round((float)W * out.inv_scale[l]);  // :1096
    g.h = cv_round((float)H * out.inv_scale[l]);
    g.scale = out.scale[l];
    g.inv_scale = out.inv_scale[l];
    g.patch_size = (float)(int)(kPatchSize * out.scale[l]);
    if (g.w - 2 * kFastBorder < 35 || g.h - 2 * kFastBorder < 35)
      return why = "pyramid level too small for the FAST grid", false;
    g.pitch = (g.w + kLevelAlign - 1) / kLevelAlign * kLevelAlign;
    g.pyr_off = l == 0 ? -1 : pyr;
    if (l > 0) pyr += g.pitch * g.h;
    g.blur_off = blur;
    blur += g.pitch * g.h;
    g.blur_tile_begin = tiles;
    g.tiles_y = (g.h + kBlurTileH - 1) / kBlurTileH;
    {
      const int fx = g.w / kBlurTileW, tw = g.w - fx * kBlurTileW, nl = (tw + 3) / 4;
#ifndef ORB_BLUR_TAIL
#define ORB_BLUR_TAIL 1  // A/B build switch: 0 = every tail is one more tile column
#endif
      if (ORB_BLUR_TAIL && tw > 0 && nl <= 32) {  // >= 2 strips a wave: a strip path
        g.tiles_x = fx;
        g.tail_nl = nl;
        g.tail_s = 64 / nl;
        const int waves = (g.h + 32 * g.tail_s - 1) / (32 * g.tail_s);
        g.tail_blocks = (waves + 3) / 4;
      } else {
        g.tiles_x = fx + (tw > 0);
        g.tail_nl = g.tail_s = g.tail_blocks = 0;
      }
    }
    tiles += g.tiles_x * g.tiles_y + g.tail_blocks;

    // resize taps for level l from level l-1 (cv::resize INTER_LINEAR)
    if (l > 0) {
      const LevelGeom& s = P.lev[l - 1];
      const double scale_x = 1. / ((double)g.w / s.w), scale_y = 1. / ((double)g.h / s.h);
      g.rs_x = (int)out.rs_tab.size();
      g.xmax = g.w;
      for (int dx = 0; dx < g.w; ++dx) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = (int)std::floor(fx);
        fx -= sx;
        if (sx < 0) fx = 0.f, sx = 0;
        if (sx + 1 >= s.w) {
          g.xmax = std::min(g.xmax, dx);
          if (sx >= s.w - 1) fx = 0.f, sx = s.w - 1;
        }
        short a0 = sat_short((1.f - fx) * 2048), a1 = sat_short(fx * 2048);
        if (dx >= g.xmax) a0 = 2048, a1 = 0;  // single-tap columns: S[sx] * ONE
        out.rs_tab.push_back(sx);
        out.rs_tab.push_back((int)(uint16_t)a0 | ((int)(uint16_t)a1 << 16));
      }
      g.rs_y = (int)out.rs_tab.size();
      for (int dy = 0; dy < g.h; ++dy) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        int sy = (int)std::floor(fy);
        fy -= sy;
        const short b0 = sat_short((1.f - fy) * 2048), b1 = sat_short(fy * 2048);
        const int r0 = std::min(std::max(sy, 0), s.h - 1), r1 = std::min(std::max(sy + 1, 0), s.h - 1);
        out.rs_tab.push_back(r0 | (r1 << 16));
        out.rs_tab.push_back((int)(uint16_t)b0 | ((int)(uint16_t)b1 << 16));
      }
      // largest source window of a kResizeTileW x kResizeTileH output tile
      g.rs_tiles_x = (g.w + kResizeTileW - 1) / kResizeTileW;
      g.rs_tiles_y = (g.h + kResizeTileH - 1) / kResizeTileH;
      // a narrow right-hand tail goes to resize_tail (lane = output row)
      g.rs_tail_x0 = 0;
      g.rs_tail_blocks = 0;
      {
#ifndef ORB_RS_TAIL
#define ORB_RS_TAIL 1  // A/B build switch: 0 = the tiles cover every column
#endif
        const int fx = g.w / kResizeTileW, ng = (g.w - fx * kResizeTileW + 3) / 4;
        if (ORB_RS_TAIL && ng > 0 && ng <= kRsTailGroups) {
          g.rs_tiles_x = fx;
          g.rs_tail_x0 = fx * kResizeTileW;
          g.rs_tail_blocks = (g.h + 63) / 64;
        }
      }
      g.rs_src_cols = 0;
      g.rs_src_rows = 0;
      const int* tab = out.rs_tab.data();
      for (int tx = 0; tx < g.rs_tiles_x; ++tx) {
        const int xa = tx * kResizeTileW, xb = std::min(xa + kResizeTileW, g.w) - 1;
        const int c0 = tab[g.rs_x + 2 * xa] & ~15;
        const int c1 = std::min(tab[g.rs_x + 2 * xb] + 1, s.w - 1) | 15;  // same as k_resize
        g.rs_src_cols = std::max(g.rs_src_cols, c1 - c0 + 1);
      }
      for (int ty = 0; ty < g.rs_tiles_y; ++ty) {
        const int ya = ty * kResizeTileH, yb = std::min(ya + kResizeTileH, g.h) - 1;
        const int r0 = tab[g.rs_y + 2 * ya] & 0xffff, r1 = tab[g.rs_y + 2 * yb] >> 16;
        g.rs_src_rows = std::max(g.rs_src_rows, r1 - r0 + 1);
      }
      if (g.rs_tail_blocks) {  // resize_tail's windows: the tail columns x 64 output rows
        const int c0 = tab[g.rs_x + 2 * g.rs_tail_x0] & ~15;
        const int c1 = std::min(tab[g.rs_x + 2 * (g.w - 1)] + 1, s.w - 1) | 15;
        for (int b = 0; b < g.rs_tail_blocks; ++b) {
          const int ya = 64 * b, yb = std::min(ya + 63, g.h - 1);
          const int r0 = tab[g.rs_y + 2 * ya] & 0xffff, r1 = tab[g.rs_y + 2 * yb] >> 16;
          const int nq = (c1 - c0 + 1) / 16;
          if ((long long)(r1 - r0 + 1) * nq * nq >= (1 << 19)) return why = "scale factor too large for the resize tail", false;
          rs_lds = std::max(rs_lds, (c1 - c0 + 1) * (r1 - r0 + 1) + 16);
        }
      }
      rs_lds = std::max(rs_lds, g.rs_src_cols * g.rs_src_rows + 16);  // + k_resize's 3-dword overreach
      // k_resize splits a staging index i < rows x nq by the multiply-shift
      // (i * ceil(2^19 / nq)) >> 19, exact while rows x nq^2 < 2^19
      {
        const long long nq = g.rs_src_cols / 16;
        if ((long long)g.rs_src_rows * nq * nq >= (1 << 19)) return why = "scale factor too large for the resize tile", false;
      }
      int x = 0;
      for (; x <= g.w - 16; x += 16) {
      }
      g.vec16_end = x;
      for (; x < g.w - 8; x += 8) {
      }
      g.vec8_end = x;
      if (resize_rounding == ORBGPU_RESIZE_SCALAR) g.vec16_end = g.vec8_end = 0;
    }

    // FAST cell grid (:748-825)
    const int min_b = kFastBorder;
    const int max_bx = g.w - kEdgeThreshold + 3, max_by = g.h - kEdgeThreshold + 3;
    const float width = (float)(max_bx - min_b), height = (float)(max_by - min_b);
    const int ncols = (int)(width / 35.f), nrows = (int)(height / 35.f);
    const int wc = (int)std::ceil(width / ncols), hc = (int)std::ceil(height / nrows);
    g.cell_begin = (int)out.cells.size();
    g.slot_begin = slots;
    for (int i = 0; i < nrows; ++i) {
      const float y0 = (float)(min_b + i * hc);
      float y1 = y0 + hc + 6;
      if (y0 >= max_by - 3) continue;
      if (y1 > max_by) y1 = (float)max_by;
      for (int j = 0; j < ncols; ++j) {
        const float x0 = (float)(min_b + j * wc);
        float x1 = x0 + wc + 6;
        if (x0 >= max_bx - 3) continue;
        if (x1 > max_bx) x1 = (float)max_bx;
        Cell c;
        c.level = l;
        c.x0 = (int)x0;
        c.y0 = (int)y0;
        c.cols = (int)x1 - c.x0;
        c.rows = (int)y1 - c.y0;
        const int dw = c.cols - 6, dh = c.rows - 6;
        c.slot_off = slots;
        c.slot_cap = (dw > 0 && dh > 0) ? ((dw + 1) / 2) * ((dh + 1) / 2) : 0;
        slots += c.slot_cap;
        max_roi = std::max(max_roi, c.cols * c.rows);
        max_roi_lds = std::max(max_roi_lds, fast_cell_lds_bytes(c.cols, c.rows));
        // the ROI row (lead <= 3 + cols) and the score-map row (dw + 2) in one pitch
        need_pitch = std::max(need_pitch, std::max(c.cols + 3, dw + 2));
        if (dw > 127 || dh > 255)  // k_fast_cells survivor encoding r << 7 | q
          return why = "FAST cell too large", false;
        out.cells.push_back(c);
      }
    }
    g.cell_end = (int)out.cells.size();
    g.slot_count = slots - g.slot_begin;

    // octree (:546-560)
    g.budget = out.feats_per_level[l];
    g.rel_w = max_bx - min_b;
    g.rel_h = max_by - min_b;
    g.n_roots = (int)std::round((float)g.rel_w / g.rel_h);
    if (g.n_roots < 1) return why = "image too tall for the octree roots", false;
    g.root_w = (float)g.rel_w / g.n_roots;
    g.out_off = kps;
    g.out_cap = std::max(g.budget + 3, 4 * g.n_roots);
    kps += g.out_cap;
    g.quad_off = quads;
    quads += (g.out_cap + 3) / 4;
    node_cap = std::max({node_cap, g.out_cap, g.cell_end - g.cell_begin, g.n_roots});
  }
  P.n_cells = (int)out.cells.size();
  P.pyr_bytes = (pyr + 255) & ~255;
  P.blur_bytes = (blur + 255) & ~255;
  P.slots = slots;
  P.kp_slots = kps;
  P.kp_quads = quads;
  P.node_cap = (node_cap + 63) & ~63;
  P.blur_tiles = tiles;
  P.max_roi = (max_roi + 15) & ~15;
  P.fast_pitch = 0;
  for (int pt = 48; pt <= 64; pt += 4)
    if (need_pitch <= pt) {
      P.fast_pitch = pt;
      break;
    }
  if (P.fast_pitch) {
    max_roi_lds = 0;
    for (const Cell& c : out.cells) max_roi_lds = std::max(max_roi_lds, fast_cell_lds_bytes_pitch(c.cols, c.rows, P.fast_pitch));
  }
  P.max_roi_lds = (max_roi_lds + 15) & ~15;
  P.rs_lds = (rs_lds + 15) & ~15;
  if (P.rs_lds > 160 * 1024) return why = "scale factor too large for the resize tile", false;
  if (P.max_roi_lds > 64 * 1024) return why = "FAST cell too large", false;
  // octree storage: the node arrays and kOctreeLdsCand candidates in LDS;
  // fewer candidates in LDS (the rest in HBM, as beyond kOctreeLdsCand) when
  // the nodes leave less room; the node arrays in HBM (k_octree<true>) when
  // they alone do not fit -- any num_features the reference accepts
  // (orb_extractor.cc:432-444 bounds no level's budget).
  {
    const size_t fixed = octree_fixed_lds_bytes(), nodes = oct_node_bytes(P.node_cap);
    if (octree_nodes != ORBGPU_OCTREE_NODES_HBM && nodes + fixed + (size_t)kOctreeLdsCand * 8 <= kOctreeLdsMax) {
      P.oct_hbm_nodes = 0;
      P.oct_kcap = kOctreeLdsCand;
    } else if (octree_nodes != ORBGPU_OCTREE_NODES_HBM && nodes + fixed + 64 * 8 <= kOctreeLdsMax) {
      P.oct_hbm_nodes = 0;
      P.oct_kcap = (int)((kOctreeLdsMax - nodes - fixed) / 8) & ~63;
    } else {
      P.oct_hbm_nodes = 1;
      P.oct_kcap = kOctreeLdsCand;
    }
  }
  return true;
}

// LDS of one FAST cell wave (k_fast_cells): ROI staged with 4-aligned rows
// (+3 lead bytes), a byte score map of the detection area with a zero border
// the u16 survivors of 64 group entries and a u32 list of the 8-pixel
// groups holding one.
#ifndef ORB_FAST_SV_FULL
#define ORB_FAST_SV_FULL 0  // A/B build switch, as in orb_kernels.hip
#endif
int fast_cell_lds_bytes(int cols, int rows) {
  const int ls = (cols + 3 + 3) & ~3;
  const int dw = std::max(cols - 6, 0), dh = std::max(rows - 6, 0);
  const int nd = dw * dh, ng = ((dw + 7) >> 3) * dh;
  const int nsc = std::max(cols - 4, 0) * std::max(rows - 4, 0);
  const int sv = ORB_FAST_SV_FULL ? (2 * nd + 15) & ~15 : 2 * (512 + 64);  // u16 survivors (kFastSvChunk + kFastSvCarry)
  return ((ls * rows + 15) & ~15) + ((nsc + 15) & ~15) + sv + 4 * ng + 16;
}

// The same with the plan's fixed pitch for the ROI and the score-map rows
// (k_fast_cells<pitch>), plus slack for the compass windows' reads past a
// row's last group.
int fast_cell_lds_bytes_pitch(int cols, int rows, int pitch) {
  const int dw = std::max(cols - 6, 0), dh = std::max(rows - 6, 0);
  const int nd = dw * dh, ng = ((dw + 7) >> 3) * dh;
  const int sv = ORB_FAST_SV_FULL ? (2 * nd + 15) & ~15 : 2 * (512 + 64);
  return ((pitch * rows + 15) & ~15) + ((pitch * (dh + 2) + 15) & ~15) + sv + 4 * ng + 16 + 16;
}

// k_octree's LDS besides the nodes: the scan scratch (256 + 1 ints) and 16
// block scalars.
size_t octree_fixed_lds_bytes() { return (256 + 1) * 4 + 16 * 4; }

size_t octree_lds_bytes(const PlanHeader& P) {
  const size_t cand = (size_t)P.oct_kcap * 8;
  return (P.oct_hbm_nodes ? 0 : oct_node_bytes(P.node_cap)) + octree_fixed_lds_bytes() + cand;
}


// The single-image dataflow launch's items in ticket order (orb_launch.h):
// the image copy, then level 0's FAST cells, level 1's resize and level 0's
// octree (the longest chain: FAST -> DistributeOctTree of level 0), level 0's
// blur; per level l >= 1 the next level's resize, its FAST cells, octree and
// blur; the describe items last, level 0's at the very end (its octree
// finishes last).
void make_df_items(const PlanHeader& P, int img_bytes, DfPlan& df, std::vector<uint32_t>& items) {
  df = DfPlan{};
  items.clear();
  const int L = P.levels;
  auto push = [&](int type, int l, int n) {
    for (int i = 0; i < n; ++i) items.push_back((uint32_t)type | ((uint32_t)l << 4) | ((uint32_t)i << 8));
  };
  df.img_bytes = img_bytes;
  df.n_bands = (img_bytes + kDfBandBytes - 1) / kDfBandBytes;
  for (int l = 0; l < L; ++l) {
    const LevelGeom& g = P.lev[l];
    df.units[l] = l ? g.rs_tiles_x * g.rs_tiles_y + g.rs_tail_blocks : 0;
    df.fast_items[l] = (g.cell_end - g.cell_begin + 3) / 4;
    df.blur_items[l] = (l + 1 < L ? P.lev[l + 1].blur_tile_begin : P.blur_tiles) - g.blur_tile_begin;
  }
  push(kDfCopy, 0, df.n_bands);
  push(kDfFast, 0, df.fast_items[0]);
  if (L > 1) push(kDfResize, 1, df.units[1]);
  push(kDfOctree, 0, 1);
  push(kDfBlur, 0, df.blur_items[0]);
  for (int l = 1; l < L; ++l) {
    if (l + 1 < L) push(kDfResize, l + 1, df.units[l + 1]);
    push(kDfFast, l, df.fast_items[l]);
    push(kDfOctree, l, 1);
    push(kDfBlur, l, df.blur_items[l]);
  }
  for (int l = L - 1; l >= 0; --l) {
    const int n = (P.lev[l].out_cap + 3) / 4;
    push(kDfDescribe, l, n);
    df.desc_items += n;
  }
  // last: the host mirror, level by level as each level's descriptors land
  // (no lapping band; with one, the last describe item assembles)
  push(kDfMirror, 0, 1);
  df.n_items = (int)items.size();
}

}  // namespace orbgpu
