// Geometry plan shared by the host planner (orb_plan.cpp) and the gfx950
// kernels (orb_kernels.hip).  Everything the reference recomputes per call
// from the image size (orb_extractor.cc:407-465, 744-849, 1093-1117) is
// computed once per (params, width, height) and lives in one device buffer.
#pragma once
#include <stddef.h>
#include <stdint.h>
#include <hip/hip_runtime.h>

namespace orbgpu {

constexpr int kMaxLevels = 16;
constexpr int kEdgeThreshold = 19;  // orb_extractor.cc:74
constexpr int kFastBorder = kEdgeThreshold - 3;  // min_border_x/y (:751)
constexpr int kPatchSize = 31;      // :72

struct LevelGeom {
  int w, h;          // level size: cvRound(W * inv_scale), cvRound(H * inv_scale)  (:1096)
  int pitch;         // row pitch of the pyramid / blurred planes (w rounded up to 16)
  int pyr_off;       // byte offset of this level in an image's pyramid block (levels >= 1)
  int blur_off;      // byte offset in an image's blurred block (all levels)
  float scale;       // scale_factors_[l]
  float inv_scale;   // inv_scale_factors_[l]
  float patch_size;  // (float)(int)(31 * scale)                                     (:834)
  // resize tables (levels >= 1), offsets into Plan::rs_tab
  int rs_x, rs_y;    // xofs|alpha pairs, yofs|beta pairs
  int xmax;          // first dst column whose right neighbour is out of range
  int rs_tiles_x, rs_tiles_y;  // resize tiles (kResizeTileW x kResizeTileH outputs)
  int rs_src_cols, rs_src_rows;  // largest source window of a tile (LDS staging)
  int rs_tail_x0;      // first column of the tail path (resize_tail), when rs_tail_blocks > 0
  int rs_tail_blocks;  // 64-row blocks of the tail path (0: the tiles cover every column)
  int vec16_end;     // VResizeLinearVec_32s8u: 16-lane blocks end here
  int vec8_end;      //                          8-lane blocks end here
  // FAST grid (:748-825)
  int cell_begin, cell_end;
  int slot_begin;    // first candidate slot of this level in an image's slot block
  int slot_count;    // sum of cell capacities of this level
  // octree (:542-742)
  int budget;        // num_feats_per_lev_[l]
  int n_roots;       // round((max_x - min_x) / (max_y - min_y))
  float root_w;      // (float)(max_x - min_x) / n_roots
  int rel_w, rel_h;  // max_x - min_x, max_y - min_y
  int out_off;       // first output slot of this level in an image's keypoint block
  int out_cap;       // node-count bound: max(budget + 3, 4 * n_roots)
  int quad_off;      // first k_describe wave (4 output slots each) of this level in an image
  // blur tiling (kBlurTileW x kBlurTileH outputs per 256-thread block): tiles_x
  // x tiles_y full-width tiles, then the tail columns [tiles_x * 256, w) when
  // they need at most 32 lanes: packed as tail_s strips of tail_nl lanes x 32
  // rows per wave (tail_blocks blocks of 4 such waves); a wider tail is one
  // more tile column (tail_blocks = 0)
  int blur_tile_begin, tiles_x, tiles_y;
  int tail_nl, tail_s, tail_blocks;
};

struct Cell {
  int level;
  int x0, y0;       // ROI origin in level pixels
  int cols, rows;   // ROI size (detection area is the ROI minus 3 px on each side)
  int slot_off;     // first candidate slot in the image's slot block
  int slot_cap;     // ceil(dw/2) * ceil(dh/2): bound for 3x3 strict maxima
};

struct PlanHeader {
  int width, height, levels;
  int ini_th, min_th;
  int n_cells;
  int pyr_bytes;    // per image, levels 1..L-1
  int blur_bytes;   // per image, all levels
  int slots;        // per image candidate slots
  int kp_slots;     // per image octree-output slots
  int kp_quads;     // per image k_describe waves: sum over levels of ceil(out_cap / 4)
  int node_cap;     // node capacity of the octree kernel (per (image, level) block)
  int oct_kcap;     // octree candidates held in LDS (the rest in HBM)
  int oct_hbm_nodes;  // 1: the node arrays live in HBM (k_octree<true>), 0: in LDS
  int blur_tiles;   // per image
  int max_roi;      // largest cell ROI (bytes)
  int max_roi_lds;  // LDS bytes of one FAST cell (staged ROI + score map + lists)
  int fast_pitch;   // 48..64: the LDS row pitch of every FAST cell (k_fast_cells<pitch>); 0 = per cell
  int rs_lds;       // LDS bytes of one resize tile
  int umax[16];     // circular patch extents (:452-464)
  LevelGeom lev[kMaxLevels];
};

constexpr int kBlurTileW = 256, kBlurTileH = 128;   // 64 threads x 4 cols, 4 waves x 32 rows
constexpr int kResizeTileW = 256, kResizeTileH = 32;  // 4 waves x 8 rows, 64 lanes x 4 px
constexpr int kRsTailGroups = 48;  // widest tail (4-column groups) taken by resize_tail
constexpr int kLevelAlign = 16;
#ifndef ORB_OCT_KCAP
#define ORB_OCT_KCAP 2048  // A/B: 1024 -> 0.099 ms per 256 images isolated (0.114), bench flat, single-image latency worse
#endif
constexpr int kOctreeLdsCand = ORB_OCT_KCAP;  // octree candidates per (image, level) kept in LDS (rest in HBM)
constexpr int kOctreeLdsMax = 160 * 1024;  // LDS of one gfx950 workgroup

// Bytes of the octree's node arrays for node capacity nc: the 64-bit best
// response, 17 per-node ints and 8 per-node child ints (k_octree's carve).
__host__ __device__ constexpr size_t oct_node_bytes(int nc) { return (size_t)nc * (8 + 17 * 4 + 8 * 4); }

}  // namespace orbgpu
