// Host-side planner interface (see orb_plan.cpp).
#pragma once
#include <string>
#include <vector>

#include "../../include/orbgpu.h"
#include "orb_plan.h"

namespace orbgpu {

struct HostPlan {
  PlanHeader hdr;
  std::vector<Cell> cells;
  std::vector<int> rs_tab;
  std::vector<float> scale, inv_scale, sigma2, inv_sigma2;
  std::vector<int> feats_per_level;
};

void scale_tables(const orbgpu_orb_params& p, std::vector<float>& scale, std::vector<float>& inv,
                  std::vector<float>& s2, std::vector<float>& inv_s2,
                  std::vector<int>& feats_per_level);
// resize_rounding: ORBGPU_RESIZE_SSE / ORBGPU_RESIZE_SCALAR (include/orbgpu.h)
// octree_nodes: ORBGPU_OCTREE_NODES_AUTO (LDS whenever the node arrays fit) or
// ORBGPU_OCTREE_NODES_HBM (always HBM: the test path for the large plans)
bool make_plan(const orbgpu_orb_params& p, int width, int height, HostPlan& out, std::string& why,
               int resize_rounding = 0, int octree_nodes = 0);
size_t octree_lds_bytes(const PlanHeader& P);
size_t octree_fixed_lds_bytes();
int fast_cell_lds_bytes(int cols, int rows);
int fast_cell_lds_bytes_pitch(int cols, int rows, int pitch);

}  // namespace orbgpu
