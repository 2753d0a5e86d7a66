// C-ABI implementation of the extractor half of include/orbgpu.h.
// Owns the per-handle HIP stream, the geometry plan and the device workspace;
// launches the kernel sequence of orb_kernels.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "../../include/orbgpu.h"
#include "orb_launch.h"
#include "orb_plan_host.h"
#include "stereo_launch.h"

using namespace orbgpu;

namespace {

template <class T>
hipError_t dalloc(T** p, size_t count) {
  *p = nullptr;
  if (count == 0) count = 1;
  return hipMalloc(reinterpret_cast<void**>(p), count * sizeof(T));
}

template <class T>
void dfree(T*& p) {
  if (p) (void)hipFree(p);
  p = nullptr;
}

}  // namespace

struct orbgpu_extractor {
  orbgpu_orb_params params{};
  int device = 0;
  int n_cu = 256;
  hipStream_t stream = nullptr;
  int max_w = 0, max_h = 0, max_images = 0;

  HostPlan plan;
  int plan_w = -1, plan_h = -1;
  int resize_rounding = ORBGPU_RESIZE_SSE;
  int octree_nodes = ORBGPU_OCTREE_NODES_AUTO;
  int pyramid_launch = ORBGPU_PYRAMID_PER_LEVEL;  // orbgpu_extractor_set_pyramid_launch
  hipEvent_t stage_event = nullptr;  // orbgpu_extractor_set_stage_event (batch launches)
  int stage_event_at = -1;
  PlanHeader* d_plan = nullptr;
  Cell* d_cells = nullptr;
  int* d_rs = nullptr;
  size_t cells_cap = 0, rs_cap = 0;

  int ws_images = 0;  // workspace sized for this many images of the plan
  size_t ws_pyr = 0, ws_blur = 0, ws_slots = 0, ws_cells = 0, ws_kp = 0;
  uint8_t *d_pyr = nullptr, *d_blur = nullptr;
  uint32_t *d_slots = nullptr, *d_dense = nullptr, *d_oct_out = nullptr;
  int *d_cell_count = nullptr, *d_knode = nullptr, *d_oct_count = nullptr;
  uint8_t* d_oct_nodes = nullptr;  // octree node arrays of HBM-node plans (per (image, level) block)
  size_t ws_nodes = 0;
  float* d_angle = nullptr;
  uint64_t* d_desc = nullptr;
  int* d_err = nullptr;

  // single-image (host-buffer) path: the outputs as ONE device block
  // [n, mono, err, pad | keypoints (kp_slots x 28, 16-B aligned) | descriptors]
  // mirrored by one pinned block, so the chain ends in a single D2H copy; the
  // pointers below are views into the blocks (d_sout / h_sout own them)
  uint8_t* d_img = nullptr;
  size_t d_img_bytes = 0;
  char* d_sout = nullptr;
  char* h_sout = nullptr;
  size_t sout_bytes = 0;
  orbgpu_keypoint* d_kps = nullptr;
  uint8_t* d_descs = nullptr;
  size_t out_cap = 0;
  int* d_nm = nullptr;     // n, mono, err (the single-image launch's error word)
  int* h_small = nullptr;  // n, mono, err (pinned)
  orbgpu_keypoint* h_kps = nullptr;
  uint8_t* h_descs = nullptr;
  // pinned (host-mapped, fine-grained) staging of the image: the graph's copy
  // or the dataflow launch's copy items read it, the host only memcpys
  uint8_t* h_img = nullptr;
  uint8_t* h_img_dev = nullptr;  // its device view
  size_t h_img_bytes = 0;
  int* h_band = nullptr;          // the dataflow launch's band flags (in the h_img block, after the image)
  const int* h_band_dev = nullptr;
  int df_seq = 0;                 // sequence number of the last dataflow call
  char* h_sout_dev = nullptr;    // device view of h_sout (the dataflow launch mirrors into it)
  // the dataflow launch (k_extract_df): control block, launch record + item list
  int single_mode = ORBGPU_SINGLE_DATAFLOW;
  int* d_df_ctrl = nullptr;
  DfLaunch* d_df_rec = nullptr;  // record, then the items
  size_t df_rec_cap = 0;         // bytes of d_df_rec
  DfLaunch df_launch{};          // what d_df_rec holds
  bool df_valid = false;
  int df_grid = 0;               // ORBGPU_DF_GRID (tools): workers, else the CU count
  unsigned long long* d_df_trace = nullptr;  // ORBGPU_DF_TRACE (tools/df_trace.py): per-ticket timeline
  size_t df_trace_cap = 0;
  hipGraph_t graph = nullptr;
  hipGraphExec_t graph_exec = nullptr;
  ExtractLaunch graph_launch{};  // what graph_exec was captured for
  ExtractLaunch eager_launch{};  // the last launch run eagerly (captured when repeated)
  int graph_wh[2] = {0, 0}, eager_wh[2] = {0, 0};  // plan size of each (grids are baked in)
  bool graph_valid = false, eager_valid = false;
  std::vector<uint8_t> host_pyr;
  bool host_pyr_valid = false;
  int last_w = 0, last_h = 0;

  // stereo matcher scratch (row lists, row ends, window distances) and the
  // host path's device outputs
  uint16_t* d_st_lists = nullptr;
  int *d_st_rowend = nullptr, *d_st_sad = nullptr;
  // host path block [error word, pad x3 | uright x kcap | depth x kcap] on the
  // device and its pinned mirror: one copy back per call
  float* d_st_out = nullptr;
  float* h_st_out = nullptr;      // host-mapped: [error word | uright | depth], then the completion word
  float* h_st_out_dev = nullptr;
  int st_seq = 0;
  size_t st_lists = 0, st_rowend = 0, st_sad = 0, st_out = 0;

  // optional per-stage event profiling of batch calls (a ring of event sets)
  std::vector<hipEvent_t> prof_events;
  int prof_slots = 0, prof_used = 0;
};

namespace {

// Any (re)allocation a captured launch refers to -- device workspace or the
// pinned staging the graph's copies read and write -- retires the captured
// graph and the eager record it was keyed on: a new allocation can come back
// at a freed address, so pointer equality alone cannot prove the graph valid.
void drop_graphs(orbgpu_extractor* h) {
  if (h->graph_exec) (void)hipGraphExecDestroy(h->graph_exec);
  if (h->graph) (void)hipGraphDestroy(h->graph);
  h->graph_exec = nullptr;
  h->graph = nullptr;
  h->graph_valid = false;
  h->eager_valid = false;
  h->df_valid = false;  // the dataflow record names the same buffers
}

// The single-image output blocks for `slots` keypoints (see orbgpu_extractor).
orbgpu_status ensure_single_out(orbgpu_extractor* h, size_t slots) {
  if (slots <= h->out_cap && h->d_sout) return ORBGPU_OK;
  drop_graphs(h);
  const size_t kp_bytes = (slots * sizeof(orbgpu_keypoint) + 15) & ~(size_t)15;
  const size_t bytes = 16 + kp_bytes + slots * 32;
  if (h->d_sout) (void)hipFree(h->d_sout);
  if (h->h_sout) (void)hipHostFree(h->h_sout);
  h->d_sout = h->h_sout = nullptr;
  h->out_cap = 0;
  if (hipMalloc(&h->d_sout, bytes) != hipSuccess ||
      hipHostMalloc(&h->h_sout, bytes, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer(reinterpret_cast<void**>(&h->h_sout_dev), h->h_sout, 0) != hipSuccess)
    return ORBGPU_ERR_NOMEM;
  if (hipMemset(h->d_sout, 0, 16) != hipSuccess) return ORBGPU_ERR_DEVICE;
  h->sout_bytes = bytes;
  h->out_cap = slots;
  h->d_nm = reinterpret_cast<int*>(h->d_sout);
  h->d_kps = reinterpret_cast<orbgpu_keypoint*>(h->d_sout + 16);
  h->d_descs = reinterpret_cast<uint8_t*>(h->d_sout + 16 + kp_bytes);
  h->h_small = reinterpret_cast<int*>(h->h_sout);
  h->h_kps = reinterpret_cast<orbgpu_keypoint*>(h->h_sout + 16);
  h->h_descs = reinterpret_cast<uint8_t*>(h->h_sout + 16 + kp_bytes);
  return ORBGPU_OK;
}

orbgpu_status ensure_plan(orbgpu_extractor* h, int w, int ht) {
  if (h->plan_w == w && h->plan_h == ht) return ORBGPU_OK;
  drop_graphs(h);
  std::string why;
  HostPlan p;
  if (!make_plan(h->params, w, ht, p, why, h->resize_rounding, h->octree_nodes)) return ORBGPU_ERR_INVALID;
  if (p.cells.size() > h->cells_cap) {
    dfree(h->d_cells);
    if (dalloc(&h->d_cells, p.cells.size()) != hipSuccess) return ORBGPU_ERR_NOMEM;
    h->cells_cap = p.cells.size();
  }
  if (p.rs_tab.size() > h->rs_cap) {
    dfree(h->d_rs);
    if (dalloc(&h->d_rs, p.rs_tab.size()) != hipSuccess) return ORBGPU_ERR_NOMEM;
    h->rs_cap = p.rs_tab.size();
  }
  if (hipMemcpyAsync(h->d_plan, &p.hdr, sizeof(PlanHeader), hipMemcpyHostToDevice, h->stream) ||
      hipMemcpyAsync(h->d_cells, p.cells.data(), p.cells.size() * sizeof(Cell),
                     hipMemcpyHostToDevice, h->stream) ||
      hipMemcpyAsync(h->d_rs, p.rs_tab.data(), p.rs_tab.size() * sizeof(int),
                     hipMemcpyHostToDevice, h->stream) ||
      hipStreamSynchronize(h->stream))
    return ORBGPU_ERR_DEVICE;
  // the plan's own LDS needs (the plan checked both against 160 KB; a device
  // with less LDS per workgroup refuses only the plans that need more)
  if (set_lds_limits(octree_lds_bytes(p.hdr), (size_t)p.hdr.rs_lds) != hipSuccess) return ORBGPU_ERR_DEVICE;
  h->plan = std::move(p);
  h->plan_w = w;
  h->plan_h = ht;
  h->ws_images = 0;  // re-check workspace sizes against the new plan
  return ORBGPU_OK;
}

orbgpu_status ensure_workspace(orbgpu_extractor* h, int n) {
  const PlanHeader& P = h->plan.hdr;
  if (h->ws_images >= n) return ORBGPU_OK;
  drop_graphs(h);
  const size_t pyr = (size_t)n * P.pyr_bytes, blur = (size_t)n * P.blur_bytes;
  const size_t slots = (size_t)n * P.slots, cells = (size_t)n * P.n_cells;
  const size_t kp = (size_t)n * P.kp_slots;
  if (pyr > h->ws_pyr) {
    dfree(h->d_pyr);
    if (dalloc(&h->d_pyr, pyr)) return ORBGPU_ERR_NOMEM;
    h->ws_pyr = pyr;
  }
  if (blur > h->ws_blur) {
    dfree(h->d_blur);
    if (dalloc(&h->d_blur, blur)) return ORBGPU_ERR_NOMEM;
    h->ws_blur = blur;
  }
  if (slots > h->ws_slots) {
    dfree(h->d_slots);
    dfree(h->d_dense);
    dfree(h->d_knode);
    if (dalloc(&h->d_slots, slots) || dalloc(&h->d_dense, slots) || dalloc(&h->d_knode, slots))
      return ORBGPU_ERR_NOMEM;
    h->ws_slots = slots;
  }
  if (cells > h->ws_cells) {
    dfree(h->d_cell_count);
    if (dalloc(&h->d_cell_count, cells)) return ORBGPU_ERR_NOMEM;
    h->ws_cells = cells;
  }
  if (P.oct_hbm_nodes) {
    const size_t nodes = (size_t)n * P.levels * oct_node_bytes(P.node_cap);
    if (nodes > h->ws_nodes) {
      dfree(h->d_oct_nodes);
      if (dalloc(&h->d_oct_nodes, nodes)) return ORBGPU_ERR_NOMEM;
      h->ws_nodes = nodes;
    }
  }
  if (kp > h->ws_kp) {
    dfree(h->d_oct_out);
    dfree(h->d_angle);
    dfree(h->d_desc);
    dfree(h->d_oct_count);
    if (dalloc(&h->d_oct_out, kp) || dalloc(&h->d_angle, kp) || dalloc(&h->d_desc, kp * 4) ||
        dalloc(&h->d_oct_count, (size_t)n * kMaxLevels))
      return ORBGPU_ERR_NOMEM;
    h->ws_kp = kp;
  }
  h->ws_images = n;
  return ORBGPU_OK;
}

ExtractLaunch make_launch(orbgpu_extractor* h, const uint8_t* imgs, size_t pitch, int stride,
                          int n, const int lap[2], void* kps, void* descs, int cap, int* d_n,
                          int* d_mono) {
  ExtractLaunch a{};
  a.host_plan = &h->plan.hdr;
  a.plan = h->d_plan;
  a.n_cu = h->n_cu;
  // the resize chain per level (default), or as one launch (k_pyramid, a
  // workgroup per image) -- bit-identical, slower at every batch size
  // measured
  a.pyramid_groups =
      h->pyramid_launch == ORBGPU_PYRAMID_FUSED ? pyramid_groups_for((size_t)h->plan.hdr.rs_lds) : 0;
  a.cells = h->d_cells;
  a.rs_tab = h->d_rs;
  a.imgs = imgs;
  a.image_pitch = pitch;
  a.stride = stride;
  a.n_images = n;
  a.pyr = h->d_pyr;
  a.blur = h->d_blur;
  a.slots = h->d_slots;
  a.cell_count = h->d_cell_count;
  a.dense = h->d_dense;
  a.knode = h->d_knode;
  a.oct_out = h->d_oct_out;
  a.oct_count = h->d_oct_count;
  a.angle = h->d_angle;
  a.desc = h->d_desc;
  a.octree_lds = octree_lds_bytes(h->plan.hdr);
  a.oct_nodes = h->plan.hdr.oct_hbm_nodes ? h->d_oct_nodes : nullptr;
  a.lap0 = lap ? lap[0] : 0;
  a.lap1 = lap ? lap[1] : 0;
  a.kps_out = kps;
  a.desc_out = descs;
  a.cap = cap;
  a.n_out = d_n;
  a.mono_out = d_mono;
  a.err = h->d_err;
  return a;
}

// Row-list entries per frame: a right keypoint spans at most
// 2 * ceil(2 * s_max) + 3 rows (frame.cc:844-849).
int stereo_list_cap(const HostPlan& p, int cap) {
  const float smax = p.scale.back();
  return cap * (2 * (int)std::ceil(2.0f * smax) + 3);
}

orbgpu_status ensure_stereo(orbgpu_extractor* h, int n_frames, int cap) {
  const size_t lists = (size_t)n_frames * stereo_list_cap(h->plan, cap);
  const size_t rowend = (size_t)n_frames * h->plan.hdr.height, sad = (size_t)n_frames * cap;
  if (lists > h->st_lists) {
    dfree(h->d_st_lists);
    if (dalloc(&h->d_st_lists, lists)) return ORBGPU_ERR_NOMEM;
    h->st_lists = lists;
  }
  if (rowend > h->st_rowend) {
    dfree(h->d_st_rowend);
    if (dalloc(&h->d_st_rowend, rowend)) return ORBGPU_ERR_NOMEM;
    h->st_rowend = rowend;
  }
  if (sad > h->st_sad) {
    dfree(h->d_st_sad);
    if (dalloc(&h->d_st_sad, sad)) return ORBGPU_ERR_NOMEM;
    h->st_sad = sad;
  }
  return ORBGPU_OK;
}

StereoLaunch make_stereo(orbgpu_extractor* h, int n_frames, int cap, float bf, float mb,
                         float* uright, float* depth, size_t out_fstride) {
  StereoLaunch a{};
  a.plan = h->d_plan;
  a.n_frames = n_frames;
  a.cap = cap;
  a.rows = h->plan.hdr.height;
  a.list_cap = stereo_list_cap(h->plan, cap);
  a.bf = bf;
  a.mb = mb;
  a.uright = uright;
  a.depth = depth;
  a.out_fstride = out_fstride;
  a.lists = h->d_st_lists;
  a.row_end = h->d_st_rowend;
  a.sad = h->d_st_sad;
  a.err = h->d_err;
  return a;
}

}  // namespace


// Field-wise equality of two launches (no padding compared).
static bool same_launch(const ExtractLaunch& x, const ExtractLaunch& y) {
  return x.host_plan == y.host_plan && x.plan == y.plan && x.cells == y.cells &&
         x.rs_tab == y.rs_tab && x.imgs == y.imgs && x.image_pitch == y.image_pitch &&
         x.stride == y.stride && x.n_images == y.n_images && x.pyr == y.pyr && x.blur == y.blur &&
         x.slots == y.slots && x.cell_count == y.cell_count && x.dense == y.dense &&
         x.knode == y.knode && x.oct_out == y.oct_out && x.oct_count == y.oct_count &&
         x.angle == y.angle && x.desc == y.desc && x.octree_lds == y.octree_lds &&
         x.oct_nodes == y.oct_nodes &&
         x.lap0 == y.lap0 && x.lap1 == y.lap1 && x.kps_out == y.kps_out &&
         x.desc_out == y.desc_out && x.cap == y.cap && x.n_out == y.n_out &&
         x.mono_out == y.mono_out && x.err == y.err && x.n_cu == y.n_cu && x.events == y.events &&
         x.stage_event == y.stage_event && x.stage_event_at == y.stage_event_at &&
         x.pyramid_groups == y.pyramid_groups;
}

// Enqueue the single-image chain between its copies: the image from pinned
// h_img, then the output block (n, mono, err, the full-capacity keypoints and
// descriptors) into pinned memory in one copy.  A launch seen twice in a row (same plan, buffers, lapping)
// is captured into a hipGraph and replayed from then on: the per-frame
// host path submits one graph instead of 13 kernels and 5 copies.  The
// first run of a launch stays eager (it also performs the one-time LDS
// opt-ins, which are not stream work).
static hipError_t enqueue_chain(orbgpu_extractor* h, const ExtractLaunch& a) {
  hipError_t e = hipMemcpyAsync(const_cast<uint8_t*>(a.imgs), h->h_img, a.image_pitch,
                                hipMemcpyHostToDevice, h->stream);
  if (e == hipSuccess) e = launch_extract(a, h->stream);
  // n, mono, err, keypoints and descriptors: one copy of the output block
  if (e == hipSuccess)
    e = hipMemcpyAsync(h->h_sout, h->d_sout, h->sout_bytes, hipMemcpyDeviceToHost, h->stream);
  return e;
}

static hipError_t run_single_chain(orbgpu_extractor* h, const ExtractLaunch& a) {
  const bool g_same = h->graph_wh[0] == h->plan_w && h->graph_wh[1] == h->plan_h;
  const bool e_same = h->eager_wh[0] == h->plan_w && h->eager_wh[1] == h->plan_h;
  if (h->graph_valid && g_same && same_launch(h->graph_launch, a))
    return hipGraphLaunch(h->graph_exec, h->stream);
  if (h->eager_valid && e_same && same_launch(h->eager_launch, a)) {
    if (h->graph_exec) (void)hipGraphExecDestroy(h->graph_exec);
    if (h->graph) (void)hipGraphDestroy(h->graph);
    h->graph_exec = nullptr;
    h->graph = nullptr;
    h->graph_valid = false;
    hipError_t e = hipStreamBeginCapture(h->stream, hipStreamCaptureModeRelaxed);
    if (e == hipSuccess) {
      const hipError_t le = enqueue_chain(h, a);
      e = hipStreamEndCapture(h->stream, &h->graph);
      if (e == hipSuccess) e = le;
    }
    if (e == hipSuccess) e = hipGraphInstantiate(&h->graph_exec, h->graph, nullptr, nullptr, 0);
    if (e == hipSuccess) {
      h->graph_launch = a;
      h->graph_wh[0] = h->plan_w;
      h->graph_wh[1] = h->plan_h;
      h->graph_valid = true;
      return hipGraphLaunch(h->graph_exec, h->stream);
    }
    (void)hipGetLastError();  // capture unsupported here: stay eager
  }
  h->eager_launch = a;
  h->eager_wh[0] = h->plan_w;
  h->eager_wh[1] = h->plan_h;
  h->eager_valid = true;
  return enqueue_chain(h, a);
}

// The single-image chain as one dataflow launch (k_extract_df): the launch
// record (device pointers, lapping, the plan's item shape) lives in device
// memory next to the item list and is rewritten only when it changes (a new
// plan or buffer, another lapping band).  The outputs reach the host through
// the launch's own mirror writes into the mapped h_sout: no copy commands.
// The launch record of a dataflow call, uploaded when it changes -- in the
// call's prepare phase, before any launch: its synchronous copy must not be
// issued while another dataflow launch of this thread waits for its image (a
// copy queued behind that launch on a shared hardware queue would wait for
// the staging this thread has not done yet).
static orbgpu_status prepare_single_df(orbgpu_extractor* h, size_t img_bytes, const int lap[2]) {
  const PlanHeader& P = h->plan.hdr;
  DfLaunch a;
  std::memset(&a, 0, sizeof a);
  a.plan = h->d_plan;
  a.cells = h->d_cells;
  a.rs_tab = h->d_rs;
  a.ctrl = h->d_df_ctrl;
  a.img_host = h->h_img_dev;
  a.img = h->d_img;
  a.pyr = h->d_pyr;
  a.blur = h->d_blur;
  a.slots = h->d_slots;
  a.cell_count = h->d_cell_count;
  a.dense = h->d_dense;
  a.knode = h->d_knode;
  a.oct_out = h->d_oct_out;
  a.oct_count = h->d_oct_count;
  a.angle = h->d_angle;
  a.desc = h->d_desc;
  a.lap0 = lap[0];
  a.lap1 = lap[1];
  a.kps_out = h->d_kps;
  a.desc_out = h->d_descs;
  a.nm = h->d_nm;
  a.nm_host = reinterpret_cast<int*>(h->h_sout_dev);
  a.done_host = reinterpret_cast<int*>(h->h_sout_dev) + 3;  // the output block's pad word
  a.kps_host = h->h_sout_dev + (reinterpret_cast<char*>(h->d_kps) - h->d_sout);
  a.desc_host = h->h_sout_dev + (reinterpret_cast<char*>(h->d_descs) - h->d_sout);
  a.cap = P.kp_slots;
  a.trace = h->d_df_trace;
  std::vector<uint32_t> items;
  if (h->df_valid) {
    a.items = h->df_launch.items;
    a.grid = h->df_launch.grid;
    a.df = h->df_launch.df;
  } else {
    make_df_items(P, (int)img_bytes, a.df, items);
    a.df.lds_bytes = (int)df_lds_bytes(P, octree_lds_bytes(P));
    a.grid = std::min(a.df.n_items, h->df_grid > 0 ? h->df_grid : h->n_cu);
    if (h->d_df_trace && 4 * (size_t)a.df.n_items + 2 > h->df_trace_cap) a.trace = nullptr;
    const size_t need = sizeof(DfLaunch) + items.size() * sizeof(uint32_t);
    if (need > h->df_rec_cap) {
      if (hipStreamSynchronize(h->stream) != hipSuccess) return ORBGPU_ERR_DEVICE;
      dfree(h->d_df_rec);
      if (hipMalloc(reinterpret_cast<void**>(&h->d_df_rec), need) != hipSuccess) return ORBGPU_ERR_NOMEM;
      h->df_rec_cap = need;
    }
    a.items = reinterpret_cast<const uint32_t*>(h->d_df_rec + 1);
    if (set_df_lds_limit((size_t)a.df.lds_bytes) != hipSuccess) return ORBGPU_ERR_DEVICE;
  }
  if (!h->df_valid || std::memcmp(&a, &h->df_launch, sizeof a) != 0) {
    // rare (a new plan, buffer or lapping band): ordered after the stream's work
    if (hipStreamSynchronize(h->stream) != hipSuccess ||
        hipMemcpy(h->d_df_rec, &a, sizeof a, hipMemcpyHostToDevice) != hipSuccess ||
        (!items.empty() && hipMemcpy(h->d_df_rec + 1, items.data(), items.size() * sizeof(uint32_t),
                                     hipMemcpyHostToDevice) != hipSuccess))
      return ORBGPU_ERR_DEVICE;
    h->df_launch = a;
    h->df_valid = true;
  }
  return ORBGPU_OK;
}

// One host-buffer extraction (orbgpu_extract, and each image of
// orbgpu_extract_stereo) in phases, so a stereo pair can have both launches in
// flight from one host thread: prepare (validation, plan, buffers), launch
// (the dataflow launch before its image is staged; the graph path stages the
// image and enqueues its copy + chain), stage_df (the dataflow launch's image,
// band by band), wait, finish (the outputs to the caller's arrays).
struct SingleCall {
  orbgpu_extractor* h;
  const uint8_t* img;
  int width, height, stride;
  const int* lapping;
  orbgpu_keypoint* kps;
  uint8_t* descs;
  int cap;
  int* n_out;
  int* mono_out;
  size_t bytes = 0;
  int pitch0 = 0, seq = 0;
  int lap[2] = {0, 0};
  bool df = false;

  orbgpu_status prepare() {
    if (!h || !n_out) return ORBGPU_ERR_INVALID;
    *n_out = 0;
    if (mono_out) *mono_out = -1;
    if (!img || width <= 0 || height <= 0) return ORBGPU_ERR_EMPTY;
    if (stride < width || cap < 0 || (cap > 0 && (!kps || !descs))) return ORBGPU_ERR_INVALID;
    if (hipSetDevice(h->device) != hipSuccess) return ORBGPU_ERR_DEVICE;
    orbgpu_status st = ensure_plan(h, width, height);
    if (st == ORBGPU_OK) st = ensure_workspace(h, 1);
    if (st != ORBGPU_OK) return st;
    const PlanHeader& P = h->plan.hdr;
    pitch0 = P.lev[0].pitch;  // 16-byte aligned rows for the vector loads
    bytes = (size_t)pitch0 * height;
    if (bytes > h->d_img_bytes || bytes > h->h_img_bytes) drop_graphs(h);  // image staging about to be reallocated
    if (bytes > h->d_img_bytes) {
      dfree(h->d_img);
      if (dalloc(&h->d_img, bytes)) return ORBGPU_ERR_NOMEM;
      h->d_img_bytes = bytes;
    }
    if (bytes > h->h_img_bytes) {
      if (h->h_img) (void)hipHostFree(h->h_img);
      h->h_img = nullptr;
      h->h_img_bytes = 0;
      // the image, then one flag per copy band of the dataflow launch
      const size_t flags_off = (bytes + 63) & ~(size_t)63;
      const size_t n_bands = (bytes + kDfBandBytes - 1) / kDfBandBytes;
      if (hipHostMalloc(&h->h_img, flags_off + 4 * n_bands, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
          hipHostGetDevicePointer(reinterpret_cast<void**>(&h->h_img_dev), h->h_img, 0) != hipSuccess)
        return ORBGPU_ERR_NOMEM;
      h->h_band = reinterpret_cast<int*>(h->h_img + flags_off);
      h->h_band_dev = reinterpret_cast<const int*>(h->h_img_dev + flags_off);
      std::memset(h->h_band, 0, 4 * n_bands);
      h->df_seq = 0;
      h->h_img_bytes = bytes;
    }
    if ((st = ensure_single_out(h, (size_t)P.kp_slots)) != ORBGPU_OK) return st;
    lap[0] = lapping ? lapping[0] : 0;
    lap[1] = lapping ? lapping[1] : 0;
    df = h->single_mode == ORBGPU_SINGLE_DATAFLOW && !P.oct_hbm_nodes;
    return df ? prepare_single_df(h, bytes, lap) : ORBGPU_OK;
  }

  // the image into pinned staging (rows at the level-0 pitch); band_done(b)
  // after each piece: the bytes below b are in place
  template <class F>
  void stage(F&& band_done) {
    if (stride == pitch0) {
      for (size_t b0 = 0; b0 < bytes; b0 += kDfBandBytes) {
        const size_t nb = std::min((size_t)kDfBandBytes, bytes - b0);
        std::memcpy(h->h_img + b0, img + b0, nb);
        band_done(b0 + nb);
      }
    } else {
      for (int r = 0; r < height; ++r) {
        std::memcpy(h->h_img + (size_t)r * pitch0, img + (size_t)r * stride, (size_t)width);
        band_done((size_t)(r + 1) * pitch0);
      }
    }
  }

  orbgpu_status launch() {
    if (df) {
      seq = h->df_seq = h->df_seq == 0x7fffffff ? 1 : h->df_seq + 1;
      return launch_extract_df(h->df_launch, h->d_df_rec, h->h_band_dev, seq, h->stream) == hipSuccess
                 ? ORBGPU_OK
                 : ORBGPU_ERR_DEVICE;
    }
    stage([](size_t) {});
    const PlanHeader& P = h->plan.hdr;
    ExtractLaunch a = make_launch(h, h->d_img, bytes, pitch0, 1, lap, h->d_kps, h->d_descs, P.kp_slots, h->d_nm,
                                  h->d_nm + 1);
    a.err = h->d_nm + 2;  // the block's error word: copied back with the outputs
    return run_single_chain(h, a) == hipSuccess ? ORBGPU_OK : ORBGPU_ERR_DEVICE;
  }

  // the dataflow launch's image, after the launch: each band's flag once its
  // bytes are written (the launch's copy items wait for them), so the copy
  // overlaps the launch's start
  void stage_df() {
    if (!df) return;
    const int n_bands = (int)((bytes + kDfBandBytes - 1) / kDfBandBytes);
    int next = 0;
    stage([&](size_t upto) {
      while (next < n_bands && std::min((size_t)(next + 1) * kDfBandBytes, bytes) <= upto)
        __atomic_store_n(&h->h_band[next++], seq, __ATOMIC_RELEASE);
    });
  }

  // band b of the dataflow launch's image (rows at the level-0 pitch, the
  // caller's stride equal to it): false past the last band
  bool stage_band(int b) {
    const size_t b0 = (size_t)b * kDfBandBytes;
    if (!df || stride != pitch0 || b0 >= bytes) return false;
    const size_t nb = std::min((size_t)kDfBandBytes, bytes - b0);
    std::memcpy(h->h_img + b0, img + b0, nb);
    __atomic_store_n(&h->h_band[b], seq, __ATOMIC_RELEASE);
    return true;
  }

  orbgpu_status wait() {
    if (!df) return hipStreamSynchronize(h->stream) == hipSuccess ? ORBGPU_OK : ORBGPU_ERR_DEVICE;
    // the launch writes the call's number after every output word: return as
    // soon as it appears (the workers' exit drains on the stream behind it);
    // past ~0.5 s, or a stream error, the stream's own synchronisation decides
    volatile int* done = reinterpret_cast<volatile int*>(h->h_small) + 3;
    bool seen = false;
    for (long spin = 0; spin < (1L << 24); ++spin) {
      if (*done == seq) {
        seen = true;
        break;
      }
      if ((spin & 4095) == 4095 && hipStreamQuery(h->stream) != hipErrorNotReady) {
        seen = *done == seq;
        break;
      }
      __builtin_ia32_pause();
    }
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
    if (!seen && hipStreamSynchronize(h->stream) != hipSuccess) return ORBGPU_ERR_DEVICE;
    if (!seen && *done != seq) return ORBGPU_ERR_DEVICE;
    return ORBGPU_OK;
  }

  orbgpu_status finish() {
    const int nm[2] = {h->h_small[0], h->h_small[1]}, err = h->h_small[2];
    h->host_pyr_valid = false;
    h->last_w = width;
    h->last_h = height;
    if (err) {
      if (std::getenv("ORBGPU_DEBUG")) fprintf(stderr, "orbgpu_extract: device error word 0x%x (df %d)\n", err, (int)df);
      (void)hipMemset(h->d_nm + 2, 0, sizeof(int));
      return ORBGPU_ERR_CAPACITY;
    }
    *n_out = nm[0];
    if (mono_out) *mono_out = nm[1];
    if (nm[0] > cap) return ORBGPU_ERR_CAPACITY;
    if (nm[0] > 0) {
      std::memcpy(kps, h->h_kps, (size_t)nm[0] * sizeof(orbgpu_keypoint));
      std::memcpy(descs, h->h_descs, (size_t)nm[0] * 32);
    }
    return ORBGPU_OK;
  }
};

extern "C" {

orbgpu_status orbgpu_extractor_create(const orbgpu_orb_params* params, int device, int max_width,
                                      int max_height, int max_images, orbgpu_extractor** out) {
  if (!params || !out || max_width <= 0 || max_height <= 0 || max_images <= 0)
    return ORBGPU_ERR_INVALID;
  *out = nullptr;
  HostPlan probe;
  std::string why;
  if (!make_plan(*params, max_width, max_height, probe, why)) return ORBGPU_ERR_INVALID;
  if (hipSetDevice(device) != hipSuccess) return ORBGPU_ERR_DEVICE;
  auto* h = new (std::nothrow) orbgpu_extractor();
  if (!h) return ORBGPU_ERR_NOMEM;
  h->params = *params;
  h->device = device;
  if (const char* e = std::getenv("ORBGPU_RESIZE"))  // A/B default for tools, read once
    if (std::strcmp(e, "fused") == 0) h->pyramid_launch = ORBGPU_PYRAMID_FUSED;
  h->max_w = max_width;
  h->max_h = max_height;
  h->max_images = max_images;
  if (hipDeviceGetAttribute(&h->n_cu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess ||
      h->n_cu < 1)
    h->n_cu = 256;
  if (const char* e = std::getenv("ORBGPU_SINGLE"))  // A/B default for tools, read once
    if (std::strcmp(e, "graph") == 0) h->single_mode = ORBGPU_SINGLE_GRAPH;
  if (const char* e = std::getenv("ORBGPU_DF_GRID")) h->df_grid = std::atoi(e);
  if (std::getenv("ORBGPU_DF_TRACE")) {
    h->df_trace_cap = 4 * 65536 + 2;
    if (dalloc(&h->d_df_trace, h->df_trace_cap) || hipMemset(h->d_df_trace, 0, 8 * h->df_trace_cap) != hipSuccess) {
      orbgpu_extractor_destroy(h);
      return ORBGPU_ERR_DEVICE;
    }
  }
  if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess ||
      dalloc(&h->d_plan, 1) || dalloc(&h->d_err, 1) || dalloc(&h->d_df_ctrl, (size_t)kDfCounters * kDfCtrStride) ||
      hipMemset(h->d_df_ctrl, 0, sizeof(int) * kDfCounters * kDfCtrStride) != hipSuccess) {
    orbgpu_extractor_destroy(h);
    return ORBGPU_ERR_DEVICE;
  }
  (void)hipMemset(h->d_err, 0, sizeof(int));
  orbgpu_status st = ensure_plan(h, max_width, max_height);
  if (st == ORBGPU_OK) st = ensure_workspace(h, max_images);
  if (st == ORBGPU_OK) st = ensure_single_out(h, (size_t)h->plan.hdr.kp_slots);
  if (st != ORBGPU_OK) {
    orbgpu_extractor_destroy(h);
    return st;
  }
  *out = h;
  return ORBGPU_OK;
}

void orbgpu_extractor_destroy(orbgpu_extractor* h) {
  if (!h) return;
  (void)hipSetDevice(h->device);
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  dfree(h->d_plan);
  dfree(h->d_cells);
  dfree(h->d_rs);
  dfree(h->d_pyr);
  dfree(h->d_blur);
  dfree(h->d_slots);
  dfree(h->d_dense);
  dfree(h->d_knode);
  dfree(h->d_cell_count);
  dfree(h->d_oct_out);
  dfree(h->d_oct_count);
  dfree(h->d_oct_nodes);
  dfree(h->d_angle);
  dfree(h->d_desc);
  dfree(h->d_err);
  dfree(h->d_img);
  dfree(h->d_df_ctrl);
  dfree(h->d_df_rec);
  dfree(h->d_df_trace);
  if (h->d_sout) (void)hipFree(h->d_sout);
  if (h->graph_exec) (void)hipGraphExecDestroy(h->graph_exec);
  if (h->graph) (void)hipGraphDestroy(h->graph);
  if (h->h_sout) (void)hipHostFree(h->h_sout);
  if (h->h_img) (void)hipHostFree(h->h_img);
  dfree(h->d_st_lists);
  dfree(h->d_st_rowend);
  dfree(h->d_st_sad);
  dfree(h->d_st_out);
  if (h->h_st_out) (void)hipHostFree(h->h_st_out);
  for (hipEvent_t e : h->prof_events) (void)hipEventDestroy(e);
  if (h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
}

orbgpu_status orbgpu_extractor_scales(const orbgpu_extractor* h, float* scale, float* inv_scale,
                                      float* sigma2, float* inv_sigma2) {
  if (!h) return ORBGPU_ERR_INVALID;
  const int L = h->params.num_levels;
  for (int l = 0; l < L; ++l) {
    if (scale) scale[l] = h->plan.scale[l];
    if (inv_scale) inv_scale[l] = h->plan.inv_scale[l];
    if (sigma2) sigma2[l] = h->plan.sigma2[l];
    if (inv_sigma2) inv_sigma2[l] = h->plan.inv_sigma2[l];
  }
  return ORBGPU_OK;
}

int orbgpu_extractor_levels(const orbgpu_extractor* h) { return h ? h->params.num_levels : 0; }

orbgpu_status orbgpu_extractor_set_resize_rounding(orbgpu_extractor* h, int mode) {
  if (!h || (mode != ORBGPU_RESIZE_SSE && mode != ORBGPU_RESIZE_SCALAR)) return ORBGPU_ERR_INVALID;
  if (hipSetDevice(h->device) != hipSuccess) return ORBGPU_ERR_DEVICE;
  if (h->stream && hipStreamSynchronize(h->stream) != hipSuccess) return ORBGPU_ERR_DEVICE;
  if (mode == h->resize_rounding) return ORBGPU_OK;
  h->resize_rounding = mode;
  const int w = h->plan_w, ht = h->plan_h;
  h->plan_w = h->plan_h = -1;  // re-plan (and retire captured graphs) with the new column split
  return ensure_plan(h, w, ht);
}

orbgpu_status orbgpu_extractor_set_octree_nodes(orbgpu_extractor* h, int mode) {
  if (!h || (mode != ORBGPU_OCTREE_NODES_AUTO && mode != ORBGPU_OCTREE_NODES_HBM)) return ORBGPU_ERR_INVALID;
  if (hipSetDevice(h->device) != hipSuccess) return ORBGPU_ERR_DEVICE;
  if (h->stream && hipStreamSynchronize(h->stream) != hipSuccess) return ORBGPU_ERR_DEVICE;
  if (mode == h->octree_nodes) return ORBGPU_OK;
  h->octree_nodes = mode;
  const int w = h->plan_w, ht = h->plan_h;
  h->plan_w = h->plan_h = -1;  // re-plan; ensure_workspace sizes the node range on the next call
  return ensure_plan(h, w, ht);
}

orbgpu_status orbgpu_extractor_set_stage_event(orbgpu_extractor* h, int stage, void* hip_event) {
  if (!h || (hip_event && (stage < 0 || stage >= kStages))) return ORBGPU_ERR_INVALID;
  h->stage_event = static_cast<hipEvent_t>(hip_event);
  h->stage_event_at = hip_event ? stage : -1;
  return ORBGPU_OK;
}

orbgpu_status orbgpu_extractor_set_pyramid_launch(orbgpu_extractor* h, int mode) {
  if (!h || (mode != ORBGPU_PYRAMID_PER_LEVEL && mode != ORBGPU_PYRAMID_FUSED)) return ORBGPU_ERR_INVALID;
  if (hipSetDevice(h->device) != hipSuccess) return ORBGPU_ERR_DEVICE;
  if (h->stream && hipStreamSynchronize(h->stream) != hipSuccess) return ORBGPU_ERR_DEVICE;
  h->pyramid_launch = mode;  // the next launch differs from a captured one: no stale graph replays
  return ORBGPU_OK;
}

// Debug (not in orbgpu.h; tools/df_trace.py): the last dataflow launch's
// per-ticket timeline, 4 u64 per item + the assembly's start / end; returns
// the item count, or -1 without ORBGPU_DF_TRACE.
int orbgpu_debug_df_trace(orbgpu_extractor* h, unsigned long long* out, int cap_items) {
  if (!h || !out || !h->d_df_trace || !h->df_valid) return -1;
  const int n = std::min(cap_items, h->df_launch.df.n_items);
  if (hipStreamSynchronize(h->stream) != hipSuccess ||
      hipMemcpy(out, h->d_df_trace, 8 * (4 * (size_t)n + 2), hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  if (n == h->df_launch.df.n_items) {  // the assembly stamps follow the items
    out[4 * (size_t)n] = 0;
  }
  if (hipMemcpy(out + 4 * (size_t)n, h->d_df_trace + 4 * (size_t)h->df_launch.df.n_items, 16,
                hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  return n;
}

orbgpu_status orbgpu_extractor_set_single_launch(orbgpu_extractor* h, int mode) {
  if (!h || (mode != ORBGPU_SINGLE_DATAFLOW && mode != ORBGPU_SINGLE_GRAPH)) return ORBGPU_ERR_INVALID;
  h->single_mode = mode;
  return ORBGPU_OK;
}

orbgpu_status orbgpu_extractor_plan(const orbgpu_orb_params* params, int width, int height,
                                    int* kp_slots, int* octree_hbm) {
  if (!params) return ORBGPU_ERR_INVALID;
  HostPlan p;
  std::string why;
  if (!make_plan(*params, width, height, p, why)) return ORBGPU_ERR_INVALID;
  if (kp_slots) *kp_slots = p.hdr.kp_slots;
  if (octree_hbm) *octree_hbm = p.hdr.oct_hbm_nodes;
  return ORBGPU_OK;
}

int orbgpu_extractor_max_keypoints(orbgpu_extractor* h, int width, int height) {
  if (!h) return -1;
  HostPlan p;
  std::string why;
  if (!make_plan(h->params, width, height, p, why)) return -1;
  return p.hdr.kp_slots;
}

orbgpu_status orbgpu_extract(orbgpu_extractor* h, const uint8_t* img, int width, int height,
                             int stride, const int lapping[2], orbgpu_keypoint* kps,
                             uint8_t* descs, int cap, int* n_out, int* mono_out) {
  SingleCall c{h, img, width, height, stride, lapping, kps, descs, cap, n_out, mono_out};
  orbgpu_status st = c.prepare();
  if (st == ORBGPU_OK) st = c.launch();
  if (st == ORBGPU_OK) c.stage_df();
  if (st == ORBGPU_OK) st = c.wait();
  return st == ORBGPU_OK ? c.finish() : st;
}

orbgpu_status orbgpu_extract_stereo(orbgpu_extractor* left, orbgpu_extractor* right, const uint8_t* img_left,
                                    const uint8_t* img_right, int width, int height, int stride,
                                    const int lapping_left[2], const int lapping_right[2],
                                    orbgpu_keypoint* kps_left, uint8_t* descs_left, int cap_left,
                                    int* n_left, int* mono_left, orbgpu_keypoint* kps_right,
                                    uint8_t* descs_right, int cap_right, int* n_right, int* mono_right) {
  if (!left || !right || left == right) return ORBGPU_ERR_INVALID;
  SingleCall c[2] = {{left, img_left, width, height, stride, lapping_left, kps_left, descs_left, cap_left, n_left,
                      mono_left},
                     {right, img_right, width, height, stride, lapping_right, kps_right, descs_right, cap_right,
                      n_right, mono_right}};
  orbgpu_status st[2];
  for (int k = 0; k < 2; ++k) st[k] = c[k].prepare();
  // both dataflow launches first (each handle's own stream), then both images
  // (each launch's copy items wait for their bands), then the results.  A
  // graph-path launch may block (capture, instantiation), so with one in the
  // pair each image is staged right after its own launch.
  if (c[0].df && c[1].df) {
    for (int k = 0; k < 2; ++k)
      if (st[k] == ORBGPU_OK) st[k] = c[k].launch();
    if (st[0] == ORBGPU_OK && st[1] == ORBGPU_OK && c[0].stride == c[0].pitch0 && c[1].stride == c[1].pitch0) {
      // the two images' bands in alternation: both launches start on level 0
      // together instead of the right one waiting for the whole left image
      for (int b = 0;; ++b) {
        const bool l = c[0].stage_band(b), r = c[1].stage_band(b);
        if (!l && !r) break;
      }
    } else {
      for (int k = 0; k < 2; ++k)
        if (st[k] == ORBGPU_OK) c[k].stage_df();
    }
  } else {
    for (int k = 0; k < 2; ++k)
      if (st[k] == ORBGPU_OK && (st[k] = c[k].launch()) == ORBGPU_OK) c[k].stage_df();
  }
  for (int k = 0; k < 2; ++k)
    if (st[k] == ORBGPU_OK) st[k] = c[k].wait();
  for (int k = 0; k < 2; ++k)
    if (st[k] == ORBGPU_OK) st[k] = c[k].finish();
  return st[0] != ORBGPU_OK ? st[0] : st[1];
}

orbgpu_status orbgpu_extractor_pyramid_level(orbgpu_extractor* h, int level, const uint8_t** data,
                                             int* width, int* height, int* stride) {
  if (!h || !data || level < 0 || level >= h->params.num_levels || h->last_w == 0)
    return ORBGPU_ERR_INVALID;
  if (hipSetDevice(h->device) != hipSuccess) return ORBGPU_ERR_DEVICE;
  const PlanHeader& P = h->plan.hdr;
  const size_t l0 = (size_t)P.lev[0].pitch * P.lev[0].h;
  if (!h->host_pyr_valid) {
    h->host_pyr.resize(l0 + P.pyr_bytes);
    if (hipMemcpyAsync(h->host_pyr.data(), h->d_img, l0, hipMemcpyDeviceToHost, h->stream) ||
        hipMemcpyAsync(h->host_pyr.data() + l0, h->d_pyr, P.pyr_bytes, hipMemcpyDeviceToHost,
                       h->stream) ||
        hipStreamSynchronize(h->stream))
      return ORBGPU_ERR_DEVICE;
    h->host_pyr_valid = true;
  }
  const LevelGeom& g = P.lev[level];
  *data = h->host_pyr.data() + (level == 0 ? 0 : l0 + g.pyr_off);
  if (width) *width = g.w;
  if (height) *height = g.h;
  if (stride) *stride = g.pitch;
  return ORBGPU_OK;
}

orbgpu_status orbgpu_extract_batch(orbgpu_extractor* h, const uint8_t* d_imgs, int n_images,
                                   int width, int height, int stride, size_t image_pitch,
                                   const int lapping[2], orbgpu_keypoint* d_kps, uint8_t* d_descs,
                                   int cap_per_image, int* d_n, int* d_mono, void* hip_stream) {
  if (!h || !d_imgs || n_images <= 0 || !d_kps || !d_descs || !d_n || !d_mono)
    return ORBGPU_ERR_INVALID;
  if (width <= 0 || height <= 0) return ORBGPU_ERR_EMPTY;
  if (stride < width || image_pitch < (size_t)stride * height) return ORBGPU_ERR_INVALID;
  if (hipSetDevice(h->device) != hipSuccess) return ORBGPU_ERR_DEVICE;
  orbgpu_status st = ensure_plan(h, width, height);
  if (st == ORBGPU_OK) st = ensure_workspace(h, n_images);
  if (st != ORBGPU_OK) return st;
  hipStream_t s = hip_stream ? (hipStream_t)hip_stream : h->stream;
  const int lap[2] = {lapping ? lapping[0] : 0, lapping ? lapping[1] : 0};
  ExtractLaunch a = make_launch(h, d_imgs, image_pitch, stride, n_images, lap, d_kps, d_descs,
                                cap_per_image, d_n, d_mono);
  if (h->prof_used < h->prof_slots) a.events = &h->prof_events[(size_t)h->prof_used++ * (kStages + 1)];
  a.stage_event = h->stage_event;
  a.stage_event_at = h->stage_event_at;
  if (launch_extract(a, s) != hipSuccess) return ORBGPU_ERR_DEVICE;
  h->host_pyr_valid = false;
  h->last_w = 0;  // the host pyramid getter serves the host-buffer path only
  return ORBGPU_OK;
}

orbgpu_status orbgpu_extractor_profile(orbgpu_extractor* h, int max_calls) {
  if (!h || max_calls < 0) return ORBGPU_ERR_INVALID;
  if (hipSetDevice(h->device) != hipSuccess) return ORBGPU_ERR_DEVICE;
  (void)hipDeviceSynchronize();
  for (hipEvent_t e : h->prof_events) (void)hipEventDestroy(e);
  h->prof_events.assign((size_t)max_calls * (kStages + 1), nullptr);
  for (hipEvent_t& e : h->prof_events)
    if (hipEventCreate(&e) != hipSuccess) return ORBGPU_ERR_DEVICE;
  h->prof_slots = max_calls;
  h->prof_used = 0;
  return ORBGPU_OK;
}

int orbgpu_extractor_profile_read(orbgpu_extractor* h, double* ms_per_stage) {
  if (!h || !ms_per_stage) return -1;
  if (hipSetDevice(h->device) != hipSuccess) return -1;
  for (int k = 0; k < kStages; ++k) ms_per_stage[k] = 0;
  for (int c = 0; c < h->prof_used; ++c) {
    hipEvent_t* ev = &h->prof_events[(size_t)c * (kStages + 1)];
    if (hipEventSynchronize(ev[kStages]) != hipSuccess) return -1;
    for (int k = 0; k < kStages; ++k) {
      float ms = 0;
      if (hipEventElapsedTime(&ms, ev[k], ev[k + 1]) != hipSuccess) return -1;
      ms_per_stage[k] += ms;
    }
  }
  const int calls = h->prof_used;
  h->prof_used = 0;
  return calls;
}

int orbgpu_extractor_stage(orbgpu_extractor* h, int which, int level, void* out, int cap) {
  if (!h || !out || level < 0 || level >= h->params.num_levels || h->plan_w < 0) return -1;
  if (hipSetDevice(h->device) != hipSuccess || hipStreamSynchronize(h->stream) != hipSuccess)
    return -1;
  const PlanHeader& P = h->plan.hdr;
  const LevelGeom& g = P.lev[level];
  if (which == 0) {
    const int n = g.w * g.h;
    if (n > cap) return -1;
    return hipMemcpy2D(out, g.w, h->d_blur + g.blur_off, g.pitch, g.w, g.h,
                       hipMemcpyDeviceToHost) == hipSuccess
               ? n
               : -1;
  }
  if (which == 1) {
    std::vector<int> cc(g.cell_end - g.cell_begin);
    if (hipMemcpy(cc.data(), h->d_cell_count + g.cell_begin, cc.size() * sizeof(int),
                  hipMemcpyDeviceToHost) != hipSuccess)
      return -1;
    int n = 0;
    for (int c : cc) n += c;
    if (n > cap) return -1;
    return hipMemcpy(out, h->d_dense + g.slot_begin, (size_t)n * 4, hipMemcpyDeviceToHost) ==
                   hipSuccess
               ? n
               : -1;
  }
  if (which == 2) {
    int n = 0;
    if (hipMemcpy(&n, h->d_oct_count + level, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess ||
        n > cap)
      return -1;
    return hipMemcpy(out, h->d_oct_out + g.out_off, (size_t)n * 4, hipMemcpyDeviceToHost) ==
                   hipSuccess
               ? n
               : -1;
  }
  return -1;
}

orbgpu_status orbgpu_stereo_match_batch(orbgpu_extractor* h, int n_frames, const uint8_t* d_imgs,
                                        int stride, size_t image_pitch, const orbgpu_keypoint* d_kps,
                                        const uint8_t* d_descs, int cap_per_image, const int* d_n,
                                        float bf, float mb, float* d_uright, float* d_depth,
                                        void* hip_stream) {
  if (!h || n_frames <= 0 || !d_imgs || !d_kps || !d_descs || !d_n || !d_uright || !d_depth ||
      cap_per_image <= 0 || cap_per_image > 65535 || !(mb > 0.0f))  // u16 row lists
    return ORBGPU_ERR_INVALID;
  if (h->plan_w < 0 || h->ws_images < 2 * n_frames) return ORBGPU_ERR_INVALID;  // no batch yet
  if (hipSetDevice(h->device) != hipSuccess) return ORBGPU_ERR_DEVICE;
  orbgpu_status st = ensure_stereo(h, n_frames, cap_per_image);
  if (st != ORBGPU_OK) return st;
  const PlanHeader& P = h->plan.hdr;
  StereoLaunch a = make_stereo(h, n_frames, cap_per_image, bf, mb, d_uright, d_depth,
                               (size_t)cap_per_image);
  const float* kps = reinterpret_cast<const float*>(d_kps);
  for (int side = 0; side < 2; ++side) {  // images 2f (left), 2f + 1 (right)
    StereoSide& s = side ? a.R : a.L;
    s.img0 = d_imgs + side * image_pitch;
    s.img_fstride = 2 * image_pitch;
    s.img_stride = stride;
    s.pyr = h->d_pyr + (size_t)side * P.pyr_bytes;
    s.pyr_fstride = 2 * (size_t)P.pyr_bytes;
    s.kps = kps + (size_t)side * cap_per_image * 7;
    s.kp_fstride = 2 * (size_t)cap_per_image;
    s.desc = d_descs + (size_t)side * cap_per_image * 32;
    s.n = d_n + side;
    s.n_fstride = 2;
  }
  hipStream_t s = hip_stream ? (hipStream_t)hip_stream : h->stream;
  return launch_stereo(a, s) == hipSuccess ? ORBGPU_OK : ORBGPU_ERR_DEVICE;
}

orbgpu_status orbgpu_stereo_match(orbgpu_extractor* left, orbgpu_extractor* right, float bf,
                                  float mb, float* uright, float* depth, int cap) {
  if (!left || !right || !uright || !depth || cap < 0 || !(mb > 0.0f)) return ORBGPU_ERR_INVALID;
  // both handles must hold a host-path extraction of one geometry and parameter set
  if (left->last_w <= 0 || right->last_w != left->last_w || right->last_h != left->last_h ||
      std::memcmp(&left->params, &right->params, sizeof(left->params)) != 0 ||
      left->device != right->device)
    return ORBGPU_ERR_INVALID;
  if (hipSetDevice(left->device) != hipSuccess) return ORBGPU_ERR_DEVICE;
  const PlanHeader& P = left->plan.hdr;
  const int kcap = P.kp_slots;
  if (kcap > 65535) return ORBGPU_ERR_INVALID;  // u16 row lists / match keys (k_stereo_match)
  orbgpu_status st = ensure_stereo(left, 1, kcap);
  if (st != ORBGPU_OK) return st;
  const size_t need = 4 + (size_t)2 * kcap;
  if (need > left->st_out) {
    dfree(left->d_st_out);
    if (left->h_st_out) (void)hipHostFree(left->h_st_out);
    left->h_st_out = nullptr;
    left->st_out = 0;
    if (dalloc(&left->d_st_out, need) ||
        hipHostMalloc(&left->h_st_out, (need + 16) * sizeof(float), hipHostMallocMapped | hipHostMallocCoherent) !=
            hipSuccess ||
        hipHostGetDevicePointer(reinterpret_cast<void**>(&left->h_st_out_dev), left->h_st_out, 0) != hipSuccess)
      return ORBGPU_ERR_NOMEM;
    reinterpret_cast<int*>(left->h_st_out)[need] = 0;
    left->st_out = need;
  }
  float* dur = left->d_st_out + 4;
  StereoLaunch a = make_stereo(left, 1, kcap, bf, mb, dur, dur + kcap, (size_t)kcap);
  int* d_call_err = reinterpret_cast<int*>(left->d_st_out);  // this call's error word
  a.err = d_call_err;
  for (int side = 0; side < 2; ++side) {
    orbgpu_extractor* h = side ? right : left;
    StereoSide& s = side ? a.R : a.L;
    s.img0 = h->d_img;
    s.img_stride = h->plan.hdr.lev[0].pitch;
    s.pyr = h->d_pyr;
    s.kps = reinterpret_cast<const float*>(h->d_kps);
    s.desc = h->d_descs;
    s.n = h->d_nm;
  }
  // the left call's keypoint count (its pinned output block, already synchronised)
  const int n = std::min(left->h_small[0], kcap);
  if (n > cap) return ORBGPU_ERR_CAPACITY;
  // error word, uright[0, kcap), depth[0, n): mirrored into the host-mapped
  // block by k_stereo_median, which then stores the call's number after it
  const size_t bytes = (4 + (size_t)kcap + (size_t)n) * sizeof(float);
  const int seq = left->st_seq = left->st_seq == 0x7fffffff ? 1 : left->st_seq + 1;
  a.zero_err = 1;  // k_stereo_rows writes the error word (no memset)
  a.mirror_src = reinterpret_cast<const uint8_t*>(left->d_st_out);
  a.mirror_dst = reinterpret_cast<uint8_t*>(left->h_st_out_dev);
  a.mirror_bytes = (int)bytes;
  a.done_host = reinterpret_cast<int*>(left->h_st_out_dev) + left->st_out;
  a.seq = seq;
  if (launch_stereo(a, left->stream) != hipSuccess) return ORBGPU_ERR_DEVICE;
  volatile int* done = reinterpret_cast<volatile int*>(left->h_st_out) + left->st_out;
  bool seen = false;
  for (long spin = 0; spin < (1L << 24); ++spin) {
    if (*done == seq) {
      seen = true;
      break;
    }
    if ((spin & 4095) == 4095 && hipStreamQuery(left->stream) != hipErrorNotReady) {
      seen = *done == seq;
      break;
    }
    __builtin_ia32_pause();
  }
  __atomic_thread_fence(__ATOMIC_ACQUIRE);
  if (!seen && (hipStreamSynchronize(left->stream) != hipSuccess || *done != seq)) return ORBGPU_ERR_DEVICE;
  int err = 0;
  std::memcpy(&err, left->h_st_out, sizeof(int));
  if (err) return ORBGPU_ERR_CAPACITY;
  if (n > 0) {
    std::memcpy(uright, left->h_st_out + 4, (size_t)n * sizeof(float));
    std::memcpy(depth, left->h_st_out + 4 + kcap, (size_t)n * sizeof(float));
  }
  return ORBGPU_OK;
}

orbgpu_status orbgpu_extractor_check(orbgpu_extractor* h) {
  if (!h) return ORBGPU_ERR_INVALID;
  if (hipSetDevice(h->device) != hipSuccess) return ORBGPU_ERR_DEVICE;
  int err = 0;
  if (hipDeviceSynchronize() != hipSuccess ||
      hipMemcpy(&err, h->d_err, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess)
    return ORBGPU_ERR_DEVICE;
  if (err) {
    (void)hipMemset(h->d_nm + 2, 0, sizeof(int));
    return ORBGPU_ERR_CAPACITY;
  }
  return ORBGPU_OK;
}

}  // extern "C"
