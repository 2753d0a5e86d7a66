// C-ABI implementation of the DBoW2 vocabulary / transform half of
// include/orbgpu.h (kernels: bow_kernels.hip).  The text loader restates
// TemplatedVocabulary::loadFromTextFile (TemplatedVocabulary.h:1248-1327)
// with the same iostream extraction rules, then the tree goes to the device
// as flat arrays (descriptors, CSR children in file order, word ids, weights).
#include <hip/hip_runtime.h>

#include <cstring>
#include <fstream>
#include <new>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/orbgpu.h"
#include "bow_launch.h"

using orbgpu::kBowMaxFeatures;

struct orbgpu_vocab {
  int device = 0;
  hipStream_t stream = nullptr;
  orbgpu::VocabDev dev{};
  void* d_tree = nullptr;  // one allocation for every tree array
  // scratch of the host-buffer path and per-feature arrays of batches
  uint8_t* d_io = nullptr;
  size_t io_bytes = 0;
  uint8_t* h_io = nullptr;
  size_t h_bytes = 0;
  void* d_feat = nullptr;
  size_t feat_cap = 0;  // features
};

namespace {

struct HostTree {
  int k = 0, L = 0, scoring = 0, weighting = 0;
  std::vector<uint8_t> desc;            // 32 per node
  std::vector<std::vector<uint32_t>> children;
  std::vector<uint32_t> word_id;
  std::vector<double> weight;
  uint32_t n_words = 0;
};

// loadFromTextFile: one node per getline until eof (a trailing empty line
// makes a childless, weightless node under the root, as in the reference;
// its descriptor, uninitialised there, is zero here).
bool parse(const char* path, HostTree& T) {
  std::ifstream f(path);
  if (!f.is_open() || f.eof()) return false;
  std::string head;
  std::getline(f, head);
  std::istringstream hs(head);
  int sc = 0, wt = 0;
  hs >> T.k >> T.L >> sc >> wt;
  if (T.k < 0 || T.k > 20 || T.L < 1 || T.L > 10 || sc < 0 || sc > 5 || wt < 0 || wt > 3)
    return false;
  T.scoring = sc, T.weighting = wt;
  T.desc.assign(32, 0);
  T.children.assign(1, {});
  T.word_id.assign(1, 0);
  T.weight.assign(1, 0.0);
  std::string line;
  while (!f.eof()) {
    std::getline(f, line);
    std::istringstream ls(line);
    const uint32_t id = (uint32_t)T.children.size();
    int parent = 0, leaf = 0;
    ls >> parent;
    if (parent < 0 || (uint32_t)parent >= id) return false;  // UB in the reference
    ls >> leaf;
    // FORB::fromString on the 32 whitespace tokens: a token that is not an
    // int leaves its byte (and every later one) as it was
    std::string toks;
    for (int i = 0; i < 32; ++i) {
      std::string tok;
      ls >> tok;
      toks += tok;
      toks += ' ';
    }
    std::istringstream ds(toks);
    uint8_t d[32] = {};
    for (int i = 0; i < 32; ++i) {
      int v;
      ds >> v;
      if (!ds.fail()) d[i] = (uint8_t)v;
    }
    double w = 0.0;
    ls >> w;
    T.desc.insert(T.desc.end(), d, d + 32);
    T.children.emplace_back();
    T.children[parent].push_back(id);
    T.weight.push_back(w);
    T.word_id.push_back(leaf > 0 ? T.n_words++ : 0u);
  }
  return true;
}

size_t al(size_t v) { return (v + 255) & ~(size_t)255; }

int pow2_at_least(int v) {
  int m = 1;
  while (m < v) m <<= 1;
  return m;
}

orbgpu_status upload(orbgpu_vocab* v, const HostTree& T) {
  const int N = (int)T.children.size();
  std::vector<int> off(N + 1, 0);
  for (int i = 0; i < N; ++i) off[i + 1] = off[i] + (int)T.children[i].size();
  std::vector<uint32_t> ids;
  ids.reserve(off[N]);
  for (const auto& c : T.children) ids.insert(ids.end(), c.begin(), c.end());
  const size_t b_desc = al(32 * (size_t)N), b_off = al(4 * (size_t)(N + 1)),
               b_ids = al(4 * ids.size() + 4), b_word = al(4 * (size_t)N), b_w = al(8 * (size_t)N);
  const size_t total = b_desc + b_off + b_ids + b_word + b_w;
  if (hipMalloc(&v->d_tree, total) != hipSuccess) return ORBGPU_ERR_NOMEM;
  std::vector<uint8_t> h(total, 0);
  uint8_t* p = h.data();
  std::memcpy(p, T.desc.data(), 32 * (size_t)N);
  std::memcpy(p + b_desc, off.data(), 4 * (size_t)(N + 1));
  if (!ids.empty()) std::memcpy(p + b_desc + b_off, ids.data(), 4 * ids.size());
  std::memcpy(p + b_desc + b_off + b_ids, T.word_id.data(), 4 * (size_t)N);
  std::memcpy(p + b_desc + b_off + b_ids + b_word, T.weight.data(), 8 * (size_t)N);
  if (hipMemcpy(v->d_tree, h.data(), total, hipMemcpyHostToDevice) != hipSuccess)
    return ORBGPU_ERR_DEVICE;
  uint8_t* d = static_cast<uint8_t*>(v->d_tree);
  orbgpu::VocabDev& D = v->dev;
  D.desc = d;
  D.child_off = reinterpret_cast<const int*>(d + b_desc);
  D.child_ids = reinterpret_cast<const uint32_t*>(d + b_desc + b_off);
  D.word_id = reinterpret_cast<const uint32_t*>(d + b_desc + b_off + b_ids);
  D.weight = reinterpret_cast<const double*>(d + b_desc + b_off + b_ids + b_word);
  D.k = T.k, D.L = T.L, D.scoring = T.scoring, D.weighting = T.weighting;
  D.n_nodes = N, D.n_words = (int)T.n_words;
  return ORBGPU_OK;
}

// per-feature scratch (word, weight, node) for `feats` features
orbgpu_status ensure_feat(orbgpu_vocab* v, size_t feats) {
  if (feats <= v->feat_cap) return ORBGPU_OK;
  if (v->d_feat) (void)hipFree(v->d_feat);
  v->d_feat = nullptr;
  v->feat_cap = 0;
  if (hipMalloc(&v->d_feat, feats * 16) != hipSuccess) return ORBGPU_ERR_NOMEM;
  v->feat_cap = feats;
  return ORBGPU_OK;
}

void set_feat(orbgpu_vocab* v, orbgpu::BowLaunch& L, size_t feats) {
  uint8_t* p = static_cast<uint8_t*>(v->d_feat);
  L.f_weight = reinterpret_cast<double*>(p);
  L.f_word = reinterpret_cast<uint32_t*>(p + 8 * feats);
  L.f_nid = reinterpret_cast<uint32_t*>(p + 12 * feats);
}

}  // namespace

extern "C" {

orbgpu_status orbgpu_vocab_load_text(int device, const char* path, orbgpu_vocab** out) {
  if (!path || !out) return ORBGPU_ERR_INVALID;
  *out = nullptr;
  HostTree T;
  if (!parse(path, T)) return ORBGPU_ERR_INVALID;
  if (hipSetDevice(device) != hipSuccess) return ORBGPU_ERR_DEVICE;
  auto* v = new (std::nothrow) orbgpu_vocab();
  if (!v) return ORBGPU_ERR_NOMEM;
  v->device = device;
  orbgpu_status st = ORBGPU_OK;
  if (hipStreamCreateWithFlags(&v->stream, hipStreamNonBlocking) != hipSuccess)
    st = ORBGPU_ERR_DEVICE;
  if (st == ORBGPU_OK) st = upload(v, T);
  if (st != ORBGPU_OK) {
    orbgpu_vocab_destroy(v);
    return st;
  }
  *out = v;
  return ORBGPU_OK;
}

void orbgpu_vocab_destroy(orbgpu_vocab* v) {
  if (!v) return;
  (void)hipSetDevice(v->device);
  if (v->stream) (void)hipStreamSynchronize(v->stream);
  if (v->d_tree) (void)hipFree(v->d_tree);
  if (v->d_io) (void)hipFree(v->d_io);
  if (v->h_io) (void)hipHostFree(v->h_io);
  if (v->d_feat) (void)hipFree(v->d_feat);
  if (v->stream) (void)hipStreamDestroy(v->stream);
  delete v;
}

orbgpu_status orbgpu_vocab_info(const orbgpu_vocab* v, int info[6]) {
  if (!v || !info) return ORBGPU_ERR_INVALID;
  info[0] = v->dev.k, info[1] = v->dev.L, info[2] = v->dev.scoring, info[3] = v->dev.weighting;
  info[4] = v->dev.n_nodes, info[5] = v->dev.n_words;
  return ORBGPU_OK;
}

orbgpu_status orbgpu_bow_transform_batch(orbgpu_vocab* v, int n_frames, const uint8_t* d_descs,
                                         const int* d_n, int stride, int levelsup,
                                         uint32_t* d_bow_words, double* d_bow_weights,
                                         int* d_n_words, uint32_t* d_fv_nodes,
                                         int32_t* d_fv_offsets, uint32_t* d_fv_features,
                                         int* d_n_nodes, void* hip_stream) {
  if (!v || n_frames <= 0 || !d_descs || !d_n || stride <= 0 || stride > kBowMaxFeatures ||
      !d_bow_words || !d_bow_weights || !d_n_words || !d_fv_nodes || !d_fv_offsets ||
      !d_fv_features || !d_n_nodes)
    return ORBGPU_ERR_INVALID;
  if (hipSetDevice(v->device) != hipSuccess) return ORBGPU_ERR_DEVICE;
  const size_t feats = (size_t)n_frames * stride;
  if (ensure_feat(v, feats) != ORBGPU_OK) return ORBGPU_ERR_NOMEM;
  orbgpu::BowLaunch L{};
  L.voc = v->dev;
  L.n_frames = n_frames, L.stride = stride, L.levelsup = levelsup;
  L.lds_m = pow2_at_least(stride);
  L.descs = d_descs, L.n = d_n;
  set_feat(v, L, v->feat_cap);
  L.bow_words = d_bow_words, L.bow_weights = d_bow_weights, L.n_words = d_n_words;
  L.fv_nodes = d_fv_nodes, L.fv_offsets = d_fv_offsets, L.fv_features = d_fv_features;
  L.n_nodes = d_n_nodes;
  hipStream_t s = hip_stream ? (hipStream_t)hip_stream : v->stream;
  return orbgpu::launch_bow(L, s) == hipSuccess ? ORBGPU_OK : ORBGPU_ERR_DEVICE;
}

orbgpu_status orbgpu_bow_transform(orbgpu_vocab* v, const uint8_t* descs, int n, int levelsup,
                                   uint32_t* bow_words, double* bow_weights, int* n_words,
                                   uint32_t* fv_nodes, int32_t* fv_offsets, uint32_t* fv_features,
                                   int* n_nodes) {
  if (!v || n < 0 || (n > 0 && (!descs || !bow_words || !bow_weights || !fv_nodes ||
                                !fv_features)) ||
      !n_words || !n_nodes || !fv_offsets)
    return ORBGPU_ERR_INVALID;
  if (n > kBowMaxFeatures) return ORBGPU_ERR_CAPACITY;
  if (hipSetDevice(v->device) != hipSuccess) return ORBGPU_ERR_DEVICE;
  const int S = n > 0 ? n : 1;
  // device layout: descs | n | outputs (words, weights, n_words, nodes, offsets, features, n_nodes)
  const size_t o_desc = 0, o_n = al(32 * (size_t)S), o_words = o_n + 256,
               o_wts = o_words + al(4 * (size_t)S), o_nw = o_wts + al(8 * (size_t)S),
               o_nodes = o_nw + 256, o_offs = o_nodes + al(4 * (size_t)S),
               o_feat = o_offs + al(4 * (size_t)(S + 1)), o_nn = o_feat + al(4 * (size_t)S),
               total = o_nn + 256;
  if (total > v->io_bytes) {
    if (v->d_io) (void)hipFree(v->d_io);
    if (v->h_io) (void)hipHostFree(v->h_io);
    v->d_io = v->h_io = nullptr;
    v->io_bytes = 0;
    if (hipMalloc(&v->d_io, total) != hipSuccess || hipHostMalloc(&v->h_io, total) != hipSuccess)
      return ORBGPU_ERR_NOMEM;
    v->io_bytes = total;
  }
  if (ensure_feat(v, S) != ORBGPU_OK) return ORBGPU_ERR_NOMEM;
  uint8_t* h = v->h_io;
  uint8_t* d = v->d_io;
  if (n > 0) std::memcpy(h + o_desc, descs, 32 * (size_t)n);
  std::memcpy(h + o_n, &n, sizeof(int));
  hipStream_t s = v->stream;
  if (hipMemcpyAsync(d, h, o_n + sizeof(int), hipMemcpyHostToDevice, s) != hipSuccess)
    return ORBGPU_ERR_DEVICE;
  orbgpu::BowLaunch L{};
  L.voc = v->dev;
  L.n_frames = 1, L.stride = S, L.levelsup = levelsup;
  L.lds_m = pow2_at_least(S);
  L.descs = d + o_desc;
  L.n = reinterpret_cast<const int*>(d + o_n);
  set_feat(v, L, v->feat_cap);
  L.bow_words = reinterpret_cast<uint32_t*>(d + o_words);
  L.bow_weights = reinterpret_cast<double*>(d + o_wts);
  L.n_words = reinterpret_cast<int*>(d + o_nw);
  L.fv_nodes = reinterpret_cast<uint32_t*>(d + o_nodes);
  L.fv_offsets = reinterpret_cast<int32_t*>(d + o_offs);
  L.fv_features = reinterpret_cast<uint32_t*>(d + o_feat);
  L.n_nodes = reinterpret_cast<int*>(d + o_nn);
  if (orbgpu::launch_bow(L, s) != hipSuccess ||
      hipMemcpyAsync(h + o_words, d + o_words, total - o_words, hipMemcpyDeviceToHost, s) !=
          hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return ORBGPU_ERR_DEVICE;
  int nw, nn;
  std::memcpy(&nw, h + o_nw, sizeof(int));
  std::memcpy(&nn, h + o_nn, sizeof(int));
  *n_words = nw;
  *n_nodes = nn;
  if (nw > 0) {
    std::memcpy(bow_words, h + o_words, 4 * (size_t)nw);
    std::memcpy(bow_weights, h + o_wts, 8 * (size_t)nw);
  }
  std::memcpy(fv_offsets, h + o_offs, 4 * (size_t)(nn + 1));
  if (nn > 0) {
    std::memcpy(fv_nodes, h + o_nodes, 4 * (size_t)nn);
    int nf;
    std::memcpy(&nf, h + o_offs + 4 * (size_t)nn, sizeof(int));
    std::memcpy(fv_features, h + o_feat, 4 * (size_t)nf);
  }
  return ORBGPU_OK;
}

}  // extern "C"
