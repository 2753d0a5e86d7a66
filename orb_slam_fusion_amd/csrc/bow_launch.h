// Launch descriptor of DBoW2's transform (TemplatedVocabulary.h:1057-1179)
// over a vocabulary tree resident in HBM.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace orbgpu {

constexpr int kBowMaxFeatures = 8192;  // per frame (LDS sort of the assembly: 16 B a feature, 128 KB)

struct VocabDev {
  const uint8_t* desc;       // [n_nodes][32]
  const int* child_off;      // [n_nodes + 1] into child_ids (children in file order)
  const uint32_t* child_ids;
  const uint32_t* word_id;   // [n_nodes] (0 for non-words, as Node())
  const double* weight;      // [n_nodes]
  int k, L, scoring, weighting, n_nodes, n_words;
};

struct BowLaunch {
  VocabDev voc;
  int n_frames, stride, levelsup;
  int lds_m;  // next power of two >= stride (assembly LDS sizing)
  const uint8_t* descs;  // [n_frames][stride][32]
  const int* n;          // features per frame
  // per-feature scratch [n_frames][stride]
  uint32_t* f_word;
  double* f_weight;
  uint32_t* f_nid;
  // outputs, per frame at f * stride (fv_offsets at f * (stride + 1))
  uint32_t* bow_words;
  double* bow_weights;
  int* n_words;
  uint32_t* fv_nodes;
  int32_t* fv_offsets;
  uint32_t* fv_features;
  int* n_nodes;
};

hipError_t launch_bow(const BowLaunch& a, hipStream_t st);

}  // namespace orbgpu
