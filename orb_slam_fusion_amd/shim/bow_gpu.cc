// Frame::ComputeBoW / KeyFrame::ComputeBoW over the gfx950 C ABI.
// Compiled inside the reference build; the originals (frame.cc:761-766,
// keyframe.cc:202-209) are guarded with ORBGPU_BOW.
// Same effect as mpORBvocabulary->transform(descriptors, mBowVec, mFeatVec, 4):
// the GPU holds its own copy of the vocabulary, loaded once per process from
// the same ORBvoc.txt the System loads (path in the ORBGPU_VOCAB environment
// variable; the DBoW2 object does not keep its file name).  KeyFrame::ComputeBoW
// runs on LocalMapping / LoopClosing threads and Frame::ComputeBoW on Tracking,
// so the vocabulary (read-only) is shared and each thread takes a lock only
// for the device call.
#include <cstdlib>
#include <mutex>
#include <stdexcept>
#include <vector>

#include "map/frame.h"
#include "map/keyframe.h"
#include "orbgpu.h"

namespace ORB_SLAM_FUSION {

namespace {

std::mutex g_bow_mutex;

orbgpu_vocab* gpu_vocab() {
  static orbgpu_vocab* v = [] {
    const char* path = std::getenv("ORBGPU_VOCAB");
    if (!path) throw std::runtime_error("ORBGPU_VOCAB is not set (path of ORBvoc.txt)");
    orbgpu_vocab* p = nullptr;
    if (orbgpu_vocab_load_text(0, path, &p) != ORBGPU_OK)
      throw std::runtime_error("orbgpu_vocab_load_text failed");
    return p;
  }();
  return v;
}

void compute_bow(const cv::Mat& desc, DBoW2::BowVector& bow, DBoW2::FeatureVector& fv) {
  const int n = desc.rows;
  std::vector<uint32_t> words(n), nodes(n), feats(n);
  std::vector<double> weights(n);
  std::vector<int32_t> offs(n + 1);
  int nw = 0, nn = 0;
  {
    std::lock_guard<std::mutex> lock(g_bow_mutex);
    if (orbgpu_bow_transform(gpu_vocab(), n > 0 ? desc.ptr<uint8_t>(0) : nullptr, n, 4,
                             words.data(), weights.data(), &nw, nodes.data(), offs.data(),
                             feats.data(), &nn) != ORBGPU_OK)
      throw std::runtime_error("orbgpu_bow_transform failed");
  }
  bow.clear();
  fv.clear();
  for (int i = 0; i < nw; ++i) bow.insert(bow.end(), {words[i], weights[i]});
  for (int j = 0; j < nn; ++j)
    fv.insert(fv.end(), {nodes[j], std::vector<unsigned int>(feats.begin() + offs[j],
                                                             feats.begin() + offs[j + 1])});
}

}  // namespace

void Frame::ComputeBoW() {
  if (mBowVec.empty()) compute_bow(mDescriptors, mBowVec, mFeatVec);
}

void KeyFrame::ComputeBoW() {
  if (mBowVec.empty() || mFeatVec.empty()) compute_bow(mDescriptors, mBowVec, mFeatVec);
}

}  // namespace ORB_SLAM_FUSION
