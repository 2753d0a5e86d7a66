// Drop-in replacement header for include/cam/orb_feature/orb_extractor.h of
// J094/orb_slam_fusion: the same class, members and signatures
// (orb_extractor.h:29-104), implemented over the gfx950 C ABI (orbgpu.h).
// Compiled only in a build that has OpenCV (the reference's own dependency);
// frame.cc / tracking.cc include it unchanged.
#ifndef ORBEXTRACTOR_H
#define ORBEXTRACTOR_H

#include <list>
#include <utility>
#include <opencv2/opencv.hpp>
#include <vector>

#include "orbgpu.h"

namespace ORB_SLAM_FUSION {

class ExtractorNode {  // kept for source compatibility (orb_extractor.h:31-42)
 public:
  ExtractorNode() : no_more_(false) {}
  void DivideNode(ExtractorNode &n_1, ExtractorNode &n_2, ExtractorNode &n_3,
                  ExtractorNode &n_4);
  std::vector<cv::KeyPoint> kps_;
  cv::Point2i UL_, UR_, BL_, BR_;
  std::list<ExtractorNode>::iterator lit_;
  bool no_more_;
};

class OrbExtractor {
 public:
  enum { kHarrisScore = 0, kFastScore = 1 };

  OrbExtractor(int num_feats, float scale_factor, int num_levs, int ini_th_fast,
               int min_th_fast);
  ~OrbExtractor();

  // Same contract as orb_extractor.cc:1011-1091: returns the mono index, -1 on
  // an empty image; asserts CV_8UC1; the mask is ignored.
  int operator()(cv::InputArray img, cv::InputArray msk, std::vector<cv::KeyPoint> &kps,
                 cv::OutputArray descs, std::vector<int> &lapping_areas);

  int inline GetLevels() { return num_levs_; }
  float inline GetScaleFactor() { return scale_factor_; }
  std::vector<float> inline GetScaleFactors() { return scale_factors_; }
  std::vector<float> inline GetInverseScaleFactors() { return inv_scale_factors_; }
  std::vector<float> inline GetScaleSigmaSquares() { return lev_sigma_2_; }
  std::vector<float> inline GetInverseScaleSigmaSquares() { return inv_lev_sigma_2_; }

  // Host levels of the last call (each a ROI inside a 19-px REFLECT_101
  // frame, as ComputePyramid leaves them); read by Frame::ComputeStereoMatches.
  std::vector<cv::Mat> img_pyramid_;

  void ComputePyramid(cv::Mat img);

  // Both images of a stereo frame from the calling thread (orbgpu_extract_stereo):
  // left's operator() on im_left and right's on im_right, both launches in
  // flight together.  Returns {left mono index, right mono index}; used by the
  // stereo Frame constructor in place of its two ExtractORB threads
  // (frame.cc:179-182, frame_stereo_gpu.cc).
  static std::pair<int, int> ExtractStereo(OrbExtractor &left, OrbExtractor &right, cv::InputArray im_left,
                                           cv::InputArray im_right, std::vector<cv::KeyPoint> &kps_left,
                                           cv::OutputArray descs_left, std::vector<cv::KeyPoint> &kps_right,
                                           cv::OutputArray descs_right, std::vector<int> &lapping_left,
                                           std::vector<int> &lapping_right);

  // The device handle (frame_stereo_gpu.cc matches on its resident outputs).
  orbgpu_extractor *gpu() const { return gpu_; }

 protected:
  int num_feats_;
  double scale_factor_;
  int num_levs_;
  int ini_th_fast_;
  int min_th_fast_;
  std::vector<float> scale_factors_;
  std::vector<float> inv_scale_factors_;
  std::vector<float> lev_sigma_2_;
  std::vector<float> inv_lev_sigma_2_;

 private:
  // the call's outputs from kp_buf_ / desc_buf_ (and img_pyramid_ without ORBGPU_STEREO)
  void finish_call(int n, std::vector<cv::KeyPoint> &kps, cv::OutputArray descs);
  int reserve_call(const cv::Mat &im);  // sizes the buffers; returns the keypoint capacity

  orbgpu_extractor *gpu_ = nullptr;
  std::vector<orbgpu_keypoint> kp_buf_;
  cv::Mat desc_buf_;
};

}  // namespace ORB_SLAM_FUSION

#endif
