// OrbExtractor over the gfx950 C ABI (see orb_extractor.h in this directory).
// Build with the reference's OpenCV and link liborbgpu.so; replaces
// src/cam/orb_feature/orb_extractor.cc in the reference's CMake source list.
#include "orb_extractor.h"

#include <cassert>
#include <cstdlib>
#include <cstring>
#include <stdexcept>

namespace ORB_SLAM_FUSION {

namespace {
const int kEdgeThreshold = 19;  // orb_extractor.cc:74
int device_from_env() {
  const char *s = std::getenv("ORBGPU_DEVICE");
  return s ? std::atoi(s) : 0;
}
}  // namespace

OrbExtractor::OrbExtractor(int num_feats, float scale_factor, int num_levs, int ini_th_fast,
                           int min_th_fast)
    : num_feats_(num_feats),
      scale_factor_(scale_factor),
      num_levs_(num_levs),
      ini_th_fast_(ini_th_fast),
      min_th_fast_(min_th_fast) {
  const orbgpu_orb_params p{num_feats, scale_factor, num_levs, ini_th_fast, min_th_fast};
  // EuRoC-sized workspace; other sizes re-plan on the first call.
  if (orbgpu_extractor_create(&p, device_from_env(), 752, 480, 1, &gpu_) != ORBGPU_OK)
    throw std::runtime_error("orbgpu_extractor_create failed");
  scale_factors_.resize(num_levs_);
  inv_scale_factors_.resize(num_levs_);
  lev_sigma_2_.resize(num_levs_);
  inv_lev_sigma_2_.resize(num_levs_);
  orbgpu_extractor_scales(gpu_, scale_factors_.data(), inv_scale_factors_.data(),
                          lev_sigma_2_.data(), inv_lev_sigma_2_.data());
  img_pyramid_.resize(num_levs_);
}

OrbExtractor::~OrbExtractor() { orbgpu_extractor_destroy(gpu_); }

int OrbExtractor::reserve_call(const cv::Mat &im) {
  assert(im.type() == CV_8UC1);
  const int cap = orbgpu_extractor_max_keypoints(gpu_, im.cols, im.rows);
  kp_buf_.resize(cap > 0 ? cap : 1);
  desc_buf_.create(cap > 0 ? cap : 1, 32, CV_8U);
  return cap;
}

void OrbExtractor::finish_call(int n, std::vector<cv::KeyPoint> &kps, cv::OutputArray descs) {
  kps = std::vector<cv::KeyPoint>(n);
  static_assert(sizeof(cv::KeyPoint) == sizeof(orbgpu_keypoint), "cv::KeyPoint layout");
  std::memcpy(kps.data(), kp_buf_.data(), sizeof(orbgpu_keypoint) * n);
  if (n == 0) {
    descs.release();
  } else {
    descs.create(n, 32, CV_8U);
    desc_buf_.rowRange(0, n).copyTo(descs.getMat());
  }

#ifndef ORBGPU_STEREO
  // img_pyramid_: host levels inside a REFLECT_101 frame (orb_extractor.cc:1098-1115).
  // Its only reader is Frame::ComputeStereoMatches; with the GPU stereo matcher
  // (frame_stereo_gpu.cc, ORBGPU_STEREO) the levels stay on the device.
  for (int l = 0; l < num_levs_; ++l) {
    const uint8_t *data;
    int w, h, s;
    if (orbgpu_extractor_pyramid_level(gpu_, l, &data, &w, &h, &s) != ORBGPU_OK)
      throw std::runtime_error("orbgpu_extractor_pyramid_level failed");
    cv::Mat tmp(h + 2 * kEdgeThreshold, w + 2 * kEdgeThreshold, CV_8U);
    cv::Mat lev(h, w, CV_8U, const_cast<uint8_t *>(data), s);
    cv::copyMakeBorder(lev, tmp, kEdgeThreshold, kEdgeThreshold, kEdgeThreshold,
                       kEdgeThreshold, cv::BORDER_REFLECT_101);
    img_pyramid_[l] = tmp(cv::Rect(kEdgeThreshold, kEdgeThreshold, w, h));
  }
#endif
}

int OrbExtractor::operator()(cv::InputArray img, cv::InputArray /*msk*/,
                             std::vector<cv::KeyPoint> &kps, cv::OutputArray descs,
                             std::vector<int> &lapping_areas) {
  if (img.empty()) return -1;
  cv::Mat im = img.getMat();
  const int cap = reserve_call(im);
  int n = 0, mono = 0;
  const int lap[2] = {lapping_areas.size() > 0 ? lapping_areas[0] : 0,
                      lapping_areas.size() > 1 ? lapping_areas[1] : 0};
  const orbgpu_status st =
      orbgpu_extract(gpu_, im.data, im.cols, im.rows, (int)im.step, lap, kp_buf_.data(),
                     desc_buf_.data, cap, &n, &mono);
  if (st != ORBGPU_OK) throw std::runtime_error("orbgpu_extract failed");
  finish_call(n, kps, descs);
  return mono;
}

std::pair<int, int> OrbExtractor::ExtractStereo(OrbExtractor &left, OrbExtractor &right, cv::InputArray im_left,
                                                cv::InputArray im_right, std::vector<cv::KeyPoint> &kps_left,
                                                cv::OutputArray descs_left, std::vector<cv::KeyPoint> &kps_right,
                                                cv::OutputArray descs_right, std::vector<int> &lapping_left,
                                                std::vector<int> &lapping_right) {
  if (im_left.empty() || im_right.empty() || im_left.size() != im_right.size() ||
      im_left.getMat().step != im_right.getMat().step)  // one geometry: otherwise one image at a time
    return {left(im_left, cv::Mat(), kps_left, descs_left, lapping_left),
            right(im_right, cv::Mat(), kps_right, descs_right, lapping_right)};
  cv::Mat iml = im_left.getMat(), imr = im_right.getMat();
  const int cap_l = left.reserve_call(iml), cap_r = right.reserve_call(imr);
  auto lap_of = [](const std::vector<int> &v, int (&l)[2]) {
    l[0] = v.size() > 0 ? v[0] : 0;
    l[1] = v.size() > 1 ? v[1] : 0;
  };
  int lap_l[2], lap_r[2];
  lap_of(lapping_left, lap_l);
  lap_of(lapping_right, lap_r);
  int n_l = 0, n_r = 0, mono_l = 0, mono_r = 0;
  if (orbgpu_extract_stereo(left.gpu_, right.gpu_, iml.data, imr.data, iml.cols, iml.rows, (int)iml.step, lap_l,
                            lap_r, left.kp_buf_.data(), left.desc_buf_.data, cap_l, &n_l, &mono_l,
                            right.kp_buf_.data(), right.desc_buf_.data, cap_r, &n_r, &mono_r) != ORBGPU_OK)
    throw std::runtime_error("orbgpu_extract_stereo failed");
  left.finish_call(n_l, kps_left, descs_left);
  right.finish_call(n_r, kps_right, descs_right);
  return {mono_l, mono_r};
}

void OrbExtractor::ComputePyramid(cv::Mat img) {
  // Public in the reference (test_compute_pyramid.cc); runs the GPU path and
  // keeps only the pyramid.
  std::vector<cv::KeyPoint> k;
  cv::Mat d;
  std::vector<int> lap = {0, 0};
  (*this)(img, cv::Mat(), k, d, lap);
}

}  // namespace ORB_SLAM_FUSION
