// Frame::ComputeStereoMatches over the gfx950 C ABI.
// Compiled inside the reference build (include paths of frame.h / the shim
// orb_extractor.h); the original definition in src/map/frame.cc:828-986 is
// guarded with ORBGPU_STEREO.  The stereo Frame
// constructor calls it right after ExtractORB on both images
// (frame.cc:179-189), so the two extractors' handles still hold this frame's
// keypoints, descriptors and pyramids on the device: the match runs there
// (no img_pyramid_ download; the extractor shim skips it under
// ORBGPU_STEREO) and only mvuRight / mvDepth come back.
#include <stdexcept>
#include <utility>
#include <vector>

#include "cam/orb_feature/orb_extractor.h"
#include "map/frame.h"
#include "orbgpu.h"

namespace ORB_SLAM_FUSION {

// The stereo constructors' extraction (frame.cc:179-182 and, with the
// KannalaBrandt8 lapping areas, :1076-1084 start a std::thread per image to
// run ExtractORB(0 / 1, ...)): under ORBGPU_STEREO the guarded blocks call
// this instead -- both images from the tracking thread, both launches in
// flight together (orbgpu_extract_stereo); the same members are written as by
// the two ExtractORB calls (:467-476).
void Frame::ExtractORBStereo(const cv::Mat &imLeft, const cv::Mat &imRight, int x0_left, int x1_left,
                             int x0_right, int x1_right) {
  vector<int> lap_left = {x0_left, x1_left}, lap_right = {x0_right, x1_right};
  const std::pair<int, int> mono =
      OrbExtractor::ExtractStereo(*orb_extractor_left_, *orb_extractor_right_, imLeft, imRight, mvKeys, mDescriptors,
                                  mvKeysRight, mDescriptorsRight, lap_left, lap_right);
  monoLeft = mono.first;
  monoRight = mono.second;
}

void Frame::ComputeStereoMatches() {
  mvuRight = std::vector<float>(N, -1.0f);
  mvDepth = std::vector<float>(N, -1.0f);
  if (N == 0) return;
  if (orbgpu_stereo_match(orb_extractor_left_->gpu(), orb_extractor_right_->gpu(), bf_, mb,
                          mvuRight.data(), mvDepth.data(), N) != ORBGPU_OK)
    throw std::runtime_error("orbgpu_stereo_match failed");
}

}  // namespace ORB_SLAM_FUSION
