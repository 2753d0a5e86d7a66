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
#include <vector>

#include "cam/orb_feature/orb_extractor.h"
#include "map/frame.h"
#include "orbgpu.h"

namespace ORB_SLAM_FUSION {

void Frame::ComputeStereoMatches() {
  mvuRight = std::vector<float>(N, -1.0f);
  mvDepth = std::vector<float>(N, -1.0f);
  if (N == 0) return;
  if (orbgpu_stereo_match(orb_extractor_left_->gpu(), orb_extractor_right_->gpu(), bf_, mb,
                          mvuRight.data(), mvDepth.data(), N) != ORBGPU_OK)
    throw std::runtime_error("orbgpu_stereo_match failed");
}

}  // namespace ORB_SLAM_FUSION
