// ORACLE (test infrastructure only; only tests/, __graft_entry__.smoke() and
// bench.py's cpu_baseline leg may load it -- never the product path).
//
// CPU restatement of ORB_SLAM_FUSION::OrbExtractor (include/cam/orb_feature/
// orb_extractor.h:44-104, src/cam/orb_feature/orb_extractor.cc:72-1117):
// pyramid -> per-cell FAST with threshold fallback -> octree distribution ->
// IC_Angle -> 7x7 Gaussian -> steered BRIEF -> mono/stereo assembly.
// OpenCV primitives follow cv_semantics.h (OpenCV 4.5.4 rules, parity UNPINNED
// at that boundary); cosf/sinf follow glibc_sincosf.h (pinned exhaustively
// against the host libm); the sample-coordinate FMA contraction follows what
// GCC 11.4 -O2 -march=native emits for orb_extractor.cc:111-113 (checked by
// tests/test_oracle_cpu.py::test_get_value_contraction).
#pragma once
#include <cstddef>
#include <cstdint>
#include <list>
#include <vector>

namespace oracle {

// Field order of cv::KeyPoint (28 bytes).
struct KeyPoint {
  float x, y, size, angle, response;
  int octave, class_id;
};

struct Plane {
  int w = 0, h = 0;
  std::vector<uint8_t> px;  // packed rows, stride == w
  const uint8_t* row(int y) const { return px.data() + (size_t)y * w; }
};

class OrbExtractor {
 public:
  OrbExtractor(int num_feats, float scale_factor, int num_levs, int ini_th_fast,
               int min_th_fast);

  // orb_extractor.cc:1011-1091.  Returns the mono index (-1 on empty input).
  int Extract(const uint8_t* img, int w, int h, int stride, std::vector<KeyPoint>& kps,
              std::vector<uint8_t>& descs, const int lapping[2]);

  void ComputePyramid(const uint8_t* img, int w, int h, int stride);  // :1093-1117

  int GetLevels() const { return num_levs_; }
  float GetScaleFactor() const { return (float)scale_factor_; }
  const std::vector<float>& GetScaleFactors() const { return scale_factors_; }
  const std::vector<float>& GetInverseScaleFactors() const { return inv_scale_factors_; }
  const std::vector<float>& GetScaleSigmaSquares() const { return lev_sigma_2_; }
  const std::vector<float>& GetInverseScaleSigmaSquares() const { return inv_lev_sigma_2_; }
  const std::vector<int>& FeaturesPerLevel() const { return num_feats_per_lev_; }
  const std::vector<int>& UMax() const { return umax_; }

  std::vector<Plane> img_pyramid_;
  std::vector<Plane> blurred_;  // per level, filled by Extract (stage dump)
  // Stage dumps of the last Extract, per level (coordinates relative to the
  // 16-px FAST border, exactly as the reference holds them before :837-838).
  std::vector<std::vector<KeyPoint>> to_dist_;
  std::vector<std::vector<KeyPoint>> octree_;

 private:
  struct Node {
    std::vector<KeyPoint> kps;
    int ulx = 0, uly = 0, urx = 0, ury = 0, blx = 0, bly = 0, brx = 0, bry = 0;
    std::list<Node>::iterator self;
    bool no_more = false;
    void Divide(Node& n1, Node& n2, Node& n3, Node& n4) const;
  };

  void ComputeKeyPointsOctTree(std::vector<std::vector<KeyPoint>>& all_kps);
  std::vector<KeyPoint> DistributeOctTree(const std::vector<KeyPoint>& kps, int min_x,
                                          int max_x, int min_y, int max_y, int num_feats);

  int num_feats_;
  double scale_factor_;
  int num_levs_, ini_th_fast_, min_th_fast_;
  std::vector<int> num_feats_per_lev_, umax_;
  std::vector<float> scale_factors_, inv_scale_factors_, lev_sigma_2_, inv_lev_sigma_2_;
  std::vector<int8_t> pattern_;  // 256 x (x0, y0, x1, y1)
};

// Stand-alone pieces, exposed for stage-level tests.
float IcAngle(const Plane& img, int cx, int cy, const std::vector<int>& umax);
void OrbDescriptor(const Plane& blurred, int cx, int cy, float angle_deg,
                   const int8_t* pattern, uint8_t desc[32]);

}  // namespace oracle
