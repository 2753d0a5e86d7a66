// ORACLE (test infrastructure only): CPU restatement of
// Frame::ComputeStereoMatches (src/map/frame.cc:828-986) over the oracle
// extractor's outputs.  Only tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg use it, as the checker.
//
// Semantics kept from the reference (file:line in frame.cc):
//   * right keypoints are listed on every row in [floor(y - 2 s), ceil(y + 2 s)]
//     with s = scale of their octave (:840-849); rows outside the level-0 image
//     are dropped (the reference would index out of its row table there);
//   * a left keypoint scans the list of row (size_t)y (:864) for octaves within
//     +-1 and uR in [uL - maxD, uL] (:868-893), maxD = bf / mb (:851-854); best
//     = first strict minimum of the Hamming distance, start TH_HIGH = 100;
//   * match accepted for dist < (TH_HIGH + TH_LOW) / 2 = 75 (:832, :896);
//   * 11x11 L1 window search over incR in [-5, 5] on the octave's level of the
//     left and right pyramids at round()ed scaled coordinates (:898-935); the
//     window may reach the +19 px reflect-101 border of the reference's padded
//     pyramid storage (orb_extractor.cc:1105-1114), read here by reflection;
//   * rejection at the sweep ends, parabola fit, |deltaR| <= 1 (:937-948);
//   * disparity in [0, maxD) with the 0.01 clamp (bestuR = uL - 0.01 in
//     double) (:950-962);
//   * median filter: drop every match whose window distance is >= 1.5f * 1.4f *
//     median of the kept distances (:965-980).  An empty match list (the
//     reference reads vDistIdx[0] of an empty vector) leaves everything as is.
// Float operations are written in the reference's order; none of them is
// affected by FMA contraction (every product in an add is an exact *2).
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <utility>
#include <vector>

namespace {

struct Kp {  // cv::KeyPoint layout
  float x, y, size, angle, response;
  int32_t octave, class_id;
};

// ORBmatcher::DescriptorDistance (orb_matcher.cc:1877-1891)
int desc_dist(const uint8_t* a, const uint8_t* b) {
  int d = 0;
  for (int i = 0; i < 8; ++i) {
    uint32_t pa, pb;
    __builtin_memcpy(&pa, a + 4 * i, 4);
    __builtin_memcpy(&pb, b + 4 * i, 4);
    uint32_t v = pa ^ pb;
    v = v - ((v >> 1) & 0x55555555u);
    v = (v & 0x33333333u) + ((v >> 2) & 0x33333333u);
    d += (int)((((v + (v >> 4)) & 0xF0F0F0Fu) * 0x1010101u) >> 24);
  }
  return d;
}

inline int reflect101(int i, int n) {
  i = i < 0 ? -i : i;
  return i >= n ? 2 * n - 2 - i : i;
}

struct Plane {
  const uint8_t* p;
  int w, h, stride;
  int at(int x, int y) const { return p[(size_t)reflect101(y, h) * stride + reflect101(x, w)]; }
};

}  // namespace

extern "C" int orc_stereo_match(const Kp* kl, int nl, const uint8_t* dl, const Kp* kr, int nr,
                                const uint8_t* dr, const float* scale, const float* inv_scale,
                                const uint8_t* const* pyr_l, const uint8_t* const* pyr_r,
                                const int* lw, const int* lh, const int* stride_l,
                                const int* stride_r, float bf,
                                float mb, float* uright, float* depth) {
  constexpr int kThHigh = 100, kThLow = 50;
  const int thOrbDist = (kThHigh + kThLow) / 2;
  for (int i = 0; i < nl; ++i) uright[i] = -1.0f, depth[i] = -1.0f;
  const int nRows = lh[0];
  std::vector<std::vector<int>> rows(nRows);
  for (int iR = 0; iR < nr; ++iR) {
    const float kpY = kr[iR].y;
    const float r = 2.0f * scale[kr[iR].octave];
    const int maxr = (int)std::ceil(kpY + r);
    const int minr = (int)std::floor(kpY - r);
    for (int yi = minr; yi <= maxr; ++yi)
      if (yi >= 0 && yi < nRows) rows[yi].push_back(iR);
  }
  const float minZ = mb, minD = 0;
  const float maxD = bf / minZ;
  std::vector<std::pair<int, int>> dist_idx;
  for (int iL = 0; iL < nl; ++iL) {
    const Kp& kpL = kl[iL];
    const int levelL = kpL.octave;
    const float vL = kpL.y, uL = kpL.x;
    const size_t row = (size_t)vL;
    if (row >= (size_t)nRows || rows[row].empty()) continue;
    const float minU = uL - maxD, maxU = uL - minD;
    if (maxU < 0) continue;
    int bestDist = kThHigh;
    int bestIdxR = 0;
    for (int iR : rows[row]) {
      const Kp& kpR = kr[iR];
      if (kpR.octave < levelL - 1 || kpR.octave > levelL + 1) continue;
      const float uR = kpR.x;
      if (uR >= minU && uR <= maxU) {
        const int dist = desc_dist(dl + 32 * (size_t)iL, dr + 32 * (size_t)iR);
        if (dist < bestDist) {
          bestDist = dist;
          bestIdxR = iR;
        }
      }
    }
    if (bestDist >= thOrbDist) continue;
    const float uR0 = kr[bestIdxR].x;
    const float scaleFactor = inv_scale[levelL];
    const float scaleduL = std::round(kpL.x * scaleFactor);
    const float scaledvL = std::round(kpL.y * scaleFactor);
    const float scaleduR0 = std::round(uR0 * scaleFactor);
    const int w = 5, L = 5;
    const float iniu = scaleduR0 + L - w;
    const float endu = scaleduR0 + L + w + 1;
    if (iniu < 0 || endu >= lw[levelL]) continue;
    const Plane PL{pyr_l[levelL], lw[levelL], lh[levelL], stride_l[levelL]};
    const Plane PR{pyr_r[levelL], lw[levelL], lh[levelL], stride_r[levelL]};
    const int yl = (int)scaledvL, xl = (int)scaleduL, xr = (int)scaleduR0;
    int sadBest = INT_MAX, bestincR = 0;
    float dists[2 * L + 1];
    for (int incR = -L; incR <= L; ++incR) {
      int s = 0;
      for (int dy = -w; dy <= w; ++dy)
        for (int dx = -w; dx <= w; ++dx)
          s += std::abs(PL.at(xl + dx, yl + dy) - PR.at(xr + incR + dx, yl + dy));
      const float dist = (float)(double)s;  // cv::norm returns double
      if (dist < sadBest) {
        sadBest = (int)dist;
        bestincR = incR;
      }
      dists[L + incR] = dist;
    }
    if (bestincR == -L || bestincR == L) continue;
    const float dist1 = dists[L + bestincR - 1];
    const float dist2 = dists[L + bestincR];
    const float dist3 = dists[L + bestincR + 1];
    const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
    if (deltaR < -1 || deltaR > 1) continue;
    float bestuR = scale[levelL] * ((float)scaleduR0 + (float)bestincR + deltaR);
    float disparity = uL - bestuR;
    if (disparity >= minD && disparity < maxD) {
      if (disparity <= 0) {
        disparity = 0.01;
        bestuR = (float)((double)uL - 0.01);
      }
      depth[iL] = bf / disparity;
      uright[iL] = bestuR;
      dist_idx.emplace_back(sadBest, iL);
    }
  }
  if (dist_idx.empty()) return 0;
  std::sort(dist_idx.begin(), dist_idx.end());
  const float median = (float)dist_idx[dist_idx.size() / 2].first;
  const float thDist = 1.5f * 1.4f * median;
  int kept = (int)dist_idx.size();
  for (int i = (int)dist_idx.size() - 1; i >= 0; --i) {
    if (dist_idx[i].first < thDist) break;
    uright[dist_idx[i].second] = -1;
    depth[dist_idx[i].second] = -1;
    --kept;
  }
  return kept;
}
