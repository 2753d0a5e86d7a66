// ORACLE (test infrastructure only): CPU restatement of the ORBmatcher
// projection searches that feed PoseOptimization in tracking, for the pinhole
// rig (Frame::Nleft == -1).  Only tests/ and bench.py's side lines use it, as
// the checker.
//
// Restated functions (reference file:line):
//   * Frame::AssignFeaturesToGrid / PosInGrid (frame.cc:438-465, 748-759),
//     Frame::GetFeaturesInArea (frame.cc:679-746): grid order ix, iy, then the
//     cell's keypoints in increasing index;
//   * Frame::isInFrustum (frame.cc:548-603) and MapPoint::PredictScale
//     (mappoint.cc:550-563), GetMin/MaxDistanceInvariance (:524-532);
//   * ORBmatcher::SearchByProjection(Frame&, const vector<MapPoint*>&, th,
//     bFarPoints, thFarPoints) (orb_matcher.cc:42-206), RadiusByViewingCos
//     (:208-213);
//   * ORBmatcher::SearchByProjection(Frame& CurrentFrame, const Frame&
//     LastFrame, th, bMono) (orb_matcher.cc:1518-1728), ComputeThreeMaxima
//     (:1841-1873), DescriptorDistance (:1877-1891);
//   * ORBmatcher::SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF,
//     const set<MapPoint*>& sAlreadyFound, th, ORBdist) (orb_matcher.cc:
//     1730-1839), Relocalization's search;
//   * ORBmatcher::SearchByBoW(KeyFrame* pKF, Frame& F, vector<MapPoint*>&)
//     (orb_matcher.cc:215-389), over the two DBoW2 FeatureVectors.
//
// Float arithmetic: the reference is g++ -O2 -march=native C++ (contraction
// on in C++ dialects), so Eigen / Sophus sums of products are fused.  The
// restatement writes every fusion explicitly, following what GCC 11.4 emits
// for the same scalar expressions (tests/test_match_cpu.py compiles them and
// checks the vfmadd/vfmsub/vfnmadd pattern): in a + b*c the product is fused;
// in a*b + c*d (and a*b - c*d) the FIRST product is fused and the second
// rounded.  Eigen itself is absent here, so the expression order inside
// Eigen's small fixed-size kernels (3x3 * 3, norm, dot, cross, Quaternion
// normalize) is restated from Eigen 3.3's scalar (non-SIMD) code paths; that
// boundary is parity-unpinned.  Everything else (grid, order of candidates,
// ties, claims, ratio test, histogram) is integer / compare logic restated
// exactly.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace {

constexpr int kGridCols = 64, kGridRows = 48;  // frame.h:40-41
constexpr int kThHigh = 100;                   // orb_matcher.cc:35
constexpr int kHistoLength = 30;               // orb_matcher.cc:37

struct Kp {  // cv::KeyPoint layout
  float x, y, size, angle, response;
  int32_t octave, class_id;
};

struct Geom {  // orbgpu_frame_geom
  float min_x, max_x, min_y, max_y;
  int32_t n_levels;
  float log_scale;
  float scale[16];
};

struct Cam {
  float fx, fy, cx, cy, bf;
};

struct ProjPoint {  // orbgpu_proj_point
  float Xw[3];
  int32_t octave;
  float angle;
  int32_t has_obs;
  uint8_t desc[32];
};

struct MapPt {  // orbgpu_map_point
  float Xw[3], normal[3];
  float min_dist, max_dist;
  int32_t flags;
  uint8_t desc[32];
};

struct View {  // orbgpu_track_view
  int32_t in_view, level;
  float proj_x, proj_y, proj_xr, depth, view_cos;
};

int desc_dist(const uint8_t* a, const uint8_t* b) {  // orb_matcher.cc:1877-1891
  int d = 0;
  for (int i = 0; i < 8; ++i) {
    uint32_t pa, pb;
    std::memcpy(&pa, a + 4 * i, 4);
    std::memcpy(&pb, b + 4 * i, 4);
    uint32_t v = pa ^ pb;
    v = v - ((v >> 1) & 0x55555555u);
    v = (v & 0x33333333u) + ((v >> 2) & 0x33333333u);
    d += (int)((((v + (v >> 4)) & 0xF0F0F0Fu) * 0x1010101u) >> 24);
  }
  return d;
}

// --- Sophus / Eigen float kernels (contracted as GCC does) -----------------
struct V3 {
  float x, y, z;
};

// a*b - c*d -> fma(a, b, -(c*d))
inline float mul_sub(float a, float b, float c, float d) { return std::fmaf(a, b, -(c * d)); }

V3 cross(const V3& a, const V3& b) {
  return {mul_sub(a.y, b.z, a.z, b.y), mul_sub(a.z, b.x, a.x, b.z), mul_sub(a.x, b.y, a.y, b.x)};
}

// Sophus::SO3::operator*(p) (so3.hpp:359-367): uv = 2 (q.vec x p);
// p + w uv + q.vec x uv -> fma(w, uv, p) + cross
V3 quat_rotate(const float q[4], const V3& p) {  // q = (x, y, z, w)
  const V3 qv{q[0], q[1], q[2]};
  V3 uv = cross(qv, p);
  uv = {uv.x + uv.x, uv.y + uv.y, uv.z + uv.z};
  const V3 c = cross(qv, uv);
  return {std::fmaf(q[3], uv.x, p.x) + c.x, std::fmaf(q[3], uv.y, p.y) + c.y,
          std::fmaf(q[3], uv.z, p.z) + c.z};
}

// Sophus::SE3::operator*(p) = so3() * p + translation() (se3.hpp:321-324)
V3 se3_apply(const float* pose7, const V3& p) {
  const V3 r = quat_rotate(pose7, p);
  return {r.x + pose7[4], r.y + pose7[5], r.z + pose7[6]};
}

// Tcw.inverse().translation() (se3.hpp:208-211): the conjugate quaternion is
// renormalised by SO3's constructor (so3.hpp:482-488, normalize :298-304).
// Eigen's 4-float squaredNorm is a packet redux: (x^2 + z^2) + (y^2 + w^2).
V3 se3_inverse_translation(const float* pose7) {
  float q[4] = {-pose7[0], -pose7[1], -pose7[2], pose7[3]};
  const float s = (q[0] * q[0] + q[2] * q[2]) + (q[1] * q[1] + q[3] * q[3]);
  const float len = std::sqrt(s);
  for (float& c : q) c /= len;
  return quat_rotate(q, V3{-pose7[4], -pose7[5], -pose7[6]});
}

// Eigen Matrix3f * Vector3f + Vector3f (row i: fma(r2, z, fma(r0, x, r1*y)) + t)
V3 mat_apply(const float* R, const float* t, const V3& p) {
  V3 o;
  float* out = &o.x;
  for (int i = 0; i < 3; ++i) {
    const float* r = R + 3 * i;
    out[i] = std::fmaf(r[2], p.z, std::fmaf(r[0], p.x, r[1] * p.y)) + t[i];
  }
  return o;
}

// Eigen dot / squaredNorm over 3 floats: fma(a2, b2, fma(a0, b0, a1*b1))
inline float dot3(const V3& a, const V3& b) {
  return std::fmaf(a.z, b.z, std::fmaf(a.x, b.x, a.y * b.y));
}

// Pinhole::Project (pinhole_model.cc:45-50): fx * X / Z + cx
inline float project_u(const Cam& c, const V3& p) { return c.fx * p.x / p.z + c.cx; }
inline float project_v(const Cam& c, const V3& p) { return c.fy * p.y / p.z + c.cy; }

// MapPoint::PredictScale (mappoint.cc:550-563).  mappoint.cc has no
// using-directive and no <math.h> in its include closure, so the unqualified
// log() / ceil() there are ::log(double) / ::ceil(double): the float ratio is
// promoted and divided by the promoted float mfLogScaleFactor (itself
// logf(mfScaleFactor): frame.cc reaches the C++ <math.h> wrapper through
// g2o_types.h, which exports std::log(float)).  A non-finite ceil() converts
// to int as x86's cvttsd2si does (INT_MIN), i.e. level 0.
int level_of_ratio(float ratio, float log_scale, int n_levels) {
  const double c = std::ceil(std::log((double)ratio) / (double)log_scale);
  int n = std::isfinite(c) && std::fabs(c) < 2147483648.0 ? (int)c : INT32_MIN;
  if (n < 0) n = 0;
  else if (n >= n_levels) n = n_levels - 1;
  return n;
}

int predict_scale(float max_distance, float dist, float log_scale, int n_levels) {
  return level_of_ratio(max_distance / dist, log_scale, n_levels);
}

// --- Frame ------------------------------------------------------------------
struct Frame {
  const Geom* g;
  const Kp* kps;
  const uint8_t* desc;
  const float* uright;  // may be null
  int n;
  float inv_w, inv_h;  // mfGridElementWidthInv / HeightInv (frame.cc:201-204)
  std::vector<int> grid[kGridCols][kGridRows];
  // mvpMapPoints: -1 empty, -2 pre-existing with observations, >= 0 query
  std::vector<int> holder;
  std::vector<char> holder_obs;  // Observations() > 0 of the held point

  Frame(const Geom* g_, const Kp* k, const uint8_t* d, const float* ur, const uint8_t* claimed,
        int n_)
      : g(g_), kps(k), desc(d), uright(ur), n(n_) {
    inv_w = (float)kGridCols / (g->max_x - g->min_x);
    inv_h = (float)kGridRows / (g->max_y - g->min_y);
    holder.assign(n, -1);
    holder_obs.assign(n, 0);
    for (int i = 0; i < n; ++i)
      if (claimed && claimed[i]) holder[i] = -2, holder_obs[i] = 1;
    for (int i = 0; i < n; ++i) {  // AssignFeaturesToGrid
      int px, py;
      if (pos_in_grid(kps[i], px, py)) grid[px][py].push_back(i);
    }
  }

  bool pos_in_grid(const Kp& kp, int& px, int& py) const {  // frame.cc:748-759
    px = (int)std::round((kp.x - g->min_x) * inv_w);
    py = (int)std::round((kp.y - g->min_y) * inv_h);
    return !(px < 0 || px >= kGridCols || py < 0 || py >= kGridRows);
  }

  // frame.cc:679-746
  std::vector<int> features_in_area(float x, float y, float r, int min_level,
                                    int max_level) const {
    std::vector<int> out;
    const int nMinCellX = std::max(0, (int)std::floor((x - g->min_x - r) * inv_w));
    if (nMinCellX >= kGridCols) return out;
    const int nMaxCellX = std::min(kGridCols - 1, (int)std::ceil((x - g->min_x + r) * inv_w));
    if (nMaxCellX < 0) return out;
    const int nMinCellY = std::max(0, (int)std::floor((y - g->min_y - r) * inv_h));
    if (nMinCellY >= kGridRows) return out;
    const int nMaxCellY = std::min(kGridRows - 1, (int)std::ceil((y - g->min_y + r) * inv_h));
    if (nMaxCellY < 0) return out;
    const bool check_levels = (min_level >= 0) || (max_level >= 0);
    for (int ix = nMinCellX; ix <= nMaxCellX; ++ix)
      for (int iy = nMinCellY; iy <= nMaxCellY; ++iy)
        for (int idx : grid[ix][iy]) {
          const Kp& kp = kps[idx];
          if (check_levels) {
            if (kp.octave < min_level) continue;
            if (max_level >= 0 && kp.octave > max_level) continue;
          }
          const float dx = kp.x - x, dy = kp.y - y;
          if (std::fabs(dx) < r && std::fabs(dy) < r) out.push_back(idx);
        }
    return out;
  }

  bool blocked(int idx) const { return holder[idx] != -1 && holder_obs[idx]; }
};

// ComputeThreeMaxima (orb_matcher.cc:1841-1873)
void three_maxima(const std::vector<int>* histo, int& ind1, int& ind2, int& ind3) {
  int max1 = 0, max2 = 0, max3 = 0;
  ind1 = ind2 = ind3 = -1;
  for (int i = 0; i < kHistoLength; ++i) {
    const int s = (int)histo[i].size();
    if (s > max1) {
      max3 = max2, max2 = max1, max1 = s;
      ind3 = ind2, ind2 = ind1, ind1 = i;
    } else if (s > max2) {
      max3 = max2, max2 = s;
      ind3 = ind2, ind2 = i;
    } else if (s > max3) {
      max3 = s, ind3 = i;
    }
  }
  if (max2 < 0.1f * (float)max1) ind2 = ind3 = -1;
  else if (max3 < 0.1f * (float)max1) ind3 = -1;
}

void write_match(const Frame& F, const std::vector<char>& nulled, int32_t* match) {
  for (int i = 0; i < F.n; ++i)
    match[i] = nulled[i] ? -2 : (F.holder[i] >= 0 ? F.holder[i] : -1);
}

}  // namespace

extern "C" {

// ORBmatcher::SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame,
// th, bMono) -- orb_matcher.cc:1518-1728 (Nleft == -1 branches).
int orc_search_last(const Geom* g, const Cam* cam, float mb, const float* Tcw, const float* Tlw,
                    const Kp* kps, const uint8_t* desc, const float* uright,
                    const uint8_t* claimed, int n, const ProjPoint* pts, int n_pts, float th,
                    int mono, int check_ori, int32_t* match) {
  Frame F(g, kps, desc, uright, claimed, n);
  int nmatches = 0;
  std::vector<int> rot_hist[kHistoLength];
  const float factor = kHistoLength / 360.0f;
  const V3 twc = se3_inverse_translation(Tcw);
  const V3 tlc = se3_apply(Tlw, twc);
  const bool forward = tlc.z > mb && !mono;
  const bool backward = -tlc.z > mb && !mono;
  for (int i = 0; i < n_pts; ++i) {
    const ProjPoint& P = pts[i];
    const V3 x3Dc = se3_apply(Tcw, V3{P.Xw[0], P.Xw[1], P.Xw[2]});
    const float invzc = (float)(1.0 / (double)x3Dc.z);
    if (invzc < 0) continue;
    const float u = project_u(*cam, x3Dc), v = project_v(*cam, x3Dc);
    if (u < g->min_x || u > g->max_x) continue;
    if (v < g->min_y || v > g->max_y) continue;
    const int oct = P.octave;
    const float radius = th * g->scale[oct];
    std::vector<int> cand;
    if (forward) cand = F.features_in_area(u, v, radius, oct, -1);
    else if (backward) cand = F.features_in_area(u, v, radius, 0, oct);
    else cand = F.features_in_area(u, v, radius, oct - 1, oct + 1);
    if (cand.empty()) continue;
    int best = 256, best_idx = -1;
    for (int i2 : cand) {
      if (F.blocked(i2)) continue;
      if (uright && uright[i2] > 0) {
        const float ur = std::fmaf(-cam->bf, invzc, u);  // u - bf * invzc
        if (std::fabs(ur - uright[i2]) > radius) continue;
      }
      const int d = desc_dist(P.desc, desc + 32 * (size_t)i2);
      if (d < best) best = d, best_idx = i2;
    }
    if (best <= kThHigh) {
      F.holder[best_idx] = i;
      F.holder_obs[best_idx] = P.has_obs != 0;
      ++nmatches;
      if (check_ori) {
        float rot = P.angle - kps[best_idx].angle;
        if (rot < 0.0) rot += 360.0f;
        int bin = (int)std::round(rot * factor);
        if (bin == kHistoLength) bin = 0;
        rot_hist[bin].push_back(best_idx);
      }
    }
  }
  std::vector<char> nulled(n, 0);
  if (check_ori) {
    int i1, i2, i3;
    three_maxima(rot_hist, i1, i2, i3);
    for (int b = 0; b < kHistoLength; ++b) {
      if (b == i1 || b == i2 || b == i3) continue;
      for (int idx : rot_hist[b]) {
        F.holder[idx] = -1;
        nulled[idx] = 1;
        --nmatches;
      }
    }
  }
  write_match(F, nulled, match);
  return nmatches;
}

// ORBmatcher::SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th,
// ORBdist) -- orb_matcher.cc:1730-1839.  pts[i]: the key frame's point of
// keypoint i (flags & 1: NULL, isBad() or in sAlreadyFound); angles[i]:
// pKF->mvKeysUn[i].angle; claimed: CurrentFrame.mvpMapPoints[k] != NULL.
int orc_search_kf(const Geom* g, const Cam* cam, const float* Tcw, const Kp* kps,
                  const uint8_t* desc, const uint8_t* claimed, int n, const MapPt* pts,
                  const float* angles, int n_pts, float th, int orb_dist, int check_ori,
                  int32_t* match) {
  Frame F(g, kps, desc, nullptr, claimed, n);
  int nmatches = 0;
  std::vector<int> rot_hist[kHistoLength];
  const float factor = kHistoLength / 360.0f;
  const V3 Ow = se3_inverse_translation(Tcw);  // Tcw.inverse().translation()
  for (int i = 0; i < n_pts; ++i) {
    const MapPt& M = pts[i];
    if (M.flags & 1) continue;
    const V3 x3Dw{M.Xw[0], M.Xw[1], M.Xw[2]};
    const V3 x3Dc = se3_apply(Tcw, x3Dw);
    const float u = project_u(*cam, x3Dc), v = project_v(*cam, x3Dc);
    if (u < g->min_x || u > g->max_x) continue;
    if (v < g->min_y || v > g->max_y) continue;
    const V3 PO{x3Dw.x - Ow.x, x3Dw.y - Ow.y, x3Dw.z - Ow.z};
    const float dist3D = std::sqrt(dot3(PO, PO));
    const float maxD = 1.2f * M.max_dist, minD = 0.8f * M.min_dist;  // mappoint.cc:524-532
    if (dist3D < minD || dist3D > maxD) continue;
    const int level = predict_scale(M.max_dist, dist3D, g->log_scale, g->n_levels);
    const float radius = th * g->scale[level];
    const std::vector<int> cand = F.features_in_area(u, v, radius, level - 1, level + 1);
    if (cand.empty()) continue;
    int best = 256, best_idx = -1;
    for (int i2 : cand) {
      if (F.holder[i2] != -1) continue;  // CurrentFrame.mvpMapPoints[i2]
      const int d = desc_dist(M.desc, desc + 32 * (size_t)i2);
      if (d < best) best = d, best_idx = i2;
    }
    if (best <= orb_dist) {
      F.holder[best_idx] = i;
      F.holder_obs[best_idx] = 1;
      ++nmatches;
      if (check_ori) {
        float rot = angles[i] - kps[best_idx].angle;
        if (rot < 0.0) rot += 360.0f;
        int bin = (int)std::round(rot * factor);
        if (bin == kHistoLength) bin = 0;
        rot_hist[bin].push_back(best_idx);
      }
    }
  }
  std::vector<char> nulled(n, 0);
  if (check_ori) {
    int i1, i2, i3;
    three_maxima(rot_hist, i1, i2, i3);
    for (int b = 0; b < kHistoLength; ++b) {
      if (b == i1 || b == i2 || b == i3) continue;
      for (int idx : rot_hist[b]) {
        F.holder[idx] = -1;
        nulled[idx] = 1;
        --nmatches;
      }
    }
  }
  write_match(F, nulled, match);
  return nmatches;
}

// ORBmatcher::SearchByBoW(KeyFrame* pKF, Frame& F, vector<MapPoint*>&
// vpMapPointMatches) -- orb_matcher.cc:215-389, Nleft == -1.  FeatureVectors
// as ascending node ids with CSR feature lists (node j: features
// [off[j], off[j + 1])); kf_valid[i]: vpMapPointsKF[i] && !isBad(); angles:
// pKF->mvKeysUn[i].angle / F.mvKeys[k].angle.  match[k] = the key-frame index
// whose point F's keypoint k receives, -1 none (vpMapPointMatches starts all
// NULL).  The right-camera branch never fires for Nleft == -1 (its best
// distance stays 256).
int orc_search_bow(const uint32_t* kf_nodes, const int32_t* kf_off, const uint32_t* kf_feat,
                   int kf_n_nodes, const uint8_t* kf_desc, const float* kf_angle,
                   const uint8_t* kf_valid, const uint32_t* f_nodes, const int32_t* f_off,
                   const uint32_t* f_feat, int f_n_nodes, const uint8_t* f_desc,
                   const float* f_angle, int f_n, float nn_ratio, int check_ori, int32_t* match) {
  constexpr int kThLow = 50;  // orb_matcher.cc:36
  for (int k = 0; k < f_n; ++k) match[k] = -1;
  int nmatches = 0;
  std::vector<int> rot_hist[kHistoLength];
  const float factor = kHistoLength / 360.0f;
  int a = 0, b = 0;
  while (a < kf_n_nodes && b < f_n_nodes) {
    if (kf_nodes[a] == f_nodes[b]) {
      for (int ia = kf_off[a]; ia < kf_off[a + 1]; ++ia) {
        const int realIdxKF = (int)kf_feat[ia];
        if (!kf_valid[realIdxKF]) continue;
        int best1 = 256, best_idx = -1, best2 = 256;
        for (int ib = f_off[b]; ib < f_off[b + 1]; ++ib) {
          const int realIdxF = (int)f_feat[ib];
          if (match[realIdxF] >= 0) continue;
          const int d = desc_dist(kf_desc + 32 * (size_t)realIdxKF, f_desc + 32 * (size_t)realIdxF);
          if (d < best1) {
            best2 = best1;
            best1 = d;
            best_idx = realIdxF;
          } else if (d < best2) {
            best2 = d;
          }
        }
        if (best1 <= kThLow && (float)best1 < nn_ratio * (float)best2) {
          match[best_idx] = realIdxKF;
          if (check_ori) {
            float rot = kf_angle[realIdxKF] - f_angle[best_idx];
            if (rot < 0.0) rot += 360.0f;
            int bin = (int)std::round(rot * factor);
            if (bin == kHistoLength) bin = 0;
            rot_hist[bin].push_back(best_idx);
          }
          ++nmatches;
        }
      }
      ++a;
      ++b;
    } else if (kf_nodes[a] < f_nodes[b]) {  // KFit = vFeatVecKF.lower_bound(Fit->first)
      a = (int)(std::lower_bound(kf_nodes + a, kf_nodes + kf_n_nodes, f_nodes[b]) - kf_nodes);
    } else {
      b = (int)(std::lower_bound(f_nodes + b, f_nodes + f_n_nodes, kf_nodes[a]) - f_nodes);
    }
  }
  if (check_ori) {
    int i1, i2, i3;
    three_maxima(rot_hist, i1, i2, i3);
    for (int bn = 0; bn < kHistoLength; ++bn) {
      if (bn == i1 || bn == i2 || bn == i3) continue;
      for (int idx : rot_hist[bn]) {
        match[idx] = -1;
        --nmatches;
      }
    }
  }
  return nmatches;
}

// Frame::isInFrustum (frame.cc:548-603) over SearchLocalPoints' loop
// (tracking.cc:2644-2661).  Only the fields the reference writes are written.
void orc_frustum(const Geom* g, const Cam* cam, const float* Rcw, const float* tcw,
                 const float* Ow, const MapPt* pts, int n_pts, float cos_limit, View* views) {
  for (int j = 0; j < n_pts; ++j) {
    const MapPt& M = pts[j];
    View& V = views[j];
    V.in_view = 0;
    if (M.flags & 1) continue;
    V.proj_x = -1, V.proj_y = -1;
    const V3 P{M.Xw[0], M.Xw[1], M.Xw[2]};
    const V3 Pc = mat_apply(Rcw, tcw, P);
    const float Pc_dist = std::sqrt(dot3(Pc, Pc));
    const float invz = 1.0f / Pc.z;
    if (Pc.z < 0.0f) continue;
    const float u = project_u(*cam, Pc), v = project_v(*cam, Pc);
    if (u < g->min_x || u > g->max_x) continue;
    if (v < g->min_y || v > g->max_y) continue;
    V.proj_x = u, V.proj_y = v;
    const float maxD = 1.2f * M.max_dist, minD = 0.8f * M.min_dist;
    const V3 PO{P.x - Ow[0], P.y - Ow[1], P.z - Ow[2]};
    const float dist = std::sqrt(dot3(PO, PO));
    if (dist < minD || dist > maxD) continue;
    const V3 Pn{M.normal[0], M.normal[1], M.normal[2]};
    const float view_cos = dot3(PO, Pn) / dist;
    if (view_cos < cos_limit) continue;
    V.level = predict_scale(M.max_dist, dist, g->log_scale, g->n_levels);
    V.in_view = 1;
    V.proj_xr = std::fmaf(-cam->bf, invz, u);  // uv(0) - bf_ * invz
    V.depth = Pc_dist;
    V.view_cos = view_cos;
  }
}

// ORBmatcher::SearchByProjection(Frame& F, const vector<MapPoint*>&, th,
// bFarPoints, thFarPoints) -- orb_matcher.cc:42-137 (Nleft == -1).
int orc_search_local(const Geom* g, const Kp* kps, const uint8_t* desc, const float* uright,
                     const uint8_t* claimed, int n, const MapPt* pts, const View* views,
                     int n_pts, float th, float nn_ratio, int far_points, float th_far,
                     int32_t* match) {
  Frame F(g, kps, desc, uright, claimed, n);
  int nmatches = 0;
  const bool factor = th != 1.0;
  for (int j = 0; j < n_pts; ++j) {
    const View& V = views[j];
    if (!V.in_view) continue;
    if (far_points && V.depth > th_far) continue;
    const int level = V.level;
    float r = V.view_cos > 0.998 ? 2.5f : 4.0f;  // RadiusByViewingCos (:208-213)
    if (factor) r *= th;
    const float rs = r * g->scale[level];
    const std::vector<int> cand = F.features_in_area(V.proj_x, V.proj_y, rs, level - 1, level);
    if (cand.empty()) continue;
    int best = 256, best_level = -1, best2 = 256, best_level2 = -1, best_idx = -1;
    for (int idx : cand) {
      if (F.blocked(idx)) continue;
      if (uright && uright[idx] > 0) {
        const float er = std::fabs(V.proj_xr - uright[idx]);
        if (er > r * g->scale[level]) continue;
      }
      const int d = desc_dist(pts[j].desc, desc + 32 * (size_t)idx);
      if (d < best) {
        best2 = best, best = d;
        best_level2 = best_level, best_level = kps[idx].octave;
        best_idx = idx;
      } else if (d < best2) {
        best_level2 = kps[idx].octave;
        best2 = d;
      }
    }
    if (best <= kThHigh) {
      if (best_level == best_level2 && best > nn_ratio * best2) continue;
      F.holder[best_idx] = j;
      F.holder_obs[best_idx] = (pts[j].flags & 2) != 0;
      ++nmatches;
    }
  }
  std::vector<char> nulled(n, 0);
  write_match(F, nulled, match);
  return nmatches;
}

int orc_predict_scale(float max_distance, float dist, float log_scale, int n_levels) {
  return predict_scale(max_distance, dist, log_scale, n_levels);
}

// Checks a PredictScale threshold table (the GPU library's
// orbgpu_level_thresholds) against the restatement on every float ratio with
// bit pattern in [lo, hi]; returns the number of disagreements.
long orc_predict_scale_check(float log_scale, int n_levels, const float* thr, uint32_t lo,
                             uint32_t hi) {
  long bad = 0;
  for (uint64_t b = lo; b <= hi; ++b) {
    float r;
    const uint32_t bits = (uint32_t)b;
    std::memcpy(&r, &bits, 4);
    int lv = 0;
    if (!(r == INFINITY))
      for (int j = 1; j < n_levels; ++j) lv += r >= thr[j - 1];
    bad += lv != level_of_ratio(r, log_scale, n_levels);
  }
  return bad;
}

// Frame grid of the current frame, for the tests: cell of keypoint i or -1.
void orc_frame_grid_cells(const Geom* g, const Kp* kps, int n, int32_t* cell) {
  Frame F(g, kps, nullptr, nullptr, nullptr, 0);
  for (int i = 0; i < n; ++i) {
    int px, py;
    cell[i] = F.pos_in_grid(kps[i], px, py) ? px * kGridRows + py : -1;
  }
}

}  // extern "C"
