// ORBmatcher searches over the gfx950 C ABI.
// Compiled inside the reference build (its include paths: frame.h, keyframe.h,
// mappoint.h, orb_matcher.h, DBoW2, Sophus, Eigen); the original definitions
// in orb_matcher.cc (:42-206, :215-389, :1518-1728 and :1730-1839) are guarded
// with ORBGPU_MATCH.
// Same reads and writes as the reference for the pinhole rig (Nleft == -1):
//   SearchByProjection(CurrentFrame, LastFrame, th, bMono): LastFrame's
//     non-outlier map points (GetWorldPos, GetDescriptor, Observations),
//     mvKeys / mvKeysUn octave and angle, both poses; CurrentFrame's mvKeysUn,
//     mDescriptors, mvuRight, mvpMapPoints (written), mb, camera; mfNNratio /
//     mbCheckOrientation of this matcher.
//   SearchByProjection(F, vpMapPoints, th, bFarPoints, thFarPoints): the
//     points' tracking fields written by Frame::isInFrustum (mbTrackInView,
//     mTrackProjX/Y/XR, mnTrackScaleLevel, mTrackViewCos, mTrackDepth), isBad,
//     Observations, GetDescriptor; F as above.
//   SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist): the key
//     frame's points (isBad, GetWorldPos, min/max distance, GetDescriptor),
//     pKF->mvKeysUn angles; CurrentFrame's pose, keypoints, descriptors,
//     mvpMapPoints (read: every held keypoint is skipped; written).
//   SearchByBoW(pKF, F, vpMapPointMatches): both mFeatVec, descriptors, the
//     key frame's points (isBad) and mvKeysUn angles, F.mvKeys angles.
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <vector>

#include <set>

#include "cam/orb_feature/orb_matcher.h"
#include "map/frame.h"
#include "map/keyframe.h"
#include "map/mappoint.h"
#include "orbgpu.h"

namespace ORB_SLAM_FUSION {

namespace {
static_assert(sizeof(cv::KeyPoint) == sizeof(orbgpu_keypoint), "cv::KeyPoint layout");

// One matcher context per calling thread (Tracking; LocalMapping does not call
// these two overloads).
orbgpu_matcher *thread_matcher() {
  thread_local struct Holder {
    orbgpu_matcher *m = nullptr;
    ~Holder() { orbgpu_matcher_destroy(m); }
  } h;
  if (!h.m && orbgpu_matcher_create(0, 8192, 65536, &h.m) != ORBGPU_OK)
    throw std::runtime_error("orbgpu_matcher_create failed");
  return h.m;
}

orbgpu_frame_geom frame_geom(const Frame &F) {
  orbgpu_frame_geom g{};
  g.min_x = Frame::mnMinX, g.max_x = Frame::mnMaxX;
  g.min_y = Frame::mnMinY, g.max_y = Frame::mnMaxY;
  g.n_levels = F.mnScaleLevels;
  g.log_scale_factor = F.mfLogScaleFactor;
  for (int l = 0; l < F.mnScaleLevels && l < ORBGPU_MAX_LEVELS; ++l)
    g.scale_factors[l] = F.mvScaleFactors[l];
  return g;
}

orbgpu_pose to_pose(const Sophus::SE3f &T) {
  const Eigen::Quaternionf q = T.unit_quaternion();
  const Eigen::Vector3f t = T.translation();
  return orbgpu_pose{q.x(), q.y(), q.z(), q.w(), t.x(), t.y(), t.z()};
}

// mvpMapPoints[i] != NULL && ->Observations() > 0 (orb_matcher.cc:86-87, 1591-1592)
std::vector<uint8_t> claimed_mask(const Frame &F) {
  std::vector<uint8_t> c(F.N, 0);
  for (int i = 0; i < F.N; ++i)
    if (F.mvpMapPoints[i] && F.mvpMapPoints[i]->Observations() > 0) c[i] = 1;
  return c;
}

void copy_desc(const cv::Mat &d, uint8_t out[32]) { std::memcpy(out, d.ptr<uint8_t>(0), 32); }

// mfMinDistance / mfMaxDistance under mMutexPos, as MapPoint::PredictScale and
// GetMin/MaxDistanceInvariance read them (mappoint.cc:524-563).  They are
// protected members without getters; a member pointer taken through a
// derived class names them without touching the reference's header.
struct MapPointDistances : MapPoint {
  static void read(MapPoint *p, float &min_d, float &max_d) {
    static constexpr float MapPoint::*kMin = &MapPointDistances::mfMinDistance;
    static constexpr float MapPoint::*kMax = &MapPointDistances::mfMaxDistance;
    static constexpr std::mutex MapPoint::*kMutex = &MapPointDistances::mMutexPos;
    std::unique_lock<std::mutex> lock(p->*kMutex);
    min_d = p->*kMin;
    max_d = p->*kMax;
  }
};

// DBoW2::FeatureVector (std::map<NodeId, vector<unsigned>>) as CSR arrays
struct FeatVecArrays {
  std::vector<uint32_t> nodes, features;
  std::vector<int32_t> offsets{0};
  explicit FeatVecArrays(const DBoW2::FeatureVector &fv) {
    for (const auto &kv : fv) {
      nodes.push_back(kv.first);
      features.insert(features.end(), kv.second.begin(), kv.second.end());
      offsets.push_back((int32_t)features.size());
    }
  }
};

}  // namespace

int ORBmatcher::SearchByProjection(Frame &CurrentFrame, const Frame &LastFrame, const float th,
                                   const bool bMono) {
  if (CurrentFrame.Nleft != -1 || LastFrame.Nleft != -1)
    throw std::logic_error("orbgpu SearchByProjection: fisheye rig not supported");
  std::vector<orbgpu_proj_point> pts;
  std::vector<MapPoint *> who;
  pts.reserve(LastFrame.N);
  who.reserve(LastFrame.N);
  for (int i = 0; i < LastFrame.N; i++) {
    MapPoint *pMP = LastFrame.mvpMapPoints[i];
    if (!pMP || LastFrame.mvbOutlier[i]) continue;
    orbgpu_proj_point p;
    const Eigen::Vector3f X = pMP->GetWorldPos();
    p.Xw[0] = X[0], p.Xw[1] = X[1], p.Xw[2] = X[2];
    p.octave = LastFrame.mvKeys[i].octave;
    p.angle = LastFrame.mvKeysUn[i].angle;
    p.has_obs = pMP->Observations() > 0;
    copy_desc(pMP->GetDescriptor(), p.desc);
    pts.push_back(p);
    who.push_back(pMP);
  }
  const orbgpu_frame_geom g = frame_geom(CurrentFrame);
  const orbgpu_camera cam{CurrentFrame.fx, CurrentFrame.fy, CurrentFrame.cx, CurrentFrame.cy,
                          CurrentFrame.bf_};
  const orbgpu_pose Tcw = to_pose(CurrentFrame.GetPose());
  const orbgpu_pose Tlw = to_pose(LastFrame.GetPose());
  const std::vector<uint8_t> claimed = claimed_mask(CurrentFrame);
  std::vector<int32_t> match(CurrentFrame.N);
  int nmatches = 0;
  if (orbgpu_search_by_projection_last(
          thread_matcher(), &g, &cam, CurrentFrame.mb, &Tcw, &Tlw,
          reinterpret_cast<const orbgpu_keypoint *>(CurrentFrame.mvKeysUn.data()),
          CurrentFrame.mDescriptors.ptr<uint8_t>(0), CurrentFrame.mvuRight.data(), claimed.data(),
          CurrentFrame.N, pts.data(), (int)pts.size(), th, bMono, mbCheckOrientation, match.data(),
          &nmatches) != ORBGPU_OK)
    throw std::runtime_error("orbgpu_search_by_projection_last failed");
  for (int i = 0; i < CurrentFrame.N; ++i) {
    if (match[i] >= 0) CurrentFrame.mvpMapPoints[i] = who[match[i]];
    else if (match[i] == -2) CurrentFrame.mvpMapPoints[i] = static_cast<MapPoint *>(NULL);
  }
  return nmatches;
}

int ORBmatcher::SearchByProjection(Frame &F, const std::vector<MapPoint *> &vpMapPoints,
                                   const float th, const bool bFarPoints,
                                   const float thFarPoints) {
  if (F.Nleft != -1) throw std::logic_error("orbgpu SearchByProjection: fisheye rig not supported");
  std::vector<orbgpu_map_point> pts;
  std::vector<orbgpu_track_view> views;
  std::vector<MapPoint *> who;
  pts.reserve(vpMapPoints.size());
  views.reserve(vpMapPoints.size());
  who.reserve(vpMapPoints.size());
  for (MapPoint *pMP : vpMapPoints) {
    // orb_matcher.cc:52-58: only points isInFrustum put in view, not bad
    if (!pMP->mbTrackInView || pMP->isBad()) continue;
    orbgpu_map_point p{};
    p.flags = pMP->Observations() > 0 ? ORBGPU_MP_HAS_OBS : 0;
    copy_desc(pMP->GetDescriptor(), p.desc);
    orbgpu_track_view v;
    v.in_view = 1;
    v.level = pMP->mnTrackScaleLevel;
    v.proj_x = pMP->mTrackProjX, v.proj_y = pMP->mTrackProjY, v.proj_xr = pMP->mTrackProjXR;
    v.depth = pMP->mTrackDepth;
    v.view_cos = pMP->mTrackViewCos;
    pts.push_back(p);
    views.push_back(v);
    who.push_back(pMP);
  }
  const orbgpu_frame_geom g = frame_geom(F);
  const std::vector<uint8_t> claimed = claimed_mask(F);
  std::vector<int32_t> match(F.N);
  int nmatches = 0;
  if (orbgpu_search_by_projection_local(
          thread_matcher(), &g, reinterpret_cast<const orbgpu_keypoint *>(F.mvKeysUn.data()),
          F.mDescriptors.ptr<uint8_t>(0), F.mvuRight.data(), claimed.data(), F.N, pts.data(),
          views.data(), (int)pts.size(), th, mfNNratio, bFarPoints, thFarPoints, match.data(),
          &nmatches) != ORBGPU_OK)
    throw std::runtime_error("orbgpu_search_by_projection_local failed");
  for (int i = 0; i < F.N; ++i)
    if (match[i] >= 0) F.mvpMapPoints[i] = who[match[i]];
  return nmatches;
}

int ORBmatcher::SearchByProjection(Frame &CurrentFrame, KeyFrame *pKF,
                                   const std::set<MapPoint *> &sAlreadyFound, const float th,
                                   const int ORBdist) {
  if (CurrentFrame.Nleft != -1)
    throw std::logic_error("orbgpu SearchByProjection: fisheye rig not supported");
  const std::vector<MapPoint *> vpMPs = pKF->GetMapPointMatches();
  std::vector<orbgpu_map_point> pts(vpMPs.size());
  std::vector<float> angles(vpMPs.size());
  for (size_t i = 0; i < vpMPs.size(); ++i) {
    MapPoint *pMP = vpMPs[i];
    orbgpu_map_point &p = pts[i];
    p = orbgpu_map_point{};
    angles[i] = pKF->mvKeysUn[i].angle;
    if (!pMP || pMP->isBad() || sAlreadyFound.count(pMP)) {
      p.flags = ORBGPU_MP_SKIP;
      continue;
    }
    const Eigen::Vector3f X = pMP->GetWorldPos();
    p.Xw[0] = X[0], p.Xw[1] = X[1], p.Xw[2] = X[2];
    MapPointDistances::read(pMP, p.min_dist, p.max_dist);
    copy_desc(pMP->GetDescriptor(), p.desc);
  }
  const orbgpu_frame_geom g = frame_geom(CurrentFrame);
  const orbgpu_camera cam{CurrentFrame.fx, CurrentFrame.fy, CurrentFrame.cx, CurrentFrame.cy,
                          CurrentFrame.bf_};
  const orbgpu_pose Tcw = to_pose(CurrentFrame.GetPose());
  std::vector<uint8_t> claimed(CurrentFrame.N);  // every held keypoint is skipped (:1791)
  for (int i = 0; i < CurrentFrame.N; ++i) claimed[i] = CurrentFrame.mvpMapPoints[i] != NULL;
  std::vector<int32_t> match(CurrentFrame.N);
  int nmatches = 0;
  if (orbgpu_search_by_projection_kf(
          thread_matcher(), &g, &cam, &Tcw,
          reinterpret_cast<const orbgpu_keypoint *>(CurrentFrame.mvKeysUn.data()),
          CurrentFrame.mDescriptors.ptr<uint8_t>(0), claimed.data(), CurrentFrame.N, pts.data(),
          angles.data(), (int)pts.size(), th, ORBdist, mbCheckOrientation, match.data(),
          &nmatches) != ORBGPU_OK)
    throw std::runtime_error("orbgpu_search_by_projection_kf failed");
  for (int i = 0; i < CurrentFrame.N; ++i) {
    if (match[i] >= 0) CurrentFrame.mvpMapPoints[i] = vpMPs[match[i]];
    else if (match[i] == -2) CurrentFrame.mvpMapPoints[i] = static_cast<MapPoint *>(NULL);
  }
  return nmatches;
}

int ORBmatcher::SearchByBoW(KeyFrame *pKF, Frame &F, std::vector<MapPoint *> &vpMapPointMatches) {
  if (F.Nleft != -1 || pKF->cam2_)
    throw std::logic_error("orbgpu SearchByBoW: fisheye rig not supported");
  const std::vector<MapPoint *> vpMapPointsKF = pKF->GetMapPointMatches();
  vpMapPointMatches = std::vector<MapPoint *>(F.N, static_cast<MapPoint *>(NULL));
  const FeatVecArrays kfv(pKF->mFeatVec), ffv(F.mFeatVec);
  const int nk = (int)vpMapPointsKF.size();
  std::vector<uint8_t> valid(nk);
  std::vector<float> ka(nk), fa(F.N);
  for (int i = 0; i < nk; ++i) {
    valid[i] = vpMapPointsKF[i] && !vpMapPointsKF[i]->isBad();
    ka[i] = pKF->mvKeysUn[i].angle;
  }
  for (int i = 0; i < F.N; ++i) fa[i] = F.mvKeys[i].angle;
  std::vector<int32_t> match(F.N);
  int nmatches = 0;
  if (orbgpu_search_by_bow(thread_matcher(), kfv.nodes.data(), kfv.offsets.data(),
                           kfv.features.data(), (int)kfv.nodes.size(),
                           pKF->mDescriptors.ptr<uint8_t>(0), ka.data(), valid.data(), nk,
                           ffv.nodes.data(), ffv.offsets.data(), ffv.features.data(),
                           (int)ffv.nodes.size(), F.mDescriptors.ptr<uint8_t>(0), fa.data(), F.N,
                           mfNNratio, mbCheckOrientation, match.data(), &nmatches) != ORBGPU_OK)
    throw std::runtime_error("orbgpu_search_by_bow failed");
  for (int i = 0; i < F.N; ++i)
    if (match[i] >= 0) vpMapPointMatches[i] = vpMapPointsKF[match[i]];
  return nmatches;
}

}  // namespace ORB_SLAM_FUSION
