// Optimizer::LocalBundleAdjustment over the gfx950 C ABI.
// Compiled inside the reference build (its include paths: keyframe.h,
// mappoint.h, map.h, Sophus, Eigen) in place of the original definition in
// optimizer.cc:1053-1441.
// The window gather and the write-back keep the reference's semantics
// (:1057-1124 and :1362-1441: local keyframes = pKF + its non-bad covisible
// keyframes of the same map, local map points = their non-bad points of that
// map, fixed cameras = other keyframes observing them; abort without a fixed
// keyframe; num_MPs untouched); the graph + optimize(10) + outlier test run on
// the GPU (orbgpu_lba_optimize).  Pinhole rigs only (the ToBody edges of
// fisheye rigs, :1312-1350, are out of scope).
#include <list>
#include <mutex>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "map/keyframe.h"
#include "map/map.h"
#include "map/mappoint.h"
#include "orbgpu.h"
#include "solver/g2o_solver/optimizer.h"

namespace ORB_SLAM_FUSION {

namespace {
// LocalMapping calls this; keep one context per calling thread.
orbgpu_lba_ctx *lba_thread_ctx() {
  thread_local struct Holder {
    orbgpu_lba_ctx *c = nullptr;
    ~Holder() { orbgpu_lba_ctx_destroy(c); }
  } h;
  if (!h.c && orbgpu_lba_ctx_create(0, &h.c) != ORBGPU_OK)
    throw std::runtime_error("orbgpu_lba_ctx_create failed");
  return h.c;
}

orbgpu_pose to_pose(const Sophus::SE3f &T) {
  const Eigen::Quaternionf q = T.unit_quaternion();
  const Eigen::Vector3f t = T.translation();
  return orbgpu_pose{q.x(), q.y(), q.z(), q.w(), t.x(), t.y(), t.z()};
}
}  // namespace

void Optimizer::LocalBundleAdjustment(KeyFrame *pKF, bool *pbStopFlag, Map *pMap,
                                      int &num_fixedKF, int &num_OptKF, int &num_MPs,
                                      int &num_edges) {
  (void)num_MPs;  // never written by the reference either
  Map *pCurrentMap = pKF->GetMap();
  if (pKF->cam2_) throw std::logic_error("orbgpu LocalBundleAdjustment: fisheye rig not supported");

  // ---- window: local keyframes, local map points, fixed cameras
  std::list<KeyFrame *> local_kfs{pKF};
  pKF->mnBALocalForKF = pKF->id_;
  for (KeyFrame *k : pKF->GetVectorCovisibleKeyFrames()) {
    k->mnBALocalForKF = pKF->id_;
    if (!k->isBad() && k->GetMap() == pCurrentMap) local_kfs.push_back(k);
  }
  num_fixedKF = 0;
  std::list<MapPoint *> local_mps;
  for (KeyFrame *k : local_kfs) {
    if (k->id_ == pMap->GetInitKFid()) num_fixedKF = 1;
    for (MapPoint *mp : k->GetMapPointMatches())
      if (mp && !mp->isBad() && mp->GetMap() == pCurrentMap && mp->mnBALocalForKF != pKF->id_) {
        local_mps.push_back(mp);
        mp->mnBALocalForKF = pKF->id_;
      }
  }
  std::list<KeyFrame *> fixed_kfs;
  for (MapPoint *mp : local_mps)
    for (const auto &obs : mp->GetObservations()) {
      KeyFrame *k = obs.first;
      if (k->mnBALocalForKF != pKF->id_ && k->mnBAFixedForKF != pKF->id_) {
        k->mnBAFixedForKF = pKF->id_;
        if (!k->isBad() && k->GetMap() == pCurrentMap) fixed_kfs.push_back(k);
      }
    }
  num_fixedKF += (int)fixed_kfs.size();
  if (num_fixedKF == 0) return;  // "LM-LBA: There are 0 fixed KF in the optimizations"

  // ---- flat graph: poses (local then fixed cameras), points, observations
  std::vector<KeyFrame *> kfs(local_kfs.begin(), local_kfs.end());
  kfs.insert(kfs.end(), fixed_kfs.begin(), fixed_kfs.end());
  std::unordered_map<KeyFrame *, int> kf_index;
  std::vector<orbgpu_pose> poses;
  std::vector<uint8_t> fixed;
  for (size_t i = 0; i < kfs.size(); ++i) {
    kf_index[kfs[i]] = (int)i;
    poses.push_back(to_pose(kfs[i]->GetPose()));
    fixed.push_back(i >= local_kfs.size() || kfs[i]->id_ == pMap->GetInitKFid() ? 1 : 0);
  }
  num_OptKF = (int)local_kfs.size();
  std::vector<MapPoint *> mps(local_mps.begin(), local_mps.end());
  std::vector<float> pts(3 * mps.size());
  std::vector<orbgpu_lba_edge> edges;
  std::vector<std::pair<KeyFrame *, MapPoint *>> edge_ref;
  for (size_t p = 0; p < mps.size(); ++p) {
    const Eigen::Vector3f X = mps[p]->GetWorldPos();
    for (int c = 0; c < 3; ++c) pts[3 * p + c] = X[c];
    for (const auto &obs : mps[p]->GetObservations()) {
      KeyFrame *k = obs.first;
      if (k->isBad() || k->GetMap() != pCurrentMap) continue;
      const int left = std::get<0>(obs.second);
      if (left == -1) continue;
      const cv::KeyPoint &kp = k->mvKeysUn[left];
      orbgpu_lba_edge e;
      e.point = (int32_t)p;
      e.kf = kf_index.at(k);
      e.u = kp.pt.x;
      e.v = kp.pt.y;
      e.ur = k->mvuRight[left];  // < 0: EdgeSE3ProjectXYZ, else EdgeStereoSE3ProjectXYZ
      e.inv_sigma2 = k->mvInvLevelSigma2[kp.octave];
      edges.push_back(e);
      edge_ref.emplace_back(k, mps[p]);
    }
  }
  num_edges = (int)edges.size();
  if (pbStopFlag && *pbStopFlag) return;

  const orbgpu_camera cam{pKF->fx, pKF->fy, pKF->cx, pKF->cy, pKF->bf_};
  std::vector<orbgpu_pose> poses_out(kfs.size());
  std::vector<float> pts_out(pts);
  std::vector<uint8_t> outlier(edges.size());
  static_assert(sizeof(bool) == 1, "pbStopFlag is read as one byte by the ABI");
  // every window runs on the device (any size: orbgpu.h); a failure -- only
  // exhausted device memory remains -- is an error, never a CPU fallback
  const orbgpu_status st =
      orbgpu_lba_optimize(lba_thread_ctx(), &cam, (int)kfs.size(), poses.data(), fixed.data(), (int)mps.size(),
                          pts.data(), (int)edges.size(), edges.data(), 0, (int)mps.size(), 10,
                          pMap->IsInertial() ? 100.0 : 0.0,  // :1137
                          reinterpret_cast<const volatile uint8_t *>(pbStopFlag), nullptr, nullptr,
                          poses_out.data(), nullptr, pts_out.data(), outlier.data(), nullptr);
  if (st != ORBGPU_OK)
    throw std::runtime_error("orbgpu_lba_optimize failed with status " + std::to_string(st));

  // ---- outliers and write-back (:1362-1441)
  std::vector<std::pair<KeyFrame *, MapPoint *>> to_erase;
  for (size_t i = 0; i < edges.size(); ++i)
    if (outlier[i] && !edge_ref[i].second->isBad()) to_erase.push_back(edge_ref[i]);
  std::unique_lock<std::mutex> lock(pMap->mMutexMapUpdate);
  for (auto &ke : to_erase) {
    ke.first->EraseMapPointMatch(ke.second);
    ke.second->EraseObservation(ke.first);
  }
  for (size_t i = 0; i < local_kfs.size(); ++i) {
    const orbgpu_pose &o = poses_out[i];
    kfs[i]->SetPose(Sophus::SE3f(Eigen::Quaternionf(o.qw, o.qx, o.qy, o.qz),
                                 Eigen::Vector3f(o.tx, o.ty, o.tz)));
  }
  for (size_t p = 0; p < mps.size(); ++p) {
    mps[p]->SetWorldPos(Eigen::Vector3f(pts_out[3 * p], pts_out[3 * p + 1], pts_out[3 * p + 2]));
    mps[p]->UpdateNormalAndDepth();
  }
  pMap->IncreaseChangeIndex();
}

}  // namespace ORB_SLAM_FUSION
