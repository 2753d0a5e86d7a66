// Optimizer::PoseOptimization over the gfx950 C ABI.
// Compiled inside the reference build (its include paths: frame.h, mappoint.h,
// Sophus, Eigen); the original definition in optimizer.cc:762-1051 is removed
// or guarded with ORBGPU_POSE.  Same reads and writes as
// the reference: N, mvpMapPoints, mvuRight, mvKeysUn, mvInvLevelSigma2, fx, fy,
// cx, cy, bf_, GetPose() in; mvbOutlier, SetPose() out; MapPoint::mGlobalMutex
// held while the world positions are read; returns the inlier count.
#include <mutex>
#include <stdexcept>
#include <vector>

#include "map/frame.h"
#include "map/mappoint.h"
#include "orbgpu.h"
#include "solver/g2o_solver/optimizer.h"

namespace ORB_SLAM_FUSION {

namespace {
// One pose context per calling thread (Tracking only, but keep it re-entrant).
orbgpu_pose_ctx *thread_ctx() {
  thread_local struct Holder {
    orbgpu_pose_ctx *c = nullptr;
    ~Holder() { orbgpu_pose_ctx_destroy(c); }
  } h;
  if (!h.c && orbgpu_pose_ctx_create(0, 1, 8192, &h.c) != ORBGPU_OK)
    throw std::runtime_error("orbgpu_pose_ctx_create failed");
  return h.c;
}
}  // namespace

int Optimizer::PoseOptimization(Frame *pFrame) {
  if (pFrame->cam2_) throw std::logic_error("orbgpu PoseOptimization: fisheye rig not supported");
  const int N = pFrame->N;
  std::vector<orbgpu_pose_obs> obs;
  std::vector<int> index;
  obs.reserve(N);
  index.reserve(N);
  {
    std::unique_lock<std::mutex> lock(MapPoint::mGlobalMutex);
    for (int i = 0; i < N; i++) {
      MapPoint *pMP = pFrame->mvpMapPoints[i];
      if (!pMP) continue;
      pFrame->mvbOutlier[i] = false;
      const Eigen::Vector3f X = pMP->GetWorldPos();
      const cv::KeyPoint &kpUn = pFrame->mvKeysUn[i];
      orbgpu_pose_obs o;
      o.Xw[0] = X[0];
      o.Xw[1] = X[1];
      o.Xw[2] = X[2];
      o.u = kpUn.pt.x;
      o.v = kpUn.pt.y;
      o.ur = pFrame->mvuRight[i];
      o.inv_sigma2 = pFrame->mvInvLevelSigma2[kpUn.octave];
      obs.push_back(o);
      index.push_back(i);
    }
  }
  if (obs.size() < 3) return 0;

  const Sophus::SE3f Tcw = pFrame->GetPose();
  const Eigen::Quaternionf q = Tcw.unit_quaternion();
  const Eigen::Vector3f t = Tcw.translation();
  const orbgpu_pose in{q.x(), q.y(), q.z(), q.w(), t.x(), t.y(), t.z()};
  const orbgpu_camera cam{pFrame->fx, pFrame->fy, pFrame->cx, pFrame->cy, pFrame->bf_};
  orbgpu_pose out;
  std::vector<uint8_t> outlier(obs.size());
  int inliers = 0;
  if (orbgpu_pose_opt(thread_ctx(), &cam, &in, obs.data(), (int)obs.size(), &out,
                      outlier.data(), &inliers) != ORBGPU_OK)
    throw std::runtime_error("orbgpu_pose_opt failed");
  for (size_t k = 0; k < index.size(); ++k) pFrame->mvbOutlier[index[k]] = outlier[k] != 0;
  pFrame->SetPose(Sophus::SE3f(Eigen::Quaternionf(out.qw, out.qx, out.qy, out.qz),
                               Eigen::Vector3f(out.tx, out.ty, out.tz)));
  return inliers;
}

}  // namespace ORB_SLAM_FUSION
