// Optimizer::PoseInertialOptimizationLastFrame / LastKeyFrame over the gfx950
// C ABI.  Compiled inside the reference build (frame.h, keyframe.h,
// mappoint.h, imu_types.h, g2o_types.h, Eigen, Sophus); the original
// definitions (optimizer.cc:4394-4760, 4762-5160) are guarded with
// ORBGPU_INERTIAL.  Same reads and writes as the
// reference for the pinhole rig (Nleft == -1): the frame's matched map points,
// keypoints, mvuRight, mvInvLevelSigma2 / Uncertainty2, mTrackDepth, the IMU
// states of the frame and of mpPrevFrame / mpLastKeyFrame, the
// preintegration, pFp->mpcpi in; mvbOutlier, SetImuPoseVelocity, mImuBias and
// the new mpcpi out.  The information matrices are formed here exactly as the
// edges' constructors form them (EdgeInertial is constructed for its
// information; the random-walk ones are the same C block inverses).
#include <mutex>
#include <stdexcept>
#include <vector>

#include "imu/imu_types.h"
#include "imu_marshal.h"
#include "map/frame.h"
#include "map/keyframe.h"
#include "map/mappoint.h"
#include "orbgpu.h"
#include "solver/g2o_solver/g2o_types.h"
#include "solver/g2o_solver/optimizer.h"

namespace ORB_SLAM_FUSION {

namespace {

using namespace orbgpu_shim;

orbgpu_inertial_ctx *thread_ctx() {
  thread_local struct Holder {
    orbgpu_inertial_ctx *c = nullptr;
    ~Holder() { orbgpu_inertial_ctx_destroy(c); }
  } h;
  if (!h.c && orbgpu_inertial_ctx_create(0, 1, 8192, &h.c) != ORBGPU_OK)
    throw std::runtime_error("orbgpu_inertial_ctx_create failed");
  return h.c;
}

orbgpu_imu_state state_of(Frame *pF) {
  orbgpu_imu_state s{};
  put(s.Rwb, pF->GetImuRotation());
  put(s.twb, pF->GetImuPosition());
  put(s.Rcw, pF->GetPose().rotationMatrix());
  put(s.tcw, pF->GetPose().translation());
  put(s.v, pF->GetVelocity());
  const float bg[3] = {pF->mImuBias.bwx, pF->mImuBias.bwy, pF->mImuBias.bwz};
  const float ba[3] = {pF->mImuBias.bax, pF->mImuBias.bay, pF->mImuBias.baz};
  for (int i = 0; i < 3; ++i) {
    s.bg[i] = bg[i];
    s.ba[i] = ba[i];
  }
  return s;
}

orbgpu_imu_state state_of(KeyFrame *pKF) {
  orbgpu_imu_state s{};
  put(s.Rwb, pKF->GetImuRotation());
  put(s.twb, pKF->GetImuPosition());
  put(s.v, pKF->GetVelocity());
  put(s.bg, pKF->GetGyroBias());
  put(s.ba, pKF->GetAccBias());
  return s;
}

int run(Frame *pFrame, bool bRecInit, int mode) {
  if (pFrame->Nleft != -1)
    throw std::logic_error("orbgpu PoseInertialOptimization: fisheye rig not supported");
  const int N = pFrame->N;
  std::vector<orbgpu_inertial_obs> obs;
  std::vector<int> index;
  obs.reserve(N);
  index.reserve(N);
  {
    std::unique_lock<std::mutex> lock(MapPoint::mGlobalMutex);
    for (int i = 0; i < N; i++) {
      MapPoint *pMP = pFrame->mvpMapPoints[i];
      if (!pMP) continue;
      pFrame->mvbOutlier[i] = false;
      const cv::KeyPoint &kpUn = pFrame->mvKeysUn[i];
      Eigen::Matrix<double, 2, 1> uv;
      uv << kpUn.pt.x, kpUn.pt.y;
      const float unc2 = pFrame->cam_->Uncertainty2(uv);
      const Eigen::Vector3f X = pMP->GetWorldPos();
      orbgpu_inertial_obs o;
      o.Xw[0] = X[0];
      o.Xw[1] = X[1];
      o.Xw[2] = X[2];
      o.u = kpUn.pt.x;
      o.v = kpUn.pt.y;
      o.ur = pFrame->mvuRight[i];
      o.inv_sigma2 = pFrame->mvInvLevelSigma2[kpUn.octave] / unc2;
      o.close = pMP->mTrackDepth < 10.f;
      obs.push_back(o);
      index.push_back(i);
    }
  }
  const orbgpu_imu_calib calib = calib_of(pFrame);
  const orbgpu_imu_state cur = state_of(pFrame);
  orbgpu_imu_state prev;
  orbgpu_imu_preint preint;
  orbgpu_imu_prior prior{};
  Frame *pFp = pFrame->mpPrevFrame;
  if (mode == ORBGPU_INERTIAL_LAST_FRAME) {
    prev = state_of(pFp);
    preint = preint_of(pFrame->mpImuPreintegratedFrame);
    if (!pFp->mpcpi) throw std::runtime_error("pFp->mpcpi does not exist");
    const ConstraintPoseImu *c = pFp->mpcpi;
    putd(prior.Rwb, c->Rwb);
    putd(prior.twb, c->twb);
    putd(prior.vwb, c->vwb);
    putd(prior.bg, c->bg);
    putd(prior.ba, c->ba);
    putd(prior.H, c->H);
  } else {
    prev = state_of(pFrame->mpLastKeyFrame);
    preint = preint_of(pFrame->mpImuPreintegrated);
  }
  orbgpu_inertial_result res;
  std::vector<uint8_t> outlier(obs.size() + 1);
  if (orbgpu_pose_inertial(thread_ctx(), mode, &calib, &cur, &prev, &preint,
                           mode == ORBGPU_INERTIAL_LAST_FRAME ? &prior : nullptr, obs.data(),
                           (int)obs.size(), bRecInit ? 1 : 0, &res, outlier.data()) != ORBGPU_OK)
    throw std::runtime_error("orbgpu_pose_inertial failed");
  for (size_t k = 0; k < index.size(); ++k) pFrame->mvbOutlier[index[k]] = outlier[k] != 0;
  Eigen::Matrix3f Rwb;
  Eigen::Vector3f twb, v;
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) Rwb(i, j) = res.Rwb[3 * i + j];
    twb[i] = res.twb[i];
    v[i] = res.v[i];
  }
  pFrame->SetImuPoseVelocity(Rwb, twb, v);
  pFrame->mImuBias = IMU::Bias(res.ba[0], res.ba[1], res.ba[2], res.bg[0], res.bg[1], res.bg[2]);
  Eigen::Matrix3d Rd;
  Eigen::Vector3d td, vd, bgd, bad;
  Matrix15d H;
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) Rd(i, j) = res.Rwb_d[3 * i + j];
    td[i] = res.twb_d[i];
    vd[i] = res.v_d[i];
    bgd[i] = res.bg_d[i];
    bad[i] = res.ba_d[i];
  }
  for (int i = 0; i < 15; ++i)
    for (int j = 0; j < 15; ++j) H(i, j) = res.H[15 * i + j];
  pFrame->mpcpi = new ConstraintPoseImu(Rd, td, vd, bgd, bad, H);
  if (mode == ORBGPU_INERTIAL_LAST_FRAME) {
    delete pFp->mpcpi;
    pFp->mpcpi = NULL;
  }
  return res.n_good;
}

}  // namespace

int Optimizer::PoseInertialOptimizationLastFrame(Frame *pFrame, bool bRecInit) {
  return run(pFrame, bRecInit, ORBGPU_INERTIAL_LAST_FRAME);
}

int Optimizer::PoseInertialOptimizationLastKeyFrame(Frame *pFrame, bool bRecInit) {
  return run(pFrame, bRecInit, ORBGPU_INERTIAL_LAST_KEYFRAME);
}

}  // namespace ORB_SLAM_FUSION
