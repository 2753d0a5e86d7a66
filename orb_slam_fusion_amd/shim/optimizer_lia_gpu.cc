// Optimizer::LocalInertialBA over the gfx950 C ABI.  Compiled inside the
// reference build (keyframe.h, mappoint.h, map.h, imu_types.h, g2o_types.h,
// Eigen, Sophus) in place of the original definition in
// optimizer.cc:2329-2902.  Key frames without IMU data
// (VertexPose only, :2466-2484) and windows of any size run on the device.  The temporal window
// (:2332-2436), the graph (:2461-2781), the FAIL test and the write-back
// (:2832-2901) keep the reference's semantics; the optimisation and the
// outlier test run on the GPU (orbgpu_lia_optimize).  Pinhole rigs only (the
// right-camera EdgeMono(1) of fisheye rigs, :2743-2778, is out of scope).
// num_fixedKF / num_OptKF / num_MPs / num_edges are left unwritten, as the
// reference leaves them.
#include <cmath>
#include <iostream>
#include <list>
#include <mutex>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "imu_marshal.h"
#include "map/keyframe.h"
#include "map/map.h"
#include "map/mappoint.h"
#include "orbgpu.h"
#include "solver/g2o_solver/optimizer.h"

namespace ORB_SLAM_FUSION {

namespace {

using namespace orbgpu_shim;

orbgpu_lba_ctx *lia_thread_ctx() {  // LocalMapping's thread: one context
  thread_local struct Holder {
    orbgpu_lba_ctx *c = nullptr;
    ~Holder() { orbgpu_lba_ctx_destroy(c); }
  } h;
  if (!h.c && orbgpu_lba_ctx_create(0, &h.c) != ORBGPU_OK)
    throw std::runtime_error("orbgpu_lba_ctx_create failed");
  return h.c;
}

// ImuCamPose(pKF) (g2o_types.cc:28-72) + the IMU vertex estimates
orbgpu_imu_state kf_state(KeyFrame *k) {
  orbgpu_imu_state s{};
  put(s.Rwb, k->GetImuRotation());
  put(s.twb, k->GetImuPosition());
  put(s.Rcw, k->GetRotation());
  put(s.tcw, k->GetTranslation());
  put(s.v, k->GetVelocity());
  put(s.bg, k->GetGyroBias());
  put(s.ba, k->GetAccBias());
  return s;
}

}  // namespace

void Optimizer::LocalInertialBA(KeyFrame *pKF, bool *pbStopFlag, Map *pMap, int &num_fixedKF,
                                int &num_OptKF, int &num_MPs, int &num_edges, bool bLarge,
                                bool bRecInit) {
  // pbStopFlag: attached after optimize() in the reference (:2794), never stops it;
  // the counters are the reference's out-params, which it leaves unwritten
  (void)pbStopFlag;
  (void)num_fixedKF;
  (void)num_OptKF;
  (void)num_MPs;
  (void)num_edges;
  if (pKF->cam2_) throw std::logic_error("orbgpu LocalInertialBA: fisheye rig not supported");
  Map *pCurrentMap = pKF->GetMap();
  const int maxOpt = bLarge ? 25 : 10, opt_it = bLarge ? 4 : 10;
  const int Nd = std::min((int)pCurrentMap->KeyFramesInMap() - 2, maxOpt);

  // ---- temporal window (:2343-2386)
  std::vector<KeyFrame *> opt{pKF};
  pKF->mnBALocalForKF = pKF->id_;
  for (int i = 1; i < Nd; i++) {
    if (!opt.back()->mPrevKF) break;
    opt.push_back(opt.back()->mPrevKF);
    opt.back()->mnBALocalForKF = pKF->id_;
  }
  std::list<MapPoint *> local_mps;
  for (KeyFrame *k : opt)
    for (MapPoint *mp : k->GetMapPointMatches())
      if (mp && !mp->isBad() && mp->mnBALocalForKF != pKF->id_) {
        local_mps.push_back(mp);
        mp->mnBALocalForKF = pKF->id_;
      }
  std::list<KeyFrame *> fixed_kfs;
  if (opt.back()->mPrevKF) {
    fixed_kfs.push_back(opt.back()->mPrevKF);
    opt.back()->mPrevKF->mnBAFixedForKF = pKF->id_;
  } else {
    opt.back()->mnBALocalForKF = 0;
    opt.back()->mnBAFixedForKF = pKF->id_;
    fixed_kfs.push_back(opt.back());
    opt.pop_back();
  }
  // maxCovKF = 0: no optimizable covisible key frames (:2388-2412)
  for (MapPoint *mp : local_mps) {  // one fixed observer per point, at most 200 (:2414-2436)
    for (const auto &obs : mp->GetObservations()) {
      KeyFrame *k = obs.first;
      if (k->mnBALocalForKF != pKF->id_ && k->mnBAFixedForKF != pKF->id_) {
        k->mnBAFixedForKF = pKF->id_;
        if (!k->isBad()) {
          fixed_kfs.push_back(k);
          break;
        }
      }
    }
    if (fixed_kfs.size() >= 200) break;
  }

  // ---- flat graph (:2461-2781)
  const int N = (int)opt.size();
  std::vector<KeyFrame *> kfs(opt);
  kfs.insert(kfs.end(), fixed_kfs.begin(), fixed_kfs.end());
  std::unordered_map<KeyFrame *, int> kf_index;
  std::vector<orbgpu_imu_state> states;
  std::vector<uint8_t> fixed, imu;
  for (size_t i = 0; i < kfs.size(); ++i) {
    kf_index[kfs[i]] = (int)i;
    states.push_back(kf_state(kfs[i]));
    fixed.push_back(i >= (size_t)N ? 1 : 0);
    imu.push_back(kfs[i]->bImu ? 1 : 0);
  }
  std::vector<orbgpu_lia_imu_edge> links;
  for (int i = 0; i < N; ++i) {
    KeyFrame *k = opt[i];
    if (!k->mPrevKF) continue;  // "NOT INERTIAL LINK TO PREVIOUS FRAME!!!!"
    if (!(k->bImu && k->mPrevKF->bImu && k->mpImuPreintegrated)) continue;
    auto it = kf_index.find(k->mPrevKF);
    if (it == kf_index.end()) continue;  // no vertex: the reference skips the edge
    k->mpImuPreintegrated->SetNewBias(k->mPrevKF->GetImuBias());  // as :2539 (no effect on the edge)
    orbgpu_lia_imu_edge l{};
    l.kf1 = it->second;
    l.kf2 = i;
    l.flags = (i == N - 1 ? ORBGPU_LIA_ROBUST | ORBGPU_LIA_DOWNWEIGHT : 0) | (bRecInit ? ORBGPU_LIA_ROBUST : 0);
    l.preint = preint_of(k->mpImuPreintegrated);
    links.push_back(l);
  }
  std::vector<MapPoint *> mps(local_mps.begin(), local_mps.end());
  std::vector<float> pts(3 * mps.size());
  std::vector<uint8_t> close(mps.size());
  std::vector<orbgpu_lba_edge> edges;
  std::vector<std::pair<KeyFrame *, MapPoint *>> edge_ref;
  for (size_t p = 0; p < mps.size(); ++p) {
    const Eigen::Vector3f X = mps[p]->GetWorldPos();
    for (int c = 0; c < 3; ++c) pts[3 * p + c] = X[c];
    close[p] = mps[p]->mTrackDepth < 10.f;
    for (const auto &obs : mps[p]->GetObservations()) {
      KeyFrame *k = obs.first;
      if (k->mnBALocalForKF != pKF->id_ && k->mnBAFixedForKF != pKF->id_) continue;
      if (k->isBad() || k->GetMap() != pCurrentMap) continue;
      const int left = std::get<0>(obs.second);
      if (left == -1) continue;
      auto it = kf_index.find(k);
      if (it == kf_index.end()) continue;
      const cv::KeyPoint &kp = k->mvKeysUn[left];
      Eigen::Matrix<double, 2, 1> uv;
      uv << kp.pt.x, kp.pt.y;
      orbgpu_lba_edge e;
      e.point = (int32_t)p;
      e.kf = it->second;
      e.u = kp.pt.x;
      e.v = kp.pt.y;
      e.ur = k->mvuRight[left];  // < 0: EdgeMono(0), else EdgeStereo(0)
      e.inv_sigma2 = k->mvInvLevelSigma2[kp.octave] / k->cam_->Uncertainty2(uv);
      edges.push_back(e);
      edge_ref.emplace_back(k, mps[p]);
    }
  }

  const orbgpu_imu_calib calib = calib_of(pKF);
  std::vector<orbgpu_imu_state> out_states(kfs.size());
  std::vector<float> pts_out(pts);
  std::vector<uint8_t> outlier(edges.size() + 1);
  double stats[7];
  const orbgpu_status st =
      orbgpu_lia_optimize(lia_thread_ctx(), &calib, (int)kfs.size(), states.data(), fixed.data(), imu.data(),
                          (int)mps.size(), pts.data(), close.data(), (int)edges.size(), edges.data(),
                          (int)links.size(), links.data(), opt_it, bLarge ? 1e-2 : 1e0, out_states.data(),
                          nullptr, pts_out.data(), outlier.data(), stats);
  if (st != ORBGPU_OK)  // exhausted device memory: an error, never a CPU fallback
    throw std::runtime_error("orbgpu_lia_optimize failed with status " + std::to_string(st));

  // ---- FAIL test, erase, write-back (:2796-2901)
  std::vector<std::pair<KeyFrame *, MapPoint *>> to_erase;
  for (int pass = 0; pass < 2; ++pass)  // mono edges first, then stereo
    for (size_t i = 0; i < edges.size(); ++i)
      if ((edges[i].ur < 0.f) == (pass == 0) && outlier[i] && !edge_ref[i].second->isBad())
        to_erase.push_back(edge_ref[i]);
  const float err = (float)stats[0], err_end = (float)stats[1];
  std::unique_lock<std::mutex> lock(pMap->mMutexMapUpdate);
  if ((2 * err < err_end || std::isnan(err) || std::isnan(err_end)) && !bLarge) {
    std::cout << "FAIL LOCAL-INERTIAL BA!!!!" << std::endl;
    return;
  }
  for (auto &ke : to_erase) {
    ke.first->EraseMapPointMatch(ke.second);
    ke.second->EraseObservation(ke.first);
  }
  for (KeyFrame *k : fixed_kfs) k->mnBAFixedForKF = 0;
  for (int i = 0; i < N; ++i) {
    const orbgpu_imu_state &o = out_states[i];
    Eigen::Matrix3f Rcw;
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) Rcw(r, c) = o.Rcw[3 * r + c];
    opt[i]->SetPose(Sophus::SE3f(Rcw, Eigen::Vector3f(o.tcw[0], o.tcw[1], o.tcw[2])));
    opt[i]->mnBALocalForKF = 0;
    if (opt[i]->bImu) {
      opt[i]->SetVelocity(Eigen::Vector3f(o.v[0], o.v[1], o.v[2]));
      opt[i]->SetNewBias(IMU::Bias(o.ba[0], o.ba[1], o.ba[2], o.bg[0], o.bg[1], o.bg[2]));
    }
  }
  for (size_t p = 0; p < mps.size(); ++p) {
    mps[p]->SetWorldPos(Eigen::Vector3f(pts_out[3 * p], pts_out[3 * p + 1], pts_out[3 * p + 2]));
    mps[p]->UpdateNormalAndDepth();
  }
  pMap->IncreaseChangeIndex();
}

}  // namespace ORB_SLAM_FUSION
