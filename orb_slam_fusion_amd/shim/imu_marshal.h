// Marshalling of the reference's IMU types into the orbgpu C ABI structs,
// shared by the inertial drop-ins (optimizer_inertial_gpu.cc,
// optimizer_lia_gpu.cc).  Compiled inside the reference build.
#pragma once
#include "imu/imu_types.h"
#include "orbgpu.h"
#include "solver/g2o_solver/g2o_types.h"

namespace ORB_SLAM_FUSION {
namespace orbgpu_shim {

template <typename M>
inline void put(float *dst, const M &m) {  // row-major copy of a float matrix / vector
  for (int i = 0; i < m.rows(); ++i)
    for (int j = 0; j < m.cols(); ++j) dst[i * m.cols() + j] = m(i, j);
}
template <typename M>
inline void putd(double *dst, const M &m) {
  for (int i = 0; i < m.rows(); ++i)
    for (int j = 0; j < m.cols(); ++j) dst[i * m.cols() + j] = m(i, j);
}

// Pinhole params_ + bf + mImuCalib (Frame or KeyFrame)
template <typename F>
inline orbgpu_imu_calib calib_of(F *pF) {
  orbgpu_imu_calib c{};
  c.fx = pF->fx;
  c.fy = pF->fy;
  c.cx = pF->cx;
  c.cy = pF->cy;
  c.bf = pF->bf_;
  put(c.Rcb, pF->mImuCalib.mTcb.rotationMatrix());
  put(c.tcb, pF->mImuCalib.mTcb.translation());
  put(c.Rbc, pF->mImuCalib.mTbc.rotationMatrix());
  put(c.tbc, pF->mImuCalib.mTbc.translation());
  return c;
}

// IMU::Preintegrated -> deltas, Jacobians, linearisation bias and the
// informations EdgeInertial / EdgeGyroRW / EdgeAccRW derive from it.
inline orbgpu_imu_preint preint_of(IMU::Preintegrated *p) {
  orbgpu_imu_preint o{};
  o.dT = p->dT;
  put(o.dR, p->dR);
  put(o.dV, p->dV);
  put(o.dP, p->dP);
  put(o.JRg, p->JRg);
  put(o.JVg, p->JVg);
  put(o.JVa, p->JVa);
  put(o.JPg, p->JPg);
  put(o.JPa, p->JPa);
  o.bg[0] = p->b.bwx;
  o.bg[1] = p->b.bwy;
  o.bg[2] = p->b.bwz;
  o.ba[0] = p->b.bax;
  o.ba[1] = p->b.bay;
  o.ba[2] = p->b.baz;
  EdgeInertial ei(p);  // its constructor forms the information (g2o_types.cc:472-492)
  putd(o.info, ei.information());
  putd(o.info_g, Eigen::Matrix3d(p->C.block<3, 3>(9, 9).cast<double>().inverse()));
  putd(o.info_a, Eigen::Matrix3d(p->C.block<3, 3>(12, 12).cast<double>().inverse()));
  return o;
}

}  // namespace orbgpu_shim
}  // namespace ORB_SLAM_FUSION
