// ORACLE (test infrastructure only): the inertial pieces shared by the
// tracking optimisations (inertial_oracle.cc: PoseInertialOptimizationLastFrame
// / LastKeyFrame) and LocalInertialBA (lia_oracle.cc) -- 3x3 algebra, the SO3
// maps of g2o_types.cc:779-848, the float side of IMU::Preintegrated
// (imu_types.cc:283-310), ImuCamPose::Update (g2o_types.cc:192-214) and
// EdgeInertial (g2o_types.cc:494-578) on two vertex sets.
#pragma once

#include <cstdint>

#include "../include/orbgpu.h"

namespace oracle {
namespace inertial {

struct M3 {
  double a[9];
  double& operator()(int r, int c) { return a[3 * r + c]; }
  double operator()(int r, int c) const { return a[3 * r + c]; }
};
struct V3 {
  double a[3];
  double& operator[](int i) { return a[i]; }
  double operator[](int i) const { return a[i]; }
};

M3 eye();
M3 mul(const M3& A, const M3& B);
M3 tr(const M3& A);
V3 mv(const M3& A, const V3& v);
V3 add(const V3& a, const V3& b);
V3 sub(const V3& a, const V3& b);
V3 scl(const V3& a, double s);
M3 hat(const V3& w);
M3 from_f(const float* f);
V3 from_f3(const float* f);
M3 from_d(const double* f);
V3 from_d3(const double* f);
M3 polar(const M3& R);
M3 ExpSO3(double x, double y, double z);
V3 LogSO3(const M3& R);
M3 InvRightJ(const V3& v);
M3 RightJ(const V3& v);

struct Preint {  // pointers into an orbgpu_imu_preint
  const float* dR;
  const float* dV;
  const float* dP;
  const float* JRg;
  const float* JVg;
  const float* JVa;
  const float* JPg;
  const float* JPa;
  const float* bg;  // linearisation bias
  const float* ba;
};
Preint preint_view(const orbgpu_imu_preint& p);

struct Calib {
  double fx, fy, cx, cy, bf;
  M3 Rcb, Rbc;
  V3 tcb, tbc;
};
Calib load_calib(const orbgpu_imu_calib& cb);

struct State {  // one frame's vertices
  M3 Rwb, Rcw;
  V3 twb, tcw, v, bg, ba;
};
State load_state(const orbgpu_imu_state& s);
void pose_update(State& s, const double* u, const Calib& c);  // ImuCamPose::Update

// IMU::GRAVITY_VALUE (float) as EdgeInertial's g = (0, 0, -9.81)
inline V3 gravity() { return V3{{0, 0, -(double)9.81f}}; }

// EdgeInertial between vertex set 1 (s1: VP1 VV1 VG1 VA1) and 2 (s2: VP2 VV2):
// error (9) and Jacobian J[9][24], columns VP1(6) VV1(3) VG1(3) VA1(3) VP2(6) VV2(3).
void inertial_edge_error(const State& s1, const State& s2, const Preint& pi, double dt, const V3& g,
                         double e[9]);
void inertial_edge_jacobian(const State& s1, const State& s2, const Preint& pi, double dt,
                            const V3& g, double J[9][24]);

// One edge's quadratic form into the n x n system (BaseMultiEdge::
// constructQuadraticForm with weight w = rho'(chi2), 1 without kernel).
// blocks: (solver offset or -1 for a fixed vertex, dim) in column order.
void add_quadratic(double* H, double* b, int n, int D, const double* J, int ldj, const double* Om,
                   const double* e, double w, const int (*blocks)[2], int nblk);
double quad(const double* Om, const double* e, int D);

}  // namespace inertial
}  // namespace oracle
