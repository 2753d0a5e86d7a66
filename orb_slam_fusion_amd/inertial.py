"""Host mirror of Optimizer::PoseInertialOptimizationLastFrame /
PoseInertialOptimizationLastKeyFrame over the gfx950 C ABI.

``PoseInertialOptimizationLastFrame(problem)`` / ``...LastKeyFrame`` follow
optimizer.h (the two static members) / optimizer.cc:4762-5160 and
:4394-4760 for the pinhole rig: the frame's (and previous frame's / last key
frame's) IMU state, the preintegration between them, the previous frame's
ConstraintPoseImu (LastFrame) and the matched observations go in; the
optimised IMU pose, velocity and biases (SetImuPoseVelocity / mImuBias), the
outlier flags (mvbOutlier), the 15x15 Hessian for the new ConstraintPoseImu
and the return value (nInitialCorrespondences - nBad) come out.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Optional

import numpy as np

from ._lib import (IMU_CALIB_DTYPE, IMU_PREINT_DTYPE, IMU_PRIOR_DTYPE, IMU_STATE_DTYPE,
                   INERTIAL_LAST_FRAME, INERTIAL_LAST_KEYFRAME, INERTIAL_OBS_DTYPE,
                   INERTIAL_RESULT_DTYPE, check, lib, ptr)
from .extractor import launch_stream


@dataclass
class InertialProblem:
    """The Frame fields the inertial pose optimisations read (one row of obs
    per i with mvpMapPoints[i] != NULL, in index order)."""

    calib: np.ndarray                  # IMU_CALIB_DTYPE ()
    cur: np.ndarray                    # IMU_STATE_DTYPE (): the frame
    prev: np.ndarray                   # IMU_STATE_DTYPE (): mpPrevFrame / mpLastKeyFrame
    preint: np.ndarray                 # IMU_PREINT_DTYPE ()
    obs: np.ndarray                    # INERTIAL_OBS_DTYPE [n]
    prior: Optional[np.ndarray] = None  # IMU_PRIOR_DTYPE (): pFp->mpcpi (LastFrame)
    result: Optional[np.ndarray] = None   # INERTIAL_RESULT_DTYPE (), written
    outlier: Optional[np.ndarray] = None  # uint8 [n], written


class PoseInertialOptimizer:
    def __init__(self, device: int = 0, max_problems: int = 1, max_obs: int = 4096):
        self._h = ctypes.c_void_p()
        self.max_obs = max_obs
        check(lib().orbgpu_inertial_ctx_create(device, max_problems, max_obs,
                                               ctypes.byref(self._h)),
              "orbgpu_inertial_ctx_create")

    def _run(self, mode: int, pb: InertialProblem, rec_init: bool) -> int:
        calib = np.ascontiguousarray(pb.calib, IMU_CALIB_DTYPE)
        cur = np.ascontiguousarray(pb.cur, IMU_STATE_DTYPE)
        prev = np.ascontiguousarray(pb.prev, IMU_STATE_DTYPE)
        pre = np.ascontiguousarray(pb.preint, IMU_PREINT_DTYPE)
        prior = None if pb.prior is None else np.ascontiguousarray(pb.prior, IMU_PRIOR_DTYPE)
        obs = np.ascontiguousarray(pb.obs, INERTIAL_OBS_DTYPE)
        n = len(obs)
        res = np.zeros((), INERTIAL_RESULT_DTYPE)
        out = np.zeros(max(n, 1), np.uint8)
        check(lib().orbgpu_pose_inertial(self._h, mode, ptr(calib), ptr(cur), ptr(prev), ptr(pre),
                                         ptr(prior), ptr(obs), n, int(rec_init), ptr(res),
                                         ptr(out)),
              "orbgpu_pose_inertial")
        pb.result = res
        pb.outlier = out[:n]
        return int(res["n_good"])

    def PoseInertialOptimizationLastFrame(self, pb: InertialProblem, bRecInit: bool = False) -> int:
        return self._run(INERTIAL_LAST_FRAME, pb, bRecInit)

    def PoseInertialOptimizationLastKeyFrame(self, pb: InertialProblem,
                                             bRecInit: bool = False) -> int:
        return self._run(INERTIAL_LAST_KEYFRAME, pb, bRecInit)

    def batch(self, mode: int, calib: np.ndarray, cur, prev, preint, prior, obs, nobs, result,
              outlier, rec_init: bool = False, stream=None) -> None:
        """Device tensors (uint8 views of the record layouts): cur/prev
        [P, 132], preint [P, 1064], prior [P, 1968] (LastFrame, else None),
        obs [P, stride, 32], nobs int32 [P], result [P, 2064], outlier uint8
        [P, stride]."""
        P, stride = obs.shape[0], obs.shape[1]
        calib = np.ascontiguousarray(calib, IMU_CALIB_DTYPE)
        with launch_stream(stream) as s:
            check(lib().orbgpu_pose_inertial_batch(
                self._h, mode, ptr(calib), P, ptr(cur), ptr(prev), ptr(preint), ptr(prior),
                ptr(obs), ptr(nobs), stride, int(rec_init), ptr(result), ptr(outlier), s),
                "orbgpu_pose_inertial_batch")

    def close(self) -> None:
        if self._h:
            lib().orbgpu_inertial_ctx_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
