"""Host mirror of Optimizer::PoseOptimization over the gfx950 C ABI.

``PoseOptimization(frame)`` follows include/solver/g2o_solver/optimizer.h:64 /
optimizer.cc:762-1051 for the pinhole rig: the frame's matched observations
go in, the optimised pose (SetPose), per-observation outlier flags
(mvbOutlier) and the inlier count (return value) come out.  Fewer than 3
correspondences return 0 and leave the pose untouched, as the reference.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Optional

import numpy as np

from ._lib import POSE_OBS_DTYPE, Camera, check, lib, ptr
from .extractor import launch_stream


@dataclass
class PoseFrame:
    """The Frame fields PoseOptimization reads, flattened (one row per i with
    mvpMapPoints[i] != NULL, in index order)."""

    cam: np.ndarray           # float32 [fx, fy, cx, cy, bf]
    pose: np.ndarray          # float32 Tcw (qx, qy, qz, qw, tx, ty, tz)
    obs: np.ndarray           # POSE_OBS_DTYPE [n]
    outlier: Optional[np.ndarray] = None  # uint8 [n], written


class PoseOptimizer:
    def __init__(self, device: int = 0, max_problems: int = 1, max_obs: int = 4096,
                 trial_groups: int | None = None):
        self._h = ctypes.c_void_p()
        self.max_obs = max_obs
        check(
            lib().orbgpu_pose_ctx_create(device, max_problems, max_obs, ctypes.byref(self._h)),
            "orbgpu_pose_ctx_create",
        )
        if trial_groups is not None:  # speculative LM trial groups (1 or 2), see orbgpu.h
            check(lib().orbgpu_pose_ctx_set_trial_groups(self._h, trial_groups, trial_groups),
                  "orbgpu_pose_ctx_set_trial_groups")

    def PoseOptimization(self, frame: PoseFrame) -> int:
        obs = np.ascontiguousarray(frame.obs, dtype=POSE_OBS_DTYPE)
        n = len(obs)
        cam = Camera(*[float(v) for v in frame.cam])
        pin = np.ascontiguousarray(frame.pose, dtype=np.float32)
        pout = np.zeros(7, np.float32)
        out = np.zeros(max(n, 1), np.uint8)
        inl = ctypes.c_int()
        check(
            lib().orbgpu_pose_opt(
                self._h, ctypes.byref(cam), ptr(pin), ptr(obs), n, ptr(pout), ptr(out),
                ctypes.byref(inl),
            ),
            "orbgpu_pose_opt",
        )
        frame.pose = pout
        frame.outlier = out[:n]
        return inl.value

    def batch(self, cam, pose_in, obs, nobs, pose_out, outlier, inliers, pose_out_d=None,
              stream=None) -> None:
        """Device tensors: pose_in/pose_out float32 [P, 7]; obs [P, stride, 7] float32
        (POSE_OBS layout); nobs int32 [P]; outlier uint8 [P, stride]; inliers int32 [P];
        pose_out_d optional float64 [P, 7]."""
        P, stride = obs.shape[0], obs.shape[1]
        c = Camera(*[float(v) for v in cam])
        with launch_stream(stream) as s:
            check(
                lib().orbgpu_pose_opt_batch(
                    self._h, ctypes.byref(c), ptr(pose_in), ptr(obs), ptr(nobs), stride, P,
                    ptr(pose_out), ptr(outlier), ptr(inliers), ptr(pose_out_d), s,
                ),
                "orbgpu_pose_opt_batch",
            )

    def close(self) -> None:
        if self._h:
            lib().orbgpu_pose_ctx_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
