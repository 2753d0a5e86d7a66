"""Seeded synthetic workloads from liborbsynth.so: stereo frames
for the extractor and pose-only problems.  Shared by tests/ and bench.py."""
from __future__ import annotations

import ctypes
from functools import lru_cache

import numpy as np

from ._lib import LIB_DIR, POSE_OBS_DTYPE

FRAME_SEED_BASE = 0x5EED0000
POSE_SEED = 7


@lru_cache(None)
def _so() -> ctypes.CDLL:
    path = LIB_DIR / "liborbsynth.so"
    if not path.exists():
        raise OSError(f"{path} is missing: run `make`")
    so = ctypes.CDLL(str(path))
    so.synth_stereo_frame.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_void_p, ctypes.c_void_p]
    so.synth_noise_image.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    so.synth_pose_problem.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_void_p]
    return so


def stereo_frame(frame_idx: int, w: int = 752, h: int = 480, disparity: int = 24):
    left = np.zeros((h, w), np.uint8)
    right = np.zeros((h, w), np.uint8)
    _so().synth_stereo_frame(FRAME_SEED_BASE + frame_idx, w, h, disparity, left.ctypes.data,
                             right.ctypes.data)
    return left, right


def noise_image(seed: int, w: int, h: int) -> np.ndarray:
    out = np.zeros((h, w), np.uint8)
    _so().synth_noise_image(seed, w, h, out.ctypes.data)
    return out


def pose_problem(seed: int = POSE_SEED, n: int = 600, outlier_pct: int = 10):
    """Returns (cam[5], pose_init[7], pose_true[7], obs[n] POSE_OBS_DTYPE)."""
    obs = np.zeros(n, POSE_OBS_DTYPE)
    cam = np.zeros(5, np.float32)
    pt = np.zeros(7, np.float32)
    pi = np.zeros(7, np.float32)
    _so().synth_pose_problem(seed, n, outlier_pct, obs.ctypes.data, cam.ctypes.data, pt.ctypes.data,
                             pi.ctypes.data)
    return cam, pi, pt, obs
