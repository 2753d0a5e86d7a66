"""Seeded synthetic workloads from liborbsynth.so: stereo frames
for the extractor and pose-only problems.  Shared by tests/ and bench.py."""
from __future__ import annotations

import ctypes
from functools import lru_cache

import numpy as np

from ._lib import LBA_EDGE_DTYPE, LIB_DIR, POSE_OBS_DTYPE

FRAME_SEED_BASE = 0x5EED0000
POSE_SEED = 7
LBA_SEED = 11


@lru_cache(None)
def _so() -> ctypes.CDLL:
    path = LIB_DIR / "liborbsynth.so"
    if not path.exists():
        raise OSError(f"{path} is missing: run `make`")
    so = ctypes.CDLL(str(path))
    so.synth_stereo_frame.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_void_p, ctypes.c_void_p]
    so.synth_track_pair.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_int] + [ctypes.c_void_p] * 4
    so.synth_sequence.argtypes = [ctypes.c_uint64] + [ctypes.c_int] * 5 + [ctypes.c_void_p] * 2
    so.synth_vocab_text.argtypes = [ctypes.c_uint64] + [ctypes.c_int] * 6 + [ctypes.c_char_p]
    so.synth_vocab_text.restype = ctypes.c_int
    so.synth_noise_image.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    so.synth_pose_problem.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_void_p]
    so.synth_lba_problem.argtypes = [ctypes.c_uint64] + [ctypes.c_int] * 5 + [ctypes.c_void_p] * 7
    so.synth_lba_problem.restype = ctypes.c_int
    return so


def stereo_frame(frame_idx: int, w: int = 752, h: int = 480, disparity: int = 24):
    left = np.zeros((h, w), np.uint8)
    right = np.zeros((h, w), np.uint8)
    _so().synth_stereo_frame(FRAME_SEED_BASE + frame_idx, w, h, disparity, left.ctypes.data,
                             right.ctypes.data)
    return left, right


def track_pair(frame_idx: int, shift: int = 6, w: int = 752, h: int = 480, disparity: int = 24):
    """Two consecutive stereo frames of a camera translating along x over the
    canvas plane: features move +shift px from the last frame to the current
    one.  Returns (last_left, last_right, cur_left, cur_right)."""
    ims = [np.zeros((h, w), np.uint8) for _ in range(4)]
    _so().synth_track_pair(FRAME_SEED_BASE + 0x10000 + frame_idx, w, h, disparity, shift,
                           *[im.ctypes.data for im in ims])
    return tuple(ims)


def sequence(seq_idx: int, n_frames: int, shift: int = 6, w: int = 752, h: int = 480,
             disparity: int = 24):
    """A stereo sequence (C3 / C5 on synthetic data): n_frames consecutive
    frames of a camera translating along x, features moving +shift px per
    frame, depth bf / disparity.  Returns (left [n, h, w], right [n, h, w])."""
    left = np.zeros((n_frames, h, w), np.uint8)
    right = np.zeros((n_frames, h, w), np.uint8)
    _so().synth_sequence(FRAME_SEED_BASE + 0x20000 + seq_idx, n_frames, w, h, disparity, shift,
                         left.ctypes.data, right.ctypes.data)
    return left, right


def vocab_text(path, seed: int = 3, k: int = 10, L: int = 6, scoring: int = 0,
               weighting: int = 0, stop_pct: int = 3, trailing_newline: bool = True) -> int:
    """Writes a DBoW2 text vocabulary (ORBvoc.txt layout, full k-ary tree of depth
    L; scoring / weighting as DBoW2's enums, default L1_NORM / TF_IDF like
    ORB-SLAM's vocabulary).  Returns the node count (root excluded)."""
    n = _so().synth_vocab_text(seed, k, L, scoring, weighting, stop_pct, int(trailing_newline),
                               str(path).encode())
    if n < 0:
        raise OSError(f"cannot write {path}")
    return n


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


class LbaProblem:
    """A LocalBundleAdjustment window (config C4 by default): cam[5];
    poses_true / poses_init [n_kf, 7] (Tcw as qx, qy, qz, qw, tx, ty, tz);
    fixed [n_kf] uint8; pts_true / pts_init [n_pts, 3]; edges LBA_EDGE_DTYPE."""

    def __init__(self, cam, poses_true, poses_init, fixed, pts_true, pts_init, edges):
        self.cam, self.poses_true, self.poses_init, self.fixed = cam, poses_true, poses_init, fixed
        self.pts_true, self.pts_init, self.edges = pts_true, pts_init, edges


def lba_problem(seed: int = LBA_SEED, n_kf: int = 20, n_pts: int = 3000, obs_per_pt: int = 6,
                n_fixed: int = 2, outlier_pct: int = 0) -> LbaProblem:
    cam = np.zeros(5, np.float32)
    pt = np.zeros((n_kf, 7), np.float32)
    pi = np.zeros((n_kf, 7), np.float32)
    fixed = np.zeros(n_kf, np.uint8)
    xt = np.zeros((n_pts, 3), np.float32)
    xi = np.zeros((n_pts, 3), np.float32)
    edges = np.zeros(n_pts * min(obs_per_pt, n_kf), LBA_EDGE_DTYPE)
    ne = _so().synth_lba_problem(seed, n_kf, n_pts, obs_per_pt, n_fixed, outlier_pct,
                                 cam.ctypes.data, pt.ctypes.data, pi.ctypes.data, fixed.ctypes.data,
                                 xt.ctypes.data, xi.ctypes.data, edges.ctypes.data)
    return LbaProblem(cam, pt, pi, fixed, xt, xi, edges[:ne])
