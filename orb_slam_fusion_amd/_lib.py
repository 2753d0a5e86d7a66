"""ctypes binding of the C ABI in include/orbgpu.h (liborbgpu.so).

The product path is the in-tree HIP library; there is no CPU fallback.  If the
library is missing or fails to load, every entry point raises -- loudly -- so a
GPU box can never pass on a silent fallback.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import numpy as np

PKG_DIR = Path(__file__).resolve().parent
LIB_DIR = PKG_DIR / "lib"
REPO_DIR = PKG_DIR.parent

ORBGPU_OK = 0
ORBGPU_ERR_INVALID = -1
ORBGPU_ERR_EMPTY = -2
ORBGPU_ERR_CAPACITY = -3
ORBGPU_ERR_DEVICE = -4
ORBGPU_ERR_NOMEM = -5
ORBGPU_RESIZE_SSE = 0
ORBGPU_LBA_SOLVER_AUTO = -1
ORBGPU_LBA_SOLVER_LDS = 0
ORBGPU_LBA_SOLVER_BLOCK = 1
ORBGPU_LBA_SOLVER_GRID = 2
ORBGPU_RESIZE_SCALAR = 1
ORBGPU_LBA_SCHUR_SPLIT = 0
ORBGPU_LBA_SCHUR_PAIR = 1
ORBGPU_LBA_SCHUR_BAND = 2
ORBGPU_OCTREE_NODES_AUTO = 0
ORBGPU_OCTREE_NODES_HBM = 1
ORBGPU_PYRAMID_PER_LEVEL = 0
ORBGPU_PYRAMID_FUSED = 1
ORBGPU_SINGLE_DATAFLOW = 0
ORBGPU_SINGLE_GRAPH = 1

STATUS_NAMES = {
    ORBGPU_OK: "OK",
    ORBGPU_ERR_INVALID: "INVALID",
    ORBGPU_ERR_EMPTY: "EMPTY",
    ORBGPU_ERR_CAPACITY: "CAPACITY",
    ORBGPU_ERR_DEVICE: "DEVICE",
    ORBGPU_ERR_NOMEM: "NOMEM",
}


class OrbGpuError(RuntimeError):
    def __init__(self, status: int, where: str):
        super().__init__(f"{where}: orbgpu status {status} ({STATUS_NAMES.get(status, '?')})")
        self.status = status


class OrbParams(ctypes.Structure):
    _fields_ = [
        ("num_features", ctypes.c_int),
        ("scale_factor", ctypes.c_float),
        ("num_levels", ctypes.c_int),
        ("ini_th_fast", ctypes.c_int),
        ("min_th_fast", ctypes.c_int),
    ]


class Camera(ctypes.Structure):
    _fields_ = [(n, ctypes.c_float) for n in ("fx", "fy", "cx", "cy", "bf")]


# cv::KeyPoint field order (28 bytes)
KEYPOINT_DTYPE = np.dtype(
    [
        ("x", "<f4"),
        ("y", "<f4"),
        ("size", "<f4"),
        ("angle", "<f4"),
        ("response", "<f4"),
        ("octave", "<i4"),
        ("class_id", "<i4"),
    ]
)
assert KEYPOINT_DTYPE.itemsize == 28

# orbgpu_pose_obs: Xw[3], u, v, ur, inv_sigma2
POSE_OBS_DTYPE = np.dtype(
    [("Xw", "<f4", (3,)), ("u", "<f4"), ("v", "<f4"), ("ur", "<f4"), ("inv_sigma2", "<f4")]
)
assert POSE_OBS_DTYPE.itemsize == 28

# orbgpu_lba_edge: point, kf, u, v, ur (< 0: mono), inv_sigma2
LBA_EDGE_DTYPE = np.dtype(
    [("point", "<i4"), ("kf", "<i4"), ("u", "<f4"), ("v", "<f4"), ("ur", "<f4"),
     ("inv_sigma2", "<f4")]
)
assert LBA_EDGE_DTYPE.itemsize == 24

# orbgpu_proj_point: a LastFrame observation projected by
# SearchByProjection(CurrentFrame, LastFrame)
PROJ_POINT_DTYPE = np.dtype(
    [("Xw", "<f4", (3,)), ("octave", "<i4"), ("angle", "<f4"), ("has_obs", "<i4"),
     ("desc", "u1", (32,))]
)
assert PROJ_POINT_DTYPE.itemsize == 56

# orbgpu_map_point: a local map point (isInFrustum + SearchByProjection(F, vpMapPoints))
MP_SKIP, MP_HAS_OBS = 1, 2
MAP_POINT_DTYPE = np.dtype(
    [("Xw", "<f4", (3,)), ("normal", "<f4", (3,)), ("min_dist", "<f4"), ("max_dist", "<f4"),
     ("flags", "<i4"), ("desc", "u1", (32,))]
)
assert MAP_POINT_DTYPE.itemsize == 68

# orbgpu_track_view: the MapPoint tracking fields isInFrustum writes
TRACK_VIEW_DTYPE = np.dtype(
    [("in_view", "<i4"), ("level", "<i4"), ("proj_x", "<f4"), ("proj_y", "<f4"),
     ("proj_xr", "<f4"), ("depth", "<f4"), ("view_cos", "<f4")]
)
assert TRACK_VIEW_DTYPE.itemsize == 28

MAX_LEVELS = 16

# PoseInertialOptimization inputs/outputs (orbgpu_imu_* in include/orbgpu.h)
_F9, _F3, _D9, _D3 = ("<f4", (9,)), ("<f4", (3,)), ("<f8", (9,)), ("<f8", (3,))
IMU_STATE_DTYPE = np.dtype([("Rwb",) + _F9, ("twb",) + _F3, ("Rcw",) + _F9, ("tcw",) + _F3,
                            ("v",) + _F3, ("bg",) + _F3, ("ba",) + _F3], align=True)
IMU_PREINT_DTYPE = np.dtype(
    [("dT", "<f4"), ("dR",) + _F9, ("dV",) + _F3, ("dP",) + _F3, ("JRg",) + _F9, ("JVg",) + _F9,
     ("JVa",) + _F9, ("JPg",) + _F9, ("JPa",) + _F9, ("bg",) + _F3, ("ba",) + _F3, ("pad_", "<f4"),
     ("info", "<f8", (81,)), ("info_g",) + _D9, ("info_a",) + _D9], align=True)
IMU_PRIOR_DTYPE = np.dtype([("Rwb",) + _D9, ("twb",) + _D3, ("vwb",) + _D3, ("bg",) + _D3,
                            ("ba",) + _D3, ("H", "<f8", (225,))], align=True)
IMU_CALIB_DTYPE = np.dtype([("fx", "<f4"), ("fy", "<f4"), ("cx", "<f4"), ("cy", "<f4"),
                            ("bf", "<f4"), ("Rcb",) + _F9, ("tcb",) + _F3, ("Rbc",) + _F9,
                            ("tbc",) + _F3], align=True)
INERTIAL_OBS_DTYPE = np.dtype([("Xw", "<f4", (3,)), ("u", "<f4"), ("v", "<f4"), ("ur", "<f4"),
                               ("inv_sigma2", "<f4"), ("close", "<i4")], align=True)
INERTIAL_RESULT_DTYPE = np.dtype(
    [("Rwb",) + _F9, ("twb",) + _F3, ("v",) + _F3, ("bg",) + _F3, ("ba",) + _F3,
     ("n_good", "<i4"), ("n_inliers", "<i4"), ("Rwb_d",) + _D9, ("twb_d",) + _D3, ("v_d",) + _D3,
     ("bg_d",) + _D3, ("ba_d",) + _D3, ("H", "<f8", (225,))], align=True)
assert (IMU_STATE_DTYPE.itemsize, IMU_PREINT_DTYPE.itemsize, IMU_PRIOR_DTYPE.itemsize,
        IMU_CALIB_DTYPE.itemsize, INERTIAL_OBS_DTYPE.itemsize,
        INERTIAL_RESULT_DTYPE.itemsize) == (132, 1064, 1968, 116, 32, 2064)
INERTIAL_LAST_FRAME, INERTIAL_LAST_KEYFRAME = 0, 1

# orbgpu_lia_imu_edge: one temporal link of LocalInertialBA (EdgeInertial +
# EdgeGyroRW + EdgeAccRW between key frames kf1 = mPrevKF and kf2)
LIA_IMU_EDGE_DTYPE = np.dtype([("kf1", "<i4"), ("kf2", "<i4"), ("flags", "<i4"), ("pad_", "<i4"),
                               ("preint", IMU_PREINT_DTYPE)], align=True)
assert LIA_IMU_EDGE_DTYPE.itemsize == 1080
LIA_ROBUST, LIA_DOWNWEIGHT = 1, 2


class FrameGeom(ctypes.Structure):
    """orbgpu_frame_geom: Frame::mnMinX/mnMaxX/mnMinY/mnMaxY, mnScaleLevels,
    mfLogScaleFactor, mvScaleFactors."""

    _fields_ = [
        ("min_x", ctypes.c_float),
        ("max_x", ctypes.c_float),
        ("min_y", ctypes.c_float),
        ("max_y", ctypes.c_float),
        ("n_levels", ctypes.c_int32),
        ("log_scale_factor", ctypes.c_float),
        ("scale_factors", ctypes.c_float * MAX_LEVELS),
    ]


_P = ctypes.c_void_p
_I = ctypes.c_int
_F = ctypes.c_float

# name -> (restype, argtypes); mirrors include/orbgpu.h
SIGNATURES = {
    "orbgpu_extractor_create": (_I, [ctypes.POINTER(OrbParams), _I, _I, _I, _I, ctypes.POINTER(_P)]),
    "orbgpu_extractor_destroy": (None, [_P]),
    "orbgpu_extractor_scales": (_I, [_P, _P, _P, _P, _P]),
    "orbgpu_extractor_levels": (_I, [_P]),
    "orbgpu_extractor_max_keypoints": (_I, [_P, _I, _I]),
    "orbgpu_extractor_set_resize_rounding": (_I, [_P, _I]),
    "orbgpu_extractor_set_octree_nodes": (_I, [_P, _I]),
    "orbgpu_extractor_set_pyramid_launch": (_I, [_P, _I]),
    "orbgpu_extractor_set_single_launch": (_I, [_P, _I]),
    "orbgpu_extractor_set_stage_event": (_I, [_P, _I, _P]),
    "orbgpu_extractor_plan": (_I, [_P, _I, _I, _P, _P]),
    "orbgpu_extract": (_I, [_P, _P, _I, _I, _I, _P, _P, _P, _I, _P, _P]),
    "orbgpu_extract_stereo": (_I, [_P, _P, _P, _P, _I, _I, _I, _P, _P, _P, _P, _I, _P, _P, _P, _P, _I, _P, _P]),
    "orbgpu_extractor_pyramid_level": (_I, [_P, _I, ctypes.POINTER(_P), _P, _P, _P]),
    "orbgpu_extract_batch": (
        _I,
        [_P, _P, _I, _I, _I, _I, ctypes.c_size_t, _P, _P, _P, _I, _P, _P, _P],
    ),
    "orbgpu_extractor_check": (_I, [_P]),
    "orbgpu_stereo_match_batch": (
        _I,
        [_P, _I, _P, _I, ctypes.c_size_t, _P, _P, _I, _P, ctypes.c_float, ctypes.c_float, _P, _P, _P],
    ),
    "orbgpu_stereo_match": (_I, [_P, _P, ctypes.c_float, ctypes.c_float, _P, _P, _I]),
    "orbgpu_extractor_stage": (_I, [_P, _I, _I, _P, _I]),
    "orbgpu_extractor_profile": (_I, [_P, _I]),
    "orbgpu_extractor_profile_read": (_I, [_P, _P]),
    "orbgpu_pose_ctx_create": (_I, [_I, _I, _I, ctypes.POINTER(_P)]),
    "orbgpu_pose_ctx_set_trial_groups": (_I, [_P, _I, _I]),
    "orbgpu_pose_ctx_destroy": (None, [_P]),
    "orbgpu_pose_opt": (_I, [_P, ctypes.POINTER(Camera), _P, _P, _I, _P, _P, _P]),
    "orbgpu_pose_opt_batch": (
        _I,
        [_P, ctypes.POINTER(Camera), _P, _P, _P, _I, _I, _P, _P, _P, _P, _P],
    ),
    "orbgpu_matcher_create": (_I, [_I, _I, _I, ctypes.POINTER(_P)]),
    "orbgpu_matcher_destroy": (None, [_P]),
    "orbgpu_matcher_status": (_I, [_P, _P, _I, ctypes.POINTER(_I)]),
    "orbgpu_search_by_projection_last": (
        _I,
        [_P, ctypes.POINTER(FrameGeom), ctypes.POINTER(Camera), _F, _P, _P, _P, _P, _P, _P, _I, _P,
         _I, _F, _I, _I, _P, _P],
    ),
    "orbgpu_search_by_projection_last_batch": (
        _I,
        [_P, _I, ctypes.POINTER(FrameGeom), ctypes.POINTER(Camera), _F, _P, _P, _P, _P, _P, _P, _P,
         _I, _P, _P, _I, _F, _I, _I, _P, _P, _P],
    ),
    "orbgpu_matches_to_pose_obs_batch": (
        _I, [_P, _I, _P, _P, _P, _P, _I, _P, _I, _P, _I, _P, _I, _P, _P, _P],
    ),
    "orbgpu_unproject_stereo_batch": (
        _I, [_P, _I, ctypes.POINTER(Camera), _P, _P, _P, _P, _P, _I, _P, _I, _P, _P],
    ),
    "orbgpu_matches_to_inertial_obs_batch": (
        _I, [_P, _I, _P, _P, _P, _P, _I, _P, _P, _I, _P, _I, _P, _I, _P, _P, _P],
    ),
    "orbgpu_frustum": (
        _I, [_P, ctypes.POINTER(FrameGeom), ctypes.POINTER(Camera), _P, _P, _P, _P, _I, _F, _P],
    ),
    "orbgpu_search_by_projection_local": (
        _I,
        [_P, ctypes.POINTER(FrameGeom), _P, _P, _P, _P, _I, _P, _P, _I, _F, _F, _I, _F, _P, _P],
    ),
    "orbgpu_search_local_points": (
        _I,
        [_P, ctypes.POINTER(FrameGeom), ctypes.POINTER(Camera), _P, _P, _P, _P, _P, _P, _P, _I, _P,
         _I, _F, _F, _F, _I, _F, _P, _P, _P],
    ),
    "orbgpu_search_by_projection_kf": (
        _I,
        [_P, ctypes.POINTER(FrameGeom), ctypes.POINTER(Camera), _P, _P, _P, _P, _I, _P, _P, _I, _F,
         _I, _I, _P, _P],
    ),
    "orbgpu_search_by_projection_kf_batch": (
        _I,
        [_P, _I, ctypes.POINTER(FrameGeom), ctypes.POINTER(Camera), _P, _P, _P, _P, _P, _I, _P, _P,
         _P, _I, _F, _I, _I, _P, _P, _P],
    ),
    "orbgpu_search_by_bow": (
        _I, [_P, _P, _P, _P, _I, _P, _P, _P, _I, _P, _P, _P, _I, _P, _P, _I, _F, _I, _P, _P],
    ),
    "orbgpu_search_by_bow_batch": (
        _I, [_P, _I, _P, _P, _P, _P, _P, _P, _P, _I, _P, _P, _P, _P, _P, _P, _I, _P, _I, _F, _I,
             _P, _P, _P],
    ),
    "orbgpu_level_thresholds": (_I, [_F, _I, _P]),
    "orbgpu_vocab_load_text": (_I, [_I, ctypes.c_char_p, ctypes.POINTER(_P)]),
    "orbgpu_vocab_destroy": (None, [_P]),
    "orbgpu_vocab_info": (_I, [_P, _P]),
    "orbgpu_bow_transform": (_I, [_P, _P, _I, _I, _P, _P, _P, _P, _P, _P, _P]),
    "orbgpu_bow_transform_batch": (
        _I, [_P, _I, _P, _P, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P],
    ),
    "orbgpu_inertial_ctx_create": (_I, [_I, _I, _I, ctypes.POINTER(_P)]),
    "orbgpu_inertial_ctx_destroy": (None, [_P]),
    "orbgpu_pose_inertial": (_I, [_P, _I, _P, _P, _P, _P, _P, _P, _I, _I, _P, _P]),
    "orbgpu_pose_inertial_batch": (
        _I, [_P, _I, _P, _I, _P, _P, _P, _P, _P, _P, _I, _I, _P, _P, _P],
    ),
    "orbgpu_lba_ctx_create": (_I, [_I, ctypes.POINTER(_P)]),
    "orbgpu_lba_ctx_set_reduce_ordered": (_I, [_P, _I]),
    "orbgpu_lba_ctx_set_solver": (_I, [_P, _I]),
    "orbgpu_lba_ctx_set_schur": (_I, [_P, _I]),
    "orbgpu_lba_ctx_set_relinearize": (_I, [_P, _I]),
    "orbgpu_lba_ctx_set_memory_limit": (_I, [_P, ctypes.c_size_t]),
    "orbgpu_lba_ctx_destroy": (None, [_P]),
    "orbgpu_lba_optimize": (
        _I,
        [_P, ctypes.POINTER(Camera), _I, _P, _P, _I, _P, _I, _P, _I, _I, _I, ctypes.c_double, _P,
         _P, _P, _P, _P, _P, _P, _P],
    ),
    "orbgpu_lia_optimize": (
        _I,
        [_P, _P, _I, _P, _P, _P, _I, _P, _P, _I, _P, _I, _P, _I, ctypes.c_double, _P, _P, _P, _P,
         _P],
    ),
}

# int (*orbgpu_lba_reduce_fn)(void* user, double* d_buf, int n, int op, void* hip_stream)
LBA_REDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                 ctypes.c_int, ctypes.c_void_p)

_lib = None


def library_path() -> Path:
    return Path(os.environ.get("ORBGPU_LIB", LIB_DIR / "liborbgpu.so"))


def lib() -> ctypes.CDLL:
    """Loads liborbgpu.so (raises if it is absent: no fallback exists)."""
    global _lib
    if _lib is None:
        path = library_path()
        if not path.exists():
            raise OSError(
                f"{path} is missing: build it with `make` (or __graft_entry__.build()); "
                "the orb_slam_fusion_amd hot path has no CPU fallback"
            )
        so = ctypes.CDLL(str(path))
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(so, name)
            fn.restype = res
            fn.argtypes = args
        _lib = so
    return _lib


def check(status: int, where: str) -> None:
    if status != ORBGPU_OK:
        raise OrbGpuError(status, where)


def ptr(a) -> ctypes.c_void_p:
    """Raw address of a numpy array or torch tensor (no copy)."""
    if a is None:
        return ctypes.c_void_p(0)
    if isinstance(a, np.ndarray):
        return ctypes.c_void_p(a.ctypes.data)
    return ctypes.c_void_p(a.data_ptr())
