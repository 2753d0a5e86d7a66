"""Host mirror of the ORBmatcher projection searches over the gfx950 C ABI.

``ORBmatcher(nnratio, checkOri)`` follows include/cam/orb_feature/orb_matcher.h
for the pinhole rig (Frame::Nleft == -1):

* ``SearchByProjection_last(F, last_points, Tcw, Tlw, th, bMono)`` --
  SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, th, bMono)
  (orb_matcher.cc:1518-1728), the motion-model search of
  Tracking::TrackWithMotionModel (tracking.cc:2163-2216);
* ``SearchByProjection_local(F, points, views, th, bFarPoints, thFarPoints)`` --
  SearchByProjection(Frame& F, const vector<MapPoint*>&, th, bFarPoints,
  thFarPoints) (orb_matcher.cc:42-206);
* ``is_in_frustum(F, points, viewingCosLimit)`` -- Frame::isInFrustum
  (frame.cc:548-603) over Tracking::SearchLocalPoints' loop;
* ``search_local_points(...)`` -- both in one call (tracking.cc:2626-2690);
* ``SearchByProjection_kf(F, kf_points, kf_angles, th, ORBdist)`` --
  SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF, const
  set<MapPoint*>& sAlreadyFound, th, ORBdist) (orb_matcher.cc:1730-1839), the
  search of Tracking::Relocalization (tracking.cc:2967-2997);
* ``SearchByBoW(kf, F)`` -- SearchByBoW(KeyFrame* pKF, Frame& F,
  vector<MapPoint*>&) (orb_matcher.cc:215-389), the search of
  Tracking::TrackReferenceKeyFrame and Relocalization (tracking.cc:2043-2067,
  2904-2926).

``MatchFrame`` carries the Frame fields the searches read.  Results: match[i]
per current keypoint (>= 0: mvpMapPoints[i] = that query point; -1:
untouched; -2: set to NULL by the rotation check) and the return value.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import Optional, Tuple

import numpy as np

from ._lib import (KEYPOINT_DTYPE, MAP_POINT_DTYPE, MAX_LEVELS, PROJ_POINT_DTYPE,
                   TRACK_VIEW_DTYPE, Camera, FrameGeom, check, lib, ptr)
from .extractor import launch_stream

TH_HIGH, TH_LOW, HISTO_LENGTH = 100, 50, 30  # orb_matcher.cc:35-37


def frame_geom(width: float, height: float, scale_factors, min_x: float = 0.0,
               min_y: float = 0.0) -> FrameGeom:
    """Frame::ComputeImageBounds for undistorted images (frame.cc:820-825) plus
    the scale tables (mvScaleFactors, mfLogScaleFactor = logf(scale[1]))."""
    sf = np.asarray(scale_factors, np.float32)
    g = FrameGeom()
    g.min_x, g.max_x, g.min_y, g.max_y = float(min_x), float(width), float(min_y), float(height)
    g.n_levels = len(sf)
    g.log_scale_factor = float(np.log(np.float32(sf[1] if len(sf) > 1 else 1.2)))
    for i in range(MAX_LEVELS):
        g.scale_factors[i] = float(sf[i]) if i < len(sf) else 0.0
    return g


@dataclass
class MatchFrame:
    """The current Frame as the searches read it."""

    geom: FrameGeom
    cam: np.ndarray                 # float32 [fx, fy, cx, cy, bf]
    mb: float                       # Frame::mb
    kps: np.ndarray                 # KEYPOINT_DTYPE [N] (mvKeysUn)
    desc: np.ndarray                # uint8 [N, 32] (mDescriptors)
    uright: Optional[np.ndarray] = None   # float32 [N] (mvuRight)
    claimed: Optional[np.ndarray] = None  # uint8 [N]: mvpMapPoints[i] with observations
    pose: Optional[np.ndarray] = None     # float32 Tcw (qx, qy, qz, qw, tx, ty, tz)


def _c(a, dtype):
    return None if a is None else np.ascontiguousarray(a, dtype=dtype)


def pose_matrices(pose: np.ndarray) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Frame::UpdatePoseMatrices inputs for isInFrustum: (Rcw row-major [9], tcw, Ow)
    from a Tcw quaternion pose, in float32 (the shim reads the Frame's own
    mRcw / mtcw / mOw instead)."""
    q = np.asarray(pose[:4], np.float64)
    x, y, z, w = q / np.linalg.norm(q)
    R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                  [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                  [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])
    t = np.asarray(pose[4:7], np.float64)
    return (R.astype(np.float32).reshape(9), t.astype(np.float32),
            (-(R.T @ t)).astype(np.float32))


class ORBmatcher:
    def __init__(self, nnratio: float = 0.6, checkOri: bool = True, device: int = 0,
                 max_keypoints: int = 8192, max_points: int = 16384):
        self.mfNNratio = float(nnratio)
        self.mbCheckOrientation = bool(checkOri)
        self._h = ctypes.c_void_p()
        check(lib().orbgpu_matcher_create(device, max_keypoints, max_points,
                                          ctypes.byref(self._h)), "orbgpu_matcher_create")

    # -- SearchByProjection(CurrentFrame, LastFrame, th, bMono) -------------
    def SearchByProjection_last(self, F: MatchFrame, last_points: np.ndarray, Tlw: np.ndarray,
                                th: float, bMono: bool) -> Tuple[int, np.ndarray]:
        kps, desc = _c(F.kps, KEYPOINT_DTYPE), _c(F.desc, np.uint8)
        pts = _c(last_points, PROJ_POINT_DTYPE)
        ur, cl = _c(F.uright, np.float32), _c(F.claimed, np.uint8)
        Tcw, Tl = _c(F.pose, np.float32), _c(Tlw, np.float32)
        n = len(kps)
        match = np.zeros(max(n, 1), np.int32)
        nm = ctypes.c_int()
        cam = Camera(*[float(v) for v in F.cam])
        check(lib().orbgpu_search_by_projection_last(
            self._h, ctypes.byref(F.geom), ctypes.byref(cam), float(F.mb), ptr(Tcw), ptr(Tl),
            ptr(kps), ptr(desc), ptr(ur), ptr(cl), n, ptr(pts), len(pts), float(th), int(bMono),
            int(self.mbCheckOrientation), ptr(match), ctypes.byref(nm)),
            "orbgpu_search_by_projection_last")
        return nm.value, match[:n]

    def search_last_batch(self, geom: FrameGeom, cam, mb: float, Tcw, Tlw, kps, desc, uright,
                          claimed, n, pts, npts, th: float, bMono: bool, match, nmatches,
                          stream=None) -> None:
        """Device tensors: Tcw / Tlw float32 [B, 7]; kps int32/float32 [B, K, 7]; desc uint8
        [B, K, 32]; uright float32 [B, K] or None; claimed uint8 [B, K] or None; n int32 [B];
        pts uint8 [B, P, 56] (PROJ_POINT layout); npts int32 [B]; match int32 [B, K];
        nmatches int32 [B]."""
        B, K = kps.shape[0], kps.shape[1]
        c = Camera(*[float(v) for v in cam])
        with launch_stream(stream) as s:
            check(lib().orbgpu_search_by_projection_last_batch(
                self._h, B, ctypes.byref(geom), ctypes.byref(c), float(mb), ptr(Tcw), ptr(Tlw),
                ptr(kps), ptr(desc), ptr(uright), ptr(claimed), ptr(n), K, ptr(pts), ptr(npts),
                pts.shape[1], float(th), int(bMono), int(self.mbCheckOrientation), ptr(match),
                ptr(nmatches), s), "orbgpu_search_by_projection_last_batch")

    def matches_to_pose_obs_batch(self, kps, uright, match, n, pts, inv_level_sigma2, obs, nobs,
                                  obs_index=None, stream=None) -> None:
        """PoseOptimization's observation list from this call's matches, on the device:
        kps [B, K, 7]; uright float32 [B, K] or None; match int32 [B, K]; n int32 [B];
        pts uint8 [B, P, 56]; obs float32 [B, S, 7] (POSE_OBS layout); nobs int32 [B];
        obs_index int32 [B, S] or None."""
        B, K = kps.shape[0], kps.shape[1]
        isg = np.ascontiguousarray(inv_level_sigma2, np.float32)
        with launch_stream(stream) as s:
            check(lib().orbgpu_matches_to_pose_obs_batch(
                self._h, B, ptr(kps), ptr(uright), ptr(match), ptr(n), K, ptr(pts),
                pts.shape[1], ptr(isg), len(isg), ptr(obs), obs.shape[1], ptr(nobs),
                ptr(obs_index), s), "orbgpu_matches_to_pose_obs_batch")

    def unproject_stereo_batch(self, cam, Tcw, kps, desc, depth, n, pts, npts,
                               stream=None) -> None:
        """Frame::UnprojectStereo of every stereo keypoint (mvDepth > 0) on the
        device -> LastFrame points: Tcw float32 [B, 7]; kps [B, K, 7]; desc uint8
        [B, K, 32]; depth float32 [B, K]; n int32 [B]; pts uint8 [B, P, 56];
        npts int32 [B]."""
        B, K = kps.shape[0], kps.shape[1]
        c = Camera(*[float(v) for v in cam])
        with launch_stream(stream) as s:
            check(lib().orbgpu_unproject_stereo_batch(
                self._h, B, ctypes.byref(c), ptr(Tcw), ptr(kps), ptr(desc), ptr(depth), ptr(n), K,
                ptr(pts), pts.shape[1], ptr(npts), s), "orbgpu_unproject_stereo_batch")

    def matches_to_inertial_obs_batch(self, kps, uright, match, n, pts, close, inv_level_sigma2,
                                      obs, nobs, obs_index=None, stream=None) -> None:
        """The same list for PoseInertialOptimizationLastFrame / LastKeyFrame:
        close uint8 [B, P] (MapPoint::mTrackDepth < 10) or None; obs uint8
        [B, S, 32] (INERTIAL_OBS layout)."""
        B, K = kps.shape[0], kps.shape[1]
        isg = np.ascontiguousarray(inv_level_sigma2, np.float32)
        with launch_stream(stream) as s:
            check(lib().orbgpu_matches_to_inertial_obs_batch(
                self._h, B, ptr(kps), ptr(uright), ptr(match), ptr(n), K, ptr(pts), ptr(close),
                pts.shape[1], ptr(isg), len(isg), ptr(obs), obs.shape[1], ptr(nobs),
                ptr(obs_index), s), "orbgpu_matches_to_inertial_obs_batch")

    def status(self, reset: bool = True, stream=None) -> int:
        """Sticky error bits of the *_batch calls (include/orbgpu.h
        orbgpu_matcher_status): 1 = frame over kp_stride (skipped), 2 = an
        observation list truncated at obs_stride, 4 = points beyond pt_stride."""
        err = ctypes.c_int()
        with launch_stream(stream) as s:
            check(lib().orbgpu_matcher_status(self._h, s, int(reset), ctypes.byref(err)),
                  "orbgpu_matcher_status")
        return err.value

    # -- SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist) ---
    def SearchByProjection_kf(self, F: MatchFrame, kf_points: np.ndarray, kf_angles: np.ndarray,
                              th: float, ORBdist: int) -> Tuple[int, np.ndarray]:
        """kf_points: MAP_POINT_DTYPE per key-frame keypoint (MP_SKIP for NULL,
        bad or already-found points); kf_angles: pKF->mvKeysUn[i].angle;
        F.claimed: CurrentFrame.mvpMapPoints[i] != NULL; F.pose = Tcw."""
        kps, desc = _c(F.kps, KEYPOINT_DTYPE), _c(F.desc, np.uint8)
        pts, ang = _c(kf_points, MAP_POINT_DTYPE), _c(kf_angles, np.float32)
        cl, Tcw = _c(F.claimed, np.uint8), _c(F.pose, np.float32)
        n = len(kps)
        match = np.zeros(max(n, 1), np.int32)
        nm = ctypes.c_int()
        cam = Camera(*[float(v) for v in F.cam])
        check(lib().orbgpu_search_by_projection_kf(
            self._h, ctypes.byref(F.geom), ctypes.byref(cam), ptr(Tcw), ptr(kps), ptr(desc),
            ptr(cl), n, ptr(pts), ptr(ang), len(pts), float(th), int(ORBdist),
            int(self.mbCheckOrientation), ptr(match), ctypes.byref(nm)),
            "orbgpu_search_by_projection_kf")
        return nm.value, match[:n]

    def search_kf_batch(self, geom: FrameGeom, cam, Tcw, kps, desc, claimed, n, pts, angles, npts,
                        th: float, ORBdist: int, match, nmatches, stream=None) -> None:
        """Device tensors: Tcw float32 [B, 7]; kps [B, K, 7]; desc uint8 [B, K, 32];
        claimed uint8 [B, K] or None; n int32 [B]; pts uint8 [B, P, 68] (MAP_POINT
        layout); angles float32 [B, P]; npts int32 [B]; match int32 [B, K];
        nmatches int32 [B]."""
        B, K = kps.shape[0], kps.shape[1]
        c = Camera(*[float(v) for v in cam])
        with launch_stream(stream) as s:
            check(lib().orbgpu_search_by_projection_kf_batch(
                self._h, B, ctypes.byref(geom), ctypes.byref(c), ptr(Tcw), ptr(kps), ptr(desc),
                ptr(claimed), ptr(n), K, ptr(pts), ptr(angles), ptr(npts), pts.shape[1],
                float(th), int(ORBdist), int(self.mbCheckOrientation), ptr(match),
                ptr(nmatches), s), "orbgpu_search_by_projection_kf_batch")

    # -- SearchByBoW(pKF, F, vpMapPointMatches) ----------------------------------
    def SearchByBoW(self, kf_featvec, kf_desc, kf_angles, kf_valid, f_featvec, f_desc,
                    f_angles) -> Tuple[int, np.ndarray]:
        """FeatureVectors as (nodes uint32 ascending, offsets int32 [n + 1],
        features uint32) -- BowVocabulary.transform's fv output; kf_valid uint8
        (point present and not bad).  -> (nmatches, match int32 [N_F]: key-frame
        feature index whose point F's keypoint receives, -1 none)."""
        kn, ko, kf = (_c(x, t) for x, t in zip(kf_featvec, (np.uint32, np.int32, np.uint32)))
        fn, fo, ff = (_c(x, t) for x, t in zip(f_featvec, (np.uint32, np.int32, np.uint32)))
        kd, fd = _c(kf_desc, np.uint8), _c(f_desc, np.uint8)
        ka, fa = _c(kf_angles, np.float32), _c(f_angles, np.float32)
        kv = _c(kf_valid, np.uint8)
        n = len(fd)
        match = np.zeros(max(n, 1), np.int32)
        nm = ctypes.c_int()
        check(lib().orbgpu_search_by_bow(
            self._h, ptr(kn), ptr(ko), ptr(kf), len(kn), ptr(kd), ptr(ka), ptr(kv), len(kd),
            ptr(fn), ptr(fo), ptr(ff), len(fn), ptr(fd), ptr(fa), n, self.mfNNratio,
            int(self.mbCheckOrientation), ptr(match), ctypes.byref(nm)), "orbgpu_search_by_bow")
        return nm.value, match[:n]

    def search_bow_batch(self, kf_fv, kf_desc, kf_angles, kf_valid, f_fv, f_desc, f_angles, f_n,
                         match, nmatches, f_angle_step: int = 1, stream=None) -> None:
        """Device tensors; kf_fv / f_fv = (nodes uint32 [B, S], offsets int32
        [B, S + 1], features uint32 [B, S], n_nodes int32 [B]) as
        BowVocabulary.transform_batch fills them; descriptors uint8 [B, S, 32];
        kf_angles float32 [B, S]; kf_valid uint8 [B, S]; f_angles: float32 [B, S]
        (step 1) or the frame keypoints' angle column (step 7); f_n int32 [B];
        match int32 [B, S]; nmatches int32 [B]."""
        B, KS, FS = kf_desc.shape[0], kf_desc.shape[1], f_desc.shape[1]
        with launch_stream(stream) as s:
            check(lib().orbgpu_search_by_bow_batch(
                self._h, B, ptr(kf_fv[0]), ptr(kf_fv[1]), ptr(kf_fv[2]), ptr(kf_fv[3]),
                ptr(kf_desc), ptr(kf_angles), ptr(kf_valid), KS, ptr(f_fv[0]), ptr(f_fv[1]),
                ptr(f_fv[2]), ptr(f_fv[3]), ptr(f_desc), ptr(f_angles), int(f_angle_step),
                ptr(f_n), FS, self.mfNNratio, int(self.mbCheckOrientation), ptr(match),
                ptr(nmatches), s), "orbgpu_search_by_bow_batch")

    # -- Frame::isInFrustum ---------------------------------------------------
    def is_in_frustum(self, F: MatchFrame, points: np.ndarray, viewingCosLimit: float,
                      views: Optional[np.ndarray] = None) -> np.ndarray:
        pts = _c(points, MAP_POINT_DTYPE)
        views = np.zeros(len(pts), TRACK_VIEW_DTYPE) if views is None else \
            np.ascontiguousarray(views, TRACK_VIEW_DTYPE)
        R, t, Ow = pose_matrices(F.pose)
        cam = Camera(*[float(v) for v in F.cam])
        check(lib().orbgpu_frustum(self._h, ctypes.byref(F.geom), ctypes.byref(cam), ptr(R),
                                   ptr(t), ptr(Ow), ptr(pts), len(pts), float(viewingCosLimit),
                                   ptr(views)), "orbgpu_frustum")
        return views

    # -- SearchByProjection(F, vpMapPoints, th, bFarPoints, thFarPoints) -----
    def SearchByProjection_local(self, F: MatchFrame, points: np.ndarray, views: np.ndarray,
                                 th: float, bFarPoints: bool = False,
                                 thFarPoints: float = 0.0) -> Tuple[int, np.ndarray]:
        kps, desc = _c(F.kps, KEYPOINT_DTYPE), _c(F.desc, np.uint8)
        pts, vw = _c(points, MAP_POINT_DTYPE), _c(views, TRACK_VIEW_DTYPE)
        ur, cl = _c(F.uright, np.float32), _c(F.claimed, np.uint8)
        n = len(kps)
        match = np.zeros(max(n, 1), np.int32)
        nm = ctypes.c_int()
        check(lib().orbgpu_search_by_projection_local(
            self._h, ctypes.byref(F.geom), ptr(kps), ptr(desc), ptr(ur), ptr(cl), n, ptr(pts),
            ptr(vw), len(pts), float(th), self.mfNNratio, int(bFarPoints), float(thFarPoints),
            ptr(match), ctypes.byref(nm)), "orbgpu_search_by_projection_local")
        return nm.value, match[:n]

    def search_local_points(self, F: MatchFrame, points: np.ndarray, viewingCosLimit: float,
                            th: float, bFarPoints: bool = False, thFarPoints: float = 0.0,
                            views: Optional[np.ndarray] = None
                            ) -> Tuple[int, np.ndarray, np.ndarray]:
        """isInFrustum over `points` then the local search: (nmatches, match, views)."""
        kps, desc = _c(F.kps, KEYPOINT_DTYPE), _c(F.desc, np.uint8)
        pts = _c(points, MAP_POINT_DTYPE)
        ur, cl = _c(F.uright, np.float32), _c(F.claimed, np.uint8)
        views = np.zeros(len(pts), TRACK_VIEW_DTYPE) if views is None else \
            np.ascontiguousarray(views, TRACK_VIEW_DTYPE)
        R, t, Ow = pose_matrices(F.pose)
        n = len(kps)
        match = np.zeros(max(n, 1), np.int32)
        nm = ctypes.c_int()
        cam = Camera(*[float(v) for v in F.cam])
        check(lib().orbgpu_search_local_points(
            self._h, ctypes.byref(F.geom), ctypes.byref(cam), ptr(R), ptr(t), ptr(Ow), ptr(kps),
            ptr(desc), ptr(ur), ptr(cl), n, ptr(pts), len(pts), float(viewingCosLimit),
            float(th), self.mfNNratio, int(bFarPoints), float(thFarPoints), ptr(views),
            ptr(match), ctypes.byref(nm)), "orbgpu_search_local_points")
        return nm.value, match[:n], views

    def close(self) -> None:
        if self._h:
            lib().orbgpu_matcher_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def level_thresholds(log_scale_factor: float, n_levels: int) -> np.ndarray:
    """The PredictScale thresholds the kernels use (host-only helper)."""
    thr = np.zeros(MAX_LEVELS - 1, np.float32)
    if lib().orbgpu_level_thresholds(float(log_scale_factor), int(n_levels), ptr(thr)) < 0:
        raise ValueError("bad PredictScale parameters")
    return thr


__all__ = ["ORBmatcher", "MatchFrame", "frame_geom", "level_thresholds", "pose_matrices",
           "TH_HIGH", "TH_LOW", "HISTO_LENGTH"]
