"""Seeded synthetic workloads from liborbsynth.so: stereo frames
for the extractor and pose-only problems.  Shared by tests/ and bench.py."""
from __future__ import annotations

import ctypes
from functools import lru_cache

import numpy as np

from ._lib import (IMU_CALIB_DTYPE, IMU_PREINT_DTYPE, IMU_STATE_DTYPE, LBA_EDGE_DTYPE, LIA_DOWNWEIGHT,
                   LIA_IMU_EDGE_DTYPE, LIA_ROBUST, LIB_DIR, POSE_OBS_DTYPE)

FRAME_SEED_BASE = 0x5EED0000
POSE_SEED = 7
LBA_SEED = 11
LIA_SEED = 13


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


# ---------------------------------------------------------------------------
# LocalInertialBA windows (numpy): a stereo-inertial body flying forward, key
# frames every 0.2 s, the temporal window of the newest n_opt key frames, the
# key frame before it and n_fixed_cov older observers as fixed key frames.
def _hat(w):
    return np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]], float)


def _exp_so3(w):
    w = np.asarray(w, float)
    d2 = float(w @ w)
    d = np.sqrt(d2)
    W = _hat(w)
    if d < 1e-5:
        return np.eye(3) + W + 0.5 * W @ W
    return np.eye(3) + W * np.sin(d) / d + W @ W * (1.0 - np.cos(d)) / d2


def _polar(R):
    U, _, Vt = np.linalg.svd(R)
    return U @ Vt


def _clean_info(M):
    M = (M + M.T) / 2
    w, V = np.linalg.eigh(M)
    w[w < 1e-12] = 0
    return V @ np.diag(w) @ V.T


LIA_G = np.array([0.0, 0.0, -float(np.float32(9.81))])
LIA_CAM = (435.2, 435.2, 376.0, 240.0, float(np.float32(435.2 * 0.11)))


def lia_calib() -> np.ndarray:
    """Pinhole + mTcb / mTbc of a forward-looking camera on a body with x
    forward, z up (the tests' inertial calibration)."""
    c = np.zeros((), IMU_CALIB_DTYPE)
    c["fx"], c["fy"], c["cx"], c["cy"], c["bf"] = LIA_CAM
    Rbc = np.array([[0, 0, 1], [-1, 0, 0], [0, -1, 0]], float) @ _exp_so3([0.01, -0.02, 0.015])
    tbc = np.array([0.05, -0.02, 0.01])
    Rbc32, tbc32 = Rbc.astype(np.float32), tbc.astype(np.float32)
    Rcb = Rbc32.astype(float).T
    tcb = -Rcb @ tbc32.astype(float)
    c["Rbc"], c["tbc"] = Rbc32.ravel(), tbc32
    c["Rcb"], c["tcb"] = Rcb.astype(np.float32).ravel(), tcb.astype(np.float32)
    return c


def lia_state(c, Rwb, twb, v, bg, ba) -> np.ndarray:
    """orbgpu_imu_state of a key frame: ImuCamPose(pKF) + the vertex estimates."""
    s = np.zeros((), IMU_STATE_DTYPE)
    Rcb = c["Rcb"].astype(float).reshape(3, 3)
    Rcw = Rcb @ Rwb.T
    tcw = Rcb @ (-Rwb.T @ twb) + c["tcb"].astype(float)
    s["Rwb"], s["twb"], s["Rcw"], s["tcw"] = Rwb.ravel(), twb, Rcw.ravel(), tcw
    s["v"], s["bg"], s["ba"] = v, bg, ba
    return s


class LiaProblem:
    """One LocalInertialBA window in the C ABI's layout: calib; kfs / kfs_true
    (IMU_STATE_DTYPE [n_kf]: the temporal key frames newest first, then the
    fixed ones, the key frame before the window first); fixed, imu uint8
    [n_kf]; pts_init / pts_true [n_pts, 3]; close uint8 [n_pts]; edges
    (LBA_EDGE_DTYPE, per point its observers in key-frame order); imu_edges
    (LIA_IMU_EDGE_DTYPE, temporal key frame i -> its mPrevKF, i = 0 .. N-1);
    iterations / lambda_init as LocalInertialBA sets them (:2334-2339,
    :2448-2459); outliers (bool per edge, the injected gross errors)."""

    def __init__(self, **kw):
        self.__dict__.update(kw)


def lia_problem(seed: int = LIA_SEED, n_opt: int = 10, n_fixed_cov: int = 10, n_pts: int = 2000,
                max_obs: int = 8, outlier_frac: float = 0.05, stereo_frac: float = 0.5,
                b_large: bool = False, rec_init: bool = False, perturb: float = 1.0,
                no_imu: tuple = (), max_depth: float = 40.0, consecutive: bool = False,
                kf_rot_scale: tuple = ()) -> LiaProblem:
    """no_imu: window indices of key frames without IMU data (`!pKFi->bImu`:
    VertexPose only, optimizer.cc:2466-2484) -- the temporal links touching
    them are left out, as :2503 skips them.  max_depth: farthest visible
    depth.  consecutive: a point's observers are max_obs consecutive key
    frames of those that see it (a banded window) instead of a random
    subset.  kf_rot_scale: per free key frame (window order), a multiplier of
    its initial rotation error only (LM updates of very different sizes within
    one trial)."""
    rng = np.random.default_rng(seed)
    c = lia_calib()
    fx, fy, cx, cy, bf = LIA_CAM
    n_tot = n_opt + 1 + n_fixed_cov
    dt = 0.2
    # true trajectory, oldest first: forward flight with a weaving yaw
    times = np.arange(n_tot) * dt
    R_true, t_true, v_true = [], [], []
    for t in times:
        yaw = 0.15 * np.sin(0.9 * t)
        R_true.append(_exp_so3([0.02 * np.sin(1.3 * t), 0.03 * np.sin(0.7 * t), yaw]))
        t_true.append(np.array([1.0 * t, 0.4 * np.sin(0.8 * t), 0.1 * np.sin(1.1 * t)]))
        v_true.append(np.array([1.0, 0.32 * np.cos(0.8 * t), 0.11 * np.cos(1.1 * t)]))
    bg0, ba0 = rng.normal(0, 0.01, 3), rng.normal(0, 0.05, 3)
    bg_true = [bg0 + rng.normal(0, 1e-4, 3) * k for k in range(n_tot)]
    ba_true = [ba0 + rng.normal(0, 1e-3, 3) * k for k in range(n_tot)]
    # key frame order of the window: newest first (pKF, mPrevKF, ...), then
    # the fixed key frame before the window, then older observers
    order = list(range(n_tot - 1, -1, -1))
    kfs_true = np.zeros(n_tot, IMU_STATE_DTYPE)
    kfs = np.zeros(n_tot, IMU_STATE_DTYPE)
    fixed = np.zeros(n_tot, np.uint8)
    fixed[n_opt:] = 1
    s = perturb
    for i, k in enumerate(order):
        kfs_true[i] = lia_state(c, R_true[k], t_true[k], v_true[k], bg_true[k], ba_true[k])
        if fixed[i]:
            kfs[i] = kfs_true[i]
        else:
            rs = kf_rot_scale[i] if i < len(kf_rot_scale) else 1.0
            kfs[i] = lia_state(c, R_true[k] @ _exp_so3(rng.normal(0, 3e-3 * s, 3) * rs),
                               t_true[k] + rng.normal(0, 2e-2 * s, 3),
                               v_true[k] + rng.normal(0, 2e-2 * s, 3),
                               bg_true[k] + rng.normal(0, 1e-3 * s, 3),
                               ba_true[k] + rng.normal(0, 5e-3 * s, 3))
    imu = np.ones(n_tot, np.uint8)
    for i in no_imu:
        assert 0 <= i < n_opt
        imu[i] = 0
    # points ahead of the flight, observed by the key frames that see them
    span = times[-1]
    P = np.stack([rng.uniform(3.0, span + 22.0, 4 * n_pts), rng.uniform(-8, 8, 4 * n_pts),
                  rng.uniform(-3, 3, 4 * n_pts)], 1)
    Rcw_t = [kfs_true[i]["Rcw"].astype(float).reshape(3, 3) for i in range(n_tot)]
    tcw_t = [kfs_true[i]["tcw"].astype(float) for i in range(n_tot)]
    # visibility of every candidate from every key frame, one key frame at a time
    vis_of = [[] for _ in range(len(P))]
    for i in range(n_tot):
        Xc = P @ Rcw_t[i].T + tcw_t[i]
        with np.errstate(divide="ignore", invalid="ignore"):
            u = fx * Xc[:, 0] / Xc[:, 2] + cx
            v = fy * Xc[:, 1] / Xc[:, 2] + cy
        ok = (Xc[:, 2] >= 0.5) & (Xc[:, 2] <= max_depth) & (u >= 0) & (u < 752) & (v >= 0) & (v < 480)
        for j in np.nonzero(ok)[0]:
            vis_of[j].append((i, Xc[j, 2], u[j], v[j]))
    pts, obs_lists = [], []
    for X, vis in zip(P, vis_of):
        if len(vis) < 2 or not any(i < n_opt for i, *_ in vis):
            continue
        if len(vis) > max_obs:
            if consecutive:
                j0 = int(rng.integers(0, len(vis) - max_obs + 1))
                keep = np.arange(j0, j0 + max_obs)
            else:
                keep = np.sort(rng.choice(len(vis), max_obs, replace=False))
            vis = [vis[j] for j in keep]
            if not any(i < n_opt for i, *_ in vis):
                continue
        pts.append(X)
        obs_lists.append(vis)
        if len(pts) == n_pts:
            break
    pts_true = np.array(pts, float)
    n_p = len(pts_true)
    rows, bad = [], []
    for p, vis in enumerate(obs_lists):
        for i, z, u, v in vis:
            octave = int(rng.integers(0, 8))
            inv_s2 = np.float32(1.0) / np.float32(1.2) ** np.float32(2 * octave)
            sig = float(np.sqrt(1.0 / inv_s2))
            uo, vo = u + rng.normal() * sig, v + rng.normal() * sig
            is_bad = rng.random() < outlier_frac
            if is_bad:
                uo += rng.choice([-1, 1]) * rng.uniform(15, 60)
            ur = u - bf / z + rng.normal() * sig if rng.random() < stereo_frac else -1.0
            rows.append((p, i, uo, vo, ur, inv_s2))
            bad.append(is_bad)
    edges = np.array(rows, LBA_EDGE_DTYPE)
    pts_init = (pts_true + rng.normal(0, 0.03 * s, pts_true.shape)).astype(np.float32)
    close = np.array([(Rcw_t[0] @ X + tcw_t[0])[2] < 10.0 for X in pts_true], np.uint8)
    # preintegration of every temporal link (kf i -> mPrevKF = kf i + 1)
    ie = np.zeros(n_opt, LIA_IMU_EDGE_DTYPE)
    for i in range(n_opt):
        k2, k1 = order[i], order[i + 1]
        R1, R2, t1, t2, v1, v2 = R_true[k1], R_true[k2], t_true[k1], t_true[k2], v_true[k1], v_true[k2]
        pi = ie[i]["preint"]
        pi["dT"] = dt
        dR = _polar(R1.T @ R2 @ _exp_so3(rng.normal(0, 2e-4, 3)))
        pi["dR"] = dR.astype(np.float32).ravel()
        pi["dV"] = R1.T @ (v2 - v1 - LIA_G * dt) + rng.normal(0, 2e-3, 3)
        pi["dP"] = R1.T @ (t2 - t1 - v1 * dt - 0.5 * LIA_G * dt * dt) + rng.normal(0, 2e-4, 3)
        a = R1.T @ ((v2 - v1) / dt - LIA_G)
        pi["JRg"] = (-dt * np.eye(3) + rng.normal(0, 1e-3, (3, 3))).ravel()
        pi["JVg"] = (0.5 * dt * dt * _hat(a) + rng.normal(0, 1e-4, (3, 3))).ravel()
        pi["JVa"] = (-dt * dR + rng.normal(0, 1e-4, (3, 3))).ravel()
        pi["JPg"] = (dt ** 3 / 6 * _hat(a) + rng.normal(0, 1e-5, (3, 3))).ravel()
        pi["JPa"] = (-0.5 * dt * dt * dR + rng.normal(0, 1e-5, (3, 3))).ravel()
        pi["bg"] = bg_true[k1] + rng.normal(0, 2e-3, 3)
        pi["ba"] = ba_true[k1] + rng.normal(0, 1e-2, 3)
        sg = np.concatenate([np.full(3, 1e-3), np.full(3, 1e-2), np.full(3, 1e-3)])
        L = rng.normal(0, 0.2, (9, 9)) * np.outer(sg, sg)
        C9 = np.diag(sg ** 2) + L @ L.T * 0.1
        pi["info"] = _clean_info(np.linalg.inv(C9.astype(np.float32).astype(float))).ravel()
        Cg = np.diag(np.full(3, (1.7e-4) ** 2 * dt)).astype(np.float32).astype(float)
        Ca = np.diag(np.full(3, (3e-3) ** 2 * dt)).astype(np.float32).astype(float)
        pi["info_g"] = np.linalg.inv(Cg).ravel()
        pi["info_a"] = np.linalg.inv(Ca).ravel()
        ie[i]["kf1"], ie[i]["kf2"] = i + 1, i
        ie[i]["flags"] = ((LIA_ROBUST | LIA_DOWNWEIGHT) if i == n_opt - 1 else 0) | \
            (LIA_ROBUST if rec_init else 0)
    ie = ie[[bool(imu[i] and imu[i + 1]) for i in range(n_opt)]]  # pKFi->bImu && mPrevKF->bImu
    return LiaProblem(calib=c, kfs=kfs, kfs_true=kfs_true, fixed=fixed, imu=imu,
                      pts_init=pts_init, pts_true=pts_true.astype(np.float32), close=close,
                      edges=edges, imu_edges=ie, outliers=np.array(bad, bool),
                      iterations=4 if b_large else 10, lambda_init=1e-2 if b_large else 1e0,
                      b_large=b_large)
