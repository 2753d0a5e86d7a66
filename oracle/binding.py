"""ORACLE binding (test infrastructure only).

ctypes access to oracle/_build/liborboracle.so -- the CPU restatement of the
reference hot path.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this module, and only as the checker / the CPU
baseline; nothing in orb_slam_fusion_amd/ may.
"""
from __future__ import annotations

import ctypes
from functools import lru_cache
from pathlib import Path

import numpy as np

ORACLE_DIR = Path(__file__).resolve().parent
LIB_PATH = ORACLE_DIR / "_build" / "liborboracle.so"

KEYPOINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                           ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
POSE_OBS_DTYPE = np.dtype([("Xw", "<f4", (3,)), ("u", "<f4"), ("v", "<f4"), ("ur", "<f4"),
                           ("inv_sigma2", "<f4")])
LBA_EDGE_DTYPE = np.dtype([("point", "<i4"), ("kf", "<i4"), ("u", "<f4"), ("v", "<f4"),
                           ("ur", "<f4"), ("inv_sigma2", "<f4")])
# int reduce(void* user, double* buf, int n, int op)   op: 0 sum, 1 max
LBA_REDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_double),
                                 ctypes.c_int, ctypes.c_int)

_P, _I, _F = ctypes.c_void_p, ctypes.c_int, ctypes.c_float


@lru_cache(None)
def lib() -> ctypes.CDLL:
    if not LIB_PATH.exists():
        raise OSError(f"{LIB_PATH} missing: run `make -C oracle`")
    so = ctypes.CDLL(str(LIB_PATH))
    sig = {
        "orc_extractor_new": (_P, [_I, _F, _I, _I, _I]),
        "orc_extractor_free": (None, [_P]),
        "orc_extract": (_I, [_P, _P, _I, _I, _I, _I, _I, _P, _P, _I, _P]),
        "orc_extract_stereo": (_I, [_P, _P, _P, _P, _I, _I, _I, _P, _P]),
        "orc_params": (None, [_P, _P, _P, _P, _P, _P, _P]),
        "orc_pyramid": (None, [_P, _P, _I, _I, _I]),
        "orc_level_size": (_I, [_P, _I, _P, _P]),
        "orc_level_copy": (None, [_P, _I, _I, _P]),
        "orc_stage": (_I, [_P, _I, _I, _P, _I]),
        "orc_resize": (None, [_P, _I, _I, _P, _I, _I]),
        "orc_set_resize_rounding": (None, [_I]),
        "orc_get_resize_rounding": (_I, []),
        "orc_gauss": (None, [_P, _I, _I, _P]),
        "orc_gauss_kernel": (None, [_P]),
        "orc_fast": (_I, [_P, _I, _I, _I, _I, _P, _I]),
        "orc_fast_atan2": (_F, [_F, _F]),
        "orc_sincosf": (None, [_P, _I, _P, _P]),
        "orc_sincosf_check_libm": (ctypes.c_long, [ctypes.c_uint, ctypes.c_uint]),
        "orc_pose_opt": (_I, [_P, _P, _P, _I, _P, _P, _P]),
        "orc_lba_edge_linearize": (_I, [_P, _P, _P, _P, _P, _P, _P]),
        "orc_se3_exp_compose": (None, [_P, _P, _P]),
        "orc_stereo_match": (_I, [_P, _I, _P, _P, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _F, _F,
                                  _P, _P]),
        "orc_lba": (_I, [_P, _I, _P, _P, _I, _P, _I, _P, _I, _I, _I, ctypes.c_double, _I,
                         LBA_REDUCE_FN, _P, _P, _P, _P, _P, _P]),
        "orc_search_last": (_I, [_P, _P, _F, _P, _P, _P, _P, _P, _P, _I, _P, _I, _F, _I, _I, _P]),
        "orc_frustum": (None, [_P, _P, _P, _P, _P, _P, _I, _F, _P]),
        "orc_search_kf": (_I, [_P, _P, _P, _P, _P, _P, _I, _P, _P, _I, _F, _I, _I, _P]),
        "orc_search_bow": (_I, [_P, _P, _P, _I, _P, _P, _P, _P, _P, _P, _I, _P, _P, _I, _F, _I,
                                _P]),
        "orc_search_local": (_I, [_P, _P, _P, _P, _P, _I, _P, _P, _I, _F, _F, _I, _F, _P]),
        "orc_predict_scale": (_I, [_F, _F, _F, _I]),
        "orc_predict_scale_check": (ctypes.c_long, [_F, _I, _P, ctypes.c_uint32, ctypes.c_uint32]),
        "orc_frame_grid_cells": (None, [_P, _P, _I, _P]),
        "orc_vocab_load": (_P, [ctypes.c_char_p]),
        "orc_vocab_free": (None, [_P]),
        "orc_vocab_info": (None, [_P, _P]),
        "orc_bow_transform": (None, [_P, _P, _I, _I, _P, _P, _P, _P, _P, _P, _P]),
        "orc_pose_inertial": (_I, [_I, _P, _P, _P, _P, _P, _P, _I, _I, _P, _P]),
        "orc_inertial_system": (None, [_I, _P, _P, _P, _P, _P, _P, _I, _I, _P, _P]),
        "orc_pose_inertial_ex": (_I, [_I, _P, _P, _P, _P, _P, _P, _I, _I, _P, _P, _P]),
        "orc_sym_pinv": (None, [_P, _I, _P]),
        "orc_lia": (_I, [_P, _I, _P, _P, _P, _I, _P, _P, _I, _P, _I, _P, _I, ctypes.c_double, _P,
                         _P, _P, _P, _P]),
        "orc_lia_system": (_I, [_P, _I, _P, _P, _P, _I, _P, _I, _P, _I, _P, _P, _P]),
        "orc_lia_vis_linearize": (None, [_P, _P, _P, _P, _P, _P, _P]),
    }
    for name, (res, args) in sig.items():
        f = getattr(so, name)
        f.restype, f.argtypes = res, args
    return so


def _p(a) -> ctypes.c_void_p:
    if a is None:
        return ctypes.c_void_p(0)
    if isinstance(a, ctypes.Structure):
        return ctypes.cast(ctypes.pointer(a), ctypes.c_void_p)
    return ctypes.c_void_p(a.ctypes.data)


class OracleExtractor:
    """CPU restatement of ORB_SLAM_FUSION::OrbExtractor (see orb_oracle.h)."""

    def __init__(self, num_feats=1000, scale_factor=1.2, num_levs=8, ini_th=20, min_th=7):
        self.L = num_levs
        self._h = lib().orc_extractor_new(num_feats, scale_factor, num_levs, ini_th, min_th)

    def __del__(self):
        try:
            lib().orc_extractor_free(self._h)
        except Exception:
            pass

    def extract(self, img: np.ndarray, lapping=(0, 0)):
        img = np.ascontiguousarray(img, np.uint8)
        h, w = img.shape
        cap = 8192
        while True:  # n is reported even when it exceeds cap: run again with room for it
            kps = np.zeros(cap, KEYPOINT_DTYPE)
            desc = np.zeros((cap, 32), np.uint8)
            n = ctypes.c_int()
            mono = lib().orc_extract(self._h, _p(img), w, h, w, int(lapping[0]), int(lapping[1]),
                                     _p(kps), _p(desc), cap, ctypes.byref(n))
            if n.value <= cap:
                break
            cap = n.value
        return mono, kps[: n.value].copy(), desc[: n.value].copy()

    def params(self):
        L = self.L
        s, i, s2, is2 = (np.zeros(L, np.float32) for _ in range(4))
        fpl = np.zeros(L, np.int32)
        umax = np.zeros(16, np.int32)
        lib().orc_params(self._h, _p(s), _p(i), _p(s2), _p(is2), _p(fpl), _p(umax))
        return dict(scale=s, inv_scale=i, sigma2=s2, inv_sigma2=is2, feats_per_level=fpl, umax=umax)

    def level(self, lev: int, blurred: bool = False) -> np.ndarray:
        w, h = ctypes.c_int(), ctypes.c_int()
        assert lib().orc_level_size(self._h, lev, ctypes.byref(w), ctypes.byref(h)) == 0
        out = np.zeros((h.value, w.value), np.uint8)
        lib().orc_level_copy(self._h, lev, int(blurred), _p(out))
        return out

    def pyramid(self, img: np.ndarray):
        img = np.ascontiguousarray(img, np.uint8)
        h, w = img.shape
        lib().orc_pyramid(self._h, _p(img), w, h, w)
        return [self.level(l) for l in range(self.L)]

    def stage(self, lev: int, which: int) -> np.ndarray:
        """which 0: FAST candidates in to_dist order; 1: octree output in list
        order.  Rows (x, y, response), coordinates relative to the 16-px border."""
        cap = 1 << 18
        buf = np.zeros((cap, 3), np.float32)
        n = lib().orc_stage(self._h, lev, which, _p(buf), cap)
        return buf[:n].copy()


RESIZE_SSE, RESIZE_SCALAR = 0, 1


class resize_rounding:
    """Context manager: the oracle's resize vertical-pass rounding
    for the duration of a block -- RESIZE_SSE (OpenCV 4.5.4, 128-bit SIMD
    body + scalar tail; the default) or RESIZE_SCALAR (every column scalar)."""

    def __init__(self, mode: int):
        self.mode = mode

    def __enter__(self):
        self.prev = lib().orc_get_resize_rounding()
        lib().orc_set_resize_rounding(self.mode)
        return self

    def __exit__(self, *exc):
        lib().orc_set_resize_rounding(self.prev)
        return False


def resize(src: np.ndarray, dw: int, dh: int) -> np.ndarray:
    src = np.ascontiguousarray(src, np.uint8)
    out = np.zeros((dh, dw), np.uint8)
    lib().orc_resize(_p(src), src.shape[1], src.shape[0], _p(out), dw, dh)
    return out


def gauss(src: np.ndarray) -> np.ndarray:
    src = np.ascontiguousarray(src, np.uint8)
    out = np.zeros_like(src)
    lib().orc_gauss(_p(src), src.shape[1], src.shape[0], _p(out))
    return out


def gauss_kernel():
    k = np.zeros(7, np.int32)
    lib().orc_gauss_kernel(_p(k))
    return k


def fast(roi: np.ndarray, th: int) -> np.ndarray:
    roi = np.ascontiguousarray(roi, np.uint8)
    cap = roi.size
    buf = np.zeros((cap, 3), np.int32)
    n = lib().orc_fast(_p(roi), roi.shape[1], roi.shape[1], roi.shape[0], th, _p(buf), cap)
    return buf[:n].copy()


def fast_atan2(y: float, x: float) -> float:
    return float(lib().orc_fast_atan2(y, x))


def sincosf(x: np.ndarray):
    x = np.ascontiguousarray(x, np.float32)
    s = np.zeros_like(x)
    c = np.zeros_like(x)
    lib().orc_sincosf(_p(x), x.size, _p(s), _p(c))
    return s, c


def sincosf_check_libm(lo_bits: int, hi_bits: int) -> int:
    return int(lib().orc_sincosf_check_libm(lo_bits, hi_bits))


def pose_opt(cam: np.ndarray, pose_in: np.ndarray, obs: np.ndarray):
    """Returns (inliers, pose_out float32[7], outlier uint8[n], pose_out float64[7])."""
    cam = np.ascontiguousarray(cam, np.float32)
    pose_in = np.ascontiguousarray(pose_in, np.float32)
    obs = np.ascontiguousarray(obs, POSE_OBS_DTYPE)
    n = len(obs)
    pout = np.zeros(7, np.float32)
    pd = np.zeros(7, np.float64)
    out = np.zeros(max(n, 1), np.uint8)
    inl = lib().orc_pose_opt(_p(cam), _p(pose_in), _p(obs), n, _p(pout), _p(out), _p(pd))
    return inl, pout, out[:n].copy(), pd


def lba(problem, iters: int = 10, pt_range=None, reduce=None, lambda_init: float = 0.0,
        stop_after_trials: int = -1):
    """LocalBundleAdjustment restatement on an LbaProblem-like object (cam,
    poses_init, fixed, pts_init, edges).  pt_range=(begin, end) restricts this
    call to a point shard; reduce(buf: np.ndarray[float64], op) -> None
    completes the shard sums in place (op 0 sum, 1 max).  lambda_init > 0:
    setUserLambdaInit; stop_after_trials >= 0: terminate() turns true once
    that many LM trials have run.  Returns dict with
    poses [n_kf, 7] f64, pts [n_pts, 3] f64 (shard rows only), outlier [E] u8
    (shard edges only), chi2 [E] f64 (each edge's chi2 at the classification:
    the last computeActiveErrors), stats [6]."""
    cam = np.ascontiguousarray(problem.cam, np.float32)
    poses = np.ascontiguousarray(problem.poses_init, np.float32)
    fixed = np.ascontiguousarray(problem.fixed, np.uint8)
    pts = np.ascontiguousarray(problem.pts_init, np.float32)
    edges = np.ascontiguousarray(problem.edges, LBA_EDGE_DTYPE)
    n_kf, n_pts, ne = len(poses), len(pts), len(edges)
    b, e = pt_range if pt_range is not None else (0, n_pts)
    po = np.zeros((n_kf, 7), np.float64)
    xo = np.zeros((n_pts, 3), np.float64)
    out = np.zeros(max(ne, 1), np.uint8)
    chi = np.zeros(max(ne, 1), np.float64)
    st = np.zeros(6, np.float64)
    if reduce is None:
        cb = LBA_REDUCE_FN(0)
    else:
        def _cb(_user, buf, n, op):
            try:
                arr = np.ctypeslib.as_array(buf, shape=(n,))
                reduce(arr, op)
                return 0
            except Exception:  # noqa: BLE001 -- reported as a failed reduce
                return -1
        cb = LBA_REDUCE_FN(_cb)
    rc = lib().orc_lba(_p(cam), n_kf, _p(poses), _p(fixed), n_pts, _p(pts), ne, _p(edges), b, e,
                       iters, float(lambda_init), int(stop_after_trials), cb, None, _p(po), _p(xo),
                       _p(out), _p(st), _p(chi))
    if rc != 0:
        raise RuntimeError(f"orc_lba failed ({rc})")
    return {"poses": po, "pts": xo, "outlier": out[:ne].copy(), "chi2": chi[:ne].copy(), "stats": st}


def lba_edge_linearize(cam, pose7, X, edge):
    """-> (depth_positive, err[3], Jl[3,3], Jp[3,6]) of one LBA edge."""
    cam = np.ascontiguousarray(cam, np.float32)
    pose7 = np.ascontiguousarray(pose7, np.float64)
    X = np.ascontiguousarray(X, np.float64)
    e = np.ascontiguousarray(np.array([edge], LBA_EDGE_DTYPE))
    err, jl, jp = np.zeros(3), np.zeros(9), np.zeros(18)
    d = lib().orc_lba_edge_linearize(_p(cam), _p(pose7), _p(X), _p(e), _p(err), _p(jl), _p(jp))
    return bool(d), err, jl.reshape(3, 3), jp.reshape(3, 6)


def se3_exp_compose(u6, pose7):
    u6 = np.ascontiguousarray(u6, np.float64)
    pose7 = np.ascontiguousarray(pose7, np.float64)
    out = np.zeros(7)
    lib().orc_se3_exp_compose(_p(u6), _p(pose7), _p(out))
    return out


def stereo_match(kps_l, desc_l, kps_r, desc_r, pyr_l, pyr_r, scale, inv_scale, bf, mb):
    """Frame::ComputeStereoMatches (frame.cc:828-986) on the oracle: returns
    (uright, depth, kept).  pyr_l / pyr_r: lists of the level planes."""
    kl = np.ascontiguousarray(kps_l, KEYPOINT_DTYPE)
    kr = np.ascontiguousarray(kps_r, KEYPOINT_DTYPE)
    dl = np.ascontiguousarray(desc_l, np.uint8)
    dr = np.ascontiguousarray(desc_r, np.uint8)
    L = len(pyr_l)
    pl = [np.ascontiguousarray(a, np.uint8) for a in pyr_l]
    pr = [np.ascontiguousarray(a, np.uint8) for a in pyr_r]
    ptr_l = (ctypes.c_void_p * L)(*[a.ctypes.data for a in pl])
    ptr_r = (ctypes.c_void_p * L)(*[a.ctypes.data for a in pr])
    lw = np.array([a.shape[1] for a in pl], np.int32)
    lh = np.array([a.shape[0] for a in pl], np.int32)
    sl = np.array([a.strides[0] for a in pl], np.int32)
    sr = np.array([a.strides[0] for a in pr], np.int32)
    sc = np.ascontiguousarray(scale, np.float32)
    isc = np.ascontiguousarray(inv_scale, np.float32)
    ur = np.zeros(len(kl), np.float32)
    dep = np.zeros(len(kl), np.float32)
    kept = lib().orc_stereo_match(_p(kl), len(kl), _p(dl), _p(kr), len(kr), _p(dr), _p(sc), _p(isc),
                                  ctypes.cast(ptr_l, ctypes.c_void_p), ctypes.cast(ptr_r, ctypes.c_void_p),
                                  _p(lw), _p(lh), _p(sl), _p(sr), float(bf), float(mb), _p(ur), _p(dep))
    return ur, dep, kept


# --- ORBmatcher projection searches (match_oracle.cc) -----------------------
PROJ_POINT_DTYPE = np.dtype([("Xw", "<f4", (3,)), ("octave", "<i4"), ("angle", "<f4"),
                             ("has_obs", "<i4"), ("desc", "u1", (32,))])
MAP_POINT_DTYPE = np.dtype([("Xw", "<f4", (3,)), ("normal", "<f4", (3,)), ("min_dist", "<f4"),
                            ("max_dist", "<f4"), ("flags", "<i4"), ("desc", "u1", (32,))])
TRACK_VIEW_DTYPE = np.dtype([("in_view", "<i4"), ("level", "<i4"), ("proj_x", "<f4"),
                             ("proj_y", "<f4"), ("proj_xr", "<f4"), ("depth", "<f4"),
                             ("view_cos", "<f4")])


def _geom(g):
    """orbgpu_frame_geom bytes from a ctypes FrameGeom (or anything with its fields)."""
    a = np.zeros(22, np.float32)
    a[0:4] = [g.min_x, g.max_x, g.min_y, g.max_y]
    a[4:5].view(np.int32)[0] = g.n_levels
    a[5] = g.log_scale_factor
    a[6:22] = list(g.scale_factors)
    return a


def _opt(a, dtype):
    return None if a is None else np.ascontiguousarray(a, dtype)


def search_last(geom, cam, mb, Tcw, Tlw, kps, desc, uright, claimed, pts, th, mono, check_ori):
    """SearchByProjection(CurrentFrame, LastFrame, th, bMono) -> (nmatches, match[N])."""
    g = _geom(geom)
    c = np.ascontiguousarray(cam, np.float32)
    k = np.ascontiguousarray(kps, KEYPOINT_DTYPE)
    d = np.ascontiguousarray(desc, np.uint8)
    p = np.ascontiguousarray(pts, PROJ_POINT_DTYPE)
    ur, cl = _opt(uright, np.float32), _opt(claimed, np.uint8)
    tc, tl = np.ascontiguousarray(Tcw, np.float32), np.ascontiguousarray(Tlw, np.float32)
    match = np.zeros(max(len(k), 1), np.int32)
    nm = lib().orc_search_last(_p(g), _p(c), float(mb), _p(tc), _p(tl), _p(k), _p(d), _p(ur),
                               _p(cl), len(k), _p(p), len(p), float(th), int(mono),
                               int(check_ori), _p(match))
    return nm, match[:len(k)]


def search_kf(geom, cam, Tcw, kps, desc, claimed, pts, angles, th, orb_dist, check_ori):
    """SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist) -> (nmatches, match)."""
    g = _geom(geom)
    c = np.ascontiguousarray(cam, np.float32)
    k = np.ascontiguousarray(kps, KEYPOINT_DTYPE)
    d = np.ascontiguousarray(desc, np.uint8)
    p = np.ascontiguousarray(pts, MAP_POINT_DTYPE)
    a = np.ascontiguousarray(angles, np.float32)
    tc = np.ascontiguousarray(Tcw, np.float32)
    match = np.zeros(max(len(k), 1), np.int32)
    nm = lib().orc_search_kf(_p(g), _p(c), _p(tc), _p(k), _p(d), _p(_opt(claimed, np.uint8)),
                             len(k), _p(p), _p(a), len(p), float(th), int(orb_dist),
                             int(check_ori), _p(match))
    return nm, match[:len(k)]


def search_bow(kf_fv, kf_desc, kf_angle, kf_valid, f_fv, f_desc, f_angle, nn_ratio, check_ori):
    """SearchByBoW(pKF, F, vpMapPointMatches); a FeatureVector is (nodes uint32
    ascending, offsets int32 [n + 1], features uint32) -> (nmatches, match)."""
    kn, ko, kf = (np.ascontiguousarray(x, t) for x, t in zip(kf_fv, (np.uint32, np.int32, np.uint32)))
    fn, fo, ff = (np.ascontiguousarray(x, t) for x, t in zip(f_fv, (np.uint32, np.int32, np.uint32)))
    kd, fd = np.ascontiguousarray(kf_desc, np.uint8), np.ascontiguousarray(f_desc, np.uint8)
    ka, fa = np.ascontiguousarray(kf_angle, np.float32), np.ascontiguousarray(f_angle, np.float32)
    kv = np.ascontiguousarray(kf_valid, np.uint8)
    match = np.zeros(max(len(fd), 1), np.int32)
    nm = lib().orc_search_bow(_p(kn), _p(ko), _p(kf), len(kn), _p(kd), _p(ka), _p(kv), _p(fn),
                              _p(fo), _p(ff), len(fn), _p(fd), _p(fa), len(fd), float(nn_ratio),
                              int(check_ori), _p(match))
    return nm, match[:len(fd)]


def frustum(geom, cam, Rcw, tcw, Ow, pts, cos_limit, views=None):
    """Frame::isInFrustum over pts -> TRACK_VIEW_DTYPE [n] (fields the reference
    does not write keep the values of `views`)."""
    g = _geom(geom)
    c = np.ascontiguousarray(cam, np.float32)
    p = np.ascontiguousarray(pts, MAP_POINT_DTYPE)
    v = np.zeros(len(p), TRACK_VIEW_DTYPE) if views is None else np.array(views, TRACK_VIEW_DTYPE)
    R, t, O = (np.ascontiguousarray(x, np.float32) for x in (Rcw, tcw, Ow))
    lib().orc_frustum(_p(g), _p(c), _p(R), _p(t), _p(O), _p(p), len(p), float(cos_limit), _p(v))
    return v


def search_local(geom, kps, desc, uright, claimed, pts, views, th, nn_ratio, far_points=False,
                 th_far=0.0):
    """SearchByProjection(F, vpMapPoints, th, bFarPoints, thFarPoints) -> (nmatches, match)."""
    g = _geom(geom)
    k = np.ascontiguousarray(kps, KEYPOINT_DTYPE)
    d = np.ascontiguousarray(desc, np.uint8)
    p = np.ascontiguousarray(pts, MAP_POINT_DTYPE)
    v = np.ascontiguousarray(views, TRACK_VIEW_DTYPE)
    ur, cl = _opt(uright, np.float32), _opt(claimed, np.uint8)
    match = np.zeros(max(len(k), 1), np.int32)
    nm = lib().orc_search_local(_p(g), _p(k), _p(d), _p(ur), _p(cl), len(k), _p(p), _p(v), len(p),
                                float(th), float(nn_ratio), int(far_points), float(th_far),
                                _p(match))
    return nm, match[:len(k)]


def predict_scale(max_dist, dist, log_scale, n_levels):
    return lib().orc_predict_scale(float(max_dist), float(dist), float(log_scale), int(n_levels))


def predict_scale_check(log_scale, n_levels, thr, lo_bits, hi_bits):
    t = np.ascontiguousarray(thr, np.float32)
    return lib().orc_predict_scale_check(float(log_scale), int(n_levels), _p(t), int(lo_bits),
                                         int(hi_bits))


def frame_grid_cells(geom, kps):
    g = _geom(geom)
    k = np.ascontiguousarray(kps, KEYPOINT_DTYPE)
    out = np.zeros(max(len(k), 1), np.int32)
    lib().orc_frame_grid_cells(_p(g), _p(k), len(k), _p(out))
    return out[:len(k)]


# --- DBoW2 (bow_oracle.cc) ---------------------------------------------------
class OracleVocab:
    """TemplatedVocabulary<FORB> restated: loadFromTextFile + transform."""

    def __init__(self, path):
        self._h = lib().orc_vocab_load(str(path).encode())
        if not self._h:
            raise ValueError(f"vocabulary load failed: {path}")

    def info(self):
        a = np.zeros(6, np.int32)
        lib().orc_vocab_info(self._h, _p(a))
        return dict(zip(("k", "L", "scoring", "weighting", "nodes", "words"), a.tolist()))

    def transform(self, descs, levelsup=4):
        """-> (bow_words, bow_weights, fv_nodes, fv_offsets, fv_features)"""
        d = np.ascontiguousarray(descs, np.uint8).reshape(-1, 32)
        n = len(d)
        S = max(n, 1)
        bw, bwt = np.zeros(S, np.uint32), np.zeros(S, np.float64)
        fn, fo, ff = np.zeros(S, np.uint32), np.zeros(S + 1, np.int32), np.zeros(S, np.uint32)
        nw, nn = ctypes.c_int(), ctypes.c_int()
        lib().orc_bow_transform(self._h, _p(d), n, int(levelsup), _p(bw), _p(bwt),
                                ctypes.byref(nw), _p(fn), _p(fo), _p(ff), ctypes.byref(nn))
        w, k = nw.value, nn.value
        return bw[:w], bwt[:w], fn[:k], fo[:k + 1], ff[:fo[k]]

    def __del__(self):
        try:
            if self._h:
                lib().orc_vocab_free(self._h)
        except Exception:
            pass


def pose_inertial(case: dict, rec_init: bool = False, with_prev: bool = False):
    """PoseInertialOptimizationLastFrame (mode 0) / LastKeyFrame (mode 1) on a
    case of tests/inertial_cases.py: returns (result record, outlier uint8[n])
    [, the previous frame's final double state]."""
    from orb_slam_fusion_amd._lib import INERTIAL_RESULT_DTYPE

    obs = case["obs"]
    n = len(obs)
    res = np.zeros((), INERTIAL_RESULT_DTYPE)
    out = np.zeros(max(n, 1), np.uint8)
    prev_out = np.zeros(21)
    prior = case.get("prior")
    lib().orc_pose_inertial_ex(case["mode"], _p(case["calib"]), _p(case["cur"]),
                               _p(case["prev"]), _p(case["preint"]), _p(prior), _p(obs), n,
                               int(rec_init), _p(res), _p(out), _p(prev_out))
    return (res, out[:n].copy(), prev_out) if with_prev else (res, out[:n].copy())


def inertial_system(case: dict, cur21: np.ndarray, prev21: np.ndarray, kernels: bool = False):
    """The oracle's Gauss-Newton (H, b) at double states [Rwb(9) twb v bg ba]."""
    n = 30 if case["mode"] == 0 else 15
    H = np.zeros((n, n))
    b = np.zeros(n)
    cur21 = np.ascontiguousarray(cur21, np.float64)
    prev21 = np.ascontiguousarray(prev21, np.float64)
    lib().orc_inertial_system(case["mode"], _p(case["calib"]), _p(cur21), _p(prev21),
                              _p(case["preint"]), _p(case.get("prior")), _p(case["obs"]),
                              len(case["obs"]), int(kernels), _p(H), _p(b))
    return H, b


def sym_pinv(A: np.ndarray) -> np.ndarray:
    A = np.ascontiguousarray(A, np.float64)
    out = np.zeros_like(A)
    lib().orc_sym_pinv(_p(A), A.shape[0], _p(out))
    return out


def lia(pb, iterations=None, lambda_init=None):
    """LocalInertialBA's solve (oracle/lia_oracle.cc) on a synth.LiaProblem:
    -> dict(kfs21 float64 [n_kf, 21] (Rwb, twb, v, bg, ba), pts float64
    [n_pts, 3], outlier uint8 [E], chi2 float64 [E] (each edge's chi2 at the
    classification), stats float64 [7])."""
    n_kf, n_p, ne, ni = len(pb.kfs), len(pb.pts_init), len(pb.edges), len(pb.imu_edges)
    ko = np.zeros((n_kf, 21))
    po = np.zeros((n_p, 3))
    out = np.zeros(max(ne, 1), np.uint8)
    chi = np.zeros(max(ne, 1))
    st = np.zeros(7)
    it = pb.iterations if iterations is None else iterations
    lam = pb.lambda_init if lambda_init is None else lambda_init
    r = lib().orc_lia(_p(pb.calib), n_kf, _p(pb.kfs), _p(pb.fixed), _p(pb.imu), n_p,
                      _p(pb.pts_init), _p(pb.close), ne, _p(pb.edges), ni, _p(pb.imu_edges), it,
                      float(lam), _p(ko), _p(po), _p(out), _p(st), _p(chi))
    assert r == 0, "orc_lia rejected the problem"
    return dict(kfs21=ko, pts=po, outlier=out[:ne].copy(), chi2=chi[:ne].copy(), stats=st)


def lia_system(pb):
    """The full g2o system (H, b) of the window at its initial state: free key
    frames' 15-blocks (VP VV VG VA) first, then 3 rows per point; Huber
    weights from the initial errors."""
    n_kf, n_p, ne, ni = len(pb.kfs), len(pb.pts_init), len(pb.edges), len(pb.imu_edges)
    free = pb.fixed == 0
    n = int(np.where(pb.imu[free] != 0, 15, 6).sum()) + 3 * n_p
    H = np.zeros((n, n))
    b = np.zeros(n)
    r = lib().orc_lia_system(_p(pb.calib), n_kf, _p(pb.kfs), _p(pb.fixed), _p(pb.imu), n_p,
                             _p(pb.pts_init), ne, _p(pb.edges), ni, _p(pb.imu_edges), _p(H), _p(b))
    assert r == 0
    return H, b


def lia_vis_linearize(calib, kf_state, X, edge):
    """One EdgeMono / EdgeStereo: error (3), Jl (3x3), Jp (3x6)."""
    X = np.ascontiguousarray(X, np.float64)
    calib, kf_state, edge = (np.array(a) for a in (calib, kf_state, edge))
    err, Jl, Jp = np.zeros(3), np.zeros(9), np.zeros(18)
    lib().orc_lia_vis_linearize(_p(calib), _p(kf_state), _p(X), _p(edge), _p(err), _p(Jl), _p(Jp))
    return err, Jl.reshape(3, 3), Jp.reshape(3, 6)
