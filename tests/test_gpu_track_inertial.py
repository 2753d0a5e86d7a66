"""The stereo-inertial tracking chain: extract -> stereo -> Tracking::
SearchLocalPoints (isInFrustum + SearchByProjection(F, vpMapPoints), the
only search once the IMU is initialised: TrackWithMotionModel returns after
PredictStateIMU, tracking.cc:2170-2176; TrackLocalMap then optimises,
tracking.cc:2262-2285) -> PoseInertialOptimizationLastFrame's observation
list (orbgpu_matches_to_inertial_obs_batch, close = mTrackDepth < 10 from
isInFrustum's depth) -> PoseInertialOptimizationLastFrame, against the
oracle chain on the same images and IMU inputs (the oracle's own frustum
depths give its close flags).  The IMU states follow the chain's
camera (identity last pose, motion-model current pose) through a synthetic
camera-body calibration; the preintegration is exact for that motion.
Observation list: bit-exact; optimisation: the tolerances of
tests/test_gpu_inertial.py."""
import sys
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tools"))


from inertial_chain import imu_inputs as _imu_inputs  # noqa: E402


def test_inertial_track_chain_matches_oracle(gpu_available):
    import torch

    import binding as oracle
    import test_gpu_inertial as tgi
    from bench_track import Chain, oracle_chain
    from orb_slam_fusion_amd._lib import (IMU_PREINT_DTYPE, IMU_PRIOR_DTYPE, IMU_STATE_DTYPE,
                                          INERTIAL_OBS_DTYPE, INERTIAL_RESULT_DTYPE)
    from orb_slam_fusion_amd.inertial import PoseInertialOptimizer

    from orb_slam_fusion_amd._lib import KEYPOINT_DTYPE, MAP_POINT_DTYPE, MP_HAS_OBS
    from orb_slam_fusion_amd.matcher import MatchFrame, ORBmatcher

    B = 2
    c = Chain(B)
    c.run()
    dev = c.dev
    P = c.d_pts.shape[1]
    TH_LOCAL = 6  # SearchLocalPoints after IMU init, before InertialBA2 (tracking.cc:2669-2673)
    scale = c.ex.GetScaleFactors()
    lk_h = c.lk.cpu().numpy().view(KEYPOINT_DTYPE).reshape(B, c.cap)
    ld_h, lnn_h, ur_h = c.ld.cpu().numpy(), c.lnn.cpu().numpy(), c.ur.cpu().numpy()
    local = ORBmatcher(0.8, True, max_keypoints=c.cap, max_points=P)
    match = np.full((B, c.cap), -1, np.int32)
    close = np.zeros((B, P), np.uint8)
    mps, frames = [], []
    for f in range(B):
        lp = c.pts[f]  # the local map points: the last frame's (Tlw = identity, Ow = 0)
        mp = np.zeros(len(lp), MAP_POINT_DTYPE)
        mp["Xw"] = lp["Xw"]
        dist = np.linalg.norm(lp["Xw"].astype(np.float32), axis=1).astype(np.float32)
        mp["normal"] = lp["Xw"] / dist[:, None]
        mp["max_dist"] = dist * scale[lp["octave"]]  # MapPoint::UpdateNormalAndDepth
        mp["min_dist"] = mp["max_dist"] / scale[-1]
        mp["flags"] = MP_HAS_OBS
        mp["desc"] = lp["desc"]
        k = int(lnn_h[f])
        F = MatchFrame(geom=c.geom, cam=c.cam, mb=c.mb, kps=lk_h[f, :k], desc=ld_h[f, :k],
                       uright=ur_h[f, :k], claimed=None, pose=c.Tcw[f])
        _, m, views = local.search_local_points(F, mp, 0.5, TH_LOCAL)
        match[f, :k] = m
        close[f, :len(mp)] = (views["in_view"] != 0) & (views["depth"] < 10.0)  # mTrackDepth < 10
        mps.append(mp)
        frames.append(F)
    local.close()
    d_match = torch.from_numpy(match).to(dev)
    d_close = torch.from_numpy(close).to(dev)
    d_iobs = torch.zeros((B, c.cap, 32), dtype=torch.uint8, device=dev)
    d_nobs = torch.zeros(B, dtype=torch.int32, device=dev)
    lk, lnn = c.lk.contiguous(), c.lnn.contiguous()
    c.matcher.matches_to_inertial_obs_batch(lk, c.ur, d_match, lnn, c.d_pts, d_close,
                                            c.inv_sigma2, d_iobs, d_nobs)
    ins = [_imu_inputs(c, f) for f in range(B)]

    def rec(k, dt):
        a = np.stack([np.asarray(x[k]).reshape(()) for x in ins]).astype(dt)
        return torch.from_numpy(a.view(np.uint8).reshape(B, dt.itemsize).copy()).to(dev)

    d_res = torch.zeros((B, INERTIAL_RESULT_DTYPE.itemsize), dtype=torch.uint8, device=dev)
    d_out = torch.zeros((B, c.cap), dtype=torch.uint8, device=dev)
    opt = PoseInertialOptimizer(max_problems=B, max_obs=c.cap)
    opt.batch(0, ins[0][0], rec(1, IMU_STATE_DTYPE), rec(2, IMU_STATE_DTYPE),
              rec(3, IMU_PREINT_DTYPE), rec(4, IMU_PRIOR_DTYPE), d_iobs, d_nobs, d_res, d_out)
    torch.cuda.synchronize()
    iobs = d_iobs.cpu().numpy().view(INERTIAL_OBS_DTYPE).reshape(B, c.cap)
    nobs = d_nobs.cpu().numpy()
    res = d_res.cpu().numpy().view(INERTIAL_RESULT_DTYPE).reshape(B)
    outs = d_out.cpu().numpy()
    opt.close()
    for f in range(B):
        # the oracle chain: its own extraction / stereo (bit-exact, test_gpu_track), its
        # own isInFrustum and local search, its own close flags from its frustum depths
        o = oracle_chain(oracle, c, f)
        F = frames[f]
        R = np.eye(3, dtype=np.float32)
        t = np.asarray(c.Tcw[f][4:], np.float32)
        views = oracle.frustum(c.geom, c.cam, R, t, -t, mps[f], 0.5)
        _, m_o = oracle.search_local(c.geom, o["kps"], o["desc"], o["ur"], None, mps[f], views,
                                     TH_LOCAL, 0.8)
        assert np.array_equal(m_o, match[f, :len(m_o)])
        sel = np.nonzero(m_o >= 0)[0]
        ref_obs = np.zeros(len(sel), INERTIAL_OBS_DTYPE)
        kl = o["kps"]
        ref_obs["Xw"] = mps[f]["Xw"][m_o[sel]]
        ref_obs["u"], ref_obs["v"], ref_obs["ur"] = kl["x"][sel], kl["y"][sel], o["ur"][sel]
        ref_obs["inv_sigma2"] = c.inv_sigma2[kl["octave"][sel]]
        vsel = views[m_o[sel]]
        ref_obs["close"] = (vsel["in_view"] != 0) & (vsel["depth"] < 10.0)
        n = int(nobs[f])
        assert n == len(sel) > 100
        assert iobs[f, :n].tobytes() == ref_obs.tobytes()
        case = dict(mode=0, calib=ins[f][0], cur=ins[f][1], prev=ins[f][2], preint=ins[f][3],
                    prior=ins[f][4], obs=ref_obs)
        ref, ref_out = oracle.pose_inertial(case)
        tgi._check(res[f], outs[f, :n], ref, ref_out)
        assert int(res[f]["n_inliers"]) > 0.8 * n
