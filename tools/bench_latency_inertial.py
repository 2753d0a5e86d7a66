"""Per-frame wall-clock of the stereo-inertial tracking thread after IMU
initialisation (the mode EuRoC MH01 runs, tests/slam_euroc_si.cc): one frame
at a time through the host-buffer ABI, as the reference calls it --

  Frame(): the left / right OrbExtractor::operator() on two threads
           (frame.cc:179-182) + ComputeStereoMatches (:189);
  TrackWithMotionModel: PredictStateIMU only, no search (tracking.cc:2170-2176);
  TrackLocalMap: SearchLocalPoints = isInFrustum + SearchByProjection(F,
           vpMapPoints, th 6, nn 0.8) (:2626-2690), then
           PoseInertialOptimizationLastFrame (:2262-2285, optimizer.cc:4762-5160)
           over the matches it left (the observation list gathered on the host
           from the Frame fields, as the reference's graph build does).

The local map is the previous frame's stereo points (tools/bench_track.Chain,
built once); the IMU inputs follow the chain's camera (tools/inertial_chain).
Timed end to end per frame (host copies included), median over frames, beside
the CPU oracle running the same sequence on the same host (2 threads for the
extractions, 1 for the rest).

    python tools/bench_latency_inertial.py [--frames 16]
"""
import argparse
import json
import sys
import threading
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "tools"))

PARAMS = (1000, 1.2, 8, 20, 7)
TH_LOCAL = 6.0  # SearchLocalPoints after IMU init, before InertialBA2 (tracking.cc:2669-2673)
NN_LOCAL = 0.8


def _local_map(c, f, scale):
    from orb_slam_fusion_amd._lib import MAP_POINT_DTYPE, MP_HAS_OBS

    lp = c.pts[f]  # the previous frame's stereo points (Tlw = identity, Ow = 0)
    mp = np.zeros(len(lp), MAP_POINT_DTYPE)
    mp["Xw"] = lp["Xw"]
    dist = np.linalg.norm(lp["Xw"].astype(np.float32), axis=1).astype(np.float32)
    mp["normal"] = lp["Xw"] / dist[:, None]
    mp["max_dist"] = dist * scale[lp["octave"]]  # MapPoint::UpdateNormalAndDepth
    mp["min_dist"] = mp["max_dist"] / scale[-1]
    mp["flags"] = MP_HAS_OBS
    mp["desc"] = lp["desc"]
    return mp


def _obs(kps, ur, match, mp, views, inv_sigma2):
    """PoseInertialOptimizationLastFrame's observations (optimizer.cc:4806-4880):
    the matched keypoints in index order, close = mTrackDepth < 10."""
    from orb_slam_fusion_amd._lib import INERTIAL_OBS_DTYPE

    sel = np.nonzero(match >= 0)[0]
    o = np.zeros(len(sel), INERTIAL_OBS_DTYPE)
    o["Xw"] = mp["Xw"][match[sel]]
    o["u"], o["v"], o["ur"] = kps["x"][sel], kps["y"][sel], ur[sel]
    o["inv_sigma2"] = inv_sigma2[kps["octave"][sel]]
    v = views[match[sel]]
    o["close"] = (v["in_view"] != 0) & (v["depth"] < 10.0)
    return o


def measure(frames: int = 16, warmup: int = 3, cpu_frames: int = 4) -> dict:
    from bench_track import Chain
    from inertial_chain import imu_inputs

    from orb_slam_fusion_amd import OrbExtractor, compute_stereo_matches
    from orb_slam_fusion_amd.inertial import InertialProblem, PoseInertialOptimizer
    from orb_slam_fusion_amd.matcher import MatchFrame, ORBmatcher

    c = Chain(frames)  # setup: the frames, the previous frames' map points, poses
    scale = c.ex.GetScaleFactors()
    inv_sigma2 = c.ex.GetInverseScaleSigmaSquares()
    maps = [_local_map(c, f, scale) for f in range(frames)]
    imus = [imu_inputs(c, f) for f in range(frames)]
    exl, exr = OrbExtractor(*PARAMS), OrbExtractor(*PARAMS)
    P = max(len(m) for m in maps)
    local = ORBmatcher(NN_LOCAL, True, max_keypoints=c.cap, max_points=P)
    opt = PoseInertialOptimizer(max_obs=c.cap)

    def one(f):
        _, _, cl, cr = c.quads[f]
        t0 = time.perf_counter()
        out = {}
        th = threading.Thread(target=lambda: out.__setitem__("r", exr(cr)))
        th.start()
        _, kl, dl = exl(cl)
        th.join()
        t1 = time.perf_counter()
        ur, _ = compute_stereo_matches(exl, exr, len(kl), c.bf, c.mb)
        t2 = time.perf_counter()
        F = MatchFrame(geom=c.geom, cam=c.cam, mb=c.mb, kps=kl, desc=dl, uright=ur, claimed=None,
                       pose=c.Tcw[f])
        _, match, views = local.search_local_points(F, maps[f], 0.5, TH_LOCAL)
        t3 = time.perf_counter()
        calib, cur, prev, pre, prior = imus[f]
        pb = InertialProblem(calib, cur, prev, pre, _obs(kl, ur, match, maps[f], views, inv_sigma2),
                             prior)
        n_good = opt.PoseInertialOptimizationLastFrame(pb)
        t4 = time.perf_counter()
        return (t1 - t0, t2 - t1, t3 - t2, t4 - t3), len(pb.obs), n_good

    parts, n_obs, good = [], [], []
    for i in range(warmup + frames):
        p, n, g = one(i % frames)
        if i >= warmup:
            parts.append(p), n_obs.append(n), good.append(g)
    med = lambda a: float(np.median(a)) * 1e3  # noqa: E731
    cols = list(zip(*parts))
    tot = [sum(p) for p in parts]
    out = {
        "workload": "stereo-inertial tracking after IMU init, one 752x480 frame at a time through "
                    "the host ABI: 2-thread extraction (1000 kp, 8 levels) + ComputeStereoMatches + "
                    "SearchLocalPoints (isInFrustum + SearchByProjection th 6, nn 0.8) + "
                    f"PoseInertialOptimizationLastFrame; median of {frames} frames",
        "gpu_ms_per_frame": round(med(tot), 3),
        "gpu_extract_ms": round(med(cols[0]), 3),
        "gpu_stereo_ms": round(med(cols[1]), 3),
        "gpu_search_local_ms": round(med(cols[2]), 3),
        "gpu_pose_inertial_ms": round(med(cols[3]), 3),
        "observations_per_frame": round(float(np.mean(n_obs)), 1),
        "inliers_per_frame": round(float(np.mean(good)), 1),
    }
    if cpu_frames > 0:
        sys.path.insert(0, str(REPO / "oracle"))
        import binding as oracle  # cpu baseline leg only

        ol, orr = oracle.OracleExtractor(*PARAMS), oracle.OracleExtractor(*PARAMS)
        p = ol.params()
        c_parts = []
        for f in range(min(cpu_frames, frames)):
            _, _, cl, cr = c.quads[f]
            t0 = time.perf_counter()
            res = {}
            th = threading.Thread(target=lambda: res.__setitem__("r", orr.extract(cr)))
            th.start()
            _, kl, dl = ol.extract(cl)
            th.join()
            _, kr, dr = res["r"]
            t1 = time.perf_counter()
            ur, _, _ = oracle.stereo_match(kl, dl, kr, dr, [ol.level(l) for l in range(8)],
                                           [orr.level(l) for l in range(8)], p["scale"],
                                           p["inv_scale"], c.bf, c.mb)
            t2 = time.perf_counter()
            R = np.eye(3, dtype=np.float32)
            t = np.asarray(c.Tcw[f][4:], np.float32)
            views = oracle.frustum(c.geom, c.cam, R, t, -t, maps[f], 0.5)
            _, match = oracle.search_local(c.geom, kl, dl, ur, None, maps[f], views, TH_LOCAL,
                                           NN_LOCAL)
            t3 = time.perf_counter()
            calib, cur, prev, pre, prior = imus[f]
            case = dict(mode=0, calib=calib, cur=cur, prev=prev, preint=pre, prior=prior,
                        obs=_obs(kl, ur, match, maps[f], views, p["inv_sigma2"]))
            oracle.pose_inertial(case)
            t4 = time.perf_counter()
            c_parts.append((t1 - t0, t2 - t1, t3 - t2, t4 - t3))
        cc = list(zip(*c_parts))
        cpu = med([sum(x) for x in c_parts])
        out.update({"cpu_ms_per_frame": round(cpu, 3), "cpu_extract_ms": round(med(cc[0]), 3),
                    "cpu_stereo_ms": round(med(cc[1]), 3), "cpu_search_local_ms": round(med(cc[2]), 3),
                    "cpu_pose_inertial_ms": round(med(cc[3]), 3), "cpu_cores": 2,
                    "speedup_vs_cpu": round(cpu / out["gpu_ms_per_frame"], 2),
                    "speedup_extract_plus_pose": round(
                        (med(cc[0]) + med(cc[3])) / (out["gpu_extract_ms"] + out["gpu_pose_inertial_ms"]),
                        2)})
    local.close()
    opt.close()
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--cpu-frames", type=int, default=4)
    a = ap.parse_args()
    print(json.dumps(measure(a.frames, cpu_frames=a.cpu_frames)))
