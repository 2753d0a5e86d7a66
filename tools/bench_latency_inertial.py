"""Per-frame wall-clock of the stereo-inertial tracking thread after IMU
initialisation (the mode EuRoC MH01 runs, tests/slam_euroc_si.cc): one frame
at a time through the host-buffer ABI, as the reference calls it --

  Frame(): the left / right extraction of frame.cc:179-182 from the tracking
           thread, both launches in flight (orbgpu_extract_stereo, the
           ORBGPU_STEREO Frame shim) + ComputeStereoMatches (:189);
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
extractions, 1 for the rest).  Two GPU legs on the same frames: this Python
process through ctypes, and tools/latency_inertial.cc (build/latency_inertial)
calling the C ABI from C++ as the drop-ins do, which also checks that every
frame's observation count and n_good equal the Python leg's; the C++ leg is
the headline (`host` names it), the Python one stays under `python_host`.

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
CPP_REPS = 4  # passes over the frames in the C++ leg (a p90 over 4 x frames samples)
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


def _dump(path, c, maps, imus, inv_sigma2, n_obs, good):
    """The C++ leg's inputs (tools/latency_inertial.cc reads them in this order)."""
    import ctypes

    from orb_slam_fusion_amd._lib import (IMU_CALIB_DTYPE, IMU_PREINT_DTYPE, IMU_PRIOR_DTYPE,
                                          IMU_STATE_DTYPE, INERTIAL_OBS_DTYPE, MAP_POINT_DTYPE,
                                          Camera, OrbParams)
    from orb_slam_fusion_amd.matcher import pose_matrices

    frames = len(n_obs)
    H, W = c.quads[0][2].shape
    cam = Camera(*[float(v) for v in c.cam])
    sizes = [ctypes.sizeof(c.geom), ctypes.sizeof(cam), MAP_POINT_DTYPE.itemsize,
             IMU_CALIB_DTYPE.itemsize, IMU_STATE_DTYPE.itemsize, IMU_PREINT_DTYPE.itemsize,
             IMU_PRIOR_DTYPE.itemsize, INERTIAL_OBS_DTYPE.itemsize]
    with open(path, "wb") as fp:
        fp.write(b"OSLATIN1")
        fp.write(np.array([frames, W, H, len(inv_sigma2), c.cap], np.int32).tobytes())
        fp.write(np.array(sizes, np.int32).tobytes())
        fp.write(bytes(OrbParams(*PARAMS)))
        fp.write(np.array([c.bf, c.mb, TH_LOCAL, NN_LOCAL, 0.5], np.float32).tobytes())
        fp.write(bytes(c.geom) + bytes(cam))
        fp.write(np.ascontiguousarray(imus[0][0], IMU_CALIB_DTYPE).tobytes())
        fp.write(np.asarray(inv_sigma2, np.float32).tobytes())
        for f in range(frames):
            _, _, cl, cr = c.quads[f]
            R, t, Ow = pose_matrices(c.Tcw[f])
            fp.write(np.ascontiguousarray(cl, np.uint8).tobytes() + np.ascontiguousarray(cr, np.uint8).tobytes())
            fp.write(R.tobytes() + t.tobytes() + Ow.tobytes())
            fp.write(np.array([len(maps[f])], np.int32).tobytes())
            fp.write(np.ascontiguousarray(maps[f], MAP_POINT_DTYPE).tobytes())
            _, cur, prev, pre, prior = imus[f]
            for a, dt in ((cur, IMU_STATE_DTYPE), (prev, IMU_STATE_DTYPE), (pre, IMU_PREINT_DTYPE),
                          (prior, IMU_PRIOR_DTYPE)):
                fp.write(np.ascontiguousarray(a, dt).tobytes())
            fp.write(np.array([n_obs[f], good[f]], np.int32).tobytes())


def _cpp_leg(c, maps, imus, inv_sigma2, n_obs, good, warmup):
    """tools/latency_inertial.cc (build/latency_inertial, built by `make`) on the
    same frames: the per-frame cost a C++ tracking thread sees through the C ABI."""
    import subprocess
    import tempfile

    exe = REPO / "build" / "latency_inertial"
    if not exe.exists():
        raise RuntimeError(f"{exe} missing: run make")
    import os

    with tempfile.TemporaryDirectory() as tmp:
        # ORBGPU_LATIN_DUMP=path keeps the inputs (e.g. to profile build/latency_inertial alone)
        path = Path(os.environ.get("ORBGPU_LATIN_DUMP") or Path(tmp) / "latin.bin")
        _dump(path, c, maps, imus, inv_sigma2, n_obs, good)
        r = subprocess.run([str(exe), str(path), str(warmup), "stereo", str(CPP_REPS)], capture_output=True,
                           text=True,
                           timeout=120)
    if r.returncode != 0:
        raise RuntimeError(f"latency_inertial exited {r.returncode}: {r.stderr.strip()[-400:]} "
                           f"{r.stdout.strip()[-600:]}")
    return json.loads(r.stdout.strip().splitlines()[-1])


def measure(frames: int = 16, warmup: int = 3, cpu_frames: int = 4, cpp_host: bool = True) -> dict:
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
        (_, kl, dl), _ = exl.extract_stereo(exr, cl, cr)
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
    order = [(i % frames) for i in range(warmup, warmup + frames)]  # frame of each timed pass
    by_frame = {f: (n, g) for f, n, g in zip(order, n_obs, good)}
    cpp = _cpp_leg(c, maps, imus, inv_sigma2, [by_frame[f][0] for f in range(frames)],
                   [by_frame[f][1] for f in range(frames)], warmup) if cpp_host else None
    med = lambda a: float(np.median(a)) * 1e3  # noqa: E731
    cols = list(zip(*parts))
    tot = [sum(p) for p in parts]
    py = {
        "host": "Python (ctypes) through the C ABI",
        "gpu_ms_per_frame": round(med(tot), 3),
        "gpu_extract_ms": round(med(cols[0]), 3),
        "gpu_stereo_ms": round(med(cols[1]), 3),
        "gpu_search_local_ms": round(med(cols[2]), 3),
        "gpu_pose_inertial_ms": round(med(cols[3]), 3),
    }
    out = {
        "workload": "stereo-inertial tracking after IMU init, one 752x480 frame at a time through "
                    "the host ABI: one-thread stereo extraction (orbgpu_extract_stereo; 1000 kp, "
                    "8 levels) + ComputeStereoMatches + SearchLocalPoints (isInFrustum + "
                    "SearchByProjection th 6, nn 0.8) + PoseInertialOptimizationLastFrame; median "
                    f"(and, C++ leg, p90 over {CPP_REPS} passes) of {frames} frames",
        "observations_per_frame": round(float(np.mean(n_obs)), 1),
        "inliers_per_frame": round(float(np.mean(good)), 1),
    }
    # headline: the C++ caller (the drop-ins are C++); the Python leg beside it
    out.update({k: v for k, v in (cpp or py).items() if k.startswith("gpu_") or k == "host"})
    if cpp is not None:
        out["same_work_as_python_leg"] = cpp["same_work_as_python_leg"]
        out["python_host"] = py
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
                    "speedup_vs_cpu_python_host": round(cpu / py["gpu_ms_per_frame"], 2),
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
    ap.add_argument("--no-cpp", action="store_true", help="skip the C++ host leg")
    a = ap.parse_args()
    print(json.dumps(measure(a.frames, cpu_frames=a.cpu_frames, cpp_host=not a.no_cpp)))
