"""Per-frame wall-clock of the reference's own call sequence (north_star:
"≥20x the CPU reference's per-frame extract+PoseOptimization wall-clock"):
one synthetic 752x480 stereo frame at a time through the host-buffer ABI --
both images of the stereo Frame constructor's extraction (frame.cc:179-182)
from the tracking thread with both launches in flight
(orbgpu_extract_stereo, the ORBGPU_STEREO Frame shim), then
Optimizer::PoseOptimization on a 600-observation problem -- timed end to
end (host copies in and out included), median and p90, beside the CPU
oracle running the same sequence on the same host (2 threads for the two
extractions, 1 for the pose).

Three GPU legs on the same frames: tools/latency.cc (build/latency) calling
the C ABI from C++ as the drop-ins do -- the headline (`host` names it) --
once with orbgpu_extract_stereo and once with the reference's own pattern
(two operator() calls on two std::threads, `two_threads`); and this Python
process through ctypes (`python_host`).  Every leg's per-frame keypoint
counts and inliers must equal the Python leg's (`same_work_as_python_leg`).
Frame::ComputeStereoMatches (frame.cc:189, on the two handles' resident
outputs) is timed as an extra column.

    python tools/bench_latency.py [--frames 100]
"""
import argparse
import json
import subprocess
import sys
import threading
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))

PARAMS = (1000, 1.2, 8, 20, 7)
FX, BASE = 435.2, 0.11


def _stereo_extract(exl, exr, left, right):
    out = {}
    th = threading.Thread(target=lambda: out.__setitem__("r", exr(right)))
    th.start()
    res_l = exl(left)
    th.join()
    return res_l, out["r"]


def _cpp_leg(frames: int, warmup: int, mode: str) -> dict:
    """build/latency (tools/latency.cc, built by `make`) on the same frames."""
    exe = REPO / "build" / "latency"
    if not exe.exists():
        raise RuntimeError(f"{exe} missing: run make")
    r = subprocess.run([str(exe), str(frames), str(warmup), mode], capture_output=True, text=True, timeout=120)
    if r.returncode != 0:
        raise RuntimeError(f"latency {mode} exited {r.returncode}: {r.stderr.strip()[-400:]}")
    return json.loads(r.stdout.strip().splitlines()[-1])


def measure(frames: int = 100, warmup: int = 5, cpu_frames: int = 8, cpp_host: bool = True) -> dict:
    from orb_slam_fusion_amd import (OrbExtractor, PoseFrame, PoseOptimizer,
                                     compute_stereo_matches, synth)

    pairs = [synth.stereo_frame(i) for i in range(frames)]
    probs = [synth.pose_problem(synth.POSE_SEED + i, 600, 10) for i in range(frames)]
    exl, exr = OrbExtractor(*PARAMS), OrbExtractor(*PARAMS)
    opt = PoseOptimizer(max_obs=600)
    bf = np.float32(FX * BASE)
    mb = np.float32(bf / np.float32(FX))
    t_ex, t_st, t_po, t_fr = [], [], [], []
    counts = {}
    for i in range(warmup + frames):
        left, right = pairs[i % frames]
        cam, pin, _, obs = probs[i % frames]
        t0 = time.perf_counter()
        (_, kl, _), (_, kr, _) = exl.extract_stereo(exr, left, right)
        t1 = time.perf_counter()
        compute_stereo_matches(exl, exr, len(kl), bf, mb)
        t2 = time.perf_counter()
        inl = opt.PoseOptimization(PoseFrame(cam=cam, pose=pin, obs=obs))
        t3 = time.perf_counter()
        if i >= warmup:
            t_ex.append(t1 - t0), t_st.append(t2 - t1), t_po.append(t3 - t2)
            t_fr.append(t1 - t0 + t3 - t2)
            counts[i % frames] = (len(kl), len(kr), int(inl))
    med = lambda a: float(np.median(a)) * 1e3  # noqa: E731
    p90 = lambda a: float(np.percentile(a, 90)) * 1e3  # noqa: E731
    py = {
        "host": "Python (ctypes) through the C ABI",
        "gpu_ms_per_frame": round(med(t_fr), 3),
        "gpu_ms_per_frame_p90": round(p90(t_fr), 3),
        "gpu_extract_ms": round(med(t_ex), 3),
        "gpu_extract_ms_p90": round(p90(t_ex), 3),
        "gpu_pose_ms": round(med(t_po), 3),
        "gpu_pose_ms_p90": round(p90(t_po), 3),
        "gpu_stereo_ms": round(med(t_st), 3),
    }
    out = {
        "workload": "one 752x480 stereo frame at a time through the host ABI: stereo extraction "
                    "from one thread (orbgpu_extract_stereo; 1000 kp, 8 levels) + PoseOptimization "
                    f"(600 obs); median and p90 of {frames} frames",
    }
    if cpp_host:
        want = [counts[f] for f in range(frames)]

        def same(leg):
            return [tuple(x) for x in zip(leg["n_left"], leg["n_right"], leg["inliers"])] == want

        pair = _cpp_leg(frames, warmup, "pair")
        two = _cpp_leg(frames, warmup, "stereo")
        keep = lambda leg: {k: v for k, v in leg.items() if k.startswith("gpu_") or k == "host"}  # noqa: E731
        out.update(keep(pair))
        out["two_threads"] = dict(keep(two), extraction="two std::threads per frame (frame.cc:179-182)")
        out["same_work_as_python_leg"] = same(pair) and same(two)
        out["python_host"] = py
    else:
        out.update(py)
    if cpu_frames > 0:
        sys.path.insert(0, str(REPO / "oracle"))
        import binding as oracle  # cpu baseline leg only

        ol, orr = oracle.OracleExtractor(*PARAMS), oracle.OracleExtractor(*PARAMS)
        c_ex, c_po = [], []
        for i in range(cpu_frames):
            left, right = pairs[i % frames]
            cam, pin, _, obs = probs[i % frames]
            t0 = time.perf_counter()
            th = threading.Thread(target=orr.extract, args=(right,))
            th.start()
            ol.extract(left)
            th.join()
            t1 = time.perf_counter()
            oracle.pose_opt(cam, pin, obs)
            t2 = time.perf_counter()
            c_ex.append(t1 - t0), c_po.append(t2 - t1)
        cpu = med(c_ex) + med(c_po)
        out["cpu_ms_per_frame"] = round(cpu, 3)
        out["cpu_extract_ms"] = round(med(c_ex), 3)
        out["cpu_pose_ms"] = round(med(c_po), 3)
        out["cpu_cores"] = 2
        out["speedup_vs_cpu"] = round(cpu / out["gpu_ms_per_frame"], 2)
        if cpp_host:
            out["speedup_vs_cpu_python_host"] = round(cpu / py["gpu_ms_per_frame"], 2)
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=100)
    ap.add_argument("--no-cpp", action="store_true", help="skip the C++ host legs")
    a = ap.parse_args()
    print(json.dumps(measure(a.frames, cpp_host=not a.no_cpp)))
