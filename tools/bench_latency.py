"""Per-frame wall-clock of the reference's own call sequence (north_star:
"≥20x the CPU reference's per-frame extract+PoseOptimization wall-clock"):
one synthetic 752x480 stereo frame at a time through the host-buffer ABI --
the left and right OrbExtractor::operator() calls on two threads, as the
stereo Frame constructor does (frame.cc:179-182), then
Optimizer::PoseOptimization on a 600-observation problem -- timed end to
end (host copies in and out included), beside the CPU oracle running the
same sequence on the same host (2 threads for the two extractions, 1 for
the pose).  Frame::ComputeStereoMatches (frame.cc:189) is timed as an extra
column (GPU: on the two handles' resident outputs).

    python tools/bench_latency.py [--frames 40]
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

PARAMS = (1000, 1.2, 8, 20, 7)
FX, BASE = 435.2, 0.11


def _stereo_extract(exl, exr, left, right):
    out = {}
    th = threading.Thread(target=lambda: out.__setitem__("r", exr(right)))
    th.start()
    res_l = exl(left)
    th.join()
    return res_l, out["r"]


def measure(frames: int = 40, warmup: int = 5, cpu_frames: int = 8) -> dict:
    from orb_slam_fusion_amd import (OrbExtractor, PoseFrame, PoseOptimizer,
                                     compute_stereo_matches, synth)

    pairs = [synth.stereo_frame(i) for i in range(frames)]
    probs = [synth.pose_problem(synth.POSE_SEED + i, 600, 10) for i in range(frames)]
    exl, exr = OrbExtractor(*PARAMS), OrbExtractor(*PARAMS)
    opt = PoseOptimizer(max_obs=600)
    bf = np.float32(FX * BASE)
    mb = np.float32(bf / np.float32(FX))
    t_ex, t_st, t_po = [], [], []
    for i in range(warmup + frames):
        left, right = pairs[i % frames]
        cam, pin, _, obs = probs[i % frames]
        t0 = time.perf_counter()
        (_, kl, _), _ = _stereo_extract(exl, exr, left, right)
        t1 = time.perf_counter()
        compute_stereo_matches(exl, exr, len(kl), bf, mb)
        t2 = time.perf_counter()
        opt.PoseOptimization(PoseFrame(cam=cam, pose=pin, obs=obs))
        t3 = time.perf_counter()
        if i >= warmup:
            t_ex.append(t1 - t0), t_st.append(t2 - t1), t_po.append(t3 - t2)
    med = lambda a: float(np.median(a)) * 1e3  # noqa: E731
    out = {
        "workload": "one 752x480 stereo frame at a time through the host ABI: 2-thread "
                    "extraction (1000 kp, 8 levels) + PoseOptimization (600 obs); median of "
                    f"{frames} frames",
        "gpu_ms_per_frame": round(med(t_ex) + med(t_po), 3),
        "gpu_extract_ms": round(med(t_ex), 3),
        "gpu_pose_ms": round(med(t_po), 3),
        "gpu_stereo_ms": round(med(t_st), 3),
    }
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
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=40)
    a = ap.parse_args()
    print(json.dumps(measure(a.frames)))
