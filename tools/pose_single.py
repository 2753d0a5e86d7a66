"""Single-problem PoseOptimization latency through the host ABI (one frame's
600 observations at a time), for each speculative trial-group count, by the
zero-copy direct launch (default) and by the copy + hipGraph path.

    python tools/pose_single.py [--frames 40]
"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def measure(frames=40, warmup=5):
    from orb_slam_fusion_amd import PoseFrame, PoseOptimizer, synth

    probs = [synth.pose_problem(synth.POSE_SEED + i, 600, 10) for i in range(frames)]
    import os

    out = {}
    for io, g in (("direct", 1), ("direct", 2), ("graph", 1)):
        os.environ["ORBGPU_POSE_IO"] = io  # read at context creation (pose_api.cpp)
        opt = PoseOptimizer(max_obs=600, trial_groups=g)
        ts = []
        for i in range(warmup + frames):
            cam, pin, _, obs = probs[i % frames]
            t0 = time.perf_counter()
            opt.PoseOptimization(PoseFrame(cam=cam, pose=pin, obs=obs))
            if i >= warmup:
                ts.append(time.perf_counter() - t0)
        out[f"{io}_groups_{g}_ms"] = round(float(np.median(ts)) * 1e3, 4)
        opt.close()
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=40)
    print(json.dumps(measure(ap.parse_args().frames)))
