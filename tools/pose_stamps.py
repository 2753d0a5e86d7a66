"""Per-phase cycle shares of the pose kernel from the ORB_STAMPS build.

    ORBGPU_LIB=orb_slam_fusion_amd/lib/liborbgpu_stamps.so python tools/pose_stamps.py [--batch B]

(--batch 1: the single-problem latency case; s_memtime ticks at 100 MHz)
"""
import argparse
import ctypes
import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))


def main():
    import torch

    from orb_slam_fusion_amd import PoseOptimizer, synth
    from orb_slam_fusion_amd._lib import library_path

    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    B = ap.parse_args().batch
    probs = [synth.pose_problem(7 + i, 600, 10) for i in range(B)]
    obs = torch.from_numpy(np.stack([p[3] for p in probs]).view(np.float32).reshape(B, 600, 7).copy()).cuda()
    pin = torch.from_numpy(np.stack([p[1] for p in probs])).cuda()
    nobs = torch.full((B,), 600, dtype=torch.int32, device="cuda")
    pout = torch.zeros((B, 7), dtype=torch.float32, device="cuda")
    outl = torch.zeros((B, 600), dtype=torch.uint8, device="cuda")
    inl = torch.zeros(B, dtype=torch.int32, device="cuda")
    opt = PoseOptimizer(max_problems=B, max_obs=600)
    lib = ctypes.CDLL(str(library_path()))
    buf = (ctypes.c_ulonglong * 16)()
    opt.batch(probs[0][0], pin, obs, nobs, pout, outl, inl)
    torch.cuda.synchronize()
    lib.orbgpu_debug_pose_stamps(buf, 16)
    iters = 5
    for _ in range(iters):
        opt.batch(probs[0][0], pin, obs, nobs, pout, outl, inl)
    torch.cuda.synchronize()
    assert lib.orbgpu_debug_pose_stamps(buf, 16) == 0
    v = list(buf)
    tot = sum(v[i] for i in range(8))
    names = {0: "control", 1: "build_sweep", 2: "ldlt", 3: "se3_exp", 4: "chi_sweep", 5: "classify"}
    print(json.dumps({"batch": B, "ticks_per_problem": tot / (B * iters), "us_per_problem_at_100MHz": tot / (B * iters) / 100, "builds_per_problem": v[8] / (B * iters),
                      "trials_per_problem": v[9] / (B * iters),
                      "trial_rounds_per_problem": v[10] / (B * iters),
                      "share": {names[i]: round(v[i] / max(tot, 1), 3) for i in names}}))


if __name__ == "__main__":
    main()
