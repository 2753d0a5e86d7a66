"""Isolated per-kernel timing of the extractor chain and the pose kernel
(no concurrency), for rocprofv3 runs and quick A/B checks on the GPU box.

    python tools/prof_stages.py [--frames 64] [--iters 20] [--mode ext|pose|both]
"""
import argparse
import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--mode", default="both")
    a = ap.parse_args()
    import torch

    from orb_slam_fusion_amd import OrbExtractor, PoseOptimizer, synth

    B = a.frames
    imgs = np.stack([im for i in range(B) for im in synth.stereo_frame(i)])
    d_imgs = torch.from_numpy(imgs).cuda()
    ex = OrbExtractor(1000, 1.2, 8, 20, 7, max_images=2 * B)
    cap = ex.max_keypoints(752, 480)
    kps = torch.zeros((2 * B, cap, 7), dtype=torch.int32, device="cuda")
    desc = torch.zeros((2 * B, cap, 32), dtype=torch.uint8, device="cuda")
    n = torch.zeros(2 * B, dtype=torch.int32, device="cuda")
    mono = torch.zeros(2 * B, dtype=torch.int32, device="cuda")
    probs = [synth.pose_problem(7 + i, 600, 10) for i in range(B)]
    obs = torch.from_numpy(np.stack([p[3] for p in probs]).view(np.float32).reshape(B, 600, 7).copy()).cuda()
    pin = torch.from_numpy(np.stack([p[1] for p in probs])).cuda()
    nobs = torch.full((B,), 600, dtype=torch.int32, device="cuda")
    pout = torch.zeros((B, 7), dtype=torch.float32, device="cuda")
    outl = torch.zeros((B, 600), dtype=torch.uint8, device="cuda")
    inl = torch.zeros(B, dtype=torch.int32, device="cuda")
    opt = PoseOptimizer(max_problems=B, max_obs=600)
    s = torch.cuda.Stream()
    res = {}
    if a.mode in ("ext", "both"):
        for _ in range(3):
            ex.extract_batch(d_imgs, kps, desc, n, mono, stream=s)
        torch.cuda.synchronize()
        ex.profile(a.iters)
        for _ in range(a.iters):
            ex.extract_batch(d_imgs, kps, desc, n, mono, stream=s)
        torch.cuda.synchronize()
        calls, ms = ex.profile_read()
        res["extract_ms"] = {k: round(v / calls, 4) for k, v in ms.items()}
        res["extract_total_ms"] = round(sum(ms.values()) / calls, 4)
    if a.mode in ("pose", "both"):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(2):
            opt.batch(probs[0][0], pin, obs, nobs, pout, outl, inl, stream=s)
        torch.cuda.synchronize()
        e0.record(s)
        for _ in range(a.iters):
            opt.batch(probs[0][0], pin, obs, nobs, pout, outl, inl, stream=s)
        e1.record(s)
        torch.cuda.synchronize()
        res["pose_ms"] = round(e0.elapsed_time(e1) / a.iters, 4)
    res["frames"] = B
    print(json.dumps(res))


if __name__ == "__main__":
    main()
