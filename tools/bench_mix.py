"""Diagnostic: the headline step's stream mix, taken apart.  Times the same
launch groups as bench.py (2 extractor pipelines of 64 images + the pose batch
of 64 problems on a high-priority stream) with and without the pose stream,
and the pose batches alone, so the cost of running them together is visible.

    python tools/bench_mix.py [--groups 40] [--pipes 2]
"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))

W, H = 752, 480
PARAMS = (1000, 1.2, 8, 20, 7)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", type=int, default=40)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--pipes", type=int, default=2)
    ap.add_argument("--pose-priority", type=int, default=-1, help="torch stream priority of the pose stream")
    a = ap.parse_args()
    import torch

    from orb_slam_fusion_amd import OrbExtractor, PoseOptimizer, synth

    Bg, P = a.batch, a.pipes
    Bp = Bg // P
    frames = [synth.stereo_frame(i) for i in range(Bg)]
    d_imgs = torch.from_numpy(np.stack([im for fr in frames for im in fr])).cuda()
    probs = [synth.pose_problem(synth.POSE_SEED + i, 600, 10) for i in range(Bg)]
    cam = probs[0][0]
    d_obs = torch.from_numpy(np.stack([p[3] for p in probs]).view(np.float32).reshape(Bg, 600, 7).copy()).cuda()
    d_pin = torch.from_numpy(np.stack([p[1] for p in probs])).cuda()
    d_n = torch.full((Bg,), 600, dtype=torch.int32, device="cuda")
    d_pout = torch.zeros((Bg, 7), dtype=torch.float32, device="cuda")
    d_out = torch.zeros((Bg, 600), dtype=torch.uint8, device="cuda")
    d_inl = torch.zeros(Bg, dtype=torch.int32, device="cuda")
    opt = PoseOptimizer(max_problems=Bg, max_obs=600)
    pipes = [OrbExtractor(*PARAMS, max_width=W, max_height=H, max_images=2 * Bp) for _ in range(P)]
    cap = pipes[0].max_keypoints(W, H)
    kps = torch.zeros((2 * Bg, cap, 7), dtype=torch.int32, device="cuda")
    desc = torch.zeros((2 * Bg, cap, 32), dtype=torch.uint8, device="cuda")
    n = torch.zeros(2 * Bg, dtype=torch.int32, device="cuda")
    mono = torch.zeros(2 * Bg, dtype=torch.int32, device="cuda")
    s_pose = torch.cuda.Stream(priority=a.pose_priority)

    def run(ext, pose):
        for _ in range(a.groups):
            if pose:
                opt.batch(cam, d_pin, d_obs, d_n, d_pout, d_out, d_inl, stream=s_pose)
            if ext:
                for k, e in enumerate(pipes):
                    sl = slice(2 * Bp * k, 2 * Bp * (k + 1))
                    e.extract_batch(d_imgs[sl], kps[sl], desc[sl], n[sl], mono[sl], stream=0)

    res = {}
    for name, ext, pose in [("both", True, True), ("extract_only", True, False), ("pose_only", False, True)]:
        run(ext, pose)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(ext, pose)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / a.groups
        res[name] = {"ms_per_group": round(ms, 4), "frames_per_s": round(Bg / ms * 1e3, 1)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
