"""Diagnostic (not a bench line): bench.py's headline step with parts switched,
to price each part's share of the concurrent mix on one GPU.

    python tools/mix_probe.py [--pose on|off] [--groups 1|2] [--pipes 2]
                              [--pose-chunk N] [--frames 2560] [--steps 6]

Prints {"frames_per_s": ..., ...}.  --pose off drops the PoseOptimization
launches (extraction alone); --groups sets the pose kernel's trial groups
per problem (orbgpu_pose_ctx_set_trial_groups)."""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))

W, H, POSE_OBS = 752, 480, 600
PARAMS = (1000, 1.2, 8, 20, 7)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pose", default="on")
    ap.add_argument("--groups", type=int, default=0)
    ap.add_argument("--pipes", type=int, default=2)
    ap.add_argument("--frames", type=int, default=2560)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--pose-chunk", type=int, default=0, help="pose problems per launch (0: the whole group)")
    a = ap.parse_args()
    import torch

    from orb_slam_fusion_amd import OrbExtractor, PoseOptimizer, synth
    from orb_slam_fusion_amd._lib import lib

    dev = torch.device("cuda", 0)
    B, Bg, P = a.frames, a.batch, a.pipes
    G, Bp = B // Bg, Bg // P
    frames = [synth.stereo_frame(i % 64) for i in range(B)]
    d_imgs = torch.from_numpy(np.stack([im for fr in frames for im in fr])).to(dev)
    probs = [synth.pose_problem(synth.POSE_SEED + i, POSE_OBS, 10) for i in range(64)]
    cam = probs[0][0]
    pipes = [OrbExtractor(*PARAMS, device=0, max_width=W, max_height=H, max_images=2 * Bp) for _ in range(P)]
    cap = pipes[0].max_keypoints(W, H)
    d_kps = torch.zeros((2 * B, cap, 7), dtype=torch.int32, device=dev)
    d_desc = torch.zeros((2 * B, cap, 32), dtype=torch.uint8, device=dev)
    d_n = torch.zeros(2 * B, dtype=torch.int32, device=dev)
    d_mono = torch.zeros(2 * B, dtype=torch.int32, device=dev)
    obs = np.stack([probs[i % 64][3] for i in range(B)]).view(np.float32).reshape(B, POSE_OBS, 7)
    d_obs = torch.from_numpy(obs.copy()).to(dev)
    d_pin = torch.from_numpy(np.stack([probs[i % 64][1] for i in range(B)])).to(dev)
    d_nobs = torch.full((B,), POSE_OBS, dtype=torch.int32, device=dev)
    d_pout = torch.zeros((B, 7), dtype=torch.float32, device=dev)
    d_out = torch.zeros((B, POSE_OBS), dtype=torch.uint8, device=dev)
    d_inl = torch.zeros(B, dtype=torch.int32, device=dev)
    opt = PoseOptimizer(device=0, max_problems=Bg, max_obs=POSE_OBS)
    if a.groups:
        lib().orbgpu_pose_ctx_set_trial_groups(opt._h, a.groups, a.groups)
    s_pose = torch.cuda.Stream(dev, priority=-1)

    def step():
        for g in range(G):
            f0 = g * Bg
            sl = slice(f0, f0 + Bg)
            if a.pose == "on":
                ck = a.pose_chunk or Bg
                for c0 in range(f0, f0 + Bg, ck):
                    cs = slice(c0, c0 + ck)
                    opt.batch(cam, d_pin[cs], d_obs[cs], d_nobs[cs], d_pout[cs], d_out[cs], d_inl[cs], stream=s_pose)
            for k, e in enumerate(pipes):
                isl = slice(2 * (f0 + Bp * k), 2 * (f0 + Bp * (k + 1)))
                e.extract_batch(d_imgs[isl], d_kps[isl], d_desc[isl], d_n[isl], d_mono[isl], stream=0)

    step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(json.dumps({"frames_per_s": round(B * a.steps / el, 1), "pose": a.pose, "groups": a.groups,
                      "pose_chunk": a.pose_chunk,
                      "pipes": P, "frames": B, "steps": a.steps}))


if __name__ == "__main__":
    main()
