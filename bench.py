#!/usr/bin/env python3
"""Throughput bench: ORB extract (stereo, 752x480, 1000 kp, 8 levels) +
PoseOptimization (600 observations) per frame on MI355X.

A step = one batch of B synthetic stereo frames per GPU: 2B images through
the gfx950 extractor (orbgpu_extract_batch) and B pose-only problems through
the gfx950 PoseOptimization (orbgpu_pose_opt_batch) on a second, concurrent
HIP stream, inputs resident in HBM.  Frames shard across ranks (contiguous
blocks of B frame ids per rank, orb_slam_fusion_amd/dist.py): no
data-path collective, weak scaling; the max over ranks of the timed region is
the job time.  Prints one JSON line on rank 0 (contract in the task README).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--frames B]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))

METRIC = "fps ORB extract+PoseOpt, 752×480 stereo @1/2/4/8 GPU; descriptors bit-exact"
W, H = 752, 480
PARAMS = (1000, 1.2, 8, 20, 7)
POSE_OBS = 600
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def level_sizes(inv_scale):
    return [(int(np.rint(np.float32(W) * s)), int(np.rint(np.float32(H) * s))) for s in inv_scale]


def stage_bytes(sizes, n_kp):
    """Algorithmic bytes per image for each extractor stage."""
    px = [w * h for w, h in sizes]
    return {
        "resize": sum(px[l - 1] + px[l] for l in range(1, len(px))),
        "blur": 2 * sum(px),
        "fast_cells": sum(px),
        "octree": 0,  # sequential list rebuilds on a few KB: latency-bound, no HBM claim
        "describe": n_kp * (749 + 512 + 4 + 32),
        "assemble": n_kp * (4 + 4 + 32 + 28 + 32),
    }


def cpu_baseline(frames, probs, budget_s: float):
    """Oracle (`kind: port`) timed on this host: stereo extraction on two threads
    (as Frame's stereo constructor, frame.cc:179-182) + PoseOptimization on one."""
    sys.path.insert(0, str(REPO / "oracle"))
    import binding as oracle  # noqa: E402  (cpu_baseline leg only)

    ex_l = oracle.OracleExtractor(*PARAMS)
    ex_r = oracle.OracleExtractor(*PARAMS)
    done, t0 = 0, time.perf_counter()
    while True:
        left, right = frames[done % len(frames)]
        th = threading.Thread(target=ex_r.extract, args=(right,))
        th.start()
        ex_l.extract(left)
        th.join()
        cam, pin, _, obs = probs[done % len(probs)]
        oracle.pose_opt(cam, pin, obs)
        done += 1
        el = time.perf_counter() - t0
        if (el >= budget_s and done >= 5) or done >= 2000:
            break
    return {
        "value": round(done / el, 3),
        "unit": "frames/s",
        "cores": 2,
        "kind": "port",
        "sample": f"{done} synthetic 752x480 stereo frames: oracle extract (2 threads, one per "
        f"image) + oracle PoseOptimization ({POSE_OBS} obs, 1 thread), {el:.1f} s",
    }


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--frames", type=int, default=64, help="stereo frames per GPU per step")
    ap.add_argument("--pipes", type=int, default=2,
                    help="extractor pipelines per GPU (each its own handle + HIP stream, "
                         "frames of a step split evenly between them)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-lba", action="store_true", help="skip the LocalBundleAdjustment side line")
    ap.add_argument("--no-stereo", action="store_true", help="skip the ComputeStereoMatches side line")
    ap.add_argument("--no-match", action="store_true",
                    help="skip the SearchByProjection (motion-model search) side line")
    ap.add_argument("--no-bow", action="store_true", help="skip the DBoW2 transform side line")
    ap.add_argument("--no-inertial", action="store_true",
                    help="skip the PoseInertialOptimizationLastFrame side line")
    ap.add_argument("--no-track", action="store_true",
                    help="skip the device-resident tracking-chain side line")
    ap.add_argument("--no-latency", action="store_true",
                    help="skip the per-frame host-path latency side line")
    args = ap.parse_args()

    import torch

    from orb_slam_fusion_amd import OrbExtractor, PoseOptimizer, dist, synth

    rank, world, local = dist.rank_world()
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}; using {world}", file=sys.stderr)
    dist.init(world, rank)  # gloo, timing coordination only: no data-path collective
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    B = args.frames
    frames = [synth.stereo_frame(i) for i in dist.frame_indices(rank, world, B)]
    imgs = np.stack([im for fr in frames for im in fr])  # [2B, H, W]: L0 R0 L1 R1 ...
    probs = [synth.pose_problem(synth.POSE_SEED + i, POSE_OBS, 10)
             for i in dist.frame_indices(rank, world, B)]
    cam = probs[0][0]

    d_imgs = torch.from_numpy(imgs).to(dev)
    P = max(1, min(args.pipes, B))
    if B % P:
        raise SystemExit(f"--frames {B} not divisible by --pipes {P}")
    Bp = B // P  # stereo frames per pipeline
    # one extractor handle per pipeline; each runs on its own library stream
    pipes = [OrbExtractor(*PARAMS, device=local, max_width=W, max_height=H, max_images=2 * Bp)
             for _ in range(P)]
    ex = pipes[0]
    cap = ex.max_keypoints(W, H)
    d_kps = torch.zeros((2 * B, cap, 7), dtype=torch.int32, device=dev)
    d_desc = torch.zeros((2 * B, cap, 32), dtype=torch.uint8, device=dev)
    d_n = torch.zeros(2 * B, dtype=torch.int32, device=dev)
    d_mono = torch.zeros(2 * B, dtype=torch.int32, device=dev)

    obs = np.stack([p[3] for p in probs]).view(np.float32).reshape(B, POSE_OBS, 7)
    d_obs = torch.from_numpy(obs.copy()).to(dev)
    d_pin = torch.from_numpy(np.stack([p[1] for p in probs])).to(dev)
    d_nobs = torch.full((B,), POSE_OBS, dtype=torch.int32, device=dev)
    d_pout = torch.zeros((B, 7), dtype=torch.float32, device=dev)
    d_out = torch.zeros((B, POSE_OBS), dtype=torch.uint8, device=dev)
    d_inl = torch.zeros(B, dtype=torch.int32, device=dev)
    opt = PoseOptimizer(device=local, max_problems=B, max_obs=POSE_OBS)

    # Two HIP streams: the extractor's kernel chain and the pose kernel run
    # concurrently (frame k's pose overlaps frame k+1's extraction in a
    # pipelined tracker; within a step the B frames are independent).
    s_pose = torch.cuda.Stream(dev, priority=-1)  # high-priority pool: its own HW queue
    pose_ev = []

    def step(timed: bool):
        # the pose kernel (64 long-lived blocks) is queued first so its blocks
        # take their CUs before the extractor's wide grids fill the device
        if timed:
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(s_pose)
        opt.batch(cam, d_pin, d_obs, d_nobs, d_pout, d_out, d_inl, stream=s_pose)
        if timed:
            e1.record(s_pose)
            pose_ev.append((e0, e1))
        for k, e in enumerate(pipes):  # stream=0: the handle's own HIP stream
            sl = slice(2 * Bp * k, 2 * Bp * (k + 1))
            e.extract_batch(d_imgs[sl], d_kps[sl], d_desc[sl], d_n[sl], d_mono[sl], stream=0)

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize()
    for e in pipes:
        e.check()

    ex.profile(args.steps)
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize()
    dist.barrier()
    elapsed = dist.job_time(time.perf_counter() - t0)
    for e in pipes:
        e.check()

    calls, stage_ms = ex.profile_read()
    pose_ms = sum(a.elapsed_time(b) for a, b in pose_ev) / max(len(pose_ev), 1)
    n_kp = d_n.cpu().numpy()
    inl = d_inl.cpu().numpy()

    total_frames = world * B * args.steps
    fps = total_frames / elapsed
    ms_per_step = elapsed / args.steps * 1e3

    sizes = level_sizes(ex.GetInverseScaleFactors())
    per_img = stage_bytes(sizes, int(n_kp.mean()))
    stage_avg = {k: v / max(calls, 1) for k, v in stage_ms.items()}
    stage_avg["pose_opt"] = pose_ms
    dom = max(stage_avg, key=stage_avg.get)
    if dom == "pose_opt" or per_img.get(dom, 0) == 0:
        # the dominant kernel is latency-bound; quote the largest HBM-bound stage too
        hbm_stages = {k: v for k, v in stage_avg.items() if per_img.get(k, 0) > 0}
        roof_stage = max(hbm_stages, key=hbm_stages.get)
    else:
        roof_stage = dom
    roof_bytes = per_img[roof_stage] * 2 * Bp  # one launch of pipeline 0 covers 2*Bp images
    roof_ms = stage_avg[roof_stage]
    achieved = roof_bytes / (roof_ms * 1e-3) / 1e9
    traffic = None
    pmc = REPO / "profiles" / "pmc_traffic.json"
    if pmc.exists():
        try:
            tj = json.loads(pmc.read_text())  # tools/pmc_traffic.sh: HBM bytes per launch
            if roof_stage in tj:  # scaled to this run's images per launch
                per = tj[roof_stage] / tj[roof_stage + "_detail"]["images_per_launch"]
                traffic = round(per * 2 * Bp)
        except Exception:
            traffic = None
    # what actually bounds the kernel: VALU-busy fraction of its SIMDs from the
    # SQ counter passes (tools/profile_round.sh -> profiles/pmc_sq.json):
    # SQ_ACTIVE_INST_VALU (quad-cycles, summed over waves) x 4 / (SQ_BUSY_CYCLES
    # (cycles summed over the 32 shader engines) x 32 SIMDs per engine)
    valu_busy = None
    sq = REPO / "profiles" / "pmc_sq.json"
    kname = {"resize": "k_resize", "blur": "k_blur", "fast_cells": "k_fast_cells", "octree": "k_octree",
             "describe": "k_describe", "assemble": "k_assemble"}.get(roof_stage)
    if sq.exists() and kname:
        try:
            k = json.loads(sq.read_text())[kname]
            valu_busy = round(4 * k["SQ_ACTIVE_INST_VALU"] / (32 * k["SQ_BUSY_CYCLES"]), 3)
        except Exception:
            valu_busy = None

    result = {
        "metric": METRIC,
        "value": round(fps, 2),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {
            "workload": "ORBextractor 752x480 stereo, 1000 kp, 8 levels, scale 1.2, FAST 20/7 "
            f"+ PoseOptimization ({POSE_OBS} obs, 70% stereo, 10% outliers, fp64 LM)",
            "frames_per_gpu_per_step": B,
            "images_per_gpu_per_step": 2 * B,
            "parallelism": f"frames sharded over {world} GPU(s), no collective",
            "streams": f"{P} extractor pipelines ({2 * Bp} images each, own HIP stream) + pose "
                       "kernel on a high-priority stream, all concurrent",
            "keypoints_per_image_mean": float(n_kp.mean()),
            "pose_inliers_mean": float(inl.mean()),
        },
        "roofline": {
            "bound": "hbm",
            "kernel": roof_stage,
            "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "algorithmic_bytes_per_launch": int(roof_bytes),
            "avg_launch_ms": round(roof_ms, 5),
            "valu_busy": valu_busy,
            "limiter": "valu issue" if valu_busy is not None and valu_busy > 0.6 else None,
        },
        "stage_ms_per_step": {k: round(v, 5) for k, v in stage_avg.items()},
        "dominant_stage": dom,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(frames, probs, args.cpu_seconds)
    if rank == 0 and world == 1 and not args.no_lba:
        # SURVEY §8 row c, reported beside the headline metric (not part of it):
        # C4 LocalBundleAdjustment window, GPU vs the CPU oracle (1 thread)
        sys.path.insert(0, str(REPO / "tools"))
        from bench_lba import measure  # noqa: E402

        result["lba"] = measure(calls=10, cpu_calls=0 if args.no_cpu_baseline else 3)
    if rank == 0 and world == 1 and not args.no_stereo:
        # SURVEY §8(f) rank 1, beside the headline metric (not part of it):
        # Frame::ComputeStereoMatches per frame on resident extractor outputs
        sys.path.insert(0, str(REPO / "tools"))
        from bench_stereo import measure as measure_stereo  # noqa: E402

        result["stereo"] = measure_stereo(frames=B, calls=20, cpu_frames=0 if args.no_cpu_baseline else 4)
    if rank == 0 and world == 1 and not args.no_match:
        # SURVEY §8(f) rank 2, beside the headline metric (not part of it):
        # SearchByProjection(CurrentFrame, LastFrame) on resident frame outputs
        sys.path.insert(0, str(REPO / "tools"))
        from bench_match import measure as measure_match  # noqa: E402

        result["match"] = measure_match(frames=B, calls=20, cpu_frames=0 if args.no_cpu_baseline else 4)
    if rank == 0 and world == 1 and not args.no_bow:
        # SURVEY §8(f) rank 4, beside the headline metric (not part of it):
        # DBoW2 transform (Frame::ComputeBoW) on resident extractor descriptors
        sys.path.insert(0, str(REPO / "tools"))
        from bench_bow import measure as measure_bow  # noqa: E402

        result["bow"] = measure_bow(frames=B, calls=20, cpu_frames=0 if args.no_cpu_baseline else 4)
    if rank == 0 and world == 1 and not args.no_inertial:
        # PoseInertialOptimizationLastFrame (stereo-inertial
        # tracking after IMU initialisation), a batch resident in HBM
        sys.path.insert(0, str(REPO / "tools"))
        from bench_inertial import measure as measure_inertial  # noqa: E402

        result["inertial"] = measure_inertial(problems=B, calls=20, mode=0,
                                              cpu_problems=0 if args.no_cpu_baseline else 4)
    if rank == 0 and world == 1 and not args.no_track:
        # config C3's path on synthetic data: extract + stereo + SearchByProjection
        # + PoseOptimization chained on the device, vs the oracle chain on the CPU
        sys.path.insert(0, str(REPO / "tools"))
        from bench_track import measure as measure_track  # noqa: E402

        result["track"] = measure_track(frames=B, calls=10, cpu_frames=0 if args.no_cpu_baseline else 4)
    if rank == 0 and world == 1 and not args.no_latency:
        # north_star's per-frame target: one stereo frame at a time through the
        # host ABI (2-thread extraction + PoseOptimization) vs the CPU oracle
        sys.path.insert(0, str(REPO / "tools"))
        from bench_latency import measure as measure_latency  # noqa: E402

        result["latency"] = measure_latency(frames=40, cpu_frames=0 if args.no_cpu_baseline else 8)
    if rank == 0:
        print(json.dumps(result), flush=True)
    dist.finalize()
    return 0


if __name__ == "__main__":
    sys.exit(main())
