#!/usr/bin/env python3
"""Throughput bench: ORB extract (stereo, 752x480, 1000 kp, 8 levels) +
PoseOptimization (600 observations) per frame on MI355X.

A step = B distinct synthetic stereo frames per GPU (default 7680, all
resident in HBM before the timed region), as one launch group: 15360
images through the gfx950 extractor (orbgpu_extract_batch, four pipelines of
3840 images, each its own HIP stream, each a stage behind the previous one)
and 7680 pose-only problems through the gfx950 PoseOptimization
(orbgpu_pose_opt_batch) on a concurrent high-priority stream.  Frames shard across ranks (contiguous
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
PROFILE_ROUND = "r06"  # profiles/<round>/kernels.json (tools/profile_round.sh)
SIDE_BATCH = 256  # frames / problems per call of the side lines (stereo, match, BoW, inertial, track)


def level_sizes(inv_scale):
    return [(int(np.rint(np.float32(W) * s)), int(np.rint(np.float32(H) * s))) for s in inv_scale]


def stage_bytes(sizes, n_kp):
    """Algorithmic bytes per image for each extractor stage (SURVEY.md §8(d),
    DESIGN.md §5): the bytes the reference algorithm must read and write once."""
    px = [w * h for w, h in sizes]
    return {
        "resize": sum(px[l - 1] + px[l] for l in range(1, len(px))),  # read l-1, write l
        "blur": 2 * sum(px),                                           # read + write every level
        "fast_cells": sum(px),                                         # read every level
        "octree": 0,  # a few KB of candidates per level: latency-bound, no HBM claim
        "describe": n_kp * (749 + 512),                                # IC_Angle circle + BRIEF samples
        "assemble": n_kp * (28 + 32),                                  # keypoint record + descriptor
    }


def describe_plane_floor(sizes, n_kp):
    """k_describe's fetch floor per image: 1000 keypoints' 31x31 (raw) and 37x37
    (blurred) patches cover every level, so the raw and blurred planes are each
    fetched about once whatever the staging: both planes + the
    angle / descriptor writes."""
    return 2 * sum(w * h for w, h in sizes) + n_kp * (4 + 32)


STAGE_KERNELS = {"resize": "k_resize", "blur": "k_blur", "fast_cells": "k_fast_cells",
                 "octree": "k_octree", "describe": "k_describe", "assemble": "k_assemble",
                 "pose_opt": "k_pose_opt"}


def host_cpu() -> dict:
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"cpu_model": model, "nproc": os.cpu_count(),
            "affinity": len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None}


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
        "build": "oracle/Makefile: g++ -O2 -march=x86-64-v3 -ffp-contract=off; a scalar "
                 "restatement -- no OpenCV SIMD in FAST / resize / GaussianBlur, so slower than "
                 "the reference's OpenCV build (the GPU/CPU ratio overstates the gap)",
        **host_cpu(),
    }


def load_profile():
    """Per-kernel evidence committed under profiles/<round>/ by
    tools/profile_round.sh: HBM bytes (FETCH_SIZE x2 + WRITE_SIZE, separate
    passes) and calibrated VALU-busy per extractor-stage launch."""
    # (BENCH_KERNELS_JSON: the kernels.json tools/profile_round.sh has just
    # written, so its bench line and its profile come from the same run)
    f = Path(os.environ.get("BENCH_KERNELS_JSON", REPO / "profiles" / PROFILE_ROUND / "kernels.json"))
    if not f.exists():
        return None
    try:
        return json.loads(f.read_text())
    except ValueError:
        return None


def load_fast_stamps():
    """k_fast_cells phase stamps (tools/stamps.py on the ORB_STAMPS build):
    the share of cells that ran the minTh fallback pass -- from the latest
    round that recorded them (-> (data, path))."""
    for r in sorted({PROFILE_ROUND, "r04", "r03", "r02"}, reverse=True):
        f = REPO / "profiles" / r / "fast_stamps.json"
        try:
            if f.exists():
                return json.loads(f.read_text()), f"profiles/{r}/fast_stamps.json"
        except ValueError:
            pass
    return None, None


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20,
                    help="timed steps (20 x ~62 ms: a timed region over 1 s, also at the driver's "
                         "--steps 20)")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--frames", type=int, default=7680,
                    help="stereo frames per GPU per step (all distinct, resident in HBM)")
    ap.add_argument("--batch", type=int, default=7680,
                    help="stereo frames per launch group (DESIGN §11: one group of the step's 7680 "
                         "frames over four pipelines measured best in the tools/ab_bench.sh sweep)")
    ap.add_argument("--pipes", type=int, default=4,
                    help="extractor pipelines per GPU (each its own handle + HIP stream, "
                         "each launch group split evenly between them)")
    ap.add_argument("--phase-stage", type=int, default=2,
                    help="pipeline k+1 starts each launch group when pipeline k has finished this "
                         "stage of it (0 pyramid .. 5 assembly; -1: no offset)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-lba", action="store_true", help="skip the LocalBundleAdjustment side line")
    ap.add_argument("--no-lia", action="store_true", help="skip the LocalInertialBA side line")
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
    ap.add_argument("--no-latency-inertial", action="store_true",
                    help="skip the stereo-inertial per-frame host-path latency side line")
    ap.add_argument("--no-c5", action="store_true",
                    help="skip the synthetic-sequence (C5 layout) side line")
    ap.add_argument("--no-lba-sharded", action="store_true",
                    help="skip the 4-rank point-sharded LBA side line")
    args = ap.parse_args()

    import torch

    from orb_slam_fusion_amd import OrbExtractor, PoseOptimizer, dist, synth

    rank, world, local = dist.rank_world()
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}; using {world}", file=sys.stderr)
    dist.init(world, rank)  # gloo, timing coordination only: no data-path collective
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    Bg = args.batch
    if args.frames % Bg:
        raise SystemExit(f"--frames {args.frames} not divisible by --batch {Bg}")
    G = args.frames // Bg  # launch groups per step
    P = max(1, min(args.pipes, Bg))
    if Bg % P:
        raise SystemExit(f"--batch {Bg} not divisible by --pipes {P}")
    Bp = Bg // P  # stereo frames per pipeline launch
    B = args.frames
    ids = dist.frame_indices(rank, world, B)
    from concurrent.futures import ThreadPoolExecutor

    with ThreadPoolExecutor(max_workers=16) as pool:  # ctypes releases the GIL
        frames = list(pool.map(synth.stereo_frame, ids))
    probs = [synth.pose_problem(synth.POSE_SEED + i, POSE_OBS, 10) for i in ids]
    cam = probs[0][0]

    d_imgs = torch.empty((2 * B, H, W), dtype=torch.uint8, device=dev)  # L0 R0 L1 R1 ...
    for k in range(0, B, 256):
        chunk = np.stack([im for fr in frames[k:k + 256] for im in fr])
        d_imgs[2 * k:2 * k + len(chunk)].copy_(torch.from_numpy(chunk))
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
    opt = PoseOptimizer(device=local, max_problems=Bg, max_obs=POSE_OBS)

    # Two kinds of HIP streams: each extractor pipeline's own, and a
    # high-priority one for the pose kernel (frame k's pose overlaps frame
    # k+1's extraction in a pipelined tracker; within a step the frames are
    # independent).
    s_pose = torch.cuda.Stream(dev, priority=-1)  # high-priority pool: its own HW queue
    pose_ev = []
    # pipeline k + 1 runs each group part-way behind pipeline k (--phase-stage):
    # its VALU-bound stages then overlap the other's latency-bound ones
    s_pipe = [torch.cuda.Stream(dev) for _ in pipes]
    ph_ev = []
    if args.phase_stage >= 0:
        for k in range(P - 1):
            ev = torch.cuda.Event()
            ev.record(s_pipe[k])  # creates the event
            pipes[k].set_stage_event(args.phase_stage, ev)
            ph_ev.append(ev)

    def step(timed: bool):
        for g in range(G):
            f0 = g * Bg
            # the pose kernel (Bg long-lived blocks) is queued first so its
            # blocks take their CUs before the extractor's wide grids fill the device
            if timed:
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(s_pose)
            sl = slice(f0, f0 + Bg)
            opt.batch(cam, d_pin[sl], d_obs[sl], d_nobs[sl], d_pout[sl], d_out[sl], d_inl[sl],
                      stream=s_pose)
            if timed:
                e1.record(s_pose)
                pose_ev.append((e0, e1))
            for k, e in enumerate(pipes):
                isl = slice(2 * (f0 + Bp * k), 2 * (f0 + Bp * (k + 1)))
                if k > 0 and ph_ev:
                    s_pipe[k].wait_event(ph_ev[k - 1])
                e.extract_batch(d_imgs[isl], d_kps[isl], d_desc[isl], d_n[isl], d_mono[isl], stream=s_pipe[k])

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize()
    for e in pipes:
        e.check()

    for e in pipes:  # stage events on every pipeline: the stage times average over all four
        e.profile(args.steps * G)
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

    calls, stage_ms = 0, {}
    for e in pipes:
        c, ms = e.profile_read()
        calls += c
        for k, v in ms.items():
            stage_ms[k] = stage_ms.get(k, 0.0) + v
    pose_ms = sum(a.elapsed_time(b) for a, b in pose_ev) / max(len(pose_ev), 1)
    n_kp = d_n.cpu().numpy()
    inl = d_inl.cpu().numpy()

    total_frames = world * B * args.steps
    fps = total_frames / elapsed
    ms_per_step = elapsed / args.steps * 1e3

    sizes = level_sizes(ex.GetInverseScaleFactors())
    kp_mean = float(n_kp.mean())
    per_img = stage_bytes(sizes, kp_mean)
    bytes_per_frame = 2 * sum(per_img.values())  # 13.76 MB per stereo frame at 1000 kp
    stage_avg = {k: v / max(calls, 1) for k, v in stage_ms.items()}  # ms per pipeline launch
    stage_avg["pose_opt"] = pose_ms
    dom = max(stage_avg, key=stage_avg.get)
    imgs_per_launch = 2 * Bp
    prof = load_profile()
    pk = (prof or {}).get("stages", {})

    # headline roofline: the whole extractor pipeline's algorithmic bytes at the
    # measured frame rate against HBM peak (SURVEY §8(d) aggregate); traffic =
    # the PMC-measured HBM bytes of the extractor kernels per stereo frame
    achieved = bytes_per_frame * fps / 1e9
    traffic = None
    if all(k in pk and pk[k].get("hbm_bytes_per_image") is not None
           for k in ("resize", "blur", "fast_cells", "octree", "describe", "assemble")):
        traffic = round(2 * sum(pk[k]["hbm_bytes_per_image"]
                                for k in ("resize", "blur", "fast_cells", "octree", "describe",
                                          "assemble")))
    kernels = {}
    # In the mix the kernels of the four pipelines and the pose stream overlap,
    # so their event durations summed over a step exceed the step.  Each
    # kernel's in-mix figure is therefore its SHARE of the step: its event
    # duration scaled by ms_per_step / (sum over kernels of duration x
    # launches per step), so the shares of one step add up to ms_per_step.
    # The kernel's own roofline is isolated_frac (the launch alone, below).
    launches = {st: (G if st == "pose_opt" else G * P) for st in stage_avg}
    overlap = sum(stage_avg[st] * launches[st] for st in stage_avg) / ms_per_step
    for st, ms in stage_avg.items():
        b = per_img.get(st, 0) * imgs_per_launch if st != "pose_opt" else 0
        kname = STAGE_KERNELS[st]
        if st == "resize" and os.environ.get("ORBGPU_RESIZE") == "fused":
            kname = "k_pyramid"  # the chain as one launch (orb_api.cpp, opt-in)
        share = ms / overlap
        row = {"kernel": kname, "share_ms_per_launch": round(share, 5), "launches_per_step": launches[st],
               "algorithmic_bytes_per_launch": int(b)}
        if b:
            row["share_frac"] = round(b / (share * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
        if st == "describe":
            pf = describe_plane_floor(sizes, kp_mean) * imgs_per_launch
            row["plane_floor_bytes_per_launch"] = int(pf)
        p = pk.get(st)
        if p:
            if p.get("hbm_bytes_per_image") is not None and st != "pose_opt":
                row["traffic_per_launch"] = round(p["hbm_bytes_per_image"] * imgs_per_launch)
                if st == "describe":
                    row["traffic_over_plane_floor"] = round(row["traffic_per_launch"] /
                                                            row["plane_floor_bytes_per_launch"], 3)
            for key in ("valu_busy", "bound"):
                if p.get(key) is not None:
                    row[key] = p[key]
            # the same launch alone on the device (the PMC pass of tools/prof_stages.py,
            # kernels serialised): in the mix each kernel shares the CUs with the other
            # pipelines' and the pose stream's, so its duration there is not its speed
            iso = p.get("pmc_pass_ms_per_launch")
            if iso and prof.get("images_per_launch") == imgs_per_launch:
                row["isolated_ms_per_launch"] = iso
                if b:
                    row["isolated_GBs"] = round(b / (iso * 1e-3) / 1e9, 2)
                    row["isolated_frac"] = round(b / (iso * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                if st == "describe":
                    row["isolated_plane_floor_frac"] = round(
                        row["plane_floor_bytes_per_launch"] / (iso * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
            if p.get("insts_valu_per_launch") is not None and prof.get("images_per_launch"):
                row["valu_insts_per_64_images"] = round(p["insts_valu_per_launch"] * 64 /
                                                        prof["images_per_launch"])
        if st == "fast_cells":
            fs, fsrc = load_fast_stamps()
            if fs:  # minTh fallback cells (stamp counters 10/11, tools/stamps.py)
                row["fallback_cell_share"] = round(fs["fallback_frac"], 4)
                row["fallback_source"] = fsrc
        kernels[st] = row
    roofline = {
        "bound": "hbm",
        "scope": "extractor pipeline: SURVEY §8(d) algorithmic bytes per stereo frame x fps",
        "achieved": round(achieved, 2),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": traffic,
        "traffic_unit": "HBM bytes per stereo frame (PMC FETCH_SIZE x2 + WRITE_SIZE, profiles/"
                        f"{PROFILE_ROUND}/kernels.json)",
        "algorithmic_bytes_per_frame": int(bytes_per_frame),
        "kernels": kernels,
        "valu_busy_definition": "kernel SQ_INSTS_VALU per ns / the same counter per ns of a "
                                "VALU-saturating kernel (tools/valu_calib.hip), same box",
        "kernel_durations": f"share_ms_per_launch: the kernel's share of a step -- its HIP-event "
                            f"duration between the stages of all {P} pipelines' launches in the timed "
                            "mix (where it runs beside the other pipelines' kernels and the pose "
                            "stream's) scaled so that share x launches_per_step summed over the "
                            f"kernels equals ms_per_step (raw in-mix durations overlap {overlap:.2f}x); "
                            "share_frac: algorithmic bytes / share; isolated_ms_per_launch / "
                            "isolated_frac: the same launch alone on the device, the kernel's "
                            "roofline (PMC pass, profiles/" + PROFILE_ROUND + "/kernels.json)",
        "in_mix_overlap": round(overlap, 3),
    }
    result = {
        "metric": METRIC,
        "value": round(fps, 2),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "timed_region_s": round(elapsed, 3),
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
            "launch_groups_per_step": G,
            "parallelism": f"frames sharded over {world} GPU(s), no collective",
            "streams": f"{P} extractor pipelines ({2 * Bp} images per launch, own HIP stream) + "
                       f"pose kernel ({Bg} problems per launch) on a high-priority stream, all "
                       "concurrent",
            "keypoints_per_image_mean": float(n_kp.mean()),
            "pose_inliers_mean": float(inl.mean()),
        },
        "roofline": roofline,
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
    if rank == 0 and world == 1 and not args.no_lia:
        # SURVEY §8(f) rank 3 (LocalMapping after IMU initialisation), beside the
        # headline metric: LocalInertialBA window, GPU vs the CPU oracle (1 thread)
        sys.path.insert(0, str(REPO / "tools"))
        from bench_lba import measure_lia  # noqa: E402

        result["lia"] = measure_lia(calls=10, cpu_calls=0 if args.no_cpu_baseline else 3)
    if rank == 0 and world == 1 and not args.no_stereo:
        # SURVEY §8(f) rank 1, beside the headline metric (not part of it):
        # Frame::ComputeStereoMatches per frame on resident extractor outputs
        sys.path.insert(0, str(REPO / "tools"))
        from bench_stereo import measure as measure_stereo  # noqa: E402

        result["stereo"] = measure_stereo(frames=SIDE_BATCH, calls=20, cpu_frames=0 if args.no_cpu_baseline else 4)
    if rank == 0 and world == 1 and not args.no_match:
        # SURVEY §8(f) rank 2, beside the headline metric (not part of it):
        # SearchByProjection(CurrentFrame, LastFrame) on resident frame outputs
        sys.path.insert(0, str(REPO / "tools"))
        from bench_match import measure as measure_match  # noqa: E402

        result["match"] = measure_match(frames=SIDE_BATCH, calls=20, cpu_frames=0 if args.no_cpu_baseline else 4)
    if rank == 0 and world == 1 and not args.no_bow:
        # SURVEY §8(f) rank 4, beside the headline metric (not part of it):
        # DBoW2 transform (Frame::ComputeBoW) on resident extractor descriptors
        sys.path.insert(0, str(REPO / "tools"))
        from bench_bow import measure as measure_bow  # noqa: E402

        result["bow"] = measure_bow(frames=SIDE_BATCH, calls=20, cpu_frames=0 if args.no_cpu_baseline else 4)
    if rank == 0 and world == 1 and not args.no_inertial:
        # PoseInertialOptimizationLastFrame (stereo-inertial
        # tracking after IMU initialisation), a batch resident in HBM
        sys.path.insert(0, str(REPO / "tools"))
        from bench_inertial import measure as measure_inertial  # noqa: E402

        result["inertial"] = measure_inertial(problems=SIDE_BATCH, calls=20, mode=0,
                                              cpu_problems=0 if args.no_cpu_baseline else 4)
    if rank == 0 and world == 1 and not args.no_track:
        # config C3's path on synthetic data: extract + stereo + SearchByProjection
        # + PoseOptimization chained on the device, vs the oracle chain on the CPU
        sys.path.insert(0, str(REPO / "tools"))
        from bench_track import measure as measure_track  # noqa: E402

        result["track"] = measure_track(frames=SIDE_BATCH, calls=10, cpu_frames=0 if args.no_cpu_baseline else 4)
    if rank == 0 and world == 1 and not args.no_latency:
        # north_star's per-frame target: one stereo frame at a time through the
        # host ABI (2-thread extraction + PoseOptimization) vs the CPU oracle
        sys.path.insert(0, str(REPO / "tools"))
        from bench_latency import measure as measure_latency  # noqa: E402

        result["latency"] = measure_latency(frames=100, cpu_frames=0 if args.no_cpu_baseline else 8)
    if rank == 0 and world == 1 and not args.no_latency_inertial:
        # the same target in the mode EuRoC MH01 runs (stereo-inertial after IMU
        # initialisation): extract + stereo + SearchLocalPoints +
        # PoseInertialOptimizationLastFrame, one frame at a time through the ABI
        sys.path.insert(0, str(REPO / "tools"))
        from bench_latency_inertial import measure as measure_lat_in  # noqa: E402

        result["latency_inertial"] = measure_lat_in(frames=16, cpu_frames=0 if args.no_cpu_baseline else 4)
    if rank == 0 and world == 1 and not args.no_c5:
        # config C5's per-GPU unit on synthetic data: 8 sequences tracked frame to
        # frame (tools/c5_runner.py), frames/s of the GPU and the drift vs truth
        sys.path.insert(0, str(REPO / "tools"))
        import c5_runner  # noqa: E402

        c = c5_runner.SequenceChain(rank, 8, 110, local)
        c.reset()
        for t in range(10):
            c.frame(t)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for t in range(10, 110):
            c.frame(t)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        nm5, inl5 = c.stats()
        result["c5"] = {"workload": "8 synthetic stereo sequences on this GPU, each tracked frame to "
                                    "frame (extract, stereo, SearchByProjection at the motion-model "
                                    "pose, PoseOptimization, UnprojectStereo), 100 timed frames",
                        "gpu_fps": round(8 * 100 / el, 1), "ms_per_frame_per_seq": round(el / 100 * 1e3, 3),
                        "matches_per_frame": round(nm5, 1), "pose_inliers_per_frame": round(inl5, 1),
                        "ate_m": c.ate()}
        del c
    if rank == 0 and world == 1 and not args.no_lba_sharded:
        sys.path.insert(0, str(REPO / "tools"))
        from bench_lba import measure_sharded  # noqa: E402

        result["lba_sharded"] = measure_sharded(calls=10)
    if rank == 0:
        print(json.dumps(result), flush=True)
    dist.finalize()
    return 0


if __name__ == "__main__":
    sys.exit(main())
