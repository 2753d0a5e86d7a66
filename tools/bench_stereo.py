"""Frame::ComputeStereoMatches timing: orbgpu_stereo_match_batch over the
frames of one extract_batch call (B synthetic 752x480 rectified pairs, the
bench's C2 extractor config), per frame, HIP events on the launch stream;
beside it the CPU oracle per frame (one core) on a few of the same frames.

    python tools/bench_stereo.py [--frames 64] [--calls 20]
"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))

FX, BASE = 435.2, 0.11


def measure(frames: int = 64, calls: int = 20, cpu_frames: int = 4) -> dict:
    import torch

    # every allocation, copy and launch on one non-default stream
    with torch.cuda.stream(torch.cuda.Stream()):
        return _measure(frames, calls, cpu_frames)


def _measure(frames: int, calls: int, cpu_frames: int) -> dict:
    import torch

    from orb_slam_fusion_amd import OrbExtractor, synth

    B = frames
    pairs = [synth.stereo_frame(i) for i in range(B)]
    imgs = torch.from_numpy(np.stack([im for p in pairs for im in p])).cuda()
    ex = OrbExtractor(1000, 1.2, 8, 20, 7, max_images=2 * B)
    cap = ex.max_keypoints(752, 480)
    kps = torch.zeros((2 * B, cap, 7), dtype=torch.int32, device="cuda")
    desc = torch.zeros((2 * B, cap, 32), dtype=torch.uint8, device="cuda")
    n = torch.zeros(2 * B, dtype=torch.int32, device="cuda")
    mono = torch.zeros(2 * B, dtype=torch.int32, device="cuda")
    ur = torch.zeros((B, cap), dtype=torch.float32, device="cuda")
    dep = torch.zeros((B, cap), dtype=torch.float32, device="cuda")
    bf = np.float32(FX * BASE)
    mb = np.float32(bf / np.float32(FX))
    s = torch.cuda.current_stream()
    ex.extract_batch(imgs, kps, desc, n, mono, stream=s)
    for _ in range(3):
        ex.stereo_match_batch(imgs, kps, desc, n, bf, mb, ur, dep, stream=s)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(calls):
        ex.stereo_match_batch(imgs, kps, desc, n, bf, mb, ur, dep, stream=s)
    e1.record(s)
    torch.cuda.synchronize()
    gpu_ms = e0.elapsed_time(e1) / calls
    matched = int((ur >= 0).sum().item())
    out = {"workload": f"Frame::ComputeStereoMatches, {B} synthetic 752x480 rectified pairs per batch "
                       "(C2 extractor outputs resident in HBM), bf = 435.2 * 0.11",
           "gpu_ms_per_batch": round(gpu_ms, 4), "gpu_us_per_frame": round(gpu_ms / B * 1e3, 3),
           "matched_per_frame": round(matched / B, 1)}
    if cpu_frames > 0:
        sys.path.insert(0, str(REPO / "oracle"))
        import binding as oracle  # cpu baseline leg only

        work = []
        for left, right in pairs[:cpu_frames]:
            exl, exr = oracle.OracleExtractor(1000, 1.2, 8, 20, 7), oracle.OracleExtractor(1000, 1.2, 8, 20, 7)
            _, kl, dl = exl.extract(left)
            _, kr, dr = exr.extract(right)
            work.append((kl, dl, kr, dr, [exl.level(l) for l in range(8)], [exr.level(l) for l in range(8)],
                         exl.params()))
        t0 = time.perf_counter()
        reps = 5
        for _ in range(reps):
            for kl, dl, kr, dr, pl, pr, p in work:
                oracle.stereo_match(kl, dl, kr, dr, pl, pr, p["scale"], p["inv_scale"], bf, mb)
        out["cpu_oracle_us_per_frame"] = round((time.perf_counter() - t0) / (reps * len(work)) * 1e6, 1)
        out["cpu_cores"] = 1
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--calls", type=int, default=20)
    a = ap.parse_args()
    print(json.dumps(measure(a.frames, a.calls)))
