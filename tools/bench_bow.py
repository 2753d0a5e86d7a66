"""DBoW2 transform timing (Frame::ComputeBoW, frame.cc:761-766:
transform(mDescriptors, mBowVec, mFeatVec, 4)) on a vocabulary of ORB-SLAM's
shape (k = 10, L = 6, L1_NORM, TF_IDF; synthetic, written in ORBvoc.txt text
format: the real vocabulary is not shipped).  B frames' descriptors come from
the GPU extractor on synthetic 752x480 images and stay in HBM;
orbgpu_bow_transform_batch is timed with HIP events on the launch stream.
Beside it: the vocabulary load time (text parse + upload), the CPU oracle per
frame on one core, and a bit-exact check against it on those frames.

    python tools/bench_bow.py [--frames 64] [--calls 20] [--L 6]
"""
import argparse
import json
import os
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))


def measure(frames: int = 64, calls: int = 20, cpu_frames: int = 4, L: int = 6) -> dict:
    import torch

    with torch.cuda.stream(torch.cuda.Stream()):
        return _measure(frames, calls, cpu_frames, L)


def _measure(frames, calls, cpu_frames, L):
    import torch

    from orb_slam_fusion_amd import OrbExtractor, synth
    from orb_slam_fusion_amd.vocab import ORBVocabulary

    tmp = tempfile.mkdtemp(prefix="orbvoc_")
    path = os.path.join(tmp, "voc.txt")
    nodes = synth.vocab_text(path, seed=3, k=10, L=L)
    t0 = time.perf_counter()
    V = ORBVocabulary()
    assert V.loadFromTextFile(path)
    load_s = time.perf_counter() - t0
    B = frames
    dev = torch.device("cuda", 0)
    imgs = torch.from_numpy(np.stack([synth.stereo_frame(i)[0] for i in range(B)])).to(dev)
    ex = OrbExtractor(1000, 1.2, 8, 20, 7, max_images=B)
    cap = ex.max_keypoints(752, 480)
    kps = torch.zeros((B, cap, 7), dtype=torch.int32, device=dev)
    desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device=dev)
    n = torch.zeros(B, dtype=torch.int32, device=dev)
    mono = torch.zeros(B, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream()
    ex.extract_batch(imgs, kps, desc, n, mono, stream=s)
    bw = torch.zeros((B, cap), dtype=torch.int32, device=dev)
    bwt = torch.zeros((B, cap), dtype=torch.float64, device=dev)
    fn = torch.zeros((B, cap), dtype=torch.int32, device=dev)
    fo = torch.zeros((B, cap + 1), dtype=torch.int32, device=dev)
    ff = torch.zeros((B, cap), dtype=torch.int32, device=dev)
    nw = torch.zeros(B, dtype=torch.int32, device=dev)
    nn = torch.zeros(B, dtype=torch.int32, device=dev)

    def run():
        V.transform_batch(desc, n, 4, bw, bwt, nw, fn, fo, ff, nn, stream=s)

    for _ in range(3):
        run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(calls):
        run()
    e1.record(s)
    torch.cuda.synchronize()
    gpu_ms = e0.elapsed_time(e1) / calls
    out = {"workload": f"DBoW2 transform(desc, BowVector, FeatureVector, 4), vocabulary k=10 L={L} "
                       f"({nodes + 1} nodes, synthetic ORBvoc.txt format, L1_NORM / TF_IDF); {B} "
                       "frames of 752x480 extractor descriptors resident in HBM",
           "gpu_ms_per_batch": round(gpu_ms, 4), "gpu_us_per_frame": round(gpu_ms / B * 1e3, 3),
           "words_per_frame": round(float(nw.float().mean().item()), 1),
           "vocab_load_s": round(load_s, 2)}
    if cpu_frames > 0:
        sys.path.insert(0, str(REPO / "oracle"))
        import binding as oracle  # cpu baseline / checker leg only

        O = oracle.OracleVocab(path)
        d_h, n_h = desc.cpu().numpy(), n.cpu().numpy()
        g = [x.cpu().numpy() for x in (bw, bwt, nw, fn, fo, ff, nn)]
        exact, work = True, []
        for f in range(min(cpu_frames, B)):
            feats = d_h[f, :n_h[f]]
            ow, owt, onn, ofo, off = O.transform(feats, 4)
            k, j = int(g[2][f]), int(g[6][f])
            exact &= (g[0][f, :k].astype(np.uint32).tobytes() == ow.tobytes() and
                      g[1][f, :k].tobytes() == owt.tobytes() and
                      g[3][f, :j].astype(np.uint32).tobytes() == onn.tobytes() and
                      g[4][f, :j + 1].tobytes() == ofo.tobytes() and
                      g[5][f, :g[4][f, j]].astype(np.uint32).tobytes() == off.tobytes())
            work.append(feats)
        reps = 3
        t0 = time.perf_counter()
        for _ in range(reps):
            for feats in work:
                O.transform(feats, 4)
        out["cpu_oracle_us_per_frame"] = round((time.perf_counter() - t0) / (reps * len(work)) * 1e6, 1)
        out["cpu_cores"] = 1
        out["bit_exact_vs_oracle"] = bool(exact)
        del O
    V.close()
    try:
        os.remove(path)
        os.rmdir(tmp)
    except OSError:
        pass
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--calls", type=int, default=20)
    ap.add_argument("--L", type=int, default=6)
    a = ap.parse_args()
    print(json.dumps(measure(a.frames, a.calls, L=a.L)))
