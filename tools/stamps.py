"""Per-phase cycle totals from the ORB_STAMPS build (make stamps).

    ORBGPU_LIB=orb_slam_fusion_amd/lib/liborbgpu_stamps.so python tools/stamps.py
"""
import ctypes
import json
import os
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))


def main():
    import torch

    from orb_slam_fusion_amd import OrbExtractor, synth
    from orb_slam_fusion_amd._lib import library_path

    B = int(os.environ.get("FRAMES", "64"))
    iters = int(os.environ.get("ITERS", "5"))
    imgs = np.stack([im for i in range(B) for im in synth.stereo_frame(i)])
    d_imgs = torch.from_numpy(imgs).cuda()
    ex = OrbExtractor(1000, 1.2, 8, 20, 7, max_images=2 * B)
    cap = ex.max_keypoints(752, 480)
    kps = torch.zeros((2 * B, cap, 7), dtype=torch.int32, device="cuda")
    desc = torch.zeros((2 * B, cap, 32), dtype=torch.uint8, device="cuda")
    n = torch.zeros(2 * B, dtype=torch.int32, device="cuda")
    mono = torch.zeros(2 * B, dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream()
    lib = ctypes.CDLL(str(library_path()))
    buf = (ctypes.c_ulonglong * 16)()
    ex.extract_batch(d_imgs, kps, desc, n, mono, stream=s)
    torch.cuda.synchronize()
    lib.orbgpu_debug_stamps(buf, 16)
    for _ in range(iters):
        ex.extract_batch(d_imgs, kps, desc, n, mono, stream=s)
    torch.cuda.synchronize()
    assert lib.orbgpu_debug_stamps(buf, 16) == 0
    v = list(buf)
    cells = max(v[13], 1)
    tot = sum(v[i] for i in range(10))
    out = {"cells": cells / iters, "fallback_frac": v[10] / cells, "n_lo_per_cell": v[11] / cells,
           "n_hi_per_cell": v[12] / cells, "nd_per_cell": v[14] / cells,
           "ticks_per_cell": round(tot / cells, 1),
           "share": {f"p{i}": round(v[i] / max(tot, 1), 3) for i in range(10)},
           }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
