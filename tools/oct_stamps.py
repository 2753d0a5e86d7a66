"""Octree phase shares from the ORB_STAMPS build.
    ORBGPU_LIB=orb_slam_fusion_amd/lib/liborbgpu_stamps.so python tools/oct_stamps.py
"""
import ctypes
import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))


def main():
    import torch

    from orb_slam_fusion_amd import OrbExtractor, synth
    from orb_slam_fusion_amd._lib import library_path

    B = 64
    imgs = np.stack([im for i in range(B) for im in synth.stereo_frame(i)])
    d = torch.from_numpy(imgs).cuda()
    ex = OrbExtractor(1000, 1.2, 8, 20, 7, max_images=2 * B)
    cap = ex.max_keypoints(752, 480)
    kps = torch.zeros((2 * B, cap, 7), dtype=torch.int32, device="cuda")
    desc = torch.zeros((2 * B, cap, 32), dtype=torch.uint8, device="cuda")
    n = torch.zeros(2 * B, dtype=torch.int32, device="cuda")
    mono = torch.zeros(2 * B, dtype=torch.int32, device="cuda")
    lib = ctypes.CDLL(str(library_path()))
    buf = (ctypes.c_ulonglong * 16)()
    ex.extract_batch(d, kps, desc, n, mono, stream=0)
    torch.cuda.synchronize()
    lib.orbgpu_debug_stamps(buf, 16)
    ex.extract_batch(d, kps, desc, n, mono, stream=0)
    torch.cuda.synchronize()
    lib.orbgpu_debug_stamps(buf, 16)
    v = list(buf)
    blocks = v[10] + v[11]
    tot = sum(v[:10])
    print(json.dumps({"blocks": blocks, "ticks_per_block": tot / max(blocks, 1),
                      "level0_ticks_per_block": v[14] / max(v[11], 1),
                      "rounds_phase1_per_block": v[12] / max(blocks, 1),
                      "rounds_phase2_per_block": v[13] / max(blocks, 1),
                      "share": {k: round(v[i] / max(tot, 1), 3)
                                for i, k in enumerate(["gather", "roots", "r_choose", "output", "r_count",
                                                       "r_pc", "r_cut", "r_scans", "r_build",
                                                       "r_reassign_copy"])}}))


if __name__ == "__main__":
    main()
