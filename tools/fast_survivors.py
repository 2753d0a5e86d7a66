"""Fraction of FAST compass survivors that are FAST-9 corners (CPU, numpy).

VERDICT r4 item 4 asks for it before choosing a cheaper corner test: the
4-point compass pre-test of `k_fast_cells` passes a pixel when
max(v - max(min(u,d), min(l,r)), min(max(u,d), max(l,r)) - v) > th, and every
survivor is then scored by the full 16-pixel arc test.  This counts, over the
bench's synthetic frames and the oracle's pyramid (orb_extractor.cc:1093-1117
levels, detection area = the level minus the 19-px edge band), how many pixels
survive the compass and how many of those are corners (9 contiguous ring
pixels all > v + th or all < v - th; orb_extractor.cc:783-801 via FAST_t<16>).

    python tools/fast_survivors.py [frames] > profiles/r05/fast_survivors.json
"""
import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))

CX = [0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1]
CY = [3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3]
EDGE = 19


def level_counts(img, th):
    im = img.astype(np.int16)
    h, w = im.shape
    y0, y1, x0, x1 = EDGE, h - EDGE, EDGE, w - EDGE
    if y1 <= y0 or x1 <= x0:
        return 0, 0, 0
    v = im[y0:y1, x0:x1]
    ring = np.stack([im[y0 + dy:y1 + dy, x0 + dx:x1 + dx] for dx, dy in zip(CX, CY)])
    u, r, d, l = ring[0], ring[4], ring[8], ring[12]
    lo = np.maximum(np.minimum(u, d), np.minimum(l, r))
    hi = np.minimum(np.maximum(u, d), np.maximum(l, r))
    comp = np.maximum(v - lo, hi - v) > th
    br = ring > v + th
    dk = ring < v - th
    corner = np.zeros_like(comp)
    for k in range(16):
        idx = [(k + j) & 15 for j in range(9)]
        corner |= br[idx].all(0) | dk[idx].all(0)
    assert not (corner & ~comp).any()  # the compass never drops a corner
    return v.size, int(comp.sum()), int(corner.sum())


def main():
    from oracle.binding import OracleExtractor
    from orb_slam_fusion_amd import synth

    frames = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    ex = OracleExtractor(1000, 1.2, 8, 20, 7)
    tot = np.zeros((8, 3), np.int64)
    for f in range(frames):
        for img in synth.stereo_frame(f):
            for lev, pl in enumerate(ex.pyramid(img)):
                tot[lev] += level_counts(pl, 20)
    per = [{"level": l, "pixels": int(t[0]), "survivor_rate": round(t[1] / t[0], 4),
            "corner_rate": round(t[2] / t[0], 4), "corners_per_survivor": round(t[2] / max(t[1], 1), 4)}
           for l, t in enumerate(tot)]
    a = tot.sum(0)
    print(json.dumps({"frames": frames, "images": 2 * frames, "th": 20,
                      "survivor_rate": round(a[1] / a[0], 4), "corner_rate": round(a[2] / a[0], 4),
                      "corners_per_survivor": round(a[2] / a[1], 4), "levels": per}, indent=1))


if __name__ == "__main__":
    main()
