"""Timeline of one single-image dataflow launch (k_extract_df): with
ORBGPU_DF_TRACE set, every worker stamps each ticket (s_memrealtime, 100 MHz:
grab, ready = dependencies met, done = published) and the assembly's start /
end.  Prints per stage (type, level) the first grab, last done, mean wait and
mean body time in µs from the first grab, and the chain that ends the launch.

    ORBGPU_DF_TRACE=1 python tools/df_trace.py [--runs 20] [--frame 3]
"""
import argparse
import ctypes
import json
import os
import sys
from collections import defaultdict
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))

TYPES = ["copy", "resize", "fast", "blur", "octree", "describe", "mirror"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=20)
    ap.add_argument("--frame", type=int, default=3)
    a = ap.parse_args()
    os.environ.setdefault("ORBGPU_DF_TRACE", "1")
    from orb_slam_fusion_amd import OrbExtractor, synth
    from orb_slam_fusion_amd._lib import lib

    so = lib()
    fn = so.orbgpu_debug_df_trace
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    img, _ = synth.stereo_frame(a.frame)
    ex = OrbExtractor(1000, 1.2, 8, 20, 7)
    cap = 1 << 16
    buf = np.zeros(4 * cap + 2, np.uint64)
    spans, per_run = [], []
    for r in range(a.runs):
        ex(img)
        n = fn(ex._h, buf.ctypes.data, cap)
        if n <= 0:
            raise SystemExit("no trace (ORBGPU_DF_TRACE unset or graph path)")
        rec = buf[:4 * n].reshape(n, 4).astype(np.int64)
        t0 = int(rec[:, 0].min())
        asm0, asm1 = int(buf[4 * n]) - t0, int(buf[4 * n + 1]) - t0
        spans.append(asm1 * 0.01)
        per_run.append((rec, t0, asm0, asm1))
    rec, t0, asm0, asm1 = per_run[int(np.argsort(spans)[len(spans) // 2])]  # the median run
    us = lambda v: round(v * 0.01, 2)  # noqa: E731  (100 MHz ticks)
    stages = defaultdict(lambda: {"n": 0, "grab": 1 << 62, "ready_first": 1 << 62, "done": 0, "wait": 0, "body": 0})
    xccs = defaultdict(int)
    for g, rd, dn, meta in rec:
        it = int(meta) & 0xffffffff
        typ, lev = it & 15, (it >> 4) & 15
        s = stages[(TYPES[typ], lev)]
        s["n"] += 1
        s["grab"] = min(s["grab"], g - t0)
        s["ready_first"] = min(s["ready_first"], rd - t0)
        s["done"] = max(s["done"], dn - t0)
        s["wait"] += rd - g
        s["body"] += dn - rd
        xccs[(int(meta) >> 60) & 15] += 1
    out = {"runs": a.runs, "span_us_median": round(float(np.median(spans)), 2),
           "span_us_min": round(float(np.min(spans)), 2),
           "assembly_us": [us(asm0), us(asm1)], "items_per_xcc": dict(sorted(xccs.items())), "stages": {}}
    for (typ, lev), s in sorted(stages.items(), key=lambda kv: kv[1]["done"]):
        out["stages"][f"{typ}{lev}"] = {"items": s["n"], "first_grab": us(s["grab"]),
                                         "first_ready": us(s["ready_first"]), "last_done": us(s["done"]),
                                         "mean_wait": us(s["wait"] / s["n"]), "mean_body": us(s["body"] / s["n"])}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
