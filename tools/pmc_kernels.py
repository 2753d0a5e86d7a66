"""Reduce one round's rocprofv3 evidence to profiles/<round>/kernels.json, the
file bench.py's roofline block reads (tools/profile_round.sh runs this).

Inputs (directories of rocprofv3 csv output):
  --traffic DIR   FETCH_SIZE and WRITE_SIZE in separate --pmc passes over
                  tools/prof_stages.py (one launch = 64 images / 32 pose problems)
  --sq DIR        SQ_INSTS_VALU (+ wave counters) over the same workload
  --calib DIR     the same SQ counters over build/valu_calib (VALU-saturating kernel)
  --stats CSV     rocprofv3 --kernel-trace --stats of the bench command itself

Per extractor stage (resize = its 7 level launches per call):
  hbm_bytes_per_image  = (2 x FETCH_SIZE + WRITE_SIZE) per launch / images per launch
                         (FETCH_SIZE doubled: gfx950 reports half the bytes of wide
                         reads, MI355X_MICROARCH.md HBM section; both in KB)
  valu_busy            = (SQ_INSTS_VALU / kernel ns) / (the same for k_valu_sat):
                         the kernel's wave64-VALU issue rate as a fraction of the
                         rate a VALU-saturating kernel reaches on the same box
  rocprof_avg_ms_per_launch = kernel-stats average duration x dispatches per launch
"""
import argparse
import csv
import glob
import json
from collections import defaultdict

STAGES = {"resize": ("k_resize", 7), "blur": ("k_blur", 1), "fast_cells": ("k_fast_cells", 1),
          "octree": ("k_octree", 1), "describe": ("k_describe", 1), "assemble": ("k_assemble", 1),
          "pose_opt": ("k_pose_opt", 1)}


def short(name: str) -> str:
    return name.split("(")[0].replace("void ", "").split("::")[-1].split("<")[0].strip('"')


def counters(d: str):
    """-> {kernel: {counter: (sum over dispatches, n dispatches, sum of ns)}}"""
    acc = defaultdict(lambda: defaultdict(lambda: [0.0, set(), 0.0]))
    for f in sorted(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            k, c = short(r["Kernel_Name"]), r["Counter_Name"]
            a = acc[k][c]
            key = (f, r["Dispatch_Id"])
            a[0] += float(r["Counter_Value"])
            if key not in a[1]:
                a[1].add(key)
                a[2] += float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    return {k: {c: (v[0], len(v[1]), v[2]) for c, v in cs.items()} for k, cs in acc.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--traffic")
    ap.add_argument("--sq")
    ap.add_argument("--calib")
    ap.add_argument("--stats")
    ap.add_argument("--images-per-launch", type=int, default=64)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    out = {"images_per_launch": a.images_per_launch, "stages": {}}
    calib_rate = None
    if a.calib:
        cc = counters(a.calib)
        rates = {}
        for k in ("k_valu_sat", "k_valu_int"):
            if k in cc and "SQ_INSTS_VALU" in cc[k]:
                s, n, ns = cc[k]["SQ_INSTS_VALU"]
                rates[k] = s / ns
        out["calib"] = {"insts_valu_per_ns": rates,
                        "kernel": "tools/valu_calib.hip k_valu_sat (8 waves/SIMD, 8 independent "
                                  "v_fma_f32 chains per lane)"}
        calib_rate = rates.get("k_valu_sat")
    tr = counters(a.traffic) if a.traffic else {}
    sq = counters(a.sq) if a.sq else {}
    stats = {}
    if a.stats:
        for r in csv.DictReader(open(a.stats)):
            stats[short(r["Name"])] = (float(r["AverageNs"]), int(r["Calls"]))
    for st, (kname, per) in STAGES.items():
        if st == "resize" and any("k_pyramid" in src for src in (tr, sq, stats)):
            kname, per = "k_pyramid", 1  # the chain as one launch (batches that fill the device)
        row = {"kernel": kname, "dispatches_per_launch": per}
        t = tr.get(kname, {})
        if "FETCH_SIZE" in t and "WRITE_SIZE" in t:
            f_sum, f_n, _ = t["FETCH_SIZE"]
            w_sum, w_n, _ = t["WRITE_SIZE"]
            fetch = 2 * 1024 * f_sum / (f_n / per)
            write = 1024 * w_sum / (w_n / per)
            row["fetch_bytes_per_launch"] = round(fetch)
            row["write_bytes_per_launch"] = round(write)
            if st != "pose_opt":
                row["hbm_bytes_per_image"] = round((fetch + write) / a.images_per_launch, 1)
        q = sq.get(kname, {})
        if "SQ_INSTS_VALU" in q:
            s, n, ns = q["SQ_INSTS_VALU"]
            row["insts_valu_per_launch"] = round(s / (n / per))
            row["pmc_pass_ms_per_launch"] = round(ns / (n / per) / 1e6, 5)
            if calib_rate:
                row["valu_busy"] = round((s / ns) / calib_rate, 3)
        if kname in stats:
            avg, calls = stats[kname]
            row["rocprof_avg_ms_per_launch"] = round(avg * per / 1e6, 5)
            row["rocprof_dispatches"] = calls
        out["stages"][st] = row
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
