"""Reduce the FETCH_SIZE / WRITE_SIZE passes of tools/pmc_traffic.sh to HBM
bytes per extractor-stage launch -> JSON {stage: bytes}.

FETCH_SIZE and WRITE_SIZE are kilobytes; FETCH_SIZE is doubled (gfx950 reports
half the bytes of wide reads, MI355X_MICROARCH.md HBM section).  A stage's
launch is the sum of its kernels per extract call (resize = its 7 level
launches).
"""
import csv
import glob
import json
import sys
from collections import defaultdict

STAGE_OF = {"k_resize": "resize", "k_blur": "blur", "k_fast_cells": "fast_cells",
            "k_octree": "octree", "k_describe": "describe", "k_assemble": "assemble"}


def main():
    d, out = sys.argv[1], sys.argv[2]
    tot = defaultdict(float)   # (counter, stage) -> KB summed over dispatches
    calls = defaultdict(int)   # (counter, stage) -> dispatches of the stage's first kernel
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].split("::")[-1]
            st = STAGE_OF.get(k)
            if st is None:
                continue
            c = r["Counter_Name"]
            tot[(c, st)] += float(r["Counter_Value"])
            calls[(c, st)] += 1
    res = {}
    for st in STAGE_OF.values():
        per = 7 if st == "resize" else 1  # level launches per call
        f_calls = calls.get(("FETCH_SIZE", st), 0) / per
        w_calls = calls.get(("WRITE_SIZE", st), 0) / per
        if not f_calls or not w_calls:
            continue
        fetch = 2 * 1024 * tot[("FETCH_SIZE", st)] / f_calls
        write = 1024 * tot[("WRITE_SIZE", st)] / w_calls
        res[st] = round(fetch + write)
        res[st + "_detail"] = {"fetch_bytes": round(fetch), "write_bytes": round(write),
                               "images_per_launch": 64}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
