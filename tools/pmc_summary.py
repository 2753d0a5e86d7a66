"""Per-kernel, per-dispatch averages of the counters collected by
tools/pmc_run.sh (all pass*_counter_collection.csv under a directory).

    python tools/pmc_summary.py gpurun_out/pmc [--json out.json]

FETCH_SIZE is doubled (gfx950 reports half the bytes of wide reads,
MI355X_MICROARCH.md HBM section); SQ_*CYCLES / SQ_WAIT_* / SQ_ACTIVE_* are in
quad-cycles.
"""
import csv
import glob
import json
import sys
from collections import defaultdict


def load(d):
    acc = defaultdict(lambda: defaultdict(float))  # kernel -> counter -> sum
    disp = defaultdict(lambda: defaultdict(set))   # kernel -> counter -> dispatch ids
    for f in sorted(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").split("::")[-1]
            c = r["Counter_Name"]
            acc[k][c] += float(r["Counter_Value"])
            disp[k][c].add((f, r["Dispatch_Id"]))
    out = {}
    for k, cs in acc.items():
        out[k] = {c: v / max(1, len(disp[k][c])) for c, v in cs.items()}
        if "FETCH_SIZE" in out[k]:
            out[k]["FETCH_BYTES"] = out[k]["FETCH_SIZE"] * 1024 * 2  # KB, x2 gfx950
        if "WRITE_SIZE" in out[k]:
            out[k]["WRITE_BYTES"] = out[k]["WRITE_SIZE"] * 1024
    return out


def main():
    d = sys.argv[1]
    out = load(d)
    for k in sorted(out, key=lambda k: -out[k].get("SQ_WAVE_CYCLES", 0)):
        c = out[k]
        w = max(c.get("SQ_WAVES", 1), 1)
        line = f"{k[:22]:22s} waves={w:9.0f}"
        for name, key in (("valu/w", "SQ_INSTS_VALU"), ("lds/w", "SQ_INSTS_LDS"), ("salu/w", "SQ_INSTS_SALU"),
                          ("vmem/w", "SQ_INSTS_VMEM")):
            if key in c:
                line += f" {name}={c[key] / w:8.1f}"
        wc = c.get("SQ_WAVE_CYCLES")
        if wc:
            line += f" cyc/w={4 * wc / w:8.0f}"
            for name, key in (("valu%", "SQ_ACTIVE_INST_VALU"), ("lds%", "SQ_ACTIVE_INST_LDS"),
                              ("wait%", "SQ_WAIT_ANY"), ("waitinst%", "SQ_WAIT_INST_ANY"),
                              ("any%", "SQ_ACTIVE_INST_ANY")):
                if key in c:
                    line += f" {name}={100 * c[key] / wc:5.1f}"
        if "SQ_LDS_BANK_CONFLICT" in c:
            line += f" ldsconf={c['SQ_LDS_BANK_CONFLICT']:.0f}"
        if "FETCH_BYTES" in c:
            line += f" fetchMB={c['FETCH_BYTES'] / 1e6:8.2f}"
        if "WRITE_BYTES" in c:
            line += f" writeMB={c['WRITE_BYTES'] / 1e6:8.2f}"
        print(line)
    if "--json" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
