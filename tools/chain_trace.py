"""Where one frame's latency goes: a rocprofv3 --kernel-trace (+ optional
--memory-copy-trace) CSV of build/latency, split into per-image extractor
chains (k_resize ... k_assemble on one queue) and pose launches.  Prints, as
JSON: per kernel of the chain the median duration and the median gap before
it (previous kernel's end -> its start, same queue), the chain span (first
kernel start -> last kernel end), the pose kernel's duration, and the copies.

    python tools/chain_trace.py KERNEL_TRACE.csv [--copies MEMORY_COPY_TRACE.csv]
"""
import argparse
import csv
import json
import re
import statistics
from collections import defaultdict


def short(name: str) -> str:
    m = re.search(r"(k_\w+)", name)
    return m.group(1) if m else name[:40]


def med(v):
    return round(statistics.median(v) / 1e3, 2) if v else None  # ns -> us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--copies")
    ap.add_argument("--skip", type=int, default=5, help="chains per queue to drop (warm-up)")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    qkey = "Queue_Id" if rows and "Queue_Id" in rows[0] else ("Stream_Id" if rows and "Stream_Id" in rows[0] else None)
    by_q = defaultdict(list)
    for r in rows:
        by_q[r.get(qkey, 0) if qkey else 0].append(
            (int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    chains, pose = [], []
    for q, ev in by_q.items():
        ev.sort()
        cur = []
        for e in ev:
            if e[2] in ("k_pose_opt", "k_pose_single") or e[2].startswith("k_pose"):
                pose.append(e[1] - e[0])
                continue
            if e[2] == "k_resize" and cur and cur[-1][2] != "k_resize":
                chains.append(cur)
                cur = []
            cur.append(e)
            if e[2] == "k_assemble":
                chains.append(cur)
                cur = []
        chains = [c for c in chains if c and c[-1][2] == "k_assemble"]
    n_skip = a.skip * max(1, len(by_q))
    chains = chains[n_skip:]
    per_pos = defaultdict(lambda: {"dur": [], "gap": []})
    spans = []
    for c in chains:
        spans.append(c[-1][1] - c[0][0])
        for i, (s, e, n) in enumerate(c):
            key = f"{i:02d}_{n}"
            per_pos[key]["dur"].append(e - s)
            if i:
                per_pos[key]["gap"].append(s - c[i - 1][1])
    out = {
        "chains": len(chains),
        "chain_span_us_median": med(spans),
        "chain_kernel_sum_us_median": med([sum(e - s for s, e, _ in c) for c in chains]),
        "kernels": {k: {"dur_us": med(v["dur"]), "gap_before_us": med(v["gap"])} for k, v in sorted(per_pos.items())},
        "pose_kernel_us_median": med(pose),
        "pose_launches": len(pose),
    }
    if a.copies:
        cr = list(csv.DictReader(open(a.copies)))
        kinds = defaultdict(list)
        for r in cr:
            k = r.get("Direction") or r.get("Operation") or r.get("Kind") or "copy"
            kinds[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        out["copies_us_median"] = {k: med(v) for k, v in kinds.items()}
        out["copies_count"] = {k: len(v) for k, v in kinds.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
