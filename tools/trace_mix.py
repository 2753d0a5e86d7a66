"""Concurrency profile of a rocprofv3 --kernel-trace CSV (the bench mix):
over the window of the last --count dispatches of --anchor, the time each kernel runs, the time it runs
ALONE (no other kernel in flight), and the share of time with k kernels
in flight.

    python tools/trace_mix.py gpurun_out/trace/trace_kernel_trace.csv [--count 120]
"""
import argparse
import csv
import re
from collections import defaultdict


def short(name: str) -> str:
    m = re.search(r"(k_\w+)", name)
    return m.group(1) if m else name[:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--anchor", default="k_fast_cells",
                    help="window = the last --count dispatches of this kernel")
    ap.add_argument("--count", type=int, default=120)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows]
    anc = sorted((s, e) for s, e, n in ev if n == a.anchor)[-a.count:]
    t0, t_end = anc[0][0], anc[-1][1]
    ev = [(max(s, t0), min(e, t_end), n) for s, e, n in ev if e > t0 and s < t_end]
    pts = sorted([(s, 1, n) for s, e, n in ev] + [(e, -1, n) for s, e, n in ev])
    busy = defaultdict(float)
    alone = defaultdict(float)
    conc = defaultdict(float)
    active = defaultdict(int)
    last = t0
    for t, d, n in pts:
        dt = t - last
        k = sum(active.values())
        conc[k] += dt
        for name, c in active.items():
            if c:
                busy[name] += dt
        if k == 1:
            (only,) = [x for x, c in active.items() if c]
            alone[only] += dt
        active[n] += d
        last = t
    span = t_end - t0
    print(f"span {span / 1e6:.2f} ms")
    for k in sorted(conc):
        print(f"  {k} kernels in flight: {conc[k] / span:.3f}")
    for n in sorted(busy, key=lambda x: -busy[x]):
        print(f"  {n:24s} busy {busy[n] / span:.3f}  alone {alone[n] / span:.3f}")


if __name__ == "__main__":
    main()
