"""Per-launch durations of one extract call from a rocprofv3 kernel trace:
    python tools/klevels.py gpurun_out/kt/kt_kernel_trace.csv"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
seq = sorted(((r["Kernel_Name"].split("(")[0].split("::")[-1], int(r["Start_Timestamp"]),
               int(r["End_Timestamp"])) for r in rows), key=lambda t: t[1])
names = [s[0] for s in seq]
first = max(i for i, n in enumerate(names) if n == "k_resize" and (i == 0 or names[i - 1] != "k_resize"))
t0 = seq[first][1]
for n, a, b in seq[first:first + 14]:
    print(f"{n:14s} {(b - a) / 1000:8.1f} us  start {(a - t0) / 1000:8.1f}")
