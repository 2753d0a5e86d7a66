"""Print a rocprofv3 kernel_stats.csv as a compact table (avg/min/max µs)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    name = r["Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")[:48]
    print(f"{name:48s} calls={int(r['Calls']):5d} avg={float(r['AverageNs'])/1e3:9.1f}us "
          f"min={float(r['MinNs'])/1e3:9.1f} max={float(r['MaxNs'])/1e3:9.1f} {float(r['Percentage']):5.1f}%")
