"""Per-basic-block instruction counts of one kernel in a hipcc -S listing
(VALU counts quarter-rate 32-bit multiplies as 4):
    python tools/isa_blocks.py listing.s <kernel-symbol-prefix>"""
import re
import sys

lines = open(sys.argv[1]).read().splitlines()
start = next(i for i, l in enumerate(lines) if l.startswith(sys.argv[2]) and l.rstrip().endswith(":") or
             (l.startswith(sys.argv[2]) and ": ;" in l))
blocks, cur = [], {"name": "entry", "note": "", "v": 0, "s": 0, "d": 0, "g": 0}
blocks.append(cur)
for ln in lines[start + 1:]:
    if "s_endpgm" in ln:
        break
    m = re.match(r"^(\.LBB\d+_\d+):(.*)", ln)
    if m:
        cur = {"name": m.group(1), "note": m.group(2).strip(), "v": 0, "s": 0, "d": 0, "g": 0}
        blocks.append(cur)
        continue
    t = ln.strip().split()
    if not t or t[0].startswith((";", ".")):
        continue
    op = t[0]
    if op.startswith("v_"):
        cur["v"] += 4 if ("mul_lo_u32" in op or "mul_hi_u32" in op or "mul_lo_i32" in op) else 1
    elif op.startswith("s_"):
        cur["s"] += 1
    elif op.startswith("ds_"):
        cur["d"] += 1
    elif op.startswith(("global_", "buffer_", "flat_")):
        cur["g"] += 1
tot = {"v": 0, "s": 0, "d": 0, "g": 0}
for b in blocks:
    for k in tot:
        tot[k] += b[k]
    if b["v"] + b["s"] > 0:
        print(f"{b['name']:10s} v{b['v']:4d} s{b['s']:4d} ds{b['d']:3d} g{b['g']:3d} {b['note'][:60]}")
print("static totals", tot)
