"""Reduce the back-end's rocprofv3 evidence (tools/ba_prof.sh) to
profiles/<round>/ba_kernels.json: per LocalBundleAdjustment / LocalInertialBA
kernel, per dispatch,

  avg_ns            kernel-trace --stats average duration
  hbm_bytes         2 x FETCH_SIZE + WRITE_SIZE (KB; FETCH_SIZE doubled: gfx950
                    reports half the bytes of wide reads, MI355X_MICROARCH.md
                    HBM section), each counter from its own --pmc pass
  hbm_GBs           hbm_bytes / avg_ns, against the 8 TB/s HBM peak
  valu_insts, mfma_f64_insts, mfma_f64_flop (SQ_INSTS_VALU_MFMA_MOPS_F64 x 512),
  mfma_busy_cycles  (SQ_VALU_MFMA_BUSY_CYCLES)
  fp64 GFLOP/s      mfma_f64_flop / avg_ns, against the fp64 matrix peak of the
                    chip (78.6 TFLOP/s, AMD MI355X data sheet) and of the CUs
                    the kernel occupies (one CU for k_lba_solve: 1/256 of it)
  mfma_busy_frac    mfma_busy_cycles / (4 SIMDs x kernel cycles x CUs used),
                    kernel cycles = GRBM_GUI_ACTIVE / 8 (the counter sums the
                    8 XCDs) per dispatch

Every number is recomputable from the CSVs under profiles/<round>/ba/.
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict

FP64_MATRIX_PEAK_TFLOPS = 78.6  # MI355X data sheet (fp64 matrix = fp64 vector on CDNA4)
HBM_PEAK_GBS = 8000.0
N_CU = 256


def short(name: str) -> str:
    """'void orbgpu::(anonymous namespace)::k_lba_solve<true>(orbgpu::LbaArgs)' -> 'k_lba_solve<true>'"""
    m = re.search(r"(k_\w+(<[^>]*>)?|__amd\w+)", name)
    return m.group(1) if m else name


def counters(d: str):
    """-> {kernel: {counter: [sum over dispatches, n dispatches]}}"""
    acc = defaultdict(lambda: defaultdict(lambda: [0.0, set()]))
    for f in sorted(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            a = acc[short(r["Kernel_Name"])][r["Counter_Name"]]
            a[0] += float(r["Counter_Value"])
            a[1].add((f, r["Dispatch_Id"]))
    return {k: {c: (v[0], len(v[1])) for c, v in cs.items()} for k, cs in acc.items()}


def stats(d: str):
    out = {}
    for f in glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Name"])
            n0, c0 = out.get(k, (0.0, 0))
            c = int(r["Calls"])
            out[k] = (n0 + float(r["AverageNs"]) * c, c0 + c)
    return {k: (t / c, c) for k, (t, c) in out.items() if c}


def per_dispatch(cs, name):
    if name not in cs:
        return None
    s, n = cs[name]
    return s / max(n, 1)


def reduce_window(d: str) -> dict:
    st = stats(f"{d}/stats")
    sq = counters(f"{d}/p1")
    fe = counters(f"{d}/p2")
    wr = counters(f"{d}/p3")
    rows = {}
    for k, (avg_ns, calls) in sorted(st.items(), key=lambda kv: -kv[1][0] * kv[1][1]):
        row = {"avg_ns": round(avg_ns, 1), "dispatches": calls,
               "share_of_kernel_time": None}
        q = sq.get(k, {})
        f = per_dispatch(fe.get(k, {}), "FETCH_SIZE")
        w = per_dispatch(wr.get(k, {}), "WRITE_SIZE")
        if f is not None and w is not None:
            b = 1024.0 * (2 * f + w)
            row["hbm_bytes"] = round(b)
            row["hbm_GBs"] = round(b / avg_ns, 2)
            row["hbm_frac"] = round(b / avg_ns / HBM_PEAK_GBS, 5)
        v = per_dispatch(q, "SQ_INSTS_VALU")
        if v is not None:
            row["valu_insts"] = round(v)
        mi = per_dispatch(q, "SQ_INSTS_VALU_MFMA_F64")
        mo = per_dispatch(q, "SQ_INSTS_VALU_MFMA_MOPS_F64")
        mb = per_dispatch(q, "SQ_VALU_MFMA_BUSY_CYCLES")
        gr = per_dispatch(q, "GRBM_GUI_ACTIVE")
        wv = per_dispatch(q, "SQ_WAVES")
        if wv is not None:
            row["waves"] = round(wv)
        if mi:
            row["mfma_f64_insts"] = round(mi)
        if mo:
            flop = 512.0 * mo
            row["mfma_f64_flop"] = round(flop)
            row["fp64_GFLOPs"] = round(flop / avg_ns, 3)
            row["fp64_frac_chip"] = flop / avg_ns / (FP64_MATRIX_PEAK_TFLOPS * 1e3)
            cus = max(1, min(N_CU, round((wv or 1) / 8)))  # solve: one 8-wave block = 1 CU
            row["cus_used"] = cus
            row["fp64_frac_cus_used"] = round(flop / avg_ns / (FP64_MATRIX_PEAK_TFLOPS * 1e3 * cus / N_CU), 5)
            if mb is not None and gr:
                cyc = gr / 8.0
                row["mfma_busy_cycles"] = round(mb)
                row["kernel_cycles"] = round(cyc)
                row["mfma_busy_frac_cus_used"] = round(mb / (4.0 * cyc * cus), 5)
        rows[k] = row
    tot = sum(r["avg_ns"] * r["dispatches"] for r in rows.values())
    for r in rows.values():
        r["share_of_kernel_time"] = round(r["avg_ns"] * r["dispatches"] / tot, 4)
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", required=True, help="tools/ba_prof.sh output directory")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    out = {"peaks": {"fp64_matrix_TFLOPs": FP64_MATRIX_PEAK_TFLOPS, "hbm_GBs": HBM_PEAK_GBS,
                     "cus": N_CU},
           "definitions": __doc__.strip()}
    for w in ("lba", "lia"):
        if os.path.isdir(f"{a.dir}/{w}"):
            out[w] = reduce_window(f"{a.dir}/{w}")
    for nf in (18, 25):
        f = f"{a.dir}/solve_stamps_nf{nf}.json"
        if os.path.exists(f):
            out[f"solve_stamps_nf{nf}"] = json.load(open(f))
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
