"""Vector-memory pipeline counters per extractor kernel (VERDICT r5 item 3:
what k_describe waits on).  Reduces the rocprofv3 --pmc passes of
tools/pmc_groups_vmem.txt (run by tools/pmc_run.sh over tools/prof_stages.py)
to per-launch figures and ratios:

  ta_busy          TA_BUSY_avr / GRBM_GUI_ACTIVE (busy share of the average TA)
  td_busy          TD_TD_BUSY_sum / (GRBM_GUI_ACTIVE x 256 TDs)
  tcp_accesses_per_vmem_inst   TCP_TOTAL_CACHE_ACCESSES / SQ_INSTS_VMEM_RD
                   (cache-line tag lookups per load instruction: one per
                   distinct 128-B line a wave's load touches)
  l1_miss_share    TCP_TCC_READ_REQ / TCP_TOTAL_CACHE_ACCESSES
  tcc_read_latency_cycles   TCP_TCC_READ_REQ_LATENCY / TCP_TCC_READ_REQ
  wait_share       SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES (wave cycles waiting on a
                   dependency: memory or LDS results)
  ...

    python tools/pmc_vmem.py gpurun_out/pmc [--out profiles/r06/describe_vmem.json]
"""
import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from pmc_kernels import counters  # noqa: E402

KERNELS = ("k_resize", "k_blur", "k_fast_cells", "k_octree", "k_describe", "k_assemble")
N_TD = 256  # one texture data unit per CU


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--out")
    a = ap.parse_args()
    cc = counters(a.dir)
    out = {}
    for k in KERNELS:
        if k not in cc:
            continue
        c = {name: v for name, v in cc[k].items()}
        per = {name: s / n for name, (s, n, ns) in c.items()}  # per dispatch
        row = {"counters_per_dispatch": {name: round(v, 1) for name, v in sorted(per.items())}}
        g = per.get("GRBM_GUI_ACTIVE")
        if g:
            if "TA_BUSY_avr" in per:
                row["ta_busy"] = round(per["TA_BUSY_avr"] / g, 4)
            if "TD_TD_BUSY_sum" in per:
                row["td_busy"] = round(per["TD_TD_BUSY_sum"] / (g * N_TD), 4)
            if "TA_ADDR_STALLED_BY_TC_CYCLES_sum" in per:
                row["ta_addr_stalled_by_tc_per_ta"] = round(per["TA_ADDR_STALLED_BY_TC_CYCLES_sum"] / (g * N_TD), 4)
        if per.get("SQ_INSTS_VMEM_RD"):
            if "TCP_TOTAL_CACHE_ACCESSES_sum" in per:
                row["tcp_accesses_per_vmem_inst"] = round(per["TCP_TOTAL_CACHE_ACCESSES_sum"] / per["SQ_INSTS_VMEM_RD"], 2)
        if per.get("TCP_TOTAL_CACHE_ACCESSES_sum") and "TCP_TCC_READ_REQ_sum" in per:
            row["l1_miss_share"] = round(per["TCP_TCC_READ_REQ_sum"] / per["TCP_TOTAL_CACHE_ACCESSES_sum"], 4)
        if per.get("TCP_TCC_READ_REQ_sum") and "TCP_TCC_READ_REQ_LATENCY_sum" in per:
            row["tcc_read_latency_cycles"] = round(per["TCP_TCC_READ_REQ_LATENCY_sum"] / per["TCP_TCC_READ_REQ_sum"], 1)
        if per.get("SQ_WAVE_CYCLES"):
            for name in ("SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS"):
                if name in per:
                    row[name.lower().replace("sq_", "") + "_share"] = round(per[name] / per["SQ_WAVE_CYCLES"], 4)
        if per.get("SQ_WAVES") and per.get("SQ_WAVE_CYCLES"):
            row["cycles_per_wave"] = round(per["SQ_WAVE_CYCLES"] / per["SQ_WAVES"], 1)
        if per.get("SQ_WAVES") and "SQ_INSTS_VMEM_RD" in per:
            row["vmem_rd_per_wave"] = round(per["SQ_INSTS_VMEM_RD"] / per["SQ_WAVES"], 2)
        out[k] = row
    txt = json.dumps(out, indent=1)
    if a.out:
        Path(a.out).write_text(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
