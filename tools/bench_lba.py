"""LocalBundleAdjustment timing on the C4 window (20 KF, 3000 MP, 18000 edges,
optimize(10)): GPU (orbgpu_lba_optimize) per call vs the CPU oracle per call.

    python tools/bench_lba.py [--calls 10]
"""
import argparse
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))


def measure(calls: int = 10, cpu_calls: int = 3) -> dict:
    from orb_slam_fusion_amd import LocalBundleAdjuster, synth

    p = synth.lba_problem()
    lba = LocalBundleAdjuster()
    for _ in range(2):
        lba.optimize(p)
    t0 = time.perf_counter()
    for _ in range(calls):
        r = lba.optimize(p)
    gpu_ms = (time.perf_counter() - t0) / calls * 1e3
    out = {"workload": "C4 LocalBundleAdjustment: 20 KF (2 fixed), 3000 MP, 18000 edges "
                       "(50% stereo), optimize(10)",
           "gpu_ms_per_call": round(gpu_ms, 3), "lm_iterations": int(r["stats"][2]),
           "lm_trials": int(r["stats"][3]), "chi2_gpu": r["stats"][1]}
    if cpu_calls > 0:
        sys.path.insert(0, str(REPO / "oracle"))
        import binding as oracle  # cpu baseline leg only

        t0 = time.perf_counter()
        for _ in range(cpu_calls):
            ref = oracle.lba(p)
        out["cpu_oracle_ms_per_call"] = round((time.perf_counter() - t0) / cpu_calls * 1e3, 3)
        out["cpu_cores"] = 1
        out["chi2_oracle"] = ref["stats"][1]
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=10)
    print(json.dumps(measure(ap.parse_args().calls)))
