"""Per-phase cycle counts of the inertial pose kernel (thread 0 of each
workgroup) from the ORB_STAMPS build.

    make stamps && ORBGPU_LIB=orb_slam_fusion_amd/lib/liborbgpu_stamps.so \\
        python tools/inertial_stamps.py [--mode 0]
"""
import argparse
import ctypes
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "tools"))


def main(mode: int):
    import torch

    import bench_inertial as bi
    from orb_slam_fusion_amd._lib import library_path

    lib = ctypes.CDLL(str(library_path()))
    buf = (ctypes.c_ulonglong * 32)()
    P, calls = 64, 5
    bi.measure(P, 1, mode, cpu_problems=0, latency_calls=1)  # warm up (and clear below)
    torch.cuda.synchronize()
    lib.orbgpu_debug_inertial_stamps(buf, 32)
    # latency_calls=0 / cpu_problems=0: only the batch launches (3 warm-up + calls)
    bi.measure(P, calls, mode, cpu_problems=0, latency_calls=0)
    torch.cuda.synchronize()
    assert lib.orbgpu_debug_inertial_stamps(buf, 32) == 0
    v = list(buf)
    runs = P * (calls + 3)
    names = {6: "imu_edges (wave 0)", 0: "visual sweep wait + reduce", 1: "assemble",
             2: "ldlt", 3: "update", 4: "classify", 5: "final hessian + marginalise"}
    sub = {10: "visual loop (wave 2)", 11: "visual DPP reduce + store (wave 2)",
           12: "solve: order + loads", 13: "solve: pivots", 14: "assemble pass 1 (+barrier)",
           7: "imu: preintegration deltas", 9: "imu: error (LogSO3)", 15: "imu: linear blocks"}
    tot = sum(v[i] for i in names)
    print(json.dumps({"ticks_per_problem": tot / runs, "iterations_per_problem": v[8] / runs,
                      "ticks_per_phase_per_problem": {names[i]: round(v[i] / runs) for i in names},
                      "sub_phases_per_problem": {sub[i]: round(v[i] / runs) for i in sub},
                      # every vis_sweep (the LM steps' and the final Hessian's)
                      "sweep_ticks_per_wave_per_problem": [round(v[16 + w] / runs) for w in range(8)]}))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", type=int, default=0)
    main(ap.parse_args().mode)
