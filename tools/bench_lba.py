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


PROFILE = REPO / "profiles" / "r06" / "ba" / "ba_kernels.json"


def roofline(window: str, n_sys: int) -> dict:
    """The back-end's roofline block from the committed rocprofv3 evidence
    (tools/ba_prof.sh -> tools/ba_roofline.py -> profiles/r06/ba/): fp64
    FLOP/s and MFMA busy of k_lba_solve against the gfx950 fp64 matrix peak
    (the chip's, and the one CU a single-workgroup solve can use), HBM GB/s
    of the per-edge / per-pair stages against 8 TB/s.  Recomputable from the
    CSVs next to the JSON."""
    import json

    if not PROFILE.exists():
        return {"source": None}
    d = json.loads(PROFILE.read_text())
    rows = d.get(window, {})
    out = {"source": str(PROFILE.relative_to(REPO)), "peaks": d.get("peaks"),
           "bound": "latency: the solve is one workgroup (one CU) working down a 16-pivot-tile "
                    "chain; the edge / pair stages move a few MB per launch"}
    solve = next((k for k in rows if k.startswith("k_lba_solve")), None)
    if solve:
        r = rows[solve]
        alg = n_sys ** 3 / 3 + 2 * n_sys ** 2  # LDL^T + the two substitutions
        out["solve"] = {"kernel": solve, "n": n_sys, "avg_us": round(r["avg_ns"] / 1e3, 2),
                        "mfma_f64_flop": r.get("mfma_f64_flop"),
                        "fp64_GFLOPs_mfma": r.get("fp64_GFLOPs"),
                        "frac_chip_fp64_peak": r.get("fp64_frac_chip"),
                        "frac_one_cu_fp64_peak": r.get("fp64_frac_cus_used"),
                        "mfma_busy_frac_one_cu": r.get("mfma_busy_frac_cus_used"),
                        "algorithmic_flop": int(alg),
                        "algorithmic_GFLOPs": round(alg / r["avg_ns"], 3)}
    out["hbm"] = {k: {"avg_us": round(r["avg_ns"] / 1e3, 2), "hbm_bytes": r.get("hbm_bytes"),
                      "GBs": r.get("hbm_GBs"), "frac": r.get("hbm_frac"),
                      "share_of_kernel_time": r.get("share_of_kernel_time")}
                  for k, r in rows.items() if not k.startswith("__") and "solve" not in k}
    return out


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
           "lm_trials": int(r["stats"][3]), "chi2_gpu": r["stats"][1],
           "roofline": roofline("lba", 6 * int((p.fixed == 0).sum()))}
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


def measure_lia(calls: int = 10, cpu_calls: int = 3, b_large: bool = False) -> dict:
    """LocalInertialBA (optimizer.cc:2329-2902) on the synthetic stereo-inertial
    window: 10 temporal key frames (15 DoF each), the key frame before them and
    10 older observers fixed, 2000 map points, ~16k visual edges, 10 IMU
    links, optimize(10) with user lambda 1 (bLarge: 25 key frames, 4
    iterations, lambda 1e-2)."""
    from orb_slam_fusion_amd import LocalBundleAdjuster, synth

    p = synth.lia_problem(b_large=b_large, **({"n_opt": 25, "n_fixed_cov": 6} if b_large else {}))
    lba = LocalBundleAdjuster()
    for _ in range(2):
        lba.optimize_inertial(p)
    t0 = time.perf_counter()
    for _ in range(calls):
        r = lba.optimize_inertial(p)
    gpu_ms = (time.perf_counter() - t0) / calls * 1e3
    n_opt = int((p.fixed == 0).sum())
    out = {"workload": f"LocalInertialBA{' bLarge' if b_large else ''}: {n_opt} temporal KF x 15 DoF, "
                       f"{len(p.kfs) - n_opt} fixed KF, {len(p.pts_init)} MP, {len(p.edges)} visual edges "
                       f"(50% stereo), {len(p.imu_edges)} IMU links, optimize({p.iterations})",
           "gpu_ms_per_call": round(gpu_ms, 3), "lm_iterations": int(r["stats"][2]),
           "lm_trials": int(r["stats"][3]), "err": r["stats"][0], "err_end": r["stats"][1]}
    if not b_large:
        out["roofline"] = roofline("lia", 15 * n_opt)
    if cpu_calls > 0:
        sys.path.insert(0, str(REPO / "oracle"))
        import binding as oracle  # cpu baseline leg only

        t0 = time.perf_counter()
        for _ in range(cpu_calls):
            ref = oracle.lia(p)
        out["cpu_oracle_ms_per_call"] = round((time.perf_counter() - t0) / cpu_calls * 1e3, 3)
        out["cpu_cores"] = 1
        out["err_end_oracle"] = ref["stats"][1]
        out["max_state_diff_vs_oracle"] = float(abs(r["kfs21"] - ref["kfs21"]).max())
    return out


def measure_sharded(calls: int = 10, world: int = 4) -> dict:
    """The C4 window point-sharded over `world` ranks on ONE GPU (fresh child
    processes, gloo all-reduce of the device buffers through lba.dist_reduce):
    a capability line (the exchange's cost with both ranks sharing the GPU),
    not a multi-GPU scaling figure."""
    import os
    import socket
    import subprocess
    import tempfile

    import numpy as np

    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    worker = REPO / "tools" / "lba_shard_worker.py"

    def run(ordered: bool):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        with tempfile.TemporaryDirectory() as tmp:
            procs = [subprocess.Popen([sys.executable, str(worker), str(r), str(world), str(port), tmp,
                                       str(calls), "1" if ordered else "0"], env=env,
                                      stdout=sys.stderr) for r in range(world)]
            # (gloo's connection messages go to stderr: bench.py's stdout is its one JSON line)
            if any(p.wait(timeout=300) != 0 for p in procs):
                return None
            return [dict(np.load(Path(tmp) / f"r{k}.npz")) for k in range(world)]

    r = run(False)
    if r is None:
        return {"error": "worker failed"}
    ro = run(True)
    out = {"workload": f"C4 LocalBundleAdjustment point-sharded over {world} ranks on 1 GPU "
                       "(gloo all-reduce of S, b, chi2, scale per LM trial)",
           "ms_per_call": round(float(max(x["ms_per_call"] for x in r)), 3),
           "lm_iterations": int(r[0]["stats"][2]), "lm_trials": int(r[0]["stats"][3]),
           "chi2": float(r[0]["stats"][1]),
           "ranks": world,
           "ranks_identical_poses": bool(all((x["poses_d"] == r[0]["poses_d"]).all() for x in r)),
           "scaling": "unmeasured (both ranks on one GPU)"}
    if ro is not None:  # the stream-ordered form (reductions enqueued on the library stream)
        out["ordered"] = {
            "ms_per_call": round(float(max(x["ms_per_call"] for x in ro)), 3),
            "chi2": float(ro[0]["stats"][1]),
            "same_poses_as_host_reduce": bool((ro[0]["poses_d"] == r[0]["poses_d"]).all()),
            "note": "gloo stages each enqueued all-reduce through the host (lba.dist_enqueue); "
                    "the device-resident LM pays off with RCCL on a multi-GPU node"}
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=10)
    ap.add_argument("--lia", action="store_true", help="LocalInertialBA instead of LBA")
    ap.add_argument("--large", action="store_true", help="LocalInertialBA bLarge window")
    ap.add_argument("--cpu-calls", type=int, default=3)
    a = ap.parse_args()
    if a.lia:
        print(json.dumps(measure_lia(a.calls, a.cpu_calls, a.large)))
    else:
        print(json.dumps(measure(a.calls, a.cpu_calls)))
