"""A/B timing of the LBA reduced-system paths (orbgpu_lba_ctx_set_solver):
the one-workgroup HBM factorisation (BLOCK) against the device-wide tile steps
(GRID) on windows of growing size, each call timed end to end through the C
ABI (the LM loop, every trial's solve included).  Prints one JSON line per
window; the results of the two paths must be bit-identical.  Picks the size
where GRID starts to win (kGridMinPad in lba_kernels.hip)."""
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from orb_slam_fusion_amd import LocalBundleAdjuster, _lib, synth  # noqa: E402


def timed(adj, call, reps):
    call()  # warm: arena, code objects
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        r = call()
        t.append(time.perf_counter() - t0)
    return r, 1e3 * float(np.median(t))


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    rows = []
    for n_kf in (22, 30, 45, 60, 70, 90, 130, 200, 346):
        p = synth.lba_problem(seed=30 + n_kf, n_kf=n_kf, n_pts=30 * n_kf, obs_per_pt=5, n_fixed=2)
        out = {"window": f"lba {n_kf - 2} free kf", "rows": 6 * (n_kf - 2)}
        res = {}
        for name, mode in (("block", _lib.ORBGPU_LBA_SOLVER_BLOCK), ("grid", _lib.ORBGPU_LBA_SOLVER_GRID),
                           ("auto", _lib.ORBGPU_LBA_SOLVER_AUTO)):
            adj = LocalBundleAdjuster()
            adj.set_solver(mode)
            try:
                res[name], out[name + "_ms"] = timed(adj, lambda: adj.optimize(p), reps)
            except _lib.OrbGpuError as e:
                out[name + "_ms"] = f"status {e.status}"
        if "block" in res and "grid" in res:
            out["identical"] = bool(np.array_equal(res["block"]["poses_d"], res["grid"]["poses_d"]) and
                                    np.array_equal(res["block"]["stats"], res["grid"]["stats"]))
        out["trials"] = int(res["auto"]["stats"][3])
        print(json.dumps(out), flush=True)
        rows.append(out)
    for large in (False, True):
        pb = synth.lia_problem(9, n_opt=25, n_fixed_cov=6, n_pts=1500, b_large=True) if large else synth.lia_problem()
        out = {"window": "lia bLarge" if large else "lia default"}
        for name, mode in (("block", _lib.ORBGPU_LBA_SOLVER_BLOCK), ("grid", _lib.ORBGPU_LBA_SOLVER_GRID),
                           ("auto", _lib.ORBGPU_LBA_SOLVER_AUTO)):
            adj = LocalBundleAdjuster()
            adj.set_solver(mode)
            try:
                _, out[name + "_ms"] = timed(adj, lambda: adj.optimize_inertial(pb), reps)
            except _lib.OrbGpuError as e:
                out[name + "_ms"] = f"status {e.status}"
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
