"""PoseInertialOptimizationLastFrame timing: a batch of B
synthetic stereo-inertial tracking problems (tests/inertial_cases.py: 50 ms
of motion, 400 matched map points, 70 % stereo, 10 % gross outliers, the
previous frame's prior) resident in HBM, one orbgpu_pose_inertial_batch call
timed with HIP events on its own stream; beside it one problem at a time
through the host ABI (the tracking thread's latency) and the CPU oracle per
problem, plus a parity spot check (flags and return value equal, states to
1e-7).

    python tools/bench_inertial.py [--problems 64] [--calls 20] [--mode 0]
"""
import argparse
import hashlib
import json
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "tests"))

N_OBS = 400


def measure(problems: int = 64, calls: int = 20, mode: int = 0, cpu_problems: int = 4,
            latency_calls: int = 20) -> dict:
    import torch

    with torch.cuda.stream(torch.cuda.Stream()):
        return _measure(problems, calls, mode, cpu_problems, latency_calls)


def _measure(P, calls, mode, cpu_problems, latency_calls):
    import torch

    import inertial_cases as ic
    from orb_slam_fusion_amd._lib import (IMU_PREINT_DTYPE, IMU_PRIOR_DTYPE, IMU_STATE_DTYPE,
                                          INERTIAL_OBS_DTYPE, INERTIAL_RESULT_DTYPE)
    from orb_slam_fusion_amd.inertial import InertialProblem, PoseInertialOptimizer

    cases = [ic.make_case(100 + i, mode=mode, n_obs=N_OBS) for i in range(P)]
    dev = torch.device("cuda", 0)

    def rec(key, dt):
        a = np.stack([np.asarray(c[key]).reshape(()) for c in cases]).astype(dt)
        return torch.from_numpy(a.view(np.uint8).reshape(P, dt.itemsize).copy()).to(dev)

    obs = np.stack([c["obs"] for c in cases]).astype(INERTIAL_OBS_DTYPE)
    d_obs = torch.from_numpy(obs.view(np.uint8).reshape(P, N_OBS, 32).copy()).to(dev)
    d_n = torch.full((P,), N_OBS, dtype=torch.int32, device=dev)
    d_cur, d_prev = rec("cur", IMU_STATE_DTYPE), rec("prev", IMU_STATE_DTYPE)
    d_pre = rec("preint", IMU_PREINT_DTYPE)
    d_pri = rec("prior", IMU_PRIOR_DTYPE) if mode == 0 else None
    d_res = torch.zeros((P, INERTIAL_RESULT_DTYPE.itemsize), dtype=torch.uint8, device=dev)
    d_out = torch.zeros((P, N_OBS), dtype=torch.uint8, device=dev)
    opt = PoseInertialOptimizer(max_problems=P, max_obs=N_OBS)
    s = torch.cuda.current_stream()

    def run():
        opt.batch(mode, cases[0]["calib"], d_cur, d_prev, d_pre, d_pri, d_obs, d_n, d_res, d_out,
                  stream=s)

    for _ in range(3):
        run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(calls):
        run()
    e1.record(s)
    torch.cuda.synchronize()
    gpu_ms = e0.elapsed_time(e1) / calls
    res = d_res.cpu().numpy().view(INERTIAL_RESULT_DTYPE).reshape(P)
    outs = d_out.cpu().numpy()
    name = "PoseInertialOptimizationLastFrame" if mode == 0 else \
        "PoseInertialOptimizationLastKeyFrame"
    out = {"workload": f"{name}: {P} synthetic stereo-inertial problems per batch ({N_OBS} "
                       "matched points, 70% stereo, 10% outliers, dt 50 ms), 4 rounds x 10 "
                       "Gauss-Newton iterations + marginalisation, inputs resident in HBM",
           "gpu_ms_per_batch": round(gpu_ms, 4),
           "gpu_problems_per_s": round(P / gpu_ms * 1e3, 1),
           "inliers_per_problem": round(float(res["n_inliers"].mean()), 1),
           # bit-identity across library builds (tools/inert_ab.sh)
           "result_sha": hashlib.sha1(res.tobytes() + outs.tobytes()).hexdigest()[:16]}
    # one problem at a time through the host ABI (the tracking thread's view)
    one = PoseInertialOptimizer(max_obs=N_OBS)
    c0 = cases[0]
    pb = InertialProblem(calib=c0["calib"], cur=c0["cur"], prev=c0["prev"], preint=c0["preint"],
                         obs=c0["obs"], prior=c0["prior"])
    fn = one.PoseInertialOptimizationLastFrame if mode == 0 else \
        one.PoseInertialOptimizationLastKeyFrame
    for _ in range(min(3, latency_calls)):
        fn(pb)
    lat = []
    for _ in range(latency_calls):
        t0 = time.perf_counter()
        fn(pb)
        lat.append(time.perf_counter() - t0)
    if lat:
        out["gpu_ms_per_problem_latency"] = round(float(np.median(lat)) * 1e3, 4)
    one.close()
    if cpu_problems > 0:
        sys.path.insert(0, str(REPO / "oracle"))
        import binding as oracle  # cpu baseline / checker leg only

        exact, dmax = True, 0.0
        t0 = time.perf_counter()
        refs = [oracle.pose_inertial(cases[i]) for i in range(min(cpu_problems, P))]
        el = time.perf_counter() - t0
        for i, (ref, ref_out) in enumerate(refs):
            exact &= bool(np.array_equal(outs[i], ref_out) and res[i]["n_good"] == ref["n_good"])
            for k in ("Rwb_d", "twb_d", "v_d", "bg_d", "ba_d"):
                dmax = max(dmax, float(np.max(np.abs(res[i][k] - ref[k]))))
        out["cpu_oracle_ms_per_problem"] = round(el / len(refs) * 1e3, 3)
        out["cpu_cores"] = 1
        out["flags_equal_vs_oracle"] = exact
        out["max_state_diff_vs_oracle"] = dmax
    opt.close()
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--problems", type=int, default=64)
    ap.add_argument("--calls", type=int, default=20)
    ap.add_argument("--mode", type=int, default=0)
    a = ap.parse_args()
    print(json.dumps(measure(a.problems, a.calls, a.mode)))
