"""The stereo-inertial tracking chain's IMU inputs for a synthetic frame pair
of tools/bench_track.Chain: the IMU states follow the chain's camera
(identity last pose, motion-model current pose) through a synthetic
camera-body calibration, the preintegration is exact for that motion, and the
previous frame's prior sits at its state.  Shared by
tests/test_gpu_track_inertial.py and tools/bench_latency_inertial.py."""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tests"))


def imu_inputs(c, f):
    import inertial_cases as ic

    base = ic.make_case(40 + f, mode=0, n_obs=0)
    calib = base["calib"]
    Rcb = calib["Rcb"].astype(float).reshape(3, 3)
    tcb = calib["tcb"].astype(float)

    def body(tcw):  # camera Tcw = (I, tcw): Twb = Twc Tcb = (Rcb, tcb - tcw)
        return Rcb.copy(), tcb - np.asarray(tcw, float)

    dt = float(base["preint"]["dT"])
    R1, t1 = body(c.Tlw[f][4:])
    R2, t2 = body(c.Tcw[f][4:])
    v = (t2 - t1) / dt
    z3 = np.zeros(3)
    cur = ic.make_state(calib, R2, t2, v, z3, z3)
    prev = ic.make_state(calib, R1, t1, v, z3, z3)
    pi = base["preint"].copy()
    R1d, R2d = prev["Rwb"].astype(float).reshape(3, 3), cur["Rwb"].astype(float).reshape(3, 3)
    p1, p2 = prev["twb"].astype(float), cur["twb"].astype(float)
    v1, v2 = prev["v"].astype(float), cur["v"].astype(float)
    pi["dR"] = ic.polar(R1d.T @ R2d).ravel()
    pi["dV"] = R1d.T @ (v2 - v1 - ic.G * dt)
    pi["dP"] = R1d.T @ (p2 - p1 - v1 * dt - 0.5 * ic.G * dt * dt)
    pi["bg"], pi["ba"] = 0, 0
    prior = base["prior"].copy()
    prior["Rwb"], prior["twb"] = prev["Rwb"].astype(float), prev["twb"].astype(float)
    prior["vwb"], prior["bg"], prior["ba"] = prev["v"].astype(float), 0, 0
    return calib, cur, prev, pi, prior
