"""Oracle for PoseInertialOptimizationLastFrame / LastKeyFrame pinned against
an independent numpy model (tests/inertial_cases.py): the analytic Jacobians
and the multi-edge assembly of every edge type against central differences
through the reference's vertex updates, Marginalize's pseudo-inverse against
numpy's eigendecomposition, the final Hessians (LastKeyFrame: the current
frame's; LastFrame: after marginalising the previous frame) against numeric
ones at the oracle's final states, and the optimisation itself against the
synthetic truth.  The reference's g2o/Eigen run is not available here:
parity with it is by these properties (tolerances in each test)."""
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "oracle"))
sys.path.insert(0, str(ROOT / "tests"))

import binding as orc  # noqa: E402
import inertial_cases as ic  # noqa: E402


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("seed", [1, 5])
def test_system_matches_numeric_jacobians(mode, seed):
    case = ic.make_case(seed, mode=mode, n_obs=40)
    cur, prev = ic.state21(case["cur"]), ic.state21(case["prev"])
    # also away from the initial estimates (non-trivial rotation errors)
    cur = ic.update21(cur, np.r_[0.02, -0.01, 0.015, 0.05, -0.02, 0.01], "P")
    prev = ic.update21(prev, np.r_[-0.01, 0.02, 0.01, 0.01, 0.03, -0.02], "P")
    H, b = orc.inertial_system(case, cur, prev, kernels=False)
    Hn, bn = ic.numeric_system(case, cur, prev)
    assert np.abs(H - Hn).max() <= 1e-6 * np.abs(Hn).max()
    assert np.abs(b - bn).max() <= 1e-6 * np.abs(bn).max()
    assert np.abs(H - H.T).max() <= 1e-12 * np.abs(H).max()


def test_sym_pinv_matches_numpy():
    rng = np.random.default_rng(3)
    for m in (6, 15):
        Q, _ = np.linalg.qr(rng.normal(size=(m, m)))
        lam = 10.0 ** rng.uniform(-4, 5, m)
        lam[: m // 3] *= -1  # indefinite
        lam[1] = 3e-7  # below the cut
        A = (Q * lam) @ Q.T
        A = (A + A.T) / 2
        w, V = np.linalg.eigh(A)
        keep = np.abs(w) > 1e-6
        ref = (V[:, keep] / w[keep]) @ V[:, keep].T
        got = orc.sym_pinv(A)
        assert np.abs(got - ref).max() <= 1e-6 * np.abs(ref).max()


@pytest.mark.parametrize("mode", [0, 1])
def test_optimisation_recovers_truth_and_outliers(mode):
    case = ic.make_case(2, mode=mode, n_obs=300)
    res, out = orc.pose_inertial(case)
    tr = case["truth"]
    R = res["Rwb_d"].reshape(3, 3)
    assert np.linalg.norm(ic.log_so3(tr["R2"].T @ R)) < 3e-3
    assert np.linalg.norm(res["twb_d"] - tr["t2"]) < 2e-2
    assert out[tr["outliers"]].all()  # every gross outlier flagged
    assert out.sum() < 0.25 * len(out)
    assert res["n_good"] == len(out) - out.sum() == res["n_inliers"]
    assert np.allclose(res["Rwb"], res["Rwb_d"].astype(np.float32))
    assert np.allclose(res["v"], res["v_d"].astype(np.float32))


def _inlier_case(case, out):
    c = dict(case)
    c["obs"] = case["obs"][out == 0]
    return c


def test_final_hessian_last_keyframe():
    case = ic.make_case(4, mode=1, n_obs=120)
    res, out = orc.pose_inertial(case)
    cur = np.concatenate([res["Rwb_d"], res["twb_d"], res["v_d"], res["bg_d"], res["ba_d"]])
    Hn, _ = ic.numeric_system(_inlier_case(case, out), cur, ic.state21(case["prev"]))
    H = res["H"].reshape(15, 15)
    assert np.abs(H - Hn).max() <= 1e-6 * np.abs(Hn).max()


def test_final_hessian_last_frame_marginalised():
    case = ic.make_case(6, mode=0, n_obs=120)
    res, out, prev = orc.pose_inertial(case, with_prev=True)
    cur = np.concatenate([res["Rwb_d"], res["twb_d"], res["v_d"], res["bg_d"], res["ba_d"]])
    Hn, _ = ic.numeric_system(_inlier_case(case, out), cur, prev)
    # solver order: current frame 0..14, previous 15..29; Schur on the previous
    Hcc, Hcp, Hpp = Hn[:15, :15], Hn[:15, 15:], Hn[15:, 15:]
    w, V = np.linalg.eigh(Hpp)
    keep = np.abs(w) > 1e-6
    ref = Hcc - Hcp @ ((V[:, keep] / w[keep]) @ V[:, keep].T) @ Hcp.T
    H = res["H"].reshape(15, 15)
    assert np.abs(H - ref).max() <= 1e-5 * np.abs(ref).max()


def test_recovery_when_few_inliers():
    """nInliers < 30 and !bRecInit: observations under chi2 18 / 24 are taken
    back as inliers and nBad is recounted (optimizer.cc:5059-5085)."""
    case = ic.make_case(7, mode=0, n_obs=40, outlier_frac=0.5)
    res0, out0 = orc.pose_inertial(case, rec_init=True)
    res1, out1 = orc.pose_inertial(case, rec_init=False)
    assert res0["n_inliers"] < 30
    assert (out1 <= out0).all()  # only clears flags
    assert res1["n_good"] >= res0["n_good"]
    assert np.array_equal(res0["Rwb_d"], res1["Rwb_d"])  # the state is not re-optimised
