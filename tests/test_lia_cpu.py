"""LocalInertialBA oracle (oracle/lia_oracle.cc) pinned against the independent
numpy model of tests/lia_model.py: visual Jacobians and the whole (key frames
+ points) system by central differences through the reference's vertex
updates, one LM trial as a dense solve, the outlier rule of
optimizer.cc:2799-2826, and truth recovery on synthetic windows."""
import numpy as np
import pytest

import binding as oracle
import lia_model as lm
from orb_slam_fusion_amd import synth


def small(seed=5, **kw):
    args = dict(n_opt=4, n_fixed_cov=2, n_pts=30, max_obs=4)
    args.update(kw)
    return synth.lia_problem(seed, **args)


def test_visual_jacobians_match_numeric():
    pb = small()
    c = pb.calib
    for e in pb.edges[:40]:
        x = lm.state21(pb.kfs[e["kf"]])
        X = pb.pts_init[e["point"]].astype(float)
        kf = np.array(pb.kfs[e["kf"]])
        err, Jl, Jp = oracle.lia_vis_linearize(c, kf, X, e)
        d = 3 if e["ur"] >= 0 else 2
        Rcw, tcw = lm.cam_of(c, None, kf)
        assert np.allclose(err[:d], lm.vis_error(c, Rcw, tcw, X, e), rtol=0, atol=1e-9)
        h = 1e-6
        Jl_n = np.zeros((d, 3))
        Jp_n = np.zeros((d, 6))
        for j in range(3):
            dx = h * np.eye(3)[j]
            Jl_n[:, j] = (lm.vis_error(c, Rcw, tcw, X + dx, e) - lm.vis_error(c, Rcw, tcw, X - dx, e)) / (2 * h)
        for j in range(6):
            dv = h * np.eye(6)[j]
            ep = lm.vis_error(c, *lm.cam_of(c, lm.update21(x, dv, "P")), X, e)
            em = lm.vis_error(c, *lm.cam_of(c, lm.update21(x, -dv, "P")), X, e)
            Jp_n[:, j] = (ep - em) / (2 * h)
        assert np.abs(Jl[:d] - Jl_n).max() <= 1e-5 * np.abs(Jl_n).max()
        assert np.abs(Jp[:d] - Jp_n).max() <= 1e-5 * np.abs(Jp_n).max()
        if d == 2:
            assert not Jl[2].any() and not Jp[2].any()


@pytest.mark.parametrize("seed,rec_init", [(5, False), (6, True)])
def test_system_matches_numeric(seed, rec_init):
    pb = small(seed, rec_init=rec_init)
    H, b = oracle.lia_system(pb)
    Hn, bn = lm.Window(pb).system()
    assert H.shape == Hn.shape
    assert np.abs(H - Hn).max() <= 1e-6 * np.abs(Hn).max()
    assert np.abs(b - bn).max() <= 1e-6 * np.abs(bn).max()
    assert np.abs(H - H.T).max() <= 1e-12 * np.abs(H).max()


def test_one_lm_step_matches_dense_solve():
    pb = small(7)
    lam = 1.0
    r = oracle.lia(pb, iterations=1, lambda_init=lam)
    assert r["stats"][3] == 1, "the first trial must be accepted for this comparison"
    w = lm.Window(pb)
    # the Schur complement + LDLT + vertex updates against a dense solve of the
    # oracle's full system (itself pinned by test_system_matches_numeric)
    x, X = w.step(lam, system=oracle.lia_system(pb))
    for k in w.free:
        ref = x[k]
        got = r["kfs21"][k]
        assert np.abs(got - ref).max() <= 1e-9 * max(1.0, np.abs(ref).max())
    for k in range(len(pb.kfs)):
        if pb.fixed[k]:
            assert np.array_equal(r["kfs21"][k], lm.state21(pb.kfs[k]))
    assert np.abs(r["pts"] - np.array(X)).max() <= 1e-9 * np.abs(np.array(X)).max()
    # chi2 bookkeeping: err at the initial state, err_end / accepted at the
    # trial state (the model evaluates the float preintegration in double)
    assert abs(r["stats"][0] - w.robust_chi2()) <= 1e-6 * r["stats"][0]
    w.x, w.X = x, X
    w.init = [None] * len(pb.kfs)
    for k in range(len(pb.kfs)):
        if pb.fixed[k]:
            w.init[k] = pb.kfs[k]
    assert abs(r["stats"][1] - w.robust_chi2()) <= 1e-6 * r["stats"][1]
    assert r["stats"][1] == r["stats"][6]


def test_outlier_rule():
    """optimizer.cc:2799-2826 on the errors of the last computeActiveErrors
    (here the accepted trial's): mono chi2 > 5.991f (far) / 1.5f * 5.991f
    (close) or depth <= 0, stereo chi2 > 7.815f."""
    pb = small(8, n_pts=200, max_obs=6, outlier_frac=0.15)
    r = oracle.lia(pb, iterations=1)
    assert r["stats"][3] == 1
    w = lm.Window(pb)
    x = [r["kfs21"][k] for k in range(len(pb.kfs))]
    init = [pb.kfs[k] if pb.fixed[k] else None for k in range(len(pb.kfs))]
    errs = w.errors(x=x, X=list(r["pts"]), init=init)
    th_m, th_mc, th_s = float(np.float32(5.991)), float(np.float32(1.5) * np.float32(5.991)), \
        float(np.float32(7.815))
    ref = np.zeros(len(pb.edges), np.uint8)
    n_close_mid = 0
    for i, e in enumerate(pb.edges):
        err, Om, _ = errs[i]
        chi = float(err @ Om @ err)
        if e["ur"] < 0:
            Rcw, tcw = lm.cam_of(pb.calib, x[e["kf"]], init[e["kf"]])
            depth = (Rcw @ r["pts"][e["point"]] + tcw)[2] > 0
            cl = bool(pb.close[e["point"]])
            ref[i] = (chi > th_m and not cl) or (chi > th_mc and cl) or not depth
            n_close_mid += cl and th_m < chi <= th_mc
        else:
            ref[i] = chi > th_s
    assert np.array_equal(r["outlier"], ref)
    assert n_close_mid > 0  # the close-point band is exercised


@pytest.mark.parametrize("b_large", [False, True])
def test_recovers_truth(b_large):
    pb = synth.lia_problem(13, b_large=b_large)
    r = oracle.lia(pb)
    st = r["stats"]
    assert st[1] < 0.6 * st[0]  # err_end well below err (no FAIL)
    assert st[2] <= pb.iterations
    n_opt = int((pb.fixed == 0).sum())
    for k in range(n_opt):
        assert np.linalg.norm(r["kfs21"][k, 9:12] - pb.kfs_true[k]["twb"]) < 1.5e-2
        R = r["kfs21"][k, :9].reshape(3, 3)
        Rt = pb.kfs_true[k]["Rwb"].astype(float).reshape(3, 3)
        assert np.linalg.norm(lm.log_so3(Rt.T @ R)) < 3e-3
    out = r["outlier"].astype(bool)
    assert out[pb.outliers].mean() > 0.95
    assert out.mean() < 0.2


def test_vertex_pose_only_keyframes_system():
    """Free key frames without IMU data (`!pKFi->bImu`, optimizer.cc:2466-2484):
    a VertexPose alone (6 rows), no temporal link touching it (:2503) -- the
    oracle's system against the numpy model's central differences."""
    pb = small(11, n_opt=5, no_imu=(1, 3))
    assert list(pb.imu[:5]) == [1, 0, 1, 0, 1]
    assert all(pb.imu[e["kf1"]] and pb.imu[e["kf2"]] for e in pb.imu_edges)
    H, b = oracle.lia_system(pb)
    w = lm.Window(pb)
    assert w.n_kf_rows == 15 * 3 + 6 * 2
    Hn, bn = w.system()
    assert H.shape == Hn.shape
    assert np.abs(H - Hn).max() <= 1e-6 * np.abs(Hn).max()
    assert np.abs(b - bn).max() <= 1e-6 * np.abs(bn).max()


def test_vertex_pose_only_keyframes_lm_step():
    """One LM trial with VertexPose-only key frames against the dense solve of
    the oracle's full system: their velocity and biases are not vertices and
    stay as given."""
    pb = small(12, n_opt=5, no_imu=(0, 2))
    r = oracle.lia(pb, iterations=1, lambda_init=1.0)
    assert r["stats"][3] == 1
    w = lm.Window(pb)
    x, X = w.step(1.0, system=oracle.lia_system(pb))
    for k in w.free:
        assert np.abs(r["kfs21"][k] - x[k]).max() <= 1e-9 * max(1.0, np.abs(x[k]).max())
        if not pb.imu[k]:
            assert np.array_equal(r["kfs21"][k, 12:], lm.state21(pb.kfs[k])[12:])
    assert np.abs(r["pts"] - np.array(X)).max() <= 1e-9 * np.abs(np.array(X)).max()


def test_vertex_pose_only_recovers_truth():
    pb = synth.lia_problem(14, n_opt=10, no_imu=(4,))
    r = oracle.lia(pb)
    assert r["stats"][1] < 0.6 * r["stats"][0]
    for k in range(10):
        assert np.linalg.norm(r["kfs21"][k, 9:12] - pb.kfs_true[k]["twb"]) < 1.5e-2


def test_banded_window_generator():
    """consecutive observers: every point's key frames are adjacent in the
    window order (a banded reduced system)."""
    pb = synth.lia_problem(15, n_opt=12, n_fixed_cov=2, n_pts=300, max_obs=3, consecutive=True)
    kfs_of = {}
    for e in pb.edges:
        kfs_of.setdefault(int(e["point"]), []).append(int(e["kf"]))
    span = np.array([max(v) - min(v) for v in kfs_of.values()])
    assert (span == 2).mean() > 0.95 and span.max() <= 10
