"""GPU LocalInertialBA (orbgpu_lia_optimize) vs the oracle (oracle/lia_oracle.cc)
on the same synthetic windows.  Floating point, so parity is by tolerance:
the GPU sums in different fixed orders and factors the 15-per-key-frame
reduced system by 16 x 16 MFMA tiles; the LM path (iterations, trials), the
outlier flags (every edge whose oracle chi2 is not within 1e-6 relative of its
threshold) and err / err_end agree, states to
~1e-7 relative."""
import sys
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "oracle"))
sys.path.insert(0, str(REPO))

import binding as oracle  # noqa: E402
from orb_slam_fusion_amd import LocalBundleAdjuster, synth  # noqa: E402
from test_gpu_lba import check_flags  # noqa: E402

pytestmark = pytest.mark.gpu


def _compare(pb, tol=1e-6):
    ref = oracle.lia(pb)
    got = LocalBundleAdjuster().optimize_inertial(pb)
    gs, rs = got["stats"], ref["stats"]
    assert gs[2] == rs[2] and gs[3] == rs[3], (gs, rs)  # LM iterations, trials
    assert abs(gs[0] - rs[0]) <= 1e-8 * rs[0], (gs[0], rs[0])  # err: one evaluation
    for k in (1, 6):  # err_end, accepted chi2: after the whole LM path
        assert abs(gs[k] - rs[k]) <= tol * rs[k], (k, gs[k], rs[k])
    # lambda follows the gain ratio rho = (chi2 - chi2') / scale, a difference
    # of nearly equal sums: its rounding shows in the last digits of lambda
    assert abs(gs[4] - rs[4]) <= 1e-3 * rs[4], (gs[4], rs[4])
    scale = np.maximum(1.0, np.abs(ref["kfs21"]))
    dk = (np.abs(got["kfs21"] - ref["kfs21"]) / scale).max()
    print(f"max state diff {dk:.3g}, chi2 rel diff {abs(gs[1] - rs[1]) / rs[1]:.3g}")
    assert dk <= tol
    assert np.allclose(got["pts"], ref["pts"], rtol=1e-5, atol=1e-5)
    # optimizer.cc:2799-2826: float thresholds 5.991f, 1.5f * 5.991f (close
    # points, mono), 7.815f (stereo), compared in double
    mono = pb.edges["ur"] < 0
    close = pb.close[pb.edges["point"]] != 0
    thr = np.where(mono, np.where(close, float(np.float32(1.5) * np.float32(5.991)), float(np.float32(5.991))),
                   float(np.float32(7.815)))
    check_flags(got["outlier"], ref, thr)
    # float outputs are the casts of the double states
    assert np.array_equal(got["kfs"]["Rwb"], got["kfs21"][:, :9].astype(np.float32))
    assert np.array_equal(got["kfs"]["ba"], got["kfs21"][:, 18:21].astype(np.float32))
    for k in range(len(pb.kfs)):
        if pb.fixed[k]:
            assert np.array_equal(got["kfs"][k], pb.kfs[k])
    return got, ref


def test_lia_small_window(gpu_available):
    _compare(synth.lia_problem(5, n_opt=4, n_fixed_cov=2, n_pts=60, max_obs=4))


def test_lia_default_window(gpu_available):
    got, ref = _compare(synth.lia_problem())  # 10 temporal KF, 11 fixed, 2000 MP, ~16k edges
    assert got["stats"][1] < 0.6 * got["stats"][0]


def test_lia_large_mode(gpu_available):
    # bLarge: maxOpt 25, opt_it 4, user lambda 1e-2 (optimizer.cc:2334-2339, 2448-2452)
    _compare(synth.lia_problem(9, n_opt=25, n_fixed_cov=6, n_pts=1500, b_large=True))


def test_lia_rec_init(gpu_available):
    # bRecInit: every EdgeInertial robust (optimizer.cc:2571)
    _compare(synth.lia_problem(10, n_opt=6, n_pts=800, rec_init=True))


def test_lia_outlier_heavy(gpu_available):
    _compare(synth.lia_problem(12, n_opt=8, n_pts=1000, outlier_frac=0.2))


def test_lia_vertex_pose_only_keyframes(gpu_available):
    """Free key frames without IMU data (`!pKFi->bImu`: VertexPose only,
    optimizer.cc:2466-2484; no EdgeInertial touches them, :2503) on the
    device, against the oracle that gives them 6 rows: same LM path, states
    within tolerance, their velocity and biases untouched."""
    pb = synth.lia_problem(16, n_opt=8, n_fixed_cov=3, n_pts=900, no_imu=(2, 5))
    assert len(pb.imu_edges) == 8 - 4
    got, _ = _compare(pb)
    for k in (2, 5):
        for f in ("v", "bg", "ba"):
            assert np.array_equal(got["kfs"][f][k], pb.kfs[f][k])


def test_lia_many_links_grid_solver(gpu_available):
    """72 temporal key frames (71 IMU links, past the round-3 64-link bound; a
    1080-row reduced system on the device-wide solver) with two VertexPose-only
    key frames, against the oracle."""
    pb = synth.lia_problem(17, n_opt=72, n_fixed_cov=4, n_pts=1500, max_obs=3, max_depth=10.0,
                           consecutive=True, no_imu=(30, 31))
    assert len(pb.imu_edges) > 64
    _compare(pb)


def test_lia_then_lba_on_one_context(gpu_available):
    """Both windows share the context's arena: an LBA call after a LocalInertialBA
    call (and back) gives the standalone results."""
    adj = LocalBundleAdjuster()
    pl = synth.lba_problem(seed=5, n_kf=5, n_pts=40, obs_per_pt=3, n_fixed=1)
    pi = synth.lia_problem(5, n_opt=4, n_fixed_cov=2, n_pts=60, max_obs=4)
    a1 = adj.optimize_inertial(pi)
    b1 = adj.optimize(pl)
    a2 = adj.optimize_inertial(pi)
    b2 = LocalBundleAdjuster().optimize(pl)
    assert np.array_equal(a1["kfs21"], a2["kfs21"]) and np.array_equal(a1["outlier"], a2["outlier"])
    assert np.array_equal(b1["poses_d"], b2["poses_d"])


def test_lia_trial_terms_equal_relinearised(gpu_available):
    """The accepted trial's visual terms and IMU link forms (written while the
    trial is evaluated) equal a fresh linearisation at the accepted state
    (orbgpu_lba_ctx_set_relinearize): bit-identical runs."""
    pb = synth.lia_problem()
    spec = LocalBundleAdjuster().optimize_inertial(pb)
    adj = LocalBundleAdjuster()
    adj.set_relinearize(True)
    relin = adj.optimize_inertial(pb)
    for k in ("stats", "kfs21", "pts", "outlier"):
        assert np.array_equal(spec[k], relin[k]), k


def test_lia_trial_states_past_lds_table(gpu_available):
    """More key frames than the trial kernel stages in LDS (kMaxKfImuLds =
    128): the trial states go through k_lia_trial_states, against the
    oracle."""
    pb = synth.lia_problem(18, n_opt=131, n_fixed_cov=2, n_pts=2000, max_obs=3, max_depth=10.0,
                           consecutive=True)
    assert len(pb.kfs) > 128
    _compare(pb)


def test_lia_zero_iterations(gpu_available):
    """iterations = 0: the results come from the one classify launch (no LM
    step is queued); states unchanged, flags and err as the oracle's."""
    pb = synth.lia_problem(6, n_opt=5, n_fixed_cov=3, n_pts=150, max_obs=4)
    got = LocalBundleAdjuster().optimize_inertial(pb, iterations=0)
    ref = oracle.lia(pb, iterations=0)
    assert got["stats"][2] == 0 and got["stats"][3] == 0
    assert abs(got["stats"][0] - ref["stats"][0]) <= 1e-8 * ref["stats"][0]
    assert np.array_equal(got["kfs"], np.ascontiguousarray(pb.kfs, got["kfs"].dtype))
    mono = pb.edges["ur"] < 0
    close = pb.close[pb.edges["point"]] != 0
    thr = np.where(mono, np.where(close, float(np.float32(1.5) * np.float32(5.991)), float(np.float32(5.991))),
                   float(np.float32(7.815)))
    check_flags(got["outlier"], ref, thr)


def test_lia_update_sizes_straddle_exp_branches(gpu_available):
    """free key frames whose initial rotation errors differ
    by four orders of magnitude, interleaved, so one trial's per-key-frame
    updates (one key frame per lane) straddle ExpSO3's d = 1e-5 and
    d^2 = 0.0025 branch points within a wave -- the case the round-3
    wave-uniform ExpSO3 got wrong."""
    scales = (1e-3, 25.0, 1.0) * 3 + (1e-3,)
    pb = synth.lia_problem(19, n_opt=10, n_fixed_cov=4, n_pts=1200, kf_rot_scale=scales)
    got, _ = _compare(pb)
    corr = []
    for k in range(10):
        M = got["kfs21"][k, :9].reshape(3, 3) @ pb.kfs["Rwb"][k].reshape(3, 3).astype(float).T
        corr.append(np.linalg.norm([M[2, 1] - M[1, 2], M[0, 2] - M[2, 0], M[1, 0] - M[0, 1]]) / 2)
    assert max(corr) > 0.1 and min(corr) < 1e-3, corr
