"""GPU LocalBundleAdjustment (orbgpu_lba_optimize) vs the oracle on the same
windows.  Floating point, so parity is by tolerance: the GPU sums in a
different (fixed) order and factors the reduced camera system by 16 x 16
MFMA tiles; poses and points agree to ~1e-6 relative, the LM path
(iterations, trials) agrees exactly, and so do the outlier flags of every
edge whose oracle chi2 is not within 1e-6 relative of its threshold.  The LM loop runs on the device (lba_kernels.hip): the stop flag,
the user lambda, the LDS / global solver paths and the point-sharded
two-rank run are each checked against the oracle or the one-rank result."""
import sys
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "oracle"))
sys.path.insert(0, str(REPO))

import binding as oracle  # noqa: E402
from orb_slam_fusion_amd import LocalBundleAdjuster, synth  # noqa: E402

pytestmark = pytest.mark.gpu


def _quat_sign(q, ref):
    return q if np.dot(q[:4], ref[:4]) >= 0 else np.concatenate([-q[:4], q[4:]])


# Outlier flags: identical on every edge except those whose oracle chi2 lies
# within CHI2_BAND (relative) of its threshold -- there the states' last-digit
# differences (poses agree to ~1e-12 relative) may decide the comparison.  The
# exempt set is listed and must stay tiny.
CHI2_BAND = 1e-6
MAX_EXEMPT = 3


def check_flags(got_out, ref, thr):
    near = np.abs(ref["chi2"] - thr) <= CHI2_BAND * thr
    diff = got_out != ref["outlier"]
    bad = np.nonzero(diff & ~near)[0]
    assert bad.size == 0, [(int(i), float(ref["chi2"][i]), float(thr[i])) for i in bad[:10]]
    exempt = np.nonzero(near)[0]
    print(f"exempt edges (chi2 within {CHI2_BAND:g} of the threshold): {exempt.tolist()}")
    assert exempt.size <= MAX_EXEMPT, exempt.tolist()


def _compare(p, iters=10, tol=1e-6, lambda_init=0.0, adj=None):
    ref = oracle.lba(p, iters=iters, lambda_init=lambda_init)
    got = (adj or LocalBundleAdjuster()).optimize(p, iterations=iters, lambda_init=lambda_init)
    assert got["stats"][2] == ref["stats"][2]  # LM iterations
    assert got["stats"][3] == ref["stats"][3]  # trials
    assert abs(got["stats"][1] - ref["stats"][1]) <= tol * ref["stats"][1]
    for k in range(len(p.poses_init)):
        g = _quat_sign(got["poses_d"][k], ref["poses"][k])
        assert np.allclose(g, ref["poses"][k], rtol=tol, atol=tol), k
    assert np.allclose(got["pts"], ref["pts"], rtol=1e-5, atol=1e-5)
    # optimizer.cc:1366-1401: chi2 > 5.991 (mono) / 7.815 (stereo), double literals
    check_flags(got["outlier"], ref, np.where(p.edges["ur"] < 0, 5.991, 7.815))
    return got, ref


def test_lba_small_window(gpu_available):
    _compare(synth.lba_problem(seed=5, n_kf=5, n_pts=40, obs_per_pt=3, n_fixed=1))


def test_lba_with_outliers(gpu_available):
    _compare(synth.lba_problem(seed=3, n_kf=8, n_pts=400, obs_per_pt=4, n_fixed=1, outlier_pct=10))


def test_lba_c4_window(gpu_available):
    got, ref = _compare(synth.lba_problem())  # 20 KF, 3000 MP, 18000 edges
    assert got["stats"][1] < got["stats"][0]


@pytest.mark.parametrize("order", ["shuffled", "one_swap"])
def test_lba_edges_in_any_order(gpu_available, order):
    # point-major input skips the layout's scatter (lba_api.cpp run_window);
    # any other order takes it: both against the oracle on the same edge list
    p = synth.lba_problem(seed=3, n_kf=8, n_pts=400, obs_per_pt=4, n_fixed=1, outlier_pct=10)
    if order == "shuffled":
        p.edges = p.edges[np.random.default_rng(11).permutation(len(p.edges))]
    else:  # sorted but for the last two edges of different points
        i = np.nonzero(np.diff(p.edges["point"]) > 0)[0][-1]
        idx = np.arange(len(p.edges))
        idx[[i, i + 1]] = idx[[i + 1, i]]
        p.edges = p.edges[idx]
    _compare(p)


def test_lba_window_past_2048_rows(gpu_available):
    """344 free key frames: a 2064-row reduced system (the HBM solve path; the
    round-2 API refused it) -- one LM iteration against the oracle."""
    _compare(synth.lba_problem(seed=21, n_kf=346, n_pts=3460, obs_per_pt=6, n_fixed=2), iters=1)


def test_lba_window_past_old_lds_bound(gpu_available):
    """1710 free key frames (a 10260-row reduced system: past the round-3 bound
    of 1706, where D and the right-hand side no longer fit LDS) on the
    device-wide solver -- one LM iteration against the oracle.  No window
    size is refused and no CPU code runs (the drop-in has no fallback)."""
    p = synth.lba_problem(seed=23, n_kf=1712, n_pts=4 * 1712, obs_per_pt=4, n_fixed=2)
    _compare(p, iters=1)


def test_lba_lds_path_at_its_bound(gpu_available):
    """26 free key frames: 156 rows, n_pad 160 -- the largest system the packed
    LDS solve takes (its dynamic block plus the kernel's static LDS within
    160 KB); 27 take the one-block HBM path."""
    from orb_slam_fusion_amd import _lib

    p = synth.lba_problem(seed=24, n_kf=28, n_pts=1400, obs_per_pt=5, n_fixed=2)
    got, _ = _compare(p)
    adj = LocalBundleAdjuster()
    adj.set_solver(_lib.ORBGPU_LBA_SOLVER_LDS)
    forced = adj.optimize(p)
    assert np.array_equal(forced["poses_d"], got["poses_d"])  # AUTO took the LDS path
    q = synth.lba_problem(seed=24, n_kf=29, n_pts=1400, obs_per_pt=5, n_fixed=2)
    with pytest.raises(_lib.OrbGpuError) as e:
        adj.optimize(q)  # 162 rows: past the LDS path
    assert e.value.status == _lib.ORBGPU_ERR_CAPACITY


@pytest.mark.parametrize("n_kf", [30, 60])
def test_lba_block_and_grid_solvers_identical(gpu_available, n_kf):
    """The one-workgroup HBM solve and the device-wide one run the same tile
    operations in the same order: bit-identical LM paths and states."""
    from orb_slam_fusion_amd import _lib

    p = synth.lba_problem(seed=25, n_kf=n_kf, n_pts=40 * n_kf, obs_per_pt=5, n_fixed=2)
    res = {}
    for mode in (_lib.ORBGPU_LBA_SOLVER_BLOCK, _lib.ORBGPU_LBA_SOLVER_GRID):
        adj = LocalBundleAdjuster()
        adj.set_solver(mode)
        res[mode] = adj.optimize(p)
    a, b = res[_lib.ORBGPU_LBA_SOLVER_BLOCK], res[_lib.ORBGPU_LBA_SOLVER_GRID]
    assert np.array_equal(a["stats"], b["stats"])
    assert np.array_equal(a["poses_d"], b["poses_d"])
    assert np.array_equal(a["pts"], b["pts"])
    assert np.array_equal(a["outlier"], b["outlier"])
    _compare(p)


def test_lba_point_seen_by_many_keyframes(gpu_available):
    """Points observed by 390 free key frames (past the 8 edges a Schur thread
    looks up per batch: the lookup walks the rest in batches) -- one LM
    iteration against the oracle."""
    p = synth.lba_problem(seed=26, n_kf=392, n_pts=12, obs_per_pt=390, n_fixed=2)
    _compare(p, iters=1)


def test_lba_all_fixed_and_empty(gpu_available):
    p = synth.lba_problem(seed=4, n_kf=4, n_pts=50, obs_per_pt=3, n_fixed=4)
    got = LocalBundleAdjuster().optimize(p)
    ref = oracle.lba(p)
    assert np.allclose(got["pts"], ref["pts"], rtol=1e-5, atol=1e-5)
    assert np.allclose(got["poses"], p.poses_init)


def test_lba_zero_iterations_and_repeat(gpu_available):
    """iterations = 0: no LM step is queued, so one classify launch writes the
    results to host memory (the other calls get them from the k_lba_sums of
    the step queued behind the LM's end); then calls of different sizes on
    one context, each against the oracle (a call must never return an
    earlier call's results)."""
    lba = LocalBundleAdjuster()
    p = synth.lba_problem(seed=9, n_kf=6, n_pts=120, obs_per_pt=3, n_fixed=1)
    got = lba.optimize(p, iterations=0)
    ref = oracle.lba(p, iters=0)
    assert got["stats"][2] == 0 and got["stats"][3] == 0
    assert np.allclose(got["poses_d"], p.poses_init)
    check_flags(got["outlier"], ref, np.where(p.edges["ur"] < 0, 5.991, 7.815))
    for seed, n_kf, n_pts in ((10, 8, 300), (11, 5, 60), (10, 8, 300)):
        q = synth.lba_problem(seed=seed, n_kf=n_kf, n_pts=n_pts, obs_per_pt=3, n_fixed=1)
        g = lba.optimize(q)
        r = oracle.lba(q)
        assert g["stats"][3] == r["stats"][3]
        assert np.allclose(g["pts"], r["pts"], rtol=1e-5, atol=1e-5)
        check_flags(g["outlier"], r, np.where(q.edges["ur"] < 0, 5.991, 7.815))


def test_lba_stop_flag(gpu_available):
    import ctypes

    p = synth.lba_problem(seed=5, n_kf=5, n_pts=40, obs_per_pt=3, n_fixed=1)
    flag = ctypes.c_uint8(1)
    got = LocalBundleAdjuster().optimize(p, stop_flag=flag)
    assert got["stats"][2] == 0  # no LM iteration ran
    assert np.allclose(got["poses"], p.poses_init)


def test_lba_shard_with_identity_reduce_matches(gpu_available):
    """Whole window as one 'shard' through the reduce path (world size 1)."""
    import torch.distributed as dist

    from orb_slam_fusion_amd import dist as odist

    p = synth.lba_problem(seed=8, n_kf=6, n_pts=120, obs_per_pt=3, n_fixed=1)
    ref = LocalBundleAdjuster().optimize(p)
    if not dist.is_initialized():
        import os
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29611")
        dist.init_process_group("nccl", rank=0, world_size=1)
    got = LocalBundleAdjuster().optimize(p, group=dist.group.WORLD)
    odist.finalize()
    assert np.array_equal(got["poses_d"], ref["poses_d"])
    assert np.array_equal(got["pts"], ref["pts"])


def test_lba_ordered_reduce_world1_matches(gpu_available):
    """The stream-ordered sharded form (reductions enqueued on the library's
    stream over RCCL, the LM loop on the device) at world size 1: bit-identical
    to the plain call, LM path included."""
    import torch.distributed as dist

    from orb_slam_fusion_amd import dist as odist

    p = synth.lba_problem()
    ref = LocalBundleAdjuster().optimize(p)
    if not dist.is_initialized():
        import os
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29613")
        dist.init_process_group("nccl", rank=0, world_size=1)
    adj = LocalBundleAdjuster()
    got = adj.optimize(p, group=dist.group.WORLD, ordered=True)
    again = adj.optimize(p, group=dist.group.WORLD, ordered=True)  # the context reused
    odist.finalize()
    for g in (got, again):
        assert np.array_equal(g["stats"], ref["stats"])
        assert np.array_equal(g["poses_d"], ref["poses_d"])
        assert np.array_equal(g["pts"], ref["pts"])
        assert np.array_equal(g["outlier"], ref["outlier"])


def test_lba_inertial_map_user_lambda(gpu_available):
    """setUserLambdaInit(100.0) when the map is inertial (optimizer.cc:1137)."""
    got, ref = _compare(synth.lba_problem(seed=6, n_kf=10, n_pts=600, obs_per_pt=4, n_fixed=2),
                        lambda_init=100.0)
    assert got["stats"][3] == ref["stats"][3]


def test_lba_large_window_global_solver(gpu_available):
    """28 free keyframes: the 168 x 168 reduced system exceeds the LDS budget and
    is factorised from global memory (k_lba_solve<false>)."""
    _compare(synth.lba_problem(seed=9, n_kf=30, n_pts=1500, obs_per_pt=5, n_fixed=2))


def test_lba_many_fixed_keyframes(gpu_available):
    """More keyframes than the trial-pose LDS table holds (k_lba_trial_poses)."""
    _compare(synth.lba_problem(seed=10, n_kf=1100, n_pts=2200, obs_per_pt=3, n_fixed=1092))


def test_lba_stop_flag_mid_run(gpu_available):
    """*pbStopFlag flipped by another thread while optimize runs (LocalMapping's
    flag, set from Tracking, localmapping.cc:226).  The device reads it where g2o
    polls terminate(); the state must equal the oracle stopped after the same
    number of trials."""
    import ctypes
    import threading
    import time

    p = synth.lba_problem(seed=9, n_kf=30, n_pts=1500, obs_per_pt=5, n_fixed=2)
    lba = LocalBundleAdjuster()
    full = lba.optimize(p)
    t0 = time.perf_counter()
    lba.optimize(p)
    span = time.perf_counter() - t0
    seen = set()
    for frac in np.linspace(0.05, 0.95, 12):
        flag = ctypes.c_uint8(0)
        go = threading.Event()

        def flip(delay=frac * span, flag=flag, go=go):
            go.wait()
            time.sleep(delay)  # releases the GIL: the main thread is inside the C call
            flag.value = 1

        th = threading.Thread(target=flip)
        th.start()
        go.set()
        got = lba.optimize(p, stop_flag=flag)
        th.join()
        trials = int(got["stats"][3])
        seen.add(trials)
        ref = oracle.lba(p, stop_after_trials=trials)
        assert got["stats"][2] == ref["stats"][2] and got["stats"][3] == ref["stats"][3]
        for k in range(len(p.poses_init)):
            g = _quat_sign(got["poses_d"][k], ref["poses"][k])
            assert np.allclose(g, ref["poses"][k], rtol=1e-6, atol=1e-6), k
        assert np.allclose(got["pts"], ref["pts"], rtol=1e-5, atol=1e-5)
    assert any(0 < t < full["stats"][3] for t in seen), (seen, full["stats"][3])


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("ordered", [False, True])
def test_lba_ranks_one_gpu(gpu_available, tmp_path, ordered, world):
    """The point-sharded C4 window on 2 and 4 ranks (fresh child processes, all
    on cuda:0), partial reduced camera systems / chi2 / LM scale summed through
    lba.dist_reduce over gloo (optimizer.cc:1359-1360, block_solver.hpp:383-460
    split by points): the same LM path and state as the one-rank GPU run.
    ordered: the stream-ordered form (lba.dist_enqueue; gloo stages through
    the host), which must issue the same collective sequence on every rank."""
    import os
    import socket
    import subprocess

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    worker = REPO / "tools" / "lba_shard_worker.py"
    procs = [subprocess.Popen([sys.executable, str(worker), str(r), str(world), str(port), str(tmp_path),
                               "0", "1" if ordered else "0"], env=env) for r in range(world)]
    for pr in procs:
        assert pr.wait(timeout=100) == 0
    r = [np.load(tmp_path / f"r{k}.npz") for k in range(world)]
    p = synth.lba_problem()
    single = LocalBundleAdjuster().optimize(p)
    cut = r[0]["cut"]
    assert len(cut) == world + 1
    for k in range(world):
        assert (r[k]["poses_d"] == r[0]["poses_d"]).all()  # every rank solves the same system
        assert (r[k]["stats"][1:5] == r[0]["stats"][1:5]).all()
    assert r[0]["stats"][2] == single["stats"][2] and r[0]["stats"][3] == single["stats"][3]
    assert abs(r[0]["stats"][1] - single["stats"][1]) <= 1e-9 * single["stats"][1]
    assert np.allclose(r[0]["poses_d"], single["poses_d"], rtol=1e-9, atol=1e-12)
    pts = np.concatenate([r[k]["pts"][cut[k]:cut[k + 1]] for k in range(world)])
    assert np.allclose(pts, single["pts"], rtol=1e-6, atol=1e-6)
    owner = np.searchsorted(cut[1:], p.edges["point"], side="right")  # rank owning each edge's point
    outl = np.choose(owner, [r[k]["outlier"] for k in range(world)])
    assert (outl == single["outlier"]).all()


def _same(a, b):
    for k in ("stats", "poses_d", "pts", "outlier"):
        assert np.array_equal(a[k], b[k]), k


def test_lba_trial_terms_equal_relinearised(gpu_available):
    """An accepted trial leaves its state's per-edge terms for the next build
    (lin_of / LbaCtrl::lin_state); re-linearising every build instead
    (orbgpu_lba_ctx_set_relinearize) computes the same values: bit-identical runs."""
    p = synth.lba_problem(seed=31, n_kf=12, n_pts=900, obs_per_pt=5, n_fixed=2, outlier_pct=5)
    spec = LocalBundleAdjuster().optimize(p)
    adj = LocalBundleAdjuster()
    adj.set_relinearize(True)
    relin = adj.optimize(p)
    _same(spec, relin)
    assert spec["stats"][3] >= 3  # several accepted trials


@pytest.mark.parametrize("mode", ["split", "pair", "band"])
def test_lba_schur_paths(gpu_available, mode):
    """The Schur complement by point range (default), by pose pair and by
    point band (orbgpu_lba_ctx_set_schur; band falls back to pairs when a
    point spans more than 15 free key frames) each match the oracle and repeat
    bit for bit."""
    from orb_slam_fusion_amd import _lib

    m = {"split": _lib.ORBGPU_LBA_SCHUR_SPLIT, "pair": _lib.ORBGPU_LBA_SCHUR_PAIR,
         "band": _lib.ORBGPU_LBA_SCHUR_BAND}[mode]
    p = synth.lba_problem(seed=32)
    adj = LocalBundleAdjuster()
    adj.set_schur(m)
    got, _ = _compare(p, adj=adj)
    _same(got, adj.optimize(p))


def test_lba_memory_limit_nomem(gpu_available):
    """a window past the context's device-memory budget returns
    ORBGPU_ERR_NOMEM before any device work, and the context stays usable
    (the same window then matches a fresh context bit for bit)."""
    from orb_slam_fusion_amd._lib import ORBGPU_ERR_NOMEM, OrbGpuError

    p = synth.lba_problem(seed=7, n_kf=8, n_pts=400, obs_per_pt=4, n_fixed=2)
    adj = LocalBundleAdjuster()
    adj.set_memory_limit(4096)
    with pytest.raises(OrbGpuError) as e:
        adj.optimize(p)
    assert e.value.status == ORBGPU_ERR_NOMEM
    adj.set_memory_limit(0)
    _same(adj.optimize(p), LocalBundleAdjuster().optimize(p))
