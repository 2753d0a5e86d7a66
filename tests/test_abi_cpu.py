"""CPU checks of the C ABI library (no compute calls: there is no GPU here).

* liborbgpu.so loads and exports every function include/orbgpu.h declares;
* the binding's signature table covers exactly those functions;
* argument validation that happens before any HIP call returns the
  documented status codes;
* the library contains gfx950 code objects and no CPU fallback symbols.
"""
import ctypes
import re
import subprocess
from pathlib import Path

import numpy as np
import pytest

from orb_slam_fusion_amd import _lib

REPO = Path(__file__).resolve().parents[1]
HEADER = REPO / "include" / "orbgpu.h"


def declared_functions():
    text = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    return sorted(set(re.findall(r"\b(orbgpu_\w+)\s*\(", text)))


def test_header_declares_expected_entry_points():
    names = declared_functions()
    for must in ["orbgpu_extractor_create", "orbgpu_extract", "orbgpu_extract_batch",
                 "orbgpu_extractor_pyramid_level", "orbgpu_pose_opt", "orbgpu_pose_opt_batch"]:
        assert must in names


def test_library_exports_every_declared_symbol():
    so = _lib.lib()
    missing = [n for n in declared_functions() if not hasattr(so, n)]
    assert not missing, missing


def test_binding_table_matches_header():
    assert sorted(_lib.SIGNATURES) == declared_functions()


def test_exported_symbols_are_c_linkage():
    out = subprocess.run(["nm", "-D", "--defined-only", str(_lib.library_path())],
                         capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (orbgpu_\w+)", out))
    assert set(declared_functions()) <= exported


def test_library_carries_gfx950_code_object():
    data = _lib.library_path().read_bytes()
    assert b"gfx950" in data


def test_invalid_params_rejected_before_device():
    so = _lib.lib()
    h = ctypes.c_void_p()
    bad = _lib.OrbParams(1000, 1.0, 8, 20, 7)  # scale_factor must be > 1
    assert so.orbgpu_extractor_create(ctypes.byref(bad), 0, 752, 480, 1, ctypes.byref(h)) == \
        _lib.ORBGPU_ERR_INVALID
    too_small = _lib.OrbParams(1000, 1.2, 8, 20, 7)
    assert so.orbgpu_extractor_create(ctypes.byref(too_small), 0, 100, 80, 1, ctypes.byref(h)) == \
        _lib.ORBGPU_ERR_INVALID
    assert so.orbgpu_extract(None, None, 0, 0, 0, None, None, None, 0, None, None) == \
        _lib.ORBGPU_ERR_INVALID
    assert so.orbgpu_pose_opt(None, None, None, None, 0, None, None, None) == _lib.ORBGPU_ERR_INVALID
    assert so.orbgpu_pose_ctx_set_trial_groups(None, 1, 1) == _lib.ORBGPU_ERR_INVALID
    # inertial entry points: null handle / bad mode / missing prior rejected before any device work
    assert so.orbgpu_pose_inertial(None, 0, None, None, None, None, None, None, 0, 0, None,
                                   None) == _lib.ORBGPU_ERR_INVALID
    assert so.orbgpu_pose_inertial_batch(None, 0, None, 1, None, None, None, None, None, None, 8,
                                         0, None, None, None) == _lib.ORBGPU_ERR_INVALID
    assert so.orbgpu_inertial_ctx_create(0, 0, 16, ctypes.byref(h)) == _lib.ORBGPU_ERR_INVALID


def test_inertial_mode_and_prior_checked_with_a_handle():
    """The mode / prior / n_obs checks of inertial_api.cpp run with a non-null
    handle: they return before the handle is dereferenced or the device is
    touched, so a dummy address exercises them on the CPU."""
    so = _lib.lib()
    dummy = ctypes.c_void_p(0x1000)  # never dereferenced on these paths
    calib = ctypes.create_string_buffer(256)
    ctypes.memmove(calib, np.array([1.0, 1.0], np.float32).tobytes(), 8)  # fx, fy > 0
    cur, prev, pre, prior, res = (ctypes.create_string_buffer(4096) for _ in range(5))
    obs, out = ctypes.create_string_buffer(64), ctypes.create_string_buffer(8)
    INV = _lib.ORBGPU_ERR_INVALID
    # bad mode
    assert so.orbgpu_pose_inertial(dummy, 5, calib, cur, prev, pre, prior, obs, 1, 0, res, out) == INV
    assert so.orbgpu_pose_inertial_batch(dummy, 5, calib, 1, cur, prev, pre, prior, obs, obs, 8, 0,
                                         res, out, None) == INV
    # LAST_FRAME (mode 0) without a prior
    assert so.orbgpu_pose_inertial(dummy, 0, calib, cur, prev, pre, None, obs, 1, 0, res, out) == INV
    assert so.orbgpu_pose_inertial_batch(dummy, 0, calib, 1, cur, prev, pre, None, obs, obs, 8, 0,
                                         res, out, None) == INV
    # negative observation count, observations without an outlier buffer
    assert so.orbgpu_pose_inertial(dummy, 1, calib, cur, prev, pre, None, obs, -1, 0, res, out) == INV
    assert so.orbgpu_pose_inertial(dummy, 1, calib, cur, prev, pre, None, obs, 1, 0, res, None) == INV
    # a calibration with fx <= 0
    zero = ctypes.create_string_buffer(256)
    assert so.orbgpu_pose_inertial(dummy, 1, zero, cur, prev, pre, None, obs, 1, 0, res, out) == INV


def test_local_inertial_ba_checked_with_a_handle():
    """orbgpu_lia_optimize's argument checks (lba_api.cpp) return before the
    context is dereferenced: a link to a key frame without IMU vertices (free
    or fixed: optimizer.cc:2503 adds an EdgeInertial only between two bImu
    key frames), a self link and a non-positive user lambda are INVALID.  A
    free key frame without IMU vertices and no link is valid (VertexPose
    only), and so is any link count -- tests/test_gpu_lia.py runs both."""
    from orb_slam_fusion_amd import synth
    from orb_slam_fusion_amd.lba import LocalBundleAdjuster

    so = _lib.lib()
    pb = synth.lia_problem(3, n_opt=3, n_fixed_cov=1, n_pts=20, max_obs=3)
    adj = LocalBundleAdjuster.__new__(LocalBundleAdjuster)  # no device context
    adj._h = ctypes.c_void_p(0x1000)  # never dereferenced on these paths
    INV = _lib.ORBGPU_ERR_INVALID

    def status(**over):
        import copy
        q = copy.deepcopy(pb)
        for k, v in over.items():
            setattr(q, k, v)
        try:
            adj.optimize_inertial(q)
        except _lib.OrbGpuError as e:
            return e.status
        return _lib.ORBGPU_OK

    try:
        imu = pb.imu.copy()
        imu[0] = 0  # a free key frame that link 0 still touches
        assert status(imu=imu) == INV
        imu = pb.imu.copy()
        imu[int((pb.fixed == 0).sum())] = 0  # the key frame before the window (a link's kf1)
        assert status(imu=imu) == INV
        links = pb.imu_edges.copy()
        links[0]["kf1"] = links[0]["kf2"]
        assert status(imu_edges=links) == INV
        assert status(lambda_init=0.0) == INV
        assert so.orbgpu_lia_optimize(None, None, 0, None, None, None, 0, None, None, 0, None, 0,
                                      None, 10, 1.0, None, None, None, None, None) == INV
    finally:
        adj._h = ctypes.c_void_p()


def test_keypoint_struct_is_cv_keypoint_layout():
    assert _lib.KEYPOINT_DTYPE.itemsize == 28
    assert list(_lib.KEYPOINT_DTYPE.names) == ["x", "y", "size", "angle", "response", "octave",
                                               "class_id"]


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    monkeypatch.setenv("ORBGPU_LIB", str(tmp_path / "nope.so"))
    monkeypatch.setattr(_lib, "_lib", None)
    with pytest.raises(OSError, match="no CPU fallback"):
        _lib.lib()


def _plan(params, w, h):
    so = _lib.lib()
    slots, hbm = ctypes.c_int(-1), ctypes.c_int(-1)
    st = so.orbgpu_extractor_plan(ctypes.byref(_lib.OrbParams(*params)), w, h,
                                  ctypes.byref(slots), ctypes.byref(hbm))
    return st, slots.value, hbm.value


@pytest.mark.parametrize("size", [(752, 480), (1241, 376), (640, 480), (1024, 768)])
def test_plan_accepts_every_reference_extractor(size):
    """no (num_features, scale <= 2, levels <= 16) the
    reference constructs is refused -- including OrbExtractor(5 * nFeatures,
    ...) (tracking.cc:202-204,811-813) and budgets far past any LDS.  Only
    geometries whose smallest level cannot hold the FAST grid are skipped
    (the reference divides by a zero cell count there, orb_extractor.cc:748-760)."""
    w, h = size
    for nf in (1, 100, 1000, 1200, 2000, 5000, 6000, 10000, 20000, 60000):
        for sf in (1.1, 1.2, 1.5, 2.0):
            for L in (1, 4, 8, 12, 16):
                if min(w, h) / sf ** (L - 1) < 80:
                    continue  # the smallest level would not hold the grid
                st, slots, hbm = _plan((nf, sf, L, 20, 7), w, h)
                assert st == _lib.ORBGPU_OK, (nf, sf, L, size)
                assert slots >= nf, (nf, sf, L, size, slots)
                assert hbm in (0, 1)


def test_plan_octree_storage_policy():
    """The octree's node arrays stay in LDS up to the reference's 5x
    extractor at EuRoC / KITTI sizes and go to HBM only beyond it."""
    assert _plan((1000, 1.2, 8, 20, 7), 752, 480)[2] == 0
    assert _plan((5000, 1.2, 8, 20, 7), 752, 480)[2] == 0
    assert _plan((6000, 1.2, 8, 20, 7), 1241, 376)[2] == 0
    st, slots, hbm = _plan((20000, 1.2, 8, 20, 7), 1241, 376)
    assert st == _lib.ORBGPU_OK and hbm == 1 and slots >= 20000


def test_plan_refuses_degenerate_geometry():
    assert _plan((1000, 1.2, 8, 20, 7), 60, 60)[0] == _lib.ORBGPU_ERR_INVALID
    assert _plan((1000, 1.0, 8, 20, 7), 752, 480)[0] == _lib.ORBGPU_ERR_INVALID
    assert _lib.lib().orbgpu_extractor_plan(None, 752, 480, None, None) == _lib.ORBGPU_ERR_INVALID
