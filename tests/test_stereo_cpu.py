"""CPU checks of the stereo-matching oracle (oracle/stereo_oracle.cc,
Frame::ComputeStereoMatches frame.cc:828-986).

The reference ships no stereo fixtures, so this row's parity is
unpinned against the reference itself; the C restatement is cross-checked here
against the independent numpy restatement tests/ref_py.py:stereo_match_py on
synthetic rectified pairs (known 24 px disparity), including the 0-disparity
clamp branch and a frame whose matches all fall to the median filter's side.
"""
import sys
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "oracle"))
sys.path.insert(0, str(REPO))

import binding as oracle  # noqa: E402
import ref_py  # noqa: E402
from orb_slam_fusion_amd import synth  # noqa: E402

FX, B = 435.2, 0.11


def cam():
    bf = np.float32(FX * B)
    return bf, np.float32(bf / np.float32(FX))


def extract_pair(left, right, params=(1000, 1.2, 8, 20, 7)):
    exl, exr = oracle.OracleExtractor(*params), oracle.OracleExtractor(*params)
    _, kl, dl = exl.extract(left)
    _, kr, dr = exr.extract(right)
    L = params[2]
    return (kl, dl, kr, dr, [exl.level(l) for l in range(L)], [exr.level(l) for l in range(L)],
            exl.params())


def run_both(left, right, params=(1000, 1.2, 8, 20, 7)):
    kl, dl, kr, dr, pl, pr, p = extract_pair(left, right, params)
    bf, mb = cam()
    ur, dep, kept = oracle.stereo_match(kl, dl, kr, dr, pl, pr, p["scale"], p["inv_scale"], bf, mb)
    ur2, dep2 = ref_py.stereo_match_py(kl, dl, kr, dr, pl, pr, p["scale"], p["inv_scale"], bf, mb)
    return kl, ur, dep, kept, ur2, dep2


@pytest.mark.parametrize("frame", [0, 7])
def test_oracle_matches_numpy_restatement(frame):
    left, right = synth.stereo_frame(frame)
    kl, ur, dep, kept, ur2, dep2 = run_both(left, right)
    assert np.array_equal(ur.view(np.uint32), ur2.view(np.uint32))
    assert np.array_equal(dep.view(np.uint32), dep2.view(np.uint32))
    m = ur >= 0
    assert kept == m.sum() > 0.3 * len(kl)
    # the synthetic pair is a 24 px shift: sub-pixel disparities land on it
    assert abs(np.median(kl["x"][m] - ur[m]) - 24) < 0.1
    bf, _ = cam()
    assert np.allclose(dep[m], bf / (kl["x"][m] - ur[m]), rtol=1e-5)


def right_with_noise(img, seed=1, amp=2):
    rng = np.random.default_rng(seed)
    return np.clip(img.astype(np.int32) + rng.integers(-amp, amp + 1, img.shape), 0, 255).astype(np.uint8)


def test_zero_disparity_clamp_branch():
    # 0-disparity pair with small noise: window distances > 0 (identical images
    # give all-zero distances and the median filter drops every match), and
    # some parabolas are flat (d1 == d3) -> disparity exactly 0
    left, _ = synth.stereo_frame(3)
    kl, ur, dep, kept, ur2, dep2 = run_both(left, right_with_noise(left))
    assert np.array_equal(ur.view(np.uint32), ur2.view(np.uint32))
    assert np.array_equal(dep.view(np.uint32), dep2.view(np.uint32))
    m = ur >= 0
    clamped = np.isclose(dep[m], cam()[0] / np.float32(0.01))
    assert clamped.any()
    # disparity <= 0 -> 0.01 (frame.cc:955-958): uR = uL - 0.01 in double
    assert np.array_equal(ur[m][clamped], (kl["x"][m][clamped].astype(np.float64) - 0.01).astype(np.float32))


def test_identical_images_lose_every_match_to_the_median_filter():
    left, _ = synth.stereo_frame(3)
    kl, ur, dep, kept, ur2, dep2 = run_both(left, left.copy())
    assert kept == 0 and (ur == -1).all() and (ur2 == -1).all()


def test_no_right_keypoints_leaves_everything_unmatched():
    left, right = synth.stereo_frame(1)
    kl, dl, kr, dr, pl, pr, p = extract_pair(left, right)
    bf, mb = cam()
    ur, dep, kept = oracle.stereo_match(kl, dl, kr[:0], dr[:0], pl, pr, p["scale"], p["inv_scale"], bf, mb)
    assert kept == 0 and (ur == -1).all() and (dep == -1).all()


def test_median_filter_drops_the_tail():
    left, right = synth.stereo_frame(2)
    kl, dl, kr, dr, pl, pr, p = extract_pair(left, right)
    bf, mb = cam()
    # noise on the right image raises the window distances of part of the matches
    rng = np.random.default_rng(5)
    noisy = right.astype(np.int32) + rng.integers(-40, 41, right.shape) * (rng.random(right.shape) < 0.3)
    noisy = np.clip(noisy, 0, 255).astype(np.uint8)
    exr = oracle.OracleExtractor(1000, 1.2, 8, 20, 7)
    _, kr2, dr2 = exr.extract(noisy)
    pr2 = [exr.level(l) for l in range(8)]
    ur, dep, kept = oracle.stereo_match(kl, dl, kr2, dr2, pl, pr2, p["scale"], p["inv_scale"], bf, mb)
    ur2, dep2 = ref_py.stereo_match_py(kl, dl, kr2, dr2, pl, pr2, p["scale"], p["inv_scale"], bf, mb)
    assert np.array_equal(ur.view(np.uint32), ur2.view(np.uint32))
    assert kept > 0
