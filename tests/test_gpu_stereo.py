"""GPU parity: Frame::ComputeStereoMatches (frame.cc:828-986) on gfx950
against the CPU oracle (oracle/stereo_oracle.cc), bit-exact on every
mvuRight / mvDepth float, through both C-ABI entry points:
  * orbgpu_stereo_match (host path: the Frame's two extractor handles);
  * orbgpu_stereo_match_batch (frames of one extract_batch call).
Parity vs the reference itself is unpinned (no reference fixtures; the oracle
is cross-checked against tests/ref_py.py in test_stereo_cpu.py).
"""
import numpy as np
import pytest

import binding as oracle
from orb_slam_fusion_amd import OrbExtractor, compute_stereo_matches, synth

pytestmark = pytest.mark.gpu

FX, B = 435.2, 0.11
C2 = (1000, 1.2, 8, 20, 7)


def cam():
    bf = np.float32(FX * B)
    return bf, np.float32(bf / np.float32(FX))


def oracle_pair(left, right, params):
    exl, exr = oracle.OracleExtractor(*params), oracle.OracleExtractor(*params)
    _, kl, dl = exl.extract(left)
    _, kr, dr = exr.extract(right)
    L = params[2]
    p = exl.params()
    bf, mb = cam()
    ur, dep, _ = oracle.stereo_match(kl, dl, kr, dr, [exl.level(l) for l in range(L)],
                                     [exr.level(l) for l in range(L)], p["scale"], p["inv_scale"], bf, mb)
    return kl, ur, dep


def noisy(img, seed=1, amp=2):
    rng = np.random.default_rng(seed)
    return np.clip(img.astype(np.int32) + rng.integers(-amp, amp + 1, img.shape), 0, 255).astype(np.uint8)


def host_path(left, right, params):
    h, w = left.shape
    exl = OrbExtractor(*params, max_width=w, max_height=h)
    exr = OrbExtractor(*params, max_width=w, max_height=h)
    _, kl, _ = exl(left)
    exr(right)
    bf, mb = cam()
    ur, dep = compute_stereo_matches(exl, exr, len(kl), bf, mb)
    return kl, ur, dep


def assert_same(got, ref, ctx):
    kl_g, ur_g, dep_g = got
    kl_r, ur_r, dep_r = ref
    assert kl_g.tobytes() == kl_r.tobytes(), f"{ctx}: keypoints differ"
    bad = np.flatnonzero(ur_g.view(np.uint32) != ur_r.view(np.uint32))
    assert bad.size == 0, f"{ctx}: {bad.size} uR differ, first {bad[:5]}: {ur_g[bad[:5]]} vs {ur_r[bad[:5]]}"
    assert np.array_equal(dep_g.view(np.uint32), dep_r.view(np.uint32)), f"{ctx}: depth differs"


@pytest.mark.parametrize("frame", [0, 4, 9])
def test_host_path_bit_exact(gpu_available, frame):
    left, right = synth.stereo_frame(frame)
    got = host_path(left, right, C2)
    ref = oracle_pair(left, right, C2)
    assert_same(got, ref, f"frame {frame}")
    assert (got[1] >= 0).sum() > 300


def test_zero_disparity_clamp_and_median(gpu_available):
    left, _ = synth.stereo_frame(3)
    assert_same(host_path(left, noisy(left), C2), oracle_pair(left, noisy(left), C2), "noisy 0-disp")
    # identical images: every distance 0, the median filter drops all matches
    got = host_path(left, left.copy(), C2)
    assert (got[1] == -1).all()


@pytest.mark.parametrize("size,params", [((641, 397), C2), ((1024, 768), (1000, 1.6, 5, 20, 7)),
                                         ((752, 480), (1200, 1.2, 8, 20, 7))])
def test_other_geometries(gpu_available, size, params):
    w, h = size
    left, right = synth.stereo_frame(11, w=w, h=h)
    assert_same(host_path(left, right, params), oracle_pair(left, right, params), f"{size} {params}")


def test_batch_matches_oracle_per_frame(gpu_available):
    import torch

    F = 6
    pairs = [synth.stereo_frame(20 + f) for f in range(F - 1)]
    base, _ = synth.stereo_frame(30)
    pairs.append((base, noisy(base)))
    imgs = torch.from_numpy(np.stack([im for p in pairs for im in p])).cuda()
    ex = OrbExtractor(*C2, max_images=2 * F)
    cap = ex.max_keypoints(752, 480)
    kps = torch.zeros((2 * F, cap, 7), dtype=torch.int32, device="cuda")
    desc = torch.zeros((2 * F, cap, 32), dtype=torch.uint8, device="cuda")
    n = torch.zeros(2 * F, dtype=torch.int32, device="cuda")
    mono = torch.zeros(2 * F, dtype=torch.int32, device="cuda")
    ur = torch.zeros((F, cap), dtype=torch.float32, device="cuda")
    dep = torch.zeros((F, cap), dtype=torch.float32, device="cuda")
    ex.extract_batch(imgs, kps, desc, n, mono)
    bf, mb = cam()
    ex.stereo_match_batch(imgs, kps, desc, n, bf, mb, ur, dep)
    torch.cuda.synchronize()
    n_h = n.cpu().numpy()
    for f, (left, right) in enumerate(pairs):
        kl, ur_r, dep_r = oracle_pair(left, right, C2)
        N = int(n_h[2 * f])
        assert N == len(kl)
        got = (kl, ur[f, :N].cpu().numpy(), dep[f, :N].cpu().numpy())
        assert_same(got, (kl, ur_r, dep_r), f"batch frame {f}")


def test_more_than_4096_right_keypoints(gpu_available):
    """Right keypoint indices past 4095: a dense-noise pair with a
    24 px disparity at 8000 features gives > 4096 keypoints per image, so the
    row candidates' indices need the full 16 bits of the match key."""
    canvas = synth.noise_image(41, 752 + 24, 480)
    left = np.ascontiguousarray(canvas[:, :752])
    right = np.ascontiguousarray(canvas[:, 24:])
    params = (8000, 1.2, 8, 20, 7)
    got = host_path(left, right, params)
    ref = oracle_pair(left, right, params)
    assert len(ref[0]) > 4096, len(ref[0])
    assert_same(got, ref, "8000 features, dense noise")
    assert (got[1] >= 0).sum() > 1000
