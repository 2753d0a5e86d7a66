"""GPU parity: the gfx950 extractor against the CPU oracle, bit-exact.

Every keypoint field (cv::KeyPoint layout), every descriptor byte, the mono
index and every pyramid level must equal the oracle's on the same seeded
input.  On a mismatch the stage buffers (blurred level, FAST candidates,
octree output) are compared to name the first diverging stage.
"""
import ctypes

import numpy as np
import pytest

import binding as oracle
from orb_slam_fusion_amd import OrbExtractor, synth
from orb_slam_fusion_amd._lib import lib, ptr

pytestmark = pytest.mark.gpu

C2 = (1000, 1.2, 8, 20, 7)      # BASELINE config 2 (ORBextractor only)
EUROC = (1200, 1.2, 8, 20, 7)   # settings/EuRoC.yaml:85-98


def _stage(ex, which, lev, cap=1 << 20):
    buf = np.zeros(cap, np.uint32)
    n = lib().orbgpu_extractor_stage(ex._h, which, lev, ptr(buf), cap * 4 if which == 0 else cap)
    assert n >= 0
    if which == 0:
        return buf.view(np.uint8)[:n]
    return buf[:n]


def _unpack(u32):
    return np.stack([(u32 & 0xFFF), (u32 >> 12) & 0xFFF, u32 >> 24], 1).astype(np.float32)


def _diagnose(ex, orc, L):
    lines = []
    for lev in range(L):
        ob = orc.level(lev, blurred=True)
        gb = _stage(ex, 0, lev)
        if gb.size == ob.size and not np.array_equal(gb.reshape(ob.shape), ob):
            lines.append(f"level {lev}: blurred plane differs")
        oc = orc.stage(lev, 0)
        gc = _unpack(_stage(ex, 1, lev))
        if not np.array_equal(oc, gc):
            lines.append(f"level {lev}: FAST candidates differ (oracle {len(oc)}, gpu {len(gc)})")
            continue
        oo = orc.stage(lev, 1)
        go = _unpack(_stage(ex, 2, lev))
        if not np.array_equal(oo, go):
            lines.append(f"level {lev}: octree output differs (oracle {len(oo)}, gpu {len(go)})")
    return "; ".join(lines) or "stages equal"


def _compare(params, img, lapping=(0, 0), rounding=None, octree_hbm=False, fused=False, single=0):
    h, w = img.shape
    ex = OrbExtractor(*params, max_width=w, max_height=h)
    ex.set_single_launch(single)  # 0: ORBGPU_SINGLE_DATAFLOW (default), 1: ORBGPU_SINGLE_GRAPH
    if fused:
        ex.set_pyramid_launch(1)  # ORBGPU_PYRAMID_FUSED
    if rounding is not None:
        ex.set_resize_rounding(rounding)
    if octree_hbm:
        ex.set_octree_nodes(1)  # ORBGPU_OCTREE_NODES_HBM
    orc = oracle.OracleExtractor(*params)
    if rounding is None:
        m_ref, k_ref, d_ref = orc.extract(img, lapping)
    else:
        with oracle.resize_rounding(rounding):  # the oracle's levels follow the same split
            m_ref, k_ref, d_ref = orc.extract(img, lapping)
    m, k, d = ex(img, None, lapping)
    ctx = (f"{w}x{h} params={params} lapping={lapping} rounding={rounding} octree_hbm={octree_hbm} "
           f"fused={fused} single={single}")
    # the reference blurs only levels that kept keypoints (orb_extractor.cc
    # operator(): `if (nkeypointsLevel == 0) continue;`), the GPU every level
    ref_levels = set(k_ref["octave"].tolist())
    for lev, lvl in enumerate(ex.img_pyramid_):
        assert np.array_equal(lvl, orc.level(lev)), f"{ctx}: pyramid level {lev} differs"
        if lev in ref_levels:
            ob = orc.level(lev, blurred=True)
            assert np.array_equal(_stage(ex, 0, lev).reshape(ob.shape), ob), f"{ctx}: blurred level {lev} differs"
    if len(k) != len(k_ref) or k.tobytes() != k_ref.tobytes() or (
        len(k) and d.tobytes() != d_ref.tobytes()
    ):
        diag = _diagnose(ex, orc, params[2])
        nk = min(len(k), len(k_ref))
        bad_k = int(np.sum(k[:nk].view(np.uint8).reshape(nk, 28) != k_ref[:nk].view(np.uint8).reshape(nk, 28)))
        bad_d = int(np.sum(d[:nk] != d_ref[:nk])) if nk and d is not None else -1
        pytest.fail(f"{ctx}: n gpu {len(k)} ref {len(k_ref)}, differing kp bytes {bad_k}, "
                    f"desc bytes {bad_d}; {diag}")
    assert m == m_ref, f"{ctx}: mono index {m} != {m_ref}"
    return len(k)


@pytest.mark.parametrize("frame", [0, 1, 2])
def test_stereo_frame_c2_bit_exact(gpu_available, frame):
    left, right = synth.stereo_frame(frame)
    assert _compare(C2, left) > 900
    assert _compare(C2, right) > 900


def test_euroc_params_bit_exact(gpu_available):
    left, _ = synth.stereo_frame(10)
    assert _compare(EUROC, left) > 1100


@pytest.mark.parametrize("rounding", [0, 1])  # ORBGPU_RESIZE_SSE, ORBGPU_RESIZE_SCALAR
def test_resize_rounding_switch(gpu_available, rounding):
    """the resize vertical pass's column split is one switch; both
    settings bit-exact against the oracle under the same setting, and the two
    pyramids differ (the switch reaches the kernel)."""
    left, _ = synth.stereo_frame(4)
    assert _compare(C2, left, rounding=rounding) > 900
    ex = OrbExtractor(*C2)
    ex.set_resize_rounding(rounding)
    ex(left, None, (0, 0))
    a = [l.copy() for l in ex.img_pyramid_]
    ex.set_resize_rounding(1 - rounding)
    ex(left, None, (0, 0))
    assert any(not np.array_equal(x, y) for x, y in zip(a, ex.img_pyramid_))


def test_lapping_partition(gpu_available):
    left, _ = synth.stereo_frame(3)
    _compare(C2, left, lapping=(200, 500))


def test_noise_image_dense_fast(gpu_available):
    img = synth.noise_image(99, 320, 256)
    _compare((500, 1.2, 4, 20, 7), img)


@pytest.mark.parametrize("size", [(641, 397), (1024, 768), (400, 300)])
def test_odd_sizes(gpu_available, size):
    w, h = size
    full, _ = synth.stereo_frame(20, w=w, h=h)
    L = 8 if min(w, h) >= 300 else 6
    _compare((1000, 1.2, L, 20, 7), full)


@pytest.mark.parametrize("size", [(400, 101), (101, 101), (752, 136)])
def test_tall_and_wide_cells(gpu_available, size):
    """Cells up to 69 px (one or two cells across a level: ceil(span / n) with
    n = span // 35): ROIs of 75 rows take k_fast_cells' clamped multi-step
    ROI load, 75 columns its per-cell-pitch instance; the 752 x 136 levels mix
    one-step and clamped ROIs (orb_extractor.cc:783-801 cell geometry)."""
    w, h = size
    full, _ = synth.stereo_frame(21, w=w, h=h)
    _compare((300, 1.2, 2, 20, 7), full)


@pytest.mark.parametrize("params", [(1000, 1.6, 5, 20, 7), (1000, 1.5, 6, 20, 7), (1000, 2.0, 4, 20, 7)])
def test_large_scale_factors(gpu_available, params):
    # coarser pyramids: wider resize tap spans, fewer and smaller levels
    full, _ = synth.stereo_frame(21, w=1024, h=768)
    _compare(params, full)


def test_low_contrast_uses_min_threshold(gpu_available):
    # contrast below iniThFAST everywhere: every cell falls back to minThFAST
    left, _ = synth.stereo_frame(5)
    low = (left.astype(np.int32) // 4 + 64).astype(np.uint8)
    _compare(C2, low)


def test_flat_image_no_keypoints(gpu_available):
    img = np.full((480, 752), 128, np.uint8)
    ex = OrbExtractor(*C2)
    m, k, d = ex(img)
    assert m == 0 and len(k) == 0 and d is None


def test_empty_image_returns_minus_one(gpu_available):
    ex = OrbExtractor(*C2)
    m, k, d = ex(np.zeros((0, 0), np.uint8))
    assert m == -1 and len(k) == 0 and d is None


def test_getters_match_oracle(gpu_available):
    ex = OrbExtractor(*EUROC)
    p = oracle.OracleExtractor(*EUROC).params()
    assert np.array_equal(ex.GetScaleFactors(), p["scale"])
    assert np.array_equal(ex.GetInverseScaleFactors(), p["inv_scale"])
    assert np.array_equal(ex.GetScaleSigmaSquares(), p["sigma2"])
    assert np.array_equal(ex.GetInverseScaleSigmaSquares(), p["inv_sigma2"])
    assert ex.GetLevels() == 8


def _batch_matches_single(fused):
    import torch

    B = 6
    imgs = np.stack([synth.stereo_frame(i // 2)[i % 2] for i in range(B)])
    ex = OrbExtractor(*C2, max_images=B)
    if fused:
        ex.set_pyramid_launch(1)
    cap = ex.max_keypoints(752, 480)
    d_imgs = torch.from_numpy(imgs).cuda()
    kps = torch.zeros((B, cap, 7), dtype=torch.int32, device="cuda")
    desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device="cuda")
    n = torch.zeros(B, dtype=torch.int32, device="cuda")
    mono = torch.zeros(B, dtype=torch.int32, device="cuda")
    ex.extract_batch(d_imgs, kps, desc, n, mono)
    torch.cuda.synchronize()
    ex.check()
    kps_h, desc_h, n_h, mono_h = kps.cpu().numpy(), desc.cpu().numpy(), n.cpu().numpy(), mono.cpu().numpy()
    orc = oracle.OracleExtractor(*C2)
    for i in range(B):
        m_ref, k_ref, d_ref = orc.extract(imgs[i])
        assert n_h[i] == len(k_ref) and mono_h[i] == m_ref
        assert kps_h[i, : n_h[i]].tobytes() == k_ref.tobytes(), f"image {i} keypoints"
        assert desc_h[i, : n_h[i]].tobytes() == d_ref.tobytes(), f"image {i} descriptors"


def test_batch_matches_single(gpu_available):
    _batch_matches_single(False)


def test_repeat_calls_deterministic(gpu_available):
    left, _ = synth.stereo_frame(7)
    ex = OrbExtractor(*C2)
    r1 = ex(left)
    r2 = ex(left)
    assert r1[0] == r2[0] and r1[1].tobytes() == r2[1].tobytes() and r1[2].tobytes() == r2[2].tobytes()


def test_graph_replay_across_sizes(gpu_available):
    """The host path replays a captured hipGraph once a launch repeats; a
    handle alternating between sizes (752x480 and its transpose 480x752 have
    the same byte count) must give each size's own result every time --
    compared with fresh handles, whose first call runs eagerly."""
    rng = np.random.default_rng(3)
    imgs = {(480, 752): synth.stereo_frame(3)[0],
            (752, 480): np.ascontiguousarray(synth.stereo_frame(4)[0].T),
            (400, 640): rng.integers(0, 255, (400, 640), dtype=np.uint8)}
    ref = {}
    for hw, im in imgs.items():
        r = OrbExtractor(*C2, max_width=800, max_height=800)(im)
        ref[hw] = (r[0], r[1].tobytes(), r[2].tobytes())
    ex = OrbExtractor(*C2, max_width=800, max_height=800)
    for hw in [(480, 752), (480, 752), (480, 752), (752, 480), (752, 480), (752, 480), (480, 752),
               (400, 640), (400, 640), (480, 752), (752, 480)]:
        r = ex(imgs[hw])
        assert (r[0], r[1].tobytes(), r[2].tobytes()) == ref[hw], hw


@pytest.mark.parametrize("kind", ["checker", "salt", "stripes"])
def test_saturated_patterns_bit_exact(gpu_available, kind):
    """Full-swing bytes: circle differences of +-255 through the f16 score
    (1024 + b is exact up to 2047), scores at 254, ties everywhere in the
    NMS and the octree, the reflected borders of resize and blur."""
    rng = np.random.default_rng(11)
    h, w = 480, 752
    y, x = np.mgrid[0:h, 0:w]
    if kind == "checker":
        img = np.where(((x // 5) + (y // 7)) % 2 == 0, 0, 255).astype(np.uint8)
    elif kind == "salt":
        img = np.where(rng.random((h, w)) < 0.03, 255, 0).astype(np.uint8)
    else:
        img = np.where((x + 2 * y) % 11 < 3, 255, 0).astype(np.uint8)
    _compare(C2, img)


def test_handles_with_different_plans_coexist(gpu_available):
    """The dynamic-LDS opt-in is a per-kernel attribute: creating a handle with
    a small octree (few features) after one with a large octree must not
    shrink the limit the first handle's launches need."""
    left, _ = synth.stereo_frame(8)
    big = OrbExtractor(4000, 1.2, 8, 20, 7)
    ref = big(left)
    small = OrbExtractor(300, 1.2, 8, 20, 7)
    small(left)
    again = big(left)
    assert ref[0] == again[0] and ref[1].tobytes() == again[1].tobytes()
    _compare((4000, 1.2, 8, 20, 7), left)


@pytest.mark.parametrize("case", ["c2", "euroc", "odd", "scale2", "scale15", "rounding1"])
def test_fused_pyramid_bit_exact(gpu_available, case):
    """The resize chain as ONE launch (k_pyramid: a workgroup per image whose
    tile groups walk the levels, the same tile code as the per-level
    launches; opt-in by orbgpu_extractor_set_pyramid_launch) gives the same bytes."""
    if case == "c2":
        assert _compare(C2, synth.stereo_frame(0)[0], fused=True) > 900
    elif case == "euroc":
        assert _compare(EUROC, synth.stereo_frame(10)[1], fused=True) > 1100
    elif case == "odd":
        full, _ = synth.stereo_frame(20, w=641, h=397)
        _compare((1000, 1.2, 8, 20, 7), full, fused=True)
    elif case == "scale2":  # a wide resize window: fewer tile groups fit a workgroup's LDS
        full, _ = synth.stereo_frame(21, w=1024, h=768)
        _compare((1000, 2.0, 4, 20, 7), full, fused=True)
    elif case == "scale15":
        full, _ = synth.stereo_frame(21, w=1024, h=768)
        _compare((1000, 1.5, 6, 20, 7), full, fused=True)
    else:
        assert _compare(C2, synth.stereo_frame(4)[0], rounding=1, fused=True) > 900


def test_fused_pyramid_batch(gpu_available):
    """A batch through the one-launch pyramid equals the oracle image by image."""
    _batch_matches_single(True)


# --- every extractor the reference constructs ---------
MONO_INIT = (5000, 1.2, 8, 20, 7)  # OrbExtractor(5 * nFeatures, ...), tracking.cc:202-204 at EuRoC's 1000


def test_mono_init_extractor_5x_features(gpu_available):
    """The monocular initialisation extractor (5 x nFeatures) on 752x480:
    over 4096 keypoint slots (the old assembly bound), bit-exact."""
    left, _ = synth.stereo_frame(2)
    assert _compare(MONO_INIT, left) > 4096


def test_kitti_size_6000_features(gpu_available):
    """(6000, 1.2, 8, 20, 7) on a 1241x376 frame (KITTI geometry), plus a
    lapping band so the chunked stereo partition crosses its 4096 chunk."""
    full, _ = synth.stereo_frame(22, w=1241, h=376)
    n = _compare((6000, 1.2, 8, 20, 7), full)
    assert n > 4096
    _compare((6000, 1.2, 8, 20, 7), full, lapping=(100, 1100))


@pytest.mark.parametrize("params", [C2, MONO_INIT])
def test_octree_nodes_in_hbm_bit_exact(gpu_available, params):
    """The HBM-node octree (k_octree<true>) forced on plans that fit LDS gives
    the same bytes: the same code with the node arrays in a per-block HBM
    range and workgroup-scoped atomics."""
    left, _ = synth.stereo_frame(6)
    assert _compare(params, left, octree_hbm=True) > 900


def test_octree_nodes_hbm_by_plan(gpu_available):
    """A budget whose node list cannot fit a workgroup's LDS (20000 features,
    dense noise responses): the plan moves the nodes to HBM by itself."""
    from orb_slam_fusion_amd._lib import OrbParams
    import ctypes

    params = (20000, 1.2, 8, 20, 7)
    slots, hbm = ctypes.c_int(), ctypes.c_int()
    assert lib().orbgpu_extractor_plan(ctypes.byref(OrbParams(*params)), 1241, 376,
                                       ctypes.byref(slots), ctypes.byref(hbm)) == 0
    assert hbm.value == 1
    img = synth.noise_image(5, 1241, 376)
    assert _compare(params, img) > 8000


def test_octree_reduced_candidate_cache(gpu_available):
    """6400 features: the octree's node arrays (1408 nodes) still fit LDS but
    leave room for only 1280 of the 2048 cached candidates (the rest in HBM,
    orb_plan.cpp's middle storage policy), bit-exact."""
    left, _ = synth.stereo_frame(12)
    assert _compare((6400, 1.2, 8, 20, 7), left) > 4096


def test_batch_5x_features(gpu_available):
    """The device batch path at 5000 features: per-image outputs past 4096
    slots, equal to the oracle image by image."""
    import torch

    B = 3
    imgs = np.stack([synth.stereo_frame(30 + i)[0] for i in range(B)])
    ex = OrbExtractor(*MONO_INIT, max_images=B)
    cap = ex.max_keypoints(752, 480)
    assert cap > 4096
    d_imgs = torch.from_numpy(imgs).cuda()
    kps = torch.zeros((B, cap, 7), dtype=torch.int32, device="cuda")
    desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device="cuda")
    n = torch.zeros(B, dtype=torch.int32, device="cuda")
    mono = torch.zeros(B, dtype=torch.int32, device="cuda")
    ex.extract_batch(d_imgs, kps, desc, n, mono, lapping_areas=(300, 400))
    torch.cuda.synchronize()
    ex.check()
    kps_h, desc_h, n_h, mono_h = kps.cpu().numpy(), desc.cpu().numpy(), n.cpu().numpy(), mono.cpu().numpy()
    orc = oracle.OracleExtractor(*MONO_INIT)
    for i in range(B):
        m_ref, k_ref, d_ref = orc.extract(imgs[i], (300, 400))
        assert n_h[i] == len(k_ref) and mono_h[i] == m_ref
        assert kps_h[i, : n_h[i]].tobytes() == k_ref.tobytes(), f"image {i} keypoints"
        assert desc_h[i, : n_h[i]].tobytes() == d_ref.tobytes(), f"image {i} descriptors"


@pytest.mark.parametrize("case", ["c2", "euroc", "odd", "lapping", "scale2"])
def test_single_launch_graph_path_bit_exact(gpu_available, case):
    """orbgpu_extract's per-stage graph path (ORBGPU_SINGLE_GRAPH) against the
    oracle; every other host-path test runs the default dataflow launch."""
    left, _ = synth.stereo_frame(7)
    if case == "c2":
        _compare(C2, left, single=1)
    elif case == "euroc":
        _compare(EUROC, left, single=1)
    elif case == "odd":
        _compare(C2, synth.stereo_frame(8, w=641, h=397)[0], single=1)
    elif case == "lapping":
        _compare(C2, left, lapping=(100, 400), single=1)
    else:
        _compare((1000, 2.0, 4, 20, 7), synth.stereo_frame(21, w=1024, h=768)[0], single=1)


def test_dataflow_repeat_and_switches(gpu_available):
    """The dataflow launch record is rewritten when the lapping band, the image
    size or the mode changes; every call equals a fresh handle's graph path."""
    imgs = [synth.stereo_frame(40 + i)[0] for i in range(3)] + [synth.stereo_frame(50, w=641, h=397)[0]]
    laps = [(0, 0), (150, 450), (0, 0), (0, 0)]
    ex = OrbExtractor(*C2)
    ref = OrbExtractor(*C2)
    ref.set_single_launch(1)
    for rnd in range(2):
        for img, lap in zip(imgs, laps):
            got = ex(img, None, lap)
            exp = ref(img, None, lap)
            assert got[0] == exp[0] and got[1].tobytes() == exp[1].tobytes()
            assert got[2].tobytes() == exp[2].tobytes()
            for a, b in zip(ex.img_pyramid_, ref.img_pyramid_):
                assert np.array_equal(a, b)
        ex.set_single_launch(1 - rnd)  # round 2 on the graph path, then back


def test_dataflow_two_handles_on_two_threads(gpu_available):
    """The stereo Frame's two extractions run concurrently (frame.cc:179-182):
    two dataflow launches in flight on two streams give each handle's
    sequential results, frame after frame."""
    import threading

    pairs = [synth.stereo_frame(60 + i) for i in range(6)]
    exl, exr = OrbExtractor(*C2), OrbExtractor(*C2)
    seq = OrbExtractor(*C2)
    expect = []
    for l, r in pairs:
        _, kl, dl = seq(l)
        _, kr, dr = seq(r)
        expect.append((kl.tobytes(), dl.tobytes(), kr.tobytes(), dr.tobytes()))
    for rnd in range(3):
        for (l, r), e in zip(pairs, expect):
            out = {}
            th = threading.Thread(target=lambda: out.__setitem__("r", exr(r)))
            th.start()
            _, kl, dl = exl(l)
            th.join()
            _, kr, dr = out["r"]
            assert (kl.tobytes(), dl.tobytes(), kr.tobytes(), dr.tobytes()) == e


@pytest.mark.parametrize("single", [0, 1])
def test_extract_stereo_pair_equals_two_calls(gpu_available, single):
    """orbgpu_extract_stereo (both images from one host thread) gives each
    handle's orbgpu_extract results, on both launch paths, frame after frame
    -- and the pair's pyramids / stereo match read back as after two calls."""
    from orb_slam_fusion_amd import compute_stereo_matches

    pairs = [synth.stereo_frame(70 + i) for i in range(4)]
    exl, exr = OrbExtractor(*C2), OrbExtractor(*C2)
    for e in (exl, exr):
        e.set_single_launch(single)
    ref_l, ref_r = OrbExtractor(*C2), OrbExtractor(*C2)
    for rnd in range(2):
        for l, r in pairs:
            (ml, kl, dl), (mr, kr, dr) = exl.extract_stereo(exr, l, r)
            el, er = ref_l(l), ref_r(r)
            assert (ml, kl.tobytes(), dl.tobytes()) == (el[0], el[1].tobytes(), el[2].tobytes())
            assert (mr, kr.tobytes(), dr.tobytes()) == (er[0], er[1].tobytes(), er[2].tobytes())
            bf, mb = np.float32(435.2 * 0.11), np.float32(np.float32(435.2 * 0.11) / np.float32(435.2))
            u1, d1 = compute_stereo_matches(exl, exr, len(kl), bf, mb)
            u2, d2 = compute_stereo_matches(ref_l, ref_r, len(el[1]), bf, mb)
            assert u1.tobytes() == u2.tobytes() and d1.tobytes() == d2.tobytes()
    (ml, kl, _), _ = exl.extract_stereo(exr, pairs[0][0], pairs[0][1], (100, 400), (0, 0))
    assert kl.tobytes() == ref_l(pairs[0][0], None, (100, 400))[1].tobytes()
