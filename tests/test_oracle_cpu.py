"""CPU tests of the oracle: pinned where a pin exists (host libm, GCC codegen,
SURVEY tables), cross-checked against independent numpy/Python restatements
(tests/ref_py.py) elsewhere, and regression-pinned by tests/golden/."""
import hashlib
import json
import platform
import shutil
import subprocess
import struct
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

import numpy as np
import pytest

import binding as oracle
import ref_py
from orb_slam_fusion_amd import synth

GOLDEN = Path(__file__).resolve().parent / "golden"
C2 = (1000, 1.2, 8, 20, 7)


def _bits(f: float) -> int:
    return struct.unpack("<I", struct.pack("<f", f))[0]


def test_sincosf_exhaustive_against_host_libm():
    """Every float in [0, 2*pi] (+ a margin): restated glibc sinf/cosf ==
    host libm bit for bit (IC_Angle angles live in that range)."""
    lo, hi = 0, _bits(6.2831855) + 64
    chunks = np.linspace(lo, hi, 17, dtype=np.int64)
    with ThreadPoolExecutor(8) as pool:
        bad = sum(pool.map(lambda ab: oracle.sincosf_check_libm(int(ab[0]), int(ab[1]) - 1),
                           zip(chunks[:-1], chunks[1:] + np.r_[np.zeros(15, np.int64), 1])))
    assert bad == 0


@pytest.mark.skipif(platform.machine() != "x86_64" or not shutil.which("g++"), reason="x86 g++")
def test_get_value_contraction(tmp_path):
    """GCC -O2 -march=native (here: haswell) fuses the descriptor sample
    coordinates of orb_extractor.cc:111-113 into fmaf(x, b, y*a) and
    fmaf(x, a, -(y*b)) -- the rule the oracle and the kernel implement."""
    src = tmp_path / "gv.cc"
    src.write_text(
        "#include <cmath>\nstruct P{int x,y;};\n"
        "int f(const unsigned char* c,const P* p,float a,float b,int s){"
        "return c[(int)lrintf(p->x*b+p->y*a)*s+(int)lrintf(p->x*a-p->y*b)];}\n")
    asm = subprocess.run(["g++", "-std=c++11", "-O2", "-march=haswell", "-S", "-o", "-", str(src)],
                         capture_output=True, text=True, check=True).stdout
    assert "vfmadd231ss" in asm and "vfmsub132ss" in asm


def test_gaussian_kernel_q8():
    assert oracle.gauss_kernel().tolist() == [18, 34, 48, 56, 48, 34, 18]


def test_scale_tables_budgets_umax():
    p = oracle.OracleExtractor(*C2).params()
    assert p["feats_per_level"].tolist() == [217, 181, 151, 126, 105, 87, 73, 60]
    assert oracle.OracleExtractor(1200, 1.2, 8, 20, 7).params()["feats_per_level"].tolist() == \
        [261, 217, 181, 151, 126, 105, 87, 72]
    assert p["umax"].tolist() == [15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3]
    assert np.float32(p["scale"][1]) == np.float32(1.2000000477)


def test_pyramid_level_sizes_752x480():
    ex = oracle.OracleExtractor(*C2)
    lv = ex.pyramid(synth.stereo_frame(0)[0])
    assert [l.shape[::-1] for l in lv] == [(752, 480), (627, 400), (522, 333), (435, 278),
                                          (363, 231), (302, 193), (252, 161), (210, 134)]


@pytest.mark.parametrize("sw,sh,dw,dh", [(752, 480, 627, 400), (627, 400, 522, 333),
                                         (363, 231, 302, 193), (101, 77, 84, 64), (40, 30, 33, 25)])
def test_resize_matches_numpy_restatement(sw, sh, dw, dh):
    rng = np.random.default_rng(sw * 7 + dh)
    src = rng.integers(0, 256, (sh, sw), dtype=np.uint8)
    assert np.array_equal(oracle.resize(src, dw, dh), ref_py.resize_linear(src, dw, dh))


@pytest.mark.parametrize("sw,sh,dw,dh", [(752, 480, 627, 400), (101, 77, 84, 64)])
def test_resize_scalar_rounding_switch(sw, sh, dw, dh):
    """SURVEY A.2's switch: every column the scalar FixedPtCast rounding; it
    matches the numpy restatement and differs from the SSE split somewhere."""
    rng = np.random.default_rng(sw + dw)
    src = rng.integers(0, 256, (sh, sw), dtype=np.uint8)
    with oracle.resize_rounding(oracle.RESIZE_SCALAR):
        sca = oracle.resize(src, dw, dh)
    assert np.array_equal(sca, ref_py.resize_linear(src, dw, dh, rounding="scalar"))
    sse = oracle.resize(src, dw, dh)  # the default is restored on exit
    assert np.array_equal(sse, ref_py.resize_linear(src, dw, dh))
    assert (sca != sse).any()


@pytest.mark.parametrize("w,h", [(64, 48), (33, 17), (210, 134)])
def test_gauss_matches_numpy_restatement(w, h):
    rng = np.random.default_rng(w * h)
    src = rng.integers(0, 256, (h, w), dtype=np.uint8)
    assert np.array_equal(oracle.gauss(src), ref_py.gauss7(src))


@pytest.mark.parametrize("seed,th", [(1, 20), (2, 7), (3, 20), (4, 0)])
def test_fast_ring_buffer_matches_definition(seed, th):
    """The restated FAST_t<16> ring-buffer NMS == the definitional score/NMS."""
    rng = np.random.default_rng(seed)
    base = rng.integers(0, 256, (44, 42), dtype=np.uint8)
    if seed % 2:  # structured: blocks + noise
        base = np.kron(rng.integers(0, 256, (11, 11)), np.ones((4, 4)))[:44, :42]
        base = np.clip(base + rng.integers(-6, 7, base.shape), 0, 255).astype(np.uint8)
    got = [tuple(r) for r in oracle.fast(base, th).tolist()]
    assert got == ref_py.fast_nms_def(base, th)


def test_fast_atan2_values():
    assert abs(oracle.fast_atan2(1.0, 1.0) - 45.0) < 0.01
    assert abs(oracle.fast_atan2(-1.0, -1.0) - 225.0) < 0.01
    assert oracle.fast_atan2(0.0, 0.0) == 0.0
    for y, x in [(3.0, -7.0), (-5.0, 2.0), (1e6, 1.0)]:
        a = oracle.fast_atan2(y, x)
        assert 0.0 <= a < 360.0
        assert abs(a - np.degrees(np.arctan2(y, x)) % 360.0) < 0.02


@pytest.mark.parametrize("frame,side", [(0, 0), (1, 1), (4, 0)])
def test_octree_matches_python_restatement(frame, side):
    """DistributeOctTree in C++ (std::list) == the Python list restatement,
    level by level, on the oracle's own FAST candidates."""
    img = synth.stereo_frame(frame)[side]
    ex = oracle.OracleExtractor(*C2)
    ex.extract(img)
    budgets = ex.params()["feats_per_level"]
    for lev in range(8):
        h, w = ex.level(lev).shape
        cand = [tuple(r) for r in ex.stage(lev, 0).tolist()]
        want = ref_py.distribute_octree(cand, 16, w - 16, 16, h - 16, int(budgets[lev]))
        got = [tuple(r) for r in ex.stage(lev, 1).tolist()]
        assert got == want, f"level {lev}"


def test_octree_python_restatement_on_noise():
    img = synth.noise_image(5, 320, 256)
    ex = oracle.OracleExtractor(500, 1.2, 4, 20, 7)
    ex.extract(img)
    budgets = ex.params()["feats_per_level"]
    for lev in range(4):
        h, w = ex.level(lev).shape
        cand = [tuple(r) for r in ex.stage(lev, 0).tolist()]
        want = ref_py.distribute_octree(cand, 16, w - 16, 16, h - 16, int(budgets[lev]))
        assert [tuple(r) for r in ex.stage(lev, 1).tolist()] == want


def _gen(g):
    if g[0] == "stereo":
        l, r = synth.stereo_frame(g[1], w=g[3], h=g[4])
        return l if g[2] == "L" else r
    return synth.noise_image(g[1], g[2], g[3])


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("case", json.loads((GOLDEN / "extractor_golden.json").read_text()),
                         ids=lambda c: c["name"])
def test_oracle_reproduces_golden(case):
    img = _gen(case["gen"])
    assert _sha(img) == case["image_sha256"], "synthetic generator drifted"
    ex = oracle.OracleExtractor(*case["params"])
    mono, k, d = ex.extract(img, case["lapping"])
    assert len(k) == case["n"] and mono == case["mono"]
    assert _sha(k) == case["keypoints_sha256"] and _sha(d) == case["descriptors_sha256"]
    assert [_sha(ex.level(l)) for l in range(case["params"][2])] == case["pyramid_sha256"]


@pytest.mark.parametrize("case", json.loads((GOLDEN / "pose_golden.json").read_text()),
                         ids=lambda c: f"seed{c['seed']}")
def test_pose_oracle_golden(case):
    cam, pin, pt, obs = synth.pose_problem(case["seed"], case["n"], case["outlier_pct"])
    assert _sha(obs) == case["obs_sha256"]
    inl, pout, out, pd = oracle.pose_opt(cam, pin, obs)
    assert inl == case["inliers"] and _sha(out) == case["outlier_sha256"]
    assert np.array_equal(pout, np.array(case["pose"], np.float32))


def test_pose_oracle_recovers_truth():
    cam, pin, pt, obs = synth.pose_problem(7, 600, 10)
    inl, pout, out, _ = oracle.pose_opt(cam, pin, obs)
    assert np.linalg.norm(pout[4:] - pt[4:]) < 0.005
    assert abs(abs(float(np.dot(pout[:4], pt[:4]))) - 1.0) < 1e-5
    assert 450 < inl < 560


def test_pose_oracle_too_few():
    cam, pin, pt, obs = synth.pose_problem(3, 2, 0)
    inl, pout, out, _ = oracle.pose_opt(cam, pin, obs)
    assert inl == 0 and np.array_equal(pout, pin)


def test_empty_image_minus_one():
    ex = oracle.OracleExtractor(*C2)
    assert ex.extract(np.zeros((0, 0), np.uint8))[0] == -1
