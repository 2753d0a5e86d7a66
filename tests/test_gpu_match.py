"""GPU parity of the ORBmatcher projection searches (match_kernels.hip through
the C ABI) against the CPU oracle (oracle/match_oracle.cc): match arrays,
return values and isInFrustum fields bit-exact."""
import numpy as np
import pytest

import binding as orc
from match_cases import last_case, local_case

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def matcher(gpu_available):
    from orb_slam_fusion_amd.matcher import ORBmatcher

    m = ORBmatcher(0.9, True, max_keypoints=8192, max_points=16384)
    yield m
    m.close()


def _frame(c):
    from orb_slam_fusion_amd.matcher import MatchFrame

    return MatchFrame(geom=c.geom, cam=c.cam, mb=c.mb, kps=c.kps, desc=c.desc, uright=c.uright,
                      claimed=c.claimed, pose=c.Tcw)


@pytest.mark.parametrize("seed,motion,th,ori,stereo,mono,n_kp,n_pts", [
    (1, "none", 7, True, True, False, 600, 400),
    (2, "forward", 7, True, True, False, 600, 400),
    (3, "backward", 15, True, True, False, 600, 400),
    (4, "none", 30, False, False, False, 1000, 700),
    (5, "forward", 15, True, True, True, 1000, 700),
    (6, "none", 14, True, True, False, 3000, 2500),
    (7, "none", 7, True, True, False, 200, 1200),   # many points per keypoint: claims
])
def test_search_last_parity(matcher, seed, motion, th, ori, stereo, mono, n_kp, n_pts):
    c = last_case(seed, n_kp=n_kp, n_pts=n_pts, stereo=stereo, motion=motion)
    matcher.mbCheckOrientation = ori
    nm, m = matcher.SearchByProjection_last(_frame(c), c.pts, c.Tlw, th, mono)
    nm_o, m_o = orc.search_last(c.geom, c.cam, c.mb, c.Tcw, c.Tlw, c.kps, c.desc, c.uright,
                                c.claimed, c.pts, th, mono, ori)
    assert nm == nm_o
    np.testing.assert_array_equal(m, m_o)
    assert nm > 0


@pytest.mark.parametrize("seed,th,stereo,far,n_kp,n_pts", [
    (11, 1, True, False, 600, 500),
    (12, 3, True, False, 600, 500),
    (13, 15, False, False, 1000, 900),
    (14, 5, True, True, 1000, 900),
    (15, 2, True, False, 4000, 6000),
    (16, 10, True, False, 150, 1500),  # dense claims
])
def test_search_local_parity(matcher, seed, th, stereo, far, n_kp, n_pts):
    c = local_case(seed, n_kp=n_kp, n_pts=n_pts, stereo=stereo)
    matcher.mfNNratio = 0.8
    F = _frame(c)
    init = np.zeros(len(c.pts), orc.TRACK_VIEW_DTYPE)
    init["level"] = 99
    init["proj_xr"] = -5.0
    v_gpu = matcher.is_in_frustum(F, c.pts, 0.5, views=init)
    v_o = orc.frustum(c.geom, c.cam, c.Rcw, c.tcw, c.Ow, c.pts, 0.5, init)
    assert v_gpu.tobytes() == v_o.tobytes()
    nm, m = matcher.SearchByProjection_local(F, c.pts, v_o, th, far, 4.0)
    nm_o, m_o = orc.search_local(c.geom, c.kps, c.desc, c.uright, c.claimed, c.pts, v_o, th, 0.8,
                                 far, 4.0)
    assert nm == nm_o
    np.testing.assert_array_equal(m, m_o)
    nm2, m2, v2 = matcher.search_local_points(F, c.pts, 0.5, th, far, 4.0, views=init)
    assert v2.tobytes() == v_o.tobytes()
    assert nm2 == nm_o
    np.testing.assert_array_equal(m2, m_o)


def test_edge_cases(matcher):
    c = last_case(21, n_kp=300, n_pts=200)
    F = _frame(c)
    matcher.mbCheckOrientation = True
    # no query points
    nm, m = matcher.SearchByProjection_last(F, c.pts[:0], c.Tlw, 7, False)
    assert nm == 0 and (m == -1).all()
    # every keypoint already held by a map point with observations
    F.claimed = np.ones(len(c.kps), np.uint8)
    nm, m = matcher.SearchByProjection_last(F, c.pts, c.Tlw, 7, False)
    assert nm == 0 and (m == -1).all()
    # identical descriptors everywhere: ties resolved by the reference's order
    F.claimed = None
    F.desc = np.zeros_like(c.desc)
    pts = c.pts.copy()
    pts["desc"] = 0
    nm, m = matcher.SearchByProjection_last(F, pts, c.Tlw, 15, False)
    nm_o, m_o = orc.search_last(c.geom, c.cam, c.mb, c.Tcw, c.Tlw, c.kps, F.desc, c.uright, None,
                                pts, 15, False, True)
    assert nm == nm_o and nm > 0
    np.testing.assert_array_equal(m, m_o)
    # empty frame
    F2 = _frame(c)
    F2.kps, F2.desc, F2.uright = c.kps[:0], c.desc[:0], None
    nm, m = matcher.SearchByProjection_last(F2, c.pts, c.Tlw, 7, False)
    assert nm == 0 and len(m) == 0


def test_last_batch_matches_single(matcher):
    import torch

    from orb_slam_fusion_amd._lib import KEYPOINT_DTYPE, PROJ_POINT_DTYPE

    B, K, P = 5, 900, 700
    cases = [last_case(40 + b, n_kp=K - 50 * b, n_pts=P - 60 * b,
                       motion=["none", "forward", "backward"][b % 3]) for b in range(B)]
    dev = torch.device("cuda", 0)
    kps = np.zeros((B, K), KEYPOINT_DTYPE)
    desc = np.zeros((B, K, 32), np.uint8)
    ur = np.full((B, K), -1.0, np.float32)
    pts = np.zeros((B, P), PROJ_POINT_DTYPE)
    n = np.array([len(c.kps) for c in cases], np.int32)
    npts = np.array([len(c.pts) for c in cases], np.int32)
    for b, c in enumerate(cases):
        kps[b, :n[b]] = c.kps
        desc[b, :n[b]] = c.desc
        ur[b, :n[b]] = c.uright
        pts[b, :npts[b]] = c.pts
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    d_kps = T(kps.view(np.int32).reshape(B, K, 7))
    d_desc, d_ur = T(desc), T(ur)
    d_pts = T(pts.view(np.uint8).reshape(B, P, 56))
    d_tcw = T(np.stack([c.Tcw for c in cases]))
    d_tlw = T(np.stack([c.Tlw for c in cases]))
    d_match = torch.zeros((B, K), dtype=torch.int32, device=dev)
    d_nm = torch.zeros(B, dtype=torch.int32, device=dev)
    matcher.mbCheckOrientation = True
    c0 = cases[0]
    matcher.search_last_batch(c0.geom, c0.cam, c0.mb, d_tcw, d_tlw, d_kps, d_desc, d_ur, None,
                              T(n), d_pts, T(npts), 7, False, d_match, d_nm)
    torch.cuda.synchronize()
    match, nm = d_match.cpu().numpy(), d_nm.cpu().numpy()
    for b, c in enumerate(cases):
        nm_o, m_o = orc.search_last(c.geom, c.cam, c.mb, c.Tcw, c.Tlw, c.kps, c.desc, c.uright,
                                    None, c.pts, 7, False, True)
        assert nm[b] == nm_o
        np.testing.assert_array_equal(match[b, :n[b]], m_o)


def test_unproject_stereo_batch(matcher):
    """Frame::UnprojectStereo over the stereo keypoints (frame.cc:1008-1020):
    compaction in index order, octave / angle / descriptor carried, Xw = mRwc
    Xc + mOw against a float64 restatement (float32 tolerance)."""
    import torch

    from orb_slam_fusion_amd._lib import KEYPOINT_DTYPE, PROJ_POINT_DTYPE

    rng = np.random.default_rng(5)
    B, K = 3, 700
    kps = np.zeros((B, K), KEYPOINT_DTYPE)
    kps["x"], kps["y"] = rng.uniform(0, 752, (B, K)), rng.uniform(0, 480, (B, K))
    kps["angle"], kps["octave"] = rng.uniform(0, 360, (B, K)), rng.integers(0, 8, (B, K))
    desc = rng.integers(0, 256, (B, K, 32), dtype=np.uint8)
    depth = np.where(rng.random((B, K)) < 0.6, rng.uniform(0.5, 9, (B, K)), -1).astype(np.float32)
    n = np.array([K, 500, 0], np.int32)
    poses = []
    for f in range(B):
        q = rng.normal(size=4)
        q /= np.linalg.norm(q)
        poses.append(np.concatenate([q, rng.normal(size=3)]).astype(np.float32))
    Tcw = np.stack(poses)
    cam = np.array([458.654, 457.296, 367.215, 248.375, 50.0], np.float32)
    dev = torch.device("cuda", 0)
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    pts = torch.zeros((B, K, 56), dtype=torch.uint8, device=dev)
    npts = torch.zeros(B, dtype=torch.int32, device=dev)
    matcher.unproject_stereo_batch(cam, d(Tcw), d(kps.view(np.float32).reshape(B, K, 7)), d(desc),
                                   d(depth), d(n), pts, npts)
    torch.cuda.synchronize()
    got = pts.cpu().numpy().view(PROJ_POINT_DTYPE).reshape(B, K)
    gn = npts.cpu().numpy()
    for f in range(B):
        sel = np.nonzero(depth[f, :n[f]] > 0)[0]
        assert gn[f] == len(sel)
        g = got[f, :len(sel)]
        assert np.array_equal(g["octave"], kps["octave"][f, sel])
        assert np.array_equal(g["angle"], kps["angle"][f, sel])
        assert np.array_equal(g["desc"], desc[f, sel]) and (g["has_obs"] == 1).all()
        qx, qy, qz, qw = Tcw[f, :4].astype(np.float64)
        R = np.array([[1 - 2 * (qy * qy + qz * qz), 2 * (qx * qy - qz * qw), 2 * (qx * qz + qy * qw)],
                      [2 * (qx * qy + qz * qw), 1 - 2 * (qx * qx + qz * qz), 2 * (qy * qz - qx * qw)],
                      [2 * (qx * qz - qy * qw), 2 * (qy * qz + qx * qw), 1 - 2 * (qx * qx + qy * qy)]])
        z = depth[f, sel].astype(np.float64)
        Xc = np.stack([(kps["x"][f, sel] - cam[2]) * z / cam[0],
                       (kps["y"][f, sel] - cam[3]) * z / cam[1], z], 1)
        Xw = Xc @ R + (-(R.T @ Tcw[f, 4:].astype(np.float64)))
        np.testing.assert_allclose(g["Xw"], Xw, rtol=2e-5, atol=2e-5)
