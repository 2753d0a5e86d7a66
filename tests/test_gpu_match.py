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


@pytest.mark.parametrize("seed,th,orb_dist,ori,n_kp,n_pts", [
    (31, 10, 100, True, 600, 500),    # Relocalization's first pass (tracking.cc:2967)
    (32, 3, 64, True, 600, 500),      # its refinement passes (:2982, :2997)
    (33, 10, 100, False, 1000, 900),
    (34, 15, 50, True, 3000, 2500),
    (35, 10, 100, True, 200, 1200),   # many points per keypoint: claims
])
def test_search_kf_parity(matcher, seed, th, orb_dist, ori, n_kp, n_pts):
    """SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist)
    (orb_matcher.cc:1730-1839) bit-exact vs the oracle."""
    c = local_case(seed, n_kp=n_kp, n_pts=n_pts)
    matcher.mbCheckOrientation = ori
    nm, m = matcher.SearchByProjection_kf(_frame(c), c.pts, c.angles, th, orb_dist)
    nm_o, m_o = orc.search_kf(c.geom, c.cam, c.Tcw, c.kps, c.desc, c.claimed, c.pts, c.angles, th,
                              orb_dist, ori)
    assert nm == nm_o
    np.testing.assert_array_equal(m, m_o)
    assert nm > 20


def test_kf_batch_matches_single(matcher):
    import torch

    from orb_slam_fusion_amd._lib import KEYPOINT_DTYPE, MAP_POINT_DTYPE

    B, K, P = 4, 900, 800
    cases = [local_case(60 + b, n_kp=K - 40 * b, n_pts=P - 70 * b) for b in range(B)]
    dev = torch.device("cuda", 0)
    kps = np.zeros((B, K), KEYPOINT_DTYPE)
    desc = np.zeros((B, K, 32), np.uint8)
    cl = np.zeros((B, K), np.uint8)
    pts = np.zeros((B, P), MAP_POINT_DTYPE)
    ang = np.zeros((B, P), np.float32)
    n = np.array([len(c.kps) for c in cases], np.int32)
    npts = np.array([len(c.pts) for c in cases], np.int32)
    for b, c in enumerate(cases):
        kps[b, :n[b]], desc[b, :n[b]], cl[b, :n[b]] = c.kps, c.desc, c.claimed
        pts[b, :npts[b]], ang[b, :npts[b]] = c.pts, c.angles
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    d_match = torch.zeros((B, K), dtype=torch.int32, device=dev)
    d_nm = torch.zeros(B, dtype=torch.int32, device=dev)
    matcher.mbCheckOrientation = True
    c0 = cases[0]
    matcher.search_kf_batch(c0.geom, c0.cam, T(np.stack([c.Tcw for c in cases])),
                            T(kps.view(np.int32).reshape(B, K, 7)), T(desc), T(cl), T(n),
                            T(pts.view(np.uint8).reshape(B, P, 68)), T(ang), T(npts), 10, 100,
                            d_match, d_nm)
    torch.cuda.synchronize()
    match, nm = d_match.cpu().numpy(), d_nm.cpu().numpy()
    for b, c in enumerate(cases):
        nm_o, m_o = orc.search_kf(c.geom, c.cam, c.Tcw, c.kps, c.desc, c.claimed, c.pts, c.angles,
                                  10, 100, True)
        assert nm[b] == nm_o
        np.testing.assert_array_equal(match[b, :n[b]], m_o)


@pytest.mark.parametrize("seed,nn,ori", [(41, 0.75, True), (42, 0.7, True), (43, 0.9, False),
                                         (44, 0.6, True), (46, 0.7, True)])
def test_search_bow_parity(seed, nn, ori, gpu_available):
    """SearchByBoW(pKF, F) (orb_matcher.cc:215-389) bit-exact vs the oracle."""
    from match_cases import bow_case, fv_arrays
    from orb_slam_fusion_amd.matcher import ORBmatcher

    c = bow_case(seed, n_kf=1500 if seed == 46 else 600, n_f=1600 if seed == 46 else 650)
    m = ORBmatcher(nn, ori)
    nm, match = m.SearchByBoW(fv_arrays(c.kf_fv), c.kf_desc, c.kf_angle, c.kf_valid,
                              fv_arrays(c.f_fv), c.f_desc, c.f_angle)
    nm_o, m_o = orc.search_bow(fv_arrays(c.kf_fv), c.kf_desc, c.kf_angle, c.kf_valid,
                               fv_arrays(c.f_fv), c.f_desc, c.f_angle, nn, ori)
    assert nm == nm_o
    np.testing.assert_array_equal(match, m_o)
    assert nm > 50
    m.close()


def test_search_bow_edge_cases(matcher):
    from match_cases import bow_case, fv_arrays

    c = bow_case(45)
    empty = (np.zeros(0, np.uint32), np.zeros(1, np.int32), np.zeros(0, np.uint32))
    nm, m = matcher.SearchByBoW(empty, c.kf_desc, c.kf_angle, c.kf_valid, fv_arrays(c.f_fv),
                                c.f_desc, c.f_angle)
    assert nm == 0 and (m == -1).all()
    shifted = {k + 100000: v for k, v in c.f_fv.items()}
    nm, m = matcher.SearchByBoW(fv_arrays(c.kf_fv), c.kf_desc, c.kf_angle, c.kf_valid,
                                fv_arrays(shifted), c.f_desc, c.f_angle)
    assert nm == 0 and (m == -1).all()
    nm, m = matcher.SearchByBoW(fv_arrays(c.kf_fv), c.kf_desc, c.kf_angle,
                                np.zeros_like(c.kf_valid), fv_arrays(c.f_fv), c.f_desc, c.f_angle)
    assert nm == 0 and (m == -1).all()


def test_track_reference_keyframe_bow_chain(gpu_available, tmp_path):
    """TrackReferenceKeyFrame's slice on the device (tracking.cc:2031-2067):
    extract the reference key frame and the current frame, ComputeBoW of both
    (orbgpu_bow_transform_batch, FeatureVectors resident in HBM), then
    SearchByBoW(pKF, F) with ORBmatcher(0.7, true) reading the frame angles
    straight from the keypoint rows -- matches bit-exact vs the oracle on the
    same FeatureVectors."""
    import torch

    from orb_slam_fusion_amd import OrbExtractor, synth
    from orb_slam_fusion_amd.matcher import ORBmatcher
    from orb_slam_fusion_amd.vocab import ORBVocabulary

    path = tmp_path / "voc.txt"
    synth.vocab_text(path, k=10, L=5)
    voc = ORBVocabulary()
    assert voc.loadFromTextFile(str(path))
    dev = torch.device("cuda", 0)
    B = 3
    imgs = []
    for b in range(B):  # frame pairs a few pixels apart: reference key frame, current frame
        last_l, _, cur_l, _ = synth.track_pair(b)
        imgs += [last_l, cur_l]
    ex = OrbExtractor(1000, 1.2, 8, 20, 7, max_images=2 * B)
    cap = 2000
    d_img = torch.from_numpy(np.stack(imgs)).to(dev)
    kps = torch.zeros((2 * B, cap, 7), dtype=torch.int32, device=dev)
    desc = torch.zeros((2 * B, cap, 32), dtype=torch.uint8, device=dev)
    n = torch.zeros(2 * B, dtype=torch.int32, device=dev)
    mono = torch.zeros(2 * B, dtype=torch.int32, device=dev)
    ex.extract_batch(d_img, kps, desc, n, mono)
    S = cap
    z = lambda *s, t=torch.int32: torch.zeros(s, dtype=t, device=dev)  # noqa: E731
    bw, bwt, nw = z(2 * B, S), z(2 * B, S, t=torch.float64), z(2 * B)
    fn, fo, ff, nn_ = z(2 * B, S), z(2 * B, S + 1), z(2 * B, S), z(2 * B)
    voc.transform_batch(desc, n, 4, bw, bwt, nw, fn, fo, ff, nn_)
    sel_k, sel_f = torch.arange(0, 2 * B, 2, device=dev), torch.arange(1, 2 * B, 2, device=dev)
    kps_f = kps[sel_f].contiguous()
    kf_valid = torch.ones((B, S), dtype=torch.uint8, device=dev)
    kf_angle = kps[sel_k].view(torch.float32)[..., 3].contiguous()
    m = ORBmatcher(0.7, True)
    d_match, d_nm = z(B, S), z(B)
    m.search_bow_batch((fn[sel_k].contiguous(), fo[sel_k].contiguous(), ff[sel_k].contiguous(),
                        nn_[sel_k].contiguous()), desc[sel_k].contiguous(), kf_angle, kf_valid,
                       (fn[sel_f].contiguous(), fo[sel_f].contiguous(), ff[sel_f].contiguous(),
                        nn_[sel_f].contiguous()), desc[sel_f].contiguous(),
                       kps_f.view(torch.float32)[..., 3], n[sel_f].contiguous(), d_match, d_nm,
                       f_angle_step=7)
    assert m.status() == 0
    torch.cuda.synchronize()
    match, nm = d_match.cpu().numpy(), d_nm.cpu().numpy()
    FN, FO, FF, NN = (x.cpu().numpy() for x in (fn, fo, ff, nn_))
    D, N, K = desc.cpu().numpy(), n.cpu().numpy(), kps.cpu().numpy().view(np.float32)
    for b in range(B):
        ik, jf = 2 * b, 2 * b + 1
        fv = lambda i: (FN[i, :NN[i]], FO[i, :NN[i] + 1], FF[i, :FO[i, NN[i]]])  # noqa: E731
        nm_o, m_o = orc.search_bow(fv(ik), D[ik, :N[ik]], K[ik, :N[ik], 3], np.ones(N[ik], np.uint8),
                                   fv(jf), D[jf, :N[jf]], K[jf, :N[jf], 3], 0.7, True)
        assert nm[b] == nm_o and nm_o > 30
        np.testing.assert_array_equal(match[b, :N[jf]], m_o)
