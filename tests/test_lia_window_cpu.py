"""The LocalInertialBA temporal window (optimizer.cc:2332-2436), graph
(:2461-2781) and FAIL test / write-back (:2796-2901) of orb_slam_fusion_amd.lba
against an independent restatement, on duck-typed maps built from the
synthetic stereo-inertial windows: the mPrevKF chain and Nd, the pop when the
chain reaches the map's first key frame, one fixed observer per map point
(the reference's `break`), bad / foreign key frames and bad points."""
import sys
from collections import OrderedDict
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "oracle"))

from orb_slam_fusion_amd import synth  # noqa: E402
from orb_slam_fusion_amd.lba import gather_inertial_window, write_back_inertial  # noqa: E402


class Map:
    def __init__(self, n):
        self.n = n

    def KeyFramesInMap(self):
        return self.n


class KP:
    def __init__(self, x, y, octave):
        self.x, self.y, self.octave = x, y, octave


class KeyFrame:
    def __init__(self, kid, mp, state, addr):
        self.id_, self._map, self.addr, self.s = kid, mp, addr, state
        self._bad = False
        self.bImu = True
        self.mPrevKF = None
        self.mpImuPreintegrated = None
        self.mnBALocalForKF = self.mnBAFixedForKF = -1
        self.mvKeysUn, self.mvuRight, self.matches = [], [], []
        self.mvInvLevelSigma2 = [float(np.float32(1.0) / np.float32(1.2) ** np.float32(2 * l))
                                 for l in range(8)]

    def isBad(self):
        return self._bad

    def GetMap(self):
        return self._map

    def GetVectorCovisibleKeyFrames(self):
        return []

    def GetMapPointMatches(self):
        return list(self.matches)

    def GetImuRotation(self):
        return self.s["Rwb"].reshape(3, 3)

    def GetImuPosition(self):
        return self.s["twb"]

    def GetRotation(self):
        return self.s["Rcw"].reshape(3, 3)

    def GetTranslation(self):
        return self.s["tcw"]

    def GetVelocity(self):
        return self.s["v"]

    def GetGyroBias(self):
        return self.s["bg"]

    def GetAccBias(self):
        return self.s["ba"]


class MapPoint:
    def __init__(self, pid, pos, depth):
        self.id_, self._pos, self.mTrackDepth = pid, pos, depth
        self._bad = False
        self.mnBALocalForKF = -1
        self.obs = {}

    def isBad(self):
        return self._bad

    def GetWorldPos(self):
        return self._pos

    def GetObservations(self):  # std::map<KeyFrame*, tuple>: key (pointer) order
        return OrderedDict(sorted(self.obs.items(), key=lambda kv: kv[0].addr))


def build_map(pb, seed=0, p_bad_mp=0.0, bad_kf=(), foreign_kf=()):
    """Key frames of a synth.LiaProblem as a map: chronological ids, mPrevKF
    chain, each key frame's preintegration from the problem's links (the
    oldest key frames get synthetic ones), observations from its edges."""
    rng = np.random.default_rng(seed)
    n = len(pb.kfs)
    order = list(range(n - 1, -1, -1))  # problem index of the chronological i-th key frame
    M, other = Map(n), Map(n)
    addrs = rng.permutation(n) * 64 + 4096
    kfs = [None] * n
    for chron, i in enumerate(order):
        kfs[i] = KeyFrame(chron, M, pb.kfs_true[i] if pb.fixed[i] else pb.kfs[i], int(addrs[i]))
    for i in range(n - 1):
        kfs[i].mPrevKF = kfs[i + 1]
    for l in pb.imu_edges:
        kfs[l["kf2"]].mpImuPreintegrated = np.array(l["preint"])
    for i in range(n):
        if kfs[i].mpImuPreintegrated is None:
            kfs[i].mpImuPreintegrated = np.array(pb.imu_edges[-1]["preint"])
    for i in bad_kf:
        kfs[i]._bad = True
    for i in foreign_kf:
        kfs[i]._map = other
    mps = [MapPoint(p, pb.pts_init[p], float(rng.uniform(2, 20))) for p in range(len(pb.pts_init))]
    for p in range(len(mps)):
        mps[p]._bad = rng.random() < p_bad_mp
    for e in pb.edges:
        k, mp = kfs[e["kf"]], mps[e["point"]]
        left = len(k.mvKeysUn)
        k.mvKeysUn.append(KP(float(e["u"]), float(e["v"]), int(round(np.log(1 / e["inv_sigma2"]) /
                                                                      np.log(1.44)))))
        k.mvuRight.append(float(e["ur"]))
        k.matches.append(mp)
        mp.obs[k] = (left, -1)
    return kfs, mps, M


def reference_window(pKF, b_large=False):
    """Independent restatement of :2340-2436 as lists and mark sets."""
    kid = pKF.id_
    Nd = min(pKF.GetMap().KeyFramesInMap() - 2, 25 if b_large else 10)
    chain = [pKF]
    while len(chain) < Nd and chain[-1].mPrevKF is not None:
        chain.append(chain[-1].mPrevKF)
    marked_local = {id(k) for k in chain}
    seen, lmps = set(), []
    for k in chain:
        for mp in k.matches:
            if mp is not None and not mp.isBad() and id(mp) not in seen:
                seen.add(id(mp))
                lmps.append(mp)
    if chain[-1].mPrevKF is not None:
        opt, fixed = chain, [chain[-1].mPrevKF]
    else:
        opt, fixed = chain[:-1], [chain[-1]]
        marked_local.discard(id(chain[-1]))
    marked_fixed = {id(fixed[0])}
    for mp in lmps:
        for k in sorted(mp.obs, key=lambda k: k.addr):
            if id(k) in marked_local or id(k) in marked_fixed:
                continue
            marked_fixed.add(id(k))
            if not k.isBad():
                fixed.append(k)
                break
        if len(fixed) >= 200:
            break
    return opt, fixed, lmps, marked_local, marked_fixed


def _reset(kfs, mps):
    for k in kfs:
        k.mnBALocalForKF = k.mnBAFixedForKF = -1
    for m in mps:
        m.mnBALocalForKF = -1


def test_window_matches_independent_restatement():
    for seed, (n_opt, n_cov) in enumerate([(10, 10), (10, 3), (4, 12), (12, 0)]):
        pb = synth.lia_problem(20 + seed, n_opt=n_opt, n_fixed_cov=n_cov, n_pts=300, max_obs=6)
        n = len(pb.kfs)
        kfs, mps, M = build_map(pb, seed, p_bad_mp=0.05, bad_kf=[n - 2], foreign_kf=[n - 3])
        for pick in (0, 1, 3):
            _reset(kfs, mps)
            pKF = kfs[pick]
            opt, fixed, lmps, ml, mf = reference_window(pKF)
            _reset(kfs, mps)
            win = gather_inertial_window(pKF, pb.calib)
            assert [k.id_ for k in win.opt_kfs] == [k.id_ for k in opt]
            assert [k.id_ for k in win.fixed_kfs] == [k.id_ for k in fixed]
            assert [m.id_ for m in win.local_mps] == [m.id_ for m in lmps]
            for k in kfs:
                assert (k.mnBALocalForKF == pKF.id_) == (id(k) in ml), k.id_
                assert (k.mnBAFixedForKF == pKF.id_) == (id(k) in mf), k.id_
            # links: one per temporal key frame whose mPrevKF is a vertex; the last one robust,
            # down-weighted
            N = len(opt)
            assert len(win.imu_edges) == N
            assert list(win.imu_edges["kf2"]) == list(range(N))
            assert [win.imu_edges["flags"][i] for i in range(N)] == [0] * (N - 1) + [3]
            # visual edges: observers that are window vertices, good, of the map
            kf_order = opt + fixed
            exp = []
            for p, mp in enumerate(lmps):
                for k in sorted(mp.obs, key=lambda k: k.addr):
                    if (id(k) in ml or id(k) in mf) and not k.isBad() and k.GetMap() is M \
                            and any(k is q for q in kf_order):
                        exp.append((p, [q.id_ for q in kf_order].index(k.id_)))
            assert [(int(e["point"]), int(e["kf"])) for e in win.edges] == exp
            assert list(win.fixed) == [0] * N + [1] * len(fixed)
            assert np.array_equal(win.close, [m.mTrackDepth < 10 for m in lmps])


def test_chain_reaching_the_first_keyframe_pops():
    """Nd larger than the chain: the oldest key frame becomes the fixed one
    (mnBALocalForKF reset to 0, :2381-2385) and gets no link."""
    pb = synth.lia_problem(31, n_opt=5, n_fixed_cov=0, n_pts=200, max_obs=5)
    kfs, mps, M = build_map(pb)
    M.n = 40  # Nd = min(38, 10) = 10 > the 6-key-frame chain
    win = gather_inertial_window(kfs[0], pb.calib)
    assert [k.id_ for k in win.opt_kfs] == [k.id_ for k in kfs[:5]]
    assert win.fixed_kfs[0] is kfs[5] and kfs[5].mnBALocalForKF == 0
    assert len(win.imu_edges) == 5 and win.imu_edges["kf1"][-1] == 5
    assert win.imu_edges["flags"][-1] == 3


def test_large_and_rec_init_flags():
    pb = synth.lia_problem(32, n_opt=25, n_fixed_cov=2, n_pts=200, max_obs=5)
    kfs, mps, M = build_map(pb)
    win = gather_inertial_window(kfs[0], pb.calib, b_large=True, b_rec_init=True)
    assert len(win.opt_kfs) == min(M.n - 2, 25) == 25
    assert (win.imu_edges["flags"] & 1).all() and win.imu_edges["flags"][-1] == 3
    assert win.iterations == 4 and win.lambda_init == 1e-2


def test_gathered_window_solves_and_writes_back():
    import binding as oracle

    pb = synth.lia_problem(33, n_opt=10, n_fixed_cov=4, n_pts=400, max_obs=6)
    kfs, mps, M = build_map(pb)
    win = gather_inertial_window(kfs[0], pb.calib)
    r = oracle.lia(win)
    assert r["stats"][1] < r["stats"][0]
    res = {"stats": r["stats"], "outlier": r["outlier"], "pts": r["pts"].astype(np.float32),
           "kfs": np.array(win.kfs)}
    res["outlier"] = np.zeros(len(win.edges), np.uint8)
    res["outlier"][::5] = 1
    win.local_mps[0]._bad = True
    wb = write_back_inertial(win, res)
    assert not wb["failed"]
    mono = win.edges["ur"] < 0
    exp = [win.edge_refs[e] for sel in (np.nonzero(mono)[0], np.nonzero(~mono)[0]) for e in sel
           if res["outlier"][e] and not win.edge_refs[e][1].isBad()]
    assert [(k.id_, m.id_) for k, m in wb["to_erase"]] == [(k.id_, m.id_) for k, m in exp]
    assert [u[0].id_ for u in wb["kf_updates"]] == [k.id_ for k in win.opt_kfs]
    # the FAIL test: 2 err < err_end (floats) fails unless bLarge; NaN fails
    for st0, st1, large, fail in [(10.0, 20.5, False, True), (10.0, 19.9, False, False),
                                  (10.0, 25.0, True, False), (np.nan, 1.0, False, True)]:
        win.b_large = large
        res["stats"] = np.array([st0, st1, 0, 0, 0, 0, 0])
        assert write_back_inertial(win, res)["failed"] == fail
