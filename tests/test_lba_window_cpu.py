"""The LocalBundleAdjustment window gather (optimizer.cc:1057-1124), graph
(:1150-1354) and write-back (:1362-1441) of orb_slam_fusion_amd.lba against an
independent set-based restatement, on synthetic map graphs with bad
keyframes / points, keyframes of another map, covisible keyframes that are
bad or foreign (marked local without joining), and the 0-fixed-keyframe
abort."""
import sys
from collections import OrderedDict
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "oracle"))

from orb_slam_fusion_amd.lba import gather_window, write_back  # noqa: E402


class Map:
    def __init__(self, init_id):
        self.init_id = init_id

    def GetInitKFid(self):
        return self.init_id


class KP:
    def __init__(self, x, y, octave):
        self.x, self.y, self.octave = x, y, octave


class KeyFrame:
    def __init__(self, kid, mp, bad, addr, pose, n_kp, rng):
        self.id_, self._map, self._bad, self.addr = kid, mp, bad, addr
        self._pose = pose
        self.mnBALocalForKF = self.mnBAFixedForKF = -1
        self.mvKeysUn = [KP(float(rng.uniform(0, 752)), float(rng.uniform(0, 480)),
                            int(rng.integers(0, 8))) for _ in range(n_kp)]
        self.mvuRight = [float(rng.uniform(0, 700)) if rng.random() < 0.5 else -1.0
                         for _ in range(n_kp)]
        self.mvInvLevelSigma2 = [float(1.0 / 1.44 ** l) for l in range(8)]
        self.matches = [None] * n_kp
        self.covis = []

    def isBad(self):
        return self._bad

    def GetMap(self):
        return self._map

    def GetPose(self):
        return self._pose

    def GetVectorCovisibleKeyFrames(self):
        return list(self.covis)

    def GetMapPointMatches(self):
        return list(self.matches)


class MapPoint:
    def __init__(self, pid, mp, bad, pos):
        self.id_, self._map, self._bad, self._pos = pid, mp, bad, pos
        self.mnBALocalForKF = -1
        self.obs = {}

    def isBad(self):
        return self._bad

    def GetMap(self):
        return self._map

    def GetWorldPos(self):
        return self._pos

    def GetObservations(self):  # std::map<KeyFrame*, ...>: key (pointer) order
        return OrderedDict(sorted(self.obs.items(), key=lambda kv: kv[0].addr))


def make_graph(seed, n_kf=30, n_mp=400, init_id=0, p_bad_kf=0.1, p_other=0.1, p_bad_mp=0.05):
    rng = np.random.default_rng(seed)
    A, B = Map(init_id), Map(init_id)
    addrs = rng.permutation(n_kf) * 64 + 4096
    kfs = []
    for k in range(n_kf):
        m = B if (k > 0 and rng.random() < p_other) else A
        bad = k > 0 and rng.random() < p_bad_kf
        pose = np.array([0, 0, 0, 1, 0.1 * k, 0, 0], np.float32)
        kfs.append(KeyFrame(k, m, bad, int(addrs[k]), pose, 300, rng))
    mps = []
    for p in range(n_mp):
        mp = MapPoint(p, B if rng.random() < p_other else A, rng.random() < p_bad_mp,
                      rng.normal(size=3).astype(np.float32) + np.array([0, 0, 5], np.float32))
        c = int(rng.integers(0, n_kf))
        for k in sorted(set(int(x) % n_kf for x in c + rng.integers(0, 6, size=int(rng.integers(2, 6))))):
            kf = kfs[k]
            free = [i for i, m in enumerate(kf.matches) if m is None]
            left = int(rng.choice(free))
            kf.matches[left] = mp
            mp.obs[kf] = (left, -1)
        mps.append(mp)
    for kf in kfs:  # covisibility by shared points, weight descending (ties by id)
        w = {}
        for mp in kf.matches:
            if mp is None:
                continue
            for o in mp.obs:
                if o is not kf:
                    w[o] = w.get(o, 0) + 1
        kf.covis = [o for o, c in sorted(w.items(), key=lambda kv: (-kv[1], kv[0].id_)) if c >= 2]
    return kfs, mps, A


def reference_sets(pKF, pMap):
    """Independent restatement: the window as sets and first-occurrence orders."""
    cur = pKF.GetMap()
    good = lambda k: not k.isBad() and k.GetMap() is cur  # noqa: E731
    cov = pKF.covis
    marked_local = {id(pKF)} | {id(k) for k in cov}
    local = [pKF] + [k for k in cov if good(k)]
    seen, local_mps = set(), []
    for k in local:
        for mp in k.matches:
            if mp is not None and not mp.isBad() and mp.GetMap() is cur and id(mp) not in seen:
                seen.add(id(mp))
                local_mps.append(mp)
    seen_f, fixed = set(), []
    for mp in local_mps:
        for k in sorted(mp.obs, key=lambda k: k.addr):
            if id(k) in marked_local or id(k) in seen_f:
                continue
            seen_f.add(id(k))
            if good(k):
                fixed.append(k)
    nfix = int(any(k.id_ == pMap.GetInitKFid() for k in local)) + len(fixed)
    edges = []
    for p, mp in enumerate(local_mps):
        for k in sorted(mp.obs, key=lambda k: k.addr):
            if good(k):
                edges.append((p, k, mp.obs[k][0]))
    return local, fixed, local_mps, nfix, edges, marked_local, seen_f


def test_window_matches_independent_restatement():
    for seed in range(12):
        kfs, mps, A = make_graph(seed)
        for pick in (5, 17, 29):
            for k in kfs:
                k.mnBALocalForKF = k.mnBAFixedForKF = -1
            for m in mps:
                m.mnBALocalForKF = -1
            pKF = kfs[pick]
            if pKF.isBad():
                continue
            ref = reference_sets(pKF, A)
            win = gather_window(pKF, A, [458.654, 457.296, 367.215, 248.375, 50.45])
            local, fixed, lmps, nfix, edges, marked_local, marked_fixed = ref
            if nfix == 0:
                assert win is None
                continue
            assert [k.id_ for k in win.local_kfs] == [k.id_ for k in local]
            assert [k.id_ for k in win.fixed_kfs] == [k.id_ for k in fixed]
            assert [m.id_ for m in win.local_mps] == [m.id_ for m in lmps]
            assert win.num_fixedKF == nfix and win.num_OptKF == len(local)
            # the marks the reference leaves behind
            for k in kfs:
                assert (k.mnBALocalForKF == pKF.id_) == (id(k) in marked_local)
                assert (k.mnBAFixedForKF == pKF.id_) == (id(k) in marked_fixed)
            kf_order = local + fixed
            assert len(win.edges) == len(edges)
            for e, (p, k, left) in zip(win.edges, edges):
                assert e["point"] == p and e["kf"] == kf_order.index(k)
                assert e["u"] == np.float32(k.mvKeysUn[left].x)
                ur = k.mvuRight[left]
                assert e["ur"] == (np.float32(ur) if ur >= 0 else -1.0)
                assert e["inv_sigma2"] == np.float32(k.mvInvLevelSigma2[k.mvKeysUn[left].octave])
            fx = win.fixed.astype(bool)
            assert all(fx[len(local):]) and \
                all(fx[i] == (k.id_ == A.GetInitKFid()) for i, k in enumerate(local))


def test_zero_fixed_keyframes_aborts():
    """Init keyframe outside the window and every observer of the local points
    local: the reference returns before building the optimizer (:1119-1124)."""
    kfs, mps, A = make_graph(3, n_kf=6, n_mp=60, init_id=99, p_bad_kf=0, p_other=0, p_bad_mp=0)
    pKF = kfs[2]
    pKF.covis = [k for k in kfs if k is not pKF]  # everyone covisible -> no fixed camera
    assert gather_window(pKF, A, [1, 1, 0, 0, 1]) is None
    assert reference_sets(pKF, A)[3] == 0


def test_write_back_order_and_solve():
    """Write-back erases mono observations first, then stereo, skipping bad
    points; the gathered problem is solvable by the oracle (chi2 decreases)."""
    import binding as oracle

    kfs, mps, A = make_graph(7, n_kf=12, n_mp=200, init_id=0, p_bad_kf=0, p_other=0, p_bad_mp=0)
    rng = np.random.default_rng(1)
    # consistent observations: project the points with the poses, small noise
    for mp in mps:
        for k, (left, _) in mp.obs.items():
            X = np.asarray(mp.GetWorldPos(), np.float64) + np.asarray(k.GetPose()[4:], np.float64)
            kp = k.mvKeysUn[left]
            kp.x = float(458.654 * X[0] / X[2] + 367.215 + rng.normal(0, 1))
            kp.y = float(457.296 * X[1] / X[2] + 248.375 + rng.normal(0, 1))
            if k.mvuRight[left] >= 0:
                k.mvuRight[left] = float(kp.x - 50.45 / X[2])
    win = gather_window(kfs[4], A, [458.654, 457.296, 367.215, 248.375, 50.45])
    assert win is not None and len(win.edges) > 50
    r = oracle.lba(win)
    assert r["stats"][1] < r["stats"][0]
    res = {"outlier": r["outlier"], "poses": r["poses"].astype(np.float32),
           "pts": r["pts"].astype(np.float32)}
    res["outlier"] = np.zeros(len(win.edges), np.uint8)
    res["outlier"][::7] = 1
    win.local_mps[0]._bad = True  # a point gone bad during the solve is skipped
    to_erase, kf_poses, mp_pos = write_back(win, res)
    mono = win.edges["ur"] < 0
    exp = [win.edge_refs[e] for sel in (np.nonzero(mono)[0], np.nonzero(~mono)[0]) for e in sel
           if res["outlier"][e] and not win.edge_refs[e][1].isBad()]
    assert [(k.id_, m.id_) for k, m in to_erase] == [(k.id_, m.id_) for k, m in exp]
    assert [k.id_ for k, _ in kf_poses] == [k.id_ for k in win.local_kfs]
    assert len(mp_pos) == len(win.local_mps)
