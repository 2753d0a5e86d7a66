"""Host mirror of Optimizer::LocalBundleAdjustment's solve over the gfx950 C ABI.

The caller gathers the window as the reference does (optimizer.cc:1057-1124:
local keyframes, their map points, fixed keyframes) into an LbaProblem-like
object (``cam``, ``poses_init``, ``fixed``, ``pts_init``, ``edges``);
``LocalBundleAdjuster.optimize`` runs optimize(10) (g2o LM with the Schur
complement on the points, :1359-1360) and the outlier test (:1362-1400) on
the GPU and returns what the reference writes back (:1402-1441).

Multi-GPU: with a torch.distributed process group, each rank
passes its point shard; the partial reduced camera system, the chi2 and the
LM scale are all-reduced through ``dist_reduce`` (RCCL for device buffers,
gloo for host arrays) and every rank solves the small system redundantly.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import numpy as np

from ._lib import (IMU_STATE_DTYPE, LBA_EDGE_DTYPE, LBA_REDUCE_FN, LIA_IMU_EDGE_DTYPE, Camera, check,
                   lib, ptr)


class _DeviceDoubles:
    """Zero-copy view of a library-owned device buffer for torch.as_tensor."""

    def __init__(self, addr: int, n: int):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "<f8", "data": (addr, False),
                                         "version": 2, "strides": None}


def dist_reduce(group=None):
    """-> reduce(buf, op) completing a point-sharded sum (op 0) / max (op 1)
    across the ranks of ``group`` in place.  ``buf`` is a torch tensor (any
    device) or a numpy array (host; shares memory through torch.from_numpy)."""
    import torch
    import torch.distributed as dist

    def reduce(buf, op: int) -> None:
        t = torch.from_numpy(buf) if isinstance(buf, np.ndarray) else buf
        rop = dist.ReduceOp.MAX if op == 1 else dist.ReduceOp.SUM
        if t.is_cuda and dist.get_backend(group) == "gloo":
            # gloo moves host memory: stage the device buffer through the host
            h = t.cpu()
            dist.all_reduce(h, op=rop, group=group)
            t.copy_(h)
        else:
            dist.all_reduce(t, op=rop, group=group)
        if t.is_cuda:
            torch.cuda.synchronize(t.device)

    return reduce


def dist_enqueue(group=None, device: int = 0):
    """-> enqueue(ptr, n, op, stream) for the stream-ordered sharded call
    (orbgpu_lba_ctx_set_reduce_ordered): the all-reduce of the library's
    device buffer goes onto the library's HIP stream.  RCCL (backend "nccl")
    runs it in stream order without a host wait (torch makes its collective
    stream wait on the current stream and the current stream on the result);
    gloo has no device path, so it stages through the host (a host wait per
    reduction: the two-ranks-on-one-GPU test path)."""
    import torch
    import torch.distributed as dist

    dev = torch.device("cuda", device)
    gloo = dist.get_backend(group) == "gloo"

    def enqueue(d_buf: int, n: int, op: int, stream: int) -> None:
        rop = dist.ReduceOp.MAX if op == 1 else dist.ReduceOp.SUM
        ext = torch.cuda.ExternalStream(stream, device=dev)
        with torch.cuda.stream(ext):
            t = torch.as_tensor(_DeviceDoubles(d_buf, n), device=dev)
            if gloo:
                h = t.cpu()  # synchronises with the stream's pending work
                dist.all_reduce(h, op=rop, group=group)
                t.copy_(h)
            else:
                dist.all_reduce(t, op=rop, group=group)

    return enqueue


class LocalBundleAdjuster:
    def __init__(self, device: int = 0):
        self.device = device
        self._h = ctypes.c_void_p()
        check(lib().orbgpu_lba_ctx_create(device, ctypes.byref(self._h)), "orbgpu_lba_ctx_create")

    def close(self) -> None:
        if self._h:
            lib().orbgpu_lba_ctx_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_solver(self, solver: int) -> None:
        """Forces the reduced-system path (_lib.ORBGPU_LBA_SOLVER_*; AUTO by
        default): A/B timing and the path-equivalence tests."""
        check(lib().orbgpu_lba_ctx_set_solver(self._h, int(solver)), "orbgpu_lba_ctx_set_solver")

    def set_schur(self, mode: int) -> None:
        """The Schur complement's path (_lib.ORBGPU_LBA_SCHUR_*: SPLIT by
        point range, the default; PAIR; BAND)."""
        check(lib().orbgpu_lba_ctx_set_schur(self._h, int(mode)), "orbgpu_lba_ctx_set_schur")

    def set_relinearize(self, on: bool) -> None:
        """Re-linearise every LM build instead of taking the accepted trial's
        terms (bit-identical; the test of that identity)."""
        check(lib().orbgpu_lba_ctx_set_relinearize(self._h, 1 if on else 0), "orbgpu_lba_ctx_set_relinearize")

    def set_memory_limit(self, nbytes: int) -> None:
        """Device-memory budget of the context (0 = none): a window over it
        raises ORBGPU_ERR_NOMEM before any device work."""
        check(lib().orbgpu_lba_ctx_set_memory_limit(self._h, int(nbytes)), "orbgpu_lba_ctx_set_memory_limit")

    def optimize(self, problem, iterations: int = 10, pt_range=None, group=None,
                 stop_flag: Optional[ctypes.c_uint8] = None, lambda_init: float = 0.0,
                 ordered: bool = False) -> dict:
        """Returns {"poses": float32 [n_kf, 7], "poses_d": float64 [n_kf, 7],
        "pts": float32 [n_pts, 3] (this shard's rows), "outlier": uint8 [E]
        (this shard's edges), "stats": float64 [6]}.  ``group``: a
        torch.distributed group whose ranks hold the other point shards.
        ``ordered``: with a group, the reductions are enqueued on the library's
        stream and the LM loop stays on the device (dist_enqueue).
        ``lambda_init`` > 0: g2o's setUserLambdaInit (100 for an inertial map,
        optimizer.cc:1137).  ``stop_flag``: the reference's pbStopFlag, read
        by the device where g2o polls terminate()."""
        cam = Camera(*[float(v) for v in problem.cam])
        poses = np.ascontiguousarray(problem.poses_init, np.float32)
        fixed = np.ascontiguousarray(problem.fixed, np.uint8)
        pts = np.ascontiguousarray(problem.pts_init, np.float32)
        edges = np.ascontiguousarray(problem.edges, LBA_EDGE_DTYPE)
        n_kf, n_pts, ne = len(poses), len(pts), len(edges)
        b, e = pt_range if pt_range is not None else (0, n_pts)
        po = np.zeros((n_kf, 7), np.float32)
        pd = np.zeros((n_kf, 7), np.float64)
        xo = np.array(pts, copy=True)
        out = np.zeros(max(ne, 1), np.uint8)
        st = np.zeros(6, np.float64)
        check(lib().orbgpu_lba_ctx_set_reduce_ordered(self._h, 1 if (ordered and group is not None) else 0),
              "orbgpu_lba_ctx_set_reduce_ordered")
        if group is None:
            cb = LBA_REDUCE_FN(0)
        elif ordered:
            enq = dist_enqueue(group, self.device)

            def _cb(_user, d_buf, n, op, stream):
                try:
                    enq(d_buf, n, op, stream)
                    return 0
                except Exception:  # noqa: BLE001 -- reported as a failed reduce
                    return -1

            cb = LBA_REDUCE_FN(_cb)
        else:
            import torch

            red = dist_reduce(group)
            dev = torch.device("cuda", self.device)

            def _cb(_user, d_buf, n, op, _stream):
                try:
                    red(torch.as_tensor(_DeviceDoubles(d_buf, n), device=dev), op)
                    return 0
                except Exception:  # noqa: BLE001 -- reported as a failed reduce
                    return -1

            cb = LBA_REDUCE_FN(_cb)
        check(
            lib().orbgpu_lba_optimize(
                self._h, ctypes.byref(cam), n_kf, ptr(poses), ptr(fixed), n_pts, ptr(pts), ne,
                ptr(edges), b, e, iterations, float(lambda_init),
                ctypes.cast(ctypes.byref(stop_flag), ctypes.c_void_p) if stop_flag is not None else None,
                cb, None, ptr(po), ptr(pd), ptr(xo), ptr(out), ptr(st),
            ),
            "orbgpu_lba_optimize",
        )
        return {"poses": po, "poses_d": pd, "pts": xo, "outlier": out[:ne].copy(), "stats": st}

    def optimize_inertial(self, problem, iterations: Optional[int] = None,
                          lambda_init: Optional[float] = None) -> dict:
        """Optimizer::LocalInertialBA's solve (optimizer.cc:2440-2826) on a
        window in the C ABI's layout (``calib``, ``kfs`` IMU_STATE_DTYPE,
        ``fixed``, ``imu``, ``pts_init``, ``close``, ``edges``, ``imu_edges``
        LIA_IMU_EDGE_DTYPE; ``iterations`` / ``lambda_init`` default to the
        problem's, i.e. opt_it and the user lambda of :2334-2339,2448-2459).
        Returns {"kfs": IMU_STATE_DTYPE [n_kf] (float casts), "kfs21": float64
        [n_kf, 21] (Rwb twb v bg ba), "pts": float32 [n_pts, 3], "outlier":
        uint8 [E], "stats": float64 [7] (err, err_end, iterations, trials,
        lambda, outliers, accepted chi2)}."""
        kfs = np.ascontiguousarray(problem.kfs, IMU_STATE_DTYPE)
        fixed = np.ascontiguousarray(problem.fixed, np.uint8)
        imu = np.ascontiguousarray(problem.imu, np.uint8)
        pts = np.ascontiguousarray(problem.pts_init, np.float32)
        close = np.ascontiguousarray(problem.close, np.uint8)
        edges = np.ascontiguousarray(problem.edges, LBA_EDGE_DTYPE)
        links = np.ascontiguousarray(problem.imu_edges, LIA_IMU_EDGE_DTYPE)
        calib = np.array(problem.calib)
        n_kf, n_pts, ne = len(kfs), len(pts), len(edges)
        it = problem.iterations if iterations is None else iterations
        lam = problem.lambda_init if lambda_init is None else lambda_init
        ko = np.zeros(n_kf, IMU_STATE_DTYPE)
        kd = np.zeros((n_kf, 21), np.float64)
        xo = np.array(pts, copy=True)
        out = np.zeros(max(ne, 1), np.uint8)
        st = np.zeros(7, np.float64)
        check(
            lib().orbgpu_lia_optimize(
                self._h, ptr(calib), n_kf, ptr(kfs), ptr(fixed), ptr(imu), n_pts, ptr(pts),
                ptr(close), ne, ptr(edges), len(links), ptr(links), int(it), float(lam), ptr(ko),
                ptr(kd), ptr(xo), ptr(out), ptr(st),
            ),
            "orbgpu_lia_optimize",
        )
        return {"kfs": ko, "kfs21": kd, "pts": xo, "outlier": out[:ne].copy(), "stats": st}


# ---------------------------------------------------------------------------
# Optimizer::LocalBundleAdjustment around the solve: the window gather
# (optimizer.cc:1057-1124), the flat graph handed to the device (:1150-1354)
# and the write-back (:1362-1441), over duck-typed KeyFrame / MapPoint / Map
# objects exposing the reference's members: KeyFrame.id_, mnBALocalForKF,
# mnBAFixedForKF, isBad(), GetMap(), GetVectorCovisibleKeyFrames(),
# GetMapPointMatches(), GetPose() (qx, qy, qz, qw, tx, ty, tz), mvKeysUn
# (objects with .x, .y, .octave), mvuRight, mvInvLevelSigma2; MapPoint.id_,
# mnBALocalForKF, isBad(), GetMap(), GetObservations() (an ordered mapping
# KeyFrame -> (leftIndex, rightIndex), in the std::map's key order),
# GetWorldPos(); Map.GetInitKFid().  (The C++ drop-in, shim/
# optimizer_lba_gpu.cc, is the same code over the real classes.)
# ---------------------------------------------------------------------------
class LbaWindow:
    """One gathered window: the local / fixed keyframes and local map points
    in the reference's list orders, the out-params, and the LbaProblem the
    device solves (edges in insertion order: per local point, its
    observations in map order; pinhole left-index observations only)."""

    def __init__(self, local_kfs, fixed_kfs, local_mps, num_fixedKF, cam, poses, fixed, pts,
                 edges, edge_refs):
        self.local_kfs, self.fixed_kfs, self.local_mps = local_kfs, fixed_kfs, local_mps
        self.num_fixedKF = num_fixedKF
        self.num_OptKF = len(local_kfs)
        self.num_edges = len(edges)
        self.cam, self.poses_init, self.fixed, self.pts_init = cam, poses, fixed, pts
        self.edges = edges
        self.edge_refs = edge_refs  # [(KeyFrame, MapPoint)] per edge


def gather_window(pKF, pMap, cam) -> Optional[LbaWindow]:
    """optimizer.cc:1057-1124 then the graph of :1150-1354.  Returns None when
    the window has no fixed keyframe (the reference prints "LM-LBA: There are
    0 fixed KF in the optimizations, LBA aborted" and returns, :1119-1124).
    The mnBALocalForKF / mnBAFixedForKF marks are written exactly as the
    reference writes them (bad and other-map covisible keyframes are marked
    local without joining the window; every observer of a local point is
    marked fixed once, joining only when good and in the current map)."""
    cur_map = pKF.GetMap()
    kid = pKF.id_
    local_kfs = [pKF]
    pKF.mnBALocalForKF = kid
    for k in pKF.GetVectorCovisibleKeyFrames():
        k.mnBALocalForKF = kid
        if not k.isBad() and k.GetMap() is cur_map:
            local_kfs.append(k)
    num_fixed = 0
    local_mps = []
    init_id = pMap.GetInitKFid()
    for k in local_kfs:
        if k.id_ == init_id:
            num_fixed = 1
        for mp in k.GetMapPointMatches():
            if mp is not None and not mp.isBad() and mp.GetMap() is cur_map \
                    and mp.mnBALocalForKF != kid:
                local_mps.append(mp)
                mp.mnBALocalForKF = kid
    fixed_kfs = []
    for mp in local_mps:
        for k in mp.GetObservations():
            if k.mnBALocalForKF != kid and k.mnBAFixedForKF != kid:
                k.mnBAFixedForKF = kid
                if not k.isBad() and k.GetMap() is cur_map:
                    fixed_kfs.append(k)
    num_fixed += len(fixed_kfs)
    if num_fixed == 0:
        return None
    # vertices: local keyframes (fixed iff the map's initial keyframe), fixed
    # cameras, points; edges per point in observation order (:1150-1310)
    kfs = local_kfs + fixed_kfs
    index = {id(k): i for i, k in enumerate(kfs)}
    poses = np.array([np.asarray(k.GetPose(), np.float32) for k in kfs], np.float32).reshape(-1, 7)
    fixed = np.array([1 if (i >= len(local_kfs) or k.id_ == init_id) else 0
                      for i, k in enumerate(kfs)], np.uint8)
    pts = np.array([np.asarray(mp.GetWorldPos(), np.float32) for mp in local_mps],
                   np.float32).reshape(-1, 3)
    rows, refs = [], []
    for p, mp in enumerate(local_mps):
        for k, (left, _right) in mp.GetObservations().items():
            if k.isBad() or k.GetMap() is not cur_map or left == -1:
                continue
            i = index.get(id(k))
            if i is None:  # a stale local mark (the reference would find no vertex)
                continue
            kp = k.mvKeysUn[left]
            ur = float(k.mvuRight[left])
            rows.append((p, i, kp.x, kp.y, ur if ur >= 0 else -1.0,
                         k.mvInvLevelSigma2[kp.octave]))
            refs.append((k, mp))
    edges = np.array(rows, LBA_EDGE_DTYPE) if rows else np.zeros(0, LBA_EDGE_DTYPE)
    return LbaWindow(local_kfs, fixed_kfs, local_mps, num_fixed, np.asarray(cam, np.float32),
                     poses, fixed, pts, edges, refs)


def write_back(win: LbaWindow, result: dict):
    """optimizer.cc:1362-1441 -> (to_erase, kf_poses, mp_positions): the
    (KeyFrame, MapPoint) observations to erase (mono edges first, then
    stereo, each in insertion order; points already bad skipped), the new
    poses of the local keyframes and the new positions of the local points
    (the caller applies them under Map::mMutexMapUpdate and calls
    UpdateNormalAndDepth / IncreaseChangeIndex)."""
    out = result["outlier"]
    mono = win.edges["ur"] < 0
    to_erase = []
    for sel in (np.nonzero(mono)[0], np.nonzero(~mono)[0]):
        for e in sel:
            k, mp = win.edge_refs[e]
            if not mp.isBad() and out[e]:
                to_erase.append((k, mp))
    kf_poses = [(k, result["poses"][i]) for i, k in enumerate(win.local_kfs)]
    mp_pos = [(mp, result["pts"][p]) for p, mp in enumerate(win.local_mps)]
    return to_erase, kf_poses, mp_pos


# ---------------------------------------------------------------------------
# Optimizer::LocalInertialBA around the solve: the temporal window
# (optimizer.cc:2332-2436), the flat graph (:2461-2781) and the FAIL test /
# write-back (:2796-2901), over duck-typed objects with the reference's
# members.  KeyFrame: id_, mPrevKF, bImu, mnBALocalForKF, mnBAFixedForKF,
# isBad(), GetMap(), GetVectorCovisibleKeyFrames(), GetMapPointMatches(),
# GetImuRotation(), GetImuPosition(), GetRotation(), GetTranslation() (Tcw),
# GetVelocity(), GetGyroBias(), GetAccBias(), mvKeysUn (.x, .y, .octave),
# mvuRight, mvInvLevelSigma2 and mpImuPreintegrated (None, or the
# IMU_PREINT_DTYPE record the C++ drop-in forms from IMU::Preintegrated and
# EdgeInertial's constructor); MapPoint: id_, mnBALocalForKF, isBad(),
# GetObservations() (ordered KeyFrame -> (left, right)), GetWorldPos(),
# mTrackDepth; Map: KeyFramesInMap().  The pinhole Uncertainty2 is 1.  (The
# C++ drop-in, shim/optimizer_lia_gpu.cc, is the same code over the real
# classes.)  LocalInertialBA leaves num_fixedKF / num_OptKF / num_MPs /
# num_edges unwritten, as the reference does.
# ---------------------------------------------------------------------------
class LiaWindow:
    """One gathered temporal window in orbgpu_lia_optimize's layout plus the
    map objects behind it: opt_kfs (pKF, its mPrevKF, ... newest first),
    fixed_kfs (the key frame before the window first), local_mps,
    edge_refs [(KeyFrame, MapPoint)] per visual edge."""

    def __init__(self, **kw):
        self.__dict__.update(kw)


def _kf_state(k):
    s = np.zeros((), IMU_STATE_DTYPE)
    s["Rwb"] = np.asarray(k.GetImuRotation(), np.float32).ravel()
    s["twb"] = np.asarray(k.GetImuPosition(), np.float32)
    s["Rcw"] = np.asarray(k.GetRotation(), np.float32).ravel()
    s["tcw"] = np.asarray(k.GetTranslation(), np.float32)
    s["v"] = np.asarray(k.GetVelocity(), np.float32)
    s["bg"] = np.asarray(k.GetGyroBias(), np.float32)
    s["ba"] = np.asarray(k.GetAccBias(), np.float32)
    return s


def gather_inertial_window(pKF, calib, b_large: bool = False, b_rec_init: bool = False) -> LiaWindow:
    """optimizer.cc:2332-2436 (marks written as the reference writes them),
    then the graph of :2461-2781."""
    cur_map = pKF.GetMap()
    kid = pKF.id_
    max_opt, opt_it = (25, 4) if b_large else (10, 10)
    Nd = min(cur_map.KeyFramesInMap() - 2, max_opt)
    opt = [pKF]
    pKF.mnBALocalForKF = kid
    for _ in range(1, Nd):
        if opt[-1].mPrevKF is None:
            break
        opt.append(opt[-1].mPrevKF)
        opt[-1].mnBALocalForKF = kid
    local_mps = []
    for k in opt:
        for mp in k.GetMapPointMatches():
            if mp is not None and not mp.isBad() and mp.mnBALocalForKF != kid:
                local_mps.append(mp)
                mp.mnBALocalForKF = kid
    fixed = []
    if opt[-1].mPrevKF is not None:
        fixed.append(opt[-1].mPrevKF)
        opt[-1].mPrevKF.mnBAFixedForKF = kid
    else:
        opt[-1].mnBALocalForKF = 0
        opt[-1].mnBAFixedForKF = kid
        fixed.append(opt[-1])
        opt.pop()
    # optimizable covisible (visual) key frames: maxCovKF = 0 admits none (:2388-2412)
    max_fix = 200
    for mp in local_mps:
        for k in mp.GetObservations():
            if k.mnBALocalForKF != kid and k.mnBAFixedForKF != kid:
                k.mnBAFixedForKF = kid
                if not k.isBad():
                    fixed.append(k)
                    break
        if len(fixed) >= max_fix:
            break
    N = len(opt)
    kfs = opt + fixed
    index = {id(k): i for i, k in enumerate(kfs)}
    states = np.array([_kf_state(k) for k in kfs], IMU_STATE_DTYPE)
    fixed_flags = np.array([0] * N + [1] * len(fixed), np.uint8)
    imu = np.array([1 if k.bImu else 0 for k in kfs], np.uint8)
    # inertial links (:2531-2604): temporal key frame i -> its mPrevKF
    links = []
    for i, k in enumerate(opt):
        prev = k.mPrevKF
        if prev is None or not (k.bImu and prev.bImu and k.mpImuPreintegrated is not None):
            continue
        if id(prev) not in index:
            continue  # the reference finds no vertex and skips the edge
        rec = np.zeros((), LIA_IMU_EDGE_DTYPE)
        rec["kf1"], rec["kf2"] = index[id(prev)], i
        rec["flags"] = ((1 | 2) if i == N - 1 else 0) | (1 if b_rec_init else 0)
        rec["preint"] = k.mpImuPreintegrated
        links.append(rec)
    imu_edges = np.array(links, LIA_IMU_EDGE_DTYPE) if links else np.zeros(0, LIA_IMU_EDGE_DTYPE)
    # map point vertices and visual edges (:2648-2781), left-camera observations
    rows, refs = [], []
    for p, mp in enumerate(local_mps):
        for k, (left, _right) in mp.GetObservations().items():
            if k.mnBALocalForKF != kid and k.mnBAFixedForKF != kid:
                continue
            if k.isBad() or k.GetMap() is not cur_map or left == -1:
                continue
            i = index.get(id(k))
            if i is None:  # a stale mark: the reference would find no vertex
                continue
            kp = k.mvKeysUn[left]
            ur = float(k.mvuRight[left])
            rows.append((p, i, kp.x, kp.y, ur if ur >= 0 else -1.0,
                         k.mvInvLevelSigma2[kp.octave] / 1.0))  # / Uncertainty2 (pinhole: 1)
            refs.append((k, mp))
    edges = np.array(rows, LBA_EDGE_DTYPE) if rows else np.zeros(0, LBA_EDGE_DTYPE)
    pts = np.array([np.asarray(mp.GetWorldPos(), np.float32) for mp in local_mps],
                   np.float32).reshape(-1, 3)
    close = np.array([mp.mTrackDepth < np.float32(10.0) for mp in local_mps], np.uint8)
    return LiaWindow(opt_kfs=opt, fixed_kfs=fixed, local_mps=local_mps, edge_refs=refs,
                     calib=np.array(calib), kfs=states, fixed=fixed_flags, imu=imu,
                     pts_init=pts, close=close, edges=edges, imu_edges=imu_edges,
                     iterations=opt_it, lambda_init=1e-2 if b_large else 1e0, b_large=b_large)


def write_back_inertial(win: LiaWindow, result: dict):
    """:2796-2901 -> dict(failed, to_erase, kf_updates, mp_positions).
    failed: the reference's "FAIL LOCAL-INERTIAL BA!!!!" return (err and
    err_end as floats, 2 err < err_end or NaN, unless bLarge): nothing is
    erased or written and the marks stay.  Otherwise to_erase = (KeyFrame,
    MapPoint) pairs, mono edges first, then stereo, bad points skipped;
    kf_updates = (KeyFrame, Rcw, tcw, v, bg, ba) per temporal key frame
    (SetPose, SetVelocity, SetNewBias, float casts); mp_positions =
    (MapPoint, Xw); the caller clears the fixed marks and the temporal
    key frames' local marks as :2847-2888 do."""
    st = result["stats"]
    err, err_end = np.float32(st[0]), np.float32(st[1])
    failed = bool((np.float32(2) * err < err_end or np.isnan(err) or np.isnan(err_end))
                  and not win.b_large)
    if failed:
        return {"failed": True, "to_erase": [], "kf_updates": [], "mp_positions": []}
    out = result["outlier"]
    mono = win.edges["ur"] < 0
    to_erase = []
    for sel in (np.nonzero(mono)[0], np.nonzero(~mono)[0]):
        for e in sel:
            k, mp = win.edge_refs[e]
            if not mp.isBad() and out[e]:
                to_erase.append((k, mp))
    kfo = result["kfs"]
    upd = [(k, kfo[i]["Rcw"].reshape(3, 3), kfo[i]["tcw"], kfo[i]["v"], kfo[i]["bg"], kfo[i]["ba"])
           for i, k in enumerate(win.opt_kfs)]
    mp_pos = [(mp, result["pts"][p]) for p, mp in enumerate(win.local_mps)]
    return {"failed": False, "to_erase": to_erase, "kf_updates": upd, "mp_positions": mp_pos}
