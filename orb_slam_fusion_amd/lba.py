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

from ._lib import LBA_EDGE_DTYPE, LBA_REDUCE_FN, Camera, check, lib, ptr


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

    def optimize(self, problem, iterations: int = 10, pt_range=None, group=None,
                 stop_flag: Optional[ctypes.c_uint8] = None, lambda_init: float = 0.0) -> dict:
        """Returns {"poses": float32 [n_kf, 7], "poses_d": float64 [n_kf, 7],
        "pts": float32 [n_pts, 3] (this shard's rows), "outlier": uint8 [E]
        (this shard's edges), "stats": float64 [6]}.  ``group``: a
        torch.distributed group whose ranks hold the other point shards.
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
        if group is None:
            cb = LBA_REDUCE_FN(0)
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
