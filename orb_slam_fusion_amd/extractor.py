"""Host mirror of ORB_SLAM_FUSION::OrbExtractor over the gfx950 C ABI.

Same constructor arguments, getters, call semantics and error behaviour as
the reference class (include/cam/orb_feature/orb_extractor.h:44-104,
src/cam/orb_feature/orb_extractor.cc:407-465, 1011-1117):

* ``OrbExtractor(num_feats, scale_factor, num_levs, ini_th_fast, min_th_fast)``
* ``extractor(img, mask, lapping_areas) -> (mono_index, keypoints, descriptors)``
  where ``keypoints`` is a structured array in cv::KeyPoint field order and
  ``descriptors`` is N x 32 uint8 (row i describes keypoint i).  An empty image
  returns ``(-1, empty, None)`` like ``operator()`` returning -1 with
  ``descs`` untouched; a non-uint8 / non-2-D image raises (the reference
  asserts CV_8UC1).  The mask is ignored, as in the reference.
* ``img_pyramid_`` holds the host copies of the pyramid levels of the last
  call (read by Frame::ComputeStereoMatches, frame.cc:834,913-933).
* ``extract_batch`` is the device-resident throughput path (torch tensors).
"""
from __future__ import annotations

import contextlib
import ctypes
from typing import Optional, Sequence, Tuple

import numpy as np

from . import _lib
from ._lib import KEYPOINT_DTYPE, OrbParams, check, lib, ptr


class OrbExtractor:
    def __init__(
        self,
        num_feats: int,
        scale_factor: float,
        num_levs: int,
        ini_th_fast: int,
        min_th_fast: int,
        *,
        device: int = 0,
        max_width: int = 752,
        max_height: int = 480,
        max_images: int = 1,
    ):
        self._params = OrbParams(num_feats, scale_factor, num_levs, ini_th_fast, min_th_fast)
        self.num_feats_ = num_feats
        self.num_levs_ = num_levs
        self._h = ctypes.c_void_p()
        check(
            lib().orbgpu_extractor_create(
                ctypes.byref(self._params), device, max_width, max_height, max_images,
                ctypes.byref(self._h),
            ),
            "orbgpu_extractor_create",
        )
        L = num_levs
        self._scale = np.zeros(L, np.float32)
        self._inv_scale = np.zeros(L, np.float32)
        self._sigma2 = np.zeros(L, np.float32)
        self._inv_sigma2 = np.zeros(L, np.float32)
        check(
            lib().orbgpu_extractor_scales(
                self._h, ptr(self._scale), ptr(self._inv_scale), ptr(self._sigma2),
                ptr(self._inv_sigma2),
            ),
            "orbgpu_extractor_scales",
        )
        self._pyr_valid = False
        self._pyr = []

    # -- getters (orb_extractor.h:60-74; return copies, like the by-value getters)
    def GetLevels(self) -> int:
        return self.num_levs_

    def GetScaleFactor(self) -> float:
        return float(self._params.scale_factor)

    def GetScaleFactors(self) -> np.ndarray:
        return self._scale.copy()

    def GetInverseScaleFactors(self) -> np.ndarray:
        return self._inv_scale.copy()

    def GetScaleSigmaSquares(self) -> np.ndarray:
        return self._sigma2.copy()

    def GetInverseScaleSigmaSquares(self) -> np.ndarray:
        return self._inv_sigma2.copy()

    def set_resize_rounding(self, mode: int) -> None:
        """The resize vertical pass's column split:
        ORBGPU_RESIZE_SSE (OpenCV 4.5.4 128-bit SIMD body + scalar tail,
        default) or ORBGPU_RESIZE_SCALAR (every column the scalar rounding)."""
        check(lib().orbgpu_extractor_set_resize_rounding(self._h, int(mode)),
              "orbgpu_extractor_set_resize_rounding")

    def set_stage_event(self, stage: int, event) -> None:
        """Record ``event`` (a torch.cuda.Event, already created by one record,
        or a raw hipEvent_t; None clears) after ``stage`` (0 pyramid .. 5
        assembly) of every later extract_batch: the signal another stream
        waits on to run its batch part-way behind this one."""
        raw = None if event is None else int(getattr(event, "cuda_event", event))
        check(lib().orbgpu_extractor_set_stage_event(self._h, int(stage), ctypes.c_void_p(raw)),
              "orbgpu_extractor_set_stage_event")

    def set_pyramid_launch(self, mode: int) -> None:
        """ORBGPU_PYRAMID_PER_LEVEL (0, default: a launch per level) or
        ORBGPU_PYRAMID_FUSED (1: one k_pyramid launch, a workgroup per image)."""
        check(lib().orbgpu_extractor_set_pyramid_launch(self._h, int(mode)),
              "orbgpu_extractor_set_pyramid_launch")

    def set_single_launch(self, mode: int) -> None:
        """How __call__ runs on the device: ORBGPU_SINGLE_DATAFLOW (0, default:
        one persistent dataflow launch) or ORBGPU_SINGLE_GRAPH (1: the per-stage
        launches replayed as a hipGraph); same results."""
        check(lib().orbgpu_extractor_set_single_launch(self._h, int(mode)),
              "orbgpu_extractor_set_single_launch")

    def set_octree_nodes(self, mode: int) -> None:
        """Where DistributeOctTree's node list lives: ORBGPU_OCTREE_NODES_AUTO
        (0: LDS when it fits the workgroup, else HBM) or ORBGPU_OCTREE_NODES_HBM
        (1: always HBM; same results)."""
        check(lib().orbgpu_extractor_set_octree_nodes(self._h, int(mode)),
              "orbgpu_extractor_set_octree_nodes")

    def max_keypoints(self, width: int, height: int) -> int:
        return int(lib().orbgpu_extractor_max_keypoints(self._h, width, height))

    def _out_buffers(self, w: int, h: int):
        """(cap, keypoints, descriptors) staging arrays for a w x h image, kept
        between calls (every result is returned as a copy of its first n rows)."""
        key = (w, h)
        if getattr(self, "_out_key", None) != key:
            cap = max(self.max_keypoints(w, h), 1)
            self._out = (cap, np.zeros(cap, KEYPOINT_DTYPE), np.zeros((cap, 32), np.uint8))
            self._out_key = key
        return self._out

    # -- operator() (orb_extractor.cc:1011-1091)
    def __call__(
        self,
        img: np.ndarray,
        mask=None,
        lapping_areas: Sequence[int] = (0, 0),
    ) -> Tuple[int, np.ndarray, Optional[np.ndarray]]:
        if img is None or img.size == 0:
            return -1, np.zeros(0, KEYPOINT_DTYPE), None
        if img.dtype != np.uint8 or img.ndim != 2:
            raise AssertionError("OrbExtractor expects a CV_8UC1 image")
        img = np.ascontiguousarray(img)
        h, w = img.shape
        cap, kps, descs = self._out_buffers(w, h)
        n = ctypes.c_int()
        mono = ctypes.c_int()
        lap = (ctypes.c_int * 2)(int(lapping_areas[0]), int(lapping_areas[1]))
        st = lib().orbgpu_extract(
            self._h, ptr(img), w, h, w, lap, ptr(kps), ptr(descs), cap, ctypes.byref(n),
            ctypes.byref(mono),
        )
        if st == _lib.ORBGPU_ERR_EMPTY:
            return -1, np.zeros(0, KEYPOINT_DTYPE), None
        check(st, "orbgpu_extract")
        self._pyr_valid = False
        N = n.value
        return mono.value, kps[:N].copy(), (descs[:N].copy() if N > 0 else None)

    def extract_stereo(self, right: "OrbExtractor", img_left: np.ndarray, img_right: np.ndarray,
                       lapping_left: Sequence[int] = (0, 0), lapping_right: Sequence[int] = (0, 0)):
        """Both images of a stereo frame from this thread (orbgpu_extract_stereo):
        this handle takes the left image, `right` the right one; returns the
        two operator() results ((mono, keypoints, descriptors) each)."""
        outs = []
        args = []
        for ex, img, lp in ((self, img_left, lapping_left), (right, img_right, lapping_right)):
            img = np.ascontiguousarray(img)
            if img.dtype != np.uint8 or img.ndim != 2:
                raise AssertionError("OrbExtractor expects a CV_8UC1 image")
            cap, kb, db = ex._out_buffers(img.shape[1], img.shape[0])
            o = (kb, db, ctypes.c_int(), ctypes.c_int(), (ctypes.c_int * 2)(int(lp[0]), int(lp[1])), img, cap)
            outs.append(o)
        (kl, dl, nl, ml, ll, il, cl), (kr, dr, nr, mr, lr, ir, cr) = outs
        if il.shape != ir.shape:
            raise ValueError("the stereo images differ in size")
        h, w = il.shape
        st = lib().orbgpu_extract_stereo(
            self._h, right._h, ptr(il), ptr(ir), w, h, w, ll, lr, ptr(kl), ptr(dl), cl, ctypes.byref(nl),
            ctypes.byref(ml), ptr(kr), ptr(dr), cr, ctypes.byref(nr), ctypes.byref(mr))
        check(st, "orbgpu_extract_stereo")
        self._pyr_valid = False
        right._pyr_valid = False
        return tuple((m.value, k[:n.value].copy(), d[:n.value].copy() if n.value > 0 else None)
                     for k, d, n, m in ((kl, dl, nl, ml), (kr, dr, nr, mr)))

    @property
    def img_pyramid_(self):
        if not self._pyr_valid:
            out = []
            for lev in range(self.num_levs_):
                data = ctypes.c_void_p()
                w, h, s = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
                check(
                    lib().orbgpu_extractor_pyramid_level(
                        self._h, lev, ctypes.byref(data), ctypes.byref(w), ctypes.byref(h),
                        ctypes.byref(s),
                    ),
                    "orbgpu_extractor_pyramid_level",
                )
                buf = (ctypes.c_uint8 * (s.value * h.value)).from_address(data.value)
                arr = np.frombuffer(buf, np.uint8).reshape(h.value, s.value)[:, : w.value]
                out.append(arr.copy())
            self._pyr = out
            self._pyr_valid = True
        return self._pyr

    # -- device-resident batch (throughput path)
    def extract_batch(self, imgs, kps_out, descs_out, n_out, mono_out, lapping_areas=(0, 0),
                      stream=None) -> None:
        """imgs: uint8 CUDA tensor [B, H, W]; kps_out: [B, cap, 7] 4-byte elements;
        descs_out: uint8 [B, cap, 32]; n_out / mono_out: int32 [B].  Asynchronous
        on ``stream`` (torch stream or raw handle; default the current torch stream)."""
        B, H, W = imgs.shape
        cap = descs_out.shape[1]
        lap = (ctypes.c_int * 2)(int(lapping_areas[0]), int(lapping_areas[1]))
        with launch_stream(stream) as s:
            check(
                lib().orbgpu_extract_batch(
                    self._h, ptr(imgs), B, W, H, imgs.stride(1), imgs.stride(0), lap, ptr(kps_out),
                    ptr(descs_out), cap, ptr(n_out), ptr(mono_out), s,
                ),
                "orbgpu_extract_batch",
            )

    def stereo_match_batch(self, imgs, kps, descs, n, bf: float, mb: float, uright, depth,
                           stream=None) -> None:
        """Frame::ComputeStereoMatches (frame.cc:828-986) for the B/2 stereo frames
        of this handle's last extract_batch call (images [L0, R0, L1, R1, ...]):
        imgs, kps, descs, n are that call's arguments; uright / depth: float32
        CUDA tensors [B/2, cap] (-1 = unmatched).  bf = Frame::bf_, mb = Frame::mb."""
        B = imgs.shape[0]
        cap = descs.shape[1]
        with launch_stream(stream) as s:
            check(
                lib().orbgpu_stereo_match_batch(
                    self._h, B // 2, ptr(imgs), imgs.stride(1), imgs.stride(0), ptr(kps), ptr(descs),
                    cap, ptr(n), float(bf), float(mb), ptr(uright), ptr(depth), s,
                ),
                "orbgpu_stereo_match_batch",
            )

    STAGES = ("resize", "blur", "fast_cells", "octree", "describe", "assemble")

    def profile(self, max_calls: int) -> None:
        """Record HIP events between the kernel stages of the next max_calls
        extract_batch calls (on the launch stream)."""
        check(lib().orbgpu_extractor_profile(self._h, max_calls), "orbgpu_extractor_profile")

    def profile_read(self):
        """-> (calls, {stage: summed ms})."""
        ms = np.zeros(6, np.float64)
        calls = lib().orbgpu_extractor_profile_read(self._h, ptr(ms))
        if calls < 0:
            raise RuntimeError("orbgpu_extractor_profile_read failed")
        return calls, dict(zip(self.STAGES, ms.tolist()))

    def check(self) -> None:
        check(lib().orbgpu_extractor_check(self._h), "orbgpu_extractor_check")

    def close(self) -> None:
        if self._h:
            lib().orbgpu_extractor_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_side_streams = {}


@contextlib.contextmanager
def launch_stream(stream):
    """Stream handle for a batch launch, ordered with torch's work.

    ``stream``: None -> torch's current stream; a torch stream; or a raw int
    handle (0 = the library handle's own stream, unordered: the caller
    synchronises).  The ABI reads a NULL handle as "the library handle's own
    stream", so torch's legacy default stream (handle 0) cannot be named
    through it: the launch then goes to a side stream that first waits for the
    default stream and that the default stream waits for afterwards, keeping
    torch's allocations, fills and copies ordered with the kernels."""
    if isinstance(stream, int):
        yield ctypes.c_void_p(stream)
        return
    import torch

    cur = torch.cuda.current_stream() if stream is None else stream
    if cur.cuda_stream != 0:
        yield ctypes.c_void_p(cur.cuda_stream)
        return
    side = _side_streams.get(cur.device)
    if side is None:
        side = _side_streams[cur.device] = torch.cuda.Stream(device=cur.device)
    side.wait_stream(cur)
    try:
        yield ctypes.c_void_p(side.cuda_stream)
    finally:
        cur.wait_stream(side)
