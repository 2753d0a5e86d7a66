"""Frame::ComputeStereoMatches (src/map/frame.cc:828-986) on the GPU.

Host-path mirror of the reference call: the stereo Frame constructor runs
ExtractORB on both images (frame.cc:179-182), then ComputeStereoMatches
(:189) over mvKeys / mvKeysRight, their descriptors and the two extractors'
pyramids.  Here the two OrbExtractor handles keep those on the device after
their __call__, and the match runs where they lie (no pyramid download).
Batched frames: OrbExtractor.stereo_match_batch.
"""
from __future__ import annotations

import ctypes
from typing import Tuple

import numpy as np

from ._lib import check, lib, ptr
from .extractor import OrbExtractor


def compute_stereo_matches(left: OrbExtractor, right: OrbExtractor, n_left: int, bf: float,
                           mb: float) -> Tuple[np.ndarray, np.ndarray]:
    """-> (mvuRight, mvDepth), float32 [n_left], -1 where unmatched.  `left` /
    `right` must have just extracted the frame's left / right image (n_left =
    len(mvKeys)); bf = Frame::bf_, mb = Frame::mb."""
    ur = np.zeros(max(n_left, 1), np.float32)
    dep = np.zeros(max(n_left, 1), np.float32)
    check(lib().orbgpu_stereo_match(left._h, right._h, float(bf), float(mb), ptr(ur), ptr(dep),
                                    n_left), "orbgpu_stereo_match")
    return ur[:n_left].copy(), dep[:n_left].copy()


__all__ = ["compute_stereo_matches"]
