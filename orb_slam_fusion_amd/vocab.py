"""Host mirror of DBoW2's ORBVocabulary (TemplatedVocabulary<FORB::TDescriptor,
FORB>) over the gfx950 C ABI: ``loadFromTextFile`` (TemplatedVocabulary.h:
1248-1327) and ``transform(features, BowVector&, FeatureVector&, levelsup)``
(:1057-1179), the call of Frame::ComputeBoW / KeyFrame::ComputeBoW
(frame.cc:761-766, keyframe.cc:202-208, levelsup = 4).

BowVector comes back as a dict {word id: weight} in ascending word order,
FeatureVector as a dict {node id: [feature indices]} in ascending node order
(the reference's std::maps)."""
from __future__ import annotations

import ctypes
from typing import Dict, List, Tuple

import numpy as np

from ._lib import check, lib, ptr
from .extractor import launch_stream

SCORING = ("L1_NORM", "L2_NORM", "CHI_SQUARE", "KL", "BHATTACHARYYA", "DOT_PRODUCT")
WEIGHTING = ("TF_IDF", "TF", "IDF", "BINARY")


class ORBVocabulary:
    def __init__(self, device: int = 0):
        self.device = device
        self._h = ctypes.c_void_p()

    def loadFromTextFile(self, path) -> bool:
        self.close()
        st = lib().orbgpu_vocab_load_text(self.device, str(path).encode(), ctypes.byref(self._h))
        if st != 0:
            self._h = ctypes.c_void_p()
            return False
        return True

    def info(self) -> dict:
        a = np.zeros(6, np.int32)
        check(lib().orbgpu_vocab_info(self._h, ptr(a)), "orbgpu_vocab_info")
        return dict(zip(("k", "L", "scoring", "weighting", "nodes", "words"), a.tolist()))

    def empty(self) -> bool:
        return not self._h or self.info()["words"] == 0

    def transform_arrays(self, descs: np.ndarray, levelsup: int = 4):
        """-> (bow_words, bow_weights, fv_nodes, fv_offsets, fv_features) arrays."""
        d = np.ascontiguousarray(descs, np.uint8).reshape(-1, 32)
        n = len(d)
        S = max(n, 1)
        bw, bwt = np.zeros(S, np.uint32), np.zeros(S, np.float64)
        fn, fo, ff = np.zeros(S, np.uint32), np.zeros(S + 1, np.int32), np.zeros(S, np.uint32)
        nw, nn = ctypes.c_int(), ctypes.c_int()
        check(lib().orbgpu_bow_transform(self._h, ptr(d), n, int(levelsup), ptr(bw), ptr(bwt),
                                         ctypes.byref(nw), ptr(fn), ptr(fo), ptr(ff),
                                         ctypes.byref(nn)), "orbgpu_bow_transform")
        w, k = nw.value, nn.value
        return bw[:w], bwt[:w], fn[:k], fo[:k + 1], ff[:fo[k]]

    def transform(self, descs: np.ndarray, levelsup: int = 4
                  ) -> Tuple[Dict[int, float], Dict[int, List[int]]]:
        bw, bwt, fn, fo, ff = self.transform_arrays(descs, levelsup)
        bow = {int(w): float(x) for w, x in zip(bw, bwt)}
        fv = {int(fn[j]): ff[fo[j]:fo[j + 1]].tolist() for j in range(len(fn))}
        return bow, fv

    def transform_batch(self, descs, n, levelsup, bow_words, bow_weights, n_words, fv_nodes,
                        fv_offsets, fv_features, n_nodes, stream=None) -> None:
        """Device tensors: descs uint8 [B, S, 32]; n int32 [B]; bow_words / fv_nodes /
        fv_features 4-byte [B, S]; bow_weights float64 [B, S]; fv_offsets int32
        [B, S + 1]; n_words / n_nodes int32 [B]."""
        B, S = descs.shape[0], descs.shape[1]
        with launch_stream(stream) as s:
            check(lib().orbgpu_bow_transform_batch(
                self._h, B, ptr(descs), ptr(n), S, int(levelsup), ptr(bow_words),
                ptr(bow_weights), ptr(n_words), ptr(fv_nodes), ptr(fv_offsets),
                ptr(fv_features), ptr(n_nodes), s), "orbgpu_bow_transform_batch")

    def close(self) -> None:
        if self._h:
            lib().orbgpu_vocab_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


__all__ = ["ORBVocabulary", "SCORING", "WEIGHTING"]
