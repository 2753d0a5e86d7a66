"""GPU parity of DBoW2 transform (bow_kernels.hip through the C ABI) against
the CPU oracle (bow_oracle.cc): BowVector words and weights, FeatureVector
nodes and feature lists bit-exact."""
import numpy as np
import pytest

import binding as orc
from orb_slam_fusion_amd import synth

pytestmark = pytest.mark.gpu


def _same(a, b):
    for x, y in zip(a, b):
        assert np.asarray(x).tobytes() == np.asarray(y).tobytes()


@pytest.mark.parametrize("k,L,scoring,weighting,levelsup,trail,n", [
    (10, 4, 0, 0, 4, True, 1000),   # ORB-SLAM setting (levelsup 4 -> FeatureVector on the root)
    (10, 4, 0, 0, 2, True, 1000),
    (8, 3, 1, 1, 1, False, 700),
    (5, 4, 5, 0, 2, False, 500),
    (6, 3, 2, 2, 1, False, 600),
    (6, 3, 3, 3, 2, True, 600),
    (20, 2, 0, 0, 1, False, 4096),  # 20 children (two 16-lane passes)
    (10, 3, 0, 0, 2, False, 6000),  # a 5 x nFeatures frame (tracking.cc:202-204): past 4096 features
    (10, 3, 1, 0, 1, False, 8192),  # capacity (kBowMaxFeatures)
    (3, 2, 0, 0, 1, False, 0),
])
def test_transform_parity(gpu_available, tmp_path, k, L, scoring, weighting, levelsup, trail, n):
    from orb_slam_fusion_amd.vocab import ORBVocabulary

    path = tmp_path / "voc.txt"
    synth.vocab_text(path, seed=k + L, k=k, L=L, scoring=scoring, weighting=weighting,
                     stop_pct=4, trailing_newline=trail)
    V = ORBVocabulary()
    assert V.loadFromTextFile(path)
    O = orc.OracleVocab(path)
    assert V.info() == O.info()
    d = np.random.default_rng(n).integers(0, 256, (n, 32), dtype=np.uint8)
    if n > 40:
        d[20:40] = d[0:20]
    _same(V.transform_arrays(d, levelsup), O.transform(d, levelsup))
    V.close()


def test_extractor_descriptors_and_batch(gpu_available, tmp_path):
    import torch

    from orb_slam_fusion_amd.vocab import ORBVocabulary

    path = tmp_path / "voc.txt"
    synth.vocab_text(path, k=10, L=5)
    V = ORBVocabulary()
    assert V.loadFromTextFile(path)
    O = orc.OracleVocab(path)
    ex = orc.OracleExtractor(1000, 1.2, 8, 20, 7)
    frames = [ex.extract(synth.stereo_frame(i)[0])[2] for i in range(4)]
    S = max(len(f) for f in frames)
    B = len(frames)
    descs = np.zeros((B, S, 32), np.uint8)
    for b, f in enumerate(frames):
        descs[b, :len(f)] = f
    dev = torch.device("cuda", 0)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    d_n = T(np.array([len(f) for f in frames], np.int32))
    bw = torch.zeros((B, S), dtype=torch.int32, device=dev)
    bwt = torch.zeros((B, S), dtype=torch.float64, device=dev)
    fn = torch.zeros((B, S), dtype=torch.int32, device=dev)
    fo = torch.zeros((B, S + 1), dtype=torch.int32, device=dev)
    ff = torch.zeros((B, S), dtype=torch.int32, device=dev)
    nw = torch.zeros(B, dtype=torch.int32, device=dev)
    nn = torch.zeros(B, dtype=torch.int32, device=dev)
    V.transform_batch(T(descs), d_n, 4, bw, bwt, nw, fn, fo, ff, nn)
    torch.cuda.synchronize()
    bw, bwt, fn, fo, ff = (x.cpu().numpy() for x in (bw, bwt, fn, fo, ff))
    nw, nn = nw.cpu().numpy(), nn.cpu().numpy()
    for b, f in enumerate(frames):
        ow, owt, onn, ofo, off = O.transform(f, 4)
        assert nw[b] == len(ow) and nn[b] == len(onn)
        assert bw[b, :nw[b]].astype(np.uint32).tobytes() == ow.tobytes()
        assert bwt[b, :nw[b]].tobytes() == owt.tobytes()
        assert fn[b, :nn[b]].astype(np.uint32).tobytes() == onn.tobytes()
        assert fo[b, :nn[b] + 1].tobytes() == ofo.tobytes()
        assert ff[b, :fo[b, nn[b]]].astype(np.uint32).tobytes() == off.tobytes()
        # the host path agrees too
        _same(V.transform_arrays(f, 4), (ow, owt, onn, ofo, off))
    V.close()
