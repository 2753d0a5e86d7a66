"""CPU tests of the DBoW2 oracle (bow_oracle.cc): text loader quirks and
transform(features, BowVector, FeatureVector, levelsup) against an
independent Python restatement, for every weighting / scoring family."""
import numpy as np
import pytest

import binding as orc
from orb_slam_fusion_amd import synth
from ref_py import bow_transform_py, load_vocab_py


def _descs(seed, n):
    return np.random.default_rng(seed).integers(0, 256, (n, 32), dtype=np.uint8)


@pytest.mark.parametrize("scoring,weighting,levelsup,trail", [
    (0, 0, 1, True),    # ORB-SLAM: L1_NORM, TF_IDF (trailing bogus node included)
    (0, 0, 4, False),   # levelsup beyond L: FeatureVector on the root
    (1, 1, 2, False),   # L2_NORM, TF
    (5, 0, 1, False),   # DOT_PRODUCT: no normalisation, TF divides by #words
    (2, 2, 1, False),   # CHI_SQUARE (L1), IDF: first weight kept
    (3, 3, 2, True),    # KL (L1), BINARY
])
def test_transform_matches_python(tmp_path, scoring, weighting, levelsup, trail):
    path = tmp_path / "voc.txt"
    synth.vocab_text(path, seed=5 + scoring, k=6, L=3, scoring=scoring, weighting=weighting,
                     stop_pct=5, trailing_newline=trail)
    V = orc.OracleVocab(path)
    P = load_vocab_py(path)
    info = V.info()
    assert info["nodes"] == len(P["nodes"]) and info["words"] == P["words"]
    assert info["nodes"] == 1 + 6 + 36 + 216 + (1 if trail else 0)
    d = _descs(scoring, 300)
    d[50:60] = d[40:50]  # repeated features: repeated words, TF sums
    bw, bwt, fn, fo, ff = V.transform(d, levelsup)
    bow, fv = bow_transform_py(P, d, levelsup)
    assert bw.tolist() == list(bow.keys())
    if scoring == 1:
        np.testing.assert_allclose(bwt, list(bow.values()), rtol=1e-15)
    else:
        assert bwt.tolist() == list(bow.values())
    assert fn.tolist() == list(fv.keys())
    assert [ff[fo[j]:fo[j + 1]].tolist() for j in range(len(fn))] == list(fv.values())
    if scoring in (0, 2, 3):
        assert abs(bwt.sum() - 1.0) < 1e-12


def test_loader_rejects_bad_header(tmp_path):
    p = tmp_path / "bad.txt"
    p.write_text("25 3 0 0\n")
    with pytest.raises(ValueError):
        orc.OracleVocab(p)
    p.write_text("10 3 6 0\n")
    with pytest.raises(ValueError):
        orc.OracleVocab(p)


def test_empty_inputs(tmp_path):
    path = tmp_path / "voc.txt"
    synth.vocab_text(path, k=4, L=2, trailing_newline=False)
    V = orc.OracleVocab(path)
    bw, bwt, fn, fo, ff = V.transform(np.zeros((0, 32), np.uint8))
    assert len(bw) == 0 and len(fn) == 0 and fo.tolist() == [0]
