"""GPU parity of the device-resident tracking chain (extract -> stereo ->
SearchByProjection(CurrentFrame, LastFrame) -> PoseOptimization observation
list -> PoseOptimization) against the CPU oracle running the same chain."""
import sys
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tools"))


def test_track_chain_matches_oracle(gpu_available):
    import torch

    import binding as oracle
    from bench_track import Chain, oracle_chain
    from orb_slam_fusion_amd._lib import KEYPOINT_DTYPE, POSE_OBS_DTYPE

    B = 3
    c = Chain(B)
    c.run()
    torch.cuda.synchronize()
    lk = c.lk.cpu().numpy().view(KEYPOINT_DTYPE).reshape(B, c.cap)
    ld, lnn, ur = c.ld.cpu().numpy(), c.lnn.cpu().numpy(), c.ur.cpu().numpy()
    match, nm = c.match.cpu().numpy(), c.nm.cpu().numpy()
    obs = c.obs.cpu().numpy().view(POSE_OBS_DTYPE).reshape(B, c.cap)
    nobs, idx = c.nobs.cpu().numpy(), c.obs_index.cpu().numpy()
    pose, outl, inl = c.pose_out.cpu().numpy(), c.outlier.cpu().numpy(), c.inliers.cpu().numpy()
    for f in range(B):
        o = oracle_chain(oracle, c, f)
        k = int(lnn[f])
        assert lk[f, :k].tobytes() == o["kps"].tobytes()
        assert ld[f, :k].tobytes() == o["desc"].tobytes()
        assert ur[f, :k].tobytes() == o["ur"].tobytes()
        assert int(nm[f]) == o["nm"] and o["nm"] > 100
        np.testing.assert_array_equal(match[f, :k], o["match"])
        n = int(nobs[f])
        assert n == len(o["obs"])
        assert obs[f, :n].tobytes() == o["obs"].tobytes()
        np.testing.assert_array_equal(idx[f, :n], np.nonzero(o["match"] >= 0)[0])
        assert int(inl[f]) == o["inliers"]
        np.testing.assert_array_equal(outl[f, :n], o["outlier"])
        assert np.max(np.abs(pose[f] - o["pose"])) <= 1e-5


def test_c5_sequence_runner_tracks(gpu_available):
    """tools/c5_runner.py's chain (one rank, two sequences batched): frame to
    frame tracking over a synthetic sequence stays on the known motion."""
    import c5_runner

    c = c5_runner.SequenceChain(0, 2, 12, 0)
    c.reset()
    for t in range(12):
        c.frame(t)
    nm, inl = c.stats()
    assert nm > 200 and inl > 200
    assert c.ate() < 0.01  # metres over 11 frames of 6 px (about 3 cm) each
