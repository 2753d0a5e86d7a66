"""World-size-2 and -4 gloo test of the point-sharded LocalBundleAdjustment layout
(SURVEY §8e): each rank runs the oracle on its half of the points, the
partial reduced camera system / chi2 / LM scale are completed by the
product's all-reduce hook (orb_slam_fusion_amd.lba.dist_reduce, gloo on host
arrays here, RCCL on device buffers on the GPU), and the result equals the
single-process solve."""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest
import torch.multiprocessing as mp

REPO = Path(__file__).resolve().parents[1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _problem():
    from orb_slam_fusion_amd import synth

    return synth.lba_problem(seed=21, n_kf=8, n_pts=300, obs_per_pt=4, n_fixed=2, outlier_pct=5)


def _worker(rank, world, port, out_dir):
    sys.path.insert(0, str(REPO))
    sys.path.insert(0, str(REPO / "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import binding as oracle
    from orb_slam_fusion_amd import dist
    from orb_slam_fusion_amd.lba import dist_reduce

    dist.init(world, rank)
    p = _problem()
    n = len(p.pts_init)
    cut = [0] + [k * n // world + 7 for k in range(1, world)] + [n]  # uneven shards on purpose
    r = oracle.lba(p, pt_range=(cut[rank], cut[rank + 1]), reduce=dist_reduce())
    np.savez(Path(out_dir) / f"r{rank}.npz", poses=r["poses"], pts=r["pts"], outlier=r["outlier"],
             stats=r["stats"], cut=np.array(cut))
    dist.finalize()


@pytest.mark.parametrize("world", [2, 4])
def test_gloo_lba_shards(tmp_path, world):
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    r = [np.load(tmp_path / f"r{k}.npz") for k in range(world)]
    sys.path.insert(0, str(REPO / "oracle"))
    sys.path.insert(0, str(REPO))
    import binding as oracle

    p = _problem()
    single = oracle.lba(p)
    cut = r[0]["cut"]
    for k in range(world):
        assert (r[k]["poses"] == r[0]["poses"]).all()  # every rank solves the same system
        assert r[k]["stats"][1] == r[0]["stats"][1]  # global chi2
    assert np.allclose(r[0]["poses"], single["poses"], rtol=1e-9, atol=1e-12)
    pts = np.concatenate([r[k]["pts"][cut[k]:cut[k + 1]] for k in range(world)])
    assert np.allclose(pts, single["pts"], rtol=1e-9, atol=1e-12)
    owner = np.searchsorted(cut[1:], p.edges["point"], side="right")
    outl = np.choose(owner, [r[k]["outlier"] for k in range(world)])
    assert (outl == single["outlier"]).all()
    assert abs(r[0]["stats"][1] - single["stats"][1]) <= 1e-9 * single["stats"][1]
