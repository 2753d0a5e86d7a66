"""World-size-2 gloo test of the point-sharded LocalBundleAdjustment layout
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
    cut = [0, n // 2 + 7, n]  # uneven shards on purpose
    r = oracle.lba(p, pt_range=(cut[rank], cut[rank + 1]), reduce=dist_reduce())
    np.savez(Path(out_dir) / f"r{rank}.npz", poses=r["poses"], pts=r["pts"], outlier=r["outlier"],
             stats=r["stats"], cut=np.array(cut))
    dist.finalize()


def test_gloo_world2_lba_shards(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    r = [np.load(tmp_path / f"r{k}.npz") for k in range(world)]
    sys.path.insert(0, str(REPO / "oracle"))
    sys.path.insert(0, str(REPO))
    import binding as oracle

    p = _problem()
    single = oracle.lba(p)
    cut = r[0]["cut"]
    assert (r[0]["poses"] == r[1]["poses"]).all()  # every rank solves the same system
    assert np.allclose(r[0]["poses"], single["poses"], rtol=1e-9, atol=1e-12)
    pts = np.concatenate([r[0]["pts"][cut[0]:cut[1]], r[1]["pts"][cut[1]:cut[2]]])
    assert np.allclose(pts, single["pts"], rtol=1e-9, atol=1e-12)
    owner = (p.edges["point"] >= cut[1]).astype(int)
    outl = np.where(owner == 0, r[0]["outlier"], r[1]["outlier"])
    assert (outl == single["outlier"]).all()
    assert r[0]["stats"][1] == r[1]["stats"][1]  # global chi2
    assert abs(r[0]["stats"][1] - single["stats"][1]) <= 1e-9 * single["stats"][1]
