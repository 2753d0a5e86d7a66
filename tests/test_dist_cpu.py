"""World-size-2 gloo test of the multi-GPU layout on CPU: frames shard with no
overlap and no gap, the job time is the max over ranks, and each rank's
oracle results on its own shard match a single-process run (independent
units: no exchange on the data path)."""
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


def _worker(rank, world, port, out_dir):
    sys.path.insert(0, str(REPO))
    sys.path.insert(0, str(REPO / "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import binding as oracle
    from orb_slam_fusion_amd import dist, synth

    dist.init(world, rank)
    ids = dist.frame_indices(rank, world, per_rank=2)
    ex = oracle.OracleExtractor(500, 1.2, 4, 20, 7)
    counts = [len(ex.extract(synth.stereo_frame(i, w=320, h=256)[0])[1]) for i in ids]
    dist.barrier()
    t = dist.job_time(float(rank + 1))
    np.save(Path(out_dir) / f"r{rank}.npy", np.array(ids + counts + [t], np.float64))
    dist.finalize()


def test_gloo_world2_sharding(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    r = [np.load(tmp_path / f"r{k}.npy") for k in range(world)]
    ids = sorted(int(v) for k in range(world) for v in r[k][:2])
    assert ids == [0, 1, 2, 3]
    assert all(rr[-1] == 2.0 for rr in r)  # max over ranks

    sys.path.insert(0, str(REPO / "oracle"))
    import binding as oracle
    from orb_slam_fusion_amd import synth

    ex = oracle.OracleExtractor(500, 1.2, 4, 20, 7)
    for k in range(world):
        for j in range(2):
            fid = int(r[k][j])
            assert r[k][2 + j] == len(ex.extract(synth.stereo_frame(fid, w=320, h=256)[0])[1])
