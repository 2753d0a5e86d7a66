"""One rank of a point-sharded LocalBundleAdjustment on cuda:0,
the shard sums completed by the product's reduce hook (lba.dist_reduce) over
a gloo group; started as a fresh interpreter before it touches the GPU by
tests/test_gpu_lba.py::test_lba_ranks_one_gpu and by bench_lba's
sharded side line.  CALLS > 0: also time that many calls (barrier first).

    python tools/lba_shard_worker.py RANK WORLD PORT OUT_DIR [CALLS] [ORDERED]

ORDERED = 1: the stream-ordered form (orbgpu_lba_ctx_set_reduce_ordered,
lba.dist_enqueue): the LM loop stays on the device and the reductions are
enqueued on the library's stream.
"""
import os
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))


def shard_cuts(n: int, world: int) -> list:
    """Point ranges of the ranks: [cut[r], cut[r + 1]), uneven on purpose
    (every inner boundary 13 points past the even split)."""
    return [0] + [k * n // world + 13 for k in range(1, world)] + [n]


def main() -> None:
    rank, world, port, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], Path(sys.argv[4])
    calls = int(sys.argv[5]) if len(sys.argv) > 5 else 0
    ordered = len(sys.argv) > 6 and sys.argv[6] == "1"
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
    import torch.distributed as dist

    from orb_slam_fusion_amd import LocalBundleAdjuster, synth

    dist.init_process_group("gloo", rank=rank, world_size=world)
    p = synth.lba_problem()  # C4: 20 KF, 3000 MP, 18000 edges
    n = len(p.pts_init)
    cut = shard_cuts(n, world)
    lba = LocalBundleAdjuster(0)
    r = lba.optimize(p, pt_range=(cut[rank], cut[rank + 1]), group=dist.group.WORLD, ordered=ordered)
    ms = 0.0
    if calls > 0:
        import time

        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(calls):
            lba.optimize(p, pt_range=(cut[rank], cut[rank + 1]), group=dist.group.WORLD, ordered=ordered)
        ms = (time.perf_counter() - t0) / calls * 1e3
    np.savez(out / f"r{rank}.npz", poses_d=r["poses_d"], pts=r["pts"], outlier=r["outlier"],
             stats=r["stats"], cut=np.array(cut), ms_per_call=np.array(ms))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
