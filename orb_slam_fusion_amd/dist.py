"""Multi-GPU layout for the extractor + pose path.

Frames (and sequences) are independent units: one process per GPU, each rank
takes its own frames, and nothing on the data path is exchanged -- weak
scaling, no collective.  torch.distributed is used only to line the ranks up
for timing (barrier) and to take the job time as the max over ranks; the
coordination group is gloo (CPU) because there is no device data to move.
"""
from __future__ import annotations

import os
from typing import List


def rank_world() -> tuple:
    return int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)), int(
        os.environ.get("LOCAL_RANK", 0))


def frame_indices(rank: int, world: int, per_rank: int, step: int = 0) -> List[int]:
    """Global frame ids processed by `rank` in `step`: contiguous blocks, so the
    union over ranks is every frame exactly once."""
    base = (step * world + rank) * per_rank
    return list(range(base, base + per_rank))


def init(world: int, rank: int) -> None:
    if world > 1:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29517")
        if not dist.is_initialized():
            dist.init_process_group("gloo", rank=rank, world_size=world)


def barrier() -> None:
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        dist.barrier()


def job_time(elapsed: float) -> float:
    """Max of the per-rank timed regions (the job finishes with its slowest rank)."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return elapsed
    t = torch.tensor([elapsed], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def finalize() -> None:
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
