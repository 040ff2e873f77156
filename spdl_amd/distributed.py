"""Multi-GPU sharding for the decode stage.

Images are independent, so N GPUs decode N disjoint slices of the input with
no collective on the data path: one process per GPU (torch.distributed
launch), each rank takes every world_size-th item like the reference's
examples/image_dataloading.py:108-112 (``i % num_workers == worker_id``) and
DistributedDeterministicSampler (src/spdl/source/_sampler.py:62-130).
The only cross-rank traffic is timing/bookkeeping: a barrier and a MAX
all-reduce of elapsed time (bench.py), or a SUM of counts.
"""

from __future__ import annotations

from collections.abc import Sequence
from typing import TypeVar

T = TypeVar("T")


def shard(items: Sequence[T], rank: int, world_size: int) -> list[T]:
    """Round-robin slice of `items` for `rank` (stable, disjoint, covering)."""
    if world_size <= 0 or not 0 <= rank < world_size:
        raise ValueError(f"invalid rank {rank} for world_size {world_size}")
    return [items[i] for i in range(rank, len(items), world_size)]


def contiguous_shard(n: int, rank: int, world_size: int) -> range:
    """Contiguous block partition of range(n) (BASELINE config 3: 2048 -> 8 x 256)."""
    if world_size <= 0 or not 0 <= rank < world_size:
        raise ValueError(f"invalid rank {rank} for world_size {world_size}")
    per, extra = divmod(n, world_size)
    start = rank * per + min(rank, extra)
    return range(start, start + per + (1 if rank < extra else 0))


def reduce_max(value: float, device=None) -> float:
    """MAX over ranks (timing); identity when torch.distributed is not initialised."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def reduce_sum(value: float, device=None) -> float:
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())
