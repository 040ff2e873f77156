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

import os
import socket
import subprocess
import sys
import time
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


def launched_world() -> tuple[int, int, int]:
    """(rank, world_size, local_rank) set by a launcher (torch.distributed.run
    or :func:`spawn_ranks`); (0, 1, 0) for a plain single process."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def spawn_ranks(nprocs: int, argv: Sequence[str], master_port: int | None = None) -> int:
    """Run ``nprocs`` copies of ``python argv...`` as ranks 0..nprocs-1 of one
    job on this node and return the worst exit code.

    This is the one-process-per-GPU launch of the reference's
    examples/image_dataloading.py:291-317 (a ``multiprocessing.Pool`` of
    ``num_workers`` workers, worker i on device i): RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_ADDR / MASTER_PORT are exported to each child, the
    parent never touches a GPU (it only waits), and a failing rank makes
    the whole job fail.  Children are started as separate programs (never
    exec'd in place of this process)."""
    if nprocs < 1:
        raise ValueError(f"invalid number of ranks {nprocs}")
    port = master_port or _free_port()
    procs = []
    for r in range(nprocs):
        env = dict(os.environ)
        env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nprocs),
                   LOCAL_WORLD_SIZE=str(nprocs), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, *argv], env=env))
    rc = 0
    try:
        # poll every rank: the first one to fail ends the job, so a rank
        # still blocked in a rendezvous or barrier with it does not hang
        live = list(procs)
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0:
                    rc = rc or code
            if rc:
                break
            if live:
                time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def init_host_group() -> tuple[int, int, int]:
    """Join the launched job's CPU process group (gloo) when WORLD_SIZE > 1.
    The bench's only cross-rank traffic -- a barrier and a MAX of elapsed
    seconds -- needs no device collective, so none is created."""
    rank, world, local = launched_world()
    if world > 1:
        import torch.distributed as dist

        if not dist.is_initialized():
            dist.init_process_group("gloo", rank=rank, world_size=world)
    return rank, world, local


def barrier() -> None:
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        dist.barrier()


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
