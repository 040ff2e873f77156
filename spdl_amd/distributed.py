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


# ---- host-core binding per rank (configs[4]: the copy pool of each rank on
# its GPU's NUMA node) -------------------------------------------------------
# The reference binds its benchmark processes externally (`numactl --membind 0
# --cpubind 0`, examples/benchmark_tarfile.py:28); here each rank binds
# itself after choosing its device, within what the process may use.


def _cpulist(text: str) -> set[int]:
    """Parse a kernel cpulist ("0-3,8,10-11")."""
    out: set[int] = set()
    for part in text.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            out.update(range(int(a), int(b) + 1))
        else:
            out.add(int(part))
    return out


def device_numa(device_index: int) -> tuple[int, set[int]]:
    """(NUMA node, local CPUs) of a GPU from its PCI address (sysfs); (-1,
    empty) when unknown."""
    import torch

    p = torch.cuda.get_device_properties(device_index)
    bdf = (f"{getattr(p, 'pci_domain_id', 0):04x}:{getattr(p, 'pci_bus_id', 0):02x}:"
           f"{getattr(p, 'pci_device_id', 0):02x}.0")
    base = f"/sys/bus/pci/devices/{bdf}"
    try:
        with open(f"{base}/numa_node") as f:
            node = int(f.read().strip())
        with open(f"{base}/local_cpulist") as f:
            cpus = _cpulist(f.read())
    except (OSError, ValueError):
        return -1, set()
    return node, cpus


def cpu_quota() -> int | None:
    """Whole cores of the cgroup v2 CPU quota, or None when unlimited."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        return None


def rank_cores(usable: set[int], nodes: Sequence[int], node_cpus: dict[int, set[int]],
               local_rank: int, quota: int | None = None) -> list[int]:
    """The cores of local rank `local_rank` among `len(nodes)` ranks of this
    node, rank k's GPU on NUMA node nodes[k]: the ranks sharing a NUMA node
    split the usable cores of that node (all usable cores when the node has
    none of them) into equal disjoint runs; a CPU quota caps each rank at
    quota / ranks cores."""
    nranks = len(nodes)
    mine = nodes[local_rank]
    peers = [k for k in range(nranks) if nodes[k] == mine]
    j = peers.index(local_rank)
    cand = sorted(usable & node_cpus.get(mine, set())) or sorted(usable)
    per = max(1, len(cand) // len(peers))
    if quota is not None:
        per = max(1, min(per, quota // nranks))
    lo = (j * per) % max(1, len(cand))
    return [cand[(lo + i) % len(cand)] for i in range(min(per, len(cand)))]


def bind_rank_cpus(device_index: int, devices: Sequence[int], local_rank: int,
                   policy: str = "node") -> dict:
    """Pin every thread of this process to host cores near its GPU.
    `devices[k]`: the device of local rank k.  policy "node": every usable
    core of the GPU's NUMA node (shared by the ranks on that node); "split":
    the rank's own disjoint share of them (rank_cores), the decoder's copy
    pool sized to it.  Returns the record for the rank's JSON."""
    usable = set(os.sched_getaffinity(0))
    cache: dict[int, tuple[int, set[int]]] = {}
    for d in set(devices):
        cache[d] = device_numa(d)
    nodes = [cache[d][0] for d in devices]
    node_cpus = {cache[d][0]: cache[d][1] for d in cache}
    if policy == "split":
        cores = rank_cores(usable, nodes, node_cpus, local_rank, cpu_quota())
    else:
        cores = sorted(usable & node_cpus.get(nodes[local_rank], set())) or sorted(usable)
    for tid in os.listdir("/proc/self/task"):
        try:
            os.sched_setaffinity(int(tid), cores)
        except OSError:
            pass
    if policy == "split":  # the copy pool (created on first use): a thread per core
        os.environ["SPDL_HJ_COPY_THREADS"] = str(len(cores))
    return {"numa_node": cache[device_index][0], "bind": policy,
            "cpus": cores if len(cores) <= 32 else f"{len(cores)} cores {cores[0]}-{cores[-1]}"}
