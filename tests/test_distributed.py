"""Multi-process sharding on CPU (gloo, world_size 2): every image is decoded
exactly once across ranks, and the timing reduction is a MAX."""

import os
import socket

import pytest
import torch.multiprocessing as mp

from spdl_amd.distributed import contiguous_shard, shard


def test_shard_partition():
    items = list(range(2048))
    for world in (1, 2, 3, 8):
        parts = [shard(items, r, world) for r in range(world)]
        assert sorted(sum(parts, [])) == items
        assert max(map(len, parts)) - min(map(len, parts)) <= 1
        blocks = [list(contiguous_shard(len(items), r, world)) for r in range(world)]
        assert sum(blocks, []) == items
    assert [len(contiguous_shard(2048, r, 8)) for r in range(8)] == [256] * 8
    with pytest.raises(ValueError):
        shard(items, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    from spdl_amd.distributed import reduce_max, reduce_sum, shard

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mine = shard(list(range(100)), rank, world)
    total = reduce_sum(len(mine))
    t = reduce_max(1.0 + rank)
    gathered = [None] * world
    dist.all_gather_object(gathered, mine)
    dist.destroy_process_group()
    q.put((rank, total, t, gathered))


def test_two_rank_gloo_sharding():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, total, t, gathered in res:
        assert total == 100
        assert t == 2.0
        flat = sorted(sum(gathered, []))
        assert flat == list(range(100))
