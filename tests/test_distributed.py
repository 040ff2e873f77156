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


def _last_json(out: str) -> dict:
    import json

    for line in reversed(out.strip().splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    raise AssertionError(f"no JSON line in output:\n{out}")


@pytest.mark.parametrize("launcher", ["self", "torchrun"])
def test_bench_launcher_spawns_ranks(launcher):
    """`python bench.py --gpus 2` starts two rank processes itself (the
    reference's examples/image_dataloading.py:291-317 one-worker-per-GPU
    launch), and under torch.distributed.run it joins the launched ranks;
    either way each rank gets a disjoint contiguous slice of the global
    batch (2048 -> 2 x 1024) and the reported time is the MAX over ranks
    (rank 1 sleeps twice as long as rank 0).  CPU-only (--dry-run, gloo)."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    args = ["bench.py", "--gpus", "2", "--dry-run", "--batch", "1024"]
    if launcher == "torchrun":
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node",
               "2", "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), *args]
    else:
        cmd = [sys.executable, *args]
    r = subprocess.run(cmd, cwd=root, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    rec = _last_json(r.stdout)
    assert rec["n_gpus"] == 2 and rec["global_batch"] == 2048
    assert rec["slices"] == [[0, 1024], [1024, 2048]]
    assert rec["elapsed"] >= 0.1  # rank 1's 2 x 50 ms, not rank 0's 50 ms


def test_bench_rejects_mismatched_world():
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "4", "--dry-run"], cwd=root,
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE" in (r.stderr + r.stdout)


def test_spawn_ranks_fails_fast_when_a_later_rank_dies(tmp_path):
    """A rank > 0 that dies (e.g. in init_process_group) ends the job at once:
    rank 0, blocked as if in a rendezvous, is killed instead of waited on."""
    import time

    from spdl_amd.distributed import spawn_ranks

    script = tmp_path / "r.py"
    script.write_text("import os, sys, time\n"
                      "r = int(os.environ['RANK'])\n"
                      "time.sleep(600) if r == 0 else sys.exit(3)\n")
    t0 = time.perf_counter()
    assert spawn_ranks(2, [str(script)]) == 3
    assert time.perf_counter() - t0 < 60


def test_rank_cores_split_a_numa_node():
    from spdl_amd.distributed import rank_cores

    usable = set(range(16))
    sets = [set(rank_cores(usable, [0] * 8, {0: set(range(32))}, r)) for r in range(8)]
    assert all(len(s) == 2 for s in sets)
    assert len(set().union(*sets)) == 16  # disjoint, covering


def test_rank_cores_follow_each_gpus_node_and_quota():
    from spdl_amd.distributed import rank_cores

    nodes = [0, 0, 0, 0, 1, 1, 1, 1]
    cpus = {0: set(range(32)), 1: set(range(32, 64))}
    sets = [rank_cores(set(range(64)), nodes, cpus, r, quota=16) for r in range(8)]
    for r, s in enumerate(sets):
        assert len(s) == 2 and all((c >= 32) == (nodes[r] == 1) for c in s), (r, s)
    assert len({c for s in sets for c in s}) == 16
    # a node with none of the usable cores: fall back to the usable set
    assert rank_cores({1, 2}, [1], cpus, 0) == [1, 2]


def test_cpulist_parse():
    from spdl_amd.distributed import _cpulist

    assert _cpulist("0-3,8,10-11\n") == {0, 1, 2, 3, 8, 10, 11}
