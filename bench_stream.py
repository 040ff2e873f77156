"""End-to-end tar stream benchmark (BASELINE.json configs[4]).

Workload: a tar archive of synthetic 480x640 q90 4:2:0 JPEGs (the
``examples/benchmark_tarfile.py`` shape: ``tarfile``-written ustar members)
per rank, in the page cache.  Each pass streams the whole archive through
``spdl_amd.io.TarImageStream``:

  pread (7+1 host threads) -> pinned ring slot -> ONE hipMemcpyAsync per batch
  on the decoder's copy stream -> decode kernels (RGB 224x224 u8, pad mode)

with batch k+1's read and copy overlapping batch k's kernels.  ``--d2h`` also
copies every output batch back into pinned host memory on a separate stream
(the "RGB tensors to the trainer out" direction), overlapped the same way.

The timed region starts with the archive on disk (page cache) and ends with
every output complete (device tensor, or host tensor with --d2h).  One process
per GPU; images are independent, no collective; value = all ranks' images /
max-over-ranks time.

Usage: python bench_stream.py [--gpus N] [--images 2048] [--batch 256]
       [--passes 3] [--d2h] [--source file|bytes]
"""

from __future__ import annotations

import argparse
import io
import json
import os
import shutil
import sys
import tarfile
import tempfile
import time

import spdl_amd  # noqa: F401  (sets the HW queue count before HIP initialises)
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import spdl_amd.io as sio  # noqa: E402
from spdl_amd.distributed import (  # noqa: E402
    bind_rank_cpus,
    barrier,
    init_host_group,
    launched_world,
    reduce_max,
    spawn_ranks,
)
from spdl_amd.synthetic import synthetic_batch  # noqa: E402


def _args():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--images", type=int, default=2048)
    p.add_argument("--batch", type=int, default=256)
    p.add_argument("--passes", type=int, default=3)
    p.add_argument("--warmup-passes", type=int, default=1)
    p.add_argument("--distinct", type=int, default=32)
    p.add_argument("--d2h", action="store_true")
    p.add_argument("--source", choices=["file", "bytes"], default="file")
    p.add_argument("--rehearse-one-gpu", action="store_true",
                   help="run every rank on device 0 (launch-path rehearsal, not a multi-GPU rate)")
    p.add_argument("--bind", choices=["node", "split", "none"], default="node",
                   help="N > 1: each rank's threads on the cores of its GPU's NUMA node (node), on "
                        "its own disjoint share of them (split), or left alone (none)")
    p.add_argument("--depth", type=int, default=4,
                   help="batches in flight (= decode pipeline lanes), 1-8")
    p.add_argument("--param", action="append", default=[], metavar="NAME=VALUE",
                   help="extra decoder parameter (spdl_hj_set_param), for A/B runs")
    p.add_argument("--sample-out", default="",
                   help="write the first batch of the last timed pass (member names + "
                        "--sample-images decoded images) to <sample-out>.r<rank>.npz")
    p.add_argument("--sample-images", type=int, default=16)
    return p.parse_args()


def _make_tar(path: str, n: int, distinct: int, rank: int) -> int:
    datas = synthetic_batch(n, distinct=distinct)
    with tarfile.open(path, "w") as t:
        for i, d in enumerate(datas):
            ti = tarfile.TarInfo(f"r{rank}/{i:07d}.jpg")
            ti.size = len(d)
            t.addfile(ti, io.BytesIO(d))
    return sum(len(d) for d in datas)


def main():
    a = _args()
    rank, world, local = launched_world()
    if a.gpus > 1 and world == 1:
        # one process per GPU, started before anything touches a device
        raise SystemExit(spawn_ranks(a.gpus, [os.path.abspath(__file__), *sys.argv[1:]]))
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    init_host_group()  # gloo: barrier + MAX of elapsed seconds only
    lrank = local
    if a.rehearse_one_gpu:
        local = 0
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    bind = None
    if world > 1 and a.bind != "none":
        lw = int(os.environ.get("LOCAL_WORLD_SIZE", world))
        devices = [0] * lw if a.rehearse_one_gpu else list(range(lw))
        bind = bind_rank_cpus(device.index, devices, lrank, a.bind)

    tmp = tempfile.mkdtemp(prefix=f"spdl_tar_r{rank}_")
    try:
        path = os.path.join(tmp, "shard.tar")
        payload = _make_tar(path, a.images, a.distinct, rank)
        tar_bytes = os.path.getsize(path)
        with open(path, "rb") as f:  # page-cache warm (the archive is "on local disk")
            data = f.read()
        src = data if a.source == "bytes" else path
        cfg = sio.cuda_config(device_index=local, stream=torch.cuda.current_stream(device).cuda_stream)
        st = sio.TarImageStream(src, batch_size=a.batch, device_config=cfg, depth=a.depth)
        for kv in a.param:
            k, v = kv.split("=", 1)
            st._dec.set_param(k, int(v))
        d2h = torch.cuda.Stream(device) if a.d2h else None
        host = [torch.empty((a.batch, 224, 224, 3), dtype=torch.uint8).pin_memory()
                for _ in range(2)] if a.d2h else None
        d2h_ev = [None, None]
        sample = {}

        def one_pass():
            n, k = 0, 0
            for names, t in st:
                if k == 0 and a.sample_out:  # outside the byte path: a view + names only
                    sample["names"], sample["t"] = list(names), t
                if d2h is not None:
                    j = k & 1
                    if d2h_ev[j] is not None:
                        d2h_ev[j].synchronize()  # host buffer j is free again
                    # t is complete (the stream waited for its ticket); only
                    # the allocator must not recycle it before the copy ends
                    with torch.cuda.stream(d2h):
                        host[j][: t.shape[0]].copy_(t, non_blocking=True)
                        t.record_stream(d2h)
                        d2h_ev[j] = torch.cuda.Event()
                        d2h_ev[j].record(d2h)
                n += t.shape[0]
                k += 1
            if d2h is not None:
                d2h.synchronize()
            return n

        for _ in range(a.warmup_passes):
            one_pass()
        torch.cuda.synchronize(device)
        barrier()
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        total = 0
        for _ in range(a.passes):
            total += one_pass()
        torch.cuda.synchronize(device)
        barrier()
        torch.cuda.synchronize(device)
        own = time.perf_counter() - t0
        elapsed = reduce_max(own)
        st.close()
        mine = {"rank": rank, "device": device.index, "images": total,
                "pci_bus_id": getattr(torch.cuda.get_device_properties(device), "pci_bus_id", None),
                "images_per_sec": round(total / own, 1),
                **(bind or {})}
        if a.sample_out and sample:
            import numpy as np

            m = min(a.sample_images, sample["t"].shape[0])
            np.savez(f"{a.sample_out}.r{rank}.npz", names=np.array(sample["names"][:m]),
                     rgb=sample["t"][:m].cpu().numpy())
        if world > 1:
            import torch.distributed as dist

            ranks = [None] * world
            dist.all_gather_object(ranks, mine)
        else:
            ranks = [mine]
        if rank == 0:
            value = world * total / elapsed
            print(json.dumps({
                "metric": "images/sec end-to-end tar (page cache) -> RGB224 on device"
                          + (" -> pinned host" if a.d2h else ""),
                "value": round(value, 1),
                "unit": "images/sec",
                "n_gpus": world,
                "passes": a.passes,
                "ms_per_batch": round(elapsed / (total / a.batch) * 1000.0, 4),
                "higher_is_better": True,
                "scaling": "weak",
                "dtype": "u8",
                "data": "synthetic",
                "config": {
                    "workload": "configs[4]: tar-packed 480x640 q90 4:2:0 JPEGs, pinned ring, "
                                "overlapped H2D + decode -> RGB 224x224 u8 (pad)",
                    "images_per_rank": a.images,
                    "batch": a.batch,
                    "source": a.source,
                    "tar_bytes_per_rank": tar_bytes,
                    "jpeg_payload_bytes_per_rank": payload,
                    "d2h": bool(a.d2h),
                    "depth": a.depth,
                    **({"rehearsal": f"{world} ranks sharing ONE GPU"} if a.rehearse_one_gpu
                       else {}),
                    "parallelism": f"{world} independent per-GPU archives, no collective",
                },
                "h2d_GBps_per_gpu": round(tar_bytes * a.passes / elapsed / 1e9, 3),
                "ranks": ranks,
            }), flush=True)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
        if world > 1:
            import torch.distributed as dist

            dist.destroy_process_group()


if __name__ == "__main__":
    main()
