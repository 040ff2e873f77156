#!/usr/bin/env python3
"""configs[0]: load local JPEG files to GPUs with a thread pool per GPU
(the workload of the reference's examples/image_dataloading.py:115-317).

One process per GPU (``--num-workers``); each reads its split of the file
list (``line_number % num_workers == worker_id``), groups ``--batch-size``
paths, and decodes the batches on ``--num-threads`` threads, each calling
``spdl_amd.io.load_image_batch`` (224x224 rgb24, ``strict=False``) with its
own per-thread decoder; up to ``--buffer-size`` finished batches wait for
the consumer.  The reference builds the same stages with
spdl.pipeline.PipelineBuilder (source -> aggregate -> pipe(decode,
concurrency=num_threads) -> sink); that scheduler is outside this
project's scope, so a bounded thread pool stands in.

    python examples/image_dataloading.py --input-flist files.txt --prefix /data/ \\
        --num-workers 8
    python examples/image_dataloading.py --synthetic 1000   # writes 1k JPEGs first

Prints one JSON line: aggregated images/sec and batches/sec over workers.
"""

from __future__ import annotations

import argparse
import collections
import json
import os
import sys
import tempfile
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from dataclasses import asdict, dataclass

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


@dataclass
class PerfResult:
    elapsed: float
    num_batches: int
    num_frames: int


def _parse_args(argv=None):
    p = argparse.ArgumentParser(description=__doc__,
                                formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--input-flist", help="file with one image path per line")
    p.add_argument("--prefix", default="", help="prepended to every path of the list")
    p.add_argument("--synthetic", type=int, default=0,
                   help="write this many synthetic 480x640 q90 JPEGs and use them")
    p.add_argument("--batch-size", type=int, default=32)
    p.add_argument("--num-threads", type=int, default=4)
    p.add_argument("--buffer-size", type=int, default=16)
    p.add_argument("--num-workers", type=int, default=1)
    p.add_argument("--sample-out", default="",
                   help="write one decoded image of every batch (with its JPEG bytes) to "
                        "<sample-out>.w<worker>.npz, for checking pixels after the run")
    p.add_argument("--worker-id", type=int, default=-1, help=argparse.SUPPRESS)
    return p.parse_args(argv)


def source(path: str, prefix: str, split_size: int, split_id: int):
    """Paths at line_number % split_size == split_id (reference source())."""
    with open(path) as f:
        for i, line in enumerate(f):
            if i % split_size == split_id and (line := line.strip()):
                yield prefix + line


def batches(it, n):
    b = []
    for x in it:
        b.append(x)
        if len(b) == n:
            yield b
            b = []
    if b:
        yield b


def worker(args) -> PerfResult:
    import torch

    import spdl_amd.io as sio

    cfg = sio.cuda_config(device_index=args.worker_id)
    torch.zeros(1, device=f"cuda:{args.worker_id}")  # warm up the context

    samples, lock, nsamp = {}, threading.Lock(), [0]

    def decode(paths):
        buf = sio.load_image_batch(paths, width=224, height=224, pix_fmt="rgb24",
                                   device_config=cfg, strict=False)
        t = sio.to_torch(buf)
        if args.sample_out:  # one image per batch, a different position each time
            with lock:
                k = nsamp[0]
                nsamp[0] += 1
            j = k % t.shape[0]
            with open(paths[j], "rb") as f:
                jpeg = np.frombuffer(f.read(), np.uint8)
            rgb = t[j].cpu().numpy()
            with lock:
                samples[f"jpeg_{k}"], samples[f"rgb_{k}"] = jpeg, rgb
        return t

    src = batches(source(args.input_flist, args.prefix, args.num_workers, args.worker_id),
                  args.batch_size)
    t0 = time.monotonic()
    frames = nb = 0
    with ThreadPoolExecutor(args.num_threads) as pool:
        pending = collections.deque()
        for paths in src:
            pending.append(pool.submit(decode, paths))
            while len(pending) >= args.buffer_size + args.num_threads:
                t = pending.popleft().result()
                frames += t.shape[0]
                nb += 1
        while pending:
            t = pending.popleft().result()
            frames += t.shape[0]
            nb += 1
    torch.cuda.synchronize(args.worker_id)
    elapsed = time.monotonic() - t0
    if args.sample_out:
        np.savez(f"{args.sample_out}.w{args.worker_id}.npz", **samples)
    return PerfResult(elapsed, nb, frames)


def _write_synthetic(n: int, root: str) -> str:
    from spdl_amd.synthetic import synthetic_jpeg

    imgs = [synthetic_jpeg(3000 + i) for i in range(min(n, 64))]
    paths = []
    for i in range(n):
        p = os.path.join(root, f"{i:06d}.jpg")
        with open(p, "wb") as f:
            f.write(imgs[i % len(imgs)])
        paths.append(p)
    flist = os.path.join(root, "flist.txt")
    with open(flist, "w") as f:
        f.write("\n".join(paths) + "\n")
    return flist


def main(argv=None) -> None:
    args = _parse_args(argv)
    if args.worker_id >= 0:  # a spawned worker: run and report on stdout
        print(json.dumps(asdict(worker(args))), flush=True)
        return
    with tempfile.TemporaryDirectory() as tmp:
        if args.synthetic:
            args.input_flist, args.prefix = _write_synthetic(args.synthetic, tmp), ""
        if not args.input_flist:
            raise SystemExit("--input-flist or --synthetic is required")
        # one process per GPU, started before this process touches a GPU
        import subprocess

        base = [sys.executable, os.path.abspath(__file__), "--input-flist", args.input_flist,
                "--prefix", args.prefix, "--batch-size", str(args.batch_size),
                "--num-threads", str(args.num_threads), "--buffer-size", str(args.buffer_size),
                "--num-workers", str(args.num_workers), "--sample-out", args.sample_out]
        procs = [subprocess.Popen(base + ["--worker-id", str(i)], stdout=subprocess.PIPE,
                                  text=True) for i in range(args.num_workers)]
        vals = []
        for p in procs:
            out, _ = p.communicate()
            if p.returncode:
                raise SystemExit(f"worker failed with exit code {p.returncode}")
            vals.append(PerfResult(**json.loads(out.strip().splitlines()[-1])))
    ave = sum(v.elapsed for v in vals) / len(vals)
    frames = sum(v.num_frames for v in vals)
    nb = sum(v.num_batches for v in vals)
    print(json.dumps({"workload": "configs[0] local JPEG files, thread pool per GPU",
                      "num_workers": args.num_workers, "num_threads": args.num_threads,
                      "batch_size": args.batch_size, "frames": frames, "batches": nb,
                      "ave_elapsed_s": round(ave, 3), "images_per_sec": round(frames / ave, 1),
                      "batches_per_sec": round(nb / ave, 2)}))


if __name__ == "__main__":
    main()
