"""Throughput of progressive vs baseline 480x640 q90 JPEGs through the
pad224 chain (decode_batch, host bytes), GPU.  python tools/prog_bench.py [batch]"""
import sys
import time

import torch

sys.path.insert(0, ".")
from spdl_amd import _lib  # noqa: E402
from spdl_amd._lib import Output  # noqa: E402
from spdl_amd.synthetic import synthetic_jpeg  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
spec = Output(pix_fmt="rgb24", resize=True, fit_w=224, fit_h=224, aspect="decrease", pad_w=224,
              pad_h=224)
dec = _lib.Decoder(0)
out = torch.empty((n, 224, 224, 3), dtype=torch.uint8, device="cuda:0")
for prog in (False, True, "one"):
    # "one": a baseline batch holding a single progressive image (the batch
    # completes with its slowest image)
    datas = [synthetic_jpeg(2000 + i % 32, progressive=(prog is True or (prog == "one" and i == 0)))
             for i in range(n)]
    for _ in range(2):
        dec.decode_batch(datas, spec, out.data_ptr(), out.numel())
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    reps = 3
    for _ in range(reps):
        dec.decode_batch(datas, spec, out.data_ptr(), out.numel())
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    print(f"progressive={prog} batch {n}: {dt * 1e3:.1f} ms/batch, {n / dt:.0f} img/s, "
          f"mean bytes {sum(map(len, datas)) / n:.0f}", flush=True)
dec.close()
