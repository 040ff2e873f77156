import sys, time
sys.path.insert(0, ".")
import torch
from spdl_amd import _lib
from spdl_amd._lib import Output
from spdl_amd.synthetic import synthetic_batch
import bench
datas = synthetic_batch(256, distinct=32)
dev, offs, sizes, infos = bench._pack_device(datas, torch.device("cuda", 0))
dec = _lib.Decoder(0)
out = torch.empty((256, 224, 224, 3), dtype=torch.uint8, device="cuda:0")
for mask in [0, 1, 2, 4, 8, 15, 6]:
    dec.set_param("debug_mask", mask)
    dec.set_profiling(True)
    tot = 0
    for i in range(6):
        dec.decode_batch_device(dev.data_ptr(), dev.numel(), offs, sizes, infos, bench.OUT_SPEC, out.data_ptr(), out.numel(), sync=True)
        if i >= 1: tot += dec.last_timings()["output"]
    print("mask", mask, "resize ms", round(tot / 5 / 1000, 3))
