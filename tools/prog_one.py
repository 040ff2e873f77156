"""A few synchronous batches of progressive 480x640 q90 JPEGs through the
pad224 chain (for rocprofv3 counter passes over multiscan_kernel).
python tools/prog_one.py [batch] [reps]"""
import sys

import torch

sys.path.insert(0, ".")
from spdl_amd import _lib  # noqa: E402
from spdl_amd._lib import Output  # noqa: E402
from spdl_amd.synthetic import synthetic_jpeg  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
spec = Output(pix_fmt="rgb24", resize=True, fit_w=224, fit_h=224, aspect="decrease", pad_w=224,
              pad_h=224)
dec = _lib.Decoder(0)
out = torch.empty((n, 224, 224, 3), dtype=torch.uint8, device="cuda:0")
datas = [synthetic_jpeg(2000 + i % 8, progressive=True) for i in range(n)]
for _ in range(reps):
    dec.decode_batch(datas, spec, out.data_ptr(), out.numel())
torch.cuda.synchronize()
dec.close()
print("done", flush=True)
