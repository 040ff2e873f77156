"""Kernel trace material for the lone progressive image (verdict r05 item 2):
synchronous batches of (a) the progressive image alone, (b) 255 baseline +
that image, (c) 255 baseline only; run under rocprofv3 --kernel-trace and
compare multiscan_kernel durations.  Prints the wall time per batch.

  rocprofv3 --kernel-trace --stats -d gpurun_out/pt -- python tools/r6_prog_trace.py
"""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from spdl_amd import _lib  # noqa: E402
from spdl_amd._lib import Output  # noqa: E402
from spdl_amd.synthetic import synthetic_jpeg  # noqa: E402

spec = Output(pix_fmt="rgb24", resize=True, fit_w=224, fit_h=224, aspect="decrease", pad_w=224,
              pad_h=224)


def pack(datas):
    offs, sizes, pos = [], [], 0
    for d in datas:
        offs.append(pos)
        sizes.append(len(d))
        pos += (len(d) + 255) // 256 * 256
    host = np.zeros(pos + 256, np.uint8)
    for o, d in zip(offs, datas):
        host[o:o + len(d)] = np.frombuffer(d, np.uint8)
    dev = torch.from_numpy(host).to("cuda:0")
    infos = (_lib.ImageInfo * len(datas))(*[_lib.get_image_info(d) for d in datas])
    return dev, np.asarray(offs, np.int64), np.asarray(sizes, np.int64), infos


prog = synthetic_jpeg(2000, progressive=True)
base = [synthetic_jpeg(2000 + i % 32) for i in range(256)]
dec = _lib.Decoder(0)
dec.set_param("lanes", 4)
for name, datas in (("alone", [prog]), ("one_in_255", [prog] + base[1:]), ("baseline", base)):
    dev, offs, sizes, infos = pack(datas)
    out = torch.empty((len(datas), 224, 224, 3), dtype=torch.uint8, device="cuda:0")
    for _ in range(4):
        dec.decode_batch_device(dev.data_ptr(), dev.numel(), offs, sizes, infos, spec,
                                out.data_ptr(), out.numel(), stream=torch.cuda.current_stream(),
                                sync=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(6):
        dec.decode_batch_device(dev.data_ptr(), dev.numel(), offs, sizes, infos, spec,
                                out.data_ptr(), out.numel(), stream=torch.cuda.current_stream(),
                                sync=True)
    print(f"{name}: {(time.perf_counter() - t0) / 6 * 1e3:.2f} ms per synchronous batch", flush=True)
