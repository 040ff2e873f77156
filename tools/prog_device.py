"""Device-resident batches holding progressive images vs baseline batches
(pad224 chain, decode_batch_device as bench.py drives it), GPU.

  python tools/prog_device.py [batches]

For each mix -- all baseline, one progressive image per batch, every batch
progressive -- prints the time per batch of one synchronous batch and of a
pipelined stream (4 lanes, 6 batches in flight), and checks the last batch's
progressive image against the oracle.
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from oracle import oracle as O  # noqa: E402
from spdl_amd import _lib  # noqa: E402
from spdl_amd._lib import Output  # noqa: E402
from spdl_amd.synthetic import synthetic_jpeg  # noqa: E402

N = 256
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 60
PAD = dict(fit_w=224, fit_h=224, aspect="decrease", pad_w=224, pad_h=224)
spec = Output(pix_fmt="rgb24", resize=True, **PAD)


def pack(datas):
    offs, sizes, pos = [], [], 0
    for d in datas:
        offs.append(pos)
        sizes.append(len(d))
        pos += (len(d) + 255) // 256 * 256
    host = np.zeros(pos, np.uint8)
    for o, d in zip(offs, datas):
        host[o:o + len(d)] = np.frombuffer(d, np.uint8)
    dev = torch.from_numpy(host).to("cuda:0")
    infos = (_lib.ImageInfo * len(datas))(*[_lib.get_image_info(d) for d in datas])
    return dev, np.asarray(offs, np.int64), np.asarray(sizes, np.int64), infos


def run(datas, lanes, inflight, nsteps):
    dev, offs, sizes, infos = pack(datas)
    dec = _lib.Decoder(0)
    dec.set_param("lanes", lanes)
    outs = [torch.empty((N, 224, 224, 3), dtype=torch.uint8, device="cuda:0")
            for _ in range(inflight + 1)]
    stream = torch.cuda.current_stream()
    k = [0]

    def submit(sync):
        o = outs[k[0] % len(outs)]
        k[0] += 1
        dec.decode_batch_device(dev.data_ptr(), dev.numel(), offs, sizes, infos, spec,
                                o.data_ptr(), o.numel(), stream=stream, sync=sync)
        return dec.last_ticket()

    for _ in range(max(3, 2 * lanes)):  # (every lane's workspace warm)
        submit(True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        submit(True)
    sync_ms = (time.perf_counter() - t0) / 5 * 1e3
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pend = []
    for _ in range(nsteps):
        pend.append(submit(False))
        if len(pend) > inflight - 1:
            assert not any(dec.wait(pend.pop(0), N))
    for t in pend:
        assert not any(dec.wait(t, N))
    torch.cuda.synchronize()
    stream_ms = (time.perf_counter() - t0) / nsteps * 1e3
    last = outs[(k[0] - 1) % len(outs)].cpu().numpy()
    ref = O.decode_resize(datas[0], O.Resize(**PAD), "rgb24")
    np.testing.assert_array_equal(last[0], ref)
    dec.close()
    return sync_ms, stream_ms


LANES = int(os.environ.get("PD_LANES", "4"))  # (A/B: lanes, batches in flight)
INFLIGHT = int(os.environ.get("PD_INFLIGHT", "6"))
base = [synthetic_jpeg(2000 + i % 32) for i in range(N)]
prog1 = [synthetic_jpeg(2000, progressive=True)] + base[1:]
allp = [synthetic_jpeg(2000 + i % 32, progressive=True) for i in range(N)]
res = {}
for name, datas, n in (("baseline", base, steps), ("one_progressive", prog1, steps),
                       ("all_progressive", allp, max(6, steps // 10))):
    s1, sp = run(datas, LANES, INFLIGHT, n)
    res[name] = (s1, sp)
    print(f"{name:16s} sync batch {s1:7.2f} ms   stream ({LANES} lanes, {INFLIGHT} in flight) {sp:7.3f} ms/batch "
          f"= {N / sp * 1e3:9.0f} img/s", flush=True)
b = res["baseline"]
o = res["one_progressive"]
print(f"one progressive / baseline: sync {o[0] / b[0]:.2f}x, stream {o[1] / b[1]:.2f}x")
