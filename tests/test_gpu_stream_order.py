"""Stream order of a batch against the caller's stream (round 6, `lean_waits`).

A batch must run after everything the caller's stream had queued when the
batch was submitted -- here the device copy of the very JPEG bytes it
decodes, behind a long GEMM on that stream -- and the library skips the
cross-stream wait only when the caller's stream has nothing pending.  Every
lane, lean waits on and off, several batches in flight: every image
bit-exact vs the oracle, no status set.
"""

import numpy as np
import pytest
import torch

from spdl_amd import _lib
from spdl_amd._lib import Output
from tests import cases

pytestmark = pytest.mark.gpu

PAD = dict(fit_w=224, fit_h=224, aspect="decrease", pad_w=224, pad_h=224)


def _pack(datas):
    offs, sizes, pos = [], [], 0
    for d in datas:
        offs.append(pos)
        sizes.append(len(d))
        pos += (len(d) + 64 + 255) // 256 * 256
    host = np.zeros(pos, np.uint8)
    for o, d in zip(offs, datas):
        host[o:o + len(d)] = np.frombuffer(d, np.uint8)
    infos = (_lib.ImageInfo * len(datas))(*[_lib.get_image_info(d) for d in datas])
    return torch.from_numpy(host).pin_memory(), np.asarray(offs), np.asarray(sizes), infos


@pytest.mark.parametrize("lean", [1, 0])
@pytest.mark.parametrize("lanes", [1, 4])
def test_batch_waits_for_the_callers_pending_copy(decoder, oracle, lean, lanes):
    datas = [cases.case(f"bench_{1000 + i}") for i in range(8)] + [cases.case("q90_444"),
                                                                   cases.case("gray")]
    refs = [oracle.decode_resize(d, oracle.Resize(**PAD), pix_fmt="rgb24") for d in datas]
    host, offs, sizes, infos = _pack(datas)
    spec = Output(pix_fmt="rgb24", resize=True, **PAD)
    prev = (decoder.get_param("lean_waits"), decoder.get_param("lanes"))
    decoder.set_param("lean_waits", lean)
    decoder.set_param("lanes", lanes)
    try:
        s = torch.cuda.Stream()
        a = torch.randn(4096, 4096, device="cuda:0", dtype=torch.bfloat16)
        outs, tickets, devs = [], [], []
        for k in range(6):
            dev = torch.zeros(host.numel(), dtype=torch.uint8, device="cuda:0")
            out = torch.empty((len(datas), 224, 224, 3), dtype=torch.uint8, device="cuda:0")
            with torch.cuda.stream(s):
                for _ in range(20 if k == 0 else 2):  # keep the caller's stream busy
                    a = (a @ a).clamp_(-1, 1)
                dev.copy_(host, non_blocking=True)  # the bytes arrive only after the GEMMs
            decoder.decode_batch_device(dev.data_ptr(), dev.numel(), offs, sizes, infos, spec,
                                        out.data_ptr(), out.numel(), stream=s, sync=False)
            tickets.append(decoder.last_ticket())
            outs.append(out)
            devs.append(dev)
        for t, out in zip(tickets, outs):
            assert not any(decoder.wait(t, len(datas)))
            hyp = out.cpu().numpy()
            for i, r in enumerate(refs):
                np.testing.assert_array_equal(hyp[i], r, strict=True, err_msg=f"image {i}")
        s.synchronize()
    finally:
        decoder.set_param("lean_waits", prev[0])
        decoder.set_param("lanes", prev[1])
