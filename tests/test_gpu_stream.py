"""GPU: the staging ring (async submission, tickets) and the tar stream
(config 5 shape), bit-exact against the oracle on every image.
"""

import io
import tarfile

import numpy as np
import pytest
import torch

import spdl_amd.io as sio
from spdl_amd import _lib
from spdl_amd._lib import Output
from spdl_amd.synthetic import synthetic_jpeg
from tests import cases

pytestmark = pytest.mark.gpu

OUT224 = Output(pix_fmt="rgb24", resize=True, fit_w=224, fit_h=224, aspect="decrease",
                pad_w=224, pad_h=224)


def _rs(oracle):
    return oracle.Resize(fit_w=224, fit_h=224, aspect="decrease", pad_w=224, pad_h=224)


def _images():
    imgs = [synthetic_jpeg(100 + i, 480, 640) for i in range(6)]
    imgs += [cases.case("odd_227x333"), cases.case("q90_444"), cases.case("restart_rows"),
             cases.case("gray")]
    # a member whose size is an exact multiple of 512: the next tar header
    # follows the image bytes with no zero padding (bytes after EOI are ignored)
    d = synthetic_jpeg(7, 240, 320)
    imgs.append(d + b"\x00" * ((-len(d)) % 512))
    return imgs


def _tar(imgs, extra=True) -> bytes:
    b = io.BytesIO()
    with tarfile.open(fileobj=b, mode="w", format=tarfile.GNU_FORMAT) as t:
        for i, d in enumerate(imgs):
            ti = tarfile.TarInfo(f"shard/{i:05d}.jpg")
            ti.size = len(d)
            t.addfile(ti, io.BytesIO(d))
            if extra and i % 3 == 0:  # webdataset-style side car, skipped by the stream
                lab = f"{i}".encode()
                ti = tarfile.TarInfo(f"shard/{i:05d}.cls")
                ti.size = len(lab)
                t.addfile(ti, io.BytesIO(lab))
    return b.getvalue()


def test_async_ring_matches_sync(decoder, oracle):
    imgs = _images()
    groups = [imgs[0:3], imgs[3:6], imgs[6:9], imgs[9:11], imgs[0:2]]
    outs, tickets = [], []
    stream = torch.cuda.current_stream()
    for g in groups[:2]:
        t = torch.empty((len(g), 224, 224, 3), dtype=torch.uint8, device="cuda:0")
        decoder.decode_batch(g, OUT224, t.data_ptr(), t.numel(), stream=stream, sync=False)
        outs.append(t)
        tickets.append(decoder.last_ticket())
    assert tickets[1] == tickets[0] + 1
    assert decoder.wait(tickets[0], len(groups[0])) == [0] * len(groups[0])
    for g in groups[2:]:
        t = torch.empty((len(g), 224, 224, 3), dtype=torch.uint8, device="cuda:0")
        decoder.decode_batch(g, OUT224, t.data_ptr(), t.numel(), stream=stream, sync=False)
        outs.append(t)
        tickets.append(decoder.last_ticket())
        decoder.wait(tickets[-2], len(groups[len(tickets) - 2]))
    decoder.wait(tickets[-1], len(groups[-1]))
    with pytest.raises(RuntimeError):
        decoder.wait(tickets[-1], len(groups[-1]))  # already waited
    rs = _rs(oracle)
    for g, t in zip(groups, outs):
        hyp = t.cpu().numpy()
        for i, d in enumerate(g):
            np.testing.assert_array_equal(hyp[i], oracle.decode_resize(d, rs, "rgb24"))


@pytest.mark.parametrize("src_kind", ["bytes", "path"])
@pytest.mark.parametrize("batch_size", [1, 4, 16])
def test_tar_stream_bit_exact(oracle, tmp_path, src_kind, batch_size):
    imgs = _images()
    data = _tar(imgs)
    src = data
    if src_kind == "path":
        src = str(tmp_path / "shard.tar")
        with open(src, "wb") as f:
            f.write(data)
    cfg = sio.cuda_config(device_index=0)
    rs = _rs(oracle)
    seen = []
    with sio.TarImageStream(src, batch_size=batch_size, device_config=cfg) as st:
        assert len(st.members) == len(imgs)
        for names, t in st:
            assert t.shape[1:] == (224, 224, 3) and t.device.type == "cuda"
            hyp = t.cpu().numpy()
            for n, h in zip(names, hyp):
                i = int(n.split("/")[1].split(".")[0])
                np.testing.assert_array_equal(h, oracle.decode_resize(imgs[i], rs, "rgb24"))
                seen.append(i)
    assert seen == list(range(len(imgs)))


def test_tar_stream_planar_fp16(oracle):
    imgs = _images()[:5]
    out = Output(pix_fmt="rgb", resize=True, fit_w=256, fit_h=256, aspect="decrease",
                 pad_w=256, pad_h=256, crop_w=224, crop_h=224, normalize=True)
    rs = oracle.Resize(fit_w=256, fit_h=256, aspect="decrease", pad_w=256, pad_h=256,
                       crop_w=224, crop_h=224)
    with sio.TarImageStream(_tar(imgs), batch_size=2, output=out,
                            device_config=sio.cuda_config(0)) as st:
        got = [t.cpu() for _, t in st]
    hyp = torch.cat(got).numpy()
    assert hyp.dtype == np.float16 and hyp.shape == (5, 3, 224, 224)
    for i, d in enumerate(imgs):
        ref = oracle.decode_resize(d, rs, "rgb", normalize=True)
        np.testing.assert_array_equal(hyp[i].view(np.uint16), ref.view(np.uint16))


def test_tar_stream_error_then_recovery(oracle):
    good = _images()[:3]
    bad = cases.truncated()
    try:
        oracle.decode_rgb(bad)
        pytest.skip("corrupt case decodes on the oracle")
    except oracle.OracleError:
        pass
    with sio.TarImageStream(_tar([good[0], bad, good[1]], extra=False), batch_size=3,
                            device_config=sio.cuda_config(0)) as st:
        with pytest.raises(RuntimeError, match="Failed to decode an image"):
            list(st)
    # the same decoder machinery keeps working afterwards
    with sio.TarImageStream(_tar(good, extra=False), batch_size=2,
                            device_config=sio.cuda_config(0)) as st:
        n = sum(t.shape[0] for _, t in st)
    assert n == 3


def test_staged_rejects_unaligned_and_stale(decoder):
    d = synthetic_jpeg(1, 64, 64)
    ptr, ticket = decoder.staging_acquire(4096)
    import ctypes

    ctypes.memmove(ptr + 100, d, len(d))
    out = torch.empty((1, 64, 64, 3), dtype=torch.uint8, device="cuda:0")
    with pytest.raises(RuntimeError, match="aligned"):
        decoder.decode_staged(ticket, 100 + len(d), [100], [len(d)], Output(pix_fmt="rgb24"),
                              out.data_ptr(), out.numel())
    with pytest.raises(RuntimeError):  # the slot was consumed by the failed call
        decoder.decode_staged(ticket, 100 + len(d), [0], [len(d)], Output(pix_fmt="rgb24"),
                              out.data_ptr(), out.numel())
    ptr, ticket = decoder.staging_acquire(4096)
    ctypes.memmove(ptr + 512, d, len(d))
    decoder.decode_staged(ticket, 512 + len(d), [512], [len(d)], Output(pix_fmt="rgb24"),
                          out.data_ptr(), out.numel())
    assert _lib is not None
