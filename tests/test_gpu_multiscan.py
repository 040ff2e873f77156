"""GPU tests of progressive and non-interleaved multi-scan JPEGs (-m gpu).

The per-case parity (planes, rgb24, JFIF) runs in test_gpu_parity.py over
cases.VALID, which includes cases.PROGRESSIVE and cases.MULTISCAN (their
oracle is pinned to libjpeg 9 coefficients in test_oracle.py).  Here: mixed
batches -- progressive and baseline images in one call, through the resize
chain and the device-resident entry point -- and the unsupported formats.
"""

import numpy as np
import pytest
import torch

import spdl_amd.io as sio
from spdl_amd import _lib
from spdl_amd._lib import Output
from tests import cases

pytestmark = pytest.mark.gpu

PAD224 = dict(fit_w=224, fit_h=224, aspect="decrease", pad_w=224, pad_h=224)


def _mixed():
    names = ["q90_420", "prog_420", "multiscan_420", "prog_gray", "q90_444", "prog_restart",
             "multiscan_422_rst", "prog_optimized"]
    return [cases.case(n) for n in names]


def test_mixed_batch_pad224(oracle):
    datas = _mixed()
    hyp = sio.to_numpy(sio.load_image_batch(datas, width=224, height=224))
    rs = oracle.Resize(**PAD224)
    for i, d in enumerate(datas):
        np.testing.assert_array_equal(hyp[i], oracle.decode_resize(d, rs, "rgb24"), strict=True)


def test_mixed_batch_device_resident(oracle):
    """decode_batch_device (bytes already in HBM) with two batches in flight."""
    datas = _mixed() * 4
    offs, sizes, total = [], [], 0
    for d in datas:
        offs.append(total)
        sizes.append(len(d))
        total += (len(d) + 64 + 255) // 256 * 256
    host = np.zeros(total, np.uint8)
    for o, d in zip(offs, datas):
        host[o:o + len(d)] = np.frombuffer(d, np.uint8)
    dev = torch.from_numpy(host).to("cuda:0")
    infos = (_lib.ImageInfo * len(datas))(*[_lib.get_image_info(d) for d in datas])
    spec = Output(pix_fmt="rgb24", resize=True, **PAD224)
    dec = _lib.Decoder(0)
    dec.set_param("lanes", 2)
    outs = [torch.zeros((len(datas), 224, 224, 3), dtype=torch.uint8, device="cuda:0")
            for _ in range(2)]
    tickets = []
    for o in outs:
        dec.decode_batch_device(dev.data_ptr(), dev.numel(), np.asarray(offs, np.int64),
                                np.asarray(sizes, np.int64), infos, spec, o.data_ptr(), o.numel(),
                                stream=torch.cuda.current_stream(), sync=False)
        tickets.append(dec.last_ticket())
    for t in tickets:
        assert not any(dec.wait(t, len(datas)))
    torch.cuda.synchronize()
    rs = oracle.Resize(**PAD224)
    refs = [oracle.decode_resize(d, rs, "rgb24") for d in datas[:8]]
    for o in outs:
        hyp = o.cpu().numpy()
        for i in range(len(datas)):
            np.testing.assert_array_equal(hyp[i], refs[i % 8], strict=True)
    dec.close()


@pytest.mark.parametrize("name", ["prog_420", "multiscan_444_odd", "prog_gray"])
def test_native_planes(oracle, name):
    """load_image(filter_desc=None) of a multi-scan image: the planes."""
    d = cases.case(name)
    hyp = sio.to_numpy(sio.load_image(d, filter_desc=None))
    ref = np.concatenate([p.reshape(-1) for p in oracle.decode_planes(d)])
    np.testing.assert_array_equal(hyp.reshape(-1), ref, strict=True)


@pytest.mark.parametrize("name", cases.LARGE_PROGRESSIVE)
def test_large_progressive_planes(oracle, name):
    """Scans larger than the decoder's LDS byte window (restaged mid-scan,
    also across restart markers), many AC-refinement chunks: planes
    bit-exact vs the oracle (whose progressive decode is pinned to libjpeg 9
    coefficients in test_oracle.py)."""
    d = cases.case(name)
    hyp = sio.to_numpy(sio.load_image(d, filter_desc=None))
    ref = np.concatenate([p.reshape(-1) for p in oracle.decode_planes(d)])
    np.testing.assert_array_equal(hyp.reshape(-1), ref, strict=True)


@pytest.mark.parametrize("subsampling", [0, 2])
@pytest.mark.parametrize("quality", [20, 50, 75, 90, 95, 100])
def test_progressive_quality_sweep(oracle, quality, subsampling):
    """The AC refinement scans' scalar symbol loop (ms_ref_fast) and its side
    paths -- codes longer than 6 bits, ZRL, EOB runs, more than 15
    correction bits (the general step) -- over the code tables and history
    densities the encoder's quality produces, smooth and noise pixels:
    planes bit-exact vs the oracle."""
    from spdl_amd.synthetic import synthetic_pixels

    for px in (synthetic_pixels(7, 240, 320), cases._noise(8, 96, 160)):
        d = cases._enc(px, quality=quality, subsampling=subsampling, progressive=True)
        assert _lib.get_image_info(d).multiscan == 1
        hyp = sio.to_numpy(sio.load_image(d, filter_desc=None))
        ref = np.concatenate([p.reshape(-1) for p in oracle.decode_planes(d)])
        np.testing.assert_array_equal(hyp.reshape(-1), ref, strict=True)


@pytest.mark.parametrize("blocks_wide,blocks_high", [(8, 8), (63, 1), (64, 1), (65, 1),
                                                    (13, 5), (1, 1), (16, 9)])
@pytest.mark.parametrize("gray", [True, False])
def test_progressive_chunk_edges(oracle, blocks_wide, blocks_high, gray):
    """Refinement scans visit a component's blocks in chunks of 64 (one per
    lane: levels and masks loaded, records applied, progress published per
    chunk): component block counts below, at and past a chunk, odd shapes
    and a single block, gray and 4:2:0 (chroma with a quarter of the blocks):
    planes bit-exact vs the oracle."""
    rng = np.random.default_rng(blocks_wide * 100 + blocks_high)
    h, w = 8 * blocks_high - (rng.integers(0, 4) if blocks_high > 1 else 0), 8 * blocks_wide
    if gray:
        px = rng.integers(0, 256, size=(h, w), dtype=np.uint8)
        d = cases._enc(px, quality=92, progressive=True)
    else:
        px = rng.integers(0, 256, size=(2 * h, 2 * w, 3), dtype=np.uint8)
        d = cases._enc(px, quality=92, subsampling=2, progressive=True)
    assert _lib.get_image_info(d).multiscan == 1
    hyp = sio.to_numpy(sio.load_image(d, filter_desc=None))
    ref = np.concatenate([p.reshape(-1) for p in oracle.decode_planes(d)])
    np.testing.assert_array_equal(hyp.reshape(-1), ref, strict=True)


def test_large_progressive_batch_pad224(oracle):
    """Large progressive images mixed with baseline ones through the resize chain."""
    datas = [cases.case(n) for n in ("prog_large_420", "q90_420", "prog_large_restart",
                                     "prog_large_noise")]
    hyp = sio.to_numpy(sio.load_image_batch(datas, width=224, height=224))
    rs = oracle.Resize(**PAD224)
    for i, d in enumerate(datas):
        np.testing.assert_array_equal(hyp[i], oracle.decode_resize(d, rs, "rgb24"), strict=True)


def _agree_or_both_fail(oracle, d):
    """The GPU decode equals the oracle's, or both reject the image; later
    calls still work."""
    try:
        ref = oracle.decode_rgb(d, 0, "rgb24")
    except oracle.OracleError:
        ref = None
    info = oracle.parse(d)
    dec = _lib.Decoder(0)
    t = torch.empty((info.height, info.width, 3), dtype=torch.uint8, device="cuda:0")
    if ref is None:
        with pytest.raises(RuntimeError, match="Failed to decode an image"):
            dec.decode_batch([d], Output(pix_fmt="rgb24"), t.data_ptr(), t.numel())
    else:
        dec.decode_batch([d], Output(pix_fmt="rgb24"), t.data_ptr(), t.numel())
        np.testing.assert_array_equal(t.cpu().numpy(), ref, strict=True)
    good = cases.case("prog_422")
    gi = oracle.parse(good)
    g = torch.empty((gi.height, gi.width, 3), dtype=torch.uint8, device="cuda:0")
    dec.decode_batch([good], Output(pix_fmt="rgb24"), g.data_ptr(), g.numel())
    np.testing.assert_array_equal(g.cpu().numpy(), oracle.decode_rgb(good, 0, "rgb24"), strict=True)
    dec.close()


@pytest.mark.parametrize("seed", range(10))
def test_corrupt_progressive_agrees_with_oracle(oracle, seed):
    """Corrupt scan data / scan headers: the two concurrent scan decoders
    either reproduce the oracle's pixels or fail the image as it does (no
    hang waiting for a scan that failed)."""
    _agree_or_both_fail(oracle, cases.corrupt_progressive(seed))


@pytest.mark.parametrize("frac", [0.3, 0.5, 0.8, 0.97])
def test_truncated_progressive(oracle, frac):
    _agree_or_both_fail(oracle, cases.truncated_progressive(frac))


@pytest.mark.parametrize("bad", ["arithmetic", "twelve_bit"])
def test_unsupported_fails_per_image(bad):
    """An unsupported image fails alone: strict=False keeps the others."""
    d = getattr(cases, bad)()
    good = [cases.case("prog_420"), cases.case("q90_420")]
    with pytest.raises(RuntimeError):
        sio.load_image_batch([d, *good], width=64, height=64, strict=True)
    buf = sio.load_image_batch([d, *good], width=64, height=64, strict=False)
    assert sio.to_numpy(buf).shape == (2, 64, 64, 3)


@pytest.mark.parametrize("name", cases.METADATA)
def test_progressive_with_ff_metadata(oracle, name):
    """Binary metadata full of 0xFF xx pairs (an APP2 blob before the frame, a
    COM segment between scans) neither fails the image nor ends a scan
    early: planes and RGB224 bit-exact vs the oracle."""
    d = cases.case(name)
    ref = oracle.decode_planes(d, oracle.IDCT_SIMPLE)
    hyp = _lib.thread_decoder(0).decode_planes(d)
    for c in range(len(ref)):
        np.testing.assert_array_equal(hyp[c], ref[c], strict=True)


def test_probe_flags_the_multiscan_path():
    """spdl_hj_image_info.multiscan (ABI 5): what lets the device-resident
    entry point run the multi-scan decoder beside the baseline stages."""
    for n in ["q90_420", "q90_444", "gray", "odd_227x333"]:
        assert _lib.get_image_info(cases.case(n)).multiscan == 0, n
    for n in ["prog_420", "prog_gray", "multiscan_420", "multiscan_cmyk", "prog_restart"]:
        assert _lib.get_image_info(cases.case(n)).multiscan == 1, n


def _with_size_mod(d: bytes, mod: int) -> bytes:
    """d with a COM segment after SOI sized so that len % 256 == mod."""
    need = (mod - (len(d) + 4)) % 256
    return d[:2] + b"\xff\xfe" + (need + 2).to_bytes(2, "big") + b"\x00" * need + d[2:]


@pytest.mark.parametrize("mod", [252, 253, 254, 255, 0])
def test_tightly_packed_device_batch(oracle, mod):
    """Images back to back at 256-byte offsets (no slack after a file): the
    multi-scan decoder's destuffed copy (side stream) must stay inside its
    own image's bytes while the next image is destuffed and decoded."""
    prog = [_with_size_mod(cases.case(n), mod) for n in ["prog_420", "multiscan_420",
                                                          "prog_optimized"]]
    base = [cases.case(n) for n in ["q90_420", "q90_444", "q75_420"]]
    datas = [x for pair in zip(prog * 4, base * 4) for x in pair]
    assert all(len(d) % 256 == mod for d in datas[::2])
    offs, total = [], 0
    for d in datas:
        offs.append(total)
        total = (total + len(d) + 255) // 256 * 256
    host = np.zeros(total + 512, np.uint8)
    for o, d in zip(offs, datas):
        host[o:o + len(d)] = np.frombuffer(d, np.uint8)
    dev = torch.from_numpy(host).to("cuda:0")
    infos = [_lib.get_image_info(d) for d in datas]
    assert sum(i.multiscan for i in infos) == len(datas) // 2
    spec = Output(pix_fmt="rgb24", resize=True, **PAD224)
    dec = _lib.Decoder(0)
    out = torch.zeros((len(datas), 224, 224, 3), dtype=torch.uint8, device="cuda:0")
    for _ in range(3):
        assert not any(dec.decode_batch_device(dev.data_ptr(), dev.numel(), offs,
                                               [len(d) for d in datas], infos, spec,
                                               out.data_ptr(), out.numel()))
    rs = oracle.Resize(**PAD224)
    hyp = out.cpu().numpy()
    for i, d in enumerate(datas):
        np.testing.assert_array_equal(hyp[i], oracle.decode_resize(d, rs, "rgb24"), strict=True)
    dec.close()
