"""GPU parity: the gfx950 decode stage vs the CPU oracle, through the C-ABI.

Bar (north_star): bit-exact for the integer stages (planes, rgb after the
integer colour conversion, resize in fixed point); normalised fp16 output
bit-exact as well (same IEEE op sequence), tolerance 0.
"""

import numpy as np
import pytest
import torch

from spdl_amd._lib import Output
from tests import cases

pytestmark = pytest.mark.gpu


def _decode(decoder, datas, out: Output, shape, dtype=torch.uint8):
    t = torch.empty((len(datas),) + tuple(shape), dtype=dtype, device="cuda:0")
    status = decoder.decode_batch(datas, out, t.data_ptr(), t.numel() * t.element_size(),
                                  stream=torch.cuda.current_stream())
    assert all(s == 0 for s in status)
    return t.cpu()


@pytest.mark.parametrize("name", cases.VALID)
@pytest.mark.parametrize("idct", ["simple", "islow"])
def test_planes_bit_exact(decoder, oracle, name, idct):
    d = cases.case(name)
    hyp = decoder.decode_planes(d, idct=idct)
    ref = oracle.decode_planes(d, idct=oracle.IDCT_ISLOW if idct == "islow" else oracle.IDCT_SIMPLE)
    assert len(hyp) == len(ref)
    for h, r in zip(hyp, ref):
        np.testing.assert_array_equal(h, r, strict=True)


@pytest.mark.parametrize("name", cases.VALID)
@pytest.mark.parametrize("pix_fmt", ["rgb", "rgb24", "bgr", "bgr24"])
def test_fullres_rgb_bit_exact(decoder, oracle, name, pix_fmt):
    d = cases.case(name)
    info = oracle.parse(d)
    W, H = info.width, info.height
    shape = (3, H, W) if pix_fmt in ("rgb", "bgr") else (H, W, 3)
    hyp = _decode(decoder, [d], Output(pix_fmt=pix_fmt), shape)[0].numpy()
    ref = oracle.decode_rgb(d, oracle.IDCT_SIMPLE, pix_fmt)
    np.testing.assert_array_equal(hyp, ref, strict=True)


@pytest.mark.parametrize("name", ["q90_420", "odd_227x333", "gray", "restart_blocks", "noise_420",
                                  "rgb_coded", "rgb_ids_only"])
def test_islow_matches_libjpeg_fixture(decoder, oracle, name):
    """islow mode end-to-end vs libjpeg 9d when the pin helper is present."""
    d = cases.case(name)
    if oracle.ljpin() is None:
        pytest.skip("libjpeg 9 not available on this host")
    info = oracle.parse(d)
    hyp = _decode(decoder, [d], Output(pix_fmt="rgb24", idct="islow", csc="jfif"),
                  (info.height, info.width, 3))
    ref = oracle.lj_decode_rgb(d)
    np.testing.assert_array_equal(hyp[0].numpy(), ref, strict=True)


RESIZES = {
    "pad224": dict(fit_w=224, fit_h=224, aspect="decrease", pad_w=224, pad_h=224),
    "crop224": dict(fit_w=224, fit_h=224, aspect="increase", crop_w=224, crop_h=224),
    "stretch160x120": dict(fit_w=160, fit_h=120),
    "imagenet": dict(fit_w=256, fit_h=256, aspect="decrease", pad_w=256, pad_h=256, crop_w=224,
                     crop_h=224),
    "upscale": dict(fit_w=700, fit_h=500),
}


@pytest.mark.parametrize("name", ["q90_420", "odd_227x333", "gray", "q90_444", "restart_rows",
                                  "large_1080p", "tiny_8x8", "cmyk_pillow_odd", "ycck_adobe",
                                  "rgb_coded_odd_rst"])
@pytest.mark.parametrize("rk", list(RESIZES))
@pytest.mark.parametrize("filt", ["bicubic", "bilinear", "lanczos"])
def test_resize_bit_exact(decoder, oracle, name, rk, filt):
    d = cases.case(name)
    kw = RESIZES[rk]
    rs = oracle.Resize(filter=filt, **kw)
    ref = oracle.decode_resize(d, rs, pix_fmt="rgb")
    out = Output(pix_fmt="rgb", resize=True, filter=filt, **kw)
    hyp = _decode(decoder, [d], out, ref.shape)[0].numpy()
    np.testing.assert_array_equal(hyp, ref, strict=True)


@pytest.mark.parametrize("name", ["q90_420", "odd_227x333", "gray", "q90_444", "q90_422",
                                  "large_1080p", "tiny_8x8", "cmyk_pillow_odd", "ycck_adobe",
                                  "rgb_coded_odd_rst"])
@pytest.mark.parametrize("rk", list(RESIZES))
@pytest.mark.parametrize("filt", ["bicubic", "bilinear", "lanczos"])
def test_resize_prepass_bit_exact(decoder, oracle, name, rk, filt):
    """The same outputs with the horizontal pass forced into hscale_kernel
    (sws_prepass=1: every source row filtered once into HBM, the bands
    staged from there) -- the path large downscales take automatically."""
    d = cases.case(name)
    kw = RESIZES[rk]
    ref = oracle.decode_resize(d, oracle.Resize(filter=filt, **kw), pix_fmt="rgb")
    out = Output(pix_fmt="rgb", resize=True, filter=filt, **kw)
    decoder.set_param("sws_prepass", 1)
    try:
        hyp = _decode(decoder, [d], out, ref.shape)[0].numpy()
    finally:
        decoder.set_param("sws_prepass", -1)
    np.testing.assert_array_equal(hyp, ref, strict=True)


@pytest.mark.parametrize("pix_fmt", ["rgb", "rgb24"])
def test_normalize_fp16_bit_exact(decoder, oracle, pix_fmt):
    d = cases.case("q90_420")
    kw = RESIZES["pad224"]
    ref = oracle.decode_resize(d, oracle.Resize(**kw), pix_fmt=pix_fmt, normalize=True)
    out = Output(pix_fmt=pix_fmt, resize=True, normalize=True, **kw)
    hyp = _decode(decoder, [d], out, ref.shape, dtype=torch.float16)[0].numpy()
    np.testing.assert_array_equal(hyp.view(np.uint16), ref.view(np.uint16), strict=True)


@pytest.mark.parametrize("norm_dtype", ["float16", "bfloat16"])
def test_normalize_matches_torch_preprocessing(decoder, oracle, norm_dtype):
    """Config 4 epilogue vs the reference's own torch ops on our u8 output:
    x.float()/255, (x - mean)/std in fp32, then .to(dtype) (reference
    examples/imagenet_classification.py:95-106,162-163, NCHW via permute at
    :265).  Tolerance 0: the fused kernel does the same IEEE fp32 ops."""
    datas = [cases.case(n) for n in ("q90_420", "odd_227x333", "gray")]
    kw = dict(fit_w=256, fit_h=256, aspect="decrease", pad_w=256, pad_h=256, crop_w=224,
              crop_h=224)
    u8 = _decode(decoder, datas, Output(pix_fmt="rgb24", resize=True, **kw), (224, 224, 3))
    tdt = torch.bfloat16 if norm_dtype == "bfloat16" else torch.float16
    out = Output(pix_fmt="rgb", resize=True, normalize=True, norm_dtype=norm_dtype, **kw)
    hyp = _decode(decoder, datas, out, (3, 224, 224), dtype=tdt)
    mean = torch.tensor([0.4850, 0.4560, 0.4060]).view(1, 3, 1, 1)
    std = torch.tensor([0.2290, 0.2240, 0.2250]).view(1, 3, 1, 1)
    x = u8.permute(0, 3, 1, 2).float() / 255.0
    ref = ((x - mean) / std).to(tdt)
    assert torch.equal(hyp.view(torch.int16), ref.view(torch.int16))
    if norm_dtype == "bfloat16":
        for i, d in enumerate(datas):
            o = oracle.decode_resize(d, oracle.Resize(**kw), pix_fmt="rgb", normalize=True,
                                     norm_dtype="bfloat16")
            np.testing.assert_array_equal(hyp[i].view(torch.int16).numpy().view(np.uint16), o)


def test_batch_mixed_sizes_resize(decoder, oracle):
    names = ["q90_420", "odd_227x333", "gray", "restart_blocks", "q90_444", "noise_420",
             "large_1080p", "optimized"]
    datas = [cases.case(n) for n in names]
    kw = RESIZES["pad224"]
    out = Output(pix_fmt="rgb24", resize=True, **kw)
    hyp = _decode(decoder, datas, out, (224, 224, 3)).numpy()
    for i, d in enumerate(datas):
        ref = oracle.decode_resize(d, oracle.Resize(**kw), pix_fmt="rgb24")
        np.testing.assert_array_equal(hyp[i], ref, strict=True)


def test_batch_shared_and_distinct_huffman_tables(decoder, oracle):
    """lut_kernel builds a Huffman table once per distinct table of the batch
    (the first image holding the bytes) and the others read that build:
    repeated files, files sharing the standard tables (gray's luma slots
    among them), files with their own optimised tables (the same slots, other
    bytes) and six-table files -- every image bit-exact vs the oracle."""
    names = ["optimized", "q90_420", "optimized", "six_tables", "q90_444", "q75_420", "q90_420",
             "six_tables", "gray", "optimized", "restart_rows", "q75_420"]
    datas = [cases.case(n) for n in names]
    kw = RESIZES["pad224"]
    out = Output(pix_fmt="rgb24", resize=True, **kw)
    hyp = _decode(decoder, datas, out, (224, 224, 3)).numpy()
    for i, d in enumerate(datas):
        ref = oracle.decode_resize(d, oracle.Resize(**kw), pix_fmt="rgb24")
        np.testing.assert_array_equal(hyp[i], ref, strict=True)


@pytest.mark.parametrize("fmt", ["rgb24", "bf16"])
def test_batch_mixed_cmyk(decoder, oracle, fmt):
    """Colour models in one batch: Adobe CMYK (K transform -> three RGB
    planes through the luma filters), YCCK (-> YCbCr 4:4:4), YCbCr + K (no
    marker: K dropped), RGB-coded 3-component frames (gbrp), YCbCr and gray:
    per-image plans and the K transform (FFmpeg's, restated by the oracle;
    parity unpinned against FFmpeg itself)."""
    names = ["cmyk_adobe", "q90_420", "ycck_adobe", "gray", "cmyk_pillow", "ycck_odd_rst",
             "cmyk_pillow_odd", "q90_444", "rgb_coded", "cmyk_no_marker", "rgb_adobe_only"]
    datas = [cases.case(n) for n in names]
    kw = RESIZES["imagenet"]
    if fmt == "rgb24":
        out, shape, dt = Output(pix_fmt="rgb24", resize=True, **kw), (224, 224, 3), torch.uint8
    else:
        out = Output(pix_fmt="rgb", resize=True, normalize=True, norm_dtype="bfloat16", **kw)
        shape, dt = (3, 224, 224), torch.bfloat16
    hyp = _decode(decoder, datas, out, shape, dtype=dt)
    for i, d in enumerate(datas):
        if fmt == "rgb24":
            ref = oracle.decode_resize(d, oracle.Resize(**kw), pix_fmt="rgb24")
            np.testing.assert_array_equal(hyp[i].numpy(), ref, strict=True)
        else:
            ref = oracle.decode_resize(d, oracle.Resize(**kw), pix_fmt="rgb", normalize=True,
                                       norm_dtype="bfloat16")
            np.testing.assert_array_equal(hyp[i].view(torch.int16).numpy().view(np.uint16), ref)


def test_batch_256_fullres(decoder, oracle):
    from spdl_amd.synthetic import synthetic_batch

    datas = synthetic_batch(256, distinct=8)
    hyp = _decode(decoder, datas, Output(pix_fmt="rgb24"), (480, 640, 3)).numpy()
    refs = {}
    for i, d in enumerate(datas):
        if d not in refs:
            refs[d] = oracle.decode_rgb(d, oracle.IDCT_SIMPLE, "rgb24")
        np.testing.assert_array_equal(hyp[i], refs[d], strict=True)


@pytest.mark.parametrize("bad", ["arithmetic", "twelve_bit", "truncated", "not_jpeg", "corrupt"])
def test_errors_then_recover(decoder, oracle, bad):
    """Rubbish raises RuntimeError and later calls still work
    (reference tests/cuda/nvjpeg_decode_test.py:51-78)."""
    if bad == "arithmetic":
        d = cases.arithmetic()
    elif bad == "twelve_bit":
        d = cases.twelve_bit()
    elif bad == "truncated":
        d = cases.truncated()
    elif bad == "not_jpeg":
        d = bytes(np.random.default_rng(0).integers(0, 256, 5000, dtype=np.uint8))
    else:
        d = cases.corrupt_scan(3)
    ok_ref = True
    try:
        oracle.decode_rgb(d)
    except oracle.OracleError:
        ok_ref = False
    if bad != "corrupt":
        assert not ok_ref
    info_ok = True
    try:
        info = oracle.parse(d)
    except oracle.OracleError:
        info_ok = False
    if info_ok:
        shape = (info.height, info.width, 3)
    else:
        shape = (8, 8, 3)
    t = torch.empty(shape, dtype=torch.uint8, device="cuda:0")
    if ok_ref:
        decoder.decode_batch([d], Output(pix_fmt="rgb24"), t.data_ptr(), t.numel())
        np.testing.assert_array_equal(t.cpu().numpy(), oracle.decode_rgb(d, 0, "rgb24"))
    else:
        with pytest.raises(RuntimeError, match="Failed to decode an image"):
            decoder.decode_batch([d], Output(pix_fmt="rgb24"), t.data_ptr(), t.numel())
    # recovery
    good = cases.case("q90_444")
    hyp = _decode(decoder, [good], Output(pix_fmt="rgb24"), (240, 320, 3))[0].numpy()
    np.testing.assert_array_equal(hyp, oracle.decode_rgb(good, 0, "rgb24"))


@pytest.mark.parametrize("seed", range(12))
def test_corrupt_streams_agree_with_oracle(decoder, oracle, seed):
    d = cases.corrupt_scan(seed)
    try:
        ref = oracle.decode_rgb(d, 0, "rgb24")
    except oracle.OracleError:
        ref = None
    info = oracle.parse(d)
    t = torch.empty((info.height, info.width, 3), dtype=torch.uint8, device="cuda:0")
    if ref is None:
        with pytest.raises(RuntimeError):
            decoder.decode_batch([d], Output(pix_fmt="rgb24"), t.data_ptr(), t.numel())
    else:
        decoder.decode_batch([d], Output(pix_fmt="rgb24"), t.data_ptr(), t.numel())
        np.testing.assert_array_equal(t.cpu().numpy(), ref)


@pytest.mark.parametrize("threads", [128, 256, 512, 1024])
@pytest.mark.parametrize("sub_bits", [32, 64, 256, 1024, 8192])
def test_subsequence_sizes(oracle, sub_bits, threads):
    """The sync result must not depend on the subsequence size or on the
    number of Huffman decoder threads per image."""
    from spdl_amd._lib import Decoder

    dec = Decoder(0)
    dec.set_param("sub_bits", sub_bits)
    dec.set_param("entropy_threads", threads)
    for name in ["q90_420", "restart_blocks", "noise_420", "gray_odd"]:
        d = cases.case(name)
        info = oracle.parse(d)
        hyp = _decode(dec, [d], Output(pix_fmt="rgb24"), (info.height, info.width, 3))[0].numpy()
        np.testing.assert_array_equal(hyp, oracle.decode_rgb(d, 0, "rgb24"))
    for seed in range(6):
        d = cases.corrupt_scan(seed)
        try:
            ref = oracle.decode_rgb(d, 0, "rgb24")
        except oracle.OracleError:
            ref = None
        info = oracle.parse(d)
        t = torch.empty((info.height, info.width, 3), dtype=torch.uint8, device="cuda:0")
        if ref is None:
            with pytest.raises(RuntimeError):
                dec.decode_batch([d], Output(pix_fmt="rgb24"), t.data_ptr(), t.numel())
        else:
            dec.decode_batch([d], Output(pix_fmt="rgb24"), t.data_ptr(), t.numel())
            np.testing.assert_array_equal(t.cpu().numpy(), ref)
    dec.close()


@pytest.mark.parametrize("pix_fmt", ["rgb", "rgb24", "bgr", "bgr24"])
@pytest.mark.parametrize("w,h", [(64, 48), (102, 70), (30, 18)])
def test_fullres_batch_unscaled_converter(decoder, oracle, pix_fmt, w, h):
    """Full-resolution batches: 420 / 422 images of one size take swscale's
    unscaled converter (idct_rgb_kernel); adding a 444 image sends the
    batch through the generic sws_kernel.  Both bit-exact vs the oracle."""
    datas = [cases._enc(cases._noise(s, h, w), quality=85 + s, subsampling=2 if s % 2 else 1)
             for s in range(5)]
    shape = (3, h, w) if pix_fmt in ("rgb", "bgr") else (h, w, 3)
    for batch in (datas, datas + [cases._enc(cases._noise(9, h, w), quality=90, subsampling=0)]):
        hyp = _decode(decoder, batch, Output(pix_fmt=pix_fmt), shape).numpy()
        for i, d in enumerate(batch):
            np.testing.assert_array_equal(hyp[i], oracle.decode_rgb(d, oracle.IDCT_SIMPLE, pix_fmt),
                                          strict=True)


@pytest.mark.parametrize("sub,h,w", [(2, 480, 640), (1, 480, 640), (2, 1080, 1920), (1, 46, 1350)])
def test_fullres_unscaled_paths_agree(decoder, sub, h, w):
    """Full-resolution u8 output three ways agree byte for byte: the fused
    IDCT + converter (idct_rgb_kernel, default), IDCT then rgb_unscaled_kernel
    (output_path 2) and the generic sws_kernel (output_path 1)."""
    datas = [cases._enc(cases._noise(s, h, w), quality=90, subsampling=sub) for s in range(3)]
    fused = _decode(decoder, datas, Output(pix_fmt="rgb24"), (h, w, 3))
    outs = []
    for path in (2, 1):
        decoder.set_param("output_path", path)
        try:
            outs.append(_decode(decoder, datas, Output(pix_fmt="rgb24"), (h, w, 3)))
        finally:
            decoder.set_param("output_path", 0)
    assert torch.equal(fused, outs[0])
    assert torch.equal(fused, outs[1])


@pytest.mark.parametrize("name", cases.LARGE_PROGRESSIVE)
def test_fullres_large_progressive(decoder, oracle, name):
    """Large progressive images at full resolution: the multiscan decoder's
    lists through the fused IDCT + converter, bit-exact vs the oracle."""
    d = cases.case(name)
    info = oracle.parse(d)
    hyp = _decode(decoder, [d, d], Output(pix_fmt="rgb24"), (info.height, info.width, 3)).numpy()
    ref = oracle.decode_rgb(d, oracle.IDCT_SIMPLE, "rgb24")
    for i in range(2):
        np.testing.assert_array_equal(hyp[i], ref, strict=True)
