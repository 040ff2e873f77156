"""GPU tests of the swscale-compatible output stage and of the surfaces the
round-1 review found untested (-m gpu, through the C-ABI).

  * the reference's edge-value assertions on a red / green / blue JPEG
    (tests/io/image_decoding_test.py:130-166), full resolution and through
    the 224 pad chain, with every pixel equal to the oracle;
  * load_image(filter_desc=None) plane layout (av_image_copy_to_buffer of
    conversion.cpp:172-303): [1, 1.5H, W] / [1, 2H, W] / [3, H, W] /
    [H, W, 1], compared with the oracle's planes concatenated Y, U, V;
  * the benchmarked entry point itself -- decode_batch_device with 1 or 2
    lanes, two batches in flight and warmup_slots 0 / 8 / 64 -- on
    256 x 480x640 q90 4:2:0 -> RGB224 pad, every image bit-exact vs oracle;
  * the JFIF colour-conversion option (pinned vs libjpeg via the oracle);
  * load_image_batch strict / non-strict failure handling
    (image_decoding_test.py:352-367).
"""

import numpy as np
import pytest
import torch

import spdl_amd.io as sio
from spdl_amd import _lib
from spdl_amd._lib import Output
from tests import cases
from tests.test_oracle import _edge_jpeg, check_edge_values

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cfg():
    return sio.cuda_config(device_index=0)


@pytest.mark.parametrize("subsampling", [2, 1, 0])
def test_edge_values(cfg, oracle, subsampling):
    d = _edge_jpeg(subsampling)
    hyp = sio.to_numpy(sio.load_image(d, device_config=None))
    assert hyp.shape == (64, 96, 3)
    np.testing.assert_array_equal(hyp, oracle.decode_rgb(d), strict=True)
    check_edge_values(hyp)


def test_edge_values_batch_resized(cfg, oracle):
    d = _edge_jpeg(2)
    hyp = sio.to_numpy(sio.load_image_batch([d, d], width=48, height=32))
    rs = oracle.Resize(fit_w=48, fit_h=32, aspect="decrease", pad_w=48, pad_h=32)
    ref = oracle.decode_resize(d, rs, "rgb24")
    for h in hyp:
        np.testing.assert_array_equal(h, ref, strict=True)


@pytest.mark.parametrize("name,shape_fn", [
    ("q90_420", lambda h, w: (1, h + h // 2, w)),
    ("q90_422", lambda h, w: (1, 2 * h, w)),
    ("q90_444", lambda h, w: (3, h, w)),
    ("gray", lambda h, w: (h, w, 1)),
])
def test_native_planes_layout(oracle, name, shape_fn):
    d = cases.case(name)
    hyp = sio.to_numpy(sio.load_image(d, filter_desc=None))
    planes = oracle.decode_planes(d)
    h, w = planes[0].shape
    assert hyp.shape == shape_fn(h, w)
    ref = np.concatenate([p.reshape(-1) for p in planes])
    np.testing.assert_array_equal(hyp.reshape(-1), ref, strict=True)


def test_native_planes_odd_420_fails_like_the_reference():
    with pytest.raises(RuntimeError, match="Failed to copy image data"):
        sio.load_image(cases.case("odd_227x333"), filter_desc=None)


def test_cmyk_through_the_io_surface(oracle):
    """load_image of Adobe CMYK / YCCK files: RGB through the default filter
    (FFmpeg's K transform, oracle-restated), and the unfiltered 4-plane frame
    refused as the reference's convert_frames refuses gbrap / yuva444p."""
    for name in ("cmyk_adobe", "ycck_odd_rst", "rgb_coded", "cmyk_no_marker"):
        d = cases.case(name)
        hyp = sio.to_numpy(sio.load_image(d))
        np.testing.assert_array_equal(hyp, oracle.decode_rgb(d), strict=True)
        with pytest.raises(RuntimeError, match="Unsupported pixel format"):
            sio.load_image(d, filter_desc=None)


def test_native_planes_batch(oracle):
    datas = [cases.case("q90_444"), cases.case("q90_444")]
    hyp = sio.to_numpy(sio.load_image_batch(datas, width=None, height=None, pix_fmt=None))
    assert hyp.shape == (2, 3, 240, 320)
    ref = np.stack(oracle.decode_planes(datas[0]))
    np.testing.assert_array_equal(hyp[1], ref, strict=True)


def test_batch_handle_failure(tmp_path):
    """strict=False drops a missing file, strict=True raises
    (reference image_decoding_test.py:352-367)."""
    paths = []
    for i in range(4):
        p = tmp_path / f"{i}.jpg"
        p.write_bytes(cases.case("q90_444"))
        paths.append(str(p))
    flist = [str(tmp_path / "NON_EXISTING_FILE.JPG"), *paths]
    buf = sio.load_image_batch(flist, width=None, height=None, pix_fmt=None, strict=False)
    assert sio.to_numpy(buf).shape == (4, 3, 240, 320)
    with pytest.raises(RuntimeError):
        sio.load_image_batch(flist, width=None, height=None, pix_fmt=None, strict=True)
    buf = sio.load_image_batch(flist, width=224, height=224, strict=False)
    assert sio.to_numpy(buf).shape == (4, 224, 224, 3)
    with pytest.raises(RuntimeError):
        sio.load_image_batch(flist, width=224, height=224, strict=True)


@pytest.mark.parametrize("name", cases.VALID)
def test_jfif_option_matches_oracle(decoder, oracle, name):
    d = cases.case(name)
    info = oracle.parse(d)
    t = torch.empty((info.height, info.width, 3), dtype=torch.uint8, device="cuda:0")
    if info.ncomp == 4:  # libjpeg's JFIF tables have no CMYK conversion
        with pytest.raises(oracle.OracleError):
            oracle.decode_rgb(d, 0, "rgb24", csc="jfif")
        with pytest.raises(RuntimeError, match="jfif"):
            decoder.decode_batch([d], Output(pix_fmt="rgb24", csc="jfif"), t.data_ptr(), t.numel())
        return
    decoder.decode_batch([d], Output(pix_fmt="rgb24", csc="jfif"), t.data_ptr(), t.numel())
    np.testing.assert_array_equal(t.cpu().numpy(), oracle.decode_rgb(d, 0, "rgb24", csc="jfif"))


def test_jfif_with_resize_is_rejected(decoder):
    t = torch.empty((224, 224, 3), dtype=torch.uint8, device="cuda:0")
    with pytest.raises(RuntimeError):
        decoder.decode_batch([cases.case("q90_420")],
                             Output(pix_fmt="rgb24", resize=True, fit_w=224, fit_h=224,
                                    csc="jfif"), t.data_ptr(), t.numel())


# ---- the benchmarked path ----------------------------------------------------

PAD224 = dict(fit_w=224, fit_h=224, aspect="decrease", pad_w=224, pad_h=224)


@pytest.fixture(scope="module")
def bench_batch(oracle):
    from spdl_amd.synthetic import synthetic_slice

    datas = synthetic_slice(range(256), distinct=32)
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
    refs = [oracle.decode_resize(d, oracle.Resize(**PAD224), "rgb24") for d in datas[:32]]
    return dev, np.asarray(offs, np.int64), np.asarray(sizes, np.int64), infos, refs


@pytest.mark.parametrize("lanes,inflight,warm,prio", [
    (1, 2, 0, 1), (1, 2, 8, 1), (1, 2, 64, 1), (2, 2, 0, 1), (2, 2, 8, 1), (2, 2, 64, 1),
    (4, 6, -1, 1),  # the driver's bench configuration: 4 lanes, lanes + 2 in flight
    (4, 6, -1, 0), (4, 6, -1, -1),  # lanes at normal / high stream priority
])
def test_bench_path_bit_exact(bench_batch, lanes, inflight, warm, prio):
    """decode_batch_device exactly as bench.py drives it: async submissions,
    `inflight` batches in flight on `lanes` pipelines, then every image of
    every batch against the oracle."""
    dev, offs, sizes, infos, refs = bench_batch
    dec = _lib.Decoder(0)
    dec.set_param("lanes", lanes)
    assert dec.get_param("lanes") == lanes  # <= 4: HIP's default queues per priority pool
    dec.set_param("lane_priority", prio)
    assert dec.get_param("lane_priority") == prio
    if warm >= 0:
        dec.set_param("warmup_slots", warm)
    spec = Output(pix_fmt="rgb24", resize=True, **PAD224)
    nbatch = inflight + 2
    outs = [torch.full((256, 224, 224, 3), 7, dtype=torch.uint8, device="cuda:0")
            for _ in range(nbatch)]
    stream = torch.cuda.current_stream()
    tickets = []
    for k in range(nbatch):
        o = outs[k]
        dec.decode_batch_device(dev.data_ptr(), dev.numel(), offs, sizes, infos, spec,
                                o.data_ptr(), o.numel(), stream=stream, sync=False)
        tickets.append(dec.last_ticket())
        if len(tickets) > inflight - 1:
            assert not any(dec.wait(tickets.pop(0), 256))
    for t in tickets:
        assert not any(dec.wait(t, 256))
    torch.cuda.synchronize()
    for o in outs:
        hyp = o.cpu().numpy()
        for i in range(256):
            np.testing.assert_array_equal(hyp[i], refs[i % 32], strict=True)
    dec.close()


def test_decode_outputs_use_the_allocator_hook(oracle):
    """cuda_config(allocator=...) serves the decode outputs too (reference
    cuda/storage.cpp:71-100): called once per batch, freed with the buffer."""
    import gc

    calls = {"alloc": 0, "free": 0}

    def alloc(size, device, stream):
        calls["alloc"] += 1
        return torch.cuda.caching_allocator_alloc(size, device, stream)

    def free(ptr):
        calls["free"] += 1
        torch.cuda.caching_allocator_delete(ptr)

    def run():
        cfg = sio.cuda_config(0, allocator=(alloc, free))
        d = cases.case("q90_420")
        buf = sio.load_image_batch([d, d], width=64, height=48, device_config=cfg)
        assert calls == {"alloc": 1, "free": 0}
        hyp = sio.to_torch(buf).cpu().numpy()
        ref = oracle.decode_resize(d, oracle.Resize(fit_w=64, fit_h=48, aspect="decrease",
                                                    pad_w=64, pad_h=48), "rgb24")
        for h in hyp:
            np.testing.assert_array_equal(h, ref, strict=True)
        buf2 = sio.decode_image_nvjpeg(d, device_config=cfg)
        assert calls["alloc"] == 2
        del buf, buf2

    run()
    gc.collect()
    assert calls["free"] == 2


def test_nvjpeg_batch_scale_size_errors(cfg):
    d = cases.case("q90_420")
    with pytest.raises(RuntimeError, match="Both"):
        sio.decode_image_nvjpeg([d], device_config=cfg)
    with pytest.raises(RuntimeError):
        sio.decode_image_nvjpeg([d], device_config=cfg, scale_width=32)
