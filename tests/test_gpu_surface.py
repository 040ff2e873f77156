"""The spdl.io-level GPU surface: decode_image_nvjpeg / load_image_batch_nvjpeg.

Mirrors the reference's tests/cuda/nvjpeg_decode_test.py cases (pix_fmt
layouts, rgb/bgr channel swap, rubbish then recovery, resize to 160x120)
and checks every pixel against the oracle, where the reference can only
check shapes (nvJPEG/NPP are not byte-exact).  The nvjpeg surface stretches
with Lanczos-3 (the reference's resize_npp kernel) unless scale_algo says
otherwise.
"""

import numpy as np
import pytest
import torch

import spdl_amd.io as sio
from tests import cases

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cfg():
    return sio.cuda_config(device_index=0)


def _stretch(oracle, d, w, h, pix_fmt, algo):
    return oracle.decode_resize(d, oracle.Resize(fit_w=w, fit_h=h, filter=algo), pix_fmt=pix_fmt)


@pytest.mark.parametrize("pix_fmt", ["rgb", "bgr", "rgb24", "bgr24"])
def test_decode_pix_fmt(cfg, oracle, pix_fmt):
    d = cases.case("q90_422")  # 240x320, as the reference test image
    t = sio.to_torch(sio.decode_image_nvjpeg(d, device_config=cfg, pix_fmt=pix_fmt))
    assert t.dtype == torch.uint8 and t.device == torch.device("cuda", 0)
    assert t.shape == ((3, 240, 320) if pix_fmt in ("rgb", "bgr") else (240, 320, 3))
    ref = oracle.decode_rgb(d, oracle.IDCT_SIMPLE, pix_fmt)
    np.testing.assert_array_equal(t.cpu().numpy(), ref, strict=True)


def test_rgb_bgr_swap(cfg):
    d = cases.case("q90_420")
    rgb = sio.to_torch(sio.decode_image_nvjpeg(d, device_config=cfg, pix_fmt="rgb"))
    bgr = sio.to_torch(sio.decode_image_nvjpeg(d, device_config=cfg, pix_fmt="bgr"))
    assert torch.equal(rgb[0], bgr[2]) and torch.equal(rgb[1], bgr[1]) and torch.equal(rgb[2], bgr[0])
    assert not torch.equal(rgb[0], rgb[1])


def test_decode_rubbish_then_recover(cfg, oracle):
    rng = np.random.default_rng(0)
    for _ in range(3):
        with pytest.raises(RuntimeError):
            sio.decode_image_nvjpeg(rng.integers(0, 256, 1000, dtype=np.uint8).tobytes(),
                                    device_config=cfg)
    d = cases.case("q90_422")
    t = sio.to_torch(sio.decode_image_nvjpeg(d, device_config=cfg))
    np.testing.assert_array_equal(t.cpu().numpy(), oracle.decode_rgb(d, oracle.IDCT_SIMPLE, "rgb"))


@pytest.mark.parametrize("algo", ["lanczos", "bicubic", "bilinear"])
@pytest.mark.parametrize("pix_fmt", ["rgb", "rgb24"])
def test_decode_resize(cfg, oracle, algo, pix_fmt):
    d = cases.case("q90_422")
    kw = {} if algo == "lanczos" else {"scale_algo": algo}  # lanczos is the default
    t = sio.to_torch(sio.decode_image_nvjpeg(d, device_config=cfg, scale_width=160,
                                             scale_height=120, pix_fmt=pix_fmt, **kw))
    assert t.shape == ((3, 120, 160) if pix_fmt == "rgb" else (120, 160, 3))
    ref = _stretch(oracle, d, 160, 120, pix_fmt, algo)
    np.testing.assert_array_equal(t.cpu().numpy(), ref, strict=True)


def test_load_image_batch_nvjpeg_stretch(cfg, oracle):
    names = ["q90_420", "odd_227x333", "gray", "q90_444", "six_tables", "restart_blocks"]
    datas = [cases.case(n) for n in names]
    t = sio.to_torch(sio.load_image_batch_nvjpeg(datas, device_config=cfg, width=224,
                                                 height=224, pix_fmt="rgb"))
    assert t.shape == (len(names), 3, 224, 224)
    hyp = t.cpu().numpy()
    for i, d in enumerate(datas):
        np.testing.assert_array_equal(hyp[i], _stretch(oracle, d, 224, 224, "rgb", "lanczos"),
                                      strict=True)


def test_bad_scale_algo(cfg):
    with pytest.raises(ValueError):
        sio.decode_image_nvjpeg(cases.case("tiny_8x8"), device_config=cfg, scale_width=4,
                                scale_height=4, scale_algo="spline")
