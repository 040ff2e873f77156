"""Host-side tests (no GPU compute): the C-ABI library loads and exports every
symbol include/spdl_hipjpeg.h declares; the host probe and output geometry
agree with the oracle; the spdl.io-compatible surface validates its
arguments like the reference."""

import ctypes
import glob
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


def _declared_symbols():
    hdr = open(os.path.join(ROOT, "include", "spdl_hipjpeg.h")).read()
    return sorted(set(re.findall(r"\b(spdl_hj_[a-z0-9_]+)\s*\(", hdr)))


def test_library_exports_every_declared_symbol():
    from spdl_amd import _lib

    L = _lib.lib()
    declared = _declared_symbols()
    assert len(declared) >= 12
    for sym in declared:
        assert hasattr(L, sym), f"missing export {sym}"
    assert set(declared) == set(_lib.EXPORTED)
    assert L.spdl_hj_abi_version() == _lib.ABI_VERSION


def test_library_is_built_for_gfx950():
    path = os.path.join(ROOT, "spdl_amd", "lib", "libspdl_hipjpeg.so")
    blob = open(path, "rb").read()
    assert b"gfx950" in blob


def _jpegs():
    out = {}
    for p in sorted(glob.glob(os.path.join(GOLD, "jpeg", "*.jpg"))):
        out[os.path.basename(p)[:-4]] = open(p, "rb").read()
    return out


def test_host_probe_matches_oracle(oracle):
    from spdl_amd import _lib

    for name, data in _jpegs().items():
        info = _lib.get_image_info(data)
        ref = oracle.parse(data)
        assert (info.width, info.height, info.ncomp) == (ref.width, ref.height, ref.ncomp), name
        for c in range(ref.ncomp):
            assert (info.h_samp[c], info.v_samp[c]) == (ref.comp_h[c], ref.comp_v[c])
        assert info.color == ref.color, name  # the frame's colour model


def test_host_probe_rejects_garbage():
    from spdl_amd import _lib
    from tests import cases

    with pytest.raises(RuntimeError, match="Failed to decode"):
        _lib.get_image_info(b"\x00" * 64)
    with pytest.raises(RuntimeError, match="Failed to decode"):
        _lib.get_image_info(cases.arithmetic())  # unsupported SOF9
    with pytest.raises(RuntimeError, match="Failed to decode"):
        _lib.get_image_info(cases.twelve_bit())  # unsupported 12-bit precision
    # 4 components, progressive or one component per scan: the probe takes them
    # (the scans are walked on the device)
    for name in ("prog_cmyk", "multiscan_cmyk", "cmyk_pillow_prog"):
        assert _lib.get_image_info(cases.case(name)).ncomp == 4


@pytest.mark.parametrize("w,h", [(640, 480), (480, 640), (333, 227), (1, 1), (1920, 1080)])
@pytest.mark.parametrize("kind", ["pad", "crop", "stretch", "imagenet", "none"])
def test_output_geometry_matches_oracle(oracle, w, h, kind):
    from spdl_amd._lib import Output, output_size

    kw = {
        "pad": dict(fit_w=224, fit_h=224, aspect="decrease", pad_w=224, pad_h=224),
        "crop": dict(fit_w=224, fit_h=224, aspect="increase", crop_w=224, crop_h=224),
        "stretch": dict(fit_w=160, fit_h=120),
        "imagenet": dict(fit_w=256, fit_h=256, aspect="decrease", pad_w=256, pad_h=256,
                         crop_w=224, crop_h=224),
        "none": dict(),
    }[kind]
    g = oracle.geometry(w, h, oracle.Resize(**kw))
    ow, oh = output_size(w, h, Output(resize=bool(kw), **kw))
    assert (ow, oh) == (g["ow"], g["oh"])


def test_decoder_without_gpu_fails_loudly():
    import torch

    from spdl_amd._lib import Decoder

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(RuntimeError, match="no HIP device|cannot create decoder"):
        Decoder(0)


def test_api_argument_validation():
    import spdl_amd.io as io

    data = next(iter(_jpegs().values()))
    with pytest.raises(ValueError, match="device_config must be provided"):
        io.decode_image_nvjpeg(data)
    cfg = io.cuda_config(device_index=0)
    with pytest.raises(RuntimeError, match="Both `scale_width` and `scale_height`"):
        io.decode_image_nvjpeg([data, data], device_config=cfg)
    with pytest.raises(RuntimeError, match="Unexpected pix_fmt"):
        io.decode_image_nvjpeg(data, device_config=cfg, pix_fmt="yuv420p")
    with pytest.raises(ValueError, match="must not be empty"):
        io.load_image_batch([], width=224, height=224)
    with pytest.raises(TypeError):
        io.cuda_config(0, allocator=(1, 2))


def test_cuda_config_defaults():
    import spdl_amd.io as io

    cfg = io.cuda_config(device_index=3)
    assert cfg.device_index == 3 and cfg.stream == 0x2 and cfg.allocator is None


def test_filter_desc_parsing():
    from spdl_amd.io import get_video_filter_desc, parse_image_filter

    out = parse_image_filter(get_video_filter_desc(scale_width=224, scale_height=224))
    assert (out.resize, out.fit_w, out.fit_h, out.aspect, out.pad_w, out.pad_h, out.pix_fmt) == (
        True, 224, 224, "decrease", 224, 224, "rgb24")
    out = parse_image_filter(get_video_filter_desc(scale_width=256, scale_height=256,
                                                   scale_mode="crop", pix_fmt="bgr24"))
    assert (out.aspect, out.crop_w, out.crop_h, out.pix_fmt) == ("increase", 256, 256, "bgr24")
    out = parse_image_filter(
        "scale=w=256:h=256:flags=bicubic:force_original_aspect_ratio=decrease,"
        "pad=w=256:h=256:x=-1:y=-1:color=black,crop=w=224:h=224,format=pix_fmts=rgb24")
    assert (out.pad_w, out.crop_w) == (256, 224)
    assert parse_image_filter(None).resize is False
    with pytest.raises(ValueError):
        parse_image_filter("hflip")
    with pytest.raises(ValueError):
        parse_image_filter("scale=w=224:h=224:flags=spline")
    assert parse_image_filter("scale=w=224:h=224:flags=lanczos").filter == "lanczos"


def test_output_spec_rejects_bad_pix_fmt():
    from spdl_amd._lib import Output

    with pytest.raises(RuntimeError, match="Unexpected pix_fmt"):
        Output(pix_fmt="gray").to_c()


def test_product_never_imports_oracle():
    """The product package must not reach the oracle (a CPU fallback would
    void every parity claim)."""
    for p in glob.glob(os.path.join(ROOT, "spdl_amd", "**", "*.py"), recursive=True):
        src = open(p).read()
        assert "from oracle" not in src and "import oracle" not in src, p
    for p in glob.glob(os.path.join(ROOT, "spdl_amd", "csrc", "*")):
        src = open(p, errors="ignore").read()
        code = re.sub(r"//[^\n]*|/\*.*?\*/", "", src, flags=re.S)  # comments may cite it
        assert "jpeg_oracle" not in code and not re.search(r"\bjo_[a-z_]+\(", code), p


def test_fast_bilinear_is_refused_not_aliased():
    """swscale's SWS_FAST_BILINEAR is a different scaler: refusing it beats
    returning bilinear pixels under its name."""
    from spdl_amd.io import parse_image_filter

    with pytest.raises(ValueError, match="fast_bilinear"):
        parse_image_filter("scale=w=224:h=224:flags=fast_bilinear")
    assert parse_image_filter("scale=w=224:h=224:flags=bilinear").filter == "bilinear"


def test_default_device_follows_local_rank(monkeypatch):
    """Without device_config the decode device is the current HIP device or
    $LOCAL_RANK -- never a hard-wired 0 for every rank of a job."""
    import torch

    from spdl_amd.io import _image

    monkeypatch.setattr(torch.cuda, "is_initialized", lambda: False)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
    monkeypatch.setenv("LOCAL_RANK", "5")
    assert _image._default_config().device_index == 5
    monkeypatch.setenv("LOCAL_RANK", "9")  # out of range: device 0
    assert _image._default_config().device_index == 0
    monkeypatch.delenv("LOCAL_RANK")
    assert _image._default_config().device_index == 0
    monkeypatch.setattr(torch.cuda, "is_initialized", lambda: True)
    monkeypatch.setattr(torch.cuda, "current_device", lambda: 3)
    monkeypatch.setenv("LOCAL_RANK", "5")
    assert _image._default_config().device_index == 3


def test_ffmpeg_configs_are_reported_not_silently_dropped():
    from spdl_amd.io import _image

    _image._IGNORED_WARNED.clear()
    kw = {"decode_config": object(), "demux_config": None}
    with pytest.warns(RuntimeWarning, match="decode_config"):
        _image._ignore_ffmpeg_configs(kw)
    assert kw == {}


def test_storage_too_small_raises_like_reference():
    """load_image_batch(storage=...) writes the host result into the caller's
    storage; a short one raises the reference's capacity error
    (src/libspdl/core/buffer.cpp:56-62)."""
    import torch

    from spdl_amd.io import _image, cpu_storage
    from spdl_amd.io._buffer import CUDABuffer

    buf = CUDABuffer(None, ptr=1, shape=(2, 224, 224, 3), dtype=torch.uint8)
    with pytest.raises(RuntimeError, match="does not have enough capacity"):
        _image._to_host(buf, cpu_storage(100, pin_memory=False))


def test_release_build_rejects_debug_mask():
    """Timing-ablation knobs that break outputs exist only in HJ_ABLATIONS
    builds; the shipped library refuses them (no context needed to check:
    the name is rejected before the context is touched, so a NULL context
    still returns INVALID_ARG for every name)."""
    from spdl_amd import _lib

    L = _lib.lib()
    v = ctypes.c_int64()
    assert L.spdl_hj_set_param(None, b"debug_mask", 1) == 8
    assert L.spdl_hj_get_param(None, b"lanes", ctypes.byref(v)) == 8
    src = open(os.path.join(ROOT, "spdl_amd", "csrc", "hj_host.cpp")).read()
    i = src.index('"debug_mask"')
    assert "#if HJ_ABLATIONS" in src[src.rindex("\n#", 0, i) - 40: i]


def test_every_knob_is_documented_in_the_header():
    """Every name spdl_hj_set_param accepts (release builds) and every name
    spdl_hj_get_param reports is documented in include/spdl_hipjpeg.h's knob
    text, and the header documents no knob the library does not take."""
    src = open(os.path.join(ROOT, "spdl_amd", "csrc", "hj_host.cpp")).read()
    s0 = src.index("int spdl_hj_set_param(")
    s1 = src.index("int spdl_hj_get_param(")
    setter = src[s0:s1]
    # (release builds: the HJ_ABLATIONS-only names are not part of the ABI)
    setter = re.sub(r"#if HJ_ABLATIONS.*?#endif", "", setter, flags=re.S)
    set_names = set(re.findall(r'strcmp\(name, "([a-z0-9_]+)"\)', setter))
    getter = src[s1:src.index("\n}\n", s1)]
    get_names = set(re.findall(r'\{"([a-z0-9_]+)",', getter))
    hdr = open(os.path.join(ROOT, "include", "spdl_hipjpeg.h")).read()
    h0 = hdr.index("/* Tuning knobs:")
    doc = hdr[h0:hdr.index("int spdl_hj_get_param(", h0)]
    doc_names = set(re.findall(r'"([a-z][a-z0-9_]*)"', doc))
    assert set_names, "no knob names found in spdl_hj_set_param"
    assert not set_names - doc_names, f"undocumented knobs: {sorted(set_names - doc_names)}"
    assert not get_names - doc_names, f"undocumented values: {sorted(get_names - doc_names)}"
    extra = doc_names - set_names - get_names - {"debug_mask"}
    assert not extra, f"documented but not taken: {sorted(extra)}"
