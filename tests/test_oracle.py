"""CPU tests of the oracle (no GPU): pinned against the committed golden
fixtures (IJG libjpeg 9d outputs and the reference's own filter strings)."""

import glob
import json
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(__file__), "golden")
CASES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLD, "jpeg", "*.jpg")))


def _jpeg(name):
    with open(os.path.join(GOLD, "jpeg", name + ".jpg"), "rb") as f:
        return f.read()


def test_fixtures_present():
    assert len(CASES) >= 10


@pytest.mark.parametrize("name", CASES)
def test_entropy_decode_matches_libjpeg_coefficients(oracle, name):
    """Huffman decode + DC prediction, bit-exact vs jpeg_read_coefficients."""
    ref = np.load(os.path.join(GOLD, name + ".libjpeg.npz"))
    _, levels = oracle.decode_coefs(_jpeg(name))
    assert len(levels) == len([k for k in ref.files if k.startswith("coef")])
    for c, lv in enumerate(levels):
        np.testing.assert_array_equal(lv, ref[f"coef{c}"], strict=True)


@pytest.mark.parametrize("name", CASES)
def test_islow_pipeline_matches_libjpeg(oracle, name):
    """IDCT islow + nearest chroma + JFIF integer CSC: bit-exact vs libjpeg 9d
    (dct_method=JDCT_ISLOW, do_fancy_upsampling=FALSE)."""
    ref = np.load(os.path.join(GOLD, name + ".libjpeg.npz"))
    if "rgb_islow" not in ref.files:
        pytest.skip("libjpeg has no CMYK/YCCK -> RGB conversion, or reads the colour cues "
                    "differently from FFmpeg (coefficients pinned only)")
    ref = ref["rgb_islow"]
    hyp = oracle.decode_rgb(_jpeg(name), oracle.IDCT_ISLOW, "rgb24", csc="jfif")
    np.testing.assert_array_equal(hyp, ref, strict=True)


@pytest.mark.parametrize("name", CASES)
def test_oracle_regression(oracle, name):
    """Simple-IDCT (FFmpeg) planes / rgb / resize / fp16: pinned regression."""
    ref = np.load(os.path.join(GOLD, name + ".oracle.npz"))
    data = _jpeg(name)
    planes = oracle.decode_planes(data, oracle.IDCT_SIMPLE)
    for c, p in enumerate(planes):
        np.testing.assert_array_equal(p, ref[f"plane{c}"], strict=True)
    np.testing.assert_array_equal(oracle.decode_rgb(data, 0, "rgb24"), ref["rgb24_simple"])
    rs = oracle.Resize(fit_w=224, fit_h=224, aspect="decrease", pad_w=224, pad_h=224)
    np.testing.assert_array_equal(oracle.decode_resize(data, rs, "rgb24"), ref["pad224_rgb24"])
    f16 = oracle.decode_resize(data, rs, "rgb", normalize=True).view(np.uint16)
    np.testing.assert_array_equal(f16, ref["pad224_f16"])


def _fdct_matrix():
    return np.array([[(np.sqrt(1 / 8) if k == 0 else np.sqrt(2 / 8)) *
                      np.cos((2 * n + 1) * k * np.pi / 16) for n in range(8)] for k in range(8)])


@pytest.mark.parametrize("idct", [0, 1])
def test_idct_accuracy_ieee1180_style(oracle, idct):
    """Both integer IDCTs stay within 1 of the exact IDCT (IEEE 1180-style)."""
    C = _fdct_matrix()
    rng = np.random.default_rng(7)
    worst = 0
    for it in range(1500):
        L = 5 if it % 2 == 0 else int(rng.integers(1, 256))
        x = rng.integers(-L, L + 1, size=(8, 8)).astype(float)
        F = np.clip(np.rint(C @ x @ C.T).astype(int), -2048, 2047)
        ref = np.clip(np.rint(C.T @ F @ C) + 128, 0, 255)
        blk = F.copy()
        blk[0, 0] += 1024  # FFmpeg DC bias carried by the coefficients
        out = oracle.idct_block(blk.astype(np.int16).reshape(64), idct).astype(int)
        worst = max(worst, int(np.abs(out - ref).max()))
    assert worst <= 1


def _py_simple_idct(blk):
    """Independent pure-Python restatement of FFmpeg simple_idct 8-bit
    (simple_idct_template.c: idctRowCondDC + idctSparseColPut)."""
    W1, W2, W3, W4, W5, W6, W7 = 22725, 21407, 19266, 16383, 12873, 8867, 4520
    M = 0xFFFFFFFF

    def s32(x):
        x &= M
        return x - (1 << 32) if x & 0x80000000 else x

    def s16(x):
        x &= 0xFFFF
        return x - 0x10000 if x & 0x8000 else x

    b = [int(v) for v in blk]
    for i in range(8):
        r = b[8 * i: 8 * i + 8]
        if not any(r[1:]):
            b[8 * i: 8 * i + 8] = [s16(r[0] << 3)] * 8
            continue
        a0 = W4 * r[0] + (1 << 10)
        a1, a2, a3 = a0, a0, a0
        a0 += W2 * r[2]; a1 += W6 * r[2]; a2 -= W6 * r[2]; a3 -= W2 * r[2]
        b0 = W1 * r[1] + W3 * r[3]; b1 = W3 * r[1] - W7 * r[3]
        b2 = W5 * r[1] - W1 * r[3]; b3 = W7 * r[1] - W5 * r[3]
        a0 += W4 * r[4] + W6 * r[6]; a1 += -W4 * r[4] - W2 * r[6]
        a2 += -W4 * r[4] + W2 * r[6]; a3 += W4 * r[4] - W6 * r[6]
        b0 += W5 * r[5] + W7 * r[7]; b1 += -W1 * r[5] - W5 * r[7]
        b2 += W7 * r[5] + W3 * r[7]; b3 += W3 * r[5] - W1 * r[7]
        o = [a0 + b0, a1 + b1, a2 + b2, a3 + b3, a3 - b3, a2 - b2, a1 - b1, a0 - b0]
        b[8 * i: 8 * i + 8] = [s16(s32(v) >> 11) for v in o]
    out = np.zeros((8, 8), np.uint8)
    for i in range(8):
        c = [b[i + 8 * k] for k in range(8)]
        a0 = W4 * (c[0] + (1 << 19) // W4)
        a1, a2, a3 = a0, a0, a0
        a0 += W2 * c[2]; a1 += W6 * c[2]; a2 -= W6 * c[2]; a3 -= W2 * c[2]
        b0 = W1 * c[1] + W3 * c[3]; b1 = W3 * c[1] - W7 * c[3]
        b2 = W5 * c[1] - W1 * c[3]; b3 = W7 * c[1] - W5 * c[3]
        a0 += W4 * c[4]; a1 -= W4 * c[4]; a2 -= W4 * c[4]; a3 += W4 * c[4]
        b0 += W5 * c[5]; b1 -= W1 * c[5]; b2 += W7 * c[5]; b3 += W3 * c[5]
        a0 += W6 * c[6]; a1 -= W2 * c[6]; a2 += W2 * c[6]; a3 -= W6 * c[6]
        b0 += W7 * c[7]; b1 -= W5 * c[7]; b2 += W3 * c[7]; b3 -= W1 * c[7]
        o = [a0 + b0, a1 + b1, a2 + b2, a3 + b3, a3 - b3, a2 - b2, a1 - b1, a0 - b0]
        for r, v in enumerate(o):
            out[r, i] = min(max(s32(v) >> 20, 0), 255)
    return out


def test_simple_idct_matches_independent_restatement(oracle):
    """Two independent restatements of FFmpeg simple_idct agree bit for bit,
    including the DC-only row shortcut (row[0] << 3, which differs from the
    full row transform for large DC values)."""
    rng = np.random.default_rng(11)
    for it in range(400):
        blk = np.zeros(64, np.int16)
        blk[0] = 1024 + int(rng.integers(-1024, 1024))
        for _ in range(int(rng.integers(0, 20))):
            blk[int(rng.integers(0, 64))] = int(rng.integers(-400, 400))
        if it % 3 == 0:
            blk[1:8] = 0
            blk[0] = int(rng.integers(1500, 4000))
        np.testing.assert_array_equal(oracle.idct_block(blk, 0), _py_simple_idct(blk))


@pytest.mark.parametrize(
    "w,h,kw,expect",
    [
        (640, 480, dict(fit_w=224, fit_h=224, aspect="decrease", pad_w=224, pad_h=224),
         dict(sw=224, sh=168, dx=0, dy=28, ow=224, oh=224)),
        (480, 640, dict(fit_w=224, fit_h=224, aspect="decrease", pad_w=224, pad_h=224),
         dict(sw=168, sh=224, dx=28, dy=0, ow=224, oh=224)),
        (640, 480, dict(fit_w=224, fit_h=224, aspect="increase", crop_w=224, crop_h=224),
         dict(sw=299, sh=224, dx=-37, dy=0, ow=224, oh=224)),
        (640, 480, dict(fit_w=256, fit_h=256, aspect="decrease", pad_w=256, pad_h=256,
                        crop_w=224, crop_h=224),
         dict(sw=256, sh=192, dx=-16, dy=16, ow=224, oh=224)),
        (333, 227, dict(fit_w=224, fit_h=224, aspect="decrease", pad_w=224, pad_h=224),
         dict(sw=224, sh=153, dx=0, dy=35, ow=224, oh=224)),
        (640, 480, dict(fit_w=160, fit_h=120), dict(sw=160, sh=120, dx=0, dy=0, ow=160, oh=120)),
    ],
)
def test_geometry_ffmpeg_semantics(oracle, w, h, kw, expect):
    """scale force_original_aspect_ratio (av_rescale rounding) + centred pad /
    crop geometry, src/spdl/io/_preprocessing.py:214-234."""
    assert oracle.geometry(w, h, oracle.Resize(**kw)) == expect


def test_filter_desc_strings_match_reference():
    """Our filter-string builder reproduces the reference's
    get_video_filter_desc (fixture generated by importing the reference)."""
    from spdl_amd.io._preprocessing import get_video_filter_desc

    for item in json.load(open(os.path.join(GOLD, "filter_desc.json"))):
        assert get_video_filter_desc(**item["args"]) == item["desc"], item


def test_oracle_errors(oracle):
    from tests import cases

    with pytest.raises(oracle.OracleError):
        oracle.decode_rgb(cases.arithmetic())
    with pytest.raises(oracle.OracleError):
        oracle.decode_rgb(cases.twelve_bit())  # 12-bit precision
    with pytest.raises(oracle.OracleError):
        oracle.decode_rgb(cases.truncated())
    with pytest.raises(oracle.OracleError):
        oracle.decode_rgb(b"\x00" * 100)


def test_bf16_rounding_matches_torch(oracle):
    """jo_f32_to_bf16 == torch's fp32 -> bfloat16 cast (RNE) on the values the
    normalisation produces and on rounding ties / specials."""
    import ctypes

    import numpy as np
    import torch

    L = oracle.lib()
    L.jo_f32_to_bf16.argtypes = [ctypes.c_float]
    L.jo_f32_to_bf16.restype = ctypes.c_uint16
    mean = np.array([0.485, 0.456, 0.406], np.float32)
    std = np.array([0.229, 0.224, 0.225], np.float32)
    v = (np.arange(256, dtype=np.float32)[:, None] / np.float32(255.0) - mean) / std
    vals = np.concatenate([v.reshape(-1), np.array(
        [0.0, -0.0, 1.0 + 2 ** -8, 1.0 + 3 * 2 ** -8, 3.0e38, -3.4e38, 1e-40, np.inf, -np.inf],
        np.float32)])
    hyp = np.array([L.jo_f32_to_bf16(float(x)) for x in vals], np.uint16)
    ref = torch.from_numpy(vals).to(torch.bfloat16).view(torch.int16).numpy().view(np.uint16)
    np.testing.assert_array_equal(hyp, ref)


# ---- libswscale restatement (oracle/sws_oracle.c) ---------------------------


def _keys(x, a=-0.6):
    """Keys cubic: Mitchell-Netravali with B = 0, C = 0.6 (swscale's default
    SWS_BICUBIC parameters), in float64."""
    x = np.abs(np.asarray(x, np.float64))
    return np.where(x < 1, (a + 2) * x ** 3 - (a + 3) * x ** 2 + 1,
                    np.where(x < 2, a * x ** 3 - 5 * a * x ** 2 + 8 * a * x - 4 * a, 0.0))


@pytest.mark.parametrize("src,dst,align,one", [
    (640, 224, 4, 1 << 14), (480, 168, 2, 1 << 12), (320, 112, 4, 1 << 14), (240, 168, 2, 1 << 12),
    (1920, 224, 4, 1 << 14), (167, 333, 4, 1 << 14), (114, 227, 2, 1 << 12), (1, 224, 4, 1 << 14),
    (100, 100, 4, 1 << 14), (100, 100, 2, 1 << 12)])
@pytest.mark.parametrize("filt", ["bicubic", "bilinear", "lanczos"])
def test_sws_filter_invariants(oracle, src, dst, align, one, filt):
    """initFilter's output contract: every row sums to `one` (the
    error-diffusing normalisation), positions are non-decreasing and keep
    every non-zero tap inside the source, sizes are aligned (x86: 4
    horizontal, 2 vertical, unpadded when unscaled), unscaled is identity."""
    pos, coef = oracle.sws_axis(src, dst, filt, align, one)
    size = coef.shape[1]
    assert (coef.astype(np.int64).sum(axis=1) == one).all()
    assert (np.diff(pos) >= 0).all() and pos.min() >= 0
    for i in range(dst):
        nz = np.nonzero(coef[i])[0]
        assert pos[i] + nz.max() < max(src, 1)
    if src == dst:  # horizontal filters stay padded to 4 on x86
        assert size == (4 if align == 4 else 1)
        dense = np.zeros((dst, src), np.int64)
        for i in range(dst):
            dense[i, pos[i]:pos[i] + size] += coef[i]
        np.testing.assert_array_equal(dense, np.eye(dst, dtype=np.int64) * one)
    else:
        assert size % align == 0


@pytest.mark.parametrize("src,dst", [(640, 224), (480, 168), (320, 112), (1920, 224)])
def test_sws_bicubic_taps_follow_the_kernel(oracle, src, dst):
    """Interior rows of the fixed-point bicubic filter equal the float64
    Keys(-0.6) kernel, widened by the downscale factor and normalised, to
    within 2 LSB of 1<<14 (the int64 coefficient arithmetic and rounding
    residual are the only differences)."""
    pos, coef = oracle.sws_axis(src, dst, "bicubic")
    s = ((src << 16) + dst // 2) // dst / 65536.0
    for i in range(4, dst - 4):
        c = (i + 0.5) * s - 0.5
        idx = pos[i] + np.arange(coef.shape[1])
        w = _keys((idx - c) / s)
        ref = w / w.sum() * (1 << 14)
        assert np.abs(coef[i] - ref).max() <= 2.0, (i, coef[i], np.rint(ref))


def _float_swscale(planes, sw, sh):
    """Independent float64 model of the scale path swscale runs for a
    yuvj420p frame -> rgb24 (bicubic, centred chroma siting, half-width
    chroma shared by pixel pairs, BT.601 full-range matrix, round)."""
    Y, U, V = [p.astype(np.float64) for p in planes]
    H, W = Y.shape

    def res(p, n_out, axis, s, off=0.0):
        f = max(s, 1.0)
        out = []
        for i in range(n_out):
            c = (i + 0.5) * s - 0.5 + off
            idx = np.arange(int(np.floor(c - 2 * f)), int(np.ceil(c + 2 * f)) + 1)
            w = _keys((idx - c) / f)
            out.append(np.tensordot(w / w.sum(), np.take(p, np.clip(idx, 0, p.shape[axis] - 1),
                                                         axis=axis), axes=([0], [axis])))
        return np.stack(out, axis=axis)

    inc = lambda a, b: ((a << 16) + b // 2) // b / 65536.0  # noqa: E731
    Yr = res(res(Y, sw, 1, inc(W, sw)), sh, 0, inc(H, sh))
    cw, ch = U.shape[1], U.shape[0]

    def chroma(P):
        h = res(P, sw // 2, 1, inc(cw, sw // 2))
        # output row y (luma grid, centre 128) -> chroma rows (centre 128 at half res)
        s = inc(ch, sh)
        return np.repeat(res(h, sh, 0, s), 2, axis=1)

    Ur, Vr = chroma(U) - 128, chroma(V) - 128
    rgb = np.stack([Yr + 1.402 * Vr, Yr - 0.344136 * Ur - 0.714136 * Vr, Yr + 1.772 * Ur], -1)
    return np.clip(np.rint(rgb), 0, 255)


@pytest.mark.parametrize("name", ["q90_420", "odd_227x333"])
def test_sws_resize_matches_float_model(oracle, name):
    """The fixed-point restatement agrees with a float64 statement of the same
    algorithm to within 2 levels (fixed-point taps, 15-bit intermediates and
    the table CSC's truncations)."""
    from tests import cases

    d = cases.case(name)
    planes = oracle.decode_planes(d)
    info = oracle.parse(d)
    rs = oracle.Resize(fit_w=224, fit_h=224, aspect="decrease", pad_w=224, pad_h=224)
    g = oracle.geometry(info.width, info.height, rs)
    hyp = oracle.decode_resize(d, rs, "rgb24").astype(int)
    hyp = hyp[g["dy"]:g["dy"] + g["sh"], g["dx"]:g["dx"] + g["sw"]]
    ref = _float_swscale(planes, g["sw"], g["sh"])
    # the first chroma rows/cols see swscale's truncating window start
    diff = np.abs(hyp - ref)[4:-4, 4:-4]
    assert diff.max() <= 2 and diff.mean() < 0.8, (diff.max(), diff.mean())


def test_sws_unscaled_420_is_nearest_chroma_tables(oracle):
    """Same-size yuvj420p -> rgb24 (even size) is the unscaled converter:
    nearest chroma through the yuv2rgb tables, within 2 of the JFIF (IJG)
    conversion of the same planes and exactly R = G = B = Y for gray."""
    from tests import cases

    d = cases.case("q90_420")
    a = oracle.decode_rgb(d).astype(int)
    b = oracle.decode_rgb(d, csc="jfif").astype(int)
    assert np.abs(a - b).max() <= 2
    g = cases.case("gray")
    rgb = oracle.decode_rgb(g)
    (y,) = oracle.decode_planes(g)
    for ch in range(3):
        np.testing.assert_array_equal(rgb[..., ch], y)


def _edge_jpeg(subsampling=2, quality=95):
    """A 96x64 JPEG of three 32-px pure red / green / blue columns -- the
    reference's edge-value sample (ffmpeg lavfi color=0xff0000|0x00ff00|
    0x0000ff, hstack, tests/io/image_decoding_test.py:130-166), encoded by
    Pillow here (no ffmpeg CLI)."""
    import io as _io

    from PIL import Image

    px = np.zeros((64, 96, 3), np.uint8)
    px[:, :32, 0] = 255
    px[:, 32:64, 1] = 255
    px[:, 64:, 2] = 255
    b = _io.BytesIO()
    Image.fromarray(px).save(b, "JPEG", quality=quality, subsampling=subsampling)
    return b.getvalue()


def check_edge_values(hyp):
    """The reference's assertions (image_decoding_test.py:154-166)."""
    red, green, blue = hyp[:, :32], hyp[:, 32:64], hyp[:, 64:]
    assert np.all(red[..., 0] >= 254) and np.all(red[..., 1] <= 1) and np.all(red[..., 2] == 0)
    assert np.all(green[..., 0] == 0) and np.all(green[..., 1] >= 253)
    assert np.all(green[..., 2] <= 1)
    assert np.all(blue[..., 0] <= 1) and np.all(blue[..., 1] <= 1) and np.all(blue[..., 2] >= 254)


def test_edge_values_oracle(oracle):
    check_edge_values(oracle.decode_rgb(_edge_jpeg()))


def test_metadata_segments_do_not_change_pixels(oracle):
    """The FF-laden APP2 / COM test files decode to the pixels of the file
    they were made from (their segments are skipped by length)."""
    from tests import cases

    ref = oracle.decode_planes(cases.case("prog_420"), oracle.IDCT_SIMPLE)
    for name in cases.METADATA:
        hyp = oracle.decode_planes(cases.case(name), oracle.IDCT_SIMPLE)
        for a, b in zip(hyp, ref):
            np.testing.assert_array_equal(a, b)


def test_cmyk_ycck_decode(oracle):
    """4-component Adobe files (FFmpeg mjpeg, parity unpinned: libjpeg has no
    CMYK/YCCK -> RGB conversion to pin against): transform 0 is inverted
    CMYK -> RGB = C * K * 257 >> 16 per channel (restated here from the raw
    planes); transform 2 YCCK inverts Y, Cb, Cr against K first and then takes
    the YCbCr path.  Both decode the fixtures' source pixels to within JPEG
    error (the fixtures were made from cases.cmyk_pixels).  Without the
    marker the frame is YCbCr + K: same planes, no transform."""
    from spdl_amd.synthetic import synthetic_pixels
    from tests import cases

    for name in cases.FOUR_COMPONENT:
        data = cases.case(name)
        info = oracle.parse(data)
        assert info.ncomp == 4
        rgb = oracle.decode_rgb(data).astype(np.int64)
        if name == "cmyk_no_marker":
            assert (info.adobe, info.color) == (-1, 5)
            ref = cases.case("cmyk_adobe")
            for a, b in zip(oracle.decode_planes(data), oracle.decode_planes(ref)):
                np.testing.assert_array_equal(a, b)
            assert np.abs(rgb - oracle.decode_rgb(ref)).mean() > 30
            continue
        if info.adobe != 2:
            p = [x.astype(np.int64) for x in oracle.decode_planes(data)]
            exp = np.stack([(p[c] * p[3] * 257) >> 16 for c in range(3)], axis=-1)
            np.testing.assert_array_equal(rgb, exp)
        if name in cases.CMYK:
            seed, h, w = cases.CMYK[name][:3]
            assert info.adobe == (2 if cases.CMYK[name][4] else 0)
        else:
            seed, h, w = {"cmyk_pillow": (26, 64, 64), "cmyk_pillow_odd": (27, 75, 111),
                          "cmyk_pillow_prog": (26, 64, 64)}[name]
        src = synthetic_pixels(seed, h, w).astype(np.int64)
        assert np.abs(rgb - src).mean() < 6.0, name  # a wrong sign or bias is > 30


def test_rgb_coded_decode(oracle):
    """3-component RGB-coded files (FFmpeg gbrp: Adobe transform 0 or ids
    'R' 'G' 'B'): full-resolution rgb24 is the planes themselves, and it is
    the source pixels to within JPEG error."""
    from spdl_amd.synthetic import synthetic_pixels
    from tests import cases

    for name in [*cases.RGB_CODED, *cases.RGB_VARIANTS]:
        data = cases.case(name)
        assert oracle.parse(data).color == 2, name
        p = oracle.decode_planes(data)
        rgb = oracle.decode_rgb(data)
        np.testing.assert_array_equal(rgb, np.stack(p, axis=-1))
        seed, h, w = cases.RGB_CODED.get(name, cases.RGB_CODED["rgb_coded"])[:3]
        src = synthetic_pixels(seed, h, w).astype(np.int64)
        assert np.abs(rgb - src).mean() < 4.0, name
