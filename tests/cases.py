"""Deterministic JPEG test inputs (generated with Pillow from seeded pixels).

Covers the edge cases the reference tests exercise (tests/io/image_decoding_test.py:
yuvj420p / 422 / 444 / gray, odd sizes) plus restart intervals, quality extremes,
noise (long codes, many 0xFF00 stuffings) and a tiny image.
"""

from __future__ import annotations

import functools
import io
import os

import numpy as np
from PIL import Image

from spdl_amd.synthetic import synthetic_pixels


def _enc(px, **kw) -> bytes:
    b = io.BytesIO()
    mode = "L" if px.ndim == 2 else "RGB"
    Image.fromarray(px, mode).save(b, "JPEG", **kw)
    return b.getvalue()


def _noise(seed, h, w, c=3):
    rng = np.random.default_rng(seed)
    shape = (h, w) if c == 1 else (h, w, c)
    return rng.integers(0, 256, size=shape, dtype=np.uint8)


@functools.lru_cache(maxsize=None)
def case(name: str) -> bytes:
    if name.startswith("bench_"):  # bench.py's synthetic images (seed 1000 + i)
        from spdl_amd.synthetic import synthetic_jpeg

        return synthetic_jpeg(int(name[6:]))
    if name == "q90_420":
        return _enc(synthetic_pixels(1), quality=90, subsampling=2)
    if name == "q75_420":
        return _enc(synthetic_pixels(2), quality=75, subsampling=2)
    if name == "q95_420":
        return _enc(synthetic_pixels(3), quality=95, subsampling=2)
    if name == "q90_444":
        return _enc(synthetic_pixels(4, 240, 320), quality=90, subsampling=0)
    if name == "q90_422":
        return _enc(synthetic_pixels(5, 240, 320), quality=90, subsampling=1)
    if name == "odd_227x333":
        return _enc(synthetic_pixels(6, 227, 333), quality=90, subsampling=2)
    if name == "odd_444_101x67":
        return _enc(synthetic_pixels(7, 101, 67), quality=85, subsampling=0)
    if name == "gray":
        return _enc(synthetic_pixels(8, 200, 300)[..., 0], quality=90)
    if name == "gray_odd":
        return _enc(synthetic_pixels(9, 77, 131)[..., 1], quality=80)
    if name == "noise_420":
        return _enc(_noise(10, 240, 320), quality=90, subsampling=2)
    if name == "noise_q100":
        return _enc(_noise(11, 120, 160), quality=100, subsampling=0)
    if name == "restart_rows":
        return _enc(synthetic_pixels(12, 240, 320), quality=90, restart_marker_rows=1)
    if name == "restart_blocks":
        return _enc(synthetic_pixels(13, 227, 333), quality=90, restart_marker_blocks=7)
    if name == "restart_every_mcu":
        return _enc(synthetic_pixels(14, 64, 96), quality=90, restart_marker_blocks=1)
    if name == "tiny_8x8":
        return _enc(synthetic_pixels(15, 8, 8), quality=90)
    if name == "tiny_1x1":
        return _enc(synthetic_pixels(16, 1, 1), quality=90)
    if name == "optimized":
        return _enc(synthetic_pixels(17, 240, 320), quality=90, optimize=True)
    if name == "six_tables":
        return six_tables(case("q90_444"))
    if name == "large_1080p":
        return _enc(synthetic_pixels(18, 1080, 1920), quality=90, subsampling=2)
    # progressive (SOF2): DC first/refine + spectral-selection and
    # successive-approximation AC scans (libjpeg's default script via Pillow)
    if name == "prog_420":
        return _enc(synthetic_pixels(19, 240, 320), quality=90, subsampling=2, progressive=True)
    if name == "prog_444_odd":
        return _enc(synthetic_pixels(20, 101, 67), quality=85, subsampling=0, progressive=True)
    if name == "prog_422":
        return _enc(synthetic_pixels(21, 120, 200), quality=92, subsampling=1, progressive=True)
    if name == "prog_gray":
        return _enc(synthetic_pixels(22, 77, 131)[..., 0], quality=80, progressive=True)
    if name == "prog_optimized":  # per-scan Huffman tables (a DHT before every scan)
        return _enc(synthetic_pixels(23, 240, 320), quality=90, progressive=True, optimize=True)
    if name == "prog_restart":
        return _enc(synthetic_pixels(24, 227, 333), quality=90, progressive=True,
                    restart_marker_blocks=5)
    if name == "prog_noise_q100":
        return _enc(_noise(25, 96, 128), quality=100, subsampling=0, progressive=True)
    # large progressive images: scans past the decoder's 16 KiB LDS byte window
    # (restaged mid-scan), many refinement chunks, restarts across restages
    if name == "prog_large_420":
        return _enc(synthetic_pixels(26, 480, 640), quality=90, subsampling=2, progressive=True)
    if name == "prog_large_noise":
        return _enc(_noise(27, 320, 480), quality=95, subsampling=2, progressive=True)
    if name == "prog_large_restart":
        return _enc(synthetic_pixels(28, 480, 640), quality=92, progressive=True,
                    restart_marker_blocks=3)
    if name == "prog_1080p":
        return _enc(synthetic_pixels(29, 1080, 1920), quality=90, subsampling=2,
                    progressive=True)
    # progressive files with binary metadata full of 0xFF xx pairs: an APP2
    # blob before the frame (an ICC profile / thumbnail stand-in) and a COM
    # segment between two scans (more marker candidates than the decoder's
    # list holds: each scan's end is then found by a forward search)
    if name == "prog_app2_blob":
        return _with_segment(case("prog_420"), 0xE2, _ff_blob(40, 30000), before_sos=0)
    if name == "prog_com_between_scans":
        return _with_segment(case("prog_420"), 0xFE, _ff_blob(41, 3000), before_sos=1)
    # Adobe 4-component files written by Pillow (inverted CMYK, transform 0)
    if name == "cmyk_pillow":
        return _cmyk_pillow(synthetic_pixels(26, 64, 64))
    if name == "cmyk_pillow_odd":
        return _cmyk_pillow(synthetic_pixels(27, 75, 111), quality=80)
    # sequential, one non-interleaved scan per component (reverse order);
    # Pillow cannot write these: libjpeg 9 wrote the committed files
    # (tests/gen_golden.py, oracle.lj_encode_multiscan)
    # one colour cue removed: the APP14 marker (ids 'R' 'G' 'B' left; a CMYK
    # file without it is YCbCr + K), or the ids (renumbered 1 2 3)
    if name == "rgb_ids_only":
        return _strip_app14(case("rgb_coded"))
    if name == "cmyk_pillow_prog":  # Pillow's progressive CMYK (libjpeg-turbo script)
        return _cmyk_pillow(synthetic_pixels(26, 64, 64), progressive=True)
    if name == "cmyk_no_marker":
        return _strip_app14(case("cmyk_adobe"))
    if name == "rgb_adobe_only":
        return _renumber_ids(case("rgb_coded"))
    if name in MULTISCAN or name in CMYK or name in RGB_CODED:
        with open(os.path.join(GOLD_JPEG, name + ".jpg"), "rb") as f:
            return f.read()
    raise KeyError(name)


GOLD_JPEG = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "jpeg")
# name -> (pixels seed, h, w, quality, h0, v0, restart blocks)
MULTISCAN = {
    "multiscan_420": (30, 240, 320, 90, 2, 2, 0),
    "multiscan_444_odd": (31, 101, 67, 85, 1, 1, 0),
    "multiscan_422_rst": (32, 120, 200, 90, 2, 1, 7),
}
# Adobe CMYK (transform 0) / YCCK (transform 2), libjpeg 9 from inverted CMYK
# pixels (tests/gen_golden.py, cmyk_pixels + oracle.lj_encode_cmyk):
# name -> (pixels seed, h, w, quality, ycck, restart blocks[, scan script])
CMYK = {
    "cmyk_adobe": (33, 120, 160, 90, False, 0),
    "ycck_adobe": (34, 120, 160, 90, True, 0),
    "ycck_odd_rst": (35, 77, 131, 85, True, 5),
    # progressive (libjpeg's jpeg_simple_progression for 4 components: DC
    # first, AC 1-5 / 6-63 first, AC refine, DC refine, AC refine per
    # component) and one component per sequential scan
    "prog_cmyk": (38, 120, 160, 90, False, 0, "progressive"),
    "prog_ycck_odd_rst": (39, 77, 131, 85, True, 5, "progressive"),
    "multiscan_cmyk": (40, 96, 128, 90, False, 0, "multiscan"),
}
FOUR_COMPONENT = [*CMYK, "cmyk_pillow", "cmyk_pillow_odd", "cmyk_no_marker", "cmyk_pillow_prog"]
# 3 components coded in RGB (FFmpeg's gbrp frames): libjpeg 9 JCS_RGB writes
# ids 'R' 'G' 'B' and an Adobe transform-0 marker; the variants keep one cue
# each. name -> (pixels seed, h, w, quality, restart blocks)
RGB_CODED = {"rgb_coded": (36, 100, 150, 90, 0), "rgb_coded_odd_rst": (37, 77, 131, 85, 4)}
RGB_VARIANTS = ["rgb_ids_only", "rgb_adobe_only"]
LARGE_PROGRESSIVE = ["prog_large_420", "prog_large_noise", "prog_large_restart", "prog_1080p"]
PROGRESSIVE = ["prog_420", "prog_444_odd", "prog_422", "prog_gray", "prog_optimized",
               "prog_restart", "prog_noise_q100"]
METADATA = ["prog_app2_blob", "prog_com_between_scans"]


VALID = [
    "q90_420", "q75_420", "q95_420", "q90_444", "q90_422", "odd_227x333", "odd_444_101x67",
    "gray", "gray_odd", "noise_420", "noise_q100", "restart_rows", "restart_blocks",
    "restart_every_mcu", "tiny_8x8", "tiny_1x1", "optimized", "six_tables", "large_1080p",
    *PROGRESSIVE, *MULTISCAN, *FOUR_COMPONENT, *RGB_CODED, *RGB_VARIANTS,
]


def six_tables(data: bytes) -> bytes:
    """A 3-component JPEG re-labelled to use six distinct Huffman tables.

    The chroma DC/AC tables (ids 1) are copied to ids 2 by an extra DHT
    segment and the third component's SOS selectors point at them, so the
    pixels are those of ``data`` while the scan holds DC0-2 + AC0-2: the
    decoder's wide-table path (more tables than the common LDS layout).
    """
    d = bytearray(data)
    tabs, pos, sos = {}, 2, None
    while pos < len(d):
        assert d[pos] == 0xFF
        m, ln = d[pos + 1], (d[pos + 2] << 8) | d[pos + 3]
        if m == 0xC4:  # DHT: one or more (class/id, 16 counts, values)
            q = pos + 4
            while q < pos + 2 + ln:
                n = sum(d[q + 1:q + 17])
                tabs[d[q]] = bytes(d[q:q + 17 + n])
                q += 17 + n
        if m == 0xDA:
            sos = pos
            break
        pos += 2 + ln
    assert sos is not None and d[sos + 4] == 3, "needs a 3-component scan"
    seg = bytes([0x02]) + tabs[0x01][1:] + bytes([0x12]) + tabs[0x11][1:]
    dht = b"\xff\xc4" + (len(seg) + 2).to_bytes(2, "big") + seg
    assert d[sos + 10] == 0x11  # third component: DC1 / AC1
    d[sos + 10] = 0x22
    return bytes(d[:sos]) + dht + bytes(d[sos:])


def progressive() -> bytes:
    return _enc(synthetic_pixels(20, 64, 64), quality=90, progressive=True)


def arithmetic() -> bytes:
    """A baseline file re-labelled SOF9 (arithmetic coding): unsupported."""
    d = bytearray(case("q90_420"))
    i = d.index(b"\xff\xc0")
    d[i + 1] = 0xC9
    return bytes(d)


def _cmyk_pillow(px, quality=90, **kw) -> bytes:
    b = io.BytesIO()
    Image.fromarray(px).convert("CMYK").save(b, "JPEG", quality=quality, **kw)
    return b.getvalue()


def _strip_app14(data: bytes) -> bytes:
    i = data.index(b"\xff\xee")
    n = int.from_bytes(data[i + 2 : i + 4], "big")
    return data[:i] + data[i + 2 + n :]


def _renumber_ids(data: bytes) -> bytes:
    """Component ids 'R' 'G' 'B' -> 1 2 3 in the SOF and the SOS."""
    d = bytearray(data)
    sof, sos = d.index(b"\xff\xc0"), d.index(b"\xff\xda")
    for c in range(3):
        assert d[sof + 10 + 3 * c] == b"RGB"[c] and d[sos + 5 + 2 * c] == b"RGB"[c]
        d[sof + 10 + 3 * c] = d[sos + 5 + 2 * c] = c + 1
    return bytes(d)


def cmyk_pixels(seed: int, h: int, w: int) -> np.ndarray:
    """HxWx4 Adobe-inverted CMYK whose product decode is ~ synthetic_pixels:
    K = max(R, G, B), C = R * 255 / K (and M, Y likewise), so R ~ C * K / 255."""
    px = synthetic_pixels(seed, h, w).astype(np.int32)
    k = px.max(axis=2, keepdims=True)
    cmy = np.where(k > 0, (px * 255 + k // 2) // np.maximum(k, 1), 255)
    return np.concatenate([cmy, k], axis=2).astype(np.uint8)


def twelve_bit() -> bytes:
    """A baseline file re-labelled 12-bit extended sequential (SOF1, P = 12):
    unsupported (FFmpeg decodes it to a 16-bit pix_fmt)."""
    d = bytearray(case("q90_420"))
    i = d.index(b"\xff\xc0")
    d[i + 1] = 0xC1
    d[i + 4] = 12
    return bytes(d)


def truncated() -> bytes:
    d = case("q90_420")
    return d[: len(d) // 2]


def corrupt_scan(seed: int = 0) -> bytes:
    d = bytearray(case("q75_420"))
    start = d.index(b"\xff\xda") + 20
    rng = np.random.default_rng(seed)
    pos = rng.integers(start, len(d) - 100, size=40)
    for p in pos:
        d[p] = int(rng.integers(0, 255))
    return bytes(d)


def corrupt_progressive(seed: int = 0) -> bytes:
    """A progressive image with 1-4 random bytes overwritten past its first scan
    header (scan data, later DHT/SOS segments; no new 0xFF bytes)."""
    d = bytearray(case("prog_420"))
    start = d.index(b"\xff\xda") + 16
    rng = np.random.default_rng(100 + seed)
    for p in rng.integers(start, len(d) - 8, size=1 + seed % 4):
        d[p] = int(rng.integers(0, 255))
    return bytes(d)


def truncated_progressive(frac: float = 0.5) -> bytes:
    d = case("prog_420")
    return d[: int(len(d) * frac)]



def _ff_blob(seed: int, n: int) -> bytes:
    """n bytes of segment payload, every other one 0xFF followed by a byte that
    would read as a marker (SOFn, DHT, SOS, EOI ...) outside a segment."""
    rng = np.random.default_rng(seed)
    nx = rng.choice(np.array([0xC0, 0xC2, 0xC4, 0xD9, 0xDA, 0xDB, 0xE1], np.uint8), size=n // 2)
    out = np.empty(2 * (n // 2), np.uint8)
    out[0::2] = 0xFF
    out[1::2] = nx
    return out.tobytes()


def _with_segment(data: bytes, marker: int, payload: bytes, before_sos: int) -> bytes:
    """`data` with one marker segment inserted: right after SOI
    (before_sos=0) or just before the before_sos-th SOS marker (1 = second)."""
    seg = bytes([0xFF, marker]) + (len(payload) + 2).to_bytes(2, "big") + payload
    if before_sos == 0:
        return data[:2] + seg + data[2:]
    pos = -1
    for _ in range(before_sos + 1):
        pos = data.index(b"\xff\xda", pos + 1)
    return data[:pos] + seg + data[pos:]


def _scan_span(d: bytes) -> tuple[int, int]:
    """[start, end) of the (first) scan's entropy-coded bytes: after its SOS
    header, up to the EOI marker."""
    sos = d.index(b"\xff\xda")
    start = sos + 2 + int.from_bytes(d[sos + 2 : sos + 4], "big")
    return start, d.rindex(b"\xff\xd9")


def trailing_scan(name: str = "q90_420", copies: int = 1) -> bytes:
    """A sequential file whose scan is followed, before EOI, by `copies` more
    copies of its own entropy-coded bytes: valid Huffman symbols past the
    frame's last block, so the parallel decoder's runs there count blocks
    beyond the image's.  The sequential decoder stops at the last block and
    ignores them (libjpeg: extraneous data; FFmpeg likewise)."""
    d = case(name)
    s, e = _scan_span(d)
    return d[:e] + d[s:e] * copies + d[e:]


def junk_before_rst(seed: int = 0, name: str = "restart_rows", n: int = 24) -> bytes:
    """A restart-interval file with `n` random bytes (no 0xFF) inserted before
    every RSTn marker: garbage after each segment's last block, which the
    sequential decoder never reads."""
    d = case(name)
    rng = np.random.default_rng(500 + seed)
    s, e = _scan_span(d)
    out = bytearray(d[:s])
    i = s  # next byte of d to copy
    j = s
    while True:
        j = d.find(b"\xff", j)
        if j == -1 or j >= e:
            break
        if 0xD0 <= d[j + 1] <= 0xD7:  # RSTn: junk in front of it
            out += d[i:j] + bytes(rng.integers(0, 255, size=n, dtype=np.uint8))
            i = j
        j += 2
    out += d[i:]
    return bytes(out)
