"""ctypes bindings for the CPU oracle (``oracle/jpeg_oracle.c``) and the libjpeg
9d pinning helper (``oracle/ljpin.c``).

TEST INFRASTRUCTURE ONLY: imported by ``tests/``, ``__graft_entry__.smoke()``
and the ``cpu_baseline`` leg of ``bench.py``. The product package ``spdl_amd``
never imports this module.
"""

from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_BUILD = os.path.join(_HERE, "_build")

IDCT_SIMPLE, IDCT_ISLOW = 0, 1
FMT = {"rgb": 0, "bgr": 1, "rgb24": 2, "bgr24": 3}
ASPECT = {None: 0, "none": 0, "decrease": 1, "increase": 2}
FILTER = {"bicubic": 0, "bilinear": 1, "lanczos": 2}
DTYPE_U8, DTYPE_F16, DTYPE_BF16 = 0, 1, 2
IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


class _Info(ctypes.Structure):
    _fields_ = [
        ("width", ctypes.c_int),
        ("height", ctypes.c_int),
        ("ncomp", ctypes.c_int),
        ("hmax", ctypes.c_int),
        ("vmax", ctypes.c_int),
        ("mcux", ctypes.c_int),
        ("mcuy", ctypes.c_int),
        ("bpm", ctypes.c_int),
        ("nblocks", ctypes.c_int),
        ("restart_interval", ctypes.c_int),
        ("comp_h", ctypes.c_int * 4),
        ("comp_v", ctypes.c_int * 4),
        ("comp_tq", ctypes.c_int * 4),
        ("comp_td", ctypes.c_int * 4),
        ("comp_ta", ctypes.c_int * 4),
        ("comp_bw", ctypes.c_int * 4),
        ("comp_bh", ctypes.c_int * 4),
        ("comp_w", ctypes.c_int * 4),
        ("comp_h_px", ctypes.c_int * 4),
        ("mcu_comp", ctypes.c_int * 10),
        ("mcu_dx", ctypes.c_int * 10),
        ("mcu_dy", ctypes.c_int * 10),
        ("qt", (ctypes.c_uint16 * 64) * 4),
        ("dc_bits", (ctypes.c_uint8 * 17) * 4),
        ("dc_vals", (ctypes.c_uint8 * 256) * 4),
        ("ac_bits", (ctypes.c_uint8 * 17) * 4),
        ("ac_vals", (ctypes.c_uint8 * 256) * 4),
        ("scan_start", ctypes.c_size_t),
        ("progressive", ctypes.c_int),
        ("multiscan", ctypes.c_int),
        ("adobe", ctypes.c_int),
        ("color", ctypes.c_int),
    ]


class _Resize(ctypes.Structure):
    _fields_ = [
        ("fit_w", ctypes.c_int),
        ("fit_h", ctypes.c_int),
        ("aspect", ctypes.c_int),
        ("pad_w", ctypes.c_int),
        ("pad_h", ctypes.c_int),
        ("crop_w", ctypes.c_int),
        ("crop_h", ctypes.c_int),
        ("filter", ctypes.c_int),
    ]


class _Geom(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in ("sw", "sh", "dx", "dy", "ow", "oh")]


@dataclass(frozen=True)
class Resize:
    """Resize spec, mirroring the FFmpeg filter chain SPDL builds
    (src/spdl/io/_preprocessing.py:214-234)."""

    fit_w: int = 0
    fit_h: int = 0
    aspect: str | None = None  # None | "decrease" | "increase"
    pad_w: int = 0
    pad_h: int = 0
    crop_w: int = 0
    crop_h: int = 0
    filter: str = "bicubic"

    def _c(self) -> _Resize:
        return _Resize(
            self.fit_w,
            self.fit_h,
            ASPECT[self.aspect],
            self.pad_w,
            self.pad_h,
            self.crop_w,
            self.crop_h,
            FILTER[self.filter],
        )


def build() -> None:
    """Compile the oracle (and the libjpeg pin helper when libjpeg 9 exists)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


_LIB = None
_LJ = None


def lib() -> ctypes.CDLL:
    global _LIB
    if _LIB is None:
        path = os.path.join(_BUILD, "libjpeg_oracle.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        vp, sz, ip = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        L.jo_parse.argtypes = [vp, sz, ctypes.POINTER(_Info)]
        L.jo_decode_coefs.argtypes = [vp, sz, ctypes.POINTER(_Info), vp, vp]
        L.jo_decode_planes.argtypes = [vp, sz, ip, vp]
        L.jo_planes_size.argtypes = [ctypes.POINTER(_Info)]
        L.jo_planes_size.restype = sz
        L.jo_decode_rgb.argtypes = [vp, sz, ip, ip, vp]
        L.jo_decode_rgb_csc.argtypes = [vp, sz, ip, ip, ip, vp]
        L.jo_sws_axis.argtypes = [ip, ip, ip, ip, ip, ip, ip, vp, vp, ip]
        L.jo_geometry.argtypes = [ip, ip, ctypes.POINTER(_Resize), ctypes.POINTER(_Geom)]
        L.jo_decode_resize.argtypes = [
            vp, sz, ip, ctypes.POINTER(_Resize), ip, ip, vp, vp, vp, ctypes.POINTER(_Geom)
        ]
        L.jo_resize_planes.argtypes = [
            ctypes.POINTER(_Info), vp, ctypes.POINTER(_Resize), ip, ip, vp, vp, vp,
            ctypes.POINTER(_Geom),
        ]
        L.jo_idct_simple.argtypes = [vp, vp, ip]
        L.jo_idct_islow.argtypes = [vp, vp, ip]
        L.jo_strerror.restype = ctypes.c_char_p
        L.jo_f32_to_f16.argtypes = [ctypes.c_float]
        L.jo_f32_to_f16.restype = ctypes.c_uint16
        L.jo_decode_resize_batch.argtypes = [
            vp, vp, ip, ip, ctypes.POINTER(_Resize), ip, ip, vp, vp, vp, sz, ip, vp
        ]
        L.jo_decode_rgb_batch.argtypes = [vp, vp, ip, ip, ip, vp, sz, ip, vp]
        _LIB = L
    return _LIB


def ljpin():
    """The libjpeg 9d pin helper, or None when it is not built here."""
    global _LJ
    if _LJ is None:
        path = os.path.join(_BUILD, "libljpin.so")
        if not os.path.exists(path):
            try:
                build()
            except Exception:
                return None
        if not os.path.exists(path):
            return None
        try:
            L = ctypes.CDLL(path)
        except OSError:
            return None
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        L.lj_read_coefs.argtypes = [vp, sz, vp, vp, sz, vp]
        L.lj_decode_rgb.argtypes = [vp, sz, vp, sz, vp, vp]
        _LJ = L
    return _LJ


class OracleError(RuntimeError):
    def __init__(self, code: int):
        super().__init__(f"oracle: {lib().jo_strerror(code).decode()} (code {code})")
        self.code = code


def _buf(data: bytes):
    arr = np.frombuffer(data, dtype=np.uint8)
    return arr, arr.ctypes.data


def parse(data: bytes) -> _Info:
    info = _Info()
    _, p = _buf(data)
    rc = lib().jo_parse(p, len(data), ctypes.byref(info))
    if rc:
        raise OracleError(rc)
    return info


def decode_coefs(data: bytes):
    """Returns (coefs [nblocks,64] int16 dequantised MCU order,
    levels per component [bh,bw,64] quantised)."""
    info = parse(data)
    coefs = np.zeros((info.nblocks, 64), np.int16)
    tot = sum(info.comp_bw[c] * info.comp_bh[c] for c in range(info.ncomp))
    levels = np.zeros((tot, 64), np.int16)
    _, p = _buf(data)
    rc = lib().jo_decode_coefs(
        p, len(data), ctypes.byref(info), coefs.ctypes.data, levels.ctypes.data
    )
    if rc:
        raise OracleError(rc)
    out, o = [], 0
    for c in range(info.ncomp):
        n = info.comp_bw[c] * info.comp_bh[c]
        out.append(levels[o : o + n].reshape(info.comp_bh[c], info.comp_bw[c], 64))
        o += n
    return coefs, out


def decode_planes(data: bytes, idct: int = IDCT_SIMPLE):
    """Per-component planes, cropped to the true component size."""
    info = parse(data)
    buf = np.zeros(lib().jo_planes_size(ctypes.byref(info)), np.uint8)
    _, p = _buf(data)
    rc = lib().jo_decode_planes(p, len(data), idct, buf.ctypes.data)
    if rc:
        raise OracleError(rc)
    planes, o = [], 0
    for c in range(info.ncomp):
        h, w = info.comp_bh[c] * 8, info.comp_bw[c] * 8
        pl = buf[o : o + h * w].reshape(h, w)
        planes.append(pl[: info.comp_h_px[c], : info.comp_w[c]].copy())
        o += h * w
    return planes


CSC = {"swscale": 0, "jfif": 1}


def decode_rgb(data: bytes, idct: int = IDCT_SIMPLE, pix_fmt: str = "rgb24",
               csc: str = "swscale") -> np.ndarray:
    """Full-resolution RGB: FFmpeg's swscale conversion (the reference CPU
    path, default) or IJG libjpeg's JFIF tables + nearest chroma ("jfif")."""
    info = parse(data)
    W, H = info.width, info.height
    out = np.zeros(W * H * 3, np.uint8)
    _, p = _buf(data)
    rc = lib().jo_decode_rgb_csc(p, len(data), idct, CSC[csc], FMT[pix_fmt], out.ctypes.data)
    if rc:
        raise OracleError(rc)
    return out.reshape((3, H, W) if pix_fmt in ("rgb", "bgr") else (H, W, 3))


def geometry(w: int, h: int, rs: Resize) -> dict:
    g = _Geom()
    rc = lib().jo_geometry(w, h, ctypes.byref(rs._c()), ctypes.byref(g))
    if rc:
        raise OracleError(rc)
    return {k: getattr(g, k) for k, _ in _Geom._fields_}


def sws_axis(src: int, dst: int, filt: str = "bicubic", align: int = 4, one: int = 1 << 14,
             src_pos: int = 128, dst_pos: int = 128):
    """(positions [dst], taps [dst, size]) of the filter libswscale's
    initFilter builds for one axis (sws_oracle.c)."""
    cap = dst * 512
    pos = np.zeros(dst, np.int32)
    coef = np.zeros(cap, np.int16)
    n = lib().jo_sws_axis(src, dst, FILTER[filt], align, one, src_pos, dst_pos, pos.ctypes.data,
                          coef.ctypes.data, cap)
    if n < 0:
        raise OracleError(7)
    return pos, coef[: dst * n].reshape(dst, n)


def decode_resize(
    data: bytes,
    rs: Resize,
    pix_fmt: str = "rgb24",
    idct: int = IDCT_SIMPLE,
    normalize: bool = False,
    mean=IMAGENET_MEAN,
    std=IMAGENET_STD,
    norm_dtype: str = "float16",
) -> np.ndarray:
    info = parse(data)
    g = geometry(info.width, info.height, rs)
    n = g["ow"] * g["oh"] * 3
    out = np.zeros(n, np.uint16 if normalize else np.uint8)
    m = np.asarray(mean, np.float32)
    s = np.asarray(std, np.float32)
    _, p = _buf(data)
    rc = lib().jo_decode_resize(
        p, len(data), idct, ctypes.byref(rs._c()), FMT[pix_fmt],
        (DTYPE_BF16 if norm_dtype == "bfloat16" else DTYPE_F16) if normalize else DTYPE_U8,
        m.ctypes.data, s.ctypes.data,
        out.ctypes.data, None,
    )
    if rc:
        raise OracleError(rc)
    if normalize and norm_dtype != "bfloat16":  # bfloat16: raw uint16 bit patterns
        out = out.view(np.float16)
    shape = (3, g["oh"], g["ow"]) if pix_fmt in ("rgb", "bgr") else (g["oh"], g["ow"], 3)
    return out.reshape(shape)


def decode_resize_batch(
    datas, rs: Resize, pix_fmt: str = "rgb24", idct: int = IDCT_SIMPLE, nthreads: int = 1,
    out_hw: tuple[int, int] | None = None,
):
    """Threaded batch (CPU baseline). All images must share the output size."""
    n = len(datas)
    arrs = [np.frombuffer(d, np.uint8) for d in datas]
    ptrs = (ctypes.c_void_p * n)(*[a.ctypes.data for a in arrs])
    sizes = (ctypes.c_size_t * n)(*[len(d) for d in datas])
    if out_hw is None:
        info = parse(datas[0])
        g = geometry(info.width, info.height, rs)
        out_hw = (g["oh"], g["ow"])
    per = out_hw[0] * out_hw[1] * 3
    out = np.zeros((n, per), np.uint8)
    status = np.zeros(n, np.int32)
    m = np.asarray(IMAGENET_MEAN, np.float32)
    s = np.asarray(IMAGENET_STD, np.float32)
    failed = lib().jo_decode_resize_batch(
        ptrs, sizes, n, idct, ctypes.byref(rs._c()), FMT[pix_fmt], DTYPE_U8,
        m.ctypes.data, s.ctypes.data, out.ctypes.data, per, nthreads, status.ctypes.data,
    )
    return out, status, failed


def decode_rgb_batch(datas, pix_fmt: str = "rgb24", idct: int = IDCT_SIMPLE, nthreads: int = 1):
    """Threaded full-resolution batch (CPU baseline); equal sizes."""
    n = len(datas)
    arrs = [np.frombuffer(d, np.uint8) for d in datas]
    ptrs = (ctypes.c_void_p * n)(*[a.ctypes.data for a in arrs])
    sizes = (ctypes.c_size_t * n)(*[len(d) for d in datas])
    info = parse(datas[0])
    per = info.width * info.height * 3
    out = np.zeros((n, per), np.uint8)
    status = np.zeros(n, np.int32)
    failed = lib().jo_decode_rgb_batch(ptrs, sizes, n, idct, FMT[pix_fmt], out.ctypes.data, per,
                                       nthreads, status.ctypes.data)
    return out, status, failed


def nv12_to_rgb(nv12: np.ndarray, coeff: int = 1, bgr: bool = False) -> np.ndarray:
    """[F, 1.5H, W] u8 NV12 -> [F, 3, H, W] u8 (jo_nv12_to_rgb; quads with
    x + 1 >= W are left 0 here, unwritten by the reference)."""
    a = np.ascontiguousarray(nv12, np.uint8)
    F, h2, W = a.shape
    H = h2 // 3 * 2
    out = np.zeros((F, 3, H, W), np.uint8)
    L = lib()
    L.jo_nv12_to_rgb.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    L.jo_nv12_to_rgb.restype = None
    L.jo_nv12_to_rgb(a.ctypes.data, F, H, W, int(bool(bgr)), int(coeff), out.ctypes.data)
    return out


def idct_block(coefs: np.ndarray, idct: int = IDCT_SIMPLE) -> np.ndarray:
    c = np.ascontiguousarray(coefs, np.int16).reshape(64)
    out = np.zeros(64, np.uint8)
    fn = lib().jo_idct_islow if idct == IDCT_ISLOW else lib().jo_idct_simple
    fn(c.ctypes.data, out.ctypes.data, 8)
    return out.reshape(8, 8)


# ---- libjpeg 9d pinning -------------------------------------------------


def lj_read_coefs(data: bytes):
    L = ljpin()
    if L is None:
        raise RuntimeError("libjpeg 9 pin helper not available")
    info = np.zeros(3 + 4 * 4, np.int32)
    cap = 64 * 200000
    out = np.zeros(cap, np.int16)
    qt = np.zeros(4 * 64, np.uint16)
    _, p = _buf(data)
    n = L.lj_read_coefs(p, len(data), info.ctypes.data, out.ctypes.data, cap, qt.ctypes.data)
    if n < 0:
        raise RuntimeError(f"libjpeg failed ({n})")
    comps, o = [], 0
    for c in range(info[2]):
        bw, bh = int(info[3 + 4 * c]), int(info[4 + 4 * c])
        comps.append(out[o * 64 : (o + bw * bh) * 64].reshape(bh, bw, 64).copy())
        o += bw * bh
    return comps


def lj_decode_rgb(data: bytes) -> np.ndarray:
    L = ljpin()
    if L is None:
        raise RuntimeError("libjpeg 9 pin helper not available")
    cap = 1 << 26
    out = np.zeros(cap, np.uint8)
    w = ctypes.c_int()
    h = ctypes.c_int()
    _, p = _buf(data)
    rc = L.lj_decode_rgb(p, len(data), out.ctypes.data, cap, ctypes.byref(w), ctypes.byref(h))
    if rc:
        raise RuntimeError(f"libjpeg failed ({rc})")
    return out[: w.value * h.value * 3].reshape(h.value, w.value, 3).copy()


def lj_encode_multiscan(px: np.ndarray, quality: int = 90, h0: int = 2, v0: int = 2,
                        restart_blocks: int = 0) -> bytes:
    """Fixture encoder (libjpeg 9): sequential JPEG with one non-interleaved
    scan per component, in reverse component order."""
    L = ljpin()
    if L is None:
        raise RuntimeError("libjpeg 9 pin helper not available")
    px = np.ascontiguousarray(px, np.uint8)
    h, w = px.shape[:2]
    nc = 1 if px.ndim == 2 else px.shape[2]
    cap = h * w * nc * 4 + 65536
    out = np.zeros(cap, np.uint8)
    f = L.lj_encode_multiscan
    f.restype = ctypes.c_long
    f.argtypes = [ctypes.c_void_p] + [ctypes.c_int] * 7 + [ctypes.c_void_p, ctypes.c_size_t]
    n = f(px.ctypes.data, w, h, nc, quality, h0, v0, restart_blocks, out.ctypes.data, cap)
    if n <= 0:
        raise RuntimeError(f"libjpeg encode failed ({n})")
    return out[:n].tobytes()


def _lj_encode_cs(px: np.ndarray, quality: int, mode: int, restart_blocks: int) -> bytes:
    L = ljpin()
    if L is None:
        raise RuntimeError("libjpeg 9 pin helper not available")
    px = np.ascontiguousarray(px, np.uint8)
    h, w = px.shape[:2]
    cap = h * w * 16 + 65536
    out = np.zeros(cap, np.uint8)
    f = L.lj_encode_cs
    f.restype = ctypes.c_long
    f.argtypes = [ctypes.c_void_p] + [ctypes.c_int] * 5 + [ctypes.c_void_p, ctypes.c_size_t]
    n = f(px.ctypes.data, w, h, quality, mode, restart_blocks, out.ctypes.data, cap)
    if n <= 0:
        raise RuntimeError(f"libjpeg encode failed ({n})")
    return out[:n].tobytes()


def lj_encode_cmyk(cmyk: np.ndarray, quality: int = 90, ycck: bool = False,
                   restart_blocks: int = 0, script: str = "sequential") -> bytes:
    """Fixture encoder (libjpeg 9): a 4-component Adobe JPEG (transform 0
    CMYK, or 2 YCCK) of HxWx4 pixels, every component 1x1.  script:
    "sequential" (one interleaved scan), "progressive" (libjpeg's
    jpeg_simple_progression) or "multiscan" (one component per scan)."""
    bits = {"sequential": 0, "progressive": 4, "multiscan": 8}[script]
    return _lj_encode_cs(cmyk, quality, (1 if ycck else 0) | bits, restart_blocks)


def lj_encode_rgb_colorspace(rgb: np.ndarray, quality: int = 90, restart_blocks: int = 0) -> bytes:
    """Fixture encoder (libjpeg 9): a 3-component JPEG coded in RGB (no
    YCbCr transform; component ids 'R' 'G' 'B', Adobe transform 0)."""
    return _lj_encode_cs(rgb, quality, 2, restart_blocks)
