"""ctypes binding of the gfx950 decode stage (``include/spdl_hipjpeg.h``).

The product path: every public operator in :mod:`spdl_amd.io` ends here, in
``spdl_amd/lib/libspdl_hipjpeg.so``.  There is no CPU fallback: a missing
library or a missing GPU raises immediately.
"""

from __future__ import annotations

import ctypes
import os
import threading
from dataclasses import dataclass

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SPDL_AMD_LIB") or os.path.join(_HERE, "lib", "libspdl_hipjpeg.so")

ABI_VERSION = 6

# enums (mirror include/spdl_hipjpeg.h)
PIX_FMTS = {"rgb": 0, "bgr": 1, "rgb24": 2, "bgr24": 3}
ASPECT = {None: 0, "none": 0, "decrease": 1, "increase": 2}
FILTERS = {"bicubic": 0, "bilinear": 1, "lanczos": 2}
IDCT = {"simple": 0, "islow": 1}
CSC = {"swscale": 0, "jfif": 1}
DTYPE_U8, DTYPE_F16, DTYPE_BF16 = 0, 1, 2
NORM_DTYPES = {"float16": DTYPE_F16, "bfloat16": DTYPE_BF16}

EXPORTED = (
    "spdl_hj_abi_version",
    "spdl_hj_get_image_info",
    "spdl_hj_output_size",
    "spdl_hj_create",
    "spdl_hj_destroy",
    "spdl_hj_decode_batch",
    "spdl_hj_decode_batch_device",
    "spdl_hj_decode_planes",
    "spdl_hj_set_profiling",
    "spdl_hj_last_timings",
    "spdl_hj_stage_name",
    "spdl_hj_set_param",
    "spdl_hj_get_param",
    "spdl_hj_debug_entropy",
    "spdl_hj_last_ticket",
    "spdl_hj_wait",
    "spdl_hj_staging_acquire",
    "spdl_hj_stream_wait",
    "spdl_hj_staging_fill",
    "spdl_hj_staging_read",
    "spdl_hj_decode_staged",
    "spdl_hj_tar_index",
    "spdl_hj_nv12_to_planar_rgb",
    "spdl_hj_copy",
)


class ImageInfo(ctypes.Structure):
    _fields_ = [
        ("width", ctypes.c_int32),
        ("height", ctypes.c_int32),
        ("ncomp", ctypes.c_int32),
        ("h_samp", ctypes.c_int32 * 4),
        ("v_samp", ctypes.c_int32 * 4),
        ("color", ctypes.c_int32),  # spdl_hj_color: GRAY YCBCR RGB CMYK YCCK YCBCRK
        ("multiscan", ctypes.c_int32),  # progressive or non-interleaved (ABI 5)
    ]


class OutputSpec(ctypes.Structure):
    _fields_ = [
        ("pix_fmt", ctypes.c_int32),
        ("dtype", ctypes.c_int32),
        ("idct", ctypes.c_int32),
        ("resize", ctypes.c_int32),
        ("fit_w", ctypes.c_int32),
        ("fit_h", ctypes.c_int32),
        ("aspect", ctypes.c_int32),
        ("pad_w", ctypes.c_int32),
        ("pad_h", ctypes.c_int32),
        ("crop_w", ctypes.c_int32),
        ("crop_h", ctypes.c_int32),
        ("filter", ctypes.c_int32),
        ("mean", ctypes.c_float * 3),
        ("std", ctypes.c_float * 3),
        ("csc", ctypes.c_int32),
    ]


@dataclass(frozen=True)
class Output:
    """What the decoder produces for every image of a batch.

    ``resize=False`` keeps the full resolution.  Otherwise the FFmpeg filter
    chain SPDL builds is applied (src/spdl/io/_preprocessing.py:214-234)::

        scale=w=fit_w:h=fit_h[:force_original_aspect_ratio=aspect]
        [,pad=w=pad_w:h=pad_h:x=-1:y=-1:color=black][,crop=w=crop_w:h=crop_h]
    """

    pix_fmt: str = "rgb"
    normalize: bool = False  # -> (x/255 - mean)/std in fp32, stored as norm_dtype
    idct: str = "simple"
    resize: bool = False
    fit_w: int = 0
    fit_h: int = 0
    aspect: str | None = None
    pad_w: int = 0
    pad_h: int = 0
    crop_w: int = 0
    crop_h: int = 0
    filter: str = "bicubic"
    mean: tuple = (0.485, 0.456, 0.406)
    std: tuple = (0.229, 0.224, 0.225)
    norm_dtype: str = "float16"  # or "bfloat16"
    # "swscale": the reference CPU path's libswscale arithmetic (scale +
    # yuvj -> rgb24); "jfif": IJG libjpeg tables, nearest chroma (full-res)
    csc: str = "swscale"

    def to_c(self) -> OutputSpec:
        if self.pix_fmt not in PIX_FMTS:
            raise RuntimeError(f"Unexpected pix_fmt: {self.pix_fmt}")
        return OutputSpec(
            PIX_FMTS[self.pix_fmt],
            NORM_DTYPES[self.norm_dtype] if self.normalize else DTYPE_U8,
            IDCT[self.idct],
            int(bool(self.resize)),
            int(self.fit_w),
            int(self.fit_h),
            ASPECT[self.aspect],
            int(self.pad_w),
            int(self.pad_h),
            int(self.crop_w),
            int(self.crop_h),
            FILTERS[self.filter],
            (ctypes.c_float * 3)(*self.mean),
            (ctypes.c_float * 3)(*self.std),
            CSC[self.csc],
        )

    @property
    def planar(self) -> bool:
        return self.pix_fmt in ("rgb", "bgr")

    @property
    def torch_dtype(self):
        import torch

        if not self.normalize:
            return torch.uint8
        return torch.bfloat16 if self.norm_dtype == "bfloat16" else torch.float16


_LIB = None
_LIB_LOCK = threading.Lock()


def lib() -> ctypes.CDLL:
    """Load the native library (raises if it has not been built)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    with _LIB_LOCK:
        if _LIB is not None:
            return _LIB
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"spdl_amd native library not found at {LIB_PATH}; "
                "build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "(make -C spdl_amd/csrc)"
            )
        L = ctypes.CDLL(LIB_PATH)
        vp, sz, i32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int32
        cp = ctypes.c_char_p
        L.spdl_hj_abi_version.restype = ctypes.c_int
        L.spdl_hj_get_image_info.argtypes = [vp, sz, ctypes.POINTER(ImageInfo)]
        L.spdl_hj_output_size.argtypes = [
            i32, i32, ctypes.POINTER(OutputSpec), ctypes.POINTER(i32), ctypes.POINTER(i32)
        ]
        L.spdl_hj_create.argtypes = [ctypes.c_int, cp, sz]
        L.spdl_hj_create.restype = vp
        L.spdl_hj_destroy.argtypes = [vp]
        L.spdl_hj_destroy.restype = None
        L.spdl_hj_decode_batch.argtypes = [
            vp, vp, vp, i32, ctypes.POINTER(OutputSpec), vp, sz, vp, i32, vp, cp, sz
        ]
        L.spdl_hj_decode_batch_device.argtypes = [
            vp, vp, sz, vp, vp, vp, i32, ctypes.POINTER(OutputSpec), vp, sz, vp, i32, vp, cp, sz
        ]
        L.spdl_hj_decode_planes.argtypes = [vp, vp, sz, i32, vp, vp, cp, sz]
        L.spdl_hj_set_profiling.argtypes = [vp, i32]
        L.spdl_hj_last_timings.argtypes = [vp, vp, i32, ctypes.POINTER(i32)]
        L.spdl_hj_stage_name.argtypes = [i32]
        L.spdl_hj_stage_name.restype = ctypes.c_char_p
        L.spdl_hj_set_param.argtypes = [vp, cp, ctypes.c_int64]
        L.spdl_hj_get_param.argtypes = [vp, cp, ctypes.POINTER(ctypes.c_int64)]
        L.spdl_hj_debug_entropy.argtypes = [vp, vp, sz, vp, sz, vp, sz, vp, cp, sz]
        i64 = ctypes.c_int64
        L.spdl_hj_last_ticket.argtypes = [vp]
        L.spdl_hj_last_ticket.restype = i64
        L.spdl_hj_wait.argtypes = [vp, i64, vp, i32, cp, sz]
        L.spdl_hj_staging_acquire.argtypes = [
            vp, sz, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(i64), cp, sz
        ]
        L.spdl_hj_stream_wait.argtypes = [vp, i64, vp, cp, sz]
        L.spdl_hj_staging_fill.argtypes = [vp, i64, sz, vp, sz, cp, sz]
        L.spdl_hj_staging_read.argtypes = [vp, i64, sz, ctypes.c_int, i64, sz, cp, sz]
        L.spdl_hj_decode_staged.argtypes = [
            vp, i64, sz, vp, vp, i32, ctypes.POINTER(OutputSpec), vp, sz, vp, i32, vp, cp, sz
        ]
        L.spdl_hj_tar_index.argtypes = [
            vp, sz, sz, i32, vp, vp, vp, vp, sz, ctypes.POINTER(i32), ctypes.POINTER(sz)
        ]
        L.spdl_hj_nv12_to_planar_rgb.argtypes = [
            vp, i32, i32, i32, i32, i32, vp, sz, ctypes.c_int, vp, i32, cp, sz
        ]
        L.spdl_hj_copy.argtypes = [vp, vp, sz, i32, ctypes.c_int, vp, i32, cp, sz]
        ver = L.spdl_hj_abi_version()
        # (an explicitly chosen older build, ABI >= 5, loads for A/B runs)
        if ver != ABI_VERSION and not (os.environ.get("SPDL_AMD_LIB") and 5 <= ver < ABI_VERSION):
            raise RuntimeError(f"libspdl_hipjpeg ABI {ver} != expected {ABI_VERSION}")
        _LIB = L
    return _LIB


def get_image_info(data) -> ImageInfo:
    """Host SOF probe (width, height, components, sampling factors, colour model)."""
    addr, size, keep = buffer_address(data)
    info = ImageInfo()
    rc = lib().spdl_hj_get_image_info(addr, size, ctypes.byref(info))
    del keep
    if rc:
        raise RuntimeError(f"Failed to decode an image. (header probe: status {rc})")
    return info


def output_size(width: int, height: int, out: Output) -> tuple[int, int]:
    ow, oh = ctypes.c_int32(), ctypes.c_int32()
    spec = out.to_c()
    rc = lib().spdl_hj_output_size(width, height, ctypes.byref(spec), ctypes.byref(ow),
                                   ctypes.byref(oh))
    if rc:
        raise RuntimeError(f"invalid output geometry for {width}x{height} ({rc})")
    return ow.value, oh.value


def buffer_address(src) -> tuple[int, int, object]:
    """(address, length, keepalive) of a bytes-like object without copying
    when it is writable or a numpy array; read-only bytes are viewed through
    numpy (no copy either)."""
    import numpy as np

    if isinstance(src, np.ndarray):
        a = np.ascontiguousarray(src).view(np.uint8).reshape(-1)
        return a.ctypes.data, a.size, a
    a = np.frombuffer(memoryview(src).cast("B"), np.uint8)
    if a.size == 0:  # numpy gives empty arrays a dangling address
        a = np.zeros(1, np.uint8)
        return a.ctypes.data, 0, a
    return a.ctypes.data, a.size, a


def tar_index(src, start: int = 0, max_entries: int = 1 << 20, with_names: bool = True):
    """Regular-file members of an in-memory tar archive: list of (name,
    offset, size) with payload offsets into `src`, plus the resume position.
    Native walk (spdl_hj_tar_index) with the reference's semantics
    (src/spdl/io/lib/archive/tar_iterator.cpp:125-195)."""
    import numpy as np

    addr, size, keep = buffer_address(src)
    out = []
    pos = start
    while len(out) < max_entries:
        want = min(max_entries - len(out), 4096)
        offs = np.zeros(want, np.int64)
        szs = np.zeros(want, np.int64)
        noffs = np.zeros(want, np.int64)
        names = ctypes.create_string_buffer(want * 128 + 65536) if with_names else None
        n = ctypes.c_int32()
        nxt = ctypes.c_size_t()
        rc = lib().spdl_hj_tar_index(
            addr, size, pos, want, offs.ctypes.data, szs.ctypes.data,
            noffs.ctypes.data if with_names else None, names, len(names) if names else 0,
            ctypes.byref(n), ctypes.byref(nxt))
        if rc:
            raise RuntimeError(f"tar index failed ({rc})")
        raw = names.raw if with_names else b""
        for i in range(n.value):
            if with_names:
                o = int(noffs[i])
                name = raw[o: raw.index(b"\0", o)].decode("utf-8", "surrogateescape")
            else:
                name = ""
            out.append((name, int(offs[i]), int(szs[i])))
        pos = nxt.value
        if n.value == 0 or pos >= size:
            break
    del keep
    return out, pos


def _stream_handle(stream) -> int | None:
    if stream is None:
        return None
    if isinstance(stream, int):
        return stream
    return int(stream.cuda_stream)


class Decoder:
    """One native context (device workspace + pinned staging) bound to a
    device.  Not thread-safe: use :func:`thread_decoder` for a per-thread one
    (the reference keeps its nvJPEG state thread_local,
    src/libspdl/cuda/nvjpeg/decoding.cpp:107-112)."""

    def __init__(self, device_index: int = 0):
        err = ctypes.create_string_buffer(512)
        h = lib().spdl_hj_create(int(device_index), err, 512)
        if not h:
            raise RuntimeError(f"spdl_amd: cannot create decoder: {err.value.decode()}")
        self._h = h
        self.device_index = int(device_index)

    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().spdl_hj_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_param(self, name: str, value: int) -> None:
        rc = lib().spdl_hj_set_param(self._h, name.encode(), int(value))
        if rc:
            raise ValueError(f"invalid decoder parameter {name}={value}")

    def get_param(self, name: str) -> int:
        v = ctypes.c_int64()
        if lib().spdl_hj_get_param(self._h, name.encode(), ctypes.byref(v)):
            raise ValueError(f"unknown decoder parameter {name}")
        return int(v.value)

    def set_profiling(self, enable: bool, stages=None) -> None:
        """HIP-event timing of every stage, or only of the named ones."""
        if stages is not None:
            names = [lib().spdl_hj_stage_name(i).decode() for i in range(16)]
            self.set_param("profile_stages", sum(1 << names.index(s) for s in stages))
        elif enable:
            try:
                self.set_param("profile_stages", 0xFF)
            except ValueError:  # an A/B build from before ABI 6 times every stage anyway
                pass
        lib().spdl_hj_set_profiling(self._h, int(bool(enable)))

    def last_timings(self) -> dict:
        buf = (ctypes.c_float * 16)()
        n = ctypes.c_int32()
        lib().spdl_hj_last_timings(self._h, buf, 16, ctypes.byref(n))
        # (stages outside "profile_stages" report -1: left out)
        return {lib().spdl_hj_stage_name(i).decode(): buf[i] for i in range(n.value)
                if buf[i] >= 0.0}

    def decode_batch(self, datas, out: Output, out_ptr: int, out_bytes: int, stream=None,
                     sync: bool = True, check: bool = True) -> list[int]:
        """Per-image statuses.  A failed image raises RuntimeError unless
        ``check`` is False (synchronous calls), which returns the statuses."""
        n = len(datas)
        if n == 0:
            raise RuntimeError("Failed to decode an image. (the batch is empty)")
        # borrowed for the duration of the call, no copy (the reference binds
        # memoryviews as string_views, src/spdl/io/lib/cuda/memoryview_utils.h:17-20)
        keep = []
        ptrs = (ctypes.c_void_p * n)()
        sizes = (ctypes.c_size_t * n)()
        for i, d in enumerate(datas):
            addr, size, k = buffer_address(d)
            keep.append(k)
            ptrs[i] = addr
            sizes[i] = size
        status = (ctypes.c_int32 * n)()
        err = ctypes.create_string_buffer(1024)
        spec = out.to_c()
        rc = lib().spdl_hj_decode_batch(
            self._h, ptrs, sizes, n, ctypes.byref(spec), out_ptr, out_bytes,
            _stream_handle(stream), int(bool(sync)), status, err, 1024,
        )
        if rc and not (not check and sync and any(status)):
            raise RuntimeError(err.value.decode() or f"Failed to decode an image. ({rc})")
        return list(status)

    def decode_batch_device(self, dev_ptr: int, dev_bytes: int, offsets, sizes, infos,
                            out: Output, out_ptr: int, out_bytes: int, stream=None,
                            sync: bool = True) -> list[int]:
        """``offsets``/``sizes``: sequences or int64 numpy arrays; ``infos``: a
        sequence of ImageInfo or a prebuilt ``(ImageInfo * n)`` array (pass the
        same objects again to skip re-marshalling on every call)."""
        import numpy as np

        n = len(offsets)
        offs = np.ascontiguousarray(offsets, dtype=np.int64)
        szs = np.ascontiguousarray(sizes, dtype=np.int64)
        inf = infos if isinstance(infos, ctypes.Array) else (ImageInfo * n)(*infos)
        status = np.zeros(n, np.int32)
        err = ctypes.create_string_buffer(1024)
        spec = self._spec(out)
        rc = lib().spdl_hj_decode_batch_device(
            self._h, dev_ptr, dev_bytes, offs.ctypes.data, szs.ctypes.data, inf, n,
            ctypes.byref(spec), out_ptr, out_bytes, _stream_handle(stream), int(bool(sync)),
            status.ctypes.data, err, 1024,
        )
        if rc:
            raise RuntimeError(err.value.decode() or f"Failed to decode an image. ({rc})")
        return status.tolist()

    def _spec(self, out: Output) -> OutputSpec:
        cache = self.__dict__.setdefault("_spec_cache", {})
        spec = cache.get(out)
        if spec is None:
            spec = cache[out] = out.to_c()
        return spec

    # ---- asynchronous submission / staging ring (include/spdl_hipjpeg.h) ----
    def last_ticket(self) -> int:
        return int(lib().spdl_hj_last_ticket(self._h))

    def wait(self, ticket: int, n: int = 0) -> list[int]:
        import numpy as np

        status = np.zeros(max(n, 1), np.int32)
        err = ctypes.create_string_buffer(1024)
        rc = lib().spdl_hj_wait(self._h, int(ticket), status.ctypes.data if n else None, n, err,
                                1024)
        if rc:
            raise RuntimeError(err.value.decode() or f"Failed to decode an image. ({rc})")
        return status[:n].tolist()

    def stream_wait(self, ticket: int, stream) -> None:
        """Make `stream` wait on the device for batch `ticket`."""
        err = ctypes.create_string_buffer(512)
        rc = lib().spdl_hj_stream_wait(self._h, int(ticket), _stream_handle(stream), err, 512)
        if rc:
            raise RuntimeError(err.value.decode())

    def staging_acquire(self, nbytes: int) -> tuple[int, int]:
        """(pinned host address, ticket) of the next ring slot (>= nbytes)."""
        ptr = ctypes.c_void_p()
        ticket = ctypes.c_int64()
        err = ctypes.create_string_buffer(1024)
        rc = lib().spdl_hj_staging_acquire(self._h, int(nbytes), ctypes.byref(ptr),
                                           ctypes.byref(ticket), err, 1024)
        if rc:
            raise RuntimeError(err.value.decode())
        return int(ptr.value), int(ticket.value)

    def staging_fill(self, ticket: int, dst_off: int, src_addr: int, nbytes: int) -> None:
        err = ctypes.create_string_buffer(512)
        rc = lib().spdl_hj_staging_fill(self._h, int(ticket), int(dst_off), src_addr, int(nbytes),
                                        err, 512)
        if rc:
            raise RuntimeError(err.value.decode())

    def staging_read(self, ticket: int, dst_off: int, fd: int, file_off: int,
                     nbytes: int) -> None:
        err = ctypes.create_string_buffer(512)
        rc = lib().spdl_hj_staging_read(self._h, int(ticket), int(dst_off), int(fd),
                                        int(file_off), int(nbytes), err, 512)
        if rc:
            raise RuntimeError(err.value.decode())

    def decode_staged(self, ticket: int, nbytes: int, offsets, sizes, out: Output, out_ptr: int,
                      out_bytes: int, stream=None, sync: bool = True) -> list[int]:
        n = len(offsets)
        offs = (ctypes.c_int64 * n)(*offsets)
        szs = (ctypes.c_int64 * n)(*sizes)
        status = (ctypes.c_int32 * max(n, 1))()
        err = ctypes.create_string_buffer(1024)
        spec = out.to_c()
        rc = lib().spdl_hj_decode_staged(
            self._h, int(ticket), int(nbytes), offs, szs, n, ctypes.byref(spec), out_ptr,
            out_bytes, _stream_handle(stream), int(bool(sync)), status, err, 1024)
        if rc:
            raise RuntimeError(err.value.decode() or f"Failed to decode an image. ({rc})")
        return list(status)[:n]

    def debug_entropy(self, data, nblocks: int):
        """Coefficients / destuffed bytes / diagnostics of one image (tests)."""
        import numpy as np

        addr, size, keep = buffer_address(data)
        coefs = np.zeros((nblocks, 64), np.int16)
        clean = np.zeros(size, np.uint8)
        diag = np.zeros(60, np.int32)
        err = ctypes.create_string_buffer(1024)
        rc = lib().spdl_hj_debug_entropy(self._h, addr, size, coefs.ctypes.data,
                                         coefs.size, clean.ctypes.data, clean.size,
                                         diag.ctypes.data, err, 1024)
        if rc:
            raise RuntimeError(err.value.decode())
        return coefs, clean[: max(int(diag[1]), 0)], {
            "status": int(diag[0]), "clean_len": int(diag[1]), "nseg": int(diag[2]),
            "sync_rounds": int(diag[3]),
            "phase_us": [round(int(x) / 100.0, 1) for x in diag[4:8]],
            "dbg": [int(x) for x in diag[8:12]],
            "scans": [tuple(int(x) for x in diag[12 + 3 * s:15 + 3 * s]) for s in range(16)]}

    def decode_planes(self, data, idct: str = "simple", stream=None):
        import numpy as np

        info = get_image_info(data)
        hmax = max(info.h_samp[c] for c in range(info.ncomp))
        vmax = max(info.v_samp[c] for c in range(info.ncomp))
        planes = []
        for c in range(info.ncomp):
            if info.ncomp == 1:
                w, h = info.width, info.height
            else:
                w = -(-info.width * info.h_samp[c] // hmax)
                h = -(-info.height * info.v_samp[c] // vmax)
            planes.append(np.zeros((h, w), np.uint8))
        ptrs = (ctypes.c_void_p * 4)(*([p.ctypes.data for p in planes] + [None] * (4 - len(planes))))
        addr, size, keep = buffer_address(data)
        err = ctypes.create_string_buffer(1024)
        rc = lib().spdl_hj_decode_planes(self._h, addr, size, IDCT[idct],
                                         ptrs, _stream_handle(stream), err, 1024)
        if rc:
            raise RuntimeError(err.value.decode())
        return planes


_TLS = threading.local()


def thread_decoder(device_index: int) -> Decoder:
    """The calling thread's decoder for `device_index` (created on first use)."""
    d = getattr(_TLS, "decoders", None)
    if d is None:
        d = _TLS.decoders = {}
    dec = d.get(device_index)
    if dec is None:
        dec = d[device_index] = Decoder(device_index)
    return dec
