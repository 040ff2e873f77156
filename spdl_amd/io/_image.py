"""Image operators (drop-in for the reference's spdl.io image surface).

Reference signatures:
  decode_image_nvjpeg      src/spdl/io/_core.py:868-915
  load_image_batch_nvjpeg  src/spdl/io/_composite.py:486-524
  load_image_batch         src/spdl/io/_composite.py:358-465
  load_image               src/spdl/io/_composite.py:254-295
All of them decode on the GPU (gfx950 kernels); there is no CPU path.
"""

from __future__ import annotations

import logging
import os
import warnings
from collections.abc import Sequence

import numpy as np
import torch

from .. import _lib
from .._lib import Output
from ._buffer import CPUBuffer, CUDABuffer
from ._config import CUDAConfig
from ._preprocessing import get_video_filter_desc, parse_image_filter

_LG = logging.getLogger(__name__)

_FILTER_DESC_DEFAULT = "__SPDL_DEFAULT__"


def _read(src) -> memoryview:
    if isinstance(src, (bytes, bytearray, memoryview)):
        return memoryview(src)
    if isinstance(src, str):
        with open(src, "rb") as f:
            return memoryview(f.read())
    if isinstance(src, np.ndarray):
        return memoryview(src.tobytes())
    raise TypeError(
        f"Source must be `str` (path), `bytes` (data), or `memoryview`. Found: {type(src)}"
    )


def _stream(cfg: CUDAConfig) -> int:
    return int(cfg.stream)


def _default_config() -> CUDAConfig:
    """The device a call without ``device_config`` decodes on: the current
    HIP device once torch has initialised it (a rank that called
    ``torch.cuda.set_device``), else ``$LOCAL_RANK`` (one process per GPU,
    torch.distributed.run), else 0 -- never a hard-wired device 0 for every
    rank of a job."""
    if torch.cuda.is_initialized():
        return CUDAConfig(torch.cuda.current_device())
    rank = int(os.environ.get("LOCAL_RANK", "0") or 0)
    count = torch.cuda.device_count()
    return CUDAConfig(rank if 0 <= rank < count else 0)


# FFmpeg demux / decoder options of the reference's CPU path.  The GPU
# decoder has no equivalent knobs (its parser and decoder are fixed), so
# they are accepted for drop-in compatibility and, when set, reported once.
_IGNORED_WARNED: set = set()


def _ignore_ffmpeg_configs(kwargs: dict) -> None:
    for k in ("demux_config", "decode_config"):
        v = kwargs.pop(k, None)
        if v is not None and k not in _IGNORED_WARNED:
            _IGNORED_WARNED.add(k)
            warnings.warn(f"`{k}` configures FFmpeg's demuxer/decoder, which the GPU decode "
                          f"stage does not use; it is ignored", RuntimeWarning, stacklevel=3)


def _alloc_out(cfg: CUDAConfig, shape, dtype) -> CUDABuffer:
    nbytes = int(np.prod(shape)) * (1 if dtype == torch.uint8 else 2)
    if cfg.allocator is None:
        t = torch.empty(shape, dtype=dtype, device=f"cuda:{cfg.device_index}")
        return CUDABuffer(t, stream=cfg.stream)
    alloc, free = cfg.allocator
    ptr = int(alloc(nbytes, cfg.device_index, cfg.stream))
    if not ptr:
        raise RuntimeError("allocator returned a null pointer")
    return CUDABuffer(None, ptr=ptr, shape=tuple(shape), dtype=dtype,
                      device_index=cfg.device_index, stream=cfg.stream, deleter=free)


def _decode(datas: list, out: Output, cfg: CUDAConfig, shape_per_image, batched: bool,
            dtype=torch.uint8) -> CUDABuffer:
    n = len(datas)
    shape = (n, *shape_per_image) if batched else tuple(shape_per_image)
    buf = _alloc_out(cfg, shape, dtype)
    dec = _lib.thread_decoder(cfg.device_index)
    nbytes = int(np.prod(shape)) * (1 if dtype == torch.uint8 else 2)
    dec.decode_batch(datas, out, buf.data_ptr(), nbytes, stream=_stream(cfg), sync=True)
    return buf


def _shape(out: Output, w: int, h: int) -> tuple:
    return (3, h, w) if out.planar else (h, w, 3)


def decode_image_nvjpeg(
    src,
    *,
    device_config: CUDAConfig | None = None,
    scale_width: int = -1,
    scale_height: int = -1,
    pix_fmt: str = "rgb",
    sync: bool = True,
    scale_algo: str = "lanczos",
) -> CUDABuffer:
    """Decode JPEG(s) on the GPU.  Same contract as the reference: a single
    source gives ``[3,H,W]`` (``"rgb"``/``"bgr"``) or ``[H,W,3]``
    (``"rgb24"``/``"bgr24"``), resized (stretch) when both scale sizes are
    positive; a sequence gives ``[B,...]`` and requires the scale sizes.

    ``scale_algo`` (an addition; the reference has no such argument) picks
    the resampling kernel.  The default ``"lanczos"`` is Lanczos-3, the
    kernel of the reference's ``resize_npp`` (NPPI_INTER_LANCZOS,
    src/libspdl/cuda/npp/detail/resize.cpp:36-116); ``"bicubic"`` /
    ``"bilinear"`` are the CPU path's swscale flags."""
    if device_config is None:
        raise ValueError("device_config must be provided.")
    if scale_algo not in _lib.FILTERS:
        raise ValueError(f"Unexpected scale_algo: {scale_algo}. Supported: {list(_lib.FILTERS)}")
    if pix_fmt not in _lib.PIX_FMTS:
        raise RuntimeError(
            f'Unexpected pix_fmt: {pix_fmt}. Supported values are "bgr", "bgr24", "rgb", "rgb24"'
        )
    if isinstance(src, Sequence) and not isinstance(src, (str, bytes, bytearray, memoryview)):
        datas = [_read(s) for s in src]
        if not datas:
            raise RuntimeError("No input is provided.")
        # the reference rejects only when both are missing
        # (nvjpeg/decoding.cpp:219-221); one missing size would size its
        # output buffer with a non-positive dimension and fail there
        if scale_width <= 0 and scale_height <= 0:
            raise RuntimeError("Both `scale_width` and `scale_height` must be specified.")
        if scale_width <= 0 or scale_height <= 0:
            raise RuntimeError(
                f"Failed to allocate the output buffer: invalid size {scale_width}x{scale_height}.")
        out = Output(pix_fmt=pix_fmt, resize=True, fit_w=scale_width, fit_h=scale_height,
                     filter=scale_algo)
        return _decode(datas, out, device_config, _shape(out, scale_width, scale_height), True)
    data = _read(src)
    if scale_width > 0 and scale_height > 0:
        out = Output(pix_fmt=pix_fmt, resize=True, fit_w=scale_width, fit_h=scale_height,
                     filter=scale_algo)
        w, h = scale_width, scale_height
    else:
        out = Output(pix_fmt=pix_fmt)
        info = _lib.get_image_info(data)
        w, h = info.width, info.height
    return _decode([data], out, device_config, _shape(out, w, h), False)


def load_image_batch_nvjpeg(
    srcs,
    *,
    device_config: CUDAConfig,
    width: int,
    height: int,
    pix_fmt: str = "rgb",
    scale_algo: str = "lanczos",
) -> CUDABuffer:
    """Batch load + resize (reference _composite.py:486-524): stretch to
    ``width`` x ``height`` with the ``resize_npp`` kernel (Lanczos-3) unless
    ``scale_algo`` says otherwise."""
    return decode_image_nvjpeg(
        [_read(s) for s in srcs],
        scale_width=width,
        scale_height=height,
        device_config=device_config,
        pix_fmt=pix_fmt,
        scale_algo=scale_algo,
    )


def _to_host(buf: CUDABuffer, storage=None) -> CPUBuffer:
    """Device result -> host buffer.  With ``storage`` (a :class:`CPUStorage`,
    usually pinned) the bytes land in it, as the reference's convert_frames
    writes the batch into the caller's storage
    (src/spdl/io/_composite.py:368,460 -> src/libspdl/core/buffer.cpp:48-69,
    which raises when the storage is too small)."""
    from ._convert import to_torch
    from ._transfer import transfer_buffer_cpu

    if storage is None:
        t = to_torch(buf).cpu()
        if t.dtype == torch.bfloat16:  # numpy has no bfloat16: keep the bit patterns
            return CPUBuffer(t.view(torch.int16).numpy().view(np.uint16), dtype=torch.bfloat16)
        return CPUBuffer(t.numpy())
    nbytes = int(np.prod(buf.shape)) * (1 if buf.dtype == torch.uint8 else 2)
    if storage.size < nbytes:
        raise RuntimeError(
            f"The provided storage does not have enough capacity. ({storage.size} < {nbytes})")
    return transfer_buffer_cpu(buf, storage=storage)


def load_image_batch(
    srcs,
    *,
    width: int | None,
    height: int | None,
    pix_fmt: str | None = "rgb24",
    filter_desc: str | None = _FILTER_DESC_DEFAULT,
    device_config: CUDAConfig | None = None,
    strict: bool = True,
    normalize: bool = False,
    mean=(0.485, 0.456, 0.406),
    std=(0.229, 0.224, 0.225),
    norm_dtype: str = "float16",
    **kwargs,
):
    """Batch load images into one ``[B,H,W,3]`` buffer with the FFmpeg filter
    semantics of the reference CPU path (scale + centred pad by default).

    Decoding runs on ``device_config``'s GPU (when absent: the current HIP
    device, or ``$LOCAL_RANK``); without a ``device_config`` the result is
    copied back to a host ``CPUBuffer`` -- into ``storage`` when one is given
    (a :func:`cpu_storage`), like the reference's return type.  ``normalize=True`` fuses the ImageNet
    epilogue ((x/255 - mean)/std in fp32 -> ``norm_dtype`` float16 or
    bfloat16), an extension for config 4."""
    if not srcs:
        raise ValueError("`srcs` must not be empty.")
    storage = kwargs.pop("storage", None)
    _ignore_ffmpeg_configs(kwargs)
    if kwargs:
        raise TypeError(f"unexpected arguments: {sorted(kwargs)}")
    if filter_desc == _FILTER_DESC_DEFAULT:
        filter_desc = get_video_filter_desc(
            scale_width=width, scale_height=height, pix_fmt=pix_fmt
        )
    cfg = device_config or _default_config()
    if filter_desc is None:
        # no scale and no output format: the decoder's own planes, batched as
        # the reference's convert_frames stacks them ([B, 3, H, W] yuvj444p,
        # [B, 1, 1.5H, W] yuvj420p, [B, H, W, 1] gray; same size and format)
        dec = _lib.thread_decoder(cfg.device_index)
        arrs = []
        for i, s in enumerate(srcs):
            try:
                data = _read(s)
                arrs.append(_native_planes(dec.decode_planes(data, stream=_stream(cfg)), data))
            except Exception as err:  # reference: log, skip, raise later if strict
                _LG.error("Failed to load image %d: %s", i, err)
        if strict and len(arrs) != len(srcs):
            raise RuntimeError("Failed to load some images.")
        if not arrs:
            raise RuntimeError("Failed to load all the images.")
        if any(a.shape != arrs[0].shape for a in arrs):
            raise RuntimeError("The input images must have the same size and pixel format.")
        arr = np.stack(arrs)
        if device_config is not None:
            return CUDABuffer(torch.from_numpy(arr).to(f"cuda:{cfg.device_index}"))
        if storage is not None:
            from ._transfer import convert_array

            return convert_array(arr, storage=storage)
        return CPUBuffer(arr)
    out = parse_image_filter(filter_desc, default_pix_fmt=pix_fmt or "rgb24")
    if normalize:
        out = Output(**{**out.__dict__, "normalize": True, "mean": tuple(mean),
                        "std": tuple(std), "norm_dtype": norm_dtype})
    datas, keep = [], []
    for i, s in enumerate(srcs):
        try:
            d = _read(s)
            _lib.get_image_info(d)
        except Exception as err:  # reference logs and skips (strict=False)
            _LG.error("Failed to load image %d: %s", i, err)
            continue
        datas.append(d)
        keep.append(i)
    if strict and len(datas) != len(srcs):
        raise RuntimeError("Failed to load some images.")
    if not datas:
        raise RuntimeError("Failed to load all the images.")
    info = _lib.get_image_info(datas[0])
    ow, oh = _lib.output_size(info.width, info.height, out)
    dtype = out.torch_dtype
    shape = _shape(out, ow, oh)
    try:
        buf = _decode(datas, out, cfg, shape, True, dtype=dtype)
    except RuntimeError:
        if strict:
            raise
        # decode one by one to find the survivors (rare path)
        good = []
        for d in datas:
            try:
                good.append(_decode([d], out, cfg, shape, True, dtype=dtype))
            except RuntimeError as err:
                _LG.error("Failed to decode an image: %s", err)
        if not good:
            raise RuntimeError("Failed to load all the images.") from None
        from ._convert import to_torch

        buf = CUDABuffer(torch.cat([to_torch(g) for g in good]), stream=cfg.stream)
    if device_config is None:
        # the reference's CPU result, in the caller's storage when given (with
        # a device_config the reference only stages through it on the way to
        # the device; here the batch is decoded on the device directly)
        return _to_host(buf, storage)
    return buf


_UNSUPPORTED_FRAMES = {2: "gbrp", 3: "gbrap", 4: "yuva444p", 5: "yuva444p"}  # by spdl_hj_color


def _native_planes(planes: list, data) -> np.ndarray:
    """The buffer the reference's convert_frames makes of an unfiltered
    frame (src/libspdl/core/detail/ffmpeg/conversion.cpp:172-303,411-454,
    single-frame form conversion.h:45-53): av_image_copy_to_buffer packs Y,
    then all of U, then all of V, each plane tightly, into
      gray8     [H, W, 1]        (convert_interleaved)
      yuvj444p  [3, H, W]        (convert_planer)
      yuvj420p  [1, H + H/2, W]  (convert_yuv420p)
      yuvj422p  [1, 2H, W]       (convert_yuv422p)
    A frame whose planes do not fit that shape (odd 4:2:0 / 4:2:2 sizes)
    fails the copy there ("Failed to copy image data."); other samplings
    (yuvj440p, yuvj411p) are "Unsupported pixel format", and so are the
    frames FFmpeg makes of RGB-coded and Adobe CMYK / YCCK files (gbrp,
    gbrap, yuva444p: not in convert_frames' list, conversion.cpp:420-444)."""
    fmt = _UNSUPPORTED_FRAMES.get(_lib.get_image_info(data).color)
    if fmt is not None:
        raise RuntimeError(f"Unsupported pixel format: {fmt}")
    if len(planes) == 1:
        return np.ascontiguousarray(planes[0])[:, :, None]
    (H, W), (ch, cw) = planes[0].shape, planes[1].shape
    flat = np.concatenate([np.ascontiguousarray(p).reshape(-1) for p in planes])
    if (ch, cw) == (H, W):
        return flat.reshape(3, H, W)
    if cw == (W + 1) // 2 and ch == (H + 1) // 2:
        shape = (1, H + H // 2, W)
    elif cw == (W + 1) // 2 and ch == H:
        shape = (1, 2 * H, W)
    else:
        raise RuntimeError(
            f"Unsupported pixel format: chroma {cw}x{ch} for a {W}x{H} image")
    if flat.size != shape[1] * shape[2]:
        raise RuntimeError("Failed to copy image data.")
    return flat.reshape(shape)


def load_image(
    src,
    *,
    filter_desc: str | None = _FILTER_DESC_DEFAULT,
    device_config: CUDAConfig | None = None,
    pix_fmt: str = "rgb24",
    **kwargs,
):
    """Single image.  ``filter_desc=None`` returns the decoded planes in the
    layout of the reference's convert_frames of an unfiltered frame (Y, U, V
    back to back: ``[1, 1.5H, W]`` yuvj420p, ``[1, 2H, W]`` yuvj422p,
    ``[3, H, W]`` yuvj444p, ``[H, W, 1]`` gray; see :func:`_native_planes`);
    otherwise RGB per the filter."""
    kwargs.pop("name", None)  # only names the source in FFmpeg demux errors
    _ignore_ffmpeg_configs(kwargs)
    if kwargs:
        raise TypeError(f"unexpected arguments: {sorted(kwargs)}")
    cfg = device_config or _default_config()
    data = _read(src)
    if filter_desc is None:
        dec = _lib.thread_decoder(cfg.device_index)
        arr = _native_planes(dec.decode_planes(data, stream=_stream(cfg)), data)
        if device_config is not None:
            return CUDABuffer(torch.from_numpy(arr).to(f"cuda:{cfg.device_index}"))
        return CPUBuffer(arr)
    if filter_desc == _FILTER_DESC_DEFAULT:
        filter_desc = get_video_filter_desc(pix_fmt=pix_fmt)
    out = parse_image_filter(filter_desc, default_pix_fmt=pix_fmt)
    info = _lib.get_image_info(data)
    ow, oh = _lib.output_size(info.width, info.height, out)
    buf = _decode([data], out, cfg, _shape(out, ow, oh), False)
    if device_config is None:
        return _to_host(buf)
    return buf
