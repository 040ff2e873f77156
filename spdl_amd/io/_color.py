"""NV12 -> planar RGB/BGR on the GPU (mirror of ``spdl.io.nv12_to_rgb`` /
``nv12_to_bgr``, reference src/spdl/io/_core.py:1201-1266, binding
src/spdl/io/lib/cuda/color_conversion.cpp, kernel
src/libspdl/cuda/detail/color_conversion.cu:90-138).

The video decoder that produces NV12 frames is outside this stage's scope;
this is the colour-conversion kernel the video path hands its frames to.
"""

from __future__ import annotations

import ctypes

import torch

from .. import _lib
from ._buffer import CUDABuffer
from ._config import CUDAConfig


def _as_tensor(buffers) -> torch.Tensor:
    if isinstance(buffers, torch.Tensor):
        return buffers
    if isinstance(buffers, CUDABuffer):
        from ._convert import to_torch

        return to_torch(buffers)
    if hasattr(buffers, "__cuda_array_interface__"):
        return torch.as_tensor(buffers, device="cuda")
    raise TypeError(f"expected a CUDABuffer or a device tensor, found {type(buffers)}")


def _nv12(buffers, device_config: CUDAConfig, coeff: int, sync: bool, bgr: bool) -> CUDABuffer:
    if device_config is None:
        raise ValueError("device_config must be provided.")
    src = _as_tensor(buffers)
    if src.dim() != 3:
        raise RuntimeError(
            f"Expected 3D buffer [num_frames, h*1.5, width]. Found: {src.dim()}D")
    if src.dtype != torch.uint8 or src.device.type != "cuda":
        raise RuntimeError("NV12 input must be a uint8 device buffer")
    src = src.contiguous()
    f, h2, w = src.shape
    if h2 % 3 != 0:
        raise RuntimeError(
            f"The height of NV12 image (h*1.5) must be divisible by 3. Found: {h2}")
    h = h2 // 3 * 2
    dev = device_config.device_index
    out = torch.empty((f, 3, h, w), dtype=torch.uint8, device=f"cuda:{dev}")
    err = ctypes.create_string_buffer(512)
    rc = _lib.lib().spdl_hj_nv12_to_planar_rgb(
        src.data_ptr(), f, h2, w, int(bool(bgr)), int(coeff), out.data_ptr(), out.numel(), dev,
        int(device_config.stream), int(bool(sync)), err, 512)
    if rc:
        raise RuntimeError(err.value.decode() or f"nv12 conversion failed ({rc})")
    return CUDABuffer(out, stream=device_config.stream)


def nv12_to_rgb(buffers, *, device_config: CUDAConfig, coeff: int = 1,
                sync: bool = False) -> CUDABuffer:
    """``[num_frames, H*1.5, W]`` NV12 -> ``[num_frames, 3, H, W]`` planar RGB.

    ``coeff`` selects the matrix: 1 BT.709 (default), 4 FCC, 5 BT.470,
    6 BT.601, 7 SMPTE240M, 8 YCgCo, 9 BT.2020, 10 BT.2020C; other values are
    silently mapped to 1, as in the reference."""
    return _nv12(buffers, device_config, coeff, sync, bgr=False)


def nv12_to_bgr(buffers, *, device_config: CUDAConfig, coeff: int = 1,
                sync: bool = False) -> CUDABuffer:
    """Same as :func:`nv12_to_rgb`, channel order BGR."""
    return _nv12(buffers, device_config, coeff, sync, bgr=True)
