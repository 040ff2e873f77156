"""Drop-in image operator surface (mirror of ``spdl.io``'s image API,
reference src/spdl/io/__init__.py:20-86), backed by gfx950 HIP kernels."""

from ._buffer import CPUBuffer, CUDABuffer
from ._color import nv12_to_bgr, nv12_to_rgb
from ._config import CUDAConfig, cuda_config
from ._convert import to_numpy, to_torch
from ._image import (
    decode_image_nvjpeg,
    load_image,
    load_image_batch,
    load_image_batch_nvjpeg,
)
from ._preprocessing import get_video_filter_desc, parse_image_filter
from ._tar import TarImageStream, iter_tarfile
from ._transfer import (
    CPUStorage,
    convert_array,
    cpu_storage,
    transfer_buffer,
    transfer_buffer_cpu,
    transfer_tensor,
)

# HIP-named aliases: same functions, named for the hardware they run on.
decode_image_hip = decode_image_nvjpeg
load_image_batch_hip = load_image_batch_nvjpeg

__all__ = [
    "CPUBuffer",
    "CPUStorage",
    "CUDABuffer",
    "CUDAConfig",
    "convert_array",
    "cpu_storage",
    "cuda_config",
    "decode_image_hip",
    "decode_image_nvjpeg",
    "get_video_filter_desc",
    "iter_tarfile",
    "TarImageStream",
    "load_image",
    "load_image_batch",
    "load_image_batch_hip",
    "load_image_batch_nvjpeg",
    "nv12_to_bgr",
    "nv12_to_rgb",
    "parse_image_filter",
    "to_numpy",
    "to_torch",
    "transfer_buffer",
    "transfer_buffer_cpu",
    "transfer_tensor",
]
