"""spdl_amd: MI355X-native (gfx950) JPEG -> RGB decode stage for SPDL.

The operator surface lives in :mod:`spdl_amd.io` and mirrors ``spdl.io``'s image
API (``decode_image_nvjpeg``, ``load_image_batch_nvjpeg``, ``load_image_batch``,
``load_image``, ``cuda_config``, ``to_torch`` ...).  All decoding runs in the
hand-written HIP kernels of ``spdl_amd/csrc`` through the C-ABI in
``include/spdl_hipjpeg.h``.
"""

__version__ = "0.1.0"
