"""spdl_amd: MI355X-native (gfx950) JPEG -> RGB decode stage for SPDL.

The operator surface lives in :mod:`spdl_amd.io` and mirrors ``spdl.io``'s image
API (``decode_image_nvjpeg``, ``load_image_batch_nvjpeg``, ``load_image_batch``,
``load_image``, ``cuda_config``, ``to_torch`` ...).  All decoding runs in the
hand-written HIP kernels of ``spdl_amd/csrc`` through the C-ABI in
``include/spdl_hipjpeg.h``.
"""

import os as _os

# Each decode pipeline lane is a HIP stream of its own.  Lane streams are
# created at low priority: HIP keeps a pool of GPU_MAX_HW_QUEUES hardware
# queues per stream priority, so the lanes get queues of their own whatever
# the variable's value (4, HIP's default, included) and whether or not torch
# initialised HIP first.  HW_QUEUES is the per-pool queue count in effect.
HW_QUEUES = int(_os.environ.get("GPU_MAX_HW_QUEUES") or 0) or 4

__version__ = "0.1.0"
