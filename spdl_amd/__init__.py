"""spdl_amd: MI355X-native (gfx950) JPEG -> RGB decode stage for SPDL.

The operator surface lives in :mod:`spdl_amd.io` and mirrors ``spdl.io``'s image
API (``decode_image_nvjpeg``, ``load_image_batch_nvjpeg``, ``load_image_batch``,
``load_image``, ``cuda_config``, ``to_torch`` ...).  All decoding runs in the
hand-written HIP kernels of ``spdl_amd/csrc`` through the C-ABI in
``include/spdl_hipjpeg.h``.
"""

import os as _os

# Each decode pipeline lane is a HIP stream of its own, beside the copy stream
# and the caller's: with HIP's default of 4 hardware queues per process, three
# or more lanes share queues and serialise (measured: 4 lanes 348k img/s with
# 4 queues, 439k with 16).  Takes effect when HIP initialises after this
# import (import spdl_amd before the first GPU call).
_os.environ["GPU_MAX_HW_QUEUES"] = str(max(16, int(_os.environ.get("GPU_MAX_HW_QUEUES") or 0)))

__version__ = "0.1.0"
