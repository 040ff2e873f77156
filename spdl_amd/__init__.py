"""spdl_amd: MI355X-native (gfx950) JPEG -> RGB decode stage for SPDL.

The operator surface lives in :mod:`spdl_amd.io` and mirrors ``spdl.io``'s image
API (``decode_image_nvjpeg``, ``load_image_batch_nvjpeg``, ``load_image_batch``,
``load_image``, ``cuda_config``, ``to_torch`` ...).  All decoding runs in the
hand-written HIP kernels of ``spdl_amd/csrc`` through the C-ABI in
``include/spdl_hipjpeg.h``.
"""

import os as _os
import sys as _sys

# Each decode pipeline lane is a HIP stream of its own, beside the copy stream
# and the caller's: with HIP's default of 4 hardware queues per process, three
# or more lanes share queues and serialise (measured: 4 lanes 348k img/s with
# 4 queues, 439k with 16).  HIP reads the variable when it initialises, so
# this only works when spdl_amd is imported before the first GPU call.
# HW_QUEUES is the value in effect; HW_QUEUES_LATE says HIP had already
# initialised (through torch) with the previous value, and decoders then
# clamp their lanes to it (spdl_hj_set_param "hw_queues").
_prev = int(_os.environ.get("GPU_MAX_HW_QUEUES") or 0)
_torch = _sys.modules.get("torch")
HW_QUEUES_LATE = bool(_torch is not None and hasattr(_torch, "cuda")
                      and _torch.cuda.is_initialized())
if HW_QUEUES_LATE:
    HW_QUEUES = _prev or 4
else:
    HW_QUEUES = max(16, _prev)
    _os.environ["GPU_MAX_HW_QUEUES"] = str(HW_QUEUES)
del _torch

__version__ = "0.1.0"
