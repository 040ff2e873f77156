"""Buffer objects returned by the operators (mirror of spdl's CUDABuffer /
CPUBuffer, reference src/spdl/io/lib/cuda/buffer.cpp:55-96)."""

from __future__ import annotations

import numpy as np
import torch


class CUDABuffer:
    """Device buffer holding decoded pixels.

    Exposes ``__cuda_array_interface__`` (version 2, typestr ``|u1`` or
    ``<f2``, strides None) and ``device_index`` like the reference, and owns
    its memory either through a torch tensor (default) or through the
    allocator pair of :func:`spdl_amd.io.cuda_config`."""

    def __init__(self, tensor: torch.Tensor | None = None, *, ptr: int = 0, shape=(),
                 dtype=torch.uint8, device_index: int = 0, stream: int = 0, deleter=None):
        self._tensor = tensor
        self._ptr = ptr
        self._shape = tuple(tensor.shape) if tensor is not None else tuple(shape)
        self._dtype = tensor.dtype if tensor is not None else dtype
        self._device_index = tensor.device.index if tensor is not None else device_index
        self._stream = stream
        self._deleter = deleter

    @property
    def device_index(self) -> int:
        return self._device_index

    @property
    def shape(self):
        return self._shape

    def data_ptr(self) -> int:
        return self._tensor.data_ptr() if self._tensor is not None else self._ptr

    @property
    def __cuda_array_interface__(self) -> dict:
        typestr = "|u1" if self._dtype == torch.uint8 else "<f2"
        return {
            "shape": self._shape,
            "typestr": typestr,
            "data": (self.data_ptr(), False),
            "version": 2,
            "strides": None,
            "stream": self._stream if self._stream not in (0,) else None,
        }

    def __del__(self):
        if self._deleter is not None and self._ptr:
            try:
                self._deleter(self._ptr)
            except Exception:
                pass
            self._ptr = 0

    def __repr__(self) -> str:
        return f"CUDABuffer(shape={self._shape}, dtype={self._dtype}, device={self._device_index})"


class CPUBuffer:
    """Host buffer with ``__array_interface__`` (reference CPUBuffer)."""

    def __init__(self, array: np.ndarray):
        self._array = np.ascontiguousarray(array)

    @property
    def __array_interface__(self) -> dict:
        return self._array.__array_interface__

    @property
    def shape(self):
        return self._array.shape

    def __repr__(self) -> str:
        return f"CPUBuffer(shape={self._array.shape}, dtype={self._array.dtype})"
