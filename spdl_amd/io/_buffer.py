"""Buffer objects returned by the operators (mirror of spdl's CUDABuffer /
CPUBuffer, reference src/spdl/io/lib/cuda/buffer.cpp:55-96)."""

from __future__ import annotations

import numpy as np
import torch


# array-interface typestr per element type.  bfloat16 has no standard
# typestr: it is exported as an opaque 2-byte record ("<V2") and to_torch /
# to_numpy reinterpret it (bf16 tensor / uint16 bit patterns).
_TYPESTR = {
    torch.uint8: "|u1", torch.int8: "|i1", torch.int16: "<i2", torch.int32: "<i4",
    torch.int64: "<i8", torch.float16: "<f2", torch.float32: "<f4", torch.float64: "<f8",
    torch.bool: "|b1", torch.bfloat16: "<V2",
}


def typestr_of(dtype: torch.dtype) -> str:
    try:
        return _TYPESTR[dtype]
    except KeyError:
        raise TypeError(f"unsupported buffer dtype {dtype}") from None


def _itemsize(dtype: torch.dtype) -> int:
    return torch.empty((), dtype=dtype).element_size()


def torch_dtype_of(np_dtype) -> torch.dtype:
    return torch.from_numpy(np.empty(0, dtype=np_dtype)).dtype


class CUDABuffer:
    """Device buffer holding decoded pixels.

    Exposes ``__cuda_array_interface__`` (version 2, typestr of the element
    type, strides None) and ``device_index`` like the reference, and owns
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
    def dtype(self) -> torch.dtype:
        return self._dtype

    @property
    def nbytes(self) -> int:
        return int(np.prod(self._shape, dtype=np.int64)) * _itemsize(self._dtype)

    @property
    def __cuda_array_interface__(self) -> dict:
        typestr = typestr_of(self._dtype)
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
    """Host buffer with ``__array_interface__`` (reference CPUBuffer).

    ``storage``: the :class:`~spdl_amd.io.CPUStorage` the array lives in (kept
    alive with the buffer; a pinned storage makes transfer_buffer copy
    asynchronously on the config stream).  ``dtype``: the element type when
    numpy has none (bfloat16: the array holds the uint16 bit patterns)."""

    def __init__(self, array: np.ndarray, *, storage=None, dtype: torch.dtype | None = None):
        self._array = np.ascontiguousarray(array)
        self._storage = storage
        self._dtype = dtype if dtype is not None else torch_dtype_of(self._array.dtype)

    @property
    def dtype(self) -> torch.dtype:
        return self._dtype

    @property
    def is_pinned(self) -> bool:
        return self._storage is not None and self._storage.is_pinned

    def data_ptr(self) -> int:
        return int(self._array.ctypes.data)

    @property
    def nbytes(self) -> int:
        return int(self._array.nbytes)

    @property
    def __array_interface__(self) -> dict:
        return self._array.__array_interface__

    @property
    def shape(self):
        return self._array.shape

    def __repr__(self) -> str:
        return f"CPUBuffer(shape={self._array.shape}, dtype={self._array.dtype})"
