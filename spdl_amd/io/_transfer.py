"""Host <-> device buffer transfer (mirror of ``spdl.io.cpu_storage``,
``convert_array``, ``transfer_buffer``, ``transfer_buffer_cpu`` and
``transfer_tensor``).

Reference surface: src/spdl/io/_config.py:296-330 (cpu_storage),
src/spdl/io/_core.py:1045-1062 (convert_array), 1168-1195 (transfer_buffer,
transfer_buffer_cpu), src/spdl/io/_transfer.py (transfer_tensor); native side
src/libspdl/core/storage.cpp:29-44 (CPUStorage: size 0 is an error) and
src/libspdl/cuda/transfer.cpp (pinned -> async copy on the config stream +
synchronise, pageable -> synchronous copy).

The copies themselves go through the C-ABI (``spdl_hj_copy``); the pinned
page-locked allocation is HIP's host allocator via torch.
"""

from __future__ import annotations

import ctypes
import os
import threading
from collections import defaultdict
from collections.abc import Mapping
from dataclasses import fields, is_dataclass

import numpy as np
import torch

from .. import _lib
from ._buffer import CPUBuffer, CUDABuffer, _itemsize, torch_dtype_of
from ._config import CUDAConfig

_H2D, _D2H = 0, 1


class CPUStorage:
    """A block of host memory, page-locked when ``pin_memory`` (reference
    CPUStorage).  Buffers made by :func:`convert_array` over it keep it alive."""

    def __init__(self, size: int, pin_memory: bool = True):
        if isinstance(size, bool) or not isinstance(size, int) or size < 0:
            # the reference binds size as size_t: a negative value does not convert
            raise TypeError(f"size must be a non-negative int, found {size!r}")
        if size == 0:
            raise RuntimeError("`size` must be greater than 0.")
        self._tensor = torch.empty(size, dtype=torch.uint8, pin_memory=bool(pin_memory))
        self._pinned = bool(pin_memory)

    @property
    def size(self) -> int:
        return self._tensor.numel()

    @property
    def is_pinned(self) -> bool:
        return self._pinned

    def data_ptr(self) -> int:
        return self._tensor.data_ptr()

    def __repr__(self) -> str:
        return f"CPUStorage(size={self.size}, pinned={self._pinned})"


def cpu_storage(size: int, pin_memory: bool = True) -> CPUStorage:
    """Allocate ``size`` bytes of host memory (page-locked by default) for
    :func:`convert_array`; a pinned source lets :func:`transfer_buffer` copy
    with DMA on the config stream."""
    return CPUStorage(size, pin_memory)


def convert_array(vals, storage: CPUStorage | None = None) -> CPUBuffer:
    """Copy an array into a :class:`CPUBuffer` (into ``storage`` when given;
    RuntimeError if it is smaller than the array).  Shape and dtype are kept."""
    arr = np.ascontiguousarray(vals)
    if storage is None:
        return CPUBuffer(arr.copy())
    if storage.size < arr.nbytes:
        raise RuntimeError(
            f"The size of storage ({storage.size}) is smaller than the array ({arr.nbytes}).")
    view = storage._tensor.numpy()[: arr.nbytes].view(arr.dtype).reshape(arr.shape)
    view[...] = arr
    return CPUBuffer(view, storage=storage)


def _err() -> ctypes.Array:
    return ctypes.create_string_buffer(512)


def _copy(dst: int, src: int, nbytes: int, kind: int, device: int, stream: int,
          pinned: bool) -> None:
    err = _err()
    rc = _lib.lib().spdl_hj_copy(dst, src, nbytes, kind, device, stream, int(pinned), err, 512)
    if rc:
        raise RuntimeError(err.value.decode() or f"copy failed ({rc})")


def _host_source(buffer):
    """(pointer, nbytes, shape, torch dtype, pinned, keep-alive) of a host buffer."""
    if isinstance(buffer, CPUBuffer):
        return buffer.data_ptr(), buffer.nbytes, buffer.shape, buffer.dtype, buffer.is_pinned, buffer
    if isinstance(buffer, torch.Tensor):
        if buffer.device.type != "cpu":
            raise TypeError("transfer_buffer expects a CPU buffer")
        t = buffer.contiguous()
        return (t.data_ptr(), t.numel() * t.element_size(), tuple(t.shape), t.dtype,
                t.is_pinned(), t)
    if hasattr(buffer, "__array_interface__") or isinstance(buffer, (list, tuple)):
        arr = np.ascontiguousarray(buffer)
        return (int(arr.ctypes.data), int(arr.nbytes), arr.shape, torch_dtype_of(arr.dtype),
                False, arr)
    raise TypeError(f"expected a CPUBuffer or a host array, found {type(buffer)}")


def transfer_buffer(buffer, *, device_config: CUDAConfig) -> CUDABuffer:
    """Move a host buffer to the device of ``device_config``.

    The destination comes from the config's allocator when one is set
    (freed with its deleter when the buffer dies), else from torch's caching
    allocator.  A pinned source is copied asynchronously on the config stream
    and the stream synchronised; a pageable one with a synchronous copy."""
    if device_config is None:
        raise ValueError("device_config must be provided.")
    ptr, nbytes, shape, dtype, pinned, _keep = _host_source(buffer)
    dev, stream = device_config.device_index, int(device_config.stream)
    if device_config.allocator is None:
        t = torch.empty(shape, dtype=dtype, device=f"cuda:{dev}")
        out = CUDABuffer(t, stream=stream)
    else:
        alloc, free = device_config.allocator
        dptr = int(alloc(max(nbytes, 1), dev, stream))
        if not dptr:
            raise RuntimeError("allocator returned a null pointer")
        out = CUDABuffer(None, ptr=dptr, shape=tuple(shape), dtype=dtype, device_index=dev,
                         stream=stream, deleter=free)
    _copy(out.data_ptr(), ptr, nbytes, _H2D, dev, stream, pinned)
    return out


def transfer_buffer_cpu(buffer) -> CPUBuffer:
    """Move a C-contiguous device buffer (CUDABuffer, device tensor or any
    ``__cuda_array_interface__`` object) to host memory."""
    # the copy is issued on the stream the buffer was produced on (its
    # `stream`, or torch's current stream for a tensor) and that stream is
    # synchronised, so pending producers are ordered before it
    if isinstance(buffer, torch.Tensor):
        if buffer.device.type != "cuda":
            raise TypeError("transfer_buffer_cpu expects a device buffer")
        t = buffer.contiguous()
        ptr, shape, dtype, dev = t.data_ptr(), tuple(t.shape), t.dtype, t.device.index
        stream = torch.cuda.current_stream(t.device).cuda_stream
    elif isinstance(buffer, CUDABuffer):
        ptr, shape, dtype, dev = buffer.data_ptr(), buffer.shape, buffer.dtype, buffer.device_index
        stream = int(buffer._stream)
    elif (iface := getattr(buffer, "__cuda_array_interface__", None)) is not None:
        if iface.get("strides") is not None:
            raise RuntimeError("transfer_buffer_cpu expects a C-contiguous buffer")
        ptr, shape = iface["data"][0], tuple(iface["shape"])
        dtype = torch_dtype_of(np.dtype(iface["typestr"]))
        dev = getattr(buffer, "device_index", torch.cuda.current_device())
        stream = int(iface.get("stream") or 0)
    else:
        raise TypeError(f"expected a device buffer, found {type(buffer)}")
    host_dtype = torch.int16 if dtype == torch.bfloat16 else dtype
    host = torch.empty(shape, dtype=host_dtype)
    nbytes = host.numel() * _itemsize(dtype)
    _copy(host.data_ptr(), ptr, nbytes, _D2H, dev, stream, True)
    if dtype == torch.bfloat16:
        return CPUBuffer(host.numpy().view(np.uint16), dtype=torch.bfloat16)
    return CPUBuffer(host.numpy())


def _recursive_apply(fn, obj):
    """Apply ``fn`` to the leaves of lists, tuples, namedtuples, dicts and
    dataclasses, rebuilding the containers (reference _transfer.py)."""
    cls = type(obj)
    if isinstance(obj, list):
        return cls(_recursive_apply(fn, v) for v in obj)
    if isinstance(obj, tuple):
        if hasattr(obj, "_fields"):
            return cls(**{k: _recursive_apply(fn, v) for k, v in obj._asdict().items()})
        return cls(_recursive_apply(fn, v) for v in obj)
    if isinstance(obj, defaultdict):
        return cls(obj.default_factory, {k: _recursive_apply(fn, v) for k, v in obj.items()})
    if isinstance(obj, Mapping):
        return cls({k: _recursive_apply(fn, v) for k, v in obj.items()})
    if is_dataclass(obj) and not isinstance(obj, type):
        new = cls(**{f.name: _recursive_apply(fn, getattr(obj, f.name))
                     for f in fields(obj) if f.init})
        for f in fields(obj):
            if not f.init:
                setattr(new, f.name, _recursive_apply(fn, getattr(obj, f.name)))
        return new
    return fn(obj)


class _TensorTransfer:
    def __init__(self, device: torch.device, num_caches: int):
        self._device = device
        self._stream = torch.cuda.Stream(device)
        self._cache: list = [None] * num_caches

    def __call__(self, batch):
        pinned = []

        def move(x):
            if isinstance(x, torch.Tensor) and x.is_cpu:
                p = x.pin_memory()
                pinned.append(p)
                return p.to(self._device, non_blocking=True)
            return x

        with torch.cuda.stream(self._stream):
            batch = _recursive_apply(move, batch)
        self._stream.synchronize()
        self._cache.append(batch)
        self._cache.pop(0)
        return batch


_TLS = threading.local()


def transfer_tensor(batch, /, *, num_caches: int = 4):
    """Move the CPU tensors of a (nested) batch to ``cuda:$LOCAL_RANK`` on a
    dedicated per-thread stream: pin, copy non-blocking, synchronise.  The
    last ``num_caches`` batches stay referenced so the caller's consumer
    stream cannot see their memory recycled early."""
    if not hasattr(_TLS, "transfer"):
        rank = int(os.environ.get("LOCAL_RANK", "0"))
        if rank >= torch.cuda.device_count():
            raise RuntimeError("The local rank is larger than the number of available GPUs.")
        _TLS.transfer = _TensorTransfer(torch.device(f"cuda:{rank}"), num_caches)
    return _TLS.transfer(batch)
