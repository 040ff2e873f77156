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


def transfer_buffer_cpu(buffer, *, storage: CPUStorage | None = None) -> CPUBuffer:
    """Move a C-contiguous device buffer (CUDABuffer, device tensor or any
    ``__cuda_array_interface__`` object) to host memory.  ``storage`` (an
    extension: the reference always allocates) receives the bytes instead of
    a fresh allocation; it must be large enough."""
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
    if storage is None:
        host = torch.empty(shape, dtype=host_dtype)
    else:
        need = int(np.prod(shape)) * _itemsize(dtype)
        if storage.size < need:
            raise RuntimeError(f"The provided storage does not have enough capacity. "
                               f"({storage.size} < {need})")
        host = storage._tensor[:need].view(host_dtype).view(shape)
    nbytes = host.numel() * _itemsize(dtype)
    _copy(host.data_ptr(), ptr, nbytes, _D2H, dev, stream, True)
    if dtype == torch.bfloat16:
        return CPUBuffer(host.numpy().view(np.uint16), dtype=torch.bfloat16, storage=storage)
    return CPUBuffer(host.numpy(), storage=storage)


# ---- transfer_tensor: one coalesced pinned H2D per batch -----------------------
#
# The reference (src/spdl/io/_transfer.py:82-177) pins and copies each CPU
# tensor of a nested batch separately on a per-thread stream.  Here the
# batch is flattened, every CPU tensor is packed into ONE page-locked staging
# area (a per-thread ring of `num_caches` slots), the staging goes to the
# device in ONE spdl_hj_copy (hipMemcpyAsync on the thread's stream + sync),
# and the returned device tensors are views of that one allocation.  The
# last `num_caches` device allocations stay referenced, the reference's
# guard against the caching allocator handing their memory to another
# stream while a consumer still reads it
# (docs/source/notes/pytorch_cuda_race_condition.rst).


def _flatten(obj, leaves: list):
    """Leaves of lists / tuples / namedtuples / mappings / dataclasses into
    `leaves`; returns a function rebuilding the same structure from an
    iterator over (possibly replaced) leaves."""
    cls = type(obj)
    if is_dataclass(obj) and not isinstance(obj, type):
        parts = [(f.name, f.init, _flatten(getattr(obj, f.name), leaves)) for f in fields(obj)]

        def build_dc(it):
            vals = [(n, init, b(it)) for n, init, b in parts]
            new = cls(**{n: v for n, init, v in vals if init})
            for n, init, v in vals:
                if not init:
                    setattr(new, n, v)
            return new

        return build_dc
    if isinstance(obj, Mapping):
        items = [(k, _flatten(v, leaves)) for k, v in obj.items()]
        if isinstance(obj, defaultdict):
            return lambda it: cls(obj.default_factory, {k: b(it) for k, b in items})
        return lambda it: cls({k: b(it) for k, b in items})
    if isinstance(obj, (list, tuple)):
        items = [_flatten(v, leaves) for v in obj]
        if hasattr(obj, "_fields"):  # namedtuple
            return lambda it: cls(*[b(it) for b in items])
        return lambda it: cls([b(it) for b in items])
    leaves.append(obj)
    return lambda it: next(it)


class _BatchMover:
    """Per-thread mover: a stream, a ring of pinned staging slots and the
    device allocations of the last `num_caches` batches."""

    _ALIGN = 256

    def __init__(self, device: int, num_caches: int):
        self.device = device
        self.stream = torch.cuda.Stream(torch.device("cuda", device))
        self.ring: list = [None] * max(1, num_caches)
        self.keep: list = [None] * max(1, num_caches)
        self.k = 0

    def __call__(self, batch):
        leaves: list = []
        rebuild = _flatten(batch, leaves)
        moved = [i for i, x in enumerate(leaves) if isinstance(x, torch.Tensor) and x.is_cpu]
        if not moved:
            return batch
        offs, total = [], 0
        for i in moved:
            offs.append(total)
            nb = leaves[i].numel() * leaves[i].element_size()
            total += (nb + self._ALIGN - 1) // self._ALIGN * self._ALIGN
        slot = self.k % len(self.ring)
        self.k += 1
        stage = self.ring[slot]
        if stage is None or stage.numel() < total:
            stage = self.ring[slot] = torch.empty(max(total, 1), dtype=torch.uint8,
                                                  pin_memory=True)
        for i, o in zip(moved, offs):  # pack (torch's multi-threaded copy)
            t = leaves[i].contiguous()
            nb = t.numel() * t.element_size()
            stage[o:o + nb].copy_(t.reshape(-1).view(torch.uint8))
        # allocate on the copy stream: the caching allocator then only hands
        # out a block whose last use was ordered on this stream, never one a
        # kernel queued on the default stream may still be reading or writing
        # (the reference allocates under `with torch.cuda.stream(...)` too)
        with torch.cuda.stream(self.stream):
            dev = torch.empty(max(total, 1), dtype=torch.uint8, device=f"cuda:{self.device}")
        _copy(dev.data_ptr(), stage.data_ptr(), total, _H2D, self.device,
              self.stream.cuda_stream, True)
        self.keep[slot] = dev
        out = list(leaves)
        for i, o in zip(moved, offs):
            t = leaves[i]
            nb = t.numel() * t.element_size()
            out[i] = dev[o:o + nb].view(t.dtype).view(t.shape)
        return rebuild(iter(out))


_TLS = threading.local()


def transfer_tensor(batch, /, *, num_caches: int = 4):
    """Move every CPU tensor of a (nested) batch to ``cuda:$LOCAL_RANK``
    (reference src/spdl/io/_transfer.py:82-177): one coalesced pinned
    host-to-device copy per batch on this thread's stream, complete when the
    call returns; the result has the batch's structure with device tensors
    in place of the CPU ones."""
    mover = getattr(_TLS, "mover", None)
    if mover is None:
        rank = int(os.environ.get("LOCAL_RANK", "0"))
        count = torch.cuda.device_count()
        if rank >= count:
            raise RuntimeError(f"LOCAL_RANK={rank} but only {count} GPU(s) are visible.")
        mover = _TLS.mover = _BatchMover(rank, num_caches)
    return mover(batch)
