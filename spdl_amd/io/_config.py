"""Device configuration (mirror of spdl.io.cuda_config, reference
src/spdl/io/_config.py:115-178 and src/libspdl/cuda/types.h:22-39)."""

from __future__ import annotations

from dataclasses import dataclass
from typing import Callable

# HIP defines the same per-thread default stream sentinel as CUDA:
# #define hipStreamPerThread ((hipStream_t)2)  (hip_runtime_api.h)
STREAM_PER_THREAD = 0x2

Allocator = tuple[Callable[[int, int, int], int], Callable[[int], None]]


@dataclass(frozen=True)
class CUDAConfig:
    """Target HIP device, stream handle (``uintptr_t``; ``0x2`` = per-thread
    default stream, ``0`` = legacy default stream) and an optional allocator
    pair ``(alloc(size, device, stream) -> ptr, free(ptr))``."""

    device_index: int
    stream: int = STREAM_PER_THREAD
    allocator: Allocator | None = None


def cuda_config(
    device_index: int,
    stream: int = STREAM_PER_THREAD,
    allocator: Allocator | None = None,
) -> CUDAConfig:
    """Specify the device, stream and memory allocator used for decoding.

    Same signature and meaning as ``spdl.io.cuda_config``.  On ROCm the
    ``torch.cuda`` namespace is HIP, so ``torch.cuda.current_stream().cuda_stream``
    and ``torch.cuda.caching_allocator_alloc/delete`` work unchanged."""
    if allocator is not None:
        if len(allocator) != 2 or not all(callable(f) for f in allocator):
            raise TypeError("allocator must be a pair of callables (alloc, free)")
    return CUDAConfig(int(device_index), int(stream), allocator)
