"""Tar ingest for the decode stage (BASELINE configs[4]).

``iter_tarfile`` mirrors the reference's operator
(src/spdl/io/_tar.py:33-82, parser src/spdl/io/lib/archive/tar_iterator.cpp):
bytes / memoryview in -> ``(name, memoryview)`` zero-copy views; a file-like
object in -> ``(name, bytes)``.

``TarImageStream`` is the streaming decode path the reference assembles from
``iter_tarfile`` + ``load_image_batch_nvjpeg`` + ``transfer_buffer``; here it
is one pipeline over the native staging ring (include/spdl_hipjpeg.h):

  archive (file: multi-threaded pread / bytes: multi-threaded memcpy)
    -> pinned ring slot (a run of consecutive members, copied as ONE region:
       tar payloads are 512-byte aligned, so no repacking)
    -> one hipMemcpyAsync on the decoder's copy stream
    -> the decode kernels on the compute stream
  while the host already fills the next slot.
"""

from __future__ import annotations

import collections
import mmap
import os
from collections.abc import Callable, Iterator

import numpy as np
import torch

from .. import _lib
from .._lib import Output
from ._config import CUDAConfig

_IMAGE_EXT = (".jpg", ".jpeg", ".jpe", ".jfif")


def iter_tarfile(src) -> Iterator:
    """Parse a TAR archive and yield ``(path, contents)`` per regular file.

    Same contract as the reference (``src/spdl/io/_tar.py:33-82``): for
    ``bytes``/``memoryview`` input the contents are zero-copy memoryviews of
    it; for a file-like object (``read(n)`` only) they are ``bytes``.
    """
    if isinstance(src, (bytes, bytearray, memoryview)):
        mv = memoryview(src).cast("B")
        members, _ = _lib.tar_index(mv)
        for name, off, size in members:
            yield name, mv[off: off + size]
        return
    yield from _iter_filelike(src)


def _iter_filelike(f) -> Iterator[tuple[str, bytes]]:
    # The native walk runs over a window [pos, len(buf)); it only reports
    # members whose payload is complete inside the window.
    buf = bytearray()
    pos = 0
    eof = False
    while True:
        if pos < len(buf):
            members, nxt = _lib.tar_index(memoryview(buf)[pos:], max_entries=1)
        else:
            members, nxt = [], 0
        if members:
            name, off, size = members[0]
            yield name, bytes(buf[pos + off: pos + off + size])
            pos += nxt
            continue
        if eof:
            return
        chunk = f.read(max(1 << 22, len(buf) - pos))
        if not chunk:
            eof = True
        else:
            del buf[:pos]
            pos = 0
            buf += chunk


class TarImageStream:
    """Decode every JPEG member of a tar archive on one GPU, batch by batch.

    Args:
        src: path of the archive, or its bytes.
        batch_size: images per batch (the last one may be short).
        device_config: :func:`spdl_amd.io.cuda_config` (device + stream).
        output: :class:`spdl_amd._lib.Output` (default: RGB24 224x224, the
            ``load_image_batch(width=224, height=224)`` filter chain).
        select: predicate on member names (default: JPEG extensions).
        depth: batches in flight, each on a decode pipeline lane of its own
            (1-8; the native ring has 10 staging slots).

    Iterating yields ``(names, tensor)`` where ``tensor`` is a device tensor
    ``[B, h, w, 3]`` / ``[B, 3, h, w]`` complete on the stream it was made on
    (the iterator waits for each batch before yielding it).
    """

    def __init__(self, src, *, batch_size: int, device_config: CUDAConfig,
                 output: Output | None = None,
                 select: Callable[[str], bool] | None = None, depth: int = 4):
        if device_config is None:
            raise ValueError("device_config must be provided.")
        if batch_size <= 0:
            raise ValueError("batch_size must be positive")
        self.cfg = device_config
        self.batch_size = int(batch_size)
        self.output = output or Output(pix_fmt="rgb24", resize=True, fit_w=224, fit_h=224,
                                       aspect="decrease", pad_w=224, pad_h=224)
        self.depth = max(1, min(int(depth), 8))
        sel = select or (lambda n: n.lower().endswith(_IMAGE_EXT))
        self._fd = -1
        self._mm = None
        if isinstance(src, (str, os.PathLike)):
            self._fd = os.open(src, os.O_RDONLY)
            size = os.fstat(self._fd).st_size
            self._mm = mmap.mmap(self._fd, size, prot=mmap.PROT_READ) if size else None
            view = np.frombuffer(self._mm, np.uint8) if self._mm else np.zeros(0, np.uint8)
            self._bytes = None
        else:
            view = np.frombuffer(memoryview(src).cast("B"), np.uint8)
            self._bytes = view
        members, _ = _lib.tar_index(view)
        self.members = [m for m in members if sel(m[0])]
        self._dec = _lib.Decoder(device_config.device_index)
        # one pipeline lane per batch in flight: later batches' kernels share
        # the CUs with earlier batches' latency-bound entropy decode
        # (completion is tracked per ticket)
        self._dec.set_param("lanes", self.depth)
        h, w = self._out_hw(view)
        self._shape = (3, h, w) if self.output.planar else (h, w, 3)
        self._dtype = self.output.torch_dtype
        del view

    def _out_hw(self, view) -> tuple[int, int]:
        if not self.members:
            return 0, 0
        name, off, size = self.members[0]
        info = _lib.get_image_info(view[off: off + min(size, 1 << 16)].tobytes()
                                   if size > 0 else b"")
        ow, oh = _lib.output_size(info.width, info.height, self.output)
        return oh, ow

    def __len__(self) -> int:
        return (len(self.members) + self.batch_size - 1) // self.batch_size

    def batches(self) -> Iterator[list]:
        for i in range(0, len(self.members), self.batch_size):
            yield self.members[i: i + self.batch_size]

    def _submit(self, group, stream):
        base = group[0][1] & ~511  # payloads are 512-byte aligned in a tar
        end = group[-1][1] + group[-1][2]
        region = end - base
        ptr, ticket = self._dec.staging_acquire(region)
        if self._bytes is not None:
            self._dec.staging_fill(ticket, 0, self._bytes.ctypes.data + base, region)
        else:
            self._dec.staging_read(ticket, 0, self._fd, base, region)
        out = torch.empty((len(group),) + self._shape, dtype=self._dtype,
                          device=f"cuda:{self.cfg.device_index}")
        self._dec.decode_staged(ticket, region, [m[1] - base for m in group],
                                [m[2] for m in group], self.output, out.data_ptr(),
                                out.numel() * out.element_size(), stream=stream, sync=False)
        return ticket, out, [m[0] for m in group]

    def __iter__(self) -> Iterator[tuple[list[str], torch.Tensor]]:
        stream = int(self.cfg.stream)
        inflight = collections.deque()
        for group in self.batches():
            inflight.append(self._submit(group, stream))
            if len(inflight) > self.depth:
                ticket, out, names = inflight.popleft()
                self._dec.wait(ticket, len(names))
                yield names, out
        while inflight:
            ticket, out, names = inflight.popleft()
            self._dec.wait(ticket, len(names))
            yield names, out

    def close(self) -> None:
        if self._dec is not None:
            self._dec.close()
            self._dec = None
        if self._mm is not None:
            self._mm.close()
            self._mm = None
        if self._fd >= 0:
            os.close(self._fd)
            self._fd = -1

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
