"""to_torch / to_numpy (mirror of reference src/spdl/io/_convert.py:100-153)."""

from __future__ import annotations

import numpy as np
import torch

from ._buffer import CPUBuffer, CUDABuffer


class _Iface:
    """An interface dict re-exported with another typestr (bfloat16 buffers
    are handed to torch as int16 and viewed back, zero-copy)."""

    def __init__(self, iface: dict, typestr: str):
        self.__cuda_array_interface__ = {**iface, "typestr": typestr}


def to_torch(buffer) -> torch.Tensor:
    """Zero-copy conversion to a torch tensor."""
    if isinstance(buffer, CUDABuffer) and buffer._tensor is not None:
        return buffer._tensor
    if (iface := getattr(buffer, "__cuda_array_interface__", None)) is not None:
        if any(s == 0 for s in iface.get("shape", [])):
            raise ValueError("0-element array is not supported.")
        ptr = iface["data"][0]
        dev = f"cuda:{buffer.device_index}"
        if iface["typestr"] == "<V2":  # bfloat16
            t = torch.as_tensor(_Iface(iface, "<i2"), device=dev).view(torch.bfloat16)
        else:
            t = torch.as_tensor(buffer, device=dev)
        if t.data_ptr() != ptr:
            raise RuntimeError(
                "[INTERNAL ERROR] Failed to perform zero-copy conversion to PyTorch Tensor. "
                f"src: {ptr}, dst: {t.data_ptr()}, device: {buffer.device_index}"
            )
        return t
    if isinstance(buffer, CPUBuffer):
        t = torch.from_numpy(buffer._array)
        return t.view(buffer.dtype) if t.dtype != buffer.dtype else t
    return torch.as_tensor(np.array(buffer, copy=False))


def to_numpy(buffer) -> np.ndarray:
    """Zero-copy conversion of a CPU buffer to a numpy array (bfloat16:
    the uint16 bit patterns)."""
    if isinstance(buffer, CPUBuffer):
        return buffer._array
    if not hasattr(buffer, "__array_interface__"):
        raise RuntimeError("The given object does not have `__array_interface__` attribute.")
    return np.array(buffer, copy=False)
