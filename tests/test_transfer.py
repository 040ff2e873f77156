"""Host <-> device transfer surface (reference tests/cuda/pin_memory_test.py,
tests/cuda/buffer_transfer_test.py, tests/cuda/transfer_tensor_test.py).

CPU tests: storage validation and convert_array; GPU tests: round trips
through the native copy entry point for each dtype, pinned and pageable
sources, the allocator pair, and decoded buffers moved back to the host."""

import gc

import numpy as np
import pytest
import torch

import spdl_amd.io as sio
from tests.cases import case


@pytest.mark.parametrize("pin_memory", [False, True])
def test_cpu_storage_invalid_size(pin_memory):
    with pytest.raises(RuntimeError):
        sio.cpu_storage(0, pin_memory=pin_memory)
    with pytest.raises(TypeError):
        sio.cpu_storage(-1, pin_memory=pin_memory)


def test_convert_array_into_storage():
    vals = np.arange(0, 10)
    storage = sio.cpu_storage(vals.nbytes, pin_memory=False)
    buf = sio.convert_array(vals, storage=storage)
    arr = sio.to_numpy(buf)
    assert arr.dtype == np.int64 and arr.shape == (10,)
    np.testing.assert_array_equal(arr, vals)
    assert arr.ctypes.data == storage.data_ptr()  # lives in the storage
    assert sio.to_torch(buf).dtype == torch.int64


def test_convert_array_storage_too_small():
    vals = np.arange(0, 10)
    storage = sio.cpu_storage(vals.nbytes // 2, pin_memory=False)
    with pytest.raises(RuntimeError):
        sio.convert_array(vals, storage=storage)


def test_convert_array_without_storage_copies():
    vals = np.arange(12, dtype=np.float32).reshape(3, 4)
    buf = sio.convert_array(vals)
    vals[0, 0] = 99
    assert sio.to_numpy(buf)[0, 0] == 0
    assert buf.shape == (3, 4)


def test_buffer_typestr():
    for dt, ts in [(torch.uint8, "|u1"), (torch.float16, "<f2"), (torch.int64, "<i8"),
                   (torch.float32, "<f4"), (torch.bfloat16, "<V2")]:
        b = sio.CUDABuffer(None, ptr=1, shape=(2,), dtype=dt)
        assert b.__cuda_array_interface__["typestr"] == ts


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [np.uint8, np.int16, np.int32, np.int64, np.float32, np.float64])
@pytest.mark.parametrize("pin_memory", [False, True])
def test_transfer_round_trip(dtype, pin_memory):
    rng = np.random.default_rng(7)
    vals = (rng.standard_normal((5, 7, 3)) * 100).astype(dtype)
    storage = sio.cpu_storage(vals.nbytes, pin_memory=pin_memory)
    buf = sio.convert_array(vals, storage=storage)
    stream = torch.cuda.Stream(device=0)
    cfg = sio.cuda_config(device_index=0, stream=stream.cuda_stream)
    cuda_buf = sio.transfer_buffer(buf, device_config=cfg)
    t = sio.to_torch(cuda_buf)
    assert t.is_cuda and t.device == torch.device("cuda:0")
    assert t.dtype == torch.from_numpy(vals).dtype and tuple(t.shape) == vals.shape
    np.testing.assert_array_equal(t.cpu().numpy(), vals)
    back = sio.to_numpy(sio.transfer_buffer_cpu(cuda_buf))
    np.testing.assert_array_equal(back, vals)


@pytest.mark.gpu
def test_transfer_plain_array_and_tensor():
    vals = np.arange(1000, dtype=np.int32)
    t = sio.to_torch(sio.transfer_buffer(vals, device_config=sio.cuda_config(0)))
    assert torch.equal(t.cpu(), torch.from_numpy(vals))
    src = torch.arange(64, dtype=torch.float16).reshape(8, 8).t()  # non-contiguous
    t2 = sio.to_torch(sio.transfer_buffer(src, device_config=sio.cuda_config(0)))
    assert torch.equal(t2.cpu(), src.contiguous())
    back = sio.to_numpy(sio.transfer_buffer_cpu(t2))
    np.testing.assert_array_equal(back, src.contiguous().numpy())


@pytest.mark.gpu
def test_transfer_with_allocator():
    calls = {"alloc": 0, "free": 0}

    def alloc(size, device, stream):
        calls["alloc"] += 1
        return torch.cuda.caching_allocator_alloc(size, device, stream)

    def free(ptr):
        calls["free"] += 1
        torch.cuda.caching_allocator_delete(ptr)

    def run():
        vals = np.arange(300, dtype=np.int64).reshape(3, 100)
        cfg = sio.cuda_config(0, allocator=(alloc, free))
        buf = sio.transfer_buffer(sio.convert_array(vals), device_config=cfg)
        assert calls["alloc"] == 1 and calls["free"] == 0
        t = sio.to_torch(buf)
        assert t.data_ptr() == buf.data_ptr()
        np.testing.assert_array_equal(t.cpu().numpy(), vals)
        del t, buf

    run()
    gc.collect()
    assert calls["free"] == 1


@pytest.mark.gpu
@pytest.mark.parametrize("norm_dtype", ["float16", "bfloat16"])
def test_transfer_decoded_batch_to_host(norm_dtype):
    datas = [case(n) for n in ("q90_420", "q90_444", "odd_227x333", "gray")]
    cfg = sio.cuda_config(0)
    buf = sio.load_image_batch(datas, width=32, height=24, device_config=cfg, normalize=True,
                               norm_dtype=norm_dtype)
    dev = sio.to_torch(buf)
    host = sio.transfer_buffer_cpu(buf)
    assert host.dtype == dev.dtype
    assert torch.equal(sio.to_torch(host), dev.cpu())


@pytest.mark.gpu
def test_transfer_tensor_nested():
    from dataclasses import dataclass

    @dataclass
    class Batch:
        x: torch.Tensor
        meta: dict

    b = Batch(torch.arange(6).reshape(2, 3), {"y": [torch.ones(4), 3], "s": "k"})
    out = sio.transfer_tensor(b)
    assert out.x.is_cuda and out.meta["y"][0].is_cuda
    assert out.meta["y"][1] == 3 and out.meta["s"] == "k"
    assert torch.equal(out.x.cpu(), b.x)


def test_transfer_tensor_structure_roundtrip():
    """The batch flattening used by transfer_tensor rebuilds every container
    kind the reference handles (list, tuple, namedtuple, defaultdict,
    Mapping, dataclass incl. non-init fields) -- CPU only."""
    from collections import defaultdict, namedtuple
    from dataclasses import dataclass, field

    from spdl_amd.io._transfer import _flatten

    P = namedtuple("P", "a b")

    @dataclass
    class D:
        x: object
        y: list
        z: int = field(init=False, default=0)

    dd = defaultdict(list, {"k": [1, (2, 3)]})
    d = D(P(1, [2, 3]), [dd, {"m": 4}])
    d.z = 5
    leaves = []
    build = _flatten(d, leaves)
    assert leaves == [1, 2, 3, 1, 2, 3, 4, 5]
    out = build(iter(v * 10 for v in leaves))
    assert isinstance(out, D) and isinstance(out.x, P) and isinstance(out.y[0], defaultdict)
    assert out.x == P(10, [20, 30]) and out.y[0]["k"] == [10, (20, 30)] and out.y[1] == {"m": 40}
    assert out.z == 50 and out.y[0].default_factory is list


@pytest.mark.gpu
def test_transfer_tensor_dtypes_one_copy():
    ts = [torch.arange(10, dtype=torch.bfloat16), torch.tensor([True, False, True]),
          torch.randn(3, 5), torch.tensor(7), torch.randint(0, 255, (33,), dtype=torch.uint8)]
    out = sio.transfer_tensor(ts)
    for a, b in zip(ts, out):
        assert b.is_cuda and b.dtype == a.dtype and b.shape == a.shape
        assert torch.equal(b.cpu(), a)
    # views of one allocation
    base = {o.untyped_storage().data_ptr() for o in out}
    assert len(base) == 1
