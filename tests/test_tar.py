"""iter_tarfile (native tar walk) vs Python's tarfile on the same archives.

Mirrors the reference's tests for its parser (tests/io/tar_iterator_test.py
compares spdl.io.iter_tarfile against tarfile): ustar, GNU long names ('L'),
pax path records ('x'), directories / symlinks skipped, empty archives,
both the bytes (zero-copy memoryview) and the file-like (bytes) forms.
Host-only: runs without a GPU.
"""

import io
import tarfile

import pytest

import spdl_amd.io as sio
from spdl_amd import _lib


def _make_tar(entries, fmt=tarfile.USTAR_FORMAT) -> bytes:
    b = io.BytesIO()
    with tarfile.open(fileobj=b, mode="w", format=fmt) as t:
        for name, data in entries:
            if data is None:  # directory
                ti = tarfile.TarInfo(name)
                ti.type = tarfile.DIRTYPE
                t.addfile(ti)
            elif isinstance(data, str):  # symlink -> target
                ti = tarfile.TarInfo(name)
                ti.type = tarfile.SYMTYPE
                ti.linkname = data
                t.addfile(ti)
            else:
                ti = tarfile.TarInfo(name)
                ti.size = len(data)
                t.addfile(ti, io.BytesIO(data))
    return b.getvalue()


def _ref(data: bytes):
    with tarfile.open(fileobj=io.BytesIO(data)) as t:
        return [(m.name, t.extractfile(m).read()) for m in t.getmembers() if m.isfile()]


ENTRIES = [
    ("a.jpg", b"x" * 100),
    ("dir", None),
    ("dir/b.jpg", bytes(range(256)) * 4),      # exactly 1024 bytes: no padding
    ("link", "a.jpg"),
    ("empty.txt", b""),
    ("c/d/e.bin", b"\xff\xd8" + b"\x00" * 511),  # 513 bytes
]


@pytest.mark.parametrize("fmt", [tarfile.USTAR_FORMAT, tarfile.GNU_FORMAT, tarfile.PAX_FORMAT])
def test_bytes_matches_tarfile(fmt):
    data = _make_tar(ENTRIES, fmt)
    hyp = [(n, bytes(v)) for n, v in sio.iter_tarfile(data)]
    assert hyp == _ref(data)


@pytest.mark.parametrize("fmt", [tarfile.GNU_FORMAT, tarfile.PAX_FORMAT])
def test_long_names(fmt):
    long = "deep/" * 30 + "name_" + "y" * 120 + ".jpg"
    data = _make_tar([(long, b"abc"), ("short.jpg", b"de")], fmt)
    hyp = [(n, bytes(v)) for n, v in sio.iter_tarfile(data)]
    assert hyp == [(long, b"abc"), ("short.jpg", b"de")] == _ref(data)


def test_memoryview_is_zero_copy():
    data = bytearray(_make_tar(ENTRIES))
    views = [v for _, v in sio.iter_tarfile(data)]
    assert isinstance(views[0], memoryview)
    off = _lib.tar_index(data)[0][0][1]
    data[off] = ord("Z")  # a write to the archive shows through the view
    assert bytes(views[0][:1]) == b"Z"


def test_filelike_matches_tarfile():
    entries = [(f"f{i}.jpg", bytes([i]) * (i * 50_000 + 7)) for i in range(40)]
    data = _make_tar(entries, tarfile.GNU_FORMAT)

    class Reader:  # only read(n), as the reference requires
        def __init__(self, b):
            self.f = io.BytesIO(b)

        def read(self, n=-1):
            return self.f.read(n)

    hyp = list(sio.iter_tarfile(Reader(data)))
    assert all(isinstance(v, bytes) for _, v in hyp)
    assert hyp == _ref(data)


def test_empty_and_garbage():
    assert list(sio.iter_tarfile(_make_tar([]))) == []
    assert list(sio.iter_tarfile(b"")) == []
    assert list(sio.iter_tarfile(b"\x01" * 4096)) == []  # invalid headers are skipped


def test_truncated_member_ends_the_walk():
    data = _make_tar([("a", b"1" * 600), ("b", b"2" * 600)])
    # cut inside b's payload: a is yielded, b is dropped
    cut = data[: _lib.tar_index(data)[0][1][1] + 100]
    assert [n for n, _ in sio.iter_tarfile(cut)] == ["a"]


def test_resume_position():
    data = _make_tar([(f"m{i}", b"q" * (i + 1) * 300) for i in range(10)])
    first, pos = _lib.tar_index(data, max_entries=4)
    rest, end = _lib.tar_index(data, start=pos)
    assert [m[0] for m in first + rest] == [f"m{i}" for i in range(10)]
    assert end == len(data)
