"""Corrupt-file policy of load_image_batch (reference src/spdl/io/_composite.py:
358-465 strict handling; FFmpeg mjpeg at src/libspdl/core/detail/ffmpeg/
decoder.cpp:53-55,76-78).

FFmpeg's mjpeg decoder often conceals a damaged scan and returns a frame,
which SPDL then keeps with a warning; this decoder fails the image instead
(SPDL_HJ_ERR_TRUNCATED / BAD_HUFFMAN / BAD_RESTART), exactly where the oracle
(oracle/jpeg_oracle.c, the restated sequential decoder) fails it.  These
tests pin which images of a mixed batch survive `strict=False` -- the
oracle's survivors, in order, each bit-exact -- and that `strict=True`
raises.  The concealment itself is unpinned.
"""

import numpy as np
import pytest

import spdl_amd.io as sio
from tests import cases

pytestmark = pytest.mark.gpu


def _batch():
    good = [cases.case("q75_420"), cases.case("q90_420")]
    bad = [cases.corrupt_scan(s) for s in range(8)] + [cases.truncated()]
    # good and damaged files interleaved (every file 240x320 or 480x640 ->
    # 224x224 pad, the bench's output)
    srcs = []
    for i, b in enumerate(bad):
        srcs.append(good[i % 2])
        srcs.append(b)
    return srcs


def _ref(oracle, d):
    rs = oracle.Resize(fit_w=224, fit_h=224, aspect="decrease", pad_w=224, pad_h=224)
    try:
        return oracle.decode_resize(d, rs, pix_fmt="rgb24")
    except oracle.OracleError:
        return None


def test_non_strict_keeps_the_oracles_survivors(oracle):
    srcs = _batch()
    refs = [_ref(oracle, d) for d in srcs]
    survivors = [r for r in refs if r is not None]
    assert 0 < len(survivors) < len(srcs)  # the batch mixes both outcomes
    cfg = sio.cuda_config(device_index=0)
    buf = sio.load_image_batch(srcs, width=224, height=224, pix_fmt="rgb24", device_config=cfg,
                               strict=False)
    hyp = sio.to_torch(buf).cpu().numpy()
    assert hyp.shape == (len(survivors), 224, 224, 3)
    for h, r in zip(hyp, survivors):
        np.testing.assert_array_equal(h, r, strict=True)


def test_strict_raises_on_a_damaged_file(oracle):
    srcs = _batch()
    assert any(_ref(oracle, d) is None for d in srcs)
    with pytest.raises(RuntimeError):
        sio.load_image_batch(srcs, width=224, height=224, pix_fmt="rgb24",
                             device_config=sio.cuda_config(device_index=0), strict=True)


@pytest.mark.parametrize("seed", range(8))
def test_which_damaged_files_fail(oracle, seed):
    """Per file: the decoder fails exactly the files the oracle fails, and a
    damaged file that both decode gives the oracle's pixels."""
    d = cases.corrupt_scan(seed)
    ref = _ref(oracle, d)
    cfg = sio.cuda_config(device_index=0)
    if ref is None:
        with pytest.raises(RuntimeError, match="Failed to"):
            sio.load_image_batch([d], width=224, height=224, device_config=cfg, strict=True)
    else:
        out = sio.to_torch(sio.load_image_batch([d], width=224, height=224, device_config=cfg))
        np.testing.assert_array_equal(out.cpu().numpy()[0], ref, strict=True)
