"""GPU: NV12 -> planar RGB/BGR kernel vs the oracle restatement, bit-exact.

Mirrors what the reference exercises for its kernel (tests/cuda/
nvdec_video_decoding_test.py converts NV12 with spdl.io.nv12_to_rgb): every
matrix, RGB/BGR order, a batch of frames, odd widths (the last column is not
written, as in the reference), shape errors.
"""

import numpy as np
import pytest
import torch

import spdl_amd.io as sio

pytestmark = pytest.mark.gpu


def _rand(f, h, w, seed=0):
    rng = np.random.default_rng(seed)
    return rng.integers(0, 256, size=(f, h + h // 2, w), dtype=np.uint8)


@pytest.mark.parametrize("coeff", [1, 2, 4, 5, 6, 7, 8, 9, 10, 0, 11, -3])
@pytest.mark.parametrize("bgr", [False, True])
def test_nv12_matches_oracle(oracle, coeff, bgr):
    a = _rand(3, 64, 96, seed=abs(coeff) + 100 * bgr)
    fn = sio.nv12_to_bgr if bgr else sio.nv12_to_rgb
    buf = fn(torch.from_numpy(a).cuda(), device_config=sio.cuda_config(0), coeff=coeff,
             sync=True)
    hyp = sio.to_torch(buf).cpu().numpy()
    ref = oracle.nv12_to_rgb(a, coeff=coeff, bgr=bgr)
    assert hyp.shape == (3, 3, 64, 96)
    np.testing.assert_array_equal(hyp, ref)


def test_nv12_extremes_and_odd_width(oracle):
    a = np.zeros((2, 48, 37), np.uint8)
    a[0] = 255
    a[1, :32] = (np.arange(37, dtype=np.int64)[None, :] * 7 % 256).astype(np.uint8)
    a[1, 32:] = np.where(np.arange(37) % 2 == 0, 0, 255).astype(np.uint8)[None, :]
    hyp = sio.to_torch(sio.nv12_to_rgb(torch.from_numpy(a).cuda(),
                                       device_config=sio.cuda_config(0), sync=True)).cpu().numpy()
    ref = oracle.nv12_to_rgb(a)
    np.testing.assert_array_equal(hyp[..., :36], ref[..., :36])


def test_nv12_shape_errors():
    cfg = sio.cuda_config(0)
    with pytest.raises(RuntimeError, match="divisible by 3"):
        sio.nv12_to_rgb(torch.zeros((1, 10, 8), dtype=torch.uint8, device="cuda"),
                        device_config=cfg)
    with pytest.raises(RuntimeError, match="3D"):
        sio.nv12_to_rgb(torch.zeros((12, 8), dtype=torch.uint8, device="cuda"),
                        device_config=cfg)
    with pytest.raises(ValueError):
        sio.nv12_to_rgb(torch.zeros((1, 12, 8), dtype=torch.uint8, device="cuda"),
                        device_config=None)
