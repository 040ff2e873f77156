"""Entropy chain rounds (chain_after): unresolved chains of runs re-decoded
by whole waves after a number of sync rounds.  The output must not change by
a bit: the mixed set (whose high-quality optimised-table images need 11-12
sync rounds), restart layouts and multi-piece images, at one and four lanes,
against the oracle."""

import functools

import numpy as np
import pytest
import torch

from spdl_amd._lib import Output
from tests import cases

pytestmark = pytest.mark.gpu

PAD224 = Output(pix_fmt="rgb24", resize=True, fit_w=224, fit_h=224, aspect="decrease",
                pad_w=224, pad_h=224)


@functools.lru_cache(maxsize=None)
def _mixed():
    from spdl_amd.synthetic import mixed_jpeg

    return [mixed_jpeg(i) for i in range(64)]


@functools.lru_cache(maxsize=None)
def _ref(oracle, d: bytes):
    rs = oracle.Resize(fit_w=224, fit_h=224, aspect="decrease", pad_w=224, pad_h=224)
    return oracle.decode_resize(d, rs, pix_fmt="rgb24")


def _decode(decoder, datas, params):
    # ("chain_after" goes back to -1, automatic: get_param reports the value in effect)
    prev = {k: (-1 if k == "chain_after" else decoder.get_param(k)) for k in params}
    for k, v in params.items():
        decoder.set_param(k, v)
    try:
        t = torch.empty((len(datas), 224, 224, 3), dtype=torch.uint8, device="cuda:0")
        st = decoder.decode_batch(datas, PAD224, t.data_ptr(), t.numel(),
                                  stream=torch.cuda.current_stream(), sync=True)
        return st, t.cpu().numpy()
    finally:
        for k, v in prev.items():
            decoder.set_param(k, v)


@pytest.mark.parametrize("lanes", [1, 4])
@pytest.mark.parametrize("chain_after", [1, 2, 3])
def test_chain_rounds_mixed_set(decoder, oracle, chain_after, lanes):
    datas = _mixed()
    st, hyp = _decode(decoder, datas, {"chain_after": chain_after, "lanes": lanes})
    assert not any(st), st
    for i, d in enumerate(datas):
        np.testing.assert_array_equal(hyp[i], _ref(oracle, d), strict=True, err_msg=f"image {i}")


NAMES = ["bench_1000", "q90_420", "restart_rows", "gray", "q90_444", "odd_227x333",
         "restart_blocks", "noise_420", "optimized", "six_tables", "large_1080p", "q95_420",
         "restart_every_mcu", "tiny_8x8", "noise_q100", "q90_422"]


@pytest.mark.parametrize("piece_kb", [0, 16, 48])
@pytest.mark.parametrize("chain_after", [1, 2])
def test_chain_rounds_cases_and_pieces(decoder, oracle, chain_after, piece_kb):
    """Every sampling / table / restart layout, and images split into pieces
    (chain rounds inside each piece's sync passes, before and after the
    hand-off), with 128-bit slots so that runs are short and chains long."""
    datas = [cases.case(n) for n in NAMES]
    for sub in (128, 384):
        st, hyp = _decode(decoder, datas, {"chain_after": chain_after, "sub_bits": sub,
                                           "entropy_piece_bytes": piece_kb * 1024, "lanes": 4})
        assert not any(st), st
        for i, d in enumerate(datas):
            np.testing.assert_array_equal(hyp[i], _ref(oracle, d), strict=True,
                                          err_msg=f"{NAMES[i]} sub {sub}")


@pytest.mark.parametrize("chain_after", [1, 2])
def test_chain_rounds_planes(decoder, oracle, chain_after):
    """The coefficient path itself (planes) of the mixed set's slowest images."""
    datas = _mixed()
    prev = -1  # (automatic)
    decoder.set_param("chain_after", chain_after)
    try:
        for i in (3, 33, 26, 27):
            hyp = decoder.decode_planes(datas[i])
            ref = oracle.decode_planes(datas[i], idct=oracle.IDCT_SIMPLE)
            for h, r in zip(hyp, ref):
                np.testing.assert_array_equal(h, r, strict=True, err_msg=f"image {i}")
    finally:
        decoder.set_param("chain_after", prev)
