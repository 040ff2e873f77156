"""Tuning knobs that change launch shapes but must not change a byte
(ADVICE r05): swscale tile width (`sws_cols`), parse_kernel workgroup size
(`parse_threads`), the entropy waves' priority (`entropy_prio`) and the
XCD-aware tile order of swscale / IDCT (`xcd_order`, round 6) and the
multi-scan launch of a batch without multi-scan images (`ms_skip_empty`), each
bit-exact vs the oracle on a few resize cases in one batch.
"""

import numpy as np
import pytest
import torch

from spdl_amd._lib import Output
from tests import cases

pytestmark = pytest.mark.gpu

NAMES = ["q90_420", "odd_227x333", "gray", "restart_rows", "large_1080p", "optimized"]
SPECS = {
    "pad224": dict(fit_w=224, fit_h=224, aspect="decrease", pad_w=224, pad_h=224),
    "crop224": dict(fit_w=224, fit_h=224, aspect="increase", crop_w=224, crop_h=224),
    "stretch160x120": dict(fit_w=160, fit_h=120),
}


@pytest.mark.parametrize("knob,value", [("sws_cols", 16), ("sws_cols", 64),
                                        ("parse_threads", 128), ("parse_threads", 256),
                                        ("entropy_prio", 3), ("xcd_order", 0), ("xcd_order", 2), ("xcd_order", 3),
                                        ("ms_skip_empty", 1)])
@pytest.mark.parametrize("sk", list(SPECS))
def test_knob_bit_exact(decoder, oracle, knob, value, sk):
    kw = SPECS[sk]
    datas = [cases.case(n) for n in NAMES]
    refs = [oracle.decode_resize(d, oracle.Resize(**kw), pix_fmt="rgb24") for d in datas]
    out = Output(pix_fmt="rgb24", resize=True, **kw)
    h, w = refs[0].shape[:2]
    prev = decoder.get_param(knob)
    decoder.set_param(knob, value)
    try:
        t = torch.empty((len(datas), h, w, 3), dtype=torch.uint8, device="cuda:0")
        st = decoder.decode_batch(datas, out, t.data_ptr(), t.numel(),
                                  stream=torch.cuda.current_stream())
    finally:
        decoder.set_param(knob, prev)
    assert not any(st), st
    hyp = t.cpu().numpy()
    for i, r in enumerate(refs):
        np.testing.assert_array_equal(hyp[i], r, strict=True, err_msg=f"{knob}={value} {NAMES[i]}")


@pytest.mark.parametrize("value", [1])
def test_ms_skip_empty_with_progressive(decoder, oracle, value):
    """A batch that holds progressive images still launches the multi-scan
    decode over every image whatever `ms_skip_empty` says."""
    names = NAMES[:3] + ["prog_420", "prog_gray"]
    kw = SPECS["pad224"]
    datas = [cases.case(n) for n in names]
    refs = [oracle.decode_resize(d, oracle.Resize(**kw), pix_fmt="rgb24") for d in datas]
    out = Output(pix_fmt="rgb24", resize=True, **kw)
    prev = decoder.get_param("ms_skip_empty")
    decoder.set_param("ms_skip_empty", value)
    try:
        t = torch.empty((len(datas), 224, 224, 3), dtype=torch.uint8, device="cuda:0")
        st = decoder.decode_batch(datas, out, t.data_ptr(), t.numel(),
                                  stream=torch.cuda.current_stream())
    finally:
        decoder.set_param("ms_skip_empty", prev)
    assert not any(st), st
    hyp = t.cpu().numpy()
    for i, r in enumerate(refs):
        np.testing.assert_array_equal(hyp[i], r, strict=True, err_msg=names[i])
