"""Generate the committed golden fixtures under tests/golden/ (run in the build
container, where IJG libjpeg 9d and the reference tree exist):

  python tests/gen_golden.py

Fixtures (data only -- inputs and expected outputs):
  jpeg/<case>.jpg               input JPEGs (Pillow-encoded, seeded; tests/cases.py)
  <case>.libjpeg.npz            IJG libjpeg 9d (/opt/conda/lib/libjpeg.so.9):
                                  quantised coefficients per component
                                  (jpeg_read_coefficients) and the islow /
                                  no-fancy-upsampling RGB decode (not for
                                  4-component CMYK/YCCK: libjpeg has no such
                                  conversion)
  <case>.oracle.npz             oracle outputs (regression pin of the restatement):
                                  simple-IDCT planes, rgb24, pad224 resize,
                                  normalised fp16
  filter_desc.json              filter strings from the reference's own
                                  spdl.io._preprocessing.get_video_filter_desc
                                  (imported from /root/reference/src)
"""

from __future__ import annotations

import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402
from tests import cases  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden")

# small enough to commit (a few MB total)
CASES = [
    "q90_444", "q90_422", "odd_227x333", "odd_444_101x67", "gray", "gray_odd",
    "noise_q100", "restart_rows", "restart_blocks", "restart_every_mcu", "tiny_8x8",
    "tiny_1x1", "optimized", "six_tables",
    # the bench's own shape: 480x640 q90 4:2:0 (bench.py's first synthetic
    # image and the q90_420 case)
    "q90_420", "bench_1000",
    *cases.PROGRESSIVE, *cases.MULTISCAN, *cases.FOUR_COMPONENT, *cases.RGB_CODED,
    *cases.RGB_VARIANTS,
]

PAD224 = O.Resize(fit_w=224, fit_h=224, aspect="decrease", pad_w=224, pad_h=224)

FILTER_ARGS = [
    dict(scale_width=224, scale_height=224, pix_fmt="rgb24"),
    dict(scale_width=256, scale_height=256, scale_mode="crop"),
    dict(scale_width=160, scale_height=120, scale_mode=None),
    dict(scale_width=224, scale_height=224, pix_fmt="bgr24"),
    dict(scale_width=300, scale_height=None),
    dict(scale_width=None, scale_height=None),
    dict(scale_width=224, scale_height=224, scale_algo="bilinear"),
    dict(scale_width=256, scale_height=256, crop_width=224, crop_height=224),
]


def main() -> None:
    os.makedirs(os.path.join(GOLD, "jpeg"), exist_ok=True)
    only = sys.argv[1:]  # optional: regenerate just these cases
    for name in CASES:
        if only and name not in only:
            continue
        if name in cases.MULTISCAN:  # libjpeg 9 writes these inputs
            seed, h, w, q, h0, v0, rst = cases.MULTISCAN[name]
            from spdl_amd.synthetic import synthetic_pixels

            data = O.lj_encode_multiscan(synthetic_pixels(seed, h, w), q, h0, v0, rst)
        elif name in cases.CMYK:  # libjpeg 9 writes these too (Adobe marker)
            seed, h, w, q, ycck, rst, *script = cases.CMYK[name]
            data = O.lj_encode_cmyk(cases.cmyk_pixels(seed, h, w), q, ycck, rst,
                                    script[0] if script else "sequential")
        elif name in cases.RGB_CODED:
            from spdl_amd.synthetic import synthetic_pixels

            seed, h, w, q, rst = cases.RGB_CODED[name]
            data = O.lj_encode_rgb_colorspace(synthetic_pixels(seed, h, w), q, rst)
        else:
            data = cases.case(name)
        with open(os.path.join(GOLD, "jpeg", f"{name}.jpg"), "wb") as f:
            f.write(data)
        comps = O.lj_read_coefs(data)
        # libjpeg converts YCbCr / gray / RGB-coded frames to RGB, no CMYK / YCCK:
        # coefficients only for those
        # (and rgb_adobe_only: libjpeg 9 takes ids 1 2 3 for YCbCr ahead of the
        # Adobe transform-0 flag, FFmpeg -- the reference -- the flag for RGB)
        skip = O.parse(data).color > 2 or name == "rgb_adobe_only"
        rgb = {} if skip else dict(rgb_islow=O.lj_decode_rgb(data))
        np.savez_compressed(
            os.path.join(GOLD, f"{name}.libjpeg.npz"),
            **rgb,
            **{f"coef{c}": comps[c] for c in range(len(comps))},
        )
        planes = O.decode_planes(data, O.IDCT_SIMPLE)
        out = dict(
            rgb24_simple=O.decode_rgb(data, O.IDCT_SIMPLE, "rgb24"),
            pad224_rgb24=O.decode_resize(data, PAD224, "rgb24"),
            pad224_f16=O.decode_resize(data, PAD224, "rgb", normalize=True).view(np.uint16),
        )
        for c, p in enumerate(planes):
            out[f"plane{c}"] = p
        np.savez_compressed(os.path.join(GOLD, f"{name}.oracle.npz"), **out)
        print(name, len(data), "bytes")
    if only:
        return
    sys.path.insert(0, "/root/reference/src")
    from spdl.io._preprocessing import get_video_filter_desc

    filt = [dict(args=a, desc=get_video_filter_desc(**a)) for a in FILTER_ARGS]
    with open(os.path.join(GOLD, "filter_desc.json"), "w") as f:
        json.dump(filt, f, indent=1)
    print("filter strings:", len(filt))


if __name__ == "__main__":
    main()
