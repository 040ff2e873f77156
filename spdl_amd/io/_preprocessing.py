"""FFmpeg filter-description helpers for the image path.

``get_video_filter_desc`` reproduces the string the reference builds
(src/spdl/io/_preprocessing.py:122-254, image-relevant arguments), and
``parse_image_filter`` turns such a string back into the decoder's output
spec, so callers that pass ``filter_desc=`` strings keep working.  Only the
filters the image path needs are understood: ``scale`` (w, h, flags,
force_original_aspect_ratio), ``pad`` (w, h, x=-1, y=-1, color=black),
``crop`` (w, h, centred) and ``format=pix_fmts=``.  Anything else raises.
"""

from __future__ import annotations

from .._lib import Output

_FILTERS = {"bicubic": "bicubic", "bilinear": "bilinear", "fast_bilinear": "bilinear",
            "lanczos": "lanczos"}


def get_video_filter_desc(
    *,
    scale_width: int | None = None,
    scale_height: int | None = None,
    scale_algo: str = "bicubic",
    scale_mode: str | None = "pad",
    crop_width: int | None = None,
    crop_height: int | None = None,
    pix_fmt: str | None = "rgb24",
    pad_mode: str | None = None,
    filter_desc: str | None = None,
    **unsupported: object,
) -> str | None:
    """Same output as the reference for the image arguments."""
    for k, v in unsupported.items():
        if v is not None:
            raise ValueError(f"`{k}` is not supported by the image path")
    parts = []
    if scale_width is not None or scale_height is not None:
        w = scale_width or 0
        h = scale_height or 0
        scale = [f"{w=}", f"{h=}", f"flags={scale_algo}"]
        if scale_mode is None:
            parts.append(f"scale={':'.join(scale)}")
        elif scale_mode == "pad":
            scale.append("force_original_aspect_ratio=decrease")
            parts.append(f"scale={':'.join(scale)}")
            parts.append(f"pad={w=}:{h=}:x=-1:y=-1:color={pad_mode or 'black'}")
        elif scale_mode == "crop":
            scale.append("force_original_aspect_ratio=increase")
            parts.append(f"scale={':'.join(scale)}")
            parts.append(f"crop={w=}:{h=}")
        else:
            raise ValueError(
                f"Unexpected `scale_mode` value ({scale_mode}). "
                'Expected values are "pad", "crop", or None.'
            )
    if crop_width is not None or crop_height is not None:
        parts.append(f"crop=w={crop_width or 0}:h={crop_height or 0}")
    if filter_desc is not None:
        parts.append(filter_desc)
    if pix_fmt is not None:
        parts.append(f"format=pix_fmts={pix_fmt}")
    if parts:
        return ",".join(parts)
    return None


def _kv(args: str) -> dict:
    out = {}
    for i, item in enumerate(a for a in args.split(":") if a):
        if "=" in item:
            k, v = item.split("=", 1)
        else:  # positional w:h
            k, v = ("w", "h", "x", "y")[i], item
        out[k.strip()] = v.strip()
    return out


def parse_image_filter(filter_desc: str | None, default_pix_fmt: str = "rgb24") -> Output:
    """Translate an image filter chain into an :class:`Output` spec."""
    spec = dict(pix_fmt=default_pix_fmt, resize=False)
    if not filter_desc:
        return Output(**spec)
    have_scale = have_pad = False
    for part in filter_desc.split(","):
        part = part.strip()
        if not part:
            continue
        name, _, args = part.partition("=")
        kv = _kv(args)
        if name == "scale":
            w, h = int(kv.get("w", 0)), int(kv.get("h", 0))
            if w < 0 or h < 0:
                raise ValueError(f"negative scale sizes are not supported: {part}")
            spec.update(resize=True, fit_w=w, fit_h=h)
            flags = kv.get("flags", "bicubic")
            if flags not in _FILTERS:
                raise ValueError(f"unsupported scale flags: {flags}")
            spec["filter"] = _FILTERS[flags]
            ar = kv.get("force_original_aspect_ratio")
            if ar in (None, "disable", "0"):
                spec["aspect"] = None
            elif ar in ("decrease", "1"):
                spec["aspect"] = "decrease"
            elif ar in ("increase", "2"):
                spec["aspect"] = "increase"
            else:
                raise ValueError(f"unsupported force_original_aspect_ratio: {ar}")
            have_scale = True
        elif name == "pad":
            if not have_scale:
                raise ValueError("pad without a preceding scale is not supported")
            if kv.get("x", "-1") != "-1" or kv.get("y", "-1") != "-1":
                raise ValueError("only centred pad (x=-1:y=-1) is supported")
            if kv.get("color", "black") != "black":
                raise ValueError("only color=black is supported")
            spec.update(resize=True, pad_w=int(kv["w"]), pad_h=int(kv["h"]))
            have_pad = True
        elif name == "crop":
            if "x" in kv or "y" in kv:
                raise ValueError("only centred crop is supported")
            spec.update(resize=True, crop_w=int(kv.get("w", 0)), crop_h=int(kv.get("h", 0)))
        elif name == "format":
            pf = kv.get("pix_fmts", kv.get("w"))
            if pf not in ("rgb24", "bgr24", "rgb", "bgr"):
                raise ValueError(f"unsupported output pix_fmt: {pf}")
            spec["pix_fmt"] = pf
        else:
            raise ValueError(f"filter `{name}` is not supported by the image decode stage")
    del have_pad
    return Output(**spec)
