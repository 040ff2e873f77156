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

_FILTERS = {"bicubic": "bicubic", "bilinear": "bilinear", "lanczos": "lanczos"}
# swscale's SWS_FAST_BILINEAR is its own horizontal scaler (7-bit position
# fractions), not the bilinear filter: rather than silently return other
# pixels, it is refused
_NOT_IMPLEMENTED = {"fast_bilinear": "swscale's fast_bilinear scaler is not implemented; "
                                     "use flags=bilinear (a different, exact bilinear filter)"}


# scale_mode -> scale's force_original_aspect_ratio and the filter that
# brings the fitted image to the requested box
_FIT = {None: (None, None), "pad": ("decrease", "pad"), "crop": ("increase", "crop")}


def _node(name: str, **opts) -> str:
    """One filter of an FFmpeg chain: ``name=k1=v1:k2=v2``."""
    return name + "=" + ":".join(f"{k}={v}" for k, v in opts.items())


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
    """The filter chain the reference builds for these image arguments
    (src/spdl/io/_preprocessing.py:122-254; byte-for-byte, pinned by
    tests/golden/filter_desc.json): optional scale (+ pad / crop to the box),
    optional centre crop, a caller chain, then the output pixel format."""
    extra = sorted(k for k, v in unsupported.items() if v is not None)
    if extra:
        raise ValueError(f"image filter arguments not supported here: {extra}")
    if scale_mode not in _FIT:
        raise ValueError(f"scale_mode must be 'pad', 'crop' or None, got {scale_mode!r}")
    chain: list[str] = []
    if (scale_width, scale_height) != (None, None):
        box = {"w": scale_width or 0, "h": scale_height or 0}
        ratio, follow = _FIT[scale_mode]
        scale = {**box, "flags": scale_algo}
        if ratio:
            scale["force_original_aspect_ratio"] = ratio
        chain.append(_node("scale", **scale))
        if follow == "pad":
            chain.append(_node("pad", **box, x=-1, y=-1, color=pad_mode or "black"))
        elif follow == "crop":
            chain.append(_node("crop", **box))
    if (crop_width, crop_height) != (None, None):
        chain.append(_node("crop", w=crop_width or 0, h=crop_height or 0))
    if filter_desc is not None:
        chain.append(filter_desc)
    if pix_fmt is not None:
        chain.append(_node("format", pix_fmts=pix_fmt))
    return ",".join(chain) or None


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
    have_scale = False
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
            if flags in _NOT_IMPLEMENTED:
                raise ValueError(_NOT_IMPLEMENTED[flags])
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
    return Output(**spec)
