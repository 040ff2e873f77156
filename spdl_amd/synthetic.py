"""Deterministic synthetic JPEG workload (BASELINE.md §2 / SURVEY.md §8(d)).

Seeded numpy image: per channel six random sinusoids (amplitude 10-40,
frequency 0.002-0.05 cycles/px) + 128 + N(0, 6) noise, clipped to u8, encoded
by Pillow (baseline, 4:2:0 by default, no restart markers).  At 480x640 q90
this is ~110 KB per image, the size BASELINE.md's roofline accounting uses.
"""

from __future__ import annotations

import io

import numpy as np


def synthetic_pixels(seed: int, height: int = 480, width: int = 640) -> np.ndarray:
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:height, 0:width].astype(np.float32)
    img = np.empty((height, width, 3), np.float32)
    for c in range(3):
        acc = np.full((height, width), 128.0, np.float32)
        for _ in range(6):
            amp = rng.uniform(10, 40)
            fx, fy = rng.uniform(0.002, 0.05, size=2)
            ph = rng.uniform(0, 2 * np.pi)
            acc += amp * np.sin(2 * np.pi * (fx * xx + fy * yy) + ph).astype(np.float32)
        acc += rng.normal(0, 6, size=(height, width)).astype(np.float32)
        img[..., c] = acc
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)


def encode_jpeg(
    pixels: np.ndarray, quality: int = 90, subsampling: int = 2, optimize: bool = False,
    progressive: bool = False,
) -> bytes:
    """Pillow JPEG (baseline unless `progressive`). subsampling: 0=4:4:4,
    1=4:2:2, 2=4:2:0."""
    from PIL import Image

    mode = "L" if pixels.ndim == 2 else "RGB"
    buf = io.BytesIO()
    kw = dict(quality=quality, optimize=optimize, progressive=progressive)
    if mode == "RGB":
        kw["subsampling"] = subsampling
    Image.fromarray(pixels, mode).save(buf, format="JPEG", **kw)
    return buf.getvalue()


def synthetic_jpeg(
    seed: int,
    height: int = 480,
    width: int = 640,
    quality: int = 90,
    subsampling: int = 2,
    progressive: bool = False,
) -> bytes:
    return encode_jpeg(synthetic_pixels(seed, height, width), quality, subsampling,
                       progressive=progressive)


def synthetic_batch(n: int, distinct: int = 32, **kw) -> list[bytes]:
    """n JPEGs cycling through `distinct` seeded images."""
    base = [synthetic_jpeg(1000 + i, **kw) for i in range(min(n, distinct))]
    return [base[i % len(base)] for i in range(n)]


def synthetic_slice(indices, distinct: int = 32, **kw) -> list[bytes]:
    """Images ``indices`` of the global synthetic dataset whose image i is
    ``synthetic_batch``'s image i (seed 1000 + i % distinct): one rank's slice
    of a global batch (BASELINE configs[2]: 2048 -> 8 x 256)."""
    cache: dict[int, bytes] = {}
    out = []
    for i in indices:
        k = int(i) % distinct
        if k not in cache:
            cache[k] = synthetic_jpeg(1000 + k, **kw)
        out.append(cache[k])
    return out


# ---- heterogeneous workload (round-5 `bench.py --workload mixed`) ----------
# ImageNet-shaped: sizes from thumbnails to multi-megapixel photos with a
# skew toward ~0.2 MP (ILSVRC train: mean ~400x350, ~110 KB), several
# samplings and qualities, per-image optimised Huffman tables on some,
# restart intervals on a few.  Each image gets its own DQT and (optimised)
# DHT, so the batch's LUT builds and table dedup see a realistic mix.
_SHAPES = [(3, 4), (4, 3), (1, 1), (9, 16), (2, 3), (3, 2)]


def mixed_spec(i: int, seed: int = 5) -> dict:
    """Encoding parameters of image i of the mixed set (deterministic)."""
    rng = np.random.default_rng(seed * 100003 + i)
    mp = float(np.exp(rng.normal(np.log(0.19), 0.9)))  # megapixels, log-normal
    mp = min(max(mp, 0.019), 12.0)
    ah, aw = _SHAPES[int(rng.integers(0, len(_SHAPES)))]
    w = int(round(np.sqrt(mp * 1e6 * aw / ah)))
    h = int(round(w * ah / aw))
    u = rng.random()
    sub = 2 if u < 0.7 else (1 if u < 0.8 else 0)
    return {
        "height": max(h, 16), "width": max(w, 16),
        "quality": int(rng.integers(60, 96)),
        "subsampling": sub,
        "optimize": bool(rng.random() < 0.3),
        "restart_rows": bool(rng.random() < 0.1),
        "gray": bool(rng.random() < 0.02),
        "seed": 5000 + i,
    }


def mixed_jpeg(i: int, seed: int = 5) -> bytes:
    from PIL import Image

    s = mixed_spec(i, seed)
    px = synthetic_pixels(s["seed"], s["height"], s["width"])
    if s["gray"]:
        px = px[..., 0]
    kw = dict(quality=s["quality"], optimize=s["optimize"])
    if not s["gray"]:
        kw["subsampling"] = s["subsampling"]
    if s["restart_rows"]:
        kw["restart_marker_rows"] = 1
    buf = io.BytesIO()
    Image.fromarray(px, "L" if s["gray"] else "RGB").save(buf, format="JPEG", **kw)
    return buf.getvalue()


def mixed_batch(n: int, distinct: int = 64, seed: int = 5) -> list[bytes]:
    """n images cycling through `distinct` images of the mixed set."""
    base = [mixed_jpeg(i, seed) for i in range(min(n, distinct))]
    return [base[i % len(base)] for i in range(n)]


def big_batch(n: int = 256, distinct: int = 32) -> list[bytes]:
    """One 12 MP (4000x3000 q90 4:2:0, ~4 MB) image followed by n - 1 bench
    images: the round-4 verdict's size-adaptivity case."""
    big = synthetic_jpeg(77, 3000, 4000, quality=90)
    return [big] + synthetic_batch(n - 1, distinct)
