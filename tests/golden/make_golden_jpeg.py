#!/usr/bin/env python3
"""Golden vectors of the densify CLI's JPEG ingest.

The reference reads views with cv::imread (modules/core/types.cpp:7-11), i.e.
libjpeg(-turbo) with its defaults (ISLOW IDCT, fancy upsampling) and EXIF
orientation applied.  Pillow ships libjpeg-turbo: this script encodes small
synthetic images with it in every layout scene folders hold and stores, per
case, the file's bytes and the BGR8 array libjpeg-turbo decodes it to (PIL's
decoder with default settings, ImageOps.exif_transpose for the EXIF cases).
OpenCV is absent here, so libjpeg-turbo's own decode (the library imread
calls) is the anchor.

    python tests/golden/make_golden_jpeg.py   -> tests/golden/jpeg_ingest.npz
"""
from __future__ import annotations

import io
import os

import numpy as np
from PIL import Image, ImageOps

HERE = os.path.dirname(os.path.abspath(__file__))


def texture(w: int, h: int, seed: int) -> np.ndarray:
    """Colourful band-limited noise with hard edges (exercises chroma and the
    IDCT range limit)."""
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w].astype(np.float64)
    img = np.zeros((h, w, 3))
    for c in range(3):
        for f in (3.0, 7.0, 17.0):
            a, b, ph = rng.normal(size=3)
            img[:, :, c] += np.sin((a * x + b * y) / f + 6.0 * ph) * (60.0 / f ** 0.3)
    img += 128.0
    img[(x // 9 + y // 7) % 5 == 0] = (250, 10, 240)  # saturated blocks
    img += rng.normal(scale=6.0, size=img.shape)
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)


def exif_with_orientation(o: int) -> bytes:
    ex = Image.Exif()
    ex[0x0112] = o
    return ex.tobytes()


def cases():
    rgb_odd = texture(61, 45, 1)
    rgb = texture(128, 96, 2)
    tall = texture(37, 70, 3)
    tiny = texture(2, 3, 4)
    one = texture(1, 1, 5)
    yield "q90_444", rgb, dict(quality=90, subsampling=0)
    yield "q85_422", rgb_odd, dict(quality=85, subsampling=1)
    yield "q75_420", rgb_odd, dict(quality=75, subsampling=2)
    yield "q95_420_even", rgb, dict(quality=95, subsampling=2)
    yield "q100_444", rgb_odd, dict(quality=100, subsampling=0)
    yield "q50_420_tall", tall, dict(quality=50, subsampling=2)
    yield "q80_420_optimized", rgb_odd, dict(quality=80, subsampling=2, optimize=True)
    yield "q85_420_restart_blocks", rgb_odd, dict(quality=85, subsampling=2, restart_marker_blocks=3)
    yield "q85_444_restart_rows", rgb, dict(quality=85, subsampling=0, restart_marker_rows=1)
    yield "q85_420_progressive", rgb_odd, dict(quality=85, subsampling=2, progressive=True)
    yield "q92_444_progressive", rgb, dict(quality=92, subsampling=0, progressive=True)
    yield "q70_422_progressive_restart", tall, dict(quality=70, subsampling=1, progressive=True,
                                                    restart_marker_blocks=5)
    yield "gray_q90", rgb_odd.mean(axis=2).astype(np.uint8), dict(quality=90)
    yield "gray_q80_progressive", rgb.mean(axis=2).astype(np.uint8), dict(quality=80, progressive=True)
    yield "tiny_2x3_420", tiny, dict(quality=90, subsampling=2)
    yield "one_1x1_422", one, dict(quality=90, subsampling=1)
    yield "exif_orient6_420", rgb_odd, dict(quality=85, subsampling=2, exif=exif_with_orientation(6))
    yield "exif_orient3_444", tall, dict(quality=85, subsampling=0, exif=exif_with_orientation(3))
    yield "exif_orient5_422", tall, dict(quality=85, subsampling=1, exif=exif_with_orientation(5))
    yield "exif_orient8_420", rgb_odd, dict(quality=85, subsampling=2, exif=exif_with_orientation(8))


def main():
    out = {}
    for name, arr, kw in cases():
        im = Image.fromarray(arr)
        buf = io.BytesIO()
        im.save(buf, format="JPEG", **kw)
        data = buf.getvalue()
        dec = ImageOps.exif_transpose(Image.open(io.BytesIO(data))).convert("RGB")
        bgr = np.ascontiguousarray(np.asarray(dec)[:, :, ::-1])
        out[name + "__jpg"] = np.frombuffer(data, dtype=np.uint8)
        out[name + "__bgr"] = bgr
    path = os.path.join(HERE, "jpeg_ingest.npz")
    np.savez_compressed(path, **out)
    print(path, len(out) // 2, "cases", os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
