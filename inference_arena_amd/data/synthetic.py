"""Synthetic COCO-shaped workload.

No dataset can be downloaded here, so the arena's benchmark and tests use
seeded synthetic images shaped like the reference's curated COCO val2017 set
(data/thesis_test_set/manifest.json: 100 images, 3-5 detections each).
Images are smooth backgrounds with a handful of textured "objects" at COCO
resolutions (most 640x480 / 480x640 / 640x427), generated deterministically
from a seed.  ``encode_jpeg`` produces the bytes a client would upload.
"""
from __future__ import annotations

import io

import numpy as np

COCO_SHAPES = [(480, 640), (427, 640), (640, 480), (480, 640), (425, 640), (640, 427), (512, 640), (480, 640)]


def synthetic_image(rng: np.random.Generator, hw: tuple[int, int] | None = None) -> np.ndarray:
    h, w = hw if hw is not None else COCO_SHAPES[int(rng.integers(len(COCO_SHAPES)))]
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    img = np.empty((h, w, 3), np.float32)
    for c in range(3):
        fx, fy = rng.uniform(0.002, 0.02, 2)
        ph = rng.uniform(0, 2 * np.pi, 2)
        img[..., c] = 110 + 60 * np.sin(xx * fx + ph[0]) * np.cos(yy * fy + ph[1])
    for _ in range(int(rng.integers(3, 7))):
        ow, oh = int(rng.integers(w // 10, w // 3)), int(rng.integers(h // 10, h // 3))
        x0, y0 = int(rng.integers(0, w - ow)), int(rng.integers(0, h - oh))
        color = rng.uniform(0, 255, 3).astype(np.float32)
        tex = rng.normal(0, 25, (oh, ow, 1)).astype(np.float32)
        if rng.random() < 0.5:
            oy, ox = np.mgrid[0:oh, 0:ow]
            m = (((oy - oh / 2) / (oh / 2)) ** 2 + ((ox - ow / 2) / (ow / 2)) ** 2) <= 1.0
            region = img[y0 : y0 + oh, x0 : x0 + ow]
            region[m] = (color + tex)[m]
        else:
            img[y0 : y0 + oh, x0 : x0 + ow] = color + tex
    img += rng.normal(0, 4, img.shape).astype(np.float32)
    return np.clip(img, 0, 255).astype(np.uint8)


def synthetic_images(n: int, seed: int = 42, hw: tuple[int, int] | None = None) -> list[np.ndarray]:
    rng = np.random.default_rng(seed)
    return [synthetic_image(rng, hw) for _ in range(n)]


def encode_jpeg(img: np.ndarray, quality: int = 90) -> bytes:
    from PIL import Image

    buf = io.BytesIO()
    Image.fromarray(img).save(buf, format="JPEG", quality=quality)
    return buf.getvalue()


def encode_png(img: np.ndarray) -> bytes:
    """Lossless encoding (tests compare server results against in-process runs on the same pixels)."""
    from PIL import Image

    buf = io.BytesIO()
    Image.fromarray(img).save(buf, format="PNG", compress_level=1)
    return buf.getvalue()
