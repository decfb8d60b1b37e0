"""Host (CPU) image transforms with the reference's exact geometry.

These NumPy implementations are (a) the CPU path of the arena (the
reference-equivalent "config 1" plumbing arm) and (b) the oracle against which
the HIP preprocessing kernels (csrc/kernels/preprocess.hip) are tested.

Reference behaviour reproduced (``/root/reference`` paths):
  * ``load_image_from_bytes``: src/shared/processing/transforms.py:77-110 —
    decode any PIL-readable format to RGB uint8, "Failed to decode" on error.
  * ``letterbox``: src/shared/processing/transforms.py:118-180 — scale =
    min(T/h, T/w), new size int-truncated, floor-centred padding, gray 114.
  * ``scale_boxes``: src/shared/processing/transforms.py:183-230.
  * ``imagenet_normalize``: src/shared/processing/transforms.py:238-272.

OpenCV is not available in this environment, so ``resize_bilinear`` is a
vectorised re-implementation of cv2 ``INTER_LINEAR`` geometry
(src = (dst + 0.5) * in/out - 0.5, border clamp, uint8 rounding).  cv2's
11-bit fixed-point weights can differ from it by one intensity level.
"""
from __future__ import annotations

import io
from pathlib import Path

import numpy as np

from ..config import get_controlled_variable

LETTERBOX_COLOR = (114, 114, 114)


def _imagenet_stats() -> tuple[np.ndarray, np.ndarray]:
    mb = get_controlled_variable("preprocessing", "mobilenet")
    return np.asarray(mb["mean"], np.float32), np.asarray(mb["std"], np.float32)


IMAGENET_MEAN, IMAGENET_STD = _imagenet_stats()


class ImageTooLargeError(ValueError):
    """An upload whose header declares more pixels than ``max_image_pixels()`` (a decompression bomb: a few KB
    of JPEG that would decode to gigabytes).  Servers answer 413."""


def max_image_pixels() -> int:
    """``ARENA_MAX_IMAGE_PIXELS`` (default 50 MP, above any camera frame the arena serves; the reference's
    cv2.imdecode stops at 2^30 pixels, CV_IO_MAX_IMAGE_PIXELS)."""
    import os

    return int(os.environ.get("ARENA_MAX_IMAGE_PIXELS", str(50_000_000)))


def _check_size(im, what: str) -> None:
    w, h = im.size
    if w * h > max_image_pixels():
        raise ImageTooLargeError(f"{what}: image too large ({w}x{h} pixels > {max_image_pixels()})")


def _decode(data: bytes | Path | str, what: str) -> np.ndarray:
    from PIL import Image, UnidentifiedImageError

    try:
        src = io.BytesIO(data) if isinstance(data, (bytes, bytearray, memoryview)) else str(data)
        with Image.open(src) as im:
            _check_size(im, what)
            if im.mode != "RGB":  # convert() of an RGB image is a full copy
                im = im.convert("RGB")
            arr = np.asarray(im, dtype=np.uint8)
    except ImageTooLargeError:
        raise
    except Image.DecompressionBombError as e:
        raise ImageTooLargeError(f"{what}: image too large ({e})") from e
    except (UnidentifiedImageError, OSError, ValueError) as e:
        raise ValueError(f"{what}: {e}") from e
    return np.ascontiguousarray(arr)


def decode_rgb(data: bytes | memoryview) -> tuple[int, int, bytes]:
    """The decode of ``load_image_from_bytes`` returning (h, w, packed RGB bytes): one pack of PIL's
    RGBX raster and no numpy round trip (the decode-pool workers copy the bytes into shared memory)."""
    from PIL import Image, UnidentifiedImageError

    if not len(data):
        raise ValueError("Failed to decode image: empty payload")
    try:
        with Image.open(io.BytesIO(data)) as im:
            _check_size(im, "Failed to decode image")
            if im.mode != "RGB":
                im = im.convert("RGB")
            w, h = im.size
            return h, w, im.tobytes()
    except ImageTooLargeError:
        raise
    except Image.DecompressionBombError as e:
        raise ImageTooLargeError(f"Failed to decode image: image too large ({e})") from e
    except (UnidentifiedImageError, OSError, ValueError) as e:
        raise ValueError(f"Failed to decode image: {e}") from e


class ImageLoadError(ValueError, FileNotFoundError):
    """A missing image file: a ``ValueError`` like the reference's ``load_image``
    (src/shared/processing/transforms.py:67-71, cv2.imread -> None), and a
    ``FileNotFoundError`` for callers that expect the OS error."""


def load_image(image_path: str | Path) -> np.ndarray:
    """Load an image file as RGB uint8 [H, W, 3]."""
    p = Path(image_path)
    if not p.exists():
        raise ImageLoadError(f"Failed to load image: {p} (not found)")
    return _decode(p, f"Failed to load image {p}")


def load_image_from_bytes(image_bytes: bytes) -> np.ndarray:
    """Decode encoded image bytes (JPEG/PNG/...) to RGB uint8 [H, W, 3]."""
    if not image_bytes:
        raise ValueError("Failed to decode image: empty payload")
    return _decode(image_bytes, "Failed to decode image")


def _lin_taps(dst: int, src: int) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    scale = np.float32(src / dst)
    f = (np.arange(dst, dtype=np.float32) + np.float32(0.5)) * scale - np.float32(0.5)
    i0 = np.floor(f).astype(np.int64)
    frac = (f - i0).astype(np.float32)
    low = i0 < 0
    i0[low] = 0
    frac[low] = 0.0
    high = i0 >= src - 1
    i0[high] = src - 1
    frac[high] = 0.0
    i1 = np.minimum(i0 + 1, src - 1)
    return i0, i1, frac


def resize_bilinear(image: np.ndarray, width: int, height: int) -> np.ndarray:
    """cv2.resize(image, (width, height), INTER_LINEAR) for uint8 HWC images."""
    if image.ndim != 3:
        raise ValueError(f"Expected HWC image, got shape {image.shape}")
    h, w = image.shape[:2]
    if (h, w) == (height, width):
        return image.copy()
    y0, y1, fy = _lin_taps(height, h)
    x0, x1, fx = _lin_taps(width, w)
    img = image.astype(np.float32)
    fxc = fx[None, :, None]
    top = img[y0][:, x0] + (img[y0][:, x1] - img[y0][:, x0]) * fxc
    bot = img[y1][:, x0] + (img[y1][:, x1] - img[y1][:, x0]) * fxc
    out = top + (bot - top) * fy[:, None, None]
    if image.dtype == np.uint8:
        return np.floor(out + np.float32(0.5)).clip(0, 255).astype(np.uint8)
    return out.astype(image.dtype)


def letterbox_geometry(h: int, w: int, target_size: int) -> tuple[float, int, int, int, int]:
    """(scale, new_w, new_h, pad_w, pad_h) exactly as the reference computes them."""
    scale = min(target_size / h, target_size / w)
    new_w, new_h = int(w * scale), int(h * scale)
    return scale, new_w, new_h, (target_size - new_w) // 2, (target_size - new_h) // 2


def letterbox(
    image: np.ndarray, target_size: int, color: tuple[int, int, int] = LETTERBOX_COLOR
) -> tuple[np.ndarray, float, tuple[int, int]]:
    """Aspect-preserving resize + centred constant padding.

    Returns (letterboxed [T, T, 3] uint8, scale, (pad_w, pad_h)).
    """
    h, w = image.shape[:2]
    scale, new_w, new_h, pad_w, pad_h = letterbox_geometry(h, w, target_size)
    resized = resize_bilinear(image, new_w, new_h)
    out = np.empty((target_size, target_size, 3), dtype=np.uint8)
    out[...] = np.asarray(color, dtype=np.uint8)
    out[pad_h : pad_h + new_h, pad_w : pad_w + new_w] = resized
    return out, scale, (pad_w, pad_h)


def scale_boxes(
    boxes: np.ndarray, scale: float, padding: tuple[int, int], original_shape: tuple[int, int]
) -> np.ndarray:
    """Map [N, 4+] xyxy boxes from letterbox space back to the original image."""
    out = np.array(boxes, copy=True)
    pad_w, pad_h = padding
    orig_h, orig_w = original_shape
    out[:, [0, 2]] -= pad_w
    out[:, [1, 3]] -= pad_h
    out[:, :4] /= scale
    out[:, [0, 2]] = np.clip(out[:, [0, 2]], 0, orig_w)
    out[:, [1, 3]] = np.clip(out[:, [1, 3]], 0, orig_h)
    return out


def imagenet_normalize(image: np.ndarray) -> np.ndarray:
    """(x / 255 - mean) / std as float32 HWC."""
    x = image.astype(np.float32)
    if image.dtype == np.uint8:
        x /= np.float32(255.0)
    elif x.size and x.max() > 1.0:
        x /= np.float32(255.0)
    return (x - IMAGENET_MEAN) / IMAGENET_STD
