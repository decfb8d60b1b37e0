"""Crop transport between the detection and classification services (arm B).

``jpeg``  reference behaviour: PIL JPEG at quality 95 on the detection side,
          PIL decode (gray -> RGB, RGBA -> RGB) on the classification side
          (architectures/microservices/detection/app/grpc_client.py:99-103,
          architectures/microservices/classification/app/servicer.py:65-76).
``png``   lossless, still a standard image format.
``raw``   arena fast path: a 12-byte header (b"ARW1", uint32 h, uint32 w)
          followed by the RGB uint8 pixels — no codec cost on either side,
          and bit-exact crops.

``decode_crop`` sniffs the format, so a classification service accepts all
three from any client.
"""
from __future__ import annotations

import io
import struct

import numpy as np
from PIL import Image

RAW_MAGIC = b"ARW1"
JPEG_QUALITY = 95


def encode_crop(crop: np.ndarray, transport: str = "jpeg") -> bytes:
    crop = np.ascontiguousarray(crop, dtype=np.uint8)
    if crop.ndim != 3 or crop.shape[2] != 3:
        raise ValueError(f"crop must be HxWx3 uint8, got {crop.shape}")
    if transport == "raw":
        return RAW_MAGIC + struct.pack("<II", crop.shape[0], crop.shape[1]) + crop.tobytes()
    buf = io.BytesIO()
    if transport == "jpeg":
        Image.fromarray(crop).save(buf, format="JPEG", quality=JPEG_QUALITY)
    elif transport == "png":
        Image.fromarray(crop).save(buf, format="PNG", compress_level=1)
    else:
        raise ValueError(f"unknown crop transport '{transport}'")
    return buf.getvalue()


def decode_crop(data: bytes) -> np.ndarray:
    if data[:4] == RAW_MAGIC:
        if len(data) < 12:
            raise ValueError("truncated raw crop header")
        h, w = struct.unpack("<II", data[4:12])
        if h <= 0 or w <= 0 or len(data) != 12 + h * w * 3:
            raise ValueError(f"raw crop size mismatch: {h}x{w} with {len(data) - 12} bytes")
        return np.frombuffer(data, dtype=np.uint8, offset=12).reshape(h, w, 3)
    img = Image.open(io.BytesIO(data))
    arr = np.asarray(img)
    if arr.ndim == 2:
        arr = np.stack([arr, arr, arr], axis=-1)
    elif arr.shape[2] == 4:
        arr = arr[:, :, :3]
    return np.ascontiguousarray(arr, dtype=np.uint8)
