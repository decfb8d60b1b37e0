"""Classifier preprocessing and crop extraction (CPU reference path).

Mirrors src/shared/processing/mobilenet_preprocess.py of the reference:
direct (non aspect-preserving) bilinear resize to the configured size,
ImageNet normalisation, HWC->CHW, batch dim (:114-160); ``extract_crop``
int-truncates the box, clamps it to the image and returns a 1x1 black crop
for an empty box (:236-269).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from ..config import get_controlled_variable
from .transforms import imagenet_normalize, resize_bilinear

MOBILENET_INPUT_SIZE = int(get_controlled_variable("preprocessing", "mobilenet")["target_size"])


@dataclass
class MobileNetPreprocessResult:
    tensor: np.ndarray
    original_shape: tuple[int, int]


class MobileNetPreprocessor:
    def __init__(self, input_size: int | None = None) -> None:
        self.input_size = int(input_size or MOBILENET_INPUT_SIZE)

    def __call__(self, crop: np.ndarray) -> MobileNetPreprocessResult:
        return self.preprocess(crop)

    def preprocess(self, crop: np.ndarray) -> MobileNetPreprocessResult:
        self._validate_input(crop)
        if crop.dtype == np.uint8:
            resized = resize_bilinear(crop, self.input_size, self.input_size)
        else:
            resized = resize_bilinear(crop.astype(np.float32), self.input_size, self.input_size)
        x = imagenet_normalize(resized).transpose(2, 0, 1)[None]
        return MobileNetPreprocessResult(np.ascontiguousarray(x, dtype=np.float32), crop.shape[:2])

    def preprocess_batch(self, crops: list[np.ndarray]) -> np.ndarray:
        if not crops:
            return np.zeros((0, 3, self.input_size, self.input_size), np.float32)
        return np.concatenate([self.preprocess(c).tensor for c in crops], axis=0)

    def _validate_input(self, crop: np.ndarray) -> None:
        if not isinstance(crop, np.ndarray):
            raise ValueError(f"Expected numpy array, got {type(crop)}")
        if crop.ndim != 3:
            raise ValueError(f"Expected 3D array [H, W, C], got {crop.ndim}D")
        if crop.shape[2] != 3:
            raise ValueError(f"Expected 3 channels, got {crop.shape[2]}")
        if crop.dtype not in (np.uint8, np.float32):
            raise ValueError(f"Expected uint8 or float32 dtype, got {crop.dtype}")
        if crop.shape[0] < 1 or crop.shape[1] < 1:
            raise ValueError(f"Invalid crop dimensions: {crop.shape[:2]}")

    def get_input_shape(self) -> tuple[int, int, int, int]:
        return (1, 3, self.input_size, self.input_size)

    @staticmethod
    def get_input_dtype() -> np.dtype:
        return np.dtype(np.float32)


def crop_bounds(box, height: int, width: int) -> tuple[int, int, int, int]:
    """Integer crop window (x1, y1, x2, y2) for a float box, reference rules."""
    x1, y1, x2, y2 = (int(v) for v in box[:4])
    return max(0, x1), max(0, y1), min(width, x2), min(height, y2)


def extract_crop(image: np.ndarray, box) -> np.ndarray:
    h, w = image.shape[:2]
    x1, y1, x2, y2 = crop_bounds(box, h, w)
    if x2 <= x1 or y2 <= y1:
        return np.zeros((1, 1, 3), dtype=np.uint8)
    return image[y1:y2, x1:x2].copy()
