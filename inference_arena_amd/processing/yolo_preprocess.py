"""Detector preprocessing (CPU reference path).

Mirrors src/shared/processing/yolo_preprocess.py:44-213 of the reference:
letterbox to the configured size, /255, HWC->CHW, batch dim ->
float32 [1, 3, T, T], keeping the geometry needed to undo the letterbox.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from ..config import get_controlled_variable
from .transforms import letterbox, scale_boxes


def _target_size() -> int:
    return int(get_controlled_variable("preprocessing", "yolo")["target_size"])


YOLO_INPUT_SIZE = _target_size()


@dataclass
class YOLOPreprocessResult:
    tensor: np.ndarray
    scale: float
    padding: tuple[int, int]
    original_shape: tuple[int, int]

    def scale_boxes_to_original(self, boxes: np.ndarray) -> np.ndarray:
        return scale_boxes(boxes, self.scale, self.padding, self.original_shape)


class YOLOPreprocessor:
    def __init__(self, target_size: int | None = None) -> None:
        self.target_size = int(target_size or YOLO_INPUT_SIZE)
        self.normalization_scale = float(get_controlled_variable("preprocessing", "yolo")["normalization_scale"])

    def __call__(self, image: np.ndarray) -> YOLOPreprocessResult:
        return self.preprocess(image)

    def preprocess(self, image: np.ndarray) -> YOLOPreprocessResult:
        self._validate_input(image)
        boxed, scale, padding = letterbox(image, self.target_size)
        t = boxed.astype(np.float32) / np.float32(self.normalization_scale)
        t = np.ascontiguousarray(t.transpose(2, 0, 1)[None])
        return YOLOPreprocessResult(t, scale, padding, (image.shape[0], image.shape[1]))

    def _validate_input(self, image: np.ndarray) -> None:
        if not isinstance(image, np.ndarray):
            raise ValueError(f"Expected numpy array, got {type(image)}")
        if image.ndim != 3:
            raise ValueError(f"Expected 3D array [H, W, C], got {image.ndim}D")
        if image.shape[2] != 3:
            raise ValueError(f"Expected 3 channels, got {image.shape[2]}")
        if image.dtype != np.uint8:
            raise ValueError(f"Expected uint8 dtype, got {image.dtype}")

    def get_input_shape(self) -> tuple[int, int, int, int]:
        return (1, 3, self.target_size, self.target_size)

    @staticmethod
    def get_input_dtype() -> np.dtype:
        return np.dtype(np.float32)
