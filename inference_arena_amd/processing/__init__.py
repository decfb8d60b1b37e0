"""Host-side image processing (reference semantics; CPU path and kernel oracle)."""
from .mobilenet_preprocess import (
    MOBILENET_INPUT_SIZE,
    MobileNetPreprocessor,
    MobileNetPreprocessResult,
    crop_bounds,
    extract_crop,
)
from .transforms import (
    IMAGENET_MEAN,
    IMAGENET_STD,
    LETTERBOX_COLOR,
    imagenet_normalize,
    letterbox,
    letterbox_geometry,
    load_image,
    load_image_from_bytes,
    resize_bilinear,
    scale_boxes,
)
from .yolo_preprocess import YOLO_INPUT_SIZE, YOLOPreprocessor, YOLOPreprocessResult

__all__ = [
    "IMAGENET_MEAN",
    "IMAGENET_STD",
    "LETTERBOX_COLOR",
    "MOBILENET_INPUT_SIZE",
    "YOLO_INPUT_SIZE",
    "MobileNetPreprocessor",
    "MobileNetPreprocessResult",
    "YOLOPreprocessor",
    "YOLOPreprocessResult",
    "crop_bounds",
    "extract_crop",
    "imagenet_normalize",
    "letterbox",
    "letterbox_geometry",
    "load_image",
    "load_image_from_bytes",
    "resize_bilinear",
    "scale_boxes",
]
