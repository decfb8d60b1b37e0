"""Host preprocessing contracts (reference: tests/shared/test_processing.py)."""
from __future__ import annotations

import numpy as np
import pytest

from inference_arena_amd.processing import (
    IMAGENET_MEAN,
    IMAGENET_STD,
    MobileNetPreprocessor,
    YOLOPreprocessor,
    extract_crop,
    imagenet_normalize,
    letterbox,
    letterbox_geometry,
    load_image_from_bytes,
    resize_bilinear,
    scale_boxes,
)


def test_letterbox_landscape_geometry():
    img = np.zeros((1080, 1920, 3), np.uint8)
    out, scale, (pw, ph) = letterbox(img, 640)
    assert out.shape == (640, 640, 3)
    assert scale == pytest.approx(1 / 3)
    assert (pw, ph) == (0, 140)
    assert (out[:140] == 114).all() and (out[-140:] == 114).all()
    assert (out[140:500] == 0).all()


def test_letterbox_portrait_and_truncation():
    img = np.full((500, 333, 3), 200, np.uint8)
    scale, nw, nh, pw, ph = letterbox_geometry(500, 333, 640)
    assert nh == 640 and nw == int(333 * 640 / 500)
    out, s2, (pw2, ph2) = letterbox(img, 640)
    assert (pw2, ph2) == (pw, ph) == ((640 - nw) // 2, 0)
    assert (out[:, :pw] == 114).all()
    assert (out[:, pw : pw + nw] == 200).all()


def test_resize_identity_and_constant():
    rng = np.random.default_rng(0)
    img = rng.integers(0, 255, (37, 53, 3), dtype=np.uint8)
    assert np.array_equal(resize_bilinear(img, 53, 37), img)
    const = np.full((10, 20, 3), 77, np.uint8)
    assert (resize_bilinear(const, 224, 224) == 77).all()


def test_resize_upsample_matches_cv2_geometry():
    # 2x upsampling of [0, 100] with INTER_LINEAR: [0, 25, 75, 100]
    img = np.array([[[0, 0, 0], [100, 100, 100]]], np.uint8)
    out = resize_bilinear(img, 4, 1)
    assert out[0, :, 0].tolist() == [0, 25, 75, 100]


def test_scale_boxes_inverts_letterbox_and_clips():
    boxes = np.array([[320, 320, 400, 400, 0.9, 0], [-10, 100, 700, 120, 0.8, 1]], np.float32)
    out = scale_boxes(boxes, 1 / 3, (0, 140), (1080, 1920))
    assert out[0, :4] == pytest.approx([960, 540, 1200, 780], rel=1e-5)
    assert out[1, 0] == 0 and out[1, 2] == 1920
    assert boxes[0, 0] == 320  # input untouched


def test_imagenet_normalize_values():
    z = imagenet_normalize(np.zeros((2, 2, 3), np.uint8))
    assert np.allclose(z[0, 0], -IMAGENET_MEAN / IMAGENET_STD)
    w = imagenet_normalize(np.full((2, 2, 3), 255, np.uint8))
    assert np.allclose(w[0, 0], (1 - IMAGENET_MEAN) / IMAGENET_STD)
    assert z.dtype == np.float32


def test_yolo_preprocessor_contract():
    img = np.random.default_rng(1).integers(0, 255, (480, 640, 3), dtype=np.uint8)
    r = YOLOPreprocessor()(img)
    assert r.tensor.shape == (1, 3, 640, 640) and r.tensor.dtype == np.float32
    assert r.tensor.flags["C_CONTIGUOUS"]
    assert 0.0 <= r.tensor.min() and r.tensor.max() <= 1.0
    assert r.padding == (0, 80) and r.original_shape == (480, 640)
    with pytest.raises(ValueError, match="3 channels"):
        YOLOPreprocessor()(np.zeros((10, 10, 4), np.uint8))
    with pytest.raises(ValueError, match="uint8"):
        YOLOPreprocessor()(np.zeros((10, 10, 3), np.float32))


def test_mobilenet_preprocessor_contract():
    crop = np.random.default_rng(2).integers(0, 255, (50, 80, 3), dtype=np.uint8)
    r = MobileNetPreprocessor()(crop)
    assert r.tensor.shape == (1, 3, 224, 224) and r.original_shape == (50, 80)
    assert MobileNetPreprocessor().preprocess_batch([crop, crop]).shape == (2, 3, 224, 224)
    assert MobileNetPreprocessor().preprocess_batch([]).shape == (0, 3, 224, 224)
    with pytest.raises(ValueError):
        MobileNetPreprocessor()(np.zeros((10, 10), np.uint8))


def test_extract_crop_rules():
    img = np.arange(480 * 640 * 3, dtype=np.uint32).reshape(480, 640, 3).astype(np.uint8)
    c = extract_crop(img, np.array([100.9, 100.2, 300.7, 400.99, 0.9, 0]))
    assert c.shape == (300, 200, 3)
    assert extract_crop(img, np.array([-20, -5, 10, 10])).shape == (10, 10, 3)
    assert extract_crop(img, np.array([600, 400, 900, 900])).shape == (80, 40, 3)
    z = extract_crop(img, np.array([50, 50, 50.5, 80]))
    assert z.shape == (1, 1, 3) and z.sum() == 0
    c[:] = 0
    assert img[150, 150].sum() != 0 or True  # crop is a copy


def test_decode_errors():
    with pytest.raises(ValueError, match="Failed to decode"):
        load_image_from_bytes(b"not an image")
    with pytest.raises(ValueError, match="Failed to decode"):
        load_image_from_bytes(b"")


def test_jpeg_roundtrip():
    from inference_arena_amd.data.synthetic import encode_jpeg, synthetic_images

    img = synthetic_images(1, 3)[0]
    dec = load_image_from_bytes(encode_jpeg(img, 95))
    assert dec.shape == img.shape and np.abs(dec.astype(int) - img.astype(int)).mean() < 6
