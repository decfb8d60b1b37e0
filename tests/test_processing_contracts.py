"""More host-preprocessing behavioural contracts, following the reference's
tests/shared/test_processing.py (letterbox :62-123, ImageNet values :149-170,
scale_boxes :173-219, decode errors :222-243, preprocessors :255-584,
extract_crop :587-643, end-to-end chain :651-691)."""
from __future__ import annotations

import io

import numpy as np
import pytest
from PIL import Image

from inference_arena_amd.processing import (
    IMAGENET_MEAN,
    IMAGENET_STD,
    MobileNetPreprocessor,
    YOLOPreprocessor,
    extract_crop,
    imagenet_normalize,
    letterbox,
    letterbox_geometry,
    load_image,
    load_image_from_bytes,
    resize_bilinear,
    scale_boxes,
)
from inference_arena_amd.processing.mobilenet_preprocess import crop_bounds


@pytest.mark.parametrize("hw", [(640, 640), (480, 640), (640, 480), (100, 1000), (1000, 100), (1, 1), (7, 3000)])
def test_letterbox_shapes_and_content_area(hw):
    h, w = hw
    img = np.full((h, w, 3), 10, np.uint8)
    out, scale, (pw, ph) = letterbox(img, 640)
    assert out.shape == (640, 640, 3) and out.dtype == np.uint8
    s, nw, nh, pw2, ph2 = letterbox_geometry(h, w, 640)
    assert (pw, ph) == (pw2, ph2) and scale == s
    assert nw <= 640 and nh <= 640 and max(nw, nh) == 640 or min(h, w) * s < 1
    # content region is the image colour, everything else is the pad colour
    assert (out[ph:ph + nh, pw:pw + nw] == 10).all()
    mask = np.ones((640, 640), bool)
    mask[ph:ph + nh, pw:pw + nw] = False
    assert (out[mask] == 114).all()


def test_letterbox_square_input_is_exact_resize():
    img = np.random.default_rng(0).integers(0, 255, (640, 640, 3), dtype=np.uint8)
    out, scale, pad = letterbox(img, 640)
    assert scale == 1.0 and pad == (0, 0)
    assert np.array_equal(out, img)


def test_letterbox_scale_is_min_ratio_and_sizes_truncate():
    for h, w in ((333, 500), (427, 640), (612, 612), (375, 500)):
        s, nw, nh, pw, ph = letterbox_geometry(h, w, 640)
        assert s == min(640 / h, 640 / w)
        assert nw == int(w * s) and nh == int(h * s)  # int() truncation, not round()
        assert pw == (640 - nw) // 2 and ph == (640 - nh) // 2  # floor-centred


def test_letterbox_custom_color_and_size():
    out, _, (pw, ph) = letterbox(np.zeros((10, 20, 3), np.uint8), 320, color=(1, 2, 3))
    assert out.shape == (320, 320, 3)
    assert out[0, 0].tolist() == [1, 2, 3]


def test_letterbox_does_not_modify_input():
    img = np.random.default_rng(1).integers(0, 255, (50, 70, 3), dtype=np.uint8)
    before = img.copy()
    letterbox(img, 640)
    assert np.array_equal(img, before)


def test_resize_downsample_and_dtype():
    img = np.random.default_rng(2).integers(0, 255, (100, 80, 3), dtype=np.uint8)
    out = resize_bilinear(img, 40, 50)
    assert out.shape == (50, 40, 3) and out.dtype == np.uint8
    f = resize_bilinear(img.astype(np.float32), 40, 50)
    assert f.dtype == np.float32
    assert np.abs(f - out.astype(np.float32)).max() <= 1.0


def test_resize_gradient_is_monotone():
    ramp = np.tile(np.arange(0, 256, 8, dtype=np.uint8)[None, :, None], (4, 1, 3))
    out = resize_bilinear(ramp, 100, 4)
    assert (np.diff(out[0, :, 0].astype(int)) >= 0).all()


@pytest.mark.parametrize("c", [0, 1, 2])
def test_imagenet_normalize_per_channel(c):
    img = np.zeros((1, 1, 3), np.uint8)
    img[0, 0, c] = 255
    out = imagenet_normalize(img)
    assert out[0, 0, c] == pytest.approx((1 - IMAGENET_MEAN[c]) / IMAGENET_STD[c], rel=1e-6)


def test_imagenet_normalize_float_inputs():
    f01 = imagenet_normalize(np.full((2, 2, 3), 0.5, np.float32))
    f255 = imagenet_normalize(np.full((2, 2, 3), 127.5, np.float32))
    assert np.allclose(f01, f255, atol=1e-6)
    assert np.allclose(f01[0, 0], (0.5 - IMAGENET_MEAN) / IMAGENET_STD)


def test_imagenet_constants():
    assert IMAGENET_MEAN.tolist() == pytest.approx([0.485, 0.456, 0.406])
    assert IMAGENET_STD.tolist() == pytest.approx([0.229, 0.224, 0.225])


def test_scale_boxes_identity_and_padding_only():
    b = np.array([[10, 20, 30, 40]], np.float32)
    assert np.allclose(scale_boxes(b, 1.0, (0, 0), (100, 100)), b)
    assert np.allclose(scale_boxes(b, 1.0, (5, 10), (100, 100)), [[5, 10, 25, 30]])
    assert np.allclose(scale_boxes(b, 2.0, (0, 0), (100, 100)), [[5, 10, 15, 20]])


def test_scale_boxes_keeps_extra_columns_and_empty():
    b = np.array([[10, 20, 30, 40, 0.75, 3]], np.float32)
    out = scale_boxes(b, 0.5, (0, 0), (1000, 1000))
    assert out[0, 4] == pytest.approx(0.75) and out[0, 5] == 3
    e = scale_boxes(np.zeros((0, 6), np.float32), 0.5, (0, 0), (10, 10))
    assert e.shape == (0, 6)


def test_scale_boxes_roundtrip_through_letterbox():
    h, w = 480, 640
    s, nw, nh, pw, ph = letterbox_geometry(h, w, 640)
    orig = np.array([[100, 50, 300, 400]], np.float32)
    lb = orig.copy()
    lb[:, [0, 2]] = lb[:, [0, 2]] * s + pw
    lb[:, [1, 3]] = lb[:, [1, 3]] * s + ph
    back = scale_boxes(lb, s, (pw, ph), (h, w))
    assert np.allclose(back, orig, atol=1e-3)


def test_load_image_errors_and_formats(tmp_path):
    with pytest.raises(ValueError, match="Failed to load"):
        load_image(tmp_path / "missing.jpg")
    img = np.random.default_rng(3).integers(0, 255, (20, 30, 3), dtype=np.uint8)
    for fmt, mode in (("PNG", "RGB"), ("PNG", "L"), ("PNG", "RGBA"), ("BMP", "RGB")):
        pil = Image.fromarray(img).convert(mode)
        buf = io.BytesIO()
        pil.save(buf, format=fmt)
        dec = load_image_from_bytes(buf.getvalue())
        assert dec.shape == (20, 30, 3) and dec.dtype == np.uint8, (fmt, mode)
        if mode == "RGB":
            assert np.array_equal(dec, img)
    p = tmp_path / "x.png"
    Image.fromarray(img).save(p)
    assert np.array_equal(load_image(p), img)
    assert np.array_equal(load_image(str(p)), img)


def test_yolo_preprocessor_values_and_geometry():
    img = np.full((320, 640, 3), 255, np.uint8)
    r = YOLOPreprocessor()(img)
    t = r.tensor[0]
    assert r.scale == 1.0 and r.padding == (0, 160)
    assert t[:, 160:480].min() == pytest.approx(1.0)
    assert t[:, :160].max() == pytest.approx(114 / 255, rel=1e-6)
    assert YOLOPreprocessor().get_input_shape() == (1, 3, 640, 640)
    assert YOLOPreprocessor.get_input_dtype() == np.float32


def test_yolo_preprocessor_scale_back():
    img = np.zeros((480, 640, 3), np.uint8)
    r = YOLOPreprocessor()(img)
    boxes = np.array([[0, 80, 640, 560, 0.9, 1]], np.float32)
    out = r.scale_boxes_to_original(boxes)
    assert out[0, :4].tolist() == pytest.approx([0, 0, 640, 480])


@pytest.mark.parametrize("bad,msg", [
    ([[1, 2, 3]], "numpy array"),
    (np.zeros((10, 10), np.uint8), "3D"),
    (np.zeros((10, 10, 1), np.uint8), "3 channels"),
    (np.zeros((10, 10, 3), np.float64), "uint8"),
])
def test_yolo_preprocessor_validation(bad, msg):
    with pytest.raises(ValueError, match=msg):
        YOLOPreprocessor()(bad)


def test_mobilenet_preprocessor_values():
    crop = np.zeros((10, 10, 3), np.uint8)
    t = MobileNetPreprocessor()(crop).tensor
    assert t.shape == (1, 3, 224, 224) and t.dtype == np.float32 and t.flags["C_CONTIGUOUS"]
    for c in range(3):
        assert np.allclose(t[0, c], -IMAGENET_MEAN[c] / IMAGENET_STD[c])
    f = MobileNetPreprocessor()(np.zeros((10, 10, 3), np.float32)).tensor
    assert np.allclose(f, t)
    assert MobileNetPreprocessor(112)(crop).tensor.shape == (1, 3, 112, 112)


def test_mobilenet_preprocessor_no_aspect_preservation():
    crop = np.zeros((10, 100, 3), np.uint8)
    crop[:, 50:] = 255
    t = MobileNetPreprocessor()(crop).tensor[0, 0]
    # direct resize: the left half of every output row is dark, the right half bright
    assert t[:, :100].max() < 0 < t[:, 130:].min()


@pytest.mark.parametrize("bad,msg", [
    ("crop", "numpy array"),
    (np.zeros((10, 10), np.uint8), "3D"),
    (np.zeros((10, 10, 4), np.uint8), "3 channels"),
    (np.zeros((10, 10, 3), np.int32), "uint8 or float32"),
    (np.zeros((0, 10, 3), np.uint8), "Invalid crop dimensions"),
])
def test_mobilenet_preprocessor_validation(bad, msg):
    with pytest.raises(ValueError, match=msg):
        MobileNetPreprocessor()(bad)


def test_crop_bounds_truncation_and_clamp():
    assert crop_bounds([10.9, 20.1, 30.99, 40.5], 100, 100) == (10, 20, 30, 40)
    assert crop_bounds([-5.5, -1, 150, 120], 100, 100) == (0, 0, 100, 100)


def test_extract_crop_is_a_copy_and_content():
    img = np.random.default_rng(4).integers(1, 255, (100, 120, 3), dtype=np.uint8)
    c = extract_crop(img, [10, 20, 50, 60])
    assert c.shape == (40, 40, 3)
    assert np.array_equal(c, img[20:60, 10:50])
    c[:] = 0
    assert img[20:60, 10:50].min() >= 1  # writing the crop leaves the image untouched


@pytest.mark.parametrize("box", [[50, 50, 50, 80], [50, 50, 80, 50], [80, 80, 50, 50], [200, 200, 300, 300],
                                 [-30, -30, -10, -10]])
def test_extract_crop_empty_boxes_give_black_pixel(box):
    img = np.full((100, 100, 3), 9, np.uint8)
    c = extract_crop(img, box)
    assert c.shape == (1, 1, 3) and c.dtype == np.uint8 and c.sum() == 0


def test_end_to_end_preprocessing_chain():
    """decode -> YOLO tensor -> boxes back to the original frame -> crops -> MobileNet batch."""
    from inference_arena_amd.data.synthetic import encode_jpeg, synthetic_images

    img = synthetic_images(1, 11)[0]
    dec = load_image_from_bytes(encode_jpeg(img, 95))
    yr = YOLOPreprocessor()(dec)
    assert yr.tensor.shape == (1, 3, 640, 640)
    h, w = dec.shape[:2]
    s, nw, nh, pw, ph = letterbox_geometry(h, w, 640)
    boxes_lb = np.array([[pw + 10, ph + 10, pw + 100, ph + 60, 0.9, 0], [pw, ph, pw + nw, ph + nh, 0.8, 1]],
                        np.float32)
    boxes = yr.scale_boxes_to_original(boxes_lb)
    assert (boxes[:, [0, 2]] <= w).all() and (boxes[:, [1, 3]] <= h).all()
    crops = [extract_crop(dec, b) for b in boxes]
    batch = MobileNetPreprocessor().preprocess_batch(crops)
    assert batch.shape == (2, 3, 224, 224) and np.isfinite(batch).all()
