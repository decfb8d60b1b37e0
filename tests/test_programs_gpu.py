"""Split-service and reference-tensor-contract programs on the native executor (MI355X only).

* ``GpuTensorModel`` (model-server tensor models, reference contract
  ``yolov5n``: FP32 [3,640,640] -> [84,8400]; ``mobilenetv2``: FP32
  [3,224,224] -> [1000]) vs the fp32 torch models of the same weights.
* ``GpuDetector`` / ``GpuClassifier`` (microservices arm) vs the fused
  ``GpuPipeline``: identical kernels per image, so results agree exactly.
"""
from __future__ import annotations

import threading

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dense_models():
    from inference_arena_amd.models.zoo import make_mobilenet, make_yolo

    return make_yolo(0, cls_shift=-20.0), make_mobilenet(1)


@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
def test_yolo_tensor_model_matches_torch(dense_models, device, dtype):
    from inference_arena_amd.data.synthetic import synthetic_images
    from inference_arena_amd.engine.pipeline import GpuTensorModel
    from inference_arena_amd.processing import YOLOPreprocessor

    yolo, _ = dense_models
    tm = GpuTensorModel.yolo(yolo, device=0, buckets=[1, 4], dtype=dtype)
    pre = YOLOPreprocessor()
    xs = np.concatenate([pre(im).tensor for im in synthetic_images(3, 31)], 0)
    got = tm.infer(xs)
    assert got.shape == (3, 84, 8400) and got.dtype == np.float32
    with torch.no_grad():
        ref = yolo.eval()(torch.from_numpy(xs)).numpy()
    # class scores are sigmoids: absolute error; boxes: error relative to the 640 canvas
    cls_err = np.abs(got[:, 4:] - ref[:, 4:])
    assert np.quantile(cls_err, 0.999) < 0.05, np.quantile(cls_err, 0.999)
    box_err = np.abs(got[:, :4] - ref[:, :4])
    assert np.median(box_err) < 1.0 and np.quantile(box_err, 0.99) < 8.0, (np.median(box_err), box_err.max())


@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
def test_mobilenet_tensor_model_matches_torch(dense_models, device, dtype):
    from inference_arena_amd.data.synthetic import synthetic_images
    from inference_arena_amd.engine.pipeline import GpuTensorModel
    from inference_arena_amd.processing import MobileNetPreprocessor

    _, mnet = dense_models
    tm = GpuTensorModel.mobilenet(mnet, device=0, buckets=[2, 8], dtype=dtype)
    xs = MobileNetPreprocessor().preprocess_batch(synthetic_images(5, 37))
    got = tm.infer(xs)
    assert got.shape == (5, 1000)
    with torch.no_grad():
        ref = mnet.eval()(torch.from_numpy(xs)).numpy()
    rel = np.abs(got - ref) / (np.abs(ref).max(1, keepdims=True) + 1e-6)
    assert np.median(rel) < 0.02 and rel.max() < 0.2, (np.median(rel), rel.max())
    assert (got.argmax(1) == ref.argmax(1)).mean() >= 0.6


@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
def test_detector_and_classifier_match_fused_pipeline(dense_models, device, dtype):
    from inference_arena_amd.data.synthetic import synthetic_images
    from inference_arena_amd.engine.pipeline import GpuClassifier, GpuDetector, GpuPipeline
    from inference_arena_amd.processing import extract_crop

    yolo, mnet = dense_models
    imgs = synthetic_images(5, 41)
    fused = GpuPipeline(yolo, mnet, device=0, buckets=[8], dtype=dtype).infer(imgs)
    det = GpuDetector(yolo, device=0, buckets=[8], dtype=dtype).infer(imgs)
    cls = GpuClassifier(mnet, device=0, buckets=[4, 16], dtype=dtype)
    assert sum(len(r) for r in fused) > 3
    for im, f, d in zip(imgs, fused, det):
        assert len(f) == len(d)
        if dtype == "bf16":
            np.testing.assert_array_equal(f.boxes, d.boxes)
        else:
            # the detector-only program is tuned on its own (conv tile choices differ from the fused
            # program's), and a different tiling is a different fp32 summation order
            np.testing.assert_allclose(f.boxes, d.boxes, rtol=1e-5, atol=2e-3)
        np.testing.assert_array_equal(f.classes, d.classes)
        if len(f) == 0:
            continue
        crops = [extract_crop(im, np.concatenate([b, [s, c]])) for b, s, c in zip(f.boxes, f.scores, f.classes)]
        out = cls.infer(crops)
        for k, (idx, logit, prob) in enumerate(out):
            np.testing.assert_array_equal(idx, f.topk_idx[k])
            tol = 1e-5 if dtype == "bf16" else 1e-4
            np.testing.assert_allclose(logit, f.topk_logit[k], rtol=tol, atol=tol)


def test_batcher_tensor_requests(dense_models, device):
    """Dynamic batcher over a raw-output executor: tensor in, per-request raw tensor out."""
    from inference_arena_amd.engine.pipeline import GpuTensorModel
    from inference_arena_amd.ops import native

    _, mnet = dense_models
    tm = GpuTensorModel.mobilenet(mnet, device=0, buckets=[4])
    C = native()
    b = C.DynamicBatcher([tm.ex], {"max_batch": 4, "max_queue_delay_us": 2000})
    rng = np.random.default_rng(0)
    xs = [rng.standard_normal((3, 224, 224)).astype(np.float32) for _ in range(6)]
    direct = tm.infer(xs)
    done = threading.Event()
    results = {}

    def cb(d):
        results[int(d["id"])] = d
        if len(results) == len(xs):
            done.set()

    ids = [b.enqueue(x, cb) for x in xs]
    assert done.wait(30)
    b.shutdown()
    for i, rid in enumerate(ids):
        d = results[rid]
        assert d["error"] == ""
        np.testing.assert_allclose(d["raw"].view(np.float32), direct[i], rtol=1e-5, atol=1e-5)
