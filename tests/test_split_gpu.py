"""Split topology (detection on one GPU, classification on another, crops handed over device to device:
csrc/runtime/split.h) vs the fused single-GPU program.  On a one-GPU box both stages share device 0 and
the hand-off is a device-to-device copy; on a node the same code issues hipMemcpyPeerAsync over xGMI."""
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


def _other_gpu() -> int:
    return 1 if torch.cuda.device_count() > 1 else 0


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_split_matches_fused(dense_models, device, dtype):
    from inference_arena_amd.data.synthetic import synthetic_images
    from inference_arena_amd.engine.pipeline import GpuPipeline, SplitPipeline

    imgs = synthetic_images(7, 81) + synthetic_images(1, 82, hw=(333, 500))
    fused = GpuPipeline(*dense_models, device=0, buckets=[8], dtype=dtype).infer(imgs)
    split = SplitPipeline(*dense_models, det_device=0, cls_device=_other_gpu(), buckets=[8], dtype=dtype)
    got = split.infer(imgs)
    assert sum(len(r) for r in fused) > 5
    for a, b in zip(fused, got):
        assert len(a) == len(b)
        if dtype == "bf16":
            np.testing.assert_array_equal(a.boxes, b.boxes)
            np.testing.assert_allclose(a.topk_logit, b.topk_logit, rtol=1e-6, atol=1e-6)
        else:
            # the split detector / classifier programs are tuned on their own: other conv tilings of the
            # same layers, i.e. other fp32 summation orders (~1e-5 relative after 60 layers and the DFL)
            np.testing.assert_allclose(a.boxes, b.boxes, rtol=2e-5, atol=5e-3)
            np.testing.assert_allclose(a.topk_logit, b.topk_logit, rtol=1e-4, atol=1e-4)
        np.testing.assert_array_equal(a.classes, b.classes)
        np.testing.assert_array_equal(a.topk_idx, b.topk_idx)


def test_split_overflow_passes_and_batcher(dense_models, device):
    """More crops than one classification pass holds (extra passes on the classifier GPU), and the split
    instance scheduled by the native dynamic batcher."""
    from inference_arena_amd.data.synthetic import synthetic_images
    from inference_arena_amd.engine.pipeline import GpuPipeline, SplitPipeline
    from inference_arena_amd.ops import native

    imgs = synthetic_images(4, 21)
    ref = GpuPipeline(*dense_models, device=0, buckets=[4], dtype="fp32", crop_cap_per_image=64).infer(imgs)
    split = SplitPipeline(*dense_models, det_device=0, cls_device=_other_gpu(), buckets=[1, 4], dtype="fp32",
                          crop_cap_per_image=1)
    got = split.infer(imgs)
    assert sum(len(r) for r in got) > 16
    for a, b in zip(ref, got):
        np.testing.assert_array_equal(a.topk_idx, b.topk_idx)
    bat = native().DynamicBatcher([split.instance], {"max_batch": 4, "max_queue_delay_us": 2000})
    done = threading.Event()
    res = {}

    def cb(d):
        res[int(d["id"])] = d
        if len(res) == len(imgs):
            done.set()

    ids = [bat.enqueue(np.ascontiguousarray(im), cb) for im in imgs]
    assert done.wait(60)
    bat.shutdown()
    for i, a in zip(ids, ref):
        d = res[i]
        assert not d["error"], d["error"]
        assert d["det_count"] == len(a)
        np.testing.assert_array_equal(d["topk_idx"], a.topk_idx)
