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


def _same_topk(a, b, tol=1e-4, boxes=None):
    """fp32 programs of other crop capacities sum in other orders (the 14x14 blocks split their hidden channels
    over more workgroups at small capacities, engine/plans.py irx_slices; the split detector is tuned on its own):
    logits agree to ~1e-6, so the top-5 may only differ where two logits are within that of each other.  With
    ``boxes`` (both sides' detections) only crops whose integer window (int() of each coordinate, the reference's
    crop rule) is the same are compared: a box ~1e-5 px from an integer crops one pixel row / column apart."""
    rows = np.arange(len(a.topk_idx))
    if boxes is not None:
        win = lambda bx: tuple(int(v) for v in bx[:4])  # noqa: E731
        rows = np.array([i for i, (p, q) in enumerate(zip(*boxes)) if win(p) == win(q)], dtype=np.int64)
        assert len(rows) >= 0.8 * len(a.topk_idx), "too many crops moved between the programs"
    np.testing.assert_allclose(a.topk_logit[rows], b.topk_logit[rows], rtol=tol, atol=tol)
    for ia, ib, la in zip(a.topk_idx[rows], b.topk_idx[rows], a.topk_logit[rows]):
        for j in np.nonzero(ia != ib)[0]:
            gaps = [abs(la[j] - la[k]) for k in (j - 1, j + 1) if 0 <= k < len(la)]
            assert min(gaps) <= 2 * tol * (1 + abs(la[j])), (ia, ib, la)


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
        np.testing.assert_array_equal(a.classes, b.classes)
        if dtype == "bf16":
            np.testing.assert_array_equal(a.topk_idx, b.topk_idx)
        else:
            _same_topk(a, b)


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
        _same_topk(a, b, boxes=(a.boxes, b.boxes))
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
        from types import SimpleNamespace

        _same_topk(a, SimpleNamespace(topk_idx=np.asarray(d["topk_idx"]), topk_logit=np.asarray(d["topk_logit"])),
                   boxes=(a.boxes, np.asarray(d["det"])[:, :4]))
