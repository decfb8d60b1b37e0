"""End-to-end: native GPU pipeline vs the fp32 torch/NumPy reference pipeline."""
from __future__ import annotations

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _iou(a, b):
    x1 = np.maximum(a[:, None, 0], b[None, :, 0])
    y1 = np.maximum(a[:, None, 1], b[None, :, 1])
    x2 = np.minimum(a[:, None, 2], b[None, :, 2])
    y2 = np.minimum(a[:, None, 3], b[None, :, 3])
    inter = np.clip(x2 - x1, 0, None) * np.clip(y2 - y1, 0, None)
    aa = (a[:, 2] - a[:, 0]) * (a[:, 3] - a[:, 1])
    bb = (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])
    return inter / (aa[:, None] + bb[None, :] - inter + 1e-9)


@pytest.fixture(scope="module")
def dense_models():
    from inference_arena_amd.models.zoo import make_mobilenet, make_yolo

    return make_yolo(0, cls_shift=-20.0), make_mobilenet(1)


@pytest.fixture(scope="module")
def gpu_pipe(dense_models, device):
    from inference_arena_amd.engine.pipeline import GpuPipeline

    return GpuPipeline(*dense_models, device=0, buckets=[1, 4, 8], dtype="bf16")


def test_pipeline_matches_reference(gpu_pipe, dense_models):
    """bf16 GPU pipeline vs fp32 reference: same detections (class-agnostic IoU > 0.7) for the
    large majority, similar counts, and classifier logits of matched crops within a few percent."""
    from inference_arena_amd.data.synthetic import synthetic_images
    from inference_arena_amd.engine.reference import ReferencePipeline

    imgs = synthetic_images(6, 21)
    ref = ReferencePipeline(*dense_models, device="cpu")
    got = gpu_pipe.infer(imgs)
    n_ref = n_got = n_match = n_cls = 0
    rel = []
    for im, g in zip(imgs, got):
        r = ref(im)
        n_ref += len(r)
        n_got += len(g)
        if len(r) == 0 or len(g) == 0:
            continue
        iou = _iou(g.boxes, r.boxes)
        for j in range(len(r)):
            i = int(np.argmax(iou[:, j]))
            if iou[i, j] > 0.7:
                n_match += 1
                n_cls += int(g.topk_idx[i, 0] == r.topk_idx[j, 0])
                rel.append(abs(g.topk_logit[i, 0] - r.topk_logit[j, 0]) / (abs(r.topk_logit[j, 0]) + 1.0))
    assert n_ref > 5, "test images should produce detections"
    assert abs(n_got - n_ref) <= 0.3 * n_ref, (n_got, n_ref)
    assert n_match >= 0.75 * n_ref, (n_match, n_ref)
    assert n_cls >= 0.5 * n_match, (n_cls, n_match)
    assert np.median(rel) < 0.1, np.median(rel)


def test_buckets_and_partial_batches(gpu_pipe):
    from inference_arena_amd.data.synthetic import synthetic_images

    imgs = synthetic_images(7, 5)
    full = gpu_pipe.infer(imgs)  # bucket 8, 7 live images
    single = [gpu_pipe.infer([im])[0] for im in imgs]  # bucket 1
    for a, b in zip(full, single):
        assert len(a) == len(b)
        if len(a):
            np.testing.assert_allclose(a.boxes, b.boxes, atol=1e-3)
            np.testing.assert_array_equal(a.topk_idx, b.topk_idx)


def test_overflow_crops_extra_pass(dense_models, device):
    """More crops than one classification pass holds -> executor runs extra passes."""
    from inference_arena_amd.data.synthetic import synthetic_images
    from inference_arena_amd.engine.pipeline import GpuPipeline

    tiny = GpuPipeline(*dense_models, device=0, buckets=[4], crop_cap_per_image=1, dtype="bf16")
    big = GpuPipeline(*dense_models, device=0, buckets=[4], crop_cap_per_image=64, dtype="bf16")
    imgs = synthetic_images(4, 21)
    a, b = tiny.infer(imgs), big.infer(imgs)
    assert sum(len(r) for r in a) > 16  # exceeds the tiny pass capacity (max(16, 4*1))
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x.topk_idx, y.topk_idx)
        np.testing.assert_allclose(x.topk_logit, y.topk_logit, rtol=1e-5, atol=1e-5)


def test_fused_stem_matches_unfused(dense_models, device, monkeypatch):
    """stem_fused (letterbox / crop gather computed into LDS inside the stem convs) vs the unfused
    letterbox_s2d + conv and crop_gather_s2d + conv programs: same stem activations and results."""
    from inference_arena_amd.data.synthetic import synthetic_images
    from inference_arena_amd.engine.pipeline import GpuPipeline

    imgs = synthetic_images(5, 33) + synthetic_images(1, 34, hw=(333, 500))
    monkeypatch.setenv("ARENA_FUSE_STEM", "0")
    plain = GpuPipeline(*dense_models, device=0, buckets=[8], share_buffers=False, dtype="bf16")  # keep b0 readable
    monkeypatch.setenv("ARENA_FUSE_STEM", "1")
    fused = GpuPipeline(*dense_models, device=0, buckets=[8], share_buffers=False, dtype="bf16")
    assert any(int(op[0]) == 15 for op in fused.program.ops) and not any(int(op[0]) == 15 for op in plain.program.ops)
    a, b = plain.infer(imgs), fused.infer(imgs)
    for i in range(len(imgs)):
        # b1 = output of the conv after the stem (fused into the same kernel unless ARENA_FUSE_STEM2=0)
        s_plain, s_fused = plain.read_buffer("b1", 8, i), fused.read_buffer("b1", 8, i)
        np.testing.assert_allclose(s_fused, s_plain, atol=0.03 + 0.01 * np.abs(s_plain).max())
    for x, y in zip(a, b):
        assert len(x) == len(y)
        if len(x):
            np.testing.assert_allclose(y.boxes, x.boxes, atol=0.5)
            assert (x.topk_idx[:, 0] == y.topk_idx[:, 0]).mean() >= 0.9
            np.testing.assert_allclose(y.topk_logit[:, 0], x.topk_logit[:, 0], rtol=0.05, atol=0.05)


def test_two_stage_stem_matches_single_stage(dense_models, device, monkeypatch):
    """letterbox + stem + 3x3 s2 conv in one kernel (stem output in LDS) vs the single-stage fused
    stem followed by the separate conv: same b1 activations (bitwise up to MFMA summation order)."""
    from inference_arena_amd.data.synthetic import synthetic_images
    from inference_arena_amd.engine.pipeline import GpuPipeline

    imgs = synthetic_images(3, 61) + synthetic_images(1, 62, hw=(333, 500)) + synthetic_images(1, 63, hw=(640, 427))
    monkeypatch.setenv("ARENA_FUSE_STEM2", "0")
    one = GpuPipeline(*dense_models, device=0, buckets=[8], share_buffers=False, dtype="bf16")
    monkeypatch.setenv("ARENA_FUSE_STEM2", "1")
    two = GpuPipeline(*dense_models, device=0, buckets=[8], share_buffers=False, dtype="bf16")
    assert any(int(op[0]) == 15 and int(op[20]) for op in two.program.ops)
    assert not any(int(op[0]) == 15 and int(op[20]) for op in one.program.ops)
    a, b = one.infer(imgs), two.infer(imgs)
    for i in range(len(imgs)):
        x1, x2 = one.read_buffer("b1", 8, i), two.read_buffer("b1", 8, i)
        np.testing.assert_allclose(x2, x1, atol=0.02 + 0.01 * np.abs(x1).max())
    for x, y in zip(a, b):
        assert len(x) == len(y)


def test_stem_first_block_matches_unfused(dense_models, device, monkeypatch):
    """crop gather + stem + MobileNetV2 block 1 in one kernel (stem output in LDS) vs the fused stem
    followed by the ir_block kernel: same block-1 activations and classifications."""
    from inference_arena_amd.data.synthetic import synthetic_images
    from inference_arena_amd.engine.pipeline import GpuPipeline

    imgs = synthetic_images(4, 71) + synthetic_images(1, 72, hw=(333, 500))
    monkeypatch.setenv("ARENA_FUSE_STEM_IR", "0")
    one = GpuPipeline(*dense_models, device=0, buckets=[8], share_buffers=False, dtype="bf16")
    monkeypatch.setenv("ARENA_FUSE_STEM_IR", "1")
    two = GpuPipeline(*dense_models, device=0, buckets=[8], share_buffers=False, dtype="bf16")
    assert any(int(op[0]) == 15 and int(op[26]) for op in two.program.ops)
    assert not any(int(op[0]) == 15 and int(op[26]) for op in one.program.ops)
    a, b = one.infer(imgs), two.infer(imgs)
    n = sum(len(r) for r in a)
    assert n > 0
    for c in range(min(n, 12)):
        x1, x2 = one.read_buffer("m0.out", 8, c), two.read_buffer("m0.out", 8, c)
        np.testing.assert_allclose(x2, x1, atol=0.03 + 0.01 * np.abs(x1).max())
    for x, y in zip(a, b):
        assert len(x) == len(y)
        if len(x):
            assert (x.topk_idx[:, 0] == y.topk_idx[:, 0]).mean() >= 0.9


def test_fused_head_pool_matches_unfused(dense_models, device, monkeypatch):
    """MobileNetV2 head conv + global average pool as one kernel (head_pool) vs conv + avgpool: same pooled
    features (fp32 sum before one bf16 rounding vs per-pixel bf16) and the same classifications."""
    from inference_arena_amd.data.synthetic import synthetic_images
    from inference_arena_amd.engine.pipeline import GpuPipeline

    imgs = synthetic_images(4, 51)
    monkeypatch.setenv("ARENA_FUSE_POOL", "0")
    plain = GpuPipeline(*dense_models, device=0, buckets=[4], share_buffers=False, dtype="bf16")
    monkeypatch.setenv("ARENA_FUSE_POOL", "1")
    fused = GpuPipeline(*dense_models, device=0, buckets=[4], share_buffers=False, dtype="bf16")
    assert any(int(op[0]) == 17 for op in fused.program.ops) and not any(int(op[0]) == 17 for op in plain.program.ops)
    a, b = plain.infer(imgs), fused.infer(imgs)
    n = sum(len(r) for r in a)
    assert n > 0
    for c in range(min(n, 8)):
        pa, pb = plain.read_buffer("m.pool", 4, c), fused.read_buffer("m.pool", 4, c)
        np.testing.assert_allclose(pb, pa, atol=0.02 + 0.01 * np.abs(pa).max())
    for x, y in zip(a, b):
        assert len(x) == len(y)
        if len(x):
            assert (x.topk_idx[:, 0] == y.topk_idx[:, 0]).mean() >= 0.9
            np.testing.assert_allclose(y.topk_logit[:, 0], x.topk_logit[:, 0], rtol=0.03, atol=0.05)


def test_fused_head_pointwise_matches_unfused(dense_models, device, monkeypatch):
    """Detect head: second 3x3 of each branch with the final 1x1 fused into its epilogue (v3 kernel) vs
    the separate 3x3 + 1x1 convs: same head outputs at every level and the same detections."""
    from inference_arena_amd.data.synthetic import synthetic_images
    from inference_arena_amd.engine.pipeline import GpuPipeline

    imgs = synthetic_images(4, 41)
    monkeypatch.setenv("ARENA_FUSE_HEAD", "0")
    plain = GpuPipeline(*dense_models, device=0, buckets=[4], share_buffers=False, dtype="bf16")
    monkeypatch.setenv("ARENA_FUSE_HEAD", "1")
    fused = GpuPipeline(*dense_models, device=0, buckets=[4], share_buffers=False, dtype="bf16")
    n_pw = sum(1 for op in fused.program.ops if int(op[0]) == 1 and int(op[34]) > 0)
    assert n_pw == 6 and len(fused.program.ops) == len(plain.program.ops) - 6
    a, b = plain.infer(imgs), fused.infer(imgs)
    for lvl in range(3):
        for i in range(len(imgs)):
            x, y = plain.read_buffer(f"det{lvl}.out", 4, i), fused.read_buffer(f"det{lvl}.out", 4, i)
            np.testing.assert_allclose(y, x, atol=0.05 + 0.01 * np.abs(x).max())
    for x, y in zip(a, b):
        assert abs(len(x) - len(y)) <= 1
        if len(x) == len(y) and len(x):
            np.testing.assert_allclose(y.boxes, x.boxes, atol=1.0)


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_head_lanes_match_sequential(dense_models, device, monkeypatch, dtype):
    """ARENA_HEAD_LANES=1: the Detect head's three levels run as parallel graph branches on side streams; the
    kernels and each branch's order are unchanged, so the results are bit-identical to the sequential program
    (buckets 1 and 8, several batches through the captured graphs)."""
    from inference_arena_amd.data.synthetic import synthetic_images
    from inference_arena_amd.engine.pipeline import GpuPipeline

    imgs = synthetic_images(7, 61) + synthetic_images(1, 62, hw=(333, 500))
    monkeypatch.setenv("ARENA_HEAD_LANES", "0")
    seq = GpuPipeline(*dense_models, device=0, buckets=[1, 2, 8], dtype=dtype)
    monkeypatch.setenv("ARENA_HEAD_LANES", "1")
    par = GpuPipeline(*dense_models, device=0, buckets=[1, 2, 8], dtype=dtype)
    assert par.program.ops[:, 46].any() and not seq.program.ops[:, 46].any()
    for batch in (imgs, imgs[:1], imgs[3:5], imgs[3:]):  # buckets 8, 1, 2 (lanes: B <= 2), 8
        for a, b in zip(seq.infer(batch), par.infer(batch)):
            np.testing.assert_array_equal(a.boxes, b.boxes)
            np.testing.assert_array_equal(a.topk_idx, b.topk_idx)
            np.testing.assert_array_equal(a.topk_logit, b.topk_logit)


@pytest.mark.parametrize("kind", ["detector", "split"])
def test_head_lanes_detector_programs_through_batcher(dense_models, device, monkeypatch, kind):
    """Lanes in the detector-only program (arm B detection service) and the split topology's detector stage,
    buckets 1 / 2 / 4, driven by concurrent requests through the native DynamicBatcher (its instance thread
    submits and collects, several slots in flight): the same answers as the lanes-off programs."""
    import asyncio

    from inference_arena_amd.data.synthetic import synthetic_images
    from inference_arena_amd.engine.registry import build_session
    from inference_arena_amd.server.batching import AsyncBatcher

    imgs = synthetic_images(10, 71) + synthetic_images(2, 72, hw=(333, 500))

    def make(lanes: str):
        monkeypatch.setenv("ARENA_HEAD_LANES", lanes)
        if kind == "split":
            return build_session("split", *dense_models, device=0, buckets=[1, 2, 4], cls_device=0)
        return build_session("detector", dense_models[0], device=0, buckets=[1, 2, 4])

    def drive(runner):
        b = AsyncBatcher([_SplitInst(runner) if kind == "split" else runner], max_batch=4, max_queue_delay_us=300)

        async def go():
            out = []
            for users in (1, 2, 3, 12):
                for r in range(3):
                    idx = [(r * users + k) % len(imgs) for k in range(users)]
                    out += list(zip(idx, await asyncio.gather(*(b.run(imgs[i]) for i in idx))))
            return out

        try:
            return asyncio.run(go())
        finally:
            b.close()

    seq, par = make("0"), make("1")
    prog = (par.det if kind == "split" else par).program
    assert prog.ops[:, 46].any()
    a, c = drive(seq), drive(par)
    assert [i for i, _ in a] == [i for i, _ in c]
    for (_, x), (_, y) in zip(a, c):
        assert x["det_count"] == y["det_count"]
        np.testing.assert_array_equal(x["det"], y["det"])
        np.testing.assert_array_equal(x["topk_idx"], y["topk_idx"])


class _SplitInst:
    """A SplitPipeline as a batcher instance (its native SplitInstance submits / collects)."""

    def __init__(self, sp):
        self.ex = sp.instance


def test_fused_c3_matches_unfused(dense_models, device, monkeypatch):
    """Whole C3 blocks as one kernel (160x160 c_=16 n=1, 80x80 c_=32 n=2, head P3 c_=32 n=1 without
    shortcut) vs the per-conv program: same block outputs and the same detections."""
    from inference_arena_amd.data.synthetic import synthetic_images
    from inference_arena_amd.engine.pipeline import GpuPipeline

    imgs = synthetic_images(3, 51) + synthetic_images(1, 52, hw=(333, 500))
    monkeypatch.setenv("ARENA_FUSE_C3", "0")
    plain = GpuPipeline(*dense_models, device=0, buckets=[4], share_buffers=False, dtype="bf16")
    monkeypatch.setenv("ARENA_FUSE_C3", "all")
    fused = GpuPipeline(*dense_models, device=0, buckets=[4], share_buffers=False, dtype="bf16")
    assert sum(1 for op in fused.program.ops if int(op[0]) == 16) == 3
    a, b = plain.infer(imgs), fused.infer(imgs)
    for name in ("b2", "cat16", "p3"):
        for i in range(len(imgs)):
            x, y = plain.read_buffer(name, 4, i), fused.read_buffer(name, 4, i)
            scale = np.abs(x).max()
            np.testing.assert_allclose(y, x, atol=0.03 + 0.02 * scale, err_msg=name)
    for x, y in zip(a, b):
        assert abs(len(x) - len(y)) <= 1
        if len(x) == len(y) and len(x):
            np.testing.assert_allclose(y.boxes, x.boxes, atol=1.5)


def test_overflow_passes_serialised_two_in_flight(dense_models, device, monkeypatch):
    """ARENA_CONCURRENT=0 (one stream, two slots): with two batches in flight, collect() of the first runs its
    overflow classification passes after the second batch's graph — every slot owns its arena and crop plan,
    so the results equal those of each batch run alone (aliased arenas mixed the batches)."""
    from inference_arena_amd.data.synthetic import synthetic_images
    from inference_arena_amd.engine.pipeline import GpuPipeline

    monkeypatch.setenv("ARENA_CONCURRENT", "0")
    tiny = GpuPipeline(*dense_models, device=0, buckets=[4], crop_cap_per_image=1, dtype="bf16")
    monkeypatch.delenv("ARENA_CONCURRENT")
    big = GpuPipeline(*dense_models, device=0, buckets=[4], crop_cap_per_image=64, dtype="bf16")
    a_imgs, b_imgs = synthetic_images(4, 21), synthetic_images(4, 45)
    sa = tiny.submit(a_imgs)
    sb = tiny.submit(b_imgs)  # second batch in flight before the first is collected
    ra, rb = tiny.collect(sa, len(a_imgs)), tiny.collect(sb, len(b_imgs))
    assert sum(len(r) for r in ra) > 16  # the first batch needs overflow passes (pass capacity 16)
    for got, imgs in ((ra, a_imgs), (rb, b_imgs)):
        for x, y in zip(got, big.infer(imgs)):
            np.testing.assert_array_equal(x.topk_idx, y.topk_idx)
            np.testing.assert_allclose(x.topk_logit, y.topk_logit, rtol=1e-5, atol=1e-5)


def test_set_weights_device_from_torch_tensor(device):
    """The N-rank weight path (bench.py: RCCL broadcast -> Executor.set_weights_device): a pipeline built with
    other weights, given another pipeline's folded weight blob as a torch CUDA tensor (device-to-device copy),
    reads back the same bytes and produces bit-identical outputs."""
    from inference_arena_amd.data.synthetic import synthetic_images
    from inference_arena_amd.engine.pipeline import GpuPipeline
    from inference_arena_amd.models.zoo import make_mobilenet, make_yolo

    a = GpuPipeline(make_yolo(0, cls_shift=-20.0), make_mobilenet(1), device=0, buckets=[4], dtype="fp32")
    b = GpuPipeline(make_yolo(5, cls_shift=-20.0), make_mobilenet(6), device=0, buckets=[4], dtype="fp32")
    blob = np.ascontiguousarray(a.program.weights)
    assert blob.nbytes == np.ascontiguousarray(b.program.weights).nbytes
    assert bytes(b.ex.weights_host()) != blob.tobytes()
    t = torch.from_numpy(blob.view(np.uint8).copy()).to("cuda:0")
    b.ex.set_weights_device(t.data_ptr(), t.numel())
    torch.cuda.synchronize()
    assert bytes(b.ex.weights_host()) == blob.tobytes()
    imgs = synthetic_images(4, 21)
    ra, rb = a.infer(imgs), b.infer(imgs)
    assert sum(len(r) for r in ra) > 0
    for x, y in zip(ra, rb):
        np.testing.assert_array_equal(x.boxes, y.boxes)
        np.testing.assert_array_equal(x.topk_idx, y.topk_idx)
        np.testing.assert_array_equal(x.topk_logit, y.topk_logit)
