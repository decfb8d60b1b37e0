"""Arm B device transport on the GPU: frames exported by another process (hipIpcGetMemHandle over dmabuf,
csrc/runtime/ipc_buffer.h) are classified straight from the mapped memory (Executor::submit_device) and give
exactly the split topology's results for the same detections (same second-stage program, same crops)."""
from __future__ import annotations

import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

# the detection side, as its own process: one IPC ring, every frame put once, refs to stdout, then it keeps the
# memory alive until the consumer says it is done (a line on stdin)
PRODUCER = r"""
import sys
import numpy as np
from inference_arena_amd.server.device_transport import DeviceImageRing
frames = [np.load(p) for p in sys.argv[1:]]
ring = DeviceImageRing(len(frames), max(f.nbytes for f in frames), device=0)
for f in frames:
    _, ref = ring.put(f)
    sys.stdout.write(ref.SerializeToString().hex() + "\n")
sys.stdout.flush()
sys.stdin.readline()
"""


@pytest.fixture(scope="module")
def dense_models():
    from inference_arena_amd.models.zoo import make_mobilenet, make_yolo

    return make_yolo(0, cls_shift=-20.0), make_mobilenet(1)


def _export(frames, tmp_path):
    paths = []
    for i, f in enumerate(frames):
        p = tmp_path / f"f{i}.npy"
        np.save(p, np.ascontiguousarray(f))
        paths.append(str(p))
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    proc = subprocess.Popen([sys.executable, "-c", PRODUCER, *paths], stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                            text=True, env=env, cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from inference_arena_amd.proto import inference_api as pb

    refs = []
    for _ in frames:
        line = proc.stdout.readline()
        assert line, f"producer exited early (rc={proc.poll()})"
        refs.append(pb.DeviceImageRef.FromString(bytes.fromhex(line.strip())))
    return proc, refs


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_ipc_frames_match_split_pipeline(dense_models, device, dtype, tmp_path):
    from inference_arena_amd.data.synthetic import synthetic_images
    from inference_arena_amd.engine.pipeline import GpuFrameClassifier, SplitPipeline
    from inference_arena_amd.ops import native

    imgs = synthetic_images(7, 81) + synthetic_images(1, 82, hw=(333, 500))
    ref = SplitPipeline(*dense_models, det_device=0, cls_device=0, buckets=[8], dtype=dtype).infer(imgs)
    assert sum(len(r) for r in ref) > 5
    cls = GpuFrameClassifier(dense_models[1], device=0, buckets=[1, 8], dtype=dtype)
    proc, refs = _export(imgs, tmp_path)
    C = native()
    try:
        base = C.ipc_open(refs[0].handle, 0)
        assert all(r.handle == refs[0].handle for r in refs)
        images = [(base + r.offset, r.height, r.width, r.device) for r in refs]
        boxes = [np.concatenate([r.boxes, r.scores[:, None], r.classes[:, None].astype(np.float32)], 1)
                 for r in ref]
        res = cls.collect(cls.submit(images, boxes))
        offs = res["crop_offset"]
        for i, r in enumerate(ref):
            a, b = int(offs[i]), int(offs[i + 1])
            assert b - a == len(r)
            np.testing.assert_array_equal(res["topk_idx"][a:b], r.topk_idx)
            np.testing.assert_array_equal(res["topk_logit"][a:b], r.topk_logit)
        # one frame at a time (bucket 1) and an empty box list in a batch
        one = cls.collect(cls.submit(images[:1], boxes[:1]))
        np.testing.assert_array_equal(one["topk_idx"], ref[0].topk_idx)
        mixed = cls.collect(cls.submit(images[:2], [np.zeros((0, 6), np.float32), boxes[1]]))
        assert list(mixed["crop_offset"]) == [0, 0, len(ref[1])]
        np.testing.assert_array_equal(mixed["topk_idx"], ref[1].topk_idx)
        C.ipc_close(base)
    finally:
        proc.stdin.write("done\n")
        proc.stdin.flush()
        assert proc.wait(60) == 0


def test_device_classifier_batches_ipc_frames(dense_models, device, tmp_path):
    """The service-side micro-batcher over the real frame classifier: concurrent frames from one mapped ring."""
    import asyncio

    from inference_arena_amd.data.synthetic import synthetic_images
    from inference_arena_amd.engine.pipeline import GpuFrameClassifier, GpuPipeline
    from inference_arena_amd.ops import native
    from inference_arena_amd.server.device_transport import DeviceClassifier, ImageKey

    imgs = synthetic_images(6, 21)
    fused = GpuPipeline(*dense_models, device=0, buckets=[8], dtype="fp32").infer(imgs)
    cls = GpuFrameClassifier(dense_models[1], device=0, buckets=[1, 2, 4, 8], dtype="fp32")
    proc, refs = _export(imgs, tmp_path)
    C = native()
    dc = DeviceClassifier(cls, lambda h: C.ipc_open(h, 0), max_batch=8,
                          max_crops=int(cls.ex.crop_cap_for(8)), max_delay_us=5000)
    try:
        async def go():
            keys = [ImageKey(r.handle, r.device, r.offset, r.height, r.width) for r in refs]
            boxes = [np.concatenate([f.boxes, f.scores[:, None], f.classes[:, None].astype(np.float32)], 1)
                     for f in fused]
            out = await asyncio.gather(*(dc.classify(k, b) for k, b in zip(keys, boxes)))
            dc.close()
            return out

        out = asyncio.run(go())
        assert dc.frames == len(imgs) and dc.batches < len(imgs)
        for f, got in zip(fused, out):
            assert [list(ids) for ids, _ in got] == f.topk_idx.tolist()
            probs = np.asarray([p for _, p in got], np.float64).reshape(-1, f.topk_prob.shape[1])  # (0, 5): no boxes
            np.testing.assert_allclose(probs, f.topk_prob, rtol=1e-4, atol=1e-6)
    finally:
        proc.stdin.write("done\n")
        proc.stdin.flush()
        assert proc.wait(60) == 0


def test_detector_exports_its_staged_frames_into_the_ring(dense_models, device):
    """The GPU detector copies each frame it staged for YOLO into the given ring slot, device to device in its
    batch (InputImage.export_dst): the slot holds the exact frame once the detection answer is back, and the
    detections are those of a run without export (server/detection_service.py's device transport)."""
    import asyncio

    from inference_arena_amd.data.synthetic import synthetic_images
    from inference_arena_amd.server.batching import AsyncBatcher
    from inference_arena_amd.engine.registry import build_session
    from inference_arena_amd.server.device_transport import DeviceImageRing

    imgs = synthetic_images(5, 41) + synthetic_images(2, 42, hw=(333, 500))
    runner = build_session("detector", dense_models[0], device=0, buckets=[1, 8])
    b = AsyncBatcher([runner], max_batch=8, max_queue_delay_us=2000)
    ring = DeviceImageRing(len(imgs), 640 * 640 * 3, device=0)
    slots = [ring.acquire() for _ in imgs]

    async def go(export: bool):
        return await asyncio.gather(*(b.run(im, export_to=ring.slot_ptr(s) if export else 0)
                                      for im, s in zip(imgs, slots)))

    try:
        plain = asyncio.run(go(False))
        exported = asyncio.run(go(True))
        for im, s, p, e in zip(imgs, slots, plain, exported):
            got = np.frombuffer(ring.buf.read(s * ring.slot_bytes, im.nbytes), np.uint8).reshape(im.shape)
            np.testing.assert_array_equal(got, im)
            np.testing.assert_array_equal(p["det"], e["det"])
    finally:
        b.close()
